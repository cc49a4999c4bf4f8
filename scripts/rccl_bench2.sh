#!/bin/bash
# bench.py --gpus 2 under torchrun on the box's one GPU over RCCL's socket transport (DFMI_RCCL_SPLIT_HOSTS):
# a functional check of the multi-GPU bench path (not a scaling measurement) for the settings in VARS
# ("name:ENV=V,ENV=V ..."; default: the halo-coupled AMG level 0 on and off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
port=29555
for v in ${VARS:-halo: bj:DFMI_OPTIONS=amg.halo_l0=0}; do
  name="${v%%:*}"; envs="${v#*:}"; port=$((port + 1))
  ( for e in $(echo "$envs" | tr ',' ' '); do export "$e"; done
    DFMI_RCCL_SPLIT_HOSTS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-flame \
      --alt-steps 0 > gpurun_out/bench_rccl2_$name.log 2>&1 )
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$name" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/bench_rccl2_{sys.argv[1]}.log") if l.startswith("{")][-1])
print(sys.argv[1], round(d["ms_per_step"], 2), "ms/step", d["solver_iters"], "levels", d["amg_levels"][-2:],
      "hex", d.get("hex_face_walk"), "classes", d.get("row_classes"))
c = d.get("comm")
if c:
    print("  comm ms/step max", round(c["comm_ms_per_step"]["max"], 3), "of", round(c["step_ms"], 2),
          "halo", round(c["halo_ms_per_step_max"], 3), "allgather", round(c["allgather_ms_per_step_max"], 3))
    for k, v in sorted(c["points"].items(), key=lambda kv: -kv[1]["ms_per_step_max"])[:12]:
        print(f"    {k:34s} calls/step {v['calls_per_step']:6.1f}  KB/call {v['bytes_per_call'] / 1e3:9.1f}  ms/step {v['ms_per_step_max']:.3f}")
PY
done
