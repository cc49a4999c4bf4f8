#!/bin/bash
# The 2-rank RCCL rehearsal of the multi-GPU bench on the box's one GPU (socket transport, not xGMI): bench.py
# --gpus 2 launches its own two ranks (DFMI_RCCL_SPLIT_HOSTS=1: each poses as its own host); in-order halos and
# DFMI_HALO_OVERLAP=1. Each line's `comm` block lists the exchange points -> gpurun_out/${TAG}_rccl2_<name>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
for v in halo:0 ov:1; do
  name="${v%%:*}"; ov="${v#*:}"
  DFMI_HALO_OVERLAP=$ov DFMI_RCCL_SPLIT_HOSTS=1 timeout -k 10 300 python3 bench.py --gpus 2 --n ${N:-128} --steps 3 \
    --warmup 1 --roof-steps 2 --no-cpu --no-flame --alt-steps 0 > gpurun_out/${TAG}_rccl2_$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/${TAG}_rccl2_$name.log | tail -1 > gpurun_out/${TAG}_rccl2_$name.json
  python3 - gpurun_out/${TAG}_rccl2_$name.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["comm"]
print(d["n_gpus"], d["config"]["parallelism"], round(d["ms_per_step"], 1), "ms/step", d["solver_iters"],
      "comm", round(c["comm_ms_per_step"]["max"], 1), "ms/step")
for k, v in sorted(c["points"].items(), key=lambda kv: -kv[1]["ms_per_step_max"])[:8]:
    print(f"  {k:28s} {v['calls_per_step']:6.1f} calls  {v['bytes_per_call'] / 1024:8.1f} KiB  {v['ms_per_step_max']:7.2f} ms")
PY
done
