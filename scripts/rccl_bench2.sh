#!/bin/bash
# bench.py --gpus 2 under torchrun on the box's one GPU over RCCL's socket transport (DFMI_RCCL_SPLIT_HOSTS),
# halo overlap off and on: a functional check of the multi-GPU bench path and of the overlap's effect when
# the wire is slow (not a scaling measurement).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ov in 0 1; do
  DFMI_HALO_OVERLAP=$ov DFMI_RCCL_SPLIT_HOSTS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29555 + ov)) bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-flame \
    > gpurun_out/bench_rccl2_ov$ov.log 2>&1
  rc=$?; echo "overlap $ov rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$ov" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_rccl2_ov{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("overlap", sys.argv[1], round(d["ms_per_step"], 2), "ms/step", d["solver_iters"])
PY
done
