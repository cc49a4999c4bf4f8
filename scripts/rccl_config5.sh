#!/bin/bash
# BASELINE config 5's layout at full size on one GPU: 256^3 = 16.8M cells, decomposePar-style 2x2x2 blocks,
# 8 torchrun ranks over RCCL (socket transport, scripts/rccl_ranks.py), one outer iteration at tight solver
# tolerances vs the undecomposed 16.8M-cell run -> gpurun_out/rccl_config5.json. (Not a timing: all 8 ranks
# share one GPU and talk through loopback sockets.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${C5_TIMEOUT:-900} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29631 scripts/rccl_ranks.py --decomp 2,2,2 --mesh ${C5_MESH:-256,256,256} --no-oracle \
  --tol ${C5_TOL:-1e-12} --out gpurun_out/rccl_config5.json > gpurun_out/rccl_config5.log 2>&1
rc=$?; echo "config5 rc=$rc"; tail -2 gpurun_out/rccl_config5.log | cut -c1-600; exit $rc
