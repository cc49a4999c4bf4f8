#!/bin/bash
# A/B of the level-0 AMG smoothing sweeps (DFMI_AMG_L0_SWEEPS) + parity of the batched path with them,
# then the 2-rank bench rehearsal over RCCL sockets (DFMI_RCCL_SPLIT_HOSTS). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_PARITY" ]; then
  DFMI_SMALL_SOLVE=0 DFMI_AMG_L0_SWEEPS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "amg_pcg" -x -q --timeout 120 --timeout-method thread > gpurun_out/amg_sweeps_parity.log 2>&1
  rc=$?; echo "parity rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PROF=1 VARIANTS="${VARIANTS}" bash scripts/gpu_session.sh || exit $?
if [ -n "$RCCL_BENCH" ]; then
  DFMI_RCCL_SPLIT_HOSTS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-flame \
    > gpurun_out/bench_rccl2.log 2>&1
  rc=$?; echo "rccl bench rc=$rc"; tail -2 gpurun_out/bench_rccl2.log | cut -c1-800; [ $rc -eq 0 ] || exit $rc
fi
exit 0
