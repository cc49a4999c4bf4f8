#!/bin/bash
# A/B session: optional parity tests under an env (PARITY_ENV="A=1 B=2", PARITY_K="pytest -k expr"), then bench
# variants (VARIANTS, see gpu_session.sh). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$PARITY_K" ]; then
  env $PARITY_ENV timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "$PARITY_K" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1
  rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/ab_parity.log; [ $rc -eq 0 ] || exit $rc
fi
SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PROF=1 VARIANTS="${VARIANTS}" bash scripts/gpu_session.sh || exit $?
exit 0
