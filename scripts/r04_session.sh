#!/bin/bash
# Round-4 GPU session: the tests named in TESTS (default: multi-rank / even-odd / RCCL / chemistry), the bench
# variants in VARIANTS (gpu_session.sh syntax "name:ENV=V,ENV=V:args;..."), optionally the 2-rank RCCL rehearsal
# (RCCL2=1). Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_multirank.py tests/test_gpu_eo.py tests/test_gpu_rccl.py tests/test_gpu_chemistry.py tests/test_gpu_headline_state.py tests/test_gpu_zero_d.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-800} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/r04_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then
  SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PROF=${SKIP_PROF:-1} BENCH_ARGS="--no-cpu --no-flame" bash scripts/gpu_session.sh || exit $?
fi
if [ -n "$RCCL2" ]; then
  VARS="halo:" bash scripts/rccl_bench2.sh || exit $?
fi
exit 0
