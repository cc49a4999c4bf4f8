#!/bin/bash
# Round-6 GPU check: the GPU tests (one process, per-test time limit), then a short headline bench.
# Stops at the first failure of the tests; never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/${TAG}_tests.log | tail -3
grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---no-cpu --no-flame --alt-steps 0} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/${TAG}_bench.log
exit $rc
