#!/bin/bash
# One GPU session: parity tests, a short bench, a rocprofv3 kernel-trace summary.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0 and 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 ${TEST_TIMEOUT:-400} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/gpu_tests.log; ok $rc || exit $rc
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_PROF" ] && exit 0
export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${BENCH_ARGS} --no-cpu > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
