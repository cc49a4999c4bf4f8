#!/bin/bash
# Round-5 GPU session. Steps (each under its own time limit, stop at the first failure):
#   TESTS   pytest files/node ids (default none)          -> gpurun_out/r05_tests.log
#   BENCH   bench.py arguments (unset: skip)              -> gpurun_out/r05_bench.log
#   PROF    bench.py arguments under rocprofv3 --kernel-trace --stats (unset: skip) -> gpurun_out/r05_prof/
#   EXTRA   one more command line (unset: skip)           -> gpurun_out/r05_extra.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -x -v --timeout ${PER_TEST:-300} --timeout-method thread > gpurun_out/r05_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/r05_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python3 bench.py $BENCH > gpurun_out/r05_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r05_bench.log; echo; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/r05_prof
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof -o run -- python3 bench.py $PROF > gpurun_out/r05_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/prof_summary.py gpurun_out/r05_prof | head -40
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${EXTRA_TIMEOUT:-400} bash -c "$EXTRA" > gpurun_out/r05_extra.log 2>&1
  rc=$?; echo "extra rc=$rc"; tail -c 1500 gpurun_out/r05_extra.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
