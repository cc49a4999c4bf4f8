#!/bin/bash
# Full GPU session: all GPU tests, smoke, bench (chemistry ODE / DNN / off), rocprofv3 summary.
# Stops at the first GPU fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for mode in ode dnn off; do
  extra="--no-cpu"; [ $mode = ode ] && extra=""
  timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 --chem $mode $extra > gpurun_out/bench_$mode.log 2>&1
  rc=$?; echo "bench $mode rc=$rc"; tail -1 gpurun_out/bench_$mode.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
