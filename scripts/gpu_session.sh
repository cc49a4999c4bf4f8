#!/bin/bash
# One GPU session: GPU parity tests, smoke, bench (ODE chemistry, the headline line) + variants given
# in VARIANTS ("name:ENV=V,ENV=V:bench args;..."), and a rocprofv3 kernel-trace summary of the
# headline bench. Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log; ok $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_ode.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_ode.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "${VS[@]}"; do
  [ -z "$v" ] && continue
  name="${v%%:*}"; rest="${v#*:}"; envs="${rest%%:*}"; args="${rest#*:}"
  ( for e in $(echo "$envs" | tr ',' ' '); do export "$e"; done
    timeout -k 10 300 python bench.py --no-cpu --no-flame $args > gpurun_out/bench_$name.log 2>&1 )
  rc=$?; echo "variant $name rc=$rc"
  python - "$name" <<'EOF'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/bench_{n}.log").read().strip().splitlines()[-1])
print(n, round(d["ms_per_step"], 3), "ms", d["solver_iters"], "roof", round(d["roofline"]["frac"] or 0, 3))
EOF
  [ $rc -eq 0 ] || exit $rc
done
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-flame --alt-steps 0 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.csv 2>&1; head -30 gpurun_out/prof_summary.csv
fi
exit 0
