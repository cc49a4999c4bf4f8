#!/bin/bash
# A/B of one environment knob on the headline (bench.py, 1 GPU, no CPU / flame / alternate-scheme lines):
# the listed GPU tests first, then the bench alternating the settings twice. Stops at the first failure.
# usage: TESTS="tests/test_x.py ..." bash scripts/knob_ab.sh "ENV=a" "ENV=b"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > gpurun_out/knob_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/knob_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    ( export $setting
      timeout -k 10 300 python bench.py --no-cpu --no-flame --alt-steps 0 ${BENCH_ARGS} > gpurun_out/knob_${rep}_${i}.log 2>&1 )
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/knob_${rep}_${i}.log; exit $rc; }
    python3 - "$setting" "gpurun_out/knob_${rep}_${i}.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], round(d["ms_per_step"], 3), "ms/step", "iters", d.get("solver_iters"), flush=True)
PY
  done
done
