#!/bin/bash
# Round-4 A/B session: the tests named in TESTS, then one short bench run per variant in VARIANTS
# ("name:ENV=V,ENV=V;..."), printing ms/step and the per-kernel rooflines named in KERNELS. Every GPU step
# has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/ab_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "${VS[@]}"; do
  [ -z "$v" ] && continue
  name="${v%%:*}"; envs="${v#*:}"
  ( for e in $(echo "$envs" | tr ',' ' '); do export "$e"; done
    timeout -k 10 300 python bench.py --no-cpu --no-flame --steps ${STEPS:-10} --alt-steps 0 ${BENCH_ARGS} > gpurun_out/ab_$name.log 2>&1 )
  rc=$?; echo "variant $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$name.log; exit $rc; }
  KERNELS="${KERNELS:-k_y_prep}" python - "$name" <<'EOF'
import json, os, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{n}.log").read().strip().splitlines()[-1])
out = [n, round(d["ms_per_step"], 3), "ms", "iters", d.get("solver_iters")]
for k in os.environ["KERNELS"].split(","):
    r = (d.get("rooflines") or {}).get(k) or {}
    out += [k, round(r.get("avg_us") or 0, 1), "us", "frac", round(r.get("frac") or 0, 3)]
ch = d.get("chemistry") or {}
if "k_chem_ms_per_step" in ch:
    out += ["chem", round(ch["k_chem_ms_per_step"], 3), "ms/step"]
print(*out)
EOF
done
exit 0
