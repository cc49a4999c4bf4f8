#!/bin/bash
# Config-4 (2M cells x 53 species, DNN) A/B: the tests named in TESTS, then per variant in VARIANTS
# ("name:ENV=V,ENV=V;...") one rocprofv3 kernel trace of scripts/config4_profile.py with the step's side stream
# off (every kernel timed alone), printing ms/step and the summed durations of the kernels matching KERNELS.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/c4ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/c4ab_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "${VS[@]}"; do
  [ -z "$v" ] && continue
  name="${v%%:*}"; envs="${v#*:}"
  ( export DFMI_STEP_OVERLAP=0
    for e in $(echo "$envs" | tr ',' ' '); do export "$e"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4ab_$name -o run -- python3 scripts/config4_profile.py > gpurun_out/c4ab_$name.log 2>&1 )
  rc=$?; echo "variant $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c4ab_$name.log; exit $rc; }
  KERNELS="${KERNELS:-k_y_prep_gen,k_y_assemble_ell_gen,k_thermo_coop,k_mlp_gemm}" python3 - "$name" <<'EOF'
import ast, csv, os, sys
n = sys.argv[1]
line = [l for l in open(f"gpurun_out/c4ab_{n}.log") if l.startswith("{")][-1]
d = ast.literal_eval(line)
steps = d["steps"] + 1   # the profile's warmup step is traced too
rows = list(csv.DictReader(open(f"gpurun_out/c4ab_{n}/run_kernel_stats.csv")))
out = [n, round(d["ms_per_step"], 2), "ms/step", "iters", d.get("solver_iters")]
for k in os.environ["KERNELS"].split(","):
    tot = sum(float(r["TotalDurationNs"]) for r in rows if k in r["Name"])
    calls = sum(int(r["Calls"]) for r in rows if k in r["Name"])
    out += [k, round(tot / 1e6 / steps, 3), "ms/step", calls, "calls"]
print(*out)
EOF
done
exit 0
