#!/bin/bash
# Per-kernel stats (rocprofv3 --kernel-trace --stats) of the headline bench for each setting of one knob;
# prints the listed kernels' average us and calls. usage: KERNELS="k_a|k_b" bash scripts/knob_prof.sh "ENV=a" "ENV=b"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
i=0
for setting in "$@"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && export $setting
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kp$i" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --roof-steps 0 --no-cpu --no-flame --alt-steps 0 > "$R/gpurun_out/kp$i.log" 2>&1 )
  rc=$?; [ $rc -eq 0 ] || { tail -3 "$R/gpurun_out/kp$i.log"; exit $rc; }
  rm -f "$R/gpurun_out/kp$i/run_kernel_trace.csv"
  echo "== $setting $(grep -o '"ms_per_step": [0-9.]*' "$R/gpurun_out/kp$i.log" | head -1)"
  python3 - "$R/gpurun_out/kp$i/run_kernel_stats.csv" "${KERNELS:-k_}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f'{float(r["AverageNs"]) / 1e3:9.1f} us x {r["Calls"]:>5}  {r["Name"][:80]}')
PY
done
