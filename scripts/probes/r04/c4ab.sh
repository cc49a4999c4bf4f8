# config-4 A/B under rocprofv3 (kernel stats): parity tests first, then one profiled run per setting
# usage: bash scripts/c4ab.sh "ENV=a" "ENV=b" ...   (each argument: space-separated VAR=value list)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_species53.py tests/test_gpu_dnn.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/t.log 2>&1
echo tests ok
cd /tmp && export TMPDIR=/tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  ( export $setting; timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab$i -o run -- python3 $R/scripts/config4_profile.py > $R/gpurun_out/ab$i.log 2>&1 )
  python3 - $R/gpurun_out/ab$i <<'PY'
import csv, os, sys
d = sys.argv[1]
rows = [r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))]
keep = [r for r in rows if any(k in r["Kernel_Name"] for k in ("thermo", "y_prep", "y_assemble", "mlp_gemm", "bcg_", "cg_"))]
with open(os.path.join(d, "trace_small.csv"), "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys())); w.writeheader(); w.writerows(keep)
os.remove(os.path.join(d, "run_kernel_trace.csv"))
PY
  echo "ab$i ($setting) ok"
done
