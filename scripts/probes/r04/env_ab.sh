# headline bench under rocprofv3 for each environment setting given (kernel stats only); GPU parity tests first
# usage: bash scripts/env_ab.sh "ENV=a" "ENV=b" ...
set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/t.log 2>&1
echo tests ok
cd /tmp && export TMPDIR=/tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  ( export $setting
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/eab$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-flame > $R/gpurun_out/eab$i.log 2>&1
    rm -f $R/gpurun_out/eab$i/run_kernel_trace.csv
    timeout -k 10 300 python3 $R/bench.py --no-cpu --no-flame > $R/gpurun_out/eabb$i.log 2>&1 )
  echo "eab$i ($setting) $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/eabb$i.log | head -1)"
done
