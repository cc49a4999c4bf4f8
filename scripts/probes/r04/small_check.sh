# GPU tests (small systems now solved in one workgroup) + 1D-flame A/B of the fused small solves
set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $R/gpurun_out/small_tests.log 2>&1 || { tail -40 $R/gpurun_out/small_tests.log; exit 1; }
tail -2 $R/gpurun_out/small_tests.log
for s in "DFMI_SMALL_SOLVE=0" "DFMI_SMALL_SOLVE=1"; do
  ( export $s; timeout -k 10 100 python3 $R/scripts/flame1d_profile.py 50 > $R/gpurun_out/flab.tmp 2>&1; echo "$s $(tail -1 $R/gpurun_out/flab.tmp | cut -c1-600)" )
done
