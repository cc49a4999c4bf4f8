set -e
R=$GRAFT_REPO_ROOT
for s in "DFMI_NONE=0" "DFMI_AMG_COARSEST=16" "DFMI_AMG_COARSE_SWEEPS=64" "DFMI_AMG_COARSEST=64" "DFMI_AMG_COARSEST=16 DFMI_AMG_COARSE_SWEEPS=16"; do
  ( export $s; timeout -k 10 100 python3 $R/scripts/flame1d_profile.py 50 > $R/gpurun_out/flab.tmp 2>&1; echo "$s $(tail -1 $R/gpurun_out/flab.tmp | grep -o "'ms_per_step': [0-9.]*")" )
done
