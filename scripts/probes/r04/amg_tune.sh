#!/bin/bash
# AMG parameter sweep on the 2M bench (one process per setting, each under its own time limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for om in ${OMEGAS:-0.6 0.7 0.8}; do
  for cs in ${SWEEPS:-12 24}; do
    DFMI_AMG_OMEGA=$om DFMI_AMG_COARSE_SWEEPS=$cs timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/tune_${om}_${cs}.log 2>&1
    rc=$?
    python -c "import json,sys; d=json.loads(open('gpurun_out/tune_${om}_${cs}.log').read().strip().splitlines()[-1]); print('omega=$om sweeps=$cs', round(d['ms_per_step'],2), 'ms', d['solver_iters'])" || exit $rc
    [ $rc -eq 0 ] || exit $rc
  done
done
