#!/bin/bash
# A/B of option settings on one box (no rebuild): the headline bench with DFMI_OPTIONS unset / set, alternated
# A B A B -> gpurun_out/${TAG}_ab_<k>.log; OPTS_B="key=value,..." is the B arm, OPTS_A (default empty) the A arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
for k in ${ORDER:-A1 B1 A2 B2}; do
  case $k in A*) O="$OPTS_A" ;; B*) O="$OPTS_B" ;; esac
  DFMI_OPTIONS="$O" timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu --no-flame --alt-steps 0 \
    > gpurun_out/${TAG}_ab_$k.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$k rc=$rc"; tail -5 gpurun_out/${TAG}_ab_$k.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${TAG}_ab_$k.log') if l.startswith('{')][0]); print('$k', '$O', round(d['ms_per_step'],3), round(d['ms_per_step_median'],3), d['solver_iters'])"
done
