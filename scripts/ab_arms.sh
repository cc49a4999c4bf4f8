#!/bin/bash
# A/B/C... of library builds and option settings on one box: ARMS="name=lib:opts ..." where lib is a path to a
# libdfmi.so build ("" = the tree's) and opts a DFMI_OPTIONS string; the arms run in turn, ROUNDS times, each a
# short headline bench -> gpurun_out/${TAG}_arm_<name><round>.log and one summary line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
L=deepflame-dev_amd/libdfmi.so
cp $L /tmp/libdfmi_tree.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in $ARMS; do
    name=${arm%%=*}; spec=${arm#*=}; lib=${spec%%:*}; opts=${spec#*:}
    if [ -n "$lib" ]; then cp "$lib" $L; else cp /tmp/libdfmi_tree.so $L; fi
    DFMI_OPTIONS="$opts" timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu --no-flame \
      --alt-steps 0 > gpurun_out/${TAG}_arm_$name$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$name$r rc=$rc"; tail -5 gpurun_out/${TAG}_arm_$name$r.log; cp /tmp/libdfmi_tree.so $L; exit $rc; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${TAG}_arm_$name$r.log') if l.startswith('{')][0]); r=d['rooflines']; print('$name$r', round(d['ms_per_step'],3), round(d['ms_per_step_median'],3), {k: round(r[k]['avg_us'],1) for k in ('k_y_assemble_ell','k_u_assemble','k_y_prep','k_e_assemble','k_bcg_eo','k_cg_spmv') if k in r}, d['solver_iters'])"
  done
done
cp /tmp/libdfmi_tree.so $L
