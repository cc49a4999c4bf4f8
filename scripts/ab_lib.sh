#!/bin/bash
# A/B of two builds of libdfmi.so on one box: A = the tree's library, B = ab/libdfmi_b.so, alternated
# A B A B (ORDER="A1 B1 A2 B2 A3 B3" for more pairs), each a short headline bench (--no-cpu --no-flame --alt-steps 0) -> gpurun_out/ab_lib_<k>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=deepflame-dev_amd/libdfmi.so
cp $L /tmp/libdfmi_a.so
for k in ${ORDER:-A1 B1 A2 B2}; do
  case $k in A*) cp /tmp/libdfmi_a.so $L ;; B*) cp ab/libdfmi_b.so $L ;; esac
  timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu --no-flame --alt-steps 0 > gpurun_out/ab_lib_$k.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$k rc=$rc"; exit $rc; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_lib_$k.log') if l.startswith('{')][0]); print('$k', round(d['ms_per_step'],3), round(d['ms_per_step_median'],3), {k: round(r['avg_us'],1) for k, r in d['rooflines'].items()})"
done
cp /tmp/libdfmi_a.so $L
