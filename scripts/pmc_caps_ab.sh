#!/bin/bash
# where the assembly kernels' traffic beyond their algorithmic bytes comes from. Per arm
# (A = the tree's library with the side-stream register caps, B = ab/libdfmi_b.so built with -DDFMI_NO_CAPS):
# one rocprofv3 pass with the L2 counters (hits, misses, fabric read / write requests) and one each with
# FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md: separate passes), counters only, on the headline workload.
# Summaries -> gpurun_out/pmc_caps_<arm>_{l2,traffic}.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepflame-dev_amd/libdfmi.so
cp $L /tmp/libdfmi_a.so
B="python3 bench.py --steps 1 --warmup 1 --roof-steps 1 --no-cpu --no-flame --alt-steps 0"
for arm in ${ARMS:-A B}; do
  case $arm in A) cp /tmp/libdfmi_a.so $L ;; B) cp ab/libdfmi_b.so $L ;; esac
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv \
    -d gpurun_out/pmc_caps_${arm}_l2 -o run -- $B > gpurun_out/pmc_caps_${arm}_l2.log 2>&1
  rc=$?; echo "$arm l2 rc=$rc"; [ $rc -eq 0 ] || { cp /tmp/libdfmi_a.so $L; exit $rc; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_caps_${arm}_$c -o run -- $B \
      > gpurun_out/pmc_caps_${arm}_$c.log 2>&1
    rc=$?; echo "$arm $c rc=$rc"; [ $rc -eq 0 ] || { cp /tmp/libdfmi_a.so $L; exit $rc; }
  done
  l2=$(find gpurun_out/pmc_caps_${arm}_l2 -name "*counter_collection.csv" | sort | tail -1)
  python3 scripts/pmc_l2_summary.py "$l2" 1000000 gpurun_out/pmc_caps_${arm}_l2.json
  f=$(find gpurun_out/pmc_caps_${arm}_FETCH_SIZE -name "*counter_collection.csv" | sort | tail -1)
  w=$(find gpurun_out/pmc_caps_${arm}_WRITE_SIZE -name "*counter_collection.csv" | sort | tail -1)
  python3 scripts/pmc_summary.py "$f" "$w" gpurun_out/pmc_caps_${arm}_traffic.json > /dev/null
  rm -rf gpurun_out/pmc_caps_${arm}_l2 gpurun_out/pmc_caps_${arm}_FETCH_SIZE gpurun_out/pmc_caps_${arm}_WRITE_SIZE
done
cp /tmp/libdfmi_a.so $L
