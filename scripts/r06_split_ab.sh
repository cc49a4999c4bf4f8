#!/bin/bash
# Level-0 prolongation + post-sweep as two passes (scripts/tmp/libdfmi_split.so, option amg.split_prolong) against
# the tree's one-pass k_prolong_smooth: the bitwise check, 3 rounds of the headline A/B, one kernel trace per arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=deepflame-dev_amd/libdfmi.so
cp $L /tmp/libdfmi_tree.so
cp scripts/tmp/libdfmi_split.so $L
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread scripts/split_prolong_check.py \
  > gpurun_out/r06w_test.log 2>&1
rc=$?; cp /tmp/libdfmi_tree.so $L; [ $rc -eq 0 ] || exit $rc
TAG=r06w ROUNDS=3 ARMS="split=scripts/tmp/libdfmi_split.so: base=:" bash scripts/ab_arms.sh || exit 1
for arm in split base; do
  if [ $arm = split ]; then cp scripts/tmp/libdfmi_split.so $L; else cp /tmp/libdfmi_tree.so $L; fi
  DFMI_STEP_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06w_prof_$arm -o run -- \
    python3 bench.py --steps 8 --warmup 3 --no-cpu --no-flame --alt-steps 0 > gpurun_out/r06w_prof_$arm.log 2>&1 || { cp /tmp/libdfmi_tree.so $L; exit 1; }
done
cp /tmp/libdfmi_tree.so $L
