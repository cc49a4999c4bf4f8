#!/bin/bash
# k_restrict with batched member loads (tree) against the plain member loop (scripts/tmp/libdfmi_base.so):
# AMG GPU tests, 3 rounds of the headline A/B, and one kernel-trace summary per arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_cg_fuse.py \
  tests/test_gpu_amg_tail.py tests/test_gpu_amg_reuse.py > gpurun_out/r06y_tests.log 2>&1 || exit 1
TAG=r06y ROUNDS=3 ARMS="new=: base=scripts/tmp/libdfmi_base.so:" bash scripts/ab_arms.sh || exit 1
L=deepflame-dev_amd/libdfmi.so
cp $L /tmp/libdfmi_new.so
for arm in new base; do
  cp /tmp/libdfmi_$arm.so $L 2>/dev/null || cp scripts/tmp/libdfmi_base.so $L
  DFMI_STEP_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06y_prof_$arm -o run -- \
    python3 bench.py --steps 8 --warmup 3 --no-cpu --no-flame --alt-steps 0 > gpurun_out/r06y_prof_$arm.log 2>&1 || { cp /tmp/libdfmi_new.so $L; exit 1; }
done
cp /tmp/libdfmi_new.so $L
