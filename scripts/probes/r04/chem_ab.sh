#!/bin/bash
# Chemistry A/B: GPU chemistry tests, then the ODE bench with cost binning on and off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_chemistry.py -q > gpurun_out/chem_tests.log 2>&1
rc=$?; echo "chem tests rc=$rc"; tail -5 gpurun_out/chem_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-5} --no-cpu > gpurun_out/bench_bin.log 2>&1
rc=$?; echo "bench bin rc=$rc"; tail -1 gpurun_out/bench_bin.log; [ $rc -eq 0 ] || exit $rc
DFMI_CHEM_BIN=0 timeout -k 10 300 python bench.py --steps ${STEPS:-5} --no-cpu > gpurun_out/bench_nobin.log 2>&1
rc=$?; echo "bench nobin rc=$rc"; tail -1 gpurun_out/bench_nobin.log; exit $rc
