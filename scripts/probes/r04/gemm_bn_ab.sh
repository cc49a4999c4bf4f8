#!/bin/bash
# DNN GEMM N-tile A/B (DFMI_GEMM_BN160): surrogate parity tests, then scripts/dnn_layers.py (53-species nets,
# 64^3 all reacting) with the 160-wide tiles on and off, twice each, and a per-layer dispatch trace with them on.
# (DFMI_GEMM_BN160 and its 160-wide tile were removed after this measurement: profiles/r03_gemm_bn160_ab.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_dnn.py tests/test_gpu_species53.py -x -v --timeout 240 --timeout-method thread > gpurun_out/bn_parity.log 2>&1
rc=$?; tail -3 gpurun_out/bn_parity.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    DFMI_GEMM_BN160=$v timeout -k 10 200 python scripts/dnn_layers.py 64 3 > gpurun_out/bn_layers_${v}_$rep.json 2>gpurun_out/bn_layers.err
    rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/bn_layers.err; exit $rc; }
    echo "BN160=$v $(cat gpurun_out/bn_layers_${v}_$rep.json)"
  done
done
bash scripts/gemm_trace.sh
