#!/bin/bash
# Per-layer DNN GEMM dispatch durations (rocprofv3 kernel trace of scripts/dnn_layers.py) -> gpurun_out/gemm_trace.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && rm -rf gpurun_out/gt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt -- python3 scripts/dnn_layers.py ${N:-64} 2 > gpurun_out/gemm_trace.log 2>&1
rc=$?; tail -2 gpurun_out/gemm_trace.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/gemm_trace.py gpurun_out/gt > gpurun_out/gemm_trace.json && cat gpurun_out/gemm_trace.json
