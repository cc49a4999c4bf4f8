#!/bin/bash
# DNN GEMM A/B (DFMI_GEMM_PIPE): surrogate parity tests with the variant, then bench --chem dnn (H2 nets)
# with and without it. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DFMI_GEMM_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_dnn.py tests/test_gpu_species53.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gemm_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/gemm_parity.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  DFMI_GEMM_PIPE=$v timeout -k 10 300 python bench.py --chem dnn --no-cpu --no-flame --steps 5 --warmup 2 > gpurun_out/bench_gemm$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_gemm{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("pipe", sys.argv[1], round(d["ms_per_step"], 2), "ms/step", "gemm", round(d["dnn"]["gemm_ms_total"], 2), "ms", "frac", round(d["dnn"]["mfma_roofline"]["frac"], 3))
PY
done
