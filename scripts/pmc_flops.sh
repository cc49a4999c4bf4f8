#!/bin/bash
# FP64 VALU work per kernel from one SQ counter pass (at most 8 SQ counters; counters only, no tracing
# domains) over the headline bench workload -> gpurun_out/pmc_flops.json (copy to profiles/). The thermo and
# chemistry kernels are FP64-VALU bound; bench.py prices their counted FLOPs against the FP64 vector peak.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES"
timeout -k 10 400 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_flops -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-flame --alt-steps 0 ${BENCH_ARGS} > gpurun_out/pmc_flops.log 2>&1
rc=$?; echo "pmc flops rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pmc_flops -name "*counter_collection.csv" | sort | tail -1)
python3 scripts/pmc_flops_summary.py "$f" gpurun_out/pmc_flops.json
