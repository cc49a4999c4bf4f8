#!/bin/bash
# Config-4 counter passes (each its own run, counters only): GRBM_GUI_ACTIVE (effective clock of the in-loop vs the
# surrogate-alone GEMMs, scripts/pmc_clock.py), FP64 VALU work per dispatch (k_thermo_coop's counted-FLOP roofline,
# scripts/pmc_flops_summary.py), then a kernel trace of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/c4_clock gpurun_out/c4_flops gpurun_out/c4_trace
timeout -k 10 500 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/c4_clock -o run -- python3 scripts/config4_profile.py 128 both > gpurun_out/c4_clock.log 2>&1
rc=$?; echo "clock rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_clock.py gpurun_out/c4_clock/run_counter_collection.csv gpurun_out/c4_clock.json --kernels k_mlp_gemm k_thermo_coop
PMC="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_LDS"
timeout -k 10 500 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/c4_flops -o run -- python3 scripts/config4_profile.py 128 > gpurun_out/c4_flops.log 2>&1
rc=$?; echo "flops rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_flops_summary.py gpurun_out/c4_flops/run_counter_collection.csv gpurun_out/c4_flops.json | head -8
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4_trace -o run -- python3 scripts/config4_profile.py 128 both > gpurun_out/c4_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py gpurun_out/c4_trace | head -24
