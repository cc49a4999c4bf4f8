#!/bin/bash
# Round-6 measurement session on the final tree, each step under its own time limit, stopping at the first failure:
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) -> gpurun_out/pmc_traffic.json, PMC FP64 FLOPs ->
# gpurun_out/pmc_flops.json, kernel-trace statistics of the headline bench with the side stream folded in
# (DFMI_STEP_OVERLAP=0: every kernel alone on the GPU) -> gpurun_out/r06_prof/, then the default bench.py line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_PMC" ]; then
  bash scripts/pmc_traffic.sh || exit $?
  bash scripts/pmc_flops.sh || exit $?
fi
rm -rf gpurun_out/r06_prof
DFMI_STEP_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_prof -o run -- \
  python3 bench.py --steps 16 --warmup 5 --no-cpu --no-flame --alt-steps 0 > gpurun_out/r06_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py gpurun_out/r06_prof > gpurun_out/r06_prof_summary.csv 2>&1; head -12 gpurun_out/r06_prof_summary.csv
timeout -k 10 600 python3 bench.py > gpurun_out/r06_bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 800 gpurun_out/r06_bench_full.log; exit $rc
