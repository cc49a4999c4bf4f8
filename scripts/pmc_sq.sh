#!/bin/bash
# One SQ-counter pass (PMC="c1 c2 ...", at most 8 SQ counters) over a short headline bench; per-kernel means of
# the kernels matching KEYS -> gpurun_out/pmc_sq_<tag>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-sq}
# CMD: the profiled program (default: a short headline bench); it must start with the interpreter itself
CMD=${CMD:-"python3 bench.py --steps 2 --warmup 1 --no-cpu --no-flame --roof-steps 1 ${BENCH_ARGS}"}
timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_$tag -o run -- $CMD > gpurun_out/pmc_$tag.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pmc_$tag -name "*counter_collection.csv" | sort | tail -1)
python3 scripts/pmc_sq.py "$f" $KEYS > gpurun_out/pmc_sq_$tag.txt; cat gpurun_out/pmc_sq_$tag.txt
