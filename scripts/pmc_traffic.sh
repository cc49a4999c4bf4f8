#!/bin/bash
# HBM traffic per kernel from PMC counters (MI355X_MICROARCH.md HBM section): FETCH_SIZE and
# WRITE_SIZE in separate passes (they do not fit one TCC pass), counters only (no tracing domains),
# on the headline bench workload; summary -> gpurun_out/pmc_traffic.json (copy to profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-flame ${BENCH_ARGS} > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
f=$(find gpurun_out/pmc_FETCH_SIZE -name "*counter_collection.csv" | sort | tail -1)
w=$(find gpurun_out/pmc_WRITE_SIZE -name "*counter_collection.csv" | sort | tail -1)
python3 scripts/pmc_summary.py "$f" "$w" gpurun_out/pmc_traffic.json
