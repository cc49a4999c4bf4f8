#!/bin/bash
# HBM traffic per kernel from PMC counters (MI355X_MICROARCH.md HBM section): FETCH_SIZE and
# WRITE_SIZE in separate passes (they do not fit one TCC pass), --kernel-trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --chem off > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find gpurun_out/pmc_* -name "*.csv" | head
