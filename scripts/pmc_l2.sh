#!/bin/bash
# L2 behaviour of the assembly kernels for one cell order: hits, misses, fabric reads/writes per dispatch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-bricks}
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d gpurun_out/pmcl2_$tag -o run -- python3 bench.py --steps 1 --warmup 1 --roof-steps 1 --no-cpu --no-flame --renumber $tag > gpurun_out/pmcl2_$tag.log 2>&1
