#!/bin/bash
# PMC pass over the DNN GEMM kernels of the config-4 profile workload (one counter set per run).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex mlp_gemm --output-format csv -d $R/gpurun_out/pmcg$i -o run -- python3 $R/scripts/config4_profile.py > $R/gpurun_out/pmcg$i.log 2>&1 || exit $?
  python3 - $R/gpurun_out/pmcg$i <<'PY'
import csv, glob, os, sys, collections
f = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]; acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
done
