#!/bin/bash
# Decomposed-AMG A/B: p-iterations per solve with and without the agglomerated coarsest level
# (Amg::global, DFMI_AMG_GLOBAL) for 1/2/4/8 in-process ranks of 64^3 (weak, the bench's layout).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in 1 0; do
  DFMI_AMG_GLOBAL=$g timeout -k 10 300 python scripts/amg_decomp_study.py ${N:-64} ${STEPS:-3} weak > gpurun_out/amg_global_$g.jsonl 2> gpurun_out/amg_global_$g.err
  rc=$?; echo "global=$g rc=$rc"; cat gpurun_out/amg_global_$g.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
