#!/bin/bash
# Decomposed-AMG A/B: p-iterations per solve and ms/step for 1/2/4/8 in-process ranks of ${N:-64}^3 (weak,
# the bench's layout) with the opt-in variants: the agglomerated coarsest level (DFMI_AMG_GLOBAL) and level 0
# smoothed with its processor couplings (DFMI_AMG_HALO_L0). VARS: space-separated "name:ENV=V,ENV=V" items.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-base: halo:DFMI_AMG_HALO_L0=1 global:DFMI_AMG_GLOBAL=1}; do
  name="${v%%:*}"; envs="${v#*:}"
  ( for e in $(echo "$envs" | tr ',' ' '); do export "$e"; done
    timeout -k 10 300 python scripts/amg_decomp_study.py ${N:-64} ${STEPS:-3} weak > gpurun_out/amg_ab_$name.jsonl 2> gpurun_out/amg_ab_$name.err )
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json,sys
for l in open('gpurun_out/amg_ab_$name.jsonl'):
    d=json.loads(l); print(d['ranks'], d['p_iters_last_solve'], round(d['ms_per_step'],2), d['amg_levels'][-2:])
"; [ $rc -eq 0 ] || exit $rc
done
