#!/usr/bin/env python3
"""Per-kernel FP64 work from scripts/pmc_flops.sh's SQ pass (mean per dispatch):
  flops      = 64 x SQ_INSTS_VALU_FLOPS_FP64: the counter counts wave-instructions weighted by their FLOPs per lane
               (measured on gfx950: it equals ADD + MUL + TRANS + 2 FMA of the per-instruction counters exactly), so
               x 64 lanes = FLOPs with every lane active (an upper bound where lanes are masked)
  flops_inst = 64 (ADD + MUL + TRANS) + 128 FMA instructions (the same sum from the instruction counters)
  flops_steady = the mean over the LAST `steady` dispatches of the kernel (default 3 = the bench's roofline pass:
               the first solves of a run start every cell from dt and take several times the steady work, round 4's
               mean over all dispatches included them), with their per-dispatch values in dispatch order
  python scripts/pmc_flops_summary.py <counter_collection.csv> <out.json> [steady]"""
import collections
import csv
import json
import sys


def main(path, out, steady=3):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    order = collections.defaultdict(dict)   # kernel -> dispatch id -> FLOPS_FP64 counter
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "SQ_INSTS_VALU_FLOPS_FP64":
            order[name][int(r["Dispatch_Id"])] = 64.0 * float(r["Counter_Value"])
    res = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        g = lambda c: m.get(c, 0.0)
        res[k] = {"dispatches": n, **{c: m[c] for c in sorted(m)},
                  "flops": 64.0 * g("SQ_INSTS_VALU_FLOPS_FP64"),
                  "flops_inst": 64.0 * (g("SQ_INSTS_VALU_ADD_F64") + g("SQ_INSTS_VALU_MUL_F64") + g("SQ_INSTS_VALU_TRANS_F64"))
                  + 128.0 * g("SQ_INSTS_VALU_FMA_F64")}
        seq = [order[k][d] for d in sorted(order[k])]
        if seq:
            tail = seq[-steady:]
            res[k].update({"flops_per_dispatch": seq, "flops_steady": sum(tail) / len(tail), "steady_dispatches": len(tail)})
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["flops"])[:12]:
        print(f"{v['flops'] / 1e9:10.2f} GFLOP/dispatch mean, {v.get('flops_steady', 0) / 1e9:10.2f} steady "
              f"({v['flops_inst'] / 1e9:8.2f} by instructions)  {k}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:4]))
