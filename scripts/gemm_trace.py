#!/usr/bin/env python3
"""Per-layer DNN GEMM durations from a rocprofv3 --kernel-trace CSV (scripts/gemm_trace.sh): dispatches of
k_mlp_gemm grouped by template variant and grid (each hidden layer has its own grid), with the layer's
algorithmic TFLOP/s for BASELINE config 4's nets [55, 1600, 800, 400, 1]. Usage: gemm_trace.py <trace dir>"""
import csv
import glob
import json
import os
import sys


def main(d):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    groups = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "k_mlp_gemm" not in name:
            continue
        var = ("pingpong" if "k_mlp_gemm_pp" in name else "wide" if "k_mlp_gemm_w" in name
               else "out" if "ILb1ELb1E" in name else "hidden")
        key = (var, int(r["Grid_Size_X"]) // int(r.get("Workgroup_Size_X") or 256), int(r["Grid_Size_Z"]))
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for (var, gx, gz), us in sorted(groups.items()):
        us = us[1:] if len(us) > 2 else us   # first dispatch of each shape warms the code object
        out.append({"variant": var, "blocks": gx, "nets": gz, "launches": len(us),
                    "avg_us": sum(us) / len(us), "min_us": min(us)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
