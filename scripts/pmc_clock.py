#!/usr/bin/env python3
"""Effective clock per dispatch from a GRBM_GUI_ACTIVE counter pass (MI355X_MICROARCH.md DVFS: the counter is summed
over the 8 XCDs, clock = GRBM_GUI_ACTIVE / 8 / kernel wall time), for the kernels whose name contains one of the given
substrings. A dispatch is 'alone' before the first dispatch of the --split kernel and 'in_loop' after it
(scripts/config4_profile.py both: surrogate alone, then the config-4 steps).
  python scripts/pmc_clock.py <counter_collection.csv> out.json --kernels k_mlp_gemm --split k_thermo_coop"""
import argparse
import collections
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("out")
    ap.add_argument("--kernels", nargs="+", default=["k_mlp_gemm"])
    ap.add_argument("--split", default="k_thermo_coop")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                     int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Grid_Size"]))
    rows.sort()
    split = next((d for d, k, _, _, _ in rows if a.split in k), None)
    out = collections.defaultdict(list)
    for d, k, v, ns, grid in rows:
        if not any(s in k for s in a.kernels) or ns <= 0:
            continue
        name = k.replace("void ", "").split("(")[0]
        arm = "alone" if split is None or d < split else "in_loop"
        out[f"{arm} {name} grid={grid}"].append({"dispatch": d, "us": ns / 1e3, "clock_ghz": v / 8.0 / ns})
    res = {}
    for key, lst in sorted(out.items()):
        res[key] = {"dispatches": len(lst), "median_us": statistics.median(x["us"] for x in lst),
                    "median_clock_ghz": statistics.median(x["clock_ghz"] for x in lst),
                    "per_dispatch": lst}
        print(f"{key:70s} n={len(lst):3d} median {res[key]['median_us']:9.1f} us  clock {res[key]['median_clock_ghz']:.3f} GHz")
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
