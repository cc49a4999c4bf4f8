#!/usr/bin/env python3
"""Per-kernel means of the counters of one rocprofv3 --pmc pass (counter_collection.csv):
  python scripts/pmc_sq.py <counter_collection.csv> [kernel substrings...]"""
import collections
import csv
import sys


def main(path, keys):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if keys and not any(k in name for k in keys):
            continue
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in sorted(agg.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
