"""Per-kernel L2 behaviour from a rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
pass (scripts/pmc_l2.sh): hit rate, fabric read/write bytes per dispatch (RDREQ x 128 B: gfx950 tallies a
128-B read as one 64-B request unit, MI355X_MICROARCH.md HBM section; WRREQ x 64 B), L2 requests."""
import collections, csv, json, re, sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    if not m or int(r["Grid_Size"]) < int(sys.argv[2] if len(sys.argv) > 2 else 1000000):
        continue
    agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, v in sorted(agg.items()):
    mean = lambda c: sum(v[c]) / len(v[c]) if v[c] else 0.0
    hit, miss = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
    out[k] = {"dispatches": len(v["TCC_HIT_sum"]), "l2_hit": hit / max(hit + miss, 1.0),
              "fabric_read_bytes": mean("TCC_EA0_RDREQ_sum") * 128, "fabric_write_bytes": mean("TCC_EA0_WRREQ_sum") * 64,
              "l2_requests": hit + miss}
    print(f"{k:28s} n={out[k]['dispatches']:4d} hit={100 * out[k]['l2_hit']:5.1f}% rd={out[k]['fabric_read_bytes'] / 1e6:7.0f}MB "
          f"wr={out[k]['fabric_write_bytes'] / 1e6:6.0f}MB req={out[k]['l2_requests'] / 1e6:6.1f}M")
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
