"""Recompute the solver SpMV rooflines from committed profiles alone: a rocprofv3 --kernel-trace --stats
summary (scripts/prof_summary.py output) and the bench JSON line of the SAME profiled command, whose
"solver_work_run" holds the system-iterations of every solve in that process and the algorithmic bytes per
unit. k_bcg_spmv: 2 SpMVs (spmv1 + spmv2 launches) per BiCGStab system-iteration; k_bcg_eo (the even-odd form,
k_eo_a..d): 2 Schur-complement applications per system-iteration; k_cg_spmv: 1 per PCG iteration. Usage: python scripts/roof_from_profile.py profiles/r02_kernel_stats.csv profiles/r02_bench_prof.json
(profiles/r02_roof_from_profile.json is its output for the committed round-2 profile)"""
import csv
import json
import sys

PEAK = 8000.0   # GB/s, MI355X HBM3E


def main(stats_csv, bench_json):
    rows = [r for r in csv.reader(l for l in open(stats_csv) if not l.startswith("#"))]
    head, rows = rows[0], rows[1:]
    ms = {}
    for r in rows:
        if len(r) < len(head):
            continue
        d = dict(zip(head[:-1], r[:len(head) - 1]))
        name = ",".join(r[len(head) - 1:]).split("::")[-1]   # kernel names contain commas
        fam = ("k_bcg_spmv" if name.startswith("k_bcg_spmv") else "k_cg_spmv" if name.startswith("k_cg_spmv") else
               "k_bcg_eo" if name[:7] in ("k_eo_a<", "k_eo_b<", "k_eo_c<", "k_eo_d<") else None)
        if fam:
            ms[fam] = ms.get(fam, 0.0) + float(d["total_ms"])
    b = json.loads([l for l in open(bench_json) if l.strip().startswith("{")][-1])
    w = b["solver_work_run"]
    it = w["system_iterations"]
    units = {"k_bcg_spmv": 2.0 * (it["U"] + it["Y"] + it["E"]), "k_cg_spmv": it["p"]}
    units["k_bcg_eo"] = units["k_bcg_spmv"]   # even-odd: one Schur application (k_eo_a..d half passes) per SpMV
    bpu = dict(w["bytes_per_unit"])
    bpu.setdefault("k_bcg_eo", bpu["k_bcg_spmv"])   # bench.py algorithmic_bytes prices both forms alike
    out = {}
    for k, t in ms.items():
        total = bpu[k] * units[k]
        if k in ("k_bcg_spmv", "k_bcg_eo") and "u_matrix_bytes" in w:   # U's shared operator counts once per three systems
            total -= 2.0 * it["U"] * (2.0 / 3.0) * w["u_matrix_bytes"]
        gbs = total / (t / 1e3) / 1e9
        out[k] = {"units": units[k], "bytes_per_unit": bpu[k], "kernel_ms": t, "achieved_GBs": gbs,
                  "frac": gbs / PEAK}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
