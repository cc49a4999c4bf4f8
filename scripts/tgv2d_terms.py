#!/usr/bin/env python3
"""Term-by-term sensitivity of the 2D reacting-TGV regression (test/corrtest.cpp:52-56) on CPU-A.

Each variant reruns scripts/tgv2d_regression.py --lib cpu_a in its own process with one EEqn / pEqn term
dropped or scaled through CPU-A's study knobs (baseline/cpu_a/cpu_a.cpp DFMI_CPUA_STUDY): diffAlphaD,
fvc::div(hDiffCorrFlux), dpdt (EEqn.H:12-45; pEqn.H:121-128), the ddtCorr flux (pEqn.H:21-25). The table
gives, per corrtest step, the sampled T and its deviation from the reference value, and the shift each
variant causes against the baseline run -- which term (if any) carries the +0.3 % mid-ignition residual.

  python scripts/tgv2d_terms.py [--out profiles/r04_tgv2d_terms.json] [--variants base,no_dpdt,...]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = {"base": "", "no_diffAlphaD": "no_diffAlphaD", "no_hDiffCorrFlux": "no_hDiffCorrFlux",
            "no_dpdt": "no_dpdt", "ddtcorr_0": "ddtcorr=0", "ddtcorr_2": "ddtcorr=2",
            "no_dAD_no_hdcf": "no_diffAlphaD,no_hDiffCorrFlux",
            # +1 % on one term: the sensitivity a small implementation difference in it would have
            "dAD_1.01": "dAD=1.01", "hdcf_1.01": "hdcf=1.01", "dpdt_1.01": "dpdt=1.01"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04_tgv2d_terms.json"))
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--extra", default="", help="extra arguments of tgv2d_regression.py")
    a = ap.parse_args()
    res = {}
    if os.path.exists(a.out):
        res = json.load(open(a.out)).get("runs", {})
    for v in a.variants.split(","):
        env = dict(os.environ, DFMI_CPUA_STUDY=VARIANTS.get(v, v))
        tmp = os.path.join("/tmp", f"tgv2d_{v}.json")
        cmd = [sys.executable, os.path.join(ROOT, "scripts", "tgv2d_regression.py"), "--lib", "cpu_a", "--out", tmp]
        cmd += a.extra.split() if a.extra else []
        print("running", v, flush=True)
        subprocess.run(cmd, env=env, check=True, stdout=subprocess.DEVNULL)
        res[v] = json.load(open(tmp))
        print(v, {k: round(s["value"], 3) for k, s in res[v]["steps"].items()}, flush=True)
    table = {}
    base = res.get("base")
    for v, r in res.items():
        row = {}
        for k, s in r["steps"].items():
            row[k] = {"T": s["value"], "dev_vs_reference_pct": 100.0 * (s["value"] - s["expected"]) / s["expected"]}
            if base:
                row[k]["shift_vs_base_pct"] = 100.0 * (s["value"] - base["steps"][k]["value"]) / base["steps"][k]["value"]
        table[v] = row
    json.dump({"case": "test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver", "lib": "cpu_a", "table": table,
               "runs": res}, open(a.out, "w"), indent=1)
    for v, row in table.items():
        print(f"{v:18s}", "  ".join(f"{k}: {r['dev_vs_reference_pct']:+.3f}%" for k, r in row.items()))


if __name__ == "__main__":
    main()
