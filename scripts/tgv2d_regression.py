#!/usr/bin/env python3
# (tests/golden/flame1d_speed_cpu_a.json is written by dfmi.regression.run_flame1d_speed on CPU-A, the same way)
"""Run the reference's 2D reacting-TGV regression (test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver,
tests/golden/tgv2d) through include/dfmi.h and print / save the values test/corrtest.cpp:51-56 asserts.

  python scripts/tgv2d_regression.py [--lib cpu_a|gpu] [--out file.json] [--schemes default|case]

--lib cpu_a runs the CPU-A baseline (the oracle's assembly, OpenMP); gpu the HIP library.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="gpu", choices=["gpu", "cpu_a"])
    ap.add_argument("--out")
    ap.add_argument("--schemes", default="case", choices=["case", "default"])
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--thermo", default="reference", choices=["reference", "fit"],
                    help="transport table: the reference's thermo_ES80_H2-7-16.txt, or fits regenerated from the YAML "
                         "by dfmi.transport_fit (what the reference CPU path's Cantera builds at run time)")
    a = ap.parse_args()
    from dfmi import regression as R
    from dfmi.schemes import DEFAULT
    golden = os.path.join(ROOT, "tests", "golden")
    lib = os.path.join(ROOT, "baseline", "cpu_a", "libdfmi_cpu_a.so") if a.lib == "cpu_a" else None
    kw = {} if a.schemes == "case" else {"schemes": dict(DEFAULT)}
    if a.thermo == "fit":
        import tempfile
        from dfmi.mech import read_yaml_mechanism, write_thermo_table
        from dfmi.transport_fit import fit_mechanism
        tab = os.path.join(tempfile.mkdtemp(), "thermo_ES80_fit.txt")
        write_thermo_table(tab, fit_mechanism(read_yaml_mechanism(os.path.join(golden, "ES80_H2-7-16.yaml"))))
        kw["thermo_table"] = tab
    t0 = time.time()
    out = R.run_tgv2d(os.path.join(golden, "tgv2d"), golden, steps=a.steps, lib_path=lib,
                      log=lambda s: print(f"[{time.time() - t0:6.1f}s] {s}", flush=True), **kw)
    res = {"case": "test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver", "lib": a.lib, "schemes": a.schemes,
           "thermo": a.thermo,
           "wall_s": time.time() - t0, "steps": {str(k): v for k, v in out.items()},
           "max_rel_dev": max(abs(v["value"] - v["expected"]) / v["expected"] for v in out.values())}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
