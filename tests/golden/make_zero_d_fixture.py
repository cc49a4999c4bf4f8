#!/usr/bin/env python3
"""BASELINE config 1 fixture: the reference df0DFoam case examples/df0DFoam/zeroD_cubicReactor/H2/
cvodeIntegrator (0/ fields: T = 1000 K, p = 101325 Pa, Y_H2/O2/N2; ES80_H2-7-16; dt 1e-6, endTime 1e-3
-> 1000 steps; constantProperty pressure) -> zeroD_cubicReactor.json: the initial state read from
the reference's 0/ files, plus the oracle trajectory (oracle.zero_d_trajectory: SciPy BDF at
rtol 1e-14 / atol 1e-25 -- the case's own odeCoeffs are relTol 1e-15 / absTol 1e-24 -- and the
oracle thermo) at every step. Run in the development container (needs /root/reference)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
CASE = "/root/reference/examples/df0DFoam/zeroD_cubicReactor/H2/cvodeIntegrator/0"


def main():
    from dfmi.foam_io import read_field
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from chem_oracle import Kinetics
    import oracle as O
    ym = read_yaml_mechanism(os.path.join(HERE, "ES80_H2-7-16.yaml"))
    sp = ym["species"]
    t = read_thermo_table(os.path.join(HERE, "thermo_ES80_H2-7-16.txt"), sp)
    vals = {}
    for name in ("T", "p", "H2", "O2", "N2"):
        v = np.atleast_1d(read_field(os.path.join(CASE, name + ".gz")))
        vals[name] = float(v[0])
    Y0 = np.zeros(len(sp))
    for name in ("H2", "O2", "N2"):
        Y0[sp.index(name)] = vals[name]
    kin = Kinetics(parse_mechanism(os.path.join(HERE, "ES80_H2-7-16.yaml")), ym["nasa"], ym["W"])
    n = int(os.environ.get("ZERO_D_STEPS", "1000"))
    T, Y = O.zero_d_trajectory(t, kin, vals["T"], vals["p"], Y0, 1e-6, n, rtol=1e-14, atol=1e-25, inert=sp.index("N2"))
    out = {"source": "reference examples/df0DFoam/zeroD_cubicReactor/H2/cvodeIntegrator (0/, system/controlDict, "
                     "constant/CanteraTorchProperties)",
           "mechanism": "ES80_H2-7-16.yaml", "species": sp, "T0": vals["T"], "p": vals["p"], "Y0": Y0.tolist(),
           "dt": 1e-6, "n_steps": n, "oracle": "oracle.zero_d_trajectory, SciPy BDF rtol 1e-14 atol 1e-25",
           "T": T.tolist(), "Y": Y.tolist()}
    with open(os.path.join(HERE, "zeroD_cubicReactor.json"), "w") as f:
        json.dump(out, f)
    print(f"T: {T[0]:.2f} -> {T[-1]:.2f} K over {n} steps")


if __name__ == "__main__":
    main()
