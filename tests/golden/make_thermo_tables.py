#!/usr/bin/env python3
"""Regenerate the thermo/transport tables the tests and bench use that the reference does not ship:
thermo_Burke2012_s9r23.txt from Burke2012_s9r23.yaml (reference test/Tu500K-Phi1/) with
dfmi.transport_fit (a restatement of Cantera 2.6 GasTransport::fitProperties), and the synthetic
53-species table of BASELINE config 4 (the 36 gri30 species of the reference's
mechanisms/CH4/gri30.yaml fitted the same way, cycled to 53, N2 last) -- thermo_gri53_synthetic.txt."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "deepflame-dev_amd"))
from dfmi.transport_fit import main  # noqa: E402
from dfmi.mech import write_thermo_table  # noqa: E402
from dfmi.synthetic import gri53_table  # noqa: E402

if __name__ == "__main__":
    rc = main([os.path.join(HERE, "Burke2012_s9r23.yaml"), os.path.join(HERE, "thermo_Burke2012_s9r23.txt")])
    write_thermo_table(os.path.join(HERE, "thermo_gri53_synthetic.txt"), gri53_table(os.path.join(HERE, "gri30.yaml")))
    sys.exit(rc)
