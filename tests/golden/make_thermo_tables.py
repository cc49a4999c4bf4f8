#!/usr/bin/env python3
"""Regenerate the thermo/transport tables the tests and bench use that the reference does not ship:
thermo_Burke2012_s9r23.txt from Burke2012_s9r23.yaml (reference test/Tu500K-Phi1/) with
dfmi.transport_fit (a restatement of Cantera 2.6 GasTransport::fitProperties)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "deepflame-dev_amd"))
from dfmi.transport_fit import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main([os.path.join(HERE, "Burke2012_s9r23.yaml"), os.path.join(HERE, "thermo_Burke2012_s9r23.txt")]))
