"""BASELINE config 4 (2M cells x 53 species, DNN source) alone, for a rocprofv3 kernel trace or PMC pass.
  python scripts/config4_profile.py [n] [both]
both: the 53-species surrogate alone first (bench.dnn53_line, the same GEMM shapes outside the time step), then the
config-4 steps, so one counter pass holds both arms of the in-loop vs alone GEMM comparison (scripts/pmc_clock.py)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from dfmi.mesh import hex_box  # noqa: E402
from dfmi.mech import read_yaml_mechanism  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
m = hex_box(n, n, n, lengths=(2 * np.pi * 1e-3,) * 3)
ym = read_yaml_mechanism(os.path.join(ROOT, "tests", "golden", bench.MECHS["burke9"][0]))
f = bench.reference_fields(m, ym["species"])
if "both" in sys.argv[2:]:
    print(bench.dnn53_line(m, f["T"], f["p"]), flush=True)
print(bench.config4_line(m, f["T"], f["U"], f["p"], steps=2, warmup=1), flush=True)
