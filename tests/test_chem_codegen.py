"""The generated mechanism code (csrc/chem_gen_*.inc) is current: regenerating it from the
mechanism files reproduces the committed files byte for byte, and the fingerprint the runtime
compares is the one of the shipped thermo tables."""
import os

import pytest

from conftest import GOLDEN, ROOT

CASES = [("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt", "burke9"),
         ("ES80_H2-7-16.yaml", "thermo_ES80_H2-7-16.txt", "es80")]


@pytest.mark.parametrize("yml,table,name", CASES)
def test_generated_code_is_current(yml, table, name):
    from dfmi.chem_codegen import generate
    from dfmi.kinetics import parse_mechanism
    from dfmi.mech import read_yaml_mechanism
    path = os.path.join(GOLDEN, yml)
    ym = read_yaml_mechanism(path)
    code = generate(parse_mechanism(path), ym["nasa"], ym["W"], name)
    with open(os.path.join(ROOT, "deepflame-dev_amd", "csrc", f"chem_gen_{name}.inc")) as f:
        assert f.read() == code


def test_burke_fingerprint_matches_shipped_table():
    from dfmi.chem_codegen import fingerprint
    from dfmi.kinetics import parse_mechanism
    from dfmi.mech import read_yaml_mechanism, read_thermo_table
    path = os.path.join(GOLDEN, "Burke2012_s9r23.yaml")
    ym = read_yaml_mechanism(path)
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), ym["species"])
    m = parse_mechanism(path)
    assert fingerprint(m, t.nasa, t.W) == fingerprint(m, ym["nasa"], ym["W"])


def test_generated_rate_constants_match_oracle(tmp_path):
    """The generated consts() (compiled on the host with g++, the CPU-A build's macros) against the oracle's
    Kinetics.rate_constants: forward k_f, reverse k_f / K_c (per-species exp(g/RT) products above the generator's
    floor temperature, the per-reaction exponential below it), the fall-off low-pressure limits and log10 Fc."""
    import subprocess
    import numpy as np
    from chem_oracle import Kinetics
    from dfmi.kinetics import parse_mechanism
    from dfmi.mech import read_yaml_mechanism
    path = os.path.join(GOLDEN, "Burke2012_s9r23.yaml")
    ym = read_yaml_mechanism(path)
    mech = parse_mechanism(path)
    src = tmp_path / "k.cpp"
    inc = os.path.join(ROOT, "deepflame-dev_amd", "csrc", "chem_gen_burke9.inc")
    src.write_text('#include <cmath>\n#include <cstdio>\n#include <cstdlib>\n#define DFMI_HD\n#define DFMI_SCHED_FENCE()\n'
                   '#define DFMI_CONTRACT() do {} while (0)\n#define DFMI_RCP(x) (1.0 / (x))\n'
                   f'#include "{inc}"\n'
                   'int main(int argc, char** argv) {\n  for (int a = 1; a < argc; ++a) {\n'
                   '    double k[ChemGen_burke9::NK]; ChemGen_burke9::consts(std::atof(argv[a]), k);\n'
                   '    for (int i = 0; i < ChemGen_burke9::NK; ++i) std::printf("%.17g ", k[i]);\n'
                   '    std::printf("\\n");\n  }\n}\n')
    exe = tmp_path / "k"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(src)], check=True)
    Ts = [90.0, 200.0, 300.0, 610.0, 999.0, 1001.0, 1500.0, 2200.0, 3000.0]
    out = subprocess.run([str(exe)] + [repr(t) for t in Ts], check=True, capture_output=True, text=True).stdout
    kin = Kinetics(mech, ym["nasa"], ym["W"])
    R = mech.R
    fo = [r for r in range(R) if mech.itype[r] >= 2]
    troe = [r for r in range(R) if mech.itype[r] == 3]
    for T, line in zip(Ts, out.strip().split("\n")):
        k = np.array([float(v) for v in line.split()])
        kf, k0, Kc = kin.rate_constants(T)
        kr = np.where(mech.reversible, kf / Kc, 0.0)
        assert np.allclose(k[:R], kf, rtol=1e-13, atol=0), T
        assert np.allclose(k[R:2 * R], kr, rtol=1e-12, atol=0), (T, np.max(np.abs(k[R:2 * R] / np.where(kr == 0, 1, kr) - 1)))
        assert np.allclose(k[2 * R:2 * R + len(fo)], k0[fo], rtol=1e-13, atol=0), T
        for i, r in enumerate(troe):
            a, T3, T1, _ = mech.troe[r]
            Fc = (1 - a) * np.exp(-T / T3) + a * np.exp(-T / T1)
            assert abs(k[2 * R + len(fo) + i] - np.log10(Fc)) <= 1e-15, T
