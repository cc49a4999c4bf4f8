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
