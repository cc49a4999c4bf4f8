"""The reference's own whole-loop regression, on the CPU (CPU-A = the oracle's assembly, OpenMP solvers,
ROS3 chemistry): test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver run for 500 steps with its own 0/
fields, fvSchemes (limitedLinear01 / limitedLinear / cubic), cyclic + empty patches, ES80 chemistry at
dfChemistryModel's default tolerances (relTol 1e-9, absTol 1e-15), T sampled with cellPoint on the
system/sample line, against the five values test/corrtest.cpp:52-56 asserts (read at :20-24).

Tolerance 0.5 % of the value. The reference's numbers come from OpenFOAM-7 + Cantera-2.6 on 4 MPI ranks
with GAMG / PBiCGStab at relTol 0.01; our solves are tight. Measured (profiles/r03_tgv2d_*.json): CPU-A
within 0.31 % at every point; the GPU path's upwind/linear schemes instead of the case's deviate 0.53 % at
t = 2e-4 s; loosening our solvers to 1e-2 moves the values by <= 0.06 %, the chemistry tolerance
(1e-6/1e-10 vs 1e-9/1e-15) by < 1e-5. Term-by-term attribution (profiles/r04_tgv2d_terms.json):
the residual's shape over the five samples matches a 0.5 % difference in the species-enthalpy diffusion terms
(diffAlphaD / hDiffCorrFlux) and no other term; no formula difference was found, so the 0.5 % stays.
"""
import json
import os

import pytest

from conftest import GOLDEN, ROOT

CPU_A = os.path.join(ROOT, "baseline", "cpu_a", "libdfmi_cpu_a.so")
TOL = 5e-3
# the 500-step rerun takes about 10 minutes of this container's 8 cores: opt-in (DFMI_REGRESSION=1, or
# scripts/tgv2d_regression.py, which wrote the committed run); the GPU test (test_gpu_regression.py)
# reruns the whole case on every round-end GPU pass and compares against the committed run
FULL = os.environ.get("DFMI_REGRESSION") == "1"


def test_committed_cpu_a_run_matches_reference_regression():
    """the committed CPU-A run (tests/golden/tgv2d_cpu_a.json) is within TOL of corrtest.cpp:52-56"""
    from dfmi.regression import TGV2D_EXPECTED
    d = json.load(open(os.path.join(GOLDEN, "tgv2d_cpu_a.json")))
    assert sorted(int(k) for k in d["steps"]) == sorted(TGV2D_EXPECTED)
    for step, (_, expected) in TGV2D_EXPECTED.items():
        r = d["steps"][str(step)]
        assert r["expected"] == expected
        assert abs(r["value"] - expected) / expected < TOL, (step, r["value"], expected)


@pytest.fixture(scope="module")
def cpu_a_run():
    from dfmi import regression as R
    if not FULL:
        pytest.skip("500-step CPU-A rerun: set DFMI_REGRESSION=1")
    if not os.path.exists(CPU_A):
        pytest.skip("CPU-A not built")
    return R.run_tgv2d(os.path.join(GOLDEN, "tgv2d"), GOLDEN, lib_path=CPU_A)


def test_tgv2d_cpu_matches_reference_regression(cpu_a_run):
    from dfmi.regression import TGV2D_EXPECTED
    assert sorted(cpu_a_run) == sorted(TGV2D_EXPECTED)
    for step, r in cpu_a_run.items():
        dev = abs(r["value"] - r["expected"]) / r["expected"]
        assert dev < TOL, (step, r["value"], r["expected"], dev)


def test_tgv2d_cpu_matches_committed_run(cpu_a_run):
    """the committed CPU-A values (tests/golden/tgv2d_cpu_a.json, scripts/tgv2d_regression.py) that the
    GPU test also compares against are what this build computes"""
    ref = json.load(open(os.path.join(GOLDEN, "tgv2d_cpu_a.json")))["steps"]
    for step, r in cpu_a_run.items():
        assert abs(r["value"] - ref[str(step)]["value"]) < 1e-6 * r["value"], step


def test_sampler_reproduces_point_interpolation_of_linear_field():
    """cellPoint interpolation is exact for a field linear in x and y (point values of a linear field
    are exact averages on the uniform 2D mesh, the tets interpolate linearly)"""
    import numpy as np
    from dfmi.regression import tgv2d_mesh
    from dfmi.sample import CellPointSampler
    m = tgv2d_mesh()
    cc = m.cell_centres
    f = 3.0 + 100.0 * cc[:, 0] - 50.0 * cc[:, 1]
    s = CellPointSampler(m, m.nodes, (True, True, False))
    for y in (0.00123, 0.0024144, 0.0031891):
        v = s.interpolate(f, (0.003, y, 0.003))
        assert abs(v - (3.0 + 100.0 * 0.003 - 50.0 * y)) < 1e-12
