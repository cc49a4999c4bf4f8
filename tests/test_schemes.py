"""Convection / interpolation schemes of the reference cases (CPU: the oracle's restatement).

The reference's dfLowMachFoam cases select div(phi,Yi_h) Gauss limitedLinear01 1 (a multivariate
scheme over every Y_i and he, YEqn.H:6-14 / createFields.H:118-129), div(phi,K) Gauss limitedLinear 1 and
div(hDiffCorrFlux) Gauss cubic (test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver/system/fvSchemes:32-40).
The oracle's restatement (oracle/df_oracle.cpp, OpenFOAM-7 LimitedScheme / Limited01 / NVDTVD /
multivariateScheme / cubic) is checked here against:
  * an independent vectorised numpy statement of the same OpenFOAM formulas (smooth fields, walls and
    cyclic patches) -- to 1e-12 (numpy sums the gradients in another order);
  * exactness invariants: the limiter of a linear field is 1 (limitedLinear = linear); limitedLinear01
    over a table holding a field outside [0, 1] is upwind wherever that field leaves the bounds; cubic
    interpolation of a quadratic on a uniform mesh is exact on faces whose cells have exact gradients.
"""
import numpy as np
import pytest

from conftest import rel_err


def test_scheme_parser():
    from dfmi.schemes import parse, scheme_codes, read_fv_schemes, LIMITED_LINEAR01, CUBIC, LIMITED_LINEAR
    assert parse("div(phi,Yi_h)", "Gauss limitedLinear01 1") == (LIMITED_LINEAR01, 1.0)
    assert parse("div(phi,K)", "limitedLinear 0.5") == (LIMITED_LINEAR, 0.5)
    assert parse("div(hDiffCorrFlux)", "Gauss cubic") == (CUBIC, 1.0)
    for bad in [("div(phi,h)", "linear"), ("div(phi,U)", "cubic"), ("div(phi,Yi_h)", "cubic"), ("div(phi,K)", "limitedLinear"),
                ("div(phi,K)", "limitedLinear 2"), ("div(hDiffCorrFlux)", "upwind")]:
        with pytest.raises(ValueError):
            parse(*bad)
    assert scheme_codes({}) == ([0, 1, 1, 1], [1.0, 1.0, 1.0])
    assert scheme_codes({"div(phi,U)": "Gauss limitedLinearV 1"}) == ([0, 1, 1, 5], [1.0, 1.0, 1.0])
    import os
    from conftest import GOLDEN
    got = read_fv_schemes(os.path.join(GOLDEN, "tgv2d", "fvSchemes"))
    assert got == {"div(phi,Yi_h)": "Gauss limitedLinear01 1", "div(phi,K)": "Gauss limitedLinear 1",
                   "div(hDiffCorrFlux)": "Gauss cubic", "div(phi,U)": "Gauss linear"}


def _box(periodic):
    from dfmi.mesh import hex_box
    return hex_box(6, 5, 4, lengths=(1.0, 0.8, 0.6), periodic=(periodic,) * 3, gradings=(1.0, 1.5, 0.7))


def _oracle(m, t, st, schemes, types=None):
    import oracle as O
    from dfmi.case import default_patch_types
    pt = default_patch_types(m)
    if types:
        pt.update(types)
    return O.Oracle(m, t, st, pt, inert=t.S - 1, rdt=1e6, schemes=schemes)


def _slot_partner(m):
    """per boundary slot: (cell, partner cell or -1, coupled)"""
    bfc = m.boundary_arrays()[4]
    part = -np.ones(m.n_boundary_slots, np.int64)
    offs, o = [], 0
    for p in m.patches:
        offs.append(o); o += p.slots
    for pi, p in enumerate(m.patches):
        if p.kind == "cyclic":
            q = p.neighbour_patch
            part[offs[pi]:offs[pi] + p.size] = bfc[offs[q]:offs[q] + p.size]
    return bfc.astype(np.int64), part


def _np_grad(m, v, bv):
    """Gauss linear gradient [3, C] (the order differs from the oracle's; compared to 1e-12)"""
    C = m.n_cells
    own, nei, w = m.owner, m.neighbour, m.weight
    fv = w * (v[own] - v[nei]) + v[nei]
    g = np.zeros((3, C))
    for k in range(3):
        np.add.at(g[k], own, m.sf[:, k] * fv)
        np.add.at(g[k], nei, -m.sf[:, k] * fv)
    bsf, _, _, bw, bfc = m.boundary_arrays()
    bfc, part = _slot_partner(m)
    bface = np.where(part >= 0, bw * v[bfc] + (1 - bw) * v[np.maximum(part, 0)], bv)
    for k in range(3):
        np.add.at(g[k], bfc, bsf[:, k] * bface)
    return g / m.volume


def _np_limiter(twoByk, b01, flux, vP, vN, gP, gN, d):
    lim = np.ones_like(flux)
    if b01:
        out = ((flux > 0) & ((vP < 0) | (vN > 1))) | ((flux < 0) & ((vN < 0) | (vP > 1)))
    else:
        out = np.zeros(flux.shape, bool)
    gradf = vN - vP
    g = np.where(flux[None, :] > 0, gP, gN)
    gradcf = (d * g).sum(axis=0)
    sg = lambda x: np.where(x >= 0, 1.0, -1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(np.abs(gradcf) >= 1000 * np.abs(gradf), 2 * 1000 * sg(gradcf) * sg(gradf) - 1, 2 * (gradcf / gradf) - 1)
    lim = np.maximum(np.minimum(twoByk * r, 1.0), 0.0)
    return np.where(out, 0.0, lim)


def _np_weights(m, fields, flux, bflux, b01, k=1.0):
    """(multivariate) limited weights [F], coupled slots [B] by the OpenFOAM formulas"""
    own, nei = m.owner, m.neighbour
    d = m.mesh_distance.T
    lims, blims = [], []
    bfc, part = _slot_partner(m)
    bd = m.boundary_delta().T
    for v, bv in fields:
        g = _np_grad(m, v, bv)
        lims.append(_np_limiter(2.0 / k, b01, flux, v[own], v[nei], g[:, own], g[:, nei], d))
        cp = part >= 0
        bl = np.ones(m.n_boundary_slots)
        bl[cp] = _np_limiter(2.0 / k, b01, bflux[cp], v[bfc[cp]], v[part[cp]], g[:, bfc[cp]], g[:, part[cp]], bd[:, cp])
        blims.append(bl)
    lim = np.min(lims, axis=0)
    blim = np.min(blims, axis=0)
    pos0 = lambda x: (x >= 0).astype(np.float64)
    return lim * m.weight + (1 - lim) * pos0(flux), blim * m.boundary_arrays()[3] + (1 - blim) * pos0(bflux)


def _state(m, t, rng, he_scale=1.0):
    """smooth fields (limiters mostly 1, limited where the waves turn), random-sign fluxes"""
    C, F, B, S = m.n_cells, m.n_faces, m.n_boundary_slots, t.S
    x = m.cell_centres / m.cell_centres.max(axis=0)
    base = rng.dirichlet(np.ones(S))
    ph = rng.uniform(0, 2 * np.pi, (S, 3))
    Y = base[:, None] * (1 + 0.3 * np.sin(2 * np.pi * x[:, 0] + ph[:, 0:1]) * np.cos(2 * np.pi * x[:, 1] + ph[:, 1:2]))
    Y /= Y.sum(axis=0)
    from dfmi.case import boundary_values
    he = he_scale * (0.5 + 0.3 * np.sin(2 * np.pi * x[:, 2] + 1.0) * np.cos(2 * np.pi * x[:, 0]))
    st = {"Y": Y, "boundary_Y": boundary_values(m, Y), "he": he, "boundary_he": boundary_values(m, he),
          "phi": rng.standard_normal(F), "boundary_phi": rng.standard_normal(B)}
    K = rng.uniform(0, 8, C)
    st["K"] = K
    st["boundary_K"] = boundary_values(m, K)
    return st


@pytest.mark.parametrize("periodic", [True, False])
@pytest.mark.parametrize("kind", ["limitedLinear01 1", "limitedLinear 1", "limitedLinear 0.5"])
def test_multivariate_weights_match_openfoam_formulas(es80, periodic, kind):
    t, _ = es80
    m = _box(periodic)
    rng = np.random.default_rng(3)
    st = _state(m, t, rng)
    o = _oracle(m, t, {k: v.copy() for k, v in st.items()}, {"div(phi,Yi_h)": kind})
    o._run("orc_conv_weights")
    k = float(kind.split()[1])
    fields = [(st["Y"][s], st["boundary_Y"][s]) for s in range(t.S)] + [(st["he"], st["boundary_he"])]
    w, bw = _np_weights(m, fields, st["phi"], st["boundary_phi"], kind.startswith("limitedLinear01"), k)
    assert rel_err(o["conv_w"], w) < 1e-12
    bfc, part = _slot_partner(m)
    assert rel_err(o["boundary_conv_w"][part >= 0], bw[part >= 0]) < 1e-12
    # the weights lie between central and upwind
    up = (st["phi"] >= 0).astype(float)
    lo, hi = np.minimum(up, m.weight), np.maximum(up, m.weight)
    assert np.all(o["conv_w"] >= lo - 1e-15) and np.all(o["conv_w"] <= hi + 1e-15)
    assert 0 < np.mean(o["conv_w"] != up) < 1   # limited somewhere, not everywhere


def test_limited01_with_he_outside_bounds_is_upwind(es80):
    """he of a real mixture is far outside [0, 1] (J/kg), so Limited01 rejects it on every face and the
    multivariate minimum makes Y and he upwind -- what the reference cases actually run"""
    t, _ = es80
    m = _box(True)
    st = _state(m, t, np.random.default_rng(5), he_scale=1e5)
    o = _oracle(m, t, st, {"div(phi,Yi_h)": "limitedLinear01 1"})
    o._run("orc_conv_weights")
    assert np.array_equal(o["conv_w"], (st["phi"] >= 0).astype(float))


def test_limited_linear_of_linear_field_is_linear(es80):
    from dfmi.mesh import FIXED_VALUE
    t, _ = es80
    m = _box(False)
    a = np.array([1.5, -2.0, 0.75])
    K = 3.0 + m.cell_centres @ a
    bK = np.zeros(m.n_boundary_slots)
    off = 0
    for p in m.patches:
        n = p.size
        nrm = p.sf / p.mag_sf[:, None]
        bK[off:off + n] = 3.0 + (m.cell_centres[p.face_cells] + nrm / p.delta_coeffs[:, None]) @ a
        off += n
    rng = np.random.default_rng(2)
    st = {"K": K, "boundary_K": bK, "phi": rng.standard_normal(m.n_faces), "boundary_phi": np.zeros(m.n_boundary_slots),
          "out_K_w": np.zeros(m.n_faces), "out_boundary_K_w": np.zeros(m.n_boundary_slots)}
    o = _oracle(m, t, st, {"div(phi,K)": "limitedLinear 1"}, {"K": m.patch_types(FIXED_VALUE)})
    o._run("orc_k_weights")
    assert np.allclose(o["out_K_w"], m.weight, rtol=0, atol=1e-14)


def test_cubic_interpolation_exact_for_quadratic(es80):
    """uniform mesh, hD = (x^2, y^2, 0): linear face values carry +h^2/4, cubic's correction removes it
    on faces whose two cells have exact (central) Gauss gradients"""
    from dfmi.mesh import hex_box
    t, _ = es80
    n = 8
    m = hex_box(n, n, 3, lengths=(1.0, 1.0, 0.3), periodic=(False, False, True))
    cc = m.cell_centres
    hD = np.stack([cc[:, 0] ** 2, cc[:, 1] ** 2, np.zeros(m.n_cells)])
    bh = np.zeros((3, m.n_boundary_slots))
    from dfmi.case import boundary_values
    bh[...] = boundary_values(m, hD)
    off = 0
    for p in m.patches:   # exact wall values
        if p.kind == "wall":
            fcen = cc[p.face_cells] + p.sf / p.mag_sf[:, None] / p.delta_coeffs[:, None]
            bh[0, off:off + p.size] = fcen[:, 0] ** 2
            bh[1, off:off + p.size] = fcen[:, 1] ** 2
        off += p.slots
    st = {"hDiffCorrFlux": hD, "boundary_hDiffCorrFlux": bh, "out_cubic_flux": np.zeros(m.n_faces),
          "out_boundary_cubic_flux": np.zeros(m.n_boundary_slots)}
    o = _oracle(m, t, st, {"div(hDiffCorrFlux)": "cubic"})
    o._run("orc_cubic_flux")
    own, nei = m.owner, m.neighbour
    w = m.weight
    lin = sum(m.sf[:, k] * (w * (hD[k, own] - hD[k, nei]) + hD[k, nei]) for k in range(3))
    tot = lin + o["out_cubic_flux"]
    fc = 0.5 * (cc[own] + cc[nei])
    exact = m.sf[:, 0] * fc[:, 0] ** 2 + m.sf[:, 1] * fc[:, 1] ** 2
    ii, jj, _ = m.local_index
    inner = lambda c: (ii[c] > 0) & (ii[c] < n - 1) & (jj[c] > 0) & (jj[c] < n - 1)
    sel = inner(own) & inner(nei) & (np.abs(m.sf[:, 2]) == 0)
    assert sel.sum() > 20
    assert np.abs(tot[sel] - exact[sel]).max() < 1e-14 * np.abs(exact[sel]).max() * 10
    assert np.abs(lin[sel] - exact[sel]).max() > 1e-4 * np.abs(exact[sel]).max()   # linear alone is not exact


@pytest.mark.parametrize("periodic", [True, False])
def test_limited_linear_v_weights_match_openfoam_formulas(es80, periodic):
    """div(phi,U) Gauss limitedLinearV 1 (the 1D flame's, test/Tu500K-Phi1/system/fvSchemes): NVDVTVDV::r
    from (U_N - U_P) . (d & grad(U)_upwind) over |U_N - U_P|^2"""
    t, _ = es80
    m = _box(periodic)
    rng = np.random.default_rng(11)
    x = m.cell_centres / m.cell_centres.max(axis=0)
    U = np.stack([np.sin(2 * np.pi * x[:, 0] + a) * np.cos(2 * np.pi * x[:, 1]) for a in (0.3, 1.1, 2.0)])
    from dfmi.case import boundary_values
    st = {"U": U, "boundary_U": boundary_values(m, U), "phi": rng.standard_normal(m.n_faces),
          "boundary_phi": rng.standard_normal(m.n_boundary_slots), "out_U_w": np.zeros(m.n_faces),
          "out_boundary_U_w": np.zeros(m.n_boundary_slots)}
    o = _oracle(m, t, st, {"div(phi,U)": "limitedLinearV 1"})
    o._run("orc_u_weights")
    # numpy: grad(U) per component, r = 2 (dU . (d & G)) / |dU|^2 - 1
    G = np.stack([_np_grad(m, U[j], st["boundary_U"][j]) for j in range(3)], axis=1)   # [i dir][j comp][C]
    own, nei = m.owner, m.neighbour
    up = np.where(st["phi"] > 0, own, nei)
    d = m.mesh_distance.T
    dU = U[:, nei] - U[:, own]
    gradf = (dU * dU).sum(axis=0)
    dG = np.einsum("if,ijf->jf", d, G[:, :, up])
    gradcf = (dU * dG).sum(axis=0)
    sg = lambda v: np.where(v >= 0, 1.0, -1.0)
    r = np.where(np.abs(gradcf) >= 1000 * np.abs(gradf), 2 * 1000 * sg(gradcf) * sg(gradf) - 1, 2 * gradcf / gradf - 1)
    lim = np.clip(2 * r, 0, 1)
    w = lim * m.weight + (1 - lim) * (st["phi"] >= 0)
    assert rel_err(o["out_U_w"], w) < 1e-12
    assert 0 < np.mean(np.abs(o["out_U_w"] - m.weight) > 1e-12) < 1
