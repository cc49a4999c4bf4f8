"""Pin the CPU oracle before trusting it (CPU only).

* Thermo/transport: against the reference's own fixture thermo_ES80_H2-7-16.txt and the
  mechanism file it was generated from (examples/dfLowMachFoam/notorch/threeD_reactingTGV/
  H2/cvodeIntegrator), plus textbook 300 K transport values.
* Finite volume: analytic invariants (the reference FV path has no golden outputs):
  exact Gauss gradients of linear fields, discrete conservation, symmetric laplacian.
"""
import numpy as np
import pytest

from conftest import rel_err


def test_thermo_table_nasa_matches_yaml_bitwise(es80):
    t, y = es80
    assert t.S == 7
    assert y["species"] == ["H", "O", "H2O", "OH", "O2", "H2", "N2"]
    assert np.array_equal(t.nasa, y["nasa"])                 # max rel diff 0.0
    assert np.allclose(t.W, [1.008, 15.999, 18.015, 17.007, 31.998, 2.016, 28.014])


def _pure_state(S, idx, T, p=101325.0):
    Y = np.zeros((S, 1)); Y[idx] = 1.0
    return Y


def test_transport_fits_reproduce_textbook_300K(es80):
    t, _ = es80
    sp = t.species
    lnT = np.log(300.0)
    poly = np.array([1, lnT, lnT ** 2, lnT ** 3, lnT ** 4])
    mu_h2 = (t.visc[sp.index("H2")] @ poly) ** 2 * np.sqrt(300.0)
    lam_n2 = (t.cond[sp.index("N2")] @ poly) * np.sqrt(300.0)
    d_h2n2 = (t.bdiff[sp.index("H2"), sp.index("N2")] @ poly) * 300.0 ** 1.5 / 101325.0
    assert abs(mu_h2 - 9.00e-6) / 9.00e-6 < 5e-3
    assert abs(lam_n2 - 0.02646) / 0.02646 < 5e-3
    assert abs(d_h2n2 - 7.79e-5) / 7.79e-5 < 5e-3


def test_oracle_thermo_pure_species_and_newton(es80):
    import oracle as O
    t, _ = es80
    L = O.lib()
    dp = O._dp
    L.orc_set_thermo(t.S, dp(np.ascontiguousarray(t.W)), dp(np.ascontiguousarray(t.nasa)), dp(np.ascontiguousarray(t.visc)),
                     dp(np.ascontiguousarray(t.cond)), dp(np.ascontiguousarray(t.bdiff)))
    n = 5
    S = t.S
    rng = np.random.default_rng(0)
    Y = rng.random((S, n)); Y /= Y.sum(axis=0)
    T = np.array([300.0, 600.0, 1000.0, 1500.0, 2400.0])
    p = np.full(n, 101325.0)
    he = np.zeros(n); psi = np.zeros(n); rho = np.zeros(n); mu = np.zeros(n); al = np.zeros(n)
    rhoD = np.zeros((S, n)); hai = np.zeros((S, n))
    L.orc_thermo_points(n, 1, dp(T), dp(he), dp(p), dp(Y), dp(psi), dp(rho), dp(mu), dp(al), dp(rhoD), dp(hai))
    # he = sum Y_i h_i
    assert rel_err(he, (Y * hai).sum(axis=0)) < 1e-13
    # ideal gas
    Wm = 1.0 / (Y / t.W[:, None]).sum(axis=0)
    assert rel_err(rho, p * Wm / (8314.46261815324 * T)) < 1e-14
    # Newton inversion recovers T from he
    T2 = T * 0.9
    L.orc_thermo_points(n, 0, dp(T2), dp(he), dp(p), dp(Y), dp(psi), dp(rho), dp(mu), dp(al), dp(rhoD), dp(hai))
    assert np.max(np.abs(T2 - T) / T) < 1e-7     # Newton rtol (dfThermo.H:89); T=1000 sits on the NASA7 range switch
    # pure species: Wilke mixture viscosity = species viscosity
    for i in range(S):
        Yp = np.zeros((S, 1)); Yp[i] = 1.0
        Tp = np.array([800.0]); hp = np.zeros(1); z = [np.zeros(1) for _ in range(5)]
        rD = np.zeros((S, 1)); ha = np.zeros((S, 1))
        L.orc_thermo_points(1, 1, dp(Tp), dp(hp), dp(np.array([101325.0])), dp(Yp), dp(z[0]), dp(z[1]), dp(z[2]),
                            dp(z[3]), dp(rD), dp(ha))
        lnT = np.log(800.0); poly = np.array([1, lnT, lnT ** 2, lnT ** 3, lnT ** 4])
        mu_i = (t.visc[i] @ poly) ** 2 * np.sqrt(800.0)
        assert abs(z[2][0] - mu_i) / mu_i < 1e-13
        assert rD[i, 0] == 0.0          # X_i = 1 -> rhoD_i = 0 (dfThermo.cu:232-235)


def _linear_box():
    from dfmi.mesh import hex_box
    return hex_box(5, 4, 3, lengths=(1.0, 0.8, 0.6), periodic=(False, False, False), gradings=(1.0, 1.5, 0.7))


def _oracle_for(m, t, state, types=None):
    import oracle as O
    from dfmi.case import default_patch_types
    from dfmi.mesh import FIXED_VALUE
    pt = default_patch_types(m)
    if types:
        pt.update(types)
    return O.Oracle(m, t, state, pt, inert=t.S - 1, rdt=1e6)


def test_oracle_gauss_gradient_exact_for_linear_field(es80):
    from dfmi.mesh import FIXED_VALUE
    t, _ = es80
    m = _linear_box()
    cc = m.cell_centres
    a = np.array([1.5, -2.0, 0.75])
    f = 3.0 + cc @ a
    # fixedValue walls carrying the exact face values
    bsf, _, _, _, bfc = m.boundary_arrays()
    # boundary face centres: cell centre + distance along the normal
    off = 0
    bval = np.zeros(m.n_boundary_slots)
    for p in m.patches:
        n = p.size
        nrm = p.sf / p.mag_sf[:, None]
        fcen = cc[p.face_cells] + nrm * (1.0 / p.delta_coeffs)[:, None]
        bval[off:off + n] = 3.0 + fcen @ a
        off += n
    st = {"phi_field": f, "boundary_phi_field": bval, "gout": np.zeros(3 * m.n_cells), "bgout": np.zeros(3 * m.n_boundary_slots)}
    o = _oracle_for(m, t, st, {"T": m.patch_types(FIXED_VALUE)})
    o._run("orc_grad_scalar", b"phi_field", b"boundary_phi_field", b"ptype_T", b"gout", b"bgout")
    g = o["gout"].reshape(3, -1)
    assert np.allclose(g, a[:, None], rtol=0, atol=1e-12)


def test_oracle_rho_eqn_conserves_mass_periodic(es80):
    from dfmi.mesh import hex_box
    t, _ = es80
    m = hex_box(6, 5, 4, gradings=(1.0, 1.4, 1.0))
    rng = np.random.default_rng(1)
    C_, F, B = m.n_cells, m.n_faces, m.n_boundary_slots
    rho_old = 1.0 + 0.1 * rng.random(C_)
    phi = 1e-7 * rng.standard_normal(F)
    # consistent cyclic fluxes: partner slots carry opposite flux
    bphi = np.zeros(B)
    off = []
    o_ = 0
    for p in m.patches:
        off.append(o_); o_ += p.slots
    for pi, p in enumerate(m.patches):
        if pi < p.neighbour_patch:
            v = 1e-7 * rng.standard_normal(p.size)
            bphi[off[pi]:off[pi] + p.size] = v
            q = p.neighbour_patch
            bphi[off[q]:off[q] + p.size] = -v
    st = {"rho": np.zeros(C_), "rho_old": rho_old, "phi": phi, "boundary_phi": bphi, "boundary_rho": np.zeros(B)}
    o = _oracle_for(m, t, st)
    o.rho_eqn()
    mass0 = (rho_old * m.volume).sum()
    mass1 = (o["rho"] * m.volume).sum()
    assert abs(mass1 - mass0) / mass0 < 1e-14
