"""Python driver of the CPU oracle (TEST INFRASTRUCTURE -- never the product path).

Loads oracle/_build/liboracle.so (oracle/df_oracle.cpp, the sequential OpenFOAM-style
restatement) and completes it with exact sparse direct solves (scipy.sparse.linalg.spsolve)
where the reference solves linear systems, so the oracle's fields after a step are the exact
solutions of the assembled equations. See df_oracle.cpp's header for the parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

ZG, FV, EMPTY, CYCLIC, PROC, PROC_CYC = 0, 1, 3, 6, 7, 10


def build():
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.orc_set_d.argtypes = [C.c_char_p, C.POINTER(C.c_double)]
        _lib.orc_set_i.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
        _lib.orc_thermo_correct.argtypes = [C.c_int]
        _lib.orc_correct_bc.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        _lib.orc_grad_scalar.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p]
        _lib.orc_last_error.argtypes = [C.c_char_p, C.c_int]
        dp = C.POINTER(C.c_double)
        _lib.orc_set_thermo.argtypes = [C.c_int, dp, dp, dp, dp, dp]
        _lib.orc_thermo_points.argtypes = [C.c_int, C.c_int, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp]
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Oracle:
    """Holds contiguous copies of every array the restatement reads or writes."""

    def __init__(self, mesh, table, state: dict, ptypes: dict, inert: int, rdt: float, schemes: dict | None = None):
        """schemes: {fvSchemes divSchemes key: scheme} for the terms the reference GPU path hard-wires
        (dfmi.schemes.TERMS; default upwind / linear / linear), e.g. the reference cases'
        {"div(phi,Yi_h)": "limitedLinear01 1", "div(phi,K)": "limitedLinear 1", "div(hDiffCorrFlux)": "cubic"}"""
        from dfmi.case import patch_kind
        from dfmi.schemes import scheme_codes
        self.m = mesh
        self.S = table.S
        self.L = lib()
        self.L.orc_clear()
        self.arr = {}
        self.iarr = {}
        m = mesh
        bsf, bmag, bdc, bw, bfc = m.boundary_arrays()
        self._i("dims", [m.n_cells, m.n_faces, m.n_boundary_slots, m.n_patches, table.S])
        self._i("owner", m.owner); self._i("neighbour", m.neighbour); self._i("patch_size", m.patch_sizes)
        self._i("cyclic_neighbor", m.cyclic_neighbour()); self._i("boundary_face_cell", bfc if bfc.size else [0])
        self._i("patch_kind", patch_kind(m)); self._i("inert_index", [inert])
        for k, v in ptypes.items():
            self._i("ptype_" + k, v)
        self._d("sf", m.sf.T.copy()); self._d("mag_sf", m.mag_sf); self._d("weight", m.weight)
        self._d("delta_coeffs", m.delta_coeffs); self._d("volume", m.volume)
        self._d("boundary_sf", bsf.T.copy() if bsf.size else np.zeros(3)); self._d("boundary_mag_sf", bmag)
        self._d("boundary_weight", bw); self._d("boundary_delta_coeffs", bdc)
        self._d("rdelta_t", [rdt])
        self._d("mesh_distance", np.asarray(m.mesh_distance).T.copy() if m.n_faces else np.zeros(3))
        bd = m.boundary_delta()
        self._d("boundary_delta", bd.T.copy() if bd.size else np.zeros(3))
        codes, ks = scheme_codes(schemes or {})
        self._i("schemes", codes)
        self._d("scheme_k", ks)
        self._d("conv_w", np.zeros(max(m.n_faces, 1)))
        self._d("boundary_conv_w", np.zeros(max(m.n_boundary_slots, 1)))
        self.rdt = rdt
        self.inert = inert
        self.ptypes = ptypes
        for k, v in state.items():
            self._d(k, v)
        if "boundary_heGradient" not in self.arr:
            self._d("boundary_heGradient", np.zeros(m.n_boundary_slots))
        self.L.orc_set_thermo(table.S, _dp(np.ascontiguousarray(table.W)), _dp(np.ascontiguousarray(table.nasa)),
                              _dp(np.ascontiguousarray(table.visc)), _dp(np.ascontiguousarray(table.cond)),
                              _dp(np.ascontiguousarray(table.bdiff)))
        self._kind = patch_kind(m)

    # ---- array registry
    def _d(self, name, a):
        a = np.ascontiguousarray(np.array(a, dtype=np.float64))
        self.arr[name] = a
        self.L.orc_set_d(name.encode(), _dp(a))
        return a

    def _i(self, name, a):
        a = np.ascontiguousarray(np.array(a, dtype=np.int32))
        self.iarr[name] = a
        self.L.orc_set_i(name.encode(), a.ctypes.data_as(C.POINTER(C.c_int)))
        return a

    def __getitem__(self, k):
        return self.arr[k]

    def set(self, k, v):
        if k in self.arr and self.arr[k].shape == np.shape(v):
            self.arr[k][...] = v
        else:
            self._d(k, v)

    def out(self, name, shape):
        return self._d(name, np.zeros(shape))

    def _run(self, fn, *args):
        rc = getattr(self.L, fn)(*args)
        if rc != 0:
            buf = C.create_string_buffer(2048)
            self.L.orc_last_error(buf, 2048)
            raise RuntimeError(f"{fn}: {buf.value.decode()}")

    # ---- stages
    def matrix_outputs(self, nsys_faces=1, nsrc=1, nb=1, extra=()):
        m = self.m
        C_, F, B = m.n_cells, m.n_faces, m.n_boundary_slots
        o = {"lower": self.out("out_lower", nsys_faces * F), "upper": self.out("out_upper", nsys_faces * F),
             "diag": self.out("out_diag", nsys_faces * C_), "source": self.out("out_source", nsrc * C_),
             "internal_coeffs": self.out("out_internal_coeffs", nb * B),
             "boundary_coeffs": self.out("out_boundary_coeffs", nb * B)}
        for e, n in extra:
            o[e] = self.out("out_" + e, n)
        return o

    def rho_eqn(self):
        C_ = self.m.n_cells
        self.out("out_rho_diag", C_); self.out("out_rho_source", C_)
        self._run("orc_rho_eqn")

    def u_assemble(self):
        m = self.m
        o = self.matrix_outputs(1, 3, 3, [("source_solve", 3 * m.n_cells), ("gradU", 9 * m.n_cells)])
        self._run("orc_u_assemble")
        for k in ("lower", "upper", "source", "internal_coeffs", "boundary_coeffs"):
            self.set("ueqn_" + k, o[k].copy())
        self.ueqn = {k: v.copy() for k, v in o.items()}
        return self.ueqn

    def u_hbya(self):
        self._run("orc_u_hbya")

    def p_assemble(self):
        m = self.m
        o = self.matrix_outputs(1, 1, 1, [("rhorAUf", m.n_faces), ("boundary_rhorAUf", m.n_boundary_slots),
                                          ("phiHbyA", m.n_faces), ("boundary_phiHbyA", m.n_boundary_slots)])
        self._run("orc_p_assemble")
        for k in ("lower", "upper", "internal_coeffs", "boundary_coeffs", "phiHbyA", "boundary_phiHbyA"):
            self.set("peqn_" + k, o[k].copy())
        self.peqn = {k: v.copy() for k, v in o.items()}
        return self.peqn

    def p_post(self):
        self._run("orc_p_post")

    def y_prep(self):
        m = self.m
        self.out("out_gradY", 3 * self.S * m.n_cells)
        for k in ("sumYDiffError", "hDiffCorrFlux"):
            self.set(k, np.zeros((3, m.n_cells)) if self.arr.get(k) is None else self.arr[k])
        self._run("orc_conv_weights")   # div(phi,Yi_h) weights from this step's Y, he, phi (YEqn.H:6-14)
        self._run("orc_y_prep")

    def y_assemble(self):
        S = self.S
        m = self.m
        o = self.matrix_outputs(S, S, S, [("phiUc", m.n_faces), ("boundary_phiUc", m.n_boundary_slots)])
        self._run("orc_y_assemble")
        self.yeqn = {k: v.copy() for k, v in o.items()}
        return self.yeqn

    def y_inert(self):
        self._run("orc_y_inert")

    def e_assemble(self, fresh_weights=False):
        """fresh_weights: recompute the div(phi,Yi_h) weights first (an EEqn inspected on its own); in
        the time step EEqn reuses the weights YEqn computed (EEqn.H's mvConvection)"""
        if fresh_weights:
            self._run("orc_conv_weights")
        o = self.matrix_outputs(1, 1, 1)
        self._run("orc_e_assemble")
        self.eeqn = {k: v.copy() for k, v in o.items()}
        return self.eeqn

    def energy_gradient(self):
        """boundary_heGradient on gradientEnergy slots (dfEEqn.cu:148, :266-287)"""
        self._run("orc_energy_gradient")

    def thermo_correct(self, from_T=False):
        self._run("orc_thermo_correct", 1 if from_T else 0)

    def correct_bc(self, field, ptype, ncomp):
        self._run("orc_correct_bc", field.encode(), ("boundary_" + field).encode(), ("ptype_" + ptype).encode(), ncomp)

    # ---- exact linear solves of the assembled LDU systems
    def _slot_info(self):
        m = self.m
        kinds = self._kind
        sp_ = []
        for pi, p in enumerate(m.patches):
            sp_ += [pi] * p.slots
        prim = []
        for p in m.patches:
            prim += [1] * p.size + ([0] * p.size if p.kind in ("processor", "processorCyclic") else [])
        bfc = m.boundary_arrays()[4]
        partner = -np.ones(m.n_boundary_slots, dtype=np.int64)
        off = 0
        offs = []
        for p in m.patches:
            offs.append(off); off += p.slots
        for pi, p in enumerate(m.patches):
            if p.kind == "cyclic":
                q = p.neighbour_patch
                partner[offs[pi]:offs[pi] + p.size] = bfc[offs[q]:offs[q] + p.size]
        return np.array(sp_, dtype=np.int64), np.array(prim, dtype=bool), bfc.astype(np.int64), partner

    def solve_ldu(self, lower, upper, diag, source, ic, bc, ptype_name):
        m = self.m
        C_ = m.n_cells
        types = np.asarray(self.ptypes[ptype_name])
        slot_patch, prim, bfc, partner = self._slot_info()
        d = diag.copy()
        b = source.copy()
        rows = [m.neighbour, m.owner]
        cols = [m.owner, m.neighbour]
        vals = [lower, upper]
        cr, cc, cv = [], [], []
        for bslot in range(m.n_boundary_slots):
            if not prim[bslot]:
                continue
            t = types[slot_patch[bslot]]
            if t == EMPTY:
                continue
            c = bfc[bslot]
            d[c] += ic[bslot]
            if t in (CYCLIC, PROC, PROC_CYC):
                cr.append(c); cc.append(partner[bslot]); cv.append(-bc[bslot])
            else:
                b[c] += bc[bslot]
        A = sp.coo_matrix((np.concatenate(vals + [d, np.array(cv)]),
                           (np.concatenate(rows + [np.arange(C_), np.array(cr, dtype=np.int64)]),
                            np.concatenate(cols + [np.arange(C_), np.array(cc, dtype=np.int64)]))),
                          shape=(C_, C_)).tocsc()
        if C_ <= 5000:
            return spla.spsolve(A, b)
        # large meshes: a direct factorisation of a 3-D operator fills in badly; a Jacobi-preconditioned
        # Krylov solve to 1e-15 of the right-hand side is exact to the comparison tolerances (1e-9)
        Dinv = sp.diags(1.0 / A.diagonal())
        nb = max(np.abs(b).max(), 1e-300)
        sym = abs(A - A.T).max() <= 1e-14 * abs(A).max()
        solvers = ([lambda: spla.cg(A, b, rtol=1e-15, atol=0.0, maxiter=5000, M=Dinv)] if sym else []) + \
                  [lambda: spla.bicgstab(A, b, rtol=1e-15, atol=0.0, maxiter=3000, M=Dinv),
                   lambda: spla.gmres(A, b, rtol=1e-15, atol=0.0, restart=60, maxiter=40, M=Dinv)]
        best = None
        for solver in solvers:
            x, info = solver()
            res = np.abs(A @ x - b).max() / nb if np.isfinite(x).all() else np.inf
            if best is None or res < best[1]:
                best = (x, res)
            if res < 1e-12:
                return x
        if best[1] < 1e-11:
            return best[0]
        return spla.spsolve(A, b)

    # ---- one full outer iteration (dfLowMachFoam.C:284-531, nOuter = 1)
    def time_step(self, n_corr=2):
        m = self.m
        C_, F, B, S = m.n_cells, m.n_faces, m.n_boundary_slots, self.S
        a = self.arr
        for n, o in (("rho_old", "rho"), ("boundary_rho_old", "boundary_rho"), ("phi_old", "phi"),
                     ("boundary_phi_old", "boundary_phi"), ("U_old", "U"), ("boundary_U_old", "boundary_U"),
                     ("K_old", "K"), ("p_old", "p"), ("boundary_p_old", "boundary_p")):
            a[n][...] = a[o]
        self.rho_eqn()
        u = self.u_assemble()
        for k in range(3):
            a["U"][k] = self.solve_ldu(u["lower"], u["upper"], u["diag"], u["source_solve"][k * C_:(k + 1) * C_],
                                       u["internal_coeffs"][k * B:(k + 1) * B], u["boundary_coeffs"][k * B:(k + 1) * B], "U")
        self.correct_bc("U", "U", 3)
        Ux, Uy, Uz = a["U"]
        a["K"][...] = 0.5 * (Ux * Ux + Uy * Uy + Uz * Uz)
        bx, by, bz = a["boundary_U"]
        a["boundary_K"][...] = 0.5 * (bx * bx + by * by + bz * bz)
        self.y_prep()
        y = self.y_assemble()
        for s in range(S):
            if s == self.inert:
                continue
            a["Y"][s] = self.solve_ldu(y["lower"][s * F:(s + 1) * F], y["upper"][s * F:(s + 1) * F],
                                       y["diag"][s * C_:(s + 1) * C_], y["source"][s * C_:(s + 1) * C_],
                                       y["internal_coeffs"][s * B:(s + 1) * B], y["boundary_coeffs"][s * B:(s + 1) * B], "Y")
        self.y_inert()
        self.energy_gradient()                    # dfEEqn.cu:148 (gradientEnergy patches)
        self.correct_bc("he", "he", 1)
        e = self.e_assemble()
        a["he"][...] = self.solve_ldu(e["lower"], e["upper"], e["diag"], e["source"], e["internal_coeffs"],
                                      e["boundary_coeffs"], "he")
        self.correct_bc("he", "he", 1)
        self.thermo_correct(False)
        for _ in range(n_corr):
            a["rho"][...] = a["p"] * a["psi"]; a["boundary_rho"][...] = a["boundary_p"] * a["boundary_psi"]
            a["psip0"][...] = a["psi"] * a["p"]; a["boundary_psip0"][...] = a["boundary_psi"] * a["boundary_p"]
            self.u_hbya()
            pq = self.p_assemble()
            a["p"][...] = self.solve_ldu(pq["lower"], pq["upper"], pq["diag"], pq["source"], pq["internal_coeffs"],
                                         pq["boundary_coeffs"], "p")
            self.p_post()
            a["rho"][...] = a["rho"] + (a["psi"] * a["p"] - a["psip0"])
            a["boundary_rho"][...] = a["boundary_rho"] + (a["boundary_psi"] * a["boundary_p"] - a["boundary_psip0"])
            self.rho_eqn()
        a["rho"][...] = a["p"] * a["psi"]
        a["boundary_rho"][...] = a["boundary_p"] * a["boundary_psi"]


def thermo_points(table, T, he, p, Y, fixT):
    """oracle thermo_point over n states (Y [S, n]): returns dict T, he, psi, rho, mu, alpha, rhoD, hai"""
    L = lib()
    L.orc_set_thermo(table.S, _dp(np.ascontiguousarray(table.W)), _dp(np.ascontiguousarray(table.nasa)),
                     _dp(np.ascontiguousarray(table.visc)), _dp(np.ascontiguousarray(table.cond)),
                     _dp(np.ascontiguousarray(table.bdiff)))
    n = np.size(T)
    o = {"T": np.array(T, dtype=np.float64).ravel().copy(), "he": np.array(he, dtype=np.float64).ravel().copy(),
         "p": np.array(p, dtype=np.float64).ravel().copy(), "Y": np.ascontiguousarray(Y, dtype=np.float64).reshape(table.S, n)}
    for k in ("psi", "rho", "mu", "alpha"):
        o[k] = np.zeros(n)
    o["rhoD"] = np.zeros((table.S, n)); o["hai"] = np.zeros((table.S, n))
    rc = L.orc_thermo_points(n, 1 if fixT else 0, _dp(o["T"]), _dp(o["he"]), _dp(o["p"]), _dp(o["Y"]), _dp(o["psi"]),
                             _dp(o["rho"]), _dp(o["mu"]), _dp(o["alpha"]), _dp(o["rhoD"]), _dp(o["hai"]))
    if rc != 0:
        raise RuntimeError("orc_thermo_points failed")
    return o


def zero_d_trajectory(table, kin, T0, p0, Y0, dt, n_steps, rtol=1e-12, atol=1e-22, inert=None):
    """df0DFoam (applications/solvers/df0DFoam/df0DFoam.C:99-113, YEqn.H, EEqn.H; constantProperty
    pressure) for one cell: per step chemistry.solve(dt) -- isothermal closed reactor from
    setState_TPY(T, p, Y), RR scaled by the thermo rho --, YEqn ddt(rho, Yi) == RR_i (Yi.max(0),
    inert = 1 - sum), he held, correctThermo (T from he), rho = thermo.rho(). Returns T [n+1], Y [n+1, S]."""
    S = table.S
    inert = S - 1 if inert is None else inert
    st = thermo_points(table, [T0], [0.0], [p0], np.asarray(Y0, dtype=np.float64).reshape(S, 1), True)
    T, he, rho, Y = st["T"][0], st["he"][0], st["rho"][0], np.asarray(Y0, dtype=np.float64).copy()
    Ts, Ys = [T], [Y.copy()]
    for _ in range(n_steps):
        rho_old = rho
        RR = kin.reaction_rates(np.array([T]), np.array([p0]), np.array([rho]), Y.reshape(S, 1), dt,
                                rtol=rtol, atol=atol)[:, 0]
        rdt = 1.0 / dt
        Yn = (rdt * rho_old * Y * 1.0 + 1.0 * RR) / (rdt * rho * 1.0)
        Yn = np.maximum(Yn, 0.0)
        tot = 0.0
        for s_ in range(S):
            if s_ != inert:
                tot += Yn[s_]
        Yn[inert] = max(1.0 - tot, 0.0)
        Y = Yn
        st = thermo_points(table, [T], [he], [p0], Y.reshape(S, 1), False)
        T, rho = st["T"][0], st["rho"][0]
        Ts.append(T); Ys.append(Y.copy())
    return np.array(Ts), np.array(Ys)
