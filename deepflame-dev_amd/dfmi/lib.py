"""ctypes binding of libdfmi.so (include/dfmi.h).

The library is the product: there is no CPU fallback. Importing this module on a machine
where libdfmi.so is missing raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libdfmi.so")

_libs = {}


def load(path: str | None = None) -> C.CDLL:
    """the HIP library (default), or another implementation of include/dfmi.h given by path (the CPU-A
    baseline, baseline/cpu_a/libdfmi_cpu_a.so, which only bench.py's cpu_baseline leg and its tests use)"""
    path = path or LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise RuntimeError(f"{os.path.basename(path)} not found at {path}; run __graft_entry__.build()")
        lib = C.CDLL(path)
        _declare(lib)
        _libs[path] = lib
    return _libs[path]


_P = C.c_void_p
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int)

SIGNATURES = {
    "dfmi_create": [C.POINTER(_P), C.c_int],
    "dfmi_destroy": [_P],
    "dfmi_last_error": [C.c_char_p, C.c_int],
    "dfmi_set_constant_values": [_P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _IP, C.c_int, C.c_double],
    "dfmi_set_cyclic_info": [_P, _IP],
    "dfmi_set_comm_info": [_P, C.c_void_p, C.c_int, C.c_int, _IP],
    "dfmi_get_unique_id": [C.c_void_p],
    "dfmi_set_comm_local": [_P, C.c_int, C.c_int, C.c_int, _IP],
    "dfmi_set_constant_indexes": [_P, _IP, _IP, _IP, _IP, C.c_int],
    "dfmi_init_constant_fields_internal": [_P, _DP, _DP, _DP, _DP, _DP, _DP],
    "dfmi_init_constant_fields_boundary": [_P, _DP, _DP, _DP, _DP, _IP, _IP, _IP],
    "dfmi_set_patch_types": [_P, C.c_char_p, _IP],
    "dfmi_set_inert_index": [_P, C.c_int],
    "dfmi_set_patch_param": [_P, C.c_char_p, C.c_int, C.c_char_p, C.c_double],
    "dfmi_set_traversal": [_P, _IP],
    "dfmi_init_boundary_delta": [_P, _DP],
    "dfmi_set_scheme": [_P, C.c_char_p, C.c_char_p],
    "dfmi_thermo_set_coeffs": [_P, C.c_int, _DP, _DP, _DP, _DP, _DP],
    "dfmi_thermo_load": [_P, C.c_char_p],
    "dfmi_set_field": [_P, C.c_char_p, _DP, C.c_long, C.c_int],
    "dfmi_get_field": [_P, C.c_char_p, _DP, C.c_long, C.c_int],
    "dfmi_pre_time_step": [_P], "dfmi_rho_process": [_P], "dfmi_U_process": [_P], "dfmi_Y_process": [_P],
    "dfmi_E_process": [_P], "dfmi_thermo_correct": [_P], "dfmi_thermo_update_energy": [_P],
    "dfmi_thermo_update_rho": [_P], "dfmi_thermo_psip0": [_P], "dfmi_thermo_correct_psip_rho": [_P],
    "dfmi_U_get_HbyA": [_P], "dfmi_p_process": [_P], "dfmi_post_time_step": [_P],
    "dfmi_time_step": [_P, C.c_int], "dfmi_sync": [_P],
    "dfmi_step_timer": [_P, C.c_int], "dfmi_step_times": [_P, _DP, C.c_int, _IP],
    "dfmi_hbm_copy_peak": [_P, C.c_double, C.c_int, _DP],
    "dfmi_assemble": [_P, C.c_char_p],
    "dfmi_get_matrix": [_P, C.c_char_p, C.c_char_p, _DP, C.c_long],
    "dfmi_get_solver_rows": [_P, C.c_char_p, C.c_char_p, _DP, C.c_long],
    "dfmi_set_solver": [_P, C.c_char_p, C.c_int, C.c_double, C.c_double],
    "dfmi_solver_stats": [_P, C.c_char_p, _IP, _DP, _DP],
    "dfmi_solver_work": [_P, C.c_char_p, _DP, C.c_int],
    "dfmi_set_preconditioner": [_P, C.c_char_p, C.c_char_p],
    "dfmi_set_option": [_P, C.c_char_p, C.c_double], "dfmi_get_option": [_P, C.c_char_p, _DP],
    "dfmi_amg_info": [_P, C.c_int, _IP, _IP, _IP],
    "dfmi_row_classes": [_P, _IP],
    "dfmi_hex_dims": [_P, _IP, _IP, _IP],
    "dfmi_correct_boundary": [_P, C.c_char_p],
    "dfmi_kernel_timer": [_P, C.c_char_p],
    "dfmi_comm_timer": [_P, C.c_int],
    "dfmi_comm_report": [_P, C.c_char_p, C.c_int, _IP],
    "dfmi_kernel_time": [_P, _DP, _IP],
    "dfmi_kernel_time_named": [_P, C.c_char_p, _DP, _IP],
    "dfmi_chem_set_mechanism": [_P, C.c_int, _IP, _IP, _DP],
    "dfmi_chem_set_options": [_P, C.c_int, C.c_double, C.c_double, C.c_double],
    "dfmi_chem_solve": [_P, C.c_double],
    "dfmi_chem_set_max_steps": [_P, C.c_int],
    "dfmi_zero_d_step": [_P, C.c_double, C.c_int],
    "dfmi_renumber_cells": [C.c_int, _DP, C.c_int, _IP, _IP, C.c_char_p, _IP],
    "dfmi_renumber_faces": [C.c_int, C.c_int, _IP, _IP, _IP, _IP, _IP, _IP, _IP],
    "dfmi_chem_info": [_P, _IP],
    "dfmi_dnn_set_model": [_P, C.c_int, C.c_int, _IP, C.POINTER(C.c_float), _DP, _DP, _DP, _DP, C.c_double,
                           C.c_double],
    "dfmi_dnn_load_model": [_P, C.c_char_p, C.c_double, C.c_double],
    "dfmi_dnn_infer": [_P, _IP],
    "dfmi_dnn_stats": [_P, _IP, _DP],
}


def _declare(lib):
    for name, args in SIGNATURES.items():
        if not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = C.c_int
        if args is not None:
            fn.argtypes = args
    lib.dfmi_version.restype = C.c_char_p


def exported_symbols() -> list:
    return list(SIGNATURES) + ["dfmi_version"]


class DfmiError(RuntimeError):
    pass


def _check(rc, name):
    if rc != 0:
        buf = C.create_string_buffer(4096)
        load().dfmi_last_error(buf, 4096)
        raise DfmiError(f"{name}: {buf.value.decode()}")


def renumber_cells(n_cells, cell_centres, owner, neighbour, method="morton"):
    """new -> old cell map (include/dfmi.h dfmi_renumber_cells)"""
    lib = load()
    cc = np.ascontiguousarray(cell_centres, dtype=np.float64).reshape(-1)
    o = np.ascontiguousarray(owner, dtype=np.int32); nb = np.ascontiguousarray(neighbour, dtype=np.int32)
    out = np.empty(n_cells, np.int32)
    _check(lib.dfmi_renumber_cells(int(n_cells), cc.ctypes.data_as(_DP), int(o.size), o.ctypes.data_as(_IP),
                                   nb.ctypes.data_as(_IP), method.encode(), out.ctypes.data_as(_IP)), "dfmi_renumber_cells")
    return out


def renumber_faces(n_cells, owner, neighbour, cell_new_to_old):
    """(face new -> old, new owner, new neighbour, flipped) (include/dfmi.h dfmi_renumber_faces)"""
    lib = load()
    o = np.ascontiguousarray(owner, dtype=np.int32); nb = np.ascontiguousarray(neighbour, dtype=np.int32)
    p = np.ascontiguousarray(cell_new_to_old, dtype=np.int32)
    F = o.size
    fo, no, nn, fl = (np.empty(F, np.int32) for _ in range(4))
    _check(lib.dfmi_renumber_faces(int(n_cells), int(F), o.ctypes.data_as(_IP), nb.ctypes.data_as(_IP),
                                   p.ctypes.data_as(_IP), fo.ctypes.data_as(_IP), no.ctypes.data_as(_IP),
                                   nn.ctypes.data_as(_IP), fl.ctypes.data_as(_IP)), "dfmi_renumber_faces")
    return fo, no, nn, fl.astype(bool)


def _dp(a):
    return a.ctypes.data_as(_DP)


def _ip(a):
    return a.ctypes.data_as(_IP)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


# Implementation options (include/dfmi.h dfmi_set_option) applied to every new HIP-library Context: the entries of
# DEFAULT_OPTIONS (tests set them around a case) and of the environment variable DFMI_OPTIONS ("key=value,..."; for
# runs in child processes and bench A/B runs). The library itself reads no option from the environment.
DEFAULT_OPTIONS: dict = {}


def env_options() -> dict:
    out = {}
    for item in os.environ.get("DFMI_OPTIONS", "").split(","):
        if item.strip():
            k, v = item.split("=")
            out[k.strip()] = float(v)
    return out


class Context:
    """One device-resident database (one rank, one GPU)."""

    def __init__(self, device: int = 0, lib_path: str | None = None):
        self.lib = load(lib_path)
        h = _P()
        self._keep = []
        self._call("dfmi_create", C.byref(h), device)
        self.h = h
        if lib_path is None or os.path.abspath(lib_path) == LIB_PATH:
            for k, v in {**env_options(), **DEFAULT_OPTIONS}.items():
                self.set_option(k, v)

    def _call(self, name, *args):
        rc = getattr(self.lib, name)(*args)
        if rc != 0:
            buf = C.create_string_buffer(4096)
            self.lib.dfmi_last_error(buf, 4096)
            raise DfmiError(f"{name}: {buf.value.decode()}")
        return rc

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.dfmi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- setup
    def set_constant_values(self, C_, Ctot, F, B, P, nproc, patch_size, S, rdt):
        ps = _i32(patch_size)
        self._call("dfmi_set_constant_values", self.h, C_, Ctot, F, B, P, nproc, _ip(ps), S, float(rdt))

    def set_cyclic_info(self, cyc):
        a = _i32(cyc); self._call("dfmi_set_cyclic_info", self.h, _ip(a))

    def set_comm_info(self, uid: bytes, nranks, rank, neighb):
        a = _i32(neighb)
        buf = C.create_string_buffer(uid, 128)
        self._call("dfmi_set_comm_info", self.h, buf, nranks, rank, _ip(a))

    def set_comm_local(self, hub_id, nranks, rank, neighb):
        a = _i32(neighb)
        self._call("dfmi_set_comm_local", self.h, int(hub_id), nranks, rank, _ip(a))

    @staticmethod
    def unique_id() -> bytes:
        lib = load()
        buf = C.create_string_buffer(128)
        if lib.dfmi_get_unique_id(buf) != 0:
            e = C.create_string_buffer(4096); lib.dfmi_last_error(e, 4096)
            raise DfmiError(e.value.decode())
        return buf.raw

    def set_constant_indexes(self, owner, neighbour, proc_rows, proc_cols, global_offset):
        o, n, r, c = _i32(owner), _i32(neighbour), _i32(proc_rows), _i32(proc_cols)
        if r.size == 0:
            r = np.zeros(1, np.int32); c = np.zeros(1, np.int32)
        self._call("dfmi_set_constant_indexes", self.h, _ip(o), _ip(n), _ip(r), _ip(c), int(global_offset))

    def init_constant_fields_internal(self, sf, mag_sf, weight, delta, volume, mesh_dist):
        arrs = [_f64(x) for x in (sf, mag_sf, weight, delta, volume, mesh_dist)]
        self._call("dfmi_init_constant_fields_internal", self.h, *[_dp(a) for a in arrs])

    def init_constant_fields_boundary(self, bsf, bmag, bdelta, bweight, bfc, ptype_calc, ptype_extrap):
        arrs = [_f64(x) for x in (bsf, bmag, bdelta, bweight)]
        for i, a in enumerate(arrs):
            if a.size == 0:
                arrs[i] = np.zeros(3)
        fc = _i32(bfc) if np.size(bfc) else np.zeros(1, np.int32)
        pc, pe = _i32(ptype_calc), _i32(ptype_extrap)
        self._call("dfmi_init_constant_fields_boundary", self.h, *[_dp(a) for a in arrs], _ip(fc), _ip(pc), _ip(pe))

    def init_boundary_delta(self, bdelta):
        a = _f64(bdelta)
        if a.size == 0:
            a = np.zeros(3)
        self._call("dfmi_init_boundary_delta", self.h, _dp(a))

    def set_scheme(self, term, scheme):
        """fvSchemes divSchemes entry for div(phi,Yi_h) / div(phi,K) / div(hDiffCorrFlux) (include/dfmi.h)"""
        self._call("dfmi_set_scheme", self.h, term.encode(), scheme.encode())

    def set_patch_types(self, field, types):
        a = _i32(types); self._call("dfmi_set_patch_types", self.h, field.encode(), _ip(a))

    def set_patch_param(self, field, patch, name, value):
        self._call("dfmi_set_patch_param", self.h, field.encode(), int(patch), name.encode(), float(value))

    def set_traversal(self, order):
        """visiting order of the gather kernels (None: natural); see include/dfmi.h"""
        if order is None:
            self._call("dfmi_set_traversal", self.h, None)
        else:
            a = _i32(order)
            self._call("dfmi_set_traversal", self.h, _ip(a))

    def set_inert_index(self, i):
        self._call("dfmi_set_inert_index", self.h, int(i))

    def thermo_set_coeffs(self, t):
        arrs = [_f64(x) for x in (t.W, t.nasa, t.visc, t.cond, t.bdiff)]
        self._call("dfmi_thermo_set_coeffs", self.h, t.S, *[_dp(a) for a in arrs])

    # --- fields
    def set_field(self, name, arr, layout=0):
        a = _f64(arr)
        count = a.shape[0] if (layout == 1 and a.ndim == 2) else (a.shape[-1] if a.ndim == 2 else a.shape[0])
        self._call("dfmi_set_field", self.h, name.encode(), _dp(a), int(count), layout)

    def get_field(self, name, shape, layout=0):
        out = np.empty(shape, dtype=np.float64)
        count = shape[0] if (layout == 1 and len(shape) == 2) else (shape[-1] if len(shape) == 2 else shape[0])
        self._call("dfmi_get_field", self.h, name.encode(), _dp(out), int(count), layout)
        return out

    def get_matrix(self, eqn, part, n):
        out = np.empty(n, dtype=np.float64)
        self._call("dfmi_get_matrix", self.h, eqn.encode(), part.encode(), _dp(out), int(n))
        return out

    def get_solver_rows(self, eqn, part, n):
        out = np.empty(n, dtype=np.float64)
        self._call("dfmi_get_solver_rows", self.h, eqn.encode(), part.encode(), _dp(out), int(n))
        return out

    # --- processes
    def call(self, name, *args):
        self._call("dfmi_" + name, self.h, *args)

    def assemble(self, eqn):
        self._call("dfmi_assemble", self.h, eqn.encode())

    def correct_boundary(self, field):
        self._call("dfmi_correct_boundary", self.h, field.encode())

    def set_solver(self, eqn, max_iter, tol, abs_tol=0.0):
        self._call("dfmi_set_solver", self.h, eqn.encode(), int(max_iter), float(tol), float(abs_tol))

    def set_option(self, key: str, value: float):
        """implementation option (include/dfmi.h dfmi_set_option; INTEGRATION.md lists the keys)"""
        self._call("dfmi_set_option", self.h, key.encode(), float(value))

    def get_option(self, key: str) -> float:
        v = C.c_double()
        self._call("dfmi_get_option", self.h, key.encode(), C.byref(v))
        return v.value

    def set_preconditioner(self, eqn, name):
        self._call("dfmi_set_preconditioner", self.h, eqn.encode(), name.encode())

    def chem_set_mechanism(self, mech):
        idata, irs, dd = mech.pack()
        self._keep_chem = (idata, irs, dd)
        self._call("dfmi_chem_set_mechanism", self.h, mech.R, _ip(idata), _ip(irs), _dp(dd))

    def chem_set_options(self, mode, rtol=1e-6, atol=1e-10, T_min=0.0):
        self._call("dfmi_chem_set_options", self.h, int(mode), float(rtol), float(atol), float(T_min))

    def chem_solve(self, dt):
        self._call("dfmi_chem_solve", self.h, float(dt))

    def zero_d_step(self, dt, n_steps=1):
        """df0DFoam time steps on every cell (include/dfmi.h dfmi_zero_d_step)"""
        self._call("dfmi_zero_d_step", self.h, float(dt), int(n_steps))

    def chem_set_max_steps(self, n):
        self._call("dfmi_chem_set_max_steps", self.h, int(n))

    def chem_info(self):
        g = C.c_int()
        self._call("dfmi_chem_info", self.h, C.byref(g))
        return g.value

    def dnn_set_model(self, dims, params, x_mu, x_std, y_mu, y_std, T_react=610.0, dt_infer=1e-6):
        """params: list over modules of [(W [out,in], b [out]) per layer] (numpy float32)."""
        from .dnn_checkpoint import pack_params
        d = _i32(dims)
        flat = pack_params(params)
        self._keep_dnn = flat
        arr = [_f64(a) for a in (x_mu, x_std, y_mu, y_std)]
        self._call("dfmi_dnn_set_model", self.h, len(params), len(dims) - 1, _ip(d),
                   flat.ctypes.data_as(C.POINTER(C.c_float)), *[_dp(a) for a in arr], float(T_react), float(dt_infer))

    def dnn_load_model(self, path, T_react=610.0, dt_infer=1e-6):
        """a packed model file (dfmi/dnn_checkpoint.py write_packed) through dfmi_dnn_load_model"""
        self._call("dfmi_dnn_load_model", self.h, str(path).encode(), float(T_react), float(dt_infer))

    def dnn_infer(self):
        n = C.c_int()
        self._call("dfmi_dnn_infer", self.h, C.byref(n))
        return n.value

    def dnn_stats(self):
        n = C.c_int(); f = C.c_double()
        self._call("dfmi_dnn_stats", self.h, C.byref(n), C.byref(f))
        return n.value, f.value

    def amg_info(self):
        n = C.c_int(); cells = np.zeros(32, np.int32); w = np.zeros(32, np.int32)
        self._call("dfmi_amg_info", self.h, 32, C.byref(n), _ip(cells), _ip(w))
        return [(int(cells[i]), int(w[i])) for i in range(n.value)]

    def row_classes(self):
        """distinct gather-row classes decoded per cell (0: explicit ELL columns)"""
        n = C.c_int()
        self._call("dfmi_row_classes", self.h, C.byref(n))
        return n.value

    def hex_dims(self):
        """(nx, ny, nz) of a detected hex box in blockMesh order (computed face walk), or (0, 0, 0)"""
        v = [C.c_int(), C.c_int(), C.c_int()]
        self._call("dfmi_hex_dims", self.h, *[C.byref(a) for a in v])
        return tuple(a.value for a in v)

    def solver_stats(self, eqn):
        it = C.c_int(); r0 = C.c_double(); rel = C.c_double()
        self._call("dfmi_solver_stats", self.h, eqn.encode(), C.byref(it), C.byref(r0), C.byref(rel))
        return it.value, r0.value, rel.value

    def solver_work(self, eqn, reset=False):
        """system-iterations performed by the solves of `eqn` since the last reset"""
        v = C.c_double()
        self._call("dfmi_solver_work", self.h, eqn.encode(), C.byref(v), int(reset))
        return v.value

    def time_step(self, n_corr=2):
        self._call("dfmi_time_step", self.h, int(n_corr))

    def comm_timer(self, on: bool = True):
        """reset and arm (or disarm) the per-exchange-point communication accounting"""
        self._call("dfmi_comm_timer", self.h, int(bool(on)))

    def comm_report(self) -> dict:
        """{exchange point: {"calls", "bytes" (sent by this rank), "ms" (HIP-event time of the transport calls)}}"""
        import json
        need = C.c_int()
        self._call("dfmi_comm_report", self.h, None, 0, C.byref(need))
        buf = C.create_string_buffer(max(need.value, 1) + 64)
        self._call("dfmi_comm_report", self.h, buf, len(buf), C.byref(need))
        return json.loads(buf.value.decode() or "{}")

    def kernel_timer(self, kernel: str):
        """Arm HIP-event timing of every launch of `kernel` on this context's stream."""
        self._call("dfmi_kernel_timer", self.h, kernel.encode())

    def kernel_time(self, name=None):
        """(total_ms, launches) of an armed kernel since arming (default: the first armed)."""
        ms = C.c_double(); n = C.c_int()
        if name is None:
            self._call("dfmi_kernel_time", self.h, C.byref(ms), C.byref(n))
        else:
            self._call("dfmi_kernel_time_named", self.h, name.encode(), C.byref(ms), C.byref(n))
        return ms.value, n.value

    def hbm_copy_peak(self, gib=4.0, reps=20):
        """measured copy bandwidth, GB/s (read + write)"""
        v = C.c_double()
        self._call("dfmi_hbm_copy_peak", self.h, float(gib), int(reps), C.byref(v))
        return v.value

    def step_timer(self, on: bool = True):
        """arm per-step HIP events on the context stream (dfmi_time_step marks the end of every step)"""
        self._call("dfmi_step_timer", self.h, int(on))

    def step_times(self, n: int) -> np.ndarray:
        """durations (ms) of the steps run since step_timer(True): end of step i minus end of step i-1"""
        out = np.zeros(max(n, 1))
        got = C.c_int(0)
        self._call("dfmi_step_times", self.h, _dp(out), int(n), C.byref(got))
        return out[:min(got.value, n)]

    def sync(self):
        self._call("dfmi_sync", self.h)
