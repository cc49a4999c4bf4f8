"""Mechanism data: Cantera YAML species/NASA7 reader and the reference thermo table.

The GPU thermo path reads a binary coefficient file ``thermo_<mech>.txt`` next to
the Cantera mechanism (reference ``src_gpu/dfThermo.cu:361-435``):

    int32 S; f64 W[S]; f64 nasa[S][15] = [T_mid, hi a0..a6, lo a0..a6];
    f64 visc[S][5]; f64 cond[S][5]; f64 bindiff[S][S][5]

with the transport fits in ln T:  sqrt(mu_i/sqrt(T)) = poly,  lambda_i/sqrt(T) = poly,
D_ij*p/T^1.5 = poly  (Cantera MixTransport fits). This module reads/writes that
format and parses Cantera YAML (PyYAML SafeLoader only; nothing is executed).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
import numpy as np
import yaml


@dataclass
class ThermoTable:
    species: list
    W: np.ndarray        # [S] kg/kmol
    nasa: np.ndarray     # [S,15]
    visc: np.ndarray     # [S,5]
    cond: np.ndarray     # [S,5]
    bdiff: np.ndarray    # [S,S,5]

    @property
    def S(self) -> int:
        return int(self.W.shape[0])


def read_thermo_table(path: str, species=None) -> ThermoTable:
    b = open(path, "rb").read()
    S = struct.unpack("i", b[:4])[0]
    a = np.frombuffer(b[4:], dtype=np.float64)
    need = S + 15 * S + 5 * S + 5 * S + 5 * S * S
    if a.size != need:
        raise ValueError(f"{path}: expected {need} doubles for S={S}, got {a.size}")
    o = 0
    W = a[o:o + S].copy(); o += S
    nasa = a[o:o + 15 * S].reshape(S, 15).copy(); o += 15 * S
    visc = a[o:o + 5 * S].reshape(S, 5).copy(); o += 5 * S
    cond = a[o:o + 5 * S].reshape(S, 5).copy(); o += 5 * S
    bdiff = a[o:o + 5 * S * S].reshape(S, S, 5).copy()
    return ThermoTable(list(species) if species is not None else [f"s{i}" for i in range(S)], W, nasa, visc, cond, bdiff)


def write_thermo_table(path: str, t: ThermoTable) -> None:
    with open(path, "wb") as f:
        f.write(struct.pack("i", t.S))
        for arr in (t.W, t.nasa, t.visc, t.cond, t.bdiff):
            f.write(np.ascontiguousarray(arr, dtype=np.float64).tobytes())


ATOMIC_W = {"H": 1.008, "O": 15.999, "N": 14.007, "C": 12.011, "Ar": 39.95, "AR": 39.95, "He": 4.002602}


def read_yaml_mechanism(path: str) -> dict:
    """Species names, compositions, molecular weights, NASA7 blocks and transport data."""
    with open(path) as f:
        doc = yaml.load(f, Loader=yaml.SafeLoader)
    phase = doc["phases"][0]
    names = phase["species"]
    spec = {s["name"]: s for s in doc["species"]}
    out = {"species": list(names), "W": [], "nasa": [], "transport": [], "composition": [], "trange": [],
           "reactions": doc.get("reactions", []), "phase": phase}
    for n in names:
        s = spec[n]
        comp = s["composition"]
        out["composition"].append(comp)
        out["W"].append(sum(ATOMIC_W[e] * c for e, c in comp.items()))
        th = s["thermo"]
        tr = th["temperature-ranges"]
        if len(th["data"]) == 1:        # one range (e.g. AR in gri30): same block on both sides of T_mid
            lo = hi = th["data"][0]
        else:
            lo, hi = th["data"]
        row = [float(tr[1])] + [float(x) for x in hi] + [float(x) for x in lo]
        out["nasa"].append(row)
        out["trange"].append((float(tr[0]), float(tr[-1])))
        out["transport"].append(s.get("transport", {}))
    out["W"] = np.array(out["W"])
    out["nasa"] = np.array(out["nasa"])
    return out


def nasa_h_mass(nasa_row: np.ndarray, W: float, T: float) -> float:
    """NASA7 enthalpy per unit mass [J/kg] (dfThermo.cu:257-275)."""
    R = 8314.46261815324
    a = nasa_row[1:8] if T > nasa_row[0] else nasa_row[8:15]
    return (a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T ** 3 / 4 + a[4] * T ** 4 / 5 + a[5] / T) * R * T / W
