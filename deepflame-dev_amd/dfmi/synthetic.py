"""BASELINE config 4: the 53-species case the repository has no mechanism for.

The reference's gri30.yaml (mechanisms/CH4) is GRI-3.0 without nitrogen chemistry: 36 species. Config 4
names 53 species (full GRI-3.0) with the DF-ODENet surrogate as the source, which needs no kinetics,
so the thermo/transport table is built synthetically as SURVEY 8d prescribes: the 36 real species'
NASA7 blocks and transport fits (dfmi.transport_fit on gri30.yaml), cycled to 53 -- species 35..51
repeat the first 17 non-N2 species (named "<species>#2") -- with N2 last (the DNN layout wants the inert
species last, dfChemistrySolver.cu:160-166). Pairs of a species and its copy use the species' self-
diffusion fit. Mass fractions are Dirichlet-like draws (seed 0).
"""
from __future__ import annotations

import numpy as np

from .mech import ThermoTable, read_yaml_mechanism

S53 = 53


def gri53_order(species36: list) -> list:
    """indices into the 36 gri30 species for the 53 synthetic ones (N2 last)"""
    base = [i for i, s in enumerate(species36) if s != "N2"]          # 35
    extra = base[: S53 - 1 - len(base)]                                # 17 repeats
    return base + extra + [species36.index("N2")]


def gri53_species(gri30_yaml: str) -> list:
    ym = read_yaml_mechanism(gri30_yaml)
    names, seen = [], {}
    for i in gri53_order(ym["species"]):
        n = ym["species"][i]
        seen[n] = seen.get(n, 0) + 1
        names.append(n if seen[n] == 1 else f"{n}#{seen[n]}")
    return names


def gri53_table(gri30_yaml: str) -> ThermoTable:
    from .transport_fit import fit_mechanism
    ym = read_yaml_mechanism(gri30_yaml)
    t36 = fit_mechanism(ym)
    idx = np.array(gri53_order(ym["species"]))
    return ThermoTable(gri53_species(gri30_yaml), t36.W[idx].copy(), t36.nasa[idx].copy(), t36.visc[idx].copy(), t36.cond[idx].copy(),
                       t36.bdiff[np.ix_(idx, idx)].copy())


def gri53_mass_fractions(n: int, seed: int = 0, alpha: float = 0.3) -> np.ndarray:
    """[53, n] Dirichlet-like mass fractions (gamma(alpha) draws, renormalised), N2-rich like air"""
    rng = np.random.default_rng(seed)
    Y = rng.gamma(alpha, 1.0, (S53, n))
    Y[-1] += 20.0 * Y[:-1].sum(axis=0) / (S53 - 1) * 2.0      # the inert (N2) dominates, as in air flames
    return Y / Y.sum(axis=0)


def gri53_smooth_fractions(prog: np.ndarray, seed: int = 0) -> np.ndarray:
    """[53, n] mass fractions varying smoothly in space: two Dirichlet-like compositions (30 % of the mass
    spread over the 52 non-inert species by gamma(0.3) draws, 70 % N2) blended by prog in [0, 1] -- the
    hot kernel's progress variable -- so that enthalpy and density stay smooth fields (a per-cell random
    composition makes the flow solution itself noise)"""
    rng = np.random.default_rng(seed)
    comp = []
    for _ in range(2):
        b = rng.gamma(0.3, 1.0, S53 - 1)
        comp.append(np.concatenate([0.3 * b / b.sum(), [0.7]]))
    prog = np.clip(np.asarray(prog, dtype=np.float64), 0.0, 1.0)
    return (1 - prog)[None, :] * comp[0][:, None] + prog[None, :] * comp[1][:, None]


def gri53_dnn(ctx, seed: int = 0):
    """52 DF-ODENet nets [55, 1600, 800, 400, 1] (inference.py:12-25 widths) with seeded N(0, 1/fan_in)
    weights; input normalisation in the H2 nets' pattern (T ~ 1300 +- 400 K, p ~ 1 atm, Box-Cox(Y) ~ -5
    +- 2, dfChemistrySolver.cu:95-105); outputs scaled by 1e-4 so the synthetic source stays small"""
    from .dnn_model import seeded_weights
    S = S53
    dims = [S + 2, 1600, 800, 400, 1]
    xmu = np.concatenate([[1.3e3, 1.01325e5], np.full(S, -5.0)])
    xstd = np.concatenate([[4.0e2, 2.0e4], np.full(S, 2.0)])
    ctx.dnn_set_model(dims, seeded_weights(n_modules=S - 1, dims=dims, seed=seed), xmu, xstd, np.zeros(S - 1),
                      np.full(S - 1, 1e-4))
