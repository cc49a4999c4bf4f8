"""OpenFOAM ASCII field files (volScalarField / volVectorField, optionally gzip'd): the reader part
of the case I/O row. Parses `internalField uniform v` / `nonuniform
List<scalar|vector> N ( ... )` and the patch types of `boundaryField`; writes the same format.
Text parsing only (nothing is executed)."""
from __future__ import annotations

import gzip
import re

import numpy as np


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def read_field(path: str):
    """-> (values, patch_types): values [n] (scalar) or [n, 3] (vector); uniform fields return a
    0-d / [3] array."""
    txt = _open(path).read()
    cls = re.search(r"class\s+(\w+);", txt).group(1)
    vector = cls.endswith("VectorField")
    m = re.search(r"internalField\s+(uniform|nonuniform)", txt)
    if m is None:
        raise ValueError(f"{path}: no internalField")
    rest = txt[m.end():]
    if m.group(1) == "uniform":
        if vector:
            v = re.match(r"\s*\(([^)]*)\)", rest).group(1)
            vals = np.array([float(x) for x in v.split()])
        else:
            vals = np.array(float(re.match(r"\s*([^;\s]+)", rest).group(1)))
    else:
        hdr = re.match(r"\s*List<(\w+)>\s*(\d+)\s*\(", rest)
        n = int(hdr.group(2))
        body = rest[hdr.end():]
        end = body.find("\n)")
        body = body[:end]
        if vector:
            nums = np.array(body.replace("(", " ").replace(")", " ").split(), dtype=np.float64)
            vals = nums.reshape(n, 3)
        else:
            vals = np.array(body.split(), dtype=np.float64)
            assert vals.size == n, (path, vals.size, n)
    types = {}
    b = txt.find("boundaryField")
    if b >= 0:
        for pm in re.finditer(r"(\w+)\s*\{\s*type\s+(\w+);", txt[b:]):
            types[pm.group(1)] = pm.group(2)
    return vals, types


def read_boundary(path: str) -> dict:
    """boundaryField of a field file -> {patch: (type, value or None)}; `value uniform v` entries
    only (scalar or vector)."""
    txt = _open(path).read()
    b = txt.find("boundaryField")
    out = {}
    if b < 0:
        return out
    for pm in re.finditer(r"(\w+)\s*\{([^{}]*)\}", txt[b + len("boundaryField"):]):
        body = pm.group(2)
        t = re.search(r"type\s+(\w+);", body)
        if not t:
            continue
        v = re.search(r"value\s+uniform\s+(\([^)]*\)|[^;\s]+)\s*;", body)
        val = None
        if v:
            txtv = v.group(1).strip("()")
            val = np.array([float(x) for x in txtv.split()])
            val = val[0] if val.size == 1 else val
        out[pm.group(1)] = (t.group(1), val)
    return out


def write_field(path: str, name: str, values: np.ndarray, patch_types: dict, dims="[0 0 0 0 0 0 0]"):
    vector = values.ndim == 2
    cls = "volVectorField" if vector else "volScalarField"
    lines = ["FoamFile", "{", "    version     2.0;", "    format      ascii;", f"    class       {cls};",
             f"    object      {name};", "}", "", f"dimensions      {dims};", "",
             f"internalField   nonuniform List<{'vector' if vector else 'scalar'}>", str(len(values)), "("]
    if vector:
        lines += [f"({float(v[0])!r} {float(v[1])!r} {float(v[2])!r})" for v in values]
    else:
        lines += [repr(float(v)) for v in values]
    lines += [")", ";", "", "boundaryField", "{"]
    for p, t in patch_types.items():
        lines += [f"    {p}", "    {", f"        type            {t};", "    }"]
    lines += ["}"]
    with (gzip.open(path, "wt") if path.endswith(".gz") else open(path, "w")) as f:
        f.write("\n".join(lines) + "\n")


def read_case_fields(directory: str, species: list):
    """T, p, U and Y of a case's 0/ directory in the species order given."""
    import os
    def rd(n):
        for ext in (".gz", ""):
            pth = os.path.join(directory, n + ext)
            if os.path.exists(pth):
                return read_field(pth)[0]
        raise FileNotFoundError(os.path.join(directory, n))
    T = rd("T")
    p = rd("p")
    U = rd("U")
    n = T.size
    Y = np.stack([np.broadcast_to(rd(s), (n,)) for s in species])
    return {"T": T, "p": np.broadcast_to(p, (n,)).copy(), "U": np.ascontiguousarray(np.broadcast_to(U, (n, 3)).T),
            "Y": np.ascontiguousarray(Y)}


def tile_fields(f: dict, n_src: int, reps=(2, 2, 2)) -> dict:
    """Tile fields of an n_src^3 block (i fastest) reps times per direction (BASELINE config 3:
    the 64^3 TGV fields tiled 2x2x2 into 128^3)."""
    def tile(a):
        lead = a.shape[:-1]
        b = a.reshape(lead + (n_src, n_src, n_src))            # [..., k, j, i]
        b = np.tile(b, (1,) * len(lead) + (reps[2], reps[1], reps[0]))
        return np.ascontiguousarray(b.reshape(lead + (-1,)))
    return {k: tile(v) for k, v in f.items()}
