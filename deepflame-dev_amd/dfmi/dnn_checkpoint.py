"""DF-ODENet weight ingestion: a trained checkpoint in the reference's layout -> the arrays dfmi_dnn_set_model
takes (include/dfmi.h), or a packed file dfmi_dnn_load_model reads.

Reference layout (test/Tu500K-Phi1/inference.py:12-25,76-106): ONE `torch.save`d dict holding the
normalisation vectors `data_in_mean` / `data_in_std` ([S + 2]: T, p, BCT(Y_i) of all species) and
`data_target_mean` / `data_target_std` ([S - 1]), plus one `state_dict` per non-inert species under `net<i>`,
i = 0 .. S - 2, of the NN_MLP module: a `torch.nn.Sequential` attribute `net` with `linear_layer_<k>` Linear
layers (GELU between them), widths [S + 2, 1600, 800, 400, 1]. The reference GPU solver loads the same nets as
TorchScript programs, one file per species (`new_Temporary_Chemical_<i>.pt`, src_gpu/dfChemistrySolver.cu:112-126)
with its normalisation hard-coded (:95-105).

Safety: the checkpoint is read with `torch.load(..., weights_only=True)` only -- tensors, dicts, lists and
numbers; anything that would execute code on load (pickled classes, TorchScript programs) is refused by torch
and reported here. TorchScript files are therefore not read: export the nets' `state_dict()`s into the dict
layout above in the environment that trusts them ("DF-ODENet weights").

Packed file (`write_packed` / `read_packed`, and `dfmi_dnn_load_model` in the library), little-endian:
  8 B magic "DFMIDNN1"; int32 n_modules, n_layers; int32 dims[n_layers + 1];
  float64 x_mu[dims[0]], x_std[dims[0]], y_mu[n_modules], y_std[n_modules];
  float32 params: per module, per layer, W [out][in] row-major then b [out] (dfmi_dnn_set_model's order).
"""
from __future__ import annotations

import re
import struct

import numpy as np

MAGIC = b"DFMIDNN1"
_NORMS = ("data_in_mean", "data_in_std", "data_target_mean", "data_target_std")


def _np(v, dtype):
    if hasattr(v, "detach"):
        v = v.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(v, dtype=dtype))


def read_checkpoint(path: str) -> dict:
    """Load a reference-layout checkpoint with weights_only=True and convert it (from_state_dict)."""
    import torch
    # numpy arrays (the normalisation vectors may be saved as such) are plain data: their reconstruction
    # function, ndarray and the float dtypes are allow-listed, nothing else
    try:
        from numpy._core.multiarray import _reconstruct
    except ImportError:   # numpy < 2
        from numpy.core.multiarray import _reconstruct
    allowed = [_reconstruct, np.ndarray, np.dtype]
    allowed += [getattr(np.dtypes, n) for n in ("Float64DType", "Float32DType") if hasattr(np, "dtypes")]
    try:
        with torch.serialization.safe_globals(allowed):
            sd = torch.load(path, map_location="cpu", weights_only=True)
    except Exception as e:   # torch's UnpicklingError for anything beyond tensors and containers
        raise ValueError(f"{path}: not loadable as a weights-only checkpoint ({type(e).__name__}: {e}); "
                         "export the nets' state_dict()s and normalisation vectors into a plain dict "
                         "(INTEGRATION.md)") from None
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: expected a dict checkpoint (inference.py's state_dict), got {type(sd).__name__}")
    return from_state_dict(sd)


def _layers(net: dict, name: str):
    """(W [out, in] float32, b [out] float32) per linear layer of one NN_MLP state_dict, in layer order."""
    found = {}
    for k, v in net.items():
        m = re.fullmatch(r"(?:module\.)?(?:net\.)?linear_layer_(\d+)\.(weight|bias)", k)
        if m is None:
            raise ValueError(f"{name}: unexpected key '{k}' (NN_MLP has net.linear_layer_<k>.weight / .bias)")
        found.setdefault(int(m.group(1)), {})[m.group(2)] = v
    if not found or sorted(found) != list(range(len(found))):
        raise ValueError(f"{name}: linear layers {sorted(found)} are not 0 .. n-1")
    out = []
    for k in range(len(found)):
        if set(found[k]) != {"weight", "bias"}:
            raise ValueError(f"{name}: linear_layer_{k} lacks its weight or bias")
        W, b = _np(found[k]["weight"], np.float32), _np(found[k]["bias"], np.float32)
        if W.ndim != 2 or b.shape != (W.shape[0],):
            raise ValueError(f"{name}: linear_layer_{k} has weight {W.shape} / bias {b.shape}")
        out.append((W, b))
    for k in range(1, len(out)):
        if out[k][0].shape[1] != out[k - 1][0].shape[0]:
            raise ValueError(f"{name}: linear_layer_{k} takes {out[k][0].shape[1]} inputs, "
                             f"linear_layer_{k - 1} gives {out[k - 1][0].shape[0]}")
    return out


def from_state_dict(sd: dict) -> dict:
    """The reference checkpoint dict -> {dims, params, x_mu, x_std, y_mu, y_std} (params: per module a list of
    (W, b) per layer, the form dfmi.lib.Context.dnn_set_model and dfmi.dnn_model.seeded_weights use)."""
    missing = [k for k in _NORMS if k not in sd]
    if missing:
        raise ValueError(f"checkpoint lacks {missing} (inference.py:77-80)")
    nets = sorted((int(m.group(1)), k) for k in sd for m in [re.fullmatch(r"net(\d+)", str(k))] if m)
    if not nets or [i for i, _ in nets] != list(range(len(nets))):
        raise ValueError(f"checkpoint nets {[i for i, _ in nets]} are not net0 .. net<S-2>")
    params = [_layers(sd[k], k) for _, k in nets]
    dims = [params[0][0][0].shape[1]] + [W.shape[0] for W, _ in params[0]]
    for (i, _), p in zip(nets, params):
        d = [p[0][0].shape[1]] + [W.shape[0] for W, _ in p]
        if d != dims:
            raise ValueError(f"net{i} has widths {d}, net0 {dims}")
    if dims[-1] != 1:
        raise ValueError(f"the nets end in {dims[-1]} outputs, the surrogate needs 1 (one species each)")
    x_mu, x_std = (_np(sd[k], np.float64).ravel() for k in _NORMS[:2])
    y_mu, y_std = (_np(sd[k], np.float64).ravel() for k in _NORMS[2:])
    nmod = len(params)
    if x_mu.size != dims[0] or x_std.size != dims[0]:
        raise ValueError(f"data_in_mean/std have {x_mu.size}/{x_std.size} entries, the nets take {dims[0]}")
    if y_mu.size != nmod or y_std.size != nmod:
        raise ValueError(f"data_target_mean/std have {y_mu.size}/{y_std.size} entries for {nmod} nets")
    if dims[0] != nmod + 3:
        raise ValueError(f"{nmod} nets (S - 1) need {nmod + 3} inputs (T, p, S mass fractions), got {dims[0]}")
    return {"dims": dims, "params": params, "x_mu": x_mu, "x_std": x_std, "y_mu": y_mu, "y_std": y_std}


def pack_params(params) -> np.ndarray:
    """The flat float32 parameter array of dfmi_dnn_set_model: per module, per layer, W [out][in] then b [out]."""
    return np.ascontiguousarray(
        np.concatenate([np.concatenate([np.ravel(W), np.ravel(b)]) for mod in params for (W, b) in mod]),
        dtype=np.float32)


def write_packed(path: str, model: dict) -> None:
    dims = [int(d) for d in model["dims"]]
    nmod, nl = len(model["params"]), len(dims) - 1
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<ii", nmod, nl))
        f.write(np.asarray(dims, dtype="<i4").tobytes())
        for k in ("x_mu", "x_std", "y_mu", "y_std"):
            f.write(np.asarray(model[k], dtype="<f8").tobytes())
        f.write(pack_params(model["params"]).astype("<f4").tobytes())


def read_packed(path: str) -> dict:
    """The packed file back as {dims, n_modules, flat, x_mu, x_std, y_mu, y_std} (flat: pack_params' array)."""
    b = open(path, "rb").read()
    if b[:8] != MAGIC:
        raise ValueError(f"{path}: not a packed DF-ODENet file")
    nmod, nl = struct.unpack_from("<ii", b, 8)
    o = 16
    dims = np.frombuffer(b, "<i4", nl + 1, o).tolist()
    o += 4 * (nl + 1)
    out = {"dims": dims, "n_modules": nmod}
    for k, n in (("x_mu", dims[0]), ("x_std", dims[0]), ("y_mu", nmod), ("y_std", nmod)):
        out[k] = np.frombuffer(b, "<f8", n, o).copy()
        o += 8 * n
    npar = nmod * sum(dims[l] * dims[l + 1] + dims[l + 1] for l in range(nl))
    if len(b) != o + 4 * npar:
        raise ValueError(f"{path}: {len(b)} bytes, the header implies {o + 4 * npar}")
    out["flat"] = np.frombuffer(b, "<f4", npar, o).copy()
    return out


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="pack a reference-layout DF-ODENet checkpoint for dfmi_dnn_load_model")
    ap.add_argument("checkpoint")
    ap.add_argument("out")
    a = ap.parse_args(argv)
    m = read_checkpoint(a.checkpoint)
    write_packed(a.out, m)
    print(f"{a.out}: {len(m['params'])} nets, widths {m['dims']}")


if __name__ == "__main__":
    main()
