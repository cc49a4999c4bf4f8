"""fvSchemes selection for the terms the reference GPU path hard-wires.

The reference GPU path interpolates Yi and ha upwind and K and hDiffCorrFlux linearly whatever the case
asks for (src_gpu/dfYEqn.cu:543,587-593, dfEEqn.cu:166-174; limitedLinear is disabled,
dfMatrixOpBase.cu:2540-2600). The reference's own dfLowMachFoam cases ask for bounded schemes
(examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/system/fvSchemes:33-41,
test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver/system/fvSchemes:32-40), which the CPU
dfLowMachFoam runs (YEqn.H:6-14 multivariate convection over every Y_i and he, createFields.H:118-129;
EEqn.H fvc::div(phi, K) and fvc::div(hDiffCorrFlux)). dfmi_set_scheme (include/dfmi.h) selects them.
"""
from __future__ import annotations

TERMS = ("div(phi,Yi_h)", "div(phi,K)", "div(hDiffCorrFlux)", "div(phi,U)")
UPWIND, LINEAR, LIMITED_LINEAR, LIMITED_LINEAR01, CUBIC, LIMITED_LINEAR_V = 0, 1, 2, 3, 4, 5
DEFAULT = {"div(phi,Yi_h)": "upwind", "div(phi,K)": "linear", "div(hDiffCorrFlux)": "linear", "div(phi,U)": "linear"}
# the reference cases' own divSchemes for these terms
REFERENCE_CASE = {"div(phi,Yi_h)": "limitedLinear01 1", "div(phi,K)": "limitedLinear 1",
                  "div(hDiffCorrFlux)": "cubic"}
_ALLOWED = {"div(phi,Yi_h)": (UPWIND, LIMITED_LINEAR, LIMITED_LINEAR01),
            "div(phi,K)": (UPWIND, LINEAR, LIMITED_LINEAR, LIMITED_LINEAR01),
            "div(hDiffCorrFlux)": (LINEAR, CUBIC), "div(phi,U)": (LINEAR, LIMITED_LINEAR_V)}


def parse(term: str, scheme: str) -> tuple[int, float]:
    """'limitedLinear01 1' -> (LIMITED_LINEAR01, 1.0); a leading 'Gauss' is accepted"""
    if term not in TERMS:
        raise ValueError(f"unknown scheme term {term!r}; expected one of {TERMS}")
    tok = scheme.split()
    if tok and tok[0] == "Gauss":
        tok = tok[1:]
    names = {"upwind": UPWIND, "linear": LINEAR, "limitedLinear": LIMITED_LINEAR,
             "limitedLinear01": LIMITED_LINEAR01, "cubic": CUBIC, "limitedLinearV": LIMITED_LINEAR_V}
    if not tok or tok[0] not in names:
        raise ValueError(f"{term}: unsupported scheme {scheme!r}")
    code = names[tok[0]]
    k = 1.0
    if code in (LIMITED_LINEAR, LIMITED_LINEAR01, LIMITED_LINEAR_V):
        if len(tok) != 2:
            raise ValueError(f"{term}: {tok[0]} needs its coefficient k")
        k = float(tok[1])
        if not 0.0 <= k <= 1.0:
            raise ValueError(f"{term}: limitedLinear coefficient must be in [0, 1]")
    elif len(tok) != 1:
        raise ValueError(f"{term}: unexpected arguments in {scheme!r}")
    if code not in _ALLOWED[term]:
        raise ValueError(f"{term}: scheme {tok[0]} not supported for this term")
    return code, k


def scheme_codes(schemes: dict) -> tuple[list, list]:
    """{term: scheme} -> (codes[4], k[3]) in TERMS order (k of Yi_h, K, U), defaults filled in"""
    full = dict(DEFAULT)
    for t, v in schemes.items():
        parse(t, v)
        full[t] = v
    codes, ks = [], [1.0, 1.0, 1.0]
    kslot = {0: 0, 1: 1, 3: 2}
    for i, t in enumerate(TERMS):
        c, k = parse(t, full[t])
        codes.append(c)
        if i in kslot:
            ks[kslot[i]] = k
    return codes, ks


def read_fv_schemes(path: str) -> dict:
    """the divSchemes entries of a case's system/fvSchemes for TERMS ({term: scheme})"""
    import re
    txt = open(path).read()
    txt = re.sub(r"//.*", "", txt)
    mo = re.search(r"divSchemes\s*\{(.*?)\}", txt, re.S)
    out = {}
    if not mo:
        return out
    for line in mo.group(1).split(";"):
        tok = line.split()
        if len(tok) >= 2 and tok[0] in TERMS:
            out[tok[0]] = " ".join(tok[1:])
    return out
