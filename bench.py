#!/usr/bin/env python3
"""dfLowMachFoam outer-iteration throughput on MI355X (BASELINE.json metric: cell-updates/s).

One step = one dfLowMachFoam outer iteration (nOuter = 1, nCorr = 2: rhoEqn, UEqn + solve,
YEqn + solves, EEqn + solve, thermo correct, 2 x {HbyA, pEqn + solve, flux/U/K update, rhoEqn})
over the whole mesh, all inputs resident in HBM. Workload: BASELINE.json configs[2], the 3D
periodic box of 128^3 = 2,097,152 hex cells (reacting Taylor-Green vortex, H2/air).

N GPUs (torchrun, one process per GPU): the box is decomposed 2x1x1 / 2x2x1 / 2x2x2 (decomposePar-
style blocks), every rank owns a 128^3 block (weak scaling: N=8 is BASELINE config 5, 256^3 = 16.8M
cells), processor-patch halos and solver reductions go over RCCL (xGMI).

Output: one JSON line (rank 0) with the driver's contract fields plus
  roofline      -- the dominant kernel's algorithmic bytes / its mean HIP-event duration,
  cpu_baseline  -- CPU-A: the OpenMP C++ implementation of the same step behind the same C ABI
                   (baseline/cpu_a), timed on this host's cores on the same 128^3 workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E (MI355X_MICROARCH.md)
PMC_FILE = "r06_pmc_traffic.json"
PMC_FLOPS_FILE = "r06_pmc_flops.json"   # scripts/pmc_flops.sh: FP64 FLOPs per dispatch (SQ_INSTS_VALU_FLOPS_FP64)
FP64_PEAK_TFS = 78.6                    # MI355X FP64 vector peak

MECHS = {   # tests/golden: the reference's ES80 table, and the Burke 9-species table made by dfmi.transport_fit
    "burke9": ("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt"),
    "es80": ("ES80_H2-7-16.yaml", "thermo_ES80_H2-7-16.txt"),
}


def algorithmic_bytes(kernel: str, C: int, F: int, B: int, S: int, Bc: int = None, W: int = 6,
                      classes: bool = False, hex_walk: bool = False, face_form: bool = False) -> float:
    """Bytes one unit of a kernel's work must move at minimum: every input element read once and every
    output element written once (fp64 values, int32 indices, int8 slot types), shared face/cell arrays
    counted ONCE per launch however many species use them. Units: one launch for the assembly/thermo
    kernels (all species of that launch); k_cg_spmv one active PCG iteration; k_bcg_spmv one SpMV of
    one active system. Bc = coupled boundary slots (cyclic / processor), W = solver row width.
    Gather topology of the cell-centric kernels: 12 B per cell (nbrStart, ownStart, cbStart) + 12 B per
    face (nbrFace, own, nei) + 9 B per coupled slot (cbSlot, partner, type). DESIGN.md 5 lists them.
    classes: the solver rows are decoded from row classes (dfmi_row_classes > 0), so the solver matrices'
    8 B of owner/neighbour ids per face become 1 B per cell. hex_walk: the assembly kernels compute their
    face and neighbour indices (dfmi_hex_dims), so only cbStart (4 B per cell) and the coupled slots'
    9 B remain of the topology. face_form: the PCG reads the symmetric p operator face-wise (FaceOp): one
    coefficient per face (8 B) and the coupled-slot list (4 B per cell) instead of both ELL halves."""
    Sa = S - 1                                     # solved species (inert excluded)
    Bc = B if Bc is None else Bc
    topo = (4.0 * C + 9.0 * Bc) if hex_walk else (12.0 * C + 12.0 * F + 9.0 * Bc)
    mat = (C * 1.0 + F * 16.0) if classes else F * 24.0   # solver matrix per SpMV (values + indices)
    if kernel == "k_y_prep":
        # Y, hai, rhoD (S each), alpha, V in; sumYDiffError, hDiffCorrFlux (3 each), diffAlphaD out;
        # faces w, Sf, magSf, dc; coupled slots bw, bSf, bmagSf, bdc
        return C * 8.0 * (3 * S + 2) + C * 56.0 + F * 48.0 + Bc * 48.0 + topo
    if kernel in ("k_y_assemble_ell", "k_y_assemble"):
        # rhoD, Y, RR (S each), rho, rho_old, V in; per solved species W row values + dS + rhs out;
        # faces phi, phiUc, w, dc, magSf; coupled slots bphi, bphiUc, bw, bdc, bmagSf
        return C * 8.0 * (3 * S + 3) + Sa * C * (8.0 * W + 16.0) + F * 40.0 + Bc * 40.0 + topo
    if kernel == "k_u_grad":
        # U (3), mu, V in; mu*dev2(T(grad U)) (9) out; faces w, Sf; coupled slots bw, bSf
        return C * 40.0 + C * 72.0 + F * 32.0 + Bc * 32.0 + topo
    if kernel == "k_u_assemble":
        # rho, rho_old, U_old (3), mu, p, tau (9), V in; diag, source (3), source_solve (3), rAU out;
        # faces w, phi, dc, magSf, Sf in, lower/upper out; slots bphi, bw, bdc, bmagSf, bSf in, ic/bc (3 each) out
        return C * 136.0 + C * 64.0 + F * (56.0 + 16.0) + Bc * (56.0 + 48.0) + topo
    if kernel == "k_e_assemble":
        # he, rho, rho_old, K, K_old, alpha, hDiffCorrFlux (3), dpdt, diffAlphaD, V in; diag, source out;
        # faces phi, w, dc, magSf, Sf in, lower/upper out; slots bphi, bw, bdc, bmagSf, bSf in, ic/bc out
        return C * 104.0 + C * 16.0 + F * (56.0 + 16.0) + Bc * (56.0 + 16.0) + topo
    if kernel == "k_p_face":
        # pEqn face fluxes (phiHbyA, rhorAUf, the laplacian's lower = upper): cells rho, rAU, rho_old, U_old (3),
        # HbyA (3) in; faces own, nei, w, Sf (3), phi_old, deltaCoeffs, magSf in, 4 values out (no slots)
        return C * 72.0 + F * (8.0 + 56.0 + 32.0)
    if kernel == "k_u_hbya":
        # U (3), source (3), V in; HbyA (3) out; faces lower, upper; slots internal/boundaryCoeffs (3 each)
        return C * 56.0 + C * 24.0 + F * 16.0 + Bc * 48.0 + topo
    if kernel == "k_cg_spmv" and face_form:
        return C * 40.0 + C * 4.0 + F * 8.0 + Bc * 12.0
    if kernel == "k_cg_spmv":
        # fused PCG step p = z + beta p_old; q = A p: cells z, p_old, dS in, p, q out (40 B);
        # matrix: per internal face lower/upper values + owner/neighbour ids (24 B, LDU minimum; the
        # ELL gather stores the same 2 x 12 B per face from the two cells' sides); coupled slots 12 B
        return C * 40.0 + mat + Bc * 12.0
    if kernel in ("k_bcg_spmv", "k_bcg_eo"):
        # mean of the two SpMVs of an iteration: v = A p reads dS, p, r0, writes v (32 B / cell);
        # t = A s with s = r - alpha v formed on the fly reads dS, r, v, r0, writes t (40 B); matrix as above.
        # k_bcg_eo (even-odd reduced BiCGStab, k_eo_a..d): one application of the Schur complement S = two
        # half-row passes over the whole operator once; per iteration its four passes read dS twice (16 B),
        # move 56 B of vectors per cell (w = H p: p in, w out; v = p - H w: w, p, r0 in, v out; w2 = H s:
        # r, v in, w2 out; t = s - H w2: w2, r, v, r0 in, t out; each a half-length vector) and read the
        # operator twice -- 2 x (36 B per cell + matrix), the bytes of the two full SpMVs it replaces
        return C * 36.0 + mat + Bc * 12.0
    if kernel == "k_thermo_cells":
        # T, he, p, Y (S) in; T, he, psi, rho, mu, alpha, rhoD (S), hai (S) out
        return C * 8.0 * (3 + S) + C * 8.0 * (6 + 2 * S)
    raise KeyError(kernel)


SOLVER_KERNELS = ("k_bcg_spmv", "k_bcg_eo", "k_cg_spmv")
ASSEMBLY_KERNELS = ("k_y_assemble_ell", "k_y_prep", "k_u_grad", "k_u_assemble", "k_e_assemble", "k_u_hbya", "k_p_face")
ROOF_KERNELS = SOLVER_KERNELS + ASSEMBLY_KERNELS + ("k_thermo_cells",)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # the chemistry's per-cell step sizes and the solvers' poll cadence settle over the first few steps (the first
    # chemistry solves issue 2-6x the steady FLOPs, profiles/r05_pmc_flops.json): 5 untimed steps reach the steady state
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", "--cells-per-dir", dest="n", type=int, default=128, help="cells per direction (128 -> 2M cells)")
    ap.add_argument("--mech", default="burke9", choices=sorted(MECHS))
    ap.add_argument("--ncorr", type=int, default=2)
    ap.add_argument("--init", default="reference", choices=["reference", "tgv"],
                    help="initial state: the reference's own 64^3 TGV 0/ fields tiled (BASELINE config 3), or the "
                         "analytic TGV")
    ap.add_argument("--dt", type=float, default=1e-6)
    ap.add_argument("--kernel", default="auto",
                    help="kernel of the primary roofline entry (auto: the HBM-bound kernel with the most time)")
    ap.add_argument("--chem", default="ode", choices=["ode", "dnn", "off"],
                    help="chemistry source: stiff ODE integration per cell (BASELINE config 3), the DF-ODENet "
                         "surrogate (MFMA fp16, config 4's path on the H2 nets) or off")
    ap.add_argument("--renumber", default="none", choices=["bricks", "morton", "rcm", "none"],
                    help="cell order (dfmi_renumber_cells): blockMesh order (default: with the owner-slot face "
                         "storage its gathers are contiguous runs and it measured fastest), 8x8x4 bricks on a Z-order "
                         "curve, plain Morton, or reverse Cuthill-McKee")
    ap.add_argument("--traversal", default="none", choices=["bricks", "strips4", "strips8", "strips16", "none"],
                    help="visiting order of the gather kernels over the blockMesh-ordered data (dfmi_set_traversal)")
    ap.add_argument("--roof-steps", type=int, default=3, help="extra steps with per-kernel HIP events (rooflines)")
    ap.add_argument("--cpu-n", type=int, default=128, help="cells per direction of the CPU-A baseline sample")
    ap.add_argument("--cpu-steps", type=int, default=2, help="timed outer iterations of the CPU-A baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-flame", action="store_true", help="skip the BASELINE config 2 (1D flame) side line")
    ap.add_argument("--schemes", default="case", choices=["case", "gpu"],
                    help="convection schemes of div(phi,Yi_h) / div(phi,K) / div(hDiffCorrFlux): the case's own "
                         "(examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/system/fvSchemes: "
                         "limitedLinear01 / limitedLinear / cubic, what the reference CPU solver runs) or the "
                         "reference GPU path's hard-wired upwind / linear / linear; the other set is timed beside")
    ap.add_argument("--alt-steps", type=int, default=5, help="timed steps with the other scheme set (0: skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks and their mesh blocks, print the line's layout fields, touch no GPU "
                         "(tests of the launcher and the decomposition on CPU)")
    return ap.parse_args()


def spawn_ranks(n_gpus: int) -> int:
    """--gpus N > 1 started as a plain `python bench.py --gpus N` (no torchrun environment): launch the N ranks
    here, one process per GPU, exactly as the driver's torchrun command would (the reference binds one GPU per
    rank inside its own init, src_gpu/dfNcclBase.cu:23-65). This process never touches the GPU: it only waits
    for the children and returns their status; rank 0's JSON line goes straight to our stdout."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:   # a free rendezvous port on the loopback
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    # torchrun's own parser takes an abbreviation of its options even among the script's arguments ("--n" is
    # ambiguous with --nnodes / --nproc-per-node): hand the children the long spelling
    own = ["--cells-per-dir" + a[3:] if a == "--n" or a.startswith("--n=") else a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + own
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def case_schemes():
    """divSchemes of the headline case (committed as tests/golden/tgv64/fvSchemes)"""
    from dfmi.schemes import read_fv_schemes
    return read_fv_schemes(os.path.join(ROOT, "tests", "golden", "tgv64", "fvSchemes"))


def gpu_schemes():
    from dfmi.schemes import DEFAULT
    return dict(DEFAULT)


def cgroup_cpus():
    """CPUs the cgroup quota grants this process (cgroup v2 cpu.max, v1 cfs quota), None if unlimited"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def host_cpu():
    """(usable cores, machine cores, CPU model string) of this host (the lscpu 'Model name' field)"""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return len(os.sched_getaffinity(0)), os.cpu_count(), model


def cpu_baseline(args, table, ym, inert):
    """CPU-A: the build's OpenMP C++ implementation of the same step behind the
    same C ABI (baseline/cpu_a/libdfmi_cpu_a.so: the oracle's FV/thermo restatement with parallel gathers,
    Jacobi-BiCGStab and AMG-PCG at the GPU path's tolerances, ROS3 chemistry with the compiled-in
    kinetics), on every core OpenMP is given on this host (OMP_NUM_THREADS), on the headline's own
    workload: the cpu_n^3 box (default 128^3 = config 3) with the same initial state and chemistry.
    Bounded sample: one untimed step, then --cpu-steps timed steps."""
    from dfmi.lib import Context
    from dfmi.kinetics import parse_mechanism
    from dfmi.mesh import hex_box
    from dfmi import case
    path = os.path.join(ROOT, "baseline", "cpu_a", "libdfmi_cpu_a.so")
    n = args.cpu_n
    L = 2 * 3.141592653589793e-3
    m = hex_box(n, n, n, lengths=(L, L, L))
    ctx = Context(0, lib_path=path)
    case.setup_context(ctx, m, table, inert, args.dt, schemes=case_schemes() if args.schemes == "case" else gpu_schemes())
    if args.chem == "ode":
        ctx.chem_set_mechanism(parse_mechanism(os.path.join(ROOT, "tests", "golden", MECHS[args.mech][0])))
        ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    f = reference_fields(m, ym["species"]) if args.init == "reference" else case.tgv_fields(m, ym["species"])
    case.init_state(ctx, m, table.S, f["T"], f["p"], f["U"], f["Y"])
    ctx.time_step(args.ncorr)                      # untimed: first-touch allocations, chemistry step sizes
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        ctx.time_step(args.ncorr)
    el = time.perf_counter() - t0
    threads = int(ctx.lib.dfmi_version().decode().split("(OpenMP, ")[1].split(" ")[0])
    iters = {e: ctx.solver_stats(e)[0] for e in ("U", "Y", "E", "p")}
    ctx.close()
    # BASELINE.md section 2 also times configs 1 and 2 on CPU-A (same step definitions as the GPU lines)
    configs = {}
    if args.chem == "ode" and not args.no_flame:
        fl = flame1d_line(steps=20, warmup=2, lib_path=path)
        configs["config2_flame1d"] = {"cell_updates_per_s": fl["cell_updates_per_s"], "ms_per_step": fl["ms_per_step"],
                                      "steps": fl["steps"]}
        zd = zero_d_line(n_steps=200, lib_path=path)
        configs["config1_zeroD"] = {"chem_integrations_per_s": zd["chem_integrations_per_s"], "steps": 200,
                                    "T_end": zd["T_end"], "T_end_oracle": zd["T_end_oracle"]}
    usable, machine, model = host_cpu()
    quota = cgroup_cpus()
    chem = "ROS3 chemistry (rtol 1e-6, atol 1e-10)" if args.chem == "ode" else "no chemistry"
    value = m.n_cells * args.cpu_steps / el
    return {"value": value, "unit": "cell-updates/s", "cores": threads, "kind": "CPU-A",
            "value_per_core": value / threads,
            "sample": f"baseline/cpu_a (OpenMP C++, fp64, same ABI and step, {args.schemes} schemes) on {n}^3 = "
                      f"{m.n_cells} cells, {table.S} species, {chem}, {args.cpu_steps} timed outer iterations in "
                      f"{el:.1f} s after 1 untimed; last-step solver iterations {iters}",
            "host": {"omp_threads": threads, "affinity_cpus": usable, "nproc": machine, "model": model,
                     "cgroup_cpu_quota": quota, "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                     "OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"), "OMP_PLACES": os.environ.get("OMP_PLACES"),
                     "note": "threads = OMP_NUM_THREADS, the box's CPU share (gpurun sets it to 16 on the 1-GPU box "
                             "and forbids raising it); cgroup_cpu_quota is the kernel's quota for this process"},
            "configs": configs}


def reference_fields(m, species):
    """The reference example's initial state (examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/
    cvodeIntegrator/0, 64^3, committed under tests/golden/tgv64) tiled periodically over this
    rank's block of the global box (BASELINE config 3: 64^3 fields tiled 2x2x2 into 128^3)."""
    import numpy as np
    from dfmi.foam_io import read_case_fields
    src = read_case_fields(os.path.join(ROOT, "tests", "golden", "tgv64"), species)
    ii, jj, kk = m.local_index
    lnx, lny, lnz = m.block_dims
    rx, ry, rz = m.block
    gi, gj, gk = rx * lnx + ii, ry * lny + jj, rz * lnz + kk
    idx = (gi % 64) + 64 * ((gj % 64) + 64 * (gk % 64))
    return {"T": src["T"][idx], "p": src["p"][idx], "U": np.ascontiguousarray(src["U"][:, idx]),
            "Y": np.ascontiguousarray(src["Y"][:, idx])}


def host_state(m, table, f):
    """Initial state computed by the oracle's own thermo (no GPU) for the CPU baseline."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from dfmi import case
    C_, F, B, S = m.n_cells, m.n_faces, m.n_boundary_slots, table.S
    st = {}
    for nme in case.SCALARS:
        st[nme] = np.zeros(C_); st["boundary_" + nme] = np.zeros(B)
    for nme in case.VECTORS:
        st[nme] = np.zeros((3, C_)); st["boundary_" + nme] = np.zeros((3, B))
    for nme in case.SPECIES:
        st[nme] = np.zeros((S, C_)); st["boundary_" + nme] = np.zeros((S, B))
    for nme in case.FACES:
        st[nme] = np.zeros(F); st["boundary_" + nme] = np.zeros(B)
    st["T"] = f["T"].copy(); st["p"] = f["p"].copy(); st["U"] = f["U"].copy(); st["Y"] = f["Y"].copy()
    for k in ("T", "p", "U", "Y"):
        st["boundary_" + k] = case.boundary_values(m, st[k])
    o = O.Oracle(m, table, st, case.default_patch_types(m), 0, 1e7)
    o.thermo_correct(True)
    s = {k: v.copy() for k, v in o.arr.items() if k in st}
    s["phi"], s["boundary_phi"] = case.face_flux(m, s["rho"], s["U"], s["boundary_rho"], s["boundary_U"])
    s["K"] = 0.5 * (s["U"] ** 2).sum(axis=0)
    s["boundary_K"] = 0.5 * (s["boundary_U"] ** 2).sum(axis=0)
    return s


def flame1d_line(steps=100, warmup=10, lib_path=None):
    """BASELINE config 2: the reference's 1D H2/air flame (test/Tu500K-Phi1, 880 cells, 9 species,
    direct chemistry, dt 1e-6) on one GPU -- a latency-bound case (one wave of cells), reported
    beside the headline line, not as it."""
    from dfmi import case
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from dfmi.lib import Context
    golden = os.path.join(ROOT, "tests", "golden")
    ym = read_yaml_mechanism(os.path.join(golden, "Burke2012_s9r23.yaml"))
    t = read_thermo_table(os.path.join(golden, "thermo_Burke2012_s9r23.txt"), ym["species"])
    from dfmi.schemes import read_fv_schemes
    m = case.flame1d_mesh()
    ctx = Context(int(os.environ.get("LOCAL_RANK", "0")), lib_path=lib_path)
    # the case's own fvSchemes (test/Tu500K-Phi1/system/fvSchemes: limitedLinear01 / limitedLinear / cubic /
    # limitedLinearV for U), as the flame-speed regression runs it (tests/test_gpu_regression.py)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.flame1d_patch_types(m),
                       schemes=read_fv_schemes(os.path.join(golden, "flame1d", "fvSchemes")))
    ctx.chem_set_mechanism(parse_mechanism(os.path.join(golden, "Burke2012_s9r23.yaml")))
    ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    f, bv = case.flame1d_fields(os.path.join(golden, "flame1d"), ym["species"])
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"], bvals=bv,
                    gammas=case.flame1d_gamma(os.path.join(golden, "flame1d")))
    for _ in range(warmup):
        ctx.time_step(2)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.time_step(2)
    ctx.sync()
    el = time.perf_counter() - t0
    ctx.close()
    return {"workload": "1D freely-propagating H2/air flame (test/Tu500K-Phi1, its fvSchemes), 880 cells, Burke2012 9 species, "
                        "waveTransmissive outlet, direct integration, dt=1e-6, nCorr=2 (BASELINE config 2)",
            "ms_per_step": el / steps * 1e3, "cell_updates_per_s": m.n_cells * steps / el, "steps": steps}


def dnn53_line(m, T, p, steps=3, warmup=1):
    """BASELINE config 4's surrogate shape: 53 species, 52 DF-ODENet nets [55, 1600, 800, 400, 1]
    (the repository has no 53-species mechanism or trained nets: seeded N(0, 1/fan_in) weights, Dirichlet-like
    mass fractions, synthetic normalisation), on the headline's 2M-cell mesh and temperature field (cells at
    T >= 610 K infer). The FV kernels are instantiated for <= 16 species, so this line times the surrogate
    alone: chem-integrations/s = reacting cells inferred per second."""
    import numpy as np
    from dfmi import case, dnn_model
    from dfmi.lib import Context
    S = 53
    C = m.n_cells
    rng = np.random.default_rng(0)
    Y = rng.gamma(0.3, 1.0, (S, C))
    Y /= Y.sum(axis=0)
    Wm = 1.0 / (Y / np.linspace(2.0, 44.0, S)[:, None]).sum(axis=0)
    rho = p * Wm / (8314.46261815324 * T)
    ctx = Context(int(os.environ.get("LOCAL_RANK", "0")))
    pt = case.default_patch_types(m)
    rows, cols = m.proc_rows_cols()
    ctx.set_constant_values(C, C, m.n_faces, m.n_boundary_slots, m.n_patches, int(rows.size), m.patch_sizes, S, 1e6)
    ctx.set_cyclic_info(m.cyclic_neighbour())
    ctx.set_constant_indexes(m.owner, m.neighbour, rows, cols, 0)
    ctx.init_constant_fields_internal(m.sf, m.mag_sf, m.weight, m.delta_coeffs, m.volume, m.mesh_distance)
    bsf, bmag, bdc, bw, bfc = m.boundary_arrays()
    ctx.init_constant_fields_boundary(bsf, bmag, bdc, bw, bfc, pt["calculated"], pt["extrapolated"])
    ctx.set_inert_index(S - 1)
    dims = [S + 2, 1600, 800, 400, 1]
    ctx.dnn_set_model(dims, dnn_model.seeded_weights(n_modules=S - 1, dims=dims), np.zeros(S + 2), np.ones(S + 2),
                      np.zeros(S - 1), np.full(S - 1, 0.01))
    ctx.chem_set_options(2)
    for n_, v in (("T", T), ("p", p), ("rho", rho), ("Y", Y)):
        ctx.set_field(n_, v)
    del Y
    for _ in range(warmup):
        ctx.dnn_infer()
    ctx.kernel_timer("k_mlp_gemm")
    ctx.dnn_stats()
    ctx.sync()
    t0 = time.perf_counter()
    nr = 0
    for _ in range(steps):
        nr = ctx.dnn_infer()
    ctx.sync()
    el = time.perf_counter() - t0
    gemm_ms, gemm_n = ctx.kernel_time("k_mlp_gemm")
    _, flops = ctx.dnn_stats()
    ctx.close()
    tf = flops / (gemm_ms / 1e3) / 1e12 if gemm_ms > 0 else None
    return {"workload": "DF-ODENet surrogate alone, 53 species (52 nets [55,1600,800,400,1], seeded weights), "
                        "2097152-cell mesh with the headline T field (BASELINE config 4 shape)",
            "metric": "chem-integrations/s", "value": nr * steps / el, "reacting_cells": nr,
            "ms_per_inference": el / steps * 1e3, "gemm_ms_per_inference": gemm_ms / steps,
            "mfma_roofline": {"bound": "mfma", "achieved": tf, "peak": 2500.0, "unit": "TFLOP/s",
                              "frac": tf / 2500.0 if tf else None}}


def zero_d_line(n_steps=1000, lib_path=None):
    """BASELINE config 1: the reference df0DFoam case (examples/df0DFoam/zeroD_cubicReactor/H2/
    cvodeIntegrator: 10^3 cells of the same reactor, ES80_H2-7-16, T0 = 1000 K, 1 atm, dt 1e-6, 1000 steps,
    constant pressure) through dfmi_zero_d_step; chem-integrations/s = cells x steps / wall time."""
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from dfmi.lib import Context
    from dfmi import case
    import numpy as np
    golden = os.path.join(ROOT, "tests", "golden")
    ref = json.load(open(os.path.join(golden, "zeroD_cubicReactor.json")))
    ym = read_yaml_mechanism(os.path.join(golden, ref["mechanism"]))
    t = read_thermo_table(os.path.join(golden, "thermo_ES80_H2-7-16.txt"), ym["species"])
    m = hex_box(10, 10, 10, lengths=(5e-3,) * 3, periodic=(False,) * 3)
    ctx = Context(int(os.environ.get("LOCAL_RANK", "0")), lib_path=lib_path)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), ref["dt"])
    ctx.chem_set_mechanism(parse_mechanism(os.path.join(golden, ref["mechanism"])))
    ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    C = m.n_cells
    case.init_state(ctx, m, t.S, np.full(C, ref["T0"]), np.full(C, ref["p"]), np.zeros((3, C)),
                    np.repeat(np.asarray(ref["Y0"])[:, None], C, axis=1))
    t0 = time.perf_counter()
    ctx.zero_d_step(ref["dt"], n_steps)
    el = time.perf_counter() - t0
    T_end = float(ctx.get_field("T", (C,))[0])
    ctx.close()
    return {"workload": "df0DFoam zeroD_cubicReactor (reference example): 1000 identical cells, ES80 7 species, "
                        "T0=1000 K, p=1 atm, dt=1e-6, 1000 steps, constant pressure, rtol 1e-6 atol 1e-10",
            "ms_total": el * 1e3, "ms_per_step": el / n_steps * 1e3, "chem_integrations_per_s": C * n_steps / el,
            "T_end": T_end, "T_end_oracle": ref["T"][n_steps] if n_steps <= ref["n_steps"] else None}


def config4_line(m, T, U, p, steps=3, warmup=1):
    """BASELINE config 4 as a full dfLowMachFoam step: the 2M-cell box with 53 species (SURVEY 8d synthetic
    table: gri30's 36 species fitted by dfmi.transport_fit, cycled to 53, N2 last; Dirichlet-like mass
    fractions blended by the hot kernel's progress) and the DF-ODENet surrogate (52 seeded nets
    [55,1600,800,400,1]) as the chemistry source."""
    import numpy as np
    from dfmi.mech import read_thermo_table
    from dfmi.lib import Context
    from dfmi import case
    from dfmi.synthetic import gri53_species, gri53_smooth_fractions, gri53_dnn
    golden = os.path.join(ROOT, "tests", "golden")
    sp = gri53_species(os.path.join(golden, "gri30.yaml"))
    t = read_thermo_table(os.path.join(golden, "thermo_gri53_synthetic.txt"), sp)
    ctx = Context(int(os.environ.get("LOCAL_RANK", "0")))
    case.setup_context(ctx, m, t, sp.index("N2"), 1e-6, schemes=case_schemes())
    gri53_dnn(ctx)
    ctx.chem_set_options(2)
    case.init_state(ctx, m, t.S, T, p, U, gri53_smooth_fractions((T - T.min()) / max(np.ptp(T), 1.0)))
    for _ in range(warmup):
        ctx.time_step(2)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.time_step(2)
    ctx.sync()
    el = time.perf_counter() - t0
    iters = {e: ctx.solver_stats(e)[0] for e in ("U", "Y", "E", "p")}
    nr = ctx.dnn_stats()[0]
    ctx.close()
    return {"workload": f"dfLowMachFoam 3D periodic box {m.n_cells} cells, 53 species (synthetic GRI table), "
                        "DF-ODENet surrogate source (52 nets, fp16 MFMA), nCorr=2, dt=1e-6 (BASELINE config 4)",
            "metric": "cell-updates/s", "value": m.n_cells * steps / el, "ms_per_step": el / steps * 1e3,
            "steps": steps, "reacting_cells": nr, "solver_iters": iters}


def comm_block(local, step_ms, steps, world, rank):
    """The multi-GPU line's communication block: every rank's per-exchange-point accounting
    (dfmi_comm_report: HIP-event time of the transport calls -- ncclSend/ncclRecv groups of the halo
    exchanges, ncclAllGather of the solver reductions -- and the bytes each rank sends) over the roofline
    pass, gathered to rank 0. Per point: calls and bytes per step, time per step (max / mean over ranks);
    totals against the step time of the same pass. DESIGN.md 7 states the rule the overlap decision follows."""
    import torch.distributed as dist
    every = [None] * world
    dist.all_gather_object(every, {"rank": rank, "points": local, "step_ms": step_ms})
    if rank != 0:
        return None
    names = sorted({k for e in every for k in e["points"]})
    pts = {}
    for k in names:
        ms = [e["points"].get(k, {}).get("ms", 0.0) / steps for e in every]
        by = [e["points"].get(k, {}).get("bytes", 0.0) / steps for e in every]
        calls = [e["points"].get(k, {}).get("calls", 0) / steps for e in every]
        pts[k] = {"calls_per_step": max(calls), "bytes_per_step_max": max(by),
                  "bytes_per_call": max(by) / max(max(calls), 1e-30),
                  "ms_per_step_max": max(ms), "ms_per_step_mean": sum(ms) / world}
    tot = [sum(v.get("ms", 0.0) for v in e["points"].values()) / steps for e in every]
    halo = [sum(v.get("ms", 0.0) for n, v in e["points"].items() if not n.startswith("allgather")) / steps for e in every]
    solver = [sum(v.get("ms", 0.0) for n, v in e["points"].items()
                  if n.split(" ")[0] in ("bicgstab", "pcg") or n.startswith("allgather")) / steps for e in every]
    step = max(e["step_ms"] for e in every)
    return {"source": "dfmi_comm_report: HIP events around every transport call on the stream it ran on, "
                      f"{steps} roofline-pass steps (kernel timers armed too)",
            "overlap": os.environ.get("DFMI_HALO_OVERLAP", "0"),
            "step_ms": step,
            "comm_ms_per_step": {"max": max(tot), "per_rank": tot},
            "halo_ms_per_step_max": max(halo), "allgather_ms_per_step_max": max(tot[i] - halo[i] for i in range(world)),
            "solver_comm_ms_per_step_max": max(solver),
            "fraction_of_step": max(tot) / step if step > 0 else None,
            "points": pts}


def chem_step_stats(ctx, C):
    """Integrator steps per cell of the last chemistry solve and how evenly 64-lane waves are loaded:
    a wave costs its slowest lane, so efficiency = mean cost / mean of per-wave max cost, in natural
    cell order and in the descending-cost order the binned launch approximates."""
    import numpy as np
    st = ctx.get_field("chem_stats", (3, C))[:2]
    cost = np.maximum(st[0], 0) + st[1]
    pad = (-C) % 64
    nat = np.concatenate([cost, np.zeros(pad)]).reshape(-1, 64).max(axis=1).mean()
    srt = np.concatenate([np.sort(cost)[::-1], np.zeros(pad)]).reshape(-1, 64).max(axis=1).mean()
    # binning unit = groups of 8 consecutive cells by their most expensive cell (chem.hip GRP = 8, measured slower)
    g = np.concatenate([cost, np.zeros((-C) % 8)]).reshape(-1, 8)
    gs = g[np.argsort(-g.max(axis=1), kind="stable")]
    gs = np.concatenate([gs, np.zeros(((-len(gs)) % 8, 8))]).reshape(-1, 64)
    grp = gs.max(axis=1).mean()
    # chem.binning = 2: cells sorted inside each tile of 4096
    t = np.concatenate([cost, np.zeros((-C) % 4096)]).reshape(-1, 4096)
    tile = (-np.sort(-t, axis=1)).reshape(-1, 64).max(axis=1).mean()
    return {"steps_mean": float(st[0].mean()), "rejects_mean": float(st[1].mean()), "steps_max": float(cost.max()),
            "wave_eff_natural": float(cost.mean() / nat) if nat else None,
            "wave_eff_sorted": float(cost.mean() / srt) if srt else None,
            "wave_eff_groups_of_8": float(cost.mean() / grp) if grp else None,
            "wave_eff_tiles_4096": float(cost.mean() / tile) if tile else None}


def decomposition(world: int):
    """decomposePar blocks of the weak-scaling box: 2x1x1 / 2x2x1 / 2x2x2 (N = 8 is BASELINE config 5)"""
    return {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}.get(world, (world, 1, 1))


def rank_block(n: int, decomp, rank: int):
    """this rank's n^3 block of the (n d0) x (n d1) x (n d2) periodic 2 pi mm-per-block box"""
    from dfmi.mesh import hex_box
    L = 6.283185307179586e-3
    return hex_box(n * decomp[0], n * decomp[1], n * decomp[2], lengths=(L * decomp[0], L * decomp[1], L * decomp[2]),
                   decomp=decomp, rank=rank)


def dry_run(args, world: int, rank: int):
    """the launcher and layout without a GPU: every rank builds its block and its processor patches, rank 0
    prints the fields of the line that describe them"""
    import torch.distributed as dist
    decomp = decomposition(world)
    m = rank_block(args.n, decomp, rank)
    mine = {"rank": rank, "cells": m.n_cells, "proc_faces": int(m.proc_rows_cols()[0].size),
            "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}
    every = [mine]
    if world > 1:
        every = [None] * world
        dist.all_gather_object(every, mine)
    if rank == 0:
        print(json.dumps({"metric": "cell-updates/s (dfLowMachFoam outer iter)", "dry_run": True, "n_gpus": world,
                          "scaling": "weak",
                          "config": {"cells_per_gpu": m.n_cells, "cells_total": sum(e["cells"] for e in every),
                                     "parallelism": parallelism(decomp, world)},
                          "ranks": every}), flush=True)


def parallelism(decomp, world: int) -> str:
    return (f"domain decomposition {decomp[0]}x{decomp[1]}x{decomp[2]}, RCCL halo" if world > 1 else "single")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))           # before anything touches the GPU: the parent only waits
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; the world size decides",
              file=sys.stderr)
    import numpy as np
    import torch                                   # loads the HIP runtime first: one runtime per process
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
        dry_run(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    if world > 1 and os.environ.get("DFMI_RCCL_SPLIT_HOSTS"):
        # rehearsal of the multi-GPU path on a box with fewer GPUs than ranks: each rank poses as its own
        # host (RCCL then connects the ranks through sockets instead of refusing two ranks per device);
        # the timing of such a run says nothing about xGMI scaling
        os.environ["NCCL_HOSTID"] = f"dfmi-bench-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.lib import Context
    from dfmi import case
    golden = os.path.join(ROOT, "tests", "golden")
    yml, tab = MECHS[args.mech]
    ym = read_yaml_mechanism(os.path.join(golden, yml))
    table = read_thermo_table(os.path.join(golden, tab), ym["species"])
    inert = ym["species"].index("N2")

    n = args.n
    decomp = decomposition(world)
    m = rank_block(n, decomp, rank)
    if args.renumber != "none":   # renumberMesh's role: cells in Morton bricks, faces re-sorted
        from dfmi.renumber import renumber_mesh
        m, _ = renumber_mesh(m, args.renumber)
    ctx = Context(local)
    comm = None
    if world > 1:
        uid = [Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = {"uid": uid[0], "nranks": world, "rank": rank}
    schemes = case_schemes() if args.schemes == "case" else gpu_schemes()
    alt_schemes = gpu_schemes() if args.schemes == "case" else case_schemes()
    case.setup_context(ctx, m, table, inert, args.dt, comm=comm, schemes=schemes)
    if args.traversal == "bricks" and hasattr(m, "local_index"):
        from dfmi.lib import renumber_cells
        ijk = np.stack(m.local_index, axis=1).astype(np.float64)
        ctx.set_traversal(renumber_cells(m.n_cells, ijk, m.owner, m.neighbour, "bricks"))
    elif args.traversal.startswith("strips") and hasattr(m, "local_index"):
        # y-strips of R full x-rows swept through z: the working set of a z-sweep (3 planes of one strip)
        # stays in an XCD's L2, rows stay whole cache lines
        i, j, k = (np.asarray(a) for a in m.local_index)
        R = int(args.traversal[6:])
        ctx.set_traversal(np.lexsort((i, j, k, j // R)).astype(np.int32))
    if args.chem == "ode":
        from dfmi.kinetics import parse_mechanism
        ctx.chem_set_mechanism(parse_mechanism(os.path.join(golden, yml)))
        ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)   # reference CVODE tolerances
    elif args.chem == "dnn":
        from dfmi import dnn_model
        dnn_model.configure(ctx)
        ctx.chem_set_options(2)
    if args.init == "reference":
        f = reference_fields(m, ym["species"])
    else:
        f = case.tgv_fields(m, ym["species"])
    case.init_state(ctx, m, table.S, f["T"], f["p"], f["U"], f["Y"])
    T0, p0 = f["T"].copy(), f["p"].copy()
    del f

    for e in ("U", "Y", "E", "p"):
        ctx.solver_work(e, reset=True)             # work counts of the whole run (profiles/: frac from rocprof)
    for _ in range(args.warmup):
        ctx.time_step(args.ncorr)
    ctx.sync()
    if world > 1:
        dist.barrier()
    # ---- headline: K steps; only an event on the context stream after every step (dfmi_step_timer, no sync)
    ctx.step_timer(True)
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.time_step(args.ncorr)
    ctx.sync()                                     # the context's stream (all the step's work)
    torch.cuda.synchronize(local)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = t1 - t0
    step_ms = ctx.step_times(args.steps)
    ctx.step_timer(False)
    med = float(np.median(step_ms)) if step_ms.size else float("nan")
    if world > 1:
        tt = torch.tensor([el, med], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el, med = float(tt[0].item()), float(tt[1].item())
    stats = {e: ctx.solver_stats(e) for e in ("U", "Y", "E", "p")}

    # ---- roofline pass: the same step, HIP events around every launch of the measured kernels and the
    # solver work counted on the device (after the headline, so the instrumentation never inflates it)
    extra = {"ode": ["k_chem", "k_bin"], "dnn": ["k_mlp_gemm"], "off": []}[args.chem]
    ctx.kernel_timer(",".join(ROOF_KERNELS + tuple(extra)))
    work_pre = {e: ctx.solver_work(e, reset=True) for e in ("U", "Y", "E", "p")}
    if args.chem == "dnn":
        ctx.dnn_stats()
    if world > 1:
        ctx.comm_timer(True)                       # per-exchange-point transport time and bytes (this pass only)
    tr0 = time.perf_counter()
    for _ in range(args.roof_steps):
        ctx.time_step(args.ncorr)
    ctx.sync()
    roof_ms = (time.perf_counter() - tr0) / max(args.roof_steps, 1) * 1e3
    comm = None
    if world > 1:
        comm = comm_block(ctx.comm_report(), roof_ms, args.roof_steps, world, rank)
        ctx.comm_timer(False)
    ktime = {k: ctx.kernel_time(k) for k in ROOF_KERNELS}
    work = {e: ctx.solver_work(e) for e in ("U", "Y", "E", "p")}
    chem_ms, chem_n = ctx.kernel_time("k_chem") if args.chem == "ode" else (0.0, 0)
    bin_ms, _ = ctx.kernel_time("k_bin") if args.chem == "ode" else (0.0, 0)
    gemm_ms, gemm_n = ctx.kernel_time("k_mlp_gemm") if args.chem == "dnn" else (0.0, 0)
    n_react, gemm_flops = ctx.dnn_stats() if args.chem == "dnn" else (0, 0.0)
    ctx.kernel_timer("")
    T = ctx.get_field("T", (m.n_cells,))
    finite = bool(np.isfinite(T).all())
    # ---- the other scheme set, timed the same way beside the headline (same state, K = alt_steps)
    alt = None
    if args.alt_steps > 0:
        for term, sch in alt_schemes.items():
            ctx.set_scheme(term, sch)
        ctx.time_step(args.ncorr)
        ctx.sync()
        if world > 1:
            dist.barrier()
        ta = time.perf_counter()
        for _ in range(args.alt_steps):
            ctx.time_step(args.ncorr)
        ctx.sync()
        ea = time.perf_counter() - ta
        if world > 1:
            tt = torch.tensor([ea], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ea = float(tt.item())
        alt = {"schemes": alt_schemes, "steps": args.alt_steps, "ms_per_step": ea / args.alt_steps * 1e3,
               "value": m.n_cells * world * args.alt_steps / ea}
        for term, sch in schemes.items():
            ctx.set_scheme(term, sch)
    # ---- several ranks: the other setting of the overlapped solver halos (option halo.overlap, read per solve),
    # timed beside the headline the same way, so one multi-GPU run decides DESIGN.md 7's rule from its own numbers
    ovl = None
    if world > 1 and args.alt_steps > 0:
        cur = ctx.get_option("halo.overlap")
        ctx.set_option("halo.overlap", 0.0 if cur else 1.0)
        ctx.time_step(args.ncorr)
        ctx.sync()
        dist.barrier()
        ta = time.perf_counter()
        for _ in range(args.alt_steps):
            ctx.time_step(args.ncorr)
        ctx.sync()
        eo_ = time.perf_counter() - ta
        tt = torch.tensor([eo_], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        eo_ = float(tt.item())
        ctx.set_option("halo.overlap", cur)
        ovl = {"halo_overlap": 0 if cur else 1, "headline_halo_overlap": int(cur), "steps": args.alt_steps,
               "ms_per_step": eo_ / args.alt_steps * 1e3, "value": m.n_cells * world * args.alt_steps / eo_,
               "speedup_vs_headline": (el / args.steps) / (eo_ / args.alt_steps)}

    ncls = ctx.row_classes()
    hexd = ctx.hex_dims()
    opt_face_hex = ctx.get_option("fv.hex_walk") != 0 and ctx.get_option("fv.csr_walk") == 0
    opt_face_form = ctx.get_option("pcg.face_form") != 0
    hexw = hexd[0] > 0 and opt_face_hex
    cells_total = m.n_cells * world
    value = cells_total * args.steps / el
    # HBM bytes per launch from the PMC passes committed under profiles/ (scripts/pmc_traffic.sh +
    # scripts/pmc_summary.py: (2 FETCH_SIZE + WRITE_SIZE) KB, gfx950 correction), same workload
    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", PMC_FILE)
    if os.path.exists(pmc_path) and n == 128 and world == 1:
        tab = json.load(open(pmc_path))
        for fam in ROOF_KERNELS:
            # every instantiation of the family (k_bcg_spmv -> k_bcg_spmv1<6>, k_bcg_spmv2<6>); variants
            # moving < 1 % of the largest one's bytes are other workloads' (the 1D flame line's W = 2)
            ent = [v for key, v in tab.items()
                   if key.split("::")[-1].split("<")[0].rstrip("12") == fam or key.split("::")[-1].startswith(fam + "<")
                   or key.split("::")[-1].split("(")[0] == fam + "_cell"   # k_p_face's cell-walk form
                   or key.split("::")[-1].startswith(fam + "_brick<")      # k_y_prep's LDS-staged form
                   or (fam == "k_bcg_eo" and key.split("::")[-1][:7] in ("k_eo_a<", "k_eo_b<", "k_eo_c<", "k_eo_d<"))]
            if not ent:
                continue
            top = max(v["hbm_bytes_mean"] for v in ent)
            ent = [v for v in ent if v["hbm_bytes_mean"] >= 0.01 * top]
            nd = sum(v["dispatches"] for v in ent)
            pmc[fam] = {"hbm_bytes_mean": sum(v["hbm_bytes_mean"] * v["dispatches"] for v in ent) / nd}
    # FP64 FLOPs per dispatch of the VALU-bound kernels (thermo, chemistry) from the committed PMC pass of the same
    # workload: their roofline is counted FLOPs / the FP64 vector peak, not bytes / the HBM peak
    flops_tab = {}
    fl_path = os.path.join(ROOT, "profiles", PMC_FLOPS_FILE)
    if os.path.exists(fl_path) and n == 128 and world == 1:
        for key, v in json.load(open(fl_path)).items():
            short = key[len("dfmi::"):] if key.startswith("dfmi::") else key   # (template arguments hold "::" too)
            for fam in ("k_thermo_cells", "k_chem"):
                if short.startswith(fam + "<") or short.startswith(fam + "_gen<"):
                    fl = v.get("flops_steady", v["flops"])   # the last (roofline-pass) dispatches, not the cold solves
                    if fl > flops_tab.get(fam, {}).get("flops", -1.0):
                        flops_tab[fam] = {"flops": fl, "kernel": key,
                                          "statistic": "steady (mean of the last dispatches)" if "flops_steady" in v
                                          else "mean over all dispatches"}
    Bc = m.n_coupled_slots
    # BiCGStab: two operator applications per system-iteration, full SpMVs (k_bcg_spmv) or applications of
    # the even-odd Schur complement (k_bcg_eo); only one of the two runs
    units = {"k_bcg_spmv": 2.0 * (work["U"] + work["Y"] + work["E"]), "k_bcg_eo": 2.0 * (work["U"] + work["Y"] + work["E"]),
             "k_cg_spmv": work["p"]}
    for k in ASSEMBLY_KERNELS + ("k_thermo_cells",):
        units[k] = float(ktime[k][1])              # one unit = one launch
    roofs = {}
    for k in ROOF_KERNELS:
        ms, nl = ktime[k]
        if not nl or ms <= 0:
            continue
        # algorithmic bytes: SURVEY 8(d)'s definition (unstructured LDU: int32 owner/neighbour ids per face
        # included), comparable across rounds; impl: the index bytes the kernels actually read (row classes,
        # computed hex walk), the floor of this implementation's traffic
        per_unit = algorithmic_bytes(k, m.n_cells, m.n_faces, m.n_boundary_slots, table.S, Bc)
        per_impl = algorithmic_bytes(k, m.n_cells, m.n_faces, m.n_boundary_slots, table.S, Bc, classes=ncls > 0,
                                     hex_walk=hexw, face_form=hexw and world == 1
                                     and opt_face_form)
        total_bytes = per_unit * units[k]
        total_impl = per_impl * units[k]
        if k in ("k_bcg_spmv", "k_bcg_eo"):   # U's three components share one operator: its bytes count once per three systems
            total_bytes -= 2.0 * work["U"] * (2.0 / 3.0) * (24.0 * m.n_faces + 12.0 * Bc)
            total_impl -= 2.0 * work["U"] * (2.0 / 3.0) * ((1.0 * m.n_cells + 16.0 * m.n_faces if ncls > 0 else
                                                             24.0 * m.n_faces) + 12.0 * Bc)
        achieved = total_bytes / (ms / 1e3) / 1e9
        achieved_impl = total_impl / (ms / 1e3) / 1e9
        tr = pmc.get(k)
        roofs[k] = {"kernel": k, "bound": "hbm",
                    "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS,
                    "traffic": tr["hbm_bytes_mean"] if tr else None,
                    "algorithmic_bytes": total_bytes / nl, "launches": nl, "work_units": units[k],
                    "bytes_per_unit": per_unit, "avg_us": ms * 1e3 / nl, "total_ms": ms,
                    "impl_bytes": total_impl / nl, "frac_impl": achieved_impl / HBM_PEAK_GBS}
        if k == "k_thermo_cells":   # FP64-VALU bound: counted FLOPs against the FP64 vector peak
            fl = flops_tab.get(k)
            tfs = fl["flops"] * nl / (ms / 1e3) / 1e12 if fl else None
            roofs[k].update({"bound": "fp64-valu", "unit": "TFLOP/s", "peak": FP64_PEAK_TFS, "achieved": tfs,
                             "frac": tfs / FP64_PEAK_TFS if tfs is not None else None,
                             "flops_per_launch": fl["flops"] if fl else None,
                             "flops_source": f"profiles/{PMC_FLOPS_FILE} (64 x SQ_INSTS_VALU_FLOPS_FP64 per dispatch, mean; = 64 (ADD + MUL + TRANS + 2 FMA) wave-instructions)"
                             if fl else "no PMC FLOP counts for this workload",
                             "hbm_achieved_GBs": achieved, "hbm_frac": achieved / HBM_PEAK_GBS})
    hbm = {k: v for k, v in roofs.items() if v["bound"] == "hbm"}
    # the north star's face-flux assembly item as one number (achieved = sum of the assembly kernels'
    # algorithmic bytes / (sum of their kernel time x 8 TB/s)), with the PMC traffic of the same kernels beside it
    asm = [k for k in ASSEMBLY_KERNELS if k in roofs]
    asm_bytes = sum(roofs[k]["algorithmic_bytes"] * roofs[k]["launches"] for k in asm)
    asm_ms = sum(roofs[k]["total_ms"] for k in asm)
    asm_traffic = (sum(roofs[k]["traffic"] * roofs[k]["launches"] for k in asm) / asm_bytes
                   if asm and all(roofs[k]["traffic"] for k in asm) else None)
    assembly_roofline = ({"kernels": asm, "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                          "achieved": asm_bytes / (asm_ms / 1e3) / 1e9, "frac": asm_bytes / (asm_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                          "algorithmic_bytes_per_step": asm_bytes / max(args.roof_steps, 1),
                          "kernel_ms_per_step": asm_ms / max(args.roof_steps, 1),
                          "traffic_over_algorithmic": asm_traffic,
                          "per_kernel_frac": {k: roofs[k]["frac"] for k in asm}} if asm and asm_ms > 0 else None)
    primary = args.kernel if args.kernel != "auto" else (max(hbm, key=lambda k: hbm[k]["total_ms"]) if hbm else None)
    out = {
        "metric": "cell-updates/s (dfLowMachFoam outer iter)",
        "value": value,
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "ms_per_step_median": med,
        "ms_per_step_events": {"min": float(step_ms.min()) if step_ms.size else None,
                               "max": float(step_ms.max()) if step_ms.size else None,
                               "mean": float(step_ms.mean()) if step_ms.size else None,
                               "note": "HIP events on the context stream after every timed step (rank 0's; the "
                                       "median is the max over ranks); ms_per_step is the bracketed wall time / K"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("reference initial fields (examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/0, "
                 "64^3, committed as tests/golden/tgv64) tiled over a hex box generated in-process"
                 if args.init == "reference" else "synthetic analytic TGV on a hex box generated in-process"),
        "config": {"workload": f"dfLowMachFoam 3D periodic box {n * decomp[0]}x{n * decomp[1]}x{n * decomp[2]} = "
                               f"{cells_total} hex cells ({m.n_cells} per GPU), H2/air {table.S} species "
                               f"({args.mech}), nOuter=1 nCorr={args.ncorr}, dt={args.dt}",
                   "cells_per_gpu": m.n_cells, "species": table.S, "cell_order": args.renumber,
                   "schemes": schemes, "schemes_source": ("the case's system/fvSchemes (tests/golden/tgv64/fvSchemes)"
                                                          if args.schemes == "case" else
                                                          "the reference GPU path's hard-wired upwind/linear"),
                   "traversal": args.traversal,
                   "parallelism": parallelism(decomp, world)},
        "roofline": None if primary is None else dict(roofs[primary], traffic_source=f"profiles/{PMC_FILE} (rocprofv3 --pmc FETCH_SIZE / "
                         "WRITE_SIZE passes, mean per dispatch, gfx950 read correction)",
                         note=f"achieved = algorithmic bytes of the work done (active systems/iterations; SURVEY 8(d): "
                              f"int32 ids per face counted) / summed HIP-event kernel time over {args.roof_steps} extra "
                              "steps after the timed region (the headline runs with no events armed; while they are "
                              "armed the step's side stream is folded into the main one, so each kernel is timed "
                              "alone); algorithmic_bytes "
                              "and traffic are per launch; impl_bytes / frac_impl: the bytes this implementation must "
                              "move (gather rows decoded from row classes: 1 B per cell instead of the ids)"),
        "rooflines": {k: {kk: v[kk] for kk in ("bound", "unit", "peak", "achieved", "frac", "traffic", "algorithmic_bytes",
                                               "avg_us", "launches", "impl_bytes", "frac_impl", "flops_per_launch",
                                               "hbm_frac") if kk in v} for k, v in roofs.items()},
        "solver_iters": {e: s[0] for e, s in stats.items()},
        "solver_work_roof_pass": work,
        "solver_work_run": {"system_iterations": {e: work_pre[e] + work[e] for e in work},
                            "time_steps": args.warmup + args.steps + args.roof_steps,
                            "note": "every solve of this process's time steps (warmup + timed + roof pass): with a "
                                    "rocprofv3 --stats summary of the same command, frac = bytes_per_unit x units / "
                                    "summed kernel time (scripts/roof_from_profile.py)",
                            "bytes_per_unit": {k: algorithmic_bytes(k, m.n_cells, m.n_faces, m.n_boundary_slots,
                                                                    table.S, m.n_coupled_slots)
                                               for k in ("k_bcg_spmv", "k_cg_spmv")},
                            # U's shared operator: each U SpMV's matrix bytes count one third
                            "u_matrix_bytes": 24.0 * m.n_faces + 12.0 * m.n_coupled_slots},
        "amg_levels": ctx.amg_info(),
        "row_classes": ncls,
        "hex_face_walk": list(hexd) if hexw else None,
        "chemistry": ({"integrator": "ROS3 Rosenbrock (order 3, adaptive), rtol 1e-6 atol 1e-10",
                       "chem_integrations_per_s": m.n_cells * world * chem_n / (chem_ms / 1e3) if chem_n else None,
                       "k_chem_ms_per_step": chem_ms / max(chem_n, 1),
                       "valu_roofline": ({"bound": "fp64-valu", "unit": "TFLOP/s", "peak": FP64_PEAK_TFS,
                                          "flops_per_launch": flops_tab["k_chem"]["flops"],
                                          "achieved": flops_tab["k_chem"]["flops"] * chem_n / (chem_ms / 1e3) / 1e12,
                                          "frac": flops_tab["k_chem"]["flops"] * chem_n / (chem_ms / 1e3) / 1e12 / FP64_PEAK_TFS,
                                          "kernel": flops_tab["k_chem"]["kernel"],
                                          "statistic": flops_tab["k_chem"]["statistic"],
                                          "flops_source": f"profiles/{PMC_FLOPS_FILE}"}
                                         if "k_chem" in flops_tab and chem_n else None),
                       "k_bin_ms_per_step": bin_ms / max(chem_n, 1),
                       **chem_step_stats(ctx, m.n_cells)} if args.chem == "ode" else None),
        "dnn": ({"reacting_cells": n_react, "gemm_launches": gemm_n, "gemm_ms_total": gemm_ms,
                 "mfma_roofline": {"bound": "mfma", "achieved": gemm_flops / (gemm_ms / 1e3) / 1e12,
                                   "peak": 2500.0, "unit": "TFLOP/s",
                                   "frac": gemm_flops / (gemm_ms / 1e3) / 1e12 / 2500.0},
                 "inferences_per_s_gemm_time": n_react * args.roof_steps / (gemm_ms / 1e3)}
                if args.chem == "dnn" and gemm_ms > 0 else None),
        "assembly_roofline": assembly_roofline,
        "finite": finite,
        "other_schemes": alt,
    }
    if ovl is not None:
        out["other_halo_overlap"] = ovl
    if comm is not None:
        out["comm"] = comm
    if world == 1 and out["roofline"] is not None:   # the headline kernel against a measured copy peak as well
        peak_copy = ctx.hbm_copy_peak(4.0, 20)     # dfmi_hbm_copy_peak: 16-B vector streaming copy
        out["roofline"]["measured_copy_peak_GBs"] = peak_copy
        out["roofline"]["frac_of_measured_copy_peak"] = out["roofline"]["achieved"] / peak_copy
    U0 = ctx.get_field("U", (3, m.n_cells)) if (rank == 0 and world == 1 and n == 128 and not args.no_flame) else None
    ctx.close()
    if rank == 0 and world == 1 and n == 128 and not args.no_flame:
        out["other_configs"] = {"config1_zeroD": zero_d_line(), "config2_flame1d": flame1d_line(),
                                "config4_gri53_dnn": config4_line(m, T0, U0, p0), "dnn53_surrogate": dnn53_line(m, T0, p0)}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args, table, ym, inert)
        out["cpu_baseline"]["ratio"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
