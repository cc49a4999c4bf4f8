/* dfmi.h -- C ABI of the MI355X-native dfLowMachFoam GPU hot path.
 *
 * Drop-in replacement for the C++ class surface of the reference libdfMatrix.so
 * (show-me-code/deepflame-dev src_gpu/ *.H headers, driven from applications/solvers/dfLowMachFoam/
 * createGPUSolver.H and *_GPU.H). Each entry point names the reference method it replaces.
 *
 * Conventions (same as the reference):
 *  - host arrays are copied during the call, never retained;
 *  - vector/tensor fields: layout DFMI_AOS = OpenFOAM [n][3] / [n][9] (the reference permutes
 *    with permute_vector_h2d, dfMatrixOpBase.cu:18-38), DFMI_SOA = [3][n] / [9][n];
 *  - species fields are species-major [S][n] (createGPUSolver.H:482-500);
 *  - boundary arrays are concatenated in OpenFOAM patch order; a processor/processorCyclic patch
 *    takes 2n slots [neighbour values | patch-internal values] (createGPUSolver.H:118-123);
 *  - patch type codes: zeroGradient 0, fixedValue 1, coupled 2, empty 3, gradientEnergy 4,
 *    calculated 5, cyclic 6, processor 7, extrapolated 8, fixedEnergy 9, processorCyclic 10
 *    (dfMatrixDataBase.H:81-93), plus waveTransmissive 11 (p only; gamma via dfmi_set_patch_param,
 *    OpenFOAM-7 advectiveFvPatchField semantics with Euler ddt) and inletOutlet 12 (U, p, Y, K;
 *    inletValue in the field "boundary_<field>_ref") -- the mixed conditions the reference GPU path
 *    rejects (dfMatrixDataBase.cu:22-27) though its own 1D-flame case uses one (test/Tu500K-Phi1/0/p);
 *  - every call returns 0 on success, non-zero on error, and never exits the process
 *    (the reference exit()s, dfMatrixDataBase.H:40-50); dfmi_last_error() gives the message.
 */
#ifndef DFMI_H
#define DFMI_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dfmi_ctx dfmi_ctx;

enum { DFMI_SOA = 0, DFMI_AOS = 1 };

/* ---- lifetime ------------------------------------------------------------------------- */
/* dfMatrixDataBase(), prepareCudaResources (dfMatrixDataBase.cu:88,103): binds `device`, one stream */
int dfmi_create(dfmi_ctx** ctx, int device);
/* ~dfMatrixDataBase + cleanCudaResources (dfMatrixDataBase.cu:90,107); frees all device memory */
int dfmi_destroy(dfmi_ctx* ctx);
/* copy of the last error message of this thread; returns its length */
int dfmi_last_error(char* buf, int len);
/* library version string */
const char* dfmi_version(void);

/* ---- dfMatrixDataBase setup (createGPUBase, createGPUSolver.H:103-351) ------------------- */
/* dfMatrixDataBase::setConstantValues (dfMatrixDataBase.cu:114-147); rdelta_t = 1/deltaT */
int dfmi_set_constant_values(dfmi_ctx* ctx, int num_cells, int num_total_cells, int num_surfaces,
                             int num_boundary_surfaces, int num_patches, int num_proc_surfaces,
                             const int* patch_size, int num_species, double rdelta_t);
/* dfMatrixDataBase::setCyclicInfo (dfMatrixDataBase.cu:179-182): partner patch index or -1 */
int dfmi_set_cyclic_info(dfmi_ctx* ctx, const int* cyclic_neighbor);
/* dfMatrixDataBase::setCommInfo + ncclInit (dfMatrixDataBase.cu:92-101, dfNcclBase.cu:23-65):
 * nccl_unique_id is the 128-byte RCCL id (rank 0 creates it, the caller broadcasts it),
 * neighb_proc_no[num_patches] the peer rank of each processor patch (-1 otherwise). Collective: every rank calls
 * it; it also splits a second communicator (ncclCommSplit) for the time step's side stream. */
int dfmi_set_comm_info(dfmi_ctx* ctx, const void* nccl_unique_id, int nranks, int rank,
                       const int* neighb_proc_no);
/* rank-0 helper: create a fresh RCCL unique id (128 bytes) */
int dfmi_get_unique_id(void* nccl_unique_id_out);
/* Same as dfmi_set_comm_info, with an in-process transport instead of RCCL: the contexts of one
 * process registered under the same hub_id exchange halos by device copies, each driven by its own
 * host thread. Lets several ranks share one GPU (RCCL refuses two ranks on one device); no
 * reference counterpart. */
int dfmi_set_comm_local(dfmi_ctx* ctx, int hub_id, int nranks, int rank, const int* neighb_proc_no);
/* dfMatrixDataBase::setConstantIndexes (dfMatrixDataBase.cu:184-277) */
int dfmi_set_constant_indexes(dfmi_ctx* ctx, const int* owner, const int* neighbour, const int* proc_rows,
                              const int* proc_cols, int global_offset);
/* dfMatrixDataBase::initConstantFieldsInternal (dfMatrixDataBase.cu:316-333); sf/mesh_distance AoS */
int dfmi_init_constant_fields_internal(dfmi_ctx* ctx, const double* sf, const double* mag_sf,
                                       const double* weight, const double* delta_coeffs,
                                       const double* volume, const double* mesh_distance);
/* dfMatrixDataBase::initConstantFieldsBoundary (dfMatrixDataBase.cu:335-351); boundary_sf AoS */
int dfmi_init_constant_fields_boundary(dfmi_ctx* ctx, const double* boundary_sf, const double* boundary_mag_sf,
                                       const double* boundary_delta_coeffs, const double* boundary_weight,
                                       const int* boundary_face_cell, const int* patch_type_calculated,
                                       const int* patch_type_extrapolated);

/* patch delta vectors [B][3] (AoS, processor patches both halves like the other boundary arrays):
 * fvPatch::delta, on coupled patches (Cf - C) - (Cf' - C') (cyclicFvPatch::delta / processorFvPatch::delta).
 * The d a limited scheme's limiter reads across a coupled face (OpenFOAM-7 LimitedScheme::calcLimiter,
 * patch().delta()); required before a time step when a limited scheme is selected and the mesh has
 * coupled patches. No reference counterpart (its limitedLinear is disabled, dfMatrixOpBase.cu:2540-2600). */
int dfmi_init_boundary_delta(dfmi_ctx* ctx, const double* boundary_delta);

/* ---- convection / interpolation schemes -------------------------------------------------------------
 * The reference GPU path hard-wires upwind for Yi and ha and linear for K and hDiffCorrFlux
 * (dfYEqn.cu:543,587-593; dfEEqn.cu:166-174) whatever system/fvSchemes says; the CPU dfLowMachFoam runs
 * the case's schemes (YEqn.H:6-14 multivariate convection over every Y_i and he, createFields.H:118-129;
 * EEqn.H). term (the fvSchemes divSchemes key) / scheme:
 *   "div(phi,Yi_h)"       "upwind" (default) | "limitedLinear <k>" | "limitedLinear01 <k>"  (Yi and he)
 *   "div(phi,K)"          "linear" (default) | "upwind" | "limitedLinear <k>" | "limitedLinear01 <k>"
 *   "div(hDiffCorrFlux)"  "linear" (default) | "cubic"
 *   "div(phi,U)"          "linear" (default) | "limitedLinearV <k>"  (the 1D flame, test/Tu500K-Phi1/system/fvSchemes)
 * a leading "Gauss" is accepted, e.g. the reference cases' "Gauss limitedLinear01 1" / "Gauss cubic"
 * (test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver/system/fvSchemes:32-40). Call it after
 * dfmi_init_constant_fields_boundary (the patch kinds must be known). On decomposed meshes (processor
 * patches) every term's schemes are supported except div(phi,U) limitedLinearV, which is an error (here
 * and again when the UEqn is assembled). Limited schemes need the mesh_distance argument of
 * dfmi_init_constant_fields_internal (a NULL there makes them an error at the first assembly) and, on
 * meshes with coupled patches, dfmi_init_boundary_delta. */
int dfmi_set_scheme(dfmi_ctx* ctx, const char* term, const char* scheme);

/* ---- cell renumbering (the role of OpenFOAM's renumberMesh; run once on the host before
 * dfmi_set_constant_indexes, then permute the mesh and field data with the returned maps) -------- */
/* new_to_old[num_cells]: method "bricks" (structured blocks: cell_centres holds the integer (i, j, k) of
 * each cell; 8x8x4 bricks along a Z-order curve, lexicographic inside a brick -- the order the gathers
 * are tuned for), "morton" (Z-order of the cell centres [C][3], any mesh), "rcm" (reverse Cuthill-McKee
 * of the face graph, no geometry) or "none" */
int dfmi_renumber_cells(int num_cells, const double* cell_centres, int num_faces, const int* owner,
                        const int* neighbour, const char* method, int* new_to_old);
/* faces of the renumbered mesh in upper-triangular order: face_new_to_old[F], new owner/neighbour
 * (owner < neighbour), flipped[F] = 1 where owner and neighbour swapped (negate Sf and face fluxes,
 * w -> 1 - w, reverse the centre-to-centre vector); boundary faces keep their order (faceCells map
 * through the cell permutation) */
int dfmi_renumber_faces(int num_cells, int num_faces, const int* owner, const int* neighbour,
                        const int* cell_new_to_old, int* face_new_to_old, int* new_owner, int* new_neighbour,
                        int* flipped);

/* the order in which the per-cell gather kernels visit cells (order[C]: a permutation; thread t works on
 * cell order[t]) -- e.g. dfmi_renumber_cells(..., "bricks", ...) of a blockMesh box: the data stay in
 * their order, only the visiting order becomes cache-compact. NULL restores the natural order. Results
 * are bitwise independent of it (each cell's arithmetic is unchanged). No reference counterpart. */
int dfmi_set_traversal(dfmi_ctx* ctx, const int* order);

/* ---- per-equation patch types ------------------------------------------------------------ */
/* dfUEqn/dfYEqn/dfEEqn/dfpEqn/dfRhoEqn/dfThermo::setConstantFields (e.g. dfUEqn.cu:364-379,
 * dfEEqn.cu setConstantFields, dfThermo.cu setConstantFields). field in
 * {"U","p","he","K","Y","T","rho"}; patch_type[num_patches] */
int dfmi_set_patch_types(dfmi_ctx* ctx, const char* field, const int* patch_type);
/* a patch parameter of a mixed condition: (field "p", name "gamma") of waveTransmissive */
int dfmi_set_patch_param(dfmi_ctx* ctx, const char* field, int patch, const char* name, double value);
/* dfYEqn inertIndex (YEqn.H:119-131) */
int dfmi_set_inert_index(dfmi_ctx* ctx, int inert_index);

/* ---- thermo (dfThermo::setConstantValue, dfThermo.cu:361-435) ---------------------------- */
/* coefficient table in memory: W[S], nasa[S][15], visc[S][5], cond[S][5], bdiff[S][S][5] */
int dfmi_thermo_set_coeffs(dfmi_ctx* ctx, int num_species, const double* W, const double* nasa,
                           const double* visc, const double* cond, const double* bdiff);
/* read the reference's binary thermo_<mech>.txt */
int dfmi_thermo_load(dfmi_ctx* ctx, const char* thermo_coeff_file);

/* ---- fields (initNonConstantFields*, getFieldPointer dfMatrixDataBase.cu:521-539) ---------- */
/* names: cells  rho rho_old p p_old he T K K_old psi mu alpha dpdt rAU diffAlphaD psip0
 *        vector U U_old HbyA hDiffCorrFlux sumYDiffError     species Y rhoD hai RR
 *        faces  phi phi_old phiUc rhorAUf phiHbyA
 *        boundary_<name> for the boundary counterparts; boundary-only: boundary_heGradient,
 *        boundary_{U,p,Y,K}_ref (inletOutlet inletValue), boundary_p_vf (waveTransmissive valueFraction),
 *        boundary_p_gamma, chem_stats [3][C]. count = values per component. */
int dfmi_set_field(dfmi_ctx* ctx, const char* name, const double* host, long count, int layout);
int dfmi_get_field(dfmi_ctx* ctx, const char* name, double* host, long count, int layout);

/* ---- one outer iteration (dfLowMachFoam.C:284-531, pEqn_GPU.H) --------------------------- */
int dfmi_pre_time_step(dfmi_ctx* ctx);          /* dfMatrixDataBase::preTimeStep (:503-517) */
int dfmi_rho_process(dfmi_ctx* ctx);            /* dfRhoEqn::process (dfRhoEqn.cu:41-92) */
int dfmi_U_process(dfmi_ctx* ctx);              /* dfUEqn::process (dfUEqn.cu:487-689) */
int dfmi_Y_process(dfmi_ctx* ctx);              /* dfYEqn::process (dfYEqn.cu:443-695); RR from dfmi_set_field("RR") or the chemistry */
int dfmi_E_process(dfmi_ctx* ctx);              /* dfEEqn::process (dfEEqn.cu:108-264) */
int dfmi_thermo_correct(dfmi_ctx* ctx);         /* dfThermo::correctThermo (dfThermo.cu:572-671) */
int dfmi_thermo_update_energy(dfmi_ctx* ctx);   /* he, psi, rho, transport from T (dfThermo::updateEnergy) */
int dfmi_thermo_update_rho(dfmi_ctx* ctx);      /* dfThermo::updateRho (:673-679) */
int dfmi_thermo_psip0(dfmi_ctx* ctx);           /* dfThermo::psip0 (:681-686) */
int dfmi_thermo_correct_psip_rho(dfmi_ctx* ctx);/* dfThermo::correctPsipRho (:688-695) */
int dfmi_U_get_HbyA(dfmi_ctx* ctx);             /* dfUEqn::getHbyA (dfUEqn.cu:824-834) */
int dfmi_p_process(dfmi_ctx* ctx);              /* dfpEqn::process (dfpEqn.cu:379-546) */
int dfmi_post_time_step(dfmi_ctx* ctx);         /* dfMatrixDataBase::postTimeStep (:519) */
/* the whole loop body above with n_corr pressure correctors */
int dfmi_time_step(dfmi_ctx* ctx, int n_corr);   /* non-zero also when chemistry hit its step limit */
int dfmi_sync(dfmi_ctx* ctx);
/* per-step HIP events on the context stream (bench: median step time); no reference counterpart (its
 * TIME_GPU host ticks, dfLowMachFoam.C:249-531). dfmi_step_times returns got = steps timed since arming */
int dfmi_step_timer(dfmi_ctx* ctx, int on);
int dfmi_step_times(dfmi_ctx* ctx, double* ms, int n, int* got);
/* diagnostic: measured device-memory copy bandwidth (read + write GB/s) of a gib-GiB buffer copied reps
 * times by a 16-B-vector streaming kernel -- the measured peak beside the datasheet's 8 TB/s */
int dfmi_hbm_copy_peak(dfmi_ctx* ctx, double gib, int reps, double* gbs);
/* correct_boundary_conditions_{scalar,vector} (dfMatrixOpBase.cu:2402-2491) for field in
 * {"U","p","he","T","rho","K","Y"} using that field's patch types */
int dfmi_correct_boundary(dfmi_ctx* ctx, const char* field);

/* ---- matrix inspection (the reference DEBUG_CHECK_LDU / compareResult path, dfYEqn.cu:566-572) */
/* eqn in {"rho","U","Y","E","p","HbyA","Y_ell","Y_ell_ref"}: run that equation's assembly only (no solve) */
int dfmi_assemble(dfmi_ctx* ctx, const char* eqn);
/* part in {"lower","upper","diag","source","source_solve","internal_coeffs","boundary_coeffs"} */
int dfmi_get_matrix(dfmi_ctx* ctx, const char* eqn, const char* part, double* host, long count);
/* the solver's rows of the YEqn batch after dfmi_assemble("Y_ell") (the production path: assembly
 * written straight into the rows) or dfmi_assemble("Y_ell_ref") (LDU assembly + the generic
 * fvMatrix::addBoundaryDiag/Source fold, the role of ldu_to_csr, dfMatrixOpBase.cu:2276-2336):
 * part "val" [S-1][W][C] (W = coupling entries per row), "dS" (diag + internalCoeffs) or "rhs"
 * [S-1][C]. eqn must be "Y". */
int dfmi_get_solver_rows(dfmi_ctx* ctx, const char* eqn, const char* part, double* host, long count);
/* solver controls (amgxUOptions / amgxpOptions): eqn in {"U","Y","E","p"} */
int dfmi_set_solver(dfmi_ctx* ctx, const char* eqn, int max_iter, double tol, double abs_tol);
/* preconditioner: "jacobi" (all) or "amg" (p; aggregation AMG V-cycle, the amgxpOptions
 * AGGREGATION solver's role) -- p defaults to "amg", U/Y/E to "jacobi" */
int dfmi_set_preconditioner(dfmi_ctx* ctx, const char* eqn, const char* name);
/* implementation options by key (the role of the reference's amgx*Options files, e.g.
 * examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/system/amgxpOptions:1-18, and of the
 * CanteraTorchProperties switches): "amg.*" (omega, overcorrection, coarsest_sweeps, coarsest_size,
 * presweeps, pairwise_passes_l0, pairwise_passes, precision 32|64, padded, tail, halo_l0, global_coarse),
 * "solver.*" (even_odd, small, row_classes), "pcg.*" (face_form, fuse_l0), "fv.*" (hex_walk, csr_walk,
 * species_generic, yprep_brick), "chem.*" (method 0 ROS3 | 1 extrapolation, generated, binning),
 * "dnn.tuned_gemm"; keys and
 * defaults in INTEGRATION.md. Solver-structure keys must be set before the first solve; unknown keys fail. */
int dfmi_set_option(dfmi_ctx* ctx, const char* key, double value);
int dfmi_get_option(dfmi_ctx* ctx, const char* key, double* value);
/* AMG hierarchy after the first p solve: level count, cells and ELL width per level (with several ranks
 * and the option amg.global_coarse the agglomerated coarsest level of all ranks is listed last) */
int dfmi_amg_info(dfmi_ctx* ctx, int max_levels, int* n_levels, int* cells, int* width);
/* gather-row classes in use (0: explicit columns): after the first solve, the number of distinct
 * (column offset, coefficient source) rows the solver / assembly gathers decode from one byte per cell
 * instead of reading 2 W ints (hex boxes in blockMesh order: 27). Measurement aid (no reference
 * counterpart; the reference's ldu_to_csr keeps explicit CSR columns, dfMatrixDataBase.cu:166-177). */
int dfmi_row_classes(dfmi_ctx* ctx, int* n_classes);
/* hex box in blockMesh order detected at the first solve (every cell's face rows checked against the
 * computed i + nx (j + ny k) walk the assembly kernels then use instead of loading indices): nx, ny, nz,
 * or zeros. Measurement aid (no reference counterpart). */
int dfmi_hex_dims(dfmi_ctx* ctx, int* nx, int* ny, int* nz);
/* last solve: iterations and final relative residual */
int dfmi_solver_stats(dfmi_ctx* ctx, const char* eqn, int* iters, double* res0, double* rel_res);
/* work done by the solves of `eqn` since the last reset: the sum over solves and systems of the
 * iterations performed (each one = one PCG SpMV, or two BiCGStab SpMVs, of one system); reset != 0
 * zeroes the counter after reading. Measurement aid for bench.py (no reference counterpart). */
int dfmi_solver_work(dfmi_ctx* ctx, const char* eqn, double* system_iterations, int reset);

/* ---- chemistry (dfChemistryModel::solveSingle, dfChemistryModel.C:737-780; GPU ABI
 * precedent opencc_ode_init/opencc_ode_all, YEqn.H:45-77) ------------------------------------- */
/* mechanism arrays as laid out by deepflame-dev_amd/dfmi/kinetics.py (Mechanism.pack):
 * idata[R][8] (type: 0 elementary, 1 three-body, 2 Lindemann, 3 Troe; reversible; n_reac; n_prod;
 * has_T2), irs[R][6] (reactant ids, product ids, -1 padded), ddata[R][17+S] (A, b, Ta, nu_r[3],
 * nu_p[3], A0, b0, Ta0, Troe A/T3/T1/T2, efficiencies[S]) in SI kmol units; the NASA7 and molecular
 * weights come from the thermo coefficients */
int dfmi_chem_set_mechanism(dfmi_ctx* ctx, int n_reactions, const int* idata, const int* irs, const double* ddata);
/* mode 0 off, 1 stiff ODE integration each YEqn (chemistry->solve(deltaT)), 2 DNN surrogate;
 * tolerances on mass fractions (reference CVODE: relTol 1e-6, absTol 1e-10); cells below T_min get RR = 0 */
int dfmi_chem_set_options(dfmi_ctx* ctx, int mode, double rtol, double atol, double T_min);
/* integrate every cell over dt as a closed constant-volume reactor at fixed T whose state is
 * Cantera's setState_TPY(T, p, Y) (Y clipped at 0 and normalised, density p W/(R T);
 * dfChemistryModel.C:755) -> field "RR" = (Y(dt) - Y) rho / dt with rho the field "rho" (the thermo
 * density, problem.rhoi; inside dfmi_time_step / dfmi_Y_process: "rho_old", the thermo density before
 * this step's rhoEqn). Field "chem_stats" [3][C] = accepted steps (-1: step limit hit), rejected steps,
 * the step size the integration ended with (the next solve's first step). Returns non-zero when any
 * cell hit the step limit (its RR is then not a completed integration). */
int dfmi_chem_solve(dfmi_ctx* ctx, double dt);
/* n_steps df0DFoam time steps (applications/solvers/df0DFoam/df0DFoam.C:99-113, YEqn.H, EEqn.H;
 * zeroDReactor constantProperty pressure): per step chemistry.solve(dt) on every cell, YEqn
 * ddt(rho, Yi) == RR_i (Yi.max(0), inert = 1 - sum), he held, correctThermo (T from he), rho = p psi.
 * Every cell is an independent 0D reactor (BASELINE config 1). The steps are queued without a host
 * synchronisation between them; a chemistry step-limit failure in any of them fails the call once the batch
 * has run (the message gives the count summed over the steps). */
int dfmi_zero_d_step(dfmi_ctx* ctx, double dt, int n_steps);
/* integrator step budget per cell and solve (default 100000); exceeding it is an error of the call */
int dfmi_chem_set_max_steps(dfmi_ctx* ctx, int max_steps);
/* which integrator the last solve used: 0 data-driven generic kernel, > 0 a mechanism compiled in
 * by dfmi/chem_codegen.py (1 Burke2012_s9r23, 2 ES80_H2-7-16) */
int dfmi_chem_info(dfmi_ctx* ctx, int* generated);

/* ---- DF-ODENet surrogate (dfChemistrySolver::setConstantValue/Inference,
 * dfChemistrySolver.cu:78-206; model test/Tu500K-Phi1/inference.py:12-25) ---------------------- */
/* n_modules = S - 1 nets (species 0..S-2; the inert species must be last), each n_layers Linear
 * layers dims[0] = S+2 -> ... -> dims[n_layers] = 1 with GELU between; params (fp32) per module, per
 * layer: weight [out][in] (torch Linear layout) then bias [out]. Normalisation Xmu/Xstd [S+2],
 * Ymu/Ystd [S-1] (the reference hard-codes the H2 values, :95-105). Cells with T >= T_react
 * (reference 610 K) react; RR = (y_new - Y) rho (p/101325) / dt_infer (reference 1e-6). Inference
 * runs in fp16 (MFMA) with fp32 accumulation, as the reference's .to(kHalf) modules. */
int dfmi_dnn_set_model(dfmi_ctx* ctx, int n_modules, int n_layers, const int* dims, const float* params,
                       const double* x_mu, const double* x_std, const double* y_mu, const double* y_std,
                       double T_react, double dt_infer);
/* the same model from a packed file (magic "DFMIDNN1", n_modules, n_layers, dims, the four normalisation vectors,
 * the params above; written by deepflame-dev_amd/dfmi/dnn_checkpoint.py from a checkpoint in inference.py's
 * state_dict layout) -- the file-path entry the reference's setConstantValue has (torch::jit::load of
 * new_Temporary_Chemical_<i>.pt, dfChemistrySolver.cu:112-126), without executing a TorchScript program */
int dfmi_dnn_load_model(dfmi_ctx* ctx, const char* path, double T_react, double dt_infer);
/* run the surrogate on the current T, p, Y -> field "RR" (0 for non-reacting cells), scaled by field
 * "rho" (inside dfmi_time_step: "rho_old", as the reference passes d_rho_old, dfYEqn.cu:449) */
int dfmi_dnn_infer(dfmi_ctx* ctx, int* n_reacting);
/* reacting cells of the last inference; algorithmic hidden-layer GEMM flops since the last call */
int dfmi_dnn_stats(dfmi_ctx* ctx, int* n_reacting, double* gemm_flops);

/* ---- communication accounting per exchange point (multi-rank runs). The reference issues one NCCL group
 * per field and processor patch (dfMatrixOpBase.cu:441-485, dispatch :2402-2491; comm set up at
 * dfNcclBase.cu:23-65) and times only whole equations (TIME_GPU, dfMatrixOpBase.H:42-82). on != 0 resets
 * and arms: every halo exchange (one ncclSend/ncclRecv group per exchange point) and every all-gather is
 * bracketed by HIP events on the stream it runs on and its bytes sent counted, keyed by the exchange point
 * ("fields rho", "bicgstab Y", "pcg p amg", "allgather pcg p", ...); on == 0 disarms. */
int dfmi_comm_timer(dfmi_ctx* ctx, int on);
/* synchronise and write {"point": {"calls": n, "bytes": b, "ms": t}, ...} (JSON) into buf (len bytes);
 * *needed = the length it takes including the terminator */
int dfmi_comm_report(dfmi_ctx* ctx, char* buf, int len, int* needed);

/* ---- kernel timing (the reference's TICK_START_EVENT / TICK_END_EVENT cudaEvent pairs,
 * src_gpu/dfMatrixOpBase.H:46-60): arm HIP-event timing of every launch of one kernel
 * (name as in the source, e.g. "k_y_assemble"; "" disarms), recorded on the context stream */
int dfmi_kernel_timer(dfmi_ctx* ctx, const char* kernels);   /* comma-separated names; re-arming resets */
/* synchronise and return the summed duration and count of the first armed kernel's launches */
int dfmi_kernel_time(dfmi_ctx* ctx, double* total_ms, int* launches);
/* the same for one named armed kernel */
int dfmi_kernel_time_named(dfmi_ctx* ctx, const char* kernel, double* total_ms, int* launches);

#ifdef __cplusplus
}
#endif
#endif /* DFMI_H */
