// fv_kernels.hip -- finite-volume assembly for dfLowMachFoam on MI355X (gfx950).
//
// Replaces the reference's face-parallel atomicAdd kernels (src_gpu/dfMatrixOpBase.cu:658-2173,
// dfUEqn.cu, dfYEqn.cu, dfEEqn.cu, dfpEqn.cu, dfRhoEqn.cu) with deterministic cell-centric gathers:
// one thread per cell walks its faces in OpenFOAM's sequential order (neighbour faces ascending,
// owned faces ascending, then its boundary slots), keeping one accumulator per fvm/fvc term, so the
// result is bit-identical to the sequential restatement in oracle/df_oracle.cpp and independent of
// scheduling. Owned-face coefficients (lower/upper) are written by the owner thread; the neighbour
// thread recomputes the same face value instead of reading it back (no grid-wide dependency).
// Whole equations are fused into one or two launches (the reference issues 10-40 per equation).
//
// Compiled with -ffp-contract=off: the arithmetic sequence is the oracle's, op for op.
#include "dfmi_ctx.h"
// Occupancy caps of the kernels that share the GPU with the side stream's chemistry: at least n
// waves' worth of registers per SIMD. -DDFMI_NO_CAPS builds the uncapped A/B variant (scripts/pmc_caps_ab.sh).
#ifdef DFMI_NO_CAPS
#define DFMI_WAVES(n)
#else
#define DFMI_WAVES(n) __attribute__((amdgpu_waves_per_eu(n, 8)))
#endif
// Stores of the YEqn assembly's ELL rows go out as sc1 stores (st_drop), which write through and drop the line from
// the XCD's L2 (MI355X_MICROARCH.md: plain / nt stores keep it), leaving the L2 to the neighbour planes the face
// gathers re-read: k_y_assemble_ell 661 -> 625 us, step 13.90 -> 13.86 ms (3 rounds each in one call, round 6,
// gpurun_out r06d). The same stores in k_u_assemble measured slower (335 -> 359 us) and stay plain (st_out).
__device__ __forceinline__ void st_drop(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_out(double* p, double v) { *p = v; }
#include <cstdlib>

namespace dfmi {

namespace {

constexpr int TPB = 256;

__device__ __forceinline__ double interp_f(double w, double vo, double vn) { return w * (vo - vn) + vn; }
__device__ __forceinline__ double interp_b(double w, double vo, double vn) { return w * vo + (1.0 - w) * vn; }

struct BCoef { double vic, vbc, gic, gbc; };

// the cell a gather-kernel thread works on: thread order, or the traversal dfmi_set_traversal installed
// (e.g. 8x8x4 bricks on a Z-order curve over blockMesh-ordered data: same data layout, cache-compact
// visiting order). Each cell's arithmetic is unchanged, so results are bitwise independent of it.
__device__ __forceinline__ int cell_of(const MeshView& m, int t) { return (m.trav && t < m.C) ? m.trav[t] : t; }
// per-slot data of the mixed conditions of one field: waveTransmissive (advectiveFvPatchField, Euler ddt:
// refValue = the old-time boundary value, valueFraction = 1 / (1 + w dt deltaCoeffs) set at the pEqn
// assembly) and inletOutlet (refValue = inletValue, valueFraction = 1 - pos0(phi))
struct MixBC {
  const double* wvf;    // waveTransmissive valueFraction [B]
  const double* wref;   // waveTransmissive refValue (old-time boundary field) [B]
  const double* bphi;   // boundary flux (inletOutlet switch) [B]
  const double* ioref;  // inletValue [ncomp][B]
};
__device__ __forceinline__ void mix_vf_ref(int t, const MixBC& x, int b, long B, int comp, double& vf, double& ref) {
  if (t == WAVE_TRANSMISSIVE) { vf = x.wvf[b]; ref = x.wref[b]; }
  else { vf = x.bphi[b] >= 0.0 ? 0.0 : 1.0; ref = x.ioref[comp * B + b]; }
}
__device__ __forceinline__ BCoef bcoef_mixed(double vf, double ref, double bdc) {
  return {1.0 - vf, vf * ref, -vf * bdc, vf * bdc * ref};
}
__device__ __forceinline__ BCoef bcoef(int t, double bval, double w, double bdc, double egrad = 0.0) {
  switch (t) {
    case ZERO_GRADIENT: case EXTRAPOLATED: return {1., 0., 0., 0.};
    case FIXED_VALUE: case FIXED_ENERGY: return {0., bval, -1 * bdc, bdc * bval};
    case GRADIENT_ENERGY: return {1., egrad / bdc, 0., egrad};
    default: return {w, 1.0 - w, -1 * bdc, bdc};
  }
}

__device__ __forceinline__ BCoef bcoef_f(int t, double bval, double w, double bdc, const MixBC& mx, int b, long B, int comp,
                                        double egrad = 0.0) {
  if (bc_mixed(t)) {
    double vf, ref;
    mix_vf_ref(t, mx, b, B, comp, vf, ref);
    return bcoef_mixed(vf, ref, bdc);
  }
  return bcoef(t, bval, w, bdc, egrad);
}

// coupled neighbour-side cell value: cyclic partner cell, or the processor halo value in the slot
__device__ __forceinline__ double nbrv(const MeshView& m, const double* vf, const double* bvf, int b) {
  int pc = m.partner[b];
  return pc >= 0 ? vf[pc] : bvf[b];
}
__device__ __forceinline__ double bface(const MeshView& m, int t, const double* vf, const double* bvf, int b, int c) {
  return bc_coupled(t) ? interp_b(m.bw[b], vf[c], nbrv(m, vf, bvf, b)) : bvf[b];
}

// visit faces of cell c in sequential order: fn(face, other_cell, is_owner).
// WT > 0 (meshes whose busiest cell has WT couplings, hex meshes: 6): read the cell's row of the solver
// gather (ELL [W][C], built once: neighbour faces ascending, owned faces ascending, then coupled slots)
// -- coalesced index loads, one indirection, all WT entries loaded up front and the loop unrolled, so
// every face's gathers are in flight together instead of one face's latency after another's.
// WT = 0: the CSR walk (nbrStart/nbrFace, ownStart), same order, any mesh.
// WT = -1: hex box in blockMesh order (MeshView::hx): the same faces in the same order from the cell's
// (i, j, k) -- neighbour faces from the z-, y-, x- cells, then the owned +x, +y, +z faces; a face of
// owner o sits at storage kslot C + o, kslot = the owner's owned faces before it -- no index loads.
template <int WT, class FN> __device__ __forceinline__ void each_face(const MeshView& m, int c, FN&& fn) {
  if constexpr (WT < 0) {
    const int nx = m.hx, ny = m.hy, nxy = m.hx * m.hy;
    const int t = c / nx, i = c - t * nx, k = t / ny, j = t - k * ny;
    const int hxp = i < nx - 1, hyp = j < ny - 1;
    const int C = m.C;
    if (k > 0) { const int o = c - nxy; fn((hxp + hyp) * C + o, o, false); }
    if (j > 0) { const int o = c - nx; fn(hxp * C + o, o, false); }
    if (i > 0) fn(c - 1, c - 1, false);
    if (hxp) fn(c, c + 1, true);
    if (hyp) fn(hxp * C + c, c + nx, true);
    if (k < m.hz - 1) fn((hxp + hyp) * C + c, c + nxy, true);
  } else if constexpr (WT > 0) {
    int es[WT], cs[WT];
    const int cl = ecls_of(m, c);
#pragma unroll
    for (int k = 0; k < WT; ++k) erow(m, cl, k, c, cs[k], es[k]);
#pragma unroll
    for (int k = 0; k < WT; ++k)
      if (es[k] >= 0) fn(es[k] >> 1, cs[k], (es[k] & 1) != 0);   // slots (< 0) and padding skipped
  } else {
    const int e1 = m.nbrStart[c + 1];
    for (int k = m.nbrStart[c]; k < e1; ++k) { const int f = m.nbrFace[k]; fn(f, m.own[f], false); }
    const int o0 = m.ownStart[c], no = m.ownStart[c + 1] - o0;
    for (int k = 0; k < no; ++k) {
      const int f = m.fslot ? k * m.C + c : o0 + k;   // storage index of the k-th owned face
      fn(f, m.nei[f], true);
    }
  }
}
// visit primary, non-empty boundary slots of c in slot order: fn(slot, type)
template <class FN> __device__ __forceinline__ void each_slot(const MeshView& m, const int8_t* ty, int c, FN&& fn) {
  const int e = m.cbStart[c + 1];
  for (int k = m.cbStart[c]; k < e; ++k) {
    const int b = m.cbSlot[k];
    const int t = ty[b];
    if (t == EMPTY) continue;
    fn(b, t);
  }
}

// ------------------------------------------------------------------ boundary correction
// correct_boundary_conditions_scalar/vector (dfMatrixOpBase.cu:2402-2491)
// gradientEnergy: cell value + gradient / deltaCoeffs (correct_boundary_conditions_gradientEnergy_scalar,
// dfMatrixOpBase.cu:351-366)
__global__ void k_bc_correct(MeshView m, const int8_t* __restrict__ ty, const double* __restrict__ vf,
                             double* __restrict__ bvf, int ncomp, const double* __restrict__ egrad, MixBC mx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const int t = ty[b];
  const int c = m.bfc[b];
  for (int k = 0; k < ncomp; ++k) {
    const double* v = vf + (long)k * m.C;
    double* bv = bvf + (long)k * m.B;
    if (bc_mixed(t)) {   // mixedFvPatchField::evaluate
      double f, ref;
      mix_vf_ref(t, mx, b, m.B, k, f, ref);
      bv[b] = f * ref + (1.0 - f) * v[c];
    } else if (t == ZERO_GRADIENT || t == EXTRAPOLATED) bv[b] = v[c];
    else if (t == CYCLIC) bv[b] = interp_b(m.bw[b], v[c], v[m.partner[b]]);
    else if (bc_proc(t) && !m.sprim[b]) bv[b] = v[c];
    else if (t == GRADIENT_ENERGY && egrad) bv[b] = v[c] + egrad[b] / m.bdc[b];
  }
}

// ------------------------------------------------------------------ limited / cubic schemes
// The terms the reference GPU path hard-wires (upwind Yi/ha, linear K and hDiffCorrFlux; dfYEqn.cu:543,
// 587-593, dfEEqn.cu:166-174) with the schemes the reference's own cases select (system/fvSchemes:
// div(phi,Yi_h) Gauss limitedLinear01 1 -- multivariate over every Y_i and he, YEqn.H:6-14; div(phi,K)
// Gauss limitedLinear 1; div(hDiffCorrFlux) Gauss cubic), OpenFOAM-7 semantics as restated in
// oracle/df_oracle.cpp (limited_weights, conv_weights, k_weights, cubic_flux) -- the same operations in
// the same order, so the weights and fluxes are bitwise the oracle's.
__device__ __forceinline__ double pos0(double x) { return x >= 0 ? 1.0 : 0.0; }
__device__ __forceinline__ double sgn(double x) { return x >= 0 ? 1.0 : -1.0; }

// limitedLinearLimiter<NVDTVD>::limiter (+ Limited01Limiter's bounds when b01); g = the upwind cell's gradient
__device__ __forceinline__ double ll_limiter(double twoByk, double faceFlux, double phiP, double phiN,
                                             const double* g, const double* dv) {
  const double gradf = phiN - phiP;
  const double gradcf = dv[0] * g[0] + dv[1] * g[1] + dv[2] * g[2];
  double r;
  if (fabs(gradcf) >= 1000 * fabs(gradf)) r = 2 * 1000 * sgn(gradcf) * sgn(gradf) - 1;
  else r = 2 * (gradcf / gradf) - 1;
  return fmax(fmin(twoByk * r, 1.0), 0.0);
}
__device__ __forceinline__ bool out01(double faceFlux, double phiP, double phiN) {
  return (faceFlux > 0 && (phiP < 0 || phiN > 1)) || (faceFlux < 0 && (phiN < 0 || phiP > 1));
}

// Gauss linear gradient of a scalar at cell c (fvc::grad; the oracle's grad_scalar: faces in
// increasing index, then the cell's boundary slots, / V)
template <int WT = 0>
__device__ __forceinline__ void cell_grad(const MeshView& m, const int8_t* __restrict__ ty, const double* __restrict__ vf,
                                          const double* __restrict__ bvf, int c, double* g) {
  const long F = m.F, B = m.B;
  const double vc = vf[c];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double w = m.w[f], vn = vf[o2];
    const double yf = own ? interp_f(w, vc, vn) : interp_f(w, vn, vc);
    const double v0 = m.Sf[f] * yf, v1 = m.Sf[F + f] * yf, v2 = m.Sf[2 * F + f] * yf;
    if (own) { s0 += v0; s1 += v1; s2 += v2; } else { s0 -= v0; s1 -= v1; s2 -= v2; }
  });
  each_slot(m, ty, c, [&](int b, int t) {
    const double yf = bface(m, t, vf, bvf, b, c);
    s0 += m.bSf[b] * yf; s1 += m.bSf[B + b] * yf; s2 += m.bSf[2 * B + b] * yf;
  });
  const double vol = m.V[c];
  g[0] = s0 / vol; g[1] = s1 / vol; g[2] = s2 / vol;
}

// multivariate limited weights of div(phi,Yi_h) over {Y_0 .. Y_{S-1}, he} on the internal faces (face
// storage order), in two passes so that no wave idles behind a few lanes:
//  k_conv_w_check -- one thread per face: Limited01's bounds for every field (he of a real mixture
//    leaves [0, 1] almost everywhere, which makes the minimum 0 without any gradient); such faces get
//    their (upwind) weight here, the others are appended to a list (the order of the list does not
//    matter: every face's weight is computed on its own);
//  k_conv_w_list -- a 16-lane group per listed face, one lane per field: the limiter from the upwind
//    cell's Gauss gradient formed on the fly, the group's minimum (fmin, exact) -> the weight.
// The list is reserved with ONE atomic per workgroup (1024 threads x 4 faces): a per-wavefront atomic on
// the single counter serialised ~10^5 times per launch (most waves hold a listed face) and cost 450 us.
constexpr int CK_TPB = 1024, CK_FPT = 4, CK_NW = CK_TPB / 64;
__global__ void __launch_bounds__(CK_TPB) k_conv_w_check(MeshView m, int S, int b01, const double* __restrict__ phi,
                                                         const double* __restrict__ Y, const double* __restrict__ he,
                                                         double* __restrict__ wout, int* __restrict__ list,
                                                         int* __restrict__ nlist) {
  __shared__ int wcnt[CK_FPT * CK_NW];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long C = m.C;
  unsigned long long mask[CK_FPT];
#pragma unroll
  for (int j = 0; j < CK_FPT; ++j) {
    const int f = (blockIdx.x * CK_FPT + j) * CK_TPB + threadIdx.x;
    bool need = false;
    const int o = f < m.F ? m.own[f] : -1;
    if (o >= 0) {   // not past the end, not owner-slot padding
      const int n = m.nei[f];
      const double ph = phi[f];
      bool zero = false;
      if (b01) {
        zero = out01(ph, he[o], he[n]);
        // the species' checks without a loop-carried exit: their loads issue together (a wave runs this
        // branch when any of its lanes passed the he check)
        for (int s0 = 0; s0 < S && !zero; s0 += 4) {
          double yo[4], yn[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int sp = s0 + q < S ? s0 + q : S - 1;
            yo[q] = Y[sp * C + o]; yn[q] = Y[sp * C + n];
          }
          bool z = false;
#pragma unroll
          for (int q = 0; q < 4; ++q) z = z || out01(ph, yo[q], yn[q]);
          zero = z;
        }
      }
      if (zero) {
        const double lim = 0.0;
        wout[f] = lim * m.w[f] + (1 - lim) * pos0(ph);
      }
      need = !zero;
    }
    mask[j] = __ballot(need);
    if (lane == 0) wcnt[j * CK_NW + wid] = (int)__popcll(mask[j]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int k = 0; k < CK_FPT * CK_NW; ++k) tot += wcnt[k];
    base = tot ? atomicAdd(nlist, tot) : 0;
  }
  __syncthreads();
  int off = base;   // entries of the (j, wave) runs before this wave's run of pass j
  for (int k = 0; k < wid; ++k) off += wcnt[k];
#pragma unroll
  for (int j = 0; j < CK_FPT; ++j) {
    if ((mask[j] >> lane) & 1ull)
      list[off + (int)__popcll(mask[j] & ((1ull << lane) - 1ull))] = (blockIdx.x * CK_FPT + j) * CK_TPB + threadIdx.x;
    // next pass: skip the remaining waves of pass j and the first waves of pass j + 1
    for (int k = wid; k < CK_NW; ++k) off += wcnt[j * CK_NW + k];
    if (j + 1 < CK_FPT)
      for (int k = 0; k < wid; ++k) off += wcnt[(j + 1) * CK_NW + k];
  }
}
constexpr int CWG = 16;   // lanes per listed face (fields beyond 16 loop)
template <int WT>
__global__ void __launch_bounds__(256) k_conv_w_list(MeshView m, int S, const int8_t* __restrict__ tyY,
    const int8_t* __restrict__ tyH, double twoByk, const double* __restrict__ phi, const double* __restrict__ Y,
    const double* __restrict__ bY, const double* __restrict__ he, const double* __restrict__ bhe,
    const int* __restrict__ list, const int* __restrict__ nlist, double* __restrict__ wout) {
  const int lane = threadIdx.x % CWG;
  const int n_items = *nlist;
  const int groups = gridDim.x * (blockDim.x / CWG);
  const long C = m.C, Fs = m.F, B = m.B;
  // a group's lanes share `it`, so each group runs the loop (and its shuffles) in lockstep
  for (int it = blockIdx.x * (blockDim.x / CWG) + threadIdx.x / CWG; it < n_items; it += groups) {
    const int f = list[it];
    const int o = m.own[f], n = m.nei[f];
    const double ph = phi[f];
    const double dv[3] = {m.md[f], m.md[Fs + f], m.md[2 * Fs + f]};
    const int cu = ph > 0 ? o : n;   // NVDTVD::r reads the upwind cell's gradient
    double lim = 2.0;                // above every limiter: the neutral element of the min
    for (int s = lane; s <= S; s += CWG) {
      const double* v = s < S ? Y + s * C : he;
      const double* bv = s < S ? bY + s * B : bhe;
      double g[3];
      cell_grad<WT>(m, s < S ? tyY : tyH, v, bv, cu, g);
      lim = fmin(lim, ll_limiter(twoByk, ph, v[o], v[n], g, dv));
    }
#pragma unroll
    for (int off = CWG / 2; off > 0; off >>= 1) lim = fmin(lim, __shfl_xor(lim, off, CWG));
    if (lane == 0) wout[f] = lim * m.w[f] + (1 - lim) * pos0(ph);
  }
}

// the same on the boundary slots: coupled (cyclic) slots with the partner cell as N and the patch delta;
// every other slot takes limiter 1 (calcLimiter's non-coupled branch), i.e. its CD weight
// bgx: on decomposed meshes the neighbour-side gradients of every field on the processor slots
// ([3(S+1)][B], exchanged: patchNeighbourField of fvc::grad), nullptr otherwise
__global__ void k_conv_w_slot(MeshView m, int S, const int8_t* __restrict__ tyY, const int8_t* __restrict__ tyH,
                              int b01, double twoByk, const double* __restrict__ bphi, const double* __restrict__ Y,
                              const double* __restrict__ bY, const double* __restrict__ he,
                              const double* __restrict__ bhe, const double* __restrict__ bgx, double* __restrict__ bwout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const long C = m.C, B = m.B;
  const int t = tyY[b];
  const double ph = bphi[b];
  double lim = 1.0;
  if (bc_coupled(t) && m.sprim[b]) {
    const int c = m.bfc[b], pc = m.partner[b];   // pc < 0: processor slot, neighbour values in the slot
    auto vn = [&](const double* v, const double* bv) { return pc >= 0 ? v[pc] : bv[b]; };
    lim = 0.0;
    bool zero = false;
    if (b01) {
      zero = out01(ph, he[c], vn(he, bhe));
      for (int s = 0; s < S && !zero; ++s) zero = out01(ph, Y[s * C + c], vn(Y + s * C, bY + s * B));
    }
    if (!zero) {
      const double dv[3] = {m.bdv[b], m.bdv[B + b], m.bdv[2 * B + b]};
      const bool own_up = ph > 0;
      for (int s = 0; s <= S; ++s) {
        const double* v = s < S ? Y + s * C : he;
        const double* bv = s < S ? bY + s * B : bhe;
        double g[3];
        if (own_up || pc >= 0) cell_grad(m, s < S ? tyY : tyH, v, bv, own_up ? c : pc, g);
        else { g[0] = bgx[(3 * s) * B + b]; g[1] = bgx[(3 * s + 1) * B + b]; g[2] = bgx[(3 * s + 2) * B + b]; }
        const double l = ll_limiter(twoByk, ph, v[c], vn(v, bv), g, dv);
        lim = s == 0 ? l : fmin(lim, l);
      }
    }
  }
  bwout[b] = lim * m.bw[b] + (1 - lim) * pos0(ph);
}

// gradients of every field of the table at the cells of the processor slots -> g [3(S+1)][C] (only those
// cells written; the halo then carries them to the neighbour ranks' processor slots)
__global__ void k_conv_proc_grad(MeshView m, int S, const int8_t* __restrict__ tyY, const int8_t* __restrict__ tyH,
                                 const double* __restrict__ Y, const double* __restrict__ bY,
                                 const double* __restrict__ he, const double* __restrict__ bhe, double* __restrict__ g) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  if (!bc_proc(tyY[b]) || !m.sprim[b]) return;
  const long C = m.C, B = m.B;
  const int c = m.bfc[b];
  for (int s = 0; s <= S; ++s) {
    double gg[3];
    cell_grad(m, s < S ? tyY : tyH, s < S ? Y + s * C : he, s < S ? bY + s * B : bhe, c, gg);
    g[(3 * s) * C + c] = gg[0]; g[(3 * s + 1) * C + c] = gg[1]; g[(3 * s + 2) * C + c] = gg[2];
  }
}

// Gauss linear gradients of NC scalar components (component k at vf + k*C, boundary bvf + k*B)
// -> g [(3k + dir)][C] (fvc::grad of each vf.component(k)); one face walk for all components, each
// component summed in cell_grad's order
template <int NC, int WT>
__global__ void __launch_bounds__(TPB) k_grad_cells(MeshView m, const int8_t* __restrict__ ty,
                                                    const double* __restrict__ vf, const double* __restrict__ bvf,
                                                    double* __restrict__ g) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  double s[NC][3], vc[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) { s[k][0] = 0.0; s[k][1] = 0.0; s[k][2] = 0.0; vc[k] = vf[k * C + c]; }
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double w = m.w[f], sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const double vn = vf[k * C + o2];
      const double yf = own ? interp_f(w, vc[k], vn) : interp_f(w, vn, vc[k]);
      const double v0 = sf0 * yf, v1 = sf1 * yf, v2 = sf2 * yf;
      if (own) { s[k][0] += v0; s[k][1] += v1; s[k][2] += v2; } else { s[k][0] -= v0; s[k][1] -= v1; s[k][2] -= v2; }
    }
  });
  each_slot(m, ty, c, [&](int b, int t) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const double yf = bface(m, t, vf + k * C, bvf + k * B, b, c);
      s[k][0] += m.bSf[b] * yf; s[k][1] += m.bSf[B + b] * yf; s[k][2] += m.bSf[2 * B + b] * yf;
    }
  });
  const double vol = m.V[c];
#pragma unroll
  for (int k = 0; k < NC; ++k)
#pragma unroll
    for (int d = 0; d < 3; ++d) g[(3 * k + d) * C + c] = s[k][d] / vol;
}

// single-field limited weights (LimitedScheme: div(phi,K)) from a precomputed gradient g [3][C]
__global__ void k_lim_w_face(MeshView m, int b01, double twoByk, const double* __restrict__ phi,
                             const double* __restrict__ v, const double* __restrict__ g, double* __restrict__ wout) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F) return;
  const int o = m.own[f];
  if (o < 0) return;
  const int n = m.nei[f];
  const long C = m.C, Fs = m.F;
  const double ph = phi[f];
  double lim = 0.0;
  if (!(b01 && out01(ph, v[o], v[n]))) {
    const double dv[3] = {m.md[f], m.md[Fs + f], m.md[2 * Fs + f]};
    const int cu = ph > 0 ? o : n;
    const double gu[3] = {g[cu], g[C + cu], g[2 * C + cu]};
    lim = ll_limiter(twoByk, ph, v[o], v[n], gu, dv);
  }
  wout[f] = lim * m.w[f] + (1 - lim) * pos0(ph);
}
// the same on a hex box in blockMesh order, one thread per cell over its owned (+x, +y, +z) faces (no owner /
// neighbour index loads, the owner's value read once); bitwise k_lim_w_face
__global__ void k_lim_w_cell(MeshView m, int b01, double twoByk, const double* __restrict__ phi,
                             const double* __restrict__ v, const double* __restrict__ g, double* __restrict__ wout) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const int nx = m.hx, ny = m.hy, nxy = m.hx * m.hy;
  const int t = c / nx, i = c - t * nx, k = t / ny, j = t - k * ny;
  const int hxp = i < nx - 1, hyp = j < ny - 1, hzp = k < m.hz - 1;
  const long C = m.C, Fs = m.F;
  const double vo = v[c];
  auto face = [&](long f, int n) {
    const double ph = phi[f], vn = v[n];
    double lim = 0.0;
    if (!(b01 && out01(ph, vo, vn))) {
      const double dv[3] = {m.md[f], m.md[Fs + f], m.md[2 * Fs + f]};
      const int cu = ph > 0 ? c : n;
      const double gu[3] = {g[cu], g[C + cu], g[2 * C + cu]};
      lim = ll_limiter(twoByk, ph, vo, vn, gu, dv);
    }
    wout[f] = lim * m.w[f] + (1 - lim) * pos0(ph);
  };
  if (hxp) face(c, c + 1);
  if (hyp) face(hxp * C + c, c + nx);
  if (hzp) face((hxp + hyp) * C + c, c + nxy);
}
// boundary slots; bg = the neighbour-side gradient on processor slots ([3][B], halo), cyclic: partner cell
__global__ void k_lim_w_slot(MeshView m, const int8_t* __restrict__ ty, int b01, double twoByk,
                             const double* __restrict__ bphi, const double* __restrict__ v, const double* __restrict__ bv,
                             const double* __restrict__ g, const double* __restrict__ bg, double* __restrict__ bwout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const long C = m.C, B = m.B;
  const int t = ty[b];
  const double ph = bphi[b];
  double lim = 1.0;
  if (bc_coupled(t) && m.sprim[b]) {
    const int c = m.bfc[b], pc = m.partner[b];
    const double vn = nbrv(m, v, bv, b);
    lim = 0.0;
    if (!(b01 && out01(ph, v[c], vn))) {
      const double dv[3] = {m.bdv[b], m.bdv[B + b], m.bdv[2 * B + b]};
      double gu[3];
      for (int q = 0; q < 3; ++q) gu[q] = ph > 0 ? g[q * C + c] : (pc >= 0 ? g[q * C + pc] : bg[q * B + b]);
      lim = ll_limiter(twoByk, ph, v[c], vn, gu, dv);
    }
  }
  bwout[b] = lim * m.bw[b] + (1 - lim) * pos0(ph);
}

__global__ void k_upwind_w_face(MeshView m, const double* __restrict__ phi, double* __restrict__ wout) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F || m.own[f] < 0) return;
  wout[f] = pos0(phi[f]);
}
__global__ void k_upwind_w_slot(MeshView m, const double* __restrict__ bphi, double* __restrict__ bwout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  bwout[b] = pos0(bphi[b]);
}

// limitedLinearV weights of div(phi,U) (limitedLinearLimiter<NVDVTVDV>) from grad(U) g [9][C]
__device__ __forceinline__ double llv_limiter(double twoByk, const double* vP, const double* vN, const double* g,
                                              const double* dv) {
  const double gv[3] = {vN[0] - vP[0], vN[1] - vP[1], vN[2] - vP[2]};
  const double gradf = gv[0] * gv[0] + gv[1] * gv[1] + gv[2] * gv[2];
  double dg[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) dg[j] = dv[0] * g[j] + dv[1] * g[3 + j] + dv[2] * g[6 + j];
  const double gradcf = gv[0] * dg[0] + gv[1] * dg[1] + gv[2] * dg[2];
  double r;
  if (fabs(gradcf) >= 1000 * fabs(gradf)) r = 2 * 1000 * sgn(gradcf) * sgn(gradf) - 1;
  else r = 2 * (gradcf / gradf) - 1;
  return fmax(fmin(twoByk * r, 1.0), 0.0);
}
__global__ void k_llv_w_face(MeshView m, double twoByk, const double* __restrict__ phi, const double* __restrict__ U,
                             const double* __restrict__ g, double* __restrict__ wout) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F) return;
  const int o = m.own[f];
  if (o < 0) return;
  const int n = m.nei[f];
  const long C = m.C, Fs = m.F;
  const double ph = phi[f];
  const double dv[3] = {m.md[f], m.md[Fs + f], m.md[2 * Fs + f]};
  const double vP[3] = {U[o], U[C + o], U[2 * C + o]}, vN[3] = {U[n], U[C + n], U[2 * C + n]};
  const int cu = ph > 0 ? o : n;
  double gu[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) gu[q] = g[q * C + cu];
  const double lim = llv_limiter(twoByk, vP, vN, gu, dv);
  wout[f] = lim * m.w[f] + (1 - lim) * pos0(ph);
}
__global__ void k_llv_w_slot(MeshView m, const int8_t* __restrict__ ty, double twoByk, const double* __restrict__ bphi,
                             const double* __restrict__ U, const double* __restrict__ g, double* __restrict__ bwout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const long C = m.C, B = m.B;
  const int t = ty[b];
  const double ph = bphi[b];
  double lim = 1.0;
  if (bc_coupled(t) && m.sprim[b] && m.partner[b] >= 0) {   // cyclic (processor patches are rejected on the host)
    const int c = m.bfc[b], pc = m.partner[b];
    const double dv[3] = {m.bdv[b], m.bdv[B + b], m.bdv[2 * B + b]};
    const double vP[3] = {U[c], U[C + c], U[2 * C + c]}, vN[3] = {U[pc], U[C + pc], U[2 * C + pc]};
    const int cu = ph > 0 ? c : pc;
    double gu[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) gu[q] = g[q * C + cu];
    lim = llv_limiter(twoByk, vP, vN, gu, dv);
  }
  bwout[b] = lim * m.bw[b] + (1 - lim) * pos0(ph);
}

// cubic::correction of a vector field (3 components), dotted with Sf: the flux cubic adds to the linear
// face flux (surfaceInterpolationScheme::dotInterpolate + Sf & correction); g = its gradients [9][C]
__device__ __forceinline__ double cubic_corr(double lam, const double* S, double ms, double dc, const double* vP,
                                             const double* vN, const double* gP, const double* gN) {
  const double kSc = lam * (1 - lam * (3 - 2 * lam));
  const double kVecP = ((1 - lam) * (1 - lam)) * lam;
  const double kVecN = (lam * lam) * (lam - 1);
  double cr[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double v = kSc * vP[c] + (-kSc) * vN[c];
    double gi[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) gi[q] = kVecP * gP[3 * c + q] + kVecN * gN[3 * c + q];
    cr[c] = v + (((gi[0] * S[0] + gi[1] * S[1] + gi[2] * S[2]) / ms) / dc);
  }
  return S[0] * cr[0] + S[1] * cr[1] + S[2] * cr[2];
}
__global__ void k_cubic_face(MeshView m, const double* __restrict__ vf, const double* __restrict__ g,
                             double* __restrict__ cf) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F) return;
  const int o = m.own[f];
  if (o < 0) return;
  const int n = m.nei[f];
  const long C = m.C, Fs = m.F;
  const double S[3] = {m.Sf[f], m.Sf[Fs + f], m.Sf[2 * Fs + f]};
  double vP[3], vN[3], gP[9], gN[9];
#pragma unroll
  for (int c = 0; c < 3; ++c) { vP[c] = vf[c * C + o]; vN[c] = vf[c * C + n]; }
#pragma unroll
  for (int q = 0; q < 9; ++q) { gP[q] = g[q * C + o]; gN[q] = g[q * C + n]; }
  cf[f] = cubic_corr(m.w[f], S, m.magSf[f], m.dc[f], vP, vN, gP, gN);
}
// the same on a hex box in blockMesh order (MeshView::hx), one thread per cell over its owned (+x, +y, +z) faces:
// the owner's value and gradient are loaded once for its three faces instead of once per face (face-parallel: 24
// gathered doubles per face); bitwise k_cubic_face (the same cubic_corr on the same operands)
__global__ void k_cubic_cell(MeshView m, const double* __restrict__ vf, const double* __restrict__ g,
                             double* __restrict__ cf) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const int nx = m.hx, ny = m.hy, nxy = m.hx * m.hy;
  const int t = c / nx, i = c - t * nx, k = t / ny, j = t - k * ny;
  const int hxp = i < nx - 1, hyp = j < ny - 1, hzp = k < m.hz - 1;
  const long C = m.C, Fs = m.F;
  double vP[3], gP[9];
#pragma unroll
  for (int q = 0; q < 3; ++q) vP[q] = vf[q * C + c];
#pragma unroll
  for (int q = 0; q < 9; ++q) gP[q] = g[q * C + c];
  auto face = [&](long f, int n) {
    const double S[3] = {m.Sf[f], m.Sf[Fs + f], m.Sf[2 * Fs + f]};
    double vN[3], gN[9];
#pragma unroll
    for (int q = 0; q < 3; ++q) vN[q] = vf[q * C + n];
#pragma unroll
    for (int q = 0; q < 9; ++q) gN[q] = g[q * C + n];
    cf[f] = cubic_corr(m.w[f], S, m.magSf[f], m.dc[f], vP, vN, gP, gN);
  };
  if (hxp) face(c, c + 1);
  if (hyp) face(hxp * C + c, c + nx);
  if (hzp) face((hxp + hyp) * C + c, c + nxy);
}
__global__ void k_cubic_slot(MeshView m, const int8_t* __restrict__ ty, const double* __restrict__ vf,
                             const double* __restrict__ bvf, const double* __restrict__ g, const double* __restrict__ bg,
                             double* __restrict__ bcf) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const long C = m.C, B = m.B;
  const int t = ty[b];
  if (!bc_coupled(t) || !m.sprim[b]) { bcf[b] = 0.0; return; }
  const int c0 = m.bfc[b], pc = m.partner[b];
  const double S[3] = {m.bSf[b], m.bSf[B + b], m.bSf[2 * B + b]};
  double vP[3], vN[3], gP[9], gN[9];
#pragma unroll
  for (int c = 0; c < 3; ++c) { vP[c] = vf[c * C + c0]; vN[c] = nbrv(m, vf + c * C, bvf + c * B, b); }
#pragma unroll
  for (int q = 0; q < 9; ++q) { gP[q] = g[q * C + c0]; gN[q] = pc >= 0 ? g[q * C + pc] : bg[q * B + b]; }
  bcf[b] = cubic_corr(m.bw[b], S, m.bmagSf[b], m.bdc[b], vP, vN, gP, gN);
}

// ------------------------------------------------------------------ old <- new (preTimeStep)
// every pair in one launch (grid.y = pair) instead of one copy launch per field
constexpr int MAXCOPY = 12;
struct CopyList { const double* src[MAXCOPY]; double* dst[MAXCOPY]; long n[MAXCOPY]; };
__global__ void k_copy_multi(CopyList L) {
  const int j = blockIdx.y;
  const double* __restrict__ a = L.src[j];
  double* __restrict__ b = L.dst[j];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < L.n[j]; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}

// ------------------------------------------------------------------ rhoEqn (dfRhoEqn.cu:41-92)
template <int WT>
__global__ void k_rho(MeshView m, const int8_t* __restrict__ ty, const double* __restrict__ rho_old,
                      const double* __restrict__ phi, const double* __restrict__ bphi, double* __restrict__ rho,
                      double* __restrict__ odiag, double* __restrict__ osrc) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  double div = 0.0;
  each_face<WT>(m, c, [&](int f, int, bool own) { if (own) div += phi[f]; else div -= phi[f]; });
  each_slot(m, ty, c, [&](int b, int) { div += bphi[b]; });
  const double diag = m.rdt * m.V[c];
  double src = m.rdt * rho_old[c] * m.V[c];
  src = src - div;
  rho[c] = src / diag;
  if (odiag) { odiag[c] = diag; osrc[c] = src; }
}

// ------------------------------------------------------------------ UEqn
// gradU (fvc_grad_vector :944-1107) -> T = mu*dev2(T(gradU)) (scale_dev2t_tensor_kernel :623) for
// cells, and for the cell's non-coupled slots the corrected boundary gradient (:1239-1327) -> bT.
__device__ __forceinline__ void dev2T(double sc, const double* v, double* o) {
  const double tr = (2. / 3.) * (v[0] + v[4] + v[8]);
  o[0] = sc * (v[0] - tr); o[1] = sc * v[3]; o[2] = sc * v[6];
  o[3] = sc * v[1]; o[4] = sc * (v[4] - tr); o[5] = sc * v[7];
  o[6] = sc * v[2]; o[7] = sc * v[5]; o[8] = sc * (v[8] - tr);
}

template <int WT>
__global__ void __launch_bounds__(TPB) DFMI_WAVES(6) k_u_grad(MeshView m, const int8_t* __restrict__ ty, const double* __restrict__ U,
                         const double* __restrict__ bU, const double* __restrict__ mu, const double* __restrict__ bmu,
                         double* __restrict__ T, double* __restrict__ bT, double* __restrict__ gout) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  double s[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) s[k] = 0.0;
  const double Uc[3] = {U[c], U[C + c], U[2 * C + c]};   // own-cell values in registers
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double w = m.w[f];
    double uf[3], sf[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double un = U[j * C + o2];
      uf[j] = own ? interp_f(w, Uc[j], un) : interp_f(w, un, Uc[j]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) sf[i] = m.Sf[i * F + f];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) { const double v = sf[i] * uf[j]; if (own) s[i * 3 + j] += v; else s[i * 3 + j] -= v; }
  });
  each_slot(m, ty, c, [&](int b, int t) {
    double uf[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) uf[j] = bface(m, t, U + j * C, bU + j * B, b, c);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) s[i * 3 + j] += m.bSf[i * B + b] * uf[j];
  });
  const double vol = m.V[c];
  double g[9], o[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) g[k] = s[k] / vol;
  if (gout) {
#pragma unroll
    for (int k = 0; k < 9; ++k) gout[k * C + c] = g[k];
  }
  dev2T(mu[c], g, o);
#pragma unroll
  for (int k = 0; k < 9; ++k) T[k * C + c] = o[k];
  each_slot(m, ty, c, [&](int b, int t) {
    if (bc_coupled(t)) return;
    const double ms = m.bmagSf[b];
    const double nv[3] = {m.bSf[b] / ms, m.bSf[B + b] / ms, m.bSf[2 * B + b] / ms};
    double bg[9], bo[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double sn = (t == FIXED_VALUE || bc_mixed(t)) ? m.bdc[b] * (bU[j * B + b] - U[j * C + c]) : 0.0;
      const double corr = sn - (nv[0] * g[0 * 3 + j] + nv[1] * g[1 * 3 + j] + nv[2] * g[2 * 3 + j]);
#pragma unroll
      for (int i = 0; i < 3; ++i) bg[i * 3 + j] = g[i * 3 + j] + nv[i] * corr;
    }
    dev2T(bmu[b], bg, bo);
#pragma unroll
    for (int k = 0; k < 9; ++k) bT[k * B + b] = bo[k];
  });
}

// UEqn matrix (UEqn.H:3-20): ddt(rho,U) + div(phi,U) - laplacian(mu,U) - div(mu dev2 T(gradU)),
// plus source_solve = source - grad(p) and rAU (dfUEqn.cu:721-738).
template <int WT>
__global__ void __launch_bounds__(TPB) DFMI_WAVES(5) k_u_assemble(MeshView m, const int8_t* __restrict__ tyU, const int8_t* __restrict__ tyP,
    const double* __restrict__ rho, const double* __restrict__ rho_old, const double* __restrict__ U_old,
    const double* __restrict__ bU, const double* __restrict__ phi, const double* __restrict__ bphi,
    const double* __restrict__ mu, const double* __restrict__ bmu, const double* __restrict__ p,
    const double* __restrict__ bp, const double* __restrict__ T, const double* __restrict__ bT,
    double* __restrict__ lower, double* __restrict__ upper, double* __restrict__ diag, double* __restrict__ src,
    double* __restrict__ srcs, double* __restrict__ ic, double* __restrict__ bc, double* __restrict__ rAU, MixBC mxU,
    const double* __restrict__ wU, const double* __restrict__ bwU) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  double d1 = 0.0, dL = 0.0;
  double dT[3] = {0.0, 0.0, 0.0}, gp[3] = {0.0, 0.0, 0.0};
  // the cell's own tensor, mu and p stay in registers; each face gathers only the other cell's values
  // (interp_f keeps its owner-first argument order, so the arithmetic is unchanged)
  double Tc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) Tc[k] = T[k * C + c];
  const double muc = mu[c], pcc = p[c];
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double w = m.w[f], ph = phi[f];
    const double L1 = -(wU ? wU[f] : w) * ph;   // div(phi,U): linear, or limitedLinearV weights
    const double U1 = L1 + ph;
    const double mun = mu[o2];
    const double UL = m.dc[f] * ((own ? interp_f(w, muc, mun) : interp_f(w, mun, muc)) * m.magSf[f]);
    if (own) { d1 -= L1; st_out(&lower[f], L1 + (-UL)); st_out(&upper[f], U1 + (-UL)); }
    else d1 -= U1;
    dL -= UL;
    const double sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
    double Tn[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) Tn[k] = T[k * C + o2];
    auto fi = [&](int k) { return own ? interp_f(w, Tc[k], Tn[k]) : interp_f(w, Tn[k], Tc[k]); };
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double v = sf0 * fi(0 + j) + sf1 * fi(3 + j) + sf2 * fi(6 + j);
      if (own) dT[j] += v; else dT[j] -= v;
    }
    const double pn = p[o2];
    const double pf = own ? interp_f(w, pcc, pn) : interp_f(w, pn, pcc);
    const double g0 = sf0 * pf, g1 = sf1 * pf, g2 = sf2 * pf;
    if (own) { gp[0] += g0; gp[1] += g1; gp[2] += g2; } else { gp[0] -= g0; gp[1] -= g1; gp[2] -= g2; }
  });
  // boundary contributions: explicit tensor divergence and the pressure gradient
  each_slot(m, tyU, c, [&](int b, int t) {
    double tt[9];
    if (bc_coupled(t)) {
      const int pc = m.partner[b];
#pragma unroll
      for (int k = 0; k < 9; ++k) tt[k] = interp_b(m.bw[b], T[k * C + c], pc >= 0 ? T[k * C + pc] : bT[k * B + b]);
    } else {
#pragma unroll
      for (int k = 0; k < 9; ++k) tt[k] = bT[k * B + b];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) dT[j] += m.bSf[b] * tt[0 + j] + m.bSf[B + b] * tt[3 + j] + m.bSf[2 * B + b] * tt[6 + j];
  });
  each_slot(m, tyP, c, [&](int b, int t) {
    const double pf = bface(m, t, p, bp, b, c);
#pragma unroll
    for (int k = 0; k < 3; ++k) gp[k] += m.bSf[k * B + b] * pf;
  });
  const double vol = m.V[c];
  const double dg = (m.rdt * rho[c] * vol + d1) + (-dL);
  st_out(&diag[c], dg);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double s = m.rdt * rho_old[c] * U_old[k * C + c] * vol + dT[k];
    st_out(&src[k * C + c], s);
    st_out(&srcs[k * C + c], s - gp[k]);
  }
  double r = dg;
  each_slot(m, tyU, c, [&](int b, int t) {
    const double gam = bc_coupled(t) ? interp_b(m.bw[b], mu[c], nbrv(m, mu, bmu, b)) : bmu[b];
    const double pG = gam * m.bmagSf[b];
    double icv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const BCoef q = bcoef_f(t, bU[k * B + b], m.bw[b], m.bdc[b], mxU, b, B, k);
      const BCoef qc = bwU ? bcoef_f(t, bU[k * B + b], bwU[b], m.bdc[b], mxU, b, B, k) : q;   // convection weights
      icv[k] = bphi[b] * qc.vic + (-(pG * q.gic));
      st_out(&ic[k * B + b], icv[k]);
      bc[k * B + b] = -bphi[b] * qc.vbc + (-(-pG * q.gbc));
    }
    r += (icv[0] + icv[1] + icv[2]) / 3;
  });
  st_out(&rAU[c], 1 / (r / vol));
}

// K = 0.5*magSqr(U) on cells (boundary K is done per slot below)
__global__ void k_kinetic(int C, const double* __restrict__ U, double* __restrict__ K) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double x = U[c], y = U[(long)C + c], z = U[2L * C + c];
  K[c] = 0.5 * (x * x + y * y + z * z);
}

// HbyA: fvMatrix::H() / V (dfUEqn.cu:753-822), unscaled; rAU scaling and constrainHbyA follow.
template <int WT>
__global__ void __launch_bounds__(TPB) k_u_hbya(MeshView m, const int8_t* __restrict__ tyU, const double* __restrict__ U,
    const double* __restrict__ bU, const double* __restrict__ lower, const double* __restrict__ upper,
    const double* __restrict__ src, const double* __restrict__ ic, const double* __restrict__ bc,
    double* __restrict__ H) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, B = m.B;
  // one pass over the faces for the three components (each face's coefficient loaded once; every
  // component still sums its faces in order)
  double Hl[3] = {0.0, 0.0, 0.0};
  each_face<WT>(m, c, [&](int f, int oc, bool own) {
    const double a = own ? upper[f] : lower[f];
#pragma unroll
    for (int k = 0; k < 3; ++k) Hl[k] -= a * U[k * C + oc];
  });
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double* Uk = U + k * C;
    double bd = 0.0;
    each_slot(m, tyU, c, [&](int b, int) { bd += ic[k * B + b]; });
    bd = -bd;
    each_slot(m, tyU, c, [&](int b, int) { bd += (ic[b] + ic[B + b] + ic[2 * B + b]) / 3; });
    double h = bd * Uk[c] + (Hl[k] + src[k * C + c]);
    each_slot(m, tyU, c, [&](int b, int t) {
      h += bc_coupled(t) ? bc[k * B + b] * nbrv(m, Uk, bU + k * B, b) : bc[k * B + b];
    });
    H[k * C + c] = h / m.V[c];
  }
}

__global__ void k_hbya_scale_cells(int C, const double* __restrict__ rAU, double* __restrict__ H) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= C) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) H[(long)k * C + c] = rAU[c] * H[(long)k * C + c];
}
__global__ void k_hbya_scale_slots(int B, const int8_t* __restrict__ tyU, const double* __restrict__ brAU,
                                   const double* __restrict__ bU, double* __restrict__ bH) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double v = brAU[b] * bH[(long)k * B + b];
    if (tyU[b] == FIXED_VALUE) v = bU[(long)k * B + b];   // constrainHbyA
    bH[(long)k * B + b] = v;
  }
}

// ------------------------------------------------------------------ pEqn (dfpEqn.cu:379-546)
// per face: rhorAUf = interpolate(rho*rAU); phiHbyA = interpolate(rho)*flux(HbyA) + rhorAUf*ddtCorr;
// symmetric laplacian coefficients lower = upper = -dc*(rhorAUf*magSf).
__global__ void k_p_face(MeshView m, const double* __restrict__ rho, const double* __restrict__ rAU,
                         const double* __restrict__ rho_old, const double* __restrict__ U_old,
                         const double* __restrict__ phi_old, const double* __restrict__ H,
                         double* __restrict__ rf, double* __restrict__ ph, double* __restrict__ lower,
                         double* __restrict__ upper) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F) return;
  const long C = m.C, F = m.F;
  const int o = m.own[f], n = m.nei[f];
  if (o < 0) return;   // padding slot of the owner-slot face storage
  const double w = m.w[f];
  const double r = interp_f(w, rho[o] * rAU[o], rho[n] * rAU[n]);
  rf[f] = r;
  const double sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
  const double ro = rho_old[o], rn = rho_old[n];
  const double phiCorr = phi_old[f] - (sf0 * interp_f(w, ro * U_old[o], rn * U_old[n]) +
                                       sf1 * interp_f(w, ro * U_old[C + o], rn * U_old[C + n]) +
                                       sf2 * interp_f(w, ro * U_old[2 * C + o], rn * U_old[2 * C + n]));
  const double coeff = 1.0 - fmin(fabs(phiCorr) / (fabs(phi_old[f]) + 1e-15), 1.0);
  const double ddtCorr = coeff * m.rdt * phiCorr;
  const double fl = sf0 * interp_f(w, H[o], H[n]) + sf1 * interp_f(w, H[C + o], H[C + n]) +
                    sf2 * interp_f(w, H[2 * C + o], H[2 * C + n]);
  ph[f] = interp_f(w, rho[o], rho[n]) * fl + r * ddtCorr;
  const double UL = m.dc[f] * (r * m.magSf[f]);
  lower[f] = -UL;
  upper[f] = -UL;
}

// Owner-slot face storage (f = k C + c): one thread per cell walks its owned face slots k, so the
// owner's nine values are loaded once instead of once per face (same per-face arithmetic as k_p_face,
// bitwise); writes stay coalesced per slot plane k.
__global__ void k_p_face_cell(MeshView m, const double* __restrict__ rho, const double* __restrict__ rAU,
                              const double* __restrict__ rho_old, const double* __restrict__ U_old,
                              const double* __restrict__ phi_old, const double* __restrict__ H,
                              double* __restrict__ rf, double* __restrict__ ph, double* __restrict__ lower,
                              double* __restrict__ upper) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= m.C) return;
  const long C = m.C, F = m.F;
  const int km = (int)(F / C);
  const double rho_c = rho[c], rr_c = rho_c * rAU[c], ro = rho_old[c];
  const double uo0 = ro * U_old[c], uo1 = ro * U_old[C + c], uo2 = ro * U_old[2 * C + c];
  const double h0 = H[c], h1 = H[C + c], h2 = H[2 * C + c];
  for (int k = 0; k < km; ++k) {
    const long f = k * C + c;
    if (m.own[f] < 0) continue;   // padding slot
    const int n = m.nei[f];
    const double w = m.w[f];
    const double r = interp_f(w, rr_c, rho[n] * rAU[n]);
    rf[f] = r;
    const double sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
    const double rn = rho_old[n];
    const double po = phi_old[f];
    const double phiCorr = po - (sf0 * interp_f(w, uo0, rn * U_old[n]) + sf1 * interp_f(w, uo1, rn * U_old[C + n]) +
                                 sf2 * interp_f(w, uo2, rn * U_old[2 * C + n]));
    const double coeff = 1.0 - fmin(fabs(phiCorr) / (fabs(po) + 1e-15), 1.0);
    const double ddtCorr = coeff * m.rdt * phiCorr;
    const double fl = sf0 * interp_f(w, h0, H[n]) + sf1 * interp_f(w, h1, H[C + n]) + sf2 * interp_f(w, h2, H[2 * C + n]);
    ph[f] = interp_f(w, rho_c, rho[n]) * fl + r * ddtCorr;
    const double UL = m.dc[f] * (r * m.magSf[f]);
    lower[f] = -UL;
    upper[f] = -UL;
  }
}

__global__ void k_p_slot(MeshView m, const int8_t* __restrict__ tyP, const int8_t* __restrict__ tyU,
                         const double* __restrict__ rho, const double* __restrict__ brho, const double* __restrict__ rAU,
                         const double* __restrict__ brAU, const double* __restrict__ rho_old,
                         const double* __restrict__ brho_old, const double* __restrict__ U_old,
                         const double* __restrict__ bU_old, const double* __restrict__ bphi_old,
                         const double* __restrict__ H, const double* __restrict__ bH, const double* __restrict__ bp,
                         double* __restrict__ brf, double* __restrict__ bph, double* __restrict__ ic,
                         double* __restrict__ bc, MixBC mxP, const double* __restrict__ bphi,
                         const double* __restrict__ bpsi, const double* __restrict__ gamma, double* __restrict__ wvf) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const long C = m.C, B = m.B;
  const int t = tyP[b];
  if (!m.sprim[b] || t == EMPTY) { brf[b] = 0.0; bph[b] = 0.0; ic[b] = 0.0; bc[b] = 0.0; return; }
  const int c = m.bfc[b], pc = m.partner[b];
  const double bw = m.bw[b];
  double r;
  if (bc_coupled(t)) r = interp_b(bw, rho[c] * rAU[c], pc >= 0 ? rho[pc] * rAU[pc] : brho[b] * brAU[b]);
  else r = brho[b] * brAU[b];
  brf[b] = r;
  const int tu = tyU[b];
  double ruo[3], Hb[3], rb;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (bc_coupled(tu)) {
      const double rn = pc >= 0 ? rho_old[pc] * U_old[k * C + pc] : brho_old[b] * bU_old[k * B + b];
      ruo[k] = interp_b(bw, rho_old[c] * U_old[k * C + c], rn);
      Hb[k] = interp_b(bw, H[k * C + c], pc >= 0 ? H[k * C + pc] : bH[k * B + b]);
    } else { ruo[k] = brho_old[b] * bU_old[k * B + b]; Hb[k] = bH[k * B + b]; }
  }
  rb = bc_coupled(tu) ? interp_b(bw, rho[c], pc >= 0 ? rho[pc] : brho[b]) : brho[b];
  const double s0 = m.bSf[b], s1 = m.bSf[B + b], s2 = m.bSf[2 * B + b];
  const double phiCorr = bphi_old[b] - (s0 * ruo[0] + s1 * ruo[1] + s2 * ruo[2]);
  const double coeff = bc_fixes_value(tu) ? 0.0 : 1.0 - fmin(fabs(phiCorr) / (fabs(bphi_old[b]) + 1e-15), 1.0);
  const double fl = s0 * Hb[0] + s1 * Hb[1] + s2 * Hb[2];
  bph[b] = rb * fl + r * (coeff * m.rdt * phiCorr);
  BCoef q;
  if (t == WAVE_TRANSMISSIVE) {
    // waveTransmissiveFvPatchField::advectionSpeed = phi_p / (rho_p |Sf|) + sqrt(gamma / psi_p);
    // advectiveFvPatchField::updateCoeffs (Euler): valueFraction = 1 / (1 + w dt deltaCoeffs),
    // refValue = p.oldTime() on the patch
    const double wsp = fmax(bphi[b] / (brho[b] * m.bmagSf[b]) + sqrt(gamma[b] / bpsi[b]), 0.0);
    const double vf = 1.0 / (1.0 + wsp * (1.0 / m.rdt) * m.bdc[b]);
    wvf[b] = vf;
    q = bcoef_mixed(vf, mxP.wref[b], m.bdc[b]);
  } else q = bcoef_f(t, bp[b], bw, m.bdc[b], mxP, b, m.B, 0);
  const double pG = r * m.bmagSf[b];
  ic[b] = -(pG * q.gic);
  bc[b] = -(-pG * q.gbc);
}

template <int WT>
__global__ void k_p_cell(MeshView m, const int8_t* __restrict__ tyP, const double* __restrict__ lower,
                         const double* __restrict__ ph, const double* __restrict__ bph, const double* __restrict__ p,
                         const double* __restrict__ p_old, const double* __restrict__ psi, const double* __restrict__ rho,
                         const double* __restrict__ rho_old, double* __restrict__ diag, double* __restrict__ src) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  double dL = 0.0, div = 0.0;
  each_face<WT>(m, c, [&](int f, int, bool own) {
    dL -= -lower[f];
    if (own) div += ph[f]; else div -= ph[f];
  });
  each_slot(m, tyP, c, [&](int b, int) { div += bph[b]; });
  const double vol = m.V[c];
  double dg = m.rdt * vol;
  double sr = m.rdt * p_old[c] * vol;
  const double APsi = -dg * p[c] + sr;
  sr = sr - APsi;
  sr = sr * psi[c];
  dg = dg * psi[c];
  sr = sr - vol * (m.rdt * (rho[c] - rho_old[c]));
  sr = sr - div;
  src[c] = sr;
  diag[c] = dg - dL;
}

// after the p solve: phi = phiHbyA + pEqn.flux() (lduMatrix::faceH + fvMatrix::flux boundary)
__global__ void k_p_flux_face(MeshView m, const double* __restrict__ ph, const double* __restrict__ lower,
                              const double* __restrict__ upper, const double* __restrict__ p, double* __restrict__ phi) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F) return;
  const int o = m.own[f];
  if (o < 0) return;
  phi[f] = ph[f] + (upper[f] * p[m.nei[f]] - lower[f] * p[o]);
}
__global__ void k_p_flux_slot(MeshView m, const int8_t* __restrict__ tyP, const double* __restrict__ bph,
                              const double* __restrict__ ic, const double* __restrict__ bc, const double* __restrict__ p,
                              const double* __restrict__ bp, double* __restrict__ bphi) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const int t = tyP[b];
  if (!m.sprim[b]) { bphi[b] = 0.0; return; }
  if (t == EMPTY) return;
  const int c = m.bfc[b];
  const double fl = bc_coupled(t) ? ic[b] * p[c] - bc[b] * nbrv(m, p, bp, b) : ic[b] * p[c] - bc[b];
  bphi[b] = bph[b] + fl;
}
// U = HbyA - rAU*grad(p); K; dpdt
template <int WT>
__global__ void k_p_cell_post(MeshView m, const int8_t* __restrict__ tyP, const double* __restrict__ p,
                              const double* __restrict__ bp, const double* __restrict__ p_old,
                              const double* __restrict__ H, const double* __restrict__ rAU, double* __restrict__ U,
                              double* __restrict__ K, double* __restrict__ dpdt) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  double g[3] = {0.0, 0.0, 0.0};
  const double pcc = p[c];
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double pn = p[o2];
    const double pf = own ? interp_f(m.w[f], pcc, pn) : interp_f(m.w[f], pn, pcc);
#pragma unroll
    for (int k = 0; k < 3; ++k) { const double v = m.Sf[k * F + f] * pf; if (own) g[k] += v; else g[k] -= v; }
  });
  each_slot(m, tyP, c, [&](int b, int t) {
    const double pf = bface(m, t, p, bp, b, c);
#pragma unroll
    for (int k = 0; k < 3; ++k) g[k] += m.bSf[k * B + b] * pf;
  });
  const double vol = m.V[c];
  double u[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { u[k] = H[k * C + c] - rAU[c] * (g[k] / vol); U[k * C + c] = u[k]; }
  K[c] = 0.5 * (u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  dpdt[c] = m.rdt * (p[c] - p_old[c]);
}
__global__ void k_kinetic_slots(int B, const double* __restrict__ bU, double* __restrict__ bK) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double x = bU[b], y = bU[(long)B + b], z = bU[2L * B + b];
  bK[b] = 0.5 * (x * x + y * y + z * z);
}

// ------------------------------------------------------------------ YEqn preparation (YEqn.H:24-118)
// per cell: grad(Y_s), sumYDiffError, hDiffCorrFlux, diffAlphaD; per non-coupled slot of the cell:
// corrected boundary gradients -> boundary sumYDiffError / hDiffCorrFlux.
// the rest of k_y_prep for cell c once its face and slot sums are in: gradients / V, sumYDiffError,
// hDiffCorrFlux, diffAlphaD, and the non-coupled slots' boundary fields (shared with the brick kernel)
// (hc: the cell's own hai values, held by the caller)
template <int S>
__device__ __forceinline__ void y_prep_tail(const MeshView& m, const int8_t* __restrict__ tyY, const double* __restrict__ Y,
    const double* __restrict__ bY, const double* __restrict__ rhoD, const double* __restrict__ brhoD,
    const double (&hc)[S], const double* __restrict__ bhai, double* __restrict__ sumE,
    double* __restrict__ bsumE, double* __restrict__ hD, double* __restrict__ bhD, double* __restrict__ dAD,
    double* __restrict__ gout, int c, double (&g)[S][3], const double (&lap)[S], const double (&yc)[S]) {
  const long C = m.C, B = m.B;
  const double vol = m.V[c];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int k = 0; k < 3; ++k) g[s][k] = g[s][k] / vol;
  if (gout) {
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int k = 0; k < 3; ++k) gout[(3L * s + k) * C + c] = g[s][k];
  }
  double se[3], hd[3], rd[S];
#pragma unroll
  for (int s = 0; s < S; ++s) rd[s] = rhoD[s * C + c];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double a = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) a += rd[s] * g[s][k];
    se[k] = a;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double a = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) a += hc[s] * (rd[s] * g[s][k] - yc[s] * se[k]);
    hd[k] = a;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) { sumE[k * C + c] = se[k]; hD[k * C + c] = hd[k]; }
  double dad = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) dad = dad + lap[s] / vol;
  dAD[c] = dad;
  // boundary fields of the non-coupled slots (coupled slots interpolate cell values downstream)
  each_slot(m, tyY, c, [&](int b, int t) {
    if (bc_coupled(t)) return;
    const double ms = m.bmagSf[b];
    const double nv[3] = {m.bSf[b] / ms, m.bSf[B + b] / ms, m.bSf[2 * B + b] / ms};
    double bg[S][3];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double sn = (t == FIXED_VALUE || t == CALCULATED || t == FIXED_ENERGY || bc_mixed(t)) ? m.bdc[b] * (bY[s * B + b] - Y[s * C + c]) : 0.0;
      const double corr = sn - (nv[0] * g[s][0] + nv[1] * g[s][1] + nv[2] * g[s][2]);
#pragma unroll
      for (int k = 0; k < 3; ++k) bg[s][k] = g[s][k] + nv[k] * corr;
    }
    double bse[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < S; ++s) a += brhoD[s * B + b] * bg[s][k];
      bse[k] = a;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double a = 0.0;
#pragma unroll
      for (int s = 0; s < S; ++s)
        a += bhai[s * B + b] * (brhoD[s * B + b] * bg[s][k] - bY[s * B + b] * bse[k]);
      bsumE[k * B + b] = bse[k];
      bhD[k * B + b] = a;
    }
  });
}

template <int S, int WT>
__global__ void __launch_bounds__(TPB) k_y_prep(MeshView m, const int8_t* __restrict__ tyY, const double* __restrict__ Y,
    const double* __restrict__ bY, const double* __restrict__ rhoD, const double* __restrict__ brhoD,
    const double* __restrict__ hai, const double* __restrict__ bhai, const double* __restrict__ alpha,
    const double* __restrict__ balpha, double* __restrict__ sumE, double* __restrict__ bsumE,
    double* __restrict__ hD, double* __restrict__ bhD, double* __restrict__ dAD, double* __restrict__ gout) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  // One pass over the cell's faces computes every species' Gauss gradient AND its diffAlphaD
  // laplacian term (the two per-species face loops of the sequential code fused; each accumulator
  // still sums in face order, so the result is bitwise the sequential one). Own-cell values live
  // in registers; each face loads the neighbour's Y_s and hai_s once.
  double g[S][3], lap[S], yc[S], ahc[S];
  const double ac = alpha[c];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    g[s][0] = 0.0; g[s][1] = 0.0; g[s][2] = 0.0; lap[s] = 0.0;
    yc[s] = Y[s * C + c];
    ahc[s] = ac * hai[s * C + c];
  }
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double w = m.w[f], sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
    const double ms = m.magSf[f], dcf = m.dc[f];
    const double an = alpha[o2];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double yn = Y[s * C + o2];
      const double ahn = an * hai[s * C + o2];
      const double yf = own ? interp_f(w, yc[s], yn) : interp_f(w, yn, yc[s]);
      const double v0 = sf0 * yf, v1 = sf1 * yf, v2 = sf2 * yf;
      const double gam = own ? interp_f(w, ahc[s], ahn) : interp_f(w, ahn, ahc[s]);
      const double dy = own ? yn - yc[s] : yc[s] - yn;
      const double v = gam * ms * (dcf * dy);
      if (own) { g[s][0] += v0; g[s][1] += v1; g[s][2] += v2; lap[s] += v; }
      else { g[s][0] -= v0; g[s][1] -= v1; g[s][2] -= v2; lap[s] -= v; }
    }
  });
  each_slot(m, tyY, c, [&](int b, int t) {
    const double bs0 = m.bSf[b], bs1 = m.bSf[B + b], bs2 = m.bSf[2 * B + b];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double yf = bface(m, t, Y + s * C, bY + s * B, b, c);
      g[s][0] += bs0 * yf; g[s][1] += bs1 * yf; g[s][2] += bs2 * yf;
      double v;
      if (bc_coupled(t)) {
        const int pc = m.partner[b];
        const double an = pc >= 0 ? alpha[pc] * hai[s * C + pc] : balpha[b] * bhai[s * B + b];
        v = interp_b(m.bw[b], ahc[s], an) * m.bmagSf[b] * (m.bdc[b] * (nbrv(m, Y + s * C, bY + s * B, b) - yc[s]));
      } else {
        const double sng = (t == FIXED_VALUE || t == CALCULATED || t == FIXED_ENERGY || bc_mixed(t)) ? m.bdc[b] * (bY[s * B + b] - yc[s]) : 0.0;
        v = balpha[b] * bhai[s * B + b] * m.bmagSf[b] * sng;
      }
      lap[s] += v;
    }
  });
  double hc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) hc[s] = hai[s * C + c];
  y_prep_tail<S>(m, tyY, Y, bY, rhoD, brhoD, hc, bhai, sumE, bsumE, hD, bhD, dAD, gout, c, g, lap, yc);
}

// k_y_prep on a hex box in blockMesh order (MeshView::hx), one YBX x YBY x YBZ brick of cells per
// workgroup: Y_s and alpha hai_s of the brick and of its face-adjacent halo are staged in LDS with
// coalesced loads (SC species at a time), and every face term reads its neighbour from LDS instead of
// two dependent global gathers per species -- the north star's "face contributions staged in LDS". The
// faces, their order and every product are those of k_y_prep<S, -1> (alpha hai formed at staging is the
// same product), so the results are bitwise the face walk's.
constexpr int YBX = 16, YBY = 4, YBZ = 4;
constexpr int YPY = YBX + 2, YPZ = (YBX + 2) * (YBY + 2), YNB = YPZ * (YBZ + 2);
static_assert(YBX * YBY * YBZ == TPB, "one thread per brick cell");
template <int S, int SC>
__global__ void __launch_bounds__(TPB) k_y_prep_brick(MeshView m, const int8_t* __restrict__ tyY, const double* __restrict__ Y,
    const double* __restrict__ bY, const double* __restrict__ rhoD, const double* __restrict__ brhoD,
    const double* __restrict__ hai, const double* __restrict__ bhai, const double* __restrict__ alpha,
    const double* __restrict__ balpha, double* __restrict__ sumE, double* __restrict__ bsumE,
    double* __restrict__ hD, double* __restrict__ bhD, double* __restrict__ dAD, double* __restrict__ gout) {
  constexpr int NCH = (S + SC - 1) / SC;
  __shared__ double sY[SC][YNB], sA[SC][YNB];
  const int nx = m.hx, ny = m.hy, nz = m.hz;
  const int nbx = nx / YBX, nby = ny / YBY;
  const int bid = xcd_block();
  const int bx = bid % nbx, bt = bid / nbx, by = bt % nby, bz = bt / nby;
  const int i0 = bx * YBX, j0 = by * YBY, k0 = bz * YBZ;
  const int t = threadIdx.x;
  const int li = t % YBX, lj = (t / YBX) % YBY, lk = t / (YBX * YBY);
  const int c = (i0 + li) + nx * ((j0 + lj) + ny * (k0 + lk));
  const int me = (li + 1) + YPY * (lj + 1) + YPZ * (lk + 1);
  const long C = m.C, F = m.F, B = m.B;
  double g[S][3], lap[S], yc[S], ahc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) { g[s][0] = 0.0; g[s][1] = 0.0; g[s][2] = 0.0; lap[s] = 0.0; }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int s0 = ch * SC;
    if (ch > 0) __syncthreads();   // every thread done with the previous chunk's values
    for (int p = t; p < YNB; p += TPB) {   // the brick and its face halo (edges and corners have no face)
      const int a = p % YPY, b = (p / YPY) % (YBY + 2), d = p / YPZ;
      const int oa = (a == 0 || a == YBX + 1), ob = (b == 0 || b == YBY + 1), od = (d == 0 || d == YBZ + 1);
      if (oa + ob + od > 1) continue;
      const int gi = i0 + a - 1, gj = j0 + b - 1, gk = k0 + d - 1;
      if (gi < 0 || gi >= nx || gj < 0 || gj >= ny || gk < 0 || gk >= nz) continue;
      const long gc = gi + (long)nx * (gj + (long)ny * gk);
      const double al = alpha[gc];
#pragma unroll
      for (int q = 0; q < SC; ++q)
        if (s0 + q < S) { sY[q][p] = Y[(s0 + q) * C + gc]; sA[q][p] = al * hai[(s0 + q) * C + gc]; }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < SC; ++q)
      if (s0 + q < S) { yc[s0 + q] = sY[q][me]; ahc[s0 + q] = sA[q][me]; }
    each_face<-1>(m, c, [&](int f, int o2, bool own) {
      const int dd = o2 - c;
      const int lo = me + (dd == 1 ? 1 : dd == -1 ? -1 : dd == nx ? YPY : dd == -nx ? -YPY : dd > 0 ? YPZ : -YPZ);
      const double w = m.w[f], sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
      const double ms = m.magSf[f], dcf = m.dc[f];
#pragma unroll
      for (int q = 0; q < SC; ++q) {
        if (s0 + q >= S) continue;
        const int s = s0 + q;
        const double yn = sY[q][lo];
        const double ahn = sA[q][lo];
        const double yf = own ? interp_f(w, yc[s], yn) : interp_f(w, yn, yc[s]);
        const double v0 = sf0 * yf, v1 = sf1 * yf, v2 = sf2 * yf;
        const double gam = own ? interp_f(w, ahc[s], ahn) : interp_f(w, ahn, ahc[s]);
        const double dy = own ? yn - yc[s] : yc[s] - yn;
        const double v = gam * ms * (dcf * dy);
        if (own) { g[s][0] += v0; g[s][1] += v1; g[s][2] += v2; lap[s] += v; }
        else { g[s][0] -= v0; g[s][1] -= v1; g[s][2] -= v2; lap[s] -= v; }
      }
    });
  }
  each_slot(m, tyY, c, [&](int b, int tt) {
    const double bs0 = m.bSf[b], bs1 = m.bSf[B + b], bs2 = m.bSf[2 * B + b];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double yf = bface(m, tt, Y + s * C, bY + s * B, b, c);
      g[s][0] += bs0 * yf; g[s][1] += bs1 * yf; g[s][2] += bs2 * yf;
      double v;
      if (bc_coupled(tt)) {
        const int pc = m.partner[b];
        const double an = pc >= 0 ? alpha[pc] * hai[s * C + pc] : balpha[b] * bhai[s * B + b];
        v = interp_b(m.bw[b], ahc[s], an) * m.bmagSf[b] * (m.bdc[b] * (nbrv(m, Y + s * C, bY + s * B, b) - yc[s]));
      } else {
        const double sng = (tt == FIXED_VALUE || tt == CALCULATED || tt == FIXED_ENERGY || bc_mixed(tt)) ? m.bdc[b] * (bY[s * B + b] - yc[s]) : 0.0;
        v = balpha[b] * bhai[s * B + b] * m.bmagSf[b] * sng;
      }
      lap[s] += v;
    }
  });
  double hc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) hc[s] = hai[s * C + c];
  y_prep_tail<S>(m, tyY, Y, bY, rhoD, brhoD, hc, bhai, sumE, bsumE, hD, bhD, dAD, gout, c, g, lap, yc);
}
// species per staged chunk: all (S <= 5) or about half (LDS 2 SC YNB doubles: 9 species -> 5 = 52 KiB)
constexpr int ybrick_sc(int S) { return S <= 5 ? S : (S + 1) / 2; }



// phiUc = linearInterpolate(sumYDiffError) & Sf
__global__ void k_phiuc_face(MeshView m, const double* __restrict__ sumE, double* __restrict__ phiUc) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= m.F) return;
  const long C = m.C, F = m.F;
  const int o = m.own[f], n = m.nei[f];
  if (o < 0) return;
  const double w = m.w[f];
  phiUc[f] = m.Sf[f] * interp_f(w, sumE[o], sumE[n]) + m.Sf[F + f] * interp_f(w, sumE[C + o], sumE[C + n]) +
             m.Sf[2 * F + f] * interp_f(w, sumE[2 * C + o], sumE[2 * C + n]);
}
__global__ void k_phiuc_slot(MeshView m, const int8_t* __restrict__ tyY, const double* __restrict__ sumE,
                             const double* __restrict__ bsumE, double* __restrict__ bphiUc) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const long C = m.C, B = m.B;
  const int t = tyY[b];
  if (!m.sprim[b] || t == EMPTY) { bphiUc[b] = 0.0; return; }
  const int c = m.bfc[b];
  double e[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    e[k] = bc_coupled(t) ? interp_b(m.bw[b], sumE[k * C + c], nbrv(m, sumE + k * C, bsumE + k * B, b)) : bsumE[k * B + b];
  bphiUc[b] = m.bSf[b] * e[0] + m.bSf[B + b] * e[1] + m.bSf[2 * B + b] * e[2];
}

// Y species matrices, all non-inert species in one pass (dfYEqn.cu:571-638 fused and batched):
// fvm::ddt(rho,Yi) + div(phi,Yi) + div(phiUc,Yi) == laplacian(rhoD_i,Yi) + RR_i
template <int S, int WT>
__global__ void __launch_bounds__(TPB) k_y_assemble(MeshView m, const int8_t* __restrict__ tyY, int inert,
    const double* __restrict__ Y, const double* __restrict__ bY, const double* __restrict__ rhoD,
    const double* __restrict__ brhoD, const double* __restrict__ RR, const double* __restrict__ rho,
    const double* __restrict__ rho_old, const double* __restrict__ phi, const double* __restrict__ bphi,
    const double* __restrict__ phiUc, const double* __restrict__ bphiUc, double* __restrict__ lower,
    double* __restrict__ upper, double* __restrict__ diag, double* __restrict__ src, double* __restrict__ ic,
    double* __restrict__ bc, MixBC mxY, const double* __restrict__ wY, const double* __restrict__ bwY) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  double d1 = 0.0, d2 = 0.0;
  double dL[S], rc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) { dL[s] = 0.0; rc[s] = rhoD[s * C + c]; }
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double ph = phi[f], pu = phiUc[f];
    const double wu = wY ? wY[f] : (ph >= 0 ? 1.0 : 0.0);
    const double L1 = -wu * ph, U1 = L1 + ph;
    const double L2 = -wu * pu, U2 = L2 + pu;
    if (own) { d1 -= L1; d2 -= L2; } else { d1 -= U1; d2 -= U2; }
    const double w = m.w[f], dcf = m.dc[f], ms = m.magSf[f];
    const double Ls = L1 + L2, Us = U1 + U2;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (s == inert) continue;
      const double rn = rhoD[s * C + o2];
      const double UL = dcf * ((own ? interp_f(w, rc[s], rn) : interp_f(w, rn, rc[s])) * ms);
      dL[s] -= UL;
      if (own) { lower[s * F + f] = Ls - UL; upper[s * F + f] = Us - UL; }
    }
  });
  const double vol = m.V[c];
  const double dd = m.rdt * rho[c] * vol + (d1 + d2);
  const double ro = m.rdt * rho_old[c];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s == inert) continue;
    diag[s * C + c] = dd - dL[s];
    src[s * C + c] = ro * Y[s * C + c] * vol + vol * RR[s * C + c];
  }
  each_slot(m, tyY, c, [&](int b, int t) {
    const double wu = bwY ? bwY[b] : (bphi[b] >= 0 ? 1.0 : 0.0);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (s == inert) continue;
      const BCoef qc = bcoef_f(t, bY[s * B + b], wu, m.bdc[b], mxY, b, B, s);
      const BCoef ql = bcoef_f(t, bY[s * B + b], m.bw[b], m.bdc[b], mxY, b, B, s);
      const double gam = bc_coupled(t) ? interp_b(m.bw[b], rhoD[s * C + c], nbrv(m, rhoD + s * C, brhoD + s * B, b)) : brhoD[s * B + b];
      const double pG = gam * m.bmagSf[b];
      ic[s * B + b] = (bphi[b] * qc.vic + bphiUc[b] * qc.vic) - pG * ql.gic;
      bc[s * B + b] = (-bphi[b] * qc.vbc + -bphiUc[b] * qc.vbc) - (-pG * ql.gbc);
    }
  });
}

// The same YEqn assembly, emitted directly in the solver's ELL layout (production path): per
// system (non-inert species) the row values [W][C] in the gather order (neighbour faces, owned
// faces, coupled slots), dS = diag + sum internalCoeffs and rhs = source + non-coupled
// boundaryCoeffs in slot order -- bitwise what k_ell_build makes from the LDU arrays, without writing
// and re-reading lower/upper/internalCoeffs/boundaryCoeffs.
// (the species in two groups, each group its own walk over the cell's faces and slots, bitwise the same: 94 VGPRs and
// no spill under the side-stream cap, but 660 against 590-610 us per launch and 13.88-13.94 against 13.70-13.76 ms
// per step, round 6 -- not kept)
template <int S, int WT>
__global__ void __launch_bounds__(TPB) DFMI_WAVES(5) k_y_assemble_ell(MeshView m, const int8_t* __restrict__ tyY, int inert,
    const double* __restrict__ Y, const double* __restrict__ bY, const double* __restrict__ rhoD,
    const double* __restrict__ brhoD, const double* __restrict__ RR, const double* __restrict__ rho,
    const double* __restrict__ rho_old, const double* __restrict__ phi, const double* __restrict__ bphi,
    const double* __restrict__ phiUc, const double* __restrict__ bphiUc, int W, long Ce, double* __restrict__ val,
    double* __restrict__ dS, double* __restrict__ rhs, MixBC mxY, const double* __restrict__ wY,
    const double* __restrict__ bwY) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const int pc = m.eopos ? m.eopos[c] : c;   // the solver row of c (even-odd layout)
  const long C = m.C, B = m.B;
  auto group = [&](const int g0) {
    constexpr int G = S;
    double d1 = 0.0, d2 = 0.0;
    double dL[G], rc[G];
#pragma unroll
    for (int j = 0; j < G; ++j) { const int s = g0 + j; dL[j] = 0.0; rc[j] = s < S ? rhoD[s * C + c] : 0.0; }
    int k = 0;
    each_face<WT>(m, c, [&](int f, int o2, bool own) {
      const double ph = phi[f], pu = phiUc[f];
      const double wu = wY ? wY[f] : (ph >= 0 ? 1.0 : 0.0);
      const double L1 = -wu * ph, U1 = L1 + ph;
      const double L2 = -wu * pu, U2 = L2 + pu;
      if (own) { d1 -= L1; d2 -= L2; } else { d1 -= U1; d2 -= U2; }
      const double w = m.w[f], dcf = m.dc[f], ms = m.magSf[f];
      const double Ls = L1 + L2, Us = U1 + U2;
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int s = g0 + j;
        if (s >= S) break;
        if (s == inert) continue;
        const int ss = s < inert ? s : s - 1;
        const double rn = rhoD[s * C + o2];
        const double UL = dcf * ((own ? interp_f(w, rc[j], rn) : interp_f(w, rn, rc[j])) * ms);
        dL[j] -= UL;
        st_drop(&val[((long)ss * W + k) * C + pc], own ? Us - UL : Ls - UL);
      }
      ++k;
    });
    const double vol = m.V[c];
    const double dd = m.rdt * rho[c] * vol + (d1 + d2);
    const double ro = m.rdt * rho_old[c];
    double dg[G], sr[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int s = g0 + j;
      if (s >= S) break;
      dg[j] = dd - dL[j];
      sr[j] = ro * Y[s * C + c] * vol + vol * RR[s * C + c];
    }
    each_slot(m, tyY, c, [&](int b, int t) {
      const double wu = bwY ? bwY[b] : (bphi[b] >= 0 ? 1.0 : 0.0);
      const bool cp = bc_coupled(t);
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int s = g0 + j;
        if (s >= S) break;
        if (s == inert) continue;
        const int ss = s < inert ? s : s - 1;
        const BCoef qc = bcoef_f(t, bY[s * B + b], wu, m.bdc[b], mxY, b, B, s);
        const BCoef ql = bcoef_f(t, bY[s * B + b], m.bw[b], m.bdc[b], mxY, b, B, s);
        const double gam = cp ? interp_b(m.bw[b], rhoD[s * C + c], nbrv(m, rhoD + s * C, brhoD + s * B, b)) : brhoD[s * B + b];
        const double pG = gam * m.bmagSf[b];
        const double icv = (bphi[b] * qc.vic + bphiUc[b] * qc.vic) - pG * ql.gic;
        const double bcv = (-bphi[b] * qc.vbc + -bphiUc[b] * qc.vbc) - (-pG * ql.gbc);
        dg[j] += icv;
        if (cp) st_drop(&val[((long)ss * W + k) * C + pc], -bcv);
        else sr[j] += bcv;
      }
      if (cp) ++k;
    });
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int s = g0 + j;
      if (s >= S) break;
      if (s == inert) continue;
      const int ss = s < inert ? s : s - 1;
      for (int kk = k; kk < W; ++kk) st_drop(&val[((long)ss * W + kk) * C + pc], 0.0);
      st_drop(&dS[ss * Ce + pc], dg[j]);
      st_drop(&rhs[ss * Ce + pc], sr[j]);
    }
  };
  group(0);
}


template <int S>
__global__ void k_y_inert(int C, int inert, double* __restrict__ Y) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sum = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s == inert) continue;
    double yi = Y[(long)s * C + c];
    yi = yi > 0 ? yi : 0;
    Y[(long)s * C + c] = yi;
    sum += yi;
  }
  sum = 1 - sum;
  Y[(long)inert * C + c] = sum > 0 ? sum : 0;
}


// ------------------------------------------------------------------ species-generic Y kernels
// Mechanisms beyond the register-resident templates (S > 16, e.g. GRI-scale 53 species, BASELINE
// config 4): the species loop runs in chunks of CH species held in registers. Every per-species
// accumulator (gradient, laplacian, matrix coefficients) depends on its own species only, and every
// cross-species sum (sumYDiffError, hDiffCorrFlux, diffAlphaD and their boundary fields) is carried
// across chunks in species order, so the results are bitwise those of the sequential restatement
// (oracle y_prep / y_assemble) -- the same sums in the same order. hDiffCorrFlux needs the finished
// sumYDiffError, so a second pass re-forms the gradients chunk by chunk (neighbour values come from
// L2 the second time; cheaper than spilling S x 3 gradients per cell to HBM).
constexpr int YCH = 8;
constexpr int YPREP_LCH = 8, YASM_LCH = 8;   // species per launch of the chunked y_prep / y_assemble_ell kernels

// gradient (and, with LAP, the diffAlphaD laplacian) of species s0 .. s0+CH-1 at cell c, divided by V
template <int CH, bool LAP, int WT>
__device__ __forceinline__ void y_chunk_grad(const MeshView& m, const int8_t* __restrict__ tyY, int S, int s0, int c,
    const double* __restrict__ Y, const double* __restrict__ bY, const double* __restrict__ hai,
    const double* __restrict__ bhai, const double* __restrict__ alpha, const double* __restrict__ balpha, double ac,
    double (&g)[CH][3], double (&lap)[CH], double (&yc)[CH]) {
  const long C = m.C, F = m.F, B = m.B;
  double ahc[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int s = s0 + j;
    g[j][0] = 0.0; g[j][1] = 0.0; g[j][2] = 0.0; lap[j] = 0.0;
    yc[j] = s < S ? Y[s * C + c] : 0.0;
    ahc[j] = (LAP && s < S) ? ac * hai[s * C + c] : 0.0;
  }
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double w = m.w[f], sf0 = m.Sf[f], sf1 = m.Sf[F + f], sf2 = m.Sf[2 * F + f];
    const double ms = m.magSf[f], dcf = m.dc[f];
    const double an = LAP ? alpha[o2] : 0.0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int s = s0 + j;
      if (s >= S) break;
      const double yn = Y[s * C + o2];
      const double yf = own ? interp_f(w, yc[j], yn) : interp_f(w, yn, yc[j]);
      const double v0 = sf0 * yf, v1 = sf1 * yf, v2 = sf2 * yf;
      if (own) { g[j][0] += v0; g[j][1] += v1; g[j][2] += v2; } else { g[j][0] -= v0; g[j][1] -= v1; g[j][2] -= v2; }
      if (LAP) {
        const double ahn = an * hai[s * C + o2];
        const double gam = own ? interp_f(w, ahc[j], ahn) : interp_f(w, ahn, ahc[j]);
        const double dy = own ? yn - yc[j] : yc[j] - yn;
        const double v = gam * ms * (dcf * dy);
        if (own) lap[j] += v; else lap[j] -= v;
      }
    }
  });
  each_slot(m, tyY, c, [&](int b, int t) {
    const double bs0 = m.bSf[b], bs1 = m.bSf[B + b], bs2 = m.bSf[2 * B + b];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int s = s0 + j;
      if (s >= S) break;
      const double yf = bface(m, t, Y + s * C, bY + s * B, b, c);
      g[j][0] += bs0 * yf; g[j][1] += bs1 * yf; g[j][2] += bs2 * yf;
      if (LAP) {
        double v;
        if (bc_coupled(t)) {
          const int pc = m.partner[b];
          const double an = pc >= 0 ? alpha[pc] * hai[s * C + pc] : balpha[b] * bhai[s * B + b];
          v = interp_b(m.bw[b], ahc[j], an) * m.bmagSf[b] * (m.bdc[b] * (nbrv(m, Y + s * C, bY + s * B, b) - yc[j]));
        } else {
          const double sng = (t == FIXED_VALUE || t == CALCULATED || t == FIXED_ENERGY || bc_mixed(t)) ? m.bdc[b] * (bY[s * B + b] - yc[j]) : 0.0;
          v = balpha[b] * bhai[s * B + b] * m.bmagSf[b] * sng;
        }
        lap[j] += v;
      }
    }
  });
  const double vol = m.V[c];
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k) g[j][k] = g[j][k] / vol;
}

// corrected gradient of the chunk's species on a non-coupled slot b of cell c (fvc_grad ... correctBC)
template <int CH>
__device__ __forceinline__ void y_chunk_bgrad(const MeshView& m, int t, int b, int S, int s0, int c,
                                              const double* __restrict__ Y, const double* __restrict__ bY,
                                              const double (&g)[CH][3], double (&bg)[CH][3]) {
  const long C = m.C, B = m.B;
  const double ms = m.bmagSf[b];
  const double nv[3] = {m.bSf[b] / ms, m.bSf[B + b] / ms, m.bSf[2 * B + b] / ms};
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int s = s0 + j;
    if (s >= S) break;
    const double sn = (t == FIXED_VALUE || t == CALCULATED || t == FIXED_ENERGY || bc_mixed(t)) ? m.bdc[b] * (bY[s * B + b] - Y[s * C + c]) : 0.0;
    const double corr = sn - (nv[0] * g[j][0] + nv[1] * g[j][1] + nv[2] * g[j][2]);
#pragma unroll
    for (int k = 0; k < 3; ++k) bg[j][k] = g[j][k] + nv[k] * corr;
  }
}

// One launch covers the species [s_lo, s_hi) of one pass (pass 2 needs the finished sumYDiffError). The
// cross-species sums are carried between launches in their output arrays (sumE / dAD, hD, and the boundary
// fields as before), in species order, so any split is bitwise the single launch. The split is for locality:
// a thread walking all S species keeps every species' Y / alpha*hai / rhoD of the cells in flight live in L2
// (2 waves per SIMD: 16k cells per XCD x 53 species x 3 arrays = 20 MB against its 4 MB), so each neighbour
// value is fetched again by each of the cells that read it; a range of species per launch shrinks that set.
template <int CH, int WT>
__global__ void __launch_bounds__(TPB) DFMI_WAVES(4) k_y_prep_gen(MeshView m, int s_lo, int s_hi, int pass,
    const int8_t* __restrict__ tyY,
    const double* __restrict__ Y, const double* __restrict__ bY, const double* __restrict__ rhoD,
    const double* __restrict__ brhoD, const double* __restrict__ hai, const double* __restrict__ bhai,
    const double* __restrict__ alpha, const double* __restrict__ balpha, double* __restrict__ sumE,
    double* __restrict__ bsumE, double* __restrict__ hD, double* __restrict__ bhD, double* __restrict__ dAD,
    double* __restrict__ gout) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, B = m.B;
  const int S = s_hi;   // species bound of this launch
  const double ac = alpha[c], vol = m.V[c];
  double se[3] = {0.0, 0.0, 0.0}, dad = 0.0;
  if (pass == 1) {
  if (s_lo > 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) se[k] = sumE[k * C + c];
    dad = dAD[c];
  }
  // pass 1: gradients + laplacians -> sumYDiffError, diffAlphaD; boundary sumYDiffError summed in place
  for (int s0 = s_lo; s0 < s_hi; s0 += CH) {
    double g[CH][3], lap[CH], yc[CH];
    y_chunk_grad<CH, true, WT>(m, tyY, S, s0, c, Y, bY, hai, bhai, alpha, balpha, ac, g, lap, yc);
    if (gout) {
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (s0 + j < S)
#pragma unroll
          for (int k = 0; k < 3; ++k) gout[(3L * (s0 + j) + k) * C + c] = g[j][k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (s0 + j < S) se[k] += rhoD[(s0 + j) * C + c] * g[j][k];
#pragma unroll
    for (int j = 0; j < CH; ++j)
      if (s0 + j < S) dad = dad + lap[j] / vol;
    each_slot(m, tyY, c, [&](int b, int t) {
      if (bc_coupled(t)) return;
      double bg[CH][3];
      y_chunk_bgrad<CH>(m, t, b, S, s0, c, Y, bY, g, bg);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        double a = s0 == 0 ? 0.0 : bsumE[k * B + b];
#pragma unroll
        for (int j = 0; j < CH; ++j)
          if (s0 + j < S) a += brhoD[(s0 + j) * B + b] * bg[j][k];
        bsumE[k * B + b] = a;
      }
    });
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) sumE[k * C + c] = se[k];
  dAD[c] = dad;
  return;
  }
  // pass 2: hDiffCorrFlux = sum_i hai_i (rhoD_i grad Y_i - Y_i sumYDiffError) (and on the slots)
#pragma unroll
  for (int k = 0; k < 3; ++k) se[k] = sumE[k * C + c];
  double hd[3] = {0.0, 0.0, 0.0};
  if (s_lo > 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) hd[k] = hD[k * C + c];
  }
  for (int s0 = s_lo; s0 < s_hi; s0 += CH) {
    double g[CH][3], lap[CH], yc[CH];
    y_chunk_grad<CH, false, WT>(m, tyY, s_hi, s0, c, Y, bY, hai, bhai, alpha, balpha, ac, g, lap, yc);
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int s = s0 + j;
        if (s < S) hd[k] += hai[s * C + c] * (rhoD[s * C + c] * g[j][k] - yc[j] * se[k]);
      }
    each_slot(m, tyY, c, [&](int b, int t) {
      if (bc_coupled(t)) return;
      double bg[CH][3];
      y_chunk_bgrad<CH>(m, t, b, S, s0, c, Y, bY, g, bg);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double bse = bsumE[k * B + b];
        double a = s0 == 0 ? 0.0 : bhD[k * B + b];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int s = s0 + j;
          if (s < S) a += bhai[s * B + b] * (brhoD[s * B + b] * bg[j][k] - bY[s * B + b] * bse);
        }
        bhD[k * B + b] = a;
      }
    });
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) hD[k * C + c] = hd[k];
}

// YEqn matrices, chunked over species (LDU form: the dfmi_assemble("Y") inspection path)
template <int CH, int WT>
__global__ void __launch_bounds__(TPB) k_y_assemble_gen(MeshView m, int S, const int8_t* __restrict__ tyY, int inert,
    const double* __restrict__ Y, const double* __restrict__ bY, const double* __restrict__ rhoD,
    const double* __restrict__ brhoD, const double* __restrict__ RR, const double* __restrict__ rho,
    const double* __restrict__ rho_old, const double* __restrict__ phi, const double* __restrict__ bphi,
    const double* __restrict__ phiUc, const double* __restrict__ bphiUc, double* __restrict__ lower,
    double* __restrict__ upper, double* __restrict__ diag, double* __restrict__ src, double* __restrict__ ic,
    double* __restrict__ bc, MixBC mxY, const double* __restrict__ wY, const double* __restrict__ bwY) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  const double vol = m.V[c];
  for (int s0 = 0; s0 < S; s0 += CH) {
    double d1 = 0.0, d2 = 0.0;
    double dL[CH], rc[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) { dL[j] = 0.0; rc[j] = s0 + j < S ? rhoD[(s0 + j) * C + c] : 0.0; }
    each_face<WT>(m, c, [&](int f, int o2, bool own) {
      const double ph = phi[f], pu = phiUc[f];
      const double wu = wY ? wY[f] : (ph >= 0 ? 1.0 : 0.0);
      const double L1 = -wu * ph, U1 = L1 + ph;
      const double L2 = -wu * pu, U2 = L2 + pu;
      if (own) { d1 -= L1; d2 -= L2; } else { d1 -= U1; d2 -= U2; }
      const double w = m.w[f], dcf = m.dc[f], ms = m.magSf[f];
      const double Ls = L1 + L2, Us = U1 + U2;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int s = s0 + j;
        if (s >= S) break;
        if (s == inert) continue;
        const double rn = rhoD[s * C + o2];
        const double UL = dcf * ((own ? interp_f(w, rc[j], rn) : interp_f(w, rn, rc[j])) * ms);
        dL[j] -= UL;
        if (own) { lower[s * F + f] = Ls - UL; upper[s * F + f] = Us - UL; }
      }
    });
    const double dd = m.rdt * rho[c] * vol + (d1 + d2);
    const double ro = m.rdt * rho_old[c];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int s = s0 + j;
      if (s >= S) break;
      if (s == inert) continue;
      diag[s * C + c] = dd - dL[j];
      src[s * C + c] = ro * Y[s * C + c] * vol + vol * RR[s * C + c];
    }
    each_slot(m, tyY, c, [&](int b, int t) {
      const double wu = bwY ? bwY[b] : (bphi[b] >= 0 ? 1.0 : 0.0);
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int s = s0 + j;
        if (s >= S) break;
        if (s == inert) continue;
        const BCoef qc = bcoef_f(t, bY[s * B + b], wu, m.bdc[b], mxY, b, B, s);
        const BCoef ql = bcoef_f(t, bY[s * B + b], m.bw[b], m.bdc[b], mxY, b, B, s);
        const double gam = bc_coupled(t) ? interp_b(m.bw[b], rhoD[s * C + c], nbrv(m, rhoD + s * C, brhoD + s * B, b)) : brhoD[s * B + b];
        const double pG = gam * m.bmagSf[b];
        ic[s * B + b] = (bphi[b] * qc.vic + bphiUc[b] * qc.vic) - pG * ql.gic;
        bc[s * B + b] = (-bphi[b] * qc.vbc + -bphiUc[b] * qc.vbc) - (-pG * ql.gbc);
      }
    });
  }
}

// YEqn in the solver's ELL rows, chunked over species (production path for S > 16)
// One launch covers the species [s_lo, s_hi) (the species are independent here; split for L2 locality of the
// neighbour rhoD gathers, as k_y_prep_gen)
template <int CH, int WT>
__global__ void __launch_bounds__(TPB) k_y_assemble_ell_gen(MeshView m, int s_lo, int S, const int8_t* __restrict__ tyY, int inert,
    const double* __restrict__ Y, const double* __restrict__ bY, const double* __restrict__ rhoD,
    const double* __restrict__ brhoD, const double* __restrict__ RR, const double* __restrict__ rho,
    const double* __restrict__ rho_old, const double* __restrict__ phi, const double* __restrict__ bphi,
    const double* __restrict__ phiUc, const double* __restrict__ bphiUc, int W, long Ce, double* __restrict__ val,
    double* __restrict__ dS, double* __restrict__ rhs, MixBC mxY, const double* __restrict__ wY,
    const double* __restrict__ bwY) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const int pc = m.eopos ? m.eopos[c] : c;   // the solver row of c (even-odd layout)
  const long C = m.C, B = m.B;
  const double vol = m.V[c];
  for (int s0 = s_lo; s0 < S; s0 += CH) {
    double d1 = 0.0, d2 = 0.0;
    double dL[CH], rc[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) { dL[j] = 0.0; rc[j] = s0 + j < S ? rhoD[(s0 + j) * C + c] : 0.0; }
    int k = 0;
    each_face<WT>(m, c, [&](int f, int o2, bool own) {
      const double ph = phi[f], pu = phiUc[f];
      const double wu = wY ? wY[f] : (ph >= 0 ? 1.0 : 0.0);
      const double L1 = -wu * ph, U1 = L1 + ph;
      const double L2 = -wu * pu, U2 = L2 + pu;
      if (own) { d1 -= L1; d2 -= L2; } else { d1 -= U1; d2 -= U2; }
      const double w = m.w[f], dcf = m.dc[f], ms = m.magSf[f];
      const double Ls = L1 + L2, Us = U1 + U2;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int s = s0 + j;
        if (s >= S) break;
        if (s == inert) continue;
        const int ss = s < inert ? s : s - 1;
        const double rn = rhoD[s * C + o2];
        const double UL = dcf * ((own ? interp_f(w, rc[j], rn) : interp_f(w, rn, rc[j])) * ms);
        dL[j] -= UL;
        val[((long)ss * W + k) * C + pc] = own ? Us - UL : Ls - UL;
      }
      ++k;
    });
    const double dd = m.rdt * rho[c] * vol + (d1 + d2);
    const double ro = m.rdt * rho_old[c];
    double dg[CH], sr[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int s = s0 + j;
      dg[j] = dd - dL[j];
      sr[j] = s < S ? ro * Y[s * C + c] * vol + vol * RR[s * C + c] : 0.0;
    }
    each_slot(m, tyY, c, [&](int b, int t) {
      const double wu = bwY ? bwY[b] : (bphi[b] >= 0 ? 1.0 : 0.0);
      const bool cp = bc_coupled(t);
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int s = s0 + j;
        if (s >= S) break;
        if (s == inert) continue;
        const int ss = s < inert ? s : s - 1;
        const BCoef qc = bcoef_f(t, bY[s * B + b], wu, m.bdc[b], mxY, b, B, s);
        const BCoef ql = bcoef_f(t, bY[s * B + b], m.bw[b], m.bdc[b], mxY, b, B, s);
        const double gam = cp ? interp_b(m.bw[b], rhoD[s * C + c], nbrv(m, rhoD + s * C, brhoD + s * B, b)) : brhoD[s * B + b];
        const double pG = gam * m.bmagSf[b];
        const double icv = (bphi[b] * qc.vic + bphiUc[b] * qc.vic) - pG * ql.gic;
        const double bcv = (-bphi[b] * qc.vbc + -bphiUc[b] * qc.vbc) - (-pG * ql.gbc);
        dg[j] += icv;
        if (cp) val[((long)ss * W + k) * C + pc] = -bcv;
        else sr[j] += bcv;
      }
      if (cp) ++k;
    });
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int s = s0 + j;
      if (s >= S) break;
      if (s == inert) continue;
      const int ss = s < inert ? s : s - 1;
      for (int kk = k; kk < W; ++kk) val[((long)ss * W + kk) * C + pc] = 0.0;
      dS[ss * Ce + pc] = dg[j];
      rhs[ss * Ce + pc] = sr[j];
    }
  }
}

__global__ void k_y_inert_gen(int C, int S, int inert, double* __restrict__ Y) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sum = 0;
  for (int s = 0; s < S; ++s) {
    if (s == inert) continue;
    double yi = Y[(long)s * C + c];
    yi = yi > 0 ? yi : 0;
    Y[(long)s * C + c] = yi;
    sum += yi;
  }
  sum = 1 - sum;
  Y[(long)inert * C + c] = sum > 0 ? sum : 0;
}

// ------------------------------------------------------------------ EEqn (EEqn.H:12-45; dfEEqn.cu:108-264)
template <int WT>
__global__ void __launch_bounds__(TPB) k_e_assemble(MeshView m, const int8_t* __restrict__ tyH, const int8_t* __restrict__ tyK,
    const double* __restrict__ he, const double* __restrict__ bhe, const double* __restrict__ rho,
    const double* __restrict__ rho_old, const double* __restrict__ K, const double* __restrict__ K_old,
    const double* __restrict__ bK, const double* __restrict__ phi, const double* __restrict__ bphi,
    const double* __restrict__ alpha, const double* __restrict__ balpha, const double* __restrict__ hD,
    const double* __restrict__ bhD, const double* __restrict__ dpdt, const double* __restrict__ dAD,
    const double* __restrict__ egrad, double* __restrict__ lower, double* __restrict__ upper,
    double* __restrict__ diag, double* __restrict__ src, double* __restrict__ ic, double* __restrict__ bc,
    const double* __restrict__ wY, const double* __restrict__ bwY, const double* __restrict__ wK,
    const double* __restrict__ bwK, const double* __restrict__ cf, const double* __restrict__ bcf) {
  const int c = cell_of(m, xcd_block() * blockDim.x + threadIdx.x);
  if (c >= m.C) return;
  const long C = m.C, F = m.F, B = m.B;
  double d1 = 0.0, dL = 0.0, divK = 0.0, divh = 0.0;
  const double ac = alpha[c], Kc = K[c], hc0 = hD[c], hc1 = hD[C + c], hc2 = hD[2 * C + c];   // own cell
  each_face<WT>(m, c, [&](int f, int o2, bool own) {
    const double ph = phi[f], w = m.w[f];
    auto fi = [&](double vc, double vn) { return own ? interp_f(w, vc, vn) : interp_f(w, vn, vc); };
    const double wu = wY ? wY[f] : (ph >= 0 ? 1.0 : 0.0);
    const double L1 = -wu * ph, U1 = L1 + ph;
    const double UL = m.dc[f] * (fi(ac, alpha[o2]) * m.magSf[f]);
    if (own) { d1 -= L1; lower[f] = L1 - UL; upper[f] = U1 - UL; } else d1 -= U1;
    dL -= UL;
    const double wk = wK ? wK[f] : w;   // div(phi,K): limited weights, or linear
    const double vk = ph * (own ? interp_f(wk, Kc, K[o2]) : interp_f(wk, K[o2], Kc));
    double vh = m.Sf[f] * fi(hc0, hD[o2]) + m.Sf[F + f] * fi(hc1, hD[C + o2]) +
                m.Sf[2 * F + f] * fi(hc2, hD[2 * C + o2]);
    if (cf) vh = vh + cf[f];            // div(hDiffCorrFlux) cubic: + Sf & correction
    if (own) { divK += vk; divh += vh; } else { divK -= vk; divh -= vh; }
  });
  each_slot(m, tyK, c, [&](int b, int t) {
    const double kb = (wK && bc_coupled(t)) ? interp_b(bwK[b], Kc, nbrv(m, K, bK, b)) : bface(m, t, K, bK, b, c);
    divK += bphi[b] * kb;
  });
  each_slot(m, tyH, c, [&](int b, int t) {
    double h[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) h[k] = bface(m, t, hD + k * C, bhD + k * B, b, c);
    double v = m.bSf[b] * h[0] + m.bSf[B + b] * h[1] + m.bSf[2 * B + b] * h[2];
    if (bcf && bc_coupled(t)) v = v + bcf[b];
    divh += v;
  });
  const double vol = m.V[c];
  diag[c] = (m.rdt * rho[c] * vol + d1) - dL;
  double sL = m.rdt * rho_old[c] * he[c] * vol;
  sL = sL - vol * (m.rdt * (rho[c] * K[c] - rho_old[c] * K_old[c]));
  sL = sL - divK;
  sL = sL + vol * dpdt[c];
  double sR = vol * dAD[c];
  sR = sR - divh;
  src[c] = sL - sR;
  each_slot(m, tyH, c, [&](int b, int t) {
    const double eg = egrad ? egrad[b] : 0.0;
    const BCoef qc = bcoef(t, bhe[b], bwY ? bwY[b] : (bphi[b] >= 0 ? 1.0 : 0.0), m.bdc[b], eg);
    const BCoef ql = bcoef(t, bhe[b], m.bw[b], m.bdc[b], eg);
    const double gam = bc_coupled(t) ? interp_b(m.bw[b], alpha[c], nbrv(m, alpha, balpha, b)) : balpha[b];
    const double pG = gam * m.bmagSf[b];
    ic[b] = bphi[b] * qc.vic - pG * ql.gic;
    bc[b] = -bphi[b] * qc.vbc - (-pG * ql.gbc);
  });
}

// ------------------------------------------------------------------ df0DFoam species update
// YEqn.H of df0DFoam (applications/solvers/df0DFoam/YEqn.H): fvm::ddt(rho, Yi) == RR_i per cell (no
// transport), solved exactly: Y_i = (rdt rho_old Y_i V + V RR_i) / (rdt rho V); Yi.max(0); inert = 1 - sum.
__global__ void k_zero_d_species(int C, int S, int inert, double rdt, const double* __restrict__ V,
                                 const double* __restrict__ rho_old, const double* __restrict__ rho,
                                 const double* __restrict__ RR, double* __restrict__ Y) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double vol = V[c];
  const double dg = rdt * rho[c] * vol, ro = rdt * rho_old[c];
  double sum = 0.0;
  for (int s = 0; s < S; ++s) {
    if (s == inert) continue;
    double y = (ro * Y[(long)s * C + c] * vol + vol * RR[(long)s * C + c]) / dg;
    y = y > 0 ? y : 0;
    Y[(long)s * C + c] = y;
    sum += y;
  }
  sum = 1 - sum;
  Y[(long)inert * C + c] = sum > 0 ? sum : 0;
}

// ------------------------------------------------------------------ elementwise thermo bookkeeping
__global__ void k_mul(long n, const double* __restrict__ a, const double* __restrict__ b, double* __restrict__ out) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}
__global__ void k_add_psip(long n, const double* __restrict__ p, const double* __restrict__ psi,
                           const double* __restrict__ psip0, double* __restrict__ rho) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) rho[i] += psi[i] * p[i] - psip0[i];
}

template <template <int> class K, class... A> void dispatch_S(int S, dim3 g, dim3 b, hipStream_t st, A... a);

}  // namespace

// ====================================================================== launchers
#define LAUNCH(kernel, n, ...) \
  do { KScope _ks(x, #kernel); if ((n) > 0) hipLaunchKernelGGL(kernel, dim3(blocks_for((n), TPB)), dim3(TPB), 0, x.stream, __VA_ARGS__); \
       DFMI_HIP(hipGetLastError()); } while (0)
// a launch timed under another kernel's name (a variant of that kernel: the bench rooflines key on the name)
#define LAUNCH_AS(name, kernel, n, ...) \
  do { KScope _ks(x, name); if ((n) > 0) hipLaunchKernelGGL(kernel, dim3(blocks_for((n), TPB)), dim3(TPB), 0, x.stream, __VA_ARGS__); \
       DFMI_HIP(hipGetLastError()); } while (0)

// kernels templated on the ELL width: the unrolled path for hex meshes (W = 6), the CSR walk otherwise
// (option fv.csr_walk forces the CSR walk everywhere: A/B measurement and parity of both paths)
bool face_rows(const Ctx& x) { return x.ell.W == 6 && !x.on("fv.csr_walk"); }
// hex boxes in blockMesh order: the computed face walk (each_face<-1>) everywhere (fv.hex_walk = 0: off)
bool face_hex(const Ctx& x) { return x.hex[0] > 0 && x.on("fv.hex_walk") && !x.on("fv.csr_walk"); }
#define LAUNCH_W(kern, n, ...) \
  do { if (face_hex(x)) LAUNCH(kern<-1>, n, __VA_ARGS__); else if (face_rows(x)) LAUNCH(kern<6>, n, __VA_ARGS__); \
       else LAUNCH(kern<0>, n, __VA_ARGS__); } while (0)
// species-chunked kernels for large mechanisms walk the CSR face lists on every mesh: 2M cells x 53 species,
// y_prep 9.5 against 17.5 ms by the face rows and 8.61 against 8.71 ms by the computed hex walk (its 179 VGPRs:
// two waves per SIMD), y_assemble_ell 4.5 / 4.43 against 6.1 / 5.84 ms (round 4, scripts/c4_ab.sh)
#define LAUNCH_SWG(kern, NS, n, ...) LAUNCH((kern<NS, 0>), n, __VA_ARGS__)
#define LAUNCH_SW(kern, NS, n, ...) \
  do { if (face_hex(x)) LAUNCH((kern<NS, -1>), n, __VA_ARGS__); else if (face_rows(x)) LAUNCH((kern<NS, 6>), n, __VA_ARGS__); \
       else LAUNCH((kern<NS, 0>), n, __VA_ARGS__); } while (0)

// the mixed-condition data of a field (MixBC): p's waveTransmissive state, every field's inletValue
MixBC mixbc(Ctx& x, const std::string& field) {
  MixBC m{nullptr, nullptr, x.f("boundary_phi"), nullptr};
  if (field == "p") { m.wvf = x.f("boundary_p_vf"); m.wref = x.f("boundary_p_old"); }
  auto it = x.fields.find("boundary_" + field + "_ref");
  if (it != x.fields.end()) m.ioref = it->second.buf.p;
  return m;
}

void k_bc_correct(Ctx& x, const char* tf, double* vf, double* bvf, int ncomp) {
  const double* eg = std::string(tf) == "he" ? x.f("boundary_heGradient") : nullptr;
  LAUNCH(k_bc_correct, x.B, x.view(), x.st(tf), vf, bvf, ncomp, eg, mixbc(x, tf));
}

void copy_old(Ctx& x) {   // dfMatrixDataBase::preTimeStep (dfMatrixDataBase.cu:503-517)
  const char* pairs[][2] = {{"rho_old", "rho"}, {"boundary_rho_old", "boundary_rho"}, {"phi_old", "phi"},
                            {"boundary_phi_old", "boundary_phi"}, {"U_old", "U"}, {"boundary_U_old", "boundary_U"},
                            {"K_old", "K"}, {"p_old", "p"}, {"boundary_p_old", "boundary_p"}};
  CopyList L{};
  int k = 0;
  for (auto& pr : pairs) {
    Field& dst = x.fields.at(pr[0]);
    if (dst.buf.n == 0) continue;
    L.src[k] = x.f(pr[1]); L.dst[k] = dst.buf.p; L.n[k] = (long)dst.buf.n; ++k;
  }
  static_assert(sizeof(pairs) / sizeof(pairs[0]) <= MAXCOPY, "CopyList capacity");
  KScope _ks(x, "k_copy_multi");
  if (k) hipLaunchKernelGGL(k_copy_multi, dim3(1024, k), dim3(TPB), 0, x.stream, L);
  DFMI_HIP(hipGetLastError());
}

void rho_process(Ctx& x, bool write_matrix) {
  double* od = write_matrix ? x.f("dbg_rho_diag") : nullptr;
  double* os = write_matrix ? x.f("dbg_rho_source") : nullptr;
  LAUNCH_W(k_rho, x.C, x.view(), x.st("rho"), x.f("rho_old"), x.f("phi"), x.f("boundary_phi"), x.f("rho"), od, os);
  k_bc_correct(x, "rho", x.f("rho"), x.f("boundary_rho"), 1);
  halo_fields(x, {"rho"});
}

// ---- schemes (dfmi_set_scheme): buffers allocated on first use
static double* scheme_buf(Ctx& x, const char* name, long n, int ncomp, bool face = false) {
  auto it = x.fields.find(name);
  if (it == x.fields.end() || it->second.n != n || it->second.ncomp != ncomp) {
    Field& f = x.fields[name];
    f.n = n; f.ncomp = ncomp; f.boundary = std::string(name).rfind("boundary_", 0) == 0; f.face = face;
    f.buf.alloc((size_t)n * ncomp);
    f.buf.zero(x.stream);
    return f.buf.p;
  }
  return it->second.buf.p;
}
static void scheme_checks(Ctx& x, bool limited) {
  bool coupled = false;
  for (int p = 0; p < x.P; ++p) coupled |= x.pkind[p] != 0;
  DFMI_CHECK(!limited || !coupled || x.have_bdelta, "limited schemes on a mesh with coupled patches need dfmi_init_boundary_delta");
  DFMI_CHECK(!limited || x.have_md, "limited schemes need mesh_distance (dfmi_init_constant_fields_internal)");
}

void u_assemble(Ctx& x) {
  Matrix& A = x.mU;
  const bool llv = x.sch.U == SCH_LLV;
  double* gout = llv ? scheme_buf(x, "gradU", x.C, 9) : x.fields.count("dbg_gradU") ? x.f("dbg_gradU") : nullptr;
  LAUNCH_W(k_u_grad, x.C, x.view(), x.st("U"), x.f("U"), x.f("boundary_U"), x.f("mu"), x.f("boundary_mu"),
         x.f("tauU"), x.f("boundary_tauU"), gout);
  halo_fields(x, {"tauU"});   // fvc_grad_vector_correctBC_processor (dfMatrixOpBase.cu:1366-1389)
  if (llv) {   // div(phi,U) limitedLinearV weights from this grad(U)
    scheme_checks(x, true);
    for (int p = 0; p < x.P; ++p)   // dfmi_set_scheme refuses it too; checked again here, where it is launched
      DFMI_CHECK(x.pkind[p] != 2, "div(phi,U) limitedLinearV on a decomposed mesh (processor patches) is not supported");
    if (x.fields.count("dbg_gradU"))
      DFMI_HIP(hipMemcpyAsync(x.f("dbg_gradU"), gout, 9 * sizeof(double) * x.C, hipMemcpyDeviceToDevice, x.stream));
    double* w = scheme_buf(x, "U_w", x.Fs, 1, true);
    double* bw = scheme_buf(x, "boundary_U_w", x.B, 1);
    const double twoByk = 2.0 / std::max(x.sch.k_U, 1e-15);
    LAUNCH(k_llv_w_face, x.Fs, x.view(), twoByk, x.f("phi"), x.f("U"), gout, w);
    LAUNCH(k_llv_w_slot, x.B, x.view(), x.st("U"), twoByk, x.f("boundary_phi"), x.f("U"), gout, bw);
  }
  LAUNCH_W(k_u_assemble, x.C, x.view(), x.st("U"), x.st("p"), x.f("rho"), x.f("rho_old"), x.f("U_old"),
           x.f("boundary_U"), x.f("phi"), x.f("boundary_phi"), x.f("mu"), x.f("boundary_mu"), x.f("p"),
           x.f("boundary_p"), x.f("tauU"), x.f("boundary_tauU"), A.lower.p, A.upper.p, A.diag.p, A.source.p,
           A.source_solve.p, A.ic.p, A.bc.p, x.f("rAU"), mixbc(x, "U"), x.sch_w(6), x.sch_w(7));
  k_bc_correct(x, "extrapolated", x.f("rAU"), x.f("boundary_rAU"), 1);
  halo_fields(x, {"rAU"});
}

void u_post_solve(Ctx& x) {
  k_bc_correct(x, "U", x.f("U"), x.f("boundary_U"), 3);
  halo_fields(x, {"U"});
  LAUNCH(k_kinetic, x.C, x.C, x.f("U"), x.f("K"));
  LAUNCH(k_kinetic_slots, x.B, x.B, x.f("boundary_U"), x.f("boundary_K"));
}

void u_hbya(Ctx& x) {
  Matrix& A = x.mU;
  LAUNCH_W(k_u_hbya, x.C, x.view(), x.st("U"), x.f("U"), x.f("boundary_U"), A.lower.p, A.upper.p, A.source.p,
         A.ic.p, A.bc.p, x.f("HbyA"));
  k_bc_correct(x, "extrapolated", x.f("HbyA"), x.f("boundary_HbyA"), 3);
  LAUNCH(k_hbya_scale_cells, x.C, x.C, x.f("rAU"), x.f("HbyA"));
  LAUNCH(k_hbya_scale_slots, x.B, x.B, x.st("U"), x.f("boundary_rAU"), x.f("boundary_U"), x.f("boundary_HbyA"));
  halo_fields(x, {"HbyA"});
}

void p_assemble(Ctx& x) {
  Matrix& A = x.mP;
  MeshView m = x.view();
  {
    // the cell walk over the owner-slot storage (measured 176 -> 150 us on the 2M box), else (face order)
    // face-parallel; one timer name for both (bench rooflines)
    const bool cellw = x.fslot;
    KScope _ks(x, "k_p_face");
    if (cellw && x.C > 0)
      hipLaunchKernelGGL(k_p_face_cell, dim3(blocks_for(x.C, TPB)), dim3(TPB), 0, x.stream, m, x.f("rho"), x.f("rAU"),
                         x.f("rho_old"), x.f("U_old"), x.f("phi_old"), x.f("HbyA"), x.f("rhorAUf"), x.f("phiHbyA"),
                         A.lower.p, A.upper.p);
    else if (!cellw && x.Fs > 0)
      hipLaunchKernelGGL(k_p_face, dim3(blocks_for(x.Fs, TPB)), dim3(TPB), 0, x.stream, m, x.f("rho"), x.f("rAU"),
                         x.f("rho_old"), x.f("U_old"), x.f("phi_old"), x.f("HbyA"), x.f("rhorAUf"), x.f("phiHbyA"),
                         A.lower.p, A.upper.p);
    DFMI_HIP(hipGetLastError());
  }
  LAUNCH(k_p_slot, x.B, m, x.st("p"), x.st("U"), x.f("rho"), x.f("boundary_rho"), x.f("rAU"), x.f("boundary_rAU"),
         x.f("rho_old"), x.f("boundary_rho_old"), x.f("U_old"), x.f("boundary_U_old"), x.f("boundary_phi_old"),
         x.f("HbyA"), x.f("boundary_HbyA"), x.f("boundary_p"), x.f("boundary_rhorAUf"), x.f("boundary_phiHbyA"),
         A.ic.p, A.bc.p, mixbc(x, "p"), x.f("boundary_phi"), x.f("boundary_psi"), x.f("boundary_p_gamma"),
         x.f("boundary_p_vf"));
  LAUNCH_W(k_p_cell, x.C, m, x.st("p"), A.lower.p, x.f("phiHbyA"), x.f("boundary_phiHbyA"), x.f("p"), x.f("p_old"),
         x.f("psi"), x.f("rho"), x.f("rho_old"), A.diag.p, A.source.p);
}

void p_post_solve(Ctx& x) {
  Matrix& A = x.mP;
  MeshView m = x.view();
  k_bc_correct(x, "p", x.f("p"), x.f("boundary_p"), 1);
  halo_fields(x, {"p"});
  LAUNCH(k_p_flux_face, x.Fs, m, x.f("phiHbyA"), A.lower.p, A.upper.p, x.f("p"), x.f("phi"));
  LAUNCH(k_p_flux_slot, x.B, m, x.st("p"), x.f("boundary_phiHbyA"), A.ic.p, A.bc.p, x.f("p"), x.f("boundary_p"),
         x.f("boundary_phi"));
  LAUNCH_W(k_p_cell_post, x.C, m, x.st("p"), x.f("p"), x.f("boundary_p"), x.f("p_old"), x.f("HbyA"), x.f("rAU"),
         x.f("U"), x.f("K"), x.f("dpdt"));
  k_bc_correct(x, "U", x.f("U"), x.f("boundary_U"), 3);
  halo_fields(x, {"U"});
  LAUNCH(k_kinetic_slots, x.B, x.B, x.f("boundary_U"), x.f("boundary_K"));
}

// species count: register-resident templates for 2..16 species, the chunked kernels above otherwise
// (or always, with the option fv.species_generic -- the parity tests run both on the same mechanisms)
bool species_generic(const Ctx& x) { return x.S > 16 || x.on("fv.species_generic"); }
#define DFMI_SWITCH_S(S, CALL, GEN)                                                              \
  if (species_generic(x)) { GEN; } else switch (S) {                                             \
    case 2: CALL(2); break; case 3: CALL(3); break; case 4: CALL(4); break; case 5: CALL(5); break; \
    case 6: CALL(6); break; case 7: CALL(7); break; case 8: CALL(8); break; case 9: CALL(9); break; \
    case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break;                  \
    case 13: CALL(13); break; case 14: CALL(14); break; case 15: CALL(15); break;                  \
    case 16: CALL(16); break;                                                                      \
    default: throw Error("dfmi: species count " + std::to_string(S) + " not supported");          \
  }

// div(phi,Yi_h) weights from this step's Y, he and phi (YEqn.H:6-14: the multivariate scheme is built at the
// start of YEqn and EEqn reuses it)
void conv_weights(Ctx& x) {
  if (x.sch.yh == SCH_UPWIND) return;
  scheme_checks(x, true);
  double* w = scheme_buf(x, "conv_w", x.Fs, 1, true);
  double* bw = scheme_buf(x, "boundary_conv_w", x.B, 1);
  const int b01 = x.sch.yh == SCH_LL01;
  const double twoByk = 2.0 / std::max(x.sch.k_yh, 1e-15);
  MeshView m = x.view();
  if (x.conv_list.n < (size_t)std::max(x.Fs, 1)) x.conv_list.alloc(std::max(x.Fs, 1));
  if (!x.conv_nlist.n) x.conv_nlist.alloc(1);
  DFMI_HIP(hipMemsetAsync(x.conv_nlist.p, 0, sizeof(int), x.stream));
  {
    KScope _ks(x, "k_conv_w_check");
    const int blocks = (int)((x.Fs + (long)CK_TPB * CK_FPT - 1) / ((long)CK_TPB * CK_FPT));
    if (blocks > 0)
      hipLaunchKernelGGL(k_conv_w_check, dim3(blocks), dim3(CK_TPB), 0, x.stream, m, x.S, b01, x.f("phi"), x.f("Y"),
                         x.f("he"), w, x.conv_list.p, x.conv_nlist.p);
    DFMI_HIP(hipGetLastError());
  }
  {
    KScope _ks(x, "k_conv_w_list");   // a fixed grid of 16-lane groups strides over the listed faces
    const int blocks = std::min(4096, std::max(1, blocks_for(x.Fs, 256 / CWG)));
    if (face_hex(x))
      hipLaunchKernelGGL(k_conv_w_list<-1>, dim3(blocks), dim3(256), 0, x.stream, m, x.S, x.st("Y"), x.st("he"), twoByk,
                         x.f("phi"), x.f("Y"), x.f("boundary_Y"), x.f("he"), x.f("boundary_he"), x.conv_list.p,
                         x.conv_nlist.p, w);
    else if (face_rows(x))
      hipLaunchKernelGGL(k_conv_w_list<6>, dim3(blocks), dim3(256), 0, x.stream, m, x.S, x.st("Y"), x.st("he"), twoByk,
                         x.f("phi"), x.f("Y"), x.f("boundary_Y"), x.f("he"), x.f("boundary_he"), x.conv_list.p,
                         x.conv_nlist.p, w);
    else
      hipLaunchKernelGGL(k_conv_w_list<0>, dim3(blocks), dim3(256), 0, x.stream, m, x.S, x.st("Y"), x.st("he"), twoByk,
                         x.f("phi"), x.f("Y"), x.f("boundary_Y"), x.f("he"), x.f("boundary_he"), x.conv_list.p,
                         x.conv_nlist.p, w);
    DFMI_HIP(hipGetLastError());
  }
  const double* bgx = nullptr;
  if (halo_active(x)) {   // processor faces: the neighbour cells' gradients (LimitedScheme::calcLimiter's pGradcN)
    double* g = scheme_buf(x, "conv_grad", x.C, 3 * (x.S + 1));
    bgx = scheme_buf(x, "boundary_conv_grad", x.B, 3 * (x.S + 1));
    LAUNCH(k_conv_proc_grad, x.B, m, x.S, x.st("Y"), x.st("he"), x.f("Y"), x.f("boundary_Y"), x.f("he"),
           x.f("boundary_he"), g);
    halo_fields(x, {"conv_grad"});
  }
  LAUNCH(k_conv_w_slot, x.B, m, x.S, x.st("Y"), x.st("he"), b01, twoByk, x.f("boundary_phi"), x.f("Y"),
         x.f("boundary_Y"), x.f("he"), x.f("boundary_he"), bgx, bw);
}

// div(phi,K) weights and div(hDiffCorrFlux)'s cubic correction (EEqn.H's fvc::div(phi, K), fvc::div(hDiffCorrFlux))
static void e_scheme_terms(Ctx& x) {
  MeshView m = x.view();
  if (x.sch.K != SCH_LINEAR) {
    const bool lim = x.sch.K == SCH_LL || x.sch.K == SCH_LL01;
    scheme_checks(x, false);
    double* w = scheme_buf(x, "K_w", x.Fs, 1, true);
    double* bw = scheme_buf(x, "boundary_K_w", x.B, 1);
    double* g = scheme_buf(x, "gradK", x.C, 3);
    double* bg = scheme_buf(x, "boundary_gradK", x.B, 3);
    if (lim) {
      DFMI_CHECK(x.have_md, "limited schemes need mesh_distance (dfmi_init_constant_fields_internal)");
      bool coupled = false;
      for (int p = 0; p < x.P; ++p) coupled |= x.pkind[p] != 0;
      DFMI_CHECK(!coupled || x.have_bdelta, "limited schemes on a mesh with coupled patches need dfmi_init_boundary_delta");
      if (face_hex(x)) LAUNCH((k_grad_cells<1, -1>), x.C, m, x.st("K"), x.f("K"), x.f("boundary_K"), g);
      else if (face_rows(x)) LAUNCH((k_grad_cells<1, 6>), x.C, m, x.st("K"), x.f("K"), x.f("boundary_K"), g);
      else LAUNCH((k_grad_cells<1, 0>), x.C, m, x.st("K"), x.f("K"), x.f("boundary_K"), g);
      halo_fields(x, {"gradK"});   // the neighbour cell's gradient on processor faces (patchNeighbourField)
    }
    // upwind: limiter 0 everywhere (Limited01 with bounds that reject every face)
    const int b01 = lim ? (x.sch.K == SCH_LL01) : 1;
    const double twoByk = 2.0 / std::max(x.sch.k_K, 1e-15);
    if (lim) {
      if (face_hex(x)) LAUNCH(k_lim_w_cell, x.C, m, b01, twoByk, x.f("phi"), x.f("K"), g, w);
      else LAUNCH(k_lim_w_face, x.Fs, m, b01, twoByk, x.f("phi"), x.f("K"), g, w);
      LAUNCH(k_lim_w_slot, x.B, m, x.st("K"), b01, twoByk, x.f("boundary_phi"), x.f("K"), x.f("boundary_K"), g, bg, bw);
    } else {
      LAUNCH(k_upwind_w_face, x.Fs, m, x.f("phi"), w);
      LAUNCH(k_upwind_w_slot, x.B, m, x.f("boundary_phi"), bw);
    }
  }
  if (x.sch.hD == SCH_CUBIC) {
    double* cf = scheme_buf(x, "cubic_flux", x.Fs, 1, true);
    double* bcf = scheme_buf(x, "boundary_cubic_flux", x.B, 1);
    double* g = scheme_buf(x, "gradHD", x.C, 9);
    scheme_buf(x, "boundary_gradHD", x.B, 9);
    if (face_hex(x)) LAUNCH((k_grad_cells<3, -1>), x.C, m, x.st("calculated"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), g);
    else if (face_rows(x)) LAUNCH((k_grad_cells<3, 6>), x.C, m, x.st("calculated"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), g);
    else LAUNCH((k_grad_cells<3, 0>), x.C, m, x.st("calculated"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), g);
    halo_fields(x, {"gradHD"});
    if (face_hex(x)) LAUNCH(k_cubic_cell, x.C, m, x.f("hDiffCorrFlux"), g, cf);
    else LAUNCH(k_cubic_face, x.Fs, m, x.f("hDiffCorrFlux"), g, cf);
    LAUNCH(k_cubic_slot, x.B, m, x.st("calculated"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), g,
           x.f("boundary_gradHD"), bcf);
  }
}

void y_prep(Ctx& x, bool weights) {
  if (weights) conv_weights(x);   // div(phi,Yi_h) weights of this step (before Y changes)
  MeshView m = x.view();
  double* gout = x.fields.count("dbg_gradY") ? x.f("dbg_gradY") : nullptr;
// (k_y_prep: the CSR walk measured faster than the gather rows -- 667 vs 848 us on the 2M box; its
// 243 VGPRs leave no room for the up-front row loads). Measured slower and removed (round 5): the species-outer
// row kernel (767-793 vs 657-673 us) and the z-marching tiles (811 vs 620 us), DESIGN.md 8.
  // LDS-staged brick kernel on hex boxes whose dimensions the brick divides (fv.yprep_brick = 0: off)
  const bool brick = face_hex(x) && !x.trav.n && x.hex[0] % YBX == 0 && x.hex[1] % YBY == 0 && x.hex[2] % YBZ == 0 &&
                     x.on("fv.yprep_brick");
#define CALL(NS)                                                                                                     \
  do {                                                                                                               \
    if (brick)                                                                                                       \
      LAUNCH_AS("k_y_prep", (k_y_prep_brick<NS, ybrick_sc(NS)>), x.C, m, x.st("Y"), x.f("Y"), x.f("boundary_Y"),    \
             x.f("rhoD"), x.f("boundary_rhoD"), x.f("hai"), x.f("boundary_hai"), x.f("alpha"), x.f("boundary_alpha"), \
             x.f("sumYDiffError"), x.f("boundary_sumYDiffError"), x.f("hDiffCorrFlux"),                              \
             x.f("boundary_hDiffCorrFlux"), x.f("diffAlphaD"), gout);                                               \
    else if (face_hex(x))                                                                                            \
      LAUNCH((k_y_prep<NS, -1>), x.C, m, x.st("Y"), x.f("Y"), x.f("boundary_Y"), x.f("rhoD"), x.f("boundary_rhoD"),  \
             x.f("hai"), x.f("boundary_hai"), x.f("alpha"), x.f("boundary_alpha"), x.f("sumYDiffError"),             \
             x.f("boundary_sumYDiffError"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), x.f("diffAlphaD"),  \
             gout);                                                                                                  \
    else                                                                                                             \
      LAUNCH((k_y_prep<NS, 0>), x.C, m, x.st("Y"), x.f("Y"), x.f("boundary_Y"), x.f("rhoD"), x.f("boundary_rhoD"),   \
             x.f("hai"), x.f("boundary_hai"), x.f("alpha"), x.f("boundary_alpha"), x.f("sumYDiffError"),             \
             x.f("boundary_sumYDiffError"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), x.f("diffAlphaD"),  \
             gout);                                                                                                  \
  } while (0)
  // the chunked kernel (4 species per chunk: 7.0 ms against 7.4-9.5 for chunks of 2 / 3 / 8 on 2M x 53 species) in
  // species ranges of YPREP_LCH species per launch (L2 locality of the neighbour gathers: 8.74 -> 8.56-8.62 ms
  // with 8 or 16), pass 1 over every range, then pass 2 (it reads the finished sumYDiffError)
#define GEN(CH)                                                                                                      \
  do {                                                                                                               \
    constexpr int lch = YPREP_LCH / CH * CH;                                                                         \
    for (int pass = 1; pass <= 2; ++pass)                                                                            \
      for (int s_lo = 0; s_lo < x.S; s_lo += lch)                                                                    \
        LAUNCH_SWG(k_y_prep_gen, CH, x.C, m, s_lo, std::min(x.S, s_lo + lch), pass, x.st("Y"), x.f("Y"),             \
                   x.f("boundary_Y"), x.f("rhoD"), x.f("boundary_rhoD"), x.f("hai"), x.f("boundary_hai"), x.f("alpha"), \
                   x.f("boundary_alpha"), x.f("sumYDiffError"), x.f("boundary_sumYDiffError"), x.f("hDiffCorrFlux"),  \
                   x.f("boundary_hDiffCorrFlux"), x.f("diffAlphaD"), pass == 1 ? gout : nullptr);                   \
  } while (0)
  DFMI_SWITCH_S(x.S, CALL, GEN(4))
#undef GEN
#undef CALL
  halo_fields(x, {"sumYDiffError", "hDiffCorrFlux"});
  LAUNCH(k_phiuc_face, x.Fs, m, x.f("sumYDiffError"), x.f("phiUc"));
  LAUNCH(k_phiuc_slot, x.B, m, x.st("Y"), x.f("sumYDiffError"), x.f("boundary_sumYDiffError"), x.f("boundary_phiUc"));
}

void y_assemble(Ctx& x) {
  Matrix& A = x.mY;
  MeshView m = x.view();
#define CALL(NS) LAUNCH_SW(k_y_assemble, NS, x.C, m, x.st("Y"), x.inert, x.f("Y"), x.f("boundary_Y"), x.f("rhoD"),   \
                        x.f("boundary_rhoD"), x.f("RR"), x.f("rho"), x.f("rho_old"), x.f("phi"), x.f("boundary_phi"), \
                        x.f("phiUc"), x.f("boundary_phiUc"), A.lower.p, A.upper.p, A.diag.p, A.source.p, A.ic.p, A.bc.p, mixbc(x, "Y"), x.sch_w(0), x.sch_w(1))
  DFMI_SWITCH_S(x.S, CALL,
                LAUNCH_SWG(k_y_assemble_gen, YCH, x.C, m, x.S, x.st("Y"), x.inert, x.f("Y"), x.f("boundary_Y"), x.f("rhoD"),
                       x.f("boundary_rhoD"), x.f("RR"), x.f("rho"), x.f("rho_old"), x.f("phi"), x.f("boundary_phi"),
                       x.f("phiUc"), x.f("boundary_phiUc"), A.lower.p, A.upper.p, A.diag.p, A.source.p, A.ic.p, A.bc.p, mixbc(x, "Y"), x.sch_w(0), x.sch_w(1)))
#undef CALL
}

void y_assemble_ell(Ctx& x, int W, long Ce, double* val, double* dS, double* rhs) {
  MeshView m = x.view();
  // (the z-marching tile form measured slower than this cell-parallel kernel, 961 vs 622 us, and is removed)
#define CALL(NS)                                                                                                     \
  LAUNCH_SW(k_y_assemble_ell, NS, x.C, m, x.st("Y"), x.inert, x.f("Y"), x.f("boundary_Y"), x.f("rhoD"),              \
            x.f("boundary_rhoD"), x.f("RR"), x.f("rho"), x.f("rho_old"), x.f("phi"),                                 \
            x.f("boundary_phi"), x.f("phiUc"), x.f("boundary_phiUc"), W, Ce, val, dS, rhs, mixbc(x, "Y"), x.sch_w(0), x.sch_w(1))
  // chunked kernel: 8 species per chunk, species ranges of YASM_LCH per launch (assembly 5.98 -> 5.86 ms per step
  // on 2M x 53 species with 8)
#define GEN(CH)                                                                                                      \
  do {                                                                                                               \
    constexpr int lch = YASM_LCH / CH * CH;                                                                          \
    for (int s_lo = 0; s_lo < x.S; s_lo += lch)                                                                      \
      LAUNCH_SWG(k_y_assemble_ell_gen, CH, x.C, m, s_lo, std::min(x.S, s_lo + lch), x.st("Y"), x.inert, x.f("Y"),    \
                 x.f("boundary_Y"), x.f("rhoD"), x.f("boundary_rhoD"), x.f("RR"), x.f("rho"), x.f("rho_old"), x.f("phi"), \
                 x.f("boundary_phi"), x.f("phiUc"), x.f("boundary_phiUc"), W, Ce, val, dS, rhs, mixbc(x, "Y"),       \
                 x.sch_w(0), x.sch_w(1));                                                                            \
  } while (0)
  DFMI_SWITCH_S(x.S, CALL, GEN(8))
#undef GEN
#undef CALL
}

void y_post_solve(Ctx& x) {
#define CALL(NS) LAUNCH(k_y_inert<NS>, x.C, x.C, x.inert, x.f("Y"))
  DFMI_SWITCH_S(x.S, CALL, LAUNCH(k_y_inert_gen, x.C, x.C, x.S, x.inert, x.f("Y")))
#undef CALL
  k_bc_correct(x, "Y", x.f("Y"), x.f("boundary_Y"), x.S);
  halo_fields(x, {"Y"});
}

// EEqn assembly in two parts: the scheme terms (K's limited weights from the UEqn's K, hDiffCorrFlux's cubic
// correction from the YEqn preparation) read nothing of the Y solve; the boundary energy gradient (the
// thermo at the solved boundary Y), he's boundary values and the matrix come after it
void e_assemble_front(Ctx& x) { e_scheme_terms(x); }
void e_assemble_back(Ctx& x) {
  Matrix& A = x.mE;
  MeshView m = x.view();
  thermo_energy_gradient(x);   // eeqn_calculate_energy_gradient (dfEEqn.cu:148, :266-287)
  k_bc_correct(x, "he", x.f("he"), x.f("boundary_he"), 1);
  const double* eg = x.f("boundary_heGradient");
  LAUNCH_W(k_e_assemble, x.C, m, x.st("he"), x.st("K"), x.f("he"), x.f("boundary_he"), x.f("rho"), x.f("rho_old"),
         x.f("K"), x.f("K_old"), x.f("boundary_K"), x.f("phi"), x.f("boundary_phi"), x.f("alpha"),
         x.f("boundary_alpha"), x.f("hDiffCorrFlux"), x.f("boundary_hDiffCorrFlux"), x.f("dpdt"), x.f("diffAlphaD"),
         eg, A.lower.p, A.upper.p, A.diag.p, A.source.p, A.ic.p, A.bc.p, x.sch_w(0), x.sch_w(1), x.sch_w(2),
         x.sch_w(3), x.sch_w(4), x.sch_w(5));
}
void e_assemble(Ctx& x) {
  e_assemble_front(x);
  e_assemble_back(x);
}

void e_post_solve(Ctx& x) {
  k_bc_correct(x, "he", x.f("he"), x.f("boundary_he"), 1);
  halo_fields(x, {"he"});
}

// one df0DFoam time step (df0DFoam.C:99-113, constantProperty pressure): chemistry.solve(deltaT) on
// every cell (a closed isothermal reactor from setState_TPY, RR scaled by the thermo rho), YEqn
// (ddt(rho, Yi) == RR), EEqn (he held: constant pressure) -> correctThermo (T from he), rho = thermo.rho()
void zero_d_step(Ctx& x, double dt) {
  DFMI_CHECK(x.chem.mode == 1 || x.chem.mode == 2, "0D step: chemistry mode must be 1 (ODE) or 2 (DNN)");
  DFMI_HIP(hipMemcpyAsync(x.f("rho_old"), x.f("rho"), sizeof(double) * x.C, hipMemcpyDeviceToDevice, x.stream));
  if (x.chem.mode == 1) chem_solve(x, dt, "rho");
  else dnn_solve(x, "rho");
  LAUNCH(k_zero_d_species, x.C, x.C, x.S, x.inert, 1.0 / dt, x.V.p, x.f("rho_old"), x.f("rho"), x.f("RR"), x.f("Y"));
  k_bc_correct(x, "Y", x.f("Y"), x.f("boundary_Y"), x.S);
  thermo_correct(x, false);
  thermo_rho_from_psi(x);
}

// ---- measured HBM copy peak (diagnostic): streaming copies with 16-B vector loads/stores, U vectors per
// thread (all loads issued before the stores), one pass over the buffer; the best of U = 1, 2, 4, 8 is the
// measured peak (read + write bytes / time), the reference point for `roofline.achieved` beside 8 TB/s.
template <int U>
__global__ void __launch_bounds__(256) k_stream_copy(long n, const double2* __restrict__ a, double2* __restrict__ b) {
  const long base = (long)blockIdx.x * 256 * U + threadIdx.x;
  double2 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long i = base + (long)k * 256;
    if (i < n) v[k] = a[i];
  }
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long i = base + (long)k * 256;
    if (i < n) b[i] = v[k];
  }
}

template <int U> double stream_copy_gbs(Ctx& x, long n, const double2* a, double2* b, int reps) {
  const dim3 g((unsigned)((n + 256L * U - 1) / (256L * U))), bl(256);
  hipLaunchKernelGGL(k_stream_copy<U>, g, bl, 0, x.stream, n, a, b);
  hipEvent_t e0, e1;
  DFMI_HIP(hipEventCreate(&e0)); DFMI_HIP(hipEventCreate(&e1));
  DFMI_HIP(hipEventRecord(e0, x.stream));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_stream_copy<U>, g, bl, 0, x.stream, n, a, b);
  DFMI_HIP(hipEventRecord(e1, x.stream));
  DFMI_HIP(hipEventSynchronize(e1));
  float ms = 0.0f;
  DFMI_HIP(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
  return 2.0 * (double)n * sizeof(double2) * reps / (ms / 1e3) / 1e9;
}

double hbm_copy_gbs(Ctx& x, size_t bytes, int reps) {
  const long n = (long)(bytes / sizeof(double2));
  DevBuf<double2> a, b;
  a.alloc(n); b.alloc(n);
  DFMI_HIP(hipMemsetAsync(a.p, 0, n * sizeof(double2), x.stream));
  double best = 0.0;
  best = std::max(best, stream_copy_gbs<1>(x, n, a.p, b.p, reps));
  best = std::max(best, stream_copy_gbs<2>(x, n, a.p, b.p, reps));
  best = std::max(best, stream_copy_gbs<4>(x, n, a.p, b.p, reps));
  best = std::max(best, stream_copy_gbs<8>(x, n, a.p, b.p, reps));
  return best;
}

void thermo_rho_from_psi(Ctx& x) {   // dfThermo::updateRho (dfThermo.cu:673-679)
  LAUNCH(k_mul, x.C, (long)x.C, x.f("p"), x.f("psi"), x.f("rho"));
  LAUNCH(k_mul, x.B, (long)x.B, x.f("boundary_p"), x.f("boundary_psi"), x.f("boundary_rho"));
}
void thermo_psip0(Ctx& x) {          // dfThermo::psip0 (:681-686)
  LAUNCH(k_mul, x.C, (long)x.C, x.f("psi"), x.f("p"), x.f("psip0"));
  LAUNCH(k_mul, x.B, (long)x.B, x.f("boundary_psi"), x.f("boundary_p"), x.f("boundary_psip0"));
}
void thermo_correct_psip_rho(Ctx& x) {   // dfThermo::correctPsipRho (:688-695)
  LAUNCH(k_add_psip, x.C, (long)x.C, x.f("p"), x.f("psi"), x.f("psip0"), x.f("rho"));
  LAUNCH(k_add_psip, x.B, (long)x.B, x.f("boundary_p"), x.f("boundary_psi"), x.f("boundary_psip0"), x.f("boundary_rho"));
}

}  // namespace dfmi
