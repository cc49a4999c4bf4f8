// amg.hip -- aggregation-AMG V-cycle preconditioner for the pressure PCG (replaces AmgX's
// AGGREGATION / V-cycle p solver, reference examples/.../system/amgxpOptions:1-18,
// src_gpu/AmgXSolver.cu:184-340).
//
// Hierarchy (built once per mesh on the host, since it depends only on geometry): three greedy
// pairwise-matching passes per level on the strength graph |Sf| * deltaCoeffs (the geometric part
// of the laplacian coefficients), so a uniform hex mesh coarsens 2x2x2 per level (AmgX SIZE_2
// selector, applied three times). Aggregates never cross ranks: the preconditioner is rank-local
// (block-Jacobi across processor faces); the outer PCG SpMV carries the halo.
// Per solve: Galerkin coarse operators P^T A P (piecewise-constant P) are summed on the device from
// precomputed contribution lists in a fixed order -- deterministic, no atomics.
// V-cycle: one weighted-Jacobi pre-sweep from zero (fused into the residual pass), restriction,
// coarse correction, prolongation fused with one post-sweep; the coarsest level (<= 4096 cells) is
// smoothed by a fixed number of Jacobi sweeps inside one workgroup (LDS-resident vectors). All pieces
// are linear and the pre/post sweeps are adjoint, so the preconditioner is symmetric (valid for CG).
#include "dfmi_ctx.h"
#include "amg.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>

namespace dfmi {
namespace {

constexpr int TPB = 256;
constexpr int COARSEST = 1024;   // k_coarsest capacity (cells); also n * W <= LDS_ENT
constexpr int CTPB = 1024;

// ---------------------------------------------------------------- kernels
// coarse values: out[s * nc + I] = sum of the fine sources listed for (slot s, cell I)
__global__ void k_galerkin(int nc, int slots, const int* __restrict__ gstart, const int* __restrict__ gsrc,
                           const double* __restrict__ fval, const double* __restrict__ fD, double* __restrict__ cval,
                           double* __restrict__ cD) {
  const int I = blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= nc) return;
  for (int s = 0; s < slots; ++s) {
    const long e0 = gstart[(long)s * nc + I], e1 = gstart[(long)s * nc + I + 1];
    double a = 0.0;
    for (long e = e0; e < e1; ++e) {
      const int src = gsrc[e];
      a += src >= 0 ? fval[src] : fD[-src - 1];
    }
    if (s < slots - 1) cval[(long)s * nc + I] = a;
    else cD[I] = a;
  }
}

// x = omega b / D (first sweep from zero); r = b - A x   (columns >= n: other ranks, dropped)
template <int WT>
__global__ void __launch_bounds__(TPB) k_smooth_res(int n, int W_, const int* __restrict__ col,
                                                    const double* __restrict__ val, const double* __restrict__ D,
                                                    const double* __restrict__ b, double omega,
                                                    double* __restrict__ x, double* __restrict__ r) {
  const int W = WT > 0 ? WT : W_;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const double xc = omega * b[c] / D[c];
  double y = D[c] * xc;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const int j = col[(long)k * n + c];
    if (j < n) y += val[(long)k * n + c] * (omega * b[j] / D[j]);
  }
  x[c] = xc;
  r[c] = b[c] - y;
}

__global__ void k_restrict(int nc, const int* __restrict__ mstart, const int* __restrict__ members,
                           const double* __restrict__ r, double* __restrict__ bc) {
  const int I = blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= nc) return;
  double a = 0.0;
  for (int e = mstart[I]; e < mstart[I + 1]; ++e) a += r[members[e]];
  bc[I] = a;
}

// y = x + P xc; out = y + omega (b - A y) / D; optional block partials of b.out (level 0: r.z)
template <int WT>
__global__ void __launch_bounds__(TPB) k_prolong_smooth(int n, int W_, const int* __restrict__ col,
                                                        const double* __restrict__ val, const double* __restrict__ D,
                                                        const double* __restrict__ b, const double* __restrict__ x,
                                                        const int* __restrict__ agg, const double* __restrict__ xc,
                                                        double omega, double* __restrict__ out, double* partial) {
  const int W = WT > 0 ? WT : W_;
  __shared__ double sh[TPB / 64];
  double acc = 0.0;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const double yc = x[c] + xc[agg[c]];
    double ay = D[c] * yc;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int j = col[(long)k * n + c];
      if (j < n) ay += val[(long)k * n + c] * (x[j] + xc[agg[j]]);
    }
    const double o = yc + omega * (b[c] - ay) / D[c];
    out[c] = o;
    acc += b[c] * o;
  }
  if (!partial) return;
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int w = 0; w < TPB / 64; ++w) a += sh[w];
    partial[blockIdx.x] = a;
  }
}

__global__ void k_dot_partial(int n, const double* __restrict__ a, const double* __restrict__ b, double* partial) {
  __shared__ double sh[TPB / 64];
  double acc = 0.0;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) acc += a[c] * b[c];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < TPB / 64; ++w) s += sh[w];
    partial[blockIdx.x] = s;
  }
}

// coarsest level: `sweeps` weighted-Jacobi sweeps from zero in one workgroup; operator and vectors
// staged in LDS (n * W <= LDS_ENT), so the sweeps run at LDS latency
constexpr int LDS_ENT = 6144;
__global__ void __launch_bounds__(CTPB) k_coarsest(int n, int W, const int* __restrict__ col,
                                                   const double* __restrict__ val, const double* __restrict__ D,
                                                   const double* __restrict__ b, double omega, int sweeps,
                                                   double* __restrict__ x) {
  __shared__ double xa[COARSEST], xb[COARSEST];
  __shared__ double sv[LDS_ENT];
  __shared__ int sc[LDS_ENT];
  __shared__ double sd[COARSEST], sb[COARSEST];
  for (int e = threadIdx.x; e < n * W; e += CTPB) { sv[e] = val[e]; sc[e] = col[e]; }
  for (int c = threadIdx.x; c < n; c += CTPB) { sd[c] = D[c]; sb[c] = b[c]; xa[c] = omega * b[c] / D[c]; }
  __syncthreads();
  double* cur = xa;
  double* nxt = xb;
  for (int s = 1; s < sweeps; ++s) {
    for (int c = threadIdx.x; c < n; c += CTPB) {
      double y = sd[c] * cur[c];
      for (int k = 0; k < W; ++k) {
        const int j = sc[k * n + c];
        if (j < n) y += sv[k * n + c] * cur[j];
      }
      nxt[c] = cur[c] + omega * (sb[c] - y) / sd[c];
    }
    __syncthreads();
    double* t = cur; cur = nxt; nxt = t;
  }
  for (int c = threadIdx.x; c < n; c += CTPB) x[c] = cur[c];
}

// ---------------------------------------------------------------- host: hierarchy
struct Graph {                  // symmetric strength graph, CSR, no self entries
  int n = 0;
  std::vector<int> start, adj;
  std::vector<double> w;
};

// one greedy pairwise matching on g: each unmatched vertex (in index order) pairs with its
// strongest unmatched neighbour (ties: lowest index). Returns group id per vertex, group count.
int pair_match(const Graph& g, std::vector<int>& grp) {
  grp.assign(g.n, -1);
  int ng = 0;
  for (int v = 0; v < g.n; ++v) {
    if (grp[v] >= 0) continue;
    int best = -1;
    double bw = -1.0;
    for (int e = g.start[v]; e < g.start[v + 1]; ++e) {
      const int u = g.adj[e];
      if (u == v || grp[u] >= 0) continue;
      // strengths within 1e-9 relative are ties (rounding must not break the geometric pattern)
      if (g.w[e] > bw * (1 + 1e-9)) { bw = g.w[e]; best = u; }
      else if (std::fabs(g.w[e] - bw) <= 1e-9 * bw && u < best) best = u;
    }
    grp[v] = ng;
    if (best >= 0) grp[best] = ng;
    ++ng;
  }
  return ng;
}

// collapse g by a grouping (edge strengths summed, intra-group edges dropped)
Graph collapse(const Graph& g, const std::vector<int>& grp, int ng) {
  std::vector<std::vector<std::pair<int, double>>> e(ng);
  for (int v = 0; v < g.n; ++v)
    for (int k = g.start[v]; k < g.start[v + 1]; ++k) {
      const int a = grp[v], b = grp[g.adj[k]];
      if (a != b) e[a].push_back({b, g.w[k]});
    }
  Graph c;
  c.n = ng;
  c.start.assign(ng + 1, 0);
  for (int a = 0; a < ng; ++a) {
    auto& l = e[a];
    std::sort(l.begin(), l.end(), [](auto& x, auto& y) { return x.first < y.first; });
    std::vector<std::pair<int, double>> m;
    for (auto& p : l) {
      if (!m.empty() && m.back().first == p.first) m.back().second += p.second;
      else m.push_back(p);
    }
    for (auto& p : m) { c.adj.push_back(p.first); c.w.push_back(p.second); }
    c.start[a + 1] = (int)c.adj.size();
  }
  return c;
}

// Build the next level from level `f` (ELL cols [Wf][nf], strength graph g). Fills f's agg/members
// and galerkin maps, returns the coarse level's ELL structure and strength graph.
void build_next(AmgLevel& f, const std::vector<int>& fcol, const Graph& g, AmgLevel& c, std::vector<int>& ccol,
                Graph& cg, hipStream_t st) {
  const int nf = f.n, Wf = f.W;
  // three pairwise passes -> aggregates of up to 8
  std::vector<int> agg(nf);
  std::iota(agg.begin(), agg.end(), 0);
  Graph cur = g;
  int ng = nf;
  for (int pass = 0; pass < 3; ++pass) {
    std::vector<int> grp;
    ng = pair_match(cur, grp);
    for (int v = 0; v < nf; ++v) agg[v] = grp[agg[v]];
    cur = collapse(cur, grp, ng);
  }
  // renumber coarse cells by their first fine member (locality)
  std::vector<int> first(ng, INT32_MAX);
  for (int v = 0; v < nf; ++v) first[agg[v]] = std::min(first[agg[v]], v);
  std::vector<int> ord(ng);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](int a, int b) { return first[a] < first[b]; });
  std::vector<int> ren(ng);
  for (int i = 0; i < ng; ++i) ren[ord[i]] = i;
  for (int v = 0; v < nf; ++v) agg[v] = ren[agg[v]];
  const int nc = ng;
  // coarse strength graph (same collapse, renumbered)
  cg = collapse(g, agg, nc);
  // members
  std::vector<int> mstart(nc + 1, 0), members(nf);
  for (int v = 0; v < nf; ++v) mstart[agg[v] + 1]++;
  for (int i = 0; i < nc; ++i) mstart[i + 1] += mstart[i];
  {
    std::vector<int> pos(mstart.begin(), mstart.end() - 1);
    for (int v = 0; v < nf; ++v) members[pos[agg[v]]++] = v;
  }
  // coarse ELL columns: sorted unique neighbour aggregates over rank-local fine couplings
  std::vector<std::vector<int>> nb(nc);
  for (int v = 0; v < nf; ++v)
    for (int k = 0; k < Wf; ++k) {
      const int j = fcol[(size_t)k * nf + v];
      if (j >= nf || j == v) continue;    // halo or padding
      const int A = agg[v], Bc = agg[j];
      if (A != Bc) nb[A].push_back(Bc);
    }
  int Wc = 1;
  for (auto& l : nb) {
    std::sort(l.begin(), l.end());
    l.erase(std::unique(l.begin(), l.end()), l.end());
    Wc = std::max(Wc, (int)l.size());
  }
  ccol.assign((size_t)Wc * nc, 0);
  for (int I = 0; I < nc; ++I)
    for (int k = 0; k < Wc; ++k) ccol[(size_t)k * nc + I] = k < (int)nb[I].size() ? nb[I][k] : I;
  // Galerkin contribution lists: slot k < Wc -> coarse entry (I, nb[I][k]); slot Wc -> diagonal.
  // Fine sources in (member ascending, fine slot ascending) order; fine diag first per member.
  const int slots = Wc + 1;
  std::vector<std::vector<int>> lists((size_t)slots * nc);
  for (int I = 0; I < nc; ++I) {
    for (int e = mstart[I]; e < mstart[I + 1]; ++e) {
      const int v = members[e];
      lists[(size_t)Wc * nc + I].push_back(-(v + 1));
      for (int k = 0; k < Wf; ++k) {
        const int j = fcol[(size_t)k * nf + v];
        if (j >= nf || j == v) continue;
        const int src = k * nf + v;
        const int Bc = agg[j];
        if (Bc == I) lists[(size_t)Wc * nc + I].push_back(src);
        else {
          const int kk = (int)(std::lower_bound(nb[I].begin(), nb[I].end(), Bc) - nb[I].begin());
          lists[(size_t)kk * nc + I].push_back(src);
        }
      }
    }
  }
  std::vector<int> gstart((size_t)slots * nc + 1, 0), gsrc;
  for (size_t s = 0; s < lists.size(); ++s) {
    for (int v : lists[s]) gsrc.push_back(v);
    gstart[s + 1] = (int)gsrc.size();
  }
  if (gsrc.empty()) gsrc.push_back(0);
  f.agg.upload(agg, st);
  f.mstart.upload(mstart, st);
  f.members.upload(members, st);
  f.gstart.upload(gstart, st);
  f.gsrc.upload(gsrc, st);
  c.n = nc;
  c.W = Wc;
  c.col.upload(ccol, st);
  c.val.alloc((size_t)Wc * nc);
  c.D.alloc(nc);
  c.b.alloc(nc); c.x.alloc(nc); c.r.alloc(nc); c.xo.alloc(nc);
}

double env_d(const char* k, double d) { const char* v = std::getenv(k); return v ? std::atof(v) : d; }

}  // namespace

void amg_setup(Ctx& x) {
  Amg& a = x.amg;
  a.lv.clear();
  a.omega = env_d("DFMI_AMG_OMEGA", 0.85);
  a.coarse_sweeps = (int)env_d("DFMI_AMG_COARSE_SWEEPS", 8);
  a.coarsest = std::min(COARSEST, std::max(8, (int)env_d("DFMI_AMG_COARSEST", 512)));
  const int C = x.C;
  // level 0: the solver ELL (columns >= C are halo entries, dropped in the preconditioner)
  std::vector<int> col((size_t)x.ell.W * C);
  DFMI_HIP(hipMemcpy(col.data(), x.ell.col.p, col.size() * sizeof(int), hipMemcpyDeviceToHost));
  // geometric strength |Sf| * deltaCoeffs per coupling (faces and cyclic slots)
  std::vector<double> mag(x.F), dcf(x.F), bmag(x.B), bdc(x.B);
  if (x.F) {
    DFMI_HIP(hipMemcpy(mag.data(), x.magSf.p, x.F * sizeof(double), hipMemcpyDeviceToHost));
    DFMI_HIP(hipMemcpy(dcf.data(), x.dc.p, x.F * sizeof(double), hipMemcpyDeviceToHost));
  }
  if (x.B) {
    DFMI_HIP(hipMemcpy(bmag.data(), x.bmagSf.p, x.B * sizeof(double), hipMemcpyDeviceToHost));
    DFMI_HIP(hipMemcpy(bdc.data(), x.bdc.p, x.B * sizeof(double), hipMemcpyDeviceToHost));
  }
  Graph g;
  g.n = C;
  {
    std::vector<std::vector<std::pair<int, double>>> e(C);
    for (int f = 0; f < x.F; ++f) {
      const double s = mag[f] * dcf[f];
      e[x.h_own[f]].push_back({x.h_nei[f], s});
      e[x.h_nei[f]].push_back({x.h_own[f], s});
    }
    for (int p = 0; p < x.P; ++p) {
      if (x.pkind[p] != 1) continue;
      const int q = x.cyc_nbr[p];
      for (int i = 0; i < x.psize[p]; ++i) {
        const int b = x.poff[p] + i;
        const int c = x.h_bfc[b], o = x.h_bfc[x.poff[q] + i];
        if (c != o) e[c].push_back({o, bmag[b] * bdc[b]});
      }
    }
    g.start.assign(C + 1, 0);
    for (int c = 0; c < C; ++c) {
      auto& l = e[c];
      std::sort(l.begin(), l.end(), [](auto& u, auto& v) { return u.first < v.first; });
      std::vector<std::pair<int, double>> m;
      for (auto& p : l) {
        if (!m.empty() && m.back().first == p.first) m.back().second += p.second;
        else m.push_back(p);
      }
      for (auto& p : m) { g.adj.push_back(p.first); g.w.push_back(p.second); }
      g.start[c + 1] = (int)g.adj.size();
    }
  }
  a.lv.emplace_back();
  a.lv[0].n = C;
  a.lv[0].W = x.ell.W;
  a.lv[0].x.alloc(C); a.lv[0].r.alloc(C); a.lv[0].xo.alloc(C);
  std::vector<int> fcol = col;
  auto too_big = [&](const AmgLevel& l) { return l.n > a.coarsest || (size_t)l.n * l.W > 6144; };
  while (too_big(a.lv.back())) {
    AmgLevel c;
    std::vector<int> ccol;
    Graph cg;
    build_next(a.lv.back(), fcol, g, c, ccol, cg, x.stream);
    DFMI_HIP(hipStreamSynchronize(x.stream));
    const bool stalled = c.n * 2 > a.lv.back().n;
    a.lv.push_back(std::move(c));
    fcol.swap(ccol);
    g = std::move(cg);
    if (stalled) break;
  }
  DFMI_CHECK(!too_big(a.lv.back()) || a.lv.back().n <= 8, "AMG coarsening stalled above the coarsest-level capacity");
  a.ready = true;
}

// Per solve: coarse operators from the level-0 values (val0 [W][C], D0 = diag + internalCoeffs).
void amg_galerkin(Ctx& x, const double* val0, const double* D0) {
  Amg& a = x.amg;
  const double* fv = val0;
  const double* fD = D0;
  for (size_t l = 0; l + 1 < a.lv.size(); ++l) {
    AmgLevel& f = a.lv[l];
    AmgLevel& c = a.lv[l + 1];
    KScope _ks(x, "k_galerkin");
    hipLaunchKernelGGL(k_galerkin, dim3(blocks_for(c.n, TPB)), dim3(TPB), 0, x.stream, c.n, c.W + 1, f.gstart.p,
                       f.gsrc.p, fv, fD, c.val.p, c.D.p);
    DFMI_HIP(hipGetLastError());
    fv = c.val.p;
    fD = c.D.p;
  }
}

// z = M^-1 r; block partials of r.z (one per block of the level-0 grid) into `partial`
void amg_apply(Ctx& x, const double* val0, const double* D0, const int* col0, const double* r, double* z,
               double* partial, int nblk) {
  Amg& a = x.amg;
  const int L = (int)a.lv.size();
  const double om = a.omega;
  auto VAL = [&](int l) { return l == 0 ? val0 : (const double*)a.lv[l].val.p; };
  auto DD = [&](int l) { return l == 0 ? D0 : (const double*)a.lv[l].D.p; };
  auto COL = [&](int l) { return l == 0 ? col0 : (const int*)a.lv[l].col.p; };
  auto B = [&](int l) { return l == 0 ? r : (const double*)a.lv[l].b.p; };
  // down
  for (int l = 0; l + 1 < L; ++l) {
    AmgLevel& f = a.lv[l];
    {
      KScope _ks(x, "k_smooth_res");
      if (f.W == 6)
        hipLaunchKernelGGL(k_smooth_res<6>, dim3(blocks_for(f.n, TPB)), dim3(TPB), 0, x.stream, f.n, f.W, COL(l),
                           VAL(l), DD(l), B(l), om, f.x.p, f.r.p);
      else
        hipLaunchKernelGGL(k_smooth_res<0>, dim3(blocks_for(f.n, TPB)), dim3(TPB), 0, x.stream, f.n, f.W, COL(l),
                           VAL(l), DD(l), B(l), om, f.x.p, f.r.p);
    }
    {
      KScope _ks(x, "k_restrict");
      hipLaunchKernelGGL(k_restrict, dim3(blocks_for(a.lv[l + 1].n, TPB)), dim3(TPB), 0, x.stream, a.lv[l + 1].n,
                         f.mstart.p, f.members.p, f.r.p, a.lv[l + 1].b.p);
    }
  }
  // coarsest
  {
    AmgLevel& c = a.lv[L - 1];
    KScope _ks(x, "k_coarsest");
    hipLaunchKernelGGL(k_coarsest, dim3(1), dim3(CTPB), 0, x.stream, c.n, c.W, COL(L - 1), VAL(L - 1), DD(L - 1),
                       B(L - 1), om, a.coarse_sweeps, L == 1 ? z : c.x.p);
  }
  if (L == 1) {
    KScope _ks(x, "k_dot_partial");
    hipLaunchKernelGGL(k_dot_partial, dim3(nblk), dim3(TPB), 0, x.stream, x.C, r, (const double*)z, partial);
  }
  // up
  for (int l = L - 2; l >= 0; --l) {
    AmgLevel& f = a.lv[l];
    double* out = l == 0 ? z : f.xo.p;
    KScope _ks(x, "k_prolong_smooth");
    const dim3 grid = l == 0 ? dim3(nblk) : dim3(blocks_for(f.n, TPB));
    if (f.W == 6)
      hipLaunchKernelGGL(k_prolong_smooth<6>, grid, dim3(TPB), 0, x.stream, f.n, f.W, COL(l), VAL(l), DD(l), B(l),
                         f.x.p, f.agg.p, a.lv[l + 1].x.p, om, out, l == 0 ? partial : nullptr);
    else
      hipLaunchKernelGGL(k_prolong_smooth<0>, grid, dim3(TPB), 0, x.stream, f.n, f.W, COL(l), VAL(l), DD(l), B(l),
                         f.x.p, f.agg.p, a.lv[l + 1].x.p, om, out, l == 0 ? partial : nullptr);
    if (l > 0) std::swap(f.x, f.xo);   // the corrected x of this level feeds the next finer prolongation
  }
  DFMI_HIP(hipGetLastError());
}

}  // namespace dfmi
