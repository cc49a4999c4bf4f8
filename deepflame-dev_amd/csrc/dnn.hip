// dnn.hip -- DF-ODENet chemistry surrogate on MI355X.
//
// Reference: dfChemistrySolver::Inference (src_gpu/dfChemistrySolver.cu:129-206) with the model of
// test/Tu500K-Phi1/inference.py:12-25 (NN_MLP: Linear + GELU stacks, one net per non-inert species,
// run in half precision). Per reacting cell (T >= 610 K):
//   x = [T, 101325, BCT(Y_0..Y_{S-1})], BCT(y) = (y^0.1 - 1) / 0.1, normalised (x - Xmu) / Xstd;
//   out_i = net_i(x) (i < S-1);  y_i = invBCT(out_i Ystd_i + Ymu_i + BCT(Y_i));
//   y_i /= (sum_{i<S-1} y_i + Y_inert);  RR_i = (y_i - Y_i) rho (p / 101325) / dt_infer.
// (construct_init_input :4-23, normalize_input :25-35, calculate_y_new :37-51, calculate_RR :53-75.)
//
// MI355X design: the reacting cells are compacted on the device (deterministic scan), then every
// hidden layer of all S-1 nets is ONE batched GEMM launch (grid.z = net) on MFMA
// v_mfma_f32_32x32x16_f16 with fp32 accumulation and the bias + exact-erf GELU + fp16 rounding fused
// into the epilogue; the 1-wide output layer and the BCT post-processing are fused into one kernel.
// GEMM tile 128x128x32, 4 waves (2x2, 64x64 each = 2x2 MFMA tiles), both operands streamed
// global -> LDS by DMA (global_load_lds, swizzled rows) through a 3-buffer ring, A and W both
// K-contiguous (W in torch Linear [out][in] layout), K and activation row strides padded to 64.
#include "dfmi_ctx.h"
#include <cmath>

namespace dfmi {
namespace {

using half8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int NBUF = 3;                   // LDS ring: two K tiles in flight while one feeds the MFMAs
constexpr int GT = 256;
constexpr int KPAD = 64;                  // every GEMM K (and activation row stride) is a multiple of this
constexpr int TILE_H = BM * BK;           // halves per staged operand tile (8 KiB)

// GELU for the GEMM epilogue: erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, branch-free), three
// orders of magnitude below the fp16 rounding the result goes through (torch's GELU is the exact-erf
// form); the library erff branches per lane on |x| < 1 and dominated the epilogue of the shallow
// (K = 11) first layer
__device__ __forceinline__ float gelu_fast(float v) {
  const float u = v * 0.70710678118654752440f, a = fabsf(u);
  const float t = __frcp_rn(1.0f + 0.3275911f * a);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float e = 1.0f - poly * __expf(-a * a);
  return 0.5f * v * (1.0f + copysignf(e, u));
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4): lane l's 16 bytes land at lds_wave + 16 l
__device__ __forceinline__ void glds16(const _Float16* g, _Float16* lds_wave) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave, 16, 0, 0);
}

// 16-B chunk c (of 4 per 64-B row) of row `row` lives at chunk c ^ ((row >> 2) & 3): the 16 rows a
// ds_read_b128 lane group reads ({0-3,12-15,20-27}, {4-11,16-19,28-31} of each half-wave) then hit 16
// distinct bank slots (conflict-free)
__device__ __forceinline__ int swz(int row, int c) { return c ^ ((row >> 2) & 3); }

// C[z][M][ldc] = act(A[z][M][lda] . W[z][N][K]^T + b[z][N]) for columns < N, 0 for N <= col < ldc;
// fp16 in/out, fp32 accumulate. K, lda, ldc multiples of 64.
// Block tile 128x128x32, 4 waves each owning a 64x64 quadrant (2x2 v_mfma_f32_32x32x16_f16 tiles).
// Both operand tiles are streamed global -> LDS by DMA (global_load_lds, 16 B per lane, 4 DMA
// instructions per thread per K tile) through a 3-buffer ring: tiles k+1 and k+2 are in flight while
// tile k feeds the MFMAs; the wait before each barrier is counted (vmcnt(4): the newest tile stays in
// flight) and the barrier is a raw s_barrier, so nothing drains the DMA queue inside the loop. The
// swizzle is applied on the global source address (each DMA still writes 1 KiB contiguously). 48 KiB
// LDS: three blocks per CU. Block ids are remapped so the consecutive ids that share an XCD walk the
// N tiles of one M tile (A rows re-read from that XCD's L2).
template <bool GELU>
__global__ void __launch_bounds__(GT, 3) k_mlp_gemm(int M, int N, int K, const _Float16* __restrict__ A, int lda,
                                                    long sA, const _Float16* __restrict__ W, long sW,
                                                    const float* __restrict__ bias, long sb,
                                                    _Float16* __restrict__ Cout, int ldc, long sC) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[NBUF * 2 * TILE_H];   // [buf][A | W][128][32]
  const int z = blockIdx.z;
  A += z * sA; W += z * sW; bias += z * sb; Cout += z * sC;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM, nwg = ntn * ntm;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // staging: wave w fills rows [32 w, 32 w + 32) of both tiles, 16 rows (1 KiB) per DMA instruction
  const _Float16* pa[2];
  const _Float16* pw[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 32 + i * 16 + (lane >> 2);
    const int gc = swz(row, lane & 3);
    const int ga = min(m0 + row, M - 1), gw = min(n0 + row, N - 1);   // clamped rows are masked on store
    pa[i] = A + (long)ga * lda + gc * 8;
    pw[i] = W + (long)gw * K + gc * 8;
  }
  auto stage = [&](int buf, int k0) {
    _Float16* la = lds + buf * 2 * TILE_H;
    _Float16* lw = la + TILE_H;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(pa[i] + k0, la + (wave * 32 + i * 16) * BK);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(pw[i] + k0, lw + (wave * 32 + i * 16) * BK);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int r = lane & 31, h = lane >> 5;
  const int nk = K / BK;
  stage(0, 0);
  if (nk > 1) stage(1, BK);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (this wave's DMAs; the newer tile may stay in flight), then the barrier makes
    // every wave's DMAs visible and frees the buffer read in iteration kt-1
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) stage(cur == 0 ? 2 : cur - 1, (kt + 2) * BK);
    const _Float16* la = lds + cur * 2 * TILE_H;
    const _Float16* lw = la + TILE_H;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks * 2 + h;   // logical 16-B chunk of this lane's 8 k values
      half8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm + 32 * i + r;
        af[i] = *reinterpret_cast<const half8*>(la + row * BK + swz(row, c) * 8);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wn + 32 * j + r;
        bf[j] = *reinterpret_cast<const half8*>(lw + row * BK + swz(row, c) * 8);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    cur = cur == NBUF - 1 ? 0 : cur + 1;
  }
  // epilogue: bias + GELU in registers (C/D map col = lane & 31, row = (e & 3) + 8 (e >> 2) +
  // 4 (lane >> 5)), the fp16 tile staged through LDS, written back as 16-B row chunks
  __syncthreads();   // every wave is done with the ring (no DMA outstanding after the last wait)
  constexpr int CLD = BN + 8;   // halves per LDS row of the output tile (row starts 16-B aligned)
  static_assert(BM * CLD <= NBUF * 2 * TILE_H, "output tile must fit the staging ring");
  _Float16* cs = lds;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = wn + 32 * j + (lane & 31), col = n0 + cl;
    const bool live = col < N;
    const float bv = live ? bias[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rl = wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        float v = acc[i][j][e] + bv;
        if (GELU) v = gelu_fast(v);
        cs[rl * CLD + cl] = live ? (_Float16)v : (_Float16)0.0f;
      }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < BM * BN / 8 / GT; ++it) {
    const int idx = tid + it * GT, rl = idx / (BN / 8), ch = idx % (BN / 8);
    const int row = m0 + rl, col = n0 + ch * 8;
    if (row < M && col < ldc)
      *reinterpret_cast<half8*>(Cout + (long)row * ldc + col) = *reinterpret_cast<const half8*>(cs + rl * CLD + ch * 8);
  }
}

// reacting-cell compaction (deterministic): per-block counts, one-block scan, scatter
constexpr int CB = 1024;
__global__ void k_react_count(int C, const double* __restrict__ T, double Tr, int* __restrict__ bc) {
  __shared__ int s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  const int c = blockIdx.x * CB + threadIdx.x;
  const bool f = c < C && T[c] >= Tr;
  const unsigned long long b = __ballot(f);
  if ((threadIdx.x & 63) == 0) atomicAdd(&s, __popcll(b));
  __syncthreads();
  if (threadIdx.x == 0) bc[blockIdx.x] = s;
}
__global__ void k_react_scan(int nb, int* __restrict__ bc, int* __restrict__ total) {
  if (threadIdx.x != 0) return;
  int a = 0;
  for (int i = 0; i < nb; ++i) { const int v = bc[i]; bc[i] = a; a += v; }
  *total = a;
}
__global__ void k_react_scatter(int C, const double* __restrict__ T, double Tr, const int* __restrict__ boff,
                                int* __restrict__ idx) {
  __shared__ int woff[CB / 64];
  const int c = blockIdx.x * CB + threadIdx.x;
  const bool f = c < C && T[c] >= Tr;
  const unsigned long long b = __ballot(f);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) woff[w] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0;
    for (int i = 0; i < CB / 64; ++i) { const int v = woff[i]; woff[i] = a; a += v; }
  }
  __syncthreads();
  if (f) {
    const int pos = boff[blockIdx.x] + woff[w] + __popcll(b & ((1ull << lane) - 1ull));
    idx[pos] = c;
  }
}

// normalised fp16 input rows [n][Kp] (zero padded)
__global__ void k_dnn_input(int n, int C, int S, int Kp, const int* __restrict__ idx, const double* __restrict__ T,
                            const double* __restrict__ Y, const double* __restrict__ Xmu,
                            const double* __restrict__ Xstd, _Float16* __restrict__ X) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = idx[i];
  _Float16* row = X + (long)i * Kp;
  row[0] = (_Float16)((T[c] - Xmu[0]) / Xstd[0]);
  row[1] = (_Float16)((101325.0 - Xmu[1]) / Xstd[1]);
  for (int s = 0; s < S; ++s) {
    const double b = (pow(Y[(long)s * C + c], 0.1) - 1.0) * 10.0;
    row[2 + s] = (_Float16)((b - Xmu[2 + s]) / Xstd[2 + s]);
  }
  for (int k = S + 2; k < Kp; ++k) row[k] = (_Float16)0.0f;
}

// output layer (K -> 1) of every net + calculate_y_new + calculate_RR
__global__ void k_dnn_output(int n, int C, int S, int K, int ldh, int nmod, const int* __restrict__ idx,
                             const _Float16* __restrict__ H, long sH, const _Float16* __restrict__ w, long sw,
                             const float* __restrict__ b, const double* __restrict__ Ymu,
                             const double* __restrict__ Ystd, const double* __restrict__ Y,
                             const double* __restrict__ rho, const double* __restrict__ p, double dt,
                             double* __restrict__ RR) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = idx[i];
  double yn[32];
  double sum = 0.0;
  for (int m = 0; m < nmod; ++m) {
    const _Float16* hr = H + m * sH + (long)i * ldh;
    const _Float16* wm = w + m * sw;
    float a = 0.0f;
    for (int k = 0; k < K; k += 8) {
      const half8 hv = *reinterpret_cast<const half8*>(hr + k);
      const half8 wv = *reinterpret_cast<const half8*>(wm + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) a += (float)hv[j] * (float)wv[j];
    }
    const double out = (double)(_Float16)(a + b[m]);   // the net's fp16 output, as .to(kDouble)
    const double ybct = (pow(Y[(long)m * C + c], 0.1) - 1.0) * 10.0;
    const double v = out * Ystd[m] + Ymu[m] + ybct;
    yn[m] = pow(v * 0.1 + 1.0, 10.0);
    sum += yn[m];
  }
  sum += Y[(long)(S - 1) * C + c];
  for (int m = 0; m < nmod; ++m) {
    const double y = yn[m] / sum;
    RR[(long)m * C + c] = (y - Y[(long)m * C + c]) * rho[c] * (p[c] / 101325.0) / dt;
  }
}

__global__ void k_zero(long n, double* __restrict__ v) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) v[i] = 0.0;
}

}  // namespace

void dnn_upload(Ctx& x, int nmod, int nlayers, const int* dims, const float* params, const double* xmu,
                const double* xstd, const double* ymu, const double* ystd, double T_react, double dt_infer) {
  Dnn& d = x.dnn;
  DFMI_CHECK(nmod == x.S - 1 && nmod <= 32, "DNN: one net per non-inert species (S - 1 <= 32) expected");
  DFMI_CHECK(nlayers >= 2 && nlayers <= 8, "DNN: 2..8 linear layers supported");
  DFMI_CHECK(dims[0] == x.S + 2 && dims[nlayers] == 1, "DNN: input must be S + 2 wide and output 1 wide");
  DFMI_CHECK(x.inert == x.S - 1, "DNN: the reference layout needs the inert species last");
  d.nmod = nmod;
  d.dims.assign(dims, dims + nlayers + 1);
  d.Kp.resize(nlayers);
  for (int l = 0; l < nlayers; ++l) {
    // K of every layer padded to the GEMM K tile; activations are stored with that row stride (the
    // padding columns are written as 0, the padded weight columns are 0)
    d.Kp[l] = (dims[l] + KPAD - 1) / KPAD * KPAD;
    if (l == nlayers - 1) DFMI_CHECK(dims[l] % 8 == 0, "DNN: last hidden width must be a multiple of 8");
  }
  // repack weights: per layer [module][out][Kp] fp16 (K zero-padded), biases fp32 [module][out]
  d.W.clear(); d.b.clear();
  d.W.resize(nlayers); d.b.resize(nlayers);
  std::vector<std::vector<_Float16>> hw(nlayers);
  std::vector<std::vector<float>> hb(nlayers);
  for (int l = 0; l < nlayers; ++l) {
    hw[l].assign((size_t)nmod * dims[l + 1] * d.Kp[l], (_Float16)0.0f);
    hb[l].assign((size_t)nmod * dims[l + 1], 0.0f);
  }
  const float* p = params;
  for (int m = 0; m < nmod; ++m)
    for (int l = 0; l < nlayers; ++l) {
      const int in = dims[l], out = dims[l + 1];
      for (int o = 0; o < out; ++o)
        for (int i = 0; i < in; ++i) hw[l][((size_t)m * out + o) * d.Kp[l] + i] = (_Float16)p[(size_t)o * in + i];
      p += (size_t)out * in;
      for (int o = 0; o < out; ++o) hb[l][(size_t)m * out + o] = p[o];
      p += out;
    }
  for (int l = 0; l < nlayers; ++l) {
    d.W[l].upload(hw[l].data(), hw[l].size(), x.stream);
    d.b[l].upload(hb[l].data(), hb[l].size(), x.stream);
  }
  d.xmu.upload(xmu, dims[0], x.stream); d.xstd.upload(xstd, dims[0], x.stream);
  d.ymu.upload(ymu, nmod, x.stream); d.ystd.upload(ystd, nmod, x.stream);
  d.T_react = T_react;
  d.dt = dt_infer;
  DFMI_HIP(hipStreamSynchronize(x.stream));
  d.ready = true;
}

void dnn_solve(Ctx& x) {
  Dnn& d = x.dnn;
  DFMI_CHECK(d.ready, "DNN model not set (dfmi_dnn_set_model)");
  const int C = x.C, S = x.S, L = (int)d.dims.size() - 1;
  const int nb = blocks_for(C, CB);
  if (d.bc.n < (size_t)nb + 1) d.bc.alloc(nb + 1);
  if (d.idx.n < (size_t)C) d.idx.alloc(C);
  double* RR = x.f("RR");
  hipLaunchKernelGGL(k_zero, dim3(blocks_for((long)S * C, 256)), dim3(256), 0, x.stream, (long)S * C, RR);
  hipLaunchKernelGGL(k_react_count, dim3(nb), dim3(CB), 0, x.stream, C, x.f("T"), d.T_react, d.bc.p);
  hipLaunchKernelGGL(k_react_scan, dim3(1), dim3(64), 0, x.stream, nb, d.bc.p, d.bc.p + nb);
  hipLaunchKernelGGL(k_react_scatter, dim3(nb), dim3(CB), 0, x.stream, C, x.f("T"), d.T_react, d.bc.p, d.idx.p);
  DFMI_HIP(hipGetLastError());
  int nr = 0;
  DFMI_HIP(hipMemcpyAsync(&nr, d.bc.p + nb, sizeof(int), hipMemcpyDeviceToHost, x.stream));
  DFMI_HIP(hipStreamSynchronize(x.stream));
  d.last_reacting = nr;
  if (nr == 0) return;
  const int chunk = std::min(nr, d.chunk);
  // activation buffers for one chunk: ping-pong [module][chunk][width]
  size_t wmax = 0;
  for (int l = 1; l < L; ++l) wmax = std::max(wmax, (size_t)d.Kp[l]);
  const size_t act = (size_t)d.nmod * chunk * wmax;
  if (d.h0.n < act) { d.h0.alloc(act); d.h1.alloc(act); }
  if (d.x0.n < (size_t)chunk * d.Kp[0]) d.x0.alloc((size_t)chunk * d.Kp[0]);
  for (int c0 = 0; c0 < nr; c0 += chunk) {
    const int n = std::min(chunk, nr - c0);
    const int* idx = d.idx.p + c0;
    hipLaunchKernelGGL(k_dnn_input, dim3(blocks_for(n, 256)), dim3(256), 0, x.stream, n, C, S, d.Kp[0], idx, x.f("T"),
                       x.f("Y"), d.xmu.p, d.xstd.p, d.x0.p);
    const _Float16* in = d.x0.p;
    long sIn = 0;
    _Float16* bufs[2] = {d.h0.p, d.h1.p};
    int lda = d.Kp[0];
    for (int l = 0; l + 1 < L; ++l) {
      const int N = d.dims[l + 1], K = d.Kp[l], ldc = d.Kp[l + 1];
      _Float16* out = bufs[l & 1];
      d.gemm_flops += 2.0 * n * N * d.dims[l] * d.nmod;   // algorithmic flops (unpadded K)
      const dim3 g(blocks_for(N, BN) * blocks_for(n, BM), 1, d.nmod);
      KScope _ks(x, "k_mlp_gemm");
      hipLaunchKernelGGL(k_mlp_gemm<true>, g, dim3(GT), 0, x.stream, n, N, K, in, lda, sIn, d.W[l].p, (long)N * K,
                         d.b[l].p, (long)N, out, ldc, (long)n * ldc);
      DFMI_HIP(hipGetLastError());
      in = out;
      sIn = (long)n * ldc;
      lda = ldc;
    }
    const int K = d.dims[L - 1];
    DFMI_CHECK(K % 8 == 0, "DNN: output layer width");
    KScope _ks(x, "k_dnn_output");
    hipLaunchKernelGGL(k_dnn_output, dim3(blocks_for(n, 256)), dim3(256), 0, x.stream, n, C, S, K, lda, d.nmod, idx,
                       in, sIn, d.W[L - 1].p, (long)d.Kp[L - 1], d.b[L - 1].p, d.ymu.p, d.ystd.p, x.f("Y"),
                       x.f("rho"), x.f("p"), d.dt, RR);
    DFMI_HIP(hipGetLastError());
  }
}

}  // namespace dfmi
