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
// v_mfma_f32_16x16x32_f16 with fp32 accumulation and the bias + erf GELU + fp16 rounding fused into the
// epilogue; the 1-wide output layer and the BCT post-processing are fused into one kernel.
// GEMM tile 256x128x32, 4 waves (2x2, 128x64 each = 8x4 MFMA tiles), both operands streamed
// global -> LDS by DMA (global_load_lds, swizzled rows) through a 3-buffer ring, A and W both
// K-contiguous (W in torch Linear [out][in] layout), K and activation row strides padded to 32.
#include "dfmi_ctx.h"
#include <cmath>
#include <cstdlib>
#include <type_traits>

namespace dfmi {
namespace {

using half8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr int BN = 128, BK = 32;
constexpr int NBUF = 3;                   // LDS ring: two K tiles in flight while one feeds the MFMAs
constexpr int KPAD = 32;                  // every GEMM K (and activation row stride) is a multiple of this
constexpr int TILE_W = BN * BK;           // halves per staged W tile (8 KiB)

// GELU for the GEMM epilogue, two values at a time: erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7,
// branch-free), three orders of magnitude below the fp16 rounding the result goes through (torch's GELU is
// the exact-erf form; the library erff branches per lane on |x| < 1). Packed fp32 arithmetic (v_pk_mul_f32 / v_pk_fma_f32, two values per instruction: no MFMA competes for the
// issue slots in the epilogue), hardware reciprocal and exp2 (<= 1 ulp each; __frcp_rn expands to the
// correctly-rounded division sequence, which dominated the epilogue), explicit fmas (-ffp-contract=off).
// The form 0.5 v (1 + sign(v) erf(|v|/sqrt2)) = 0.5 fma(|v|, erf(|v|/sqrt2), v), with 1/sqrt2 folded into the
// constants: no copysign, one abs per value, 12% faster at full occupancy than evaluating u = v/sqrt2 first
// (scripts/probes/gelu_probe.hip); the epilogue is VALU-bound on it (a 64-deep K leaves it nothing to hide behind).
using f32x2 = __attribute__((ext_vector_type(2))) float;
using half2v = __attribute__((ext_vector_type(2))) _Float16;
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 v) {
  const f32x2 a = __builtin_elementwise_abs(v);
  const f32x2 d = __builtin_elementwise_fma(a, f32x2(0.23164202848f), f32x2(1.0f));   // 1 + 0.3275911 |v| / sqrt2
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 q = __builtin_elementwise_fma(t, f32x2(1.061405429f), f32x2(-1.453152027f));
  q = __builtin_elementwise_fma(t, q, f32x2(1.421413741f));
  q = __builtin_elementwise_fma(t, q, f32x2(-0.284496736f));
  q = __builtin_elementwise_fma(t, q, f32x2(0.254829592f));
  const f32x2 w = v * (v * -0.72134752044448170368f);                                 // -(v^2 / 2) log2(e)
  const f32x2 ex = {__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  const f32x2 e = __builtin_elementwise_fma(-(t * q), ex, f32x2(1.0f));                // erf(|v| / sqrt2)
  return __builtin_elementwise_fma(a, e, v) * 0.5f;
}

// fp16 rounding kept in fp32 registers: torch's fp16 Linear writes its output (x W^T + b, fp32
// accumulation) as fp16 before the GELU reads it, and the GELU's own output is rounded again
// (v_cvt_pk_f16_f32: one conversion per pair)
__device__ __forceinline__ half2v to16(f32x2 v) { return __builtin_convertvector(v, half2v); }
__device__ __forceinline__ f32x2 round16(f32x2 v) { return __builtin_convertvector(to16(v), f32x2); }

using f32x4 = __attribute__((ext_vector_type(4))) float;

// GEMM epilogue shared by the kernels below, for one wave's 16 NI x 16 NJ accumulator tile (NI x NJ blocks of 16 x 16,
// C/D map col = lane & 15, row = 4 (lane >> 4) + e) at tile-local rows wm.., columns wn.. of the N tile at n0:
// bias + GELU, rounded to fp16, into the LDS output tile cs (row stride CLD). 16-column blocks wholly past N (the
// padded tail of the last N tile: 224 of the 1,024 columns of an 800-wide layer) are written as zeros without
// evaluating the GELU -- a wave-uniform test; the GELU is the epilogue's whole cost.
template <bool GELU, int CLD, int NI = 8, int NJ = 4>
__device__ __forceinline__ void stage_out_tile(const f32x4 (&acc)[NI][NJ], _Float16* cs, int wm, int wn, int n0, int N,
                                               const float* __restrict__ bias, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int cl = wn + 16 * j + (lane & 15), col = n0 + cl;
    if (n0 + wn + 16 * j >= N) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[(wm + 16 * i + 4 * g + e) * CLD + cl] = (_Float16)0.0f;
      continue;
    }
    const bool live = col < N;
    const float bv = live ? bias[col] : 0.0f;
    auto block = [&](auto full_c) {   // full: all 16 columns live (no per-lane select)
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int rl = wm + 16 * i + 4 * g + e;
          f32x2 v = round16(f32x2{acc[i][j][e], acc[i][j][e + 1]} + bv);
          if (GELU) v = gelu_fast2(v);
          half2v h = to16(v);
          if (!decltype(full_c)::value && !live) h = half2v{(_Float16)0.0f, (_Float16)0.0f};
          cs[rl * CLD + cl] = h.x;
          cs[(rl + 1) * CLD + cl] = h.y;
        }
    };
    if (n0 + wn + 16 * j + 16 <= N) block(std::true_type{});
    else block(std::false_type{});
  }
}

// OUT epilogue (the last hidden layer): the net's 1-wide output layer fused in instead of storing the tile --
// each fp16-rounded activation times its output weight wo[col], summed per row (fp32, fixed order: over the
// lane's four 16-column blocks, then a 16-lane xor tree) into the wave's partial Pw[row]. Blocks wholly past N
// are skipped (their products are zeros).
template <bool GELU>
__device__ __forceinline__ void out_layer_partials(const f32x4 (&acc)[8][4], float* __restrict__ Pw, int M, int m0, int wm,
                                                   int wn, int n0, int N, const float* __restrict__ bias,
                                                   const _Float16* __restrict__ wo, int lane) {
  float bv[4], wv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn + 16 * j + (lane & 15);
    bv[j] = col < N ? bias[col] : 0.0f;
    wv[j] = col < N ? (float)wo[col] : 0.0f;   // dead columns contribute 0
  }
  f32x2 sacc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i) sacc[i][0] = sacc[i][1] = f32x2{0.0f, 0.0f};
  // column blocks outermost (one wave-uniform test each; the per-row sums still run over j in order)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (n0 + wn + 16 * j >= N) break;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        f32x2 v = round16(f32x2{acc[i][j][e], acc[i][j][e + 1]} + bv[j]);   // the Linear's fp16 output
        if (GELU) v = gelu_fast2(v);
        sacc[i][e / 2] = __builtin_elementwise_fma(round16(v), f32x2(wv[j]), sacc[i][e / 2]);   // the fp16 activation
      }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
      f32x2 sa = sacc[i][e / 2];
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) {
        sa.x += __shfl_xor(sa.x, off);
        sa.y += __shfl_xor(sa.y, off);
      }
      const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + e;
      if ((lane & 15) == 0) {
        if (row < M) Pw[row] = sa.x;
        if (row + 1 < M) Pw[row + 1] = sa.y;
      }
    }
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4): lane l's 16 bytes land at lds_wave + 16 l
__device__ __forceinline__ void glds16(const _Float16* g, _Float16* lds_wave) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_wave, 16, 0, 0);
}

// 16x16x32 operand reads: lane l reads row (l & 15) of a 16-row block at logical chunk (l >> 4). A
// ds_read_b128 lane group then holds rows {0-3,12-15} at chunk c and rows {4-11} at chunk c ^ 1 (or the
// converse); chunk c of row r lives at c ^ H((r >> 2) & 3), H = {0, 2, 3, 1}, which puts the four rows of
// each bank-row position on four distinct 16-B slots (conflict-free)
__device__ __forceinline__ int swz16(int row, int c) { return c ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3); }

// C[z][M][ldc] = act(A[z][M][lda] . W[z][N][K]^T + b[z][N]) for columns < N, 0 for N <= col < ldc;
// fp16 in/out, fp32 accumulate, K, lda, ldc multiples of 32.
// Block tile 256 x 128 x 32, 4 waves (2 x 2) each owning a 128 x 64 tile of 8 x 4 v_mfma_f32_16x16x32_f16
// accumulators (12 fragment reads per 32 MFMAs: half the LDS read traffic per flop of a 64 x 64 wave tile,
// twice the MFMA work between barriers). Both operand tiles are streamed global -> LDS by DMA
// (global_load_lds, 16 B per lane, 6 DMA instructions per wave per K tile) through a 3-buffer ring: tiles
// k+1 and k+2 are in flight while tile k feeds the MFMAs; the wait before each barrier is counted
// (vmcnt(6): the newest tile stays in flight) and the barrier is a raw s_barrier, so nothing drains the DMA
// queue inside the loop. The swizzle is applied on the global source address (each DMA still writes 1 KiB
// contiguously). 72 KiB LDS: two blocks (8 waves) per CU. Block ids are remapped so the consecutive ids
// that share an XCD walk the N tiles of one M tile (A rows re-read from that XCD's L2).
//
// OUT (the last hidden layer): the net's 1-wide output layer is fused into the epilogue instead of storing
// the tile -- each fp16-rounded activation is multiplied by its output weight wo[col] and the products are
// summed per row (fp32, fixed order: over the lane's 4 columns, then a 16-lane xor tree); the two waves of
// a row band write separate partial sums P[z][2 tile_n + wave_n][M], which k_dnn_output adds in order.
template <bool GELU, bool OUT>
__global__ void __launch_bounds__(256, 2)
    k_mlp_gemm(int M, int N, int K, const _Float16* __restrict__ A, int lda, long sA, const _Float16* __restrict__ W,
               long sW, const float* __restrict__ bias, long sb, _Float16* __restrict__ Cout, int ldc, long sC,
               const _Float16* __restrict__ wo, long swo, float* __restrict__ P, long sP) {
  constexpr int BMW = 256, GTW = 256;
  constexpr int TILE_A = BMW * BK, STAGE = TILE_A + TILE_W;
  __shared__ __attribute__((aligned(16))) _Float16 lds[NBUF * STAGE];   // [buf][A (256 x 32) | W (128 x 32)]
  const int z = blockIdx.z;
  A += z * sA; W += z * sW; bias += z * sb; Cout += z * sC; wo += z * swo; P += z * sP;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BMW - 1) / BMW, nwg = ntn * ntm;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int m0 = (wg / ntn) * BMW, n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // staging: wave w fills A rows [64 w, 64 w + 64) and W rows [32 w, 32 w + 32), 16 rows per DMA
  const _Float16* pa[4];
  const _Float16* pw[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 64 + i * 16 + (lane >> 2);
    pa[i] = A + (long)min(m0 + row, M - 1) * lda + swz16(row, lane & 3) * 8;   // clamped rows masked on store
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 32 + i * 16 + (lane >> 2);
    pw[i] = W + (long)min(n0 + row, N - 1) * K + swz16(row, lane & 3) * 8;
  }
  auto stage = [&](int buf, int k0) {
    _Float16* la = lds + buf * STAGE;
    _Float16* lw = la + TILE_A;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(pa[i] + k0, la + (wave * 64 + i * 16) * BK);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(pw[i] + k0, lw + (wave * 32 + i * 16) * BK);
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 64;
  const int r = lane & 15, c = lane >> 4;
  const int nk = K / BK;
  auto frag_reads = [&](int buf, half8 (&af)[8], half8 (&bf)[4]) {
    const _Float16* la = lds + buf * STAGE;
    const _Float16* lw = la + TILE_A;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn + 16 * j + r;
      bf[j] = *reinterpret_cast<const half8*>(lw + row * BK + swz16(row, c) * 8);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wm + 16 * i + r;
      af[i] = *reinterpret_cast<const half8*>(la + row * BK + swz16(row, c) * 8);
    }
  };
  // 16-column blocks of this wave that hold output columns (< N): the padded tail of the last N tile
  // (N = 400 / 800 pad to 512 / 896) issues no MFMAs, freeing the SIMD for the co-resident block
  const int jlive = min(4, max(0, (N - (n0 + wn) + 15) / 16));
  auto mfmas = [&](const half8 (&af)[8], const half8 (&bf)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < jlive)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
  };
  stage(0, 0);
  if (nk > 1) stage(1, BK);
  {
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) stage(cur == 0 ? 2 : cur - 1, (kt + 2) * BK);
      half8 af[8], bf[4];
      frag_reads(cur, af, bf);
      // all 12 fragment reads issued before the first MFMA (counted lgkmcnt waits follow): left to itself the
      // compiler re-reads A two fragments at a time behind lgkmcnt(0), exposing the LDS latency 4x per tile
      __builtin_amdgcn_sched_barrier(0);
      mfmas(af, bf);
      cur = cur == NBUF - 1 ? 0 : cur + 1;
    }
  }
  if constexpr (OUT) {
    out_layer_partials<GELU>(acc, P + (long)(2 * (wg % ntn) + (wave & 1)) * M, M, m0, wm, wn, n0, N, bias, wo, lane);
    return;
  }
  // the fp16 tile staged through LDS, written back as 16-B row chunks
  __syncthreads();
  constexpr int CLD = BN + 8;
  static_assert(BMW * CLD <= NBUF * STAGE, "output tile must fit the staging ring");
  _Float16* cs = lds;
  stage_out_tile<GELU, CLD>(acc, cs, wm, wn, n0, N, bias, lane);
  __syncthreads();
#pragma unroll
  for (int it = 0; it < BMW * BN / 8 / GTW; ++it) {
    const int idx = tid + it * GTW, rl = idx / (BN / 8), ch = idx % (BN / 8);
    const int row = m0 + rl, col = n0 + ch * 8;
    if (row < M && col < ldc)
      *reinterpret_cast<half8*>(Cout + (long)row * ldc + col) = *reinterpret_cast<const half8*>(cs + rl * CLD + ch * 8);
  }
}

// Input-layer variant (K <= 64: the 55 -> 1600 first layer, K padded to 64): with one K tile there is nothing for
// a DMA ring to overlap, and the layer's time is its epilogue -- 5.45 G GELUs per 65,536-row chunk of the 52 nets,
// VALU-bound, plus 10.9 GB of fp16 activations written. So the tile is small enough for four workgroups (16
// waves) per CU to hide the GELU's dependent transcendental latencies behind one another: 128 x 128 x 64, 4 waves
// (2 x 2) of 64 x 64 (4 x 4 MFMA blocks), the whole K staged by DMA at once (A and W 128 rows x 128 B each,
// rows swizzled as the ping-pong kernel below), then the output tile staged through the same LDS (35 KiB) and written as
// 16-B row chunks. Same MFMA order per output as k_mlp_gemm (K halves in order), so the same results.
template <bool GELU, int BMI>
__global__ void __launch_bounds__(256, BMI == 64 ? 6 : 4)
    k_mlp_gemm_in(int M, int N, int K, const _Float16* __restrict__ A, int lda, long sA, const _Float16* __restrict__ W,
                  long sW, const float* __restrict__ bias, long sb, _Float16* __restrict__ Cout, int ldc, long sC) {
  // BMI = 128: 4 waves (2 x 2) of 64 x 64; BMI = 64: 4 waves (1 x 4) of 64 x 32 (six workgroups per CU)
  constexpr int BNI = 128, BKI = 64, NT = 256, NWN = BMI == 128 ? 2 : 4, NJ = BNI / NWN / 16, PA = BMI / 32;
  constexpr int CLD = BNI + 8;
  constexpr int TILE_A = BMI * BKI, TILE_W = BNI * BKI;
  constexpr int LDS_H = TILE_A + TILE_W > BMI * CLD ? TILE_A + TILE_W : BMI * CLD;
  __shared__ __attribute__((aligned(16))) _Float16 lds[LDS_H];   // [A (BMI x 64) | W (128 x 64)], then C
  const int z = blockIdx.z;
  A += z * sA; W += z * sW; bias += z * sb; Cout += z * sC;
  const int ntn = (N + BNI - 1) / BNI, ntm = (M + BMI - 1) / BMI, nwg = ntn * ntm;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int m0 = (wg / ntn) * BMI, n0 = (wg % ntn) * BNI;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave / NWN) * 64, wn = (wave % NWN) * (16 * NJ);
  const int r = lane & 15, g = lane >> 4;
  const int fo[2] = {r * BKI + ((g) ^ (r >> 1)) * 8, r * BKI + ((4 + g) ^ (r >> 1)) * 8};
  // staging: wave w fills A rows [BMI/4 w, ..) and W rows [32 w, 32 w + 32), 8 rows (1 KiB) per DMA piece
  const _Float16* pa[PA];
  const _Float16* pw[4];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = wave * (BMI / 4) + i * 8 + (lane >> 3), ch = (lane & 7) ^ ((row >> 1) & 7);
    pa[i] = A + (long)min(m0 + row, M - 1) * lda + ch * 8;   // clamped rows masked on store
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + (lane >> 3), ch = (lane & 7) ^ ((row >> 1) & 7);
    pw[i] = W + (long)min(n0 + row, N - 1) * K + ch * 8;
  }
  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int jl = min(NJ, max(0, (N - (n0 + wn) + 15) / 16));   // live 16-column blocks of this wave
  for (int k0 = 0; k0 < K; k0 += BKI) {
    const int kh_n = min(2, (K - k0) / 32);                    // K halves in this tile (K % 32 == 0)
    if (k0 > 0) __syncthreads();                               // the previous tile's reads done
#pragma unroll
    for (int i = 0; i < PA; ++i) glds16(pa[i] + k0, lds + (wave * (BMI / 4) + i * 8) * BKI);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(pw[i] + k0, lds + TILE_A + (wave * 32 + i * 8) * BKI);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int kh = 0; kh < kh_n; ++kh) {
      half8 af[4], bf[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = *reinterpret_cast<const half8*>(lds + TILE_A + (wn + 16 * j) * BKI + fo[kh]);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const half8*>(lds + (wm + 16 * i) * BKI + fo[kh]);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (j < jl)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();
  stage_out_tile<GELU, CLD, 4, NJ>(acc, lds, wm, wn, n0, N, bias, lane);
  __syncthreads();
#pragma unroll 4
  for (int it = 0; it < BMI * BNI / 8 / NT; ++it) {
    const int idx = tid + it * NT, rl = idx / (BNI / 8), ch = idx % (BNI / 8);
    const int row = m0 + rl, col = n0 + ch * 8;
    if (row < M && col < ldc)
      *reinterpret_cast<half8*>(Cout + (long)row * ldc + col) = *reinterpret_cast<const half8*>(lds + rl * CLD + ch * 8);
  }
}

// 128-B LDS rows (8 chunks of 16 B): chunk c of row r at c ^ ((r >> 1) & 7), which puts each ds_read_b128 lane
// group ({0-3,12-15,20-27}, ... : rows 0-15 of a 16-row block at two adjacent logical chunks) on 16 distinct 16-B
// bank slots; DMA pieces are 8 rows x 128 B (1 KiB contiguous, the swizzle applied on the source address).
// (Round 5: the single-group 256 x 256 x 64 variants, 9.77 / 10.07 ms per chunk against the ping-pong kernel's
// 8.72, are removed.)

// Ping-pong variant of the wide-layer GEMM (the guide's 256x256 eight-phase schedule, cdna_hip_programming.md
// section 5): the same 256 x 256 x 64 tile and 8 waves, but each 64-deep K tile runs as four phases, one per
// C quadrant of the wave's 128 x 64 tile (16 MFMAs: 4 row blocks x 2 column blocks x 2 K halves), and the two
// wave rows run one barrier apart -- while waves 0-3 issue a phase's MFMAs, waves 4-7 issue their next phase's
// fragment reads and DMA, so each SIMD always has one wave feeding the MFMA pipe. LDS holds two K tiles as
// four half-tiles each (A rows of row-half 0 / 1 of both wave rows, W rows of column-half 0 / 1 of all four
// wave columns: 128 rows x 128 B, swizzled as above), and every half-tile is re-staged (two DMA pieces per
// wave) one phase after its last read: per tile t, phase 0 reads A0 B0 and stages B0 of t+1, phase 1 reads B1
// and stages A0 of t+2, phase 2 reads A1 and stages B1 of t+2, phase 3 reads B0 and stages A1 of t+2, then
// waits vmcnt(6) (the three newest half-tiles stay in flight, tile t+1 has landed). Every phase retires its own
// reads (lgkmcnt(0)) before its first barrier, which makes the one-phase restage safe with the groups
// staggered; each read follows the wait that retires its data by at least one barrier of both groups.
// Past the last tile the stages re-load the last tile's data (in bounds, never read) so that every phase
// issues the same DMA count; the epilogue drains them first. Accumulation order per output: K tiles in
// order, K halves in order -- the same MFMA sequence as k_mlp_gemm, so the same results.
// OUT (the last hidden layer, K zero-padded to a multiple of 64): the 1-wide output layer fused into the
// epilogue as in k_mlp_gemm -- per row, the products with wo over each wave's 64 columns, summed over the
// lane's four 16-column blocks and a 16-lane xor tree, written as partial P[z][4 tile_n + wave_n][M]: the
// same 64-column groups in the same order as k_mlp_gemm's two 64-column partials per 128-wide tile.
//
// TS > 0 (N = 256 q + t, 0 < t <= 32: the 800-wide layer): q column tiles instead of q + 1, the last 32 / TS of
// them also computing TS of the tail columns as a 256 x TS strip -- wave (wr, wc) owns its rows 32 wc.. of the
// strip (2 x TS/16 MFMA blocks). Its A fragments are the ones the wave already holds for that half of its rows
// (phase 0 for wc < 2, phase 2 otherwise); its W rows (TS x 64 per K tile) are staged by waves 0 .. TS/8 - 1 (one
// DMA piece each, with A row-half 1 at phase 3: the strip's reads end in phase 2) into a slot per stage.
// A 32-column tile of its own streams all of A for 1/8 of a tile's MFMAs (63 % of a full tile's time).
template <bool GELU, bool OUT = false, int TS = 0>
__global__ void __launch_bounds__(512, 1)
    k_mlp_gemm_pp(int M, int N, int K, const _Float16* __restrict__ A, int lda, long sA, const _Float16* __restrict__ W,
                  long sW, const float* __restrict__ bias, long sb, _Float16* __restrict__ Cout, int ldc, long sC,
                  const _Float16* __restrict__ wo = nullptr, long swo = 0, float* __restrict__ P = nullptr, long sP = 0) {
  constexpr bool TAIL = TS > 0;
  static_assert(!(OUT && TAIL) && (TS == 0 || TS == 16 || TS == 32), "tail strips: 16 or 32 columns, no OUT");
  constexpr int BMW = 256, BNW = 256, BKW = 64, NT = 512, TW = TS, NJT = TS / 16, NSTRIP = TAIL ? 32 / TS : 0;
  constexpr int HALF = 128 * BKW;                // halves (fp16 elements) per half-tile: 16 KiB
  constexpr int STAGE = 4 * HALF;                // [A row-half 0 | A row-half 1 | W col-half 0 | W col-half 1]
  constexpr int TSLOT = TW * BKW;                // tail W rows per stage (TS x 128 B), after the two stages
  constexpr int CLD = BNW + (TAIL ? TW : 0) + 8;
  constexpr int LDS_IN = 2 * STAGE + (TAIL ? 2 * TSLOT : 0);
  constexpr int LDS_H = LDS_IN > BMW * CLD ? LDS_IN : BMW * CLD;
  __shared__ __attribute__((aligned(16))) _Float16 lds[LDS_H];
  const int z = blockIdx.z;
  A += z * sA; W += z * sW; bias += z * sb; Cout += z * sC;
  if constexpr (OUT) { wo += z * swo; P += z * sP; }
  const int ntn = TAIL ? N / BNW : (N + BNW - 1) / BNW, ntm = (M + BMW - 1) / BMW, nwg = ntn * ntm;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int m0 = (wg / ntn) * BMW, n0 = (wg % ntn) * BNW;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  // DMA sources: half-tile h, piece q: half-row hr = 16 wave + 8 q + (lane >> 3), 16-B chunk lane & 7 of the
  // LDS row holding logical chunk (lane & 7) ^ ((hr >> 1) & 7). A half h < 2: tile row (hr / 64) 128 + 64 h +
  // hr % 64 (rows of both wave rows); W half h = 2 + jh: tile row (hr / 32) 64 + 32 jh + hr % 32 (all columns)
  const _Float16* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int hr = 16 * wave + 8 * q + (lane >> 3), ch = (lane & 7) ^ ((hr >> 1) & 7);
      if (h < 2) {
        const int row = (hr >> 6) * 128 + h * 64 + (hr & 63);
        src[h][q] = A + (long)min(m0 + row, M - 1) * lda + ch * 8;   // clamped rows masked on store
      } else {
        const int row = (hr >> 5) * 64 + (h - 2) * 32 + (hr & 31);   // the wave-column-major LDS position
        src[h][q] = W + (long)min(n0 + row, N - 1) * K + ch * 8;
      }
    }
  auto stage_half = [&](int buf, int h, int k0) {
    _Float16* d = lds + buf * STAGE + h * HALF + 16 * wave * BKW;
    glds16(src[h][0] + k0, d);
    glds16(src[h][1] + k0, d + 8 * BKW);
  };
  // this tile's strip (the last NSTRIP tiles: strip si at columns nt0 + TS si); its W rows: wave w < TS / 8
  // stages rows 8 w .. 8 w + 7 (clamped to N - 1: dead columns masked on store)
  const int nt0 = ntn * BNW, si = TAIL ? wg % ntn - (ntn - NSTRIP) : -1, so = nt0 + TS * si;
  const _Float16* tsrc;
  {
    const int trow = 8 * (wave & 3) + (lane >> 3), ch = (lane & 7) ^ ((trow >> 1) & 7);
    tsrc = W + (long)min(max(so, 0) + trow, N - 1) * K + ch * 8;
  }
  auto stage_tail = [&](int buf, int k0) { glds16(tsrc + k0, lds + 2 * STAGE + buf * TSLOT + 8 * (wave & 3) * BKW); };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int r = lane & 15, g = lane >> 4;
  const int fo[2] = {r * BKW + ((g) ^ (r >> 1)) * 8, r * BKW + ((4 + g) ^ (r >> 1)) * 8};
  half8 af[4][2], bf[2][2];   // the quadrant's fragments: 4 row blocks / 2 column blocks x 2 K halves
  auto read_a = [&](int buf, int ih) {
    const _Float16* s0 = lds + buf * STAGE + ih * HALF + (wr * 64) * BKW;
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) af[ib][kh] = *reinterpret_cast<const half8*>(s0 + ib * 16 * BKW + fo[kh]);
  };
  auto read_b = [&](int buf, int jh) {
    const _Float16* s0 = lds + buf * STAGE + (2 + jh) * HALF + (wc * 32) * BKW;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) bf[jb][kh] = *reinterpret_cast<const half8*>(s0 + jb * 16 * BKW + fo[kh]);
  };
  constexpr int NJ1 = NJT > 0 ? NJT : 1;
  f32x4 acct[2][NJ1];   // the tail strip: rows 32 wc + 16 ib of the wave's 128, columns 16 jb of the strip
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ1; ++j) acct[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  half8 bt[NJ1][2];
  auto read_bt = [&](int buf) {
    const _Float16* s0 = lds + 2 * STAGE + buf * TSLOT;
#pragma unroll
    for (int jb = 0; jb < NJT; ++jb)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) bt[jb][kh] = *reinterpret_cast<const half8*>(s0 + jb * 16 * BKW + fo[kh]);
  };
  const int nk = K / BKW;
  auto kloop = [&](auto jl_c, auto tail_c) {
    constexpr int JL = decltype(jl_c)::value;
    constexpr bool TT = decltype(tail_c)::value;   // this tile computes the tail strip
    auto tail_from = [&](auto o_c) {   // rows of the strip in af[O + ib], O = 2 (wc & 1); K half outer
      constexpr int O = decltype(o_c)::value;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int jb = 0; jb < NJT; ++jb)
#pragma unroll
          for (int ib = 0; ib < 2; ++ib)
            acct[ib][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[O + ib][kh], bt[jb][kh], acct[ib][jb], 0, 0, 0);
    };
    auto tail_mfmas = [&]() {
      if (wc & 1) tail_from(std::integral_constant<int, 2>{});
      else tail_from(std::integral_constant<int, 0>{});
    };
    auto quad = [&](int ih, int jh) {   // 16 MFMAs, K half outer so that dependent MFMAs are 8 apart
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
          if (2 * jh + jb < JL)
#pragma unroll
            for (int ib = 0; ib < 4; ++ib)
              acc[4 * ih + ib][2 * jh + jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ib][kh], bf[jb][kh],
                                                                                   acc[4 * ih + ib][2 * jh + jb], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    // one phase: fragment reads and one half-tile's DMA, own reads retired, barrier, MFMAs, barrier
    // tail strip of the half ih: the waves whose strip rows lie in it (wc < 2: half 0, else half 1)
    auto sync_mfma = [&](int ih, int jh, bool tail) {
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this phase's reads retired before its first barrier
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      quad(ih, jh);
      if constexpr (TT) {
        if (tail) {
          __builtin_amdgcn_s_setprio(1);
          tail_mfmas();
          __builtin_amdgcn_s_setprio(0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    const bool tw0 = TT && wc < 2, tw1 = TT && wc >= 2, tstage = TT && wave < TS / 8;
    __builtin_amdgcn_s_waitcnt(0xC07F);   // no scalar load outstanding into the loop
    // prologue: tile 0 complete, tile 1's A0 B1 A1 in flight (the steady-state issue order); the tail strip's
    // W rows of tile 0 with tile 0, of tile 1 after tile 1's A0 (as in the loop: one more piece in flight)
    const int k1 = min(1, nk - 1) * BKW;
    stage_half(0, 0, 0); stage_half(0, 3, 0); stage_half(0, 1, 0); stage_half(0, 2, 0);
    if (tstage) stage_tail(0, 0);
    stage_half(1, 0, k1);
    if (tstage) stage_tail(1, k1);
    stage_half(1, 3, k1); stage_half(1, 1, k1);
    if (tstage) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();   // the stagger: waves 4-7 run one barrier behind
    __builtin_amdgcn_sched_barrier(0);
    for (int t = 0; t < nk; ++t) {
      const int b = t & 1;
      const int kn = min(t + 1, nk - 1) * BKW, k2 = min(t + 2, nk - 1) * BKW;
      read_b(b, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_a(b, 0);
      if (tw0) read_bt(b);
      stage_half(b ^ 1, 2, kn);          // W col-half 0 of tile t+1 (its slot's last read: tile t-1, phase 3)
      sync_mfma(0, 0, tw0);
      read_b(b, 1);
      stage_half(b, 0, k2);              // A row-half 0 of tile t+2 (last read: phase 0)
      sync_mfma(0, 1, false);
      read_a(b, 1);
      if (tw1) read_bt(b);
      stage_half(b, 3, k2);              // W col-half 1 of tile t+2 (last read: phase 1)
      sync_mfma(1, 1, tw1);
      read_b(b, 0);
      stage_half(b, 1, k2);              // A row-half 1 of tile t+2 (last read: phase 2)
      if (tstage) {
        stage_tail(b, k2);               // the strip's W rows of tile t+2 (last read: phase 2)
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile t+1 landed (t+2's first three halves in flight)
      }
      sync_mfma(1, 0, false);
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();   // both groups end on the same barrier count
    __builtin_amdgcn_s_waitcnt(0);              // the re-staging DMAs past the last tile drained
  };
  const int wm = wr * 128, wn = wc * 64;
  const bool tail_tile = TAIL && si >= 0;
  if constexpr (TAIL) {   // every main tile is full
    if (tail_tile) kloop(std::integral_constant<int, 4>{}, std::true_type{});
    else kloop(std::integral_constant<int, 4>{}, std::false_type{});
  } else {
    switch (min(4, max(0, (N - (n0 + wn) + 15) / 16))) {
      case 4: kloop(std::integral_constant<int, 4>{}, std::false_type{}); break;
      case 3: kloop(std::integral_constant<int, 3>{}, std::false_type{}); break;
      case 2: kloop(std::integral_constant<int, 2>{}, std::false_type{}); break;
      case 1: kloop(std::integral_constant<int, 1>{}, std::false_type{}); break;
      default: kloop(std::integral_constant<int, 0>{}, std::false_type{}); break;
    }
  }
  if constexpr (OUT) {   // the fused output layer (no LDS use: the drained stages are not touched)
    out_layer_partials<GELU>(acc, P + (long)(4 * (wg % ntn) + wc) * M, M, m0, wm, wn, n0, N, bias, wo, lane);
    return;
  }
  // epilogue: bias + GELU in registers, the fp16 tile staged through LDS, written back as 16-B row chunks
  __syncthreads();
  _Float16* cs = lds;
  stage_out_tile<GELU, CLD>(acc, cs, wm, wn, n0, N, bias, lane);
  if constexpr (TAIL)
    if (tail_tile) stage_out_tile<GELU, CLD, 2, NJT>(acct, cs, wm + 32 * wc, BNW, so - BNW, N, bias, lane);
  __syncthreads();
#pragma unroll 4
  for (int it = 0; it < BMW * BNW / 8 / NT; ++it) {
    const int idx = tid + it * NT, rl = idx / (BNW / 8), ch = idx % (BNW / 8);
    const int row = m0 + rl, col = n0 + ch * 8;
    if (row < M && col < ldc)
      *reinterpret_cast<half8*>(Cout + (long)row * ldc + col) = *reinterpret_cast<const half8*>(cs + rl * CLD + ch * 8);
  }
  if (tail_tile) {   // the strip, and (last tile) zeros for the padding columns nt0 + 32 .. ldc (at most 32)
    constexpr int NSC = TS / 8, NCH = NSC + 4;
    const bool last = si == NSTRIP - 1;
    for (int idx = tid; idx < BMW * NCH; idx += NT) {
      const int rl = idx / NCH, ch = idx % NCH;
      if (ch >= NSC && !last) continue;
      const int row = m0 + rl, col = ch < NSC ? so + ch * 8 : nt0 + 32 + (ch - NSC) * 8;
      if (row < M && col < ldc) {
        half8 v = {};
        if (ch < NSC) v = *reinterpret_cast<const half8*>(cs + rl * CLD + BNW + ch * 8);
        *reinterpret_cast<half8*>(Cout + (long)row * ldc + col) = v;
      }
    }
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
// exclusive scan of the per-block counts in one 1024-thread workgroup (chunks of 1024, wave prefix sums)
__global__ void __launch_bounds__(1024) k_react_scan(int nb, int* __restrict__ bc, int* __restrict__ total) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + t;
    const int v = i < nb ? bc[i] : 0;
    int incl = v;   // inclusive prefix within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int wo = 0;
    for (int k = 0; k < w; ++k) wo += wsum[k];
    const int c0 = carry;
    if (i < nb) bc[i] = c0 + wo + incl - v;
    __syncthreads();
    if (t == 1023) carry = c0 + wo + incl;
    __syncthreads();
  }
  if (t == 0) *total = carry;
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
  row[0] = (_Float16)(float)((T[c] - Xmu[0]) / Xstd[0]);   // torch's double -> half goes through float
  row[1] = (_Float16)(float)((101325.0 - Xmu[1]) / Xstd[1]);
  for (int s = 0; s < S; ++s) {
    const double b = (pow(Y[(long)s * C + c], 0.1) - 1.0) * 10.0;
    row[2 + s] = (_Float16)(float)((b - Xmu[2 + s]) / Xstd[2 + s]);
  }
  for (int k = S + 2; k < Kp; ++k) row[k] = (_Float16)0.0f;
}

// output layer (K -> 1) of every net + calculate_y_new + calculate_RR
// one workgroup per 64 reacting cells, 8 waves: wave g evaluates species g, g + 8, ... of the 64 cells (coalesced
// partial-sum reads across the cells), the renormalising sum runs over the species in order by wave 0 (the
// sequential sum of the one-thread-per-cell form, bitwise; that form ran one wave per SIMD -- 1,024 waves for a
// 65,536-row chunk -- and kept yn[] in scratch: 270 us per chunk)
constexpr int OG = 8;
__global__ void __launch_bounds__(64 * OG) k_dnn_output(int n, int C, int S, int nq, int nmod, const int* __restrict__ idx,
                             const float* __restrict__ P, long sP, const float* __restrict__ b,
                             const double* __restrict__ Ymu, const double* __restrict__ Ystd,
                             const double* __restrict__ Y, const double* __restrict__ rho,
                             const double* __restrict__ p, double dt, double* __restrict__ RR,
                             const double* __restrict__ hc, double* __restrict__ Qdot) {
  __shared__ double syn[64][64], ssum[64];   // [species][cell]; nmod <= 63
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + cl;
  const bool live = i < n;
  const int c = live ? idx[i] : 0;
  if (live)
    for (int m = g; m < nmod; m += OG) {
      float a = 0.0f;
      for (int q = 0; q < nq; ++q) a += P[m * sP + (long)q * n + i];   // the GEMM's partial dot products, in order
      const double out = (double)(_Float16)(a + b[m]);   // the net's fp16 output, as .to(kDouble)
      const double ybct = (pow(Y[(long)m * C + c], 0.1) - 1.0) * 10.0;
      const double v = out * Ystd[m] + Ymu[m] + ybct;
      syn[m][cl] = pow(v * 0.1 + 1.0, 10.0);
    }
  __syncthreads();
  if (g == 0 && live) {
    double sum = 0.0;
    for (int m = 0; m < nmod; ++m) sum += syn[m][cl];
    ssum[cl] = sum + Y[(long)(S - 1) * C + c];
  }
  __syncthreads();
  if (live) {
    const double rc = rho[c], pc = p[c] / 101325.0, sum = ssum[cl];
    for (int m = g; m < nmod; m += OG) {
      const double y = syn[m][cl] / sum;
      const double rr = (y - Y[(long)m * C + c]) * rc * pc / dt;
      RR[(long)m * C + c] = rr;
      syn[m][cl] = rr;   // only this thread reads syn[m][cl]; it now holds RR for the heat release below
    }
  }
  __syncthreads();
  // Qdot = -sum_i hc_i RR_i in species order (pytorchFunctions.H:233-238; the inert species' RR is 0 here)
  if (g == 0 && live && hc) {   // hc == nullptr: no thermo table uploaded (a surrogate-only context)
    double q = 0.0;
    for (int m = 0; m < nmod; ++m) q -= hc[m] * syn[m][cl];
    Qdot[c] = q;
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
  DFMI_CHECK(nmod == x.S - 1 && nmod <= 63, "DNN: one net per non-inert species (S - 1 <= 63) expected");
  DFMI_CHECK(nlayers >= 2 && nlayers <= 8, "DNN: 2..8 linear layers supported");
  DFMI_CHECK(dims[0] == x.S + 2 && dims[nlayers] == 1, "DNN: input must be S + 2 wide and output 1 wide");
  DFMI_CHECK(x.inert == x.S - 1, "DNN: the reference layout needs the inert species last");
  d.nmod = nmod;
  d.dims.assign(dims, dims + nlayers + 1);
  d.Kp.resize(nlayers);
  for (int l = 0; l < nlayers; ++l) {
    // K of every layer padded to the GEMM K tile; activations are stored with that row stride (the
    // padding columns are written as 0, the padded weight columns are 0)
    // (widths >= 512 to 64: the ping-pong kernel's K tile; the extra zero columns add exact zeros)
    const int kp = dims[l] >= 512 ? 64 : KPAD;
    d.Kp[l] = (dims[l] + kp - 1) / kp * kp;
    if (l == nlayers - 1) DFMI_CHECK(dims[l] % 8 == 0, "DNN: last hidden width must be a multiple of 8");
  }
  // repack weights: per layer [module][out][Kp] fp16 (K zero-padded), biases fp16-rounded, kept as fp32 [module][out]
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
      for (int o = 0; o < out; ++o) hb[l][(size_t)m * out + o] = (float)(_Float16)p[o];   // module.to(kHalf)
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

void dnn_prepare(Ctx& x) {
  Dnn& d = x.dnn;
  DFMI_CHECK(d.ready, "DNN model not set (dfmi_dnn_set_model)");
  const int C = x.C;
  const int nb = blocks_for(C, CB);
  if (d.bc.n < (size_t)nb + 1) d.bc.alloc(nb + 1);
  if (d.idx.n < (size_t)C) d.idx.alloc(C);
  hipLaunchKernelGGL(k_react_count, dim3(nb), dim3(CB), 0, x.stream, C, x.f("T"), d.T_react, d.bc.p);
  hipLaunchKernelGGL(k_react_scan, dim3(1), dim3(1024), 0, x.stream, nb, d.bc.p, d.bc.p + nb);
  hipLaunchKernelGGL(k_react_scatter, dim3(nb), dim3(CB), 0, x.stream, C, x.f("T"), d.T_react, d.bc.p, d.idx.p);
  DFMI_HIP(hipGetLastError());
  d.nr_host.ensure(1);
  if (!d.nr_ev) DFMI_HIP(hipEventCreateWithFlags(&d.nr_ev, hipEventDisableTiming));
  DFMI_HIP(hipMemcpyAsync(d.nr_host.p, d.bc.p + nb, sizeof(int), hipMemcpyDeviceToHost, x.stream));
  DFMI_HIP(hipEventRecord(d.nr_ev, x.stream));
  d.prepared = true;
}

void dnn_solve(Ctx& x, const char* rho_field) {
  Dnn& d = x.dnn;
  DFMI_CHECK(d.ready, "DNN model not set (dfmi_dnn_set_model)");
  const int C = x.C, S = x.S, L = (int)d.dims.size() - 1;
  if (!d.prepared) dnn_prepare(x);
  d.prepared = false;
  double* RR = x.f("RR");
  hipLaunchKernelGGL(k_zero, dim3(blocks_for((long)S * C, 256)), dim3(256), 0, x.stream, (long)S * C, RR);
  hipLaunchKernelGGL(k_zero, dim3(blocks_for((long)C, 256)), dim3(256), 0, x.stream, (long)C, x.f("Qdot"));
  // the count was copied behind an event at the step start; the solver polls since then have passed it
  DFMI_HIP(hipEventSynchronize(d.nr_ev));
  const int nr = d.nr_host.p[0];
  d.last_reacting = nr;
  if (nr == 0) return;
  const int chunk = std::min(nr, d.chunk);
  // the wide layers (K % 64 == 0, N >= 512: the 1600 -> 800 layer) through the 256x256x64 ping-pong kernel (8.72 ms
  // per 65,536-row chunk against k_mlp_gemm's 9.66), N = 256 q + t (t <= 32) with two 16-column tail strips in the
  // last two tiles (7.48-7.57 against 7.62-7.64 for one 32-column strip and 8.48 for a (q+1)-th tile); K = 64 layers
  // (the 55 -> 1600 input layer) through the 128 x 128 four-blocks-per-CU kernel (2.93 against 3.01 ms for a
  // 64 x 128 tile); DESIGN.md 8
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
    // the last hidden layer by the ping-pong kernel where its K allows (four 64-column partials per 256-wide
    // tile) or by k_mlp_gemm (two per 128-wide tile): partial sums per row of the fused output layer
    const bool tuned = x.on("dnn.tuned_gemm");
    const bool pp_out = tuned && d.Kp[L - 2] % 64 == 0 && d.Kp[L - 2] >= 512;
    const int nq = pp_out ? 4 * blocks_for(d.dims[L - 1], 256) : 2 * blocks_for(d.dims[L - 1], BN);
    const long sP = (long)nq * n;
    if (d.part.n < (size_t)d.nmod * sP) d.part.alloc((size_t)d.nmod * sP);
    for (int l = 0; l + 1 < L; ++l) {
      const int N = d.dims[l + 1], K = d.Kp[l], ldc = d.Kp[l + 1];
      _Float16* out = bufs[l & 1];
      d.gemm_flops += 2.0 * n * N * d.dims[l] * d.nmod;   // algorithmic flops (unpadded K)
      const dim3 g(blocks_for(N, BN) * blocks_for(n, 256), 1, d.nmod);
      KScope _ks(x, "k_mlp_gemm");
      if (l + 2 == L) {   // last hidden layer: the output layer fused into the epilogue
        d.gemm_flops += 2.0 * n * N * d.nmod;
        if (pp_out)
          hipLaunchKernelGGL((k_mlp_gemm_pp<true, true>), dim3(blocks_for(N, 256) * blocks_for(n, 256), 1, d.nmod),
                             dim3(512), 0, x.stream, n, N, K, in, lda, sIn, d.W[l].p, (long)N * K, d.b[l].p, (long)N, out,
                             ldc, (long)n * ldc, d.W[L - 1].p, (long)d.Kp[L - 1], d.part.p, sP);
        else
          hipLaunchKernelGGL((k_mlp_gemm<true, true>), g, dim3(256), 0, x.stream, n, N, K, in, lda, sIn, d.W[l].p,
                             (long)N * K, d.b[l].p, (long)N, out, ldc, (long)n * ldc, d.W[L - 1].p, (long)d.Kp[L - 1],
                             d.part.p, sP);
      } else if (tuned && K % 64 == 0 && K >= 512 && N >= 512) {   // the 1600 -> 800 layer
        const dim3 gw(blocks_for(N, 256) * blocks_for(n, 256), 1, d.nmod);
        // N = 256 q + t, 0 < t <= 16 q: q tiles, the last two with 16-column tail strips
        const bool tail = N % 256 != 0 && N % 256 <= 32 && ldc <= N / 256 * 256 + 64 && N / 256 >= 2;
        const dim3 gt(N / 256 * blocks_for(n, 256), 1, d.nmod);
        if (tail)
          hipLaunchKernelGGL((k_mlp_gemm_pp<true, false, 16>), gt, dim3(512), 0, x.stream, n, N, K, in, lda, sIn,
                             d.W[l].p, (long)N * K, d.b[l].p, (long)N, out, ldc, (long)n * ldc, nullptr, 0L, nullptr, 0L);
        else
          hipLaunchKernelGGL((k_mlp_gemm_pp<true>), gw, dim3(512), 0, x.stream, n, N, K, in, lda, sIn, d.W[l].p,
                             (long)N * K, d.b[l].p, (long)N, out, ldc, (long)n * ldc);
      } else if (tuned && K == 64) {   // the 55 -> 1600 input layer of the 53-species nets
        hipLaunchKernelGGL((k_mlp_gemm_in<true, 128>), dim3(blocks_for(N, 128) * blocks_for(n, 128), 1, d.nmod),
                           dim3(256), 0, x.stream, n, N, K, in, lda, sIn, d.W[l].p, (long)N * K, d.b[l].p, (long)N, out,
                           ldc, (long)n * ldc);
      } else {
        hipLaunchKernelGGL((k_mlp_gemm<true, false>), g, dim3(256), 0, x.stream, n, N, K, in, lda, sIn, d.W[l].p,
                           (long)N * K, d.b[l].p, (long)N, out, ldc, (long)n * ldc, nullptr, 0L, nullptr, 0L);
      }
      DFMI_HIP(hipGetLastError());
      in = out;
      sIn = (long)n * ldc;
      lda = ldc;
    }
    KScope _ks(x, "k_dnn_output");
    hipLaunchKernelGGL(k_dnn_output, dim3(blocks_for(n, 64)), dim3(64 * OG), 0, x.stream, n, C, S, nq, d.nmod, idx,
                       d.part.p, sP, d.b[L - 1].p, d.ymu.p, d.ystd.p, x.f("Y"), x.f(rho_field), x.f("p"), d.dt, RR,
                       x.thermo.dhc.n == (size_t)S ? (const double*)x.thermo.dhc.p : nullptr, x.f("Qdot"));
    DFMI_HIP(hipGetLastError());
  }
}

}  // namespace dfmi
