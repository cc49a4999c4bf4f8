// dfmi_common.h -- shared host/device definitions for the MI355X-native dfLowMachFoam hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

// The library is written for MI355X alone: wave_sum's v_permlane16/32_swap, the MFMA tiles of dnn.hip and the
// LDS-DMA staging exist on gfx950 only. A device pass for any other target stops here with a clear message.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "dfmi targets gfx950 (MI355X) only: build with --offload-arch=gfx950 (Makefile ARCH)"
#endif

namespace dfmi {

// Block -> cell range for the per-cell (gather) kernels: the dispatcher deals consecutive blocks
// round-robin to the 8 XCDs, each with its own L2. Remapped so that XCD x works through one contiguous
// slab of blocks, a cell's y- and z-neighbours (a row / a plane away) are gathered from lines its own
// L2 already holds (measured: the FV assembly kernels 12-18 % faster). Bijective for any grid.
__device__ __forceinline__ int xcd_block() {
  const int nb = gridDim.x, b = blockIdx.x;
  if (nb < 16) return b;
  const int x = b % 8, q = nb / 8, r = nb % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}


// Boundary-condition codes, identical to the reference enum (src_gpu/dfMatrixDataBase.H:81-93)
// plus two mixed conditions the reference GPU path rejects (dfMatrixDataBase.cu:22-27) but its CPU
// cases use: waveTransmissive (test/Tu500K-Phi1/0/p:34) and inletOutlet
enum BC : int8_t {
  ZERO_GRADIENT = 0, FIXED_VALUE = 1, COUPLED = 2, EMPTY = 3, GRADIENT_ENERGY = 4, CALCULATED = 5,
  CYCLIC = 6, PROCESSOR = 7, EXTRAPOLATED = 8, FIXED_ENERGY = 9, PROCESSOR_CYCLIC = 10,
  WAVE_TRANSMISSIVE = 11, INLET_OUTLET = 12
};

__host__ __device__ inline bool bc_coupled(int t) { return t == CYCLIC || t == PROCESSOR || t == PROCESSOR_CYCLIC || t == COUPLED; }
__host__ __device__ inline bool bc_proc(int t) { return t == PROCESSOR || t == PROCESSOR_CYCLIC; }
__host__ __device__ inline bool bc_fixes_value(int t) { return t == FIXED_VALUE || t == FIXED_ENERGY; }
// mixedFvPatchField: value = f ref + (1 - f) cell (refGrad = 0)
__host__ __device__ inline bool bc_mixed(int t) { return t == WAVE_TRANSMISSIVE || t == INLET_OUTLET; }

struct Error : std::runtime_error { using std::runtime_error::runtime_error; };

#define DFMI_HIP(call)                                                                              \
  do {                                                                                              \
    hipError_t _e = (call);                                                                         \
    if (_e != hipSuccess)                                                                           \
      throw ::dfmi::Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + __FILE__ + \
                          ":" + std::to_string(__LINE__) + " in " #call);                           \
  } while (0)

#define DFMI_CHECK(cond, msg) \
  do { if (!(cond)) throw ::dfmi::Error(std::string("dfmi: ") + (msg)); } while (0)

// Owning device allocation (the reference never frees, dfMatrixDataBase.cu:111; we do).
template <class T> struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; return *this; }
  ~DevBuf() { release(); }
  void release() { if (p) { (void)hipFree(p); p = nullptr; n = 0; } }
  void alloc(size_t count) {
    release();
    n = count;
    if (count) DFMI_HIP(hipMalloc(&p, count * sizeof(T)));
  }
  void zero(hipStream_t s) { if (n) DFMI_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s)); }
  void upload(const T* h, size_t count, hipStream_t s) {
    if (count != n) alloc(count);
    if (count) DFMI_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
  }
  void upload(const std::vector<T>& v, hipStream_t s) { upload(v.data(), v.size(), s); }
  operator T*() const { return p; }
};

// Owning pinned host allocation (device-visible; async copies into it need no staging).
template <class T> struct PinnedBuf {
  T* p = nullptr;
  T* d = nullptr;   // device view (ensure_mapped only)
  size_t n = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() { release(); }
  void release() { if (p) { (void)hipHostFree(p); p = nullptr; n = 0; } d = nullptr; }
  void ensure(size_t count) {
    if (count <= n) return;
    release();
    DFMI_HIP(hipHostMalloc(&p, count * sizeof(T), hipHostMallocDefault));
    n = count;
  }
  // mapped into the device's address space: kernels store into it directly (read by the host after a sync)
  void ensure_mapped(size_t count) {
    if (count <= n && d) return;
    release();
    DFMI_HIP(hipHostMalloc(&p, count * sizeof(T), hipHostMallocMapped));
    DFMI_HIP(hipHostGetDevicePointer((void**)&d, p, 0));
    n = count;
  }
};

// Convergence record a solver kernel posts into host-coherent pinned memory (linsolve.hip Poller): the host
// spins on `seq` (stored last, system-scope release) instead of waiting on an event behind a copy.
struct PollRec {
  long long seq;       // snapshot number, written last
  int stopped;         // every system of the solve has stopped
  int iters;           // the largest iteration count among the systems
};
struct HostRecs {      // two alternating records, mapped into the device's address space
  PollRec* h = nullptr;
  PollRec* d = nullptr;
  HostRecs() = default;
  HostRecs(const HostRecs&) = delete;
  HostRecs& operator=(const HostRecs&) = delete;
  ~HostRecs() { if (h) (void)hipHostFree(h); }
  void ensure() {
    if (h) return;
    DFMI_HIP(hipHostMalloc((void**)&h, 2 * sizeof(PollRec), hipHostMallocCoherent | hipHostMallocMapped));
    for (int i = 0; i < 2; ++i) { h[i].seq = 0; h[i].stopped = 0; h[i].iters = 0; }
    DFMI_HIP(hipHostGetDevicePointer((void**)&d, h, 0));
  }
};

inline int blocks_for(long n, int tpb) { return (int)((n + tpb - 1) / tpb); }

// Columns of the per-cell gather rows [W][C] (the solver ELL, linsolve.hip build_ell). Row classes: on
// meshes where few distinct rows occur relative to the cell (a hex box in blockMesh order: 27 -- interior,
// faces, edges, corners), cell c stores one byte, its class, and the class table holds the W column
// offsets j - c; an entry the table cannot express (a processor halo column) is read from the explicit
// array. A gather then reads 1 B per cell instead of 4 W B (24 B on hex meshes). cls == nullptr: explicit.
constexpr int CEXPL = -2147483647 - 1;   // class-table entry: read the explicit array
constexpr int CT_MAX = 1536;              // class-table entries (ncls x W) a kernel stages in LDS
struct ColView {
  const int* col = nullptr;         // explicit [W][C]
  const uint8_t* cls = nullptr;     // [C] row class, or nullptr
  const int* tab = nullptr;         // [ncls][W] column offsets
  int W = 0;
  int ntab = 0;                     // ncls * W <= CT_MAX
  // every thread of the block, before any divergent exit: the class table into LDS (sh: CT_MAX ints)
  __device__ __forceinline__ void stage(int* sh) const {
    if (cls) {
      for (int i = threadIdx.x; i < ntab; i += blockDim.x) sh[i] = tab[i];
      __syncthreads();
    }
  }
  // the row's offset into the staged table (-1: explicit columns)
  __device__ __forceinline__ int row(int c) const { return cls ? (int)cls[c] * W : -1; }
  __device__ __forceinline__ int get(const int* sh, int rb, long C, int k, int c) const {
    if (rb >= 0) {
      const int o = sh[rb + k];
      if (o != CEXPL) return c + o;
    }
    return col[k * C + c];
  }
  // all W columns of the row before any gather: the class offsets (LDS) and the explicit columns a row
  // needs are read first, so the row's W gathers issue together instead of each waiting at the join of
  // the class / explicit branch for every load before it (get() per entry serialises the gathers).
  // Measured on the even-odd kernels: 40.4 -> 40.2 us per launch -- with 8 waves per SIMD in flight they
  // were bandwidth- rather than latency-bound already; the same change to face_row made k_cg_spmv slower
  // (44.7 -> 49.7 us: more VGPRs, loads for the absent neighbours) and was not kept.
  template <int W> __device__ __forceinline__ void get_all(const int* sh, int rb, long C, int c,
                                                           int (&j)[W]) const {
    int o[W];
#pragma unroll
    for (int k = 0; k < W; ++k) o[k] = rb >= 0 ? sh[rb + k] : CEXPL;
#pragma unroll
    for (int k = 0; k < W; ++k) j[k] = o[k] != CEXPL ? c + o[k] : col[k * C + c];
  }
};
// f(k, j) over row c's entries: columns first (get_all) when the width is a compile-time WT > 0
template <int WT, class F>
__device__ __forceinline__ void for_cols(const ColView& col, const int* sh, int rb, long C, int W, int c, F&& f) {
  if constexpr (WT > 0) {
    int j[WT];
    col.get_all<WT>(sh, rb, C, c, j);
#pragma unroll
    for (int k = 0; k < WT; ++k) f(k, j[k]);
  } else {
    for (int k = 0; k < W; ++k) f(k, col.get(sh, rb, C, k, c));
  }
}

// The symmetric pressure operator read face-wise on a hex box in blockMesh order (FaceOp::on; the cell's
// rows are the ELL's, checked at build_ell): faces from the computed (i, j, k) walk with their coefficient at
// the owner-slot storage index (lower == upper for the laplacian), then the cell's coupled slots in slot
// order with -boundaryCoeffs -- the ELL row's entries in the ELL's order without reading its 48 B of values
// (the face array holds each coefficient once: 24 B per cell) or padding. T: fp64, or the V-cycle's fp32
// copies (the ELL's rounding: (float) upper, -(float) bc).
template <class T> struct FaceOp {
  int on = 0;
  int nx = 0, ny = 0, nz = 0;
  long C = 0;
  const T* up = nullptr;           // face coefficients [kslot][C]
  const T* bc = nullptr;           // boundaryCoeffs [B]
  const int* csStart = nullptr;    // coupled slots of each cell [C + 1] ...
  const int* csSlot = nullptr;     // ... ascending slot index
  const int* scol = nullptr;       // column of a coupled slot: cyclic partner cell, or C + halo index
};
template <class T, class FN> __device__ __forceinline__ void face_row(const FaceOp<T>& o, int c, FN&& fn) {
  const int nx = o.nx, ny = o.ny, nxy = o.nx * o.ny;
  const int C = (int)o.C;
  const int t = c / nx, i = c - t * nx, k = t / ny, j = t - k * ny;
  const int hxp = i < nx - 1, hyp = j < ny - 1;
  if (k > 0) { const int q = c - nxy; fn(q, o.up[(hxp + hyp) * C + q]); }
  if (j > 0) { const int q = c - nx; fn(q, o.up[hxp * C + q]); }
  if (i > 0) fn(c - 1, o.up[c - 1]);
  if (hxp) fn(c + 1, o.up[c]);
  if (hyp) fn(c + nx, o.up[hxp * C + c]);
  if (k < o.nz - 1) fn(c + nxy, o.up[(hxp + hyp) * C + c]);
  const int e1 = o.csStart[c + 1];
  for (int e = o.csStart[c]; e < e1; ++e) {
    const int b = o.csSlot[e];
    fn(o.scol[b], -o.bc[b]);
  }
}

// ---- fixed-order reductions of per-block partials (solvers: linsolve.hip; the PCG stop test the AMG's
// first V-cycle kernel repeats, amg.hip). Blocks of RED_TPB threads.
constexpr int RED_TPB = 256, RED_NW = RED_TPB / 64;
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum over the wave, every lane ending with the same bits: lane pairings that are involutions, each step
// v + v(partner) (IEEE addition commutes, so both lanes of a pair agree): quad swaps, the half-row and row
// mirrors (DPP), then gfx950's row and half-wave swaps (v_permlane16/32_swap: both outputs hold the even /
// odd row, the lower / upper half, so the sum is formed in the same order everywhere). No LDS round trips
// (a __shfl butterfly is six dependent ds_bpermute pairs). Call with every lane of the wave active.
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
  {
    const auto l = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  {
    const auto l = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  return v;
}

// value(s, i, k) = p[i * si + s * ss + k], i < np: the per-block partials (single rank) or the
// all-gathered per-rank sums (multi-rank)
struct Red { const double* p; int np; long si, ss; };

// fixed-order block-wide sum, result in every thread
template <int NV> __device__ __forceinline__ void red_sum(const Red& r, int s, double (&out)[NV]) {
  __shared__ double sh[RED_NW][NV];
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  for (int i = threadIdx.x; i < r.np; i += RED_TPB)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += r.p[(long)i * r.si + (long)s * r.ss + k];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) { const double t = wave_sum(v[k]); if (lane == 0) sh[wid][k] = t; }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < RED_NW; ++w) a += sh[w][k];
    out[k] = a;
  }
  __syncthreads();
}

}  // namespace dfmi
