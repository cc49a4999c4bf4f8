// gelu_probe.hip -- issue-rate probe for the DNN GEMM epilogue's GELU (dnn.hip gelu_fast2): the same
// Abramowitz-Stegun erf form evaluated (0) with packed fp32 instructions (v_pk_fma_f32 / v_pk_mul_f32, as in
// dnn.hip) and (1) with scalar fp32 instructions (this file is built with -fno-slp-vectorize so the scalar
// form stays scalar), both inside the fp16 rounding the epilogue applies. Every lane runs 8 independent
// chains over registers only; the result is stored so nothing is dead.
//   hipcc -O3 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 gelu_probe.hip -o gelu_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

using f32x2 = __attribute__((ext_vector_type(2))) float;

__device__ __forceinline__ f32x2 gelu_pk(f32x2 v) {
  const f32x2 u = v * 0.70710678118654752440f;
  const f32x2 a = __builtin_elementwise_abs(u);
  const f32x2 d = __builtin_elementwise_fma(a, f32x2(0.3275911f), f32x2(1.0f));
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 q = __builtin_elementwise_fma(t, f32x2(1.061405429f), f32x2(-1.453152027f));
  q = __builtin_elementwise_fma(t, q, f32x2(1.421413741f));
  q = __builtin_elementwise_fma(t, q, f32x2(-0.284496736f));
  q = __builtin_elementwise_fma(t, q, f32x2(0.254829592f));
  const f32x2 poly = t * q;
  const f32x2 w = (a * a) * -1.44269504088896340736f;
  const f32x2 ex = {__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  const f32x2 e = __builtin_elementwise_fma(-poly, ex, f32x2(1.0f));
  const f32x2 hv = v * 0.5f;
  const f32x2 se = {copysignf(e.x, u.x), copysignf(e.y, u.y)};
  return __builtin_elementwise_fma(hv, se, hv);
}

__device__ __forceinline__ float gelu_sc(float v) {
  const float u = v * 0.70710678118654752440f;
  const float a = fabsf(u);
  const float d = fmaf(a, 0.3275911f, 1.0f);
  const float t = __builtin_amdgcn_rcpf(d);
  float q = fmaf(t, 1.061405429f, -1.453152027f);
  q = fmaf(t, q, 1.421413741f);
  q = fmaf(t, q, -0.284496736f);
  q = fmaf(t, q, 0.254829592f);
  const float poly = t * q;
  const float w = (a * a) * -1.44269504088896340736f;
  const float ex = __builtin_amdgcn_exp2f(w);
  const float e = fmaf(-poly, ex, 1.0f);
  const float hv = v * 0.5f;
  return fmaf(hv, copysignf(e, u), hv);
}

// the lean form: 0.5 v (1 + sign(v) erf|u|) = fma(|0.5 v|, erf|u|, 0.5 v); 1/sqrt2 folded into the constants,
// |.| as source modifiers (scalar VOP3) or one v_and (packed: VOP3P has no abs modifier)
__device__ __forceinline__ float gelu_lean(float v) {
  const float hv = v * 0.5f;
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(v), 0.23164202848f, 1.0f));
  float q = fmaf(t, 1.061405429f, -1.453152027f);
  q = fmaf(t, q, 1.421413741f);
  q = fmaf(t, q, -0.284496736f);
  q = fmaf(t, q, 0.254829592f);
  const float ex = __builtin_amdgcn_exp2f(v * (v * -0.72134752044448170368f));
  const float e = fmaf(-(t * q), ex, 1.0f);
  return fmaf(fabsf(hv), e, hv);
}
__device__ __forceinline__ f32x2 gelu_lean2(f32x2 v) {
  const f32x2 hv = v * 0.5f;
  const f32x2 a = __builtin_elementwise_abs(v);
  const f32x2 d = __builtin_elementwise_fma(a, f32x2(0.23164202848f), f32x2(1.0f));
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 q = __builtin_elementwise_fma(t, f32x2(1.061405429f), f32x2(-1.453152027f));
  q = __builtin_elementwise_fma(t, q, f32x2(1.421413741f));
  q = __builtin_elementwise_fma(t, q, f32x2(-0.284496736f));
  q = __builtin_elementwise_fma(t, q, f32x2(0.254829592f));
  const f32x2 w = v * (v * -0.72134752044448170368f);
  const f32x2 ex = {__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  const f32x2 e = __builtin_elementwise_fma(-(t * q), ex, f32x2(1.0f));
  return __builtin_elementwise_fma(a * 0.5f, e, hv);
}

__device__ __forceinline__ float r16(float v) { return (float)(_Float16)v; }

template <int MODE>
__global__ void __launch_bounds__(256) k_probe(int iters, const float* __restrict__ in, float* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = in[(tid * 8 + i) & 4095];
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0 || MODE == 3) {
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        f32x2 x = {r16(v[i] + 0.25f), r16(v[i + 1] + 0.25f)};
        x = MODE == 0 ? gelu_pk(x) : gelu_lean2(x);
        v[i] = r16(x.x);
        v[i + 1] = r16(x.y);
      }
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = r16(gelu_sc(r16(v[i] + 0.25f)));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = r16(gelu_lean(r16(v[i] + 0.25f)));
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += v[i];
  out[tid] = acc;
}

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 256;
  float *in, *out;
  hipMalloc(&in, 4096 * sizeof(float));
  hipMalloc(&out, (size_t)blocks * threads * sizeof(float));
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = -4.0f + 8.0f * (float)i / 4096.0f;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double vals = (double)blocks * threads * iters * 8;
  const char* names[4] = {"packed", "scalar", "lean-scalar", "lean-packed"};
  for (int mode = 0; mode < 4; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(threads), 0, 0, iters, in, out);
      else if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(threads), 0, 0, iters, in, out);
      else if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(threads), 0, 0, iters, in, out);
      else hipLaunchKernelGGL(k_probe<3>, dim3(blocks), dim3(threads), 0, 0, iters, in, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("mode %s rep %d: %.3f ms, %.1f G gelu/s, %.3f ms per 5.45 G values\n", names[mode], rep, ms,
             vals / ms * 1e-6, 5.45e3 / (vals / ms * 1e-6));
    }
  return 0;
}
