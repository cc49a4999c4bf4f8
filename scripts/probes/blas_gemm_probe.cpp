// Library calibration for the DNN hidden layers: rocBLAS gemm_strided_batched_ex on the shapes of
// BASELINE config 4's nets -- 52 nets x 65,536 rows, fp16 in/out, fp32 accumulate, C[M][N] = A[M][K] W[N][K]^T --
// timed with HIP events (no bias / GELU epilogue: the plain GEMM only). Build:
//   hipcc --offload-arch=gfx950 -O2 scripts/probes/blas_gemm_probe.cpp -lrocblas -o scripts/probes/blas_gemm_probe
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>

#define CK(x) do { auto e = (x); if (e != 0) { std::printf("error %d at %s:%d\n", (int)e, __FILE__, __LINE__); return 1; } } while (0)

int main() {
  const int M = 65536, B = 52;
  const int shapes[3][2] = {{1600, 64}, {800, 1600}, {400, 800}};   // (N, K): 55(->64)->1600, 1600->800, 800->400
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(rocblas_set_stream(h, st));
  for (auto& s : shapes) {
    const int N = s[0], K = s[1];
    const size_t na = (size_t)M * K * B, nw = (size_t)N * K * B, nc = (size_t)M * N * B;
    _Float16 *A, *W, *Cm;
    CK(hipMalloc(&A, na * 2)); CK(hipMalloc(&W, nw * 2)); CK(hipMalloc(&Cm, nc * 2));
    CK(hipMemset(A, 0x3c, na * 2)); CK(hipMemset(W, 0x1c, nw * 2));
    const float alpha = 1.0f, beta = 0.0f;
    auto run = [&]() {
      return rocblas_gemm_strided_batched_ex(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &alpha,
                                             W, rocblas_datatype_f16_r, K, (rocblas_stride)N * K,
                                             A, rocblas_datatype_f16_r, K, (rocblas_stride)M * K, &beta,
                                             Cm, rocblas_datatype_f16_r, N, (rocblas_stride)M * N,
                                             Cm, rocblas_datatype_f16_r, N, (rocblas_stride)M * N, B,
                                             rocblas_datatype_f32_r, rocblas_gemm_algo_standard, 0, 0);
    };
    for (int i = 0; i < 3; ++i) CK(run());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int reps = 10;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) CK(run());
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double fl = 2.0 * M * N * K * (double)B;
    std::printf("{\"N\": %d, \"K\": %d, \"ms_per_chunk\": %.3f, \"tflops\": %.1f, \"frac_of_2500\": %.3f}\n", N, K, ms,
                fl / (ms * 1e-3) / 1e12, fl / (ms * 1e-3) / 1e12 / 2500.0);
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(Cm));
  }
  rocblas_destroy_handle(h);
  return 0;
}
