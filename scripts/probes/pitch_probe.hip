// Species-plane pitch probe: each thread c reads NA arrays laid out at buf[a * pitch + c] (the [S][C]
// field layout) and writes their sum. Measures GB/s for power-of-two pitches (C = 2^21 doubles = 16 MiB
// planes) against padded pitches, to see whether many concurrently streamed planes at a 16-MiB stride
// lose bandwidth (address-translation or channel conflicts).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_sum(const double* __restrict__ buf, long pitch, int na, long C, double* __restrict__ out) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int a = 0; a < na; ++a) s += buf[a * pitch + c];
  out[c] = s;
}

// same reads, but each thread handles 8 consecutive arrays per pass over the cells (chunked species loop)
__global__ void k_sum_chunk(const double* __restrict__ buf, long pitch, int na, long C, double* __restrict__ out) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int a0 = 0; a0 < na; a0 += 8) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = a0 + j < na ? buf[(a0 + j) * pitch + c] : 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  out[c] = s;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
  const long C = 1L << 21;
  const int nas[] = {1, 9, 27, 53, 106};
  const long pads[] = {0, 8, 64, 512, 4096, 65536 + 128};
  const long maxpitch = C + 65536 + 128;
  double *buf, *out;
  CK(hipMalloc(&buf, sizeof(double) * maxpitch * 106));
  CK(hipMalloc(&out, sizeof(double) * C));
  CK(hipMemset(buf, 0, sizeof(double) * maxpitch * 106));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int kind = 0; kind < 2; ++kind)
    for (int na : nas)
      for (long pad : pads) {
        const long pitch = C + pad;
        auto run = [&]() {
          if (kind == 0) hipLaunchKernelGGL(k_sum, dim3(C / 256), dim3(256), 0, 0, buf, pitch, na, C, out);
          else hipLaunchKernelGGL(k_sum_chunk, dim3(C / 256), dim3(256), 0, 0, buf, pitch, na, C, out);
        };
        run(); run();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) run();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        const double gbs = (double)(na + 1) * C * 8 / (us * 1e-6) / 1e9;
        printf("{\"kernel\": \"%s\", \"arrays\": %d, \"pad_doubles\": %ld, \"us\": %.1f, \"GBs\": %.0f}\n",
               kind ? "chunk8" : "loop", na, pad, us, gbs);
        fflush(stdout);
      }
  return 0;
}
