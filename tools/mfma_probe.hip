// Microbenchmark: cycles per MFMA instruction on gfx950 (one wave per SIMD, 4 independent accumulators).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ void probe(float* out, long long* cyc, int iters) {
  bf16x8 a8, b8; s16x4 a4, b4;
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(threadIdx.x * 0.001f + i); b8[i] = (__bf16)(i * 0.5f); }
  for (int i = 0; i < 4; ++i) { a4[i] = (short)(threadIdx.x + i); b4[i] = (short)(i * 3); }
  f32x4 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  f32x16 d0 = {0}, d1 = {0};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c3, 0, 0, 0);
    } else if constexpr (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c3, 0, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d1, 0, 0, 0);
    }
  }
  long long t1 = clock64();
  float s = c0[0] + c1[1] + c2[2] + c3[3] + d0[0] + d1[5];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float* out; long long* cyc; hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 8);
  const int iters = 4096;
  const char* names[3] = {"16x16x32_bf16 x4", "16x16x16_bf16_1k x4", "32x32x16_bf16 x2"};
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (k == 0) probe<0><<<1024, 256>>>(out, cyc, iters);
      if (k == 1) probe<1><<<1024, 256>>>(out, cyc, iters);
      if (k == 2) probe<2><<<1024, 256>>>(out, cyc, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      double flops_per_iter = (k == 0) ? 4 * 16 * 16 * 32 * 2.0 : (k == 1) ? 4 * 16 * 16 * 16 * 2.0 : 2 * 32 * 32 * 16 * 2.0;
      double tf = flops_per_iter * iters * 1024 * 4 / (ms * 1e-3) / 1e12;
      if (rep) printf("%-22s clock64 cycles/iter %.1f  (%.1f per MFMA)  chip %.0f TFLOP/s\n", names[k],
                      (double)c / iters, (double)c / iters / (k == 2 ? 2 : 4), tf);
    }
  }
  return 0;
}
