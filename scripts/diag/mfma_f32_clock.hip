// fp32 MFMA ceiling probe: back-to-back v_mfma_f32_16x16x4_f32 (4 or 8 waves per CU, 4
// independent accumulator chains per wave, operands in registers, no memory in the loop) on
// random vs zero operands.  Prints wall time, achieved TF/s and the in-kernel clock
// (s_memtime / s_memrealtime x 100 MHz, median over workgroups) -- whether the fp32 conv
// kernels' ~60 % "MFMA busy" is a DVFS clock ceiling or lost issue cycles.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_f32_clock scripts/diag/mfma_f32_clock.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int ITERS>
__global__ __launch_bounds__(512) void mfma_loop(const float* in, float* out, unsigned long long* clk) {
  const int t = threadIdx.x;
  float a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = in[(t * 8 + i) & 4095];
    b[i] = in[(t * 8 + i + 2048) & 4095];
  }
  f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  const unsigned long long m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; i += 4) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1], b[i + 1], c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 2], b[i + 2], c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 3], b[i + 3], c3, 0, 0, 0);
    }
  }
  const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + t] = s[0] + s[1] + s[2] + s[3];
  if (t == 0) {
    clk[2 * blockIdx.x] = m1 - m0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  constexpr int ITERS = 20000;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float *in, *out;
  unsigned long long* clk;
  hipMalloc(&in, 4096 * sizeof(float));
  hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
  hipMalloc(&clk, (size_t)cus * 2 * sizeof(unsigned long long));
  std::vector<float> h(4096);
  for (int zero = 0; zero < 2; ++zero) {
    for (auto& x : h) x = zero ? 0.f : (float)rand() / RAND_MAX - 0.5f;
    hipMemcpy(in, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
    for (int threads : {256, 512}) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int w = 0; w < 400; ++w) mfma_loop<ITERS><<<cus, threads>>>(in, out, clk);  // >= 2 s hot
      hipEventRecord(e0);
      mfma_loop<ITERS><<<cus, threads>>>(in, out, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> c(2 * cus);
      hipMemcpy(c.data(), clk, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      std::vector<double> ghz(cus);
      for (int i = 0; i < cus; ++i) ghz[i] = c[2 * i] / (c[2 * i + 1] * 0.01) / 1000.0;  // memrealtime: 100 MHz
      std::sort(ghz.begin(), ghz.end());
      const double flop = 2.0 * 1024 * 8 * (double)ITERS * cus * (threads / 64);
      const double cyc_per_mfma = c[0] / (8.0 * ITERS) / 1.0;
      printf("%s operands, %d waves/CU: %.3f ms, %.1f TF/s, in-kernel clock median %.2f GHz (min %.2f max %.2f), "
             "%.1f cycles per MFMA per wave\n",
             zero ? "zero" : "random", threads / 64, ms, flop / ms / 1e9, ghz[cus / 2], ghz[0], ghz[cus - 1],
             cyc_per_mfma);
    }
  }
  return 0;
}
