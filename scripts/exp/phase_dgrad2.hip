// Phase timing of the conv2 dgrad kernel (experiment; not part of the library build).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/phase_dgrad2.hip -o /tmp/phase && /tmp/phase
#include "../../ape-x_amd/ops/csrc/common.h"
#include <cstdio>
#include <vector>

using namespace apex;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int DY_PIX = 144;

__device__ __forceinline__ bool bf16_pos(uint16_t v) { return v != 0 && !(v & 0x8000); }

template <int OH, int OW, int TH, int TW, int BORDER>
__device__ __forceinline__ void stage_dy_padded(const uint16_t* __restrict__ dy, char* t) {
  constexpr int CH = 8;
  stage_all<OH * OW * CH>(reinterpret_cast<const uint4*>(dy), t, [](int q) {
    const int pix = q / CH, cc = q % CH;
    return ((pix / OW + BORDER) * TW + pix % OW + BORDER) * DY_PIX + cc * 16;
  });
}

__global__ __launch_bounds__(256) void dgrad2_t(const uint16_t* __restrict__ dy2, const uint16_t* __restrict__ wt2,
                                                const uint16_t* __restrict__ a1, uint16_t* __restrict__ dy1, int B,
                                                long long* tm, int skip_mask) {
  constexpr int T = 11, TILE = T * T * DY_PIX;
  constexpr int SPW = 2;
  __shared__ __attribute__((aligned(16))) char smem[SPW * TILE + 16 * 32 * DY_PIX];
  char* wts = smem + SPW * TILE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  long long t0 = clock64();
  for (int q = threadIdx.x; q < SPW * T * T * DY_PIX / 16; q += blockDim.x) reinterpret_cast<uint4*>(smem)[q] = uint4{0, 0, 0, 0};
  stage_all<16 * 32 * 8>(reinterpret_cast<const uint4*>(wt2), wts, [](int q) { return (q / 8) * DY_PIX + (q % 8) * 16; });
  __syncthreads();
  long long t1 = clock64(), t2 = 0, t3 = 0;
  for (int b0 = blockIdx.x * SPW; b0 < B; b0 += gridDim.x * SPW) {
    __syncthreads();
    for (int sw = 0; sw < SPW; ++sw)
      if (b0 + sw < B) stage_dy_padded<9, 9, T, T, 1>(dy2 + (size_t)(b0 + sw) * 81 * 64, smem + sw * TILE);
    __syncthreads();
    t2 = clock64();
    for (int it = wave; it < SPW * 16; it += 4) {
      const int sw = it / 16, cls = (it / 4) % 4, mt = it % 4;
      const int b = b0 + sw;
      if (b >= B) continue;
      const int ry = cls >> 1, rx = cls & 1;
      const int m = mt * 32 + r32;
      const int mc = m < 100 ? m : 99;
      const int i = mc / 10, j = mc % 10;
      const char* abase = smem + sw * TILE + ((i + 1) * T + (j + 1)) * DY_PIX + h * 16;
      const char* bbase = wts + r32 * DY_PIX + h * 16;
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int sub = s / 4, dyy = sub >> 1, dxx = sub & 1, n0 = (s % 4) * 16;
        const int tap = (ry + 2 * dyy) * 4 + (rx + 2 * dxx);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(abase - (dyy * T + dxx) * DY_PIX + n0 * 2);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(bbase + tap * 32 * DY_PIX + n0 * 2);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc, 0, 0, 0);
      }
      const int c = r32;
      const uint16_t* ab = a1 + (size_t)b * 400 * 32 + c;
      uint16_t* ob = dy1 + (size_t)b * 400 * 32 + c;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (mm < 100) {
          const int q = (2 * (mm / 10) + ry) * 20 + 2 * (mm % 10) + rx;
          ob[q * 32] = (skip_mask || bf16_pos(ab[q * 32])) ? f2bf(acc[r]) : (uint16_t)0;
        }
      }
    }
    t3 = clock64();
  }
  __syncthreads();
  long long t4 = clock64();
  if (threadIdx.x == 0 || threadIdx.x == 64 || threadIdx.x == 128 || threadIdx.x == 192) {
    long long* o = tm + (blockIdx.x * 4 + wave) * 5;
    o[0] = t0; o[1] = t1; o[2] = t2; o[3] = t3; o[4] = t4;
  }
}

int main() {
  const int B = 512, grid = 256;
  uint16_t *dy2, *wt2, *a1, *dy1;
  long long* tm;
  hipMalloc(&dy2, (size_t)B * 81 * 64 * 2);
  hipMalloc(&wt2, 16 * 32 * 64 * 2);
  hipMalloc(&a1, (size_t)B * 400 * 32 * 2);
  hipMalloc(&dy1, (size_t)B * 400 * 32 * 2);
  hipMalloc(&tm, grid * 4 * 5 * 8);
  hipMemset(dy2, 0x3c, (size_t)B * 81 * 64 * 2);
  hipMemset(wt2, 0x3c, 16 * 32 * 64 * 2);
  hipMemset(a1, 0x3c, (size_t)B * 400 * 32 * 2);
  for (int skip = 0; skip < 2; ++skip) {
    for (int w = 0; w < 3; ++w) dgrad2_t<<<grid, 256>>>(dy2, wt2, a1, dy1, B, tm, skip);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int w = 0; w < 20; ++w) dgrad2_t<<<grid, 256>>>(dy2, wt2, a1, dy1, B, tm, skip);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(grid * 4 * 5);
    hipMemcpy(h.data(), tm, h.size() * 8, hipMemcpyDeviceToHost);
    double ph[4] = {0, 0, 0, 0};
    long long mn = h[0];
    for (int i = 0; i < grid * 4; ++i) mn = std::min(mn, h[i * 5]);
    double end_max = 0;
    for (int i = 0; i < grid * 4; ++i) {
      for (int k = 0; k < 4; ++k) ph[k] += (double)(h[i * 5 + k + 1] - h[i * 5 + k]);
      end_max = std::max(end_max, (double)(h[i * 5 + 4] - mn));
    }
    printf("skip_mask=%d: %.2f us/launch; mean cycles: weights %.0f, stage_dy %.0f, compute+epilogue %.0f, tail %.0f; span %.0f\n",
           skip, ms * 1000 / 20, ph[0] / (grid * 4), ph[1] / (grid * 4), ph[2] / (grid * 4), ph[3] / (grid * 4), end_max);
  }
  return 0;
}
