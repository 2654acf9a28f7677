// FC1 of the dueling heads (Linear 3136 -> 2 x 128, adv | value hidden) for gfx950.
//
// z[B][256] = a3[B][3136] . W[256][3136]^T is skinny (M = batch, N = 256, K = 3136): a
// library GEMM tiles only M x N (at B = 512: 128 32x32 tiles for 256 CUs) and walks the
// long K serially.  Here K is split 4 ways and, inside a workgroup, across its 4 waves:
//
//   * workgroup = 32 rows x 64 columns x K/4 (49 k-steps of 16); grid = B/32 x 4 x 4
//     (256 workgroups at B = 512, 128 for the 256-env actor batch);
//   * both MFMA operands are read straight from global memory into registers (A rows and
//     W rows are K-contiguous: one 16-byte load per lane per fragment, L2-resident), all
//     of a wave's loads issued before its MFMA chain -- no LDS staging;
//   * the 4 waves' partial tiles are summed in LDS in fixed order and written as one fp32
//     split-K partial [4][B][256]; heads_fwd sums the 4 partials (fixed order, so the
//     result is deterministic) before bias + ReLU + the dueling heads.
#include "common.h"
#include "kernels.h"

namespace apex {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int FC_K = 3136, FC_N = 256, FC_KSTEPS = FC_K / 16;  // 196
constexpr int FC_KSPLIT = 4, FC_KS_PER_SPLIT = FC_KSTEPS / FC_KSPLIT;  // 49
constexpr int FC_KS_PER_WAVE = (FC_KS_PER_SPLIT + 3) / 4;            // 13
static_assert(FC_KSTEPS % FC_KSPLIT == 0, "K split");
}  // namespace

int fc1_splits() { return FC_KSPLIT; }

// grid.x runs over the M tiles of all problems of the set (problem = tile / ceil(B/32))
__global__ __launch_bounds__(256) void fc1_fwd_k(FcSet set) {
  __shared__ float red[4][32 * 65];  // per-wave 32 x 64 tiles, padded rows
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  const int B = set.B, MT = (B + 31) / 32;
  const int pb = blockIdx.x / MT, mtile = blockIdx.x - pb * MT, ntile = blockIdx.y, split = blockIdx.z;
  const uint16_t* __restrict__ a = set.p[pb].a;
  const uint16_t* __restrict__ w = set.p[pb].w;
  float* __restrict__ part = set.p[pb].part;
  const int row = mtile * 32 + r32;
  const int rowc = row < B ? row : B - 1;
  // this wave's k-steps: split * 49 + [wave * 13, min(49, wave * 13 + 13))
  const int ks0 = split * FC_KS_PER_SPLIT + wave * FC_KS_PER_WAVE;
  const int nks = min(FC_KS_PER_WAVE, FC_KS_PER_SPLIT - wave * FC_KS_PER_WAVE);  // 13, 13, 13, 10
  const uint16_t* ar = a + (size_t)rowc * FC_K + 8 * h;
  const uint16_t* w0 = w + (size_t)(ntile * 64 + r32) * FC_K + 8 * h;
  const uint16_t* w1 = w0 + (size_t)32 * FC_K;
  bf16x8 fa[FC_KS_PER_WAVE], fb0[FC_KS_PER_WAVE], fb1[FC_KS_PER_WAVE];
#pragma unroll
  for (int i = 0; i < FC_KS_PER_WAVE; ++i) {
    if (i < nks) {
      const int k = (ks0 + i) * 16;
      fa[i] = *reinterpret_cast<const bf16x8*>(ar + k);
      fb0[i] = *reinterpret_cast<const bf16x8*>(w0 + k);
      fb1[i] = *reinterpret_cast<const bf16x8*>(w1 + k);
    }
  }
  f32x16 acc0 = {}, acc1 = {};
#pragma unroll
  for (int i = 0; i < FC_KS_PER_WAVE; ++i) {
    if (i < nks) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb0[i], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb1[i], acc1, 0, 0, 0);
    }
  }
  // fixed-order sum of the 4 waves' tiles: rows = M (the C/D row map), cols = N
  float* rw = red[wave];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = (r & 3) + 8 * (r >> 2) + 4 * h;
    rw[m * 65 + r32] = acc0[r];
    rw[m * 65 + 32 + r32] = acc1[r];
  }
  __syncthreads();
  // 32 x 64 outputs / 256 threads = 8 per thread: row = t / 8, 8 consecutive columns
  const int orow = threadIdx.x >> 3, oc = (threadIdx.x & 7) * 8;
  const int grow = mtile * 32 + orow;
  if (grow < B) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = orow * 65 + oc + j;
      v[j] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
    }
    float4* dst = reinterpret_cast<float4*>(part + ((size_t)split * B + grow) * FC_N + ntile * 64 + oc);
    dst[0] = make_float4(v[0], v[1], v[2], v[3]);
    dst[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

void fc1_fwd_multi(const FcSet& set, hipStream_t s) {
  if (set.B <= 0) return;
  if (set.n < 1 || set.n > kMaxProbs) throw std::invalid_argument("fc1_fwd: 1..3 problems");
  const dim3 grid(set.n * ((set.B + 31) / 32), FC_N / 64, FC_KSPLIT);
  fc1_fwd_k<<<grid, 256, 0, s>>>(set);
  LAUNCH_CHECK();
}

void fc1_fwd(const uint16_t* a, const uint16_t* w, float* part, int B, hipStream_t s) {
  FcSet set{};
  set.p[0] = FcProb{a, w, part};
  set.n = 1;
  set.B = B;
  fc1_fwd_multi(set, s);
}

}  // namespace apex
