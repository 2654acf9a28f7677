// FC1 of the dueling heads (Linear 3136 -> 2 x 128, adv | value hidden) for gfx950.
//
// z[M][256] = a3[M][3136] . W[256][3136]^T is skinny (N = 256) with a long K; at the
// learner's M = 3 x 512 (one launch for Q(s), Q(s'), Q_target(s')) the limit is the
// per-CU L2 -> CU read rate (~70 GB/s per CU, MI355X_MICROARCH.md 'Indexed rows'), so
// the tiling minimises bytes per CU rather than maximising workgroups:
//
//   * workgroup = 128 rows x all 256 columns x one K slice (S slices, S adaptive so the
//     grid is ~170-250 workgroups); W bytes per CU = 256 x K/S x 2 -- the W slice is read
//     ONCE per workgroup into LDS (115 KB at S = 14), shared by the 4 waves, and each
//     wave streams its own 32 A rows straight into registers (all loads issued first);
//   * each wave computes 32 rows x 256 columns (8 accumulator tiles of
//     v_mfma_f32_32x32x16_bf16), writing its fp32 split-K partial slab [S][M][256];
//     heads_fwd sums the S slabs in fixed order (deterministic) before bias + ReLU.
//   * LDS W rows are padded by 16 B (464 / 240 B): 16 consecutive lanes' ds_read_b128 hit
//     16 distinct 4-bank groups (conflict free).
#include "common.h"
#include "kernels.h"

namespace apex {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int FC_K = 3136, FC_N = 256;
constexpr int FC_TM = 128;                       // rows per workgroup
}  // namespace

int fc1_splits() { return 28; }  // the most any launch uses (workspace sizing)

int fc1_splits_for(int total_rows) {
  // 196 k-steps split 14 ways (14 k-steps per slice) when that already gives ~160+
  // workgroups, else 28 ways (fewer bytes per CU, more partial slabs)
  const int mt = (total_rows + FC_TM - 1) / FC_TM;
  return mt * 14 >= 160 ? 14 : 28;
}

template <int KS>  // k-steps per slice
__global__ __launch_bounds__(256) void fc1_fwd_k(FcSet set) {
  constexpr int FC_WPITCH = KS * 32 + 16;  // LDS bytes per W row: 464 (KS 14) / 240 (KS 7)
  __shared__ __attribute__((aligned(16))) char wsm[FC_N * FC_WPITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  const int B = set.B, MT = (B + FC_TM - 1) / FC_TM;
  const int pb = blockIdx.x / MT, mtile = blockIdx.x - pb * MT, split = blockIdx.y;
  const uint16_t* __restrict__ a = set.p[pb].a;
  const uint16_t* __restrict__ w = set.p[pb].w;
  float* __restrict__ part = set.p[pb].part;
  const int k0 = split * KS * 16;
  // A fragments of this wave's 32 rows for the whole slice (row clamped; stores masked)
  const int row = mtile * FC_TM + wave * 32 + r32;
  const int rowc = row < B ? row : B - 1;
  const bf16x8* ar = reinterpret_cast<const bf16x8*>(a + (size_t)rowc * FC_K + k0 + 8 * h);
  bf16x8 fa[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) fa[i] = ar[2 * i];
  // W slice [256][KS*16] -> LDS in 16-byte chunks, loads issued in rounds of 7
  constexpr int CPR = KS * 2;        // 16-byte chunks per W row
  constexpr int TOTAL = FC_N * CPR;
  constexpr int PER = TOTAL / 256;
  static_assert(TOTAL % 256 == 0 && PER % 7 == 0, "W slice chunking");
#pragma unroll
  for (int r0 = 0; r0 < PER; r0 += 7) {
    u32v4 v[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int q = threadIdx.x + 256 * (r0 + j);
      const int n = q / CPR, c = q % CPR;
      v[j] = *reinterpret_cast<const u32v4*>(w + (size_t)n * FC_K + k0 + c * 8);
    }
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int q = threadIdx.x + 256 * (r0 + j);
      const int n = q / CPR, c = q % CPR;
      *reinterpret_cast<u32v4*>(wsm + n * FC_WPITCH + c * 16) = v[j];
    }
  }
  __syncthreads();
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    bf16x8 fb[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
      fb[t] = *reinterpret_cast<const bf16x8*>(wsm + (t * 32 + r32) * FC_WPITCH + i * 32 + h * 16);
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[t], acc[t], 0, 0, 0);
  }
  // partial slab rows (r&3)+8(r>>2)+4h of the wave's 32, column t*32 + r32
  const int rbase = mtile * FC_TM + wave * 32;
  float* dst = part + ((size_t)split * B + rbase) * FC_N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (rbase + m < B) {
#pragma unroll
      for (int t = 0; t < 8; ++t) dst[(size_t)m * FC_N + t * 32 + r32] = acc[t][r];
    }
  }
}

int fc1_fwd_multi(const FcSet& set, hipStream_t s) {
  if (set.B <= 0) return 0;
  if (set.n < 1 || set.n > kMaxProbs) throw std::invalid_argument("fc1_fwd: 1..3 problems");
  const int MT = (set.B + FC_TM - 1) / FC_TM;
  const int S = fc1_splits_for(set.n * set.B);
  const dim3 grid(set.n * MT, S);
  if (S == 14) {
    fc1_fwd_k<14><<<grid, 256, 0, s>>>(set);
  } else {
    fc1_fwd_k<7><<<grid, 256, 0, s>>>(set);
  }
  LAUNCH_CHECK();
  return S;
}

int fc1_fwd(const uint16_t* a, const uint16_t* w, float* part, int B, hipStream_t s) {
  FcSet set{};
  set.p[0] = FcProb{a, w, part};
  set.n = 1;
  set.B = B;
  return fc1_fwd_multi(set, s);
}

}  // namespace apex
