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

// ====================================================================== FC1 backward
// One launch, two workgroup roles (dL/dz = dz [B][256] bf16 from dqn_heads_bwd):
//
//  * dX (blocks [0, DXB)): da3 = dz . W, K = 256 -- both operands K-contiguous (dz rows,
//    W^T rows of the packed wfc1t [3136][256]), so fragments are plain 16-byte loads;
//    the ReLU backward of conv3 (a3 > 0) and the bf16 cast are fused into the coalesced
//    tile epilogue, writing dy3 (what wgrad3 / dgrad3 read) directly;
//  * dW (blocks [DXB, ...)): dW[n][k] = sum_b dz[b][n] a3[b][k] -- the reduction runs over
//    rows of both operands, so a batch slice of dz and a3 is staged in LDS and both
//    fragments are gathered with ds_read_b64_tr_b16 (padded pitches: conflict free per
//    32-lane half); each workgroup writes an fp32 partial slab [G][256][3136] in natural
//    (p, c) column order and grad_finalize reduces the G slabs and scatters them into the
//    reference [n][c*49+p] layout (FC1 is a 7x7 "conv" over a3's 7x7x64).
// Replaces two hipBLASLt GEMMs + the unpack and ReLU-mask kernels (four launches).
namespace {
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 tr_read4(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(__attribute__((address_space(3))) char*)p);
}
constexpr int FB_DX_TM = 128, FB_DX_TN = 64;      // dX workgroup tile (4 waves x 32 rows, 2 N tiles)
constexpr int FB_DW_TN = 128, FB_DW_TK = 64;      // dW workgroup tile: 128 n x 64 k
constexpr int FB_G = 2;                           // batch slices of the dW reduction
constexpr int FB_DZ_PITCH = FB_DW_TN * 2 + 64;    // 320 B: tr-read rows 16 banks apart
constexpr int FB_A3_PITCH = FB_DW_TK * 2 + 64;    // 192 B
constexpr int FB_MAXB = 256;                      // batch rows per dW slice held in LDS
constexpr int FB_LDS = FB_MAXB * (FB_DZ_PITCH + FB_A3_PITCH);  // 128 KB
}  // namespace

int fc1_bwd_slices() { return FB_G; }

__global__ __launch_bounds__(256) void fc1_bwd_k(const uint16_t* __restrict__ dz, const uint16_t* __restrict__ a3,
                                                 const uint16_t* __restrict__ wt, uint16_t* __restrict__ dy3,
                                                 float* __restrict__ part, int B, int dxb) {
  __shared__ __attribute__((aligned(16))) char smem[FB_LDS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  if ((int)blockIdx.x < dxb) {
    // ---------------------------------------------------------------- dX role
    const int NB = FC_K / FB_DX_TN;  // 49
    const int mb = blockIdx.x / NB, nb = blockIdx.x % NB;
    const int row = mb * FB_DX_TM + wave * 32 + r32;
    const int rowc = row < B ? row : B - 1;
    const bf16x8* ar = reinterpret_cast<const bf16x8*>(dz + (size_t)rowc * FC_N + 8 * h);
    const bf16x8* br0 = reinterpret_cast<const bf16x8*>(wt + (size_t)(nb * FB_DX_TN + r32) * FC_N + 8 * h);
    const bf16x8* br1 = reinterpret_cast<const bf16x8*>(wt + (size_t)(nb * FB_DX_TN + 32 + r32) * FC_N + 8 * h);
    bf16x8 fa[16], fb0[16], fb1[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      fa[i] = ar[2 * i];
      fb0[i] = br0[2 * i];
      fb1[i] = br1[2 * i];
    }
    f32x16 acc0 = {}, acc1 = {};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb0[i], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb1[i], acc1, 0, 0, 0);
    }
    char* ep = smem + wave * TILE_EP_BYTES;
    const int rbase = mb * FB_DX_TM + wave * 32;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const long col0 = (long)nb * FB_DX_TN + 32 * t;
      tile_store_bf16(t ? acc1 : acc0, ep, [](int, int, float v) { return f2bf(v); },
                      [&](int r) -> long { return rbase + r < B ? (long)(rbase + r) * FC_K + col0 : -1; }, dy3,
                      a3);
    }
    return;
  }
  // ---------------------------------------------------------------- dW role
  const int blk = blockIdx.x - dxb;
  const int KB = FC_K / FB_DW_TK;  // 49
  const int g = blk / (2 * KB), rem = blk % (2 * KB), nbk = rem / KB, kb = rem % KB;
  const int rows = (B + FB_G - 1) / FB_G, b0 = g * rows, nrows = min(rows, B - b0);
  char* dzs = smem;
  char* a3s = smem + FB_MAXB * FB_DZ_PITCH;
  // stage dz[b0 .. +256][nbk*128 .. +128] and a3[b0 .. +256][kb*64 .. +64] in 16-B chunks,
  // every load of the thread issued before the first LDS store (rows past nrows are zero)
  const int nr16 = (nrows + 15) & ~15;
  {
    constexpr int DZC = FB_MAXB * 16 / 256, A3C = FB_MAXB * 8 / 256;  // 16 + 8 chunks per thread
    u32v4 vd[DZC], va[A3C];
#pragma unroll
    for (int j = 0; j < DZC; ++j) {
      const int q = threadIdx.x + 256 * j, r = q >> 4, c = q & 15;
      const int rr = r < nrows ? r : nrows - 1;
      vd[j] = *reinterpret_cast<const u32v4*>(dz + (size_t)(b0 + rr) * FC_N + nbk * FB_DW_TN + c * 8);
    }
#pragma unroll
    for (int j = 0; j < A3C; ++j) {
      const int q = threadIdx.x + 256 * j, r = q >> 3, c = q & 7;
      const int rr = r < nrows ? r : nrows - 1;
      va[j] = *reinterpret_cast<const u32v4*>(a3 + (size_t)(b0 + rr) * FC_K + kb * FB_DW_TK + c * 8);
    }
#pragma unroll
    for (int j = 0; j < DZC; ++j) {
      const int q = threadIdx.x + 256 * j, r = q >> 4, c = q & 15;
      if (r < nr16) *reinterpret_cast<u32v4*>(dzs + r * FB_DZ_PITCH + c * 16) = r < nrows ? vd[j] : u32v4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < A3C; ++j) {
      const int q = threadIdx.x + 256 * j, r = q >> 3, c = q & 7;
      if (r < nr16) *reinterpret_cast<u32v4*>(a3s + r * FB_A3_PITCH + c * 16) = r < nrows ? va[j] : u32v4{0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();
  // wave (wn, wk): n tiles 2 wn, 2 wn + 1 (of 4), k tile wk (of 2)
  const int wn = wave >> 1, wk = wave & 1;
  const int q4 = (lane & 15) >> 2, p4 = lane & 3, grp = (lane >> 4) & 1;
  const int colsel = 16 * grp + 4 * p4;
  f32x16 acc0 = {}, acc1 = {};
  for (int s = 0; s < nr16 / 16; ++s) {
    const int r0 = 16 * s + 8 * h + q4;
    const char* d0 = dzs + r0 * FB_DZ_PITCH + (64 * wn + colsel) * 2;
    const char* x0 = a3s + r0 * FB_A3_PITCH + (32 * wk + colsel) * 2;
    const bf16x4 al0 = tr_read4(d0), ah0 = tr_read4(d0 + 4 * FB_DZ_PITCH);
    const bf16x4 al1 = tr_read4(d0 + 64), ah1 = tr_read4(d0 + 64 + 4 * FB_DZ_PITCH);
    const bf16x4 bl = tr_read4(x0), bh = tr_read4(x0 + 4 * FB_A3_PITCH);
    const bf16x8 fa0{al0[0], al0[1], al0[2], al0[3], ah0[0], ah0[1], ah0[2], ah0[3]};
    const bf16x8 fa1{al1[0], al1[1], al1[2], al1[3], ah1[0], ah1[1], ah1[2], ah1[3]};
    const bf16x8 fb{bl[0], bl[1], bl[2], bl[3], bh[0], bh[1], bh[2], bh[3]};
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, fb, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, fb, acc1, 0, 0, 0);
  }
  // partial slab g: [256][3136], rows n = C/D row map, columns k = lane
  float* dst = part + (size_t)g * FC_N * FC_K;
  const int ncol = kb * FB_DW_TK + 32 * wk + r32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = (r & 3) + 8 * (r >> 2) + 4 * h;
    dst[(size_t)(nbk * FB_DW_TN + 64 * wn + m) * FC_K + ncol] = acc0[r];
    dst[(size_t)(nbk * FB_DW_TN + 64 * wn + 32 + m) * FC_K + ncol] = acc1[r];
  }
}

void fc1_bwd(const uint16_t* dz, const uint16_t* a3, const uint16_t* wt, uint16_t* dy3, float* part, int B,
             hipStream_t s) {
  if (B <= 0) return;
  if ((B + FB_G - 1) / FB_G > FB_MAXB) throw std::invalid_argument("fc1_bwd: batch <= 512");
  const int dxb = ((B + FB_DX_TM - 1) / FB_DX_TM) * (FC_K / FB_DX_TN);
  const int dwb = FB_G * 2 * (FC_K / FB_DW_TK);
  fc1_bwd_k<<<dxb + dwb, 256, 0, s>>>(dz, a3, wt, dy3, part, B, dxb);
  LAUNCH_CHECK();
}

size_t fc1_bwd_workspace_floats() { return (size_t)FB_G * FC_N * FC_K; }

}  // namespace apex
