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
//    rows of both operands, so 128-row batch chunks of dz and a3 are staged in LDS and both
//    fragments are gathered with ds_read_b64_tr_b16 (padded pitches: conflict free per
//    32-lane half; the next chunk is prefetched into registers); each workgroup owns a
//    complete 64 x 64 tile (no split-K slabs, 48 KB LDS: 3 workgroups per CU), written
//    in natural (p, c) column order; grad_finalize's row-transpose job scatters it into the
//    reference [n][c*49+p] layout through LDS (coalesced both ways).
// Replaces two hipBLASLt GEMMs + the unpack and ReLU-mask kernels (four launches).
namespace {
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 tr_read4(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(__attribute__((address_space(3))) char*)p);
}
constexpr int FB_DX_TM = 128, FB_DX_TN = 64;      // dX workgroup tile (4 waves x 32 rows, 2 N tiles)
constexpr int FB_DW_TN = 64, FB_DW_TK = 64;       // dW workgroup tile: 64 n x 64 k (one 32x32 per wave)
constexpr int FB_PITCH = 64 * 2 + 64;             // 192 B LDS rows: tr-read rows 16 banks apart
constexpr int FB_CH = 128;                        // batch rows per LDS chunk
constexpr int FB_LDS = 2 * FB_CH * FB_PITCH;      // dz + a3 chunk = 48 KB (3 workgroups per CU)
}  // namespace

int fc1_bwd_slices() { return 1; }  // dW is complete per workgroup (one slab)

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
  const int nbk = blk / KB, kb = blk % KB;
  char* dzs = smem;
  char* a3s = smem + FB_CH * FB_PITCH;
  const int wn = wave >> 1, wk = wave & 1;  // the wave's 32 x 32 tile
  const int q4 = (lane & 15) >> 2, p4 = lane & 3, grp = (lane >> 4) & 1;
  const int colsel = 16 * grp + 4 * p4;
  f32x16 acc = {};
  // the whole batch in 128-row chunks through LDS; the next chunk's loads are in flight
  // (registers) while the current one is multiplied.  Thread t moves 16-byte chunk
  // q = t + 256 j (j < 4) of each operand: row q >> 3, column chunk q & 7.
  u32v4 vd[4], va[4];
  auto load = [&](int b0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = threadIdx.x + 256 * j, r = q >> 3, c = q & 7;
      const int rr = min(b0 + r, B - 1);
      vd[j] = *reinterpret_cast<const u32v4*>(dz + (size_t)rr * FC_N + nbk * FB_DW_TN + c * 8);
      va[j] = *reinterpret_cast<const u32v4*>(a3 + (size_t)rr * FC_K + kb * FB_DW_TK + c * 8);
    }
  };
  load(0);
  for (int b0 = 0; b0 < B; b0 += FB_CH) {
    const int nrows = min(FB_CH, B - b0), nr16 = (nrows + 15) & ~15;
    if (b0) __syncthreads();  // the previous chunk's fragment reads are done
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = threadIdx.x + 256 * j, r = q >> 3, c = q & 7;
      const u32v4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u32v4*>(dzs + r * FB_PITCH + c * 16) = r < nrows ? vd[j] : z;
      *reinterpret_cast<u32v4*>(a3s + r * FB_PITCH + c * 16) = r < nrows ? va[j] : z;
    }
    __syncthreads();
    if (b0 + FB_CH < B) load(b0 + FB_CH);
    for (int s = 0; s < nr16 / 16; ++s) {
      const int r0 = 16 * s + 8 * h + q4;
      const char* d0 = dzs + r0 * FB_PITCH + (32 * wn + colsel) * 2;
      const char* x0 = a3s + r0 * FB_PITCH + (32 * wk + colsel) * 2;
      const bf16x4 al = tr_read4(d0), ah = tr_read4(d0 + 4 * FB_PITCH);
      const bf16x4 bl = tr_read4(x0), bh = tr_read4(x0 + 4 * FB_PITCH);
      const bf16x8 fa{al[0], al[1], al[2], al[3], ah[0], ah[1], ah[2], ah[3]};
      const bf16x8 fb{bl[0], bl[1], bl[2], bl[3], bh[0], bh[1], bh[2], bh[3]};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
    }
  }
  // dW [256][3136] in natural (p, c) column order: rows n = C/D row map, columns k = lane
  const int ncol = kb * FB_DW_TK + 32 * wk + r32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = (r & 3) + 8 * (r >> 2) + 4 * h;
    part[(size_t)(nbk * FB_DW_TN + 32 * wn + m) * FC_K + ncol] = acc[r];
  }
}

void fc1_bwd(const uint16_t* dz, const uint16_t* a3, const uint16_t* wt, uint16_t* dy3, float* part, int B,
             hipStream_t s) {
  if (B <= 0) return;
  const int dxb = ((B + FB_DX_TM - 1) / FB_DX_TM) * (FC_K / FB_DX_TN);
  const int dwb = (FC_N / FB_DW_TN) * (FC_K / FB_DW_TK);
  fc1_bwd_k<<<dxb + dwb, 256, 0, s>>>(dz, a3, wt, dy3, part, B, dxb);
  LAUNCH_CHECK();
}

size_t fc1_bwd_workspace_floats() { return (size_t)FC_N * FC_K; }

}  // namespace apex
