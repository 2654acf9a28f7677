// Pre-split exact ("px") forward GEMMs of the reference-precision network on bf16 MFMA (gfx950).
//
// The reference computes in fp32 (origin_repo/learner.py:139-145).  gfx950's fp32 MFMA
// (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate, so an fp32 GEMM costs 512 MFMA
// cycles per 32x32x16 block.  Writing every fp32 operand element as three bf16 terms,
// x = h + m + l (RNE split, common.h split3_rne: h = bf16(x), m = bf16(x - h),
// l = bf16(x - h - m), exact), the product of two elements is
//
//     x y = hh' + (hm' + mh') + (mm' + hl' + lh') + (ml' + lm' + ll')
//
// with |m| <= 2^-8 |x| and |l| <= 2^-16 |x|: the last group is <= 2^-23 |x y| (one fp32
// rounding of the product is 2^-24), so the first six terms -- each bf16 x bf16 product
// exact in fp32 -- carry fp32 accuracy.  They cost 6 x 32 = 192 MFMA cycles per 32x32x16
// (v_mfma_f32_32x32x16_bf16) instead of 512: 2.7x fewer.  The hh' term is accumulated
// alone and the five smaller ones in a second accumulator (added once at the end), so the
// small terms never round against the large running sum.  Knob (19, 2) adds ml' + lm' (8
// products, 256 cycles): only ll' (<= 2^-32 |x y|) is dropped, so the per-product
// representation error falls far below one fp32 rounding (MI355X, 6 terms: layer errors
// 2-3.5x the fp32-MFMA body's; learner step-0 parity 2.0e-4 vs 7.8e-5 of the update length).
//
// The round-2 attempt split both operands while staging them into LDS (gemm_x9_k in
// f32_kernels.hip): ~5.5 VALU per element ate the MFMA savings.  Here nothing is split in
// the GEMM: the PRODUCERS write planes -- the optimizer writes the packed weights' planes in
// its update pass (learner_kernels.hip PackMap.arena_x / FcPack.wp_x), each forward layer's
// epilogue writes its activation planes beside the fp32 activation (conv1 -> a1x, conv2 ->
// a2x, conv3 -> a3x) -- and the loaders move 16-byte chunks of 8 bf16 straight into LDS.
//
// Body: 64 x 64 tiles (whole N for conv2 / conv3), BK = 32, 4 waves in a 2 x 2 grid of
// 32 x 32 wave tiles; LDS holds [3 planes][64 rows][BK + 8] bf16 per operand (pitch 80 B:
// conflict-free ds_read_b128 fragment reads), double buffered = 60 KB (2 workgroups per CU);
// one register prefetch of the next k-block, one barrier per k-block.  Per 16-k step a wave
// issues 6 ds_read_b128 and 6 MFMAs.  The fp32 output (for the backward) and its planes (for
// the next layer) are stored by the same epilogue.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace apex {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ F32Prob pick_px(const F32Set& s, int i) {
  return i == 0 ? s.p[0] : (i == 1 ? s.p[1] : s.p[2]);
}
// XCD-chunked tile order (see f32_kernels.hip xcd_chunk): XCD j walks a contiguous range
__device__ __forceinline__ int xcd_chunk_px(int b, int G) {
  const int G8 = G & ~7;
  return b >= G8 ? b : (b & 7) * (G8 >> 3) + (b >> 3);
}

template <class P>
struct GeoPx {
  static constexpr int BM = P::BM, BN = P::BN, BK = P::BK, WM = P::WM, WN = 4 / P::WM;
  static constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static constexpr int PITCH = BK + 8;                    // bf16 per LDS row
  static constexpr int SA = BM * PITCH, SB = BN * PITCH;  // one plane
  static constexpr int STAGE = 3 * (SA + SB);
  static constexpr int LDS_HALVES = 2 * STAGE;
  static constexpr int RA = BK / 8;                       // 16-byte chunks per row
  static constexpr int CA = BM * RA, CB = BN * RA;
  static constexpr int NA = (CA + 255) / 256, NB = (CB + 255) / 256;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves of 32 x 32 blocks");
  static_assert(BK % 16 == 0, "k-steps of 16");
};

template <class P, int NTERM, int PIPE>
__device__ __forceinline__ void gemm_body_px(const F32Set& args, int block, uint16_t* lds) {
  static_assert(NTERM == 6 || NTERM == 8, "6 or 8 term products");
  using G = GeoPx<P>;
  typename P::Ctx ctx;
  P::decode(args, block, ctx);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave % G::WM, wn = wave / G::WM;
  const int r = lane & 31, h = lane >> 5;
  const int64_t psa = ctx.p.inx_ps, psb = ctx.p.wx_ps;
  f32x16 acc[G::TM][G::TN], acc2[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = acc2[i][j][e] = 0.f;
  const uint16_t* rowa[G::NA];
  const uint16_t* rowb[G::NB];
#pragma unroll
  for (int j = 0; j < G::NA; ++j) {
    const int q = min(t + 256 * j, G::CA - 1);
    rowa[j] = P::row_a(ctx, q / G::RA, q % G::RA);
  }
#pragma unroll
  for (int j = 0; j < G::NB; ++j) {
    const int q = min(t + 256 * j, G::CB - 1);
    rowb[j] = P::row_b(ctx, q / G::RA, q % G::RA);
  }
  uint4 ra0[G::NA][3], rb0[G::NB][3], ra1[G::NA][3], rb1[G::NB][3];
  auto gload = [&](int kb, uint4 (&ra)[G::NA][3], uint4 (&rb)[G::NB][3]) {
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      if (G::CA % 256 == 0 || t + 256 * j < G::CA) {
        const uint16_t* a = rowa[j] ? rowa[j] + P::koff_a(kb) : nullptr;
#pragma unroll
        for (int u = 0; u < 3; ++u) ra[j][u] = a ? *reinterpret_cast<const uint4*>(a + u * psa) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      if (G::CB % 256 == 0 || t + 256 * j < G::CB) {
        const uint16_t* b = rowb[j] + P::koff_b(kb);
#pragma unroll
        for (int u = 0; u < 3; ++u) rb[j][u] = *reinterpret_cast<const uint4*>(b + u * psb);
      }
    }
  };
  auto sstore = [&](int buf, const uint4 (&ra)[G::NA][3], const uint4 (&rb)[G::NB][3]) {
    uint16_t* As = lds + buf * G::STAGE;
    uint16_t* Bs = As + 3 * G::SA;
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      const int q = t + 256 * j;
      if (G::CA % 256 == 0 || q < G::CA) {
        uint16_t* d = As + (q / G::RA) * G::PITCH + 8 * (q % G::RA);
#pragma unroll
        for (int u = 0; u < 3; ++u) *reinterpret_cast<uint4*>(d + u * G::SA) = ra[j][u];
      }
    }
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      const int q = t + 256 * j;
      if (G::CB % 256 == 0 || q < G::CB) {
        uint16_t* d = Bs + (q / G::RA) * G::PITCH + 8 * (q % G::RA);
#pragma unroll
        for (int u = 0; u < 3; ++u) *reinterpret_cast<uint4*>(d + u * G::SB) = rb[j][u];
      }
    }
  };
  auto compute = [&](int buf) {
    const uint16_t* As = lds + buf * G::STAGE;
    const uint16_t* Bs = As + 3 * G::SA;
#pragma unroll
    for (int kc = 0; kc < G::BK / 16; ++kc) {
      bfx8 a[G::TM][3], b[G::TN][3];
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi) {
        const uint16_t* ap = As + (wm * G::WTM + mi * 32 + r) * G::PITCH + kc * 16 + 8 * h;
#pragma unroll
        for (int u = 0; u < 3; ++u) a[mi][u] = *reinterpret_cast<const bfx8*>(ap + u * G::SA);
      }
#pragma unroll
      for (int ni = 0; ni < G::TN; ++ni) {
        const uint16_t* bp = Bs + (wn * G::WTN + ni * 32 + r) * G::PITCH + kc * 16 + 8 * h;
#pragma unroll
        for (int u = 0; u < 3; ++u) b[ni][u] = *reinterpret_cast<const bfx8*>(bp + u * G::SB);
      }
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < G::TN; ++ni) {
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][0], b[ni][0], acc[mi][ni], 0, 0, 0);
          f32x16 c2 = acc2[mi][ni];
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][0], b[ni][1], c2, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][1], b[ni][0], c2, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][1], b[ni][1], c2, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][0], b[ni][2], c2, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][2], b[ni][0], c2, 0, 0, 0);
          if constexpr (NTERM == 8) {  // the 2^-24 terms too: only ll' (2^-32) is dropped
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][1], b[ni][2], c2, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][2], b[ni][1], c2, 0, 0, 0);
          }
          acc2[mi][ni] = c2;
        }
    }
  };
  if constexpr (PIPE == 0) {  // two LDS stages, the next k-block prefetched in registers
    int kb = ctx.kb0, cur = 0;
    if (kb < ctx.kb1) {
      gload(kb, ra0, rb0);
      sstore(0, ra0, rb0);
    }
    __syncthreads();
    for (; kb < ctx.kb1; ++kb) {
      const bool more = kb + 1 < ctx.kb1;
      if (more) gload(kb + 1, ra0, rb0);
      __builtin_amdgcn_sched_barrier(0);
      compute(cur);
      if (more) sstore(cur ^ 1, ra0, rb0);
      __syncthreads();
      cur ^= 1;
    }
  } else {  // one LDS stage (4 workgroups per CU), k-blocks kb+1 and kb+2 in flight in registers
    int kb = ctx.kb0;
    if (kb < ctx.kb1) gload(kb, ra0, rb0);
    if (kb + 1 < ctx.kb1) gload(kb + 1, ra1, rb1);
    for (; kb < ctx.kb1; kb += 2) {
      __syncthreads();  // every wave is done reading the stage
      sstore(0, ra0, rb0);
      __syncthreads();
      if (kb + 2 < ctx.kb1) gload(kb + 2, ra0, rb0);
      compute(0);
      if (kb + 1 >= ctx.kb1) break;
      __syncthreads();
      sstore(0, ra1, rb1);
      __syncthreads();
      if (kb + 3 < ctx.kb1) gload(kb + 3, ra1, rb1);
      compute(0);
    }
  }
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * h;  // 32x32 MFMA C/D layout
        P::store(ctx, wm * G::WTM + mi * 32 + row, wn * G::WTN + ni * 32 + r, acc[mi][ni][e] + acc2[mi][ni][e]);
      }
}

template <class P, int NTERM>
__global__ __launch_bounds__(256, 2) void gemm_px_k(F32Set args, int remap) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[GeoPx<P>::LDS_HALVES];
  gemm_body_px<P, NTERM, 0>(args, remap ? xcd_chunk_px(blockIdx.x, gridDim.x) : blockIdx.x, lds);
}
// PIPE 1: one LDS stage + a 2-deep register ring (MI355X, conv2 forward: the 2-stage form ran
// at 19 % MFMA busy with 2 workgroups per CU -- each k-block's loads waited ~1 us of memory
// latency behind ~450 MFMA cycles; 4 resident workgroups x 2 k-blocks in flight hide it)
template <class P, int NTERM>
__global__ __launch_bounds__(256, 3) void gemm_px1_k(F32Set args, int remap) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[GeoPx<P>::STAGE];
  gemm_body_px<P, NTERM, 1>(args, remap ? xcd_chunk_px(blockIdx.x, gridDim.x) : blockIdx.x, lds);
}

// ------------------------------------------------------------------ policies
// conv2: a2[m][n] = relu(sum_k a1(m, k) w2p[n][k] + b2[n]), m = (b, oy, ox) of 9 x 9,
// k = tap * 32 + ci (tap = ky * 4 + kx), a1 channels-last [B][20][20][32]
template <int BM_, int BN_, int BK_, int WM_>
struct Conv2FwdX {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  // a k-block lies inside one tap, or (BK = 64) covers taps (ky, 2j) and (ky, 2j + 1): adjacent
  // pixels, so one k-block row is 64 contiguous channels -- a full 128-byte line per plane
  static_assert((32 % BK == 0 || BK == 64) && BN <= 64, "k-block within one tap or one even tap pair");
  static constexpr int NT = 64 / BN;
  struct Ctx {
    F32Prob p;
    int M, m0, n0, kb0, kb1;
  };
  static __host__ __device__ int tiles(int B) { return NT * ((B * 81 + BM - 1) / BM); }
  static __device__ void decode(const F32Set& a, int block, Ctx& c) {
    const int tp = tiles(a.B);
    c.p = pick_px(a, block / tp);
    c.M = a.B * 81;
    const int t = block % tp;
    c.m0 = (t / NT) * BM;
    c.n0 = (t % NT) * BN;
    c.kb0 = 0;
    c.kb1 = 512 / BK;
  }
  static __device__ const uint16_t* row_a(const Ctx& c, int row, int ch) {
    const int m = c.m0 + row;
    if (m >= c.M) return nullptr;
    const int b = m / 81, p = m - b * 81, oy = p / 9, ox = p - oy * 9;
    return c.p.inx + ((size_t)b * 400 + 2 * oy * 20 + 2 * ox) * 32 + 8 * ch;
  }
  static __device__ int koff_a(int kb) {
    const int k0 = kb * BK, tap = k0 >> 5;  // wave-uniform
    return ((tap >> 2) * 20 + (tap & 3)) * 32 + (k0 & 31);
  }
  static __device__ const uint16_t* row_b(const Ctx& c, int n, int ch) { return c.p.wx + (c.n0 + n) * 512 + 8 * ch; }
  static __device__ int koff_b(int kb) { return kb * BK; }
  static __device__ void store(const Ctx& c, int ml, int n, float v) {
    const int m = c.m0 + ml;
    if (m >= c.M) return;
    const size_t i = (size_t)m * 64 + c.n0 + n;
    const float y = fmaxf(v + c.p.bias[c.n0 + n], 0.f);
    c.p.out[i] = y;
    if (c.p.outx) store_planes(c.p.outx, c.p.outx_ps, i, y);
  }
};

// conv3: a3 = relu(conv(a2, W3) + b3), m = (b, oy, ox) of 7 x 7, k = tap * 64 + ci, a2 [B][9][9][64]
template <int BM_, int BN_, int BK_, int WM_>
struct Conv3FwdX {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  static_assert(64 % BK == 0 && BN <= 64, "a k-block lies inside one tap");
  static constexpr int NT = 64 / BN;
  struct Ctx {
    F32Prob p;
    int M, m0, n0, kb0, kb1;
  };
  static __host__ __device__ int tiles(int B) { return NT * ((B * 49 + BM - 1) / BM); }
  static __device__ void decode(const F32Set& a, int block, Ctx& c) {
    const int tp = tiles(a.B);
    c.p = pick_px(a, block / tp);
    c.M = a.B * 49;
    const int t = block % tp;
    c.m0 = (t / NT) * BM;
    c.n0 = (t % NT) * BN;
    c.kb0 = 0;
    c.kb1 = 576 / BK;
  }
  static __device__ const uint16_t* row_a(const Ctx& c, int row, int ch) {
    const int m = c.m0 + row;
    if (m >= c.M) return nullptr;
    const int b = m / 49, p = m - b * 49, oy = p / 7, ox = p - oy * 7;
    return c.p.inx + ((size_t)b * 81 + oy * 9 + ox) * 64 + 8 * ch;
  }
  static __device__ int koff_a(int kb) {
    const int k0 = kb * BK, tap = k0 >> 6, ky = tap / 3, kx = tap - ky * 3;  // wave-uniform
    return (ky * 9 + kx) * 64 + (k0 & 63);
  }
  static __device__ const uint16_t* row_b(const Ctx& c, int n, int ch) { return c.p.wx + (c.n0 + n) * 576 + 8 * ch; }
  static __device__ int koff_b(int kb) { return kb * BK; }
  static __device__ void store(const Ctx& c, int ml, int n, float v) {
    const int m = c.m0 + ml;
    if (m >= c.M) return;
    const size_t i = (size_t)m * 64 + c.n0 + n;
    const float y = fmaxf(v + c.p.bias[c.n0 + n], 0.f);
    c.p.out[i] = y;
    if (c.p.outx) store_planes(c.p.outx, c.p.outx_ps, i, y);
  }
};

// FC1 (both dueling heads fused, N = 256), split-K into 7 slabs of 448:
// z[s][b][n] = sum_{k in slab s} a3[b][k] wfc1p[n][k], k = p * 64 + c
constexpr int kPxFcSplits = 7;
template <int BM_, int BN_, int BK_, int WM_>
struct Fc1FwdX {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  static constexpr int KBS = 3136 / BK / kPxFcSplits;
  static_assert(KBS * BK * kPxFcSplits == 3136 && 256 % BN == 0, "split-K tiling");
  static constexpr int NT = 256 / BN;
  struct Ctx {
    F32Prob p;
    int B, m0, n0, split, kb0, kb1;
  };
  static __host__ __device__ int tiles(int B) { return ((B + BM - 1) / BM) * NT * kPxFcSplits; }
  static __device__ void decode(const F32Set& a, int block, Ctx& c) {
    const int tp = tiles(a.B);
    c.p = pick_px(a, block / tp);
    int t = block % tp;
    c.B = a.B;
    c.n0 = (t % NT) * BN;
    t /= NT;
    c.split = t % kPxFcSplits;
    c.m0 = (t / kPxFcSplits) * BM;
    c.kb0 = c.split * KBS;
    c.kb1 = c.kb0 + KBS;
  }
  static __device__ const uint16_t* row_a(const Ctx& c, int row, int ch) {
    const int b = c.m0 + row;
    return b < c.B ? c.p.inx + (size_t)b * 3136 + 8 * ch : nullptr;
  }
  static __device__ int koff_a(int kb) { return kb * BK; }
  static __device__ const uint16_t* row_b(const Ctx& c, int n, int ch) {
    return c.p.wx + (size_t)(c.n0 + n) * 3136 + 8 * ch;
  }
  static __device__ int koff_b(int kb) { return kb * BK; }
  static __device__ void store(const Ctx& c, int ml, int nl, float v) {
    const int b = c.m0 + ml;
    if (b < c.B) c.p.out[((size_t)c.split * c.B + b) * 256 + c.n0 + nl] = v;
  }
};

__global__ void split_planes_k(const float* __restrict__ src, uint16_t* __restrict__ dst, int64_t n, int64_t ps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    store_planes(dst, ps, i, src[i]);
}

int g_px = 0;     // f32_set_variant(19, 0|1|2): off | 6 term products | 8 term products
int g_px_xcd = 1;
int g_px_bk = 32;   // f32_set_variant(22, 32|64): k-block depth (64: 128-byte plane rows = full lines)
int g_px_pipe = 0;  // f32_set_variant(21, 0|1): pipeline form of the px / pxb bodies (see gemm_px1_k; 1 measured slower)

template <class P>
void px_launch(const F32Set& set, hipStream_t s) {
  const int blocks = set.n * P::tiles(set.B);
  if (blocks <= 0) return;
  if (g_px_pipe == 1) {
    if (g_px == 2) gemm_px1_k<P, 8><<<blocks, 256, 0, s>>>(set, g_px_xcd);
    else gemm_px1_k<P, 6><<<blocks, 256, 0, s>>>(set, g_px_xcd);
  } else {
    if (g_px == 2) gemm_px_k<P, 8><<<blocks, 256, 0, s>>>(set, g_px_xcd);
    else gemm_px_k<P, 6><<<blocks, 256, 0, s>>>(set, g_px_xcd);
  }
  LAUNCH_CHECK();
}

void check_px(const F32Set& set) {
  if (set.n < 1 || set.n > kMaxProbs || set.B <= 0) throw std::invalid_argument("px: 1..3 problems, B > 0");
  for (int i = 0; i < set.n; ++i) {
    const F32Prob& p = set.p[i];
    if (!p.inx || !p.wx || !p.out || p.inx_ps <= 0 || p.wx_ps <= 0 || (p.outx && p.outx_ps <= 0))
      throw std::invalid_argument("px: every problem needs input / weight planes with positive plane strides");
    if ((reinterpret_cast<uintptr_t>(p.inx) | reinterpret_cast<uintptr_t>(p.wx)) & 15 || (p.inx_ps | p.wx_ps) & 7)
      throw std::invalid_argument("px: planes must be 16-byte aligned");
  }
}

}  // namespace

bool px_enabled() { return g_px != 0; }

int px_terms() { return g_px == 2 ? 8 : 6; }

int px_pipe() { return g_px_pipe; }

void px_set_pipe(int v) { g_px_pipe = v; }

void px_set_bk(int v) { g_px_bk = v; }

void px_set(int v) { g_px = v; }

void px_conv_fwd_multi(int layer, const F32Set& set, hipStream_t s) {
  check_px(set);
  if (g_px_bk == 64) {
    if (layer == 2) px_launch<Conv2FwdX<64, 64, 64, 2>>(set, s);
    else if (layer == 3) px_launch<Conv3FwdX<64, 64, 64, 2>>(set, s);
    else throw std::invalid_argument("px_conv_fwd_multi: layer 2 or 3");
    return;
  }
  if (layer == 2) px_launch<Conv2FwdX<64, 64, 32, 2>>(set, s);
  else if (layer == 3) px_launch<Conv3FwdX<64, 64, 32, 2>>(set, s);
  else throw std::invalid_argument("px_conv_fwd_multi: layer 2 or 3");
}

void px_fc1_fwd_multi(const F32Set& set, hipStream_t s) {
  check_px(set);
  if (g_px_bk == 64) px_launch<Fc1FwdX<64, 64, 64, 2>>(set, s);
  else px_launch<Fc1FwdX<64, 64, 32, 2>>(set, s);
}

void f32_split_planes(const float* src, uint16_t* dst, int64_t n, int64_t plane, hipStream_t s) {
  if (n <= 0) return;
  if (plane < n) throw std::invalid_argument("f32_split_planes: plane stride < n");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  split_planes_k<<<blocks, 256, 0, s>>>(src, dst, n, plane);
  LAUNCH_CHECK();
}

}  // namespace apex
