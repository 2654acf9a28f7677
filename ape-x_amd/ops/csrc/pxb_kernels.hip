// Pre-split exact ("px") BACKWARD GEMMs of the reference-precision network on bf16 MFMA (gfx950).
//
// Same arithmetic as the px forward (px_kernels.hip): every fp32 operand arrives as three exact
// bf16 planes x = h + m + l written by its producer, and each output is the fp32 sum of 6 (knob
// (19, 1)) or 8 (knob (19, 2)) exact bf16 x bf16 term products on v_mfma_f32_32x32x16_bf16, the
// big hh' term in its own accumulator.  Producers of the backward's planes:
//   dz   (FC1 pre-activation gradient)   dqn_heads_bwd_k         (loss_heads_kernels.hip)
//   dy3  (conv3 output gradient)         FC1 dgrad epilogue      (here)
//   dy2  (conv2 output gradient)         conv3 dgrad epilogue    (here)
//   a1 / a2 / a3                         forward epilogues        (px forward)
//   wfc1p / w3t / w2t                    optimizer pack pass      (learner_kernels.hip pack_store)
//
// The weight gradients reduce over the batch (FC1) or over (sample, position) rows (conv2 /
// conv3), i.e. over the ROW index of both stored operands.  Both are staged into LDS exactly as
// they lie in memory -- one 16-byte chunk of 8 channels per thread and plane, [k row][column] --
// and read as MFMA fragments with gfx950's hardware-transposing ds_read_b64_tr_b16 (T10 of the
// CDNA guide): lane 4q + p of each 16-lane group addresses row q, columns 4p .. 4p + 3 of a
// 4 x 16 block, and receives column (lane & 15) of the 4 rows.  Two reads give the 8 k values
// of a 32x32x16 operand fragment.  The transposed image's row pitch is 32 (mod 128) bf16 --
// 64 B (mod 256 B) -- so the 4 rows of a 32-lane half land on disjoint 16-bank quarters:
// conflict-free.  Row-read operands (the input gradients: k = (tap, channel) contiguous in both
// dy and the transposed weights) use the px forward's [row][BK + 8] image and ds_read_b128.
//
// One generic body (A and/or B transposed, optional row sums of A for the bias gradient via
// an extra MFMA against a ones fragment), policies per GEMM, and two-problem launches (weight
// gradient + input gradient of a layer, as the fp32 gemm2_k pairs them).  BK = 32, 4 waves of
// 32 x 32 wave tiles, double-buffered LDS, one register prefetch, one barrier per k-block.
#include <algorithm>
#include <string>

#include "common.h"
#include "kernels.h"

namespace apex {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

struct PxbArgs {
  const uint16_t* ax;  // A operand planes (plane stride a_ps elements)
  const uint16_t* bx;  // B operand planes
  const float* mask;   // input gradient: post-ReLU activation of the layer below (ReLU backward)
  float* out;          // input gradient (fp32) | weight-gradient partials
  float* out2;         // weight gradient: bias partials (conv) | value-head rows (FC1 in place)
  uint16_t* outx;      // input gradient planes (null: none)
  int64_t a_ps, b_ps, out_ps;
  int B, kbps, splits;
};

// smallest pitch >= c with pitch = 32 (mod 64) elements -- 64 or 192 B (mod 256 B): the 4 rows
// of a transposed read's 32-lane half start on 4 disjoint 16-bank quarters
constexpr int tr_pitch(int c) { return c % 64 == 32 ? c : c + 32 - c % 64 + (c % 64 > 32 ? 64 : 0); }
static_assert(tr_pitch(32) == 32 && tr_pitch(64) == 96 && tr_pitch(128) == 160, "transposed pitches");

template <class P>
struct GeoB {
  static constexpr int BM = P::BM, BN = P::BN, BK = 32, WM = P::WM, WN = 4 / P::WM;
  static constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static constexpr int RP = BK + 8;                              // row image pitch
  static constexpr int TPA = tr_pitch(BM), TPB = tr_pitch(BN);   // transposed image pitches
  static constexpr int SA = P::A_TR ? BK * TPA : BM * RP;        // one plane
  static constexpr int SB = P::B_TR ? BK * TPB : BN * RP;
  static constexpr int STAGE = 3 * (SA + SB);
  static constexpr int LDS = 2 * STAGE;
  static constexpr int CA = BM * BK / 8, CB = BN * BK / 8;      // 16-byte chunks per plane and k-block
  static constexpr int NA = (CA + 255) / 256, NB = (CB + 255) / 256;
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "4 waves of 32 x 32 blocks");
  static_assert(CA % 64 == 0 && CB % 64 == 0, "whole waves per chunk round");
};

__device__ __forceinline__ s16x4 ds_tr(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
// 32x32x16 operand fragment (lane: row / column l & 31, k = 8 (l >> 5) + j) of the block at
// (k step kc, column c0) of a transposed image [k][column] with pitch TP
template <int TP>
__device__ __forceinline__ bfx8 frag_tr(const uint16_t* img, int kc, int c0, int lane) {
  const uint16_t* p = img + (kc * 16 + 8 * (lane >> 5) + ((lane & 15) >> 2)) * TP + c0 + 16 * ((lane >> 4) & 1) +
                      4 * (lane & 3);
  const s16x4 lo = ds_tr(p), hi = ds_tr(p + 4 * TP);
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bfx8, v);
}
// the same fragment from a row image [row][k] with pitch RP
template <int RP>
__device__ __forceinline__ bfx8 frag_row(const uint16_t* img, int kc, int r0, int lane) {
  return *reinterpret_cast<const bfx8*>(img + (r0 + (lane & 31)) * RP + kc * 16 + 8 * (lane >> 5));
}

template <class P, int NTERM, int PIPE>
__device__ __forceinline__ void pxb_body(const PxbArgs& args, int block, uint16_t* lds) {
  using G = GeoB<P>;
  static_assert(NTERM == 6 || NTERM == 8, "6 or 8 term products");
  typename P::Ctx ctx;
  P::decode(args, block, ctx);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave % G::WM, wn = wave / G::WM;
  const int64_t psa = args.a_ps, psb = args.b_ps;
  constexpr bool CS = P::COLSUM;
  const bool want_cs = CS && P::want_colsum(ctx) && wn == 0;  // wave-uniform
  f32x16 acc[G::TM][G::TN], acc2[G::TM][G::TN], cs[G::TM];
#pragma unroll
  for (int i = 0; i < G::TM; ++i) {
#pragma unroll
    for (int e = 0; e < 16; ++e) cs[i][e] = 0.f;
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = acc2[i][j][e] = 0.f;
  }
  // per-thread loader states: row operands keep a row pointer (k offsets are uniform per
  // k-block), transposed operands a (k row, chunk) state the policy turns into an address
  typename P::LA la[G::NA];
  typename P::LB lb[G::NB];
  // (a last partial round of chunks, e.g. the 32-column B of conv2's input gradient: the
  // threads beyond it keep the last chunk's state and skip the loads and stores; wave-uniform)
#pragma unroll
  for (int j = 0; j < G::NA; ++j) la[j] = P::init_a(args, ctx, min(t + 256 * j, G::CA - 1));
#pragma unroll
  for (int j = 0; j < G::NB; ++j) lb[j] = P::init_b(args, ctx, min(t + 256 * j, G::CB - 1));
  uint4 ra0[G::NA][3], rb0[G::NB][3], ra1[G::NA][3], rb1[G::NB][3];
  auto gload = [&](int kb, uint4 (&ra)[G::NA][3], uint4 (&rb)[G::NB][3]) {
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      if (G::CA % 256 != 0 && t + 256 * j >= G::CA) continue;
      const uint16_t* a = P::ptr_a(args, ctx, la[j], kb);
#pragma unroll
      for (int u = 0; u < 3; ++u) ra[j][u] = a ? *reinterpret_cast<const uint4*>(a + u * psa) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      if (G::CB % 256 != 0 && t + 256 * j >= G::CB) continue;
      const uint16_t* b = P::ptr_b(args, ctx, lb[j], kb);
#pragma unroll
      for (int u = 0; u < 3; ++u) rb[j][u] = b ? *reinterpret_cast<const uint4*>(b + u * psb) : make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf, const uint4 (&ra)[G::NA][3], const uint4 (&rb)[G::NB][3]) {
    uint16_t* As = lds + buf * G::STAGE;
    uint16_t* Bs = As + 3 * G::SA;
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      const int q = t + 256 * j;
      if (G::CA % 256 != 0 && q >= G::CA) continue;
      // transposed: chunk q = (k row q / (BM/8), columns 8 (q % (BM/8))); row: (row q / 4, k 8 (q % 4))
      uint16_t* d = P::A_TR ? As + (q / (G::BM / 8)) * G::TPA + 8 * (q % (G::BM / 8))
                            : As + (q / (G::BK / 8)) * G::RP + 8 * (q % (G::BK / 8));
#pragma unroll
      for (int u = 0; u < 3; ++u) *reinterpret_cast<uint4*>(d + u * G::SA) = ra[j][u];
    }
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      const int q = t + 256 * j;
      if (G::CB % 256 != 0 && q >= G::CB) continue;
      uint16_t* d = P::B_TR ? Bs + (q / (G::BN / 8)) * G::TPB + 8 * (q % (G::BN / 8))
                            : Bs + (q / (G::BK / 8)) * G::RP + 8 * (q % (G::BK / 8));
#pragma unroll
      for (int u = 0; u < 3; ++u) *reinterpret_cast<uint4*>(d + u * G::SB) = rb[j][u];
    }
  };
  const s16x8 ones_s = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};  // bf16 1.0
  const bfx8 ones = __builtin_bit_cast(bfx8, ones_s);
  auto compute = [&](int buf) {
    const uint16_t* As = lds + buf * G::STAGE;
    const uint16_t* Bs = As + 3 * G::SA;
#pragma unroll
    for (int kc = 0; kc < G::BK / 16; ++kc) {
      bfx8 a[G::TM][3], b[G::TN][3];
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int m0 = wm * G::WTM + mi * 32;
          if constexpr (P::A_TR) a[mi][u] = frag_tr<G::TPA>(As + u * G::SA, kc, m0, lane);
          else a[mi][u] = frag_row<G::RP>(As + u * G::SA, kc, m0, lane);
        }
#pragma unroll
      for (int ni = 0; ni < G::TN; ++ni)
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int n0 = wn * G::WTN + ni * 32;
          if constexpr (P::B_TR) b[ni][u] = frag_tr<G::TPB>(Bs + u * G::SB, kc, n0, lane);
          else b[ni][u] = frag_row<G::RP>(Bs + u * G::SB, kc, n0, lane);
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
          if constexpr (NTERM == 8) {
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][1], b[ni][2], c2, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][2], b[ni][1], c2, 0, 0, 0);
          }
          acc2[mi][ni] = c2;
        }
      if constexpr (CS) {
        if (want_cs) {  // bias gradient: row sums of A (h + m + l, each exact against 1.0)
#pragma unroll
          for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
            for (int u = 0; u < 3; ++u) cs[mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi][u], ones, cs[mi], 0, 0, 0);
        }
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
  } else {  // one LDS stage, k-blocks kb+1 and kb+2 in flight in registers (px_kernels.hip gemm_px1_k)
    int kb = ctx.kb0;
    if (kb < ctx.kb1) gload(kb, ra0, rb0);
    if (kb + 1 < ctx.kb1) gload(kb + 1, ra1, rb1);
    for (; kb < ctx.kb1; kb += 2) {
      __syncthreads();
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
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * h;  // 32x32 MFMA C/D layout
        P::store(args, ctx, wm * G::WTM + mi * 32 + row, wn * G::WTN + ni * 32 + r, acc[mi][ni][e] + acc2[mi][ni][e]);
      }
  if constexpr (CS) {
    if (want_cs && r == 0) {  // every column of A * ones is the row sum: lanes 0 and 32 hold all rows
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int e = 0; e < 16; ++e) P::store_colsum(args, ctx, wm * G::WTM + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * h, cs[mi][e]);
    }
  }
}

template <int A, int B>
struct MaxOf {
  static constexpr int v = A > B ? A : B;
};

template <class P1, class P2, int NTERM>
__global__ __launch_bounds__(256, 2) void pxb2_k(PxbArgs a1, PxbArgs a2, int n1) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[MaxOf<GeoB<P1>::LDS, GeoB<P2>::LDS>::v];
  if ((int)blockIdx.x < n1) pxb_body<P1, NTERM, 0>(a1, blockIdx.x, lds);
  else pxb_body<P2, NTERM, 0>(a2, blockIdx.x - n1, lds);
}
template <class P1, class P2, int NTERM>
__global__ __launch_bounds__(256, 2) void pxb2p1_k(PxbArgs a1, PxbArgs a2, int n1) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[MaxOf<GeoB<P1>::STAGE, GeoB<P2>::STAGE>::v];
  if ((int)blockIdx.x < n1) pxb_body<P1, NTERM, 1>(a1, blockIdx.x, lds);
  else pxb_body<P2, NTERM, 1>(a2, blockIdx.x - n1, lds);
}

// ------------------------------------------------------------------ policies
// Shared by the row-read operands: LA / LB = the chunk's row pointer (null: zero row).
struct RowPtr {
  const uint16_t* p;
};
// A stored ReLU'd input gradient: y = (mask > 0) v, fp32 + planes
__device__ __forceinline__ void store_dgrad(const PxbArgs& a, size_t o, float v) {
  const float y = a.mask[o] > 0.f ? v : 0.f;
  a.out[o] = y;
  if (a.outx) store_planes(a.outx, a.out_ps, o, y);
}

// FC1 input gradient: dy3[b][k'] = (a3 > 0) sum_n dz[b][n] wfc1p[n][k'];  A = dz planes (row
// read, k = n), B = wfc1p planes staged [n][k'] and read transposed.  64 x 64 tiles.
struct Fc1DgradX {
  static constexpr int BM = 64, BN = 64, WM = 2;
  static constexpr bool A_TR = false, B_TR = true, COLSUM = false;
  struct Ctx {
    int m0, n0, kb0, kb1;
  };
  using LA = RowPtr;
  struct LB {
    int kr, c8;
  };
  static __host__ __device__ int tiles(int B) { return ((B + BM - 1) / BM) * 49; }
  static __device__ void decode(const PxbArgs&, int block, Ctx& c) {
    c.n0 = (block % 49) * BN;
    c.m0 = (block / 49) * BM;
    c.kb0 = 0;
    c.kb1 = 256 / 32;
  }
  static __device__ LA init_a(const PxbArgs& a, const Ctx& c, int q) {
    const int b = c.m0 + q / 4;
    return {b < a.B ? a.ax + (size_t)b * 256 + 8 * (q % 4) : nullptr};
  }
  static __device__ const uint16_t* ptr_a(const PxbArgs&, const Ctx&, const LA& s, int kb) {
    return s.p ? s.p + kb * 32 : nullptr;
  }
  static __device__ LB init_b(const PxbArgs&, const Ctx& c, int q) { return {q / (BN / 8), c.n0 + 8 * (q % (BN / 8))}; }
  static __device__ const uint16_t* ptr_b(const PxbArgs& a, const Ctx&, const LB& s, int kb) {
    return a.bx + (size_t)(kb * 32 + s.kr) * 3136 + s.c8;
  }
  static __device__ bool want_colsum(const Ctx&) { return false; }
  static __device__ void store_colsum(const PxbArgs&, const Ctx&, int, float) {}
  static __device__ void store(const PxbArgs& a, const Ctx& c, int ml, int nl, float v) {
    const int b = c.m0 + ml;
    if (b < a.B) store_dgrad(a, (size_t)b * 3136 + c.n0 + nl, v);
  }
};

// FC1 weight gradient: dW[n][k'] = sum_b dz[b][n] a3[b][k'];  both operands staged [b][...] and
// read transposed.  a.splits > 0: batch slices of a.kbps k-blocks, natural-order partials
// out[slice][256][3136] (grad_finalize's FC1 job sums + transposes); 0: reference layout in
// place (out = advantage rows, out2 = value rows), as Fc1Wgrad of f32_kernels.hip.
struct Fc1WgradX {
  static constexpr int BM = 64, BN = 64, WM = 2;
  static constexpr bool A_TR = true, B_TR = true, COLSUM = false;
  struct Ctx {
    int m0, n0, split, kb0, kb1;
  };
  struct LA {
    int kr, c8;
  };
  using LB = LA;
  static __host__ __device__ int tiles(int) { return 4 * 49; }
  static __device__ void decode(const PxbArgs& a, int block, Ctx& c) {
    const int t = block % (4 * 49);
    c.split = block / (4 * 49);
    c.n0 = (t % 49) * BN;
    c.m0 = (t / 49) * BM;
    const int nkb = (a.B + 31) / 32;
    c.kb0 = a.splits > 0 ? c.split * a.kbps : 0;
    c.kb1 = a.splits > 0 ? min(nkb, c.kb0 + a.kbps) : nkb;
  }
  static __device__ LA init_a(const PxbArgs&, const Ctx& c, int q) { return {q / (BM / 8), c.m0 + 8 * (q % (BM / 8))}; }
  static __device__ const uint16_t* ptr_a(const PxbArgs& a, const Ctx&, const LA& s, int kb) {
    const int b = kb * 32 + s.kr;
    return b < a.B ? a.ax + (size_t)b * 256 + s.c8 : nullptr;
  }
  static __device__ LB init_b(const PxbArgs&, const Ctx& c, int q) { return {q / (BN / 8), c.n0 + 8 * (q % (BN / 8))}; }
  static __device__ const uint16_t* ptr_b(const PxbArgs& a, const Ctx&, const LB& s, int kb) {
    const int b = kb * 32 + s.kr;
    return b < a.B ? a.bx + (size_t)b * 3136 + s.c8 : nullptr;
  }
  static __device__ bool want_colsum(const Ctx&) { return false; }
  static __device__ void store_colsum(const PxbArgs&, const Ctx&, int, float) {}
  static __device__ void store(const PxbArgs& a, const Ctx& c, int ml, int nl, float v) {
    const int n = c.m0 + ml, k = c.n0 + nl;
    if (a.splits > 0) {
      a.out[((size_t)c.split * 256 + n) * 3136 + k] = v;
      return;
    }
    const int ref = (k & 63) * 49 + (k >> 6);
    if (n < 128) a.out[n * 3136 + ref] = v;
    else a.out2[(n - 128) * 3136 + ref] = v;
  }
};

// conv weight gradient (layers 2, 3): part[s][co][tap*C + ci] = sum_{rows (b, p) of split s}
// dy[b][p][co] x[b][window(p, tap)][ci];  k-blocks are POSITION-major (p, block of 32 samples)
// as in ConvWgrad of f32_kernels.hip, so a k-block's rows are 32 samples at one output position.
// A = dy planes staged [row][co], B = the input planes' im2col rows staged [row][(tap, ci)],
// both read transposed; the bias partial is A's row sum (the n0 == 0 tile).
template <int L>
struct ConvWgradX {
  static constexpr int C = L == 3 ? 64 : 32, K = L == 3 ? 3 : 4, S = L == 3 ? 1 : 2;
  static constexpr int IH = L == 3 ? 9 : 20, OH = L == 3 ? 7 : 9, P = OH * OH;
  static constexpr int N = K * K * C;
  static constexpr int BM = 64, BN = 64, WM = 2;
  static constexpr bool A_TR = true, B_TR = true, COLSUM = true;
  struct Ctx {
    int n0, split, kb0, kb1, nbb;
  };
  struct LA {
    int kr, c8;
  };
  struct LB {
    int kr, off;  // off = (ky * IH + kx) * C + ci of the chunk's 8 columns
  };
  static __host__ __device__ int kblocks(int B) { return P * ((B + 31) / 32); }
  static __host__ __device__ int tiles(int, int splits) { return (N / BN) * splits; }
  static __device__ void decode(const PxbArgs& a, int block, Ctx& c) {
    constexpr int NT = N / BN;
    c.split = block / NT;
    c.n0 = (block % NT) * BN;
    c.nbb = (a.B + 31) / 32;
    c.kb0 = c.split * a.kbps;
    c.kb1 = min(c.kb0 + a.kbps, kblocks(a.B));
  }
  static __device__ LA init_a(const PxbArgs&, const Ctx&, int q) { return {q / (BM / 8), 8 * (q % (BM / 8))}; }
  static __device__ const uint16_t* ptr_a(const PxbArgs& a, const Ctx& c, const LA& s, int kb) {
    const int p = kb / c.nbb, b = (kb - p * c.nbb) * 32 + s.kr;  // p, block base: wave-uniform
    return b < a.B ? a.ax + ((size_t)b * P + p) * 64 + s.c8 : nullptr;
  }
  static __device__ LB init_b(const PxbArgs&, const Ctx& c, int q) {
    const int n = c.n0 + 8 * (q % (BN / 8)), tap = n / C, ci = n - tap * C, ky = tap / K, kx = tap - ky * K;
    return {q / (BN / 8), (ky * IH + kx) * C + ci};
  }
  static __device__ const uint16_t* ptr_b(const PxbArgs& a, const Ctx& c, const LB& s, int kb) {
    const int p = kb / c.nbb, b = (kb - p * c.nbb) * 32 + s.kr;
    if (b >= a.B) return nullptr;
    const int oy = p / OH, ox = p - oy * OH;
    return a.bx + ((size_t)b * IH * IH + S * oy * IH + S * ox) * C + s.off;
  }
  static __device__ bool want_colsum(const Ctx& c) { return c.n0 == 0; }
  static __device__ void store_colsum(const PxbArgs& a, const Ctx& c, int m, float v) { a.out2[c.split * 64 + m] = v; }
  static __device__ void store(const PxbArgs& a, const Ctx& c, int m, int nl, float v) {
    a.out[((size_t)c.split * 64 + m) * N + c.n0 + nl] = v;
  }
};

// conv3 input gradient, position-major (Conv3DgradPT of f32_kernels.hip): rows = 64 samples at
// one input position pi, k = (valid tap, co); A = dy3 planes [b][49][64], B = w3t planes
// [tap][ci][co] (row reads).  dy2 = (a2 > 0) v, fp32 + planes (the conv2 backward's operand).
struct Conv3DgradX {
  static constexpr int BM = 64, BN = 64, WM = 2;
  static constexpr bool A_TR = false, B_TR = false, COLSUM = false;
  struct Ctx {
    int b0, pos, iy, ix, ky0, kx0, nkx, kb0, kb1;
  };
  using LA = RowPtr;
  using LB = RowPtr;
  static __host__ __device__ int tiles(int B) { return 81 * ((B + BM - 1) / BM); }
  static __device__ void decode(const PxbArgs& a, int block, Ctx& c) {
    const int tpp = (a.B + BM - 1) / BM;
    c.pos = block / tpp;
    c.b0 = (block - c.pos * tpp) * BM;
    c.iy = c.pos / 9;
    c.ix = c.pos - c.iy * 9;
    c.ky0 = max(0, c.iy - 6);
    c.kx0 = max(0, c.ix - 6);
    const int nky = min(2, c.iy) - c.ky0 + 1;
    c.nkx = min(2, c.ix) - c.kx0 + 1;
    c.kb0 = 0;
    c.kb1 = 2 * nky * c.nkx;
  }
  static __device__ void tap_of(const Ctx& c, int kb, int& ky, int& kx) {
    const int ti = kb >> 1, r = ti / c.nkx;
    ky = c.ky0 + r;
    kx = c.kx0 + ti - r * c.nkx;
  }
  static __device__ LA init_a(const PxbArgs& a, const Ctx& c, int q) {
    const int b = c.b0 + q / 4;
    return {b < a.B ? a.ax + (size_t)b * 49 * 64 + 8 * (q % 4) : nullptr};
  }
  static __device__ const uint16_t* ptr_a(const PxbArgs&, const Ctx& c, const LA& s, int kb) {
    int ky, kx;
    tap_of(c, kb, ky, kx);
    return s.p ? s.p + ((c.iy - ky) * 7 + c.ix - kx) * 64 + (kb & 1) * 32 : nullptr;
  }
  static __device__ LB init_b(const PxbArgs& a, const Ctx&, int q) { return {a.bx + (q / 4) * 64 + 8 * (q % 4)}; }
  static __device__ const uint16_t* ptr_b(const PxbArgs&, const Ctx& c, const LB& s, int kb) {
    int ky, kx;
    tap_of(c, kb, ky, kx);
    return s.p + (ky * 3 + kx) * 4096 + (kb & 1) * 32;
  }
  static __device__ bool want_colsum(const Ctx&) { return false; }
  static __device__ void store_colsum(const PxbArgs&, const Ctx&, int, float) {}
  static __device__ void store(const PxbArgs& a, const Ctx& c, int ml, int n, float v) {
    const int b = c.b0 + ml;
    if (b < a.B) store_dgrad(a, ((size_t)b * 81 + c.pos) * 64 + n, v);
  }
};

// conv2 input gradient, position-major sub-pixel classes (Conv2DgradP of f32_kernels.hip):
// input pixel (2 jy + py, 2 jx + px) takes taps (py + 2 ty, px + 2 tx) from output pixel
// (jy - ty, jx - tx); rows = 128 samples of one (class, jy, jx), N = 32 input channels.
// A = dy2 planes [b][81][64], B = w2t planes [ky][kx][ci][co].  dy1 = (a1 > 0) v (fp32 only:
// the conv1 weight gradient splits it itself).
struct Conv2DgradX {
  static constexpr int BM = 128, BN = 32, WM = 4;
  static constexpr bool A_TR = false, B_TR = false, COLSUM = false;
  struct Ctx {
    int b0, cls, jy, jx, ty0, tx0, ntx, kb0, kb1;
  };
  using LA = RowPtr;
  using LB = RowPtr;
  static __host__ __device__ int tiles(int B) { return 400 * ((B + BM - 1) / BM); }
  static __device__ void decode(const PxbArgs& a, int block, Ctx& c) {
    const int tpp = (a.B + BM - 1) / BM;
    const int pos = block / tpp;  // cls * 100 + jy * 10 + jx
    c.b0 = (block - pos * tpp) * BM;
    c.cls = pos / 100;
    const int jj = pos - c.cls * 100;
    c.jy = jj / 10;
    c.jx = jj - c.jy * 10;
    c.ty0 = c.jy == 9 ? 1 : 0;
    c.tx0 = c.jx == 9 ? 1 : 0;
    const int nty = (c.jy == 0 ? 0 : 1) - c.ty0 + 1;
    c.ntx = (c.jx == 0 ? 0 : 1) - c.tx0 + 1;
    c.kb0 = 0;
    c.kb1 = 2 * nty * c.ntx;
  }
  static __device__ void tap_of(const Ctx& c, int kb, int& ty, int& tx) {
    const int ti = kb >> 1, r = c.ntx == 2 ? ti >> 1 : ti;
    ty = c.ty0 + r;
    tx = c.tx0 + ti - r * c.ntx;
  }
  static __device__ LA init_a(const PxbArgs& a, const Ctx& c, int q) {
    const int b = c.b0 + q / 4;
    return {b < a.B ? a.ax + (size_t)b * 81 * 64 + 8 * (q % 4) : nullptr};
  }
  static __device__ const uint16_t* ptr_a(const PxbArgs&, const Ctx& c, const LA& s, int kb) {
    int ty, tx;
    tap_of(c, kb, ty, tx);
    return s.p ? s.p + ((c.jy - ty) * 9 + c.jx - tx) * 64 + (kb & 1) * 32 : nullptr;
  }
  static __device__ LB init_b(const PxbArgs& a, const Ctx&, int q) { return {a.bx + (q / 4) * 64 + 8 * (q % 4)}; }
  static __device__ const uint16_t* ptr_b(const PxbArgs&, const Ctx& c, const LB& s, int kb) {
    int ty, tx;
    tap_of(c, kb, ty, tx);
    const int ky = (c.cls >> 1) + 2 * ty, kx = (c.cls & 1) + 2 * tx;
    return s.p + (ky * 4 + kx) * 32 * 64 + (kb & 1) * 32;
  }
  static __device__ bool want_colsum(const Ctx&) { return false; }
  static __device__ void store_colsum(const PxbArgs&, const Ctx&, int, float) {}
  static __device__ void store(const PxbArgs& a, const Ctx& c, int ml, int n, float v) {
    const int b = c.b0 + ml;
    if (b >= a.B) return;
    const int iy = 2 * c.jy + (c.cls >> 1), ix = 2 * c.jx + (c.cls & 1);
    store_dgrad(a, ((size_t)b * 400 + iy * 20 + ix) * 32 + n, v);
  }
};

int g_pxb = 0;  // f32_set_variant(20, 0|1): the backward GEMMs on the pre-split kernels (needs knob 19)

template <class P1, class P2>
void launch_pair(const PxbArgs& a1, int n1, const PxbArgs& a2, int n2, hipStream_t s) {
  if (n1 + n2 <= 0) return;
  if (px_pipe() == 1) {
    if (px_terms() == 8) pxb2p1_k<P1, P2, 8><<<n1 + n2, 256, 0, s>>>(a1, a2, n1);
    else pxb2p1_k<P1, P2, 6><<<n1 + n2, 256, 0, s>>>(a1, a2, n1);
  } else {
    if (px_terms() == 8) pxb2_k<P1, P2, 8><<<n1 + n2, 256, 0, s>>>(a1, a2, n1);
    else pxb2_k<P1, P2, 6><<<n1 + n2, 256, 0, s>>>(a1, a2, n1);
  }
  LAUNCH_CHECK();
}

void check_planes(const void* p, int64_t ps, const char* what) {
  if (!p || ps <= 0 || (reinterpret_cast<uintptr_t>(p) & 15) || (ps & 7))
    throw std::invalid_argument(std::string("pxb: ") + what + " planes must be 16-byte aligned with a positive plane stride (multiple of 8)");
}

}  // namespace

bool pxb_enabled() { return g_pxb != 0 && px_enabled(); }

void pxb_set(int v) { g_pxb = v; }

void pxb_fc1_bwd(const PxbFc1& f, int B, hipStream_t s) {
  if (B <= 0) return;
  check_planes(f.dzx, f.dz_ps, "dz");
  check_planes(f.a3x, f.a3_ps, "a3");
  check_planes(f.wx, f.w_ps, "wfc1p");
  if (f.dy3x) check_planes(f.dy3x, f.dy3_ps, "dy3");
  PxbArgs d{};
  d.ax = f.dzx;
  d.a_ps = f.dz_ps;
  d.bx = f.wx;
  d.b_ps = f.w_ps;
  d.mask = f.a3;
  d.out = f.dy3;
  d.outx = f.dy3x;
  d.out_ps = f.dy3_ps;
  d.B = B;
  PxbArgs w{};
  w.ax = f.dzx;
  w.a_ps = f.dz_ps;
  w.bx = f.a3x;
  w.b_ps = f.a3_ps;
  w.out = f.gw;
  w.out2 = f.gw2;
  w.B = B;
  int slices = 1;
  if (f.slices > 0) {  // natural-order partials in f.slices batch slices (f32_fc1_wgrad_slices)
    const int nkb = (B + 31) / 32;
    w.kbps = (nkb + f.slices - 1) / f.slices;
    w.splits = slices = (nkb + w.kbps - 1) / w.kbps;
  }
  launch_pair<Fc1WgradX, Fc1DgradX>(w, Fc1WgradX::tiles(B) * slices, d, Fc1DgradX::tiles(B), s);
}

void pxb_conv_bwd(int layer, const PxbConv& c, int B, int splits, int kbps, hipStream_t s) {
  if (B <= 0) return;
  check_planes(c.dyx, c.dy_ps, "dy");
  check_planes(c.xx, c.x_ps, "x");
  check_planes(c.wtx, c.wt_ps, "wt");
  if (c.dxx) check_planes(c.dxx, c.dx_ps, "dx");
  PxbArgs g{};
  g.ax = c.dyx;
  g.a_ps = c.dy_ps;
  g.bx = c.xx;
  g.b_ps = c.x_ps;
  g.out = c.ws;
  g.out2 = c.ws_bias;
  g.B = B;
  g.kbps = kbps;
  g.splits = splits;
  PxbArgs d{};
  d.ax = c.dyx;
  d.a_ps = c.dy_ps;
  d.bx = c.wtx;
  d.b_ps = c.wt_ps;
  d.mask = c.mask;
  d.out = c.dx;
  d.outx = c.dxx;
  d.out_ps = c.dx_ps;
  d.B = B;
  if (layer == 3) launch_pair<ConvWgradX<3>, Conv3DgradX>(g, ConvWgradX<3>::tiles(B, splits), d, Conv3DgradX::tiles(B), s);
  else if (layer == 2) launch_pair<ConvWgradX<2>, Conv2DgradX>(g, ConvWgradX<2>::tiles(B, splits), d, Conv2DgradX::tiles(B), s);
  else throw std::invalid_argument("pxb_conv_bwd: layer 2 or 3");
}

}  // namespace apex
