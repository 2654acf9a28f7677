// Reference-precision (fp32) Nature-CNN dueling network on CDNA4 fp32 MFMA (gfx950).
//
// The reference trains entirely in fp32 (origin_repo/learner.py:139-145, utils.py:64-97,
// model.py:31-68).  gfx950 has exact-f32 matrix instructions -- v_mfma_f32_32x32x2_f32 is
// bit-for-bit a k-ordered fmaf chain at 64 FLOP/clk/SIMD (157 TF chip) -- so every GEMM-shaped
// op of the learner step (three forwards, the whole backward) runs on them here, with fp32
// operands and fp32 activations.  Weights are read from exact fp32 PACKED copies in GEMM
// layouts (k-contiguous rows), which the optimizer rewrites in the same pass as the master
// update (learner_kernels.hip PackMap / FcPack): gathering a weight chunk from the reference
// layout took four strided dword loads per 16 bytes, and the texture-address work of those
// scattered loads, not the MFMA pipe, bounded conv2/conv3/FC1 (MI355X: FC1 forward 60 -> 35 us,
// conv2 114 -> 90 us per 1536-sample launch).  Packed layouts (models/fused_f32.py):
//   conv1 W1 [32][c*64 + ky*8 + kx] (= reference)   w2p [64][tap*32 + ci]   w3p [64][tap*64 + ci]
//   wfc1p [256][p*64 + c] (FC1 forward, and row-major the input-gradient B operand)
//   w2t [ky][kx][ci][co], w3t [ky][kx][ci][co] (dgrad B operands, co contiguous)
//
// One templated LDS-staged GEMM body serves all 13 GEMMs; a policy per layer supplies the
// tile decode, the operand chunk loaders (implicit im2col / col2im / sub-pixel gathers,
// u8 frames converted in the loader) and the epilogue (bias+ReLU, ReLU-backward mask,
// split-K partials, conv bias column sums):
//
//   * C[M][N] = sum_k A(m,k) B(k,n); 256 threads = 4 waves on a WM x WN wave grid, each wave
//     TM x TN 32x32 accumulators (16 fp32 each).
//   * each operand tile is staged global -> registers -> LDS in its natural global layout:
//     "K-major" [row][BK] (k contiguous) or "MN-major" [k][BM|BN] (m|n contiguous), 16-byte
//     chunks; LDS double buffer + register prefetch of the next k-block (one barrier per
//     k-block; a sched_barrier pins the prefetch ahead of the MFMA block, otherwise the
//     scheduler sinks late-needed loads next to their LDS store and exposes their latency);
//     pitches padded so the fragment reads are bank-conflict free.
//   * k-chunk mapping: for a chunk of 8 k, lane (r = l & 31, h = l >> 5) holds elements
//     k = 4h .. 4h+3 of its A row / B column (one ds_read_b128 when K-major, four ds_read_b32
//     when MN-major); MFMA i of the chunk consumes element i of both -- the 32x32x2 MFMA's
//     k-slot h is then k = 4h + i, and the four MFMAs together cover all 8.
//
// Layer GEMMs (B samples, activations channels-last fp32: a1 [B][400][32], a2 [B][81][64],
// a3 [B][49][64]):
//   fwd  conv1 M=B*400 N=32 K=256 (c,ky,kx; u8 frames)   conv2 M=B*81 N=64 K=512 (tap,ci)
//        conv3 M=B*49 N=64 K=576                          fc1 M=B N=256 K=3136 (split-K 7)
//   bwd  fc1 dgrad M=B N=3136 K=256 (+ReLU mask)          fc1 wgrad M=256 N=3136 K=B
//        conv3/conv2 wgrad M=Cout N=taps*Cin K=B*P (split) conv3 dgrad M=B*81 N=64 K=576
//        conv2 dgrad: 4 stride-2 sub-pixel classes, M=4*B*100 N=32 K=4*64
//        conv1 wgrad M=32 N=256 K=B*400 (sample-resident kernel, partial per 2 samples)
// Independent backward GEMMs share one launch (gemm2_k: fc1 dgrad+wgrad, conv3 wgrad+dgrad,
// conv2 wgrad+dgrad), so the backward is 4 GEMM launches + one grad_finalize.  conv1 (forward
// and weight gradient) has its own sample-resident kernels: u8 frame planes staged in LDS.
//
// Two forms of the same GEMM body (bit-identical results, tests/test_gpu_f32_net.py):
//  * register split: operands staged as fp32 in LDS; every wave splits every fragment it reads
//    into bf16 hi / mid / lo (split8, 44 VALU per fragment and 16 k -- 11-18 VALU per MFMA);
//  * stage split (GeoS): the thread that stages a 4-value chunk splits it ONCE and stores the three
//    bf16 planes; fragments are read back ready (ds_read_b128 for K-major operands,
//    ds_read_b64_tr_b16 -- the hardware transpose -- for MN-major ones): 3-8 VALU per MFMA, one
//    LDS image (the next k-block waits in registers) so the footprint stays at the fp32 form's.
// The forward launches run the stage split (co-running with the actor's forward, they gain most
// from the VALU they no longer issue); the backward pairs keep the register split (measured no
// faster staged: profiles/r6_stage_split.md).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "tree_dev.h"

namespace apex {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
// 4 u8 pixels (one dword) -> 4 floats (v_cvt_f32_ubyte0..3); 0..255 exact
__device__ __forceinline__ f32x4 u8x4(uint32_t w) {
  return f32x4{(float)(w & 0xFFu), (float)((w >> 8) & 0xFFu), (float)((w >> 16) & 0xFFu), (float)(w >> 24)};
}

constexpr int kPlane = 84 * 84;

// Raw buffer resources for the backward GEMM operands: a load at a byte offset past the
// operand's range returns zeros (the range check of a raw buffer), and the rows of every
// backward operand are sample-major, so the rows of a tile past the batch lie past the range.
// The loaders then keep ONE 32-bit byte offset per chunk (k-invariant, computed once) plus
// the k-block's wave-uniform offset: a single VALU add per 16-byte load, no 64-bit address
// math and no "sample < B" select (operands below 2 GiB: host check).
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* p, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)nbytes, 0x00020000);
}
__device__ __forceinline__ f32x4 bld4(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
struct BufRow {
  uint32_t off;  // byte offset of the chunk at k-block 0
};


struct NoSmem {
  int unused;
};

template <class P>
struct Geo {
  static constexpr int BM = P::BM, BN = P::BN, BK = P::BK, WM = P::WM, WN = 4 / P::WM;
  static constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  static constexpr int TM = WTM / 32, TN = WTN / 32;
  static constexpr int PA = P::A_KMAJ ? BK + 4 : BM + 8;  // LDS pitches (floats)
  static constexpr int PB = P::B_KMAJ ? BK + 4 : BN + 8;
  static constexpr int RA = P::A_KMAJ ? BK / 4 : BM / 4;  // 16-byte chunks per LDS row
  static constexpr int RB = P::B_KMAJ ? BK / 4 : BN / 4;
  static constexpr int SA = (P::A_KMAJ ? BM : BK) * PA;
  static constexpr int SB = (P::B_KMAJ ? BN : BK) * PB;
  static constexpr int CA = BM * BK / 4, CB = BN * BK / 4;
  static constexpr int NA = (CA + 255) / 256, NB = (CB + 255) / 256;
  static constexpr int LDS_FLOATS = 2 * (SA + SB);
  static_assert(WM * WN == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "32x32 wave blocks");
  static_assert(BK % 8 == 0, "k-chunks of 8");
  static_assert(LDS_FLOATS >= 4 * 256, "colsum reduction reuses the LDS tile");
};

// Policies may opt into an A column-sum (conv bias gradient = sum of dY over pixels):
// only for MN-major A, where each thread's chunks always cover the same 4 columns.
template <class P, class = void>
struct HasColsum {
  static constexpr bool value = false;
};
template <class P>
struct HasColsum<P, decltype((void)P::A_COLSUM, void())> {
  static constexpr bool value = P::A_COLSUM;
};

// The next k-block is loaded into registers while the current one computes (its LDS store
// follows the MFMA block).  Policies may precompute a per-thread row state once (the k-invariant part of an operand
// chunk's address: im2col divisions by the output width, sample / channel offsets) and load
// each k-block from it with a scalar offset: row_a(args, ctx, row, ch) -> RowA and
// load_a_row(args, ctx, RowA, kb) (same for B).  Without it the loaders re-derive the whole
// address per chunk and k-block (~20 VALU per 16-byte load: 5-7 VALU per MFMA measured).
template <class P, class = void>
struct HasRowA : std::false_type {};
template <class P>
struct HasRowA<P, std::void_t<typename P::RowA>> : std::true_type {};
template <class P, class = void>
struct HasRowB : std::false_type {};
template <class P>
struct HasRowB<P, std::void_t<typename P::RowB>> : std::true_type {};
template <class P, bool = HasRowA<P>::value>
struct RowAOf {
  using type = int;
};
template <class P>
struct RowAOf<P, true> {
  using type = typename P::RowA;
};
template <class P, bool = HasRowB<P>::value>
struct RowBOf {
  using type = int;
};
template <class P>
struct RowBOf<P, true> {
  using type = typename P::RowB;
};

// XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs (b and b + 8 share an
// L2), so with the identity order the N-tiles of one M-tile -- and neighbouring M-tiles,
// whose im2col windows overlap -- land on different XCDs and each L2 fetches them again.
// Chunked: XCD j walks the contiguous logical tiles [j G/8, (j+1) G/8) in order.  A pure
// permutation of the tiles (bit-identical results); the tail past a multiple of 8 keeps
// the identity.
__device__ __forceinline__ int xcd_chunk(int b, int G) {
  const int G8 = G & ~7;
  return b >= G8 ? b : (b & 7) * (G8 >> 3) + (b >> 3);
}

// bf16 helpers of the exact-split conv1 kernels below (every fp32 term split by truncation)
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t pack_bf16_hi(float lo, float hi) {  // two exact bf16 halves
  return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}
__device__ __forceinline__ float trunc_bf16(float x) { return __uint_as_float(__float_as_uint(x) & 0xFFFF0000u); }

// Exact three-term split of 8 fp32 values (two 4-element k-runs of a fragment) into bf16
// hi / mid / lo vectors, x = hi + mid + lo EXACTLY (truncation: 8 + 8 + 8 significant bits).
// The products of every pair of terms are exact in fp32; the six kept pairs (hi.hi, hi.mid,
// mid.hi, hi.lo, mid.mid, lo.hi) leave out terms below 2^-23 |a||b| -- the size of the fp32
// rounding of the product itself -- so the GEMM is fp32-class on the bf16 matrix cores
// (1024 FLOP/clk/SIMD vs 64 for v_mfma_f32_32x32x2_f32: six of them still run 2.7x faster).
// (A round-to-nearest split through v_cvt_pk_bf16_f32 -- fewer VALU instructions on paper --
// measured 3-5 % slower per launch and 3 % slower per step on MI355X: profiles/r5_x6.md.)
struct Split8 {
  bfx8 h, m, l;
};
typedef float f32x2 __attribute__((ext_vector_type(2)));
// One pair (a, b) -> packed bf16 words of its hi / mid / lo terms.  PK: the two residual
// subtractions as one v_pk_add_f32 each (the same IEEE operations: bit-identical terms),
// 9 VALU per pair instead of 11 -- measured 3.5 % SLOWER per step inside the register-split
// GEMM loop (register pairs constrain the allocation, profiles/archive_r5.md (r5_ab_split_packed_sub.txt)),
// so only the stage-split store (outside the MFMA loop) uses it.
template <bool PK>
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  if constexpr (PK) {
    const f32x2 v = {a, b};
    const f32x2 r = v - f32x2{trunc_bf16(a), trunc_bf16(b)};
    const f32x2 rl = r - f32x2{trunc_bf16(r[0]), trunc_bf16(r[1])};
    h = pack_bf16_hi(a, b);  // (the perm takes the upper halves: truncation)
    m = pack_bf16_hi(r[0], r[1]);
    l = pack_bf16_hi(rl[0], rl[1]);  // exact: <= 8 significant bits
  } else {
    const float ar = a - trunc_bf16(a), br = b - trunc_bf16(b);
    const float am = trunc_bf16(ar), bm = trunc_bf16(br);
    h = pack_bf16_hi(a, b);
    m = pack_bf16_hi(am, bm);
    l = pack_bf16_hi(ar - am, br - bm);
  }
}
__device__ __forceinline__ Split8 split8(f32x4 x0, f32x4 x1) {
  uint32_t h[4], m[4], l[4];
  split_pair<false>(x0[0], x0[1], h[0], m[0], l[0]);
  split_pair<false>(x0[2], x0[3], h[1], m[1], l[1]);
  split_pair<false>(x1[0], x1[1], h[2], m[2], l[2]);
  split_pair<false>(x1[2], x1[3], h[3], m[3], l[3]);
  return {__builtin_bit_cast(bfx8, make_uint4(h[0], h[1], h[2], h[3])),
          __builtin_bit_cast(bfx8, make_uint4(m[0], m[1], m[2], m[3])),
          __builtin_bit_cast(bfx8, make_uint4(l[0], l[1], l[2], l[3]))};
}

// Stage-split LDS image (gemm_body<P, true>): each fp32 operand chunk is split ONCE, by the
// thread that stages it, into three bf16 planes (hi / mid / lo) in LDS; the waves read the
// planes back as ready MFMA fragments.  In the register-split form every wave splits every
// fragment it reads -- each element 2x (2 x 2 wave grids) to 4x (the shared B operand of a
// 4 x 1 grid), 44 VALU per fragment and 16 k -- which bounds the GEMMs on the VALU
// (14-20 VALU per MFMA, 15-29 % MFMA busy: profiles/r5_fp32_pmc.md).  Same terms, same
// k-slot of every product (bit-identical results):
//  * K-major operand: plane rows [row][BK] bf16; the 4-element staging chunk u of a 16-k
//    block lands in 16-byte chunk (u & 1), 8-byte half (u >> 1) -- so lane (r, h) reads slots
//    8h..8h+7 = k {4h..4h+3, 8+4h..8+4h+3} (split8's map) as ONE ds_read_b128 per plane;
//    chunks XOR-swizzled by row so a read's 16-lane groups hit 64 distinct banks.
//  * MN-major operand: plane rows [k][BM] bf16 (the staged chunk's 4 m at one k, natural
//    order); a fragment is two ds_read_b64_tr_b16 per plane (k rows 4h..+3 and 8+4h..+3:
//    lane 4q + p of a 16-lane group addresses k row q, columns 4p..4p+3; lane i receives
//    column i) -- the hardware transpose; chunks XOR-swizzled so a 32-lane half's four k rows
//    hit distinct banks.
template <class P>
struct GeoS {
  using G = Geo<P>;
  static constexpr int BM = P::BM, BN = P::BN, BK = P::BK;
  static constexpr int RBA = P::A_KMAJ ? BK * 2 : BM * 2;  // plane row bytes (no padding)
  static constexpr int RBB = P::B_KMAJ ? BK * 2 : BN * 2;
  static constexpr int PLA = (P::A_KMAJ ? BM : BK) * RBA;  // plane bytes
  static constexpr int PLB = (P::B_KMAJ ? BN : BK) * RBB;
  static constexpr int SA = 3 * PLA, SB = 3 * PLB;
  static constexpr int LDS_BYTES = 2 * (SA + SB);
  static_assert(BK == 16 || BK == 32, "K-major swizzle: 2 or 4 chunks per row");
  static_assert((P::A_KMAJ || BM == 32 || BM == 64 || BM == 128) && (P::B_KMAJ || BN == 32 || BN == 64 || BN == 128),
                "MN-major swizzle");
};
// K-major: row of NC = BK / 8 16-byte chunks; 16 / NC rows share a 256-byte bank line
template <int BK>
__device__ __forceinline__ int swz_k(int row) {
  constexpr int NC = BK / 8;
  return (row / (16 / NC)) & (NC - 1);
}
// MN-major: row of W bf16 (W / 8 chunks); a half-wave transposed read takes 4 rows x 4 chunks
template <int W>
__device__ __forceinline__ int swz_m(int row) {
  if constexpr (W == 32) return 0;
  else if constexpr (W == 64) return 4 * ((row >> 1) & 1);
  else return 4 * (row & 3);
}
// one staged fp32 chunk (4 values) -> its hi / mid / lo bf16 words (split_pair: split8's terms)
__device__ __forceinline__ void split4(f32x4 x, uint2& h, uint2& m, uint2& l) {
  split_pair<true>(x[0], x[1], h.x, m.x, l.x);
  split_pair<true>(x[2], x[3], h.y, m.y, l.y);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__device__ __forceinline__ uint2 ds_tr16(const char* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

// Every fp32 GEMM of the learner (gemm_body) on the bf16 matrix cores through split8: the
// fp32-MFMA form (v_mfma_f32_32x32x2_f32) it replaced in round 5 ran 2142 vs 2378 learner
// steps/s at the same fp32-class accuracy (profiles/r5_x6.md, tests/test_gpu_f32_net.py).
template <class P, int SS>
__device__ __forceinline__ void gemm_body(const typename P::Args& args, int block, float* lds,
                                          typename P::Smem& sm) {
  using G = Geo<P>;
  using GS = GeoS<P>;
  constexpr bool COLSUM = HasColsum<P>::value;
  static_assert(!COLSUM || (!P::A_KMAJ && 256 % G::RA == 0), "colsum needs MN-major A");
  typename P::Ctx ctx;
  P::decode(args, block, ctx, sm);
  if constexpr (P::SMEM) __syncthreads();
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave % G::WM, wn = wave / G::WM;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  constexpr int NSET = 1;
  f32x4 ra[NSET][G::NA], rb[NSET][G::NB];
  f32x4 csum = zero4();
  typename RowAOf<P>::type rowa[G::NA];
  typename RowBOf<P>::type rowb[G::NB];
  if constexpr (HasRowA<P>::value) {
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      const int q = min(t + 256 * j, G::CA - 1);
      rowa[j] = P::row_a(args, ctx, q / G::RA, q % G::RA);
    }
  }
  if constexpr (HasRowB<P>::value) {
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      const int q = min(t + 256 * j, G::CB - 1);
      rowb[j] = P::row_b(args, ctx, q / G::RB, q % G::RB);
    }
  }

  auto gload = [&](int kb, auto S) {
    constexpr int st = decltype(S)::value;
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      const int q = t + 256 * j;
      if (G::CA % 256 == 0 || q < G::CA) {
        if constexpr (HasRowA<P>::value) ra[st][j] = P::load_a_row(args, ctx, rowa[j], kb);
        else ra[st][j] = P::load_a(args, ctx, sm, kb, q / G::RA, q % G::RA);
      }
    }
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      const int q = t + 256 * j;
      if (G::CB % 256 == 0 || q < G::CB) {
        if constexpr (HasRowB<P>::value) rb[st][j] = P::load_b_row(args, ctx, rowb[j], kb);
        else rb[st][j] = P::load_b(args, ctx, sm, kb, q / G::RB, q % G::RB);
      }
    }
  };
  // stage-split store: chunk q of a K-major operand = row q / R, k 4 (q % R) .. +3; of an
  // MN-major operand = k row q / R, m 4 (q % R) .. +3 (R: fp32 chunks per row)
  auto ss_store = [&](char* base, int plane, auto KMAJ, auto W, int R, int q, f32x4 v) {
    uint2 hi, mi, lo;
    split4(v, hi, mi, lo);
    const int row = q / R, ch = q % R;
    int off;
    if constexpr (decltype(KMAJ)::value) {
      constexpr int BK = decltype(W)::value;
      const int u = ch & 3, pc = ((ch >> 2) * 2 + (u & 1)) ^ swz_k<BK>(row);
      off = row * (BK * 2) + pc * 16 + (u >> 1) * 8;
    } else {
      constexpr int Wd = decltype(W)::value;
      const int pc = (ch >> 1) ^ swz_m<Wd>(row);
      off = row * (Wd * 2) + pc * 16 + (ch & 1) * 8;
    }
    *reinterpret_cast<uint2*>(base + off) = hi;
    *reinterpret_cast<uint2*>(base + plane + off) = mi;
    *reinterpret_cast<uint2*>(base + 2 * plane + off) = lo;
  };
  auto sstore = [&](int buf, auto S) {
    constexpr int st = decltype(S)::value;
    if constexpr (SS) {
      char* As = reinterpret_cast<char*>(lds) + buf * (GS::SA + GS::SB);
      char* Bs = As + GS::SA;
      using KA = std::integral_constant<bool, P::A_KMAJ>;
      using KB = std::integral_constant<bool, P::B_KMAJ>;
      using WA = std::integral_constant<int, P::A_KMAJ ? G::BK : G::BM>;
      using WB = std::integral_constant<int, P::B_KMAJ ? G::BK : G::BN>;
#pragma unroll
      for (int j = 0; j < G::NA; ++j) {
        const int q = t + 256 * j;
        if (G::CA % 256 == 0 || q < G::CA) {
          ss_store(As, GS::PLA, KA{}, WA{}, G::RA, q, ra[st][j]);
          if constexpr (COLSUM) csum += ra[st][j];
        }
      }
#pragma unroll
      for (int j = 0; j < G::NB; ++j) {
        const int q = t + 256 * j;
        if (G::CB % 256 == 0 || q < G::CB) ss_store(Bs, GS::PLB, KB{}, WB{}, G::RB, q, rb[st][j]);
      }
      return;
    }
    float* As = lds + buf * (G::SA + G::SB);
    float* Bs = As + G::SA;
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      const int q = t + 256 * j;
      if (G::CA % 256 == 0 || q < G::CA) {
        *reinterpret_cast<f32x4*>(As + (q / G::RA) * G::PA + 4 * (q % G::RA)) = ra[st][j];
        if constexpr (COLSUM) csum += ra[st][j];
      }
    }
#pragma unroll
    for (int j = 0; j < G::NB; ++j) {
      const int q = t + 256 * j;
      if (G::CB % 256 == 0 || q < G::CB)
        *reinterpret_cast<f32x4*>(Bs + (q / G::RB) * G::PB + 4 * (q % G::RB)) = rb[st][j];
    }
  };
  using S0 = std::integral_constant<int, 0>;
  // the cross terms accumulate apart from hi.hi (summed in the epilogue)
  f32x16 accx[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) accx[i][j][e] = 0.f;
  auto frag_a = [&](const float* As, int mi, int kc) {
    const int m = wm * G::WTM + mi * 32 + r;
    f32x4 v;
    if constexpr (P::A_KMAJ) {
      v = *reinterpret_cast<const f32x4*>(As + m * G::PA + kc * 8 + 4 * h);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = As[(kc * 8 + 4 * h + i) * G::PA + m];
    }
    return v;
  };
  auto frag_b = [&](const float* Bs, int ni, int kc) {
    const int n = wn * G::WTN + ni * 32 + r;
    f32x4 v;
    if constexpr (P::B_KMAJ) {
      v = *reinterpret_cast<const f32x4*>(Bs + n * G::PB + kc * 8 + 4 * h);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = Bs[(kc * 8 + 4 * h + i) * G::PB + n];
    }
    return v;
  };
  // stage-split fragment of 16 k (k16 step s) for MFMA row/column `mn` of the wave tile
  auto ss_frag = [&](const char* base, int plane, auto KMAJ, auto W, int mn0, int s) {
    Split8 f;
    if constexpr (decltype(KMAJ)::value) {
      constexpr int BK = decltype(W)::value;
      const int row = mn0 + r;
      const char* p = base + row * (BK * 2) + (((2 * s + h) ^ swz_k<BK>(row)) * 16);
      f.h = __builtin_bit_cast(bfx8, *reinterpret_cast<const uint4*>(p));
      f.m = __builtin_bit_cast(bfx8, *reinterpret_cast<const uint4*>(p + plane));
      f.l = __builtin_bit_cast(bfx8, *reinterpret_cast<const uint4*>(p + 2 * plane));
    } else {
      constexpr int Wd = decltype(W)::value;
      const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
      const int col = mn0 + 16 * (g & 1) + 4 * pp, c = col >> 3, hb = ((col >> 2) & 1) * 8;
      const int k1 = 16 * s + 4 * (g >> 1) + qq, k2 = k1 + 8;
      const char* p1 = base + k1 * (Wd * 2) + ((c ^ swz_m<Wd>(k1)) * 16) + hb;
      const char* p2 = base + k2 * (Wd * 2) + ((c ^ swz_m<Wd>(k2)) * 16) + hb;
      uint2 x1, x2;
      x1 = ds_tr16(p1);
      x2 = ds_tr16(p2);
      f.h = __builtin_bit_cast(bfx8, make_uint4(x1.x, x1.y, x2.x, x2.y));
      x1 = ds_tr16(p1 + plane);
      x2 = ds_tr16(p2 + plane);
      f.m = __builtin_bit_cast(bfx8, make_uint4(x1.x, x1.y, x2.x, x2.y));
      x1 = ds_tr16(p1 + 2 * plane);
      x2 = ds_tr16(p2 + 2 * plane);
      f.l = __builtin_bit_cast(bfx8, make_uint4(x1.x, x1.y, x2.x, x2.y));
    }
    return f;
  };
  auto compute = [&](int buf) {
    if constexpr (SS) {
      const char* As = reinterpret_cast<const char*>(lds) + buf * (GS::SA + GS::SB);
      const char* Bs = As + GS::SA;
      using KA = std::integral_constant<bool, P::A_KMAJ>;
      using KB = std::integral_constant<bool, P::B_KMAJ>;
      using WA = std::integral_constant<int, P::A_KMAJ ? G::BK : G::BM>;
      using WB = std::integral_constant<int, P::B_KMAJ ? G::BK : G::BN>;
#pragma unroll
      for (int s = 0; s < G::BK / 16; ++s) {
        Split8 a[G::TM], b[G::TN];
#pragma unroll
        for (int mi = 0; mi < G::TM; ++mi) a[mi] = ss_frag(As, GS::PLA, KA{}, WA{}, wm * G::WTM + mi * 32, s);
#pragma unroll
        for (int ni = 0; ni < G::TN; ++ni) b[ni] = ss_frag(Bs, GS::PLB, KB{}, WB{}, wn * G::WTN + ni * 32, s);
#pragma unroll
        for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < G::TN; ++ni) {
            f32x16 x = accx[mi][ni];
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].l, b[ni].h, x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].m, b[ni].m, x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].h, b[ni].l, x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].m, b[ni].h, x, 0, 0, 0);
            x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].h, b[ni].m, x, 0, 0, 0);
            accx[mi][ni] = x;
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].h, b[ni].h, acc[mi][ni], 0, 0, 0);
          }
      }
      return;
    }
    const float* As = lds + buf * (G::SA + G::SB);
    const float* Bs = As + G::SA;
    static_assert(G::BK % 16 == 0, "k-blocks of 16");
    // 16 k per step: lane (r, h) holds k = 4h..4h+3 of chunk kc and of chunk kc + 1 -> bf16
    // k-slots 8h..8h+7 of the 32x32x16 MFMA (the same slot map for A and B)
#pragma unroll
    for (int kc = 0; kc < G::BK / 8; kc += 2) {
      Split8 a[G::TM], b[G::TN];
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi) a[mi] = split8(frag_a(As, mi, kc), frag_a(As, mi, kc + 1));
#pragma unroll
      for (int ni = 0; ni < G::TN; ++ni) b[ni] = split8(frag_b(Bs, ni, kc), frag_b(Bs, ni, kc + 1));
#pragma unroll
      for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < G::TN; ++ni) {
          f32x16 x = accx[mi][ni];
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].l, b[ni].h, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].m, b[ni].m, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].h, b[ni].l, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].m, b[ni].h, x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].h, b[ni].m, x, 0, 0, 0);
          accx[mi][ni] = x;
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi].h, b[ni].h, acc[mi][ni], 0, 0, 0);
        }
    }
  };

  int kb = ctx.kb0;
  int cur = 0;
  if (kb < ctx.kb1) {
    gload(kb, S0{});
    sstore(0, S0{});
  }
  __syncthreads();
  if constexpr (SS == 2) {  // one LDS image (half the footprint): the next k-block waits in
                            // registers and is stored after a second barrier
    for (; kb < ctx.kb1; ++kb) {
      const bool more = kb + 1 < ctx.kb1;
      if (more) gload(kb + 1, S0{});
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      if (more) {
        __syncthreads();
        sstore(0, S0{});
      }
      __syncthreads();
    }
  } else
  for (; kb < ctx.kb1; ++kb) {
    const bool more = kb + 1 < ctx.kb1;
    if (more) gload(kb + 1, S0{});
    // every MFMA of the block is issued before the LDS store waits on the next block's
    // global loads: unfenced, the scheduler sinks late-needed loads next to their store and
    // exposes their latency
    __builtin_amdgcn_sched_barrier(0);
    compute(cur);
    if (more) sstore(cur ^ 1, S0{});
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni) acc[mi][ni] += accx[mi][ni];

#pragma unroll
  for (int mi = 0; mi < G::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < G::TN; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
        P::store(args, ctx, wm * G::WTM + mi * 32 + row, wn * G::WTN + ni * 32 + r, acc[mi][ni][e]);
      }

  if constexpr (COLSUM) {
    if (P::want_colsum(ctx)) {  // block-uniform
      // the last loop barrier retired every LDS read: reuse the tile buffer
      *reinterpret_cast<f32x4*>(lds + 4 * t) = csum;
      __syncthreads();
      if (t < G::BM) {
        const int c4 = t >> 2, comp = t & 3;
        float s = 0.f;
        for (int g = 0; g < 256 / G::RA; ++g) s += lds[4 * (c4 + g * G::RA) + comp];  // fixed order
        P::store_colsum(args, ctx, t, s);
      }
    }
  }
}


template <int A, int B>
struct MaxI {
  static constexpr int value = A > B ? A : B;
};
// form SS: 0 = register split (Geo image), 1 = stage-split double buffer, 2 = stage-split single
// buffer, 3 = form 2 compiled for >= 3 waves per SIMD (amdgpu_waves_per_eu: the 128 x 64 conv2
// tile 204 -> 150 VGPRs, the others 104 -> 92, no spills)
template <class P, int SS>
struct LdsFloats {
  static constexpr int value =
      SS ? MaxI<GeoS<P>::LDS_BYTES / (SS >= 2 ? 8 : 4), 4 * 256>::value : Geo<P>::LDS_FLOATS;
};
template <int SS>
struct BodyForm {
  static constexpr int value = SS == 3 ? 2 : SS;
};

template <class P, int SS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SS == 3 ? 3 : 1))) void gemm_k(
    typename P::Args args) {
  __shared__ __attribute__((aligned(16))) float lds[LdsFloats<P, SS>::value];
  __shared__ typename P::Smem sm;
  gemm_body<P, BodyForm<SS>::value>(args, xcd_chunk(blockIdx.x, gridDim.x), lds, sm);
}

// Two independent GEMMs in one launch: blocks [0, n1) run P1, the rest P2 (P1 first: the
// longer per-block problem starts early).
// r (stage > 0): the learner's priority-tree write riding the launch as extra workgroups
// (tree_dev.h tree_ride: the leaves in block 0, a level's recompute past the GEMM tiles).
template <class P1, class P2, int SS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SS == 3 ? 3 : 1))) void gemm2_k(
    typename P1::Args a1, typename P2::Args a2, int n1, TreeRide r) {
  __shared__ __attribute__((aligned(16))) float lds[MaxI<LdsFloats<P1, SS>::value, LdsFloats<P2, SS>::value>::value];
  __shared__ union {
    typename P1::Smem s1;
    typename P2::Smem s2;
  } sm;
  int b = blockIdx.x;
  if (r.stage && tree_ride(r, r.nhost, lds, &b)) return;  // (grid-uniform stage, block-uniform role)
  if (b < n1)
    gemm_body<P1, BodyForm<SS>::value>(a1, b, lds, sm.s1);
  else
    gemm_body<P2, BodyForm<SS>::value>(a2, b - n1, lds, sm.s2);
}

__device__ __forceinline__ F32Prob pick(const F32Set& s, int i) {
  return i == 0 ? s.p[0] : (i == 1 ? s.p[1] : s.p[2]);
}

// ------------------------------------------------------------------ forward policies
template <int BM_, int BN_, int BK_, int WM_>
struct Conv2FwdT {  // a2 = relu(conv(a1, W2) + b2); k = (ky, kx, ci) = tap * 32 + ci; w = w2p
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  static constexpr bool A_KMAJ = true, B_KMAJ = true, SMEM = false;
  static_assert(512 % BK == 0 && BN <= 64, "k-blocks tile K = 512");
  using Args = F32Set;
  using Smem = NoSmem;
  struct Ctx {
    F32Prob p;
    int M, m0, n0, kb0, kb1;
    Rsrc in, w;
  };
  static constexpr int NT = 64 / BN;
  static __host__ __device__ int tiles(int B) { return NT * ((B * 81 + BM - 1) / BM); }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    const int tp = tiles(a.B);
    c.p = pick(a, block / tp);
    c.M = a.B * 81;
    const int t = block % tp;
    c.m0 = (t / NT) * BM;
    c.n0 = (t % NT) * BN;
    c.kb0 = 0;
    c.kb1 = 512 / BK;
    c.in = make_rsrc(c.p.in, (uint32_t)a.B * 400 * 32 * 4);
    c.w = make_rsrc(c.p.w, 64 * 512 * 4);
  }
  static __device__ f32x4 load_a(const Args&, const Ctx& c, const Smem&, int kb, int row, int ch) {
    const int m = c.m0 + row;
    if (m >= c.M) return zero4();
    const int k = kb * BK + 4 * ch, tap = k >> 5, ci = k & 31, ky = tap >> 2, kx = tap & 3;
    const int b = m / 81, p = m - b * 81, oy = p / 9, ox = p - oy * 9;
    const float* in = static_cast<const float*>(c.p.in);
    return ld4(in + ((size_t)b * 400 + (2 * oy + ky) * 20 + 2 * ox + kx) * 32 + ci);
  }
  static __device__ f32x4 load_b(const Args&, const Ctx& c, const Smem&, int kb, int n, int ch) {
    return ld4(c.p.w + (c.n0 + n) * 512 + kb * BK + 4 * ch);
  }
  // row states (32 % BK == 0: a k-block lies inside one tap; 4*ch is the chunk's channel
  // offset within the block, the block's tap / channel base is wave-uniform): byte offsets into
  // raw buffers -- rows past the last sample lie past the range and load zeros
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    static_assert(32 % BK == 0, "a k-block inside one tap");
    const int m = c.m0 + row;
    const int b = m / 81, p = m - b * 81, oy = p / 9, ox = p - oy * 9;
    return {(uint32_t)(((b * 400 + 2 * oy * 20 + 2 * ox) * 32 + 4 * ch) * 4)};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    const int k0 = kb * BK, tap = k0 >> 5, ky = tap >> 2, kx = tap & 3;  // wave-uniform
    return bld4(c.in, r.off + (uint32_t)(((ky * 20 + kx) * 32 + (k0 & 31)) * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int n, int ch) {
    return {(uint32_t)(((c.n0 + n) * 512 + 4 * ch) * 4)};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    return bld4(c.w, r.off + (uint32_t)(kb * BK * 4));
  }
  static __device__ void store(const Args&, const Ctx& c, int ml, int n, float v) {
    const int m = c.m0 + ml;
    if (m < c.M) c.p.out[(size_t)m * 64 + c.n0 + n] = fmaxf(v + c.p.bias[c.n0 + n], 0.f);
  }
};

template <int BM_, int BN_, int BK_, int WM_>
struct Conv3FwdT {  // a3 = relu(conv(a2, W3) + b3); k = tap * 64 + ci; w = w3p
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  static constexpr bool A_KMAJ = true, B_KMAJ = true, SMEM = false;
  static_assert(576 % BK == 0 && 64 % BK == 0 || BK == 64, "a k-block stays inside one tap");
  using Args = F32Set;
  using Smem = NoSmem;
  struct Ctx {
    F32Prob p;
    int M, m0, n0, kb0, kb1;
    Rsrc in, w;
  };
  static constexpr int NT = 64 / BN;
  static __host__ __device__ int tiles(int B) { return NT * ((B * 49 + BM - 1) / BM); }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    const int tp = tiles(a.B);
    c.p = pick(a, block / tp);
    c.M = a.B * 49;
    const int t = block % tp;
    c.m0 = (t / NT) * BM;
    c.n0 = (t % NT) * BN;
    c.kb0 = 0;
    c.kb1 = 576 / BK;
    c.in = make_rsrc(c.p.in, (uint32_t)a.B * 81 * 64 * 4);
    c.w = make_rsrc(c.p.w, 64 * 576 * 4);
  }
  static __device__ f32x4 load_a(const Args&, const Ctx& c, const Smem&, int kb, int row, int ch) {
    const int m = c.m0 + row;
    if (m >= c.M) return zero4();
    const int k = kb * BK + 4 * ch, tap = k >> 6, ci = k & 63, ky = tap / 3, kx = tap - ky * 3;
    const int b = m / 49, p = m - b * 49, oy = p / 7, ox = p - oy * 7;
    const float* in = static_cast<const float*>(c.p.in);
    return ld4(in + ((size_t)b * 81 + (oy + ky) * 9 + ox + kx) * 64 + ci);
  }
  static __device__ f32x4 load_b(const Args&, const Ctx& c, const Smem&, int kb, int n, int ch) {
    return ld4(c.p.w + (c.n0 + n) * 576 + kb * BK + 4 * ch);
  }
  // row states (64 % BK == 0: a k-block lies inside one tap of 64 channels, chunk 4*ch): byte
  // offsets into raw buffers (rows past the last sample: past the range, zeros)
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    static_assert(64 % BK == 0, "a k-block inside one tap");
    const int m = c.m0 + row;
    const int b = m / 49, p = m - b * 49, oy = p / 7, ox = p - oy * 7;
    return {(uint32_t)(((b * 81 + oy * 9 + ox) * 64 + 4 * ch) * 4)};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    const int k0 = kb * BK, tap = k0 >> 6, ky = tap / 3, kx = tap - ky * 3;  // wave-uniform
    return bld4(c.in, r.off + (uint32_t)(((ky * 9 + kx) * 64 + (k0 & 63)) * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int n, int ch) {
    return {(uint32_t)(((c.n0 + n) * 576 + 4 * ch) * 4)};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    return bld4(c.w, r.off + (uint32_t)(kb * BK * 4));
  }
  static __device__ void store(const Args&, const Ctx& c, int ml, int n, float v) {
    const int m = c.m0 + ml;
    if (m < c.M) c.p.out[(size_t)m * 64 + c.n0 + n] = fmaxf(v + c.p.bias[c.n0 + n], 0.f);
  }
};

constexpr int kFcSplits = 7;  // FC1 forward split-K: 3136 = 7 x 448 (14 splits: FC1 34.6 -> 30.9 us but the heads kernel reduces twice the slabs: step neutral)
template <int BM_, int BN_, int BK_, int WM_>
struct Fc1FwdT {  // z[s][b][n] = sum_{k' in split s} a3[b][k'] wfc1p[n][k'], k' = p*64 + c
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  static constexpr bool A_KMAJ = true, B_KMAJ = true, SMEM = false;
  static constexpr int KBS = 3136 / BK / kFcSplits;  // k-blocks per split
  static_assert(KBS * BK * kFcSplits == 3136 && 256 % BN == 0, "split-K tiling");
  static constexpr int NT = 256 / BN;
  using Args = F32Set;
  using Smem = NoSmem;
  struct Ctx {
    F32Prob p;
    int B, m0, n0, split, kb0, kb1;
    Rsrc in, w;
  };
  static __host__ __device__ int tiles(int B) { return ((B + BM - 1) / BM) * NT * kFcSplits; }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    const int tp = tiles(a.B);
    c.p = pick(a, block / tp);
    int t = block % tp;
    c.B = a.B;
    c.n0 = (t % NT) * BN;
    t /= NT;
    c.split = t % kFcSplits;
    c.m0 = (t / kFcSplits) * BM;
    c.kb0 = c.split * KBS;
    c.kb1 = c.kb0 + KBS;
    c.in = make_rsrc(c.p.in, (uint32_t)a.B * 3136 * 4);
    c.w = make_rsrc(c.p.w, 256 * 3136 * 4);
  }
  static __device__ f32x4 load_a(const Args&, const Ctx& c, const Smem&, int kb, int row, int ch) {
    const int b = c.m0 + row;
    if (b >= c.B) return zero4();
    return ld4(static_cast<const float*>(c.p.in) + (size_t)b * 3136 + kb * BK + 4 * ch);
  }
  static __device__ f32x4 load_b(const Args&, const Ctx& c, const Smem&, int kb, int nl, int ch) {
    return ld4(c.p.w + (size_t)(c.n0 + nl) * 3136 + kb * BK + 4 * ch);
  }
  static __device__ void store(const Args&, const Ctx& c, int ml, int nl, float v) {
    const int b = c.m0 + ml;
    if (b < c.B) c.p.out[((size_t)c.split * c.B + b) * 256 + c.n0 + nl] = v;
  }
  // row states: the chunk's k-invariant byte offsets (rows past the batch: past the range, zeros)
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)(((c.m0 + row) * 3136 + 4 * ch) * 4)};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    return bld4(c.in, r.off + (uint32_t)(kb * BK * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int nl, int ch) {
    return {(uint32_t)(((c.n0 + nl) * 3136 + 4 * ch) * 4)};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    return bld4(c.w, r.off + (uint32_t)(kb * BK * 4));
  }
};

constexpr int kPlaneDw = kPlane / 4;  // 1764 dwords per plane

// conv1 forward at reference precision on the bf16 matrix cores (exact three-term split).
//  * Input pixels are u8 (0..255, 8 significant bits): exactly representable in bf16.
//  * An fp32 weight splits EXACTLY into three bf16 terms by truncation: hi = w with its low
//    16 bits cleared, mid = (w - hi) likewise, lo = w - hi - mid (each subtraction is exact;
//    lo has <= 8 significant bits).  A bf16 x bf16 product is exact in fp32.
//  So x*w = x*hi + x*mid + x*lo with every product exact, accumulated in fp32 -- the hi
//  products, the mid products and the lo products (2^-8 and 2^-16 smaller) in three
//  accumulators, summed small-to-large at the end, so the extra terms add no rounding at the
//  fp32 chain's scale (error vs fp64: tests/test_gpu_f32_net.py).  On v_mfma_f32_16x16x32_bf16
//  (16 cycles per 16x16x32) the 3 terms cost 48 cycles where v_mfma_f32_16x16x4_f32 pays
//  8 x 32 = 256 for the same 16x16x32 of fp32: 5.3x fewer MFMA cycles.
//  Persistent over samples, two workgroups per CU (56 KB of LDS each: the sample's four
//  planes as bf16, converted once while staging); the weight split is redone only when
//  the problem changes.  Wave w: channels 16 (w >> 1) .. +15, output tiles w & 1, +2, ...
//  of 16 pixels; lane (i = l & 15, q = l >> 4) holds A[pixel i][k = 8q + j] = plane c =
//  kb >> 1, row 4 oy + 4 (kb & 1) + q, columns 4 ox + j: 8 consecutive bf16 of one row.
struct W1Split {
  bfx8 hi[8], mid[8], lo[8];
};

// this lane's weight fragments for all 8 k-blocks, split into 3 terms.  k order inside a
// k-block (input channel kb >> 1, kernel rows 4 (kb & 1) .. +3): lane group q = 2 p + h holds
// rows 2p, 2p + 1 (j >> 2) x columns 4h .. 4h + 3 (j & 3) -- see f32_conv1_fwd_x3_k's fragments;
// wrow = W1 row + (2p) * 8 + 4h
__device__ __forceinline__ void split_w1(const float* wrow, W1Split& w) {
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    const f32x4 v0 = ld4(wrow + 32 * kb), v1 = ld4(wrow + 32 * kb + 8);
    const float x[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = x[2 * j], b = x[2 * j + 1];
      const float ah = trunc_bf16(a), bh = trunc_bf16(b);
      const float ar = a - ah, br = b - bh;
      const float am = trunc_bf16(ar), bm = trunc_bf16(br);
      h[j] = pack_bf16_hi(ah, bh);
      m[j] = pack_bf16_hi(am, bm);
      l[j] = pack_bf16_hi(ar - am, br - bm);  // exact: <= 8 significant bits
    }
    w.hi[kb] = __builtin_bit_cast(bfx8, make_uint4(h[0], h[1], h[2], h[3]));
    w.mid[kb] = __builtin_bit_cast(bfx8, make_uint4(m[0], m[1], m[2], m[3]));
    w.lo[kb] = __builtin_bit_cast(bfx8, make_uint4(l[0], l[1], l[2], l[3]));
  }
}

// (A double-buffered 512-thread variant -- one workgroup per CU, the next sample staged from
// inside the MFMA loop -- timed 42.9-43.5 vs 46.4-47.4 us alone but cost the whole learner step
// ~3 % (2063-2067 vs 2125-2131 steps/s, scripts/ab/conv1_fullstep_ab.sh): its 113 KB of LDS per
// CU leave no room for the actor graph's kernels running beside it.)
// two workgroups per CU, each walking a contiguous run of samples (next sample prefetched):
// 512 / 1024 workgroups 42.2 / 41.5-43.9 us, one sample per workgroup (1536) 44.4-45.0 us
// (3 x 512 samples, interleaved on one box)
constexpr int kC1xGrid = 512;
// the learner's 3 x 512 samples on 384 workgroups (4 each): with the PER draw folded in, the
// 512-workgroup launch filled every CU's LDS (2 x 56 KB) from the step's first microsecond and
// starved the actor graph's conv1 beside it (the sampling launch used to give it a head start):
// whole step, alternated on one box, draw folded at 384 / 448 / 320 / 512 workgroups 2546.5 /
// 2549.8 / 2441.3 / 2446.5 (another box), sampling launch + 512: 2525.3 (profiles/r6_step_kernels.md)
constexpr int kC1xGridLearner = 384;
// small launches (the actor's 256 envs beside the learner's forward) at 2 samples per workgroup:
// 128 workgroups 2566.9, 256 (one sample each, the round-5 shape) 2466.3, 192 2517.0, 96 2538.1,
// 64 2492.0 learner steps/s (one box, alternated; profiles/r6_step_kernels.md)
constexpr int kC1xDrawMax = 8;  // samples per workgroup with the folded draw (2 per wave)
constexpr int kC1xChunks = 4 * (kPlane / 16), kC1xPer = (kC1xChunks + 255) / 256;  // 16-byte u8 chunks

// the sample's 4 x 441 16-byte u8 chunks -> registers (issued, not waited on); fid (the folded
// draw): the sample's 4 frame ids, drawn by this workgroup
__device__ __forceinline__ void c1x_load(const F32Set& set, int smp, uint4 (&v)[kC1xPer], const int* fid) {
  const int B = set.B, prob = smp / B, b = smp - prob * B, t = threadIdx.x;
  const F32Prob p = pick(set, prob);
  const uint8_t* fr = static_cast<const uint8_t*>(p.in);
  const FrameSrc f{fr, p.ids, p.idx};
  const uint4* s0 = reinterpret_cast<const uint4*>(fid ? fr + (size_t)fid[0] * kPlane : frame_plane(f, b, 0, kPlane));
  const uint4* s1 = reinterpret_cast<const uint4*>(fid ? fr + (size_t)fid[1] * kPlane : frame_plane(f, b, 1, kPlane));
  const uint4* s2 = reinterpret_cast<const uint4*>(fid ? fr + (size_t)fid[2] * kPlane : frame_plane(f, b, 2, kPlane));
  const uint4* s3 = reinterpret_cast<const uint4*>(fid ? fr + (size_t)fid[3] * kPlane : frame_plane(f, b, 3, kPlane));
#pragma unroll
  for (int k = 0; k < kC1xPer; ++k) {  // (no dynamically indexed pointer array: it would live in scratch)
    const int e = min(t + 256 * k, kC1xChunks - 1), c = e / 441;  // tail lanes reload a valid chunk
    const uint4* sc = c == 0 ? s0 : (c == 1 ? s1 : (c == 2 ? s2 : s3));
    v[k] = sc[e - c * 441];
  }
}

// registers -> LDS as bf16: chunk e = bf16 elements 16e .. 16e + 15 (7056 = 441 x 16)
__device__ __forceinline__ void c1x_store(const uint4 (&v)[kC1xPer], uint32_t* xs) {
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kC1xPer; ++k) {
    const int e = t + 256 * k;
    if (e < kC1xChunks) {
      const f32x4 a = u8x4(v[k].x), bq = u8x4(v[k].y), c = u8x4(v[k].z), d = u8x4(v[k].w);
      uint4* dst = reinterpret_cast<uint4*>(xs) + 2 * e;
      dst[0] = make_uint4(pack_bf16_hi(a[0], a[1]), pack_bf16_hi(a[2], a[3]), pack_bf16_hi(bq[0], bq[1]),
                          pack_bf16_hi(bq[2], bq[3]));
      dst[1] = make_uint4(pack_bf16_hi(c[0], c[1]), pack_bf16_hi(c[2], c[3]), pack_bf16_hi(d[0], d[1]),
                          pack_bf16_hi(d[2], d[3]));
    }
  }
}

// Software-pipelined over the workgroup's samples: the next sample's frame chunks are
// loaded into registers before this sample's MFMA loop, so the frame-ring (HBM) latency
// hides behind compute; they are converted into LDS after the loop.
// The two 8-byte halves of a pixel fragment load as two ds_read_b64 (2 LDS cycles each,
// 256 B/clk) instead of the ds_read2_b64 the compiler would merge them into (8 cycles,
// 128 B/clk): the second address is hidden from the load/store merger (one v_add per fragment;
// MI355X, 3 x 512 samples: 44.6 vs 46.5 us)
__device__ __forceinline__ int opaque_i(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
// cs.out_idx (the learner): the PER draw folded in -- wave k draws sample s0 + k's slot (the
// per_sample_k descent, same arithmetic: identical slots and IS weights) and its 4 frame ids go
// to LDS before the first frame load; workgroups past cs.nhost scatter the staged actor rows.
__global__ __launch_bounds__(256, 2) void f32_conv1_fwd_x3_k(F32Set set, ConvSample cs) {
  __shared__ __attribute__((aligned(16))) uint32_t xs[2 * kPlaneDw * 4];  // 4 planes of bf16
  __shared__ int fid[kC1xDrawMax][4];  // (the draw) frame ids of the workgroup's samples
  const int B = set.B, total = set.n * B;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i = lane & 15, q = lane >> 4, nh = wave >> 1;
  const bool draw = cs.out_idx != nullptr;  // grid-uniform
  const int G = draw ? cs.nhost : (int)gridDim.x;
  if (draw && (int)blockIdx.x >= G) {  // block-uniform: the staged-row scatter
    staged_scatter(cs.rows, blockIdx.x - G);
    return;
  }
  const __bf16* xb = reinterpret_cast<const __bf16*>(xs);
  W1Split w;
  int cur = -1;
  uint4 v[kC1xPer];
  // a contiguous run of samples per workgroup: the weight split is redone only at a
  // problem boundary (a grid-strided walk crossed one at every sample: ~25 % of the VALU)
  const int per = (total + G - 1) / G;
  const int s0 = blockIdx.x * per, s1 = min(total, s0 + per);
  if (draw) {  // (per <= kC1xDrawMax: checked by the launcher)
    for (int k = wave; k < s1 - s0; k += 4) {  // wave-uniform
      const int smp = s0 + k, prob = smp / B, b = smp - prob * B;
      const int64_t len64 = cs.length[0];
      const int length = (int)(len64 < (int64_t)cs.t.size[0] ? len64 : (int64_t)cs.t.size[0]);
      const float pmin = cs.t.node_min[cs.t.levels - 1][0];
      float p;
      const int node = tree_sample_leaf(cs.t, b, B, length, cs.exclude_last, cs.seed, (uint64_t)cs.counter[0], lane,
                                        &p);
      const int se = staged_row_of(cs.rows, node, lane);
      const F32Prob pp = pick(set, prob);
      const int* ids = se < 0 ? pp.ids : (pp.ids == cs.rows.dst.s_ids ? cs.rows.st.s_ids : cs.rows.st.s2_ids);
      if (lane < 4) fid[k][lane] = ids[4 * (se < 0 ? node : se) + lane];
      if (prob == 0 && lane == 0) {
        cs.out_idx[b] = node;
        cs.out_w[b] = per_is_weight(p, pmin, 1.f, cs.beta[0]);
      }
    }
    __syncthreads();
  }
  if (s0 < s1) c1x_load(set, s0, v, draw ? fid[0] : nullptr);
  for (int smp = s0; smp < s1; ++smp) {
    const int prob = smp / B, b = smp - prob * B;
    const F32Prob p = pick(set, prob);
    if (prob != cur) {  // block-uniform
      cur = prob;
      split_w1(p.w + (nh * 16 + i) * 256 + (q >> 1) * 16 + (q & 1) * 4, w);
    }
    __syncthreads();  // the previous sample's tiles are done with xs
    c1x_store(v, xs);
    __syncthreads();
    if (smp + 1 < s1) c1x_load(set, smp + 1, v, draw ? fid[smp + 1 - s0] : nullptr);  // in flight during the MFMAs
    // roles swapped on the MFMA (A = the weight slice, B = the pixels: identical lane maps),
    // so lane (i, q) ends with channels 4q .. 4q+3 of pixel i -- one 16-byte store
    float* out = p.out + (size_t)b * 400 * 32 + nh * 16 + 4 * q;
    float4 bias4;
    bias4.x = p.bias[nh * 16 + 4 * q];
    bias4.y = p.bias[nh * 16 + 4 * q + 1];
    bias4.z = p.bias[nh * 16 + 4 * q + 2];
    bias4.w = p.bias[nh * 16 + 4 * q + 3];
    // pixel fragments: lane (i, q = 2p + h) reads 4 columns 4 ox + 4h .. +3 of kernel rows 2p and
    // 2p + 1 (two ds_read_b64, 42 dwords apart).  Within a 32-lane LDS group (q = 0, 1) lane
    // (ox, h = 1) reads the same dwords as lane (ox + 1, h = 0) -- stride-4 windows overlap by 4
    // columns -- so the group touches ~34 consecutive dwords and broadcasts the rest: no bank
    // conflicts (rows in the lane groups gave 1.84 conflict cycles per LDS cycle)
    auto frags = [&](int tile, bfx8 (&a)[8]) {
      const int m = tile * 16 + i, oy = m / 20, ox = m - oy * 20;
      const __bf16* a0 = xb + (4 * oy + 2 * (q >> 1)) * 84 + 4 * ox + 4 * (q & 1);
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {  // 8-byte aligned: two ds_read_b64
        const uint2* ap = reinterpret_cast<const uint2*>(a0 + (kb >> 1) * kPlane + (kb & 1) * 4 * 84);
        const uint2 lo = ap[0], hi = ap[opaque_i(21)];  // next kernel row (84 bf16 = 21 x 8 bytes)
        a[kb] = __builtin_bit_cast(bfx8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
    };
    auto tile_mfma = [&](int tile, const bfx8 (&a)[8]) {
      // three accumulators (hi / mid / lo products): no MFMA waits on its predecessor's result
      f32x4 ah = zero4(), am = zero4(), al = zero4();
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        ah = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.hi[kb], a[kb], ah, 0, 0, 0);
        am = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.mid[kb], a[kb], am, 0, 0, 0);
        al = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w.lo[kb], a[kb], al, 0, 0, 0);
      }
      float4 y;
      y.x = fmaxf(ah[0] + (am[0] + al[0]) + bias4.x, 0.f);
      y.y = fmaxf(ah[1] + (am[1] + al[1]) + bias4.y, 0.f);
      y.z = fmaxf(ah[2] + (am[2] + al[2]) + bias4.z, 0.f);
      y.w = fmaxf(ah[3] + (am[3] + al[3]) + bias4.w, 0.f);
      *reinterpret_cast<float4*>(out + (size_t)(tile * 16 + i) * 32) = y;
    };
    // ping-pong fragment buffers: the next tile's LDS reads are in flight during this tile's MFMAs.
    // Wave parity t0 owns tiles t0, t0 + 2, ...: 6 pairs (+ tile 24 for t0 = 0); every fragment
    // load is unconditional (the one past parity 1's last tile re-reads tile 24, unused), so the
    // buffers keep fixed registers (guarded loads + a mid-loop exit made the compiler copy them)
    bfx8 fa[8], fb[8];
    const int t0 = wave & 1;
    frags(t0, fa);
    for (int pr = 0; pr < 6; ++pr) {
      const int tile = t0 + 4 * pr;
      frags(tile + 2, fb);
      tile_mfma(tile, fa);
      frags(min(tile + 4, 24), fa);
      tile_mfma(tile + 2, fb);
    }
    if (t0 == 0) tile_mfma(24, fa);
  }
}

// ------------------------------------------------------------------ backward policies
struct BwdArgs {
  const void* x;        // layer input (u8 frames for conv1: FrameSrc fields)
  const int* ids;
  const int* idx;
  const float* dy;      // gradient w.r.t. the layer's (post-ReLU-masked) output
  const float* w;       // packed weights: wfc1p (FC1 dgrad), w3t / w2t (conv dgrad)
  const float* mask;    // post-ReLU activation of the layer below (dgrad ReLU backward)
  float* out;           // dgrad output | wgrad partials / FC1 advantage grad
  float* out2;          // wgrad bias partials | FC1 value grad
  int B;
  int kbps;             // wgrad: k-blocks per split
  int splits;
};

struct Fc1Dgrad {  // dy3[b][k'] = (a3 > 0) * sum_n dz[b][n] wfc1p[n][k']
  static constexpr int BM = 64, BN = 64, BK = 32, WM = 2;
  static constexpr bool A_KMAJ = true, B_KMAJ = false, SMEM = false;
  using Args = BwdArgs;
  using Smem = NoSmem;
  struct Ctx {
    int m0, n0, kb0, kb1;
    Rsrc dy, w;
  };
  static __host__ __device__ int tiles(int B) { return ((B + BM - 1) / BM) * 49; }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    c.n0 = (block % 49) * BN;
    c.m0 = (block / 49) * BM;
    c.kb0 = 0;
    c.kb1 = 256 / BK;
    c.dy = make_rsrc(a.dy, (uint32_t)a.B * 256 * 4);
    c.w = make_rsrc(a.w, 256 * 3136 * 4);
  }
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)((c.m0 + row) * 256 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    return bld4(c.dy, r.off + (uint32_t)(kb * BK * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)(row * 3136 + c.n0 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    return bld4(c.w, r.off + (uint32_t)(kb * BK * 3136 * 4));
  }
  static __device__ void store(const Args& a, const Ctx& c, int ml, int nl, float v) {
    const int b = c.m0 + ml;
    if (b >= a.B) return;
    const size_t o = (size_t)b * 3136 + c.n0 + nl;
    a.out[o] = a.mask[o] > 0.f ? v : 0.f;
  }
};

struct Fc1Wgrad {  // dW[n][k'] = sum_b dz[b][n] a3[b][k'], stored to the reference [n][c*49 + p]
  // a.splits > 0: the batch is split into a.splits slices of a.kbps k-blocks (196 tiles per
  // slice) and each slice writes its partial in the natural [n][p*64 + c] order to
  // a.out[slice][256][3136]; grad_finalize's FC1 row job sums the slices in a fixed order and
  // transposes (f32_fc1_finalize_job).  a.splits == 0: one pass, the reference-layout grads
  // written in place (a.out = advantage rows, a.out2 = value rows).
  static constexpr int BM = 64, BN = 64, BK = 32, WM = 2;
  static constexpr bool A_KMAJ = false, B_KMAJ = false, SMEM = false;
  using Args = BwdArgs;
  using Smem = NoSmem;
  struct Ctx {
    int m0, n0, kb0, kb1, split;
    Rsrc dy, x;
  };
  static __host__ __device__ int tiles(int) { return 4 * 49; }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    const int t = block % (4 * 49);
    c.split = block / (4 * 49);
    c.n0 = (t % 49) * BN;
    c.m0 = (t / 49) * BM;
    const int nkb = (a.B + BK - 1) / BK;
    c.kb0 = a.splits > 0 ? c.split * a.kbps : 0;
    c.kb1 = a.splits > 0 ? min(nkb, c.kb0 + a.kbps) : nkb;
    c.dy = make_rsrc(a.dy, (uint32_t)a.B * 256 * 4);
    c.x = make_rsrc(a.x, (uint32_t)a.B * 3136 * 4);
  }
  // k = sample: chunk rows are samples kb * BK + row (past the batch: past the range)
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)(row * 256 + c.m0 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    return bld4(c.dy, r.off + (uint32_t)(kb * BK * 256 * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)(row * 3136 + c.n0 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    return bld4(c.x, r.off + (uint32_t)(kb * BK * 3136 * 4));
  }
  static __device__ void store(const Args& a, const Ctx& c, int ml, int nl, float v) {
    const int n = c.m0 + ml, k = c.n0 + nl;
    if (a.splits > 0) {  // coalesced natural-order partial
      a.out[((size_t)c.split * 256 + n) * 3136 + k] = v;
      return;
    }
    // scattered stores (write-combined in L2) instead of gathered operand loads
    const int ref = (k & 63) * 49 + (k >> 6);
    if (n < 128) a.out[n * 3136 + ref] = v;
    else a.out2[(n - 128) * 3136 + ref] = v;
  }
};

// conv wgrad (layers 2, 3): part[s][co][tap*C + ci] = sum_{rows in split s} dy[row][co] x_col[row][tap, ci]
// with POSITION-MAJOR rows: k-block kb = (output position p, block of 32 samples), so the
// im2col address of a row is (sample) * plane + (position, tap) offset -- the position is
// uniform per k-block (scalar), where sample-major rows paid ~30 VALU per 16-byte load
// dividing the row index by P and OH (MI355X: conv3 wgrad 45 -> see profiles).
template <int L>
struct ConvWgrad {
  static constexpr int C = L == 3 ? 64 : 32, K = L == 3 ? 3 : 4, S = L == 3 ? 1 : 2;
  static constexpr int IH = L == 3 ? 9 : 20, OH = L == 3 ? 7 : 9, P = OH * OH;
  static constexpr int N = K * K * C;
  static constexpr int BM = 64, BN = 64, BK = 32, WM = 2;
  static_assert(N % BN == 0, "whole tiles");
  static constexpr bool A_KMAJ = false, B_KMAJ = false, SMEM = false, A_COLSUM = true;
  using Args = BwdArgs;
  using Smem = NoSmem;
  struct Ctx {
    int n0, split, kb0, kb1, nbb;
    Rsrc dy, x;
  };
  static __host__ __device__ int kblocks(int B) { return P * ((B + BK - 1) / BK); }
  static __host__ __device__ int tiles(int, int splits) { return (N / BN) * splits; }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    constexpr int NT = N / BN;
    c.split = block / NT;
    c.n0 = (block % NT) * BN;
    c.nbb = (a.B + BK - 1) / BK;
    c.kb0 = c.split * a.kbps;
    c.kb1 = min(c.kb0 + a.kbps, kblocks(a.B));
    c.dy = make_rsrc(a.dy, (uint32_t)a.B * P * 64 * 4);
    c.x = make_rsrc(a.x, (uint32_t)a.B * IH * IH * C * 4);
  }
  // row states: the chunk's sample row within a 32-sample k-block (+ its channel chunk / its
  // (tap, ci) column offset) as a byte offset; the k-block adds (sample block, position)
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx&, int row, int ch) {
    return {(uint32_t)(row * P * 64 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    const int p = kb / c.nbb, bb = kb - p * c.nbb;  // wave-uniform
    return bld4(c.dy, r.off + (uint32_t)((bb * BK * P + p) * 64 * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int row, int ch) {
    const int n = c.n0 + 4 * ch, tap = n / C, ci = n - tap * C, ky = tap / K, kx = tap - ky * K;
    return {(uint32_t)(row * IH * IH * C + (ky * IH + kx) * C + ci) * 4};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    const int p = kb / c.nbb, bb = kb - p * c.nbb, oy = p / OH, ox = p - oy * OH;  // wave-uniform
    return bld4(c.x, r.off + (uint32_t)((bb * BK * IH * IH + S * oy * IH + S * ox) * C * 4));
  }
  static __device__ void store(const Args& a, const Ctx& c, int m, int nl, float v) {
    a.out[((size_t)c.split * 64 + m) * N + c.n0 + nl] = v;
  }
  static __device__ bool want_colsum(const Ctx& c) { return c.n0 == 0; }
  static __device__ void store_colsum(const Args& a, const Ctx& c, int m, float v) {
    a.out2[c.split * 64 + m] = v;
  }
};

// conv1 weight gradient, sample-resident: workgroup g (8 waves) holds samples 2g, 2g+1
// (their frame planes staged in LDS once), wave w takes sample w >> 2 and input channel
// c = w & 3, i.e. the 64 columns kk = c*64 + ky*8 + kx of dW1[32][256], as 2 (co halves) x 4
// 16x16 tiles on v_mfma_f32_16x16x4_f32 with the PIXEL as the reduction index:
//   A[i = co][slot q] = dy1[pixel p0 + q][co]              (one float per lane per 4 pixels)
//   B[slot q][j]      = frame(pixel p0 + q, kk(j, i'))      with kk = c*64 + (j >> 1)*8 + 4 (j & 1) + i'
// so ONE ds_read_b32 (4 u8 = kx 4(j&1)..+3 of row 4oy + (j >> 1)) feeds the 4 tiles i' and
// both co halves: 8 independent accumulators per 4 pixels.  The two samples' partials are
// added through LDS (fixed order) into partial g: ws[g][co][kk] + bias partials ws_b[g][co]
// (sum of dy1 over the pixels), reduced over g by grad_finalize like the other layers.
constexpr int kConv1WgradS = 2;  // default samples per workgroup (partials = ceil(B / 2))
// staging dump (dwords): the chunk loop's tail past S samples' 1764 S chunks (256 S threads)
template <int S>
constexpr int c1w_dump() {
  return 4 * (((S * 4 * (kPlane / 16) + 256 * S - 1) / (256 * S)) * 256 * S - S * 4 * (kPlane / 16));
}
// conv1 weight gradient at reference precision on bf16 MFMA (the exact split of the
// forward above, applied to dy): the u8 frame operand is exact in bf16 and each dy value
// splits exactly into hi + mid + lo bf16, so every product is exact and only the fp32
// accumulation rounds (hi, mid and lo products in separate accumulators).
// Workgroup = 8 waves = 2 samples x 4 input channels c; wave c owns columns
// kk = c*64 + (col >> 1)*8 + 4 (col & 1) + i of the 4 tiles i, both co halves, and the
// reduction runs over PIXEL GROUPS of 8 on v_mfma_f32_16x16x32_bf16: group g = (output row
// g / 3, columns 8 (g % 3) .. +7; the third group of a row has 4 real pixels, dy = 0 on the 4
// pad slots), 4 groups (lane q) per k-step, 15 k-steps per sample.  Lane (col, q) reads the
// 8 consecutive plane dwords (4oy + (col >> 1)) * 21 + ox0 + jj + (col & 1) once per k-step;
// tile i takes byte i of each (kx & 3 == i), so the 4 B fragments share one set of LDS reads.
// The A fragments (dy of the k-step's 4 groups, both co halves, as hi / mid / lo bf16) are the
// same for the sample's 4 channel waves: each wave splits ONE quarter (co half c >> 1, slots
// 4 (c & 1) .. +3) into an LDS double buffer and all four read the whole set back (6 x 16 B
// per lane), one workgroup barrier per k-step -- the split (~5 VALU per value) was 4x redundant
// and bounded the kernel (9.7 VALU per MFMA, 15 % MFMA busy, round 3).  One workgroup per CU
// either way (~180 VGPRs: 2 waves per SIMD), so the 82 KB of LDS cost no occupancy.
// S = samples per workgroup (4 S waves); S = 1 writes one partial per sample.
constexpr int kC1wAf = 2 * 3 * 64;  // uint4 per (buffer, sample): [half][term][lane]
template <int S>
__global__ __launch_bounds__(256 * S) void f32_conv1_wgrad_x3_k(BwdArgs a) {
  constexpr int NT = 256 * S;
  __shared__ __attribute__((aligned(16))) uint32_t pl[S * 4 * kPlaneDw + 16 + c1w_dump<S>()];  // + pad: row-end groups
  __shared__ uint4 af[2][S][kC1wAf];  // split dy fragments, double-buffered over k-steps
  __shared__ int64_t wplanes[S * 4];  // plane byte offsets from the frames base
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int col = lane & 15, q = lane >> 4, sl = wave >> 2, c = wave & 3;
  const int b0 = blockIdx.x * S, ns = min(S, a.B - b0);
  // this wave's quarter of every k-step's dy: co = 16 hq + col, slots j0 .. j0 + 3 of group g.
  // All 15 k-steps' values are loaded up front (60 registers), in flight with the plane
  // staging: loaded one k-step ahead, each k-step (~400 MFMA cycles) waited out most of a
  // global round trip
  const int hq = c >> 1, j0 = 4 * (c & 1);
  const bool live = sl < ns;  // a missing second sample (odd batch tail): zero dy, barriers kept
  const float* dy = a.dy + (size_t)(b0 + (live ? sl : 0)) * 400 * 32 + 16 * hq + col;
  float dyv[15][4];
#pragma unroll
  for (int ks = 0; ks < 15; ++ks) {  // unconditional loads from clamped pixel slots, zeroed at use
    const int g = 4 * ks + q, oy = g / 3, ox0 = 8 * (g - 3 * oy), nv = min(8, 20 - ox0);
    const float* dp = dy + (oy * 20 + ox0) * 32;
#pragma unroll
    for (int j = 0; j < 4; ++j) dyv[ks][j] = dp[min(j0 + j, nv - 1) * 32];
  }
  {  // stage the samples' planes (u8): S x 4 x 441 16-byte chunks
    const FrameSrc f{static_cast<const uint8_t*>(a.x), a.ids, a.idx};
    constexpr int kChunks = 4 * (kPlane / 16), kPer = (S * kChunks + NT - 1) / NT;
    // the 8 plane addresses once (frame_plane reads idx then ids: two dependent round trips,
    // paid per chunk when resolved inside the loop below)
    // (kept as offsets from the kernel-argument base: a pointer read back from LDS is a flat
    // pointer, and flat loads may alias the LDS stores below -- each waited out before its store)
    const uint8_t* fb = static_cast<const uint8_t*>(a.x);
    if (t < S * 4) wplanes[t] = frame_plane(f, b0 + min(t >> 2, ns - 1), t & 3, kPlane) - fb;
    __syncthreads();
    uint4 v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = min(t + NT * i, ns * kChunks - 1), s2 = e / kChunks, r = e - s2 * kChunks, ch = r / 441;
      v[i] = reinterpret_cast<const uint4*>(fb + wplanes[s2 * 4 + ch])[r - ch * 441];
    }
    // unconditional stores (a guarded store sank its load into the branch: one round trip per
    // chunk); the tail chunks past both samples land in the dump past the planes (and pad)
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = t + NT * i;
      reinterpret_cast<uint4*>(pl)[e < S * kChunks ? e : e + 4] = v[i];
    }
    if (t < 16) pl[S * 4 * kPlaneDw + t] = 0u;
  }
  // hi / mid / lo products in three accumulators: no MFMA waits on its predecessor's result
  f32x4 ah[2][4], am[2][4], al[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) ah[h][i] = am[h][i] = al[h][i] = zero4();
  float bs = 0.f;  // bias partial of co = 16 hq + col over this wave's slots
  auto split_store = [&](int ks, int buf) {
    const int g = 4 * ks + q, oy = g / 3, ox0 = 8 * (g - 3 * oy), nv = min(8, 20 - ox0);
    float d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d[j] = (live && j0 + j < nv) ? dyv[ks][j] : 0.f;
      bs += d[j];
    }
    uint32_t hw[2], mw[2], lw[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float x = d[2 * j], y = d[2 * j + 1];
      const float xh = trunc_bf16(x), yh = trunc_bf16(y);
      const float xr = x - xh, yr = y - yh;
      const float xm = trunc_bf16(xr), ym = trunc_bf16(yr);
      hw[j] = pack_bf16_hi(xh, yh);
      mw[j] = pack_bf16_hi(xm, ym);
      lw[j] = pack_bf16_hi(xr - xm, yr - ym);
    }
    uint32_t* base = reinterpret_cast<uint32_t*>(&af[buf][sl][hq * 3 * 64 + lane]) + (c & 1) * 2;
    *reinterpret_cast<uint2*>(base) = make_uint2(hw[0], hw[1]);
    *reinterpret_cast<uint2*>(base + 64 * 4) = make_uint2(mw[0], mw[1]);
    *reinterpret_cast<uint2*>(base + 2 * 64 * 4) = make_uint2(lw[0], lw[1]);
  };
  const uint32_t* pc = pl + (sl * 4 + c) * kPlaneDw + (col >> 1) * 21 + (col & 1);
  split_store(0, 0);
  __syncthreads();  // the planes and the first k-step's fragments are staged
#pragma unroll
  for (int ks = 0; ks < 15; ++ks) {  // unrolled: dyv[ks] stays in registers
    const int cur = ks & 1;
    const int g = 4 * ks + q, oy = g / 3, ox0 = 8 * (g - 3 * oy);
    bfx8 A[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 3; ++k) A[h][k] = __builtin_bit_cast(bfx8, af[cur][sl][(h * 3 + k) * 64 + lane]);
    // B: 8 plane dwords (pixels ox0 + jj of row 4 oy + ky), byte i -> tile i
    const uint32_t* px = pc + 4 * oy * 21 + ox0;
    uint32_t wv[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) wv[jj] = px[jj];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t bw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 lo = u8x4(wv[2 * j]), hi = u8x4(wv[2 * j + 1]);
        bw[j] = pack_bf16_hi(lo[i], hi[i]);
      }
      const bfx8 Bf = __builtin_bit_cast(bfx8, make_uint4(bw[0], bw[1], bw[2], bw[3]));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        ah[h][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[h][0], Bf, ah[h][i], 0, 0, 0);
        am[h][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[h][1], Bf, am[h][i], 0, 0, 0);
        al[h][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[h][2], Bf, al[h][i], 0, 0, 0);
      }
    }
    if (ks + 1 < 15) split_store(ks + 1, cur ^ 1);  // the buffer read at ks - 1 (barrier below)
    __syncthreads();
  }
  // bias partials: co = 16 hq + col summed over the wave's 4 groups q, then the two waves
  // (c & 1) of the half and the two samples through LDS (fixed order)
  bs += __shfl_xor(bs, 16, 64);
  bs += __shfl_xor(bs, 32, 64);
  float* red = reinterpret_cast<float*>(pl);  // [4 waves][8 tiles x 4 regs][64 lanes] + bias [S samples][4 waves][16]
  float* bred = red + (S == 2 ? 4 * 32 * 64 : 0);
  if (q == 0) bred[(sl * 4 + c) * 16 + col] = bs;
  if (S == 2 && sl == 1) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          red[((c * 8 + h * 4 + i) * 4 + e) * 64 + lane] = ah[h][i][e] + (am[h][i][e] + al[h][i][e]);
  }
  __syncthreads();
  if (sl == 0) {
    float* out = a.out + (size_t)blockIdx.x * 32 * 256;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float own = ah[h][i][e] + (am[h][i][e] + al[h][i][e]);
          const float v = S == 2 ? own + red[((c * 8 + h * 4 + i) * 4 + e) * 64 + lane] : own;
          const int co = h * 16 + 4 * q + e, kk = c * 64 + (col >> 1) * 8 + 4 * (col & 1) + i;
          out[co * 256 + kk] = v;
        }
    if (t < 32) {  // co = t: half t >> 4, waves 2 (t >> 4) and +1 of every sample
      const int h = t >> 4, cc = t & 15;
      float v = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < S; ++s2) v += bred[(s2 * 4 + 2 * h) * 16 + cc] + bred[(s2 * 4 + 2 * h + 1) * 16 + cc];
      a.out2[blockIdx.x * 32 + t] = v;
    }
  }
}

// Input-gradient GEMMs with POSITION-MAJOR rows: row m = (spatial position, sample), so all
// rows of a tile share one input position and the same set of in-range taps.  The k loop runs
// over exactly those taps -- the sample-major forms above multiply the zero border: 40% of
// the conv3 dgrad MFMA work (21 of 27 (ky, iy) pairs in range per axis) and 19% of conv2's.
// BM x BN tiles of (samples at one input position) x (input channels): 128 x 32 (two n-tiles;
// 64 x 64 with each dy3 row staged once measured no better)
template <int BM_, int BN_, int WM_, int BK_ = 32>
struct Conv3DgradPT {  // dy2[b][pi][ci] = (a2 > 0) * sum_{valid taps, co} dy3[b][pi - tap][co] w3t[tap][ci][co]
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_;
  static constexpr int KPT = 64 / BK;  // k-blocks per tap (64 output channels)
  static constexpr int NT = 64 / BN;
  static_assert(NT * BN == 64, "n-tiles cover the 64 input channels");
  static constexpr bool A_KMAJ = true, B_KMAJ = true, SMEM = false;
  using Args = BwdArgs;
  using Smem = NoSmem;
  struct Ctx {
    int b0, pos, iy, ix, ky0, kx0, nkx, n0, kb0, kb1;
    Rsrc dy, w;
  };
  static __host__ __device__ int tiles(int B) { return 81 * NT * ((B + BM - 1) / BM); }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
    const int tpp = (a.B + BM - 1) / BM;
    c.n0 = (block % NT) * BN;
    block /= NT;
    c.pos = block / tpp;
    c.b0 = (block - c.pos * tpp) * BM;
    c.iy = c.pos / 9;
    c.ix = c.pos - c.iy * 9;
    c.ky0 = max(0, c.iy - 6);
    c.kx0 = max(0, c.ix - 6);
    const int nky = min(2, c.iy) - c.ky0 + 1;
    c.nkx = min(2, c.ix) - c.kx0 + 1;
    c.kb0 = 0;
    c.kb1 = KPT * nky * c.nkx;
    c.dy = make_rsrc(a.dy, (uint32_t)a.B * 49 * 64 * 4);
    c.w = make_rsrc(a.w, 9 * 64 * 64 * 4);
  }
  static __device__ void tap_of(const Ctx& c, int kb, int& ky, int& kx) {
    const int ti = kb / KPT, r = ti / c.nkx;
    ky = c.ky0 + r;
    kx = c.kx0 + ti - r * c.nkx;
  }
  // row states: sample row b0 + row (past the batch: past the range) / weight row n; the
  // k-block adds the tap's (wave-uniform) offset
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)((c.b0 + row) * 49 * 64 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    int ky, kx;
    tap_of(c, kb, ky, kx);
    return bld4(c.dy, r.off + (uint32_t)((((c.iy - ky) * 7 + c.ix - kx) * 64 + (kb % KPT) * BK) * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx& c, int n, int ch) {
    return {(uint32_t)((c.n0 + n) * 64 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    int ky, kx;
    tap_of(c, kb, ky, kx);
    return bld4(c.w, r.off + (uint32_t)(((ky * 3 + kx) * 64 * 64 + (kb % KPT) * BK) * 4));
  }
  static __device__ void store(const Args& a, const Ctx& c, int ml, int n, float v) {
    const int b = c.b0 + ml;
    if (b >= a.B) return;
    const size_t o = ((size_t)b * 81 + c.pos) * 64 + c.n0 + n;
    a.out[o] = a.mask[o] > 0.f ? v : 0.f;
  }
};

// BK 16 (half the LDS: more workgroups per CU beside the weight-gradient ones of the same
// launch): conv3 backward 47.2 vs 50.0 us, conv2 65.3 vs 68.8 us at BK 32 (B = 512)
using Conv3DgradP = Conv3DgradPT<128, 32, 4, 16>;
using Conv3DgradP32 = Conv3DgradPT<128, 32, 4, 32>;

// conv2: input pixel (iy, ix) = (2 jy + py, 2 jx + px) takes taps (py + 2 ty, px + 2 tx) from
// output pixel (jy - ty, jx - tx); rows = (class, jy, jx, sample), only in-range (ty, tx)
template <int BK_ = 32>
struct Conv2DgradPT {
  static constexpr int BM = 128, BN = 32, BK = BK_, WM = 4;
  static constexpr int KPT = 64 / BK;  // k-blocks per tap (64 output channels)
  static constexpr bool A_KMAJ = true, B_KMAJ = true, SMEM = false;
  using Args = BwdArgs;
  using Smem = NoSmem;
  struct Ctx {
    int b0, cls, jy, jx, ty0, tx0, ntx, kb0, kb1;
    Rsrc dy, w;
  };
  static __host__ __device__ int tiles(int B) { return 400 * ((B + BM - 1) / BM); }
  static __device__ void decode(const Args& a, int block, Ctx& c, Smem&) {
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
    c.kb1 = KPT * nty * c.ntx;
    c.dy = make_rsrc(a.dy, (uint32_t)a.B * 81 * 64 * 4);
    c.w = make_rsrc(a.w, 16 * 32 * 64 * 4);
  }
  static __device__ void tap_of(const Ctx& c, int kb, int& ty, int& tx) {
    const int ti = kb / KPT, r = c.ntx == 2 ? ti >> 1 : ti;
    ty = c.ty0 + r;
    tx = c.tx0 + ti - r * c.ntx;
  }
  using RowA = BufRow;
  using RowB = BufRow;
  static __device__ RowA row_a(const Args&, const Ctx& c, int row, int ch) {
    return {(uint32_t)((c.b0 + row) * 81 * 64 + 4 * ch) * 4};
  }
  static __device__ f32x4 load_a_row(const Args&, const Ctx& c, const RowA& r, int kb) {
    int ty, tx;
    tap_of(c, kb, ty, tx);
    return bld4(c.dy, r.off + (uint32_t)((((c.jy - ty) * 9 + c.jx - tx) * 64 + (kb % KPT) * BK) * 4));
  }
  static __device__ RowB row_b(const Args&, const Ctx&, int n, int ch) { return {(uint32_t)(n * 64 + 4 * ch) * 4}; }
  static __device__ f32x4 load_b_row(const Args&, const Ctx& c, const RowB& r, int kb) {
    int ty, tx;
    tap_of(c, kb, ty, tx);
    const int ky = (c.cls >> 1) + 2 * ty, kx = (c.cls & 1) + 2 * tx;
    return bld4(c.w, r.off + (uint32_t)(((ky * 4 + kx) * 32 * 64 + (kb % KPT) * BK) * 4));
  }
  static __device__ void store(const Args& a, const Ctx& c, int ml, int n, float v) {
    const int b = c.b0 + ml;
    if (b >= a.B) return;
    const int iy = 2 * c.jy + (c.cls >> 1), ix = 2 * c.jx + (c.cls & 1);
    const size_t o = ((size_t)b * 400 + iy * 20 + ix) * 32 + n;
    a.out[o] = a.mask[o] > 0.f ? v : 0.f;
  }
};
using Conv2DgradP = Conv2DgradPT<16>;
using Conv2DgradP32 = Conv2DgradPT<32>;

// default: the forward GEMMs on the stage-split single-image form at >= 3 waves per SIMD (form
// 3), the backward pairs on the register split.  Whole step, separate processes alternated on one
// box (scripts/ab/apex_engine_ab.py, profiles/r6_stage_split.md): register split 2466, forward
// form 2 2526.5, both directions form 2 2509; another box: register split 2434, forward form 2
// 2478, forward form 3 2489 steps/s.  The backward pairs gain nothing (backward-only form 2:
// 2341 vs 2345): their wgrad halves' LDS and the MN-major transposed reads eat the VALU saved.
// The actor's small forward launches (256 envs, beside the learner's forward) on the register
// split: 2497 vs 2489 (both rounds of an alternated A/B).
constexpr int kStageSplitDefault = 3 + 16 * (0 + 1);  // (+ the actor's small launches on form 0)

// wgrad split sizing: ~target blocks over (n-tiles x splits)
struct SplitPlan {
  int splits, kbps;
};

SplitPlan plan_splits(int kbt, int ntiles, int target_blocks) {
  int s = std::max(1, target_blocks / ntiles);
  int kbps = std::max(1, (kbt + s - 1) / s);
  s = (kbt + kbps - 1) / kbps;
  return {s, kbps};
}

// conv2 / conv3 weight gradient: ~`target` workgroups over (64-wide n-tiles x batch splits);
// target <= 0: the default (~one per CU)
SplitPlan wgrad_plan(int layer, int B, int target) {
  switch (layer) {
    case 1: {  // f32_conv1_wgrad_x3_k<S> workgroups (target 1: one sample per workgroup)
      const int S = target == 1 ? 1 : kConv1WgradS;
      return {(B + S - 1) / S, S};
    }
    case 2: return plan_splits(ConvWgrad<2>::kblocks(B), 512 / 64, target > 0 ? target : 256);
    case 3: return plan_splits(ConvWgrad<3>::kblocks(B), 576 / 64, target > 0 ? target : 252);
    default: throw std::invalid_argument("f32 wgrad layer");
  }
}

// GEMM form per direction, read at launch time (a captured graph keeps the form it was
// captured with): mask = forward form + 4 x backward-pair form (+ 16 x (1 + form) of the
// forward launches below the learner's size, the actor's; unset = the forward form), form 0 =
// register split, 1 = stage-split (double-buffered LDS image), 2 = stage-split, single LDS
// image, 3 = form 2 held to >= 3 waves per SIMD.  Every form gives bit-identical results.
int g_stage_split = -1;
int stage_split_mask() {
  if (g_stage_split < 0) {
    const char* e = std::getenv("APEX_F32_STAGE_SPLIT");
    g_stage_split = e ? std::atoi(e) : kStageSplitDefault;
  }
  return g_stage_split;
}

// small: a launch below the learner's size (the actor's / evaluator's forward) -- bits 4-5 of the
// mask, when set, give those launches a form of their own (form + 1; 0 = the forward form)
template <class P>
void launch1(const typename P::Args& a, int blocks, hipStream_t s, bool small = false) {
  if (blocks <= 0) return;
  const int m = stage_split_mask();
  const int form = small && ((m >> 4) & 3) ? ((m >> 4) & 3) - 1 : m & 3;
  switch (form) {
    case 1: gemm_k<P, 1><<<blocks, 256, 0, s>>>(a); break;
    case 2: gemm_k<P, 2><<<blocks, 256, 0, s>>>(a); break;
    case 3: gemm_k<P, 3><<<blocks, 256, 0, s>>>(a); break;
    default: gemm_k<P, 0><<<blocks, 256, 0, s>>>(a);
  }
  LAUNCH_CHECK();
}

template <class P1, class P2>
void launch2(const typename P1::Args& a1, int n1, const typename P2::Args& a2, int n2, hipStream_t s,
             const TreeRide* ride = nullptr) {
  if (n1 + n2 <= 0) return;
  TreeRide r{};
  if (ride && ride->stage) {
    r = *ride;
    r.nhost = n1 + n2;
  }
  const int nb = n1 + n2 + tree_ride_blocks(r);
  switch ((stage_split_mask() >> 2) & 3) {
    case 1: gemm2_k<P1, P2, 1><<<nb, 256, 0, s>>>(a1, a2, n1, r); break;
    case 2: gemm2_k<P1, P2, 2><<<nb, 256, 0, s>>>(a1, a2, n1, r); break;
    case 3: gemm2_k<P1, P2, 3><<<nb, 256, 0, s>>>(a1, a2, n1, r); break;
    default: gemm2_k<P1, P2, 0><<<nb, 256, 0, s>>>(a1, a2, n1, r);
  }
  LAUNCH_CHECK();
}

void check_set(const F32Set& set) {
  if (set.n < 1 || set.n > kMaxProbs) throw std::invalid_argument("f32: 1..3 problems");
  if (set.B <= 0) throw std::invalid_argument("f32: B must be positive");
  if ((int64_t)(set.B + 128) * 400 * 32 * 4 >= (int64_t)1 << 31)  // 32-bit operand byte offsets (raw buffers)
    throw std::invalid_argument("f32: batch too large for 32-bit operand offsets");
}

template <class P>
void fwd_launch(const F32Set& set, hipStream_t s) {
  launch1<P>(set, set.n * P::tiles(set.B), s, set.n * set.B < 1024);
}

}  // namespace

void f32_set_stage_split(int mask) { g_stage_split = mask; }
int f32_stage_split() { return stage_split_mask(); }

// ------------------------------------------------------------------ host launchers
// Tiles (MI355X, measured): the learner's launches (2-3 passes of its batch: >= 1024 rows) on
// 64 x 64 tiles (every A row staged once, 2 x 2 waves of 32 x 32: conv2 / conv3 1947 vs 1934
// steps/s for 128 x 32), the actor's single 256-env pass on 128 x 32 (4 x 1 waves: twice the
// workgroups); FC1 on 64 x 64 (31.6 vs 36.9 us for 128 x 64); the tuning log is
// profiles/r2_f32_kernel_tuning.md.
static bool learner_sized(const F32Set& set) { return set.n * set.B >= 1024; }

// c1_grid: conv1 workgroups (<= 0: kC1xGrid); tile (learner-sized launches, microbench
// alternatives to the defaults): 1 = conv2 on 64 x 64, 2 = conv2 on 128 x 64 as 4 x 1 waves of
// 32 x 64 / conv3 on 128 x 64 (2 x 2 waves), 3 = conv3 on 128 x 32 (4 x 1 waves)
// the learner-sized forward tiles when the caller passes tile 0: APEX_F32_TILES="c2,c3" (the
// microbench tile codes below, or "c2/c3"; unset = the defaults), read once -- a whole-step A/B knob
static int default_tile(int layer) {
  static int t2 = -1, t3 = -1;
  if (t2 < 0) {
    t2 = t3 = 0;
    if (const char* e = std::getenv("APEX_F32_TILES")) std::sscanf(e, "%d%*c%d", &t2, &t3);  // "c2,c3" or "c2/c3"
  }
  return layer == 2 ? t2 : t3;
}

void f32_conv_fwd_multi(int layer, const F32Set& set, hipStream_t s, int c1_grid, int tile, const ConvSample* draw) {
  check_set(set);
  if (draw && draw->out_idx && layer != 1) throw std::invalid_argument("f32_conv_fwd_multi: the draw folds into conv1");
  if (tile == 0 && (layer == 2 || layer == 3)) tile = default_tile(layer);
  switch (layer) {
    case 1: {
      if (c1_grid <= 0) c1_grid = learner_sized(set) ? kC1xGridLearner : (set.n * set.B + 1) / 2;
      const int G = std::min(set.n * set.B, c1_grid > 0 ? c1_grid : kC1xGrid);
      ConvSample c{};
      if (draw && draw->out_idx) {
        c = *draw;
        c.nhost = G;
        if ((set.n * set.B + G - 1) / G > kC1xDrawMax)
          throw std::invalid_argument("f32 conv1 draw: <= 8 samples per workgroup");
        if (!c.length || !c.beta || !c.counter || !c.out_w || set.p[0].idx != c.out_idx)
          throw std::invalid_argument("f32 conv1 draw: fill level, beta, counter, weights, and problem 0 reading idx");
        for (int k = 0; k < set.n; ++k)
          if (!set.p[k].ids || (c.rows.E > 0 && set.p[k].ids != c.rows.dst.s_ids && set.p[k].ids != c.rows.dst.s2_ids))
            throw std::invalid_argument("f32 conv1 draw: every problem reads the replay's frame-id tables");
      }
      f32_conv1_fwd_x3_k<<<G + (c.out_idx ? (c.rows.E + 255) / 256 : 0), 256, 0, s>>>(set, c);
      LAUNCH_CHECK();
      break;
    }
    case 2:  // learner: 128 x 64 tiles at BK 32 (64 x 32 per wave): on the split-bf16 MFMA 66.6-67.5 us
             // vs 73-79 for 64 x 64 (under fp32 MFMA 64 x 64 had won) and 76-88 for 256 x 64 (64 x 64
             // per wave: one wave per SIMD); whole step 2456-2466 vs 2193-2200 steps/s for 256 x 64
      if (learner_sized(set) && tile == 1) fwd_launch<Conv2FwdT<64, 64, 32, 2>>(set, s);
      else if (learner_sized(set) && tile == 2) fwd_launch<Conv2FwdT<128, 64, 32, 4>>(set, s);
      else if (learner_sized(set)) fwd_launch<Conv2FwdT<128, 64, 32, 2>>(set, s);
      else fwd_launch<Conv2FwdT<128, 32, 32, 4>>(set, s);  // (the actor: 128 x 64 / 64 x 64 measured no better)
      break;
    case 3:  // learner: 64 x 64 (46.7-46.8 us vs 80.6-84.5 for 256 x 64)
      if (learner_sized(set) && tile == 2) fwd_launch<Conv3FwdT<128, 64, 32, 2>>(set, s);
      else if (learner_sized(set) && tile == 3) fwd_launch<Conv3FwdT<128, 32, 32, 4>>(set, s);
      else if (learner_sized(set)) fwd_launch<Conv3FwdT<64, 64, 32, 2>>(set, s);
      // the actor: 128 x 64 tiles (98 workgroups for 256 envs beside the learner's forward):
      // 2622.6 vs 2564.0 learner steps/s for 128 x 32 (196), 64 x 64 (196) 2558.2 (one box)
      else fwd_launch<Conv3FwdT<128, 64, 32, 2>>(set, s);
      break;
    default: throw std::invalid_argument("f32_conv_fwd_multi: layer must be 1, 2 or 3");
  }
}

int f32_fc1_splits() { return kFcSplits; }

int f32_fc1_fwd_multi(const F32Set& set, hipStream_t s) {
  check_set(set);
  fwd_launch<Fc1FwdT<64, 64, 32, 2>>(set, s);
  return kFcSplits;
}

// FC1 weight gradient: ONE batch slice of natural-order partials, reduced and transposed by
// grad_finalize (coalesced stores; more slices did not pay for their partial traffic:
// 1947 vs 1929 / 1892 steps/s for 2 / 4)
constexpr int kFc1WgSlices = 1;

int f32_fc1_wgrad_splits() { return kFc1WgSlices; }

size_t f32_fc1_wgrad_workspace_floats() { return (size_t)kFc1WgSlices * 256 * 3136; }

// the backward loaders address operands by 32-bit byte offsets (raw buffer resources)
static void check_bwd_batch(int B) {
  if ((int64_t)B * 400 * 32 * 4 + (int64_t)64 * 400 * 32 * 4 >= (int64_t)1 << 31)
    throw std::invalid_argument("f32 backward: batch too large for 32-bit operand offsets");
}

void f32_fc1_bwd_split(const float* dz, const float* a3, const float* wfc1p, float* dy3, float* ws, int B,
                       hipStream_t s, const TreeRide* ride) {
  if (B <= 0) return;
  check_bwd_batch(B);
  BwdArgs d{};
  d.dy = dz;
  d.w = wfc1p;
  d.mask = a3;
  d.out = dy3;
  d.B = B;
  BwdArgs w{};
  w.x = a3;
  w.dy = dz;
  w.out = ws;
  w.B = B;
  const int nkb = (B + Fc1Wgrad::BK - 1) / Fc1Wgrad::BK;
  w.splits = std::min(kFc1WgSlices, nkb);
  w.kbps = (nkb + w.splits - 1) / w.splits;
  w.splits = (nkb + w.kbps - 1) / w.kbps;  // every slice non-empty
  launch2<Fc1Wgrad, Fc1Dgrad>(w, Fc1Wgrad::tiles(B) * w.splits, d, Fc1Dgrad::tiles(B), s, ride);
}

int f32_fc1_wgrad_slices(int B) {
  const int nkb = (B + Fc1Wgrad::BK - 1) / Fc1Wgrad::BK;
  const int g = std::min(kFc1WgSlices, nkb), kbps = (nkb + g - 1) / g;
  return (nkb + kbps - 1) / kbps;
}

int f32_wgrad_splits(int layer, int B, int target) { return wgrad_plan(layer, B, target).splits; }

int f32_wgrad_kbps(int layer, int B, int target) { return wgrad_plan(layer, B, target).kbps; }

size_t f32_wgrad_workspace_floats(int layer, int B, int target) {
  const SplitPlan p = wgrad_plan(layer, B, target);
  const size_t per = layer == 1 ? 32 * 256 : (layer == 2 ? 64 * 512 : 64 * 576);
  const size_t cout = layer == 1 ? 32 : 64;
  return (size_t)p.splits * (per + cout);
}

// wgrad + dgrad of conv layer 3 or 2 in one launch; layer 1: wgrad only (x = frames)
void f32_conv_bwd(int layer, const void* x, const int* ids, const int* idx, const float* dy, const float* w,
                  const float* mask, float* dx, float* ws, int B, hipStream_t s, int target, int tile,
                  const TreeRide* ride) {
  if (B <= 0) return;
  check_bwd_batch(B);
  if (ride && ride->stage && layer == 1) throw std::invalid_argument("f32_conv_bwd: no tree rider on layer 1");
  const SplitPlan p = wgrad_plan(layer, B, target);
  const size_t per = layer == 1 ? 32 * 256 : (layer == 2 ? 64 * 512 : 64 * 576);
  BwdArgs g{};
  g.x = x;
  g.ids = ids;
  g.idx = idx;
  g.dy = dy;
  g.out = ws;
  g.out2 = ws + (size_t)p.splits * per;
  g.B = B;
  g.kbps = p.kbps;
  g.splits = p.splits;
  BwdArgs d{};
  d.dy = dy;
  d.w = w;
  d.mask = mask;
  d.out = dx;
  d.B = B;
  // microbench knob (read once): APEX_F32_BWD_HALF=1 runs only the weight-gradient half of a conv
  // pair, 2 only the input-gradient half (profiles/r6_ab_ledger.md: what each half costs alone)
  static const int halves = [] {
    const char* e = std::getenv("APEX_F32_BWD_HALF");
    return e ? std::atoi(e) : 0;
  }();
  if (halves && layer != 1) {
    const int nw = (layer == 2 ? 512 / 64 : 576 / 64) * p.splits;
    const int nd = layer == 2 ? Conv2DgradP::tiles(B) : Conv3DgradP::tiles(B);
    if (layer == 2) launch2<ConvWgrad<2>, Conv2DgradP>(g, halves == 1 ? nw : 0, d, halves == 2 ? nd : 0, s, nullptr);
    else launch2<ConvWgrad<3>, Conv3DgradP>(g, halves == 1 ? nw : 0, d, halves == 2 ? nd : 0, s, nullptr);
    return;
  }
  switch (layer) {
    case 3:  // tile 1: input gradient at BK 32 (the alternative to the default)
      if (tile == 1) launch2<ConvWgrad<3>, Conv3DgradP32>(g, (576 / 64) * p.splits, d, Conv3DgradP32::tiles(B), s, ride);
      else launch2<ConvWgrad<3>, Conv3DgradP>(g, (576 / 64) * p.splits, d, Conv3DgradP::tiles(B), s, ride);
      break;
    case 2:
      if (tile == 1) launch2<ConvWgrad<2>, Conv2DgradP32>(g, (512 / 64) * p.splits, d, Conv2DgradP32::tiles(B), s, ride);
      else launch2<ConvWgrad<2>, Conv2DgradP>(g, (512 / 64) * p.splits, d, Conv2DgradP::tiles(B), s, ride);
      break;
    case 1:
      if (p.kbps == 1) f32_conv1_wgrad_x3_k<1><<<p.splits, 256, 0, s>>>(g);
      else f32_conv1_wgrad_x3_k<2><<<p.splits, 512, 0, s>>>(g);
      LAUNCH_CHECK();
      break;
    default: throw std::invalid_argument("f32_conv_bwd: layer must be 1, 2 or 3");
  }
}

FinalizeJob f32_conv_finalize_job(int layer, int B, const float* ws, float* grad, float* bias_grad, int target) {
  const SplitPlan p = wgrad_plan(layer, B, target);
  FinalizeJob j{};
  j.kind = 0;
  j.G = p.splits;
  j.part = ws;
  const int cout = layer == 1 ? 32 : 64;
  const int K = layer == 1 ? 256 : (layer == 2 ? 512 : 576);
  j.pstride = cout * K;
  j.bpart = ws + (size_t)p.splits * cout * K;
  j.bstride = cout;
  j.n_main = cout * K;
  j.n_bias = cout;
  if (layer == 1) {  // partials already in the reference [co][c][ky][kx] order
    j.C = 1;
    j.KH = 1;
    j.KW = 256;
  } else {  // [co][ky][kx][ci] -> reference [co][ci][ky][kx]
    j.C = layer == 2 ? 32 : 64;
    j.KH = j.KW = layer == 2 ? 4 : 3;
  }
  j.out[0] = grad;
  j.out[1] = bias_grad;
  return j;
}

FinalizeJob norm_only_job(const float* g, int n) {
  FinalizeJob j{};
  j.kind = 3;
  j.G = 1;
  j.part = g;
  j.pstride = 0;
  j.n_main = n;
  j.n_bias = 0;
  return j;
}

}  // namespace apex
