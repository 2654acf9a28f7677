// MFMA backward kernels for the Nature-CNN trunk on gfx950.
//
// dgrad (input gradient) as an implicit GEMM  M = input pixels, N = input channels,
// K = (tap, output channel), fused with the ReLU backward of the layer below:
//   * conv3 (3x3, stride 1): dy3 staged in LDS with a 2-pixel zero border, so every tap of
//     every output row is a plain 16-byte read (no bounds checks in the K loop);
//   * conv2 (4x4, stride 2): sub-pixel decomposition -- input pixels are grouped by
//     parity class (qy%2, qx%2); inside a class exactly 2x2 taps contribute, so K = 4 taps
//     x 64 instead of 16 taps x 64 with 3/4 zeros.
//   B operand = transposed packed weights W^T [tap][c][n] (n contiguous, 16-byte frags).
//
// wgrad (weight gradient) dW[n][(ky,kx,c)] = sum_{b,p} dy[b][p][n] x[b][S p + (ky,kx)][c]:
//   the reduction runs over output pixels, which are strided in the channels-last tiles,
//   so both MFMA operands are fetched with ds_read_b64_tr_b16 (hardware 4x16 transpose;
//   every lane supplies its own row address, so the strided im2col rows of the input are
//   gathered for free).  Each workgroup accumulates a batch slice in registers and writes
//   one fp32 partial; wgrad_reduce sums the partials in fixed order (deterministic) and
//   scatters into the reference [N][C][KH][KW] gradient layout.
#include "common.h"
#include "kernels.h"
#include "tree_dev.h"

namespace apex {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(__attribute__((address_space(3))) char*)p);
}

__device__ __forceinline__ bool bf16_pos(uint16_t v) { return v != 0 && !(v & 0x8000); }


// ====================================================================== dgrad
// Stage a [OH][OW][64] bf16 dy tile into LDS at offset `border` inside a zeroed
// [TH][TW] grid (pixel stride 144 B = 128 + 16 pad).
constexpr int DY_PIX = 144;

template <int OH, int OW, int TH, int TW, int BORDER>
__device__ __forceinline__ int dy_pad_off(int q) {
  constexpr int CH = 8;  // 16-byte chunks per pixel (64 channels)
  const int pix = q / CH, cc = q % CH;
  return ((pix / OW + BORDER) * TW + pix % OW + BORDER) * DY_PIX + cc * 16;
}

// Stage a [OH][OW][64] bf16 dy tile into a zero-bordered LDS grid; with `mask` (the
// post-ReLU activation of the same shape) the ReLU backward is applied on the way in
// (coalesced 16-B reads of both, instead of a strided gather in a producer's epilogue).
template <int OH, int OW, int TH, int TW, int BORDER>
__device__ __forceinline__ void stage_dy_padded(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ mask,
                                                char* t) {
  constexpr int TOTAL = OH * OW * 8;
  static_assert(TOTAL <= 8 * 256, "one Pf8 block");
  auto off = [](int q) { return dy_pad_off<OH, OW, TH, TW, BORDER>(q); };
  Pf8 v;
  pf_load<TOTAL>(v, reinterpret_cast<const uint4*>(dy));
  if (mask) {  // block-uniform
    Pf8 m;
    pf_load<TOTAL>(m, reinterpret_cast<const uint4*>(mask));
    pf_mask<TOTAL>(v, m);
  }
  pf_store<TOTAL>(v, t, off);
}

template <int ROWS>
__device__ __forceinline__ void zero_lds(char* t) {
  for (int q = threadIdx.x; q < ROWS * DY_PIX / 16; q += blockDim.x) reinterpret_cast<uint4*>(t)[q] = uint4{0, 0, 0, 0};
}

// W^T packed [taps][C][64] bf16 -> LDS rows (tap, c) with stride 144 B
template <int TAPS, int C>
__device__ __forceinline__ void stage_wt(const uint16_t* __restrict__ wt, char* t) {
  constexpr int CH = 8;
  stage_all<TAPS * C * CH>(reinterpret_cast<const uint4*>(wt), t,
                           [](int q) { return (q / CH) * DY_PIX + (q % CH) * 16; });
}

// conv3 dgrad: dy3 [B][49][64] (already ReLU-masked) -> dx2 [B][81][64]; with out_mask
// (= a2) the ReLU backward is applied in the coalesced epilogue (writes dy2)
// dgrad kernels: 8 waves per workgroup (2 per SIMD at one LDS-limited workgroup per CU);
// waves 0-3 stage (the copy helpers are written for 256 threads)
constexpr int kDgWaves = 8;

__global__ __launch_bounds__(64 * kDgWaves) void dgrad3_k(const uint16_t* __restrict__ dy3, const uint16_t* __restrict__ mask3,
                                                const uint16_t* __restrict__ wt3, uint16_t* __restrict__ dx2,
                                                const uint16_t* __restrict__ out_mask, int B) {
  constexpr int T = 11, TILE = T * T * DY_PIX;     // 7x7 grid + 2-pixel border
  constexpr int SPW = 2;
  __shared__ __attribute__((aligned(16))) char smem[SPW * TILE + 9 * 64 * DY_PIX + kDgWaves * TILE_EP_BYTES];
  char* wts = smem + SPW * TILE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  const bool stager = threadIdx.x < 256;  // wave-uniform
  char* ep = wts + 9 * 64 * DY_PIX + wave * TILE_EP_BYTES;
  zero_lds<SPW * T * T>(smem);
  if (stager) stage_wt<9, 64>(wt3, wts);
  for (int b0 = blockIdx.x * SPW; b0 < B; b0 += gridDim.x * SPW) {
    __syncthreads();
    if (stager)
      for (int sw = 0; sw < SPW; ++sw)
        if (b0 + sw < B)
          stage_dy_padded<7, 7, T, T, 2>(dy3 + (size_t)(b0 + sw) * 49 * 64,
                                         mask3 ? mask3 + (size_t)(b0 + sw) * 49 * 64 : nullptr, smem + sw * TILE);
    __syncthreads();
    // items: (sample, m-tile of 32 input pixels (3), n-tile of 32 channels (2)) = 12
    for (int it = wave; it < SPW * 6; it += kDgWaves) {
      const int sw = it / 6, mt = (it / 2) % 3, nt = it % 2;
      const int b = b0 + sw;
      if (b >= B) continue;
      const int q = mt * 32 + r32;
      const int qc = q < 81 ? q : 80;
      const int qy = qc / 9, qx = qc % 9;
      // output pixel for tap (ky,kx): (qy-ky, qx-kx) -> padded index (qy-ky+2, qx-kx+2)
      const char* abase = smem + sw * TILE + ((qy + 2) * T + (qx + 2)) * DY_PIX + h * 16;
      const char* bbase = wts + (nt * 32 + r32) * DY_PIX + h * 16;
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 36; ++s) {
        const int tap = s / 4, ky = tap / 3, kx = tap % 3, n0 = (s % 4) * 16;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(abase - (ky * T + kx) * DY_PIX + n0 * 2);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(bbase + tap * 64 * DY_PIX + n0 * 2);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc, 0, 0, 0);
      }
      const long base = (long)b * 81 * 64 + nt * 32;
      tile_store_bf16(acc, ep, [](int, int, float v) { return f2bf(v); },
                      [&](int row) -> long {
                        const int qq = mt * 32 + row;
                        return qq < 81 ? base + qq * 64 : -1;
                      }, dx2, out_mask);
    }
  }
}

// conv2 dgrad (sub-pixel): dy2 (optionally masked while staging) -> dx1 [B][400][32];
// with out_mask (= a1) the ReLU backward is applied in the coalesced epilogue (writes dy1)
__global__ __launch_bounds__(64 * kDgWaves) void dgrad2_k(const uint16_t* __restrict__ dx2, const uint16_t* __restrict__ mask2,
                                                const uint16_t* __restrict__ wt2, uint16_t* __restrict__ dx1,
                                                const uint16_t* __restrict__ out_mask, int B) {
  constexpr int T = 11, TILE = T * T * DY_PIX;     // 9x9 grid + 1-pixel border
  constexpr int SPW = 2;
  __shared__ __attribute__((aligned(16))) char smem[SPW * TILE + 16 * 32 * DY_PIX + kDgWaves * TILE_EP_BYTES];
  char* wts = smem + SPW * TILE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  const bool stager = threadIdx.x < 256;  // wave-uniform
  char* ep = wts + 16 * 32 * DY_PIX + wave * TILE_EP_BYTES;
  zero_lds<SPW * T * T>(smem);
  if (stager) stage_wt<16, 32>(wt2, wts);
  for (int b0 = blockIdx.x * SPW; b0 < B; b0 += gridDim.x * SPW) {
    __syncthreads();
    if (stager)
      for (int sw = 0; sw < SPW; ++sw)
        if (b0 + sw < B)
          stage_dy_padded<9, 9, T, T, 1>(dx2 + (size_t)(b0 + sw) * 81 * 64,
                                         mask2 ? mask2 + (size_t)(b0 + sw) * 81 * 64 : nullptr, smem + sw * TILE);
    __syncthreads();
    // items: (sample, parity class (4), m-tile of 32 class pixels (4 -> 128 >= 100)) = 32
    for (int it = wave; it < SPW * 16; it += kDgWaves) {
      const int sw = it / 16, cls = (it / 4) % 4, mt = it % 4;
      const int b = b0 + sw;
      if (b >= B) continue;
      const int ry = cls >> 1, rx = cls & 1;
      const int m = mt * 32 + r32;
      const int mc = m < 100 ? m : 99;
      const int i = mc / 10, j = mc % 10;  // qy = 2i + ry, qx = 2j + rx
      // contributing taps: ky = ry + 2 dyy, kx = rx + 2 dxx ; output pixel (i - dyy, j - dxx) -> padded +1
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
      const long base = (long)b * 400 * 32;
      tile_store_bf16(acc, ep, [](int, int, float v) { return f2bf(v); },
                      [&](int row) -> long {
                        const int mm = mt * 32 + row;
                        if (mm >= 100) return -1;
                        const int q = (2 * (mm / 10) + ry) * 20 + 2 * (mm % 10) + rx;
                        return base + q * 32;
                      }, dx1, out_mask);
    }
  }
}

void conv_dgrad(int layer, const uint16_t* dy, const uint16_t* dy_mask, const uint16_t* wt, uint16_t* dx,
                const uint16_t* dx_mask, int B, hipStream_t s) {
  if (B <= 0) return;
  const int grid = std::min((B + 1) / 2, 512);
  if (layer == 3) {
    dgrad3_k<<<grid, 64 * kDgWaves, 0, s>>>(dy, dy_mask, wt, dx, dx_mask, B);
  } else if (layer == 2) {
    dgrad2_k<<<grid, 64 * kDgWaves, 0, s>>>(dy, dy_mask, wt, dx, dx_mask, B);
  } else {
    throw std::invalid_argument("conv_dgrad: layer must be 2 or 3");
  }
  LAUNCH_CHECK();
}

// ====================================================================== wgrad
// GRID batch slices x KSPLIT kidx-tile groups = workgroups (256: one per CU).  Splitting
// the kidx tiles (instead of more batch slices) keeps the fp32 partial workspace
// [GRID][N][K] -- and the reduce that reads it -- small.
template <int H_, int W_, int C_, int KH_, int KW_, int S_, int N_, int GRID_, int KSPLIT_, int GROUPS_ = 1,
          bool XCD_ = true>
struct WG {
  static constexpr bool XCD = XCD_;  // XCD-aware blockIdx mapping (see wgrad_k)
  static constexpr int H = H_, W = W_, C = C_, KH = KH_, KW = KW_, S = S_, N = N_, GRID = GRID_;
  static constexpr int KSPLIT = KSPLIT_;
  // sample groups per workgroup: each group of 4 waves stages and multiplies its own
  // sample (2 groups = 8 waves = 2 per SIMD at the LDS-limited one workgroup per CU), the
  // groups' accumulators are summed before the one partial write (same workspace size)
  static constexpr int GROUPS = GROUPS_;
  static constexpr int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1, P = OH * OW;
  static constexpr int K = KH * KW * C;
  static constexpr int KT = K / 32;            // 32-wide kidx tiles
  static constexpr int NT = N / 32;
  static constexpr int KS = (P + 15) / 16;     // pixel k-steps
  static constexpr int PPAD = KS * 16;
  static constexpr int PIX = (C == 4) ? 8 : (C * 2 + 16);
  // C == 4 (the u8 frame stack): 8-B pixels plus 16 B of padding after every 16 pixels,
  // so the staging threads' 128-B runs land on distinct banks (conflict-free b128 writes)
  static constexpr int X_BYTES = (C == 4) ? H * W * PIX + (H * W / 16) * 16 : H * W * PIX;
  static constexpr int DYROW = N * 2 + 16;
  static constexpr int DY_BYTES = PPAD * DYROW;
  static constexpr int KTB = (KT + KSPLIT - 1) / KSPLIT;  // kidx tiles per workgroup
  static constexpr int KTW = (KTB + 3) / 4;               // kidx tiles per wave
};
using WG1 = WG<84, 84, 4, 8, 8, 4, 32, 128, 2, 1>;  // 95 KB of LDS per sample: one group
using WG2 = WG<20, 20, 32, 4, 4, 2, 64, 64, 4, 2>;
using WG3 = WG<9, 9, 64, 3, 3, 1, 64, 64, 4, 1, false>;

// LDS byte address of input pixel `pix` in the wgrad x tile
template <class G>
__device__ __forceinline__ int x_pix_off(int pix) {
  if constexpr (G::C == 4) return pix * G::PIX + (pix >> 4) * 16;
  else return pix * G::PIX;
}

// Frame stack -> padded NHWC bf16 (16 pixels per thread-chunk, 16-B pad after each chunk),
// split into a register prefetch (4 planes x <= 2 groups per thread) and an LDS commit.
template <class G>
__device__ __forceinline__ void frames_load(const FrameSrc& f, int b, Pf8& p) {
  constexpr int HW = G::H * G::W, GROUPS = HW / 16;
  static_assert(GROUPS <= 512, "two 16-pixel groups per thread");
  const uint4* p0 = reinterpret_cast<const uint4*>(frame_plane(f, b, 0, HW));
  const uint4* p1 = reinterpret_cast<const uint4*>(frame_plane(f, b, 1, HW));
  const uint4* p2 = reinterpret_cast<const uint4*>(frame_plane(f, b, 2, HW));
  const uint4* p3 = reinterpret_cast<const uint4*>(frame_plane(f, b, 3, HW));
  const int g0 = threadIdx.x & 255, g1 = g0 + 256;
  auto ld = [](const uint4* q, int i) { return reinterpret_cast<const u32v4*>(q)[i]; };
  p.r0 = ld(p0, g0); p.r1 = ld(p1, g0); p.r2 = ld(p2, g0); p.r3 = ld(p3, g0);
  const int g1c = g1 < GROUPS ? g1 : GROUPS - 1;  // always assigned (stores are guarded)
  p.r4 = ld(p0, g1c); p.r5 = ld(p1, g1c); p.r6 = ld(p2, g1c); p.r7 = ld(p3, g1c);
}

template <class G>
__device__ __forceinline__ void frames_store(const Pf8& p, char* xs) {
  constexpr int GROUPS = G::H * G::W / 16;
  const int g0 = threadIdx.x & 255, g1 = g0 + 256;
  uint4* d = reinterpret_cast<uint4*>(xs + g0 * 144);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    u8x4words_to_lds(p.r0[k], p.r1[k], p.r2[k], p.r3[k], d + 2 * k);
  if (g1 < GROUPS) {
    d = reinterpret_cast<uint4*>(xs + g1 * 144);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      u8x4words_to_lds(p.r4[k], p.r5[k], p.r6[k], p.r7[k], d + 2 * k);
  }
}

// LDS byte offset of kidx tile kt's column-block origin relative to an output pixel's window
template <class G>
__device__ __forceinline__ int kt_origin(int kt) {
  if constexpr (G::C == 4) {
    return kt * G::W;  // PIXEL delta: tile = kernel row ky (8 taps x 4 channels); see x_pix_off
  } else {
    constexpr int CB = G::C / 32;
    const int tap = kt / CB, c0 = (kt % CB) * 32;
    return ((tap / G::KW) * G::W + tap % G::KW) * G::PIX + c0 * 2;
  }
}

template <class G>
__device__ __forceinline__ void wg_issue(const void* __restrict__ x, const FrameSrc& fs,
                                         const uint16_t* __restrict__ dy, const uint16_t* __restrict__ mask, int bb,
                                         Pf8& px, Pf8& pd, Pf8& pm) {
  if constexpr (G::C == 4) {
    frames_load<G>(fs, bb, px);
  } else {
    pf_load<G::H * G::W * G::C / 8>(px, reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(x) +
                                                                       (size_t)bb * G::H * G::W * G::C * 2));
  }
  pf_load<G::P * G::N / 8>(pd, reinterpret_cast<const uint4*>(dy + (size_t)bb * G::P * G::N));
  if (mask) pf_load<G::P * G::N / 8>(pm, reinterpret_cast<const uint4*>(mask + (size_t)bb * G::P * G::N));
}

template <class G>
struct WgFrags {
  bf16x8 a[G::NT];   // dy^T fragments (rows n, k = 16 pixels)
  bf16x8 b[G::KTW];  // im2col x fragments (k = 16 pixels, cols kidx)
};

// LDS byte offset of the B (im2col x) fragment of pixel k-step ks, half t, kidx tile kt
// for this lane: sample-independent, so computed once per workgroup (the integer
// division by OW per k-step was most of the kernels' VALU, PMC)
template <class G>
__device__ __forceinline__ int wg_boff(int ks, int t, int h, int q4, int colsel, int kt) {
  const int p = ks * 16 + 8 * h + 4 * t + q4;
  const int pc = p < G::P ? p : G::P - 1;
  const int oy = pc / G::OW, ox = pc % G::OW;
  const int xpix = (G::S * oy) * G::W + G::S * ox;
  if constexpr (G::C == 4) return x_pix_off<G>(xpix + kt_origin<G>(kt) + colsel / 4);
  else return xpix * G::PIX + kt_origin<G>(kt) + colsel * 2;
}

template <class G>
struct WgAddr {
  int b[G::KS][2][G::KTW];
  bool ok[G::KTW];
};

template <class G>
__device__ __forceinline__ void wg_frags_pre(const char* xs, const char* dys, int ks, int arow, int colsel,
                                             const WgAddr<G>& ad, WgFrags<G>& f) {
  // A (dy^T): rows p = 16 ks + 8 h + 4 t + q4 (arow = 8 h + q4), columns n
#pragma unroll
  for (int nt = 0; nt < G::NT; ++nt) {
    const char* a0 = dys + (ks * 16 + arow) * G::DYROW + (nt * 32 + colsel) * 2;
    const bf16x4 lo = tr_read(a0), hi = tr_read(a0 + 4 * G::DYROW);
    f.a[nt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
#pragma unroll
  for (int k = 0; k < G::KTW; ++k) {
    f.b[k] = bf16x8{};
    if (ad.ok[k]) {
      const bf16x4 lo = tr_read(xs + ad.b[ks][0][k]), hi = tr_read(xs + ad.b[ks][1][k]);
      f.b[k] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  }
}

template <class G>
__device__ __forceinline__ void wg_mfma(const WgFrags<G>& f, int, int, f32x16 (&acc)[G::NT][G::KTW]) {
#pragma unroll
  for (int k = 0; k < G::KTW; ++k) {
#pragma unroll
    for (int nt = 0; nt < G::NT; ++nt)
      acc[nt][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[nt], f.b[k], acc[nt][k], 0, 0, 0);
  }
}

// bias gradient from the prefetched dy registers: chunk q = 8 channels (group q % (N/8))
// of pixel q / (N/8); a thread's chunks all have group t % (N/8)
template <class G>
__device__ __forceinline__ void wg_bias_acc(const Pf8& pd, float (&bs)[8]) {
  constexpr int DCH = G::P * G::N / 8;
  const int t = threadIdx.x & 255;  // local to the sample group
#define APEX_WG_BIAS(K, R)                                     \
  if constexpr (K * 256 < DCH) {                               \
    if (t + K * 256 < DCH) {                                   \
      _Pragma("unroll") for (int j = 0; j < 4; ++j) {          \
        const uint32_t w = pd.R[j];                            \
        bs[2 * j] += __uint_as_float(w << 16);                 \
        bs[2 * j + 1] += __uint_as_float(w & 0xFFFF0000u);     \
      }                                                        \
    }                                                          \
  }
  APEX_PF_SLOTS(APEX_WG_BIAS)
#undef APEX_WG_BIAS
}

template <class G>
__global__ __launch_bounds__(256 * G::GROUPS) void wgrad_k(const void* __restrict__ x, FrameSrc fs,
                                                          const uint16_t* __restrict__ dy,
                                                          const uint16_t* __restrict__ mask, int B, int gridb,
                                                          float* __restrict__ partial,
                                                          float* __restrict__ bias_partial) {
  constexpr int GB = G::X_BYTES + G::DY_BYTES;  // LDS bytes per sample group
  __shared__ __attribute__((aligned(16))) char smem[G::GROUPS * GB];
  const int grp = threadIdx.x >> 8;           // sample group (wave-uniform)
  char* xs = smem + grp * GB;
  char* dys = xs + G::X_BYTES;
  const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3;  // wave within the group
  const int g = lane >> 4, q4 = (lane >> 2) & 3, pp = lane & 3, h = g >> 1;
  const int colsel = 16 * (g & 1) + 4 * pp;  // column (within a 32-wide tile) this lane addresses
  // XCD-aware mapping: workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8), and
  // the KSPLIT workgroups of one batch slice read the same samples -- give them blockIdx
  // values 8 apart so they share one XCD's L2 (one HBM/MALL read per sample instead of
  // KSPLIT).  Needs gridDim.x % (8 * KSPLIT) == 0, else the plain mapping.
  int bg, kg;
  if (G::XCD && gridDim.x % (8 * G::KSPLIT) == 0) {
    const int xcd = blockIdx.x & 7, r = blockIdx.x >> 3;
    kg = r % G::KSPLIT;
    bg = (r / G::KSPLIT) * 8 + xcd;
  } else {
    bg = blockIdx.x / G::KSPLIT;
    kg = blockIdx.x % G::KSPLIT;
  }
  const int kt0 = kg * G::KTB;
  const bool do_bias = kg == 0;  // block-uniform: one kidx group owns the bias gradient
  // zero the padded dy rows once (they stay zero)
  for (int q = threadIdx.x & 255; q < (G::PPAD - G::P) * G::DYROW / 16; q += 256)
    reinterpret_cast<uint4*>(dys + G::P * G::DYROW)[q] = uint4{0, 0, 0, 0};
  float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16 acc[G::NT][G::KTW];
#pragma unroll
  for (int a = 0; a < G::NT; ++a)
#pragma unroll
    for (int k = 0; k < G::KTW; ++k) acc[a][k] = f32x16{};
  // sample-independent fragment addresses (B: im2col x rows for every pixel k-step)
  WgAddr<G> ad;
  const int arow = 8 * h + q4;
#pragma unroll
  for (int k = 0; k < G::KTW; ++k) {
    const int kl = wave + 4 * k, kt = kt0 + kl;
    ad.ok[k] = kl < G::KTB && kt < G::KT;
    const int ktc = kt < G::KT ? kt : G::KT - 1;
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t) ad.b[ks][t][k] = wg_boff<G>(ks, t, h, q4, colsel, ktc);
  }
  // register prefetch: the group's next sample's x and dy loads are in flight during this
  // sample's MFMA loop (one LDS buffer per group; committed after the compute)
  constexpr int XCH = (G::C == 4) ? 0 : G::H * G::W * G::C / 8;
  constexpr int DCH = G::P * G::N / 8;
  constexpr int STEP = G::GROUPS;  // samples of this batch slice per iteration
  Pf8 px, pd, pm;
  if (bg + grp * gridb < B) wg_issue<G>(x, fs, dy, mask, bg + grp * gridb, px, pd, pm);
  for (int b0 = bg; b0 < B; b0 += STEP * gridb) {  // block-uniform trip count
    const int b = b0 + grp * gridb;
    const bool valid = b < B;  // group-uniform
    __syncthreads();  // the previous sample's compute is done with LDS
    if (valid) {
      if constexpr (G::C == 4) {
        frames_store<G>(px, xs);
      } else {
        constexpr int CH16 = G::C / 8;
        pf_store<XCH>(px, xs, [](int q) { return (q / CH16) * G::PIX + (q % CH16) * 16; });
      }
      {
        constexpr int CH16 = G::N / 8;
        if (mask) pf_mask<DCH>(pd, pm);  // ReLU backward of the layer output, applied at staging
        pf_store<DCH>(pd, dys, [](int q) { return (q / CH16) * G::DYROW + (q % CH16) * 16; });
      }
      if (do_bias) wg_bias_acc<G>(pd, bs);
    }
    __syncthreads();
    if (b + STEP * gridb < B) wg_issue<G>(x, fs, dy, mask, b + STEP * gridb, px, pd, pm);  // group-uniform
    if (valid) {
      // fully unrolled pixel k-steps on precomputed fragment addresses, software
      // pipelined: the fragments of ks + 1 are read while ks multiplies
      WgFrags<G> cur;
      wg_frags_pre<G>(xs, dys, 0, arow, colsel, ad, cur);
#pragma unroll
      for (int ks = 0; ks < G::KS; ++ks) {
        WgFrags<G> nxt;
        if (ks + 1 < G::KS) wg_frags_pre<G>(xs, dys, ks + 1, arow, colsel, ad, nxt);
        wg_mfma<G>(cur, wave, kt0, acc);
        if (ks + 1 < G::KS) cur = nxt;
      }
    }
  }
  if (do_bias) {  // fixed-order combine of the per-thread bias sums (reuse the LDS tiles)
    constexpr int NG = G::N / 8;  // channel groups; thread t owns group t % NG
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = bs[j];
    __syncthreads();
    if (threadIdx.x < G::N) {
      const int n = threadIdx.x, cg = n / 8, j = n % 8;
      float t = 0.f;
      for (int src = cg; src < 256 * G::GROUPS; src += NG) t += red[src * 8 + j];
      bias_partial[(size_t)bg * G::N + n] = t;
    }
  }
  if constexpr (G::GROUPS > 1) {  // group 1's accumulators into group 0's, one k-tile column at a time
    static_assert(G::GROUPS == 2, "two sample groups");
    static_assert(4 * G::NT * 16 * 64 * 4 <= G::GROUPS * GB, "accumulator exchange fits the tiles");
    float* xch = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int k = 0; k < G::KTW; ++k) {
      __syncthreads();
      if (grp == 1) {
#pragma unroll
        for (int nt = 0; nt < G::NT; ++nt)
#pragma unroll
          for (int r = 0; r < 16; ++r) xch[((wave * G::NT + nt) * 16 + r) * 64 + lane] = acc[nt][k][r];
      }
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int nt = 0; nt < G::NT; ++nt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[nt][k][r] += xch[((wave * G::NT + nt) * 16 + r) * 64 + lane];
      }
    }
    if (grp != 0) return;
  }
  // partial[bg][n][kidx]: C/D map row = n (A rows), col = kidx (B cols)
  float* out = partial + (size_t)bg * G::N * G::K;
  const int hh = lane >> 5, col = lane & 31;
#pragma unroll
  for (int nt = 0; nt < G::NT; ++nt)
#pragma unroll
    for (int k = 0; k < G::KTW; ++k) {
      const int kl = wave + 4 * k;
      const int kt = kt0 + kl;
      if (kl < G::KTB && kt < G::KT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int n = nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          out[(size_t)n * G::K + kt * 32 + col] = acc[nt][k][r];
        }
      }
    }
}

// Sum the [G][N][K] partials (kidx order (ky,kx,c)) and the [G][N] bias partials.
// Block = 64 outputs x 4 waves; wave w sums partials g = w, w+4, ... (coalesced, 4x the
// loads in flight), fixed-order combine in LDS; writes the reference [N][C][KH][KW] grad.
__global__ __launch_bounds__(256) void wgrad_reduce_k(const float* __restrict__ partial,
                                                      const float* __restrict__ bpart, int G, int N, int C, int KH,
                                                      int KW, float* __restrict__ grad, float* __restrict__ bias_grad) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = C * KH * KW;
  const int e = blockIdx.x * 64 + lane;
  const int total = N * K + N;
  float s = 0.f;
  if (e < N * K) {
#pragma unroll 4
    for (int g = wave; g < G; g += 4) s += partial[(size_t)g * N * K + e];
  } else if (e < total) {
#pragma unroll 4
    for (int g = wave; g < G; g += 4) s += bpart[(size_t)g * N + (e - N * K)];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < total) {
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if (e < N * K) {
      const int n = e / K, kidx = e % K;
      const int c = kidx % C, tap = kidx / C;
      grad[((n * C + c) * KH + tap / KW) * KW + tap % KW] = t;
    } else {
      bias_grad[e - N * K] = t;
    }
  }
}

template <class G>
static void launch_wgrad(const void* x, FrameSrc fs, const uint16_t* dy, const uint16_t* mask, int B, float* ws,
                         float* grad, float* bias_grad, hipStream_t s) {
  const int grid = std::min(G::GRID, B);  // batch slices; x KSPLIT kidx groups
  float* partial = ws;
  float* bpart = ws + (size_t)G::GRID * G::N * G::K;
  wgrad_k<G><<<grid * G::KSPLIT, 256 * G::GROUPS, 0, s>>>(x, fs, dy, mask, B, grid, partial, bpart);
  LAUNCH_CHECK();
  if (!grad) return;  // partials only: grad_finalize reduces them with the other layers'
  const int total = G::N * G::K + G::N;
  wgrad_reduce_k<<<(total + 63) / 64, 256, 0, s>>>(partial, bpart, grid, G::N, G::C, G::KH, G::KW, grad, bias_grad);
  LAUNCH_CHECK();
}

size_t wgrad_workspace_floats(int layer) {
  switch (layer) {
    case 1: return (size_t)WG1::GRID * WG1::N * (WG1::K + 1);
    case 2: return (size_t)WG2::GRID * WG2::N * (WG2::K + 1);
    case 3: return (size_t)WG3::GRID * WG3::N * (WG3::K + 1);
    default: throw std::invalid_argument("wgrad layer");
  }
}

void conv_wgrad(int layer, const void* x, const int* ids, const int* idx, const uint16_t* dy, const uint16_t* dy_mask,
                int B, float* workspace, float* grad, float* bias_grad, hipStream_t s) {
  if (B <= 0) return;
  const FrameSrc fs{reinterpret_cast<const uint8_t*>(x), ids, idx};
  switch (layer) {
    case 1: launch_wgrad<WG1>(x, fs, dy, dy_mask, B, workspace, grad, bias_grad, s); break;
    case 2: launch_wgrad<WG2>(x, fs, dy, dy_mask, B, workspace, grad, bias_grad, s); break;
    case 3: launch_wgrad<WG3>(x, fs, dy, dy_mask, B, workspace, grad, bias_grad, s); break;
    default: throw std::invalid_argument("conv_wgrad: layer must be 1, 2 or 3");
  }
}

// ------------------------------------------------------------------ grad finalize
// One launch for every batch-sliced gradient reduction of the learner step: the three conv
// wgrad partial sets and the dqn_heads_bwd head/FC1-bias partials (previously four launches).
// Each workgroup owns 64 outputs of one job; its 4 waves split the partial slices and the
// slices are summed in a fixed order (deterministic).
int wgrad_grid(int layer, int B) {
  switch (layer) {
    case 1: return std::min(WG1::GRID, B);
    case 2: return std::min(WG2::GRID, B);
    case 3: return std::min(WG3::GRID, B);
    default: throw std::invalid_argument("wgrad layer");
  }
}

// outputs per workgroup: 64 when the 4 waves split many slices (G >= kWideG), 256 (one per
// thread, 4 independent chains) when the job has few slices; kind 2 (FC1 rows): one row of
// 3136 per workgroup, transposed through LDS so reads and writes are both coalesced
constexpr int kWideG = 16;
constexpr int kRowLen = 49 * 64;
// norm-only job: 8 elements per thread (3136 -> 392 workgroups for the FC1 gradient: fewer
// partials for every optimizer workgroup to re-reduce).  A last-workgroup (ticket) reduction
// of the partials was measured 5x slower (50 vs 9.5 us): each workgroup's device-scope release
// fence writes back the XCD L2.
constexpr int kNormOnlyPer = 256 * 8;

__host__ __device__ inline int finalize_blocks(const FinalizeJob& j) {
  if (j.kind == 2) return j.n_main / kRowLen;
  if (j.kind == 3) return (j.n_main + kNormOnlyPer - 1) / kNormOnlyPer;
  const int per = j.G >= kWideG ? 64 : 256;
  return (j.n_main + j.n_bias + per - 1) / per;
}

__device__ __forceinline__ void finalize_sumsq_q(double q, const FinalizeSet& fs, int gb) {
  // block-wide fixed-order sum of the threads' q (all 256 threads call this)
  __shared__ double red[4];
  q = wave_sum(q);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = q;
  __syncthreads();
  if (threadIdx.x == 0) fs.sumsq[gb] = (red[0] + red[1]) + (red[2] + red[3]);
}

__device__ __forceinline__ void finalize_sumsq(float v, const FinalizeSet& fs, bool active, int gb) {
  finalize_sumsq_q(active ? (double)v * (double)v : 0.0, fs, gb);
}

// r (stage 3): the top walk of the learner's priority-tree write riding the launch as block 0
// (tree_dev.h tree_ride; the finalize blocks and their sum-of-squares partials keep their index)
__global__ __launch_bounds__(256) void grad_finalize_k(FinalizeSet fs, TreeRide r) {
  __shared__ float red[4][64];
  __shared__ float row[kRowLen];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int gb = blockIdx.x;
  if (r.stage && tree_ride(r, r.nhost, &red[0][0], &gb)) return;  // (block-uniform role)
  int j = 0;
  while (j + 1 < fs.n && gb >= fs.job[j + 1].block0) ++j;
  const FinalizeJob& jb = fs.job[j];
  if (jb.kind == 3) {  // norm only: the gradient was written in place by its producer
    if (!fs.sumsq) return;
    const int e0 = (gb - jb.block0) * kNormOnlyPer + threadIdx.x;
    float v[8];
    // unconditional loads from clamped indices, zeroed after: guarded, each load compiled to a
    // branch + wait (8 serial round trips per workgroup)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = jb.part[min(e0 + 256 * k, max(jb.n_main - 1, 0))];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = e0 + 256 * k < jb.n_main ? v[k] : 0.f;
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) q += (double)v[k] * (double)v[k];
    finalize_sumsq_q(q, fs, gb);
    return;
  }
  if (jb.kind == 2) {  // FC1 weight rows: natural [n][p*64 + c] -> reference [n][c*49 + p]
    const int n = gb - jb.block0;
    const float* src = jb.part + (size_t)n * kRowLen;
    // the thread's 13 elements of each slice loaded together (clamped index, zeroed after):
    // a loop load -> store per element paid a round trip each
    constexpr int kPer = (kRowLen + 255) / 256;
    float t[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) t[i] = src[min((int)threadIdx.x + 256 * i, kRowLen - 1)];
    for (int g = 1; g < jb.G; ++g) {
#pragma unroll
      for (int i = 0; i < kPer; ++i) t[i] += src[(size_t)g * jb.pstride + min((int)threadIdx.x + 256 * i, kRowLen - 1)];
    }
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int k = threadIdx.x + 256 * i;
      if (k < kRowLen) {
        row[(k & 63) * 49 + (k >> 6)] = t[i];
        q += t[i] * t[i];
      }
    }
    __syncthreads();
    float* dst = jb.out[0] + (size_t)n * kRowLen;
    for (int e = threadIdx.x; e < kRowLen; e += 256) dst[e] = row[e];
    if (fs.sumsq) {
      // per-thread fp32 partial of <= 13 squares, then the fixed-order fp64 block sum
      __shared__ double rq[4];
      double d = wave_sum((double)q);
      if (lane == 0) rq[wave] = d;
      __syncthreads();
      if (threadIdx.x == 0) fs.sumsq[gb] = (rq[0] + rq[1]) + (rq[2] + rq[3]);
    }
    return;
  }
  const int total = jb.n_main + jb.n_bias;
  int e;
  float t = 0.f;
  bool have = false;
  if (jb.G >= kWideG) {
    e = (gb - jb.block0) * 64 + lane;
    float s = 0.f;
    // (16 slices per unrolled batch: the loads of a batch are in flight together, the adds
    // stay in slice order)
    if (e < jb.n_main) {
#pragma unroll 16
      for (int g = wave; g < jb.G; g += 4) s += jb.part[(size_t)g * jb.pstride + e];
    } else if (e < total) {
#pragma unroll 16
      for (int g = wave; g < jb.G; g += 4) s += jb.bpart[(size_t)g * jb.bstride + (e - jb.n_main)];
    }
    red[wave][lane] = s;
    __syncthreads();
    have = wave == 0 && e < total;
    if (have) t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  } else {
    e = (gb - jb.block0) * 256 + threadIdx.x;
    have = e < total;
    if (have) {
      const float* src = e < jb.n_main ? jb.part + e : jb.bpart + (e - jb.n_main);
      const size_t st = e < jb.n_main ? (size_t)jb.pstride : (size_t)jb.bstride;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      int g = 0;
      for (; g + 4 <= jb.G; g += 4) {
        s0 += src[(size_t)g * st];
        s1 += src[(size_t)(g + 1) * st];
        s2 += src[(size_t)(g + 2) * st];
        s3 += src[(size_t)(g + 3) * st];
      }
      for (; g < jb.G; ++g) s0 += src[(size_t)g * st];
      t = (s0 + s1) + (s2 + s3);
    }
  }
  if (fs.sumsq) finalize_sumsq(t, fs, have, gb);
  if (!have) return;
  if (jb.kind == 0) {  // conv: [N][KH*KW*C] (c fastest) -> reference [N][C][KH][KW]
    if (e < jb.n_main) {
      const int K = jb.C * jb.KH * jb.KW, n = e / K, kidx = e % K, c = kidx % jb.C, tap = kidx / jb.C;
      jb.out[0][((n * jb.C + c) * jb.KH + tap / jb.KW) * jb.KW + tap % jb.KW] = t;
    } else {
      jb.out[1][e - jb.n_main] = t;
    }
  } else {  // heads: [A][128] W_adv2 | [128] W_val2 | [A] b_adv2 | [1] b_val2 | [128] b_adv1 | [128] b_val1
    const int A = jb.C;
    if (e < A * 128) jb.out[0][e] = t;
    else if (e < (A + 1) * 128) jb.out[2][e - A * 128] = t;
    else if (e < (A + 1) * 128 + A) jb.out[1][e - (A + 1) * 128] = t;
    else if (e < (A + 1) * 129) jb.out[3][0] = t;
    else {
      const int n = e - (A + 1) * 129;
      if (n < 128) jb.out[4][n] = t; else jb.out[5][n - 128] = t;
    }
  }
}

int grad_finalize(FinalizeSet fs, hipStream_t s, const TreeRide* ride) {
  if (fs.n < 1 || fs.n > kMaxFinalizeJobs) throw std::invalid_argument("grad_finalize: 1..6 jobs");
  int blocks = 0;
  for (int j = 0; j < fs.n; ++j) {
    fs.job[j].block0 = blocks;
    blocks += finalize_blocks(fs.job[j]);
  }
  TreeRide r{};
  if (ride && ride->stage) {
    if (ride->stage != 3) throw std::invalid_argument("grad_finalize: takes the top-walk rider only");
    r = *ride;
    r.nhost = blocks;
  }
  grad_finalize_k<<<blocks + tree_ride_blocks(r), 256, 0, s>>>(fs, r);
  LAUNCH_CHECK();
  return blocks;
}

int grad_finalize_blocks(const FinalizeSet& fs) {
  int blocks = 0;
  for (int j = 0; j < fs.n; ++j) blocks += finalize_blocks(fs.job[j]);
  return blocks;
}

FinalizeJob conv_finalize_job(int layer, int B, const float* ws, float* grad, float* bias_grad) {
  FinalizeJob j{};
  auto fill = [&](auto geo) {
    using G = decltype(geo);
    j.kind = 0;
    j.G = std::min(G::GRID, B);
    j.part = ws;
    j.pstride = G::N * G::K;
    j.bpart = ws + (size_t)G::GRID * G::N * G::K;
    j.bstride = G::N;
    j.n_main = G::N * G::K;
    j.n_bias = G::N;
    j.C = G::C;
    j.KH = G::KH;
    j.KW = G::KW;
  };
  switch (layer) {
    case 1: fill(WG1{}); break;
    case 2: fill(WG2{}); break;
    case 3: fill(WG3{}); break;
    default: throw std::invalid_argument("conv_finalize_job: layer");
  }
  j.out[0] = grad;
  j.out[1] = bias_grad;
  return j;
}

FinalizeJob f32_fc1_finalize_job(int half, int G, const float* ws, float* grad) {
  // fp32 learner: G batch slices of FC1 weight-gradient partials [G][256][p*64 + c]
  // (f32_fc1_bwd_split) -> reference [n][c*49 + p], same row-transpose job as the bf16 slabs
  FinalizeJob j = fc1_finalize_job(half, ws, grad);
  j.G = G;
  return j;
}

FinalizeJob fc1_finalize_job(int half, const float* ws, float* grad) {
  // [G][256][7*7*64] natural (p, c) order -> reference [n][c*49 + p] (row-transpose job)
  constexpr int K = 49 * 64;
  FinalizeJob j{};
  j.kind = 2;
  j.G = fc1_bwd_slices();
  j.part = ws + (size_t)half * 128 * K;
  j.pstride = 256 * K;
  j.bpart = nullptr;
  j.bstride = 0;
  j.n_main = 128 * K;
  j.n_bias = 0;
  j.C = 64;
  j.KH = 7;
  j.KW = 7;
  j.out[0] = grad;
  j.out[1] = nullptr;
  return j;
}

FinalizeJob heads_finalize_job(int G, int A, const float* part, float* g_wadv2, float* g_badv2, float* g_wval2,
                               float* g_bval2, float* g_badv1, float* g_bval1) {
  FinalizeJob j{};
  const int stride = (A + 1) * 128 + (A + 1) + 256;
  j.kind = 1;
  j.G = G;
  j.part = part;
  j.pstride = stride;
  j.bpart = part;
  j.bstride = stride;
  j.n_main = stride;
  j.n_bias = 0;
  j.C = A;
  j.out[0] = g_wadv2;
  j.out[1] = g_badv2;
  j.out[2] = g_wval2;
  j.out[3] = g_bval2;
  j.out[4] = g_badv1;
  j.out[5] = g_bval1;
  return j;
}

// fp32 [N][C][KH][KW] -> bf16 W^T [KH][KW][C][N]
__global__ void pack_conv_wt_k(const float* __restrict__ src, uint16_t* __restrict__ dst, int N, int C, int KH,
                               int KW) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = N * C * KH * KW;
  if (i >= total) return;
  const int n = i % N, c = (i / N) % C, kx = (i / (N * C)) % KW, ky = i / (N * C * KW);
  dst[i] = f2bf(src[((n * C + c) * KH + ky) * KW + kx]);
}

void pack_conv_wt(const float* src, uint16_t* dst, int N, int C, int KH, int KW, hipStream_t s) {
  const int total = N * C * KH * KW;
  pack_conv_wt_k<<<(total + 255) / 256, 256, 0, s>>>(src, dst, N, C, KH, KW);
  LAUNCH_CHECK();
}

}  // namespace apex
