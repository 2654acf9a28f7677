// MFMA kernels for the Nature-CNN dueling Q-network on gfx950.
//
// Layouts (chosen for CDNA4, not copied from any NCHW/cuDNN convention):
//   * activations are channels-last bf16: a1 [B][400][32], a2 [B][81][64], a3 [B][49][64]
//     (a3 flattened as p*64+c; the FC1 weight is repacked to that order);
//   * conv weights are packed bf16 [N][KH][KW][C] (== channels_last of [N][C][KH][KW]), so
//     the implicit-GEMM K index is (ky, kx, c) with c fastest and every MFMA A/B fragment
//     (8 consecutive k) is ONE 16-byte LDS read.
//   * the u8 frames of the replay are converted to bf16 (exact for 0..255) while
//     being staged into LDS -- no separate cast kernel, no NCHW->NHWC transpose kernel.
//
// conv_fwd: persistent workgroups (4 waves) stage the packed weights into LDS once, then
// loop over sample pairs: stage both samples' input into LDS (padded pixel stride to break
// the 2-4 way ds_read_b128 bank conflicts of stride-S pixel rows), and each wave runs whole
// 32x32 output tiles as a chain of v_mfma_f32_32x32x16_bf16 over K, with the bias + ReLU +
// bf16 pack fused into the epilogue.
#include "common.h"
#include "kernels.h"

namespace apex {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int H_, int W_, int C_, int KH_, int KW_, int S_, int N_>
struct ConvGeo {
  static constexpr int H = H_, W = W_, C = C_, KH = KH_, KW = KW_, S = S_, N = N_;
  static constexpr int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1, P = OH * OW;
  static constexpr int K = KH * KW * C, KSTEPS = K / 16;
  static constexpr int MT = (P + 31) / 32, NT = N / 32;
  static constexpr int PIX = (C == 4) ? 8 : (C * 2 + 16);  // LDS bytes per input pixel (padded)
  // LDS bytes of padding after every input row: chosen with the ds_read_b128 bank model
  // (MI355X_MICROARCH §LDS: 4 groups of 16 lanes, bank (a/4) % 64) over the A-fragment
  // reads of every (M tile, k-step): conv2 11.3 -> 8.0 LDS cycles per read, conv3
  // 8.0 -> 5.0 (ideal 4; pixel strides stay 16-byte aligned)
  static constexpr int ROWPAD = (C == 32) ? 16 : ((C == 64) ? 224 : 0);
  static constexpr int ROW = W * PIX + ROWPAD;
  static constexpr int X_BYTES = H * ROW;
  static constexpr int W_ROW = K * 2 + 16;                 // LDS bytes per weight row (padded)
  static constexpr int W_BYTES = N * W_ROW;
  static constexpr int SPW = 2;                             // samples per workgroup iteration
  static constexpr int LDS = SPW * X_BYTES + W_BYTES;
  static_assert(K % 16 == 0, "K must be a multiple of 16");
  static_assert(N % 32 == 0, "N must be a multiple of 32");
};

using Conv1 = ConvGeo<84, 84, 4, 8, 8, 4, 32>;
using Conv2 = ConvGeo<20, 20, 32, 4, 4, 2, 64>;
using Conv3 = ConvGeo<9, 9, 64, 3, 3, 1, 64>;
static_assert(Conv1::P == 400 && Conv2::P == 81 && Conv3::P == 49, "Nature-CNN geometry");
static_assert(Conv2::LDS + 8 * TILE_EP_BYTES <= 160 * 1024 && Conv3::LDS + 8 * TILE_EP_BYTES <= 160 * 1024, "LDS");

// Stage one sample's input into LDS as padded NHWC bf16 (blockDim must be 256).
template <class G, bool U8IN>
__device__ __forceinline__ void stage_input(const void* __restrict__ in, const FrameSrc& fs, int b, char* xs) {
  if constexpr (U8IN) {
    static_assert(G::C == 4 && G::PIX == 8, "u8 path is the 4-frame stack");
    stage_frames_bf16<G::H * G::W>(fs, b, xs);
  } else {
    constexpr int CH16 = G::C / 8;  // 16-byte chunks per pixel
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(in) +
                                                      (size_t)b * G::H * G::W * G::C * 2);
    stage_all<G::H * G::W * CH16>(src, xs, [](int q) {
      const int pi = q / CH16;
      return (pi / G::W) * G::ROW + (pi % G::W) * G::PIX + (q % CH16) * 16;
    });
  }
}

template <class G>
__device__ __forceinline__ void stage_weights(const uint16_t* __restrict__ wp, char* ws) {
  constexpr int CH16 = G::K / 8;
  stage_all<G::N * CH16>(reinterpret_cast<const uint4*>(wp), ws,
                            [](int q) { return (q / CH16) * G::W_ROW + (q % CH16) * 16; });
}

// LDS byte offset (relative to the output pixel's window origin) of implicit-GEMM k index kk
// (8 consecutive k starting at kk are contiguous: one tap x 8 channels, or for the 4-channel
// frame stack two adjacent taps x 4 channels).
template <class G>
__device__ __forceinline__ constexpr int a_off(int kk) {
  if constexpr (G::C == 4) {
    const int ky = kk / (4 * G::KW), kx = (kk / 4) % G::KW;
    return ky * G::ROW + kx * G::PIX;
  } else {
    const int tap = kk / G::C, c0 = kk % G::C;
    return (tap / G::KW) * G::ROW + (tap % G::KW) * G::PIX + c0 * 2;
  }
}

// Problem set (kernels.h ConvSet): sample pairs never straddle two problems (a problem of
// B samples has ceil(B/2) pairs); the weights are restaged only when the problem's weight
// pointer changes (the learner's Q(s) and Q(s') passes share the online weights).
// Eight waves per workgroup: the LDS footprint (two samples + the weights) allows one
// workgroup per CU, and with four waves each SIMD had a single wave to hide every LDS and
// MFMA latency; waves 4-7 share the staged tiles (waves 0-3 stage: the copy helpers are
// written for 256 threads).
constexpr int kConvWaves = 8;

template <class G, bool U8IN>
__global__ __launch_bounds__(64 * kConvWaves) void conv_fwd_k(ConvSet set) {
  __shared__ __attribute__((aligned(16))) char smem[G::LDS + kConvWaves * TILE_EP_BYTES];
  char* ws = smem + G::SPW * G::X_BYTES;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  const bool stager = threadIdx.x < 256;  // wave-uniform
  char* ep = smem + G::LDS + wave * TILE_EP_BYTES;  // per-wave epilogue scratch
  const int B = set.B, PP = (B + G::SPW - 1) / G::SPW, pairs = set.n * PP;
  const uint16_t* wcur = nullptr;
  // bf16 inputs: the NEXT pair's two samples are prefetched into registers while this
  // pair multiplies (one workgroup per CU: without it every pair paid a full HBM round
  // trip before its MFMAs could start)
  static_assert(G::SPW == 2, "two prefetch blocks");
  constexpr int XCH = G::H * G::W * G::C / 8;  // 16-byte chunks per sample
  constexpr int CH16 = G::C / 8;
  Pf8 nx0, nx1;
  auto sample_src = [&](int pb, int b) {
    return reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(set.p[pb].in) +
                                          (size_t)b * G::H * G::W * G::C * 2);
  };
  auto issue = [&](int q) {
    const int pb = q / PP, b0 = (q - pb * PP) * G::SPW;
    pf_load<XCH>(nx0, sample_src(pb, b0));
    pf_load<XCH>(nx1, sample_src(pb, b0 + 1 < B ? b0 + 1 : b0));
  };
  if constexpr (!U8IN) {
    static_assert(XCH <= 8 * 256, "one Pf8 per sample");
    if (stager && (int)blockIdx.x < pairs) issue(blockIdx.x);
  }
  for (int q = blockIdx.x; q < pairs; q += gridDim.x) {
    const int pb = q / PP, b0 = (q - pb * PP) * G::SPW;
    const ConvProb& pr = set.p[pb];
    const FrameSrc fs{reinterpret_cast<const uint8_t*>(pr.in), pr.ids, pr.idx};
    __syncthreads();
    if (pr.w != wcur) {  // block-uniform
      wcur = pr.w;
      if (stager) stage_weights<G>(wcur, ws);
    }
    if (stager) {
      if constexpr (U8IN) {
#pragma unroll
        for (int sw = 0; sw < G::SPW; ++sw)
          if (b0 + sw < B) stage_input<G, U8IN>(pr.in, fs, b0 + sw, smem + sw * G::X_BYTES);
      } else {
        auto off = [](int c) {
          const int pi = c / CH16;
          return (pi / G::W) * G::ROW + (pi % G::W) * G::PIX + (c % CH16) * 16;
        };
        pf_store<XCH>(nx0, smem, off);
        if (b0 + 1 < B) pf_store<XCH>(nx1, smem + G::X_BYTES, off);
      }
    }
    __syncthreads();
    if constexpr (!U8IN) {
      if (stager && q + (int)gridDim.x < pairs) issue(q + gridDim.x);
    }
    const float* bias = pr.bias;
    uint16_t* out = pr.out;
    constexpr int ITEMS = G::SPW * G::MT * G::NT;
    for (int it = wave; it < ITEMS; it += kConvWaves) {
      const int sw = it / (G::MT * G::NT);
      const int mt = (it / G::NT) % G::MT;
      const int nt = it % G::NT;
      const int b = b0 + sw;
      if (b >= B) continue;  // wave-uniform
      const char* xs = smem + sw * G::X_BYTES;
      int p = mt * 32 + r32;
      const int pc = p < G::P ? p : G::P - 1;
      const int oy = pc / G::OW, ox = pc % G::OW;
      const char* abase = xs + (G::S * oy) * G::ROW + (G::S * ox) * G::PIX;
      const char* bbase = ws + (nt * 32 + r32) * G::W_ROW + h * 16;
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        // after unrolling, both candidate offsets are compile-time constants
        const int off = h ? a_off<G>(16 * s + 8) : a_off<G>(16 * s);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(abase + off);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(bbase + 32 * s);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc, 0, 0, 0);
      }
      const float bn = bias[nt * 32 + r32];
      const long base = (long)b * G::P * G::N + nt * 32;
      tile_store_bf16(acc, ep, [bn](int, int, float v) { return f2bf(fmaxf(v + bn, 0.f)); },
                      [&](int row) -> long {
                        const int pp = mt * 32 + row;
                        return pp < G::P ? base + (long)pp * G::N : -1;
                      }, out);
    }
  }
}

template <class G, bool U8IN>
static void launch_conv_fwd(const ConvSet& set, hipStream_t s) {
  const int pairs = set.n * ((set.B + G::SPW - 1) / G::SPW);
  if (pairs <= 0) return;
  // one workgroup per CU (the LDS footprint allows no more): 256 persistent workgroups
  const int grid = std::min(pairs, 256);
  conv_fwd_k<G, U8IN><<<grid, 64 * kConvWaves, 0, s>>>(set);
  LAUNCH_CHECK();
}

void conv_fwd_multi(int layer, const ConvSet& set, hipStream_t s) {
  if (set.n < 1 || set.n > kMaxProbs) throw std::invalid_argument("conv_fwd: 1..3 problems");
  switch (layer) {
    case 1: conv1_fwd_multi(set, s); break;  // conv1_kernels.hip
    case 2: launch_conv_fwd<Conv2, false>(set, s); break;
    case 3: launch_conv_fwd<Conv3, false>(set, s); break;
    default: throw std::invalid_argument("conv_fwd: layer must be 1, 2 or 3");
  }
}

void conv_fwd(int layer, const void* in, const int* ids, const int* idx, const uint16_t* wp, const float* bias,
              uint16_t* out, int B, hipStream_t s) {
  ConvSet set{};
  set.p[0] = ConvProb{in, ids, idx, wp, bias, out};
  set.n = 1;
  set.B = B;
  conv_fwd_multi(layer, set, s);
}

// ------------------------------------------------------------------ dueling heads
// z [nsplit][B][256] = FC1 pre-activation split-K partials (fc_kernels.hip; adv hidden
// 0..127 | value hidden 128..255, no bias), summed here in fixed order.
// A workgroup stages the head weights (A+1)x128 in LDS and handles 4 rows (one per
// wave, B/4 workgroups so a 512-row batch spreads over 128 CUs): h = relu(z + b1) ->
// LDS; lane a < A computes adv_a, lane A the value; q = V + A - mean(A)
// (model.py:60-68).  h is kept (fp32) for the backward.
constexpr int kHeadRows = 4;

__global__ __launch_bounds__(256) void heads_fwd_k(HeadsSet set) {
  // row a (a < A: adv, a == A: value); pitch 132 floats: 16-byte rows for ds_read_b128, lane
  // a's read starting at bank 4a (mod 64), so 16 lanes per LDS cycle are conflict-free
  constexpr int kWp = 132;
  __shared__ __attribute__((aligned(16))) float ws[64 * kWp];
  __shared__ __attribute__((aligned(16))) float hs[4][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int B = set.B, A = set.A, nsplit = set.nsplit, RB = (B + kHeadRows - 1) / kHeadRows;
  int pb, rb;
  if (set.xcd_map) {
    // The learner's 3 x 512 rows: fc1_fwd's grid (12 row tiles m, 14 splits s) puts slab
    // (m, s) on XCD (m + 12 s) % 8, i.e. row tile m's partials live in the L2s of the two
    // XCDs x == m (mod 4).  Deal this kernel's 384 row blocks so each reads its row tile
    // from those L2s (workgroups go to XCD blockIdx % 8): XCD pair {c, c + 4} takes the
    // 96 row blocks of tiles c, c + 4, c + 8 (48 each, balanced).
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, c = x & 3;
    const int k = j + 48 * (x >> 2);
    pb = k / 32;
    rb = c * 32 + (k & 31);
  } else {
    pb = blockIdx.x / RB;
    rb = blockIdx.x - pb * RB;
  }
  const HeadsProb& pr = set.p[pb];
  const float* __restrict__ z = pr.z;
  static_assert(kHeadRows == 4, "one row per wave");
  const int b = rb * kHeadRows + wave;
  const bool valid = b < B;
  const float* zr = z + (size_t)(valid ? b : 0) * 256;
  // split-K slabs summed in fixed (slab) order; 4 columns per lane, 8 slabs (32 loads) in
  // flight ahead of the adds (the actor's 256-row FC1 uses 28 slabs: 2 in flight cost ~12 us).
  // The first 8 slabs' loads are issued BEFORE the head-weight staging: the two global round
  // trips overlap instead of following each other.
  const size_t sstride = (size_t)B * 256;
  constexpr int U = 8;
  float v[U][4];
  auto zload = [&](int sp) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[u][k] = sp + u < nsplit ? zr[(size_t)(sp + u) * sstride + lane + 64 * k] : 0.f;
  };
  zload(0);
  // head weights staged 8 loads at a time (a rolled load -> LDS store loop waits out one L2
  // round trip per element: ~10 per thread before the first row)
  const float* __restrict__ wa2 = pr.w_adv2;
  const float* __restrict__ wv2 = pr.w_val2;
  for (int e0 = threadIdx.x; e0 < (A + 1) * 128; e0 += 8 * 256) {
    float wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = min(e0 + 256 * u, (A + 1) * 128 - 1), a = e / 128, j = e % 128;
      wv[u] = a < A ? wa2[a * 128 + j] : wv2[j];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 256 * u;
      if (e < (A + 1) * 128) ws[(e / 128) * kWp + e % 128] = wv[u];
    }
  }
  const float bo = lane < A ? pr.b_adv2[lane] : (lane == A ? pr.b_val2[0] : 0.f);
  {
    float zs[4] = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < nsplit; sp += U) {
      if (sp > 0) zload(sp);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) zs[k] += v[u][k];  // adding 0.f past nsplit is exact
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = lane + 64 * k;
      const float bias = j < 128 ? pr.b_adv1[j] : pr.b_val1[j - 128];
      const float v = fmaxf(zs[k] + bias, 0.f);
      hs[wave][j] = v;
      if (pr.hout && valid) pr.hout[(size_t)b * 256 + j] = v;
    }
    __syncthreads();
    float o = 0.f;
    if (lane <= A) {  // 16-byte LDS reads, the same j-ordered fp32 chain as a scalar loop
      const f32x4v* wr = reinterpret_cast<const f32x4v*>(ws + lane * kWp);
      const f32x4v* hr = reinterpret_cast<const f32x4v*>(hs[wave] + (lane < A ? 0 : 128));
#pragma unroll 8
      for (int j = 0; j < 32; ++j) {
        const f32x4v hv = hr[j], wv = wr[j];
        o += hv[0] * wv[0];
        o += hv[1] * wv[1];
        o += hv[2] * wv[2];
        o += hv[3] * wv[3];
      }
      o += bo;
    }
    const float adv_sum = wave_sum(lane < A ? o : 0.f);
    const float v = __shfl(o, A, 64);
    const float qv = v + o - adv_sum / (float)A;
    if (valid && lane < A) pr.q[(size_t)b * A + lane] = qv;
    if (pb == 0 && set.act.eps != nullptr && valid) {
      // eps-greedy epilogue (select_actions_k's semantics and Philox draw): first argmax
      // by a wave (value, index) reduction, ties to the lower index
      float bv = lane < A ? qv : -INFINITY;
      int bi = lane < A ? lane : 64;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      if (lane == 0) {
        float u[4];
        uniform4(set.act.seed, (uint64_t)b, set.act.counter ? (uint64_t)set.act.counter[0] : 0ull, u);
        if (!(u[0] > set.act.eps[b])) {
          const int r = (int)(u[1] * (float)A);
          bi = r < A ? r : A - 1;
        }
        set.act.actions[b] = bi;
      }
    }
  }
}

void heads_fwd_multi(const HeadsSet& set, hipStream_t s) {
  if (set.A < 1 || set.A > 63) throw std::invalid_argument("heads_fwd: 1 <= A <= 63");
  if (set.nsplit < 1 || set.nsplit > 64) throw std::invalid_argument("heads_fwd: 1 <= nsplit <= 64");
  if (set.n < 1 || set.n > kMaxProbs) throw std::invalid_argument("heads_fwd: 1..3 problems");
  if (set.B <= 0) return;
  HeadsSet hs = set;
  // the mapping assumes fc1_fwd's 128-row tiles x 14 splits over 3 x 512 rows (FcSet)
  hs.xcd_map = (set.n == 3 && set.B == 512 && set.nsplit == 14 && kHeadRows == 4) ? 1 : 0;
  heads_fwd_k<<<set.n * ((set.B + kHeadRows - 1) / kHeadRows), 256, 0, s>>>(hs);
  LAUNCH_CHECK();
}

void heads_fwd(const float* z, int nsplit, const float* b_adv1, const float* b_val1, const float* w_adv2,
               const float* b_adv2, const float* w_val2, const float* b_val2, float* hout, float* q, int B, int A,
               hipStream_t s) {
  HeadsSet set{};
  set.p[0] = HeadsProb{z, b_adv1, b_val1, w_adv2, b_adv2, w_val2, b_val2, hout, q};
  set.n = 1;
  set.B = B;
  set.A = A;
  set.nsplit = nsplit;
  heads_fwd_multi(set, s);
}

// Backward of the heads for one row per wave:
//   dv = sum_a dq_a ; dadv_a = dq_a - mean(dq) ; dh_j = sum_a dadv_a W_adv2[a][j] (j<128),
//   dh_{128+j} = dv W_val2[j] ; dz = dh * (h > 0).
// Writes dz as fp32 (bias grads) and bf16 (FC1 GEMMs), and dA = [dadv | dv] for the head
// weight gradients.
__global__ __launch_bounds__(256) void heads_bwd_k(const float* __restrict__ dq, const float* __restrict__ h,
                                                   const float* __restrict__ w_adv2, const float* __restrict__ w_val2,
                                                   float* __restrict__ dA, float* __restrict__ dz,
                                                   uint16_t* __restrict__ dz_bf, int B, int A) {
  __shared__ float da_s[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + wave;
  const bool valid = b < B;
  const float g = (valid && lane < A) ? dq[(size_t)b * A + lane] : 0.f;
  const float tot = wave_sum(g);
  const float dadv = lane < A ? g - tot / (float)A : 0.f;
  if (lane < A) da_s[wave][lane] = dadv;
  if (valid && lane < A) dA[(size_t)b * (A + 1) + lane] = dadv;
  if (valid && lane == 0) dA[(size_t)b * (A + 1) + A] = tot;
  __syncthreads();
  if (!valid) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = lane + 64 * k;
    float d;
    if (j < 128) {
      d = 0.f;
      for (int a = 0; a < A; ++a) d += da_s[wave][a] * w_adv2[a * 128 + j];
    } else {
      d = tot * w_val2[j - 128];
    }
    d = h[(size_t)b * 256 + j] > 0.f ? d : 0.f;
    dz[(size_t)b * 256 + j] = d;
    dz_bf[(size_t)b * 256 + j] = f2bf(d);
  }
}

void heads_bwd(const float* dq, const float* h, const float* w_adv2, const float* w_val2, float* dA, float* dz,
               uint16_t* dz_bf, int B, int A, hipStream_t s) {
  if (A < 1 || A > 63) throw std::invalid_argument("heads_bwd: 1 <= A <= 63");
  heads_bwd_k<<<(B + 3) / 4, 256, 0, s>>>(dq, h, w_adv2, w_val2, dA, dz, dz_bf, B, A);
  LAUNCH_CHECK();
}

// Head/FC1-bias gradients as one batch reduction (replaces 2 GEMMs + 4 sums):
//   dW_adv2[a][j] = sum_b dadv[b][a] h[b][j]   dW_val2[j] = sum_b dv[b] h[b][128+j]
//   db_adv2[a] = sum_b dadv[b][a]   db_val2 = sum_b dv[b]   db_fc1[n] = sum_b dz[b][n]
// Stage 1: HG_SPLIT blocks x 256 threads (thread = hidden column j) over row slices ->
// fp32 partials; stage 2 sums the partials in fixed order (deterministic).
constexpr int HG_SPLIT = 64;  // 8 rows per block at B = 512: latency-bound, so spread wide
constexpr int HG_MAXA = 32;

__global__ __launch_bounds__(256) void heads_wgrad_partial_k(const float* __restrict__ dA, const float* __restrict__ h,
                                                             const float* __restrict__ dz, int B, int A,
                                                             float* __restrict__ part) {
  __shared__ float da_s[64][HG_MAXA + 1];
  const int j = threadIdx.x;
  const int rows = (B + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows, r1 = min(B, r0 + rows);
  float acc[HG_MAXA];
#pragma unroll
  for (int a = 0; a < HG_MAXA; ++a) acc[a] = 0.f;
  float dsum = 0.f, bsum = 0.f;  // db_fc1[j]; bias of head output (threads j <= A)
  for (int c0 = r0; c0 < r1; c0 += 64) {
    const int cn = min(64, r1 - c0);
    __syncthreads();
    for (int e = threadIdx.x; e < cn * (A + 1); e += 256) da_s[e / (A + 1)][e % (A + 1)] = dA[(size_t)(c0 + e / (A + 1)) * (A + 1) + e % (A + 1)];
    __syncthreads();
    for (int r = 0; r < cn; ++r) {
      const float hj = h[(size_t)(c0 + r) * 256 + j];
      dsum += dz[(size_t)(c0 + r) * 256 + j];
      if (j <= A) bsum += da_s[r][j];
      if (j < 128) {
#pragma unroll
        for (int a = 0; a < HG_MAXA; ++a)
          if (a < A) acc[a] += da_s[r][a] * hj;
      } else {
        acc[0] += da_s[r][A] * hj;
      }
    }
  }
  // partial layout per block: [A][128] adv, [128] val, [A] db_adv2, [1] db_val2, [256] db_fc1
  const int stride = (A + 1) * 128 + (A + 1) + 256;
  float* p = part + (size_t)blockIdx.x * stride;
  if (j < 128) {
    for (int a = 0; a < A; ++a) p[a * 128 + j] = acc[a];
  } else {
    p[A * 128 + (j - 128)] = acc[0];
  }
  if (j <= A) p[(A + 1) * 128 + j] = bsum;
  p[(A + 1) * 129 + j] = dsum;
}

__global__ void heads_wgrad_reduce_k(const float* __restrict__ part, int G, int A, float* __restrict__ g_wadv2,
                                     float* __restrict__ g_badv2, float* __restrict__ g_wval2,
                                     float* __restrict__ g_bval2, float* __restrict__ g_badv1,
                                     float* __restrict__ g_bval1) {
  const int stride = (A + 1) * 128 + (A + 1) + 256;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= stride) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // 4 independent chains: loads stay in flight
  int g = 0;
  for (; g + 4 <= G; g += 4) {
    s0 += part[(size_t)g * stride + e];
    s1 += part[(size_t)(g + 1) * stride + e];
    s2 += part[(size_t)(g + 2) * stride + e];
    s3 += part[(size_t)(g + 3) * stride + e];
  }
  for (; g < G; ++g) s0 += part[(size_t)g * stride + e];
  const float s = (s0 + s1) + (s2 + s3);
  if (e < A * 128) g_wadv2[e] = s;
  else if (e < (A + 1) * 128) g_wval2[e - A * 128] = s;
  else if (e < (A + 1) * 128 + A) g_badv2[e - (A + 1) * 128] = s;
  else if (e < (A + 1) * 129) g_bval2[0] = s;
  else {
    const int n = e - (A + 1) * 129;
    if (n < 128) g_badv1[n] = s; else g_bval1[n - 128] = s;
  }
}

void heads_wgrad(const float* dA, const float* h, const float* dz, int B, int A, float* ws, float* g_wadv2,
                 float* g_badv2, float* g_wval2, float* g_bval2, float* g_badv1, float* g_bval1, hipStream_t s) {
  if (A < 1 || A > HG_MAXA) throw std::invalid_argument("heads_wgrad: 1 <= A <= 32");
  const int G = std::min(HG_SPLIT, B);
  heads_wgrad_partial_k<<<G, 256, 0, s>>>(dA, h, dz, B, A, ws);
  LAUNCH_CHECK();
  const int stride = (A + 1) * 128 + (A + 1) + 256;
  heads_wgrad_reduce_k<<<(stride + 255) / 256, 256, 0, s>>>(ws, G, A, g_wadv2, g_badv2, g_wval2, g_bval2, g_badv1,
                                                           g_bval1);
  LAUNCH_CHECK();
}

size_t heads_wgrad_workspace_floats(int A) { return (size_t)HG_SPLIT * ((A + 1) * 128 + (A + 1) + 256); }

// ------------------------------------------------------------------ packing / masks
// conv weight fp32 [N][C][KH][KW] (reference layout) -> bf16 [N][KH][KW][C]
__global__ void pack_conv_w_k(const float* __restrict__ src, uint16_t* __restrict__ dst, int N, int C, int KH,
                              int KW) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // dst index
  const int total = N * C * KH * KW;
  if (i >= total) return;
  const int c = i % C, kx = (i / C) % KW, ky = (i / (C * KW)) % KH, n = i / (C * KW * KH);
  dst[i] = f2bf(src[((n * C + c) * KH + ky) * KW + kx]);
}

// FC1 weights: adv.0.weight / value.0.weight fp32 [128][C*P] (order c*P+p) -> bf16 [256][P*C]
__global__ void pack_fc1_k(const float* __restrict__ adv, const float* __restrict__ val, uint16_t* __restrict__ dst,
                           int P, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int F = P * C;
  if (i >= 256 * F) return;
  const int n = i / F, r = i % F, p = r / C, c = r % C;
  const float* src = n < 128 ? adv + (size_t)n * F : val + (size_t)(n - 128) * F;
  dst[i] = f2bf(src[c * P + p]);
}

// gradient of the packed FC1 weight (fp32 [256][P*C]) -> reference-layout grads (assign)
__global__ void unpack_fc1_grad_k(const float* __restrict__ gp, float* __restrict__ g_adv, float* __restrict__ g_val,
                                  int P, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // reference index
  const int F = P * C;
  if (i >= 256 * F) return;
  const int n = i / F, r = i % F, c = r / P, p = r % P;
  const float v = gp[(size_t)n * F + p * C + c];
  if (n < 128) g_adv[(size_t)n * F + r] = v; else g_val[(size_t)(n - 128) * F + r] = v;
}

// y = x * (a > 0) for bf16 tensors (ReLU backward through the stored activation)
__global__ void relu_mask_bf16_k(const uint16_t* __restrict__ g, const uint16_t* __restrict__ a,
                                 uint16_t* __restrict__ out, int64_t n8) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  uint4 gv = reinterpret_cast<const uint4*>(g)[i];
  const uint4 av = reinterpret_cast<const uint4*>(a)[i];
  uint32_t* gw = reinterpret_cast<uint32_t*>(&gv);
  const uint32_t* aw = reinterpret_cast<const uint32_t*>(&av);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // bf16 > 0  <=>  sign bit clear and not +0
    const uint32_t lo = aw[k] & 0xFFFF, hi = aw[k] >> 16;
    const uint32_t mlo = (lo != 0 && !(lo & 0x8000)) ? 0xFFFFu : 0u;
    const uint32_t mhi = (hi != 0 && !(hi & 0x8000)) ? 0xFFFF0000u : 0u;
    gw[k] &= (mlo | mhi);
  }
  reinterpret_cast<uint4*>(out)[i] = gv;
}

// u8 NCHW [B][4][84][84] -> bf16 NHWC [B][84][84][4] (the conv1 input for its weight gradient)
__global__ void u8_to_bf16_nhwc_k(const uint8_t* __restrict__ in, uint16_t* __restrict__ out, int B, int HW) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // group of 4 pixels
  const int64_t groups = (int64_t)B * HW / 4;
  if (g >= groups) return;
  const int64_t b = g / (HW / 4), off = (g % (HW / 4)) * 4;
  const uint8_t* src = in + b * 4 * HW + off;
  uint32_t v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = *reinterpret_cast<const uint32_t*>(src + c * HW);
  uint4 lo, hi;
  lo.x = pack_bf16x2_u8(v[0] & 0xFF, v[1] & 0xFF);
  lo.y = pack_bf16x2_u8(v[2] & 0xFF, v[3] & 0xFF);
  lo.z = pack_bf16x2_u8((v[0] >> 8) & 0xFF, (v[1] >> 8) & 0xFF);
  lo.w = pack_bf16x2_u8((v[2] >> 8) & 0xFF, (v[3] >> 8) & 0xFF);
  hi.x = pack_bf16x2_u8((v[0] >> 16) & 0xFF, (v[1] >> 16) & 0xFF);
  hi.y = pack_bf16x2_u8((v[2] >> 16) & 0xFF, (v[3] >> 16) & 0xFF);
  hi.z = pack_bf16x2_u8(v[0] >> 24, v[1] >> 24);
  hi.w = pack_bf16x2_u8(v[2] >> 24, v[3] >> 24);
  uint4* d = reinterpret_cast<uint4*>(out + (b * HW + off) * 4);
  d[0] = lo;
  d[1] = hi;
}

void pack_conv_w(const float* src, uint16_t* dst, int N, int C, int KH, int KW, hipStream_t s) {
  const int total = N * C * KH * KW;
  pack_conv_w_k<<<(total + 255) / 256, 256, 0, s>>>(src, dst, N, C, KH, KW);
  LAUNCH_CHECK();
}
void pack_fc1(const float* adv, const float* val, uint16_t* dst, int P, int C, hipStream_t s) {
  const int total = 256 * P * C;
  pack_fc1_k<<<(total + 255) / 256, 256, 0, s>>>(adv, val, dst, P, C);
  LAUNCH_CHECK();
}
void unpack_fc1_grad(const float* gp, float* g_adv, float* g_val, int P, int C, hipStream_t s) {
  const int total = 256 * P * C;
  unpack_fc1_grad_k<<<(total + 255) / 256, 256, 0, s>>>(gp, g_adv, g_val, P, C);
  LAUNCH_CHECK();
}
void relu_mask_bf16(const uint16_t* g, const uint16_t* a, uint16_t* out, int64_t n, hipStream_t s) {
  if (n % 8) throw std::invalid_argument("relu_mask_bf16: n must be a multiple of 8");
  const int64_t n8 = n / 8;
  relu_mask_bf16_k<<<(unsigned)((n8 + 255) / 256), 256, 0, s>>>(g, a, out, n8);
  LAUNCH_CHECK();
}
void u8_to_bf16_nhwc(const uint8_t* in, uint16_t* out, int B, int HW, hipStream_t s) {
  if (HW % 4) throw std::invalid_argument("u8_to_bf16_nhwc: HW must be a multiple of 4");
  const int64_t groups = (int64_t)B * HW / 4;
  u8_to_bf16_nhwc_k<<<(unsigned)((groups + 255) / 256), 256, 0, s>>>(in, out, B, HW);
  LAUNCH_CHECK();
}

}  // namespace apex
