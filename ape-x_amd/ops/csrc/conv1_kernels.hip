// conv1 forward (Conv 4->32, k8, s4 on 84x84 u8 frame stacks) for gfx950.
//
// The first conv dominates the forward pass (3.28 M MAC per sample, 3 learner passes + 1
// actor pass per Ape-X step).  Design (measured: the previous NHWC-bf16 staging kernel was
// bound by 8-way ds_write_b128 conflicts in its u8->bf16 staging and 16 VALU per MFMA):
//
//   * LDS holds the sample's 4 planes as bf16 [4][84][84] (56,448 B), converted ONCE per
//     input byte while staging (each byte feeds 4 output windows; converting per use cost
//     12 VALU per MFMA, measured), written with lane-contiguous 16-byte stores (conflict
//     free); two stages (double buffer) = 113 KB, one workgroup per CU.
//   * implicit-GEMM K order is (c, ky, kx) == the reference weight layout [32][4][8][8]:
//     the 8 k of one MFMA fragment are 8 consecutive kx = 16 consecutive bytes of one
//     plane row (two 8-byte-aligned ds_read_b64).
//   * all 32 output channels are one 32-wide N tile, so each wave keeps the whole B operand
//     (16 k-steps x 8 bf16 = 64 VGPRs) in registers for the life of the kernel: per MFMA
//     only the A fragment touches LDS.
//   * the next sample's frames are loaded into registers before the current sample's MFMA
//     loop and written to the other LDS stage after it (one barrier per sample).
//   * epilogue: bias + ReLU + bf16, channels-last a1 [B][400][32] (what conv2 reads).
#include "common.h"
#include "kernels.h"

namespace apex {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int C1_HW = 84 * 84;              // pixels per plane
constexpr int C1_STAGE = 4 * C1_HW * 2;     // 56,448 B per sample as bf16 planes
constexpr int C1_Q = 4 * C1_HW / 8;         // 3528 8-byte u8 chunks per sample
constexpr int C1_PER = (C1_Q + 255) / 256;  // 14 per thread
constexpr int C1_P = 400, C1_OW = 20, C1_MT = 13, C1_N = 32, C1_K = 256;

// 8 u8 (two dwords) -> 8 bf16: v_cvt_f32_ubyte{0..3} + v_cvt_pk_bf16_f32 (exact: integers
// 0..255 have 8 significant bits)
__device__ __forceinline__ uint4 u8x8_to_bf16(uint2 w) {
  bf16x8 r;
  r[0] = (__bf16)(float)(w.x & 0xFF);
  r[1] = (__bf16)(float)((w.x >> 8) & 0xFF);
  r[2] = (__bf16)(float)((w.x >> 16) & 0xFF);
  r[3] = (__bf16)(float)(w.x >> 24);
  r[4] = (__bf16)(float)(w.y & 0xFF);
  r[5] = (__bf16)(float)((w.y >> 8) & 0xFF);
  r[6] = (__bf16)(float)((w.y >> 16) & 0xFF);
  r[7] = (__bf16)(float)(w.y >> 24);
  return __builtin_bit_cast(uint4, r);
}

// 14 8-byte chunks per thread in named registers (an array ends up in scratch: SROA runs
// before the loops are unrolled)
struct Stage14 {
  uint2 v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13;
};
static_assert(C1_PER == 14, "Stage14 holds 14 chunks per thread");

struct Planes {
  const uint2 *p0, *p1, *p2, *p3;
};

__device__ __forceinline__ Planes planes_of(const FrameSrc& f, int b) {
  return {reinterpret_cast<const uint2*>(frame_plane(f, b, 0, C1_HW)),
          reinterpret_cast<const uint2*>(frame_plane(f, b, 1, C1_HW)),
          reinterpret_cast<const uint2*>(frame_plane(f, b, 2, C1_HW)),
          reinterpret_cast<const uint2*>(frame_plane(f, b, 3, C1_HW))};
}

__device__ __forceinline__ uint2 load_chunk(const Planes& pl, int q) {
  // chunk q: plane q / 882, byte offset (q % 882) * 8
  const int c = q / (C1_HW / 8), o = q % (C1_HW / 8);
  const uint2* p = c == 0 ? pl.p0 : (c == 1 ? pl.p1 : (c == 2 ? pl.p2 : pl.p3));
  return p[o];
}

__device__ __forceinline__ void load_sample(const FrameSrc& f, int b, Stage14& st) {
  const Planes pl = planes_of(f, b);  // 4 frame-id lookups per sample, not per chunk
  const int t = threadIdx.x;
  st.v0 = load_chunk(pl, t);
  st.v1 = load_chunk(pl, t + 256);
  st.v2 = load_chunk(pl, t + 512);
  st.v3 = load_chunk(pl, t + 768);
  st.v4 = load_chunk(pl, t + 1024);
  st.v5 = load_chunk(pl, t + 1280);
  st.v6 = load_chunk(pl, t + 1536);
  st.v7 = load_chunk(pl, t + 1792);
  st.v8 = load_chunk(pl, t + 2048);
  st.v9 = load_chunk(pl, t + 2304);
  st.v10 = load_chunk(pl, t + 2560);
  st.v11 = load_chunk(pl, t + 2816);
  st.v12 = load_chunk(pl, t + 3072);
  if (t + 3328 < C1_Q) st.v13 = load_chunk(pl, t + 3328);
}

// u8 -> bf16 once per input byte while writing LDS: lane-contiguous 16-B stores
// (8 lanes cover a 128-B bank row: conflict-free ds_write_b128)
__device__ __forceinline__ void store_sample(char* xs, const Stage14& st) {
  uint4* d = reinterpret_cast<uint4*>(xs);
  const int t = threadIdx.x;
  d[t] = u8x8_to_bf16(st.v0);
  d[t + 256] = u8x8_to_bf16(st.v1);
  d[t + 512] = u8x8_to_bf16(st.v2);
  d[t + 768] = u8x8_to_bf16(st.v3);
  d[t + 1024] = u8x8_to_bf16(st.v4);
  d[t + 1280] = u8x8_to_bf16(st.v5);
  d[t + 1536] = u8x8_to_bf16(st.v6);
  d[t + 1792] = u8x8_to_bf16(st.v7);
  d[t + 2048] = u8x8_to_bf16(st.v8);
  d[t + 2304] = u8x8_to_bf16(st.v9);
  d[t + 2560] = u8x8_to_bf16(st.v10);
  d[t + 2816] = u8x8_to_bf16(st.v11);
  d[t + 3072] = u8x8_to_bf16(st.v12);
  if (t + 3328 < C1_Q) d[t + 3328] = u8x8_to_bf16(st.v13);
}

__device__ __forceinline__ FrameSrc frames_of(const ConvProb& p) {
  return FrameSrc{reinterpret_cast<const uint8_t*>(p.in), p.ids, p.idx};
}

// B operand (weights, reference layout [n][c][ky][kx] = [n][k]): lane holds column n = r32,
// k = 16 s + 8 h + j, for all 16 k-steps -- the whole B stays in 64 VGPRs
__device__ __forceinline__ void load_wb(const uint16_t* w, int r32, int h, bf16x8 (&wb)[16]) {
  const uint4* wr = reinterpret_cast<const uint4*>(w + (size_t)r32 * C1_K + 8 * h);
#pragma unroll
  for (int s = 0; s < 16; ++s) wb[s] = __builtin_bit_cast(bf16x8, wr[2 * s]);
}

}  // namespace

// Samples i in [0, n*B) of the problem set (problem i / B), grid-strided; a workgroup
// reloads its register-resident weights only when the problem's weights change.
__global__ __launch_bounds__(256, 1) void conv1_fwd_k(ConvSet set) {
  __shared__ __attribute__((aligned(16))) char smem[2][C1_STAGE];
  __shared__ __attribute__((aligned(16))) char eps[4][TILE_EP_BYTES];  // per-wave epilogue scratch
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, r32 = lane & 31;
  const int B = set.B, total = set.n * B;
  int i = blockIdx.x;
  if (i >= total) return;  // block-uniform
  bf16x8 wb[16];
  const uint16_t* wcur = set.p[i / B].w;
  load_wb(wcur, r32, h, wb);
  float bn = set.p[i / B].bias[r32];
  Stage14 v;
  load_sample(frames_of(set.p[i / B]), i % B, v);
  store_sample(smem[0], v);
  __syncthreads();
  int stage = 0;
  int tile0 = wave;  // round-robin tiles across samples keeps the 4 waves balanced
  for (; i < total; i += gridDim.x) {
    const int pb = i / B, b = i - pb * B;
    const int i_next = i + gridDim.x;
    const bool more = i_next < total;  // block-uniform
    if (more) load_sample(frames_of(set.p[i_next / B]), i_next % B, v);
    if (set.p[pb].w != wcur) {  // block-uniform
      wcur = set.p[pb].w;
      load_wb(wcur, r32, h, wb);
      bn = set.p[pb].bias[r32];
    }
    uint16_t* out = set.p[pb].out;
    const char* xs = smem[stage];
    for (int mt = tile0; mt < C1_MT; mt += 4) {
      const int p = mt * 32 + r32;
      const int pc = p < C1_P ? p : C1_P - 1;
      const int oy = pc / C1_OW, ox = pc % C1_OW;
      // bf16 plane c, row (4 oy + ky), columns 4 ox .. 4 ox + 7; k-step s: c = s / 4,
      // ky = 2 (s % 4) + h.  8-byte aligned: two ds_read_b64 per fragment.
      const char* abase = xs + 2 * ((4 * oy + h) * 84 + 4 * ox);
      // issue all 16 A-fragment reads of the tile before the MFMA chain (one wave per SIMD:
      // nothing else hides LDS latency)
      uint4 ar[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int off = 2 * ((s >> 2) * C1_HW + 2 * (s & 3) * 84);
        const uint2* a2 = reinterpret_cast<const uint2*>(abase + off);
        const uint2 lo = a2[0], hi = a2[1];
        ar[s] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the chain
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < 16; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ar[s]), wb[s], acc, 0, 0, 0);
      const long base = (long)b * C1_P * C1_N;
      tile_store_bf16(acc, eps[wave], [bn](int, int, float v) { return f2bf(fmaxf(v + bn, 0.f)); },
                      [&](int row) -> long {
                        const int pp = mt * 32 + row;
                        return pp < C1_P ? base + (long)pp * C1_N : -1;
                      }, out);
    }
    tile0 = (tile0 + 4 * ((C1_MT - tile0 + 3) / 4)) - C1_MT;  // next sample continues the rotation
    if (more) store_sample(smem[stage ^ 1], v);
    __syncthreads();
    stage ^= 1;
  }
}

void conv1_fwd_multi(const ConvSet& set, hipStream_t s) {
  const int total = set.n * set.B;
  if (total <= 0) return;
  if (set.n < 1 || set.n > kMaxProbs) throw std::invalid_argument("conv1_fwd: 1..3 problems");
  // >= two samples per workgroup: the next sample's load overlaps the current MFMA loop
  const int grid = std::min(std::max(1, (total + 1) / 2), 256);  // one workgroup per CU (113 KB LDS)
  conv1_fwd_k<<<grid, 256, 0, s>>>(set);
  LAUNCH_CHECK();
}

void conv1_fwd(const uint8_t* frames, const int* ids, const int* idx, const uint16_t* w, const float* bias,
               uint16_t* out, int B, hipStream_t s) {
  ConvSet set{};
  set.p[0] = ConvProb{frames, ids, idx, w, bias, out};
  set.n = 1;
  set.B = B;
  conv1_fwd_multi(set, s);
}

}  // namespace apex
