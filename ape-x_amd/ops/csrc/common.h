// Shared device helpers for the gfx950 kernels (wave64 reductions, Philox RNG,
// bf16 packing, launch checking).  CDNA4 only: wave width is hard-coded to 64.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#define APEX_WAVE 64

#define HIP_CHECK(expr)                                                                      \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

#define LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

namespace apex {

// Ape-X priority mix (utils.py:77, learner.py): 0.9 max|delta| + 0.1 |delta| + 1e-6, rounded
// step by step in torch's fp32 order -- no fma contraction, so every kernel that forms it
// (sequential and batched tree writes, the loss kernel) agrees bit for bit whatever the
// compiler does around it
__device__ __forceinline__ float prio_mix(float dmax, float d) {
#pragma clang fp contract(off)
  return (0.9f * dmax + 0.1f * d) + 1e-6f;
}

// ---------------------------------------------------------------- wave reductions
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

// K independent wave reductions, step-major: every value's exchange of one butterfly step is
// issued before the next step (one LDS-permute latency per step instead of one per value and
// step), each value's arithmetic exactly as wave_sum / wave_min
template <int K, typename T>
__device__ __forceinline__ void wave_sum_k(T (&v)[K]) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = __shfl_xor(v[k], o, 64);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += w[k];
  }
}
template <int K, typename T>
__device__ __forceinline__ void wave_min_k(T (&v)[K]) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = __shfl_xor(v[k], o, 64);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = w[k] < v[k] ? w[k] : v[k];
  }
}

// Tree-node reductions on DPP lane moves (VALU, no LDS permute round trips): quad xor 1, xor
// 2, half-row mirror, row mirror (every lane of a row then holds the row's value), row
// broadcasts 15 / 31 into the next rows; the result is read from lane 63.  A fixed association
// order (not wave_sum's butterfly): every priority-tree kernel reduces node children with
// these, so all tree paths agree bit for bit.  K values step-major, as wave_sum_k.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_id, double fill) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v), f = __builtin_bit_cast(uint64_t, fill);
  const int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
  const int flo = (int)(uint32_t)f, fhi = (int)(uint32_t)(f >> 32);
  int rlo, rhi;
  switch (ctrl_id) {  // (the DPP control must be a compile-time constant)
    case 0: rlo = __builtin_amdgcn_update_dpp(flo, lo, 0xB1, 0xF, 0xF, false);
            rhi = __builtin_amdgcn_update_dpp(fhi, hi, 0xB1, 0xF, 0xF, false); break;
    case 1: rlo = __builtin_amdgcn_update_dpp(flo, lo, 0x4E, 0xF, 0xF, false);
            rhi = __builtin_amdgcn_update_dpp(fhi, hi, 0x4E, 0xF, 0xF, false); break;
    case 2: rlo = __builtin_amdgcn_update_dpp(flo, lo, 0x141, 0xF, 0xF, false);
            rhi = __builtin_amdgcn_update_dpp(fhi, hi, 0x141, 0xF, 0xF, false); break;
    case 3: rlo = __builtin_amdgcn_update_dpp(flo, lo, 0x140, 0xF, 0xF, false);
            rhi = __builtin_amdgcn_update_dpp(fhi, hi, 0x140, 0xF, 0xF, false); break;
    case 4: rlo = __builtin_amdgcn_update_dpp(flo, lo, 0x142, 0xA, 0xF, false);
            rhi = __builtin_amdgcn_update_dpp(fhi, hi, 0x142, 0xA, 0xF, false); break;
    default: rlo = __builtin_amdgcn_update_dpp(flo, lo, 0x143, 0xC, 0xF, false);
             rhi = __builtin_amdgcn_update_dpp(fhi, hi, 0x143, 0xC, 0xF, false); break;
  }
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)rhi << 32) | (uint32_t)rlo);
}
__device__ __forceinline__ float dpp_f32(float v, int ctrl_id, float fill) {
  const int x = __builtin_bit_cast(int, v), f = __builtin_bit_cast(int, fill);
  int r;
  switch (ctrl_id) {
    case 0: r = __builtin_amdgcn_update_dpp(f, x, 0xB1, 0xF, 0xF, false); break;
    case 1: r = __builtin_amdgcn_update_dpp(f, x, 0x4E, 0xF, 0xF, false); break;
    case 2: r = __builtin_amdgcn_update_dpp(f, x, 0x141, 0xF, 0xF, false); break;
    case 3: r = __builtin_amdgcn_update_dpp(f, x, 0x140, 0xF, 0xF, false); break;
    case 4: r = __builtin_amdgcn_update_dpp(f, x, 0x142, 0xA, 0xF, false); break;
    default: r = __builtin_amdgcn_update_dpp(f, x, 0x143, 0xC, 0xF, false); break;
  }
  return __builtin_bit_cast(float, r);
}
__device__ __forceinline__ double lane63_f64(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int K>
__device__ __forceinline__ void tree_sum_k(double (&v)[K]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    double w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = dpp_f64(v[k], c, 0.0);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += w[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = lane63_f64(v[k]);
}
template <int K>
__device__ __forceinline__ void tree_min_k(float (&v)[K]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    float w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = dpp_f32(v[k], c, INFINITY);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = w[k] < v[k] ? w[k] : v[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[k]), 63));
}
__device__ __forceinline__ double tree_sum(double v) {
  double a[1] = {v};
  tree_sum_k<1>(a);
  return a[0];
}
__device__ __forceinline__ float tree_min(float v) {
  float a[1] = {v};
  tree_min_k<1>(a);
  return a[0];
}

// inclusive prefix sum across the 64 lanes (Hillis-Steele, fixed order => deterministic)
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T w = __shfl_up(v, o, 64);
    if (lane >= o) v += w;
  }
  return v;
}

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c.x, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, &hi1);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 4 uniforms in [0,1) for (seed, stream, counter).
__device__ __forceinline__ void uniform4(uint64_t seed, uint64_t stream, uint64_t counter, float out[4]) {
  u32x4 c{(uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  u32x4 r = philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float s = 5.9604644775390625e-08f;  // 2^-24
  out[0] = (r.x >> 8) * s;
  out[1] = (r.y >> 8) * s;
  out[2] = (r.z >> 8) * s;
  out[3] = (r.w >> 8) * s;
}

// Box-Muller standard normal from two uniforms in [0,1)
__device__ __forceinline__ float std_normal(float u1, float u2) {
  const float r = sqrtf(-2.f * logf(fmaxf(u1, 1e-12f)));
  return r * cospif(2.f * u2);
}

__device__ __forceinline__ double uniform_double(uint64_t seed, uint64_t stream, uint64_t counter) {
  u32x4 c{(uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  u32x4 r = philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uint64_t bits = ((uint64_t)r.x << 21) ^ (uint64_t)r.y;  // 53 random bits
  return (double)(bits & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
}

// One wave draws stratified proportional sample i of B from a fanout-64 sum tree (TreeDesc of
// kernels.h): mass (u_i + i) * total / B with u_i from Philox (seed, i, counter), descended with
// a wave-wide inclusive scan of the 64 child sums per level; returns the leaf.  ``length``
// live slots; ``exclude_last``: the newest slot's leaf is left out of the mass (reference Q5).
// Shared by per_sample_k (replay_kernels.hip) and the AQL learner forward, which samples its
// own row (aql_engine_kernels.hip).
template <class TD>
__device__ __forceinline__ int tree_sample_leaf(const TD& t, int i, int B, int length, int exclude_last,
                                                uint64_t seed, uint64_t ctr, int lane, float* leaf_p = nullptr) {
  // leaf_p: the drawn leaf's stored value (leaf_sum[node]), taken from the last level's
  // children instead of a dependent re-read after the descent
  const int L = t.levels;
  double total = t.node_sum[L - 1][0];
  if (exclude_last && length > 0 && length <= t.size[0]) total -= (double)t.leaf_sum[length - 1];
  const double u = uniform_double(seed, (uint64_t)i, ctr);
  double mass = (u + (double)i) * total / (double)B;
  int node = 0;
  for (int level = L; level >= 1; --level) {
    const int child = node * 64 + lane;
    const int csize = t.size[level - 1];
    double v = 0.0;
    float raw = 0.f;
    if (child < csize) {
      if (level == 1) {
        raw = t.leaf_sum[child];
        v = (double)raw;
      } else {
        v = t.node_sum[level - 2][child];
      }
    }
    if (exclude_last && level == 1 && child == length - 1) v = 0.0;
    const double incl = wave_inclusive_scan(v, lane);
    unsigned long long hit = __ballot(incl > mass);
    int k;
    if (hit) {
      k = __ffsll((long long)hit) - 1;
    } else {  // rounding at the top end: take the last child with mass
      unsigned long long nz = __ballot(v > 0.0);
      k = nz ? 63 - __clzll((long long)nz) : 0;
    }
    const double before = __shfl(incl - v, k, 64);
    if (level == 1 && leaf_p) *leaf_p = __shfl(raw, k, 64);
    mass -= before;
    if (mass < 0.0) mass = 0.0;
    node = node * 64 + k;
  }
  return node;
}

// ---------------------------------------------------------------- bf16
__device__ __forceinline__ uint16_t f2bf(float f) {
  return __bfloat16_as_ushort(__float2bfloat16(f));  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ void atomic_max_pos_float(float* addr, float v) {
  // valid for non-negative floats: IEEE order == signed-int order
  atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
}

// Where a conv1 input sample lives.  With `ids`, sample b's frame c is frame
// ids[(idx ? idx[b] : b) * 4 + c] of the HBM frame ring (the replay / actor stack is read
// in place, no gather); without, the input is a dense u8 [B][4][84][84] tensor.
struct FrameSrc {
  const uint8_t* frames;
  const int* ids;
  const int* idx;
};

__device__ __forceinline__ const uint8_t* frame_plane(const FrameSrc& f, int b, int c, int plane_bytes) {
  if (f.ids) {
    const int row = f.idx ? f.idx[b] : b;
    return f.frames + (size_t)f.ids[row * 4 + c] * plane_bytes;
  }
  return f.frames + ((size_t)b * 4 + c) * plane_bytes;
}

__device__ __forceinline__ uint32_t pack_bf16x2_u8(uint32_t b0, uint32_t b1) {
  // integers 0..255 are exact in bf16: bf16 = high half of the f32
  const uint32_t f0 = __float_as_uint((float)b0), f1 = __float_as_uint((float)b1);
  return (f0 >> 16) | (f1 & 0xFFFF0000u);
}

__device__ __forceinline__ uint32_t word_of(const uint4& v, int k) {
  return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));  // k is a compile-time constant
}

// 4 channel planes x 4 consecutive u8 pixels (one 32-bit word each) -> 4 pixels x 4
// channels bf16 = 32 bytes (two uint4), written straight to LDS.
__device__ __forceinline__ void u8x4words_to_lds(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint4* d) {
  uint4 a, b;
  a.x = pack_bf16x2_u8(w0 & 0xFF, w1 & 0xFF);
  a.y = pack_bf16x2_u8(w2 & 0xFF, w3 & 0xFF);
  a.z = pack_bf16x2_u8((w0 >> 8) & 0xFF, (w1 >> 8) & 0xFF);
  a.w = pack_bf16x2_u8((w2 >> 8) & 0xFF, (w3 >> 8) & 0xFF);
  b.x = pack_bf16x2_u8((w0 >> 16) & 0xFF, (w1 >> 16) & 0xFF);
  b.y = pack_bf16x2_u8((w2 >> 16) & 0xFF, (w3 >> 16) & 0xFF);
  b.z = pack_bf16x2_u8(w0 >> 24, w1 >> 24);
  b.w = pack_bf16x2_u8(w2 >> 24, w3 >> 24);
  d[0] = a;
  d[1] = b;
}

// Stage a 4-frame u8 stack (84x84) into LDS as NHWC bf16 with 8-byte pixels: every
// thread issues all of its 16-byte global loads before the first LDS write.
template <int HW>
__device__ __forceinline__ void stage_frames_bf16(const FrameSrc& f, int b, char* xs) {
  constexpr int GROUPS = HW / 16;                 // 16-pixel groups
  constexpr int PER = (GROUPS + 255) / 256;
  const uint8_t* const pl[4] = {frame_plane(f, b, 0, HW), frame_plane(f, b, 1, HW), frame_plane(f, b, 2, HW),
                                frame_plane(f, b, 3, HW)};
  static_assert(PER <= 2, "frame staging keeps <= 8 loads in flight per thread");
  const int g0 = threadIdx.x, g1 = threadIdx.x + 256;
  const bool ok1 = PER > 1 && g1 < GROUPS;
  uint4 a0 = {}, a1 = {}, a2 = {}, a3 = {}, b0 = {}, b1 = {}, b2 = {}, b3 = {};
  if (g0 < GROUPS) {
    a0 = reinterpret_cast<const uint4*>(pl[0])[g0];
    a1 = reinterpret_cast<const uint4*>(pl[1])[g0];
    a2 = reinterpret_cast<const uint4*>(pl[2])[g0];
    a3 = reinterpret_cast<const uint4*>(pl[3])[g0];
  }
  if (ok1) {
    b0 = reinterpret_cast<const uint4*>(pl[0])[g1];
    b1 = reinterpret_cast<const uint4*>(pl[1])[g1];
    b2 = reinterpret_cast<const uint4*>(pl[2])[g1];
    b3 = reinterpret_cast<const uint4*>(pl[3])[g1];
  }
  if (g0 < GROUPS) {
    uint4* d = reinterpret_cast<uint4*>(xs + g0 * 16 * 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) u8x4words_to_lds(word_of(a0, k), word_of(a1, k), word_of(a2, k), word_of(a3, k), d + 2 * k);
  }
  if (ok1) {
    uint4* d = reinterpret_cast<uint4*>(xs + g1 * 16 * 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) u8x4words_to_lds(word_of(b0, k), word_of(b1, k), word_of(b2, k), word_of(b3, k), d + 2 * k);
  }
}

// Pipelined 16-byte copy global -> LDS of TOTAL chunks with a destination remap: rounds
// of 4 loads issued back to back before their LDS writes (bounded register footprint,
// no private-memory arrays).
template <int TOTAL, class DstOff>
__device__ __forceinline__ void stage_chunks(const uint4* __restrict__ src, char* dst, DstOff dst_off) {
  constexpr int PER = (TOTAL + 255) / 256;
#pragma unroll
  for (int k0 = 0; k0 < PER; k0 += 4) {
    const int q0 = threadIdx.x + 256 * k0, q1 = q0 + 256, q2 = q0 + 512, q3 = q0 + 768;
    uint4 v0 = {}, v1 = {}, v2 = {}, v3 = {};
    if (q0 < TOTAL) v0 = src[q0];
    if (k0 + 1 < PER && q1 < TOTAL) v1 = src[q1];
    if (k0 + 2 < PER && q2 < TOTAL) v2 = src[q2];
    if (k0 + 3 < PER && q3 < TOTAL) v3 = src[q3];
    if (q0 < TOTAL) *reinterpret_cast<uint4*>(dst + dst_off(q0)) = v0;
    if (k0 + 1 < PER && q1 < TOTAL) *reinterpret_cast<uint4*>(dst + dst_off(q1)) = v1;
    if (k0 + 2 < PER && q2 < TOTAL) *reinterpret_cast<uint4*>(dst + dst_off(q2)) = v2;
    if (k0 + 3 < PER && q3 < TOTAL) *reinterpret_cast<uint4*>(dst + dst_off(q3)) = v3;
  }
}

}  // namespace apex

namespace apex {

// ---------------------------------------------------------------- register prefetch
// Up to 8 x 256 16-byte chunks per workgroup held in NAMED registers (a uint4 array here
// is demoted to scratch: SROA runs before the unroller), so a persistent kernel can issue
// the global loads of its NEXT sample before computing the current one, and commit them
// to LDS after the compute (one LDS buffer, global latency hidden behind the MFMAs).
typedef unsigned int u32v4 __attribute__((ext_vector_type(4)));  // native vector: SROA-friendly
struct Pf8 {
  u32v4 r0, r1, r2, r3, r4, r5, r6, r7;
};

#define APEX_PF_SLOTS(X) X(0, r0) X(1, r1) X(2, r2) X(3, r3) X(4, r4) X(5, r5) X(6, r6) X(7, r7)

// pf_load / pf_store: chunks q = t + 256 (BASE + K), K = 0..7, of a TOTAL-chunk copy
template <int TOTAL, int BASE = 0>
__device__ __forceinline__ void pf_load(Pf8& p, const uint4* __restrict__ src4) {
  static_assert(TOTAL <= 32 * 256, "at most 4 Pf8 blocks per copy");
  const u32v4* src = reinterpret_cast<const u32v4*>(src4);
  const int t = threadIdx.x & 255;  /* local to a 256-thread staging group */
#define APEX_PF_LD(K, R) \
  if constexpr ((BASE + K) * 256 < TOTAL) p.R = src[min(t + (BASE + K) * 256, TOTAL - 1)];  /* always assigned */
  APEX_PF_SLOTS(APEX_PF_LD)
#undef APEX_PF_LD
}

template <int TOTAL, int BASE = 0, class DstOff>
__device__ __forceinline__ void pf_store(const Pf8& p, char* dst, DstOff dst_off) {
  const int t = threadIdx.x & 255;  /* local to a 256-thread staging group */
#define APEX_PF_ST(K, R) \
  if constexpr ((BASE + K) * 256 < TOTAL) {                                     \
    const int q = t + (BASE + K) * 256;                                         \
    if (((BASE + K) + 1) * 256 <= TOTAL || q < TOTAL)                           \
      *reinterpret_cast<u32v4*>(dst + dst_off(q)) = p.R;                        \
  }
  APEX_PF_SLOTS(APEX_PF_ST)
#undef APEX_PF_ST
}

// Global -> LDS copy of TOTAL 16-byte chunks with every load of the copy issued before
// the first LDS store (up to 32 per thread in flight, named vector registers): the
// latency is paid once per copy, not once per round of loads.
template <int TOTAL, class DstOff>
__device__ __forceinline__ void stage_all(const uint4* __restrict__ src, char* dst, DstOff dst_off) {
  Pf8 a, b, c, d;
  pf_load<TOTAL, 0>(a, src);
  if constexpr (TOTAL > 8 * 256) pf_load<TOTAL, 8>(b, src);
  if constexpr (TOTAL > 16 * 256) pf_load<TOTAL, 16>(c, src);
  if constexpr (TOTAL > 24 * 256) pf_load<TOTAL, 24>(d, src);
  pf_store<TOTAL, 0>(a, dst, dst_off);
  if constexpr (TOTAL > 8 * 256) pf_store<TOTAL, 8>(b, dst, dst_off);
  if constexpr (TOTAL > 16 * 256) pf_store<TOTAL, 16>(c, dst, dst_off);
  if constexpr (TOTAL > 24 * 256) pf_store<TOTAL, 24>(d, dst, dst_off);
}

}  // namespace apex

namespace apex {

// ---------------------------------------------------------------- ReLU-backward mask
// keep bf16 element of v where the matching element of m (a post-ReLU activation) is > 0
__device__ __forceinline__ uint32_t relu_mask_bf16x2(uint32_t v, uint32_t m) {
  const uint32_t lo = ((m & 0xFFFFu) != 0u && !(m & 0x8000u)) ? 0x0000FFFFu : 0u;
  const uint32_t hi = ((m >> 16) != 0u && !(m & 0x80000000u)) ? 0xFFFF0000u : 0u;
  return v & (lo | hi);
}

__device__ __forceinline__ u32v4 relu_mask_chunk(u32v4 v, u32v4 m) {
  return u32v4{relu_mask_bf16x2(v[0], m[0]), relu_mask_bf16x2(v[1], m[1]), relu_mask_bf16x2(v[2], m[2]),
               relu_mask_bf16x2(v[3], m[3])};
}

// mask every prefetched chunk of p by the matching chunk of m (same TOTAL / BASE geometry)
template <int TOTAL, int BASE = 0>
__device__ __forceinline__ void pf_mask(Pf8& p, const Pf8& m) {
#define APEX_PF_MK(K, R) \
  if constexpr ((BASE + K) * 256 < TOTAL) p.R = relu_mask_chunk(p.R, m.R);
  APEX_PF_SLOTS(APEX_PF_MK)
#undef APEX_PF_MK
}

// ---------------------------------------------------------------- MFMA tile epilogue
// Store a 32x32 fp32 MFMA tile (C/D map: row = (r&3) + 8(r>>2) + 4h, col = lane&31) as bf16
// rows of 64 contiguous bytes through a per-wave LDS scratch (32 x 80 B): 16 two-byte LDS
// writes + 2 coalesced 16-byte global stores per lane instead of 16 strided 2-byte global
// stores.  cvt(r, row, v) -> bf16 bits.  Wave-synchronous (LDS ops of one wave complete
// in order).
constexpr int TILE_EP_PITCH = 80;
constexpr int TILE_EP_BYTES = 32 * TILE_EP_PITCH;

template <class Acc, class Cvt, class RowOff>
__device__ __forceinline__ void tile_store_bf16(const Acc& acc, char* ep, Cvt cvt, RowOff row_off, uint16_t* out,
                                                const uint16_t* mask = nullptr) {
  // row_off(row) -> element offset of the row in `out` (< 0: skip); `mask` (optional): a
  // ReLU-backward mask with the layout of `out`, applied per 16-B chunk (coalesced read)
  const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    *reinterpret_cast<uint16_t*>(ep + row * TILE_EP_PITCH + col * 2) = cvt(r, row, acc[r]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = lane + 64 * i, row = id >> 2, ch = id & 3;
    u32v4 v = *reinterpret_cast<const u32v4*>(ep + row * TILE_EP_PITCH + ch * 16);
    const long off = row_off(row);
    if (off >= 0) {
      if (mask) v = relu_mask_chunk(v, *reinterpret_cast<const u32v4*>(mask + off + ch * 8));
      *reinterpret_cast<u32v4*>(out + off + ch * 8) = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();  // the scratch is reused by the wave's next tile
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace apex
