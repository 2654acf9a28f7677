// Learner-side fused kernels for gfx950.
//
// * dqn_loss: double-DQN n-step target + Huber(1) * IS weight + batch-max priority
//   mixing + dL/dQ in ONE workgroup (reference utils.py:64-81 runs ~15 torch ops and a
//   device->host copy of the priorities every step).
// * grad_sumsq + rmsprop_step / adam_step: global-L2 clip (torch clip_grad_norm_
//   semantics) fused into a single pass of the optimizer over the flat fp32 parameter
//   buffer.  The norm is reduced deterministically: per-(tensor, block) fp64 partials,
//   re-reduced in fixed order by every update block, so no atomics and no host sync.
//   The same partials give the reference's logged 'grad_norm' formula.
#include "common.h"
#include "kernels.h"
#include "opt_dev.h"

namespace apex {

__device__ __forceinline__ float block_sum_f(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += smem[i];  // fixed order
  return t;
}

__device__ __forceinline__ float block_max_f(float v, float* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, smem[i]);
  return t;
}

// ------------------------------------------------------------------ loss
__global__ void dqn_loss_k(const float* __restrict__ q, const float* __restrict__ q2, const float* __restrict__ q2t,
                           int ldq, const int* __restrict__ act, const float* __restrict__ rew,
                           const float* __restrict__ done, const int* __restrict__ idx, const float* __restrict__ w,
                           int B, int A, float gamma_n, float* __restrict__ loss_out, float* __restrict__ dq,
                           float* __restrict__ prio) {
  __shared__ float red[16];
  const int b = threadIdx.x;
  float delta = 0.f, lw = 0.f, g = 0.f;
  int a = 0;
  if (b < B) {
    const float* qr = q + (size_t)b * ldq;
    const float* q2r = q2 + (size_t)b * ldq;
    const float* q2tr = q2t + (size_t)b * ldq;
    const int row = idx ? idx[b] : b;  // read (a, r, d) straight from the replay's transition table
    a = act[row];
    int astar = 0;
    float best = q2r[0];
    for (int k = 1; k < A; ++k)
      if (q2r[k] > best) { best = q2r[k]; astar = k; }
    const float y = rew[row] + gamma_n * q2tr[astar] * (1.f - done[row]);
    const float qa = qr[a];
    delta = fabsf(y - qa);
    const float h = delta < 1.f ? 0.5f * delta * delta : delta - 0.5f;
    lw = w[b] * h;
    g = w[b] / (float)B * fminf(fmaxf(qa - y, -1.f), 1.f);
  }
  const float total = block_sum_f(lw, red);
  const float dmax = block_max_f(b < B ? delta : -INFINITY, red);
  if (b < B) {
    prio[b] = prio_mix(dmax, delta);
    float* dr = dq + (size_t)b * ldq;
    for (int k = 0; k < A; ++k) dr[k] = (k == a) ? g : 0.f;
  }
  if (b == 0) loss_out[0] = total / (float)B;
}

void dqn_loss(const float* q, const float* q2, const float* q2t, int ldq, const int* a, const float* r, const float* d,
              const int* idx, const float* w, int B, int A, float gamma_n, float* loss_out, float* dq, float* prio,
              hipStream_t s) {
  if (B < 1 || B > 1024) throw std::invalid_argument("dqn_loss: batch must be in [1, 1024]");
  const int threads = ((B + 63) / 64) * 64;
  dqn_loss_k<<<1, threads, 0, s>>>(q, q2, q2t, ldq, a, r, d, idx, w, B, A, gamma_n, loss_out, dq, prio);
  LAUNCH_CHECK();
}

// ------------------------------------------------------------------ grad norm partials
// kNormBlocks blocks cover the flat gradient in contiguous chunks (all CUs busy no matter
// how the parameters are split into tensors); each writes one fp64 partial.
constexpr int kNormBlocks = 256;

__global__ void grad_sumsq_k(const float* __restrict__ g, int64_t n, double* __restrict__ partials) {
  __shared__ double red[4];
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
  double acc = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const float v = g[i];
    acc += (double)v * (double)v;
  }
  acc = wave_sum(acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

void grad_sumsq(const float* g, int64_t n, double* partials, hipStream_t s) {
  grad_sumsq_k<<<kNormBlocks, 256, 0, s>>>(g, n, partials);
  LAUNCH_CHECK();
}

int grad_norm_partials() { return kNormBlocks; }

__device__ __forceinline__ void pack_store(const PackMap& pk, int64_t i, float v) {
  if (pk.arena_f32) {  // fp32 network: exact copies in the GEMM layouts
    const int d1 = pk.dst1[i], d2 = pk.dst2[i];
    if (d1 >= 0) pk.arena_f32[d1] = v;
    if (d2 >= 0) pk.arena_f32[d2] = v;
    return;
  }
  if (!pk.arena) return;
  const uint16_t b = f2bf(v);
  const int d1 = pk.dst1[i], d2 = pk.dst2[i];
  if (d1 >= 0) pk.arena[d1] = b;
  if (d2 >= 0) pk.arena[d2] = b;
}

// FC1 weights (advantage.0 / value.0, reference [128][C3*P3] with column c*P3 + p) are
// updated in tiles of 8 rows x 8 channels x all 49 positions: fp32 reads/writes stay
// coalesced in the reference order, the bf16 results are staged in LDS and leave as
// 16-byte runs in both packed layouts -- wfc1p [256][p*64 + c] (forward) and wfc1t
// [p*64 + c][256] (FC1 input-gradient GEMM).  Writing them element by element through
// the scatter maps cost ~1.6M scattered 2-byte stores per step (the old 20 us pass).
constexpr int kFcN = 128, kFcC = 64, kFcP = 49, kFcTn = 8, kFcTc = 8;
constexpr int kFcTile = kFcTn * kFcTc * kFcP;                                       // 3136
constexpr int kFcTilesPerMat = (kFcN / kFcTn) * (kFcC / kFcTc);                      // 128
constexpr int kOptThreads = 256, kOptGenBlocksMax = 1024;

template <class Rule>
__device__ __forceinline__ void opt_elem(float* p, const float* g, float* s1, float* s2, int64_t i, float clip,
                                         const Rule& rule, const PackMap& pk) {
  float a = s1[i], b = s2[i];
  const float np = rule(p[i], opaque(g[i] * clip), a, b);
  s1[i] = a;
  s2[i] = b;
  p[i] = np;
  pack_store(pk, i, np);
}

// The update of one parameter set by workgroup `bid` of `nblk` (opt_step_k: the whole grid;
// opt_step2_k: two sets split at a block-uniform boundary).
template <class Params>
__device__ __forceinline__ void opt_body(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ s1,
                                         float* __restrict__ s2, int64_t n, const double* __restrict__ partials,
                                         int n_partials, const Params& hp, const int64_t* __restrict__ step,
                                         float* __restrict__ norms_out, const PackMap& pk, const FcPack& fc,
                                         int n_fc_blocks, int bid, int nblk) {
  const float max_norm = hp.max_norm;
  float lr;
  const auto rule = make_rule(hp, step ? step[0] : 0, lr);
  auto norms = [&]() {
    const NormInfo ni = reduce_norms(partials, n_partials, max_norm, hp.grad_scale);
    if (bid == 0 && threadIdx.x == 0 && norms_out) {
      norms_out[0] = ni.l2;
      norms_out[2] = fminf(max_norm > 0.f ? max_norm / (ni.l2 + 1e-6f) : 1.f, 1.f);
      norms_out[3] = lr;
    }
    return ni;
  };
  if (bid < n_fc_blocks) {
    __shared__ uint16_t tile[kFcTn][kFcTc * kFcP];
    __shared__ float tile_f[kFcTn][kFcTc * kFcP];
    const int mat = bid / kFcTilesPerMat, t = bid % kFcTilesPerMat;
    const int n0 = (t / (kFcC / kFcTc)) * kFcTn, c0 = (t % (kFcC / kFcTc)) * kFcTc;
    const int64_t base = fc.off[mat];
    // all loads of the thread's ~12 elements issued up front (memory-level parallelism:
    // one workgroup per CU), then the updates, then the stores
    constexpr int kIt = (kFcTile + kOptThreads - 1) / kOptThreads;
    float vp[kIt], vg[kIt], va[kIt], vb[kIt];
    int64_t vi[kIt];
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int e = threadIdx.x + k * kOptThreads;
      const int ec = e < kFcTile ? e : kFcTile - 1;  // clamp: the tail lanes reload a valid element
      const int r = ec / (kFcTc * kFcP), col = ec - r * (kFcTc * kFcP);
      vi[k] = base + (int64_t)(n0 + r) * (kFcC * kFcP) + c0 * kFcP + col;
      vp[k] = p[vi[k]];
      vg[k] = g[vi[k]];
      va[k] = s1[vi[k]];
      vb[k] = s2[vi[k]];
    }
    // the global grad norm (a reduction over the finalize partials) is reduced while the
    // tile's loads above are in flight: the update needs it, the loads do not
    const NormInfo ni = norms();
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int e = threadIdx.x + k * kOptThreads;
      const float np = rule(vp[k], opaque(vg[k] * ni.clip), va[k], vb[k]);
      if (e < kFcTile) {
        const int r = e / (kFcTc * kFcP), col = e - r * (kFcTc * kFcP);
        s1[vi[k]] = va[k];
        s2[vi[k]] = vb[k];
        p[vi[k]] = np;
        if (fc.wp_f32) tile_f[r][col] = np;
        else tile[r][col] = f2bf(np);
      }
    }
    const int nrow = mat * kFcN + n0;
    if (fc.wp_f32) {  // fp32 network: wfc1p rows only, 8 channels = two 16-byte runs per position
      __syncthreads();
      for (int e = threadIdx.x; e < kFcTn * kFcP * 2; e += kOptThreads) {
        const int half = e & 1, rp = e >> 1, r = rp / kFcP, pp = rp - r * kFcP;
        float4 v;
        v.x = tile_f[r][(4 * half + 0) * kFcP + pp];
        v.y = tile_f[r][(4 * half + 1) * kFcP + pp];
        v.z = tile_f[r][(4 * half + 2) * kFcP + pp];
        v.w = tile_f[r][(4 * half + 3) * kFcP + pp];
        const size_t o = (size_t)(nrow + r) * (kFcC * kFcP) + pp * kFcC + c0 + 4 * half;
        *reinterpret_cast<float4*>(fc.wp_f32 + o) = v;
      }
      return;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * kFcTn * kFcP; e += kOptThreads) {
      union { uint16_t h[8]; uint4 v; } u;
      if (e < kFcTn * kFcP) {  // wfc1p row nrow + r, positions p*64 + c0 .. +7
        const int r = e / kFcP, pp = e - r * kFcP;
#pragma unroll
        for (int c = 0; c < kFcTc; ++c) u.h[c] = tile[r][c * kFcP + pp];
        *reinterpret_cast<uint4*>(fc.wp + (size_t)(nrow + r) * (kFcC * kFcP) + pp * kFcC + c0) = u.v;
      } else {  // wfc1t row p*64 + c0 + c, columns nrow .. +7
        const int e2 = e - kFcTn * kFcP, c = e2 / kFcP, pp = e2 - c * kFcP;
#pragma unroll
        for (int r = 0; r < kFcTn; ++r) u.h[r] = tile[r][c * kFcP + pp];
        *reinterpret_cast<uint4*>(fc.wt + (size_t)(pp * kFcC + c0 + c) * (2 * kFcN) + nrow) = u.v;
      }
    }
    return;
  }
  // generic part: every element outside the FC1 ranges, scalar, through the scatter maps
  const int gb = bid - n_fc_blocks, ngb = nblk - n_fc_blocks;
  const int64_t stride = (int64_t)ngb * kOptThreads;
  int64_t lo[3], hi[3];
  int nr = 0;
  if (n_fc_blocks) {
    const int64_t F = (int64_t)kFcN * kFcC * kFcP;
    const int64_t a0 = min(fc.off[0], fc.off[1]), a1 = max(fc.off[0], fc.off[1]);
    lo[0] = 0;      hi[0] = a0;
    lo[1] = a0 + F; hi[1] = a1;
    lo[2] = a1 + F; hi[2] = n;
    nr = 3;
  } else {
    lo[0] = 0; hi[0] = n; nr = 1;
  }
  bool one_pass = true;  // (grid-uniform) the grid covers every range in one element per thread
  for (int k = 0; k < nr; ++k) one_pass = one_pass && hi[k] - lo[k] <= stride;
  if (one_pass) {
    // every load of the thread's (<= 3) elements and their packed-copy slots in flight before
    // the norm reduction: the grid-stride loop below pays a dependent round trip per element
    // (MI355X, fp32 DQN learner: 9.9 -> 8.3 us per optimizer launch, scripts/diag/opt_tail.py)
    float vp[3], vg[3], va[3], vb[3];
    int64_t vi[3];
    int d1[3], d2[3];
    const bool packed = pk.arena_f32 != nullptr || pk.arena != nullptr;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      vi[k] = k < nr ? lo[k] + (int64_t)gb * kOptThreads + threadIdx.x : -1;
      const int64_t c = k < nr && vi[k] < hi[k] ? vi[k] : 0;  // clamp: the idle lanes reload element 0
      vp[k] = p[c];
      vg[k] = g[c];
      va[k] = s1[c];
      vb[k] = s2[c];
      d1[k] = packed ? pk.dst1[c] : -1;
      d2[k] = packed ? pk.dst2[c] : -1;
    }
    const NormInfo ni = norms();
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k >= nr || vi[k] >= hi[k]) continue;
      const float np = rule(vp[k], opaque(vg[k] * ni.clip), va[k], vb[k]);
      s1[vi[k]] = va[k];
      s2[vi[k]] = vb[k];
      p[vi[k]] = np;
      if (pk.arena_f32) {
        if (d1[k] >= 0) pk.arena_f32[d1[k]] = np;
        if (d2[k] >= 0) pk.arena_f32[d2[k]] = np;
      } else if (pk.arena) {
        const uint16_t b = f2bf(np);
        if (d1[k] >= 0) pk.arena[d1[k]] = b;
        if (d2[k] >= 0) pk.arena[d2[k]] = b;
      }
    }
    return;
  }
  const NormInfo ni = norms();
  for (int k = 0; k < nr; ++k)
    for (int64_t i = lo[k] + (int64_t)gb * kOptThreads + threadIdx.x; i < hi[k]; i += stride)
      opt_elem(p, g, s1, s2, i, ni.clip, rule, pk);
}

template <class Params>
__global__ __launch_bounds__(kOptThreads) void opt_step_k(float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ s1, float* __restrict__ s2, int64_t n,
                                                          const double* __restrict__ partials, int n_partials,
                                                          Params hp, const int64_t* __restrict__ step,
                                                          float* __restrict__ norms_out, PackMap pk, FcPack fc,
                                                          int n_fc_blocks) {
  opt_body(p, g, s1, s2, n, partials, n_partials, hp, step, norms_out, pk, fc, n_fc_blocks, blockIdx.x, gridDim.x);
}

// Two independent parameter sets (own partials, norms, clip) in ONE launch: blocks
// [0, a.nblk) update set a, the rest set b (AQL: critic + proposal Adam, AQL_dis.py).
template <class Params>
__global__ __launch_bounds__(kOptThreads) void opt_step2_k(OptSet a, OptSet b, Params hp,
                                                           const int64_t* __restrict__ step) {
  const bool second = (int)blockIdx.x >= a.nblk;  // block-uniform
  const OptSet& o = second ? b : a;
  opt_body(o.p, o.g, o.s1, o.s2, o.n, o.partials, o.n_partials, hp, step, o.norms_out,
           PackMap{nullptr, nullptr, nullptr, nullptr}, FcPack{}, 0, second ? (int)blockIdx.x - a.nblk : (int)blockIdx.x,
           o.nblk);
}

template <class Params>
static void launch_opt(float* p, const float* g, float* s1, float* s2, int64_t n, const double* partials,
                       int n_partials, const Params& hp, const int64_t* step, float* norms_out, const PackMap* pack,
                       const FcPack* fc, hipStream_t s) {
  const PackMap pk = pack ? *pack : PackMap{nullptr, nullptr, nullptr, nullptr};
  if ((pk.arena || pk.arena_f32) && (!pk.dst1 || !pk.dst2))
    throw std::invalid_argument("opt_step: packed copies need both scatter maps (dst1, dst2)");
  FcPack f{};
  int nfc = 0;
  if (fc && (fc->wp || fc->wp_f32)) {
    const int64_t F = (int64_t)kFcN * kFcC * kFcP;
    if (fc->off[0] < 0 || fc->off[1] < 0 || fc->off[0] + F > n || fc->off[1] + F > n ||
        std::llabs(fc->off[0] - fc->off[1]) < F)
      throw std::invalid_argument("opt_step: FC1 ranges out of bounds / overlapping");
    if ((reinterpret_cast<uintptr_t>(fc->wp) | reinterpret_cast<uintptr_t>(fc->wt) |
         reinterpret_cast<uintptr_t>(fc->wp_f32)) & 15)
      throw std::invalid_argument("opt_step: packed FC1 layouts must be 16-byte aligned");
    f = *fc;
    nfc = 2 * kFcTilesPerMat;
  }
  const int64_t gen = n - (nfc ? 2 * (int64_t)kFcN * kFcC * kFcP : 0);
  // one element per thread (the one-pass path) up to kOptGenBlocksMax workgroups
  const int ngb = (int)std::max<int64_t>(1, std::min<int64_t>((gen + kOptThreads - 1) / kOptThreads,
                                                               kOptGenBlocksMax));
  opt_step_k<Params><<<nfc + ngb, kOptThreads, 0, s>>>(p, g, s1, s2, n, partials, n_partials, hp, step, norms_out,
                                                       pk, f, nfc);
  LAUNCH_CHECK();
}

void rmsprop_step(float* p, const float* g, float* sq, float* gavg, int64_t n, const double* partials,
                  int n_partials, const RMSpropParams& hp, const int64_t* step, float* norms_out, hipStream_t s,
                  const PackMap* pack, const FcPack* fc) {
  launch_opt(p, g, sq, gavg, n, partials, n_partials, hp, step, norms_out, pack, fc, s);
}

void adam_step2(OptSet a, OptSet b, const AdamParams& hp, const int64_t* step, hipStream_t s) {
  auto blocks = [](int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 4 * kOptThreads - 1) / (4 * kOptThreads), kOptGenBlocksMax));
  };
  if (a.n <= 0 || b.n <= 0) throw std::invalid_argument("adam_step2: both sets must be non-empty");
  a.nblk = blocks(a.n);
  b.nblk = blocks(b.n);
  opt_step2_k<AdamParams><<<a.nblk + b.nblk, kOptThreads, 0, s>>>(a, b, hp, step);
  LAUNCH_CHECK();
}

void adam_step(float* p, const float* g, float* m, float* v, int64_t n, const double* partials, int n_partials,
               const AdamParams& hp, const int64_t* step, float* norms_out, hipStream_t s, const PackMap* pack,
               const FcPack* fc) {
  launch_opt(p, g, m, v, n, partials, n_partials, hp, step, norms_out, pack, fc, s);
}

__global__ void spin_k(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

void spin_us(int us, hipStream_t s) {
  if (us < 0 || us > 100000) throw std::invalid_argument("spin_us: 0..100000 us");
  int dev = 0, khz = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;  // 100 MHz
  spin_k<<<1, 64, 0, s>>>((uint64_t)khz * (uint64_t)us / 1000ull);
  LAUNCH_CHECK();
}

void copy_f32(float* dst, const float* src, int64_t n, hipStream_t s) {
  HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, s));
}

}  // namespace apex
