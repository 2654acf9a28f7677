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
    prio[b] = 0.9f * dmax + 0.1f * delta + 1e-6f;
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

// Every update block re-reduces the partials in the same fixed order (deterministic,
// identical in all blocks).  The reference's per-tensor 'grad_norm' log value is computed
// on demand on the host side (DQNLearner.stats), not on every step.
struct NormInfo {
  float clip, l2;
};
__device__ NormInfo reduce_norms(const double* partials, int n_partials, float max_norm) {
  __shared__ double red[256];
  double t = 0.0;
  for (int k = threadIdx.x; k < n_partials; k += blockDim.x) t += partials[k];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int off = blockDim.x >> 1; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  NormInfo ni;
  ni.l2 = (float)sqrt(red[0]);
  const float coef = max_norm > 0.f ? max_norm / (ni.l2 + 1e-6f) : 1.f;
  ni.clip = fminf(coef, 1.f);
  return ni;
}

__device__ __forceinline__ float step_lr(float lr0, float gamma, int step_size, int offset, int64_t step) {
  if (gamma == 1.f || step_size <= 0) return lr0;
  const int64_t k = (step + offset) / step_size;
  return lr0 * powf(gamma, (float)k);
}

__device__ __forceinline__ void pack_store(const PackMap& pk, int64_t i, float v) {
  if (!pk.arena) return;
  const uint16_t b = f2bf(v);
  const int d1 = pk.dst1[i], d2 = pk.dst2[i];
  if (d1 >= 0) pk.arena[d1] = b;
  if (d2 >= 0) pk.arena[d2] = b;
}

__global__ __launch_bounds__(256) void rmsprop_step_k(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ sq, float* __restrict__ gavg, int64_t n,
                                                      const double* __restrict__ partials, int n_partials,
                                                      RMSpropParams hp, const int64_t* __restrict__ step,
                                                      float* __restrict__ norms_out, PackMap pk) {
  const NormInfo ni = reduce_norms(partials, n_partials, hp.max_norm);
  const int64_t st = step ? step[0] : 0;
  const float lr = step_lr(hp.lr0, hp.lr_gamma, hp.lr_step_size, hp.lr_step_offset, st);
  if (blockIdx.x == 0 && threadIdx.x == 0 && norms_out) {
    norms_out[0] = ni.l2;
    norms_out[2] = ni.clip;
    norms_out[3] = lr;
  }
  const float a = hp.alpha, oma = 1.f - hp.alpha;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * ni.clip;
    const float s2 = sq[i] * a + oma * gi * gi;
    sq[i] = s2;
    float avg;
    if (hp.centered) {
      float ga = gavg[i];
      ga = ga + oma * (gi - ga);
      gavg[i] = ga;
      avg = sqrtf(fmaxf(s2 - ga * ga, 0.f)) + hp.eps;
    } else {
      avg = sqrtf(s2) + hp.eps;
    }
    const float np = p[i] - lr * gi / avg;
    p[i] = np;
    pack_store(pk, i, np);
  }
}

void rmsprop_step(float* p, const float* g, float* sq, float* gavg, int64_t n, const double* partials,
                  int n_partials, const RMSpropParams& hp, const int64_t* step, float* norms_out, hipStream_t s,
                  const PackMap* pack) {
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  const PackMap pk = pack ? *pack : PackMap{nullptr, nullptr, nullptr};
  rmsprop_step_k<<<blocks, 256, 0, s>>>(p, g, sq, gavg, n, partials, n_partials, hp, step, norms_out, pk);
  LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void adam_step_k(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const double* __restrict__ partials, int n_partials, AdamParams hp,
                                                   const int64_t* __restrict__ step, float* __restrict__ norms_out,
                                                   PackMap pk) {
  const NormInfo ni = reduce_norms(partials, n_partials, hp.max_norm);
  const int64_t st = step ? step[0] : 0;
  const float lr = step_lr(hp.lr0, hp.lr_gamma, hp.lr_step_size, hp.lr_step_offset, st);
  const float t = (float)(st + 1);
  const float bc1 = 1.f - powf(hp.beta1, t), bc2 = 1.f - powf(hp.beta2, t);
  const float step_size = lr / bc1, rbc2 = 1.f / sqrtf(bc2);
  if (blockIdx.x == 0 && threadIdx.x == 0 && norms_out) {
    norms_out[0] = ni.l2;
    norms_out[2] = ni.clip;
    norms_out[3] = lr;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * ni.clip;
    if (hp.weight_decay != 0.f) gi += hp.weight_decay * p[i];
    float mi = m[i];
    mi = mi + (1.f - hp.beta1) * (gi - mi);
    const float vi = v[i] * hp.beta2 + (1.f - hp.beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float np = p[i] - step_size * mi / (sqrtf(vi) * rbc2 + hp.eps);
    p[i] = np;
    pack_store(pk, i, np);
  }
}

void adam_step(float* p, const float* g, float* m, float* v, int64_t n, const double* partials, int n_partials,
               const AdamParams& hp, const int64_t* step, float* norms_out, hipStream_t s, const PackMap* pack) {
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  const PackMap pk = pack ? *pack : PackMap{nullptr, nullptr, nullptr};
  adam_step_k<<<blocks, 256, 0, s>>>(p, g, m, v, n, partials, n_partials, hp, step, norms_out, pk);
  LAUNCH_CHECK();
}

void copy_f32(float* dst, const float* src, int64_t n, hipStream_t s) {
  HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, s));
}

}  // namespace apex
