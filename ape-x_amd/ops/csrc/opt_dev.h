// Device-side optimizer pieces shared by the learner's optimizer launches
// (learner_kernels.hip: opt_step_k / opt_step2_k) and the AQL learner's fused step tail
// (aql_engine_kernels.hip: aql_step_tail_k), so both round every update identically.
#pragma once

#include "common.h"
#include "kernels.h"

namespace apex {

// Every update block re-reduces the partials in the same fixed order (deterministic,
// identical in all blocks): strided per-thread sums, a wave64 butterfly, then the 4 wave
// sums in order -- one __syncthreads instead of a 256-wide LDS tree.  The reference's
// per-tensor 'grad_norm' log value is computed on demand on the host side
// (DQNLearner.stats), not on every step.  ``grad_scale`` (1/world for data-parallel
// replicas) turns the all-reduced SUM into the mean inside this pass (no scaling kernel).
struct NormInfo {
  float clip, l2;
};
__device__ inline NormInfo reduce_norms(const double* partials, int n_partials, float max_norm, float grad_scale) {
  __shared__ double red[4];
  double t = 0.0;
  // 4 loads in flight per round, added in the same (k-ascending) order as one at a time
  const int bd = blockDim.x;
  int k = threadIdx.x;
  for (; k + 3 * bd < n_partials; k += 4 * bd) {
    const double a0 = partials[k], a1 = partials[k + bd], a2 = partials[k + 2 * bd], a3 = partials[k + 3 * bd];
    t += a0;
    t += a1;
    t += a2;
    t += a3;
  }
  for (; k < n_partials; k += bd) t += partials[k];
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  NormInfo ni;
  ni.l2 = (float)(sqrt((red[0] + red[1]) + (red[2] + red[3])) * (double)grad_scale);
  const float coef = max_norm > 0.f ? max_norm / (ni.l2 + 1e-6f) : 1.f;
  ni.clip = fminf(coef, 1.f) * grad_scale;  // applied to the raw (summed) gradient
  return ni;
}

__device__ __forceinline__ float step_lr(float lr0, float gamma, int step_size, int offset, int64_t step) {
  if (gamma == 1.f || step_size <= 0) return lr0;
  const int64_t k = (step + offset) / step_size;
  return lr0 * powf(gamma, (float)k);
}

// Per-element update rules: (param, clipped grad, state1, state2) -> new param, written
// with explicit fmaf so every call site -- the FC1 tile path and the generic path --
// rounds identically.  The build uses -ffp-contract=fast, under which the backend may
// fuse a multiply into a later add differently per call site (the source pragma does
// not stop that): the clipped gradient is therefore passed through ``opaque`` (an
// empty asm that hides the multiply from the combiner, no instruction emitted).
__device__ __forceinline__ float opaque(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
struct RmsRule {
  float lr, a, oma, eps;
  int centered;
  __device__ __forceinline__ float operator()(float p, float gi, float& s1, float& s2) const {
#pragma clang fp contract(off)
    s1 = fmaf(s1, a, oma * gi * gi);  // square average
    float avg;
    if (centered) {
      s2 = fmaf(oma, gi - s2, s2);  // grad average
      avg = sqrtf(fmaxf(fmaf(-s2, s2, s1), 0.f)) + eps;
    } else {
      avg = sqrtf(s1) + eps;
    }
    return fmaf(-lr, gi / avg, p);
  }
};
struct AdamRule {
  float b1, b2, eps, wd, step_size, rbc2;
  __device__ __forceinline__ float operator()(float p, float gi, float& m, float& v) const {
#pragma clang fp contract(off)
    if (wd != 0.f) gi = fmaf(wd, p, gi);
    m = fmaf(1.f - b1, gi - m, m);
    v = fmaf(v, b2, (1.f - b2) * gi * gi);
    return fmaf(-step_size, m / fmaf(sqrtf(v), rbc2, eps), p);
  }
};

__device__ __forceinline__ RmsRule make_rule(const RMSpropParams& hp, int64_t st, float& lr) {
  lr = step_lr(hp.lr0, hp.lr_gamma, hp.lr_step_size, hp.lr_step_offset, st);
  return RmsRule{lr, hp.alpha, 1.f - hp.alpha, hp.eps, hp.centered};
}
__device__ __forceinline__ AdamRule make_rule(const AdamParams& hp, int64_t st, float& lr) {
  lr = step_lr(hp.lr0, hp.lr_gamma, hp.lr_step_size, hp.lr_step_offset, st);
  const float t = (float)(st + 1);
  const float bc1 = 1.f - powf(hp.beta1, t), bc2 = 1.f - powf(hp.beta2, t);
  return AdamRule{hp.beta1, hp.beta2, hp.eps, hp.weight_decay, lr / bc1, 1.f / sqrtf(bc2)};
}

}  // namespace apex
