// Device-side building blocks of the fanout-64 HBM priority tree (replay_kernels.hip), shared
// with the kernels that fold a tree write into another launch (aql_engine_kernels.hip).
#pragma once

#include "common.h"
#include "kernels.h"

namespace apex {

__device__ __forceinline__ float block_reduce_1024(float v, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = is_max ? -INFINITY : 0.f;
  for (int i = 0; i < nw; ++i) t = is_max ? fmaxf(t, red[i]) : t + red[i];  // fixed order
  return t;
}

// Writes one leaf; returns the priority to fold into the running max (0 if none).
__device__ __forceinline__ float write_leaf(const TreeDesc& t, int id, float p, float alpha) {
  if (p > 0.f && isfinite(p)) {
    const float v = powf(p, alpha);
    t.leaf_sum[id] = v;
    t.leaf_min[id] = v;
    return p;
  }
  t.leaf_sum[id] = 0.f;
  t.leaf_min[id] = INFINITY;
  return 0.f;
}

// ------------------------------------------------------------------ fused small updates
// Node recompute by one wave, reading through L2 (the children may have been written by
// other waves of this workgroup earlier in the same kernel).
// Scope: __HIP_MEMORY_SCOPE_AGENT when the children were written by other workgroups
// (ordered by fences + a ticket), __HIP_MEMORY_SCOPE_WORKGROUP inside one workgroup
// (ordered by the barrier).
template <int Scope = __HIP_MEMORY_SCOPE_AGENT>
__device__ __forceinline__ void recompute_node(const TreeDesc& t, int level, int node, int lane) {
  const int child = node * kTreeFanout + lane;
  const int csize = t.size[level - 1];
  double s = 0.0;
  float m = INFINITY;
  if (child < csize) {
    if (level == 1) {
      s = (double)__hip_atomic_load(t.leaf_sum + child, __ATOMIC_RELAXED, Scope);
      m = __hip_atomic_load(t.leaf_min + child, __ATOMIC_RELAXED, Scope);
    } else {
      s = __hip_atomic_load(t.node_sum[level - 2] + child, __ATOMIC_RELAXED, Scope);
      m = __hip_atomic_load(t.node_min[level - 2] + child, __ATOMIC_RELAXED, Scope);
    }
  }
  s = wave_sum(s);
  m = wave_min(m);
  if (lane == 0) {
    t.node_sum[level - 1][node] = s;
    t.node_min[level - 1][node] = m;
  }
}

// Recompute levels lo..hi of the dirty paths of `ids` (run order, staged in LDS) inside
// ONE workgroup: candidate w goes to wave w % nw (strided, so a small batch still spreads
// over every wave; blocks of 64 per wave put a 32-row batch's whole walk on wave 0), which
// recomputes its ancestor if it is the first of its run.  Level-synchronous: only this
// workgroup reads what it wrote, so the barrier (workgroup-scope release / acquire) orders
// the levels for workgroup-scope loads.  A device-scope __threadfence per level wrote the
// XCD L2 back each time.
// K candidates per wave (B <= K x waves, e.g. AQL's 32 rows: K = 8 on 4 waves, 2 on 16): a
// wave's candidates load their 64 children together -- unconditional loads from clamped
// addresses, selected after, so nothing serialises on a per-candidate wait -- then reduce:
// one L2 round trip per level instead of one per candidate.  Same per-node arithmetic, so the
// sums are bit-identical to the one-at-a-time loop.
template <int K>
__device__ __forceinline__ void update_levels_ilp(const TreeDesc& t, const int* sids, int B, int lo, int hi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int level = lo; level <= hi; ++level) {
    __syncthreads();
    const int shift = kTreeLog2Fanout * level, csize = t.size[level - 1], n0 = t.size[0];
    int node[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int w = wave + j * nw;
      const int id = sids[min(w, B - 1)], prev = sids[max(min(w, B - 1) - 1, 0)];
      const int nd = id >> shift;
      const bool first = w == 0 || !(prev >= 0 && prev < n0 && (prev >> shift) == nd);
      node[j] = (w < B && id >= 0 && id < n0 && first) ? nd : -1;
    }
    double s[K];
    float m[K];
    if (level == 1) {
      float fs[K], fm[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int c = min(max(node[j], 0) * kTreeFanout + lane, csize - 1);
        fs[j] = __hip_atomic_load(t.leaf_sum + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        fm[j] = __hip_atomic_load(t.leaf_min + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const bool ok = node[j] >= 0 && node[j] * kTreeFanout + lane < csize;
        s[j] = ok ? (double)fs[j] : 0.0;
        m[j] = ok ? fm[j] : INFINITY;
      }
    } else {
      double ds[K];
      float dm[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int c = min(max(node[j], 0) * kTreeFanout + lane, csize - 1);
        ds[j] = __hip_atomic_load(t.node_sum[level - 2] + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        dm[j] = __hip_atomic_load(t.node_min[level - 2] + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const bool ok = node[j] >= 0 && node[j] * kTreeFanout + lane < csize;
        s[j] = ok ? ds[j] : 0.0;
        m[j] = ok ? dm[j] : INFINITY;
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const double sj = wave_sum(s[j]);
      const float mj = wave_min(m[j]);
      if (node[j] >= 0 && lane == 0) {
        t.node_sum[level - 1][node[j]] = sj;
        t.node_min[level - 1][node[j]] = mj;
      }
    }
  }
}

__device__ __forceinline__ void update_levels_block(const TreeDesc& t, const int* sids, int B, int lo, int hi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // block-uniform dispatch on candidates per wave: the grouped loads pay from 3 per wave (the
  // 256-thread AQL launches: 8); at 1-2 (per_batch_leaves_k's 16 waves) the loop below measured
  // as fast
  const int k = (B + nw - 1) / nw;
  if (k >= 3 && k <= 4) return update_levels_ilp<4>(t, sids, B, lo, hi);
  if (k >= 5 && k <= 8) return update_levels_ilp<8>(t, sids, B, lo, hi);
  for (int level = lo; level <= hi; ++level) {
    __syncthreads();
    const int shift = kTreeLog2Fanout * level;
    for (int w = wave; w < B; w += nw) {  // wave-uniform
      const int id = sids[w];
      if (id < 0 || id >= t.size[0]) continue;
      const int node = id >> shift;
      if (w > 0) {
        const int prev = sids[w - 1];
        if (prev >= 0 && prev < t.size[0] && (prev >> shift) == node) continue;
      }
      recompute_node<__HIP_MEMORY_SCOPE_WORKGROUP>(t, level, node, lane);
    }
  }
}

// The batched tree write of one workgroup (any block size >= 64 and >= B): the actor rows'
// leaves, the learner priority mix + loss mean, deduplicated learner leaves, the running max
// and counters; with ``small_levels_in_block`` every level of the dirty paths too.  ``red``:
// 16 floats, ``sids``: E + B ints of LDS.  Used by per_batch_leaves_k and by the AQL learner's
// noise-reset launch (aql_post_k), which runs it in one extra workgroup.
__device__ __forceinline__ void batch_leaves_block(const TreeDesc& t, const BatchWrite& w, int small_levels_in_block,
                                                   float* red, int* sids) {
  const int k = threadIdx.x;
  // the running max priority: one block-reduced atomic (per-leaf atomics on one address
  // serialise at L2: ~40 us for 768 leaves)
  float pmax = 0.f;
  // actor rows first (they precede this step's learner priorities in time)
  for (int i = k; i < w.E; i += blockDim.x) {
    const int id = w.pre_idx[i];
    sids[i] = id;
    w.list[i] = id;
    if (id >= 0 && id < t.size[0]) pmax = fmaxf(pmax, write_leaf(t, id, w.pre_prio[i], w.alpha));
  }
  float p = 0.f;
  if (w.B > 0) {
    if (w.mix.delta) {
      const float dl = k < w.B ? w.mix.delta[k] : 0.f;
      const float total = block_reduce_1024(k < w.B ? w.mix.lw[k] : 0.f, red, false);
      const float dmax = block_reduce_1024(k < w.B ? dl : -INFINITY, red, true);
      p = prio_mix(dmax, dl);
      if (k < w.B && w.mix.prio_out) w.mix.prio_out[k] = p;
      if (k == 0 && w.mix.loss_out) w.mix.loss_out[0] = total / (float)w.B;
    } else if (k < w.B) {
      p = w.prio ? w.prio[k] : *w.max_prio;
    }
  }
  __syncthreads();  // actor leaves land before any learner leaf (last write wins)
  const int id = k < w.B ? w.idx[k] : -1;
  const bool ok = id >= 0 && id < t.size[0];
  if (k < w.B) {
    sids[w.E + k] = id;
    w.list[w.E + k] = id;
  }
  if (ok) atomicMax(w.owner + id, k);  // device atomics: performed at L2
  __syncthreads();
  if (ok && __hip_atomic_load(w.owner + id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k) {
    const float wp = write_leaf(t, id, p, w.alpha);
    if (w.mix.delta != nullptr || w.prio != nullptr) pmax = fmaxf(pmax, wp);
    w.owner[id] = -1;  // release the claim (only the winner writes; losers never touch it again)
  }
  pmax = block_reduce_1024(pmax, red, true);
  if (k == 0 && pmax > 0.f) atomic_max_pos_float(w.max_prio, pmax);
  if (k == 0) {
    if (w.pre_bump) *w.pre_bump += w.E;
    if (w.bump) *w.bump += 1;
  }
  if (small_levels_in_block) {  // tiny trees: every level in this block
    update_levels_block(t, sids, w.E + w.B, 1, t.levels);
  }
}

}  // namespace apex
