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
  s = tree_sum(s);
  m = tree_min(m);
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
    tree_sum_k<K>(s);
    tree_min_k<K>(m);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (node[j] >= 0 && lane == 0) {
        t.node_sum[level - 1][node[j]] = s[j];
        t.node_min[level - 1][node[j]] = m[j];
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

// Every level of the dirty paths of sids[0, n) (any order, duplicates allowed; n <= 64) in ONE
// memory round trip: the children of every ancestor to recompute, at every level, are
// loaded up front -- all but the dirty ones are final already, and the dirty ones are the
// nodes this workgroup recomputes one level below, substituted from LDS -- then the levels
// are reduced bottom-up through LDS only.  The level-synchronous walk (update_levels_ilp)
// paid a load round trip and a store drain per level (~14 us for a 1M-slot tree, 4 levels).
// Same per-node arithmetic (tree_sum of the 64 children as doubles, tree_min): the sums are
// bit-identical.  K: nodes per wave per level (distinct ancestors per level <= K x waves);
// LP: the deepest tree handled (levels <= LP).
template <int K, int LP>
__device__ __forceinline__ void update_levels_oneshot(const TreeDesc& t, const int* sids, int n,
                                                      long long* dbg = nullptr, int lo = 1, int hi = 1 << 30) {
  __shared__ int s_first[LP][64];    // per level: rank -> candidate index of each distinct ancestor's first
  __shared__ int s_rank[LP][64];     // per level: first candidate -> its rank
  __shared__ int s_firstof[LP][64];  // per level: candidate -> the first candidate of its ancestor
  __shared__ int s_nfirst[LP];
  __shared__ int s_inv[64][64];             // per node rank: child slot -> dirty child's first-rank (-1)
  __shared__ double s_ns[2][64];            // new sums / mins by first-rank, ping-pong over levels
  __shared__ float s_nm[2][64];
  __shared__ double s_os[LP][64];           // every level's new values, stored at the end
  __shared__ float s_om[LP][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6, tid = threadIdx.x;
  // levels lo..L of the walk (lo > 1: levels below are final in memory -- written by an earlier
  // launch -- so level lo substitutes nothing, as level 1 over the leaves)
  const int L = min(t.levels, hi), n0 = t.size[0];
  __syncthreads();  // the caller's leaf writes (workgroup scope) and sids are in place
  // 1) the distinct ancestors per level: one wave per level, lane = candidate, the ancestors
  //    compared through readlane (no LDS round trips); compacted in candidate order (ballot),
  //    so the work split is deterministic
  for (int l = lo + wave; l <= L; l += nw) {
    const int sh = kTreeLog2Fanout * l;
    const int id = lane < n ? sids[lane] : -1;
    const bool ok = id >= 0 && id < n0;
    const int anc = ok ? id >> sh : -1 - lane;  // (invalid candidates match nothing)
    int fo = lane;
    for (int v = 0; v < n; ++v) {  // wave-uniform
      const int av = __builtin_amdgcn_readlane(anc, v);
      if (v < fo && av == anc) fo = v;
    }
    const bool first = ok && fo == lane;
    const uint64_t m = __ballot(first);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (first) {
      s_first[l - 1][rank] = lane;
      s_rank[l - 1][lane] = rank;
    }
    s_firstof[l - 1][lane] = fo;
    if (lane == 0) s_nfirst[l - 1] = __popcll(m);
  }
  __syncthreads();
  if (dbg && threadIdx.x == 0) dbg[0] = (long long)clock64();
  // 2) every level's children, all loads in flight (clamped addresses; selected at use)
  double ps[LP][K];
  float pm[LP][K];
#pragma unroll
  for (int l = 1; l <= LP; ++l) {
    if (l > L) break;  // uniform
    if (l < lo) continue;
    const int sh = kTreeLog2Fanout * l, csize = t.size[l - 1], nf = s_nfirst[l - 1];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int r = wave + k * nw;
      const int node = r < nf ? sids[s_first[l - 1][r]] >> sh : 0;
      const int c = min(node * kTreeFanout + lane, csize - 1);
      if (l == 1) {
        ps[0][k] = (double)__hip_atomic_load(t.leaf_sum + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        pm[0][k] = __hip_atomic_load(t.leaf_min + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        ps[l - 1][k] = __hip_atomic_load(t.node_sum[l - 2] + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        pm[l - 1][k] = __hip_atomic_load(t.node_min[l - 2] + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  // 3) bottom-up through LDS.  The dirty children of a wave's K nodes are substituted by
  //    scatter / gather through a per-wave slot map (all K nodes' LDS traffic batched: a
  //    per-node list walk paid several dependent LDS latencies per node, ~10 us per write)
#pragma unroll
  for (int l = 1; l <= LP; ++l) {
    if (l > L) break;  // uniform
    if (l < lo) continue;
    const int sh = kTreeLog2Fanout * l, csize = t.size[l - 1], nf = s_nfirst[l - 1];
    double sv[K];
    float mv[K];
    int node[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int r = wave + k * nw;
      node[k] = r < nf ? sids[s_first[l - 1][r]] >> sh : 0;
      const bool okc = r < nf && node[k] * kTreeFanout + lane < csize;
      sv[k] = okc ? ps[l - 1][k] : 0.0;
      mv[k] = okc ? pm[l - 1][k] : INFINITY;
    }
    if (l > lo) {
      const int nfc = s_nfirst[l - 2];
#pragma unroll
      for (int k = 0; k < K; ++k) s_inv[wave + k * nw][lane] = -1;
      __syncthreads();
      // one lane per level-(l-1) first: its parent's rank (-> owning wave, k) and child slot
      for (int e = tid; e < nfc; e += blockDim.x) {
        const int w1 = s_first[l - 2][e];
        const int rep = s_rank[l - 1][s_firstof[l - 1][w1]];
        s_inv[rep][(sids[w1] >> (sh - kTreeLog2Fanout)) & (kTreeFanout - 1)] = e;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = s_inv[wave + k * nw][lane];
        if (e >= 0) {
          sv[k] = s_ns[(l - 2) & 1][e];
          mv[k] = s_nm[(l - 2) & 1][e];
        }
      }
    }
    // the reductions, step-major over the wave's nodes; only as many as this level has per wave
    // (levels near the root have 1-4 nodes)
    const int kn = nf > wave ? (nf - wave + nw - 1) / nw : 0;  // wave-uniform
    if (kn > K / 2) {
      tree_sum_k<K>(sv);
      tree_min_k<K>(mv);
    } else if (kn > 1) {
      double s2[(K / 2 > 0 ? K / 2 : 1)];
      float m2[(K / 2 > 0 ? K / 2 : 1)];
#pragma unroll
      for (int k = 0; k < K / 2; ++k) { s2[k] = sv[k]; m2[k] = mv[k]; }
      tree_sum_k<(K / 2 > 0 ? K / 2 : 1)>(s2);
      tree_min_k<(K / 2 > 0 ? K / 2 : 1)>(m2);
#pragma unroll
      for (int k = 0; k < K / 2; ++k) { sv[k] = s2[k]; mv[k] = m2[k]; }
    } else if (kn == 1) {
      sv[0] = tree_sum(sv[0]);
      mv[0] = tree_min(mv[0]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int r = wave + k * nw;
      if (r < nf && lane == 0) {  // (global stores deferred: a barrier waits out pending stores)
        s_ns[(l - 1) & 1][r] = sv[k];
        s_nm[(l - 1) & 1][r] = mv[k];
        s_os[l - 1][r] = sv[k];
        s_om[l - 1][r] = mv[k];
      }
    }
    __syncthreads();
    if (dbg && threadIdx.x == 0) dbg[l] = (long long)clock64();
  }
  // 4) every new node value out at once (nothing in this workgroup reads them back)
  for (int l = lo; l <= L; ++l) {
    const int sh = kTreeLog2Fanout * l;
    for (int r = tid; r < s_nfirst[l - 1]; r += blockDim.x) {
      const int node = sids[s_first[l - 1][r]] >> sh;
      t.node_sum[l - 1][node] = s_os[l - 1][r];
      t.node_min[l - 1][node] = s_om[l - 1][r];
    }
  }
}

// update_levels_oneshot when the batch and the tree fit it, else the level-synchronous walk.
// KMAX caps the per-wave node count compiled in (its prefetch registers: 3 LP KMAX VGPRs),
// e.g. 4 for 1024-thread workgroups (128 VGPRs)
template <int KMAX = 16>
__device__ __forceinline__ void update_levels_fast(const TreeDesc& t, const int* sids, int n, long long* dbg = nullptr,
                                                   int lo = 1, int hi = 1 << 30) {
  const int nw = blockDim.x >> 6;
  hi = min(hi, t.levels);
  if (lo > hi) return;
  // (the one-shot walk's per-wave slot maps index rows wave + k nw < K nw of its 64-row LDS
  // tables: only a K with K nw <= 64 is safe for this workgroup size)
  if (n >= 1 && n <= 64 && t.levels <= 5) {  // block-uniform
    if (n <= 4 * nw && 4 * nw <= 64) return update_levels_oneshot<4, 5>(t, sids, n, dbg, lo, hi);
    if (KMAX >= 8 && n <= 8 * nw && 8 * nw <= 64)
      return update_levels_oneshot<(KMAX >= 8 ? 8 : 4), 5>(t, sids, n, dbg, lo, hi);
    if (KMAX >= 16 && n <= 16 * nw && 16 * nw <= 64)
      return update_levels_oneshot<(KMAX >= 16 ? 16 : 4), 5>(t, sids, n, dbg, lo, hi);
  }
  update_levels_block(t, sids, n, lo, hi);
}

// The batched tree write of one workgroup (any block size >= 64 and >= B): the actor rows'
// leaves, the learner priority mix + loss mean, deduplicated learner leaves, the running max
// and counters; with ``small_levels_in_block`` every level of the dirty paths too.  ``red``:
// 16 floats, ``sids``: E + B ints of LDS.  Used by per_batch_leaves_k and by the AQL learner's
// noise-reset launch (aql_post_k), which runs it in one extra workgroup.
template <int KMAX = 16>
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
    update_levels_fast<KMAX>(t, sids, w.E + w.B);
  }
}

// IS weight of a drawn leaf (memory.py:284-298 as (p / p_min)^-beta) times the shard scale
__device__ __forceinline__ float per_is_weight(float p, float pmin, float wscale, float beta) {
  return wscale * ((p > 0.f && pmin > 0.f && isfinite(pmin)) ? powf(p / pmin, -beta) : 1.f);
}

// The staging row of slot `node` if this launch scatters it (prio > 0), else -1 (wave-uniform)
__device__ __forceinline__ int staged_row_of(const StagedRows& rows, int node, int lane) {
  int se = -1;
  for (int e = lane; e < rows.E; e += 64)
    if (rows.slot[e] == node && rows.prio[e] > 0.f) se = e;
  return wave_max(se);
}

// One staged actor row per thread into the tables (apply_staged_rows), block `rb` of the
// scatter workgroups of a sampling launch
__device__ __forceinline__ void staged_scatter(const StagedRows& rows, int rb) {
  const int e = rb * blockDim.x + threadIdx.x;
  if (e >= rows.E || !(rows.prio[e] > 0.f)) return;
  const int j = rows.slot[e];
  reinterpret_cast<int4*>(rows.dst.s_ids)[j] = reinterpret_cast<const int4*>(rows.st.s_ids)[e];
  reinterpret_cast<int4*>(rows.dst.s2_ids)[j] = reinterpret_cast<const int4*>(rows.st.s2_ids)[e];
  rows.dst.action[j] = rows.st.action[e];
  rows.dst.reward[j] = rows.st.reward[e];
  rows.dst.done[j] = rows.st.done[e];
}

// Block reduction of rows v[0, n) in the order of block_reduce_1024 over a 1024-thread block
// holding one row per thread (wave j sums rows [64 j, 64 j + 64); the wave totals are added in
// order j = 0, 1, ..): any block size gives the same bits as the one-row-per-thread kernels
// (per_write_leaves_sorted_k), so a rider workgroup of 256 threads reproduces their loss mean.
// red: >= (n + 63) / 64 floats.
__device__ __forceinline__ float block_reduce_rows(const float* __restrict__ v, int n, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6, nj = (n + 63) >> 6;
  __syncthreads();
  for (int j = wave; j < nj; j += nw) {  // wave-uniform
    const int r = 64 * j + lane;
    float x = r < n ? v[r] : (is_max ? -INFINITY : 0.f);
    x = is_max ? wave_max(x) : wave_sum(x);
    if (lane == 0) red[j] = x;
  }
  __syncthreads();
  float t = is_max ? -INFINITY : 0.f;
  for (int j = 0; j < nj; ++j) t = is_max ? fmaxf(t, red[j]) : t + red[j];  // fixed order
  return t;
}

// Ride stage 1: batch_leaves_block for any block size (rows strided over the threads), with
// the loss mean / max TD error reduced as the 1024-thread kernels do.  The learner rows' mixed
// priorities are recomputed where used (prio_mix is a pure function of dmax and delta_i).
__device__ __forceinline__ void ride_leaves(const TreeDesc& t, const BatchWrite& w, float* red) {
  const int k = threadIdx.x, nt = blockDim.x;
  float pmax = 0.f;
  for (int i = k; i < w.E; i += nt) {  // actor rows first (they precede the learner's in time)
    const int id = w.pre_idx[i];
    w.list[i] = id;
    if (id >= 0 && id < t.size[0]) pmax = fmaxf(pmax, write_leaf(t, id, w.pre_prio[i], w.alpha));
  }
  float dmax = 0.f;
  if (w.mix.delta && w.B > 0) {
    const float total = block_reduce_rows(w.mix.lw, w.B, red, false);
    dmax = block_reduce_rows(w.mix.delta, w.B, red, true);
    if (k == 0 && w.mix.loss_out) w.mix.loss_out[0] = total / (float)w.B;
  }
  __syncthreads();  // actor leaves land before any learner leaf (last write wins)
  for (int i = k; i < w.B; i += nt) {
    const int id = w.idx[i];
    w.list[w.E + i] = id;
    if (id >= 0 && id < t.size[0]) atomicMax(w.owner + id, i);  // device atomics: performed at L2
  }
  __syncthreads();
  for (int i = k; i < w.B; i += nt) {
    const int id = w.idx[i];
    const float p = w.mix.delta ? prio_mix(dmax, w.mix.delta[i]) : (w.prio ? w.prio[i] : *w.max_prio);
    if (w.mix.delta && w.mix.prio_out) w.mix.prio_out[i] = p;
    if (id >= 0 && id < t.size[0] &&
        __hip_atomic_load(w.owner + id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i) {
      const float wp = write_leaf(t, id, p, w.alpha);
      if (w.mix.delta != nullptr || w.prio != nullptr) pmax = fmaxf(pmax, wp);
      w.owner[id] = -1;  // release the claim (only the winner writes; losers never touch it again)
    }
  }
  pmax = block_reduce_1024(pmax, red, true);
  if (k == 0) {
    if (pmax > 0.f) atomic_max_pos_float(w.max_prio, pmax);
    if (w.pre_bump) *w.pre_bump += w.E;
    if (w.bump) *w.bump += 1;
  }
}

// Ride stage 2: rider workgroup `rb` recomputes level `level` of listed slots (one wave per
// slot; a slot whose predecessor in the list shares the ancestor skips it -- the actor's
// ring-ordered runs).  No ticket / fence: the level above waits for the next launch.
__device__ __forceinline__ void ride_level(const TreeDesc& t, const BatchWrite& w, int level, int rb) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int n = w.E + w.B, i = rb * nw + (threadIdx.x >> 6), sh = kTreeLog2Fanout * level;
  if (i >= n) return;
  const int id = w.list[i];
  const int prev = i > 0 ? w.list[i - 1] : -1;
  const bool dup = prev >= 0 && prev < t.size[0] && id >= 0 && (prev >> sh) == (id >> sh);
  if (id >= 0 && id < t.size[0] && !dup) recompute_node(t, level, id >> sh, lane);
}

// Ride stage 3: every node of levels top_from.. in ONE workgroup (the levels below are final:
// written by earlier launches; level top_from has <= 64 nodes).  One global round trip: each wave
// loads the children of all its level-top_from nodes together, and the levels above reduce
// their children out of LDS.  Same per-node arithmetic as recompute_node (tree_sum of the 64
// children as doubles, tree_min): bit-identical node values.  No device-scope fence (on
// gfx950 a __threadfence writes back the XCD's whole L2 -- inside a GEMM launch its dirty
// output tiles: a ticketed top walk riding the conv2 pair took that launch from 55 to 84 us).
__device__ __forceinline__ void ride_top(const TreeDesc& t, int lo) {
  __shared__ double s_sum[2][64];
  __shared__ float s_min[2][64];
  constexpr int K = 16;  // nodes per wave at level lo (64 nodes over >= 4 waves)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n = t.size[lo], csize = t.size[lo - 1];
  double sv[K];
  float mv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {  // every load in flight (clamped addresses, selected after)
    const int node = wave + k * nw, c = min(min(node, n - 1) * kTreeFanout + lane, csize - 1);
    if (lo == 1) {
      sv[k] = (double)t.leaf_sum[c];
      mv[k] = t.leaf_min[c];
    } else {
      sv[k] = t.node_sum[lo - 2][c];
      mv[k] = t.node_min[lo - 2][c];
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int node = wave + k * nw;
    if (node >= n) break;  // wave-uniform
    const bool ok = node * kTreeFanout + lane < csize;
    const double s = tree_sum(ok ? sv[k] : 0.0);
    const float m = tree_min(ok ? mv[k] : INFINITY);
    if (lane == 0) {
      t.node_sum[lo - 1][node] = s;
      t.node_min[lo - 1][node] = m;
      s_sum[lo & 1][node] = s;
      s_min[lo & 1][node] = m;
    }
  }
  for (int lv = lo + 1; lv <= t.levels; ++lv) {  // <= 64 children per level, from LDS
    __syncthreads();
    const int cs = t.size[lv - 1];
    for (int node = wave; node < t.size[lv]; node += nw) {
      const int c = node * kTreeFanout + lane;
      const double s = tree_sum(c < cs ? s_sum[(lv - 1) & 1][c] : 0.0);
      const float m = tree_min(c < cs ? s_min[(lv - 1) & 1][c] : INFINITY);
      if (lane == 0) {
        t.node_sum[lv - 1][node] = s;
        t.node_min[lv - 1][node] = m;
        s_sum[lv & 1][node] = s;
        s_min[lv & 1][node] = m;
      }
    }
  }
}

// The rider part of a host launch: true when this workgroup was a rider (it has returned from
// its tree work); *gb = the host kernel's own block index otherwise.  Riders of stages 1 and 3
// take block 0 (they start with the launch), level riders the blocks past the host's grid.
__device__ __forceinline__ bool tree_ride(const TreeRide& r, int nhost, float* red, int* gb) {
  const int b = blockIdx.x;
  *gb = b;
  if (r.stage == 1 || r.stage == 3) {
    if (b == 0) {
      if (r.stage == 1) ride_leaves(r.t, r.w, red);
      else ride_top(r.t, r.top_from);
      return true;
    }
    *gb = b - 1;
  } else if (r.stage == 2 && b >= nhost) {
    ride_level(r.t, r.w, r.level, b - nhost);
    return true;
  }
  return false;
}

}  // namespace apex
