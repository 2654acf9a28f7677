// HBM-resident prioritized replay for gfx950.
//
// Instead of the reference's binary segment tree walked in Python under a lock
// (memory.py:10-143, origin_repo/replay.py:92-143), the tree here has fanout 64 =
// one child per lane of a wave64:
//   * a prefix descent is ceil(log64 C) dependent 64-wide loads + a wave prefix scan
//     (2M leaves -> 4 levels instead of 21),
//   * a batched priority update recomputes each dirty node with ONE wave reading its
//     64 children (coalesced 256-512 B) and a fixed-order reduction, so results are
//     deterministic and independent of arrival order.  Duplicate indices resolve
//     last-write-wins like the reference's sequential loop; parents are recomputed
//     level-synchronously (one launch per level), never incrementally, so there is
//     no fp drift and no race on shared ancestors.
// Leaves are fp32, internal sums fp64, mins fp32 (+inf neutral).
#include "common.h"
#include "kernels.h"
#include "tree_dev.h"

namespace apex {

// ------------------------------------------------------------------ leaf writes
// Learner updates (dedup = 1, B <= 1024): one workgroup rank-sorts the (slot, position)
// pairs in LDS; the last position of every run of equal slots wins (the reference applies
// updates sequentially, memory.py:313-320), and the sorted slot list is written out so the
// level kernels dedup parents by comparing with their predecessor (O(1)).
// Actor inserts (dedup = 0) are unique, already ordered ring slots.
// `bump*` are device counters advanced by this kernel (it never reads them), which saves
// a separate counter launch per step.
constexpr int kSortMax = 1024;

// `mix` (optional, the learner's fused loss path): prio is derived here from the per-row
// TD errors, prio_i = 0.9 max_j delta_j + 0.1 delta_i + 1e-6 (utils.py:77), and the loss
// mean sum_i lw_i / B is written -- the batch-wide max/sum the row-parallel loss kernel
// cannot do without another launch.  Reductions in the same fixed order as dqn_loss_k.


__global__ __launch_bounds__(1024) void per_write_leaves_sorted_k(TreeDesc t, const int* __restrict__ idx,
                                                                  const float* __restrict__ prio, int B, float alpha,
                                                                  float* max_prio, int* __restrict__ sorted_out,
                                                                  int64_t* bump0, int64_t d0, int64_t* bump1,
                                                                  int64_t d1, PrioMix mix) {
  __shared__ unsigned long long key[kSortMax], unsorted[kSortMax];
  __shared__ float pmix[kSortMax];
  __shared__ float red[16];
  if (mix.delta) {
    const int k = threadIdx.x;  // B <= blockDim.x
    const float dl = k < B ? mix.delta[k] : 0.f;
    const float total = block_reduce_1024(k < B ? mix.lw[k] : 0.f, red, false);
    const float dmax = block_reduce_1024(k < B ? dl : -INFINITY, red, true);
    if (k < B) {
      const float p = prio_mix(dmax, dl);
      pmix[k] = p;
      if (mix.prio_out) mix.prio_out[k] = p;
    }
    if (k == 0 && mix.loss_out) mix.loss_out[0] = total / (float)B;
    prio = nullptr;
  }
  // rank sort: keys (slot << 32 | position) are unique, so key k's sorted position is the
  // number of smaller keys -- B broadcast LDS reads per thread and no barrier, where a
  // bitonic network paid log2(B)(log2(B)+1)/2 barrier stages (45 for B = 512: ~50 us on a
  // CU shared with the backward's GEMM waves)
  for (int k = threadIdx.x; k < B; k += blockDim.x)
    unsorted[k] = (((unsigned long long)(unsigned)idx[k]) << 32) | (unsigned)k;
  __syncthreads();
  for (int k = threadIdx.x; k < B; k += blockDim.x) {
    const unsigned long long mine = unsorted[k];
    int rank = 0;
#pragma unroll 8
    for (int j = 0; j < B; ++j) rank += unsorted[j] < mine;  // same address in every lane
    key[rank] = mine;
  }
  __syncthreads();
  // the running max priority: one block-reduced atomic (per-leaf atomics on one address
  // serialise at L2; MI355X: 46 us for 512 learner priorities)
  float pmax = 0.f;
  for (int k = threadIdx.x; k < B; k += blockDim.x) {
    const int id = (int)(key[k] >> 32);
    sorted_out[k] = id;
    const bool last = (k == B - 1) || ((int)(key[k + 1] >> 32) != id);
    if (!last || id < 0 || id >= t.size[0]) continue;
    const int src = (int)(key[k] & 0xFFFFFFFFu);
    const float p = mix.delta ? pmix[src] : (prio ? prio[src] : *max_prio);
    const float wp = write_leaf(t, id, p, alpha);
    if (prio || mix.delta) pmax = fmaxf(pmax, wp);
  }
  pmax = block_reduce_1024(pmax, red, true);
  if (threadIdx.x == 0) {
    if (pmax > 0.f) atomic_max_pos_float(max_prio, pmax);
    if (bump0) *bump0 += d0;
    if (bump1) *bump1 += d1;
  }
}

__global__ void per_write_leaves_k(TreeDesc t, const int* __restrict__ idx, const float* __restrict__ prio, int B,
                                   float alpha, float* max_prio, int64_t* bump0, int64_t d0, int64_t* bump1,
                                   int64_t d1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    if (bump0) *bump0 += d0;
    if (bump1) *bump1 += d1;
  }
  if (i >= B) return;
  const int id = idx[i];
  if (id < 0 || id >= t.size[0]) return;
  const float p = prio ? prio[i] : *max_prio;
  if (p > 0.f && isfinite(p)) {
    const float v = powf(p, alpha);
    t.leaf_sum[id] = v;
    t.leaf_min[id] = v;
    if (prio) atomic_max_pos_float(max_prio, p);
  } else {  // empty / invalid slot: no sampling mass, neutral for the min
    t.leaf_sum[id] = 0.f;
    t.leaf_min[id] = INFINITY;
  }
}

// ------------------------------------------------------------------ level recompute
// One wave per (sorted or ring-ordered) slot; children of a node are a contiguous id
// range, so equal parents form runs and only the first of a run recomputes the node.
__global__ void per_update_level_k(TreeDesc t, const int* __restrict__ ids, int B, int level) {
  const int lane = threadIdx.x & 63;
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (w >= B) return;
  const int id = ids[w];
  if (id < 0 || id >= t.size[0]) return;
  const int shift = kTreeLog2Fanout * level;
  const int node = id >> shift;
  if (w > 0) {
    const int prev = ids[w - 1];
    if (prev >= 0 && prev < t.size[0] && (prev >> shift) == node) return;  // wave-uniform
  }
  const int child = node * kTreeFanout + lane;
  const int csize = t.size[level - 1];
  double s = 0.0;
  float m = INFINITY;
  if (child < csize) {
    if (level == 1) {
      s = (double)t.leaf_sum[child];
      m = t.leaf_min[child];
    } else {
      s = t.node_sum[level - 2][child];
      m = t.node_min[level - 2][child];
    }
  }
  s = tree_sum(s);
  m = tree_min(m);
  if (lane == 0) {
    t.node_sum[level - 1][node] = s;
    t.node_min[level - 1][node] = m;
  }
}



// Actor inserts: B (<= kRingFusedMax) unique ring-ordered slots -> leaves AND every level in
// one launch (a ring chunk dirties only a handful of nodes per level).  Up to 4096 slots in one
// workgroup: the central learner's ingest writes R links x E rows per step (3136 at R = 7, E =
// 448) on the tree stream beside the backward, where every extra single-workgroup launch of a
// 1024-slot chunking waited for CU room on its own.
constexpr int kRingFusedMax = 4096;
__global__ __launch_bounds__(1024) void per_write_ring_fused_k(TreeDesc t, const int* __restrict__ idx,
                                                               const float* __restrict__ prio, int B, float alpha,
                                                               float* max_prio, int64_t* bump0, int64_t d0,
                                                               int64_t* bump1, int64_t d1) {
  __shared__ int sids[kRingFusedMax];
  __shared__ float red[16];
  float pmax = 0.f;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const int id = idx[i];
    sids[i] = id;
    if (id < 0 || id >= t.size[0]) continue;
    const float wp = write_leaf(t, id, prio ? prio[i] : *max_prio, alpha);
    if (prio) pmax = fmaxf(pmax, wp);
  }
  pmax = block_reduce_1024(pmax, red, true);  // one atomic, not one per leaf
  if (threadIdx.x == 0) {
    if (pmax > 0.f) atomic_max_pos_float(max_prio, pmax);
    if (bump0) *bump0 += d0;
    if (bump1) *bump1 += d1;
  }
  // a ring chunk dirties ~B / 64 level-1 nodes: one representative slot per distinct level-1
  // node (ring order: duplicates are adjacent), then the one-round-trip walk over those
  __shared__ int comp[64];
  __shared__ int ncomp;
  if (threadIdx.x == 0) ncomp = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const int id = sids[i];
    if (id < 0 || id >= t.size[0]) continue;
    const int prev = i > 0 ? sids[i - 1] : -1;
    if (prev >= 0 && prev < t.size[0] && (prev >> kTreeLog2Fanout) == (id >> kTreeLog2Fanout)) continue;
    const int k = atomicAdd(&ncomp, 1);
    if (k < 64) comp[k] = id;
  }
  __syncthreads();
  if (ncomp <= 64) update_levels_fast<4>(t, comp, ncomp);  // (order-free: node values deterministic)
  else update_levels_block(t, sids, B, 1, t.levels);
}

// The small top levels of a batched (random-slot) update in one workgroup.
__global__ __launch_bounds__(1024) void per_update_top_k(TreeDesc t, const int* __restrict__ ids, int B, int lo) {
  __shared__ int sids[1024];
  for (int i = threadIdx.x; i < B; i += blockDim.x) sids[i] = ids[i];
  update_levels_block(t, sids, B, lo, t.levels);
}

// ------------------------------------------------------------------ stratified sampling
// One wave per sample: mass_i = (u_i + i) * total / B, descend levels with a wave-wide
// inclusive scan of the 64 child sums; IS weight = (p_i / p_min)^-beta
// ( == (p_i N / S)^-beta / (p_min N / S)^-beta, memory.py:284-298 ).
__global__ void per_sample_k(TreeDesc t, int B, const int64_t* length_ptr, int64_t length_const,
                             const float* beta_ptr, float beta_const, uint64_t seed,
                             const int64_t* __restrict__ counter, int* __restrict__ out_idx,
                             float* __restrict__ out_w, int exclude_last, const float* __restrict__ glob,
                             ShardGlob sg, StagedRows rows, SampleRowsOut ro, int sample_blocks) {
  if ((int)blockIdx.x >= sample_blocks) {  // fused staged-row scatter (apply_staged_rows)
    staged_scatter(rows, blockIdx.x - sample_blocks);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (i >= B) return;
  int64_t len64 = length_ptr ? length_ptr[0] : length_const;
  const int length = (int)(len64 < (int64_t)t.size[0] ? len64 : (int64_t)t.size[0]);
  const float beta = beta_ptr ? beta_ptr[0] : beta_const;
  const int L = t.levels;
  const uint64_t ctr = counter ? (uint64_t)counter[0] : 0ull;
  // the root min / global pair read before the descent (independent of it)
  float pmin = glob ? glob[0] : t.node_min[L - 1][0];
  float wscale = glob ? glob[1] : 1.f;
  float p;
  const int node = tree_sample_leaf(t, i, B, length, exclude_last, seed, ctr, lane, &p);
  if (sg.slots) {  // global min priority + k M_rank / sum M over the shards (world <= 64)
    const bool ok = lane < sg.world;
    const double m = wave_sum(ok ? (double)sg.slots[2 * lane] : 0.0);
    pmin = wave_min(ok ? sg.slots[2 * lane + 1] : INFINITY);
    wscale = (float)((double)sg.world * (double)sg.slots[2 * sg.rank] / fmax(m, 1e-300));
  }
  if (lane == 0) {
    out_idx[i] = node;
    out_w[i] = per_is_weight(p, pmin, wscale, beta);
  }
  if (ro.out.s_ids) {  // private row copy: the staged row if this launch scatters the slot (no race with
                       // the scatter blocks), else the table row (a slot nobody writes in this launch)
    const int se = staged_row_of(rows, node, lane);
    const TransTable& src = se >= 0 ? rows.st : ro.src;
    const int r = se >= 0 ? se : node;
    if (lane < 4) ro.out.s_ids[4 * i + lane] = src.s_ids[4 * r + lane];
    else if (lane < 8) ro.out.s2_ids[4 * i + lane - 4] = src.s2_ids[4 * r + lane - 4];
    else if (lane == 8) ro.out.action[i] = src.action[r];
    else if (lane == 9) ro.out.reward[i] = src.reward[r];
    else if (lane == 10) ro.out.done[i] = src.done[r];
  }
}

// ------------------------------------------------------------------ gathers
// Frames are stored once in a u8 ring; a transition holds 4+4 frame ids, so a
// sampled (s, s') pair is assembled by id (7,056 B per frame, not 2x28 KB
// per transition).  One workgroup copies one 84x84 frame with 16-B loads/stores.
__global__ void gather_transitions_k(const uint8_t* __restrict__ frames, int frame_bytes,
                                     const int* __restrict__ s_ids, const int* __restrict__ s2_ids,
                                     const int* __restrict__ act, const float* __restrict__ rew,
                                     const float* __restrict__ done, const int* __restrict__ idx,
                                     uint8_t* __restrict__ out_s, uint8_t* __restrict__ out_s2,
                                     int* __restrict__ out_a, float* __restrict__ out_r,
                                     float* __restrict__ out_d) {
  const int b = blockIdx.x;
  const int which = blockIdx.y;  // 0..3: s frames, 4..7: s' frames
  const int slot = idx[b];
  const int f = (which < 4 ? s_ids : s2_ids)[slot * 4 + (which & 3)];
  const uint4* src = reinterpret_cast<const uint4*>(frames + (size_t)f * frame_bytes);
  uint8_t* dst_base = (which < 4 ? out_s : out_s2) + ((size_t)b * 4 + (which & 3)) * frame_bytes;
  uint4* dst = reinterpret_cast<uint4*>(dst_base);
  const int n16 = frame_bytes >> 4;
  for (int k = threadIdx.x; k < n16; k += blockDim.x) dst[k] = src[k];
  if (which == 0 && threadIdx.x == 0) {
    out_a[b] = act[slot];
    out_r[b] = rew[slot];
    out_d[b] = done[slot];
  }
}

__global__ void gather_frames_k(const uint8_t* __restrict__ frames, int frame_bytes, const int* __restrict__ ids,
                                int stack, uint8_t* __restrict__ out) {
  const int n = blockIdx.x, c = blockIdx.y;
  const int f = ids[n * stack + c];
  const uint4* src = reinterpret_cast<const uint4*>(frames + (size_t)f * frame_bytes);
  uint4* dst = reinterpret_cast<uint4*>(out + ((size_t)n * stack + c) * frame_bytes);
  const int n16 = frame_bytes >> 4;
  for (int k = threadIdx.x; k < n16; k += blockDim.x) dst[k] = src[k];
}

__global__ void bump_counter_k(int64_t* c, int n, int64_t by) {
  const int i = threadIdx.x;
  if (i < n) c[i] += by;
}

// ------------------------------------------------------------------ fast batched writes
// The learner step's whole tree update -- the staged actor rows of the previous actor
// step (E unique ring slots, their initial priorities) followed by this step's B sampled
// slots (mixed priorities, duplicates last-write-wins) -- in three short launches:
//   K1 (one workgroup): actor leaves; learner priority mix + loss mean; dedup by claiming
//      owner[slot] with atomicMax over the batch position (the largest position wins,
//      like the reference's sequential loop) instead of a bitonic sort; winner leaves;
//      the claims are released by the winners; counters bumped; the slot list (actor
//      then learner) written for the level kernels.
//   K2 (wide, per big level): one wave per listed slot recomputes its ancestor at this
//      level from the 64 children.  Several waves may recompute the same node: each
//      reads the same (final) children and writes the same value -- deterministic.
//   The last big level's kernel also finishes the small top levels (<= 64 nodes): the
//      last block to arrive (ticket counter, fenced) recomputes them.
// vs the single-workgroup level walk (per_write_ring_fused_k + per_write_leaves_sorted_k
// + per_update_top_k, ~60 us of latency per step on MI355X) this is ~3 short kernels.


__global__ __launch_bounds__(1024) void per_batch_leaves_k(TreeDesc t, BatchWrite w, int small_levels_in_block) {
  __shared__ float red[16];
  __shared__ int sids[2048];
  batch_leaves_block<4>(t, w, small_levels_in_block, red, sids);  // (1024 threads: 128 VGPRs)
}

// One wave per listed slot: recompute its level-`level` ancestor.  With `top_from` > 0
// the last block to finish also recomputes every node of levels top_from..levels.
__global__ __launch_bounds__(256) void per_batch_level_k(TreeDesc t, const int* __restrict__ list, int n, int level,
                                                         int top_from, int* ticket) {
  const int lane = threadIdx.x & 63;
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (i < n) {
    const int id = list[i];
    if (id >= 0 && id < t.size[0]) recompute_node(t, level, id >> (kTreeLog2Fanout * level), lane);
  }
  if (top_from <= 0) return;
  __shared__ int last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ticket, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int lv = top_from; lv <= t.levels; ++lv) {
    for (int node = wave; node < t.size[lv]; node += nw) recompute_node(t, lv, node, lane);
    __threadfence();
    __syncthreads();
  }
  if (threadIdx.x == 0) *ticket = 0;
}

void per_write_batch(const TreeDesc& t, const BatchWrite& w, int* ticket, hipStream_t s) {
  const int n = w.E + w.B;
  if (n <= 0) return;
  // (the leaves workgroup stages E + B slots in LDS; its learner rows are one per thread)
  if (w.B > 1024 || w.E + w.B > 2048) throw std::invalid_argument("per_write_batch: B <= 1024, E + B <= 2048");
  if (w.B > 0 && !w.idx) throw std::invalid_argument("per_write_batch: learner slots missing");
  if (w.E > 0 && (!w.pre_idx || !w.pre_prio)) throw std::invalid_argument("per_write_batch: actor rows missing");
  if (w.mix.delta && !w.mix.lw) throw std::invalid_argument("per_write_batch: mixing needs lw");
  // big levels (> 64 nodes) get a wide launch each; the rest go to the last one's
  // last block, or -- when no level is big -- to the leaves kernel itself
  int last_big = 0;
  for (int lv = 1; lv <= t.levels; ++lv)
    if (t.size[lv] > 64) last_big = lv;
  // a small batch (<= 64 dirty paths, e.g. AQL's 32-sample learner write) walks every level
  // inside the leaves workgroup: cheaper than the wide launches + ticketed top levels
  if (n <= 64) last_big = 0;
  per_batch_leaves_k<<<1, 1024, 0, s>>>(t, w, last_big == 0 ? 1 : 0);
  LAUNCH_CHECK();
  if (last_big == 0) return;
  const int waves_per_block = 4;
  const int grid = (n + waves_per_block - 1) / waves_per_block;
  for (int lv = 1; lv <= last_big; ++lv) {
    const int top = (lv == last_big && last_big < t.levels) ? last_big + 1 : 0;
    per_batch_level_k<<<grid, 64 * waves_per_block, 0, s>>>(t, w.list, n, lv, top, ticket);
    LAUNCH_CHECK();
  }
}

int tree_ride_blocks(const TreeRide& r) {
  if (r.stage == 1 || r.stage == 3) return 1;
  if (r.stage == 2) return (r.w.E + r.w.B + 3) / 4;  // one wave per listed slot, 4 waves per workgroup
  return 0;
}

int tree_ride_level_stages(const TreeDesc& t) {
  int last_big = 0;
  for (int lv = 1; lv <= t.levels; ++lv)
    if (t.size[lv] > 64) last_big = lv;
  return last_big <= 1 ? 1 : (last_big == 2 ? 2 : -1);
}

// ------------------------------------------------------------------ launchers
void per_write_leaves(const TreeDesc& t, const int* idx, const float* prio, int B, float alpha, float* max_prio,
                      int dedup, int* sorted_scratch, int64_t* bump0, int64_t d0, int64_t* bump1, int64_t d1,
                      hipStream_t s, const float* mix_delta, const float* mix_lw, float* mix_prio_out,
                      float* mix_loss_out) {
  if (B <= 0) return;
  if (mix_delta && (!dedup || !mix_lw)) throw std::invalid_argument("per_write_leaves: mixing needs dedup + lw");
  if (dedup) {
    if (B > kSortMax) throw std::invalid_argument("per_write_leaves: dedup batch must be <= 1024");
    if (!sorted_scratch) throw std::invalid_argument("per_write_leaves: dedup needs a sorted scratch buffer");
    const PrioMix mix{mix_delta, mix_lw, mix_prio_out, mix_loss_out};
    per_write_leaves_sorted_k<<<1, 1024, 0, s>>>(t, idx, prio, B, alpha, max_prio, sorted_scratch, bump0, d0, bump1,
                                                  d1, mix);
    LAUNCH_CHECK();
    per_update_levels(t, sorted_scratch, B, s);
  } else if (B <= kRingFusedMax) {
    per_write_ring_fused_k<<<1, 1024, 0, s>>>(t, idx, prio, B, alpha, max_prio, bump0, d0, bump1, d1);
    LAUNCH_CHECK();
  } else {
    per_write_leaves_k<<<(B + 255) / 256, 256, 0, s>>>(t, idx, prio, B, alpha, max_prio, bump0, d0, bump1, d1);
    LAUNCH_CHECK();
    per_update_levels(t, idx, B, s);
  }
}

// Random-slot batches: one wide launch per level while the level is big, then the
// remaining top levels (<= 64 nodes each) in a single workgroup launch.
void per_update_levels(const TreeDesc& t, const int* idx, int B, hipStream_t s) {
  if (B <= 0) return;
  const int waves_per_block = 4;
  const int grid = (B + waves_per_block - 1) / waves_per_block;
  int level = 1;
  for (; level <= t.levels; ++level) {
    if (level > 1 && t.size[level] <= 64 && B <= 1024) break;
    per_update_level_k<<<grid, 64 * waves_per_block, 0, s>>>(t, idx, B, level);
    LAUNCH_CHECK();
  }
  if (level <= t.levels) {
    per_update_top_k<<<1, 1024, 0, s>>>(t, idx, B, level);
    LAUNCH_CHECK();
  }
}

void per_sample(const TreeDesc& t, int B, const int64_t* length_ptr, int64_t length_const, const float* beta_ptr,
                float beta_const, uint64_t seed, const int64_t* counter, int* out_idx, float* out_w,
                int exclude_last, const float* glob, hipStream_t s, ShardGlob sg, const StagedRows* rows,
                const SampleRowsOut* rows_out) {
  if (B <= 0) return;
  if (sg.slots && (sg.world < 1 || sg.world > 64 || sg.rank < 0 || sg.rank >= sg.world))
    throw std::invalid_argument("per_sample: sharded world must be in [1, 64] with 0 <= rank < world");
  const int waves_per_block = 4;
  const int sblocks = (B + waves_per_block - 1) / waves_per_block;
  const StagedRows r = rows ? *rows : StagedRows{};
  const SampleRowsOut ro = rows_out ? *rows_out : SampleRowsOut{};
  const int rblocks = r.E > 0 ? (r.E + 64 * waves_per_block - 1) / (64 * waves_per_block) : 0;
  per_sample_k<<<sblocks + rblocks, 64 * waves_per_block, 0, s>>>(
      t, B, length_ptr, length_const, beta_ptr, beta_const, seed, counter, out_idx, out_w, exclude_last, glob, sg, r,
      ro, sblocks);
  LAUNCH_CHECK();
}

__global__ void pack_shard_slots_k(TreeDesc t, float* slots, int world, int rank) {
  const int i = threadIdx.x;
  if (i < 2 * world) {
    float v = 0.f;
    if (i == 2 * rank) v = (float)t.node_sum[t.levels - 1][0];
    if (i == 2 * rank + 1) v = t.node_min[t.levels - 1][0];
    slots[i] = v;
  }
}

void pack_shard_slots(const TreeDesc& t, float* slots, int world, int rank, hipStream_t s) {
  if (world < 1 || world > 64 || rank < 0 || rank >= world) throw std::invalid_argument("pack_shard_slots: bad world");
  pack_shard_slots_k<<<1, 128, 0, s>>>(t, slots, world, rank);
  LAUNCH_CHECK();
}

void gather_transitions(const uint8_t* frames, int frame_bytes, const int* s_ids, const int* s2_ids,
                        const int* act, const float* rew, const float* done, const int* idx, int B, uint8_t* out_s,
                        uint8_t* out_s2, int* out_a, float* out_r, float* out_d, hipStream_t s) {
  if (B <= 0) return;
  if (frame_bytes % 16) throw std::invalid_argument("frame_bytes must be a multiple of 16");
  gather_transitions_k<<<dim3(B, 8), 256, 0, s>>>(frames, frame_bytes, s_ids, s2_ids, act, rew, done, idx, out_s,
                                                  out_s2, out_a, out_r, out_d);
  LAUNCH_CHECK();
}

void gather_frames(const uint8_t* frames, int frame_bytes, const int* ids, int N, int stack, uint8_t* out,
                   hipStream_t s) {
  if (N <= 0) return;
  if (frame_bytes % 16) throw std::invalid_argument("frame_bytes must be a multiple of 16");
  gather_frames_k<<<dim3(N, stack), 256, 0, s>>>(frames, frame_bytes, ids, stack, out);
  LAUNCH_CHECK();
}

void bump_counter(int64_t* counter, int n, int64_t by, hipStream_t s) {
  bump_counter_k<<<1, 64, 0, s>>>(counter, n, by);
  LAUNCH_CHECK();
}

}  // namespace apex
