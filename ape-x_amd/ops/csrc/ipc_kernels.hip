// Central-replay experience transport over HIP IPC (xGMI peer writes), device side.
//
// Reference: actor.py:105-115 pushes pickled 50-transition batches over ZeroMQ with a credit
// window of 3; replay.py:77-107 unpickles them under one asyncio lock; learner.py:57-68 /
// actor.py:40-49 publish parameters PUB/SUB with CONFLATE.  Here (parallel/ipc.py):
//
//   * rank 0 owns an UNCACHED device arena (hipDeviceMallocUncached: every access bypasses
//     L2, so writes that peers DMA into it over xGMI are never shadowed by a stale L2 line):
//       ring[R][D] packets  (packet = E frames [E][7056] u8 | E metadata rows [E][14] i32)
//       seq[R][D]  int64    (packet number + 1 of what the slot holds; 0 = never written)
//       params[2][P] fp32   (versioned double buffer the actors pull)
//   * an actor DMAs its packet into ring[r][n % D] (hipMemcpyAsync to the IPC-mapped pointer),
//     then -- same stream, so after the data has landed -- ipc_seq_k stores n + 1 into
//     seq[r][n % D] with a system-scope release.
//   * rank 0's learner graph, between learner steps, runs
//       ipc_scan_k    : per link, how many packets are ready in order from consumed[r]
//                       (system-scope acquire loads of seq; capped per link = pacing);
//       ipc_apply_k   : scatters every ready packet's frames and rows into the link's region
//                       of the HBM replay, emits (global slot | -1, priority) pairs for
//                       the tree write (per_write_* skip slot -1) and advances the replay's
//                       fill counter by the real rows (filler rows, slot -1, carry frames only);
//       ipc_release_k : consumed[r] += ready[r], published to the host control block
//                       (system-scope store into hipHostRegister'ed /dev/shm, which the actor
//                       processes read as their credit).
//     No host polling and no host sync: the whole ingest is four captured launches.
//   * AQL packets (kind 1, parallel/ipc.py AQL_PACKET): rows appended in (link, packet) order to
//     the ONE replay ring at its cursor, then a max-priority leaf write (AQL_dis.py:120-123).
//   * parameters: rank 0 copies the master weights into params[v & 1] on its stream, then
//     ipc_flag_k publishes v to the control block; actors read v there and pull the slot
//     (seqlock check on the version around the copy).
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace apex {
namespace {

constexpr int kMetaCols = 14;
constexpr int kFrameBytes = 84 * 84;
constexpr int kFrameVec = kFrameBytes / 16;  // 441 x 16 B
static_assert(kFrameBytes % 16 == 0, "frames are copied in 16-byte vectors");

__device__ __forceinline__ int64_t load_acquire_sys(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void store_release_sys(int64_t* p, int64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void ipc_scan_k(IpcIngest g) {
  __shared__ int nready[1024];
  const int r = threadIdx.x;
  int n = 0;
  if (r < g.R && (g.live == nullptr || g.live[r])) {
    const int64_t c = g.consumed[r];
    for (int j = 0; j < g.cap; ++j) {
      const int64_t want = c + j + 1;
      if (load_acquire_sys(g.seq + (int64_t)r * g.D + (want - 1) % g.D) != want) break;
      ++n;
    }
  }
  if (r < g.R) {
    g.ready[r] = n;
    nready[r] = n;
  }
  if (!g.prefix) return;  // (uniform branch)
  __syncthreads();
  if (r < g.R) {  // exclusive prefix over the links: where this link's packets go in ring order
    int p = 0;
    for (int q = 0; q < r; ++q) p += nready[q];
    g.prefix[r] = p;
  }
}

// AQL packets (structure of arrays, E rows): st [E][obs] | st2 [E][obs] | amu [E][TA] | act [E]
// (i32) | rew [E] | done [E].  Every ready packet's rows are appended to the ONE replay ring at
// (aql.filled + row) % aql.C in (link, packet) order; slots_out gets the slot (the max-priority
// leaf write that follows) or -1 for an empty window position.
// grid: R * cap * (E / kAqlRows) blocks of 256 threads = 4 waves, one row per wave.
constexpr int kAqlRows = 4;

__global__ __launch_bounds__(256) void ipc_apply_aql_k(IpcIngest g) {
  const int chunks = g.E / kAqlRows;
  const int b = blockIdx.x;
  const int r = b / (g.cap * chunks);
  const int j = (b / chunks) % g.cap;
  const int lane = threadIdx.x & 63, e = (b % chunks) * kAqlRows + (threadIdx.x >> 6);
  const int64_t out = ((int64_t)r * g.cap + j) * g.E + e;
  if (j >= g.ready[r]) {
    if (lane == 0) g.slots_out[out] = -1;
    return;
  }
  const int k = (int)((g.consumed[r] + j) % g.D);
  const float* pk = reinterpret_cast<const float*>(g.ring + ((int64_t)r * g.D + k) * g.packet_bytes);
  const int E = g.E, obs = g.obs, TA = g.TA;
  const float* st = pk;
  const float* st2 = st + (size_t)E * obs;
  const float* amu = st2 + (size_t)E * obs;
  const int* act = reinterpret_cast<const int*>(amu + (size_t)E * TA);
  const float* rew = reinterpret_cast<const float*>(act + E);
  const float* done = rew + E;
  const int64_t row = (int64_t)(g.prefix[r] + j) * E + e;
  const int64_t slot = (g.aql.filled[0] + row) % g.aql.C;
  for (int c = lane; c < obs; c += 64) {
    g.aql.st[slot * obs + c] = st[(size_t)e * obs + c];
    g.aql.st2[slot * obs + c] = st2[(size_t)e * obs + c];
  }
  for (int c = lane; c < TA; c += 64) g.aql.amu[slot * TA + c] = amu[(size_t)e * TA + c];
  if (lane == 0) {
    g.aql.act[slot] = act[e];
    g.aql.rew[slot] = rew[e];
    g.aql.done[slot] = done[e];
    g.slots_out[out] = (int32_t)slot;
  }
}

// grid: R * cap * (E / kRows) blocks of 256 threads; block -> (link r, window j, env rows)
constexpr int kRows = 4;

__global__ __launch_bounds__(256) void ipc_apply_k(IpcIngest g) {
  const int chunks = g.E / kRows;
  const int b = blockIdx.x;
  const int r = b / (g.cap * chunks);
  const int j = (b / chunks) % g.cap;
  const int e0 = (b % chunks) * kRows;
  const int t = threadIdx.x;
  const int64_t out0 = ((int64_t)r * g.cap + j) * g.E + e0;
  if (j >= g.ready[r]) {  // nothing landed in this window position: mask the tree write
    if (t < kRows) g.slots_out[out0 + t] = -1;
    return;
  }
  const int k = (int)((g.consumed[r] + j) % g.D);
  const uint8_t* pkt = g.ring + ((int64_t)r * g.D + k) * g.packet_bytes;
  const int32_t* meta = reinterpret_cast<const int32_t*>(pkt + (int64_t)g.E * kFrameBytes);
  const int64_t fbase = g.frame_base[r], sbase = g.slot_base[r];
  // frames: kRows x 441 16-byte vectors, strided over the block (uncached source, HBM target)
  for (int v = t; v < kRows * kFrameVec; v += 256) {
    const int e = e0 + v / kFrameVec, w = v % kFrameVec;
    const int32_t fs = meta[e * kMetaCols + 13];
    if (fs < 0) continue;  // filler row
    const uint4 x = reinterpret_cast<const uint4*>(pkt + (int64_t)e * kFrameBytes)[w];
    reinterpret_cast<uint4*>(g.frames + (fbase + fs) * kFrameBytes)[w] = x;
  }
  if (t < kRows) {
    const int e = e0 + t;
    const int32_t* m = meta + e * kMetaCols;
    const int32_t ls = m[12];
    // replay fill counter: transition rows written (filler rows, e.g. the reset-frame
    // packet's, carry frames only); one atomic per block from the first lane
    const unsigned long long real = __ballot(ls >= 0) & ((1ull << kRows) - 1);
    if (t == 0 && g.filled && real)
      atomicAdd(reinterpret_cast<unsigned long long*>(g.filled), (unsigned long long)__popcll(real));
    if (ls < 0) {
      g.slots_out[out0 + t] = -1;
      return;
    }
    const int64_t slot = sbase + ls;
    const int32_t fb = (int32_t)fbase;
    int4 s = make_int4(m[0] + fb, m[1] + fb, m[2] + fb, m[3] + fb);
    int4 s2 = make_int4(m[4] + fb, m[5] + fb, m[6] + fb, m[7] + fb);
    reinterpret_cast<int4*>(g.s_ids)[slot] = s;
    reinterpret_cast<int4*>(g.s2_ids)[slot] = s2;
    g.action[slot] = m[8];
    g.reward[slot] = __int_as_float(m[9]);
    g.done[slot] = __int_as_float(m[10]);
    g.slots_out[out0 + t] = (int32_t)slot;
    g.prio_out[out0 + t] = __int_as_float(m[11]);
  }
}

__global__ void ipc_release_k(IpcIngest g) {
  // DQN: the replay's fill counter was advanced per real transition row by ipc_apply_k;
  // AQL: it is the ring cursor the apply read, advanced here by every applied row
  __shared__ unsigned long long total;
  if (threadIdx.x == 0) total = 0;
  __syncthreads();
  const int r = threadIdx.x;
  if (r < g.R) {
    const int n = g.ready[r];
    const int64_t c = g.consumed[r] + n;
    g.consumed[r] = c;
    if (g.applied) g.applied[r] += n;
    // the ring slots are free again: the actor processes read this word as their credit
    if (g.host_consumed) store_release_sys(g.host_consumed + r, c);
    if (g.kind == 1 && n) atomicAdd(&total, (unsigned long long)n);
  }
  __syncthreads();
  if (threadIdx.x == 0 && g.kind == 1 && g.filled && total) g.filled[0] += (int64_t)total * g.E;
  if (threadIdx.x == 0 && g.gate) {  // the SGD steps this ingest's rows pay for (carry kept in budget)
    const int64_t b = g.budget[0] + (int64_t)total * g.E;
    const int64_t n = b / g.gate_batch < (int64_t)g.gate_max ? b / g.gate_batch : (int64_t)g.gate_max;
    g.budget[0] = b - n * g.gate_batch;
    g.gate[0] = (int)n;
  }
}

// one workgroup per env row: its new frame (441 x 16 B) and its 14 metadata words
__global__ __launch_bounds__(128) void ipc_stage_dqn_k(IpcStage st) {
  const int e = blockIdx.x, t = threadIdx.x;
  const int32_t nf = st.new_frame[e];
  const uint4* src = reinterpret_cast<const uint4*>(st.frames + (int64_t)nf * kFrameBytes);
  uint4* dst = reinterpret_cast<uint4*>(st.packet + (int64_t)e * kFrameBytes);
  for (int w = t; w < kFrameVec; w += 128) dst[w] = src[w];
  if (t >= kMetaCols) return;
  int32_t* m = reinterpret_cast<int32_t*>(st.packet + (int64_t)st.E * kFrameBytes) + e * kMetaCols;
  int32_t v = 0;
  if (st.initial) {
    if (t < 8) v = st.hist[e * 4 + (t & 3)];
    else if (t == 8) v = st.actions[e];
    else if (t == 12) v = -1;
    else if (t == 13) v = nf;
  } else {
    const int32_t j = st.slot[e];
    if (t == 12) v = j;
    else if (t == 13) v = nf;
    else if (t == 11) v = __float_as_int(st.prio[e]);
    else if (j >= 0) {
      if (t < 4) v = st.s_ids[j * 4 + t];
      else if (t < 8) v = st.s2_ids[j * 4 + t - 4];
      else if (t == 8) v = st.action[j];
      else if (t == 9) v = __float_as_int(st.reward[j]);
      else v = __float_as_int(st.done[j]);
    }
  }
  m[t] = v;
}

// --- link emulation (IpcEmu): decide per link, write the packets, then publish them
__global__ void ipc_emu_decide_k(IpcEmu g) {
  const int r = threadIdx.x;
  if (r < g.R) g.go[r] = g.sent[r] - __hip_atomic_load(g.consumed + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g.D;
}

__device__ __forceinline__ uint32_t emu_hash(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// grid R * E blocks of 128 threads: (link r, env e)
__global__ __launch_bounds__(128) void ipc_emu_write_k(IpcEmu g) {
  const int r = blockIdx.x / g.E, e = blockIdx.x % g.E, t = threadIdx.x;
  if (!g.go[r]) return;
  const int64_t n = g.sent[r];
  uint8_t* pkt = g.ring + ((int64_t)r * g.D + n % g.D) * g.pkt;
  const int64_t q = n * g.E + e;
  const uint4* src = reinterpret_cast<const uint4*>(g.pool + (q % g.pool_n) * kFrameBytes);
  uint4* dst = reinterpret_cast<uint4*>(pkt + (int64_t)e * kFrameBytes);
  for (int w = t; w < kFrameVec; w += 128) dst[w] = src[w];
  if (t >= kMetaCols) return;
  const int32_t fs = (int32_t)(q % g.F_r), ls = (int32_t)(q % g.C_r);
  const uint32_t h = emu_hash(g.seed ^ ((uint64_t)r << 40) ^ (uint64_t)q);
  int32_t v;
  if (t < 4) v = (int32_t)((q + g.F_r - 4 + t) % g.F_r);          // the stack ending before the new frame
  else if (t < 8) v = (int32_t)((q + g.F_r - 4 + (t - 4) + 3) % g.F_r);  // n-step later (any frames in the region)
  else if (t == 8) v = (int32_t)(h % (uint32_t)g.n_actions);
  else if (t == 9) v = __float_as_int((float)((int)(h >> 8) % 3 - 1));
  else if (t == 10) v = __float_as_int((h >> 4) % 100 == 0 ? 1.f : 0.f);
  else if (t == 11) v = __float_as_int(0.05f + (float)(h >> 12) * (1.f / 1048576.f));
  else if (t == 12) v = ls;
  else v = fs;
  reinterpret_cast<int32_t*>(pkt + (int64_t)g.E * kFrameBytes)[e * kMetaCols + t] = v;
}

__global__ void ipc_emu_publish_k(IpcEmu g) {
  const int r = threadIdx.x;
  if (r >= g.R || !g.go[r]) return;
  const int64_t n = g.sent[r];
  store_release_sys(g.seq + (int64_t)r * g.D + n % g.D, n + 1);  // after the packet (kernel boundary)
  g.sent[r] = n + 1;
}

// --- pinned parameter publish
__global__ void ipc_param_pick_k(int64_t* ctrl, int pin_off, int R, int begin_off, int K, int64_t v, int* pick) {
  if (threadIdx.x != 0) return;
  uint64_t busy = 1ull << (__hip_atomic_load(ctrl + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) & 0xFF);
  for (int r = 0; r < R; ++r) {
    const int64_t p = __hip_atomic_load(ctrl + pin_off + r, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (p != 0) busy |= 1ull << (p & 0xFF);
  }
  int b = 0;
  while (b < K - 1 && ((busy >> b) & 1ull)) ++b;  // (K = R + 2 > #busy: a free one exists)
  pick[0] = b;
  store_release_sys(ctrl + begin_off + b, v);  // begun: a reader whose pull overlaps sees it
}

__global__ __launch_bounds__(256) void ipc_param_copy_k(float* params, const float* __restrict__ src, int64_t P,
                                                        int64_t stride_f, const int* __restrict__ pick) {
  float* dst = params + (int64_t)pick[0] * stride_f;
  const int64_t n4 = P >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) dst[i] = src[i];
}

__global__ void ipc_param_release_k(int64_t* ctrl, int64_t v, const int* __restrict__ pick) {
  if (threadIdx.x == 0) store_release_sys(ctrl + 2, (v << 8) | (int64_t)pick[0]);
}

__global__ void ipc_flag_k(int64_t* p, int64_t v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) store_release_sys(p, v);
}

}  // namespace

void ipc_ingest(const IpcIngest& g, hipStream_t s) {
  if (g.R < 1 || g.R > 1024 || g.D < 1 || g.cap < 1 || g.cap > g.D || g.E < kRows || g.E % kRows)
    throw std::invalid_argument("ipc_ingest: bad geometry (R <= 1024, 1 <= cap <= D, E a multiple of 4)");
  if (!g.ring || !g.seq || !g.consumed || !g.ready || !g.slots_out)
    throw std::invalid_argument("ipc_ingest: null pointer");
  if (g.kind == 0) {
    if (g.packet_bytes < (int64_t)g.E * (kFrameBytes + kMetaCols * 4))
      throw std::invalid_argument("ipc_ingest: packet stride smaller than a packet");
    if (!g.frames || !g.s_ids || !g.s2_ids || !g.action || !g.reward || !g.done || !g.prio_out || !g.frame_base ||
        !g.slot_base)
      throw std::invalid_argument("ipc_ingest: null DQN table pointer");
  } else if (g.kind == 1) {
    if (g.obs < 1 || g.TA < 1 || g.packet_bytes < (int64_t)g.E * (2 * g.obs + g.TA + 3) * 4)
      throw std::invalid_argument("ipc_ingest: AQL packet stride smaller than a packet");
    if (g.packet_bytes % 4) throw std::invalid_argument("ipc_ingest: AQL packet stride must be a multiple of 4");
    const AqlInsert& a = g.aql;
    if (!g.prefix || !a.st || !a.st2 || !a.amu || !a.act || !a.rew || !a.done || !a.filled || !g.filled ||
        a.C < (int64_t)g.R * g.cap * g.E)
      throw std::invalid_argument("ipc_ingest: AQL tables (capacity >= R * cap * E)");
  } else {
    throw std::invalid_argument("ipc_ingest: kind must be 0 (DQN) or 1 (AQL)");
  }
  if (g.gate && (g.kind != 1 || !g.budget || g.gate_batch < 1 || g.gate_max < 0))
    throw std::invalid_argument("ipc_ingest: the step gate needs AQL rows, a budget, batch >= 1");
  const int thr = ((g.R + 63) / 64) * 64;
  ipc_scan_k<<<1, thr, 0, s>>>(g);
  LAUNCH_CHECK();
  if (g.kind == 0) ipc_apply_k<<<g.R * g.cap * (g.E / kRows), 256, 0, s>>>(g);
  else ipc_apply_aql_k<<<g.R * g.cap * (g.E / kAqlRows), 256, 0, s>>>(g);
  LAUNCH_CHECK();
  ipc_release_k<<<1, thr, 0, s>>>(g);
  LAUNCH_CHECK();
}

void ipc_stage_dqn(const IpcStage& st, hipStream_t s) {
  if (st.E < 1 || !st.frames || !st.new_frame || !st.packet) throw std::invalid_argument("ipc_stage_dqn: frames");
  if (st.initial ? (!st.hist || !st.actions)
                 : (!st.s_ids || !st.s2_ids || !st.action || !st.reward || !st.done || !st.slot || !st.prio))
    throw std::invalid_argument("ipc_stage_dqn: row sources");
  ipc_stage_dqn_k<<<st.E, 128, 0, s>>>(st);
  LAUNCH_CHECK();
}

void ipc_emu_push(const IpcEmu& g, hipStream_t s) {
  if (g.R < 1 || g.R > 1024 || g.D < 1 || g.E < 1 || g.C_r < g.E || g.F_r < g.C_r || g.pool_n < 1 || g.n_actions < 1 ||
      g.pkt < (int64_t)g.E * (kFrameBytes + kMetaCols * 4))
    throw std::invalid_argument("ipc_emu_push: geometry");
  if (!g.ring || !g.seq || !g.consumed || !g.sent || !g.go || !g.pool) throw std::invalid_argument("ipc_emu_push: null");
  const int thr = ((g.R + 63) / 64) * 64;
  ipc_emu_decide_k<<<1, thr, 0, s>>>(g);
  LAUNCH_CHECK();
  ipc_emu_write_k<<<g.R * g.E, 128, 0, s>>>(g);
  LAUNCH_CHECK();
  ipc_emu_publish_k<<<1, thr, 0, s>>>(g);
  LAUNCH_CHECK();
}

void ipc_param_publish(int64_t* ctrl, int pin_off, int R, int begin_off, int K, float* params, int64_t stride_f,
                       const float* src, int64_t P, int64_t v, int* pick, hipStream_t s) {
  if (!ctrl || !params || !src || !pick || R < 1 || K < R + 2 || K > 64 || P < 1 || v < 1 || stride_f < P)
    throw std::invalid_argument("ipc_param_publish: K in [R + 2, 64], pointers, P and v positive, stride >= P");
  if ((reinterpret_cast<uintptr_t>(params) | reinterpret_cast<uintptr_t>(src)) & 15 || stride_f % 4)
    throw std::invalid_argument("ipc_param_publish: 16-byte aligned buffers and stride");
  ipc_param_pick_k<<<1, 64, 0, s>>>(ctrl, pin_off, R, begin_off, K, v, pick);
  LAUNCH_CHECK();
  const int64_t n4 = P / 4;
  const int blocks = (int)std::min<int64_t>(1024, (n4 + 255) / 256);
  ipc_param_copy_k<<<std::max(blocks, 1), 256, 0, s>>>(params, src, P, stride_f, pick);
  LAUNCH_CHECK();
  ipc_param_release_k<<<1, 64, 0, s>>>(ctrl, v, pick);
  LAUNCH_CHECK();
}

void ipc_flag(int64_t* p, int64_t v, hipStream_t s) {
  if (!p) throw std::invalid_argument("ipc_flag: null pointer");
  ipc_flag_k<<<1, 64, 0, s>>>(p, v);
  LAUNCH_CHECK();
}

}  // namespace apex
