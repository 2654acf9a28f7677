// AQL (amortized Q-learning) kernels for gfx950 (reference
// model.py:132-164 NoisyLinear, 209-335 Q_Network, 337-390 Proposal_Network).
//
// * aql_noisy_eff: W_eff = mu + sigma * eps for both NoisyLinear layers (train mode) or
//   mu (eval), once per call into a small workspace (the factorised noise buffers are
//   read as the reference stores them).
// * aql_candidate_q: Q[b, t] for every (state, candidate) pair -- q_feature MLP,
//   action encoder MLP, concat, NoisyLinear(128->64)-ReLU-NoisyLinear(64->1) fused; one
//   wave per candidate, the three 64x128 matrices staged once per workgroup in LDS
//   (odd row pitch: conflict-free column reads).
// * aql_propose: candidate sets on device -- state embedding, proposal MLP, then
//   `uniform` candidates (U(low, high) per dim, or distinct actions = a random
//   permutation prefix for discrete spaces) followed by `propose` samples of
//   MVN(mu, diag(var)) (Box-Muller on Philox) or Categorical(softmax(logits))
//   (model.py:361-374 order: uniform first, then proposal samples).
// * aql_select: per-row epsilon-greedy over the T candidates + gather of the env action.
#include "common.h"
#include "kernels.h"

namespace apex {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int AQ_H = 64;        // hidden units of q_feature / action_out / advantage1
constexpr int AQ_CAT = 128;     // concat width
constexpr int AQ_PITCH = 129;   // LDS row pitch (floats) for 128-wide rows
constexpr int kAqGroup = 8;     // candidates per work item of aql_candidate_q_k

// workspace layout (floats): W1eff [64][128] | b1eff [64] | w2eff [64] | b2eff [1]
size_t aql_workspace_floats() { return AQ_H * AQ_CAT + AQ_H + AQ_H + 1; }

__device__ __forceinline__ void noisy_eff_elem(const AQLNet& net, float* __restrict__ ws, int i);

__global__ void aql_noisy_eff_k(AQLNet net, float* __restrict__ ws) {
  noisy_eff_elem(net, ws, blockIdx.x * blockDim.x + threadIdx.x);
}

__global__ __launch_bounds__(256) void aql_candidate_q_k(AQLNet net, const float* __restrict__ ws,
                                                         const float* __restrict__ state,
                                                         const float* __restrict__ a_mu, int B,
                                                         float* __restrict__ q) {
  // LDS: W1eff [64][129], ao_w2 [64][129], qf_w2 [64][65], per-wave scratch
  __shared__ float w1s[AQ_H * AQ_PITCH];
  __shared__ float ao2s[AQ_H * AQ_PITCH];
  __shared__ float qf2s[AQ_H * (AQ_H + 1)];
  __shared__ float hbuf[4][AQ_CAT];
  __shared__ float xbuf[4][AQ_CAT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < AQ_H * AQ_CAT; e += 256) {
    const int r = e / AQ_CAT, c = e % AQ_CAT;
    w1s[r * AQ_PITCH + c] = ws[e];
    if (net.cont) ao2s[r * AQ_PITCH + c] = net.ao_w2[e];
  }
  for (int e = threadIdx.x; e < AQ_H * AQ_H; e += 256) qf2s[(e / AQ_H) * (AQ_H + 1) + e % AQ_H] = net.qf_w2[e];
  __syncthreads();
  const float* b1eff = ws + AQ_H * AQ_CAT;
  const float* w2eff = b1eff + AQ_H;
  const float b2eff = w2eff[AQ_H];
  // work item = (state b, group of kAqGroup candidates): the state's q_feature and the state
  // half of advantage1 (its input is [action_out | q_feature]) are computed once per item, not
  // once per candidate (they do not depend on the action: ~45 % of a candidate's MACs)
  const int T = net.T, ng = (T + kAqGroup - 1) / kAqGroup, items = B * ng;
  for (int it = blockIdx.x * 4 + wave; it < items; it += gridDim.x * 4) {  // wave-uniform loop
    const int b = it / ng, t0 = (it - b * ng) * kAqGroup, t1 = min(T, t0 + kAqGroup);
    const float* s = state + (size_t)b * net.obs;
    // q_feature: obs -> 64 -> 64 (ReLU both)
    float acc = net.qf_b1[lane];
    for (int i = 0; i < net.obs; ++i) acc += net.qf_w1[lane * net.obs + i] * s[i];
    hbuf[wave][lane] = fmaxf(acc, 0.f);
    __builtin_amdgcn_wave_barrier();
    acc = net.qf_b2[lane];
#pragma unroll 8
    for (int j = 0; j < AQ_H; ++j) acc += qf2s[lane * (AQ_H + 1) + j] * hbuf[wave][j];
    xbuf[wave][AQ_H + lane] = fmaxf(acc, 0.f);
    __builtin_amdgcn_wave_barrier();
    float sadv = b1eff[lane];  // advantage1 bias + its state half
#pragma unroll 8
    for (int j = 0; j < AQ_H; ++j) sadv += w1s[lane * AQ_PITCH + AQ_H + j] * xbuf[wave][AQ_H + j];
    for (int t = t0; t < t1; ++t) {
      const int c = b * T + t;
      // action encoder
      if (net.cont) {
        const float* a = a_mu + (size_t)c * net.adim;
        float h0 = net.ao_b1[lane], h1 = net.ao_b1[lane + 64];
        for (int d = 0; d < net.adim; ++d) {
          const float ad = a[d];
          h0 += net.ao_w1[lane * net.adim + d] * ad;
          h1 += net.ao_w1[(lane + 64) * net.adim + d] * ad;
        }
        __builtin_amdgcn_wave_barrier();
        hbuf[wave][lane] = fmaxf(h0, 0.f);
        hbuf[wave][lane + 64] = fmaxf(h1, 0.f);
        __builtin_amdgcn_wave_barrier();
        acc = net.ao_b2[lane];
#pragma unroll 8
        for (int j = 0; j < AQ_CAT; ++j) acc += ao2s[lane * AQ_PITCH + j] * hbuf[wave][j];
        xbuf[wave][lane] = fmaxf(acc, 0.f);
      } else {
        xbuf[wave][lane] = fmaxf(net.ao_w1[lane] * a_mu[c] + net.ao_b1[lane], 0.f);
      }
      __builtin_amdgcn_wave_barrier();
      // advantage1 (NoisyLinear 128 -> 64): the action half on top of the state half; advantage2 (64 -> 1)
      acc = sadv;
#pragma unroll 8
      for (int j = 0; j < AQ_H; ++j) acc += w1s[lane * AQ_PITCH + j] * xbuf[wave][j];
      const float qv = wave_sum(w2eff[lane] * fmaxf(acc, 0.f)) + b2eff;
      if (lane == 0) q[c] = qv;
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// Four states per 256-thread workgroup: dist_feature.0's weight [128][128] is staged in LDS once
// per workgroup (pitch 132: lane j's 16-byte row reads cover all 64 banks per 16 lanes) -- one
// wave per state read it from global with a 512-byte lane stride (64 cache lines per load,
// ~14 us for 256 states).  Same fma order as the one-wave-per-state version: bit-identical.
// Blocks past prop_blocks compute the acting net's effective NoisyLinear weights (aql_noisy_eff)
// into eff_ws when it is given, so the acting chain has one launch fewer.
constexpr int kPropStates = 4, kPropPitch = 132;

__device__ __forceinline__ void noisy_eff_elem(const AQLNet& net, float* __restrict__ ws, int i) {
  const int n1 = AQ_H * AQ_CAT;
  auto eff = [&](const float* mu, const float* sg, const float* ep, int k) {
    return net.noisy ? mu[k] + sg[k] * ep[k] : mu[k];
  };
  if (i < 0) return;
  if (i < n1) ws[i] = eff(net.a1_wmu, net.a1_wsig, net.a1_weps, i);
  else if (i < n1 + AQ_H) ws[i] = eff(net.a1_bmu, net.a1_bsig, net.a1_beps, i - n1);
  else if (i < n1 + 2 * AQ_H) ws[i] = eff(net.a2_wmu, net.a2_wsig, net.a2_weps, i - n1 - AQ_H);
  else if (i == n1 + 2 * AQ_H) ws[i] = eff(net.a2_bmu, net.a2_bsig, net.a2_beps, 0);
}

__global__ __launch_bounds__(256) void aql_propose_k(AQLNet net, const float* __restrict__ state, int B,
                                                     const float* __restrict__ low, const float* __restrict__ high,
                                                     const float* __restrict__ var, uint64_t seed,
                                                     const int64_t* __restrict__ counter, float* __restrict__ a_mu,
                                                     float* __restrict__ mu_out, float* __restrict__ eff_ws,
                                                     int prop_blocks) {
  if ((int)blockIdx.x >= prop_blocks) {  // block-uniform: the fused effective-weight blocks
    noisy_eff_elem(net, eff_ws, ((int)blockIdx.x - prop_blocks) * 256 + (int)threadIdx.x);
    return;
  }
  __shared__ __attribute__((aligned(16))) float w1[AQ_CAT * kPropPitch];
  __shared__ __attribute__((aligned(16))) float w2[64 * kPropPitch];  // dist_feature.2 [na <= 64][128]
  __shared__ float fw[AQ_CAT * 65];                                  // q.features [128][obs <= 64] (pitch 65)
  __shared__ float sst[kPropStates][64];                             // the workgroup's states
  __shared__ __attribute__((aligned(16))) float emb[kPropStates][AQ_CAT], hid[kPropStates][AQ_CAT];
  __shared__ float mu[kPropStates][64];
  __shared__ int perm[kPropStates][64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b0 = blockIdx.x * kPropStates;
  {  // stage dist_feature.0 [128][128]: every load in flight before the stores
    if ((reinterpret_cast<uintptr_t>(net.df_w1) & 15) == 0) {  // block-uniform
      const f32x4* src = reinterpret_cast<const f32x4*>(net.df_w1);
      f32x4 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = src[t + 256 * k];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int e4 = t + 256 * k, r = e4 >> 5, c = (e4 & 31) * 4;
        *reinterpret_cast<f32x4*>(&w1[r * kPropPitch + c]) = v[k];
      }
    } else {
      for (int e = t; e < AQ_CAT * AQ_CAT; e += 256) w1[(e >> 7) * kPropPitch + (e & 127)] = net.df_w1[e];
    }
    // dist_feature.2 [na][128] (a row per lane below: one wave read 64 rows 512 bytes apart per
    // load, 128 loads deep)
    for (int e = t; e < net.na * AQ_CAT; e += 256) w2[(e >> 7) * kPropPitch + (e & 127)] = net.df_w2[e];
    // q.features and the states: a runtime-length loop of global loads feeding FMAs waited out
    // one L2 round trip per input (obs of them) for the embedding
    for (int e = t; e < AQ_CAT * net.obs; e += 256) fw[(e / net.obs) * 65 + e % net.obs] = net.f_w[e];
    for (int e = t; e < kPropStates * net.obs; e += 256) {
      const int s2 = e / net.obs;
      sst[s2][e - s2 * net.obs] = state[(size_t)min(b0 + s2, B - 1) * net.obs + (e - s2 * net.obs)];
    }
  }
  __syncthreads();
  // state embedding: features = Linear(obs -> 128) + ReLU (model.py:289-291); thread (j, half):
  // states half, half + 2 of the workgroup (clamped past B: computed, never written out)
  const int j = t & 127, hs = t >> 7;
#pragma unroll
  for (int s2 = hs; s2 < kPropStates; s2 += 2) {
    float acc = net.f_b[j];
    for (int i = 0; i < net.obs; ++i) acc += fw[j * 65 + i] * sst[s2][i];
    emb[s2][j] = fmaxf(acc, 0.f);
  }
  __syncthreads();
  // dist_feature: Linear(128 -> 128) + ReLU + Linear(128 -> A)
  {
    const float bj = net.df_b1[j];
    float a0 = bj, a1 = bj;
    const float* wr = w1 + j * kPropPitch;
#pragma unroll 8
    for (int i = 0; i < AQ_CAT; i += 4) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(wr + i);
      const f32x4 e0 = *reinterpret_cast<const f32x4*>(&emb[hs][i]);
      const f32x4 e1 = *reinterpret_cast<const f32x4*>(&emb[hs + 2][i]);
      a0 += w[0] * e0[0]; a0 += w[1] * e0[1]; a0 += w[2] * e0[2]; a0 += w[3] * e0[3];
      a1 += w[0] * e1[0]; a1 += w[1] * e1[1]; a1 += w[2] * e1[2]; a1 += w[3] * e1[3];
    }
    hid[hs][j] = fmaxf(a0, 0.f);
    hid[hs + 2][j] = fmaxf(a1, 0.f);
  }
  __syncthreads();
  const int A = net.na;  // continuous: action dim; discrete: number of actions
  const int b = b0 + wave;  // sampling: one wave per state
  const bool valid = b < B;
  if (lane < A) {
    float acc = net.df_b2[lane];
    for (int i = 0; i < AQ_CAT; ++i) acc += w2[lane * kPropPitch + i] * hid[wave][i];
    mu[wave][lane] = acc;
    if (mu_out && valid) mu_out[(size_t)b * A + lane] = acc;
  }
  __syncthreads();
  const uint64_t ctr = counter ? (uint64_t)counter[0] : 0ull;
  const int U = net.uniform, T = net.T;
  float u[4];
  if (net.cont) {
    if (!valid) return;
    float* out = a_mu + (size_t)b * T * A;
    for (int e = lane; e < T * A; e += 64) {
      const int tt = e / A, d = e % A;
      uniform4(seed, (uint64_t)b * 4096 + e, ctr, u);
      out[e] = tt < U ? low[d] + (high[d] - low[d]) * u[0] : mu[wave][d] + sqrtf(var[d]) * std_normal(u[1], u[2]);
    }
  } else {
    if (lane == 0 && valid) {  // uniform without replacement: partial Fisher-Yates over 0..A-1
      for (int i = 0; i < A; ++i) perm[wave][i] = i;
      for (int i = 0; i < U; ++i) {
        uniform4(seed, (uint64_t)b * 4096 + 4000 + i, ctr, u);
        const int jj = i + min((int)(u[0] * (float)(A - i)), A - i - 1);
        const int tmp = perm[wave][i];
        perm[wave][i] = perm[wave][jj];
        perm[wave][jj] = tmp;
      }
    }
    __syncthreads();
    if (!valid) return;
    float* out = a_mu + (size_t)b * T;
    float mx = -INFINITY;
    for (int i = 0; i < A; ++i) mx = fmaxf(mx, mu[wave][i]);
    float z = 0.f;
    for (int i = 0; i < A; ++i) z += expf(mu[wave][i] - mx);
    for (int tt = lane; tt < T; tt += 64) {
      if (tt < U) {
        out[tt] = (float)perm[wave][tt];
      } else {  // inverse-CDF categorical sample of softmax(logits)
        uniform4(seed, (uint64_t)b * 4096 + tt, ctr, u);
        const float target = u[0] * z;
        float c = 0.f;
        int k = A - 1;
        for (int i = 0; i < A; ++i) {
          c += expf(mu[wave][i] - mx);
          if (c > target) { k = i; break; }
        }
        out[tt] = (float)k;
      }
    }
  }
}

__global__ void aql_select_k(const float* __restrict__ q, const float* __restrict__ a_mu, int B, int T, int adim,
                             const float* __restrict__ eps, uint64_t seed, const int64_t* __restrict__ counter,
                             int* __restrict__ act_idx, float* __restrict__ env_act) {
  const int lane = threadIdx.x & 63;
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (b >= B) return;
  float best = -INFINITY;
  int arg = 0x7fffffff;
  for (int t = lane; t < T; t += 64) {
    const float v = q[(size_t)b * T + t];
    if (v > best || (v == best && t < arg)) { best = v; arg = t; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (ov > best || (ov == best && oa < arg)) { best = ov; arg = oa; }
  }
  float u[4];
  uniform4(seed, (uint64_t)b, counter ? (uint64_t)counter[0] : 0ull, u);
  if (u[0] <= eps[b]) arg = min((int)(u[1] * (float)T), T - 1);  // random candidate (model.py:331-333)
  if (lane == 0) act_idx[b] = arg;
  for (int d = lane; d < adim; d += 64) env_act[(size_t)b * adim + d] = a_mu[((size_t)b * T + arg) * adim + d];
}

void aql_candidate_q(const AQLNet& net, float* ws, const float* state, const float* a_mu, int B, float* q,
                     hipStream_t s) {
  if (B <= 0) return;
  const int n = (int)aql_workspace_floats();
  aql_noisy_eff_k<<<(n + 255) / 256, 256, 0, s>>>(net, ws);
  LAUNCH_CHECK();
  const int items = B * ((net.T + kAqGroup - 1) / kAqGroup);
  const int grid = std::min((items + 3) / 4, 512);
  aql_candidate_q_k<<<grid, 256, 0, s>>>(net, ws, state, a_mu, B, q);
  LAUNCH_CHECK();
}

void aql_noisy_eff(const AQLNet& net, float* ws, hipStream_t s) {
  const int n = (int)aql_workspace_floats();
  aql_noisy_eff_k<<<(n + 255) / 256, 256, 0, s>>>(net, ws);
  LAUNCH_CHECK();
}

void aql_propose(const AQLNet& net, const float* state, int B, const float* low, const float* high, const float* var,
                 uint64_t seed, const int64_t* counter, float* a_mu, float* mu_out, hipStream_t s, float* eff_ws) {
  if (B <= 0) return;
  if (net.na < 1 || net.na > 64) throw std::invalid_argument("aql_propose: 1 <= actions <= 64");
  if (net.obs < 1 || net.obs > 64) throw std::invalid_argument("aql_propose: 1 <= obs <= 64");
  if (!net.cont && net.uniform > net.na) throw std::invalid_argument("aql_propose: uniform > actions (discrete)");
  const int pb = (B + kPropStates - 1) / kPropStates;
  const int eb = eff_ws ? (int)((aql_workspace_floats() + 255) / 256) : 0;
  aql_propose_k<<<pb + eb, 256, 0, s>>>(net, state, B, low, high, var, seed, counter, a_mu, mu_out, eff_ws, pb);
  LAUNCH_CHECK();
}

void aql_select(const float* q, const float* a_mu, int B, int T, int adim, const float* eps, uint64_t seed,
                const int64_t* counter, int* act_idx, float* env_act, hipStream_t s) {
  if (B <= 0) return;
  aql_select_k<<<(B + 3) / 4, 256, 0, s>>>(q, a_mu, B, T, adim, eps, seed, counter, act_idx, env_act);
  LAUNCH_CHECK();
}

}  // namespace apex
