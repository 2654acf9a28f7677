// GPU AQL engine kernels for gfx950 (BASELINE config 4).
//
// One learner step of AQL_dis (reference AQL_dis.py:63-108, utils.py:44-61,
// model.py:132-390) is five launches plus the shared replay / optimizer kernels:
//
//   per_sample -> aql_learn_fwd -> aql_learn_bwd -> per_write_leaves(mix) -> aql_grad
//              -> adam_step(critic) -> adam_step(proposal) -> aql_post
//
// * aql_learn_fwd: Q over every (state, candidate) pair of the batch for the three
//   evaluations of compute_loss_AQL -- online Q(s, .), online Q(s', .), target Q(s', .)
//   (the candidate set a_mu sampled at s_t is re-used for s', utils.py:44-49).  The action
//   encoder and the candidate half of advantage1 do not depend on the state, so the
//   online encodings are computed once for s and s'; the state half of advantage1
//   (W1[:, 64:] q_feature(s) + b1) is one 64-vector per state.  Workgroup = (net, sample,
//   16 candidates); 4 waves split the 64 output columns; both candidate GEMMs
//   (ao_h1[16x128] x ao_w2^T, ao_out[16x64] x W1a^T) run on v_mfma_f32_16x16x4_f32 with
//   the weights staged in LDS at bank-conflict-free pitches (132 / 68 floats: row n,
//   k-slot q -> bank 4n + q).  ao_h1 is generated in the A-operand registers (adim FMAs).
// * aql_learn_bwd: per sample -- the two argmaxes, the Double-Q TD target, Huber/IS
//   gradient, the forward recomputed for the ONE taken candidate (the critic loss only
//   reaches Q(s, a)), its backward to every layer input, and the proposal forward +
//   analytic log-prob/entropy gradient (MVN with fixed diagonal variance: the entropy is
//   constant; Categorical: the reference's [B,1] vs [B] broadcast, see below).  Writes
//   the per-sample vectors of aqlv:: -- no per-sample weight-gradient partials.
// * aql_grad: each parameter's gradient as a length-B contraction of those vectors
//   (NoisyLinear sigma = mu-gradient x epsilon), plus per-group sums of squares for the
//   two clip_grad_norm_(40) calls (critic / proposal are clipped separately).
// * aql_post: reset_noise() on the online and target critics (factorised Gaussian, Philox)
//   and the per-step proposal hard copy online -> target, then the step counter bump
//   (last-block ticket).
// * aql_env_reset / aql_env_step: vectorised GPU envs (BipedalWalker-shaped, CartPole,
//   Pendulum: envs/classic.py dynamics) that also insert the raw (s, a, r, s', d, a_mu)
//   transition into the replay ring (batchrecoder_AQL.py:48-51: no n-step, no actor
//   priorities; the slots go to per_write_leaves at max priority).
//
// Discrete proposal quirk kept from AQL_dis.py:84-86: the best candidate is reshaped to
// [B, 1] and scored by a Categorical of batch shape [B], so log_prob broadcasts to [B, B]
// and loss_p = mean_ij(-log pi_j(best_i)) - ent_lam * mean_j H_j.  Per sample j that is
// -(1/B) sum_k cnt_k log p_jk - ent_lam H_j with cnt_k = #{i : best_i = k}.
#include <algorithm>

#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "opt_dev.h"
#include "tree_dev.h"

namespace apex {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kH = 64, kCat = 128, kP132 = 132, kP68 = 68, kMaxAdim = 8;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float noisy_w(const float* mu, const float* sg, const float* ep, int i, int noisy) {
  const float m = mu[i];
  return noisy ? fmaf(sg[i], ep[i], m) : m;
}
__device__ __forceinline__ float relu(float x) { return fmaxf(x, 0.f); }
// a + sum_k w[k] v[k] over 64 columns, sequential fma order; w: one LDS row, v: a broadcast LDS
// vector, both 16-byte aligned.  Eight 16-byte loads of each are issued before their FMAs: with
// scalar loads the compiler re-used one register quad and waited out an LDS latency every
// 2-4 FMAs (~3k cycles per 64-term row)
__device__ __forceinline__ float lds_dot64(const float* w, const float* v, float a) {
#pragma unroll
  for (int c = 0; c < 64; c += 32) {
    f32x4 x[8], y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      x[i] = *reinterpret_cast<const f32x4*>(w + c + 4 * i);
      y[i] = *reinterpret_cast<const f32x4*>(v + c + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a = fmaf(x[i].x, y[i].x, a);
      a = fmaf(x[i].y, y[i].y, a);
      a = fmaf(x[i].z, y[i].z, a);
      a = fmaf(x[i].w, y[i].w, a);
    }
  }
  return a;
}
// phase timestamp (diagnostics): block 0, thread 0, after a barrier
#define AQL_STAMP(L, k)                                                   \
  do {                                                                    \
    if ((L).dbg && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) \
      (L).dbg[k] = (long long)clock64();                                  \
  } while (0)

// (value, index) argmax over a row of length T by one wave; ties -> lowest index
__device__ __forceinline__ int wave_argmax(const float* row, int T, int lane) {
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int t = lane; t < T; t += 64) {
    const float v = row[t];
    if (v > bv || (v == bv && t < bi)) { bv = v; bi = t; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  return bi == 0x7fffffff ? 0 : bi;
}

// ------------------------------------------------------------------ forward over candidates
// Effective NoisyLinear weights come precomputed (aql_post writes mu + sigma * eps after each
// update): the forward reads one array per layer instead of three.
constexpr int kEffB1 = kH * kCat, kEffW2 = kEffB1 + kH, kEffB2 = kEffW2 + kH;

// H = 2: 512 threads, the two halves take alternate candidate tiles of the item (2 waves per
// SIMD instead of 1: the tile's dependent MFMA chains overlap); the staging and the state MLP
// stay on the first half
template <int H>
__global__ __launch_bounds__(256 * H) void aql_learn_fwd_k(AqlLearn L) {
  __shared__ __attribute__((aligned(16))) float ao2[kH * kP132];  // action_out.2 weight [n][k]
  __shared__ __attribute__((aligned(16))) float w1[kH * kP132];   // advantage1 effective weight [n][k]
  // q_feature.0 [n][obs -> 64, zero-padded], .2 [n][k]: pitch 68 = 4 x odd, so the 16-byte row
  // reads of 16 lanes (one row each) cover all 64 banks
  __shared__ __attribute__((aligned(16))) float qw1[kH * kP68], qw2[kH * kP68];
  __shared__ float xt[H][16 * kP68];                               // ao_out tile [16 candidates][64]
  __shared__ __attribute__((aligned(16))) float ao1w[kCat * kMaxAdim];  // [k][8], zero-padded past adim
  __shared__ float ao1b[kCat], ao2b[kH], w2e[kH], b1e[kH], qb1[kH], qb2[kH];
  __shared__ __attribute__((aligned(16))) float sv[2][64], hq[2][kH], qf[2][kH];
  __shared__ float stp[2][kH];
  __shared__ float qpart[H][4][2][16];
  __shared__ int srow;
  if (L.gate && L.gate_j >= *L.gate) return;  // (grid-uniform) a gated-off step
  const bool tgt = blockIdx.y != 0;
  const AQLNet& N = tgt ? L.tg : L.on;
  const float* eff = tgt ? L.eff_tg : L.eff_on;
  const int T = N.T, RT = (T + 15) >> 4;
  const int nst = (tgt || L.act_mode) ? 1 : 2;  // online: {s, s'} (acting: {s}), target: {s'}
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, j = lane & 15, q = lane >> 4;
  const int half = H == 2 ? t >> 8 : 0, wl = wave & 3, t8 = t & 255;
  const int obs = N.obs, adim = N.adim, cont = N.cont;
  AQL_STAMP(L, 8);
  // the PER draw of sample b (fused sampling) by wave 0: identical in every workgroup of b (same
  // Philox stream); the (tile 0, online) workgroup also writes the slot and its IS weight
  auto draw = [&](int b, int rt) {
    const int64_t f = L.filled[0];
    const int length = (int)(f < (int64_t)L.tree.size[0] ? f : (int64_t)L.tree.size[0]);
    const bool wr = rt == 0 && !tgt;
    const float pmin = wr ? L.tree.node_min[L.tree.levels - 1][0] : 0.f, beta = wr ? L.beta[0] : 0.f;
    float p;
    const int node = tree_sample_leaf(L.tree, b, L.B, length, L.exclude_last, L.seed, (uint64_t)L.ctr[0], lane, &p);
    if (lane == 0) {
      srow = node;
      if (wr) {
        L.idx_out[b] = node;
        L.w_out[b] = (p > 0.f && pmin > 0.f && isfinite(pmin)) ? powf(p / pmin, -beta) : 1.f;
      }
    }
  };
  // (measured: drawing on wave 0 WHILE waves 1-3 stage the weights was slower than the two in
  // sequence -- 25.4k vs 18.0k cycles: the descent's dependent loads queue behind the staging
  // traffic in the CU's memory pipeline)
  if (t < 256) {  // stage every weight with ALL loads in flight before the first store (in separate groups,
     // each group's stores waited out its loads before the next group's loads issued: ~3 serial
     // global round trips): the two 64x128 matrices as 16-byte loads, q_feature.0 / .2 (clamped
     // column index: unconditional loads; .0's columns past obs stored as zeros), action_out.0
     // and the bias vectors
    const f32x4* a4 = reinterpret_cast<const f32x4*>(N.ao_w2);
    const f32x4* w4 = reinterpret_cast<const f32x4*>(eff);
    const int nao1 = cont ? kCat : kH;
    f32x4 va[8], vw[8];
    float x1[16], x2[16], y1[4];  // action_out.0: nao1 * adim <= 128 x 8
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (cont) va[k] = a4[t + 256 * k];
      vw[k] = w4[t + 256 * k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = t + 256 * k, r = e >> 6, i = e & 63;
      x1[k] = N.qf_w1[r * obs + min(i, obs - 1)];
      x2[k] = N.qf_w2[e];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) y1[k] = N.ao_w1[min(t + 256 * k, nao1 * adim - 1)];
    const float b_ao1 = N.ao_b1[min(t, nao1 - 1)], b_ao2 = cont ? N.ao_b2[t & 63] : 0.f;
    const float b_w2 = eff[kEffW2 + (t & 63)], b_b1 = eff[kEffB1 + (t & 63)];
    const float b_q1 = N.qf_b1[t & 63], b_q2 = N.qf_b2[t & 63];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e4 = t + 256 * k, r = e4 >> 5, c = (e4 & 31) * 4;
      if (cont) *reinterpret_cast<f32x4*>(&ao2[r * kP132 + c]) = va[k];
      *reinterpret_cast<f32x4*>(&w1[r * kP132 + c]) = vw[k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = t + 256 * k, r = e >> 6, i = e & 63;
      qw1[r * kP68 + i] = i < obs ? x1[k] : 0.f;
      qw2[r * kP68 + i] = x2[k];
    }
    // action_out.0 [n][adim] -> [n][8] zero-padded
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = t + 256 * k;
      if (e < nao1 * adim) ao1w[(e / adim) * kMaxAdim + e % adim] = y1[k];
    }
    for (int e = t; e < nao1 * (kMaxAdim - adim); e += 256) {
      const int r = e / (kMaxAdim - adim);
      ao1w[r * kMaxAdim + adim + (e - r * (kMaxAdim - adim))] = 0.f;
    }
    if (t < nao1) ao1b[t] = b_ao1;
    if (t < kH) {
      if (cont) ao2b[t] = b_ao2;
      w2e[t] = b_w2;
      b1e[t] = b_b1;
      qb1[t] = b_q1;
      qb2[t] = b_q2;
    }
  }
  // work items (sample b, group g of its candidate tiles: tiles [g RT / NG, (g + 1) RT / NG)): the
  // staged weights (~110 KB of LDS, one workgroup per CU), the PER draw and the state half serve
  // every tile of the group.  The acting launch (act_mode) runs a small grid that loops over the
  // items, so most CUs stay free for the learner's kernels running beside it
  const int NG = L.tile_groups > 0 ? min(L.tile_groups, RT) : RT;
  for (int item = blockIdx.x; item < L.B * NG; item += gridDim.x) {
  const int b = item / NG, g = item - b * NG, rt0 = g * RT / NG, rt1 = (g + 1) * RT / NG;
  __syncthreads();  // the staging / the previous item is done with sv / xt / stp / qpart / srow
  if (item == blockIdx.x) AQL_STAMP(L, 9);
  if (L.fused_sample) {
    if (wave == 0) draw(b, rt0);
    __syncthreads();
  }
  if (item == blockIdx.x) AQL_STAMP(L, 10);
  const int row = L.fused_sample ? srow : (L.idx ? L.idx[b] : b);
  if (t < 128) {
    const int si = t >> 6, i = t & 63;
    if (si < nst) sv[si][i] = i < obs ? ((tgt || si) ? L.st2 : L.st)[(size_t)row * obs + i] : 0.f;
  }
  __syncthreads();
  if (item == blockIdx.x) AQL_STAMP(L, 11);
  // continuous candidates: this lane's action row of a tile (clamped, unconditional loads; zeroed
  // past adim at use), loaded one tile ahead -- the first before the state MLP, so no tile waits
  // out a global round trip in front of its encoder
  float avn[kMaxAdim];
  auto load_av = [&](int rtx) {
    const float* am = L.amu + ((size_t)row * T + min(rtx * 16 + j, T - 1)) * adim;
#pragma unroll
    for (int d = 0; d < kMaxAdim; ++d) avn[d] = am[min(d, adim - 1)];
  };
  if (cont) load_av(rt0 + half);
  // state halves, from LDS: wave si < nst handles state si (q_feature MLP, W1[:, 64:] . qf + b1)
  if (wave < nst) {
    hq[wave][lane] = relu(lds_dot64(qw1 + lane * kP68, sv[wave], qb1[lane]));  // (zero past obs)
    __builtin_amdgcn_wave_barrier();
    qf[wave][lane] = relu(lds_dot64(qw2 + lane * kP68, hq[wave], qb2[lane]));
    __builtin_amdgcn_wave_barrier();
    stp[wave][lane] = lds_dot64(w1 + lane * kP132 + kH, qf[wave], b1e[lane]);
  }
  for (int rb = rt0; rb < rt1; rb += H) {
  const int rt = rb + half;
  const bool live = rt < rt1;  // wave-uniform (the barriers below are kept)
  float* xth = xt[half];
  // action encodings of candidates rt*16 .. +15: wave w computes columns 16w .. 16w+15
  const int n = 16 * wl + j;
  if (!live) {
  } else if (cont) {  // (tail rows recompute a valid candidate, discarded)
    float av[kMaxAdim];
#pragma unroll
    for (int d = 0; d < kMaxAdim; ++d) av[d] = d < adim ? avn[d] : 0.f;
    if (rt + H < rt1) load_av(rt + H);
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll 4
    for (int k0 = 0; k0 < kCat; k0 += 8) {
      float h0 = ao1b[k0 + q], h1 = ao1b[k0 + 4 + q];
      const f32x4* w0 = reinterpret_cast<const f32x4*>(&ao1w[(k0 + q) * kMaxAdim]);
      const f32x4* w1r = reinterpret_cast<const f32x4*>(&ao1w[(k0 + 4 + q) * kMaxAdim]);
      const f32x4 x0 = w0[0], x1 = w0[1], y0 = w1r[0], y1 = w1r[1];  // zero past adim (av too)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        h0 = fmaf(x0[d], av[d], h0);
        h1 = fmaf(y0[d], av[d], h1);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        h0 = fmaf(x1[d], av[4 + d], h0);
        h1 = fmaf(y1[d], av[4 + d], h1);
      }
      acc0 = mfma4(relu(h0), ao2[n * kP132 + k0 + q], acc0);
      acc1 = mfma4(relu(h1), ao2[n * kP132 + k0 + 4 + q], acc1);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) xth[(4 * q + i) * kP68 + n] = relu(acc0[i] + acc1[i] + ao2b[n]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = min(rt * 16 + 4 * q + i, T - 1);
      xth[(4 * q + i) * kP68 + n] = relu(fmaf(ao1w[n * kMaxAdim], L.amu[(size_t)row * T + r], ao1b[n]));
    }
  }
  __syncthreads();
  if (item == blockIdx.x) AQL_STAMP(L, 12);
  // advantage1 candidate half: pre[16][64] = ao_out . W1a^T; wave w -> columns 16w..16w+15
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
  for (int k0 = 0; k0 < kH; k0 += 8) {
    c0 = mfma4(xth[j * kP68 + k0 + q], w1[n * kP132 + k0 + q], c0);
    c1 = mfma4(xth[j * kP68 + k0 + 4 + q], w1[n * kP132 + k0 + 4 + q], c1);
  }
  for (int si = 0; si < (live ? nst : 0); ++si) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = w2e[n] * relu(c0[i] + c1[i] + stp[si][n]);
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (j == 0) qpart[half][wl][si][4 * q + i] = v;
    }
  }
  __syncthreads();
  if (item == blockIdx.x) AQL_STAMP(L, 13);
  if (live && t8 < 16 * nst) {
    const int m = t8 & 15, si = t8 >> 4, tt = rt * 16 + m;
    if (tt < T) {
      const float (*qp)[2][16] = qpart[half];
      const float qv = ((qp[0][si][m] + qp[1][si][m]) + (qp[2][si][m] + qp[3][si][m])) + eff[kEffB2];
      float* out = tgt ? L.qt_s2 : (si ? L.q_s2 : L.q_s);
      out[(size_t)b * T + tt] = qv;
    }
  }
  }  // tiles
  }  // work items
  AQL_STAMP(L, 14);
}

// ------------------------------------------------------------------ per-sample loss + backward
// sum_r W[r][k] g[r] for column k (one thread per column, R <= RMAX rows, all loads issued
// before the FMAs; each row is read coalesced across the threads)
template <int RMAX>
__device__ __forceinline__ float cols_dot(const float* __restrict__ W, int K, int R, const float* g, int k) {
  float w[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) w[r] = r < R ? W[(size_t)r * K + k] : 0.f;
  float a = 0.f;
#pragma unroll
  for (int r = 0; r < RMAX; ++r) a = r < R ? fmaf(w[r], g[r], a) : a;
  return a;
}

// sum_i W[r][i] v[i] for one row of n = 4*N4 inputs (16-byte aligned rows): all N4 16-byte
// loads of the row issued before the FMAs -- no cross-lane reduction (the ds_bpermute
// butterflies of a wave-per-row scheme serialise: 33 us for this phase)
template <int N4>
__device__ __forceinline__ float row_dot4(const float* __restrict__ W, int r, const float* v) {
  const f32x4* w = reinterpret_cast<const f32x4*>(W + (size_t)r * 4 * N4);
  f32x4 x[N4];
#pragma unroll
  for (int k = 0; k < N4; ++k) x[k] = w[k];
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int k = 0; k < N4; ++k) {
    a0 = fmaf(x[k].x, v[4 * k], a0);
    a1 = fmaf(x[k].y, v[4 * k + 1], a1);
    a0 = fmaf(x[k].z, v[4 * k + 2], a0);
    a1 = fmaf(x[k].w, v[4 * k + 3], a1);
  }
  return a0 + a1;
}

// row_dot4 on a row already in registers (same fma order)
template <int N4>
__device__ __forceinline__ float regs_dot4(const f32x4* x, const float* v) {
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int k = 0; k < N4; ++k) {
    a0 = fmaf(x[k].x, v[4 * k], a0);
    a1 = fmaf(x[k].y, v[4 * k + 1], a1);
    a0 = fmaf(x[k].z, v[4 * k + 2], a0);
    a1 = fmaf(x[k].w, v[4 * k + 3], a1);
  }
  return a0 + a1;
}

// small first-layer matrices (inputs obs / adim <= 64) from LDS: one thread per output row,
// rows zero-padded to n8 (a multiple of 8) so the dot product is branch-free and unrolled
__device__ __forceinline__ float lds_row_dot(const float* Wl, int n8, const float* v, float bias) {
  float a = bias;
  for (int i0 = 0; i0 < n8; i0 += 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a = fmaf(Wl[i0 + i], v[i0 + i], a);
  }
  return a;
}

// Double-Q TD target, Huber + IS weight (utils.py:50-60) of sample b: |td|, w * Huber and the
// loss gradient w.r.t. Q(s, a).  Shared by the backward and the fused step's tree workgroup.
struct AqlTd {
  float dl, lw, gq;
};
__device__ __forceinline__ AqlTd aql_td_vals(const AqlLearn& L, float qa, float qt, float r, float dn, float wb) {
  const float y = r + L.gamma_n * qt * (1.f - dn);
  const float diff = y - qa, dl = fabsf(diff);
  const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
  return AqlTd{dl, wb * (dl < 1.f ? 0.5f * dl * dl : dl - 0.5f), -sg * fminf(dl, 1.f) * wb / (float)L.B};
}
__device__ __forceinline__ AqlTd aql_td(const AqlLearn& L, int b, int row, int a_idx, int s_next) {
  const int T = L.on.T;
  return aql_td_vals(L, L.q_s[(size_t)b * T + a_idx], L.qt_s2[(size_t)b * T + s_next], L.rew[row], L.done[row],
                     L.w[b]);
}

// the backward of sample b by one workgroup (aql_learn_bwd_k) of NT = 256 or 512 threads.  The
// computing phases map thread tt < 256 to a row / column; with 512 threads the second half
// shares the staging that dominates the workgroup (the ~110 KB of layer weights it reads:
// 13k of ~30k cycles at 256 threads, profiles/r5_aql_engine.md): half the first-layer loads
// per thread and half of every prefetched second-layer row, whose two partial dot products
// are added through LDS.
template <int NT>
__device__ __forceinline__ void aql_bwd_block(const AqlLearn& L, int b) {
  static_assert(NT == 256 || NT == 512, "256 or 512 threads");
  constexpr int NH = NT / 256;  // thread halves
  __shared__ __attribute__((aligned(16))) float s_s[64];
  __shared__ float s_a[kMaxAdim], qfh[kH], aoh[kCat], x[kCat], pre[kH], gh[kH], gx[kCat];
  __shared__ float emb[kCat], hid[kCat], mu[64], gmu[64];
  __shared__ int cnt[64];
  __shared__ int s_best, s_next;
  __shared__ float s_gq;
  // first layers [row][in]: q_feature.0 / features.0 zero-padded to 64 columns at pitch 68 (16-byte
  // row reads, conflict-free), action_out.0 zero-padded to 8 at pitch 9
  __shared__ __attribute__((aligned(16))) float sw_qf1[kH * kP68], sw_f[kCat * kP68];
  __shared__ float sw_ao1[kCat * (kMaxAdim + 1)];
  __shared__ float red2[NH > 1 ? 256 : 1];  // the second half's partial second-layer dots
  const AQLNet& N = L.on;
  const float* eff = L.eff_on;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, tt = t & 255, hf = t >> 8;
  const int T = N.T, obs = N.obs, adim = N.adim, na = N.na, B = L.B, cont = N.cont;
  const int row = L.idx[b];
  const int a_idx = L.act[row];
  AQL_STAMP(L, 0);
  // the second-layer row this thread contracts later (q_feature.2 / action_out.2 /
  // dist_feature.0), prefetched now: its loads fly under the staging and the first layers
  // instead of opening a phase of their own
  const float* w2row = tt < kH ? N.qf_w2 + (size_t)tt * kH
                               : (tt < 2 * kH ? (cont ? N.ao_w2 + (size_t)(tt - kH) * kCat : nullptr)
                                              : N.df_w1 + (size_t)(tt - 2 * kH) * kCat);
  constexpr int XR = kCat / 4 / NH;  // 16-byte chunks of the (half) row per thread
  const int myN4 = (tt < kH ? kH / 4 : kCat / 4) / NH;
  f32x4 xr[XR];
  if (w2row) {
#pragma unroll
    for (int k = 0; k < XR; ++k)
      if (k < myN4) xr[k] = reinterpret_cast<const f32x4*>(w2row)[hf * myN4 + k];
  }
  const int pa = kMaxAdim + 1, nao1 = cont ? kCat : kH;
  {  // first layers, every load in flight before the stores (clamped column index:
     // unconditional loads; columns past obs / adim stored as zeros)
    float y1[16 / NH], y2[32 / NH], y3[4 / NH];
#pragma unroll
    for (int k = 0; k < 16 / NH; ++k) {
      const int e = t + NT * k, r = e >> 6, i = e & 63;
      y1[k] = N.qf_w1[r * obs + min(i, obs - 1)];
    }
#pragma unroll
    for (int k = 0; k < 32 / NH; ++k) {
      const int e = t + NT * k, r = e >> 6, i = e & 63;
      y2[k] = N.f_w[r * obs + min(i, obs - 1)];
    }
#pragma unroll
    for (int k = 0; k < 4 / NH; ++k) {
      const int e = t + NT * k, r = e >> 3, i = e & 7;
      y3[k] = N.ao_w1[min(r, nao1 - 1) * adim + min(i, adim - 1)];
    }
#pragma unroll
    for (int k = 0; k < 16 / NH; ++k) {
      const int e = t + NT * k, r = e >> 6, i = e & 63;
      sw_qf1[r * kP68 + i] = i < obs ? y1[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 32 / NH; ++k) {
      const int e = t + NT * k, r = e >> 6, i = e & 63;
      sw_f[r * kP68 + i] = i < obs ? y2[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4 / NH; ++k) {
      const int e = t + NT * k, r = e >> 3, i = e & 7;
      if (r < nao1) sw_ao1[r * pa + i] = i < adim ? y3[k] : 0.f;
    }
  }
  if (wave == 0) {
    const int bi = wave_argmax(L.q_s + (size_t)b * T, T, lane);
    if (lane == 0) s_best = bi;
  } else if (wave == 1) {
    const int bi = wave_argmax(L.q_s2 + (size_t)b * T, T, lane);
    if (lane == 0) s_next = bi;
  }
  if (t < 64) cnt[t] = 0;
  if (t < 64) s_s[t] = t < obs ? L.st[(size_t)row * obs + t] : 0.f;
  if (t < kMaxAdim) s_a[t] = t < adim ? L.amu[((size_t)row * T + a_idx) * adim + t] : 0.f;
  __syncthreads();
  AQL_STAMP(L, 1);
  if (!cont) {  // counts of every sample's best candidate (the [B, B] log-prob broadcast)
    for (int i = wave; i < B; i += NT / 64) {
      const int ri = L.idx[i];
      const int bi = wave_argmax(L.q_s + (size_t)i * T, T, lane);
      if (lane == 0) {
        const int k = (int)L.amu[(size_t)ri * T + bi];
        if (k >= 0 && k < 64) atomicAdd(&cnt[k], 1);
      }
    }
  }
  if (t == 0) {
    const AqlTd td = aql_td(L, b, row, a_idx, s_next);
    L.delta[b] = td.dl;
    L.lw[b] = td.lw;
    s_gq = td.gq;
  }
  // forward of the taken candidate (s, a_mu[a]) + the proposal trunk.  First layers from
  // the LDS-staged matrices (thread per row), then the 64/128-wide layers wave-per-row.
  if (hf == 0) {
    if (t < kH) {
      qfh[t] = relu(lds_dot64(sw_qf1 + t * kP68, s_s, N.qf_b1[t]));  // (zero past obs)
    } else if (t < kH + (cont ? kCat : kH)) {
      const int k = t - kH;
      aoh[k] = relu(lds_row_dot(sw_ao1 + k * pa, kMaxAdim, s_a, N.ao_b1[k]));
    }
    if (t >= 2 * kH) {
      const int k = t - 2 * kH;  // state embedding q.features (model.py:289-291)
      emb[k] = relu(lds_dot64(sw_f + k * kP68, s_s, N.f_b[k]));
    }
  }
  __syncthreads();
  AQL_STAMP(L, 2);
  if constexpr (NH == 1) {
    if (t < kH) {  // q_feature.2 (from the prefetched row)
      x[kH + t] = relu(regs_dot4<kH / 4>(xr, qfh) + N.qf_b2[t]);
    } else if (t < 2 * kH) {  // action_out.2 (continuous) / identity (discrete)
      const int nn = t - kH;
      x[nn] = cont ? relu(regs_dot4<kCat / 4>(xr, aoh) + N.ao_b2[nn]) : aoh[nn];
    } else {  // proposal dist_feature.0
      const int k = t - 2 * kH;
      hid[k] = relu(regs_dot4<kCat / 4>(xr, emb) + N.df_b1[k]);
    }
  } else {  // each half contracts its half of the row; the first half adds the second's
    float part = 0.f;
    if (tt < kH) part = regs_dot4<kH / 8>(xr, qfh + hf * (kH / 2));
    else if (tt < 2 * kH) part = cont ? regs_dot4<kCat / 8>(xr, aoh + hf * (kCat / 2)) : 0.f;
    else part = regs_dot4<kCat / 8>(xr, emb + hf * (kCat / 2));
    if (hf == 1) red2[tt] = part;
    __syncthreads();
    if (hf == 0) {
      const float a = part + red2[tt];
      if (tt < kH) {
        x[kH + tt] = relu(a + N.qf_b2[tt]);
      } else if (tt < 2 * kH) {
        const int nn = tt - kH;
        x[nn] = cont ? relu(a + N.ao_b2[nn]) : aoh[nn];
      } else {
        hid[tt - 2 * kH] = relu(a + N.df_b1[tt - 2 * kH]);
      }
    }
  }
  __syncthreads();
  AQL_STAMP(L, 3);
  if constexpr (NH == 1) {
    if (t < kH) {  // advantage1 pre-activation (effective noisy weight)
      pre[t] = row_dot4<kCat / 4>(eff, t, x) + eff[kEffB1 + t];
    } else if (t >= 2 * kH && t - 2 * kH < na) {  // proposal mean / logits
      const int d = t - 2 * kH;
      mu[d] = row_dot4<kCat / 4>(N.df_w2, d, hid) + N.df_b2[d];
    }
  } else {  // half rows, the partial dots added through LDS
    const float* wrow = nullptr;
    const float* vin = nullptr;
    if (tt < kH) {
      wrow = eff + (size_t)tt * kCat;
      vin = x;
    } else if (tt >= 2 * kH && tt - 2 * kH < na) {
      wrow = N.df_w2 + (size_t)(tt - 2 * kH) * kCat;
      vin = hid;
    }
    float part = 0.f;
    if (wrow) {
      f32x4 xw[kCat / 8];
#pragma unroll
      for (int k = 0; k < kCat / 8; ++k) xw[k] = reinterpret_cast<const f32x4*>(wrow + hf * (kCat / 2))[k];
      part = regs_dot4<kCat / 8>(xw, vin + hf * (kCat / 2));
    }
    if (hf == 1) red2[tt] = part;
    __syncthreads();
    if (hf == 0 && wrow) {
      const float a = part + red2[tt];
      if (tt < kH) pre[tt] = a + eff[kEffB1 + tt];
      else mu[tt - 2 * kH] = a + N.df_b2[tt - 2 * kH];
    }
  }
  __syncthreads();
  AQL_STAMP(L, 4);
  if (t < kH) {
    gh[t] = pre[t] > 0.f ? s_gq * eff[kEffW2 + t] : 0.f;
  } else if (wave == 3) {  // proposal loss gradient w.r.t. mu (analytic)
    float lp = 0.f;
    if (cont) {
      float d2 = 0.f, lv = 0.f;
      if (lane < na) {
        const float best = L.amu[((size_t)row * T + s_best) * adim + lane];
        const float var = L.var[lane], diff = best - mu[lane];
        gmu[lane] = -diff / var / (float)B;
        d2 = diff * diff / var;
        lv = logf(var);
      }
      d2 = wave_sum(d2);
      lv = wave_sum(lv);
      const float l2pi = 1.8378770664093453f;
      const float logp = -0.5f * (d2 + lv + (float)na * l2pi);
      const float ent = 0.5f * ((float)na * (1.f + l2pi) + lv);
      lp = -logp - L.ent_lam * ent;
    } else {
      const float m = lane < na ? mu[lane] : -INFINITY;
      const float mx = wave_max(m);
      const float ex = lane < na ? expf(m - mx) : 0.f;
      const float z = wave_sum(ex);
      const float logp = lane < na ? (m - mx) - logf(z) : 0.f;
      const float p = lane < na ? ex / z : 0.f;
      const float ent = -wave_sum(p * logp);
      const float c = lane < na ? (float)cnt[lane] / (float)B : 0.f;
      if (lane < na) gmu[lane] = ((p - c) + L.ent_lam * p * (logp + ent)) / (float)B;
      lp = -wave_sum(c * logp) - L.ent_lam * ent;
    }
    if (lane == 0) L.lossp[b] = lp;
  }
  __syncthreads();
  AQL_STAMP(L, 5);
  float* V = L.vec + (size_t)b * aqlv::STRIDE;
  // the column contractions over 64 rows: with two halves, rows 32 hf .. 32 hf + 31 each
  float c5 = 0.f;
  if (tt < kCat) {  // advantage1 input gradient
    c5 = NH == 1 ? cols_dot<kH>(eff, kCat, kH, gh, t)
                 : cols_dot<kH / 2>(eff + (size_t)hf * (kH / 2) * kCat, kCat, kH / 2, gh + hf * (kH / 2), tt);
  } else {  // proposal hidden gradient
    const int k = tt - kCat;
    c5 = NH == 1 ? cols_dot<64>(N.df_w2, kCat, na, gmu, k)
                 : cols_dot<32>(N.df_w2 + (size_t)hf * 32 * kCat, kCat, max(0, min(32, na - 32 * hf)), gmu + 32 * hf, k);
  }
  if (NH > 1) {
    if (hf == 1) red2[tt] = c5;
    __syncthreads();
    if (hf == 0) c5 += red2[tt];
  }
  if (hf == 0) {
    if (t < kCat) {
      gx[t] = x[t] > 0.f ? c5 : 0.f;
    } else {
      const int k = t - kCat;
      V[aqlv::GHID + k] = hid[k] > 0.f ? c5 : 0.f;
      V[aqlv::HID + k] = hid[k];
      V[aqlv::EMB + k] = emb[k];
    }
  }
  __syncthreads();
  AQL_STAMP(L, 6);
  float c6 = 0.f;
  if (tt < kCat) {  // action_out.0 input gradient
    if (cont)
      c6 = NH == 1 ? cols_dot<kH>(N.ao_w2, kCat, kH, gx, t)
                   : cols_dot<kH / 2>(N.ao_w2 + (size_t)hf * (kH / 2) * kCat, kCat, kH / 2, gx + hf * (kH / 2), tt);
  } else if (tt < kCat + kH) {  // q_feature.0 input gradient
    const int k = tt - kCat;
    c6 = NH == 1 ? cols_dot<kH>(N.qf_w2, kH, kH, gx + kH, k)
                 : cols_dot<kH / 2>(N.qf_w2 + (size_t)hf * (kH / 2) * kH, kH, kH / 2, gx + kH + hf * (kH / 2), k);
  }
  if (NH > 1) {
    if (hf == 1) red2[tt] = c6;
    __syncthreads();
    if (hf == 0) c6 += red2[tt];
  }
  if (hf == 1) {
  } else if (t < kCat) {
    if (cont) {
      V[aqlv::GAOH + t] = aoh[t] > 0.f ? c6 : 0.f;
      V[aqlv::AOH + t] = aoh[t];
    }
    V[aqlv::X + t] = x[t];
    V[aqlv::GX + t] = gx[t];
  } else if (t < kCat + kH) {
    const int k = t - kCat;
    const float a = c6;
    V[aqlv::GQFH + k] = qfh[k] > 0.f ? a : 0.f;
    V[aqlv::QFH + k] = qfh[k];
    V[aqlv::H + k] = relu(pre[k]);
    V[aqlv::GH + k] = gh[k];
  } else if (t < 256) {
    const int k = t - kCat - kH;
    if (k < na) V[aqlv::GMU + k] = gmu[k];
    if (k < obs) V[aqlv::S + k] = s_s[k];
    if (k < adim) V[aqlv::A + k] = s_a[k];
    if (k == 0) V[aqlv::GQ] = s_gq;
  }
  AQL_STAMP(L, 7);
}

// this step's priority write by one workgroup: the B TD terms recomputed from the forward's Q
// rows (aql_td: the formula the backward writes L.delta / L.lw with), then the batched tree
// write (leaves, mix, loss mean, every level).  Only the next step's sampler reads the tree.
__device__ __forceinline__ void td_tree_block(const AqlLearn& L, const TreeDesc& tree, BatchWrite w, int levels) {
  __shared__ float s_dl[64], s_lw[64], tred[16], s_r[64], s_dn[64], s_wb[64];
  __shared__ int sids[64], s_next[64], s_act[64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = (int)(blockDim.x >> 6), T = L.on.T, B = L.B;
  auto stamp = [&](int k) {  // diagnostics (APEX_AQL_DBG): tree-workgroup phase timestamps
    if (L.dbg && t == 0) L.dbg[16 + k] = (long long)clock64();
  };
  stamp(0);
  // the B TD terms with every sample's loads in flight together (a wave-per-sample loop paid ~4
  // dependent round trips per sample, ~29 us for 32 samples): the scalar chains idx -> act ->
  // Q(s, a) on one thread per sample, the argmaxes of Q(s', .) 4 samples per wave at a time
  const int tc = t - ((int)blockDim.x - 64);  // the last wave: its chain beside the others' argmaxes
  if (tc >= 0 && tc < B) {  // (Q(s, a) is loaded after the barrier, beside Q_tgt(s', argmax): one round trip)
    const int row = L.idx[tc];
    s_act[tc] = L.act[row];
    s_r[tc] = L.rew[row];
    s_dn[tc] = L.done[row];
    s_wb[tc] = L.w[tc];
  }
  if (T <= 256) {
    for (int b0 = wave * 4; b0 < B; b0 += 4 * nw) {  // wave-uniform
      float v[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* row = L.q_s2 + (size_t)min(b0 + j, B - 1) * T;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[j][k] = row[min(lane + 64 * k, T - 1)];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // ascending t per lane, as wave_argmax
          const int tt = lane + 64 * k;
          if (tt < T && (v[j][k] > bv || (v[j][k] == bv && tt < bi))) { bv = v[j][k]; bi = tt; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float ov = __shfl_xor(bv, o, 64);
          const int oi = __shfl_xor(bi, o, 64);
          if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (lane == 0 && b0 + j < B) s_next[b0 + j] = bi == 0x7fffffff ? 0 : bi;
      }
    }
  } else {
    for (int b = wave; b < B; b += nw) {
      const int sn = wave_argmax(L.q_s2 + (size_t)b * T, T, lane);
      if (lane == 0) s_next[b] = sn;
    }
  }
  __syncthreads();
  if (t < B) {
    const float qa = L.q_s[(size_t)t * T + s_act[t]], qt = L.qt_s2[(size_t)t * T + s_next[t]];
    const AqlTd td = aql_td_vals(L, qa, qt, s_r[t], s_dn[t], s_wb[t]);
    s_dl[t] = td.dl;
    s_lw[t] = td.lw;
  }
  __syncthreads();
  stamp(1);
  w.mix.delta = s_dl;
  w.mix.lw = s_lw;
  batch_leaves_block(tree, w, 0, tred, sids);
  stamp(2);
  if (levels > 0)  // levels 1..levels (dbg[24..29]: walk phases)
    update_levels_fast<8>(tree, sids, B, L.dbg ? L.dbg + 24 : nullptr, 1, levels);
  stamp(3);
}

template <int NT>
__global__ __launch_bounds__(NT) void aql_learn_bwd_k(AqlLearn L) {
  if (L.gate && L.gate_j >= *L.gate) return;  // (grid-uniform) a gated-off step
  if (L.bwd_tree && blockIdx.x == L.B) {  // block-uniform: the priority write (aql_learn_set_tree)
    td_tree_block(L, L.tree, L.bw, L.bwd_tree == 1 ? 1 << 30 : L.bwd_levels);
    return;
  }
  aql_bwd_block<NT>(L, blockIdx.x);
}

// ------------------------------------------------------------------ weight gradients
constexpr int kGradThreads = 256;

// the weight gradients of flat elements [bid * 256, +256) and the block's per-group sums of
// squares (aql_grad_k); returns the thread's gradient
// (a 512-thread launch: waves 4..7 of a gradient block hold no element -- they exist for the
// launch's level-walk workgroup -- and add zeros to nothing: the partials are bit-identical)
__device__ __forceinline__ float aql_grad_block(const AqlGrad& G, int bid, int nblk) {
  __shared__ double red[2][4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t i = t < kGradThreads ? (int64_t)bid * kGradThreads + t : G.n;
  float g = 0.f;
  int grp = -1;
  if (i < G.n) {
    int jb = 0;
    for (int k = 1; k < G.njobs; ++k)
      if (i >= G.job[k].off) jb = k;
    const AqlGradJob& J = G.job[jb];
    const int e = (int)(i - J.off), r = e / J.cols, c = e - r * J.cols;
    grp = J.group;
    if (!J.zero) {
      // the batch contraction in chunks of 32 samples, every load of a chunk in flight: the
      // loads are unconditional (clamped sample index, results selected after), a guarded
      // load compiled to a branch + wait each
      float acc = 0.f;
      const float* gp = G.vec + J.goff + r;
      const float* xp = G.vec + (J.xoff >= 0 ? J.xoff + c : 0);
      const bool hasx = J.xoff >= 0;
      for (int b0 = 0; b0 < G.B; b0 += 32) {
        float gv[32], xv[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
          const size_t bb = (size_t)min(b0 + k, G.B - 1) * aqlv::STRIDE;
          gv[k] = gp[bb];
          xv[k] = xp[bb];
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) {
          const bool ok = b0 + k < G.B;
          acc = fmaf(ok ? gv[k] : 0.f, (ok && hasx) ? xv[k] : 1.f, acc);
        }
      }
      g = J.eps ? acc * J.eps[e] : acc;
    }
    G.grad[i] = g;
  }
  double s0 = grp == 0 ? (double)g * (double)g : 0.0, s1 = grp == 1 ? (double)g * (double)g : 0.0;
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (lane == 0 && wave < 4) {
    red[0][wave] = s0;
    red[1][wave] = s1;
  }
  __syncthreads();
  if (t == 0) {
    G.part[bid] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    G.part[nblk + bid] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
  if (bid == 0 && wave == 1 && G.lossp_out) {
    float a = 0.f;
    for (int b = lane; b < G.B; b += 64) a += G.lossp[b];
    a = wave_sum(a);
    if (lane == 0) G.lossp_out[0] = a / (float)G.B;
  }
  return g;
}

// ------------------------------------------------------------------ noise reset + proposal copy
__device__ __forceinline__ float scaled_noise(uint64_t seed, int layer, int kind, int i, uint64_t ctr) {
  float u[4];
  uniform4(seed, ((uint64_t)layer << 40) | ((uint64_t)kind << 32) | (uint32_t)i, ctr, u);
  const float x = std_normal(u[0], u[1]);
  return copysignf(sqrtf(fabsf(x)), x);  // f(x) = sign(x) sqrt(|x|) (model.py:160-163)
}

// noise reset / effective weights / proposal copy for the elements of this block
__device__ __forceinline__ void aql_post_block(const AqlPost& P, int regen, uint64_t st) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const AqlNoise& z = P.layer[l];
    const int64_t nw = (int64_t)z.out * z.in;
    if (i >= 0 && i < nw) {
      const int o = (int)(i / z.in), c = (int)(i - (int64_t)o * z.in);
      float e = z.weps[i];
      if (regen) {
        e = scaled_noise(P.seed, l, 0, o, st) * scaled_noise(P.seed, l, 1, c, st);
        z.weps[i] = e;
      }
      z.weff[i] = fmaf(z.wsig[i], e, z.wmu[i]);
    } else if (i >= nw && i < nw + z.out) {
      const int o = (int)(i - nw);
      float e = z.beps[o];
      if (regen) {
        e = scaled_noise(P.seed, l, 2, o, st);
        z.beps[o] = e;
      }
      z.beff[o] = fmaf(z.bsig[o], e, z.bmu[o]);
    }
    i -= nw + z.out;
  }
  if (!regen) return;
  if (i >= 0 && i < P.n_copy) P.dst[i] = P.src[i];
}

// the step counter (Adam's bias correction, the noise stream) advances once all G workgroups are
// done with it.  No fence before the ticket: a workgroup's only obligation is to have READ the
// counter (consumed long before), and the new value reaches later launches at the kernel
// boundary -- an agent-scope release per workgroup wrote the XCD L2s back every step
__device__ __forceinline__ void step_ticket(const AqlPost& P, int G, uint64_t st) {
  const int t = threadIdx.x;
  __syncthreads();
  if (t == 0) {
    const int tk = atomicAdd(P.ticket, 1);
    if (tk == G - 1) {
      P.step[0] = (int64_t)st + 1;
      P.ticket[0] = 0;
    }
  }
}

__global__ __launch_bounds__(256) void aql_post_k(AqlPost P, int regen) {
  const uint64_t st = (uint64_t)P.step[0];
  aql_post_block(P, regen, st);
  if (!regen) return;
  step_ticket(P, (int)gridDim.x, st);
}

// ------------------------------------------------------------------ update launch helpers
__device__ __forceinline__ float noise_w(uint64_t seed, int l, int o, int c, uint64_t st) {
  return scaled_noise(seed, l, 0, o, st) * scaled_noise(seed, l, 1, c, st);
}

// element i of noisy layer l's [weights | biases]: fresh epsilon, effective weight from the
// layer's parameters as they are in memory (the target critic: not updated by this step)
__device__ __forceinline__ void noise_elem(const AqlNoise& z, int l, int64_t i, uint64_t seed, uint64_t st) {
  const int64_t nw = (int64_t)z.out * z.in;
  if (i < nw) {
    const int o = (int)(i / z.in), c = (int)(i - (int64_t)o * z.in);
    const float e = noise_w(seed, l, o, c, st);
    z.weps[i] = e;
    z.weff[i] = fmaf(z.wsig[i], e, z.wmu[i]);
  } else if (i < nw + z.out) {
    const int o = (int)(i - nw);
    const float e = scaled_noise(seed, l, 2, o, st);
    z.beps[o] = e;
    z.beff[o] = fmaf(z.bsig[o], e, z.bmu[o]);
  }
}

constexpr int kStepDrawBlocks = 8;  // update-launch workgroups of the next step's draw (4 waves each)

// the update of workgroup bid (< nblk: its parameter elements, thread gradient g): both clipped
// Adam steps, the online noise reset (the thread owning a sigma element also updates its mu
// partner, then draws the new epsilon and writes mu + sigma eps) and the proposal hard copy
// online -> target.
__device__ __forceinline__ void update_block(const AqlStep& D, int bid, float g, uint64_t st) {
  const int t = threadIdx.x;
  // this thread's element (and, for an online sigma, its mu partner): its parameter / moments /
  // partner gradient loaded and its new noise drawn BEFORE the grad-norm reduction (which
  // barriers), so their latency and the Philox work overlap the partials' round trip
  const int64_t i = (int64_t)bid * 256 + t;
  const bool live = bid < D.nblk && i < D.n;
  int kind = 0, l = 0;
  int64_t e = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // online noisy tensors: mu elements are updated by their sigma partner's thread
    const int64_t nw = (int64_t)D.P.layer[k].out * D.P.layer[k].in, nb = D.P.layer[k].out;
    if ((i >= D.mu_w[k] && i < D.mu_w[k] + nw) || (i >= D.mu_b[k] && i < D.mu_b[k] + nb)) kind = 1;
    if (i >= D.sig_w[k] && i < D.sig_w[k] + nw) { kind = 2; l = k; e = i - D.sig_w[k]; }
    if (i >= D.sig_b[k] && i < D.sig_b[k] + nb) { kind = 3; l = k; e = i - D.sig_b[k]; }
  }
  const bool upd = live && kind != 1;
  const int64_t ic = upd ? i : 0;
  float a = D.m[ic], b = D.v[ic], pv = D.p[ic];
  const int64_t im = kind >= 2 ? (kind == 2 ? D.mu_w[l] : D.mu_b[l]) + e : 0;
  float a2 = 0.f, b2 = 0.f, pm = 0.f, gm = 0.f, ep = 0.f;
  if (upd && kind >= 2) {
    a2 = D.m[im];
    b2 = D.v[im];
    pm = D.p[im];
    gm = D.G.grad[im];
    if (kind == 2) {
      const AqlNoise& z = D.P.layer[l];
      const int o = (int)(e / z.in), c = (int)(e - (int64_t)o * z.in);
      ep = noise_w(D.P.seed, l, o, c, st);
    } else {
      ep = scaled_noise(D.P.seed, l, 2, (int)e, st);
    }
  }
  float lr;
  const AdamRule rule = make_rule(D.hp, (int64_t)st, lr);
  const NormInfo nq = reduce_norms(D.G.part, D.nblk, D.hp.max_norm, D.hp.grad_scale);
  __syncthreads();  // reduce_norms' LDS is reused
  const NormInfo np = reduce_norms(D.G.part + D.nblk, D.nblk, D.hp.max_norm, D.hp.grad_scale);
  if (bid == 0 && t == 0) {
    const float mn = D.hp.max_norm;
    D.norms_q[0] = nq.l2;
    D.norms_q[2] = fminf(mn > 0.f ? mn / (nq.l2 + 1e-6f) : 1.f, 1.f);
    D.norms_q[3] = lr;
    D.norms_p[0] = np.l2;
    D.norms_p[2] = fminf(mn > 0.f ? mn / (np.l2 + 1e-6f) : 1.f, 1.f);
    D.norms_p[3] = lr;
  }
  if (!upd) return;
  const bool prop = i >= D.P_q;
  const float pn = rule(pv, opaque(g * (prop ? np.clip : nq.clip)), a, b);
  D.m[i] = a;
  D.v[i] = b;
  D.p[i] = pn;
  if (D.pub_p) D.pub_p[i] = pn;
  if (prop) D.P.dst[i - D.P_q] = pn;
  if (kind >= 2) {
    const AqlNoise& z = D.P.layer[l];
    const float mun = rule(pm, opaque(gm * nq.clip), a2, b2);
    D.m[im] = a2;
    D.v[im] = b2;
    D.p[im] = mun;
    if (D.pub_p) D.pub_p[im] = mun;
    if (kind == 2) {
      z.weps[e] = ep;
      if (D.pub_weps[l]) D.pub_weps[l][e] = ep;
      z.weff[e] = fmaf(pn, ep, mun);
    } else {
      z.beps[e] = ep;
      if (D.pub_beps[l]) D.pub_beps[l][e] = ep;
      z.beff[e] = fmaf(pn, ep, mun);
    }
  }
}

// the NEXT step's PER draw by draw workgroup k of kStepDrawBlocks (one wave per sample)
__device__ __forceinline__ void draw_block(const AqlStep& D, int k, uint64_t st) {
  const int t = threadIdx.x, B = D.L.B;
  if (D.draw && k >= 0 && k < kStepDrawBlocks) {  // block-uniform
    const int lane = t & 63;
    const TreeDesc& tr = D.tree;
    const int64_t f = D.filled[0];
    const int length = (int)(f < (int64_t)tr.size[0] ? f : (int64_t)tr.size[0]);
    const float pmin = tr.node_min[tr.levels - 1][0], beta = D.beta[0];
    for (int b = k * 4 + (t >> 6); b < B; b += 4 * kStepDrawBlocks) {  // wave-uniform
      float pr;
      const int node = tree_sample_leaf(tr, b, B, length, D.exclude_last, D.seed, st + 1, lane, &pr);
      if (lane == 0) {  // (as aql_learn_fwd_k's fused draw writes them)
        const_cast<int*>(D.L.idx)[b] = node;
        const_cast<float*>(D.L.w)[b] = (pr > 0.f && pmin > 0.f && isfinite(pmin)) ? powf(pr / pmin, -beta) : 1.f;
      }
    }
  }
}

// aql_grad_k: the gradient blocks, then (G.tree_leaves) one workgroup walking the priority
// tree's levels levels_lo.. of this step's dirty list -- the backward launch's tree workgroup
// wrote the leaves, the list and the lowest levels
// NT = 512: the level-walk workgroup runs 8 waves (update_levels_fast: 4 ancestors per wave per
// level instead of 8) -- that walk, not the gradient blocks, is the launch's critical path
// (profiles/r5_aql_engine.md: the walk takes the launch from 5.5 to 9.0 us)
template <int NT>
__global__ __launch_bounds__(NT) void aql_grad_k(AqlGrad G) {
  if (G.gate && G.gate_j >= *G.gate) return;  // (grid-uniform) a gated-off step
  if (G.step_snap && blockIdx.x == 0 && threadIdx.x == 0) *G.step_snap = *G.step_src;
  const int ng = (int)gridDim.x - (G.tree_leaves ? 1 : 0);
  if (G.tree_leaves && (int)blockIdx.x == ng) {  // block-uniform: the level walk
    __shared__ int sids[64];
    for (int i = threadIdx.x; i < G.bw.B; i += blockDim.x) sids[i] = G.bw.list[i];
    update_levels_fast<8>(G.tree, sids, G.bw.B, nullptr, max(G.levels_lo, 1));
    return;
  }
  aql_grad_block(G, blockIdx.x, ng);
}

// The step's update as its own launch after aql_grad_k (no grid barrier): blocks [0, nblk) the
// clipped Adam steps + online noise + proposal copy (update_block, gradients from G.grad), then
// the target critic's noise reset, then (AqlStep::draw) the next step's PER draw -- the tree is
// final (the backward launch's priority write, aql_learn_set_tree).  Replaces opt_step2_k +
// aql_post_k with the same arithmetic (bit-identical, tests/test_gpu_aql_engine.py).
int aql_update_noise_blocks(const AqlStep& d) {
  const int64_t n = (int64_t)d.P.layer[2].out * d.P.layer[2].in + d.P.layer[2].out +
                    (int64_t)d.P.layer[3].out * d.P.layer[3].in + d.P.layer[3].out;
  return (int)((n + 255) / 256);
}

__global__ __launch_bounds__(256) void aql_update_k(const AqlStep* __restrict__ Dp, int noise_blocks, int gate_j) {
  const AqlStep& D = *Dp;
  if (D.gate && gate_j >= *D.gate) return;  // (grid-uniform) a gated-off step
  const int bid = blockIdx.x, t = threadIdx.x;
  // the step from the gradient launch's copy when there is one (then block 0 bumps the counter:
  // no block of this launch reads it), else from the counter (bumped by the last block)
  const int64_t* snap = D.G.step_snap;
  const uint64_t st = (uint64_t)(snap ? snap[0] : D.P.step[0]);
  if (bid < D.nblk) {
    const int64_t i = (int64_t)bid * 256 + t;
    update_block(D, bid, i < D.n ? D.G.grad[i] : 0.f, st);
  } else if (bid < D.nblk + noise_blocks) {
    const int64_t n2 = (int64_t)D.P.layer[2].out * D.P.layer[2].in + D.P.layer[2].out;
    const int64_t n3 = (int64_t)D.P.layer[3].out * D.P.layer[3].in + D.P.layer[3].out;
    const int64_t i = (int64_t)(bid - D.nblk) * 256 + t;
    if (i < n2) noise_elem(D.P.layer[2], 2, i, D.P.seed, st);
    else if (i < n2 + n3) noise_elem(D.P.layer[3], 3, i - n2, D.P.seed, st);
  } else {
    draw_block(D, bid - D.nblk - noise_blocks, st);
  }
  if (!snap) step_ticket(D.P, (int)gridDim.x, st);
  else if (bid == 0 && t == 0) D.P.step[0] = (int64_t)st + 1;
}

// ------------------------------------------------------------------ vector envs
constexpr int kBwObs = 24, kBwAct = 4;

__device__ __forceinline__ float env_normal(uint64_t seed, int e, int i, int kind, uint64_t ctr) {
  float u[4];
  uniform4(seed, ((uint64_t)kind << 48) | ((uint64_t)(uint32_t)e << 8) | (uint32_t)i, ctr, u);
  return std_normal(u[0], u[1]);
}
__device__ __forceinline__ float env_uniform(uint64_t seed, int e, int i, int kind, uint64_t ctr) {
  float u[4];
  uniform4(seed, ((uint64_t)kind << 48) | ((uint64_t)(uint32_t)e << 8) | (uint32_t)i, ctr, u);
  return u[2];
}

// reset env e (one wave): new observation into obs_buf / phys
__device__ void env_reset_one(const AqlEnv& V, int e, int lane, uint64_t ctr) {
  float* o = V.obs_buf + (size_t)e * V.obs;
  if (V.kind == 0) {  // s ~ N(0, 0.1)
    if (lane < kBwObs) o[lane] = 0.1f * env_normal(V.seed, e, lane, 1, ctr);
  } else if (V.kind == 1) {  // CartPole: U(-0.05, 0.05)^4
    if (lane < 4) {
      const float v = -0.05f + 0.1f * env_uniform(V.seed, e, lane, 1, ctr);
      o[lane] = v;
      V.phys[(size_t)e * 4 + lane] = v;
    }
  } else {  // Pendulum: th ~ U(-pi, pi), thdot ~ U(-1, 1)
    const float th = -3.14159265f + 6.2831853f * env_uniform(V.seed, e, 0, 1, ctr);
    const float thd = -1.f + 2.f * env_uniform(V.seed, e, 1, 1, ctr);
    if (lane == 0) {
      V.phys[(size_t)e * 4] = th;
      V.phys[(size_t)e * 4 + 1] = thd;
      o[0] = cosf(th);
      o[1] = sinf(th);
      o[2] = thd;
    }
  }
  if (lane == 0) {
    V.ep_len[e] = 0;
    V.ep_ret[e] = 0.f;
  }
}

__global__ __launch_bounds__(256) void aql_env_reset_k(AqlEnv V) {
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= V.E) return;
  env_reset_one(V, e, threadIdx.x & 63, 0xFFFFFFFFull);
}

// One env's step by one wave: dynamics, reward, the raw transition into replay slot `slot`,
// episode bookkeeping / reset.  `a`: this env's action vector (adim floats; the discrete envs'
// action index as a float), `aidx`: its candidate index.
__device__ __forceinline__ void env_step_wave(const AqlEnv& V, int e, int lane, const float* a_in, int aidx,
                                              const float* __restrict__ amu, const AqlInsert& I, int64_t slot,
                                              uint64_t ctr) {
  const int obs = V.obs;
  const float* s = V.obs_buf + (size_t)e * obs;
  float s2 = 0.f, r = 0.f;
  bool term = false;
  if (V.kind == 0) {  // BipedalWalker-shaped (envs/classic.py BipedalWalkerShapedEnv.step)
    float a[kBwAct], pen = 0.f;
#pragma unroll
    for (int d = 0; d < kBwAct; ++d) {
      a[d] = fminf(fmaxf(a_in[d], -1.f), 1.f);
      pen += fabsf(a[d]);
    }
    if (lane < kBwObs) {
      float z = 0.01f * env_normal(V.seed, e, lane, 0, ctr);
      for (int k = 0; k < kBwObs; ++k) z = fmaf(V.dynA[lane * kBwObs + k], s[k], z);
#pragma unroll
      for (int d = 0; d < kBwAct; ++d) z = fmaf(V.dynB[lane * kBwAct + d], a[d], z);
      s2 = tanhf(z);
    }
    const float progress = 0.05f * wave_sum(lane < kBwObs ? V.dynw[lane] * s2 : 0.f);
    r = progress - 0.00035f * 80.f * pen;
    const float s0 = __shfl(s2, 0, 64);
    if (fabsf(s0) > 0.995f) {  // "hull touches ground"
      r = -100.f;
      term = true;
    }
  } else if (V.kind == 1) {  // CartPole (Barto et al. 1983; envs/classic.py CartPoleEnv)
    float* ph = V.phys + (size_t)e * 4;
    const float x = ph[0], xd = ph[1], th = ph[2], thd = ph[3];
    const float force = ((int)a_in[0] == 1) ? 10.f : -10.f;
    const float ct = cosf(th), sn = sinf(th);
    const float tmp = (force + 0.05f * thd * thd * sn) / 1.1f;
    const float tha = (9.8f * sn - ct * tmp) / (0.5f * (4.f / 3.f - 0.1f * ct * ct / 1.1f));
    const float xa = tmp - 0.05f * tha * ct / 1.1f;
    const float nv[4] = {x + 0.02f * xd, xd + 0.02f * xa, th + 0.02f * thd, thd + 0.02f * tha};
    if (lane < 4) s2 = nv[lane];
    r = 1.f;
    term = nv[0] < -2.4f || nv[0] > 2.4f || nv[2] < -0.20943951f || nv[2] > 0.20943951f;
    __builtin_amdgcn_wave_barrier();
    if (lane < 4) ph[lane] = nv[lane];
  } else {  // Pendulum (envs/classic.py PendulumEnv)
    float* ph = V.phys + (size_t)e * 4;
    const float th = ph[0], thd = ph[1];
    const float u = fminf(fmaxf(a_in[0], -2.f), 2.f);
    const float an = remainderf(th, 6.2831853f);  // normalised angle in [-pi, pi]
    const float cost = an * an + 0.1f * thd * thd + 0.001f * u * u;
    float nthd = thd + (-3.f * 10.f / 2.f * sinf(th + 3.14159265f) + 3.f * u) * 0.05f;
    const float nth = th + nthd * 0.05f;
    nthd = fminf(fmaxf(nthd, -8.f), 8.f);
    const float nv[3] = {cosf(nth), sinf(nth), nthd};
    if (lane < 3) s2 = nv[lane];
    r = -cost;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      ph[0] = nth;
      ph[1] = nthd;
    }
  }
  const int len = V.ep_len[e] + 1;
  const bool done = term || len >= V.max_steps;  // TimeLimit sets done (stored as terminal)
  // raw transition into the replay ring
  if (lane < obs) {
    I.st[slot * obs + lane] = s[lane];
    I.st2[slot * obs + lane] = s2;
  }
  const int TA = V.T * V.adim;
  for (int k = lane; k < TA; k += 64) I.amu[slot * TA + k] = amu[(size_t)e * TA + k];
  if (lane == 0) {
    I.act[slot] = aidx;
    I.rew[slot] = r;
    I.done[slot] = done ? 1.f : 0.f;
    I.slots[e] = (int)slot;
  }
  __builtin_amdgcn_wave_barrier();
  if (done) {
    if (lane == 0) {
      const int k = atomicAdd(V.ep_count, 1);
      float* lg = V.ep_log + (size_t)(k % V.log_cap) * 2;
      lg[0] = V.ep_ret[e] + r;
      lg[1] = (float)len;
    }
    __builtin_amdgcn_wave_barrier();
    env_reset_one(V, e, lane, ctr);
  } else {
    if (lane < obs) V.obs_buf[(size_t)e * obs + lane] = s2;
    if (lane == 0) {
      V.ep_len[e] = len;
      V.ep_ret[e] += r;
    }
  }
}

__global__ __launch_bounds__(256) void aql_env_step_k(AqlEnv V, const float* __restrict__ act,
                                                      const int* __restrict__ act_idx, const float* __restrict__ amu,
                                                      AqlInsert I) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= V.E) return;
  env_step_wave(V, e, lane, act + (size_t)e * V.adim, act_idx[e], amu, I, (I.filled[0] + e) % I.C,
                (uint64_t)V.counter[0]);
}

// The serial engine's acting tail in ONE launch (aql_act_tail): a wave per env picks its
// candidate (eps-greedy, aql_select_k's draw) and steps the env into its ring slot; one extra
// workgroup writes the E ring leaves at the max priority and walks their levels (the
// per_write_ring_fused_k write: it needs only the slots, (filled + e) mod C); the last
// workgroup to finish advances `filled` by E and the acting counter by 1 (every workgroup has
// read both by then) and writes the learner's PER beta for this iteration.  Replaces
// select + env step + ring write + the host's beta fill (4 launches).
__global__ __launch_bounds__(256) void aql_act_tail_k(AqlTail A) {
  const AqlEnv& V = A.V;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nenv = (V.E + 3) / 4;
  if ((int)blockIdx.x < nenv) {
    __shared__ float s_act[4][kMaxAdim];
    const int e = blockIdx.x * 4 + wave;
    if (e < V.E) {  // wave-uniform
      const uint64_t ctr = (uint64_t)A.counter[0];
      const int T = V.T, adim = V.adim;
      float best = -INFINITY;
      int arg = 0x7fffffff;
      for (int c = lane; c < T; c += 64) {
        const float v = A.q[(size_t)e * T + c];
        if (v > best || (v == best && c < arg)) { best = v; arg = c; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oa = __shfl_xor(arg, o, 64);
        if (ov > best || (ov == best && oa < arg)) { best = ov; arg = oa; }
      }
      float u[4];
      uniform4(A.sel_seed, (uint64_t)e, ctr, u);
      if (u[0] <= A.eps[e]) arg = min((int)(u[1] * (float)T), T - 1);  // random candidate (model.py:331-333)
      if (lane == 0) A.act_idx[e] = arg;
      if (lane < adim) {
        const float av = A.amu[((size_t)e * T + arg) * adim + lane];
        A.env_act[(size_t)e * adim + lane] = av;
        s_act[wave][lane] = av;
      }
      __builtin_amdgcn_wave_barrier();
      env_step_wave(V, e, lane, s_act[wave], arg, A.amu, A.I, (A.filled[0] + e) % A.I.C, ctr);
    }
  } else {
    __shared__ int sids[1024];
    __shared__ int comp[64];
    __shared__ int ncomp;
    const TreeDesc& tr = A.tree;
    const int64_t f = A.filled[0];
    const float p = *A.max_prio;
    for (int i = t; i < V.E; i += blockDim.x) {
      const int id = (int)((f + i) % A.I.C);
      sids[i] = id;
      if (id < tr.size[0]) write_leaf(tr, id, p, A.alpha);
    }
    if (t == 0) {
      ncomp = 0;
      if (A.beta_out) {  // AQL_dis.py:59 in the host's double arithmetic, then to fp32
#pragma clang fp contract(off)
        const double it = (double)A.iter[0];
        const double r = A.beta0 + it * A.beta_omb / A.beta_max_step * A.beta_workers;
        A.beta_out[0] = (float)(r < 1.0 ? r : 1.0);
      }
    }
    __syncthreads();
    for (int i = t; i < V.E; i += blockDim.x) {  // one slot per distinct level-1 node (ring order)
      const int id = sids[i];
      if (id >= tr.size[0]) continue;
      const int prev = i > 0 ? sids[i - 1] : -1;
      if (prev >= 0 && prev < tr.size[0] && (prev >> kTreeLog2Fanout) == (id >> kTreeLog2Fanout)) continue;
      const int k = atomicAdd(&ncomp, 1);
      if (k < 64) comp[k] = id;
    }
    __syncthreads();
    if (ncomp <= 64) update_levels_fast<4>(tr, comp, ncomp);
    else update_levels_block(tr, sids, V.E, 1, tr.levels);
  }
  __syncthreads();
  if (t == 0) {
    __threadfence();
    if (atomicAdd(A.ticket, 1) == (int)gridDim.x - 1) {  // the last workgroup: every read of the counters is done
      A.filled[0] += V.E;
      A.counter[0] += 1;
      if (A.iter) A.iter[0] += 1;
      A.ticket[0] = 0;
    }
  }
}

// staged transitions (rows 0..E-1 of src, written by the acting stream) -> replay ring slots
// (dst.filled + e) % dst.C, slot list into dst.slots; the learner's stream applies them before
// its priority-tree write, so the acting step never touches a table the learner reads
__global__ __launch_bounds__(256) void aql_apply_staged_k(AqlInsert src, AqlInsert dst, int E, int obs, int TA) {
  const int lane = threadIdx.x & 63, e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= E) return;
  const int64_t slot = (dst.filled[0] + e) % dst.C;
  if (lane < obs) {
    dst.st[slot * obs + lane] = src.st[(size_t)e * obs + lane];
    dst.st2[slot * obs + lane] = src.st2[(size_t)e * obs + lane];
  }
  for (int k = lane; k < TA; k += 64) dst.amu[slot * TA + k] = src.amu[(size_t)e * TA + k];
  if (lane == 0) {
    dst.act[slot] = src.act[e];
    dst.rew[slot] = src.rew[e];
    dst.done[slot] = src.done[e];
    dst.slots[e] = (int)slot;
  }
}

}  // namespace

// ------------------------------------------------------------------ launchers
static void check_net(const AQLNet& n) {
  if (n.obs < 1 || n.obs > 64) throw std::invalid_argument("aql learner: 1 <= obs <= 64");
  if (n.adim < 1 || n.adim > kMaxAdim) throw std::invalid_argument("aql learner: 1 <= action dim <= 8");
  if (n.T < 1 || n.T > 4096) throw std::invalid_argument("aql learner: 1 <= candidates <= 4096");
  if (n.na < 1 || n.na > 64) throw std::invalid_argument("aql learner: 1 <= proposal outputs <= 64");
  if (!n.f_w || !n.df_w1 || !n.df_w2 || (n.cont && !n.ao_w2)) throw std::invalid_argument("aql learner: weights");
}

static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return cus;
}

void aql_learn_fwd(const AqlLearn& L, hipStream_t s) {
  check_net(L.on);
  if (!L.eff_on || !L.eff_tg) throw std::invalid_argument("aql learner: effective-weight workspaces");
  for (const float* w : {L.on.qf_w2, L.on.ao_w2, L.on.df_w1, L.on.df_w2})
    if (w && (reinterpret_cast<uintptr_t>(w) & 15))
      throw std::invalid_argument("aql learner: weight matrices must be 16-byte aligned (flatten with align=4)");
  if (((reinterpret_cast<uintptr_t>(L.eff_on) | reinterpret_cast<uintptr_t>(L.eff_tg) |
        reinterpret_cast<uintptr_t>(L.on.ao_w2) | reinterpret_cast<uintptr_t>(L.tg.ao_w2)) & 15))
    throw std::invalid_argument("aql learner: action_out.2 weights / workspaces must be 16-byte aligned");
  if (L.tg.T != L.on.T || L.tg.cont != L.on.cont || L.tg.obs != L.on.obs || L.tg.adim != L.on.adim)
    throw std::invalid_argument("aql learner: online / target shapes differ");
  if (L.B < 1) return;
  const int RT = (L.on.T + 15) / 16;
  AqlLearn Lk = L;
  if (Lk.tile_groups <= 0)  // about one workgroup per CU for the two nets (LDS: one per CU)
    Lk.tile_groups = std::max(1, std::min(RT, device_cus() / (2 * L.B)));
  Lk.tile_groups = std::min(Lk.tile_groups, RT);
  if (Lk.fwd_halves == 1) aql_learn_fwd_k<1><<<dim3(L.B * Lk.tile_groups, 2), 256, 0, s>>>(Lk);
  else aql_learn_fwd_k<2><<<dim3(L.B * Lk.tile_groups, 2), 512, 0, s>>>(Lk);
  LAUNCH_CHECK();
}

void aql_act_q(const AqlLearn& L, hipStream_t s) {
  check_net(L.on);
  if (!L.act_mode || !L.eff_on || !L.st || !L.amu || !L.q_s) throw std::invalid_argument("aql_act_q: acting config");
  if (((reinterpret_cast<uintptr_t>(L.eff_on) | reinterpret_cast<uintptr_t>(L.on.ao_w2) |
        reinterpret_cast<uintptr_t>(L.on.qf_w2)) & 15))
    throw std::invalid_argument("aql_act_q: weights / workspace must be 16-byte aligned");
  if (L.B < 1) return;
  const int RT = (L.on.T + 15) / 16;
  AqlLearn Lk = L;
  // tile groups as the learner's (one weight staging per group of a state's tiles: one
  // workgroup per (state, tile) staged the ~110 KB of weights 3328 times for 256 envs, 37.8 us)
  if (Lk.tile_groups <= 0) Lk.tile_groups = std::max(1, std::min(RT, device_cus() / L.B));
  Lk.tile_groups = std::min(Lk.tile_groups, RT);
  const int items = L.B * Lk.tile_groups;
  const int blocks = std::max(1, std::min(items, L.act_blocks > 0 ? L.act_blocks : items));
  aql_learn_fwd_k<2><<<dim3(blocks, 1), 512, 0, s>>>(Lk);  // grid.y = 1: the online net only
  LAUNCH_CHECK();
}

// 512 threads per backward workgroup: bench.py --algo aql 19648 -> 20857 SGD steps/s (two
// alternated processes each, one box; profiles/r6_aql.md)
constexpr int kAqlBwdThreadsDefault = 512;

void aql_learn_bwd(const AqlLearn& L, hipStream_t s) {
  check_net(L.on);
  if (L.B < 1) return;
  if (L.bwd_tree && (L.B > 64 || L.bw.B != L.B || L.bw.E != 0 || !L.bw.idx || !L.bw.list || !L.bw.owner ||
                     !L.bw.max_prio || !L.act || !L.idx))
    throw std::invalid_argument("aql_learn_bwd: the priority write needs B <= 64 and every pointer");
  // APEX_AQL_BWD_THREADS = 256 | 512: one or two thread halves per sample workgroup (and per tree
  // workgroup)
  static const int nt = [] {
    const char* e = std::getenv("APEX_AQL_BWD_THREADS");
    return e ? (std::atoi(e) == 256 ? 256 : 512) : kAqlBwdThreadsDefault;
  }();
  if (nt == 512) aql_learn_bwd_k<512><<<L.B + (L.bwd_tree ? 1 : 0), 512, 0, s>>>(L);
  else aql_learn_bwd_k<256><<<L.B + (L.bwd_tree ? 1 : 0), 256, 0, s>>>(L);
  LAUNCH_CHECK();
}

int aql_grad_blocks(int64_t n) { return (int)((n + kGradThreads - 1) / kGradThreads); }

// 512 threads per gradient workgroup (the level-walk workgroup's extra halves; the gradient rows
// keep 256): 20843 -> 21726 SGD steps/s (profiles/r6_aql.md)
constexpr int kAqlGradThreadsDefault = 512;

void aql_grad(const AqlGrad& g, hipStream_t s) {
  if (g.njobs < 1 || g.njobs > kAqlMaxJobs || g.job[0].off != 0) throw std::invalid_argument("aql_grad: jobs");
  for (int k = 0; k < g.njobs; ++k) {
    const AqlGradJob& J = g.job[k];
    const int64_t end = k + 1 < g.njobs ? g.job[k + 1].off : g.n;
    if (J.off + (int64_t)J.rows * J.cols != end) throw std::invalid_argument("aql_grad: jobs must tile [0, n)");
    if (J.goff < 0 || J.goff + J.rows > aqlv::STRIDE || J.xoff + J.cols > aqlv::STRIDE)
      throw std::invalid_argument("aql_grad: vector offsets");
  }
  if (g.tree_leaves && (g.bw.B < 1 || g.bw.B > 64 || !g.bw.list))
    throw std::invalid_argument("aql_grad: the level walk takes a list of 1..64 learner rows");
  static const int nt = [] {  // APEX_AQL_GRAD_THREADS = 256 | 512
    const char* e = std::getenv("APEX_AQL_GRAD_THREADS");
    return e ? (std::atoi(e) == 512 ? 512 : 256) : kAqlGradThreadsDefault;
  }();
  if (nt == 512) aql_grad_k<512><<<aql_grad_blocks(g.n) + (g.tree_leaves ? 1 : 0), 512, 0, s>>>(g);
  else aql_grad_k<256><<<aql_grad_blocks(g.n) + (g.tree_leaves ? 1 : 0), 256, 0, s>>>(g);
  LAUNCH_CHECK();
}

void aql_post(const AqlPost& p, int regen, hipStream_t s) {
  int64_t n = regen ? p.n_copy : 0;
  for (int l = 0; l < 4; ++l) n += (int64_t)p.layer[l].out * p.layer[l].in + p.layer[l].out;
  aql_post_k<<<(int)((n + 255) / 256), 256, 0, s>>>(p, regen);
  LAUNCH_CHECK();
}

void aql_step_check(const AqlStep& d) {
  check_net(d.L.on);
  const AqlGrad& G = d.G;
  if (d.nblk != aql_grad_blocks(G.n) || d.n != G.n)
    throw std::invalid_argument("aql_step: gradient blocks / parameter count");
  if (d.P_q <= 0 || d.P_q > d.n || !d.p || !d.m || !d.v || !d.norms_q || !d.norms_p || !G.grad || !G.part)
    throw std::invalid_argument("aql_step: optimizer tensors");
  if (!d.P.step || !d.P.ticket || !d.P.dst || d.P.n_copy != d.n - d.P_q)
    throw std::invalid_argument("aql_step: counter / proposal copy");
  if (d.draw && (!d.filled || !d.beta || !d.L.idx || !d.L.w))
    throw std::invalid_argument("aql_step: the next step's draw needs filled / beta / idx / w");
  for (int k = 0; k < 2; ++k) {
    const int64_t nw = (int64_t)d.P.layer[k].out * d.P.layer[k].in, nb = d.P.layer[k].out;
    for (int64_t o : {d.mu_w[k], d.sig_w[k]})
      if (o < 0 || o + nw > d.P_q) throw std::invalid_argument("aql_step: online noisy weights outside the critic");
    for (int64_t o : {d.mu_b[k], d.sig_b[k]})
      if (o < 0 || o + nb > d.P_q) throw std::invalid_argument("aql_step: online noisy biases outside the critic");
  }
}

int aql_update_grid(const AqlStep& d, int* noise_blocks) {
  const int nb = aql_update_noise_blocks(d);
  if (noise_blocks) *noise_blocks = nb;
  return d.nblk + nb + (d.draw ? kStepDrawBlocks : 0);
}

void aql_update(const AqlStep* dev, int grid, int noise_blocks, hipStream_t s, int gate_j) {
  aql_update_k<<<grid, 256, 0, s>>>(dev, noise_blocks, gate_j);
  LAUNCH_CHECK();
}

void aql_env_reset(const AqlEnv& e, hipStream_t s) {
  if (e.kind < 0 || e.kind > 2) throw std::invalid_argument("aql env: kind 0 (bipedal) / 1 (cartpole) / 2 (pendulum)");
  if (e.E < 1) return;
  aql_env_reset_k<<<(e.E + 3) / 4, 256, 0, s>>>(e);
  LAUNCH_CHECK();
}

void aql_env_step(const AqlEnv& e, const float* env_act, const int* act_idx, const float* amu, const AqlInsert& ins,
                  hipStream_t s) {
  static const int obs_of[3] = {kBwObs, 4, 3}, adim_of[3] = {kBwAct, 1, 1};
  if (e.kind < 0 || e.kind > 2) throw std::invalid_argument("aql env: kind");
  if (e.obs != obs_of[e.kind] || e.adim != adim_of[e.kind]) throw std::invalid_argument("aql env: obs/action dims");
  if (ins.C < e.E) throw std::invalid_argument("aql env: replay capacity < envs");
  if (e.E < 1) return;
  aql_env_step_k<<<(e.E + 3) / 4, 256, 0, s>>>(e, env_act, act_idx, amu, ins);
  LAUNCH_CHECK();
}

void aql_act_tail(const AqlTail& a, hipStream_t s) {
  static const int obs_of[3] = {kBwObs, 4, 3}, adim_of[3] = {kBwAct, 1, 1};
  const AqlEnv& e = a.V;
  if (e.kind < 0 || e.kind > 2) throw std::invalid_argument("aql env: kind");
  if (e.obs != obs_of[e.kind] || e.adim != adim_of[e.kind]) throw std::invalid_argument("aql env: obs/action dims");
  if (a.I.C < e.E) throw std::invalid_argument("aql env: replay capacity < envs");
  if (e.E > 1024) throw std::invalid_argument("aql_act_tail: at most 1024 envs (one tree workgroup)");
  if (e.adim > kMaxAdim) throw std::invalid_argument("aql_act_tail: action dim");
  if (a.I.C > ((int64_t)1 << 31) || a.tree.size[0] < a.I.C)
    throw std::invalid_argument("aql_act_tail: the tree must cover the ring");
  if (!a.q || !a.amu || !a.eps || !a.act_idx || !a.env_act || !a.max_prio || !a.filled || !a.counter || !a.ticket ||
      (a.beta_out && !a.iter))
    throw std::invalid_argument("aql_act_tail: missing buffers");
  if (e.E < 1) return;
  aql_act_tail_k<<<(e.E + 3) / 4 + 1, 256, 0, s>>>(a);
  LAUNCH_CHECK();
}

void aql_apply_staged(const AqlInsert& src, const AqlInsert& dst, int E, int obs, int TA, hipStream_t s) {
  if (E <= 0) return;
  if (obs < 1 || obs > 64 || TA < 1) throw std::invalid_argument("aql_apply_staged: 1 <= obs <= 64, T * adim >= 1");
  if (!src.st || !src.st2 || !src.amu || !src.act || !src.rew || !src.done || !dst.st || !dst.st2 || !dst.amu ||
      !dst.act || !dst.rew || !dst.done || !dst.filled || !dst.slots || dst.C < E)
    throw std::invalid_argument("aql_apply_staged: tables");
  aql_apply_staged_k<<<(E + 3) / 4, 256, 0, s>>>(src, dst, E, obs, TA);
  LAUNCH_CHECK();
}

}  // namespace apex
