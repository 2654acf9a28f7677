// Fused double-DQN loss + dueling-heads backward + head weight-gradient partials (gfx950).
//
// Replaces three launches of the learner step (dqn_loss_k: one 512-thread workgroup,
// heads_bwd_k, heads_wgrad_partial_k) with ONE row-parallel launch: every loss quantity
// except two batch-wide reductions is row-local, so
//
//   * one wave per row computes a* = argmax Q(s'), y = r + gamma^n Q_t(s', a*)(1 - d),
//     delta = |y - Q(s, a)|, the PER-weighted Huber term and its gradient
//     g = w / B * clamp(Q(s,a) - y, -1, 1) (utils.py:64-81; dL/dQ is g at action a only);
//   * the same wave runs the heads backward for its row: dv = g, dadv = g (e_a - 1/A),
//     dz_j = g (W_adv2[a][j] - colsum_j / A) (j < 128), g W_val2[j] (j >= 128), masked by
//     the forward ReLU (h > 0), written as bf16 for the FC1 backward GEMMs;
//   * the workgroup (R rows) then forms its partial of every head/FC1-bias gradient --
//     the layout heads_wgrad_reduce_k / grad_finalize consume;
//   * the batch max of delta (priority mixing 0.9 max + 0.1 delta, utils.py:77) and the
//     loss mean are left to the priority-tree write (PrioMix), which runs on a forked
//     stream concurrently with the rest of the backward.
#include "common.h"
#include "kernels.h"

namespace apex {

namespace {
// rows per workgroup = waves per workgroup (one row per wave: each row is a chain of
// dependent loads (idx -> a, r, d; q rows), two rows per wave serialised them).  8 rows:
// B = 512 -> 64 workgroups (4 rows: 128 workgroups and twice the partials, measured slower).
constexpr int LH_MAXA = 63;
constexpr int kLhRows = 8;
}  // namespace

template <int LH_ROWS>
__global__ __launch_bounds__(64 * LH_ROWS) void dqn_heads_bwd_k(LossHeadsArgs p) {
  constexpr int LH_WAVES = LH_ROWS;
  static_assert(64 * LH_WAVES >= 256, "the partials take one column per thread of 256");
  __shared__ float colsum[128];
  __shared__ float gs[LH_ROWS];
  __shared__ int as[LH_ROWS];
  __shared__ float dzs[LH_ROWS][256];
  __shared__ float adv[LH_MAXA][128];
  __shared__ float wadv[LH_MAXA][128];  // W_adv2 (+ W_val2 below): the row's dz reads LDS, not
  __shared__ float wval[128];           // a global load that waited on the action load
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, t = threadIdx.x;
  const int B = p.B, A = p.A;
  const int r0 = blockIdx.x * LH_ROWS, nr = min(LH_ROWS, B - r0);
  if (blockIdx.x == 0 && t == 0 && p.step_snap) p.step_snap[0] = p.step[0];
  if (t < 128) {
    // 16 loads in flight per batch (the rolled loop waited out one L2 round trip per action:
    // ~18 of them before the first row could start), summed in action order
    float c = 0.f;
    wval[t] = p.w_val2[t];
    for (int a0 = 0; a0 < A; a0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p.w_adv2[min(a0 + u, A - 1) * 128 + t];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (a0 + u < A) {
          c += v[u];
          wadv[a0 + u][t] = v[u];
        }
    }
    colsum[t] = c;
  }
  for (int e = t; e < A * 128; e += 64 * LH_WAVES) adv[e / 128][e % 128] = 0.f;
  __syncthreads();
  const float gn = p.gamma_n;
  for (int rr = wave; rr < LH_ROWS; rr += LH_WAVES) {
    const int b = r0 + rr;
    if (rr >= nr) {  // wave-uniform
      if (lane == 0) {
        gs[rr] = 0.f;
        as[rr] = 0;
      }
      for (int k = 0; k < 4; ++k) dzs[rr][lane + 64 * k] = 0.f;
      continue;
    }
    const float* qr = p.q + (size_t)b * A;
    const float* q2r = p.q2 + (size_t)b * A;
    const float* q2tr = p.q2t + (size_t)b * A;
    const int row = p.idx ? p.idx[b] : b;  // (a, r, d) straight from the replay's transition table
    const int a = p.act[row];
    const float rw = p.rew[row], dn = p.done[row], wb = p.w[b];
    const float qv = lane < A ? qr[lane] : 0.f;
    const float q2tv = lane < A ? q2tr[lane] : 0.f;
    // argmax_a Q(s', a), ties -> lowest index (as the sequential scan of dqn_loss_k)
    float bv = lane < A ? q2r[lane] : -INFINITY;
    int bi = lane < A ? lane : 64;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    const float y = rw + gn * __shfl(q2tv, bi, 64) * (1.f - dn);
    const float qa = __shfl(qv, a, 64);
    const float delta = fabsf(y - qa);
    const float hub = delta < 1.f ? 0.5f * delta * delta : delta - 0.5f;
    const float g = wb / (float)B * fminf(fmaxf(qa - y, -1.f), 1.f);
    if (lane == 0) {
      p.delta[b] = delta;
      p.lw[b] = wb * hub;
      gs[rr] = g;
      as[rr] = a;
    }
    const float* hr = p.h + (size_t)b * 256;
    const float ga = g / (float)A;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = lane + 64 * k;
      float d = j < 128 ? g * wadv[a][j] - ga * colsum[j] : g * wval[j - 128];
      d = hr[j] > 0.f ? d : 0.f;
      dzs[rr][j] = d;
      if (p.dz) {
        p.dz[(size_t)b * 256 + j] = d;
      } else {
        p.dz_bf[(size_t)b * 256 + j] = f2bf(d);
      }
    }
  }
  __syncthreads();
  if (t >= 256) return;  // the partials below are one column per thread (no barriers follow)
  // workgroup partials: [A][128] dW_adv2, [128] dW_val2, [A] db_adv2, [1] db_val2, [256] db_fc1
  const int stride = (A + 1) * 128 + (A + 1) + 256;
  float* part = p.part + (size_t)blockIdx.x * stride;
  float S = 0.f, dsum = 0.f;
  float hvs[LH_ROWS];  // every row's h loaded before the (row-ordered) accumulation
#pragma unroll
  for (int r = 0; r < LH_ROWS; ++r) hvs[r] = p.h[(size_t)(r0 + min(r, nr - 1)) * 256 + t];
#pragma unroll
  for (int r = 0; r < LH_ROWS; ++r) {
    if (r >= nr) break;
    const float hv = hvs[r];
    S += gs[r] * hv;
    if (t < 128) adv[as[r]][t] += gs[r] * hv;  // column t is this thread's alone
    dsum += dzs[r][t];
  }
  if (t < 128) {
    const float sa = S / (float)A;
    for (int a = 0; a < A; ++a) part[a * 128 + t] = adv[a][t] - sa;
  } else {
    part[A * 128 + (t - 128)] = S;
  }
  if (t <= A) {
    float gsum = 0.f, ga = 0.f;
    for (int r = 0; r < nr; ++r) {
      gsum += gs[r];
      if (as[r] == t) ga += gs[r];
    }
    part[(A + 1) * 128 + t] = t < A ? ga - gsum / (float)A : gsum;
  }
  part[(A + 1) * 129 + t] = dsum;
}

int dqn_heads_bwd_blocks(int B) { return (B + kLhRows - 1) / kLhRows; }

void dqn_heads_bwd(const LossHeadsArgs& args, hipStream_t s) {
  if (args.A < 1 || args.A > LH_MAXA) throw std::invalid_argument("dqn_heads_bwd: 1 <= A <= 63");
  if (args.B <= 0) return;
  dqn_heads_bwd_k<kLhRows><<<dqn_heads_bwd_blocks(args.B), 64 * kLhRows, 0, s>>>(args);
  LAUNCH_CHECK();
}

}  // namespace apex
