// Actor-shard kernels for gfx950: vectorised synthetic Atari env, on-device
// epsilon-greedy, and the n-step batcher with actor-computed priorities
// (reference memory.py:393-478, origin_repo/actor.py:52-115).
//
// The reference runs one env + one B=1 CPU forward per actor process and ships
// pickled 50-transition chunks over TCP.  Here an actor shard is E envs on one GPU:
// the env renders 84x84 u8 frames straight into the HBM frame ring, the Q-network
// runs once for all E envs, actions are drawn on device with a per-env epsilon, and
// the n-step kernel writes transitions + initial priorities directly into the replay
// (slot = (step*E + e) mod C, so a transition's lifetime is exactly C/E steps and the
// frame ring (F >= C + (2n+8)E) always outlives the transitions that reference it).
#include "common.h"
#include "kernels.h"

namespace apex {

// ------------------------------------------------------------------ env state layout
enum : int {
  S_PX = 0, S_PY = 1, S_EX = 2, S_EY = 8, S_EVX = 14, S_BX = 20, S_BY = 21, S_BACT = 22, S_LIVES = 23,
  S_T = 24, S_EPRET = 25, S_EPLEN = 26, S_POINTS = 27, S_STRIDE = 32
};
constexpr int kEnemies = 6;
constexpr int kLives = 3;
constexpr int kScreen = 84;

// action -> (dx, dy, fire) using the ALE full action-meaning order
// NOOP FIRE UP RIGHT LEFT DOWN UPRIGHT UPLEFT DOWNRIGHT DOWNLEFT UPFIRE RIGHTFIRE LEFTFIRE
// DOWNFIRE UPRIGHTFIRE UPLEFTFIRE DOWNRIGHTFIRE DOWNLEFTFIRE; minimal sets (Pong: 6) map
// onto NOOP FIRE RIGHT LEFT RIGHTFIRE LEFTFIRE.
__device__ __forceinline__ void decode_action(int a, int n_actions, int& dx, int& dy, int& fire) {
  if (n_actions == 18) {
    const signed char DX[18] = {0, 0, 0, 1, -1, 0, 1, -1, 1, -1, 0, 1, -1, 0, 1, -1, 1, -1};
    const signed char DY[18] = {0, 0, -1, 0, 0, 1, -1, -1, 1, 1, -1, 0, 0, 1, -1, -1, 1, 1};
    const signed char FI[18] = {0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1};
    dx = DX[a]; dy = DY[a]; fire = FI[a];
  } else {
    const signed char DX[6] = {0, 0, 1, -1, 1, -1};
    const signed char FI[6] = {0, 1, 0, 0, 1, 1};
    const int k = a < 6 ? a : a % 6;
    dx = DX[k]; dy = 0; fire = FI[k];
  }
}

__device__ __forceinline__ void env_reset_state(float* st, uint64_t seed, int e, uint64_t ctr) {
  float u[4];
  st[S_PX] = 40.f;
  st[S_PY] = 70.f;
#pragma unroll
  for (int k = 0; k < kEnemies; ++k) {
    uniform4(seed, (uint64_t)e * 64 + 32 + k, ctr, u);
    st[S_EX + k] = 4.f + 72.f * u[0];
    st[S_EY + k] = 8.f + 6.f * k;
    st[S_EVX + k] = (u[1] < 0.5f ? -1.f : 1.f) * (0.4f + 0.8f * u[2]);
  }
  st[S_BX] = 0.f; st[S_BY] = 0.f; st[S_BACT] = 0.f;
  st[S_LIVES] = (float)kLives;
  st[S_T] = 0.f;
  st[S_POINTS] = 0.f;
}

// One workgroup renders one env's 84x84 frame (thread 0 has already updated the state).
__device__ void render_frame(const float* st, uint8_t* dst) {
  __shared__ int rect[(kEnemies + 2) * 4];
  __shared__ int val[kEnemies + 2];
  if (threadIdx.x == 0) {
    rect[0] = (int)st[S_PY]; rect[1] = (int)st[S_PY] + 4; rect[2] = (int)st[S_PX]; rect[3] = (int)st[S_PX] + 4;
    val[0] = 200;
    for (int k = 0; k < kEnemies; ++k) {
      rect[4 + 4 * k] = (int)st[S_EY + k]; rect[5 + 4 * k] = (int)st[S_EY + k] + 3;
      rect[6 + 4 * k] = (int)st[S_EX + k]; rect[7 + 4 * k] = (int)st[S_EX + k] + 6;
      val[1 + k] = (k & 1) ? 150 : 110;
    }
    const int ba = st[S_BACT] > 0.5f;
    rect[4 + 4 * kEnemies] = ba ? (int)st[S_BY] : -10; rect[5 + 4 * kEnemies] = ba ? (int)st[S_BY] + 2 : -10;
    rect[6 + 4 * kEnemies] = (int)st[S_BX]; rect[7 + 4 * kEnemies] = (int)st[S_BX] + 1;
    val[1 + kEnemies] = 255;
  }
  __syncthreads();
  uint32_t* out = reinterpret_cast<uint32_t*>(dst);
  for (int w = threadIdx.x; w < kScreen * kScreen / 4; w += blockDim.x) {
    const int y = (w * 4) / kScreen, x0 = (w * 4) % kScreen;
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = x0 + j;
      int v = y < 5 ? 40 : (y >= 80 ? 90 : 20);
#pragma unroll
      for (int r = 0; r < kEnemies + 2; ++r)
        if (y >= rect[4 * r] && y < rect[4 * r + 1] && x >= rect[4 * r + 2] && x < rect[4 * r + 3]) v = val[r];
      packed |= (uint32_t)v << (8 * j);
    }
    out[w] = packed;
  }
}

__global__ void vec_env_reset_k(float* state, uint64_t seed, uint8_t* frames, VecEnvParams p,
                                const int64_t* step_counter, int* new_frame, int* hist, float* ep_log) {
  const int e = blockIdx.x;
  float* st = state + (size_t)e * S_STRIDE;
  const int64_t step = step_counter ? step_counter[0] : 0;
  const int slot = (int)(((int64_t)step * p.E + e) % p.F);
  if (threadIdx.x == 0) {
    env_reset_state(st, seed, e, (uint64_t)step * 16 + 1);
    st[S_EPRET] = 0.f; st[S_EPLEN] = 0.f;
    new_frame[e] = slot;
    if (hist) for (int c = 0; c < 4; ++c) hist[e * 4 + c] = slot;
    if (ep_log) for (int c = 0; c < 4; ++c) ep_log[e * 4 + c] = 0.f;
  }
  __syncthreads();
  render_frame(st, frames + (size_t)slot * p.frame_bytes);
}

// One agent step = action_repeat emulator frames (MaxAndSkipEnv semantics: rewards
// summed, stop at game over).  episode_life: a lost life is an agent-level terminal
// but the game continues (EpisodicLifeEnv); game over / time limit reset the game.
__global__ void vec_env_step_k(float* state, const int* __restrict__ actions, uint64_t seed,
                               const int64_t* step_counter, uint8_t* frames, VecEnvParams p,
                               float* reward, float* done, int* new_frame, float* ep_log) {
  const int e = blockIdx.x;
  float* gst = state + (size_t)e * S_STRIDE;
  __shared__ float sst[S_STRIDE];
  const int64_t step = step_counter ? step_counter[0] : 0;
  const int slot = (int)(((int64_t)(step + 1) * p.E + e) % p.F);
  if (threadIdx.x == 0) {
    // the serial game logic runs on a register copy of the state (every index below is
    // a compile-time constant after unrolling): on the global copy each of its ~150
    // dependent accesses was an L2 round trip (17 us per step for 256 envs)
    float st[S_STRIDE];
#pragma unroll
    for (int i = 0; i < S_STRIDE; ++i) st[i] = gst[i];
    int dx, dy, fire;
    decode_action(actions[e], p.n_actions, dx, dy, fire);
    float r_raw = 0.f;
    bool life_lost = false, game_over = false;
    for (int f = 0; f < p.action_repeat && !game_over; ++f) {
      st[S_T] += 1.f;
      st[S_PX] = fminf(fmaxf(st[S_PX] + dx, 0.f), 80.f);
      st[S_PY] = fminf(fmaxf(st[S_PY] + dy, 42.f), 76.f);
      if (fire && st[S_BACT] < 0.5f) { st[S_BACT] = 1.f; st[S_BX] = st[S_PX] + 1.5f; st[S_BY] = st[S_PY] - 2.f; }
      const bool descend = ((int)st[S_T] % 64) == 0;
      bool crash = false;
#pragma unroll
      for (int k = 0; k < kEnemies; ++k) {
        float ex = st[S_EX + k] + st[S_EVX + k];
        if (ex < 0.f || ex > 78.f) { st[S_EVX + k] = -st[S_EVX + k]; ex = fminf(fmaxf(ex, 0.f), 78.f); }
        st[S_EX + k] = ex;
        if (descend) st[S_EY + k] += 2.f;
        if (fabsf(ex + 3.f - st[S_PX] - 2.f) < 4.5f && fabsf(st[S_EY + k] + 1.5f - st[S_PY] - 2.f) < 3.5f) crash = true;
        if (st[S_EY + k] > 78.f) crash = true;
      }
      if (st[S_BACT] > 0.5f) {
        st[S_BY] -= 3.f;
        int hit = -1;
#pragma unroll
        for (int k = 0; k < kEnemies; ++k)
          if (hit < 0 && fabsf(st[S_EX + k] + 3.f - st[S_BX]) < 3.5f && fabsf(st[S_EY + k] + 1.5f - st[S_BY]) < 2.5f)
            hit = k;
        if (hit >= 0) {
          float u[4];
          uniform4(seed, (uint64_t)e * 64 + hit, (uint64_t)step * 16 + 2 + f, u);
          r_raw += (p.n_actions == 18) ? 20.f : 1.f;
#pragma unroll
          for (int k = 0; k < kEnemies; ++k)
            if (k == hit) {  // register-resident: no dynamic index
              st[S_EX + k] = 4.f + 72.f * u[0];
              st[S_EY + k] = 8.f;
            }
          st[S_BACT] = 0.f;
        } else if (st[S_BY] < 0.f) {
          st[S_BACT] = 0.f;
        }
      }
      if (crash) {
#pragma unroll
        for (int k = 0; k < kEnemies; ++k) st[S_EY + k] = 8.f + 6.f * k;
        if (p.n_actions == 18) {
          st[S_LIVES] -= 1.f;
          life_lost = true;
          game_over = st[S_LIVES] <= 0.f;
        } else {  // Pong-like: opponent scores, game ends at 21
          r_raw -= 1.f;
          st[S_POINTS] += 1.f;
          game_over = st[S_POINTS] >= 21.f;
        }
      }
    }
    const float r = p.clip_rewards ? (r_raw > 0.f ? 1.f : (r_raw < 0.f ? -1.f : 0.f)) : r_raw;
    st[S_EPRET] += r;
    st[S_EPLEN] += 1.f;
    const bool time_up = p.max_episode_steps > 0 && st[S_EPLEN] >= (float)p.max_episode_steps;
    const bool agent_done = game_over || time_up || (p.episode_life && life_lost);
    reward[e] = r;
    done[e] = agent_done ? 1.f : 0.f;
    if (agent_done) {
      if (ep_log) {
        ep_log[e * 4 + 0] = st[S_EPRET];
        ep_log[e * 4 + 1] = st[S_EPLEN];
        ep_log[e * 4 + 2] += 1.f;
      }
      st[S_EPRET] = 0.f;
      st[S_EPLEN] = 0.f;
      if (game_over || time_up) env_reset_state(st, seed, e, (uint64_t)step * 16 + 7);
    }
    new_frame[e] = slot;
#pragma unroll
    for (int i = 0; i < S_STRIDE; ++i) {
      gst[i] = st[i];
      sst[i] = st[i];
    }
  }
  __syncthreads();
  render_frame(sst, frames + (size_t)slot * p.frame_bytes);
}

// ------------------------------------------------------------------ epsilon-greedy
__global__ void select_actions_k(const float* __restrict__ q, int E, int A, const float* __restrict__ eps,
                                 uint64_t seed, const int64_t* counter, int* __restrict__ actions) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float* row = q + (size_t)e * A;
  int best = 0;
  float bv = row[0];
  for (int a = 1; a < A; ++a)
    if (row[a] > bv) { bv = row[a]; best = a; }
  float u[4];
  uniform4(seed, (uint64_t)e, counter ? (uint64_t)counter[0] : 0ull, u);
  if (!(u[0] > eps[e])) {
    int r = (int)(u[1] * (float)A);
    best = r < A ? r : A - 1;
  }
  actions[e] = best;
}

// ------------------------------------------------------------------ n-step batcher
__device__ __forceinline__ void nstep_one(const NStepParams& p, const NStepState& st, const TransTable& tt,
                                          const float* __restrict__ q, const int* __restrict__ actions,
                                          const float* __restrict__ reward, const float* __restrict__ done,
                                          const int* __restrict__ new_frame, int64_t step, int e,
                                          int* __restrict__ slot_out, float* __restrict__ prio_out);

__global__ void nstep_emit_k(NStepParams p, NStepState st, TransTable tt, const float* __restrict__ q,
                             const int* __restrict__ actions, const float* __restrict__ reward,
                             const float* __restrict__ done, const int* __restrict__ new_frame,
                             int64_t* step_counter, int* __restrict__ slot_out,
                             float* __restrict__ prio_out, int bump) {
  const int64_t step = step_counter ? step_counter[0] : 0;
  if (bump) {
    // one workgroup strides over all envs, then advances the step counter once every
    // thread has read it (replaces a separate +1 launch on the actor stream)
    for (int e = threadIdx.x; e < p.E; e += blockDim.x) nstep_one(p, st, tt, q, actions, reward, done, new_frame,
                                                                  step, e, slot_out, prio_out);
    __syncthreads();
    if (threadIdx.x == 0) step_counter[0] = step + 1;
    return;
  }
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < p.E) nstep_one(p, st, tt, q, actions, reward, done, new_frame, step, e, slot_out, prio_out);
}

__device__ __forceinline__ void nstep_one(const NStepParams& p, const NStepState& st, const TransTable& tt,
                                          const float* __restrict__ q, const int* __restrict__ actions,
                                          const float* __restrict__ reward, const float* __restrict__ done,
                                          const int* __restrict__ new_frame, int64_t step, int e,
                                          int* __restrict__ slot_out, float* __restrict__ prio_out) {
  const int n = p.n, A = p.A;
  const int slot = (int)(((int64_t)step * p.E + e) % p.C);
  const int row = p.stage ? e : slot;  // staged: the learner scatters the row later
  int* meta = st.win_meta + e * 4;
  int start = meta[0], len = meta[1], qstart = meta[2], qlen = meta[3];
  int* hist = st.hist + e * 4;
  const float* qt = q + (size_t)e * A;
  const int at = actions[e];
  const float rt = reward[e];
  const bool dt = done[e] > 0.5f;
  const float gn = powf(p.gamma, (float)n);
  float qmax = qt[0];
  for (int a = 1; a < A; ++a) qmax = fmaxf(qmax, qt[a]);

  bool emitted = false;
  float prio = 0.f;
  auto write_trans = [&](const int* s0, int a0, float R, float d) {
    for (int c = 0; c < 4; ++c) {
      tt.s_ids[row * 4 + c] = s0[c];
      tt.s2_ids[row * 4 + c] = hist[c];
    }
    tt.action[row] = a0;
    tt.reward[row] = R;
    tt.done[row] = d;
  };

  if (p.mode == 0) {
    // ---- reference semantics (memory.py:415-440)
    if ((len == n || dt) && len > 0) {
      float R = 0.f, g = 1.f;
      for (int i = 0; i < len; ++i) { R += g * st.win_r[e * n + (start + i) % n]; g *= p.gamma; }
      R += g * rt;
      const int k0 = start;
      const int a0 = st.win_a[e * n + k0];
      const float q0a = st.win_q[((size_t)e * n + qstart) * A + a0];
      const float target = R + gn * qmax * (dt ? 0.f : 1.f);
      prio = fabsf(target - q0a) + 1e-6f;
      write_trans(st.win_ids + (e * n + k0) * 4, a0, R, dt ? 1.f : 0.f);
      emitted = true;
    }
    if (dt) {
      len = 0;  // state/action/reward deques cleared; the Q deque is not
    } else {
      int pos;
      if (len < n) { pos = (start + len) % n; ++len; } else { pos = start; start = (start + 1) % n; }
      for (int c = 0; c < 4; ++c) st.win_ids[(e * n + pos) * 4 + c] = hist[c];
      st.win_a[e * n + pos] = at;
      st.win_r[e * n + pos] = rt;
      int qpos;
      if (qlen < n) { qpos = (qstart + qlen) % n; ++qlen; } else { qpos = qstart; qstart = (qstart + 1) % n; }
      for (int a = 0; a < A; ++a) st.win_q[((size_t)e * n + qpos) * A + a] = qt[a];
    }
  } else {
    // ---- textbook n-step: R = sum_{i<n} gamma^i r, bootstrap gamma^n max Q(s_t)
    if (len == n) {
      float R = 0.f, g = 1.f;
      for (int i = 0; i < n; ++i) { R += g * st.win_r[e * n + (start + i) % n]; g *= p.gamma; }
      const int a0 = st.win_a[e * n + start];
      const float q0a = st.win_q[((size_t)e * n + start) * A + a0];
      prio = fabsf(R + gn * qmax - q0a) + 1e-6f;
      write_trans(st.win_ids + (e * n + start) * 4, a0, R, 0.f);
      emitted = true;
      start = (start + 1) % n;
      --len;
    }
    {  // push (s_t, a_t, r_t, Q(s_t))
      const int pos = (start + len) % n;
      ++len;
      for (int c = 0; c < 4; ++c) st.win_ids[(e * n + pos) * 4 + c] = hist[c];
      st.win_a[e * n + pos] = at;
      st.win_r[e * n + pos] = rt;
      for (int a = 0; a < A; ++a) st.win_q[((size_t)e * n + pos) * A + a] = qt[a];
    }
    int* dmeta = st.drain_meta + e * 2;
    if (dt) {
      // flush the window as terminal transitions: one now (if the slot is free), the
      // rest through the drain queue, one per following step.  A pending older drain is
      // dropped (only possible for episodes shorter than n-1 steps).
      int dl = 0;
      for (int j = 0; j < len; ++j) {
        float R = 0.f, g = 1.f;
        for (int i = j; i < len; ++i) { R += g * st.win_r[e * n + (start + i) % n]; g *= p.gamma; }
        const int k = (start + j) % n;
        const int a0 = st.win_a[e * n + k];
        const float pr = fabsf(R - st.win_q[((size_t)e * n + k) * A + a0]) + 1e-6f;
        if (!emitted) {
          write_trans(st.win_ids + (e * n + k) * 4, a0, R, 1.f);
          prio = pr;
          emitted = true;
        } else {
          for (int c = 0; c < 4; ++c) st.drain_ids[(e * n + dl) * 4 + c] = st.win_ids[(e * n + k) * 4 + c];
          st.drain_a[e * n + dl] = a0;
          st.drain_r[e * n + dl] = R;
          st.drain_q[e * n + dl] = pr;
          ++dl;
        }
      }
      for (int c = 0; c < 4; ++c) st.drain_s2[e * 4 + c] = hist[c];
      dmeta[0] = 0;
      dmeta[1] = dl;
      len = 0;
      start = 0;
    } else if (!emitted && dmeta[1] > 0) {
      const int k = dmeta[0];
      for (int c = 0; c < 4; ++c) {
        tt.s_ids[row * 4 + c] = st.drain_ids[(e * n + k) * 4 + c];
        tt.s2_ids[row * 4 + c] = st.drain_s2[e * 4 + c];
      }
      tt.action[row] = st.drain_a[e * n + k];
      tt.reward[row] = st.drain_r[e * n + k];
      tt.done[row] = 1.f;
      prio = st.drain_q[e * n + k];
      emitted = true;
      dmeta[0] = k + 1;
      dmeta[1] -= 1;
    }
    qstart = start;
    qlen = len;
  }
  meta[0] = start; meta[1] = len; meta[2] = qstart; meta[3] = qlen;
  // advance the observation stack (FrameStack: the reset frame is repeated k times)
  const int f = new_frame[e];
  if (dt) {
    for (int c = 0; c < 4; ++c) hist[c] = f;
  } else {
    hist[0] = hist[1]; hist[1] = hist[2]; hist[2] = hist[3]; hist[3] = f;
  }
  slot_out[e] = slot;
  prio_out[e] = emitted ? prio : 0.f;
}

// staged rows -> replay tables (overlapped actor/learner: the learner stream applies the
// previous actor step's rows right before its tree write, so a row is never rewritten
// while the learner can still sample its slot)
__global__ void apply_staged_rows_k(TransTable st, TransTable dst, const int* __restrict__ slot,
                                    const float* __restrict__ prio, int E) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E || !(prio[e] > 0.f)) return;
  const int j = slot[e];
  reinterpret_cast<int4*>(dst.s_ids)[j] = reinterpret_cast<const int4*>(st.s_ids)[e];
  reinterpret_cast<int4*>(dst.s2_ids)[j] = reinterpret_cast<const int4*>(st.s2_ids)[e];
  dst.action[j] = st.action[e];
  dst.reward[j] = st.reward[e];
  dst.done[j] = st.done[e];
}

// evaluator envs (no n-step batcher): advance each env's observation stack and the step
// counter that seeds the env / action draws (lane 0 of block 0)
__global__ void frame_hist_step_k(int* __restrict__ hist, const int* __restrict__ new_frame,
                                  const float* __restrict__ done, int E, int64_t* counter) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0 && counter) counter[0] += 1;
  if (e >= E) return;
  const int f = new_frame[e];
  int* h = hist + e * 4;
  if (done[e] > 0.f) {
    h[0] = h[1] = h[2] = h[3] = f;
  } else {
    h[0] = h[1]; h[1] = h[2]; h[2] = h[3]; h[3] = f;
  }
}

// ------------------------------------------------------------------ launchers
void frame_hist_step(int* hist, const int* new_frame, const float* done, int E, int64_t* counter, hipStream_t s) {
  if (E <= 0) return;
  frame_hist_step_k<<<(E + 255) / 256, 256, 0, s>>>(hist, new_frame, done, E, counter);
  LAUNCH_CHECK();
}

void vec_env_reset(float* state, uint64_t seed, uint8_t* frames, const VecEnvParams& p,
                   const int64_t* step_counter, int* new_frame, int* hist, float* ep_log, hipStream_t s) {
  if (p.frame_bytes != kScreen * kScreen) throw std::invalid_argument("vec env renders 84x84 frames");
  vec_env_reset_k<<<p.E, 256, 0, s>>>(state, seed, frames, p, step_counter, new_frame, hist, ep_log);
  LAUNCH_CHECK();
}

void vec_env_step(float* state, const int* actions, uint64_t seed, const int64_t* step_counter, uint8_t* frames,
                  const VecEnvParams& p, float* reward, float* done, int* new_frame, float* ep_log, hipStream_t s) {
  if (p.frame_bytes != kScreen * kScreen) throw std::invalid_argument("vec env renders 84x84 frames");
  if (p.n_actions != 18 && p.n_actions > 6) throw std::invalid_argument("vec env supports 18 or <=6 actions");
  vec_env_step_k<<<p.E, 256, 0, s>>>(state, actions, seed, step_counter, frames, p, reward, done, new_frame, ep_log);
  LAUNCH_CHECK();
}

void select_actions(const float* q, int E, int A, const float* eps, uint64_t seed, const int64_t* counter,
                    int* actions, hipStream_t s) {
  select_actions_k<<<(E + 255) / 256, 256, 0, s>>>(q, E, A, eps, seed, counter, actions);
  LAUNCH_CHECK();
}

void nstep_emit(const NStepParams& p, NStepState st, TransTable tt, const float* q, const int* actions,
                const float* reward, const float* done, const int* new_frame, int64_t* step_counter,
                int* slot_out, float* prio_out, hipStream_t s, bool bump) {
  if (p.n < 1 || p.n > 16) throw std::invalid_argument("n-step must be in [1, 16]");
  if (bump && !step_counter) throw std::invalid_argument("nstep_emit: bump needs a step counter");
  if (bump) {  // one workgroup (see nstep_emit_k)
    const int threads = std::min(1024, std::max(64, (p.E + 63) / 64 * 64));
    nstep_emit_k<<<1, threads, 0, s>>>(p, st, tt, q, actions, reward, done, new_frame, step_counter, slot_out,
                                       prio_out, 1);
  } else {
    nstep_emit_k<<<(p.E + 127) / 128, 128, 0, s>>>(p, st, tt, q, actions, reward, done, new_frame, step_counter,
                                                   slot_out, prio_out, 0);
  }
  LAUNCH_CHECK();
}

void apply_staged_rows(TransTable stage, TransTable dst, const int* slot, const float* prio, int E, hipStream_t s) {
  if (E <= 0) return;
  apply_staged_rows_k<<<(E + 255) / 256, 256, 0, s>>>(stage, dst, slot, prio, E);
  LAUNCH_CHECK();
}

}  // namespace apex
