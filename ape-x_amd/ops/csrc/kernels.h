// Host-visible launcher declarations for the gfx950 kernels.  Every launcher takes
// raw device pointers and the caller's hipStream_t (torch's current stream), never
// allocates and never synchronises, so a sequence of them can be captured into a
// hipGraph (cdna_hip_programming.md Guideline 9).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace apex {

constexpr int kTreeFanout = 64;       // one child per lane of a wave64
constexpr int kTreeLog2Fanout = 6;
constexpr int kMaxTreeLevels = 8;     // 64^8 leaves >> any HBM capacity

// Wide prioritized-replay tree: level 0 = leaves (fp32 sum / fp32 min), levels
// 1..levels = internal nodes (fp64 sum / fp32 min), level `levels` has one node.
struct TreeDesc {
  float* leaf_sum;
  float* leaf_min;
  double* node_sum[kMaxTreeLevels];
  float* node_min[kMaxTreeLevels];
  int size[kMaxTreeLevels + 1];
  int levels;
};
// Sharded replay (parallel.sharded): the exchanged per-shard (mass, min priority) slots;
// the sampler derives the global min priority and this shard's IS-weight scale
// world * M_rank / sum_r M_r in-kernel (no host-side or torch-op finalize).
struct ShardGlob {
  const float* slots;  // [world][2]
  int world, rank;
};
// Fast batched tree update (replay_kernels.hip: BatchWrite, per_write_batch): staged
// actor rows + learner priorities in one leaves kernel + one wide kernel per big level.
struct PrioMix {
  const float* delta;  // [B] |y - Q(s,a)|
  const float* lw;     // [B] w_i * Huber(delta_i)
  float* prio_out;     // [B] mixed priorities (as dqn_loss writes them)
  float* loss_out;     // [1]
};
struct BatchWrite {
  const int* pre_idx;     // [E] actor slots (unique) or null
  const float* pre_prio;  // [E] raw priorities
  int E;
  int64_t* pre_bump;      // e.g. replay.filled += E (or null)
  const int* idx;         // [B] learner slots (may repeat) or null
  const float* prio;      // [B] raw priorities (ignored with mix)
  int B;
  PrioMix mix;
  int64_t* bump;          // e.g. learner step counter += 1 (or null)
  int* owner;             // [capacity] scratch, all -1 between calls
  int* list;              // [E + B] out: slots whose ancestors are dirty
  float* max_prio;
  float alpha;
};
void per_write_batch(const TreeDesc& t, const BatchWrite& w, int* ticket, hipStream_t s);
// The same batched write riding the learner's backward launches as extra workgroups (no
// tree stream, no fork / join in the learner graph): stage 1 = the leaves (one workgroup,
// block 0 of the FC1 backward pair), stage 2 = level `level` of the listed slots (one wave
// per slot, workgroups after the GEMM tiles), stage 3 = every node of levels top_from.. in one
// workgroup (block 0).  Each stage reads what an earlier launch wrote: no fences, no tickets.
// stage 0: no rider.
struct TreeRide {
  TreeDesc t;
  BatchWrite w;
  int stage, level, top_from;
  int nhost;  // the host launch's own workgroups (set by the launcher)
};
// workgroups a rider adds to its host launch
int tree_ride_blocks(const TreeRide& r);
// wide level stages of a ridden write on this tree: 1 (level 1; every level above it in the top
// walk), 2 (levels 1 and 2; the rest in the top walk), or -1 (a level above 2 has > 64 nodes)
int tree_ride_level_stages(const TreeDesc& t);
// Zero `slots` [world][2] and write this shard's (root mass, root min priority) into
// slot `rank`: after a SUM all-reduce every rank holds all shards' pairs (an all-gather
// folded into the learner's conv-gradient all-reduce).
void pack_shard_slots(const TreeDesc& t, float* slots, int world, int rank, hipStream_t s);

// ---- replay_kernels.hip
// Write prio**alpha into the leaves of `idx` AND recompute every dirty ancestor.
// dedup = 1: duplicates resolve last-write-wins (B <= 1024, needs `sorted_scratch` [B]);
// dedup = 0: `idx` must be unique ring-ordered slots (actor inserts).
// bump0/bump1: optional device counters advanced by d0/d1 (fused counter updates).
// mix_* (optional, dedup only): priorities from per-row TD errors with the batch-max mix
// of utils.py:77, and the loss mean (see replay_kernels.hip PrioMix)
void per_write_leaves(const TreeDesc& t, const int* idx, const float* prio, int B, float alpha, float* max_prio,
                      int dedup, int* sorted_scratch, int64_t* bump0, int64_t d0, int64_t* bump1, int64_t d1,
                      hipStream_t s, const float* mix_delta = nullptr, const float* mix_lw = nullptr,
                      float* mix_prio_out = nullptr, float* mix_loss_out = nullptr);
void per_update_levels(const TreeDesc& t, const int* idx, int B, hipStream_t s);
// length/beta are read from device memory when the pointers are non-null (so a captured
// graph sees the live replay fill level and annealed beta), else the constants are used.
// ``glob`` (sharded replay, nullable): glob[0] = global min priority used for the IS
// weights, glob[1] = this shard's weight scale (apex_amd.parallel.sharded).
void per_sample(const TreeDesc& t, int B, const int64_t* length_ptr, int64_t length_const, const float* beta_ptr,
                float beta_const, uint64_t seed, const int64_t* counter, int* out_idx, float* out_w,
                int exclude_last, const float* glob, hipStream_t s, ShardGlob sg = ShardGlob{nullptr, 0, 0},
                const struct StagedRows* rows = nullptr, const struct SampleRowsOut* rows_out = nullptr);
void gather_transitions(const uint8_t* frames, int frame_bytes, const int* s_ids, const int* s2_ids,
                        const int* act, const float* rew, const float* done, const int* idx, int B, uint8_t* out_s,
                        uint8_t* out_s2, int* out_a, float* out_r, float* out_d, hipStream_t s);
void gather_frames(const uint8_t* frames, int frame_bytes, const int* ids, int N, int stack, uint8_t* out,
                   hipStream_t s);
void bump_counter(int64_t* counter, int n, int64_t by, hipStream_t s);
// evaluator envs: FrameStack advance (done: the new frame repeated 4x) + counter += 1
void frame_hist_step(int* hist, const int* new_frame, const float* done, int E, int64_t* counter, hipStream_t s);

// ---- actor_kernels.hip
struct VecEnvParams {
  int E;              // envs in this shard
  int n_actions;
  int frame_bytes;    // 84*84
  int F;              // frame-ring capacity (frames)
  int action_repeat;  // 4 (MaxAndSkip)
  int clip_rewards;
  int episode_life;
  int max_episode_steps;
};
void vec_env_reset(float* state, uint64_t seed, uint8_t* frames, const VecEnvParams& p,
                   const int64_t* step_counter, int* new_frame, int* hist, float* ep_log, hipStream_t s);
void vec_env_step(float* state, const int* actions, uint64_t seed, const int64_t* step_counter, uint8_t* frames,
                  const VecEnvParams& p, float* reward, float* done, int* new_frame, float* ep_log, hipStream_t s);
void select_actions(const float* q, int E, int A, const float* eps, uint64_t seed, const int64_t* counter,
                    int* actions, hipStream_t s);

struct NStepParams {
  int E, A, n, C;   // envs, actions, n-step, transition capacity
  float gamma;
  int mode;         // 0 = reference, 1 = textbook
  int stage;        // 1: rows go to staging row e (TransTable of E rows), slot_out = ring slot
};
struct NStepState {
  int* win_ids;     // [E][n][4]
  int* win_a;       // [E][n]
  float* win_r;     // [E][n]
  float* win_q;     // [E][n][A]
  int* win_meta;    // [E][4]: start, len, q_start, q_len
  int* hist;        // [E][4]  current observation stack (frame ids)
  int* drain_ids;   // [E][n][4]   textbook-mode tail
  int* drain_a;     // [E][n]
  float* drain_r;   // [E][n]
  float* drain_q;   // [E][n]      Q(s, a) only
  int* drain_meta;  // [E][2]: start, len
  int* drain_s2;    // [E][4]
};
struct TransTable {
  int* s_ids;       // [C][4]
  int* s2_ids;      // [C][4]
  int* action;      // [C]
  float* reward;    // [C]
  float* done;      // [C]
};
void nstep_emit(const NStepParams& p, NStepState st, TransTable tt, const float* q, const int* actions,
                const float* reward, const float* done, const int* new_frame, int64_t* step_counter,
                int* slot_out, float* prio_out, hipStream_t s, bool bump = false);
// staged actor rows [E] -> replay tables at slot[e] (emitted rows only: prio[e] > 0);
// also fused into per_sample's launch (extra blocks: the scatter writes table rows the
// sampler never reads, and both must precede the learner's forward)
struct StagedRows {
  TransTable st, dst;
  const int* slot;
  const float* prio;
  int E;
};
void apply_staged_rows(TransTable stage, TransTable dst, const int* slot, const float* prio, int E, hipStream_t s);
// per_sample's private copy of every sampled row (the learner's sampled-ahead batch):
// out.*[i] = the row of slot out_idx[i] -- from the staged rows when this very launch
// scatters that slot, else from ``src`` (the replay tables)
struct SampleRowsOut {
  TransTable src, out;
};

// ---- conv_bwd_kernels.hip: one launch for all batch-sliced gradient reductions
constexpr int kMaxFinalizeJobs = 6;
struct FinalizeJob {
  int kind;                 // 0: conv wgrad (C, KH, KW), 1: heads (C = A), 2: FC1 weight rows
  const float* part;        // [G][pstride]
  const float* bpart;       // [G][bstride] (conv bias partials)
  int G, pstride, bstride, n_main, n_bias;
  int C, KH, KW;
  float* out[6];
  int block0;               // set by grad_finalize
};
struct FinalizeSet {
  FinalizeJob job[kMaxFinalizeJobs];
  int n;
  double* sumsq;            // optional: one fp64 partial of sum(g^2) per workgroup (grad norm)
};
int wgrad_grid(int layer, int B);
// returns the finalize workgroup (= sumsq partial) count; ride: a stage-3 tree rider (block 0)
int grad_finalize(FinalizeSet fs, hipStream_t s, const TreeRide* ride = nullptr);
int grad_finalize_blocks(const FinalizeSet& fs);
FinalizeJob conv_finalize_job(int layer, int B, const float* ws, float* grad, float* bias_grad);
// FC1 weight half (0: advantage rows 0..127, 1: value rows 128..255) of fc1_bwd's slabs
FinalizeJob fc1_finalize_job(int half, const float* ws, float* grad);
FinalizeJob f32_fc1_finalize_job(int half, int G, const float* ws, float* grad);  // fp32 FC1 slices
FinalizeJob heads_finalize_job(int G, int A, const float* part, float* g_wadv2, float* g_badv2, float* g_wval2,
                               float* g_bval2, float* g_badv1, float* g_bval1);

// ---- loss_heads_kernels.hip: dqn_loss + heads_bwd + head weight-grad partials, fused
struct LossHeadsArgs {
  const float *q, *q2, *q2t;       // [B][A] Q(s), Q(s'), Q_target(s')
  const int* act;                  // replay transition table, read through idx
  const float *rew, *done;
  const int* idx;                  // sampled slots (nullptr: row b)
  const float* w;                  // [B] IS weights
  const float* h;                  // [B][256] post-ReLU hidden of the Q(s) pass
  const float *w_adv2, *w_val2;    // head weights [A][128], [128]
  int B, A;
  float gamma_n;
  float* delta;                    // [B] out: |y - Q(s,a)|
  float* lw;                       // [B] out: w * Huber(delta)
  uint16_t* dz_bf;                 // [B][256] out: dL/dz (FC1 pre-activation), bf16
  float* part;                     // [blocks][(A+1)*128 + (A+1) + 256] out: gradient partials
  float* dz;                       // [B][256] out (optional, replaces dz_bf): dL/dz in fp32
  const int64_t* step;             // learner step counter (read)
  int64_t* step_snap;              // out: its value for this step's optimizer (may be null)
};
int dqn_heads_bwd_blocks(int B);
void dqn_heads_bwd(const LossHeadsArgs& args, hipStream_t s);

// ---- learner_kernels.hip
// (a, r, d) are read through idx (the sampled replay slots) when idx != nullptr.
void dqn_loss(const float* q, const float* q2, const float* q2t, int ldq, const int* a, const float* r, const float* d,
              const int* idx, const float* w, int B, int A, float gamma_n, float* loss_out, float* dq, float* prio,
              hipStream_t s);
void grad_sumsq(const float* g, int64_t n, double* partials, hipStream_t s);
int grad_norm_partials();
struct RMSpropParams {
  float lr0, alpha, eps, max_norm;
  float lr_gamma;        // StepLR gamma (1 = constant)
  int lr_step_size;      // StepLR step size
  int lr_step_offset;    // 1 reproduces scheduler.step() before optimizer.step()
  int centered;
  float grad_scale = 1.f;  // gradient multiplier (1/world: the DP all-reduce sums)
};
// ``pack`` (nullable): after the update, bf16(p[i]) is also written to pack->arena at
// pack->dst1[i] and pack->dst2[i] (-1 = none): the MFMA kernels' packed weight layouts
// are refreshed inside the optimizer pass instead of by separate pack kernels.
struct PackMap {
  const int* dst1;
  const int* dst2;
  uint16_t* arena;      // bf16 packed copies (bf16 network) ...
  float* arena_f32;     // ... or fp32 packed copies (reference-precision network)
};
// FC1 weights (Nature-CNN dueling net): flat offsets of advantage.0.weight and
// value.0.weight ([128][64*49] each) and the two packed bf16 layouts they refresh,
// wp = wfc1p [256][49*64] and wt = wfc1t [49*64][256].  With it the optimizer updates
// FC1 in LDS-transposed tiles (coalesced packed stores) instead of through the scatter
// maps (whose FC1 entries are then ignored).  fp32 network: wp_f32 = [256][49*64] fp32
// (its forward B operand and, read row-major, the input-gradient GEMM's), no transpose.
struct FcPack {
  int64_t off[2];
  uint16_t* wp;
  uint16_t* wt;
  float* wp_f32;
};
void rmsprop_step(float* p, const float* g, float* sq, float* gavg, int64_t n, const double* partials,
                  int n_partials, const RMSpropParams& hp, const int64_t* step, float* norms_out, hipStream_t s,
                  const PackMap* pack = nullptr, const FcPack* fc = nullptr);
struct AdamParams {
  float lr0, beta1, beta2, eps, weight_decay, max_norm;
  float lr_gamma;
  int lr_step_size, lr_step_offset;
  float grad_scale = 1.f;
};
// one parameter set of a fused two-set optimizer launch (adam_step2)
struct OptSet {
  float* p;
  const float* g;
  float* s1;
  float* s2;
  int64_t n;
  const double* partials;
  int n_partials;
  float* norms_out;
  int nblk;  // set by the launcher
};
void adam_step2(OptSet a, OptSet b, const AdamParams& hp, const int64_t* step, hipStream_t s);
void adam_step(float* p, const float* g, float* m, float* v, int64_t n, const double* partials, int n_partials,
               const AdamParams& hp, const int64_t* step, float* norms_out, hipStream_t s,
               const PackMap* pack = nullptr, const FcPack* fc = nullptr);
void copy_f32(float* dst, const float* src, int64_t n, hipStream_t s);
// One wave busy-waits `us` microseconds on the constant-rate wall clock (bounded; used by
// the engine's stream-concurrency probe).
void spin_us(int us, hipStream_t s);

// ---- conv_kernels.hip (Nature-CNN dueling net, bf16 MFMA)
// layer 1: `in` is the u8 frame ring (ids/idx: FrameSrc, see common.h) or a dense u8 stack
// Multi-problem forward launches: up to kMaxProbs independent passes of the same layer
// (the learner's Q(s), Q(s') and Q_target(s')) in ONE launch -- every kernel boundary
// costs ~4.5 us on MI355X, and the 3x larger grid amortises weight staging.  All
// problems share the batch size B; problem i covers samples [i*B, (i+1)*B).
constexpr int kMaxProbs = 3;
struct ConvProb {
  const void* in;       // layer 1: u8 frames (dense [B][4][84][84] or the frame ring)
  const int* ids;       // layer 1 frame-ring ids [*][4] (nullptr = dense)
  const int* idx;       // row map into ids (nullptr = identity)
  const uint16_t* w;    // packed bf16 weights
  const float* bias;
  uint16_t* out;        // channels-last bf16 activations
};
struct ConvSet {
  ConvProb p[kMaxProbs];
  int n, B;
};
void conv_fwd_multi(int layer, const ConvSet& set, hipStream_t s);
void conv_fwd(int layer, const void* in, const int* ids, const int* idx, const uint16_t* wp, const float* bias,
              uint16_t* out, int B, hipStream_t s);
void heads_wgrad(const float* dA, const float* h, const float* dz, int B, int A, float* ws, float* g_wadv2,
                 float* g_badv2, float* g_wval2, float* g_bval2, float* g_badv1, float* g_bval1, hipStream_t s);
size_t heads_wgrad_workspace_floats(int A);
void heads_fwd(const float* z, int nsplit, const float* b_adv1, const float* b_val1, const float* w_adv2,
               const float* b_adv2, const float* w_val2, const float* b_val2, float* hout, float* q, int B, int A,
               hipStream_t s);
// fc_kernels.hip: split-K FC1 (a3 [B][3136] bf16 . W [256][3136]^T) -> fp32 partials [fc1_splits()][B][256]
int fc1_splits();                   // max slabs any launch writes (workspace sizing)
int fc1_splits_for(int total_rows);  // slabs a launch over total_rows rows writes
int fc1_fwd(const uint16_t* a, const uint16_t* w, float* part, int B, hipStream_t s);  // returns slabs
struct FcProb {
  const uint16_t* a;  // a3 [B][3136] bf16
  const uint16_t* w;  // [256][3136] bf16
  float* part;        // [slabs][B][256] fp32 split-K partials
};
struct FcSet {
  FcProb p[kMaxProbs];
  int n, B;
};
int fc1_fwd_multi(const FcSet& set, hipStream_t s);  // returns the slab count
// FC1 backward: dy3 = relu_mask(dz . W, a3) (bf16) and dW partial slabs [fc1_bwd_slices()]
// [256][3136] (natural k order; reduce + scatter with two grad_finalize conv-style jobs)
int fc1_bwd_slices();
size_t fc1_bwd_workspace_floats();
void fc1_bwd(const uint16_t* dz, const uint16_t* a3, const uint16_t* wt, uint16_t* dy3, float* part, int B,
             hipStream_t s);
struct HeadsProb {
  const float* z;  // FC1 split-K partials [nsplit][B][256]
  const float *b_adv1, *b_val1, *w_adv2, *b_adv2, *w_val2, *b_val2;
  float* hout;     // [B][256] post-ReLU hidden (nullptr: not kept)
  float* q;        // [B][A]
};
// Optional epsilon-greedy epilogue of problem 0 (the actor's inference pass): the wave that
// finishes row b's Q also picks its action (first argmax; uniform action with prob eps[b]),
// drawing the same Philox numbers as select_actions_k, so the standalone launch goes away.
struct ActSel {
  const float* eps;        // [B] per-env epsilon (nullptr: no epilogue)
  const int64_t* counter;  // actor step counter (RNG counter)
  int* actions;            // [B]
  uint64_t seed;
};
struct HeadsSet {
  HeadsProb p[kMaxProbs];
  int n, B, A, nsplit;
  int xcd_map;  // set by heads_fwd_multi: XCD-aware row-block mapping (see heads_fwd_k)
  ActSel act;
};
void heads_fwd_multi(const HeadsSet& set, hipStream_t s);
void heads_bwd(const float* dq, const float* h, const float* w_adv2, const float* w_val2, float* dA, float* dz,
               uint16_t* dz_bf, int B, int A, hipStream_t s);
void pack_conv_w(const float* src, uint16_t* dst, int N, int C, int KH, int KW, hipStream_t s);
void pack_fc1(const float* adv, const float* val, uint16_t* dst, int P, int C, hipStream_t s);
void unpack_fc1_grad(const float* gp, float* g_adv, float* g_val, int P, int C, hipStream_t s);
void relu_mask_bf16(const uint16_t* g, const uint16_t* a, uint16_t* out, int64_t n, hipStream_t s);
void u8_to_bf16_nhwc(const uint8_t* in, uint16_t* out, int B, int HW, hipStream_t s);

// ---- conv_bwd_kernels.hip
// dgrad of layer 2/3: dy (optionally ReLU-masked by dy_mask while staging) -> dx,
// optionally ReLU-masked by dx_mask in the (coalesced) epilogue
void conv_dgrad(int layer, const uint16_t* dy, const uint16_t* dy_mask, const uint16_t* wt, uint16_t* dx,
                const uint16_t* dx_mask, int B, hipStream_t s);
size_t wgrad_workspace_floats(int layer);
void conv_wgrad(int layer, const void* x, const int* ids, const int* idx, const uint16_t* dy, const uint16_t* dy_mask,
                int B, float* workspace, float* grad, float* bias_grad, hipStream_t s);
void pack_conv_wt(const float* src, uint16_t* dst, int N, int C, int KH, int KW, hipStream_t s);


// ---- conv1_kernels.hip: conv1 forward from raw u8 planes; w = bf16 [32][4][8][8] (reference layout)
void conv1_fwd_multi(const ConvSet& set, hipStream_t s);
void conv1_fwd(const uint8_t* frames, const int* ids, const int* idx, const uint16_t* w, const float* bias,
               uint16_t* out, int B, hipStream_t s);

// ---- f32_kernels.hip: reference-precision (fp32 MFMA) dueling net, fp32 activations
// channels-last, weights from exact fp32 packed copies (models/fused_f32.py layouts)
struct F32Prob {
  const void* in;     // layer input: u8 frames (conv1, FrameSrc with ids/idx) or fp32 activations
  const int* ids;
  const int* idx;
  const float* w;     // conv1: W1 (reference layout); conv2/conv3: w2p/w3p; FC1: wfc1p
  const float* w2;    // unused
  const float* bias;
  float* out;         // activations (conv) | split-K partials [7][B][256] (FC1)
};
struct F32Set {
  F32Prob p[kMaxProbs];
  int n, B;
};
// The learner's PER draw folded into the fp32 conv1 forward (f32_conv1_fwd_x3_k): every
// workgroup draws the slots of its own samples (one wave each, the per_sample_k descent) before
// staging their frames, and problem 0's workgroups write out_idx / out_w.  rows.E > 0: the staged
// actor rows this launch scatters into the tables (extra workgroups, as per_sample_k's); a drawn
// slot among them is read from the staging rows.  out_idx == nullptr: no draw.
struct ConvSample {
  TreeDesc t;
  const int64_t* length;   // live fill level (replay.filled)
  const float* beta;
  const int64_t* counter;  // RNG step counter
  uint64_t seed;
  int* out_idx;
  float* out_w;
  int exclude_last;
  StagedRows rows;
  int nhost;  // set by the launcher
};
void f32_conv_fwd_multi(int layer, const F32Set& set, hipStream_t s, int c1_grid = 0, int tile = 0,
                        const ConvSample* draw = nullptr);  // draw: layer 1 only
int f32_fc1_splits();
// GEMM form: mask = forward form + 4 x backward-pair form; form 0 = per-wave register split,
// 1 = stage-split LDS image (split once per staged element, double-buffered), 2 = the same
// with one LDS image, 3 = form 2 held to >= 3 waves per SIMD; -1 reads APEX_F32_STAGE_SPLIT.  Bit-identical in every form; read at
// launch (graphs keep the form they captured).
void f32_set_stage_split(int mask);
int f32_stage_split();
int f32_fc1_fwd_multi(const F32Set& set, hipStream_t s);  // returns the slab count
// target: conv2 / conv3 weight-gradient workgroups (<= 0: the default); the workspace, the
// launch and the finalize job of one gradient must use the same value
int f32_wgrad_splits(int layer, int B, int target = 0);
int f32_wgrad_kbps(int layer, int B, int target = 0);  // k-blocks (32 rows) per split
size_t f32_wgrad_workspace_floats(int layer, int B, int target = 0);
int f32_fc1_wgrad_splits();
int f32_fc1_wgrad_slices(int B);
size_t f32_fc1_wgrad_workspace_floats();
void f32_fc1_bwd_split(const float* dz, const float* a3, const float* wfc1p, float* dy3, float* ws, int B,
                       hipStream_t s, const TreeRide* ride = nullptr);
// conv backward: layers 3/2 = wgrad partials + dgrad (w = w3t / w2t, masked by `mask`) in
// one launch, layer 1 = wgrad partials from the u8 frames (x/ids/idx as FrameSrc)
void f32_conv_bwd(int layer, const void* x, const int* ids, const int* idx, const float* dy, const float* w,
                  const float* mask, float* dx, float* ws, int B, hipStream_t s, int target = 0, int tile = 0,
                  const TreeRide* ride = nullptr);  // ride: layers 3 / 2 only
FinalizeJob f32_conv_finalize_job(int layer, int B, const float* ws, float* grad, float* bias_grad, int target = 0);
// grad_finalize job that only adds sum(g^2) of g[0..n) to the norm partials
FinalizeJob norm_only_job(const float* g, int n);

// ---- aql_kernels.hip (AQL candidate critic / proposal)
struct AQLNet {
  int obs, adim, cont, T, na, uniform, propose, noisy;
  const float *qf_w1, *qf_b1, *qf_w2, *qf_b2;        // q_feature: obs->64->64
  const float *ao_w1, *ao_b1, *ao_w2, *ao_b2;        // action_out: adim->128->64 (cont) | 1->64
  const float *a1_wmu, *a1_wsig, *a1_weps, *a1_bmu, *a1_bsig, *a1_beps;  // NoisyLinear 128->64
  const float *a2_wmu, *a2_wsig, *a2_weps, *a2_bmu, *a2_bsig, *a2_beps;  // NoisyLinear 64->1
  const float *f_w, *f_b;                            // q.features: obs->128 (state embedding)
  const float *df_w1, *df_b1, *df_w2, *df_b2;        // proposal.dist_feature: 128->128->na
};
size_t aql_workspace_floats();
void aql_noisy_eff(const AQLNet& net, float* ws, hipStream_t s);  // W_eff = mu + sigma eps into ws
void aql_candidate_q(const AQLNet& net, float* ws, const float* state, const float* a_mu, int B, float* q,
                     hipStream_t s);
void aql_propose(const AQLNet& net, const float* state, int B, const float* low, const float* high, const float* var,
                 uint64_t seed, const int64_t* counter, float* a_mu, float* mu_out, hipStream_t s,
                 float* eff_ws = nullptr);  // + aql_noisy_eff into eff_ws (extra workgroups)
void aql_select(const float* q, const float* a_mu, int B, int T, int adim, const float* eps, uint64_t seed,
                const int64_t* counter, int* act_idx, float* env_act, hipStream_t s);

// ---- aql_engine_kernels.hip (GPU AQL engine: fused learner step, vector envs + replay insert)
// Per-sample backward vectors written by aql_learn_bwd and contracted over the batch by
// aql_grad (every weight gradient is sum_b G[b][row] * X[b][col]).  Offsets in floats.
namespace aqlv {
constexpr int GQ = 0, H = 8, GH = 72, X = 136, GX = 264, AOH = 392, GAOH = 520, A = 648, QFH = 656, GQFH = 720,
              S = 784, EMB = 848, HID = 976, GHID = 1104, GMU = 1232, STRIDE = 1296;
}
constexpr int kAqlMaxJobs = 32;
struct AqlLearn {
  AQLNet on, tg;                             // online / target critic + proposal weights
  const float *eff_on, *eff_tg;              // effective NoisyLinear weights (aql_workspace_floats layout)
  const float *st, *st2, *rew, *done, *amu;  // replay tables [C][obs] x2, [C], [C], [C][T][adim]
  const int* act;                            // [C] taken candidate index
  const int* idx;                            // [B] sampled slots
  const float* w;                            // [B] IS weights
  int B;
  float gamma_n, ent_lam;
  const float* var;                          // proposal MVN diagonal [na]
  float *q_s, *q_s2, *qt_s2;                 // [B][T] Q(s,.), Q(s',.), Q_tgt(s',.)
  float* vec;                                // [B][aqlv::STRIDE]
  float *delta, *lw, *lossp;                 // [B] |td|, w*Huber, per-sample proposal loss
  long long* dbg;                            // optional phase timestamps (block 0, s_memtime) or null
  int act_mode;                              // 1: acting -- online Q(st[row], .) only, row = idx ? idx[b] : b
  int act_blocks;                            // acting: workgroups (each loops over its items); 0 = one per item
  // fused sampling (aql_learn_set_sample): every forward workgroup draws its sample's row from
  // the PER tree itself (tree_sample_leaf, as per_sample_k) and the (tile 0, online) workgroup
  // writes idx / IS weight for the backward -- no per_sample launch
  int fused_sample, exclude_last;
  TreeDesc tree;
  const int64_t* filled;                     // live slots (min with the capacity)
  const float* beta;
  const int64_t* ctr;                        // Philox counter (the learner step)
  uint64_t seed;
  int* idx_out;
  float* w_out;
  // priority write in the backward launch (aql_learn_set_tree): one extra workgroup recomputes
  // the B TD terms from the forward's Q rows (aql_td, the backward's own formula) and runs the
  // batched tree write (leaves + every level, B <= 64) beside the per-sample backward
  int bwd_tree;  // 1: leaves + every level, 2: leaves + levels 1..bwd_levels (aql_grad_set_levels walks the rest)
  int bwd_levels;
  BatchWrite bw;
  // learner forward: candidate-tile groups per (sample, net) workgroup item (0 = about one
  // workgroup per CU; act_mode: 0 = one tile per item)
  int tile_groups;
  int fwd_halves;  // learner forward workgroup: 2 = 512 threads (alternate tiles per half), 1 = 256
  // step gate (central AQL learner): this launch belongs to step gate_j of the iteration and
  // does nothing unless gate_j < *gate (the steps the ingest's new rows paid for, IpcIngest)
  const int* gate;
  int gate_j;
};
void aql_learn_fwd(const AqlLearn& L, hipStream_t s);
// acting on the learner's MFMA forward: q_s[b][t] = Q_on(st[b], amu[b][t]) for B states
void aql_act_q(const AqlLearn& L, hipStream_t s);
void aql_learn_bwd(const AqlLearn& L, hipStream_t s);
struct AqlGradJob {
  int64_t off;         // flat offset of the parameter tensor
  int rows, cols;      // [rows][cols]; a bias has cols = 1 and xoff < 0
  int goff, xoff;      // aqlv offsets of the output-gradient / input vectors
  const float* eps;    // NoisyLinear sigma: grad = grad_mu * eps (nullable)
  int group;           // 0 = critic (optimizer_q), 1 = proposal (optimizer_proposal)
  int zero;            // identically zero (q.features: only the proposal loss reaches it)
};
struct AqlGrad {
  AqlGradJob job[kAqlMaxJobs];
  int njobs;
  int64_t n;           // flat parameters (jobs cover [0, n) in offset order)
  const float* vec;
  int B;
  float* grad;
  double* part;        // [2][blocks] sum of squares per group
  const float* lossp;  // [B]
  float* lossp_out;    // [1] proposal loss mean
  // the priority tree's level walk (aql_grad_set_levels): one extra workgroup walks levels
  // levels_lo.. of the dirty list the backward launch's tree workgroup wrote (with the leaves)
  int tree_leaves;  // 0 / 2 (the walk)
  int levels_lo;
  TreeDesc tree;
  BatchWrite bw;
  const int* gate;  // step gate (AqlLearn::gate)
  int gate_j;
  // (aql_grad_set_step_snap) block 0 copies the learner step counter here: the update launch
  // that follows reads its step from the copy, so one of its blocks can bump the counter
  // without a last-block ticket (an atomic round trip at the end of every update workgroup)
  int64_t* step_snap = nullptr;
  const int64_t* step_src = nullptr;
};
int aql_grad_blocks(int64_t n);
void aql_grad(const AqlGrad& g, hipStream_t s);
struct AqlNoise {
  float *weps, *beps;                    // NoisyLinear epsilon buffers [out][in], [out]
  const float *wmu, *wsig, *bmu, *bsig;  // parameters (post-update)
  float *weff, *beff;                    // effective weight mu + sigma * eps (learner workspace)
  int out, in;
};
struct AqlPost {
  AqlNoise layer[4];   // online advantage1/2, target advantage1/2
  const float* src;    // online proposal parameters ...
  float* dst;          // ... hard-copied into the target's (AQL_dis.py:92)
  int64_t n_copy;
  int64_t* step;       // learner step counter (+1 by the last block)
  int* ticket;
  uint64_t seed;
};
// regen = 1: fresh factorised noise for all four layers (reset_noise), effective weights,
// proposal copy, step + 1.  regen = 0: effective weights from the current noise only
// (after initialisation / a target sync).
void aql_post(const AqlPost& p, int regen, hipStream_t s);
// The learner step's update (aql_engine_kernels.hip: aql_update_k) after the gradient launch:
// both clipped Adam steps + the noise reset of both critics + the proposal copy + the step bump
// (+ the next step's PER draw, + the acting copies), replacing adam_step2 + aql_post when the
// priority write ran in the backward launch.  The descriptor lives in device memory (too large
// for kernel arguments).
struct AqlStep {
  AqlLearn L;              // the backward's view (online net, replay tables, per-sample outputs)
  AqlGrad G;               // gradient jobs, grad, partials [2][nblk], proposal loss mean
  AqlPost P;               // noisy layers (online 0-1, target 2-3), proposal copy, step, ticket
  TreeDesc tree;
  AdamParams hp;
  float *p, *m, *v;        // flat parameters and Adam moments
  int64_t n, P_q;          // critic [0, P_q), proposal [P_q, n)
  float *norms_q, *norms_p;
  int64_t mu_w[2], sig_w[2], mu_b[2], sig_b[2];  // flat offsets of the online noisy layers' tensors
  int nblk;                // gradient workgroups (aql_grad_blocks(n))
  // the NEXT step's PER draw (draw = 1): extra workgroups sample step st + 1's
  // rows into L.idx / L.w -- what the next forward's fused sampling would draw (same tree,
  // counter, mass, beta) -- and that forward runs on the plain descriptor, without its descent.
  // An iteration's last step does not draw (the actors insert before the next one).
  int draw;
  const int64_t* filled;
  const float* beta;
  uint64_t seed;
  int exclude_last;
  // optional publish (the iteration's last step): every updated parameter and the online noise
  // also written into the acting copies (set_worker_weights without the two copy launches)
  float* pub_p;
  float* pub_weps[2];
  float* pub_beps[2];
  const int* gate;  // step gate (AqlLearn::gate); the step index is aql_update's gate_j
};
void aql_step_check(const AqlStep& d);
int aql_update_grid(const AqlStep& d, int* noise_blocks);
void aql_update(const AqlStep* dev, int grid, int noise_blocks, hipStream_t s, int gate_j = 0);
struct AqlEnv {
  int kind;            // 0 BipedalWalker-shaped, 1 CartPole, 2 Pendulum
  int E, obs, adim, T, max_steps;
  float* obs_buf;      // [E][obs]
  float* phys;         // [E][4] internal state (CartPole, Pendulum)
  int* ep_len;
  float* ep_ret;
  const float *dynA, *dynB, *dynw;  // BipedalWalker-shaped dynamics [24][24], [24][4], [24]
  uint64_t seed;
  const int64_t* counter;           // actor step counter (Philox)
  int* ep_count;                    // finished episodes (monotone)
  float* ep_log;                    // [log_cap][2] (return, length) ring
  int log_cap;
};
struct AqlInsert {
  float *st, *st2, *rew, *done, *amu;
  int* act;
  int64_t C;
  const int64_t* filled;
  int* slots;          // [E] out: ring slots written this step
};
void aql_env_reset(const AqlEnv& e, hipStream_t s);
void aql_env_step(const AqlEnv& e, const float* env_act, const int* act_idx, const float* amu, const AqlInsert& ins,
                  hipStream_t s);
// the serial engine's acting tail: eps-greedy select + env step + ring tree write + counter bumps
// (+ the learner's PER beta) in one launch (aql_engine_kernels.hip aql_act_tail_k)
struct AqlTail {
  AqlEnv V;
  AqlInsert I;         // the replay ring (I.filled is read; `filled` below is bumped)
  TreeDesc tree;
  const float *q, *amu, *eps;  // candidate Q [E][T], candidates [E][T][adim], per-env epsilon
  uint64_t sel_seed;
  int* act_idx;
  float* env_act;
  float alpha;
  const float* max_prio;
  int64_t* filled;     // += E by the last workgroup
  int64_t* counter;    // acting counter (V.counter), += 1 by the last workgroup
  int* ticket;         // zero between launches
  float* beta_out;     // optional: beta_start + iter (1 - beta_start) / max_step * workers, min 1
  int64_t* iter;       // iterations so far (+= 1 by the last workgroup)
  double beta0, beta_omb, beta_max_step, beta_workers;
};
void aql_act_tail(const AqlTail& a, hipStream_t s);
// rows 0..E-1 of the staging tables ``src`` -> ring slots (dst.filled + e) % dst.C (slot list in dst.slots)
void aql_apply_staged(const AqlInsert& src, const AqlInsert& dst, int E, int obs, int TA, hipStream_t s);

// ---- central-replay experience transport over HIP IPC (ipc_kernels.hip, parallel/ipc.py)
struct IpcIngest {
  int kind;                         // 0: Ape-X DQN packets (frames + rows into per-link regions)
                                    // 1: AQL packets (SoA rows appended to one global replay ring)
  int R, D, E, cap;                 // actor links, ring depth, envs per packet, packets per link per ingest
  int64_t packet_bytes;             // ring slot stride (DQN: >= E * (7056 + 56); AQL: >= E * (2 obs + TA + 3) * 4)
  int* prefix;                      // [R] scratch: ready packets of the links before r (AQL ring order)
  int obs, TA;                      // AQL: state width, candidates x action dims
  AqlInsert aql;                    // AQL: destination tables; ring slot (aql.filled + row) % aql.C
  const uint8_t* ring;              // [R][D] packets (uncached arena)
  const int64_t* seq;               // [R][D] packet number + 1 held by each slot
  int64_t* consumed;                // [R] packets applied so far (device)
  int* ready;                       // [R] scratch: packets applied by this ingest
  const int* live;                  // [R] 0 = link dropped (optional)
  int64_t* host_consumed;           // [R] device view of the host control block (credit; optional)
  int64_t* applied;                 // [R] statistics (optional)
  int64_t* filled;                  // replay fill counter (DQN: += real rows; AQL: += E per packet)
  uint8_t* frames;                  // replay frame ring [F][7056]
  int32_t *s_ids, *s2_ids, *action; // [C][4], [C][4], [C]
  float *reward, *done;             // [C]
  const int64_t *frame_base, *slot_base;  // [R] region offsets
  int32_t* slots_out;               // [R * cap * E] global slot or -1 (tree write input)
  float* prio_out;                  // [R * cap * E]
  // AQL step gate (optional): the reference trains total_rows // batch SGD steps per recorded
  // batch (AQL_dis.py:117-118) -- budget += rows applied, gate = min(gate_max, budget // batch),
  // budget -= gate * batch; the learner's step j runs iff j < gate (AqlLearn::gate)
  int64_t* budget;
  int* gate;
  int gate_batch, gate_max;
};
void ipc_ingest(const IpcIngest& g, hipStream_t s);
// An actor rank's packet for one actor step (Ape-X DQN, ONE launch): E new frames copied out of
// the local frame ring + E metadata rows gathered from the local mirror's transition tables at
// the rows' slots (kMetaCols = 14: s_ids 4 | s2_ids 4 | action | reward | done | priority | slot
// | new-frame slot).  initial = 1: the reset-frame packet (rows from `hist` / `actions`, slot -1).
struct IpcStage {
  const uint8_t* frames;            // local frame ring [F][7056]
  const int32_t* new_frame;         // [E] local frame slot of each env's new frame
  const int32_t *s_ids, *s2_ids;    // local mirror tables [C][4]
  const int32_t* action;            // [C]
  const float *reward, *done;       // [C]
  const int32_t* slot;              // [E] local transition slot of each env's row (-1: none)
  const float* prio;                // [E] actor priority
  const int32_t* hist;              // initial: [E][4] current stacks (both s and s')
  const int32_t* actions;           // initial: [E]
  uint8_t* packet;                  // E frames | E x 14 meta
  int E, initial;
};
void ipc_stage_dqn(const IpcStage& st, hipStream_t s);
// In-process emulation of R actor links (bench.py --emulate-links): every call pushes one
// synthetic packet per link whose credit window (D) allows it, straight into the learner's ring
// slot (the bytes an actor's xGMI peer copy would land), then stores the slot's sequence word --
// the same release protocol the ingest acquires.  Packet n of link r: frames from a pool,
// rows at local slots (n E + e) mod C_r with frame ids inside the link's region.
struct IpcEmu {
  uint8_t* ring;                    // [R][D] packet slots (stride pkt)
  int64_t* seq;                     // [R][D]
  const int64_t* consumed;          // [R] the ingest's device counters (credit)
  int64_t* sent;                    // [R] packets pushed (device)
  int32_t* go;                      // [R] scratch: this call's decision per link
  const uint8_t* pool;              // [pool_n][7056] frame pool
  int pool_n, R, D, E, C_r, F_r, n_actions;
  int64_t pkt;                      // ring slot stride
  uint64_t seed;
};
void ipc_emu_push(const IpcEmu& e, hipStream_t s);
void ipc_flag(int64_t* p, int64_t v, hipStream_t s);  // system-scope release store of v (one thread)
// The pinned parameter publish (parallel/ipc.py): at execution time pick buffer b of K -- not
// the current word's (word & 0xFF), not any reader's pinned word's -- store begin[b] = v, copy
// src [P] into params + b stride_f, then release word = v << 8 | b.  ctrl: the control block's
// device address (int64 words); pin_off / begin_off / word 2: word offsets.
void ipc_param_publish(int64_t* ctrl, int pin_off, int R, int begin_off, int K, float* params, int64_t stride_f,
                       const float* src, int64_t P, int64_t v, int* pick, hipStream_t s);

}  // namespace apex
