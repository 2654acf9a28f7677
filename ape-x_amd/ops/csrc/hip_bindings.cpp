// pybind11 bindings for the gfx950 kernel library `_apex_hip`.
//
// Pointers cross the boundary as integers (torch `tensor.data_ptr()`) and the stream
// as `torch.cuda.current_stream().cuda_stream`; descriptor structs are built once in
// Python and held by small handle classes so each per-step call is a plain function
// call with scalars (sub-microsecond binding overhead, graph-capturable launches).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <optional>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace py = pybind11;
using namespace apex;

namespace {

template <typename T>
T* P(uint64_t v) {
  return reinterpret_cast<T*>(static_cast<uintptr_t>(v));
}
hipStream_t S(uint64_t v) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(v)); }

struct TreeHandle {
  TreeDesc d{};
};

TreeHandle make_tree(uint64_t leaf_sum, uint64_t leaf_min, const std::vector<uint64_t>& node_sum,
                     const std::vector<uint64_t>& node_min, const std::vector<int>& sizes) {
  TreeHandle h;
  if (node_sum.size() != node_min.size() || sizes.size() != node_sum.size() + 1)
    throw std::invalid_argument("tree: inconsistent level lists");
  if ((int)node_sum.size() > kMaxTreeLevels || node_sum.empty()) throw std::invalid_argument("tree: bad level count");
  h.d.leaf_sum = P<float>(leaf_sum);
  h.d.leaf_min = P<float>(leaf_min);
  h.d.levels = (int)node_sum.size();
  for (size_t i = 0; i < node_sum.size(); ++i) {
    h.d.node_sum[i] = P<double>(node_sum[i]);
    h.d.node_min[i] = P<float>(node_min[i]);
  }
  for (size_t i = 0; i < sizes.size(); ++i) h.d.size[i] = sizes[i];
  for (size_t i = 1; i < sizes.size(); ++i)
    if (sizes[i] != (sizes[i - 1] + kTreeFanout - 1) / kTreeFanout) throw std::invalid_argument("tree: bad sizes");
  if (sizes.back() != 1) throw std::invalid_argument("tree: top level must have one node");
  return h;
}

BatchWrite batch_write(uint64_t pre_idx, uint64_t pre_prio, int E, uint64_t pre_bump, uint64_t idx, uint64_t prio,
                       int B, uint64_t mix_delta, uint64_t mix_lw, uint64_t mix_prio_out, uint64_t mix_loss_out,
                       uint64_t bump, uint64_t owner, uint64_t list, uint64_t max_prio, float alpha) {
  BatchWrite w{};
  w.pre_idx = P<const int>(pre_idx);
  w.pre_prio = P<const float>(pre_prio);
  w.E = E;
  w.pre_bump = P<int64_t>(pre_bump);
  w.idx = P<const int>(idx);
  w.prio = P<const float>(prio);
  w.B = B;
  w.mix = PrioMix{P<const float>(mix_delta), P<const float>(mix_lw), P<float>(mix_prio_out), P<float>(mix_loss_out)};
  w.bump = P<int64_t>(bump);
  w.owner = P<int>(owner);
  w.list = P<int>(list);
  w.max_prio = P<float>(max_prio);
  w.alpha = alpha;
  return w;
}

const TreeRide* ride_of(const py::object& o) { return o.is_none() ? nullptr : o.cast<const TreeRide*>(); }

TransTable trans_table(py::dict d) {
  auto g = [&](const char* k) { return d[k].cast<uint64_t>(); };
  return TransTable{P<int>(g("s_ids")), P<int>(g("s2_ids")), P<int>(g("action")), P<float>(g("reward")),
                    P<float>(g("done"))};
}

struct NStepHandle {
  NStepParams p{};
  NStepState st{};
  TransTable tt{};
};

}  // namespace

void register_comm(py::module_& m);  // comm.cpp (direct RCCL)
void register_ipc(py::module_& m);   // ipc.cpp (HIP IPC experience transport)

PYBIND11_MODULE(_apex_hip, m) {
  register_comm(m);
  register_ipc(m);
  m.doc() = "apex_amd gfx950 kernels (HBM replay, actor shard, fused learner)";
  m.attr("arch") = "gfx950";

  py::class_<TreeHandle>(m, "TreeHandle").def_property_readonly("levels", [](const TreeHandle& h) {
    return h.d.levels;
  });
  m.def("make_tree", &make_tree);
  m.def("per_write_batch", [](const TreeHandle& t, uint64_t pre_idx, uint64_t pre_prio, int E, uint64_t pre_bump,
                              uint64_t idx, uint64_t prio, int B, uint64_t mix_delta, uint64_t mix_lw,
                              uint64_t mix_prio_out, uint64_t mix_loss_out, uint64_t bump, uint64_t owner,
                              uint64_t list, uint64_t max_prio, float alpha, uint64_t ticket, uint64_t s) {
    const BatchWrite w = batch_write(pre_idx, pre_prio, E, pre_bump, idx, prio, B, mix_delta, mix_lw, mix_prio_out,
                                     mix_loss_out, bump, owner, list, max_prio, alpha);
    per_write_batch(t.d, w, P<int>(ticket), S(s));
  });
  // the batched write as riders of the learner's backward launches (f32_fc1_bwd_split /
  // f32_conv_bwd ride=): stage 1 leaves, stage 2 level `level`, stage 3 levels top_from.. in
  // one workgroup
  py::class_<TreeRide>(m, "TreeRide")
      .def_readonly("stage", &TreeRide::stage)
      .def_readonly("level", &TreeRide::level)
      .def_readonly("top_from", &TreeRide::top_from)
      .def_property_readonly("blocks", [](const TreeRide& r) { return tree_ride_blocks(r); });
  m.def("make_tree_ride", [](const TreeHandle& t, int stage, int level, int top_from, uint64_t pre_idx,
                             uint64_t pre_prio, int E, uint64_t pre_bump, uint64_t idx, int B, uint64_t mix_delta,
                             uint64_t mix_lw, uint64_t mix_prio_out, uint64_t mix_loss_out, uint64_t bump,
                             uint64_t owner, uint64_t list, uint64_t max_prio, float alpha) {
    TreeRide r{};
    r.t = t.d;
    r.w = batch_write(pre_idx, pre_prio, E, pre_bump, idx, 0, B, mix_delta, mix_lw, mix_prio_out, mix_loss_out, bump,
                      owner, list, max_prio, alpha);
    r.stage = stage;
    r.level = level;
    r.top_from = top_from;
    if (stage < 1 || stage > 3)
      throw std::invalid_argument("make_tree_ride: stage 1 (leaves), 2 (a level) or 3 (the top levels)");
    if (stage == 3 && (top_from < 1 || top_from > t.d.levels || t.d.size[top_from] > 64))
      throw std::invalid_argument("make_tree_ride: the top walk starts at a level in 1..levels of <= 64 nodes");
    if (E < 0 || B < 0 || E + B > 2048 || (E > 0 && (!pre_idx || !pre_prio)) || (B > 0 && !idx))
      throw std::invalid_argument("make_tree_ride: 0 <= E + B <= 2048 with their slots / priorities");
    if (!owner || !list || !max_prio || (mix_delta && !mix_lw) || (B > 0 && !mix_delta))
      throw std::invalid_argument("make_tree_ride: owner, list, max_prio and the learner mix (delta + lw)");
    if (stage == 2 && (level < 1 || level > t.d.levels))
      throw std::invalid_argument("make_tree_ride: level in 1..levels");
    return r;
  });
  m.def("tree_ride_level_stages", [](const TreeHandle& t) { return tree_ride_level_stages(t.d); });
  m.def("pack_shard_slots", [](const TreeHandle& t, uint64_t slots, int world, int rank, uint64_t s) {
    pack_shard_slots(t.d, P<float>(slots), world, rank, S(s));
  });

  // ---- replay
  m.def("per_write_leaves", [](const TreeHandle& t, uint64_t idx, uint64_t prio, int B, float alpha,
                               uint64_t max_prio, int dedup, uint64_t sorted_scratch, uint64_t bump0, int64_t d0,
                               uint64_t bump1, int64_t d1, uint64_t s, uint64_t mix_delta, uint64_t mix_lw,
                               uint64_t mix_prio_out, uint64_t mix_loss_out) {
    per_write_leaves(t.d, P<const int>(idx), P<const float>(prio), B, alpha, P<float>(max_prio), dedup,
                     P<int>(sorted_scratch), P<int64_t>(bump0), d0, P<int64_t>(bump1), d1, S(s),
                     P<const float>(mix_delta), P<const float>(mix_lw), P<float>(mix_prio_out), P<float>(mix_loss_out));
  }, py::arg("t"), py::arg("idx"), py::arg("prio"), py::arg("B"), py::arg("alpha"), py::arg("max_prio"),
     py::arg("dedup"), py::arg("sorted_scratch"), py::arg("bump0"), py::arg("d0"), py::arg("bump1"), py::arg("d1"),
     py::arg("s"), py::arg("mix_delta") = 0, py::arg("mix_lw") = 0, py::arg("mix_prio_out") = 0,
     py::arg("mix_loss_out") = 0);
  m.def("per_sample", [](const TreeHandle& t, int B, uint64_t length_ptr, int64_t length, uint64_t beta_ptr,
                         float beta, uint64_t seed, uint64_t counter, uint64_t out_idx, uint64_t out_w,
                         int exclude_last, uint64_t s, uint64_t glob, uint64_t gathered, int world, int rank,
                         py::object rows_stage, py::object rows_dst, uint64_t rows_slot, uint64_t rows_prio,
                         int rows_E, py::object src, py::object out) {
    auto tab = trans_table;
    StagedRows rows{};
    if (rows_E > 0)
      rows = StagedRows{tab(rows_stage.cast<py::dict>()), tab(rows_dst.cast<py::dict>()), P<const int>(rows_slot),
                        P<const float>(rows_prio), rows_E};
    SampleRowsOut ro{};
    if (!out.is_none()) ro = SampleRowsOut{tab(src.cast<py::dict>()), tab(out.cast<py::dict>())};
    per_sample(t.d, B, P<const int64_t>(length_ptr), length, P<const float>(beta_ptr), beta, seed,
               P<const int64_t>(counter), P<int>(out_idx), P<float>(out_w), exclude_last, P<const float>(glob), S(s),
               ShardGlob{P<const float>(gathered), world, rank}, rows_E > 0 ? &rows : nullptr,
               out.is_none() ? nullptr : &ro);
  }, py::arg("t"), py::arg("B"), py::arg("length_ptr"), py::arg("length"), py::arg("beta_ptr"), py::arg("beta"),
     py::arg("seed"), py::arg("counter"), py::arg("out_idx"), py::arg("out_w"), py::arg("exclude_last"),
     py::arg("s"), py::arg("glob") = 0, py::arg("slots") = 0, py::arg("world") = 0, py::arg("rank") = 0,
     py::arg("rows_stage") = py::none(), py::arg("rows_dst") = py::none(), py::arg("rows_slot") = 0,
     py::arg("rows_prio") = 0, py::arg("rows_E") = 0, py::arg("src") = py::none(), py::arg("out") = py::none());
  m.def("gather_transitions", [](uint64_t frames, int frame_bytes, uint64_t s_ids, uint64_t s2_ids, uint64_t act,
                                 uint64_t rew, uint64_t done, uint64_t idx, int B, uint64_t out_s, uint64_t out_s2,
                                 uint64_t out_a, uint64_t out_r, uint64_t out_d, uint64_t s) {
    gather_transitions(P<const uint8_t>(frames), frame_bytes, P<const int>(s_ids), P<const int>(s2_ids),
                       P<const int>(act), P<const float>(rew), P<const float>(done), P<const int>(idx), B,
                       P<uint8_t>(out_s), P<uint8_t>(out_s2), P<int>(out_a), P<float>(out_r), P<float>(out_d),
                       S(s));
  });
  m.def("gather_frames", [](uint64_t frames, int frame_bytes, uint64_t ids, int N, int stack, uint64_t out,
                            uint64_t s) {
    gather_frames(P<const uint8_t>(frames), frame_bytes, P<const int>(ids), N, stack, P<uint8_t>(out), S(s));
  });
  m.def("frame_hist_step", [](uint64_t hist, uint64_t new_frame, uint64_t done, int E, uint64_t counter, uint64_t s) {
    frame_hist_step(P<int>(hist), P<const int>(new_frame), P<const float>(done), E, P<int64_t>(counter), S(s));
  });
  m.def("bump_counter", [](uint64_t c, int n, int64_t by, uint64_t s) { bump_counter(P<int64_t>(c), n, by, S(s)); });

  // ---- actor shard
  py::class_<VecEnvParams>(m, "VecEnvParams")
      .def(py::init([](int E, int A, int frame_bytes, int F, int repeat, int clip, int life, int max_steps) {
             VecEnvParams p{E, A, frame_bytes, F, repeat, clip, life, max_steps};
             return p;
           }),
           py::arg("E"), py::arg("n_actions"), py::arg("frame_bytes"), py::arg("F"), py::arg("action_repeat") = 4,
           py::arg("clip_rewards") = 1, py::arg("episode_life") = 1, py::arg("max_episode_steps") = 50000)
      .def_readonly("E", &VecEnvParams::E)
      .def_readonly("F", &VecEnvParams::F);
  m.def("vec_env_reset", [](uint64_t state, uint64_t seed, uint64_t frames, const VecEnvParams& p, uint64_t step,
                            uint64_t new_frame, uint64_t hist, uint64_t ep_log, uint64_t s) {
    vec_env_reset(P<float>(state), seed, P<uint8_t>(frames), p, P<const int64_t>(step), P<int>(new_frame),
                  P<int>(hist), P<float>(ep_log), S(s));
  });
  m.def("vec_env_step", [](uint64_t state, uint64_t actions, uint64_t seed, uint64_t step, uint64_t frames,
                           const VecEnvParams& p, uint64_t reward, uint64_t done, uint64_t new_frame, uint64_t ep_log,
                           uint64_t s) {
    vec_env_step(P<float>(state), P<const int>(actions), seed, P<const int64_t>(step), P<uint8_t>(frames), p,
                 P<float>(reward), P<float>(done), P<int>(new_frame), P<float>(ep_log), S(s));
  });
  m.def("select_actions", [](uint64_t q, int E, int A, uint64_t eps, uint64_t seed, uint64_t counter,
                             uint64_t actions, uint64_t s) {
    select_actions(P<const float>(q), E, A, P<const float>(eps), seed, P<const int64_t>(counter), P<int>(actions),
                   S(s));
  });

  py::class_<NStepHandle>(m, "NStepHandle");
  m.def("make_nstep", [](int E, int A, int n, int C, float gamma, int mode, py::dict st, py::dict tt, int stage) {
    NStepHandle h;
    h.p = NStepParams{E, A, n, C, gamma, mode, stage};
    auto g = [&](py::dict d, const char* k) { return d[k].cast<uint64_t>(); };
    h.st.win_ids = P<int>(g(st, "win_ids"));
    h.st.win_a = P<int>(g(st, "win_a"));
    h.st.win_r = P<float>(g(st, "win_r"));
    h.st.win_q = P<float>(g(st, "win_q"));
    h.st.win_meta = P<int>(g(st, "win_meta"));
    h.st.hist = P<int>(g(st, "hist"));
    h.st.drain_ids = P<int>(g(st, "drain_ids"));
    h.st.drain_a = P<int>(g(st, "drain_a"));
    h.st.drain_r = P<float>(g(st, "drain_r"));
    h.st.drain_q = P<float>(g(st, "drain_q"));
    h.st.drain_meta = P<int>(g(st, "drain_meta"));
    h.st.drain_s2 = P<int>(g(st, "drain_s2"));
    h.tt.s_ids = P<int>(g(tt, "s_ids"));
    h.tt.s2_ids = P<int>(g(tt, "s2_ids"));
    h.tt.action = P<int>(g(tt, "action"));
    h.tt.reward = P<float>(g(tt, "reward"));
    h.tt.done = P<float>(g(tt, "done"));
    return h;
  }, py::arg("E"), py::arg("A"), py::arg("n"), py::arg("C"), py::arg("gamma"), py::arg("mode"), py::arg("st"),
     py::arg("tt"), py::arg("stage") = 0);
  m.def("apply_staged_rows", [](py::dict st, py::dict dst, uint64_t slot, uint64_t prio, int E, uint64_t s) {
    auto tab = [](py::dict d) {
      auto g = [&](const char* k) { return d[k].cast<uint64_t>(); };
      return TransTable{P<int>(g("s_ids")), P<int>(g("s2_ids")), P<int>(g("action")), P<float>(g("reward")),
                        P<float>(g("done"))};
    };
    apply_staged_rows(tab(st), tab(dst), P<const int>(slot), P<const float>(prio), E, S(s));
  });
  m.def("nstep_emit", [](const NStepHandle& h, uint64_t q, uint64_t actions, uint64_t reward, uint64_t done,
                         uint64_t new_frame, uint64_t step, uint64_t slot_out, uint64_t prio_out, uint64_t s,
                         bool bump) {
    nstep_emit(h.p, h.st, h.tt, P<const float>(q), P<const int>(actions), P<const float>(reward),
               P<const float>(done), P<const int>(new_frame), P<int64_t>(step), P<int>(slot_out),
               P<float>(prio_out), S(s), bump);
  }, py::arg("h"), py::arg("q"), py::arg("actions"), py::arg("reward"), py::arg("done"), py::arg("new_frame"),
     py::arg("step"), py::arg("slot_out"), py::arg("prio_out"), py::arg("s"), py::arg("bump") = false);

  // ---- learner
  m.def("dqn_loss", [](uint64_t q, uint64_t q2, uint64_t q2t, int ldq, uint64_t a, uint64_t r, uint64_t d,
                       uint64_t idx, uint64_t w, int B, int A, float gamma_n, uint64_t loss, uint64_t dq,
                       uint64_t prio, uint64_t s) {
    dqn_loss(P<const float>(q), P<const float>(q2), P<const float>(q2t), ldq, P<const int>(a), P<const float>(r),
             P<const float>(d), P<const int>(idx), P<const float>(w), B, A, gamma_n, P<float>(loss), P<float>(dq),
             P<float>(prio), S(s));
  });
  m.def("grad_sumsq", [](uint64_t g, int64_t n, uint64_t partials, uint64_t s) {
    grad_sumsq(P<const float>(g), n, P<double>(partials), S(s));
  });
  m.def("grad_norm_partials", &grad_norm_partials);
  py::class_<RMSpropParams>(m, "RMSpropParams")
      .def(py::init([](float lr, float alpha, float eps, float max_norm, float lr_gamma, int lr_step_size,
                       int lr_step_offset, bool centered) {
             return RMSpropParams{lr, alpha, eps, max_norm, lr_gamma, lr_step_size, lr_step_offset, centered ? 1 : 0};
           }),
           py::arg("lr"), py::arg("alpha") = 0.99f, py::arg("eps") = 1e-8f, py::arg("max_norm") = 0.f,
           py::arg("lr_gamma") = 1.f, py::arg("lr_step_size") = 0, py::arg("lr_step_offset") = 0,
           py::arg("centered") = false)
      .def_readwrite("grad_scale", &RMSpropParams::grad_scale);
  m.def("rmsprop_step", [](uint64_t p, uint64_t g, uint64_t sq, uint64_t gavg, int64_t n, uint64_t partials,
                           int n_partials, const RMSpropParams& hp, uint64_t step, uint64_t norms, uint64_t s,
                           uint64_t dst1, uint64_t dst2, uint64_t arena, int64_t fc_off0, int64_t fc_off1,
                           uint64_t fc_wp, uint64_t fc_wt, uint64_t arena_f32, uint64_t fc_wp_f32) {
    const PackMap pk{P<const int>(dst1), P<const int>(dst2), P<uint16_t>(arena), P<float>(arena_f32)};
    const FcPack fc{{fc_off0, fc_off1}, P<uint16_t>(fc_wp), P<uint16_t>(fc_wt), P<float>(fc_wp_f32)};
    rmsprop_step(P<float>(p), P<const float>(g), P<float>(sq), P<float>(gavg), n, P<const double>(partials),
                 n_partials, hp, P<const int64_t>(step), P<float>(norms), S(s), (arena || arena_f32) ? &pk : nullptr,
                 (fc_wp || fc_wp_f32) ? &fc : nullptr);
  }, py::arg("p"), py::arg("g"), py::arg("sq"), py::arg("gavg"), py::arg("n"), py::arg("partials"),
     py::arg("n_partials"), py::arg("hp"), py::arg("step"), py::arg("norms"), py::arg("s"), py::arg("dst1") = 0,
     py::arg("dst2") = 0, py::arg("arena") = 0, py::arg("fc_off0") = -1, py::arg("fc_off1") = -1,
     py::arg("fc_wp") = 0, py::arg("fc_wt") = 0, py::arg("arena_f32") = 0, py::arg("fc_wp_f32") = 0);
  py::class_<AdamParams>(m, "AdamParams")
      .def(py::init([](float lr, float b1, float b2, float eps, float wd, float max_norm, float lr_gamma,
                       int lr_step_size, int lr_step_offset) {
             return AdamParams{lr, b1, b2, eps, wd, max_norm, lr_gamma, lr_step_size, lr_step_offset};
           }),
           py::arg("lr"), py::arg("beta1") = 0.9f, py::arg("beta2") = 0.999f, py::arg("eps") = 1e-8f,
           py::arg("weight_decay") = 0.f, py::arg("max_norm") = 0.f, py::arg("lr_gamma") = 1.f,
           py::arg("lr_step_size") = 0, py::arg("lr_step_offset") = 0)
      .def_readwrite("grad_scale", &AdamParams::grad_scale);
  m.def("adam_step", [](uint64_t p, uint64_t g, uint64_t mm, uint64_t v, int64_t n, uint64_t partials,
                        int n_partials, const AdamParams& hp, uint64_t step, uint64_t norms, uint64_t s,
                        uint64_t dst1, uint64_t dst2, uint64_t arena, int64_t fc_off0, int64_t fc_off1,
                        uint64_t fc_wp, uint64_t fc_wt, uint64_t arena_f32, uint64_t fc_wp_f32) {
    const PackMap pk{P<const int>(dst1), P<const int>(dst2), P<uint16_t>(arena), P<float>(arena_f32)};
    const FcPack fc{{fc_off0, fc_off1}, P<uint16_t>(fc_wp), P<uint16_t>(fc_wt), P<float>(fc_wp_f32)};
    adam_step(P<float>(p), P<const float>(g), P<float>(mm), P<float>(v), n, P<const double>(partials), n_partials,
              hp, P<const int64_t>(step), P<float>(norms), S(s), (arena || arena_f32) ? &pk : nullptr,
              (fc_wp || fc_wp_f32) ? &fc : nullptr);
  }, py::arg("p"), py::arg("g"), py::arg("mm"), py::arg("v"), py::arg("n"), py::arg("partials"),
     py::arg("n_partials"), py::arg("hp"), py::arg("step"), py::arg("norms"), py::arg("s"), py::arg("dst1") = 0,
     py::arg("dst2") = 0, py::arg("arena") = 0, py::arg("fc_off0") = -1, py::arg("fc_off1") = -1,
     py::arg("fc_wp") = 0, py::arg("fc_wt") = 0, py::arg("arena_f32") = 0, py::arg("fc_wp_f32") = 0);
  m.def("adam_step2", [](std::array<uint64_t, 8> a, std::array<uint64_t, 8> b, const AdamParams& hp, uint64_t step,
                         uint64_t s) {
    // (p, g, m, v, n, partials, n_partials, norms) per set
    auto mk = [](const std::array<uint64_t, 8>& t) {
      return OptSet{P<float>(t[0]), P<const float>(t[1]), P<float>(t[2]), P<float>(t[3]), (int64_t)t[4],
                    P<const double>(t[5]), (int)t[6], P<float>(t[7]), 0};
    };
    adam_step2(mk(a), mk(b), hp, P<const int64_t>(step), S(s));
  });
  // ---- network kernels
  m.def("conv_fwd", [](int layer, uint64_t in, uint64_t ids, uint64_t idx, uint64_t wp, uint64_t bias, uint64_t out,
                       int B, uint64_t s) {
    conv_fwd(layer, P<const void>(in), P<const int>(ids), P<const int>(idx), P<const uint16_t>(wp),
             P<const float>(bias), P<uint16_t>(out), B, S(s));
  });
  m.def("heads_wgrad", [](uint64_t dA, uint64_t h, uint64_t dz, int B, int A, uint64_t ws, uint64_t gwa, uint64_t gba,
                          uint64_t gwv, uint64_t gbv, uint64_t gba1, uint64_t gbv1, uint64_t s) {
    heads_wgrad(P<const float>(dA), P<const float>(h), P<const float>(dz), B, A, P<float>(ws), P<float>(gwa),
                P<float>(gba), P<float>(gwv), P<float>(gbv), P<float>(gba1), P<float>(gbv1), S(s));
  });
  m.def("heads_wgrad_workspace_floats", &heads_wgrad_workspace_floats);
  // multi-problem forward launches: lists of per-problem pointer tuples (<= 3 problems)
  m.def("conv_fwd_multi", [](int layer, const std::vector<std::array<uint64_t, 6>>& probs, int B, uint64_t s) {
    if (probs.empty() || probs.size() > (size_t)kMaxProbs) throw std::invalid_argument("1..3 problems");
    ConvSet set{};
    for (size_t i = 0; i < probs.size(); ++i) {
      const auto& t = probs[i];
      set.p[i] = ConvProb{P<const void>(t[0]), P<const int>(t[1]), P<const int>(t[2]), P<const uint16_t>(t[3]),
                          P<const float>(t[4]), P<uint16_t>(t[5])};
    }
    set.n = (int)probs.size();
    set.B = B;
    conv_fwd_multi(layer, set, S(s));
  });
  m.def("fc1_fwd_multi", [](const std::vector<std::array<uint64_t, 3>>& probs, int B, uint64_t s) -> int {
    if (probs.empty() || probs.size() > (size_t)kMaxProbs) throw std::invalid_argument("1..3 problems");
    FcSet set{};
    for (size_t i = 0; i < probs.size(); ++i)
      set.p[i] = FcProb{P<const uint16_t>(probs[i][0]), P<const uint16_t>(probs[i][1]), P<float>(probs[i][2])};
    set.n = (int)probs.size();
    set.B = B;
    return fc1_fwd_multi(set, S(s));
  });
  m.def("heads_fwd_multi", [](const std::vector<std::array<uint64_t, 9>>& probs, int nsplit, int B, int A,
                              uint64_t s, std::optional<std::array<uint64_t, 4>> act) {
    if (probs.empty() || probs.size() > (size_t)kMaxProbs) throw std::invalid_argument("1..3 problems");
    HeadsSet set{};
    for (size_t i = 0; i < probs.size(); ++i) {
      const auto& t = probs[i];
      set.p[i] = HeadsProb{P<const float>(t[0]), P<const float>(t[1]), P<const float>(t[2]), P<const float>(t[3]),
                           P<const float>(t[4]), P<const float>(t[5]), P<const float>(t[6]), P<float>(t[7]),
                           P<float>(t[8])};
    }
    set.n = (int)probs.size();
    set.B = B;
    set.A = A;
    set.nsplit = nsplit;
    if (act) {  // (eps, rng seed, counter, actions): eps-greedy epilogue on problem 0
      const auto& a = *act;
      set.act = ActSel{P<const float>(a[0]), P<const int64_t>(a[2]), P<int>(a[3]), a[1]};
    }
    heads_fwd_multi(set, S(s));
  }, py::arg("probs"), py::arg("nsplit"), py::arg("B"), py::arg("A"), py::arg("s"), py::arg("act") = py::none());
  m.def("fc1_splits", &fc1_splits);
  m.def("fc1_fwd", [](uint64_t a, uint64_t w, uint64_t part, int B, uint64_t s) {
    return fc1_fwd(P<const uint16_t>(a), P<const uint16_t>(w), P<float>(part), B, S(s));
  });
  m.def("fc1_splits_for", &fc1_splits_for);
  m.def("heads_fwd", [](uint64_t z, int nsplit, uint64_t ba1, uint64_t bv1, uint64_t wa2, uint64_t ba2, uint64_t wv2,
                        uint64_t bv2, uint64_t hout, uint64_t q, int B, int A, uint64_t s) {
    heads_fwd(P<const float>(z), nsplit, P<const float>(ba1), P<const float>(bv1), P<const float>(wa2), P<const float>(ba2),
              P<const float>(wv2), P<const float>(bv2), P<float>(hout), P<float>(q), B, A, S(s));
  });
  m.def("heads_bwd", [](uint64_t dq, uint64_t h, uint64_t wa2, uint64_t wv2, uint64_t dA, uint64_t dz, uint64_t dzb,
                        int B, int A, uint64_t s) {
    heads_bwd(P<const float>(dq), P<const float>(h), P<const float>(wa2), P<const float>(wv2), P<float>(dA),
              P<float>(dz), P<uint16_t>(dzb), B, A, S(s));
  });
  m.def("pack_conv_w", [](uint64_t src, uint64_t dst, int N, int C, int KH, int KW, uint64_t s) {
    pack_conv_w(P<const float>(src), P<uint16_t>(dst), N, C, KH, KW, S(s));
  });
  m.def("pack_fc1", [](uint64_t adv, uint64_t val, uint64_t dst, int Pp, int C, uint64_t s) {
    pack_fc1(P<const float>(adv), P<const float>(val), P<uint16_t>(dst), Pp, C, S(s));
  });
  m.def("unpack_fc1_grad", [](uint64_t gp, uint64_t ga, uint64_t gv, int Pp, int C, uint64_t s) {
    unpack_fc1_grad(P<const float>(gp), P<float>(ga), P<float>(gv), Pp, C, S(s));
  });
  m.def("relu_mask_bf16", [](uint64_t g, uint64_t a, uint64_t out, int64_t n, uint64_t s) {
    relu_mask_bf16(P<const uint16_t>(g), P<const uint16_t>(a), P<uint16_t>(out), n, S(s));
  });
  m.def("u8_to_bf16_nhwc", [](uint64_t in, uint64_t out, int B, int HW, uint64_t s) {
    u8_to_bf16_nhwc(P<const uint8_t>(in), P<uint16_t>(out), B, HW, S(s));
  });
  m.def("conv_dgrad", [](int layer, uint64_t dy, uint64_t dy_mask, uint64_t wt, uint64_t dx, uint64_t dx_mask, int B,
                         uint64_t s) {
    conv_dgrad(layer, P<const uint16_t>(dy), P<const uint16_t>(dy_mask), P<const uint16_t>(wt), P<uint16_t>(dx),
               P<const uint16_t>(dx_mask), B, S(s));
  });
  m.def("wgrad_workspace_floats", &wgrad_workspace_floats);
  py::class_<FinalizeJob>(m, "FinalizeJob");
  m.def("conv_finalize_job", [](int layer, int B, uint64_t ws, uint64_t grad, uint64_t bias_grad) {
    return conv_finalize_job(layer, B, P<const float>(ws), P<float>(grad), P<float>(bias_grad));
  });
  m.def("heads_finalize_job", [](int G, int A, uint64_t part, uint64_t wadv2, uint64_t badv2, uint64_t wval2,
                                 uint64_t bval2, uint64_t badv1, uint64_t bval1) {
    return heads_finalize_job(G, A, P<const float>(part), P<float>(wadv2), P<float>(badv2), P<float>(wval2),
                              P<float>(bval2), P<float>(badv1), P<float>(bval1));
  });
  m.def("fc1_finalize_job", [](int half, uint64_t ws, uint64_t grad) {
    return fc1_finalize_job(half, P<const float>(ws), P<float>(grad));
  });
  m.def("fc1_bwd_slices", &fc1_bwd_slices);
  m.def("fc1_bwd_workspace_floats", &fc1_bwd_workspace_floats);
  m.def("fc1_bwd", [](uint64_t dz, uint64_t a3, uint64_t wt, uint64_t dy3, uint64_t part, int B, uint64_t s) {
    fc1_bwd(P<const uint16_t>(dz), P<const uint16_t>(a3), P<const uint16_t>(wt), P<uint16_t>(dy3), P<float>(part), B,
            S(s));
  });
  m.def("grad_finalize", [](const std::vector<FinalizeJob>& jobs, uint64_t s, uint64_t sumsq, py::object ride) {
    if (jobs.empty() || jobs.size() > (size_t)kMaxFinalizeJobs) throw std::invalid_argument("1..6 jobs");
    FinalizeSet fs{};
    for (size_t i = 0; i < jobs.size(); ++i) fs.job[i] = jobs[i];
    fs.n = (int)jobs.size();
    fs.sumsq = P<double>(sumsq);
    return grad_finalize(fs, S(s), ride_of(ride));
  }, py::arg("jobs"), py::arg("s"), py::arg("sumsq") = 0, py::arg("ride") = py::none());
  m.def("wgrad_grid", &wgrad_grid);
  m.def("dqn_heads_bwd_blocks", &dqn_heads_bwd_blocks);
  m.def("dqn_heads_bwd", [](py::dict d, int B, int A, float gamma_n, uint64_t s) {
    auto g = [&](const char* k) { return d.contains(k) ? d[k].cast<uint64_t>() : (uint64_t)0; };
    LossHeadsArgs a{};
    a.q = P<const float>(g("q"));
    a.q2 = P<const float>(g("q2"));
    a.q2t = P<const float>(g("q2t"));
    a.act = P<const int>(g("act"));
    a.rew = P<const float>(g("rew"));
    a.done = P<const float>(g("done"));
    a.idx = P<const int>(g("idx"));
    a.w = P<const float>(g("w"));
    a.h = P<const float>(g("h"));
    a.w_adv2 = P<const float>(g("w_adv2"));
    a.w_val2 = P<const float>(g("w_val2"));
    a.B = B;
    a.A = A;
    a.gamma_n = gamma_n;
    a.delta = P<float>(g("delta"));
    a.lw = P<float>(g("lw"));
    a.dz_bf = P<uint16_t>(g("dz_bf"));
    a.dz = P<float>(g("dz"));
    a.part = P<float>(g("part"));
    a.step = P<const int64_t>(g("step"));
    a.step_snap = P<int64_t>(g("step_snap"));
    if (!a.q || !a.q2 || !a.q2t || !a.act || !a.rew || !a.done || !a.w || !a.h || !a.w_adv2 || !a.w_val2 ||
        !a.delta || !a.lw || !(a.dz_bf || a.dz) || !a.part || !a.step)
      throw std::invalid_argument("dqn_heads_bwd: missing pointer");
    dqn_heads_bwd(a, S(s));
  });
  m.def("conv_wgrad", [](int layer, uint64_t x, uint64_t ids, uint64_t idx, uint64_t dy, uint64_t dy_mask, int B,
                         uint64_t ws, uint64_t grad, uint64_t bgrad, uint64_t s) {
    conv_wgrad(layer, P<const void>(x), P<const int>(ids), P<const int>(idx), P<const uint16_t>(dy),
               P<const uint16_t>(dy_mask), B, P<float>(ws), P<float>(grad), P<float>(bgrad), S(s));
  });
  m.def("pack_conv_wt", [](uint64_t src, uint64_t dst, int N, int C, int KH, int KW, uint64_t s) {
    pack_conv_wt(P<const float>(src), P<uint16_t>(dst), N, C, KH, KW, S(s));
  });
  // ---- fp32 (reference-precision) network kernels (f32_kernels.hip)
  // a problem: (in, ids, idx, w, w2, bias, out)
  auto f32set = [](const std::vector<std::vector<uint64_t>>& probs, int B) {
    if (probs.empty() || probs.size() > (size_t)kMaxProbs) throw std::invalid_argument("1..3 problems");
    F32Set set{};
    for (size_t i = 0; i < probs.size(); ++i) {
      const auto& t = probs[i];
      if (t.size() != 7) throw std::invalid_argument("f32 problem: 7 fields");
      set.p[i] = F32Prob{P<const void>(t[0]), P<const int>(t[1]), P<const int>(t[2]), P<const float>(t[3]),
                         P<const float>(t[4]), P<const float>(t[5]), P<float>(t[6])};
    }
    set.n = (int)probs.size();
    set.B = B;
    return set;
  };
  // probs: (in, ids, idx, w, w2, bias, out)
  m.def("f32_conv_fwd_multi", [f32set](int layer, const std::vector<std::vector<uint64_t>>& probs, int B,
                                       uint64_t s, int c1_grid, int tile, py::object draw) {
    f32_conv_fwd_multi(layer, f32set(probs, B), S(s), c1_grid, tile,
                       draw.is_none() ? nullptr : draw.cast<const ConvSample*>());
  }, py::arg("layer"), py::arg("probs"), py::arg("B"), py::arg("s"), py::arg("c1_grid") = 0, py::arg("tile") = 0,
     py::arg("draw") = py::none());
  // the learner's PER draw folded into the conv1 forward (f32_conv_fwd_multi(1, draw=)): the
  // per_sample arguments of the plain single-replay path (+ the staged actor rows it scatters)
  py::class_<ConvSample>(m, "ConvSample");
  m.def("make_conv_sample", [](const TreeHandle& t, uint64_t length_ptr, uint64_t beta_ptr, uint64_t seed,
                               uint64_t counter, uint64_t out_idx, uint64_t out_w, int exclude_last,
                               py::object rows_stage, py::object rows_dst, uint64_t rows_slot, uint64_t rows_prio,
                               int rows_E) {
    if (!length_ptr || !beta_ptr || !counter || !out_idx || !out_w)
      throw std::invalid_argument("make_conv_sample: fill level, beta, counter, idx and weight pointers");
    ConvSample c{};
    c.t = t.d;
    c.length = P<const int64_t>(length_ptr);
    c.beta = P<const float>(beta_ptr);
    c.counter = P<const int64_t>(counter);
    c.seed = seed;
    c.out_idx = P<int>(out_idx);
    c.out_w = P<float>(out_w);
    c.exclude_last = exclude_last;
    if (rows_E > 0) {
      if (!rows_slot || !rows_prio) throw std::invalid_argument("make_conv_sample: staged slots / priorities");
      c.rows = StagedRows{trans_table(rows_stage.cast<py::dict>()), trans_table(rows_dst.cast<py::dict>()),
                          P<const int>(rows_slot), P<const float>(rows_prio), rows_E};
    }
    return c;
  }, py::arg("t"), py::arg("length_ptr"), py::arg("beta_ptr"), py::arg("seed"), py::arg("counter"),
     py::arg("out_idx"), py::arg("out_w"), py::arg("exclude_last"), py::arg("rows_stage") = py::none(),
     py::arg("rows_dst") = py::none(), py::arg("rows_slot") = 0, py::arg("rows_prio") = 0, py::arg("rows_E") = 0);
  m.def("f32_fc1_fwd_multi", [f32set](const std::vector<std::vector<uint64_t>>& probs, int B, uint64_t s) {
    return f32_fc1_fwd_multi(f32set(probs, B), S(s));
  });
  m.def("f32_fc1_splits", &f32_fc1_splits);
  m.def("f32_set_stage_split", &f32_set_stage_split);
  m.def("f32_stage_split", &f32_stage_split);
  m.def("f32_fc1_bwd_split", [](uint64_t dz, uint64_t a3, uint64_t wfc1p, uint64_t dy3, uint64_t ws, int B,
                                uint64_t s, py::object ride) {
    f32_fc1_bwd_split(P<const float>(dz), P<const float>(a3), P<const float>(wfc1p), P<float>(dy3), P<float>(ws), B,
                      S(s), ride_of(ride));
  }, py::arg("dz"), py::arg("a3"), py::arg("wfc1p"), py::arg("dy3"), py::arg("ws"), py::arg("B"), py::arg("s"),
     py::arg("ride") = py::none());
  m.def("f32_fc1_wgrad_splits", &f32_fc1_wgrad_splits);
  m.def("f32_fc1_wgrad_slices", &f32_fc1_wgrad_slices);
  m.def("f32_fc1_wgrad_workspace_floats", &f32_fc1_wgrad_workspace_floats);
  m.def("f32_fc1_finalize_job", [](int half, int G, uint64_t ws, uint64_t grad) {
    return f32_fc1_finalize_job(half, G, P<const float>(ws), P<float>(grad));
  });
  m.def("f32_wgrad_splits", &f32_wgrad_splits, py::arg("layer"), py::arg("B"), py::arg("target") = 0);
  m.def("f32_wgrad_workspace_floats", &f32_wgrad_workspace_floats, py::arg("layer"), py::arg("B"),
        py::arg("target") = 0);
  m.def("f32_conv_bwd", [](int layer, uint64_t x, uint64_t ids, uint64_t idx, uint64_t dy, uint64_t w, uint64_t mask,
                           uint64_t dx, uint64_t ws, int B, uint64_t s, int target, int tile, py::object ride) {
    f32_conv_bwd(layer, P<const void>(x), P<const int>(ids), P<const int>(idx), P<const float>(dy), P<const float>(w),
                 P<const float>(mask), P<float>(dx), P<float>(ws), B, S(s), target, tile, ride_of(ride));
  }, py::arg("layer"), py::arg("x"), py::arg("ids"), py::arg("idx"), py::arg("dy"), py::arg("w"), py::arg("mask"),
     py::arg("dx"), py::arg("ws"), py::arg("B"), py::arg("s"), py::arg("target") = 0, py::arg("tile") = 0,
     py::arg("ride") = py::none());
  m.def("f32_conv_finalize_job", [](int layer, int B, uint64_t ws, uint64_t grad, uint64_t bgrad, int target) {
    return f32_conv_finalize_job(layer, B, P<const float>(ws), P<float>(grad), P<float>(bgrad), target);
  }, py::arg("layer"), py::arg("B"), py::arg("ws"), py::arg("grad"), py::arg("bgrad"), py::arg("target") = 0);
  m.def("norm_only_job", [](uint64_t g, int n) { return norm_only_job(P<const float>(g), n); });

  // A stream on its OWN hardware queue: a CU-masked stream always gets a dedicated HSA
  // queue (the mask is a queue property), here with every CU enabled.  Plain streams of
  // one priority are spread round-robin over GPU_MAX_HW_QUEUES (4) shared queues, where
  // two logically concurrent streams (actor / learner) can land on one queue and
  // serialise.  Returns the hipStream_t as an integer (torch.cuda.ExternalStream).
  m.def("create_dedicated_stream", [](int device) {
    auto hip_ok = [](hipError_t e) {
      if (e != hipSuccess) throw std::runtime_error(std::string("create_dedicated_stream: ") + hipGetErrorString(e));
    };
    int cus = 0;
    hip_ok(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    std::vector<uint32_t> mask((cus + 31) / 32, 0xFFFFFFFFu);
    if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
    int prev = 0;
    hip_ok(hipGetDevice(&prev));
    hip_ok(hipSetDevice(device));
    hipStream_t st = nullptr;
    hip_ok(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    hip_ok(hipSetDevice(prev));
    return (uint64_t)reinterpret_cast<uintptr_t>(st);
  });
  m.def("spin_us", [](int us, uint64_t s) { spin_us(us, S(s)); });

  // ---- stream-ordering events without the system-scope fence (device-local hand-offs
  // between this process's streams: hipEventDisableSystemFence skips the L2 writeback /
  // invalidate a default event's record and wait carry)
  m.def("event_create", [](bool light) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | (light ? hipEventDisableSystemFence : 0u)));
    return reinterpret_cast<uint64_t>(e);
  });
  m.def("event_record", [](uint64_t e, uint64_t s) {
    HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(e), S(s)));
  });
  m.def("stream_wait_event", [](uint64_t s, uint64_t e) {
    HIP_CHECK(hipStreamWaitEvent(S(s), reinterpret_cast<hipEvent_t>(e), 0));
  });
  m.def("event_destroy", [](uint64_t e) { HIP_CHECK(hipEventDestroy(reinterpret_cast<hipEvent_t>(e))); });
  m.def("copy_f32", [](uint64_t dst, uint64_t src, int64_t n, uint64_t s) {
    copy_f32(P<float>(dst), P<const float>(src), n, S(s));
  });

  // ---- AQL kernels
  py::class_<AQLNet>(m, "AQLNet");
  m.def("make_aql_net", [](py::dict ints, py::dict ptrs) {
    AQLNet n{};
    auto gi = [&](const char* k) { return ints[k].cast<int>(); };
    n.obs = gi("obs"); n.adim = gi("adim"); n.cont = gi("cont"); n.T = gi("T"); n.na = gi("na");
    n.uniform = gi("uniform"); n.propose = gi("propose"); n.noisy = gi("noisy");
    auto gp = [&](const char* k) -> const float* {
      return ptrs.contains(k) ? reinterpret_cast<const float*>(ptrs[k].cast<uint64_t>()) : nullptr;
    };
    n.qf_w1 = gp("qf_w1"); n.qf_b1 = gp("qf_b1"); n.qf_w2 = gp("qf_w2"); n.qf_b2 = gp("qf_b2");
    n.ao_w1 = gp("ao_w1"); n.ao_b1 = gp("ao_b1"); n.ao_w2 = gp("ao_w2"); n.ao_b2 = gp("ao_b2");
    n.a1_wmu = gp("a1_wmu"); n.a1_wsig = gp("a1_wsig"); n.a1_weps = gp("a1_weps");
    n.a1_bmu = gp("a1_bmu"); n.a1_bsig = gp("a1_bsig"); n.a1_beps = gp("a1_beps");
    n.a2_wmu = gp("a2_wmu"); n.a2_wsig = gp("a2_wsig"); n.a2_weps = gp("a2_weps");
    n.a2_bmu = gp("a2_bmu"); n.a2_bsig = gp("a2_bsig"); n.a2_beps = gp("a2_beps");
    n.f_w = gp("f_w"); n.f_b = gp("f_b");
    n.df_w1 = gp("df_w1"); n.df_b1 = gp("df_b1"); n.df_w2 = gp("df_w2"); n.df_b2 = gp("df_b2");
    if (!n.qf_w1 || !n.ao_w1 || !n.a1_wmu || !n.a2_wmu) throw std::invalid_argument("make_aql_net: missing weights");
    if (n.cont && (!n.ao_w2 || n.adim < 1)) throw std::invalid_argument("make_aql_net: continuous encoder");
    return n;
  });
  m.def("aql_workspace_floats", &aql_workspace_floats);
  m.def("aql_candidate_q", [](const AQLNet& n, uint64_t ws, uint64_t state, uint64_t a_mu, int B, uint64_t q,
                              uint64_t s) {
    aql_candidate_q(n, P<float>(ws), P<const float>(state), P<const float>(a_mu), B, P<float>(q), S(s));
  });
  m.def("aql_propose", [](const AQLNet& n, uint64_t state, int B, uint64_t low, uint64_t high, uint64_t var,
                          uint64_t seed, uint64_t counter, uint64_t a_mu, uint64_t mu_out, uint64_t s,
                          uint64_t eff_ws) {
    if (!n.f_w || !n.df_w1 || !n.df_w2) throw std::invalid_argument("aql_propose: proposal weights missing");
    aql_propose(n, P<const float>(state), B, P<const float>(low), P<const float>(high), P<const float>(var), seed,
                P<const int64_t>(counter), P<float>(a_mu), P<float>(mu_out), S(s), P<float>(eff_ws));
  }, py::arg("net"), py::arg("state"), py::arg("B"), py::arg("low"), py::arg("high"), py::arg("var"), py::arg("seed"),
     py::arg("counter"), py::arg("a_mu"), py::arg("mu_out"), py::arg("s"), py::arg("eff_ws") = 0);
  // ---- GPU AQL engine (aql_engine_kernels.hip): descriptors built once, per-step calls take a stream
  py::class_<AqlLearn>(m, "AqlLearn");
  m.def("make_aql_learn", [](const AQLNet& on, const AQLNet& tg, py::dict p, int B, float gamma_n, float ent_lam) {
    auto g = [&](const char* k) { return p[k].cast<uint64_t>(); };
    AqlLearn L{};
    L.on = on;
    L.tg = tg;
    L.st = P<const float>(g("st")); L.st2 = P<const float>(g("st2")); L.rew = P<const float>(g("rew"));
    L.done = P<const float>(g("done")); L.amu = P<const float>(g("amu")); L.act = P<const int>(g("act"));
    L.idx = P<const int>(g("idx")); L.w = P<const float>(g("w")); L.var = P<const float>(g("var"));
    L.q_s = P<float>(g("q_s")); L.q_s2 = P<float>(g("q_s2")); L.qt_s2 = P<float>(g("qt_s2"));
    L.vec = P<float>(g("vec")); L.delta = P<float>(g("delta")); L.lw = P<float>(g("lw"));
    L.lossp = P<float>(g("lossp"));
    L.eff_on = P<const float>(g("eff_on")); L.eff_tg = P<const float>(g("eff_tg"));
    L.dbg = p.contains("dbg") ? P<long long>(g("dbg")) : nullptr;
    L.B = B;
    L.gamma_n = gamma_n;
    L.ent_lam = ent_lam;
    return L;
  });
  m.def("make_aql_act", [](const AQLNet& on, uint64_t state, uint64_t amu, uint64_t eff, uint64_t q, int B,
                           int blocks) {
    AqlLearn L{};
    L.on = on;
    L.tg = on;
    L.st = P<const float>(state);
    L.st2 = L.st;
    L.amu = P<const float>(amu);
    L.eff_on = L.eff_tg = P<const float>(eff);
    L.q_s = P<float>(q);
    L.B = B;
    L.act_mode = 1;
    L.act_blocks = blocks;
    return L;
  });
  m.def("aql_act_q", [](const AqlLearn& L, uint64_t s) { aql_act_q(L, S(s)); });
  // the learner forward samples its own rows (replaces per_sample before aql_learn_fwd)
  m.def("aql_learn_set_sample", [](const AqlLearn& L0, const TreeHandle& t, uint64_t filled, uint64_t beta,
                                   uint64_t ctr, uint64_t seed, int exclude_last) {
    AqlLearn L = L0;
    L.fused_sample = 1;
    L.tree = t.d;
    L.filled = P<const int64_t>(filled);
    L.beta = P<const float>(beta);
    L.ctr = P<const int64_t>(ctr);
    L.seed = seed;
    L.exclude_last = exclude_last;
    L.idx_out = const_cast<int*>(L.idx);
    L.w_out = const_cast<float*>(L.w);
    if (!L.filled || !L.beta || !L.ctr || !L.idx_out || !L.w_out) throw std::invalid_argument("aql_learn_set_sample");
    return L;
  });
  // the priority write as an extra workgroup of the backward launch (replaces the split write)
  m.def("aql_learn_set_tree", [](const AqlLearn& L0, const TreeHandle& t, uint64_t prio_out, uint64_t loss_out,
                                 uint64_t owner, uint64_t list, uint64_t max_prio, float alpha, int levels) {
    AqlLearn L = L0;
    BatchWrite w{};
    w.idx = L.idx;
    w.B = L.B;
    w.mix = PrioMix{nullptr, nullptr, P<float>(prio_out), P<float>(loss_out)};  // delta / lw: the block's LDS
    w.owner = P<int>(owner);
    w.list = P<int>(list);
    w.max_prio = P<float>(max_prio);
    w.alpha = alpha;
    if (!w.idx || !w.owner || !w.list || !w.max_prio || L.B < 1 || L.B > 64)
      throw std::invalid_argument("aql_learn_set_tree: 1 <= B <= 64 and every pointer");
    L.bwd_tree = levels < 0 ? 1 : 2;  // levels < 0: every level; else levels 1..levels (0: leaves only)
    L.bwd_levels = levels < 0 ? 0 : levels;
    L.tree = t.d;
    L.bw = w;
    return L;
  }, py::arg("L"), py::arg("tree"), py::arg("prio_out"), py::arg("loss_out"), py::arg("owner"), py::arg("list"),
     py::arg("max_prio"), py::arg("alpha"), py::arg("levels") = -1);
  m.def("aql_grad_set_levels", [](const AqlGrad& g0, const TreeHandle& t, uint64_t list, int B, int lo) {
    AqlGrad g = g0;
    BatchWrite w{};
    w.list = P<int>(list);
    w.B = B;
    if (!w.list || B < 1 || B > 64) throw std::invalid_argument("aql_grad_set_levels: 1 <= B <= 64 and a list");
    g.tree_leaves = 2;
    g.levels_lo = lo;
    g.tree = t.d;
    g.bw = w;
    return g;
  }, py::arg("G"), py::arg("tree"), py::arg("list"), py::arg("B"), py::arg("lo") = 1);
  m.def("aql_grad_set_step_snap", [](const AqlGrad& g0, uint64_t snap, uint64_t step) {
    AqlGrad g = g0;
    if (!snap || !step) throw std::invalid_argument("aql_grad_set_step_snap: both pointers");
    g.step_snap = P<int64_t>(snap);
    g.step_src = P<const int64_t>(step);
    return g;
  }, py::arg("G"), py::arg("snap"), py::arg("step"));
  m.def("aql_learn_set_groups", [](const AqlLearn& L0, int groups, int halves) {  // groups 0: the launcher picks
    if (halves != 0 && halves != 1 && halves != 2) throw std::invalid_argument("aql_learn_set_groups: halves 0, 1 or 2");
    AqlLearn L = L0;
    L.tile_groups = groups;
    L.fwd_halves = halves;
    return L;
  }, py::arg("L"), py::arg("groups"), py::arg("halves") = 0);
  m.def("aql_noisy_eff", [](const AQLNet& net, uint64_t ws, uint64_t s) { aql_noisy_eff(net, P<float>(ws), S(s)); });
  // gate / j: the step gate (kernels.h AqlLearn::gate) -- a by-value copy per launch
  m.def("aql_learn_fwd", [](AqlLearn L, uint64_t s, uint64_t gate, int j) {
    L.gate = P<const int>(gate);
    L.gate_j = j;
    aql_learn_fwd(L, S(s));
  }, py::arg("L"), py::arg("s"), py::arg("gate") = 0, py::arg("j") = 0);
  m.def("aql_learn_bwd", [](AqlLearn L, uint64_t s, uint64_t gate, int j) {
    L.gate = P<const int>(gate);
    L.gate_j = j;
    aql_learn_bwd(L, S(s));
  }, py::arg("L"), py::arg("s"), py::arg("gate") = 0, py::arg("j") = 0);
  m.def("aql_vec_layout", []() {
    py::dict d;
    d["GQ"] = aqlv::GQ; d["H"] = aqlv::H; d["GH"] = aqlv::GH; d["X"] = aqlv::X; d["GX"] = aqlv::GX;
    d["AOH"] = aqlv::AOH; d["GAOH"] = aqlv::GAOH; d["A"] = aqlv::A; d["QFH"] = aqlv::QFH; d["GQFH"] = aqlv::GQFH;
    d["S"] = aqlv::S; d["EMB"] = aqlv::EMB; d["HID"] = aqlv::HID; d["GHID"] = aqlv::GHID; d["GMU"] = aqlv::GMU;
    d["STRIDE"] = aqlv::STRIDE;
    return d;
  });
  py::class_<AqlGrad>(m, "AqlGrad");
  // jobs: (off, rows, cols, goff, xoff, eps_ptr, group, zero)
  m.def("make_aql_grad", [](const std::vector<std::array<int64_t, 8>>& jobs, int64_t n, uint64_t vec, int B,
                            uint64_t grad, uint64_t part, uint64_t lossp, uint64_t lossp_out) {
    if (jobs.empty() || (int)jobs.size() > kAqlMaxJobs) throw std::invalid_argument("make_aql_grad: 1..32 jobs");
    AqlGrad G{};
    for (size_t k = 0; k < jobs.size(); ++k) {
      const auto& j = jobs[k];
      G.job[k] = AqlGradJob{j[0], (int)j[1], (int)j[2], (int)j[3], (int)j[4], P<const float>((uint64_t)j[5]),
                            (int)j[6], (int)j[7]};
    }
    G.njobs = (int)jobs.size();
    G.n = n;
    G.vec = P<const float>(vec);
    G.B = B;
    G.grad = P<float>(grad);
    G.part = P<double>(part);
    G.lossp = P<const float>(lossp);
    G.lossp_out = P<float>(lossp_out);
    return G;
  });
  m.def("aql_grad", [](AqlGrad G, uint64_t s, uint64_t gate, int j) {
    G.gate = P<const int>(gate);
    G.gate_j = j;
    aql_grad(G, S(s));
  }, py::arg("G"), py::arg("s"), py::arg("gate") = 0, py::arg("j") = 0);
  m.def("aql_grad_blocks", &aql_grad_blocks);
  py::class_<AqlPost>(m, "AqlPost");
  // layers: 4 x (weps, beps, wmu, wsig, bmu, bsig, weff, beff, out, in)
  m.def("make_aql_post", [](const std::vector<std::array<uint64_t, 10>>& layers, uint64_t src, uint64_t dst,
                            int64_t n_copy, uint64_t step, uint64_t ticket, uint64_t seed) {
    if (layers.size() != 4) throw std::invalid_argument("make_aql_post: 4 noisy layers");
    AqlPost p{};
    for (int l = 0; l < 4; ++l) {
      const auto& y = layers[l];
      p.layer[l] = AqlNoise{P<float>(y[0]), P<float>(y[1]), P<const float>(y[2]), P<const float>(y[3]),
                            P<const float>(y[4]), P<const float>(y[5]), P<float>(y[6]), P<float>(y[7]), (int)y[8],
                            (int)y[9]};
    }
    p.src = P<const float>(src);
    p.dst = P<float>(dst);
    p.n_copy = n_copy;
    p.step = P<int64_t>(step);
    p.ticket = P<int>(ticket);
    p.seed = seed;
    return p;
  });
  m.def("aql_post", [](const AqlPost& p, int regen, uint64_t s) { aql_post(p, regen, S(s)); });
  // the learner step's update launch: the descriptor is validated, copied into `desc` (device
  // memory of aql_step_nbytes() bytes, owned by the caller) and launched from there
  struct AqlStepHandle {
    const AqlStep* dev;
    int grid;
    int noise_blocks;  // target-noise workgroups
    int draw;          // the descriptor carries the next step's draw
  };
  py::class_<AqlStepHandle>(m, "AqlStepHandle").def_readonly("grid", &AqlStepHandle::grid);
  m.def("aql_step_nbytes", []() { return sizeof(AqlStep); });
  m.def("make_aql_step", [](const AqlLearn& L, const AqlGrad& G, const AqlPost& Pst, const TreeHandle& t,
                            const AdamParams& hp, py::dict p, uint64_t desc) {
    auto g = [&](const char* k) { return p[k].cast<uint64_t>(); };
    auto gi = [&](const char* k) { return p[k].cast<int64_t>(); };
    AqlStep d{};
    d.L = L;
    d.G = G;
    d.P = Pst;
    d.tree = t.d;
    d.hp = hp;
    d.p = P<float>(g("p")); d.m = P<float>(g("m")); d.v = P<float>(g("v"));
    d.n = gi("n"); d.P_q = gi("P_q");
    d.norms_q = P<float>(g("norms_q")); d.norms_p = P<float>(g("norms_p"));
    d.nblk = aql_grad_blocks(d.n);
    for (int k = 0; k < 2; ++k) {  // offsets of the online noisy tensors in the flat buffer
      const AqlNoise& z = Pst.layer[k];
      d.mu_w[k] = z.wmu - d.p; d.sig_w[k] = z.wsig - d.p; d.mu_b[k] = z.bmu - d.p; d.sig_b[k] = z.bsig - d.p;
    }
    if (p.contains("draw") && p["draw"].cast<int>()) {  // + the next step's PER draw (same stream as
      d.draw = 1;                                       // aql_learn_set_sample's)
      d.filled = P<const int64_t>(g("filled"));
      d.beta = P<const float>(g("beta"));
      d.seed = g("seed");
      d.exclude_last = p["exclude_last"].cast<int>();
    }
    if (p.contains("gate")) d.gate = P<const int>(g("gate"));  // the step gate (aql_update's j)
    if (p.contains("pub_p")) {  // the acting copies (the iteration's last step publishes)
      d.pub_p = P<float>(g("pub_p"));
      d.pub_weps[0] = P<float>(g("pub_weps0")); d.pub_weps[1] = P<float>(g("pub_weps1"));
      d.pub_beps[0] = P<float>(g("pub_beps0")); d.pub_beps[1] = P<float>(g("pub_beps1"));
    }
    aql_step_check(d);
    HIP_CHECK(hipMemcpy(reinterpret_cast<void*>(desc), &d, sizeof(AqlStep), hipMemcpyHostToDevice));
    int nb = 0;
    const int grid = aql_update_grid(d, &nb);
    return AqlStepHandle{reinterpret_cast<const AqlStep*>(desc), grid, nb, d.draw};
  });
  m.def("aql_update", [](const AqlStepHandle& h, uint64_t s, int j) {
    aql_update(h.dev, h.grid, h.noise_blocks, S(s), j);
  }, py::arg("h"), py::arg("s"), py::arg("j") = 0);
  py::class_<AqlEnv>(m, "AqlEnv");
  m.def("make_aql_env", [](py::dict d) {
    auto g = [&](const char* k) { return d[k].cast<uint64_t>(); };
    auto gi = [&](const char* k) { return d[k].cast<int>(); };
    AqlEnv e{};
    e.kind = gi("kind"); e.E = gi("E"); e.obs = gi("obs"); e.adim = gi("adim"); e.T = gi("T");
    e.max_steps = gi("max_steps");
    e.obs_buf = P<float>(g("obs_buf")); e.phys = P<float>(g("phys")); e.ep_len = P<int>(g("ep_len"));
    e.ep_ret = P<float>(g("ep_ret")); e.dynA = P<const float>(g("dynA")); e.dynB = P<const float>(g("dynB"));
    e.dynw = P<const float>(g("dynw")); e.seed = g("seed"); e.counter = P<const int64_t>(g("counter"));
    e.ep_count = P<int>(g("ep_count")); e.ep_log = P<float>(g("ep_log")); e.log_cap = gi("log_cap");
    return e;
  });
  py::class_<AqlInsert>(m, "AqlInsert");
  m.def("make_aql_insert", [](py::dict d) {
    auto g = [&](const char* k) { return d[k].cast<uint64_t>(); };
    AqlInsert i{};
    i.st = P<float>(g("st")); i.st2 = P<float>(g("st2")); i.rew = P<float>(g("rew")); i.done = P<float>(g("done"));
    i.amu = P<float>(g("amu")); i.act = P<int>(g("act")); i.C = d["C"].cast<int64_t>();
    i.filled = P<const int64_t>(g("filled")); i.slots = P<int>(g("slots"));
    return i;
  });
  m.def("aql_env_reset", [](const AqlEnv& e, uint64_t s) { aql_env_reset(e, S(s)); });
  m.def("aql_apply_staged", [](const AqlInsert& src, const AqlInsert& dst, int E, int obs, int TA, uint64_t s) {
    aql_apply_staged(src, dst, E, obs, TA, S(s));
  });
  m.def("aql_env_step", [](const AqlEnv& e, uint64_t env_act, uint64_t act_idx, uint64_t amu, const AqlInsert& ins,
                           uint64_t s) {
    aql_env_step(e, P<const float>(env_act), P<const int>(act_idx), P<const float>(amu), ins, S(s));
  });
  py::class_<AqlTail>(m, "AqlTail");
  m.def("make_aql_tail", [](const AqlEnv& env, const AqlInsert& ins, const TreeHandle& tree, py::dict d) {
    auto g = [&](const char* k) { return d[k].cast<uint64_t>(); };
    auto opt = [&](const char* k) { return d.contains(k) ? d[k].cast<uint64_t>() : (uint64_t)0; };
    AqlTail a{};
    a.V = env;
    a.I = ins;
    a.tree = tree.d;
    a.q = P<const float>(g("q")); a.amu = P<const float>(g("amu")); a.eps = P<const float>(g("eps"));
    a.sel_seed = g("sel_seed"); a.act_idx = P<int>(g("act_idx")); a.env_act = P<float>(g("env_act"));
    a.alpha = d["alpha"].cast<float>(); a.max_prio = P<const float>(g("max_prio"));
    a.filled = P<int64_t>(g("filled")); a.counter = P<int64_t>(g("counter")); a.ticket = P<int>(g("ticket"));
    a.beta_out = P<float>(opt("beta_out")); a.iter = P<int64_t>(opt("iter"));
    a.beta0 = d.contains("beta0") ? d["beta0"].cast<double>() : 0.0;
    a.beta_omb = d.contains("beta_omb") ? d["beta_omb"].cast<double>() : 0.0;
    a.beta_max_step = d.contains("beta_max_step") ? d["beta_max_step"].cast<double>() : 1.0;
    a.beta_workers = d.contains("beta_workers") ? d["beta_workers"].cast<double>() : 0.0;
    if ((const void*)a.counter != (const void*)env.counter || (const void*)a.filled != (const void*)ins.filled)
      throw std::invalid_argument("make_aql_tail: counter / filled must be the env's and the ring's");
    return a;
  });
  m.def("aql_act_tail", [](const AqlTail& a, uint64_t s) { aql_act_tail(a, S(s)); });
  m.def("aql_select", [](uint64_t q, uint64_t a_mu, int B, int T, int adim, uint64_t eps, uint64_t seed,
                         uint64_t counter, uint64_t act_idx, uint64_t env_act, uint64_t s) {
    aql_select(P<const float>(q), P<const float>(a_mu), B, T, adim, P<const float>(eps), seed,
               P<const int64_t>(counter), P<int>(act_idx), P<float>(env_act), S(s));
  });
}
