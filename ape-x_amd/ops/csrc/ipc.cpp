// HIP IPC primitives for the central-replay transport (parallel/ipc.py), host side:
// arena allocation with an explicit coherence mode, IPC handle export / import, pinned
// mapping of a /dev/shm control block, stream-ordered copies into peer memory, and the
// ingest / flag launches of ipc_kernels.hip.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace py = pybind11;

namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
template <typename T>
T* P(uint64_t v) {
  return reinterpret_cast<T*>(static_cast<uintptr_t>(v));
}
template <typename T>
T* P_(uint64_t v) {  // (P names a parameter count in some bindings)
  return P<T>(v);
}
uint64_t U(const void* p) { return (uint64_t)reinterpret_cast<uintptr_t>(p); }
hipStream_t S(uint64_t v) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(v)); }

struct IpcIngestHandle {
  apex::IpcIngest g{};
};

}  // namespace

void register_ipc(py::module_& m) {
  // mode 0: plain device memory (L2-cached), 1: fine-grained, 2: uncached (every access
  // bypasses L2: the right mode for memory that peers write over xGMI while this GPU reads it)
  m.def("ipc_alloc", [](int64_t bytes, int mode) {
    if (bytes <= 0) throw std::invalid_argument("ipc_alloc: bytes must be > 0");
    void* p = nullptr;
    if (mode == 0) hip_ok(hipMalloc(&p, (size_t)bytes), "hipMalloc");
    else if (mode == 1) hip_ok(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained), "hipExtMallocWithFlags(fine)");
    else if (mode == 2) hip_ok(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
    else throw std::invalid_argument("ipc_alloc: mode must be 0 (default), 1 (fine-grained) or 2 (uncached)");
    hip_ok(hipMemset(p, 0, (size_t)bytes), "hipMemset");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return U(p);
  }, py::arg("bytes"), py::arg("mode") = 2);
  // multi-GPU preflight (parallel/preflight.py): can ``device`` map ``peer``'s memory (xGMI)?
  m.def("device_can_access_peer", [](int device, int peer) {
    int can = 0;
    hip_ok(hipDeviceCanAccessPeer(&can, device, peer), "hipDeviceCanAccessPeer");
    return can;
  });
  m.def("device_count", []() {
    int n = 0;
    hip_ok(hipGetDeviceCount(&n), "hipGetDeviceCount");
    return n;
  });
  m.def("ipc_free", [](uint64_t p) {
    if (p) hip_ok(hipFree(P<void>(p)), "hipFree");
  });
  m.def("ipc_handle", [](uint64_t p) {
    hipIpcMemHandle_t h;
    hip_ok(hipIpcGetMemHandle(&h, P<void>(p)), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  });
  m.def("ipc_open", [](py::bytes hb, int device) {
    std::string s = hb;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("ipc_open: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    hip_ok(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return U(p);
  }, py::arg("handle"), py::arg("device"));
  m.def("ipc_close", [](uint64_t p) {
    if (p) hip_ok(hipIpcCloseMemHandle(P<void>(p)), "hipIpcCloseMemHandle");
  });
  m.def("memcpy_async", [](uint64_t dst, uint64_t src, int64_t n, uint64_t stream) {
    if (n <= 0) return;
    hip_ok(hipMemcpyAsync(P<void>(dst), P<const void>(src), (size_t)n, hipMemcpyDefault, S(stream)), "hipMemcpyAsync");
  });
  m.def("memcpy_sync", [](uint64_t dst, uint64_t src, int64_t n) {
    if (n <= 0) return;
    hip_ok(hipMemcpy(P<void>(dst), P<const void>(src), (size_t)n, hipMemcpyDefault), "hipMemcpy");
  });
  // pin + map a host range (a /dev/shm control block) for GPU access; returns the device pointer
  m.def("host_register", [](uint64_t host, int64_t bytes) {
    hip_ok(hipHostRegister(P<void>(host), (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable),
           "hipHostRegister");
    void* d = nullptr;
    hip_ok(hipHostGetDevicePointer(&d, P<void>(host), 0), "hipHostGetDevicePointer");
    return U(d);
  });
  m.def("host_unregister", [](uint64_t host) {
    if (host) hip_ok(hipHostUnregister(P<void>(host)), "hipHostUnregister");
  });

  py::class_<IpcIngestHandle>(m, "IpcIngestHandle");
  m.def("make_ipc_ingest", [](py::dict d) {
    IpcIngestHandle h;
    auto& g = h.g;
    auto i = [&](const char* k) { return d[k].cast<int64_t>(); };
    auto p = [&](const char* k) -> uint64_t { return d.contains(k) ? d[k].cast<uint64_t>() : 0; };
    g.kind = d.contains("kind") ? (int)i("kind") : 0;
    g.prefix = P<int>(p("prefix"));
    if (g.kind == 1) {
      g.obs = (int)i("obs");
      g.TA = (int)i("TA");
      g.aql.st = P<float>(p("aql_st"));
      g.aql.st2 = P<float>(p("aql_st2"));
      g.aql.amu = P<float>(p("aql_amu"));
      g.aql.act = P<int>(p("aql_act"));
      g.aql.rew = P<float>(p("aql_rew"));
      g.aql.done = P<float>(p("aql_done"));
      g.aql.C = i("aql_C");
      g.aql.filled = P<const int64_t>(p("filled"));
    }
    g.R = (int)i("R");
    g.D = (int)i("D");
    g.E = (int)i("E");
    g.cap = (int)i("cap");
    g.packet_bytes = i("packet_bytes");
    g.ring = P<const uint8_t>(p("ring"));
    g.seq = P<const int64_t>(p("seq"));
    g.consumed = P<int64_t>(p("consumed"));
    g.ready = P<int>(p("ready"));
    g.live = P<const int>(p("live"));
    g.host_consumed = P<int64_t>(p("host_consumed"));
    g.applied = P<int64_t>(p("applied"));
    g.filled = P<int64_t>(p("filled"));
    g.frames = P<uint8_t>(p("frames"));
    g.s_ids = P<int32_t>(p("s_ids"));
    g.s2_ids = P<int32_t>(p("s2_ids"));
    g.action = P<int32_t>(p("action"));
    g.reward = P<float>(p("reward"));
    g.done = P<float>(p("done"));
    g.frame_base = P<const int64_t>(p("frame_base"));
    g.slot_base = P<const int64_t>(p("slot_base"));
    g.slots_out = P<int32_t>(p("slots_out"));
    g.prio_out = P<float>(p("prio_out"));
    g.budget = P<int64_t>(p("budget"));
    g.gate = P<int>(p("gate"));
    g.gate_batch = d.contains("gate_batch") ? (int)i("gate_batch") : 0;
    g.gate_max = d.contains("gate_max") ? (int)i("gate_max") : 0;
    return h;
  });
  m.def("ipc_ingest", [](const IpcIngestHandle& h, uint64_t s) { apex::ipc_ingest(h.g, S(s)); });
  m.def("ipc_flag", [](uint64_t p, int64_t v, uint64_t s) { apex::ipc_flag(P<int64_t>(p), v, S(s)); });
  m.def("ipc_param_publish", [](uint64_t ctrl, int pin_off, int R, int begin_off, int K, uint64_t params,
                                int64_t stride_f, uint64_t src, int64_t P, int64_t v, uint64_t pick, uint64_t s) {
    apex::ipc_param_publish(P_<int64_t>(ctrl), pin_off, R, begin_off, K, P_<float>(params), stride_f,
                            P_<const float>(src), P, v, P_<int>(pick), S(s));
  });
  m.def("ipc_stage_dqn", [](py::dict d, uint64_t s) {
    auto p = [&](const char* k) -> uint64_t { return d.contains(k) ? d[k].cast<uint64_t>() : 0; };
    apex::IpcStage st{};
    st.frames = P<const uint8_t>(p("frames"));
    st.new_frame = P<const int32_t>(p("new_frame"));
    st.s_ids = P<const int32_t>(p("s_ids"));
    st.s2_ids = P<const int32_t>(p("s2_ids"));
    st.action = P<const int32_t>(p("action"));
    st.reward = P<const float>(p("reward"));
    st.done = P<const float>(p("done"));
    st.slot = P<const int32_t>(p("slot"));
    st.prio = P<const float>(p("prio"));
    st.hist = P<const int32_t>(p("hist"));
    st.actions = P<const int32_t>(p("actions"));
    st.packet = P<uint8_t>(p("packet"));
    st.E = d["E"].cast<int>();
    st.initial = d.contains("initial") ? d["initial"].cast<int>() : 0;
    apex::ipc_stage_dqn(st, S(s));
  });
  py::class_<apex::IpcEmu>(m, "IpcEmu");
  m.def("make_ipc_emu", [](py::dict d) {
    auto p = [&](const char* k) { return d[k].cast<uint64_t>(); };
    auto i = [&](const char* k) { return d[k].cast<int64_t>(); };
    apex::IpcEmu g{};
    g.ring = P<uint8_t>(p("ring"));
    g.seq = P<int64_t>(p("seq"));
    g.consumed = P<const int64_t>(p("consumed"));
    g.sent = P<int64_t>(p("sent"));
    g.go = P<int32_t>(p("go"));
    g.pool = P<const uint8_t>(p("pool"));
    g.pool_n = (int)i("pool_n");
    g.R = (int)i("R"); g.D = (int)i("D"); g.E = (int)i("E");
    g.C_r = (int)i("C_r"); g.F_r = (int)i("F_r"); g.n_actions = (int)i("n_actions");
    g.pkt = i("pkt");
    g.seed = p("seed");
    return g;
  });
  m.def("ipc_emu_push", [](const apex::IpcEmu& g, uint64_t s) { apex::ipc_emu_push(g, S(s)); });
}
