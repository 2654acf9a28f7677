// Direct RCCL (NCCL API on ROCm) for the data-parallel learner: one communicator per
// process group, collectives enqueued on a caller-chosen HIP stream.
//
// torch.distributed's ProcessGroupNCCL costs ~30 us of host time per async collective
// (work objects, watchdog bookkeeping, its own stream + two event hops), measured with
// roctx ranges on MI355X; the learner issues two collectives per SGD step at ~0.3 ms
// per step, so that overhead alone made the data-parallel step host-bound.  Here a
// collective is one ncclAllReduce call on a stream the engine owns (ordering by HIP
// events it records itself).  The communicator is bootstrapped from an ncclUniqueId
// that rank 0 broadcasts over the existing process group (parallel/rccl.py).
//
// The library is the one torch already loaded (same SONAME librccl.so.1), so these
// communicators live beside torch's inside one RCCL instance.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

ncclComm_t C(uint64_t v) { return reinterpret_cast<ncclComm_t>(static_cast<uintptr_t>(v)); }
hipStream_t St(uint64_t v) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(v)); }

ncclDataType_t dtype_of(const std::string& d) {
  if (d == "f32") return ncclFloat32;
  if (d == "f64") return ncclFloat64;
  if (d == "bf16") return ncclBfloat16;
  if (d == "i64") return ncclInt64;
  if (d == "u8") return ncclUint8;
  throw std::invalid_argument("rccl: dtype must be f32|f64|bf16|i64|u8");
}

}  // namespace

void register_comm(py::module_& m) {
  m.def("rccl_version", []() {
    int v = 0;
    nccl_ok(ncclGetVersion(&v), "ncclGetVersion");
    return v;
  });
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.def("rccl_comm_init", [](py::bytes id_bytes, int world, int rank, int device) {
    std::string s = id_bytes;
    if (s.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("rccl_comm_init: bad unique id size");
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("rccl_comm_init: bad rank/world");
    ncclUniqueId id;
    std::memcpy(&id, s.data(), sizeof(id));
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl_comm_init: hipSetDevice failed");
    ncclComm_t comm = nullptr;
    {
      py::gil_scoped_release nogil;  // collective bootstrap: every rank blocks here
      nccl_ok(ncclCommInitRank(&comm, world, id, rank), "ncclCommInitRank");
    }
    return (uint64_t)reinterpret_cast<uintptr_t>(comm);
  }, py::arg("unique_id"), py::arg("world"), py::arg("rank"), py::arg("device"));
  m.def("rccl_all_reduce_sum", [](uint64_t buf, int64_t n, const std::string& dtype, uint64_t comm, uint64_t stream) {
    if (!comm) throw std::invalid_argument("rccl_all_reduce_sum: null communicator");
    if (n <= 0) return;
    void* p = reinterpret_cast<void*>(static_cast<uintptr_t>(buf));
    nccl_ok(ncclAllReduce(p, p, (size_t)n, dtype_of(dtype), ncclSum, C(comm), St(stream)), "ncclAllReduce");
  }, py::arg("buf"), py::arg("n"), py::arg("dtype"), py::arg("comm"), py::arg("stream"));
  m.def("rccl_broadcast", [](uint64_t buf, int64_t n, const std::string& dtype, int root, uint64_t comm,
                             uint64_t stream) {
    if (!comm) throw std::invalid_argument("rccl_broadcast: null communicator");
    void* p = reinterpret_cast<void*>(static_cast<uintptr_t>(buf));
    nccl_ok(ncclBroadcast(p, p, (size_t)n, dtype_of(dtype), root, C(comm), St(stream)), "ncclBroadcast");
  }, py::arg("buf"), py::arg("n"), py::arg("dtype"), py::arg("root"), py::arg("comm"), py::arg("stream"));
  m.def("rccl_comm_count", [](uint64_t comm) {
    if (!comm) throw std::invalid_argument("rccl_comm_count: null communicator");
    int n = 0;
    nccl_ok(ncclCommCount(C(comm), &n), "ncclCommCount");
    return n;
  });
  m.def("rccl_comm_destroy", [](uint64_t comm) {
    if (comm) nccl_ok(ncclCommDestroy(C(comm)), "ncclCommDestroy");
  });
}
