// `_rccl`: direct binding of the RCCL C API.
//
// The collective layer of the framework talks to RCCL itself instead of going through a
// torch.distributed process group: rank 0 creates the ncclUniqueId, the launcher's
// rendezvous store hands the 128 bytes to the other ranks, every rank calls
// ncclCommInitRank on its own GPU, and collectives are enqueued on the caller's HIP stream
// (passed as an integer, torch.cuda.current_stream().cuda_stream) on raw device pointers,
// so they are ordered with the kernels around them and can overlap compute when issued
// on a side stream.  Errors raise RuntimeError with RCCL's message; ``abort()`` tears a
// communicator down without waiting for peers (restart after a rank failure).
//
// The library is linked by SONAME (librccl.so.1): inside a Python process that imported
// torch first, the dynamic loader resolves it to the RCCL torch already mapped, so one
// RCCL instance serves the process.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress) {
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
  }
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("HIP ") + what + " failed: " + hipGetErrorString(e));
  }
}

ncclDataType_t dtype_of(int code) {
  if (code < 0 || code >= static_cast<int>(ncclNumTypes)) throw std::invalid_argument("bad RCCL dtype code");
  return static_cast<ncclDataType_t>(code);
}

ncclRedOp_t op_of(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
    default: throw std::invalid_argument("bad RCCL reduction op");
  }
}

inline void* P(std::uintptr_t p) { return reinterpret_cast<void*>(p); }
inline hipStream_t S(std::uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

class Comm {
 public:
  Comm(py::bytes uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank), device_(device) {
    std::string s = uid;
    if (s.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("ncclUniqueId must be 128 bytes");
    if (rank < 0 || rank >= nranks) throw std::invalid_argument("rank out of range");
    ncclUniqueId id;
    std::memcpy(id.internal, s.data(), sizeof(id.internal));
    check_hip(hipSetDevice(device), "hipSetDevice");
    py::gil_scoped_release nogil;  // blocks until every rank joined
    check(ncclCommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
  }
  ~Comm() {
    // at interpreter shutdown the HIP runtime may already be going away: leak rather
    // than call into RCCL then (the Python side destroys communicators explicitly)
    if (comm_ != nullptr && !_Py_IsFinalizing()) ncclCommDestroy(comm_);
  }

  void broadcast(std::uintptr_t send, std::uintptr_t recv, size_t count, int dt, int root, std::uintptr_t stream) {
    live();
    check(ncclBroadcast(P(send), P(recv), count, dtype_of(dt), root, comm_, S(stream)), "ncclBroadcast");
  }
  void all_reduce(std::uintptr_t send, std::uintptr_t recv, size_t count, int dt, int op, std::uintptr_t stream) {
    live();
    check(ncclAllReduce(P(send), P(recv), count, dtype_of(dt), op_of(op), comm_, S(stream)), "ncclAllReduce");
  }
  void all_gather(std::uintptr_t send, std::uintptr_t recv, size_t sendcount, int dt, std::uintptr_t stream) {
    live();
    check(ncclAllGather(P(send), P(recv), sendcount, dtype_of(dt), comm_, S(stream)), "ncclAllGather");
  }
  void reduce_scatter(std::uintptr_t send, std::uintptr_t recv, size_t recvcount, int dt, int op,
                      std::uintptr_t stream) {
    live();
    check(ncclReduceScatter(P(send), P(recv), recvcount, dtype_of(dt), op_of(op), comm_, S(stream)),
          "ncclReduceScatter");
  }
  // point-to-point (inside a group_start / group_end pair: an all-to-all with per-peer
  // counts is one send + one recv per peer, all in one group)
  void send(std::uintptr_t buf, size_t count, int dt, int peer, std::uintptr_t stream) {
    live();
    check(ncclSend(P(buf), count, dtype_of(dt), peer, comm_, S(stream)), "ncclSend");
  }
  void recv(std::uintptr_t buf, size_t count, int dt, int peer, std::uintptr_t stream) {
    live();
    check(ncclRecv(P(buf), count, dtype_of(dt), peer, comm_, S(stream)), "ncclRecv");
  }
  // returns "" while healthy, else RCCL's error string (peer failure, network error)
  std::string async_error() {
    if (comm_ == nullptr) return "communicator destroyed";
    ncclResult_t r = ncclSuccess;
    check(ncclCommGetAsyncError(comm_, &r), "ncclCommGetAsyncError");
    return r == ncclSuccess || r == ncclInProgress ? std::string() : std::string(ncclGetErrorString(r));
  }
  void abort() {
    if (comm_ != nullptr) {
      ncclComm_t c = comm_;
      comm_ = nullptr;
      py::gil_scoped_release nogil;
      ncclCommAbort(c);
    }
  }
  void destroy() {
    if (comm_ != nullptr) {
      ncclComm_t c = comm_;
      comm_ = nullptr;
      py::gil_scoped_release nogil;
      check(ncclCommDestroy(c), "ncclCommDestroy");
    }
  }
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  int device() const { return device_; }

 private:
  void live() const {
    if (comm_ == nullptr) throw std::runtime_error("RCCL communicator was destroyed/aborted");
  }
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_, device_;
};

}  // namespace

PYBIND11_MODULE(_rccl, m) {
  m.doc() = "direct RCCL C-API binding (broadcast / all-reduce / all-gather / reduce-scatter on HIP streams)";
  m.def("version", [] {
    int v = 0;
    check(ncclGetVersion(&v), "ncclGetVersion");
    return v;
  });
  m.def("unique_id", [] {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, sizeof(id.internal));
  });
  m.def("group_start", [] { check(ncclGroupStart(), "ncclGroupStart"); });
  m.def("group_end", [] { check(ncclGroupEnd(), "ncclGroupEnd"); });
  py::class_<Comm>(m, "Comm")
      .def(py::init<py::bytes, int, int, int>(), py::arg("unique_id"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"))
      .def("broadcast", &Comm::broadcast)
      .def("all_reduce", &Comm::all_reduce)
      .def("all_gather", &Comm::all_gather)
      .def("reduce_scatter", &Comm::reduce_scatter)
      .def("send", &Comm::send)
      .def("recv", &Comm::recv)
      .def("async_error", &Comm::async_error)
      .def("abort", &Comm::abort)
      .def("destroy", &Comm::destroy)
      .def_property_readonly("nranks", &Comm::nranks)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("device", &Comm::device);
}
