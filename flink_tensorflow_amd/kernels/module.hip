// pybind11 entry point of the `_hip` kernel library.  Each kernel TU exposes a
// register_* function; launchers take raw device pointers + shapes + a hipStream_t
// (passed as an integer from torch.cuda.current_stream().cuda_stream), so every launch
// lands on the caller's stream and is captured by hipGraph capture.
#include <pybind11/pybind11.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

void register_igemm(pybind11::module_& m);
void register_nn_misc(pybind11::module_& m);
void register_transformer(pybind11::module_& m);
void register_embedding(pybind11::module_& m);
void register_fp8(pybind11::module_& m);
void register_attention(pybind11::module_& m);
void register_dconv(pybind11::module_& m);
void register_elementwise(pybind11::module_& m);
void register_conv3x3c64(pybind11::module_& m);
void register_bottleneck(pybind11::module_& m);
void register_bottleneck_chain(pybind11::module_& m);
void register_gemm_pp(pybind11::module_& m);
void register_conv_pp(pybind11::module_& m);
void register_widedeep(pybind11::module_& m);
void register_sort_segments(pybind11::module_& m);
void register_pw_res(pybind11::module_& m);
void register_gemm_train(pybind11::module_& m);

PYBIND11_MODULE(_hip, m) {
  m.doc() = "flink_tensorflow_amd CDNA4 (gfx950) kernels";
  m.attr("arch") = "gfx950";
  register_igemm(m);
  register_nn_misc(m);
  register_transformer(m);
  register_embedding(m);
  register_fp8(m);
  register_attention(m);
  register_dconv(m);
  register_elementwise(m);
  register_conv3x3c64(m);
  register_bottleneck(m);
  register_bottleneck_chain(m);
  register_gemm_pp(m);
  register_conv_pp(m);
  register_widedeep(m);
  register_sort_segments(m);
  register_pw_res(m);
  register_gemm_train(m);
  // Streams owned by the framework (not torch's round-robin pool of 32 per device): a pooled
  // stream handed to a runner can be the very stream another thread is capturing a hipGraph
  // on, and then that thread's launches land in the capture (or are rejected).
  m.def("stream_create", [](int priority) {
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
    if (e != hipSuccess) throw std::runtime_error(std::string("hipStreamCreateWithPriority: ") + hipGetErrorString(e));
    return reinterpret_cast<std::uintptr_t>(s);
  }, pybind11::arg("priority") = 0);
  m.def("stream_destroy", [](std::uintptr_t s) {
    hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(s));
    if (e != hipSuccess) throw std::runtime_error(std::string("hipStreamDestroy: ") + hipGetErrorString(e));
  });
}
