// OCP FP8 (e4m3fn) kernels: placeholder TU, filled in with the fp8 implicit GEMM.
#include <pybind11/pybind11.h>

#include "common.h"

void register_fp8(pybind11::module_& m) {}
