// Embedding kernels (Wide&Deep / BERT): placeholder TU, filled in with the embedding
// bag forward/backward kernels.
#include <pybind11/pybind11.h>

#include "common.h"

void register_embedding(pybind11::module_& m) {}
