// Shared declarations of the `_native` host runtime: each csrc/*.cpp registers its
// bindings through one of these hooks from native.cpp's module init.
#pragma once

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;

void register_arena(py::module_& m);     // arena.cpp: plan_offsets, OffsetAllocator
void register_shm_ring(py::module_& m);  // shm_ring.cpp: ShmRing (SPSC shared-memory channel)
