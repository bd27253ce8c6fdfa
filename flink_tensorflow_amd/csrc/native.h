// Shared declarations of the `_native` host runtime: each csrc/*.cpp registers its
// bindings through one of these hooks from native.cpp's module init.
#pragma once

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <functional>

namespace py = pybind11;

void register_arena(py::module_& m);     // arena.cpp: plan_offsets, OffsetAllocator
void register_shm_ring(py::module_& m);  // shm_ring.cpp: ShmRing (SPSC shared-memory channel)
void register_jpeg(py::module_& m);      // jpeg.cpp: jpeg_decode_into (baseline JPEG -> staging rows)

// fn(i) for i in [0, n) on up to `threads` threads of the process-wide persistent host pool
// (native.cpp CopyPool; the caller's thread included) — call without the GIL
void pool_run(int n, int threads, const std::function<void(int)>& fn);
