// Tensor-arena memory management for a subtask's device (HBM) and pinned-host memory
// (the reference copies every record JVM heap <-> native buffers per
// Session.run, LIB/types/TensorValue.java:132,259-260; here a subtask owns one arena and
// every plan buffer is an offset into it).
//
//  * plan_offsets  — static planning of a compiled plan's activation buffers: buffers with
//    known lifetimes [first, last] (inclusive step indices) get byte offsets in one slab so
//    that buffers alive at the same time never overlap.  Greedy by size: largest first,
//    each into the smallest gap (best fit) among the already-placed buffers whose lifetimes
//    intersect its own, else above the highest of them.
//  * OffsetAllocator — dynamic first-fit allocator with coalescing over a fixed-size
//    region (persistent arena allocations: plan inputs/outputs, staging slots, weights).
//    Thread-safe: operator threads of one process may share a device arena.
#include "native.h"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <iterator>
#include <map>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <vector>

namespace {

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

py::tuple plan_offsets(const std::vector<int64_t>& sizes, const std::vector<int64_t>& first,
                       const std::vector<int64_t>& last, int64_t align) {
  const size_t n = sizes.size();
  if (first.size() != n || last.size() != n) throw std::invalid_argument("plan_offsets: length mismatch");
  if (align <= 0 || (align & (align - 1))) throw std::invalid_argument("plan_offsets: align must be a power of 2");
  for (size_t i = 0; i < n; ++i) {
    if (sizes[i] < 0) throw std::invalid_argument("plan_offsets: negative size");
    if (last[i] < first[i]) throw std::invalid_argument("plan_offsets: lifetime ends before it starts");
  }
  std::vector<size_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  // largest first; ties: earlier birth first (deterministic plans)
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    if (sizes[a] != sizes[b]) return sizes[a] > sizes[b];
    return first[a] < first[b];
  });
  std::vector<int64_t> off(n, -1);
  std::vector<size_t> placed;  // kept sorted by offset
  placed.reserve(n);
  int64_t total = 0;
  for (size_t idx : order) {
    const int64_t sz = align_up(std::max<int64_t>(sizes[idx], 1), align);
    int64_t best = -1, best_gap = INT64_MAX, cursor = 0;
    for (size_t p : placed) {  // ascending offsets
      if (last[p] < first[idx] || last[idx] < first[p]) continue;  // lifetimes disjoint
      const int64_t gap = off[p] - cursor;
      if (gap >= sz && gap < best_gap) {
        best = cursor;
        best_gap = gap;
      }
      cursor = std::max(cursor, off[p] + align_up(std::max<int64_t>(sizes[p], 1), align));
    }
    if (best < 0) best = cursor;
    off[idx] = best;
    total = std::max(total, best + sz);
    placed.insert(std::upper_bound(placed.begin(), placed.end(), idx,
                                   [&](size_t a, size_t b) { return off[a] < off[b]; }),
                  idx);
  }
  return py::make_tuple(off, total);
}

class OffsetAllocator {
 public:
  OffsetAllocator(int64_t capacity, int64_t align) : capacity_(capacity), align_(align) {
    if (capacity < 0) throw std::invalid_argument("OffsetAllocator: negative capacity");
    if (align <= 0 || (align & (align - 1))) throw std::invalid_argument("OffsetAllocator: align must be a power of 2");
    if (capacity > 0) free_[0] = capacity;
  }

  // first fit; returns -1 when no free block is large enough
  int64_t alloc(int64_t nbytes) {
    const int64_t sz = align_up(std::max<int64_t>(nbytes, 1), align_);
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = free_.begin(); it != free_.end(); ++it) {
      if (it->second >= sz) {
        const int64_t o = it->first, rest = it->second - sz;
        free_.erase(it);
        if (rest > 0) free_[o + sz] = rest;
        used_[o] = sz;
        in_use_ += sz;
        peak_ = std::max(peak_, in_use_);
        return o;
      }
    }
    return -1;
  }

  void release(int64_t offset) {
    std::lock_guard<std::mutex> g(mu_);
    auto u = used_.find(offset);
    if (u == used_.end()) throw std::invalid_argument("OffsetAllocator.free: offset not allocated");
    int64_t o = offset, sz = u->second;
    used_.erase(u);
    in_use_ -= sz;
    auto next = free_.lower_bound(o);
    if (next != free_.end() && next->first == o + sz) {  // merge with the following block
      sz += next->second;
      next = free_.erase(next);
    }
    if (next != free_.begin()) {  // merge with the preceding block
      auto prev = std::prev(next);
      if (prev->first + prev->second == o) {
        prev->second += sz;
        return;
      }
    }
    free_[o] = sz;
  }

  int64_t capacity() const { return capacity_; }
  int64_t in_use() {
    std::lock_guard<std::mutex> g(mu_);
    return in_use_;
  }
  int64_t peak() {
    std::lock_guard<std::mutex> g(mu_);
    return peak_;
  }
  int64_t largest_free() {
    std::lock_guard<std::mutex> g(mu_);
    int64_t m = 0;
    for (auto& kv : free_) m = std::max(m, kv.second);
    return m;
  }
  size_t num_free_blocks() {
    std::lock_guard<std::mutex> g(mu_);
    return free_.size();
  }
  size_t num_allocations() {
    std::lock_guard<std::mutex> g(mu_);
    return used_.size();
  }

 private:
  int64_t capacity_, align_;
  int64_t in_use_ = 0, peak_ = 0;
  std::map<int64_t, int64_t> free_;  // offset -> size
  std::map<int64_t, int64_t> used_;  // offset -> size
  std::mutex mu_;
};

}  // namespace

void register_arena(py::module_& m) {
  m.def("plan_offsets", &plan_offsets, py::arg("sizes"), py::arg("first"), py::arg("last"), py::arg("align") = 256,
        "Byte offsets for buffers with lifetimes [first, last] in one slab: (offsets, slab_bytes)");
  py::class_<OffsetAllocator>(m, "OffsetAllocator")
      .def(py::init<int64_t, int64_t>(), py::arg("capacity"), py::arg("align") = 256)
      .def("alloc", &OffsetAllocator::alloc, py::arg("nbytes"))
      .def("free", &OffsetAllocator::release, py::arg("offset"))
      .def_property_readonly("capacity", &OffsetAllocator::capacity)
      .def_property_readonly("in_use", &OffsetAllocator::in_use)
      .def_property_readonly("peak", &OffsetAllocator::peak)
      .def_property_readonly("largest_free", &OffsetAllocator::largest_free)
      .def_property_readonly("num_free_blocks", &OffsetAllocator::num_free_blocks)
      .def_property_readonly("num_allocations", &OffsetAllocator::num_allocations);
}
