// Static-shape key grouping for the row-sparse gradient pipeline (ops/embedding.py):
// keys -> (stable order, run boundaries, unique keys) in five launches, no host sync.
//
//   prep      key' = key in [0, num_rows) ? key : num_rows (one bucket for invalid ids),
//             iota, seg[] = n, uids[] = -1
//   radix     hipcub::DeviceRadixSort::SortPairs over ceil(log2(num_rows + 1)) bits only
//             (stable LSD radix: the same order as a stable comparison sort)
//   flags     first[i] = sorted[i] != sorted[i - 1]
//   scan      hipcub::DeviceScan::InclusiveSum -> run index + 1 of every sorted position
//   starts    seg[run] = i, uids[run] = key (or -1 for the invalid bucket) at run starts
//
// Replaces a chain of ~25 framework kernels per table (where/compare/fill/sort merge passes,
// cumsum, dtype copies).  Temp storage and buffers are caller-allocated (stream-ordered
// allocator; inside hipGraph capture they come from the graph's pool).
#include <hipcub/hipcub.hpp>
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

__global__ __launch_bounds__(256) void seg_prep_kernel(const int* __restrict__ keys, int* __restrict__ kq,
                                                       int* __restrict__ iota, int* __restrict__ seg,
                                                       int* __restrict__ uids, int n, int num_rows) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int k = keys[i];
    kq[i] = (k >= 0 && k < num_rows) ? k : num_rows;
    iota[i] = i;
    uids[i] = -1;
  }
  if (i <= n) seg[i] = n;
}

__global__ __launch_bounds__(256) void seg_flags_kernel(const int* __restrict__ sorted, int* __restrict__ first,
                                                        int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) first[i] = (i == 0 || sorted[i] != sorted[i - 1]) ? 1 : 0;
}

// run index r = incl[i] - 1; the first position of each run writes its start and key
__global__ __launch_bounds__(256) void seg_starts_kernel(const int* __restrict__ sorted, const int* __restrict__ incl,
                                                         int* __restrict__ seg_id, int* __restrict__ seg,
                                                         int* __restrict__ uids, int n, int num_rows) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int r = incl[i] - 1;
  seg_id[i] = r;
  const int k = sorted[i];
  if (i == 0 || sorted[i - 1] != k) {
    seg[r] = i;
    uids[r] = k >= num_rows ? -1 : k;
  }
}

int key_bits(int num_rows) {
  int b = 1;
  while (b < 31 && (1LL << b) <= (long long)num_rows) ++b;  // keys are 0..num_rows inclusive
  return b;
}

}  // namespace

// bytes of hipcub temp storage for n keys below num_rows + 1
size_t sort_segments_temp_bytes(int n, int num_rows) {
  size_t a = 0, b = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const int*)nullptr, (int*)nullptr, (const int*)nullptr, (int*)nullptr,
                                     n, 0, key_bits(num_rows));
  hipcub::DeviceScan::InclusiveSum(nullptr, b, (const int*)nullptr, (int*)nullptr, n);
  return (a > b ? a : b) + 256;
}

// keys int32 [n] -> sorted int32 [n], perm int32 [n] (stable), seg_id int32 [n],
// seg int32 [n + 1] (run starts, n past the last run), uids int32 [n] (-1 past the runs / for
// the invalid bucket).  work: int32 [3 n] scratch; temp: sort_segments_temp_bytes bytes.
void sort_segments(uintptr_t keys, int n, int num_rows, uintptr_t sorted, uintptr_t perm, uintptr_t seg_id,
                   uintptr_t seg, uintptr_t uids, uintptr_t work, uintptr_t temp, size_t temp_bytes,
                   uintptr_t stream) {
  if (n <= 0) return;
  if (num_rows < 0 || num_rows >= (1 << 30)) throw std::invalid_argument("sort_segments: num_rows out of range");
  if (temp_bytes < sort_segments_temp_bytes(n, num_rows)) throw std::invalid_argument("sort_segments: temp too small");
  auto s = reinterpret_cast<hipStream_t>(stream);
  int* kq = reinterpret_cast<int*>(work);
  int* iota = kq + n;
  int* tmp = iota + n;
  const dim3 grid((n + 256) / 256), block(256);
  hipLaunchKernelGGL(seg_prep_kernel, grid, block, 0, s, reinterpret_cast<const int*>(keys), kq, iota,
                     reinterpret_cast<int*>(seg), reinterpret_cast<int*>(uids), n, num_rows);
  size_t tb = temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(reinterpret_cast<void*>(temp), tb, kq, reinterpret_cast<int*>(sorted), iota,
                                         reinterpret_cast<int*>(perm), n, 0, key_bits(num_rows), s) != hipSuccess)
    throw std::runtime_error("sort_segments: radix sort failed");
  hipLaunchKernelGGL(seg_flags_kernel, grid, block, 0, s, reinterpret_cast<const int*>(sorted), tmp, n);
  tb = temp_bytes;
  if (hipcub::DeviceScan::InclusiveSum(reinterpret_cast<void*>(temp), tb, tmp, kq, n, s) != hipSuccess)
    throw std::runtime_error("sort_segments: scan failed");
  hipLaunchKernelGGL(seg_starts_kernel, grid, block, 0, s, reinterpret_cast<const int*>(sorted), kq,
                     reinterpret_cast<int*>(seg_id), reinterpret_cast<int*>(seg), reinterpret_cast<int*>(uids), n,
                     num_rows);
  FTM_CHECK_LAUNCH();
}

void register_sort_segments(pybind11::module_& m) {
  m.def("sort_segments_temp_bytes", &sort_segments_temp_bytes);
  m.def("sort_segments", &sort_segments);
}
