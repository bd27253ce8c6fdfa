// Embedding kernels for the Wide&Deep online-training path (and BERT-style lookups).
//
//   embedding_bag_fwd   out[b, f*D + d] = sum_l table[ids[b, f, l], d]     (ids < 0 skipped)
//                       fp32 master table -> bf16 activations (16-B vector loads/stores)
//   segment_sum_rows    row-sparse backward: gradient rows are grouped by destination with a
//                       sort (done by the caller on the GPU), then every destination row is
//                       summed by ONE wave in a fixed order — deterministic, no float atomics
//                       (guide Appendix B "Scatter / gather / embedding": store-and-sum form)
//   sparse_adagrad      table[u] -= lr * g / (sqrt(acc[u] += g^2) + eps) on the touched rows
//
// D % 8 == 0; one wave per (bag, field) row / destination row, 8 elements per lane.
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

__global__ __launch_bounds__(256) void embedding_bag_fwd_kernel(const int* __restrict__ ids,
                                                                const float* __restrict__ table,
                                                                bf16* __restrict__ out, int rows, int L, int D,
                                                                int out_ld, int V) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);  // r = b * F + f
  if (r >= rows) return;
  const int* idp = ids + (size_t)r * L;
  for (int c = lane * 8; c < D; c += 64 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < L; ++l) {
      const int id = idp[l];
      if (id < 0 || id >= V) continue;
      const f32x4* src = reinterpret_cast<const f32x4*>(table + (size_t)id * D + c);
      const f32x4 a = src[0], b = src[1];
      acc[0] += a[0]; acc[1] += a[1]; acc[2] += a[2]; acc[3] += a[3];
      acc[4] += b[0]; acc[5] += b[1]; acc[6] += b[2]; acc[7] += b[3];
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    // out row b, field f -> column f*D (the F field blocks are contiguous per row)
    *reinterpret_cast<bf16x8*>(out + (size_t)r * D + c) = o;
  }
  (void)out_ld;
}

// grad rows: grad_out[(b*F+f), :] (bf16 or fp32, pitch D); perm lists source rows sorted
// by destination; seg[u]..seg[u+1] is destination u's range in perm.
// One wave per destination row.  The wave's lanes are CW column chunks (8 elements each)
// x RG = 64 / CW row groups: row group g sums rows s0+g, s0+g+RG, ... (many independent
// loads in flight for hot ids), then the RG partials are combined by a fixed xor-shuffle
// tree — the summation order depends only on the segment, so results are bit-identical
// run to run.  D > 8 * 64 loops over 512-column blocks with RG = 1.
template <typename T, int CW>
__global__ __launch_bounds__(256) void segment_sum_rows_kernel(const T* __restrict__ grad, const int* __restrict__ perm,
                                                               const int* __restrict__ seg, float* __restrict__ out,
                                                               int U, int D, int L) {
  constexpr int RG = 64 / CW;
  const int lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U) return;
  const int s0 = seg[u], s1 = seg[u + 1];
  const int cl = lane % CW;
  const int rg = lane / CW;
  for (int c0 = 0; c0 < D; c0 += CW * 8) {
    const int c = c0 + cl * 8;
    const bool cv = c < D;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cv) {
      for (int i = s0 + rg; i < s1; i += RG) {
        const int src = perm[i] / L;  // bag element -> its (b, f) output row
        if constexpr (sizeof(T) == 2) {
          const bf16x8 g = *reinterpret_cast<const bf16x8*>(grad + (size_t)src * D + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += (float)g[e];
        } else {
          const f32x4* gp = reinterpret_cast<const f32x4*>(grad + (size_t)src * D + c);
          const f32x4 a = gp[0], b = gp[1];
          acc[0] += a[0]; acc[1] += a[1]; acc[2] += a[2]; acc[3] += a[3];
          acc[4] += b[0]; acc[5] += b[1]; acc[6] += b[2]; acc[7] += b[3];
        }
      }
    }
#pragma unroll
    for (int off = CW; off < 64; off <<= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], off, 64);
    }
    if (rg == 0 && cv) {
      f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)u * D + c);
      dst[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
      dst[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
    }
  }
}

// Segment boundaries of a sorted key array, static shapes: for every i that starts a run
// (i == 0 or sorted[i] != sorted[i-1]) with run index s = seg_id[i]:  seg[s] = i and
// uids[s] = key (or -1 for the invalid bucket key == num_rows).  Each run is written by
// exactly one thread: deterministic, no atomics, no host round trip.
__global__ __launch_bounds__(256) void segment_starts_kernel(const long long* __restrict__ sorted,
                                                             const int* __restrict__ seg_id, int* __restrict__ seg,
                                                             int* __restrict__ uids, int n, long long num_rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long k = sorted[i];
  if (i == 0 || sorted[i - 1] != k) {
    const int sidx = seg_id[i];
    seg[sidx] = i;
    uids[sidx] = k >= num_rows ? -1 : (int)k;
  }
}

__global__ __launch_bounds__(256) void sparse_adagrad_kernel(float* __restrict__ table, float* __restrict__ accum,
                                                             const int* __restrict__ uids, const float* __restrict__ g,
                                                             int U, int D, int V, float lr, float eps) {
  const int lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U) return;
  const int id = uids[u];
  if (id < 0 || id >= V) return;  // padding of the static-shape sparse pipeline
  const size_t row = (size_t)id * D;
  for (int c = lane * 4; c < D; c += 64 * 4) {
    f32x4 gv = *reinterpret_cast<const f32x4*>(g + (size_t)u * D + c);
    f32x4 av = *reinterpret_cast<f32x4*>(accum + row + c);
    f32x4 tv = *reinterpret_cast<f32x4*>(table + row + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      av[e] += gv[e] * gv[e];
      tv[e] -= lr * gv[e] / (sqrtf(av[e]) + eps);
    }
    *reinterpret_cast<f32x4*>(accum + row + c) = av;
    *reinterpret_cast<f32x4*>(table + row + c) = tv;
  }
}

}  // namespace

void embedding_bag_fwd(uintptr_t ids, uintptr_t table, uintptr_t out, int rows, int L, int D, int V, uintptr_t stream) {
  if (D % 8) throw std::invalid_argument("embedding_bag_fwd: D % 8 != 0");
  if (table % 16 || out % 16) throw std::invalid_argument("embedding_bag_fwd: 16-byte alignment required");
  if (rows <= 0) return;
  hipLaunchKernelGGL(embedding_bag_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const int*>(ids), reinterpret_cast<const float*>(table),
                     reinterpret_cast<bf16*>(out), rows, L, D, D, V);
  FTM_CHECK_LAUNCH();
}

template <typename T>
void launch_segment_sum(const void* grad, const int* P, const int* S, float* O, int U, int D, int L, hipStream_t s) {
  const T* g = reinterpret_cast<const T*>(grad);
  const dim3 grid((U + 3) / 4), block(256);
  switch (D / 8) {  // column chunks per row: pick the widest power of two that divides the work
    case 1: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 1>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 2: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 2>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 4: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 4>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 8: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 8>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 16: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 16>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 32: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 32>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    default: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 64>), grid, block, 0, s, g, P, S, O, U, D, L); break;
  }
}

void segment_sum_rows(uintptr_t grad, uintptr_t perm, uintptr_t seg, uintptr_t out, int U, int D, int L,
                      int grad_is_fp32, uintptr_t stream) {
  if (D % 8) throw std::invalid_argument("segment_sum_rows: D % 8 != 0");
  if (grad % 16 || out % 16) throw std::invalid_argument("segment_sum_rows: 16-byte alignment required");
  if (U <= 0) return;
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto P = reinterpret_cast<const int*>(perm);
  auto S = reinterpret_cast<const int*>(seg);
  auto O = reinterpret_cast<float*>(out);
  if (grad_is_fp32) launch_segment_sum<float>(reinterpret_cast<const void*>(grad), P, S, O, U, D, L, s);
  else launch_segment_sum<bf16>(reinterpret_cast<const void*>(grad), P, S, O, U, D, L, s);
  FTM_CHECK_LAUNCH();
}

void sparse_adagrad(uintptr_t table, uintptr_t accum, uintptr_t uids, uintptr_t g, int U, int D, int V, float lr,
                    float eps, uintptr_t stream) {
  if (D % 4) throw std::invalid_argument("sparse_adagrad: D % 4 != 0");
  if (table % 16 || accum % 16 || g % 16) throw std::invalid_argument("sparse_adagrad: 16-byte alignment required");
  if (U <= 0) return;
  hipLaunchKernelGGL(sparse_adagrad_kernel, dim3((U + 3) / 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<float*>(table), reinterpret_cast<float*>(accum), reinterpret_cast<const int*>(uids),
                     reinterpret_cast<const float*>(g), U, D, V, lr, eps);
  FTM_CHECK_LAUNCH();
}

void segment_starts(uintptr_t sorted, uintptr_t seg_id, uintptr_t seg, uintptr_t uids, int n, long long num_rows,
                    uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(segment_starts_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const long long*>(sorted), reinterpret_cast<const int*>(seg_id),
                     reinterpret_cast<int*>(seg), reinterpret_cast<int*>(uids), n, num_rows);
  FTM_CHECK_LAUNCH();
}

void register_embedding(pybind11::module_& m) {
  m.def("segment_starts", &segment_starts);
  m.def("embedding_bag_fwd", &embedding_bag_fwd);
  m.def("segment_sum_rows", &segment_sum_rows);
  m.def("sparse_adagrad", &sparse_adagrad);
}
