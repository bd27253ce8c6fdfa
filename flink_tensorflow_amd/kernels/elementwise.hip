// Standalone elementwise / normalisation kernels for ops the graph compiler cannot fuse
// into a producer epilogue ("standalone: one vectorized 16 B/lane HIP
// elementwise kernel"), and LRN for the GoogLeNet / inception5h body.
//
// binary:  out[i] = act(a[i] OP b(i)), bf16 in/out, fp32 math; b is a scalar, a vector
//          broadcast along the last dimension (bias-like, fp32), or a full bf16 tensor.
//          8 elements (16 B) per thread per step, grid-stride.
// lrn:     TF LRN over NHWC channels: y = x / (bias + alpha * sum_{|d|<=r} x[c+d]^2)^beta;
//          one thread per (pixel, 8-channel chunk), the 2r-channel halo read from the
//          neighbouring chunks (L1 hits: the pixel's channels are contiguous).
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

enum BinOp : int { OP_ADD = 0, OP_SUB = 1, OP_MUL = 2, OP_DIV = 3, OP_MAX = 4, OP_MIN = 5, OP_RSUB = 6, OP_RDIV = 7 };
enum BMode : int { B_SCALAR = 0, B_LASTDIM = 1, B_FULL = 2 };

template <int OP>
FTM_DEVICE float bin(float a, float b) {
  if constexpr (OP == OP_ADD) return a + b;
  else if constexpr (OP == OP_SUB) return a - b;
  else if constexpr (OP == OP_MUL) return a * b;
  else if constexpr (OP == OP_DIV) return a / b;
  else if constexpr (OP == OP_MAX) return fmaxf(a, b);
  else if constexpr (OP == OP_MIN) return fminf(a, b);
  else if constexpr (OP == OP_RSUB) return b - a;
  else return b / a;
}

template <int OP, int BM, int ACT>
__global__ __launch_bounds__(256) void binary_kernel(const bf16* __restrict__ a, const void* __restrict__ b,
                                                     bf16* __restrict__ y, long n8, int blen, float bscalar) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 av = reinterpret_cast<const bf16x8*>(a)[i];
    float bv[8];
    if constexpr (BM == B_SCALAR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = bscalar;
    } else if constexpr (BM == B_LASTDIM) {
      const int c = (int)((i * 8) % blen);
      const f32x4* bp = reinterpret_cast<const f32x4*>(static_cast<const float*>(b) + c);
      const f32x4 b0 = bp[0], b1 = bp[1];
      bv[0] = b0[0]; bv[1] = b0[1]; bv[2] = b0[2]; bv[3] = b0[3];
      bv[4] = b1[0]; bv[5] = b1[1]; bv[6] = b1[2]; bv[7] = b1[3];
    } else {
      const bf16x8 t = reinterpret_cast<const bf16x8*>(b)[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = (float)t[e];
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(apply_act<ACT>(bin<OP>((float)av[e], bv[e])));
    reinterpret_cast<bf16x8*>(y)[i] = o;
  }
}

__global__ __launch_bounds__(256) void lrn_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long P, int C,
                                                  int r, float bias, float alpha, float beta) {
  const int chunks = C / 8;
  const long total = P * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / chunks;
    const int c0 = (int)(i % chunks) * 8;
    const bf16* px = x + p * C;
    float sq[8 + 2 * 8];  // channels c0-8 .. c0+15 (r <= 8)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int cb = c0 + (k - 1) * 8;
      bf16x8 v = bf16x8{};
      if (cb >= 0 && cb < C) v = *reinterpret_cast<const bf16x8*>(px + cb);
#pragma unroll
      for (int e = 0; e < 8; ++e) sq[k * 8 + e] = (float)v[e] * (float)v[e];
    }
    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(px + c0);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
      for (int d = -r; d <= r; ++d) s += sq[8 + e + d];  // out-of-range channels were zero-filled
      o[e] = f2bf((float)xv[e] * __powf(bias + alpha * s, -beta));
    }
    reinterpret_cast<bf16x8*>(y + p * C)[c0 / 8] = o;
  }
}

int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

template <int OP, int BM>
void launch_act(const bf16* a, const void* b, bf16* y, long n8, int blen, float bs, int act, hipStream_t s) {
  dim3 g(grid_for(n8, 256)), t(256);
  switch (act) {
    case ACT_NONE: hipLaunchKernelGGL((binary_kernel<OP, BM, ACT_NONE>), g, t, 0, s, a, b, y, n8, blen, bs); break;
    case ACT_RELU: hipLaunchKernelGGL((binary_kernel<OP, BM, ACT_RELU>), g, t, 0, s, a, b, y, n8, blen, bs); break;
    case ACT_RELU6: hipLaunchKernelGGL((binary_kernel<OP, BM, ACT_RELU6>), g, t, 0, s, a, b, y, n8, blen, bs); break;
    case ACT_SIGMOID: hipLaunchKernelGGL((binary_kernel<OP, BM, ACT_SIGMOID>), g, t, 0, s, a, b, y, n8, blen, bs); break;
    case ACT_TANH: hipLaunchKernelGGL((binary_kernel<OP, BM, ACT_TANH>), g, t, 0, s, a, b, y, n8, blen, bs); break;
    case ACT_GELU_TANH:
      hipLaunchKernelGGL((binary_kernel<OP, BM, ACT_GELU_TANH>), g, t, 0, s, a, b, y, n8, blen, bs);
      break;
    default: throw std::invalid_argument("elementwise: unknown activation " + std::to_string(act));
  }
}

template <int OP>
void launch_mode(const bf16* a, const void* b, bf16* y, long n8, int mode, int blen, float bs, int act, hipStream_t s) {
  switch (mode) {
    case B_SCALAR: launch_act<OP, B_SCALAR>(a, b, y, n8, blen, bs, act, s); break;
    case B_LASTDIM: launch_act<OP, B_LASTDIM>(a, b, y, n8, blen, bs, act, s); break;
    case B_FULL: launch_act<OP, B_FULL>(a, b, y, n8, blen, bs, act, s); break;
    default: throw std::invalid_argument("elementwise: unknown broadcast mode");
  }
}

}  // namespace

// out = act(a OP b); mode 0: b = bscalar, 1: b fp32 [blen] along the last dim, 2: b bf16 [n]
void binary_bf16(int op, uintptr_t a, uintptr_t b, uintptr_t y, long n, int mode, int blen, float bscalar, int act,
                 uintptr_t stream) {
  if (n % 8) throw std::invalid_argument("binary_bf16: element count must be a multiple of 8");
  if (mode == B_LASTDIM && (blen % 8 || blen <= 0)) throw std::invalid_argument("binary_bf16: vector length % 8");
  if (a % 16 || y % 16 || (mode != B_SCALAR && b % 16)) throw std::invalid_argument("binary_bf16: 16-byte alignment");
  if (n == 0) return;
  auto A = reinterpret_cast<const bf16*>(a);
  auto Bp = reinterpret_cast<const void*>(b);
  auto Y = reinterpret_cast<bf16*>(y);
  auto s = reinterpret_cast<hipStream_t>(stream);
  const long n8 = n / 8;
  switch (op) {
    case OP_ADD: launch_mode<OP_ADD>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_SUB: launch_mode<OP_SUB>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_MUL: launch_mode<OP_MUL>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_DIV: launch_mode<OP_DIV>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_MAX: launch_mode<OP_MAX>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_MIN: launch_mode<OP_MIN>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_RSUB: launch_mode<OP_RSUB>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    case OP_RDIV: launch_mode<OP_RDIV>(A, Bp, Y, n8, mode, blen, bscalar, act, s); break;
    default: throw std::invalid_argument("binary_bf16: unknown op " + std::to_string(op));
  }
  FTM_CHECK_LAUNCH();
}

void lrn_bf16(uintptr_t x, uintptr_t y, long P, int C, int r, float bias, float alpha, float beta, uintptr_t stream) {
  if (C % 8) throw std::invalid_argument("lrn_bf16: C % 8 != 0");
  if (r < 0 || r > 8) throw std::invalid_argument("lrn_bf16: depth_radius must be in [0, 8]");
  if (x % 16 || y % 16) throw std::invalid_argument("lrn_bf16: 16-byte alignment");
  if (P == 0) return;
  hipLaunchKernelGGL(lrn_kernel, dim3(grid_for(P * (C / 8), 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const bf16*>(x), reinterpret_cast<bf16*>(y),
                     P, C, r, bias, alpha, beta);
  FTM_CHECK_LAUNCH();
}

// Row gather out[r] = x[idx[r]] (rows of `row_bytes`, a multiple of 16): the first-token
// (CLS) rows of a token-packed encoder.  One thread per 16-byte chunk; an index outside
// [0, n_src) writes zeros (a padded batch row has no token).
namespace {
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint4* __restrict__ x, const int* __restrict__ idx,
                                                          uint4* __restrict__ y, int n_out, int n_src, int chunks) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)n_out * chunks) return;
  const int r = (int)(i / chunks), c = (int)(i % chunks);
  const int src = idx[r];
  y[i] = (src >= 0 && src < n_src) ? x[(long)src * chunks + c] : make_uint4(0u, 0u, 0u, 0u);
}
}  // namespace

void gather_rows(uintptr_t x, uintptr_t idx, uintptr_t y, int n_out, int n_src, long row_bytes, uintptr_t stream) {
  if (row_bytes % 16 || row_bytes <= 0) throw std::invalid_argument("gather_rows: row bytes must be a positive multiple of 16");
  if (x % 16 || y % 16 || idx % 4) throw std::invalid_argument("gather_rows: 16-byte aligned rows, 4-byte indices");
  if (n_out <= 0) return;
  const int chunks = (int)(row_bytes / 16);
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)(((long)n_out * chunks + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint4*>(x),
                     reinterpret_cast<const int*>(idx), reinterpret_cast<uint4*>(y), n_out, n_src, chunks);
  FTM_CHECK_LAUNCH();
}

namespace {

// One wave that holds its stream for ``ticks`` of the 100 MHz constant real-time counter
// (s_memrealtime: a counter read, sleeping between reads) — a stream-ordered delay that
// occupies one wave slot of one CU.  Used to start a restarting pipeline's second lane a
// fraction of a batch after the first (batching/engine.py, lane phase).
__global__ __launch_bounds__(64) void stream_delay_kernel(long long ticks) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

}  // namespace

// delays ``stream`` by ``us`` microseconds (GPU-side; returns immediately)
void stream_delay(double us, uintptr_t stream) {
  if (us <= 0) return;
  if (us > 1e6) throw std::invalid_argument("stream_delay: at most one second");
  hipLaunchKernelGGL(stream_delay_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     (long long)(us * 100.0));
  FTM_CHECK_LAUNCH();
}

void register_elementwise(pybind11::module_& m) {
  m.def("stream_delay", &stream_delay);
  m.def("gather_rows", &gather_rows);
  m.def("binary_bf16", &binary_bf16);
  m.def("lrn_bf16", &lrn_bf16);
}
