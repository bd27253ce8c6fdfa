// Transformer kernels (BERT-base path): LayerNorm with fused residual add.
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

// y = LN(x + r) * gamma + beta over the last dim D (D % 8 == 0, D <= 64*8*MAXV).
// One wave per row; each lane holds ceil(D/512) 16-byte chunks in registers.
template <int MAXV>
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        bf16* __restrict__ y, bf16* __restrict__ sum_out, int rows,
                                                        int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* xp = x + (size_t)row * D;
  const bf16* rp = r ? r + (size_t)row * D : nullptr;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < D) {
      bf16x8 a = *reinterpret_cast<const bf16x8*>(xp + c);
      bf16x8 b;
      if (rp) b = *reinterpret_cast<const bf16x8*>(rp + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = (float)a[e] + (rp ? (float)b[e] : 0.f);
        v[i][e] = t;
        s += t;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  const float mean = wave_reduce_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < D)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = v[i][e] - mean;
        q += d * d;
      }
  }
  const float rstd = rsqrtf(wave_reduce_sum(q) / D + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c >= D) continue;
    bf16x8 o, so;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf((v[i][e] - mean) * rstd * gamma[c + e] + beta[c + e]);
      so[e] = f2bf(v[i][e]);
    }
    *reinterpret_cast<bf16x8*>(y + (size_t)row * D + c) = o;
    if (sum_out) *reinterpret_cast<bf16x8*>(sum_out + (size_t)row * D + c) = so;
  }
}

}  // namespace

void layernorm_bf16(uintptr_t x, uintptr_t r, uintptr_t gamma, uintptr_t beta, uintptr_t y, uintptr_t sum_out,
                    int rows, int D, float eps, uintptr_t stream) {
  if (D % 8) throw std::invalid_argument("layernorm: D must be a multiple of 8");
  if (D > 64 * 8 * 4) throw std::invalid_argument("layernorm: D > 2048 not supported");
  dim3 grid((rows + 3) / 4), block(256);
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto X = reinterpret_cast<const bf16*>(x);
  auto R = reinterpret_cast<const bf16*>(r);
  auto G = reinterpret_cast<const float*>(gamma);
  auto Bt = reinterpret_cast<const float*>(beta);
  auto Y = reinterpret_cast<bf16*>(y);
  auto S = reinterpret_cast<bf16*>(sum_out);
  if (D <= 512) hipLaunchKernelGGL(layernorm_kernel<1>, grid, block, 0, s, X, R, G, Bt, Y, S, rows, D, eps);
  else if (D <= 1024) hipLaunchKernelGGL(layernorm_kernel<2>, grid, block, 0, s, X, R, G, Bt, Y, S, rows, D, eps);
  else hipLaunchKernelGGL(layernorm_kernel<4>, grid, block, 0, s, X, R, G, Bt, Y, S, rows, D, eps);
  FTM_CHECK_LAUNCH();
}

void register_transformer(pybind11::module_& m) { m.def("layernorm_bf16", &layernorm_bf16); }
