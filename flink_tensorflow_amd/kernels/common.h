// Shared helpers for the CDNA4 (gfx950) kernels of flink_tensorflow_amd.
//
// Conventions: wave = 64 lanes; bf16 values move as 16-byte vectors (8 x bf16) in every
// memory-bound path (guide Guideline 13); MFMA fragments use the gfx950
// v_mfma_f32_16x16x32_bf16 lane maps (guide §3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define FTM_DEVICE __device__ __forceinline__

FTM_DEVICE float bf2f(bf16 v) { return (float)v; }
FTM_DEVICE bf16 f2bf(float v) { return (bf16)v; }  // RNE, v_cvt_pk_bf16_f32 at -O3

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU_TANH = 2, ACT_SIGMOID = 3, ACT_TANH = 4, ACT_RELU6 = 5 };

template <int ACT>
FTM_DEVICE float apply_act(float x) {
  if constexpr (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == ACT_RELU6) return fminf(fmaxf(x, 0.f), 6.f);
  else if constexpr (ACT == ACT_GELU_TANH) {
    // 0.5 x (1 + tanh(u)) == x * sigmoid(2u): one v_exp_f32 + one v_rcp_f32 instead of a
    // libm tanhf (the FFN1 epilogue runs it on every one of B*S*3072 outputs)
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u2 = 2.f * k0 * (x + k1 * x * x * x);
    return __fdividef(x, 1.f + __expf(-u2));
  } else if constexpr (ACT == ACT_SIGMOID) return __fdividef(1.f, 1.f + __expf(-x));
  else if constexpr (ACT == ACT_TANH) return 2.f * __fdividef(1.f, 1.f + __expf(-2.f * x)) - 1.f;
  else return x;
}

// Bijective XCD-aware block remap (guide §5 "XCD swizzle must be bijective", T1):
// consecutive logical tiles land on the same XCD (blocks b and b+8 share one XCD).
FTM_DEVICE int xcd_remap(int orig, int nwg) {
  constexpr int NXCD = 8;
  if (nwg <= NXCD) return orig;
  int q = nwg / NXCD, r = nwg % NXCD;
  int xcd = orig % NXCD;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / NXCD;
}

FTM_DEVICE float wave_reduce_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
FTM_DEVICE float wave_reduce_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

#define FTM_CHECK_LAUNCH()                                                                   \
  do {                                                                                       \
    hipError_t e_ = hipGetLastError();                                                       \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP launch failed: ") + hipGetErrorString(e_)); \
  } while (0)
