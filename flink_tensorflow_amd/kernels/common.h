// Shared helpers for the CDNA4 (gfx950) kernels of flink_tensorflow_amd.
//
// Conventions: wave = 64 lanes; bf16 values move as 16-byte vectors (8 x bf16) in every
// memory-bound path (guide Guideline 13); MFMA fragments use the gfx950
// v_mfma_f32_16x16x32_bf16 lane maps (guide §3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

// Wave priority (s_setprio 1) around the MFMA clusters of the persistent / direct conv
// kernels (conv3x3c64, pw_res, dconv) stays off: measured neutral for these (ResNet-50
// 78.36k vs 78.30k, 3 pairs; they hold most of a CU's LDS, so little of the sibling lane
// co-resides with them: profiles/r02_igemm_prio), unlike igemm / gemm_pp / conv_pp.
constexpr int ftm_mfma_prio() { return 0; }
#define FTM_PRIO_HI(p)                          \
  do {                                          \
    if (p) __builtin_amdgcn_s_setprio(1);       \
  } while (0)
#define FTM_PRIO_LO(p)                          \
  do {                                          \
    if (p) __builtin_amdgcn_s_setprio(0);       \
  } while (0)

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define FTM_DEVICE __device__ __forceinline__

FTM_DEVICE float bf2f(bf16 v) { return (float)v; }
FTM_DEVICE bf16 f2bf(float v) { return (bf16)v; }  // RNE, v_cvt_pk_bf16_f32 at -O3

// ACT_DRELU (GEMM epilogues with a residual operand only): y = res > 0 ? acc : 0 — the
// ReLU backward mask of the layer input, fused into the dX GEMM of a training step.
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU_TANH = 2, ACT_SIGMOID = 3, ACT_TANH = 4, ACT_RELU6 = 5, ACT_DRELU = 6 };

template <int ACT>
FTM_DEVICE float apply_act(float x) {
  if constexpr (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == ACT_RELU6) return fminf(fmaxf(x, 0.f), 6.f);
  else if constexpr (ACT == ACT_GELU_TANH) {
    // 0.5 x (1 + tanh(u)) == x / (1 + exp(-2u)), u = k0 (x + k1 x^3): 7 VALU per output —
    // mul, fma, mul, v_exp_f32 (base 2, log2(e) folded into the constants), add, v_rcp_f32,
    // mul.  (__fdividef / __expf lower to the IEEE division sequence here: ~20 VALU per
    // output, which made GELU ~20 % of the FFN1 GEMM.)  Large |u|: exp2 -> inf or 0, so the
    // result -> 0 or x, no NaN.
    constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f;
    constexpr float c1 = c0 * 0.044715f;
    const float t = x * __builtin_fmaf(c1, x * x, c0);
    return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
  } else if constexpr (ACT == ACT_SIGMOID) {
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
  } else if constexpr (ACT == ACT_TANH) {
    return 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * x)) - 1.f;
  } else return x;
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
