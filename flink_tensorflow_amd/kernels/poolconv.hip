// A 3x3 / stride-2 max pool and the 1x1 convolution that consumes it as ONE fp8 kernel
// (Inception-v3's MaxPool_3a -> Conv2d_3b_1x1: 147x147x64 -> 73x73x64 -> 73x73x80).
//
// Apart, the pool reads the 147x147 tensor and writes the 73x73 one, and the 1x1 conv —
// a K = 64 GEMM, far too short to hide its loads — reads it back: two memory-bound
// launches (≈140 + 137 µs at B = 256, profiles/r04_j).  Here a workgroup owns 256 pooled
// pixels:
//   1. it builds their pooled rows in LDS straight from the pre-pool tensor: each thread
//      takes (pixel, 16-B channel chunk) items, issues the nine 16-B window loads, and
//      reduces them with byte-wise maxima over an order-preserving key of the e4m3 bytes
//      (sign-magnitude -> unsigned: any sign, exactly the max of the fp8 values);
//   2. one MFMA K-step (v_mfma_scale 16x16x128 f8f6f4; K = Cin bytes zero-padded to 128)
//      per 16x16 fragment: 4 waves x 4 pixel fragments x (Cout / 16) channel fragments,
//      the [Cout][Cin] filter bank in LDS;
//   3. dequantise (w_scale * x_scale per channel) + bias + activation, requantise to e4m3
//      with the consumer's scale and store each lane's 4 channels straight from the
//      accumulators (16 contiguous bytes per pixel per fragment; concat-offset capable).
// Load items are groups of 4 adjacent pooled pixels x one 16-B chunk: inside a pooled row
// they share window columns (27 loads for 4 outputs instead of 36).
// The pooled tensor never exists in memory: one read of the pre-pool tensor (L2 serves
// the window overlap) and one write of the conv output.
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));

namespace {

struct PoolConvParams {
  const uint8_t* x;    // [N, H, W, CIN] e4m3
  const uint8_t* w;    // [Cout][CIN] e4m3
  const float* cs;     // [Cout]: w_scale * x_scale
  const float* bias;   // [Cout]
  uint8_t* y;          // [M][ldy] e4m3 (at y_coff)
  float out_q;         // 1 / consumer scale
  int H, W, Hp, Wp, Cout, ldy, y_coff;
  long M;              // N * Hp * Wp pooled pixels
};

constexpr int PX = 256;  // pooled pixels per workgroup: 4 waves x 4 fragments x 16

// e4m3 byte -> unsigned key ordered like the value (positive: b | 0x80, negative: ~b)
FTM_DEVICE u8x16 fp8_key(u8x16 v) { return v ^ ((v >> 7) * (unsigned char)0x7F + (unsigned char)0x80); }
FTM_DEVICE u8x16 fp8_unkey(u8x16 k) {
  return k ^ (((k >> 7) ^ (unsigned char)1) * (unsigned char)0x7F + (unsigned char)0x80);
}

FTM_DEVICE uint32_t pack4_e4m3(float a, float b, float c, float d) {
  const float M = 448.f;
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -M), M), fminf(fmaxf(b, -M), M), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -M), M), fminf(fmaxf(d, -M), M), w, true);
  return (uint32_t)w;
}

FTM_DEVICE i32x8 ld32(const uint8_t* p) {
  const u32x4 lo = *reinterpret_cast<const u32x4*>(p), hi = *reinterpret_cast<const u32x4*>(p + 16);
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

// one pooled pixel's 16-B channel chunk: the max of its 3x3 window (keys, order-preserving)
FTM_DEVICE u8x16 pool_chunk(const uint8_t* base, int W, int cin) {
  u8x16 v[9];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) v[dy * 3 + dx] = *reinterpret_cast<const u8x16*>(base + ((size_t)dy * W + dx) * cin);
  u8x16 k = fp8_key(v[0]);
#pragma unroll
  for (int i = 1; i < 9; ++i) k = __builtin_elementwise_max(k, fp8_key(v[i]));
  return fp8_unkey(k);
}

template <int CIN, int I, int ACT>
__global__ __launch_bounds__(256) void pool_conv1x1_fp8_kernel(PoolConvParams p) {
  static_assert(CIN == 64, "one 128-byte MFMA K-step with half of it zero");
  constexpr int XP = CIN + 16;      // pooled-row pitch in LDS (bytes; +16 spreads banks)
  constexpr int OC = I * 16;        // output channels (Cout == OC)
  constexpr int CH = CIN / 16;      // 16-B chunks per pooled row
  constexpr int G = 4;              // pooled pixels per load item (adjacent along the row)
  static_assert(PX / G * CH == 256, "one load item per thread");
  __shared__ __attribute__((aligned(16))) uint8_t Xs[PX * XP];
  __shared__ __attribute__((aligned(16))) uint8_t Ws[OC * XP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long m0 = (long)blockIdx.x * PX;

  // ---- 1. filter bank and pooled rows into LDS
  for (int q = tid; q < OC * CH; q += 256) {
    const int r = q / CH, c = q - r * CH;
    *reinterpret_cast<u32x4*>(Ws + r * XP + c * 16) = *reinterpret_cast<const u32x4*>(p.w + (size_t)r * CIN + c * 16);
  }
  {
    // thread = (group of G adjacent pooled pixels, 16-B chunk): a group inside one pooled
    // row shares window columns — 3 rows x (2G + 1) loads for G outputs instead of 9 G
    const int c = tid % CH, g = tid / CH;
    const long mg = m0 + (long)g * G;
    const long t = mg / p.Wp;
    const int pw = (int)(mg - t * p.Wp), ph = (int)(t % p.Hp), n = (int)(t / p.Hp);
    u8x16 out[G];
    if (mg + G <= p.M && pw + G <= p.Wp) {
      const uint8_t* base = p.x + (((size_t)n * p.H + 2 * ph) * p.W + 2 * pw) * CIN + c * 16;
      u8x16 k[G];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        u8x16 v[2 * G + 1];
#pragma unroll
        for (int x = 0; x < 2 * G + 1; ++x)
          v[x] = fp8_key(*reinterpret_cast<const u8x16*>(base + ((size_t)dy * p.W + x) * CIN));
#pragma unroll
        for (int o = 0; o < G; ++o) {
          const u8x16 r = __builtin_elementwise_max(__builtin_elementwise_max(v[2 * o], v[2 * o + 1]), v[2 * o + 2]);
          k[o] = dy == 0 ? r : __builtin_elementwise_max(k[o], r);
        }
      }
#pragma unroll
      for (int o = 0; o < G; ++o) out[o] = fp8_unkey(k[o]);
    } else {  // the group crosses a pooled row or the end: pixel by pixel
#pragma unroll
      for (int o = 0; o < G; ++o) {
        const long m = mg + o;
        out[o] = u8x16{};
        if (m < p.M) {
          const long tt = m / p.Wp;
          const int pwo = (int)(m - tt * p.Wp), pho = (int)(tt % p.Hp), no = (int)(tt / p.Hp);
          out[o] = pool_chunk(p.x + (((size_t)no * p.H + 2 * pho) * p.W + 2 * pwo) * CIN + c * 16, p.W, CIN);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < G; ++o) *reinterpret_cast<u8x16*>(Xs + (g * G + o) * XP + c * 16) = out[o];
  }
  __syncthreads();

  // ---- 2./3. per pixel fragment: one MFMA K-step (lane groups fq = 0, 1 carry the 64
  // channel bytes, 2, 3 zeros), then dequantise + bias + act + requantise and store each
  // lane's 4 channels of its pixel (16 contiguous bytes per pixel per 16-channel fragment)
  const int frow = lane & 15, fq = lane >> 4;
  const bool kval = fq * 32 < CIN;
  const i32x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  i32x8 a[I];
#pragma unroll
  for (int i = 0; i < I; ++i) a[i] = kval ? ld32(Ws + (i * 16 + frow) * XP + fq * 32) : zero;
  f32x4 sv[I], bv[I];
#pragma unroll
  for (int i = 0; i < I; ++i) {
    sv[i] = *reinterpret_cast<const f32x4*>(p.cs + i * 16 + fq * 4);
    bv[i] = *reinterpret_cast<const f32x4*>(p.bias + i * 16 + fq * 4);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pl = (wave * 4 + j) * 16 + frow;
    const i32x8 b = kval ? ld32(Xs + pl * XP + fq * 32) : zero;
    const long m = m0 + pl;
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const f32x4 acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0,
                                                                         127, 0, 127);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act<ACT>(acc[r] * sv[i][r] + bv[i][r]) * p.out_q;
      if (m < p.M)
        *reinterpret_cast<uint32_t*>(p.y + m * p.ldy + p.y_coff + i * 16 + fq * 4) = pack4_e4m3(v[0], v[1], v[2], v[3]);
    }
  }
}

template <int I>
void launch_i(const PoolConvParams& p, int act, hipStream_t s) {
  const dim3 grid((unsigned)((p.M + PX - 1) / PX)), block(256);
  if (act == ACT_RELU) hipLaunchKernelGGL((pool_conv1x1_fp8_kernel<64, I, ACT_RELU>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((pool_conv1x1_fp8_kernel<64, I, ACT_NONE>), grid, block, 0, s, p);
}

}  // namespace

bool pool_conv1x1_fp8_supported(int Cin, int Cout) {
  return Cin == 64 && (Cout == 64 || Cout == 80 || Cout == 96 || Cout == 128);
}

// x: [N, H, W, Cin] e4m3; pooled 3x3 / stride 2 VALID -> [N, Hp, Wp, Cin]; w: [Cout][Cin] e4m3.
void pool_conv1x1_fp8(uintptr_t x, uintptr_t w, uintptr_t cs, uintptr_t bias, uintptr_t y, int N, int H, int W,
                      int Cin, int Cout, int ldy, int y_coff, float out_q, int act, uintptr_t stream) {
  if (!pool_conv1x1_fp8_supported(Cin, Cout))
    throw std::invalid_argument("pool_conv1x1_fp8: Cin 64 and Cout in {64, 80, 96, 128} (got " + std::to_string(Cin) +
                                ", " + std::to_string(Cout) + ")");
  if (act != ACT_NONE && act != ACT_RELU) throw std::invalid_argument("pool_conv1x1_fp8: activation none / relu");
  if (H < 3 || W < 3 || N < 1) throw std::invalid_argument("pool_conv1x1_fp8: input smaller than the window");
  if (ldy % 16 || y_coff % 16 || y_coff + Cout > ldy) throw std::invalid_argument("pool_conv1x1_fp8: ldy / y_coff");
  if (x % 16 || w % 16 || y % 16 || cs % 16 || bias % 16) throw std::invalid_argument("pool_conv1x1_fp8: alignment");
  PoolConvParams p{};
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.cs = reinterpret_cast<const float*>(cs);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.out_q = out_q;
  p.H = H; p.W = W; p.Hp = (H - 3) / 2 + 1; p.Wp = (W - 3) / 2 + 1;
  p.Cout = Cout; p.ldy = ldy; p.y_coff = y_coff;
  p.M = (long)N * p.Hp * p.Wp;
  auto s = reinterpret_cast<hipStream_t>(stream);
  switch (Cout / 16) {
    case 4: launch_i<4>(p, act, s); break;
    case 5: launch_i<5>(p, act, s); break;
    case 6: launch_i<6>(p, act, s); break;
    default: launch_i<8>(p, act, s); break;
  }
  FTM_CHECK_LAUNCH();
}

void register_poolconv(pybind11::module_& m) {
  m.def("pool_conv1x1_fp8", &pool_conv1x1_fp8);
  m.def("pool_conv1x1_fp8_supported", &pool_conv1x1_fp8_supported);
}
