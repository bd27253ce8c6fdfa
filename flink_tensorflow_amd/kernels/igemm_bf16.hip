// Implicit-GEMM convolution / GEMM on CDNA4 MFMA (bf16 in, fp32 accumulate, bf16 out)
// with a fused epilogue:  y = act(acc + bias[c] + residual[m, c]).
//
// Used for every Conv2D / MatMul of the compiled GPU plan (ResNet-50, Inception-v3,
// BERT projections, Wide&Deep towers).  Layouts (TF-native NHWC):
//   x  [N, H, W, Cin]  bf16, Cin % 8 == 0 (the stem pads 3 -> 8 in the preprocess kernel)
//   w  [Cout, KH, KW, Cin] bf16  ("OHWI", K-contiguous rows; BN folded in at load time)
//   y  [N, Ho, Wo, ldy] bf16, written at channel offset y_coff (concat-by-stride-write)
// GEMM view: C^T[Cout, M] = W[Cout, K] . X^T[K, M]; M = N*Ho*Wo pixels, K = KH*KW*Cin.
// MFMA operand A = weight rows (output channels), operand B = im2col pixel rows, so an
// accumulator lane holds 4 consecutive channels of one pixel (8-byte bf16 stores).
//
// Tiling: 128 pixels x 128 channels x BK=64 per 256-thread workgroup (4 waves, 2x2, each
// 64x64 = 4x4 tiles of v_mfma_f32_16x16x32_bf16).  Register-staged global->LDS double
// buffer (issue the next tile's 16-B loads before the MFMAs, write them to the other
// LDS buffer after: guide T14), one barrier per K-tile.  LDS rows are 128 B, chunk-XOR
// swizzled (chunk ^ (row & 7)) so the ds_read_b128 fragment reads are conflict-free
// (guide T2).  Blocks are remapped XCD-aware so the channel tiles of one pixel tile
// share an L2 (guide T1).
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int BM = 128;  // pixels per tile
constexpr int BN = 128;  // output channels per tile
constexpr int BK = 64;   // K per stage
constexpr int NT = 256;  // threads

struct IgemmParams {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  bf16* y;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, sh, sw, ph, pw, dh, dw;
  int M, K;
  int ldx;          // GEMM mode: row stride of X in elements
  int ldy, y_coff;  // output pixel stride (elements) and channel offset
  int ldr;          // residual pixel stride
  int tiles_m, tiles_n;
};

FTM_DEVICE int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

template <bool CONV, int ACT, bool HAS_BIAS, bool HAS_RES>
__global__ __launch_bounds__(NT, 2) void igemm_bf16_kernel(IgemmParams p) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (BM + BN) * BK];  // 64 KiB
  bf16* Xs = smem;                 // [2][BM][BK]
  bf16* Ws = smem + 2 * BM * BK;   // [2][BN][BK]

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile % p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wp = wave & 1;   // pixel half of the tile
  const int wc = wave >> 1;  // channel half

  // ---- per-thread staging assignment: fixed k-chunk, 4 rows (r0 + 32 i)
  const int kc = tid & 7;
  const int r0 = tid >> 3;

  // pixel-row precompute (conv): base offset of image n, top-left input coords
  int xbase[4], hb[4], wb[4];
  bool mvalid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = m0 + r0 + 32 * i;
    mvalid[i] = m < p.M;
    int mm = mvalid[i] ? m : 0;
    if constexpr (CONV) {
      int wo = mm % p.Wo;
      int t = mm / p.Wo;
      int ho = t % p.Ho;
      int n = t / p.Ho;
      xbase[i] = n * p.H * p.W * p.Cin;
      hb[i] = ho * p.sh - p.ph;
      wb[i] = wo * p.sw - p.pw;
    } else {
      xbase[i] = mm * p.ldx;
      hb[i] = 0;
      wb[i] = 0;
    }
  }
  const bf16* wrow[4];
  bool nvalid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int co = n0 + r0 + 32 * i;
    nvalid[i] = co < p.Cout;
    wrow[i] = p.w + (size_t)(nvalid[i] ? co : 0) * p.K;
  }

  u32x4 xr[4], wr[4];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

  auto load_tile = [&](int k0) {
    const int k = k0 + kc * 8;
    const bool kvalid = k < p.K;
    if constexpr (CONV) {
      int kidx = k / p.Cin;
      int ci = k - kidx * p.Cin;
      int kh = kidx / p.KW;
      int kw = kidx - kh * p.KW;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int hi = hb[i] + kh * p.dh;
        int wi = wb[i] + kw * p.dw;
        bool ok = kvalid && mvalid[i] && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        xr[i] = ok ? *reinterpret_cast<const u32x4*>(p.x + xbase[i] + ((size_t)hi * p.W + wi) * p.Cin + ci) : zero4;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bool ok = kvalid && mvalid[i];
        xr[i] = ok ? *reinterpret_cast<const u32x4*>(p.x + (size_t)xbase[i] + k) : zero4;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = kvalid && nvalid[i];
      wr[i] = ok ? *reinterpret_cast<const u32x4*>(wrow[i] + k) : zero4;
    }
  };
  auto store_tile = [&](int buf) {
    bf16* xs = Xs + buf * BM * BK;
    bf16* ws = Ws + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = r0 + 32 * i;
      *reinterpret_cast<u32x4*>(xs + swz(row, kc)) = xr[i];
      *reinterpret_cast<u32x4*>(ws + swz(row, kc)) = wr[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fchunk = lane >> 4;  // 0..3 -> k offset 8*fchunk within a 32-deep substep

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
    const bf16* xs = Xs + buf * BM * BK;
    const bf16* ws = Ws + buf * BN * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4], b[4];
      const int chunk = ks * 4 + fchunk;
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ws + swz(wc * 64 + i * 16 + frow, chunk));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(xs + swz(wp * 64 + j * 16 + frow, chunk));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds channels c..c+3 of pixel m for each (i, j) fragment
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = n0 + wc * 64 + i * 16 + (lane >> 4) * 4;
    if (c >= p.Cout) continue;
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if constexpr (HAS_BIAS) bv = *reinterpret_cast<const f32x4*>(p.bias + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wp * 64 + j * 16 + (lane & 15);
      if (m >= p.M) continue;
      f32x4 v = acc[i][j] + bv;
      if constexpr (HAS_RES) {
        bf16x4 r = *reinterpret_cast<const bf16x4*>(p.res + (size_t)m * p.ldr + c);
        v[0] += (float)r[0];
        v[1] += (float)r[1];
        v[2] += (float)r[2];
        v[3] += (float)r[3];
      }
      bf16x4 o;
      o[0] = f2bf(apply_act<ACT>(v[0]));
      o[1] = f2bf(apply_act<ACT>(v[1]));
      o[2] = f2bf(apply_act<ACT>(v[2]));
      o[3] = f2bf(apply_act<ACT>(v[3]));
      *reinterpret_cast<bf16x4*>(p.y + (size_t)m * p.ldy + p.y_coff + c) = o;
    }
  }
}

template <bool CONV, int ACT>
void launch_act(const IgemmParams& p, hipStream_t s) {
  dim3 grid(p.tiles_m * p.tiles_n), block(NT);
  const bool hb = p.bias != nullptr, hr = p.res != nullptr;
  if (hb && hr) hipLaunchKernelGGL((igemm_bf16_kernel<CONV, ACT, true, true>), grid, block, 0, s, p);
  else if (hb) hipLaunchKernelGGL((igemm_bf16_kernel<CONV, ACT, true, false>), grid, block, 0, s, p);
  else if (hr) hipLaunchKernelGGL((igemm_bf16_kernel<CONV, ACT, false, true>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((igemm_bf16_kernel<CONV, ACT, false, false>), grid, block, 0, s, p);
}

template <bool CONV>
void launch(const IgemmParams& p, int act, hipStream_t s) {
  switch (act) {
    case ACT_NONE: launch_act<CONV, ACT_NONE>(p, s); break;
    case ACT_RELU: launch_act<CONV, ACT_RELU>(p, s); break;
    case ACT_GELU_TANH: launch_act<CONV, ACT_GELU_TANH>(p, s); break;
    case ACT_SIGMOID: launch_act<CONV, ACT_SIGMOID>(p, s); break;
    case ACT_TANH: launch_act<CONV, ACT_TANH>(p, s); break;
    case ACT_RELU6: launch_act<CONV, ACT_RELU6>(p, s); break;
    default: throw std::invalid_argument("unknown activation " + std::to_string(act));
  }
  FTM_CHECK_LAUNCH();
}

void check_align(uintptr_t ptr, int bytes, const char* what) {
  if (ptr % bytes) throw std::invalid_argument(std::string(what) + " is not " + std::to_string(bytes) + "-byte aligned");
}

}  // namespace

// Conv2D NHWC implicit GEMM.  Shapes are validated here (host side) before any launch.
void conv2d_nhwc_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int N, int H, int W,
                      int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw, int Ho, int Wo,
                      int ldy, int y_coff, int ldr, int act, uintptr_t stream) {
  if (Cin % 8) throw std::invalid_argument("conv2d_nhwc_bf16: Cin must be a multiple of 8");
  if (Cout % 4 || ldy % 4 || y_coff % 4) throw std::invalid_argument("conv2d_nhwc_bf16: Cout/ldy/y_coff % 4 != 0");
  if (res && ldr % 4) throw std::invalid_argument("conv2d_nhwc_bf16: residual stride % 4 != 0");
  if (N <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0) throw std::invalid_argument("conv2d_nhwc_bf16: empty problem");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 8, "y");
  if (bias) check_align(bias, 16, "bias");
  if (res) check_align(res, 8, "residual");
  IgemmParams p{};
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const bf16*>(res);
  p.y = reinterpret_cast<bf16*>(y);
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.KH = KH; p.KW = KW; p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.M = N * Ho * Wo;
  p.K = KH * KW * Cin;
  p.ldx = Cin;
  p.ldy = ldy; p.y_coff = y_coff; p.ldr = ldr;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (Cout + BN - 1) / BN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool pointwise = KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
  if (pointwise) {
    p.ldx = Cin;
    launch<false>(p, act, s);  // 1x1/s1: the input IS the [M, Cin] matrix
  } else {
    launch<true>(p, act, s);
  }
}

// Y[M, N] = act(X[M, K] . W[N, K]^T + bias + res).  X row stride ldx, Y row stride ldy.
void gemm_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int M, int N, int K, int ldx,
               int ldy, int ldr, int act, uintptr_t stream) {
  if (K % 8 || ldx % 8) throw std::invalid_argument("gemm_bf16: K and ldx must be multiples of 8");
  if (N % 4 || ldy % 4) throw std::invalid_argument("gemm_bf16: N and ldy must be multiples of 4");
  if (M <= 0 || N <= 0) throw std::invalid_argument("gemm_bf16: empty problem");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 8, "y");
  if (bias) check_align(bias, 16, "bias");
  IgemmParams p{};
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const bf16*>(res);
  p.y = reinterpret_cast<bf16*>(y);
  p.M = M; p.Cout = N; p.K = K; p.ldx = ldx; p.ldy = ldy; p.y_coff = 0; p.ldr = ldr;
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = (N + BN - 1) / BN;
  launch<false>(p, act, reinterpret_cast<hipStream_t>(stream));
}

void register_igemm(pybind11::module_& m) {
  m.def("conv2d_nhwc_bf16", &conv2d_nhwc_bf16);
  m.def("gemm_bf16", &gemm_bf16);
}
