// Implicit-GEMM convolution / GEMM on CDNA4 MFMA (bf16 in, fp32 accumulate, bf16 out)
// with a fused epilogue:  y = act(acc + bias[c] + residual[m, c]).
//
// Used for every Conv2D / MatMul of the compiled GPU plan (ResNet-50, Inception-v3,
// BERT projections, Wide&Deep towers).  Layouts (TF-native NHWC):
//   x  [N, H, W, Cin]  bf16, Cin % 8 == 0 (the stem input comes from the preprocess kernel
//      already padded / space-to-depth packed)
//   w  [Cout, KH, KW, Cin] bf16  ("OHWI", K-contiguous rows; BN folded in at load time)
//   y  [N, Ho, Wo, ldy] bf16, written at channel offset y_coff (concat-by-stride-write)
// GEMM view: C^T[Cout, M] = W[Cout, K] . X^T[K, M]; M = N*Ho*Wo pixels, K = KH*KW*Cin.
// MFMA operand A = weight rows (output channels), operand B = im2col pixel rows.
//
// Tile configurations (4 waves = 256 threads, each wave 64 channels x TM pixels of
// v_mfma_f32_16x16x32_bf16 fragments):
//   <BM=128, BN=128>  wide layers            (2 x 2 waves, 64 x 64 per wave)
//   <BM=256, BN=64>   Cout <= 64 layers      (4 x 1 waves, 64 x 64 per wave; no wasted MFMA)
// K is staged 64 deep per step.  Register-staged global->LDS double buffer: the next
// tile's 16-B loads are issued before the MFMAs and written to the other LDS buffer after
// (guide T14); one barrier per K-tile.  LDS rows are 128 B, chunk-XOR swizzled
// (chunk ^ (row & 7)) so every ds_read_b128 fragment read is conflict-free (guide T2).
// Epilogue: acc + bias is rounded to bf16 into an LDS tile (padded rows), then each
// thread streams 16-B row segments: residual loads, activation and output stores are all
// fully coalesced 16-B accesses (the memory-bound 1x1 layers live on this).  Blocks are
// remapped XCD-aware so the channel tiles of one pixel tile share an L2 (guide T1).
#include <pybind11/pybind11.h>

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"

namespace {

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
  int kq, kr;  // CONV: divmod(BK, Cin), the (tap, channel) advance of one K tile
  int prio;    // raise the wave priority around each MFMA cluster (igemm_prio)
  // DUAL (pointwise GEMM + fused strided 1x1 shortcut): K = K1 + C2; k >= K1 reads the
  // second source x2 [N, H2, W2, C2] at pixel (n, ho*s2, wo*s2) of output pixel (n, ho, wo)
  const bf16* x2;
  int K1, C2, H2, W2, s2;
};

FTM_DEVICE int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

template <int BM, int BN, int STAGES, bool CONV, int ACT, bool HAS_BIAS, bool HAS_RES, bool DUAL = false,
          bool RES_PF = false>
__global__ __launch_bounds__(NT, 2) void igemm_bf16_kernel(IgemmParams p) {
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / WAVES_M;     // pixels per wave
  constexpr int J = TM / 16;           // pixel fragments per wave
  constexpr int XR = BM / 32;          // X chunks staged per thread
  constexpr int WR = BN / 32;          // W chunks staged per thread
  constexpr int OPAD = 8;              // epilogue row padding (bf16)
  constexpr int STAGE_ELEMS = STAGES * (BM + BN) * BK;
  constexpr int EPI_ELEMS = BM * (BN + OPAD);
  constexpr int LDS_ELEMS = STAGE_ELEMS > EPI_ELEMS ? STAGE_ELEMS : EPI_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16 smem[LDS_ELEMS];
  bf16* Xs = smem;                      // [STAGES][BM][BK]
  bf16* Ws = smem + STAGES * BM * BK;   // [STAGES][BN][BK]

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile % p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wp = wave % WAVES_M;  // pixel slab of the tile
  const int wc = wave / WAVES_M;  // channel slab

  // ---- per-thread staging assignment: fixed k-chunk, rows r0 + 32 i
  const int kc = tid & 7;
  const int r0 = tid >> 3;

  // CONV: per staged row the byte offset of its receptive field's (tap 0) corner pixel and a
  // bitmask of the filter taps that land inside the image (padding taps and rows past M read
  // through the buffer descriptor's range check as zeros).  The K loop then needs no
  // divides and no bounds compares: it walks (tap, channel) incrementally.
  int xbase[XR];
  uint64_t tmask[CONV ? XR : 1];
  int x2base[DUAL ? XR : 1];
  bool mvalid[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    int m = m0 + r0 + 32 * i;
    mvalid[i] = m < p.M;
    int mm = mvalid[i] ? m : 0;
    if constexpr (DUAL) {
      const int wo = mm % p.Wo;
      const int t = mm / p.Wo;
      const int ho = t % p.Ho;
      const int n = t / p.Ho;
      x2base[i] = ((n * p.H2 + ho * p.s2) * p.W2 + wo * p.s2) * p.C2;
    }
    if constexpr (CONV) {
      const int wo = mm % p.Wo;
      const int t = mm / p.Wo;
      const int ho = t % p.Ho;
      const int n = t / p.Ho;
      const int hb = ho * p.sh - p.ph, wb = wo * p.sw - p.pw;
      xbase[i] = (((n * p.H + hb) * p.W + wb) * p.Cin) * 2;  // bytes; only used for in-image taps
      uint64_t cols = 0, tm = 0;  // in-image filter columns, then rows x columns
      for (int kw = 0; kw < p.KW; ++kw)
        if ((unsigned)(wb + kw * p.dw) < (unsigned)p.W) cols |= 1ull << kw;
      if (mvalid[i])
        for (int kh = 0; kh < p.KH; ++kh)
          if ((unsigned)(hb + kh * p.dh) < (unsigned)p.H) tm |= cols << (kh * p.KW);
      tmask[i] = tm;
    } else {
      xbase[i] = mm * p.ldx;
    }
  }
  // weight rows: CONV reads them through a buffer descriptor (rows past Cout and the K tail
  // read as zeros, no branches); the GEMM modes keep plain predicated loads
  int wrow[WR];  // byte offset of this thread's weight row (0x7fffffff: past Cout)
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    const int co = n0 + r0 + 32 * i;
    wrow[i] = co < p.Cout ? co * p.K * 2 : 0x7fffffff;
  }
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.w), 0, CONV ? p.Cout * p.K * 2 : 0, 0x00020000);

  u32x4 xr[XR], wr[WR];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

  // CONV K walk: this thread's 8-channel chunk sits at channel ci of filter tap `tap`
  // (= kh * KW + kw); tapoff = the tap's byte offset relative to the corner pixel.  One
  // K tile advances (tap, ci) by (kq, kr) = divmod(BK, Cin) (host-computed): no divides.
  const int cin2 = p.Cin * 2;
  int tap = 0, ci = 0, kh = 0, kw = 0, tapoff = 0;
  if constexpr (CONV) {
    tap = kc * 8 / p.Cin;
    ci = kc * 8 - tap * p.Cin;
    kh = tap / p.KW;
    kw = tap - kh * p.KW;
    tapoff = (kh * p.dh * p.W + kw * p.dw) * cin2;
  }
  auto advance_k = [&]() {
    ci += p.kr;
    tap += p.kq;
    kw += p.kq;
    if (ci >= p.Cin) { ci -= p.Cin; ++tap; ++kw; }
    while (kw >= p.KW) { kw -= p.KW; ++kh; }
    tapoff = (kh * p.dh * p.W + kw * p.dw) * cin2;
  };
  const __amdgpu_buffer_rsrc_t xrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.x), 0, CONV ? p.N * p.H * p.W * cin2 : 0, 0x00020000);
  const int ntaps = p.KH * p.KW;

  auto load_tile = [&](int k0) {
    const int k = k0 + kc * 8;
    const bool kvalid = k < p.K;
    if constexpr (CONV) {
      const bool tvalid = tap < ntaps;
      const int koff = tapoff + ci * 2;
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        const bool ok = tvalid && ((tmask[i] >> tap) & 1);
        xr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrsrc, ok ? xbase[i] + koff : 0x7fffffff, 0, 0));
      }
      advance_k();
    } else if constexpr (DUAL) {
      const bool second = k >= p.K1;  // chunk-uniform: K1 % 8 == 0
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        bool ok = kvalid && mvalid[i];
        const bf16* src = second ? p.x2 + (size_t)x2base[i] + (k - p.K1) : p.x + (size_t)xbase[i] + k;
        xr[i] = ok ? *reinterpret_cast<const u32x4*>(src) : zero4;
      }
    } else {
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        bool ok = kvalid && mvalid[i];
        xr[i] = ok ? *reinterpret_cast<const u32x4*>(p.x + (size_t)xbase[i] + k) : zero4;
      }
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const bool ok = kvalid && wrow[i] != 0x7fffffff;
      if constexpr (CONV)
        wr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, ok ? wrow[i] + k * 2 : 0x7fffffff, 0, 0));
      else
        wr[i] = ok ? *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint8_t*>(p.w) + wrow[i] + k * 2) : zero4;
    }
  };
  auto store_tile = [&](int buf) {
    bf16* xs = Xs + buf * BM * BK;
    bf16* ws = Ws + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < XR; ++i) *reinterpret_cast<u32x4*>(xs + swz(r0 + 32 * i, kc)) = xr[i];
#pragma unroll
    for (int i = 0; i < WR; ++i) *reinterpret_cast<u32x4*>(ws + swz(r0 + 32 * i, kc)) = wr[i];
  };

  f32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // RES_PF: the residual tile is prefetched into registers before the K loop — for the
  // short-K 1x1 expansion convs (K <= 128) the residual read is otherwise a second exposed
  // HBM round trip after the MFMAs; for long K the extra 32 VGPRs cost more occupancy
  // than they hide (bench/conv_tune.py)
  constexpr int CPR_R = BN / 8;
  constexpr int RIT = RES_PF ? (BM * CPR_R + NT - 1) / NT : 1;
  bf16x8 rres[RIT];
  if constexpr (RES_PF) {
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int q = tid + it * NT;
      const int m = m0 + q / CPR_R;
      const int c = n0 + (q % CPR_R) * 8;
      rres[it] = (q < BM * CPR_R && m < p.M && c < p.Cout)
                     ? *reinterpret_cast<const bf16x8*>(p.res + (size_t)m * p.ldr + c)
                     : bf16x8{};
    }
  }

  const int nk = (p.K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fchunk = lane >> 4;  // 0..3 -> k offset 8*fchunk within a 32-deep substep

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = STAGES == 2 ? (kt & 1) : 0;
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
    const bf16* xs = Xs + buf * BM * BK;
    const bf16* ws = Ws + buf * BN * BK;
    if (p.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4], b[J];
      const int chunk = ks * 4 + fchunk;
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ws + swz(wc * 64 + i * 16 + frow, chunk));
#pragma unroll
      for (int j = 0; j < J; ++j) b[j] = *reinterpret_cast<const bf16x8*>(xs + swz(wp * TM + j * 16 + frow, chunk));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (p.prio) __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < nk) {
      if constexpr (STAGES == 1) __syncthreads();  // single buffer: everyone done reading
      store_tile(STAGES == 2 ? (buf ^ 1) : 0);
    }
    __syncthreads();
  }

  // ---- epilogue phase 1: (acc + bias) -> bf16 LDS tile [BM][BN + OPAD]
  constexpr int OLD = BN + OPAD;
  bf16* Os = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cl = wc * 64 + i * 16 + (lane >> 4) * 4;  // local channel of this lane's 4 rows
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if constexpr (HAS_BIAS) {
      if (n0 + cl < p.Cout) bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int pl = wp * TM + j * 16 + (lane & 15);
      f32x4 v = acc[i][j] + bv;
      bf16x4 o;
      if constexpr (HAS_RES) {
        o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
      } else {
        o[0] = f2bf(apply_act<ACT>(v[0]));
        o[1] = f2bf(apply_act<ACT>(v[1]));
        o[2] = f2bf(apply_act<ACT>(v[2]));
        o[3] = f2bf(apply_act<ACT>(v[3]));
      }
      *reinterpret_cast<bf16x4*>(Os + pl * OLD + cl) = o;
    }
  }
  __syncthreads();

  // ---- epilogue phase 2: coalesced 16-B row segments (+ residual, activation)
  constexpr int CPR = BN / 8;  // 16-B chunks per tile row
#pragma unroll
  for (int it = 0; it < (BM * CPR + NT - 1) / NT; ++it) {
    const int q = tid + it * NT;
    const int pl = q / CPR;
    const int cc = q % CPR;
    const int m = m0 + pl;
    const int c = n0 + cc * 8;
    if (q >= BM * CPR || m >= p.M || c >= p.Cout) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(Os + pl * OLD + cc * 8);
    if constexpr (HAS_RES) {
      const bf16x8 r = RES_PF ? rres[RES_PF ? it : 0]
                              : *reinterpret_cast<const bf16x8*>(p.res + (size_t)m * p.ldr + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(apply_act<ACT>((float)v[e] + (float)r[e]));
    }
    *reinterpret_cast<bf16x8*>(p.y + (size_t)m * p.ldy + p.y_coff + c) = v;
  }
}

// The bias pointer is always set (the launcher substitutes a zero vector).
template <int BM, int BN, int STAGES, bool CONV, int ACT>
void launch_act(const IgemmParams& p0, hipStream_t s) {
  IgemmParams p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.Cout + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n), block(NT);
  if (p.res && p.K <= 128)
    hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, STAGES, CONV, ACT, true, true, false, true>), grid, block, 0, s, p);
  else if (p.res)
    hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, STAGES, CONV, ACT, true, true>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, STAGES, CONV, ACT, true, false>), grid, block, 0, s, p);
}

template <int BM, int BN, int STAGES, int ACT>
void launch_dual(const IgemmParams& p0, hipStream_t s) {
  IgemmParams p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.Cout + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n), block(NT);
  hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, STAGES, false, ACT, true, false, true>), grid, block, 0, s, p);
}

// Tile configurations: 0 = 128x128 double-buffered, 1 = 256x64 double-buffered,
// 2 = 128x128 single-buffered (more blocks/CU), 3 = 256x64 single-buffered, 4 = 64x128.
constexpr int NCFG = 5;

// Measured on the ResNet-50 layer set (bench/conv_tune.py, profiles/r01_tune): the
// single-buffered tiles win almost everywhere — 4 blocks/CU of occupancy hide the
// global-load latency better than a second LDS stage at 2 blocks/CU.
int auto_config(const IgemmParams& p) {
  if (p.Cout <= 64) return 3;
  return 2;
}

template <bool CONV, int ACT>
void launch_tile(const IgemmParams& p, int cfg, hipStream_t s) {
  if (cfg < 0) cfg = auto_config(p);
  switch (cfg) {
    case 0: launch_act<128, 128, 2, CONV, ACT>(p, s); break;
    case 1: launch_act<256, 64, 2, CONV, ACT>(p, s); break;
    case 2: launch_act<128, 128, 1, CONV, ACT>(p, s); break;
    case 3: launch_act<256, 64, 1, CONV, ACT>(p, s); break;
    case 4: launch_act<64, 128, 2, CONV, ACT>(p, s); break;
    default: throw std::invalid_argument("unknown igemm config " + std::to_string(cfg));
  }
}

template <bool CONV>
void launch(const IgemmParams& p, int act, int cfg, hipStream_t s) {
  if constexpr (CONV) {
    switch (act) {
      case ACT_NONE: launch_tile<CONV, ACT_NONE>(p, cfg, s); break;
      case ACT_RELU: launch_tile<CONV, ACT_RELU>(p, cfg, s); break;
      case ACT_RELU6: launch_tile<CONV, ACT_RELU6>(p, cfg, s); break;
      default: throw std::invalid_argument("conv activation must be none/relu/relu6");
    }
  } else {
    switch (act) {
      case ACT_NONE: launch_tile<CONV, ACT_NONE>(p, cfg, s); break;
      case ACT_RELU: launch_tile<CONV, ACT_RELU>(p, cfg, s); break;
      case ACT_GELU_TANH: launch_tile<CONV, ACT_GELU_TANH>(p, cfg, s); break;
      case ACT_SIGMOID: launch_tile<CONV, ACT_SIGMOID>(p, cfg, s); break;
      case ACT_TANH: launch_tile<CONV, ACT_TANH>(p, cfg, s); break;
      case ACT_RELU6: launch_tile<CONV, ACT_RELU6>(p, cfg, s); break;
      default: throw std::invalid_argument("unknown activation " + std::to_string(act));
    }
  }
  FTM_CHECK_LAUNCH();
}

// s_setprio(1) around each K-tile's MFMA cluster.  With two
// compute lanes a CU holds this kernel's waves next to the sibling lane's (loads, LDS
// stores, epilogues): raising the MFMA phase's priority keeps the matrix cores fed.  Single
// lane it is neutral (3861 vs 3863 µs per 256 images); end to end +1.0 % (79.7k -> 80.5k,
// profiles/r02_igemm_prio).
constexpr int igemm_prio() { return 1; }

// No allocation in the launch path (it may be captured into a hipGraph): a layer without
// bias passes a zero vector owned by the caller.
void require_bias(const float* b) {
  if (!b) throw std::invalid_argument("igemm: bias pointer is required (pass zeros for no bias)");
}

void check_align(uintptr_t ptr, int bytes, const char* what) {
  if (ptr % bytes) throw std::invalid_argument(std::string(what) + " is not " + std::to_string(bytes) + "-byte aligned");
}

}  // namespace

// Conv2D NHWC implicit GEMM.  Shapes are validated here (host side) before any launch.
void conv2d_nhwc_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int N, int H, int W,
                      int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw, int Ho, int Wo,
                      int ldy, int y_coff, int ldr, int act, uintptr_t stream, int cfg) {
  if (Cin % 8) throw std::invalid_argument("conv2d_nhwc_bf16: Cin must be a multiple of 8");
  if (Cout % 8 || ldy % 8 || y_coff % 8) throw std::invalid_argument("conv2d_nhwc_bf16: Cout/ldy/y_coff % 8 != 0");
  if (res && ldr % 8) throw std::invalid_argument("conv2d_nhwc_bf16: residual stride % 8 != 0");
  if (N <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0) throw std::invalid_argument("conv2d_nhwc_bf16: empty problem");
  if ((long)N * H * W * Cin * 2 >= (1L << 31) || (long)N * Ho * Wo >= (1L << 31))
    throw std::invalid_argument("conv2d_nhwc_bf16: tensor too large for 32-bit (byte) indexing");
  if (KH * KW > 64) throw std::invalid_argument("conv2d_nhwc_bf16: more than 64 filter taps");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  if (bias) check_align(bias, 16, "bias");
  if (res) check_align(res, 16, "residual");
  IgemmParams p{};
  p.prio = igemm_prio();
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
  p.kq = BK / Cin;
  p.kr = BK % Cin;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  require_bias(p.bias);
  const bool pointwise = KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
  if (pointwise) launch<false>(p, act, cfg, s);  // 1x1/s1: the input IS the [M, Cin] matrix
  else launch<true>(p, act, cfg, s);
}

// Y[M, N] = act(X[M, K] . W[N, K]^T + bias + res).  X row stride ldx, Y row stride ldy.
void gemm_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int M, int N, int K, int ldx,
               int ldy, int ldr, int act, uintptr_t stream, int cfg) {
  if (K % 8 || ldx % 8) throw std::invalid_argument("gemm_bf16: K and ldx must be multiples of 8");
  if (N % 8 || ldy % 8) throw std::invalid_argument("gemm_bf16: N and ldy must be multiples of 8");
  if (res && ldr % 8) throw std::invalid_argument("gemm_bf16: residual stride % 8 != 0");
  if (M <= 0 || N <= 0) throw std::invalid_argument("gemm_bf16: empty problem");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  if (bias) check_align(bias, 16, "bias");
  if (res) check_align(res, 16, "residual");
  IgemmParams p{};
  p.prio = igemm_prio();
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const bf16*>(res);
  p.y = reinterpret_cast<bf16*>(y);
  p.M = M; p.Cout = N; p.K = K; p.ldx = ldx; p.ldy = ldy; p.y_coff = 0; p.ldr = ldr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  require_bias(p.bias);
  launch<false>(p, act, cfg, s);
}

// y = act(x[M, K1] . W[:, :K1]^T + x2_strided[M, C2] . W[:, K1:]^T + bias): a pointwise
// conv with its 1x1 (optionally strided) projection shortcut fused into the same K loop,
// so the shortcut's output never round-trips through HBM (ResNet bottleneck unit 1).
void conv1x1_dual_bf16(uintptr_t x, uintptr_t x2, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int Ho, int Wo,
                       int K1, int C2, int H2, int W2, int s2, int Cout, int ldy, int y_coff, int act,
                       uintptr_t stream, int cfg) {
  if (K1 % 8 || C2 % 8 || Cout % 8 || ldy % 8 || y_coff % 8)
    throw std::invalid_argument("conv1x1_dual_bf16: channel counts must be multiples of 8");
  if ((Ho - 1) * s2 >= H2 || (Wo - 1) * s2 >= W2) throw std::invalid_argument("conv1x1_dual_bf16: shortcut geometry");
  if ((long)N * H2 * W2 * C2 >= (1L << 31) || (long)N * Ho * Wo * K1 >= (1L << 31))
    throw std::invalid_argument("conv1x1_dual_bf16: tensor too large for 32-bit indexing");
  require_bias(reinterpret_cast<const float*>(bias));
  check_align(x, 16, "x");
  check_align(x2, 16, "x2");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  check_align(bias, 16, "bias");
  IgemmParams p{};
  p.prio = igemm_prio();
  p.x = reinterpret_cast<const bf16*>(x);
  p.x2 = reinterpret_cast<const bf16*>(x2);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<bf16*>(y);
  p.N = N; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.M = N * Ho * Wo;
  p.K1 = K1; p.C2 = C2; p.H2 = H2; p.W2 = W2; p.s2 = s2;
  p.K = K1 + C2;
  p.ldx = K1;
  p.ldy = ldy; p.y_coff = y_coff;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (cfg < 0) cfg = Cout <= 64 ? 3 : 2;
  if (act != ACT_RELU && act != ACT_NONE) throw std::invalid_argument("conv1x1_dual_bf16: act must be none/relu");
#define FTM_DUAL(BM_, BN_, ST_)                                                    \
  do {                                                                             \
    if (act == ACT_RELU) launch_dual<BM_, BN_, ST_, ACT_RELU>(p, s);               \
    else launch_dual<BM_, BN_, ST_, ACT_NONE>(p, s);                               \
  } while (0)
  switch (cfg) {
    case 0: FTM_DUAL(128, 128, 2); break;
    case 1: FTM_DUAL(256, 64, 2); break;
    case 2: FTM_DUAL(128, 128, 1); break;
    case 3: FTM_DUAL(256, 64, 1); break;
    case 4: FTM_DUAL(64, 128, 2); break;
    default: throw std::invalid_argument("conv1x1_dual_bf16: unknown config");
  }
#undef FTM_DUAL
  FTM_CHECK_LAUNCH();
}

void register_igemm(pybind11::module_& m) {
  m.def("conv1x1_dual_bf16", &conv1x1_dual_bf16);
  m.def("conv2d_nhwc_bf16", &conv2d_nhwc_bf16);
  m.def("gemm_bf16", &gemm_bf16);
  m.attr("igemm_num_configs") = NCFG;
}
