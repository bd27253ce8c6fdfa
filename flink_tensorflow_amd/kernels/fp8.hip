// OCP FP8 (e4m3fn) inference path for CDNA4 (BASELINE config "Inception-v3 fp8 weights").
//
// Quantisation scheme (static, calibrated by the graph compiler):
//   weights      per-output-channel scale  w = wq * sw[c]            (wq e4m3, |wq| <= 448)
//   activations  per-tensor scale          x = xq * sx               (one scale per buffer;
//                the branches of a concat share the concat buffer's scale)
//   conv/GEMM    acc = sum_k wq * xq (fp32, v_mfma_scale_f32_16x16x128_f8f6f4, unit E8M0
//                block scales), then y = act(acc * (sw[c] * sx) + bias[c]) and either
//                yq = sat(y / sy) written as fp8 (the next layer's input) or bf16.
//
// The implicit GEMM follows the bf16 kernel (igemm_bf16.hip) with the K stage widened to
// 128 one-byte elements: an LDS row is still 128 B = 8 chunks of 16 B with the
// chunk ^ (row & 7) swizzle, and one 16x16x128 MFMA per fragment pair consumes a whole
// stage (2x the K per instruction of bf16 at the same LDS traffic per byte).  The A
// (weights) and B (pixels) fragments are read with the SAME (lane group, byte) -> k
// assignment, so the product is independent of the instruction's internal K order.
// A layer whose producer writes bf16 (the stem) is quantised on load (IN_BF16).
//
// Also here: quantise / dequantise, max/avg pooling on fp8 with requantisation (pool
// branches write straight into concat buffers of another scale), and global average
// pooling fp8 -> bf16 (classifier input).
#include <pybind11/pybind11.h>

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"

typedef int i32x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int BK = 128;  // K (bytes) per stage
constexpr int NT = 256;
constexpr float FP8_MAX = 448.f;
constexpr int E8M0_ONE = 127;  // unit block scale

FTM_DEVICE float sat(float v) { return fminf(fmaxf(v, -FP8_MAX), FP8_MAX); }

// 4 floats -> 4 e4m3 bytes (RNE, saturated first: the converter does not clamp)
FTM_DEVICE uint32_t pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(d), w, true);
  return (uint32_t)w;
}

FTM_DEVICE void unpack4(uint32_t w, float* o) {
  o[0] = __builtin_amdgcn_cvt_f32_fp8((int)w, 0);
  o[1] = __builtin_amdgcn_cvt_f32_fp8((int)w, 1);
  o[2] = __builtin_amdgcn_cvt_f32_fp8((int)w, 2);
  o[3] = __builtin_amdgcn_cvt_f32_fp8((int)w, 3);
}

// 16 bf16 (two 16-B vectors) * q -> 16 fp8 (one 16-B vector)
FTM_DEVICE u32x4 quant16(u32x4 lo, u32x4 hi, float q) {
  bf16x8 a = __builtin_bit_cast(bf16x8, lo), b = __builtin_bit_cast(bf16x8, hi);
  u32x4 r;
  r[0] = pack4((float)a[0] * q, (float)a[1] * q, (float)a[2] * q, (float)a[3] * q);
  r[1] = pack4((float)a[4] * q, (float)a[5] * q, (float)a[6] * q, (float)a[7] * q);
  r[2] = pack4((float)b[0] * q, (float)b[1] * q, (float)b[2] * q, (float)b[3] * q);
  r[3] = pack4((float)b[4] * q, (float)b[5] * q, (float)b[6] * q, (float)b[7] * q);
  return r;
}

struct Fp8Params {
  const uint8_t* x;    // fp8 activations (bf16 when IN_BF16)
  const uint8_t* w;    // fp8 weights [Cout][K]
  const float* scale;  // per output channel: sw[c] * sx
  const float* bias;   // per output channel (zeros when absent)
  uint8_t* y;          // fp8 or bf16 output (OUT_FP8)
  float in_q;          // IN_BF16: 1 / sx
  float out_q;         // OUT_FP8: 1 / sy
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, sh, sw, ph, pw, dh, dw;
  int M, K;
  int ldx;          // GEMM mode: row stride of X in elements
  int ldy, y_coff;  // output pixel stride / channel offset (elements)
  int tiles_m, tiles_n;
  int prio;  // s_setprio(1) around each K-tile's MFMA cluster (fp8_prio)
  unsigned long long* stamp;  // conv_lite_fp8 STAMP diagnostics: [64 workgroups][64 K-tiles][5] clocks
};

// Multi-output epilogue of conv_lite_fp8 (horizontally fused sibling 1x1 convs of one
// input): output channels [c0[s], c0[s+1]) go to destination s — its own buffer, pixel
// stride, channel offset and e4m3 scale (or bf16) — and each channel has its own lower
// clamp (0 = ReLU, -inf = none).  Passed by value (a captured launch keeps it).
constexpr int MAX_SEGS = 6;
struct Fp8Segs {
  uint8_t* y[MAX_SEGS];
  int c0[MAX_SEGS + 1];
  int ld[MAX_SEGS], off[MAX_SEGS], bf16[MAX_SEGS];
  float q[MAX_SEGS];
  const float* lo;  // per output channel lower clamp
  int n;
};

FTM_DEVICE int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 4); }

// No wave-priority raise around the MFMA phase (igemm_bf16 has one): here it measured SLOWER
// (Inception-v3 fp8 61.2k -> 60.4k static, 54.4k -> 53.1k dynamic): an fp8 K-tile is 128
// deep, so the MFMA cluster is long and prioritising it starves the sibling lane's loads.
constexpr int fp8_prio() { return 0; }

template <int BM, int BN, bool CONV, bool IN_BF16, bool OUT_FP8, int ACT>
__global__ __launch_bounds__(NT, 2) void igemm_fp8_kernel(Fp8Params p) {
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / WAVES_M;
  constexpr int J = TM / 16;
  constexpr int XR = BM / 32;
  constexpr int WR = BN / 32;
  constexpr int OB = OUT_FP8 ? 1 : 2;            // output bytes per element
  constexpr int OLD = BN * OB + 16;              // epilogue LDS row pitch (bytes)
  constexpr int STAGE_BYTES = (BM + BN) * BK;
  constexpr int EPI_BYTES = BM * OLD;
  constexpr int LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES];
  uint8_t* Xs = smem;
  uint8_t* Ws = smem + BM * BK;

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile % p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wp = wave % WAVES_M;
  const int wc = wave / WAVES_M;

  const int kc = tid & 7;   // 16-byte k chunk staged by this thread
  const int r0 = tid >> 3;  // rows r0 + 32 i

  int xbase[XR], hb[XR], wb[XR];
  bool mvalid[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
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
  const uint8_t* wrow[WR];
  bool nvalid[WR];
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    int co = n0 + r0 + 32 * i;
    nvalid[i] = co < p.Cout;
    wrow[i] = p.w + (size_t)(nvalid[i] ? co : 0) * p.K;
  }

  constexpr int XV = IN_BF16 ? 2 : 1;  // 16-B global loads per staged chunk
  u32x4 xr[XR][XV], wr[WR];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

  auto load_tile = [&](int k0) {
    const int k = k0 + kc * 16;
    const bool kvalid = k < p.K;
    size_t off[XR];
    bool ok[XR];
    if constexpr (CONV) {
      int kidx = k / p.Cin;
      int ci = k - kidx * p.Cin;
      int kh = kidx / p.KW;
      int kw = kidx - kh * p.KW;
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        int hi = hb[i] + kh * p.dh;
        int wi = wb[i] + kw * p.dw;
        ok[i] = kvalid && mvalid[i] && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        off[i] = (size_t)xbase[i] + ((size_t)hi * p.W + wi) * p.Cin + ci;
      }
    } else {
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        ok[i] = kvalid && mvalid[i];
        off[i] = (size_t)xbase[i] + k;
      }
    }
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      if constexpr (IN_BF16) {
        const u32x4* src = reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16*>(p.x) + off[i]);
        xr[i][0] = ok[i] ? src[0] : zero4;
        xr[i][1] = ok[i] ? src[1] : zero4;
      } else {
        xr[i][0] = ok[i] ? *reinterpret_cast<const u32x4*>(p.x + off[i]) : zero4;
      }
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      bool okw = kvalid && nvalid[i];
      wr[i] = okw ? *reinterpret_cast<const u32x4*>(wrow[i] + k) : zero4;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      u32x4 v;
      if constexpr (IN_BF16) v = quant16(xr[i][0], xr[i][1], p.in_q);
      else v = xr[i][0];
      *reinterpret_cast<u32x4*>(Xs + swz(r0 + 32 * i, kc)) = v;
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) *reinterpret_cast<u32x4*>(Ws + swz(r0 + 32 * i, kc)) = wr[i];
  };

  f32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  load_tile(0);
  store_tile();
  __syncthreads();

  const int frow = lane & 15;
  const int c0 = 2 * (lane >> 4);  // this lane group's two 16-B chunks of the 128-deep stage

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
    if (p.prio) __builtin_amdgcn_s_setprio(1);
    i32x8 a[4], b[J];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wc * 64 + i * 16 + frow;
      u32x4 lo = *reinterpret_cast<const u32x4*>(Ws + swz(row, c0));
      u32x4 hi = *reinterpret_cast<const u32x4*>(Ws + swz(row, c0 + 1));
      a[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int row = wp * TM + j * 16 + frow;
      u32x4 lo = *reinterpret_cast<const u32x4*>(Xs + swz(row, c0));
      u32x4 hi = *reinterpret_cast<const u32x4*>(Xs + swz(row, c0 + 1));
      b[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, E8M0_ONE, 0,
                                                                     E8M0_ONE);
    if (p.prio) __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < nk) {
      __syncthreads();  // single LDS stage: everyone is done reading it
      store_tile();
    }
    __syncthreads();
  }

  // ---- epilogue phase 1: dequant + bias + act (+ requant) -> LDS tile [BM][OLD bytes]
  uint8_t* Os = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cl = wc * 64 + i * 16 + (lane >> 4) * 4;
    f32x4 sv = {0.f, 0.f, 0.f, 0.f}, bv = {0.f, 0.f, 0.f, 0.f};
    if (n0 + cl < p.Cout) {
      sv = *reinterpret_cast<const f32x4*>(p.scale + n0 + cl);
      bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int pl = wp * TM + j * 16 + (lane & 15);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act<ACT>(acc[i][j][r] * sv[r] + bv[r]);
      if constexpr (OUT_FP8) {
        *reinterpret_cast<uint32_t*>(Os + pl * OLD + cl) =
            pack4(v[0] * p.out_q, v[1] * p.out_q, v[2] * p.out_q, v[3] * p.out_q);
      } else {
        bf16x4 o;
        o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
        *reinterpret_cast<bf16x4*>(Os + pl * OLD + cl * 2) = o;
      }
    }
  }
  __syncthreads();

  // ---- epilogue phase 2: coalesced 16-B row segments
  constexpr int EPC = 16 / OB;   // elements per 16-B chunk
  constexpr int CPR = BN / EPC;  // chunks per tile row
#pragma unroll
  for (int q = tid; q < BM * CPR; q += NT) {
    const int pl = q / CPR;
    const int cc = q % CPR;
    const int m = m0 + pl;
    const int c = n0 + cc * EPC;
    if (m >= p.M || c >= p.Cout) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(Os + pl * OLD + cc * 16);
    *reinterpret_cast<u32x4*>(p.y + ((size_t)m * p.ldy + p.y_coff + c) * OB) = v;
  }
}

template <int BM, int BN, bool CONV, bool IN_BF16, bool OUT_FP8>
void launch_cfg(const Fp8Params& p0, int act, hipStream_t s) {
  Fp8Params p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.Cout + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n), block(NT);
  switch (act) {
    case ACT_NONE: hipLaunchKernelGGL((igemm_fp8_kernel<BM, BN, CONV, IN_BF16, OUT_FP8, ACT_NONE>), grid, block, 0, s, p); break;
    case ACT_RELU: hipLaunchKernelGGL((igemm_fp8_kernel<BM, BN, CONV, IN_BF16, OUT_FP8, ACT_RELU>), grid, block, 0, s, p); break;
    default: throw std::invalid_argument("fp8 igemm: activation must be none/relu");
  }
}

// Tile configurations: 0 = 128x128, 1 = 256x64 (Cout <= 64), 2 = 128x64.
constexpr int NCFG = 3;

template <bool CONV, bool IN_BF16, bool OUT_FP8>
void launch_tile(const Fp8Params& p, int act, int cfg, hipStream_t s) {
  if (cfg < 0) {
    // measured on the Inception-v3 layer set (bench/conv_tune_fp8.py): narrow layers with a
    // short K take 256x64; otherwise the channel tile that pads Cout least (64 on ties
    // loses to 128's higher intensity); 256x64 with bf16 staging spills
    const int pad64 = (p.Cout + 63) / 64 * 64, pad128 = (p.Cout + 127) / 128 * 128;
    if (p.Cout <= 64) cfg = (p.K <= 512 && !IN_BF16) ? 1 : 2;
    else cfg = pad64 < pad128 ? 2 : 0;
  }
  switch (cfg) {
    case 0: launch_cfg<128, 128, CONV, IN_BF16, OUT_FP8>(p, act, s); break;
    case 1: launch_cfg<256, 64, CONV, IN_BF16, OUT_FP8>(p, act, s); break;
    case 2: launch_cfg<128, 64, CONV, IN_BF16, OUT_FP8>(p, act, s); break;
    default: throw std::invalid_argument("unknown fp8 igemm config " + std::to_string(cfg));
  }
}

// ---------------------------------------------------------------------------------------
// conv_lite_fp8: the fp8 counterpart of conv_pp.hip's conv_lite — a 128x128 tile of four
// waves (64 x 64 outputs each, one v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair
// and K-tile) on two 32 KiB LDS stages filled by buffer_load ... lds (no VGPR staging, no
// ds_write), one barrier per K-tile, so two workgroups (or one and a sibling lane's
// kernel) share a CU.  The K walk is per lane: each lane stages one fixed logical 16-B
// chunk of every K-tile (the XOR swizzle is applied on the source address), so any
// Cin % 16 == 0 works (Inception's 192 / 288 / 768 ...): the lane's (filter tap, channel)
// advances by divmod(128, Cin) per K-tile — no divides in the loop — and chunks past K or
// in the zero padding read zeros through the buffer range check.  Epilogue as
// igemm_fp8_kernel (per-channel dequant scale + bias + act, e4m3 or bf16 output at a
// channel offset of a wider buffer).
// ---------------------------------------------------------------------------------------
// BN_ = 96 / 64 for Cout that a 128-wide channel tile would pad badly (96, 192 = 2 x 96,
// 80, 160, 288 on 96; 320, 448, <= 64 on 64); NSTG = 1 (a single LDS stage) when the whole K fits one
// K-tile (K <= 128: no prefetch to overlap, and half the LDS lets more workgroups hide the
// load latency of these streaming layers).
// STAMP (diagnostics, bench/conv_stamp_probe.py --fp8): as conv_pp.hip's conv_lite STAMP —
// wave 0 of the first 64 workgroups records s_memtime around each K-tile's phases.
// (An eight-wave form with the DMA and MFMA roles split measured 4.5 % slower on
// Inception-v3, profiles/r04_w, and was removed.)
template <bool OUT_FP8, int ACT, int BN_, int NSTG, bool MULTI, bool STAMP>
__device__ __forceinline__ void conv_lite_fp8_body(const Fp8Params& p, const Fp8Segs& sg) {
  static_assert(BN_ == 192 || BN_ == 160 || BN_ == 128 || BN_ == 96 || BN_ == 64, "channel tile 192 .. 64");
  constexpr int BM = 128, BN = BN_;
  constexpr int NI = BN / 32;  // weight fragments per wave (a wave covers BN / 2 channels)
  constexpr int WQ = BN / 32;  // weight DMA rows-of-8 per wave
  constexpr int QD = WQ > 4 ? WQ : 4;  // DMA pieces per wave and operand pair (X: 4)
  constexpr int XB = BM * BK, WB = BN * BK, STG = XB + WB;
  constexpr int OB = (OUT_FP8 && !MULTI) ? 1 : 2;  // MULTI stages bf16, quantises per segment at the store
  constexpr int OLD = BN * OB + 16;
  constexpr int LDS = NSTG * STG > BM * OLD ? NSTG * STG : BM * OLD;
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS];

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  constexpr int NT = 256;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;

  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;  // this lane's logical 16-B chunk of every K-tile
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.x, 0, (int)((unsigned)p.N * (unsigned)(p.H * p.W) * (unsigned)p.Cin), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.w, 0, (int)((unsigned)p.Cout * (unsigned)p.K), 0x00020000);
  int pb[4], ihw[4];
  unsigned wrow[6];  // fixed size (WQ <= 6): see conv_pp.hip on template-sized arrays
  const int ohw = p.Ho * p.Wo;
#pragma unroll
  for (int q = 0; q < QD; ++q) {
    const unsigned co = n0 + 8 * (WQ * wave + q) + drow;  // weight rows: WQ rows-of-8 per wave
    wrow[q] = (q < WQ && co < (unsigned)p.Cout) ? co * (unsigned)p.K : 0x80000000u;
    if (q >= 4) continue;
    const int r = 8 * (4 * wave + q) + drow;
    const int m = m0 + r;
    const bool live = m < p.M;
    const int n = live ? m / ohw : 0;
    const int rem = live ? m - n * ohw : 0;
    const int oh = rem / p.Wo;
    const int ow = rem - oh * p.Wo;
    const int ih0 = live ? oh * p.sh - p.ph : -16384;
    const int iw0 = ow * p.sw - p.pw;
    pb[q] = ((n * p.H + ih0) * p.W + iw0) * p.Cin;
    ihw[q] = (ih0 << 16) | (iw0 & 0xFFFF);
  }
  // K walk of this lane's chunk: k = kt * 128 + dchunk * 16 -> (tap, ci), tap -> (kh, kw)
  const int ntaps = p.KH * p.KW;
  const int kq = BK / p.Cin, kr = BK - kq * p.Cin;
  int k = dchunk * 16;
  int tap = k / p.Cin;
  int ci = k - tap * p.Cin;
  int kh = tap / p.KW;
  int kw = tap - kh * p.KW;
  auto dma = [&](int stage) {
    const bool kin = tap < ntaps;
    const int dih = kh * p.dh, diw = kw * p.dw;
    const int toff = (dih * p.W + diw) * p.Cin + ci;
    uint8_t* bx = smem + stage * STG + 4 * wave * 8 * BK;
    uint8_t* bw = smem + stage * STG + XB + WQ * wave * 8 * BK;
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      if (q < 4) {
        const int ih = (ihw[q] >> 16) + dih;
        const int iw = ((ihw[q] << 16) >> 16) + diw;
        const bool ok = kin && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(bx + q * 8 * BK), 16,
                                                 ok ? (unsigned)(pb[q] + toff) : 0x80000000u, 0, 0, 0);
      }
      if (q < WQ) {
        const unsigned wo = (k < p.K && wrow[q] != 0x80000000u) ? wrow[q] + (unsigned)k : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(bw + q * 8 * BK), 16,
                                                 wo, 0, 0, 0);
      }
    }
    // advance to the next K-tile
    k += BK;
    ci += kr;
    int dt = kq;
    if (ci >= p.Cin) {
      ci -= p.Cin;
      ++dt;
    }
    tap += dt;
    kw += dt;
    while (kw >= p.KW) {
      kw -= p.KW;
      ++kh;
    }
  };

  const int frow = lane & 15;
  const int c0 = 2 * (lane >> 4);
  const int sl0 = (c0 ^ (frow & 7)) << 4, sl1 = ((c0 + 1) ^ (frow & 7)) << 4;
  f32x4 acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = NSTG == 1 ? 1 : (p.K + BK - 1) / BK;  // NSTG 1: the host guarantees K <= BK
  unsigned long long* sp = nullptr;
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  if constexpr (STAMP) {
    if (threadIdx.x == 0 && blockIdx.x < 64) sp = p.stamp + (size_t)blockIdx.x * 64 * 5;
  }
  dma(0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = NSTG == 1 ? 0 : (kt & 1);
    if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (STAMP) t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if constexpr (STAMP) t2 = __builtin_amdgcn_s_memtime();
    if (NSTG > 1 && kt + 1 < nk) dma(st ^ 1);
    if constexpr (STAMP) t3 = __builtin_amdgcn_s_memtime();
    const uint8_t* xs = smem + st * STG;
    const uint8_t* ws = xs + XB;
    i32x8 a[NI], b[4];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint8_t* r = ws + (wn * (BN / 2) + i * 16 + frow) * BK;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(r + sl0), hi = *reinterpret_cast<const u32x4*>(r + sl1);
      a[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint8_t* r = xs + (wm * 64 + j * 16 + frow) * BK;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(r + sl0), hi = *reinterpret_cast<const u32x4*>(r + sl1);
        b[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, E8M0_ONE, 0,
                                                                       E8M0_ONE);
    }
    if constexpr (STAMP) {
      const unsigned long long t4 = __builtin_amdgcn_s_memtime();
      if (sp && kt < 64) {
        sp[kt * 5 + 0] = t0;
        sp[kt * 5 + 1] = t1;
        sp[kt * 5 + 2] = t2;
        sp[kt * 5 + 3] = t3;
        sp[kt * 5 + 4] = t4;
      }
    }
  }
  __syncthreads();  // the epilogue tile reuses the stage images

  uint8_t* Os = smem;
  {
  #pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int cl = wn * (BN / 2) + i * 16 + (lane >> 4) * 4;
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, bv = {0.f, 0.f, 0.f, 0.f}, lv = {0.f, 0.f, 0.f, 0.f};
      if (n0 + cl < p.Cout) {
        sv = *reinterpret_cast<const f32x4*>(p.scale + n0 + cl);
        bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
        if constexpr (MULTI) lv = *reinterpret_cast<const f32x4*>(sg.lo + n0 + cl);
      }
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pl = wm * 64 + j * 16 + frow;
        float v[4];
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (MULTI) v[r] = fmaxf(acc[i][j][r] * sv[r] + bv[r], lv[r]);
          else v[r] = apply_act<ACT>(acc[i][j][r] * sv[r] + bv[r]);
        }
        if constexpr (OUT_FP8 && !MULTI) {
          *reinterpret_cast<uint32_t*>(Os + pl * OLD + cl) =
              pack4(v[0] * p.out_q, v[1] * p.out_q, v[2] * p.out_q, v[3] * p.out_q);
        } else {
          bf16x4 o;
          o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
          *reinterpret_cast<bf16x4*>(Os + pl * OLD + cl * 2) = o;
        }
      }
    }
  }
  __syncthreads();
  if constexpr (MULTI) {
    constexpr int CPR16 = BN / 16;  // 16-channel chunks (32 B of the bf16 tile) per row
#pragma unroll 2
    for (int q = threadIdx.x; q < BM * CPR16; q += NT) {
      const int pl = q / CPR16;
      const int cc = q % CPR16;
      const int m = m0 + pl;
      const int c = n0 + cc * 16;
      if (m >= p.M || c >= p.Cout) continue;
      int sgi = 0;
#pragma unroll
      for (int t = 1; t < MAX_SEGS; ++t) sgi += (t < sg.n && c >= sg.c0[t]) ? 1 : 0;
      const int cl = c - sg.c0[sgi];
      const u32x4 lo = *reinterpret_cast<const u32x4*>(Os + pl * OLD + cc * 32);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(Os + pl * OLD + cc * 32 + 16);
      const size_t e = (size_t)m * sg.ld[sgi] + sg.off[sgi] + cl;  // elements of that destination
      if (sg.bf16[sgi]) {
        u32x4* dst = reinterpret_cast<u32x4*>(sg.y[sgi] + e * 2);
        dst[0] = lo;
        dst[1] = hi;
      } else {
        *reinterpret_cast<u32x4*>(sg.y[sgi] + e) = quant16(lo, hi, sg.q[sgi]);
      }
    }
    return;
  }
  constexpr int EPC = 16 / OB;
  constexpr int CPR = BN / EPC;
#pragma unroll 4
  for (int q = threadIdx.x; q < BM * CPR; q += NT) {
    const int pl = q / CPR;
    const int cc = q % CPR;
    const int m = m0 + pl;
    const int c = n0 + cc * EPC;
    if (m >= p.M || c >= p.Cout) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(Os + pl * OLD + cc * 16);
    *reinterpret_cast<u32x4*>(p.y + ((size_t)m * p.ldy + p.y_coff + c) * OB) = v;
  }
}

template <bool OUT_FP8, int ACT, int BN_ = 128, int NSTG = 2, bool MULTI = false, bool STAMP = false>
__global__ __launch_bounds__(256, 2) void conv_lite_fp8_kernel(Fp8Params p, Fp8Segs sg) {
  conv_lite_fp8_body<OUT_FP8, ACT, BN_, NSTG, MULTI, STAMP>(p, sg);
}

template <bool OUT_FP8, int BN_, int NSTG, bool MULTI = false>
void launch_lite_fp8_t(Fp8Params p, int act, hipStream_t s, const Fp8Segs& sg) {
  p.tiles_m = (p.M + 127) / 128;
  p.tiles_n = (p.Cout + BN_ - 1) / BN_;
  dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if constexpr (MULTI) {  // the per-channel clamp replaces the activation
    hipLaunchKernelGGL((conv_lite_fp8_kernel<false, ACT_NONE, BN_, NSTG, true>), grid, block, 0, s, p, sg);
    return;
  }
  if constexpr (OUT_FP8 && NSTG == 2) {
    if (p.stamp && act == ACT_RELU) {  // diagnostics only (conv_lite_fp8_stamp)
      hipLaunchKernelGGL((conv_lite_fp8_kernel<true, ACT_RELU, BN_, 2, false, true>), grid, block, 0, s, p, sg);
      return;
    }
  }
  switch (act) {
    case ACT_NONE: hipLaunchKernelGGL((conv_lite_fp8_kernel<OUT_FP8, ACT_NONE, BN_, NSTG>), grid, block, 0, s, p, sg); break;
    case ACT_RELU: hipLaunchKernelGGL((conv_lite_fp8_kernel<OUT_FP8, ACT_RELU, BN_, NSTG>), grid, block, 0, s, p, sg); break;
    default: throw std::invalid_argument("fp8 conv_lite: activation must be none/relu");
  }
}

// channel tile: the one of 192 / 160 / 128 / 96 / 64 that stages the fewest rows per
// 128-pixel tile and K-tile — the channel tiles' count x (128 pixel rows + BN weight rows),
// as the K loop is bound by the bytes it fills (profiles/r04_ac, r04_af); ties go to the
// wider tile.  (Least padding among 128 / 96 / 64, with or without 192, and the same count
// over whole waves of 512 workgroups measured slower: r04_ac, r04_ah.)  One LDS stage when
// K fits one K-tile.
int lite_fp8_bn(int Cout) {
  int best = 128;
  long cost = 1L << 62;
  for (int bn : {192, 160, 128, 96, 64}) {
    const long c = (long)((Cout + bn - 1) / bn) * (128 + bn);
    if (c < cost) best = bn, cost = c;
  }
  return best;
}

template <bool OUT_FP8, bool MULTI = false>
void launch_lite_fp8(const Fp8Params& p, int act, hipStream_t s, const Fp8Segs& sg = Fp8Segs{}, int bn = 0) {
  const int b = bn ? bn : lite_fp8_bn(p.Cout);
  const bool one = p.K <= BK;
#define FTM_LITE(BN_)                                                     \
  do {                                                                    \
    if (one) launch_lite_fp8_t<OUT_FP8, BN_, 1, MULTI>(p, act, s, sg);    \
    else launch_lite_fp8_t<OUT_FP8, BN_, 2, MULTI>(p, act, s, sg);        \
  } while (0)
  if (b == 64) FTM_LITE(64);
  else if (b == 96) FTM_LITE(96);
  else if (b == 192) FTM_LITE(192);
  else if (b == 160) FTM_LITE(160);
  else FTM_LITE(128);
#undef FTM_LITE
}

// conv_lite_fp8 STAMP diagnostics target (0 = off): set by conv_lite_fp8_stamp
unsigned long long* g_lite_fp8_stamp = nullptr;

// cfg value selecting conv_lite_fp8 (fp8 input only; any conv geometry with Cin % 16 == 0)
constexpr int LITE_CFG = 11;

template <bool CONV>
void launch_io(const Fp8Params& p, bool in_bf16, bool out_fp8, int act, int cfg, hipStream_t s) {
  if (in_bf16) {
    if (out_fp8) launch_tile<CONV, true, true>(p, act, cfg, s);
    else launch_tile<CONV, true, false>(p, act, cfg, s);
  } else {
    if (out_fp8) launch_tile<CONV, false, true>(p, act, cfg, s);
    else launch_tile<CONV, false, false>(p, act, cfg, s);
  }
  FTM_CHECK_LAUNCH();
}

void check_align(uintptr_t ptr, int bytes, const char* what) {
  if (ptr % bytes) throw std::invalid_argument(std::string(what) + " is not " + std::to_string(bytes) + "-byte aligned");
}

// ---------------------------------------------------------------- elementwise / pooling
__global__ __launch_bounds__(256) void quantize_kernel(const bf16* __restrict__ x, uint8_t* __restrict__ y, long n16,
                                                       float q) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) {
    const u32x4* src = reinterpret_cast<const u32x4*>(x + i * 16);
    reinterpret_cast<u32x4*>(y)[i] = quant16(src[0], src[1], q);
  }
}

__global__ __launch_bounds__(256) void dequantize_kernel(const uint8_t* __restrict__ x, bf16* __restrict__ y, long n16,
                                                         float s) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) {
    u32x4 v = reinterpret_cast<const u32x4*>(x)[i];
    bf16x8 o0, o1;
    float f[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unpack4(v[w], f);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (w < 2) o0[w * 4 + e] = f2bf(f[e] * s);
        else o1[(w - 2) * 4 + e] = f2bf(f[e] * s);
      }
    }
    reinterpret_cast<bf16x8*>(y + i * 16)[0] = o0;
    reinterpret_cast<bf16x8*>(y + i * 16)[1] = o1;
  }
}

// NHWC fp8 pooling, 16 channels x PX adjacent output pixels per thread: the PX outputs
// share the (PX-1)*sw + kw input columns of each window row, and 2 e4m3 values decode per
// instruction (v_cvt_pk_f32_fp8) into packed-f32 sums (v_pk_add_f32).  Avg divides by
// the in-bounds count (TF SAME).  Output = pooled * rq (rq = sx / sy requantises into the
// destination buffer, e.g. a concat of another scale).
typedef float f32x2 __attribute__((ext_vector_type(2)));

FTM_DEVICE void decode16(u32x4 v, f32x2* d) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    d[2 * w] = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[w], false);
    d[2 * w + 1] = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[w], true);
  }
}

template <bool MAX, int PX>
__global__ __launch_bounds__(256) void pool_fp8_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int N,
                                                       int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh,
                                                       int sw, int ph, int pw, int ldy, int y_coff, float rq) {
  const int cchunks = C / 16;
  const int wgroups = (Wo + PX - 1) / PX;
  const long total = (long)N * Ho * wgroups * cchunks;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int cc = idx % cchunks;
    long t = idx / cchunks;
    const int oxg = t % wgroups;
    t /= wgroups;
    const int oy = t % Ho;
    const int n = t / Ho;
    const int ox0 = oxg * PX;
    f32x2 acc[PX][8];
    int cnt_w[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[p][e] = MAX ? f32x2{-INFINITY, -INFINITY} : f32x2{0.f, 0.f};
      const int lo = max((ox0 + p) * sw - pw, 0), hi = min((ox0 + p) * sw - pw + kw, W);
      cnt_w[p] = max(hi - lo, 0);
    }
    int cnt_h = 0;
    const int iy0 = oy * sh - ph, ixs = ox0 * sw - pw;
    const int ncols = (PX - 1) * sw + kw;
    for (int dy = 0; dy < kh; ++dy) {
      const int iy = iy0 + dy;
      if ((unsigned)iy >= (unsigned)H) continue;
      ++cnt_h;
      const uint8_t* row = x + ((size_t)n * H + iy) * W * C + cc * 16;
      for (int c = 0; c < ncols; ++c) {
        const int ix = ixs + c;
        if ((unsigned)ix >= (unsigned)W) continue;
        f32x2 d[8];
        decode16(*reinterpret_cast<const u32x4*>(row + (size_t)ix * C), d);
#pragma unroll
        for (int p = 0; p < PX; ++p) {
          const int rel = c - p * sw;  // column inside output p's window?
          if (rel < 0 || rel >= kw) continue;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if constexpr (MAX) acc[p][e] = f32x2{fmaxf(acc[p][e][0], d[e][0]), fmaxf(acc[p][e][1], d[e][1])};
            else acc[p][e] += d[e];
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int ox = ox0 + p;
      if (ox >= Wo) break;
      const float sc = MAX ? rq : rq / (float)max(cnt_h * cnt_w[p], 1);
      u32x4 o;
#pragma unroll
      for (int w = 0; w < 4; ++w)
        o[w] = pack4(acc[p][2 * w][0] * sc, acc[p][2 * w][1] * sc, acc[p][2 * w + 1][0] * sc, acc[p][2 * w + 1][1] * sc);
      *reinterpret_cast<u32x4*>(y + (((size_t)n * Ho + oy) * Wo + ox) * ldy + y_coff + cc * 16) = o;
    }
  }
}

// 3x3 fp8 max pool (Inception's stem / grid-reduction pools), 16 channels x 2 adjacent
// outputs per thread with every window load issued before the first use: the generic
// kernel's runtime-bounded loops load, wait and decode one window pixel at a time (9
// dependent L2 round trips per output).  Out-of-range pixels read a clamped in-range
// address and are replaced by -448 (e4m3's lowest finite value, neutral for the max:
// quantisation saturates, so no stored value is below it).
template <int SW>
__global__ __launch_bounds__(256) void maxpool3_fp8_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int N,
                                                           int H, int W, int C, int Ho, int Wo, int ph, int pw, int ldy,
                                                           int y_coff, float rq) {
  constexpr int PX = 2, NC = (PX - 1) * SW + 3;
  const int cchunks = C / 16;
  const int wgroups = (Wo + PX - 1) / PX;
  const long total = (long)N * Ho * wgroups * cchunks;
  const u32x4 lowest = {0xFEFEFEFEu, 0xFEFEFEFEu, 0xFEFEFEFEu, 0xFEFEFEFEu};
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int cc = idx % cchunks;
    long t = idx / cchunks;
    const int oxg = t % wgroups;
    t /= wgroups;
    const int oy = t % Ho;
    const int n = t / Ho;
    const int ox0 = oxg * PX;
    const int iy0 = oy * 2 - ph, ixs = ox0 * SW - pw;  // (the row stride of these pools is 2 as well)
    u32x4 v[3][NC];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = iy0 + dy;
      const int iyc = min(max(iy, 0), H - 1);
      const uint8_t* row = x + ((size_t)n * H + iyc) * W * C + cc * 16;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ix = ixs + c;
        const int ixc = min(max(ix, 0), W - 1);
        v[dy][c] = *reinterpret_cast<const u32x4*>(row + (size_t)ixc * C);
      }
    }
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const bool yok = (unsigned)(iy0 + dy) < (unsigned)H;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bool ok = yok && (unsigned)(ixs + c) < (unsigned)W;
        if (!ok) v[dy][c] = lowest;
      }
    }
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int ox = ox0 + p;
      if (ox >= Wo) break;
      f32x2 acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = f32x2{-INFINITY, -INFINITY};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          f32x2 d[8];
          decode16(v[dy][p * SW + dx], d);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] = f32x2{fmaxf(acc[e][0], d[e][0]), fmaxf(acc[e][1], d[e][1])};
        }
      u32x4 o;
#pragma unroll
      for (int w = 0; w < 4; ++w)
        o[w] = pack4(acc[2 * w][0] * rq, acc[2 * w][1] * rq, acc[2 * w + 1][0] * rq, acc[2 * w + 1][1] * rq);
      *reinterpret_cast<u32x4*>(y + (((size_t)n * Ho + oy) * Wo + ox) * ldy + y_coff + cc * 16) = o;
    }
  }
}

// Average pool (TF SAME: the sum divided by the in-bounds count) over a bf16 NHWC tensor,
// then the bias + activation of the conv that PRODUCED it, written as fp8 (sat(y * out_q))
// or bf16 into a (concat) buffer at a channel offset.  Inception's AvgPool(3x3/1) -> 1x1
// conv branches run as 1x1 conv (no bias / act, bf16 out) -> this kernel: pool and
// pointwise conv are both linear, so they commute, and the pool then reads Cout (32-192)
// channels instead of Cin (192-2048).  16 channels x PX adjacent outputs per thread.
template <bool OUT_FP8, int ACT, int PX>
__global__ __launch_bounds__(256) void avgpool_epi_kernel(const bf16* __restrict__ x, const float* __restrict__ bias,
                                                          uint8_t* __restrict__ y, int N, int H, int W, int C, int Ho,
                                                          int Wo, int kh, int kw, int sh, int sw, int ph, int pw,
                                                          int ldy, int y_coff, float out_q) {
  const int cchunks = C / 16;
  const int wgroups = (Wo + PX - 1) / PX;
  const long total = (long)N * Ho * wgroups * cchunks;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int cc = idx % cchunks;
    long t = idx / cchunks;
    const int oxg = t % wgroups;
    t /= wgroups;
    const int oy = t % Ho;
    const int n = t / Ho;
    const int ox0 = oxg * PX;
    float acc[PX][16];
    int cnt_w[PX];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[p][e] = 0.f;
      const int lo = max((ox0 + p) * sw - pw, 0), hi = min((ox0 + p) * sw - pw + kw, W);
      cnt_w[p] = max(hi - lo, 0);
    }
    int cnt_h = 0;
    const int iy0 = oy * sh - ph, ixs = ox0 * sw - pw;
    const int ncols = (PX - 1) * sw + kw;
    for (int dy = 0; dy < kh; ++dy) {
      const int iy = iy0 + dy;
      if ((unsigned)iy >= (unsigned)H) continue;
      ++cnt_h;
      const bf16* row = x + ((size_t)n * H + iy) * W * C + cc * 16;
      for (int c = 0; c < ncols; ++c) {
        const int ix = ixs + c;
        if ((unsigned)ix >= (unsigned)W) continue;
        const bf16x8* src = reinterpret_cast<const bf16x8*>(row + (size_t)ix * C);
        const bf16x8 a = src[0], b = src[1];
#pragma unroll
        for (int p = 0; p < PX; ++p) {
          const int rel = c - p * sw;  // column inside output p's window?
          if (rel < 0 || rel >= kw) continue;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            acc[p][e] += (float)a[e];
            acc[p][8 + e] += (float)b[e];
          }
        }
      }
    }
    float bv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bv[e] = bias[cc * 16 + e];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int ox = ox0 + p;
      if (ox >= Wo) break;
      const float inv = 1.f / (float)max(cnt_h * cnt_w[p], 1);
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = apply_act<ACT>(__builtin_fmaf(acc[p][e], inv, bv[e]));
      const size_t o = (((size_t)n * Ho + oy) * Wo + ox) * ldy + y_coff + cc * 16;
      if constexpr (OUT_FP8) {
        u32x4 q;
#pragma unroll
        for (int w = 0; w < 4; ++w) q[w] = pack4(v[4 * w] * out_q, v[4 * w + 1] * out_q, v[4 * w + 2] * out_q, v[4 * w + 3] * out_q);
        *reinterpret_cast<u32x4*>(y + o) = q;
      } else {
        bf16x8 o0, o1;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o0[e] = f2bf(v[e]);
          o1[e] = f2bf(v[8 + e]);
        }
        bf16x8* dst = reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(y) + o);
        dst[0] = o0;
        dst[1] = o1;
      }
    }
  }
}

// avgpool_epi_kernel for 3x3 / stride-1 windows (Inception's commuted AvgPool branches):
// 16 channels x 2 adjacent outputs per thread, all 12 window pixels (24 16-B loads) issued
// before the first add — the generic kernel's runtime loops wait for each one in turn.
// Out-of-range pixels read a clamped in-range address and are masked out of the sum.
template <bool OUT_FP8, int ACT>
__global__ __launch_bounds__(256) void avgpool3_epi_kernel(const bf16* __restrict__ x, const float* __restrict__ bias,
                                                           uint8_t* __restrict__ y, int N, int H, int W, int C, int Ho,
                                                           int Wo, int ph, int pw, int ldy, int y_coff, float out_q) {
  constexpr int PX = 2, NC = PX + 2;
  const int cchunks = C / 16;
  const int wgroups = (Wo + PX - 1) / PX;
  const long total = (long)N * Ho * wgroups * cchunks;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int cc = idx % cchunks;
    long t = idx / cchunks;
    const int oxg = t % wgroups;
    t /= wgroups;
    const int oy = t % Ho;
    const int n = t / Ho;
    const int ox0 = oxg * PX;
    const int iy0 = oy - ph, ixs = ox0 - pw;
    bf16x8 va[3][NC], vb[3][NC];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int iyc = min(max(iy0 + dy, 0), H - 1);
      const bf16* row = x + ((size_t)n * H + iyc) * W * C + cc * 16;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ixc = min(max(ixs + c, 0), W - 1);
        const bf16x8* src = reinterpret_cast<const bf16x8*>(row + (size_t)ixc * C);
        va[dy][c] = src[0];
        vb[dy][c] = src[1];
      }
    }
    float bv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bv[e] = bias[cc * 16 + e];
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int ox = ox0 + p;
      if (ox >= Wo) break;
      float acc[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      int cnt = 0;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const bool yok = (unsigned)(iy0 + dy) < (unsigned)H;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const bool ok = yok && (unsigned)(ixs + p + dx) < (unsigned)W;
          cnt += ok ? 1 : 0;
          const float m = ok ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            acc[e] = __builtin_fmaf((float)va[dy][p + dx][e], m, acc[e]);
            acc[8 + e] = __builtin_fmaf((float)vb[dy][p + dx][e], m, acc[8 + e]);
          }
        }
      }
      const float inv = 1.f / (float)max(cnt, 1);
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = apply_act<ACT>(__builtin_fmaf(acc[e], inv, bv[e]));
      const size_t o = (((size_t)n * Ho + oy) * Wo + ox) * ldy + y_coff + cc * 16;
      if constexpr (OUT_FP8) {
        u32x4 q;
#pragma unroll
        for (int w = 0; w < 4; ++w) q[w] = pack4(v[4 * w] * out_q, v[4 * w + 1] * out_q, v[4 * w + 2] * out_q, v[4 * w + 3] * out_q);
        *reinterpret_cast<u32x4*>(y + o) = q;
      } else {
        bf16x8 o0, o1;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o0[e] = f2bf(v[e]);
          o1[e] = f2bf(v[8 + e]);
        }
        bf16x8* dst = reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(y) + o);
        dst[0] = o0;
        dst[1] = o1;
      }
    }
  }
}

// [N, HW, C] fp8 -> [N, C] bf16 mean * s.  One block per image, 16 channels per thread.
__global__ __launch_bounds__(256) void gap_fp8_kernel(const uint8_t* __restrict__ x, bf16* __restrict__ y, int HW, int C,
                                                      float s) {
  const int n = blockIdx.x;
  const float inv = s / (float)HW;
  for (int cc = threadIdx.x; cc < C / 16; cc += blockDim.x) {
    float acc[16] = {};
    const uint8_t* p = x + (size_t)n * HW * C + cc * 16;
#pragma unroll 8
    for (int i = 0; i < HW; ++i) {  // unrolled: 8 independent row loads in flight per thread
      u32x4 v = *reinterpret_cast<const u32x4*>(p + (size_t)i * C);
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        float f[4];
        unpack4(v[w], f);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[w * 4 + e] += f[e];
      }
    }
    bf16x8 o0, o1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o0[e] = f2bf(acc[e] * inv);
      o1[e] = f2bf(acc[8 + e] * inv);
    }
    bf16x8* dst = reinterpret_cast<bf16x8*>(y + (size_t)n * C + cc * 16);
    dst[0] = o0;
    dst[1] = o1;
  }
}

int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

// Conv2D NHWC on fp8 (see header).  x: fp8 [N,H,W,Cin] (bf16 when in_bf16), w: fp8
// [Cout, KH*KW*Cin], scale/bias fp32 [Cout]; out_fp8 selects fp8 (out_q = 1/sy) or bf16.
void conv2d_nhwc_fp8(uintptr_t x, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t y, int N, int H, int W,
                     int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw, int Ho, int Wo,
                     int ldy, int y_coff, int in_bf16, float in_q, int out_fp8, float out_q, int act, uintptr_t stream,
                     int cfg) {
  const int ealign = out_fp8 ? 16 : 8;
  if (Cin % 16) throw std::invalid_argument("conv2d_nhwc_fp8: Cin must be a multiple of 16");
  if (Cout % ealign || ldy % ealign || y_coff % ealign)
    throw std::invalid_argument("conv2d_nhwc_fp8: Cout/ldy/y_coff not a multiple of the 16-byte output chunk");
  if (Cout % 4) throw std::invalid_argument("conv2d_nhwc_fp8: Cout % 4 != 0");
  if (N <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0) throw std::invalid_argument("conv2d_nhwc_fp8: empty problem");
  if ((long)N * H * W * Cin >= (1L << 31) || (long)N * Ho * Wo >= (1L << 31))
    throw std::invalid_argument("conv2d_nhwc_fp8: tensor too large for 32-bit indexing");
  if (!scale || !bias) throw std::invalid_argument("conv2d_nhwc_fp8: scale and bias pointers are required");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  check_align(scale, 16, "scale");
  check_align(bias, 16, "bias");
  Fp8Params p{};
  p.prio = fp8_prio();
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = reinterpret_cast<const float*>(scale);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.in_q = in_q;
  p.out_q = out_q;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.KH = KH; p.KW = KW; p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.M = N * Ho * Wo;
  p.K = KH * KW * Cin;
  p.ldx = Cin;
  p.ldy = ldy; p.y_coff = y_coff;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (cfg == LITE_CFG) {
    p.stamp = g_lite_fp8_stamp;
    if (in_bf16) throw std::invalid_argument("conv2d_nhwc_fp8: the conv_lite tile takes fp8 input");
    if (ph >= 1024 || pw >= 1024 || H >= 16384 || W >= 16384) throw std::invalid_argument("conv2d_nhwc_fp8: geometry");
    if ((long)Cout * p.K >= (1L << 31)) throw std::invalid_argument("conv2d_nhwc_fp8: weights larger than 2 GiB");
    if (out_fp8) launch_lite_fp8<true>(p, act, s);
    else launch_lite_fp8<false>(p, act, s);
    FTM_CHECK_LAUNCH();
    return;
  }
  const bool pointwise = KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
  if (pointwise) launch_io<false>(p, in_bf16, out_fp8, act, cfg, s);
  else launch_io<true>(p, in_bf16, out_fp8, act, cfg, s);
}

// Horizontally fused sibling convs on the conv_lite_fp8 tile: one implicit GEMM over the
// concatenated filters [Cout_total][K], whose output channel ranges go to different
// destinations.  segs: [(y, c0, c1, ldy, y_coff, is_bf16, out_q)] covering [0, Cout) in
// order, every bound a multiple of 16; lo: fp32 [Cout] lower clamp (0 ReLU / -inf none).
void conv2d_nhwc_fp8_multi(uintptr_t x, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t lo, int N, int H,
                           int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw,
                           int Ho, int Wo, pybind11::list segs, uintptr_t stream, int mode) {
  const int ns = (int)pybind11::len(segs);
  if (ns < 1 || ns > MAX_SEGS) throw std::invalid_argument("conv2d_nhwc_fp8_multi: 1.." + std::to_string(MAX_SEGS) + " segments");
  if (Cin % 16 || Cout % 16) throw std::invalid_argument("conv2d_nhwc_fp8_multi: Cin / Cout % 16 != 0");
  if (N <= 0 || Ho <= 0 || Wo <= 0) throw std::invalid_argument("conv2d_nhwc_fp8_multi: empty problem");
  if ((long)N * H * W * Cin >= (1L << 31) || (long)N * Ho * Wo >= (1L << 31))
    throw std::invalid_argument("conv2d_nhwc_fp8_multi: tensor too large for 32-bit indexing");
  if (ph >= 1024 || pw >= 1024 || H >= 16384 || W >= 16384) throw std::invalid_argument("conv2d_nhwc_fp8_multi: geometry");
  if (!scale || !bias || !lo) throw std::invalid_argument("conv2d_nhwc_fp8_multi: scale, bias and clamp pointers required");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(scale, 16, "scale");
  check_align(bias, 16, "bias");
  check_align(lo, 16, "lo");
  Fp8Segs sg{};
  sg.n = ns;
  sg.lo = reinterpret_cast<const float*>(lo);
  int expect = 0;
  for (int i = 0; i < ns; ++i) {
    pybind11::tuple t = segs[i].cast<pybind11::tuple>();
    if (t.size() != 7) throw std::invalid_argument("segment tuple (y, c0, c1, ldy, y_coff, is_bf16, out_q)");
    const uintptr_t y = t[0].cast<uintptr_t>();
    const int c0 = t[1].cast<int>(), c1 = t[2].cast<int>(), ld = t[3].cast<int>(), off = t[4].cast<int>();
    const int isb = t[5].cast<int>();
    if (c0 != expect || c1 <= c0 || c0 % 16 || c1 % 16) throw std::invalid_argument("conv2d_nhwc_fp8_multi: segments must tile [0, Cout) in 16s");
    if (ld % 16 || off % 16 || off + (c1 - c0) > ld) throw std::invalid_argument("conv2d_nhwc_fp8_multi: segment pitch / offset");
    check_align(y, 16, "segment y");
    sg.y[i] = reinterpret_cast<uint8_t*>(y);
    sg.c0[i] = c0;
    sg.ld[i] = ld;
    sg.off[i] = off;
    sg.bf16[i] = isb;
    sg.q[i] = t[6].cast<float>();
    expect = c1;
  }
  if (expect != Cout) throw std::invalid_argument("conv2d_nhwc_fp8_multi: segments do not cover Cout");
  sg.c0[ns] = Cout;
  Fp8Params p{};
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = reinterpret_cast<const float*>(scale);
  p.bias = reinterpret_cast<const float*>(bias);
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.KH = KH; p.KW = KW; p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.M = N * Ho * Wo;
  p.K = KH * KW * Cin;
  p.ldx = Cin;
  if ((long)Cout * p.K >= (1L << 31)) throw std::invalid_argument("conv2d_nhwc_fp8_multi: weights larger than 2 GiB");
  (void)mode;
  launch_lite_fp8<false, true>(p, ACT_NONE, reinterpret_cast<hipStream_t>(stream), sg);
  FTM_CHECK_LAUNCH();
}

// Y[M, N] = act(Xq[M, K] . Wq[N, K]^T * scale + bias)
void gemm_fp8(uintptr_t x, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t y, int M, int N, int K, int ldx,
              int ldy, int in_bf16, float in_q, int out_fp8, float out_q, int act, uintptr_t stream, int cfg) {
  const int ealign = out_fp8 ? 16 : 8;
  if (K % 16 || ldx % 16) throw std::invalid_argument("gemm_fp8: K and ldx must be multiples of 16");
  if (N % ealign || ldy % ealign) throw std::invalid_argument("gemm_fp8: N/ldy not a multiple of the output chunk");
  if (M <= 0 || N <= 0) throw std::invalid_argument("gemm_fp8: empty problem");
  if (!scale || !bias) throw std::invalid_argument("gemm_fp8: scale and bias pointers are required");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  check_align(scale, 16, "scale");
  check_align(bias, 16, "bias");
  Fp8Params p{};
  p.prio = fp8_prio();
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = reinterpret_cast<const float*>(scale);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.in_q = in_q;
  p.out_q = out_q;
  p.M = M; p.Cout = N; p.K = K; p.ldx = ldx; p.ldy = ldy; p.y_coff = 0;
  launch_io<false>(p, in_bf16, out_fp8, act, cfg, reinterpret_cast<hipStream_t>(stream));
}

void quantize_bf16_fp8(uintptr_t x, uintptr_t y, long n, float q, uintptr_t stream) {
  if (n % 16) throw std::invalid_argument("quantize_bf16_fp8: n % 16 != 0");
  check_align(x, 16, "x");
  check_align(y, 16, "y");
  if (n == 0) return;
  hipLaunchKernelGGL(quantize_kernel, dim3(grid_for(n / 16, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16*>(x), reinterpret_cast<uint8_t*>(y), n / 16, q);
  FTM_CHECK_LAUNCH();
}

void dequantize_fp8_bf16(uintptr_t x, uintptr_t y, long n, float s, uintptr_t stream) {
  if (n % 16) throw std::invalid_argument("dequantize_fp8_bf16: n % 16 != 0");
  check_align(x, 16, "x");
  check_align(y, 16, "y");
  if (n == 0) return;
  hipLaunchKernelGGL(dequantize_kernel, dim3(grid_for(n / 16, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint8_t*>(x),
                     reinterpret_cast<bf16*>(y), n / 16, s);
  FTM_CHECK_LAUNCH();
}

void pool2d_nhwc_fp8(uintptr_t x, uintptr_t y, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh,
                     int sw, int ph, int pw, int ldy, int y_coff, int is_max, float rq, uintptr_t stream) {
  if (C % 16 || ldy % 16 || y_coff % 16) throw std::invalid_argument("pool2d_nhwc_fp8: C/ldy/y_coff % 16 != 0");
  check_align(x, 16, "x");
  check_align(y, 16, "y");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto X = reinterpret_cast<const uint8_t*>(x);
  auto Y = reinterpret_cast<uint8_t*>(y);
  if (is_max && kh == 3 && kw == 3 && sh == 2 && (sw == 1 || sw == 2) && H > 0 && W > 0) {
    const long work = (long)N * Ho * ((Wo + 1) / 2) * (C / 16);
    if (sw == 2)
      hipLaunchKernelGGL((maxpool3_fp8_kernel<2>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, Y, N, H, W, C, Ho, Wo,
                         ph, pw, ldy, y_coff, rq);
    else
      hipLaunchKernelGGL((maxpool3_fp8_kernel<1>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, Y, N, H, W, C, Ho, Wo,
                         ph, pw, ldy, y_coff, rq);
    FTM_CHECK_LAUNCH();
    return;
  }
  // stride-1 windows: 2 outputs per thread share window columns; strided: 1
  if (sw == 1) {
    const long work = (long)N * Ho * ((Wo + 1) / 2) * (C / 16);
    if (is_max)
      hipLaunchKernelGGL((pool_fp8_kernel<true, 2>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, Y, N, H, W, C, Ho,
                         Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, rq);
    else
      hipLaunchKernelGGL((pool_fp8_kernel<false, 2>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, Y, N, H, W, C, Ho,
                         Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, rq);
  } else {
    const long work = (long)N * Ho * Wo * (C / 16);
    if (is_max)
      hipLaunchKernelGGL((pool_fp8_kernel<true, 1>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, Y, N, H, W, C, Ho,
                         Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, rq);
    else
      hipLaunchKernelGGL((pool_fp8_kernel<false, 1>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, Y, N, H, W, C, Ho,
                         Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, rq);
  }
  FTM_CHECK_LAUNCH();
}

template <bool OUT_FP8, int ACT>
void launch_avgpool_epi(const bf16* X, const float* B, uint8_t* Y, int N, int H, int W, int C, int Ho, int Wo, int kh,
                        int kw, int sh, int sw, int ph, int pw, int ldy, int y_coff, float out_q, hipStream_t s) {
  if (kh == 3 && kw == 3 && sh == 1 && sw == 1 && H > 0 && W > 0) {
    const long work = (long)N * Ho * ((Wo + 1) / 2) * (C / 16);
    hipLaunchKernelGGL((avgpool3_epi_kernel<OUT_FP8, ACT>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, B, Y, N, H,
                       W, C, Ho, Wo, ph, pw, ldy, y_coff, out_q);
    return;
  }
  if (sw == 1) {
    const long work = (long)N * Ho * ((Wo + 1) / 2) * (C / 16);
    hipLaunchKernelGGL((avgpool_epi_kernel<OUT_FP8, ACT, 2>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, B, Y, N, H,
                       W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, out_q);
  } else {
    const long work = (long)N * Ho * Wo * (C / 16);
    hipLaunchKernelGGL((avgpool_epi_kernel<OUT_FP8, ACT, 1>), dim3(grid_for(work, 256)), dim3(256), 0, s, X, B, Y, N, H,
                       W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, out_q);
  }
}

// y[.., y_coff:y_coff+C] = act(avgpool(x) + bias) (* out_q as fp8 when out_fp8, else bf16);
// x bf16 [N, H, W, C], bias fp32 [C], act NONE or RELU.
void avgpool_bias_act(uintptr_t x, uintptr_t bias, uintptr_t y, int N, int H, int W, int C, int Ho, int Wo, int kh,
                      int kw, int sh, int sw, int ph, int pw, int ldy, int y_coff, int out_fp8, float out_q, int act,
                      uintptr_t stream) {
  if (C % 16 || ldy % 16 || y_coff % 16) throw std::invalid_argument("avgpool_bias_act: C/ldy/y_coff % 16 != 0");
  if (act != ACT_NONE && act != ACT_RELU) throw std::invalid_argument("avgpool_bias_act: act must be NONE or RELU");
  if (N <= 0 || Ho <= 0 || Wo <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0)
    throw std::invalid_argument("avgpool_bias_act: empty problem");
  if (y_coff + C > ldy) throw std::invalid_argument("avgpool_bias_act: channel slot exceeds the output row");
  check_align(x, 16, "x");
  check_align(y, 16, "y");
  if (!bias) throw std::invalid_argument("avgpool_bias_act: bias pointer is required");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto X = reinterpret_cast<const bf16*>(x);
  auto B = reinterpret_cast<const float*>(bias);
  auto Y = reinterpret_cast<uint8_t*>(y);
  if (out_fp8) {
    if (act == ACT_RELU) launch_avgpool_epi<true, ACT_RELU>(X, B, Y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, out_q, s);
    else launch_avgpool_epi<true, ACT_NONE>(X, B, Y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, out_q, s);
  } else {
    if (act == ACT_RELU) launch_avgpool_epi<false, ACT_RELU>(X, B, Y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, out_q, s);
    else launch_avgpool_epi<false, ACT_NONE>(X, B, Y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff, out_q, s);
  }
  FTM_CHECK_LAUNCH();
}

void global_avgpool_fp8(uintptr_t x, uintptr_t y, int N, int HW, int C, float s, uintptr_t stream) {
  if (C % 16) throw std::invalid_argument("global_avgpool_fp8: C % 16 != 0");
  check_align(x, 16, "x");
  check_align(y, 16, "y");
  hipLaunchKernelGGL(gap_fp8_kernel, dim3(N), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const uint8_t*>(x), reinterpret_cast<bf16*>(y), HW, C, s);
  FTM_CHECK_LAUNCH();
}

void register_fp8(pybind11::module_& m) {
  m.def("conv2d_nhwc_fp8", &conv2d_nhwc_fp8);
  m.def("conv_lite_fp8_stamp", [](uintptr_t b) { g_lite_fp8_stamp = reinterpret_cast<unsigned long long*>(b); });
  m.def("gemm_fp8", &gemm_fp8);
  m.def("quantize_bf16_fp8", &quantize_bf16_fp8);
  m.def("dequantize_fp8_bf16", &dequantize_fp8_bf16);
  m.def("pool2d_nhwc_fp8", &pool2d_nhwc_fp8);
  m.def("global_avgpool_fp8", &global_avgpool_fp8);
  m.def("avgpool_bias_act", &avgpool_bias_act);
  m.def("conv2d_nhwc_fp8_multi", &conv2d_nhwc_fp8_multi);
  // the channel tile conv_lite_fp8 picks (host logic only; tests/test_fp8.py)
  m.def("lite_fp8_tile", [](int Cout) { return lite_fp8_bn(Cout); });
  m.attr("fp8_igemm_num_configs") = NCFG;
}
