// Pipelined implicit-GEMM convolution / GEMM for CDNA4: 256-pixel tiles, 8 waves, operands
// streamed global -> LDS by the LDS-DMA path (global_load_lds_dwordx4) through a 3-stage
// ring whose next tile stays in flight across the per-K-tile barrier (counted vmcnt + raw
// s_barrier, guide §5 "Pipelining across barriers").  One kernel body serves bf16
// (16x16x32 MFMA, 64-deep K tiles) and OCP fp8 (16x16x128 f8f6f4 MFMA, 128-deep K tiles):
// an LDS row is 128 B in both.
//
// im2col with DMA: the LDS image must be lane-linear per wave instruction (64 lanes x 16 B =
// 8 rows x 128 B), so the XOR swizzle (chunk ^ (row & 7), conflict-free fragment reads) is
// applied on the per-lane SOURCE address, and padding / K-tail / out-of-range lanes point
// at a 16-byte zero page instead of being masked.
//
// Epilogue (as igemm_bf16.hip / fp8.hip): acc [* per-channel dequant scale] + bias -> act
// -> LDS tile -> coalesced 16-B row segments [+ residual, act] -> bf16 or e4m3 (x 1/sy)
// at a channel offset of a wider output (concat-by-stride-write).
//
// Tiles: BM = 256 pixels x BN = 128 channels (8 waves as 4 x 2, 64 x 64 per wave) or
// BN = 64 (8 x 1, 32 x 64 per wave).  LDS: 3 x (256 + BN) x 128 B = 144 / 120 KiB, one
// workgroup per CU; the 8 waves (2 per SIMD) interleave MFMA with the DMA and ds_reads.
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

typedef int i32x8 __attribute__((ext_vector_type(8)));

namespace {

__device__ __attribute__((aligned(16))) uint32_t g_zero16[4];  // zero page for padded lanes

constexpr int BM = 256;
constexpr int ROWB = 128;  // LDS row bytes = one K tile of one row
// LDS ring stages: 3 (two tiles in flight) for BN <= 128; the 256 x 256 tile fits only 2
template <int BN>
constexpr int stages() { return BN >= 256 ? 2 : 3; }
constexpr int NT = 512;

struct V2Params {
  const uint8_t* x;
  const uint8_t* w;
  const float* scale;  // fp8: per-channel dequant scale (sw[c] * sx); unused for bf16
  const float* bias;
  const uint8_t* res;  // bf16 residual [M, ldr] (bf16 output only)
  uint8_t* y;
  float out_q;  // fp8 output: 1 / sy
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, sh, sw, ph, pw, dh, dw;
  int M, K;
  int ldx, ldy, y_coff, ldr;
  int tiles_m, tiles_n;
};

FTM_DEVICE int swz(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 7)) << 4); }

FTM_DEVICE void glds16(const void* src, uint8_t* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
FTM_DEVICE void wait_then_barrier() {
  // retire all but the newest N DMA ops of this wave, finish this wave's LDS reads, then
  // meet the other waves: the tile waited for is now visible to every wave and nobody
  // still reads the stage that the next DMA will overwrite
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

FTM_DEVICE uint32_t pack4_fp8(float a, float b, float c, float d) {
  const float M = 448.f;
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -M), M), fminf(fmaxf(b, -M), M), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -M), M), fminf(fmaxf(d, -M), M), w, true);
  return (uint32_t)w;
}

// ABL (diagnostic builds only, igemm_v2_ablate): 1 = no MFMA, 2 = no DMA loads, 4 = no
// fragment ds_reads — timing-only variants that locate the kernel's bottleneck.
template <int ES, int BN, bool CONV, bool OUT_FP8, int ACT, bool HAS_RES, int ABL = 0>
__global__ __launch_bounds__(NT, 1) void igemm_v2_kernel(V2Params p) {
  constexpr int EPC = 16 / ES;          // elements per 16-B chunk
  constexpr int BKE = ROWB / ES;        // K elements per tile
  constexpr int NS = stages<BN>();
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 8 / WAVES_N;
  constexpr int TM = BM / WAVES_M;      // pixels per wave
  constexpr int J = TM / 16;
  constexpr int XG = BM / 64;           // X row groups (8 rows) per wave per stage
  constexpr int WG = BN / 64;           // W row groups per wave per stage
  constexpr int GL = XG + WG;           // DMA instructions per wave per stage
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int OB = OUT_FP8 ? 1 : 2;
  constexpr int OLD = BN * OB + 16;     // epilogue LDS row pitch (bytes)
  constexpr int LDS_BYTES = BM * OLD > NS * STAGE ? BM * OLD : NS * STAGE;  // ring, reused by the epilogue
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS_BYTES];

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

  // ---- DMA lane roles: row (lane >> 3) of an 8-row group, source chunk pre-swizzled
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  int xbase[XG], hb[XG], wb[XG];
  bool mvalid[XG];
#pragma unroll
  for (int i = 0; i < XG; ++i) {
    const int m = m0 + (wave * XG + i) * 8 + lrow;
    mvalid[i] = m < p.M;
    const int mm = mvalid[i] ? m : 0;
    if constexpr (CONV) {
      const int wo = mm % p.Wo;
      const int t = mm / p.Wo;
      const int ho = t % p.Ho;
      const int n = t / p.Ho;
      xbase[i] = n * p.H * p.W * p.Cin;
      hb[i] = ho * p.sh - p.ph;
      wb[i] = wo * p.sw - p.pw;
    } else {
      xbase[i] = mm * p.ldx;
      hb[i] = wb[i] = 0;
    }
  }
  const uint8_t* wrow[WG];
  bool nvalid[WG];
#pragma unroll
  for (int i = 0; i < WG; ++i) {
    const int co = n0 + (wave * WG + i) * 8 + lrow;
    nvalid[i] = co < p.Cout;
    wrow[i] = p.w + (size_t)(nvalid[i] ? co : 0) * p.K * ES;
  }
  const void* zero = g_zero16;

  auto issue = [&](int kt, int buf) {
    if constexpr (ABL & 2) return;
    uint8_t* xs = smem + buf * STAGE;
    uint8_t* ws = xs + BM * ROWB;
    const int k = kt * BKE + lchunk * EPC;
    const bool kvalid = k < p.K;
    if constexpr (CONV) {
      const int kidx = k / p.Cin;
      const int ci = k - kidx * p.Cin;
      const int kh = kidx / p.KW;
      const int kw = kidx - kh * p.KW;
#pragma unroll
      for (int i = 0; i < XG; ++i) {
        const int hi = hb[i] + kh * p.dh;
        const int wi = wb[i] + kw * p.dw;
        const bool ok = kvalid && mvalid[i] && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        const void* src = ok ? (const void*)(p.x + ((size_t)xbase[i] + ((size_t)hi * p.W + wi) * p.Cin + ci) * ES) : zero;
        glds16(src, xs + (wave * XG + i) * 8 * ROWB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < XG; ++i) {
        const bool ok = kvalid && mvalid[i];
        const void* src = ok ? (const void*)(p.x + ((size_t)xbase[i] + k) * ES) : zero;
        glds16(src, xs + (wave * XG + i) * 8 * ROWB);
      }
    }
#pragma unroll
    for (int i = 0; i < WG; ++i) {
      const void* src = (kvalid && nvalid[i]) ? (const void*)(wrow[i] + (size_t)k * ES) : zero;
      glds16(src, ws + (wave * WG + i) * 8 * ROWB);
    }
  };

  f32x4 acc[4][J];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int nk = (p.K + BKE - 1) / BKE;

  constexpr int PD = NS - 1;  // prefetch distance (tiles)
  issue(0, 0);
  if (PD > 1 && nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (PD > 1 && kt + 1 < nk) wait_then_barrier<GL>();  // tile kt+1 may stay in flight
    else wait_then_barrier<0>();
    if (kt + PD < nk) issue(kt + PD, (kt + PD) % NS);
    const uint8_t* xs = smem + (kt % NS) * STAGE;
    const uint8_t* ws = xs + BM * ROWB;
    if constexpr (ES == 2) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[4], b[J];
        const int chunk = ks * 4 + fq;
        if constexpr (ABL & 4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = bf16x8{} + (bf16)(float)(kt + i);
#pragma unroll
          for (int j = 0; j < J; ++j) b[j] = bf16x8{} + (bf16)(float)(ks + j);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ws + swz(wc * 64 + i * 16 + frow, chunk));
#pragma unroll
          for (int j = 0; j < J; ++j) b[j] = *reinterpret_cast<const bf16x8*>(xs + swz(wp * TM + j * 16 + frow, chunk));
        }
        if constexpr (ABL & 1) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < J; ++j) acc[i][j][0] += (float)a[i][0] * (float)b[j][1];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
      }
    } else {
      i32x8 a[4], b[J];
      const int c0 = 2 * fq;
      if constexpr (ABL & 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = i32x8{} + (kt + i);
#pragma unroll
        for (int j = 0; j < J; ++j) b[j] = i32x8{} + (kt * 3 + j);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wc * 64 + i * 16 + frow;
          const u32x4 lo = *reinterpret_cast<const u32x4*>(ws + swz(row, c0));
          const u32x4 hi = *reinterpret_cast<const u32x4*>(ws + swz(row, c0 + 1));
          a[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int row = wp * TM + j * 16 + frow;
          const u32x4 lo = *reinterpret_cast<const u32x4*>(xs + swz(row, c0));
          const u32x4 hi = *reinterpret_cast<const u32x4*>(xs + swz(row, c0 + 1));
          b[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
      }
      if constexpr (ABL & 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < J; ++j) acc[i][j][0] += (float)(a[i][0] ^ b[j][7]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < J; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, 127, 0, 127);
      }
    }
  }
  wait_then_barrier<0>();  // ring idle: reuse it for the output tile

  // ---- epilogue phase 1: [dequant] + bias + act (act after residual when HAS_RES)
  uint8_t* Os = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cl = wc * 64 + i * 16 + fq * 4;
    f32x4 sv = {1.f, 1.f, 1.f, 1.f}, bv = {0.f, 0.f, 0.f, 0.f};
    if (n0 + cl < p.Cout) {
      if constexpr (ES == 1) sv = *reinterpret_cast<const f32x4*>(p.scale + n0 + cl);
      bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int pl = wp * TM + j * 16 + frow;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] * sv[r] + bv[r];
        if constexpr (!HAS_RES) v[r] = apply_act<ACT>(v[r]);
      }
      if constexpr (OUT_FP8) {
        *reinterpret_cast<uint32_t*>(Os + pl * OLD + cl) =
            pack4_fp8(v[0] * p.out_q, v[1] * p.out_q, v[2] * p.out_q, v[3] * p.out_q);
      } else {
        bf16x4 o;
        o[0] = f2bf(v[0]); o[1] = f2bf(v[1]); o[2] = f2bf(v[2]); o[3] = f2bf(v[3]);
        *reinterpret_cast<bf16x4*>(Os + pl * OLD + cl * 2) = o;
      }
    }
  }
  __syncthreads();

  // ---- epilogue phase 2: coalesced 16-B row segments
  constexpr int EPO = 16 / OB;
  constexpr int CPR = BN / EPO;
#pragma unroll
  for (int q = tid; q < BM * CPR; q += NT) {
    const int pl = q / CPR;
    const int cc = q % CPR;
    const int m = m0 + pl;
    const int c = n0 + cc * EPO;
    if (m >= p.M || c >= p.Cout) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(Os + pl * OLD + cc * 16);
    if constexpr (HAS_RES) {
      bf16x8 o = __builtin_bit_cast(bf16x8, v);
      const bf16x8 r = *reinterpret_cast<const bf16x8*>(p.res + ((size_t)m * p.ldr + c) * 2);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(apply_act<ACT>((float)o[e] + (float)r[e]));
      v = __builtin_bit_cast(u32x4, o);
    }
    *reinterpret_cast<u32x4*>(p.y + ((size_t)m * p.ldy + p.y_coff + c) * OB) = v;
  }
}

template <int ES, int BN, bool CONV, bool OUT_FP8, int ACT>
void launch_res(const V2Params& p0, hipStream_t s) {
  V2Params p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.Cout + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n), block(NT);
  if constexpr (ES == 2 && !OUT_FP8) {
    if (p.res) {
      hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, CONV, OUT_FP8, ACT, true>), grid, block, 0, s, p);
      return;
    }
  }
  if (p.res) throw std::invalid_argument("igemm_v2: residual needs bf16 in/out");
  hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, CONV, OUT_FP8, ACT, false>), grid, block, 0, s, p);
}

template <int ES, int BN, bool CONV, bool OUT_FP8>
void launch_act(const V2Params& p, int act, hipStream_t s) {
  switch (act) {
    case ACT_NONE: launch_res<ES, BN, CONV, OUT_FP8, ACT_NONE>(p, s); break;
    case ACT_RELU: launch_res<ES, BN, CONV, OUT_FP8, ACT_RELU>(p, s); break;
    case ACT_GELU_TANH:
      if constexpr (!CONV && ES == 2 && !OUT_FP8) {  // transformer FFN GEMMs
        launch_res<ES, BN, CONV, OUT_FP8, ACT_GELU_TANH>(p, s);
        break;
      }
      [[fallthrough]];
    default: throw std::invalid_argument("igemm_v2: activation must be none/relu (gelu: bf16 GEMM only)");
  }
}

template <int ES, bool CONV>
void launch_v2(const V2Params& p, int bn, bool out_fp8, int act, hipStream_t s) {
  if (bn == 256) {
    if constexpr (!CONV) {  // large plain GEMMs (transformer projections / FFN)
      if (out_fp8) launch_act<ES, 256, CONV, true>(p, act, s);
      else launch_act<ES, 256, CONV, false>(p, act, s);
    } else {
      throw std::invalid_argument("igemm_v2: bn 256 is a GEMM-mode tile");
    }
  } else if (bn == 128) {
    if (out_fp8) launch_act<ES, 128, CONV, true>(p, act, s);
    else launch_act<ES, 128, CONV, false>(p, act, s);
  } else {
    if (out_fp8) launch_act<ES, 64, CONV, true>(p, act, s);
    else launch_act<ES, 64, CONV, false>(p, act, s);
  }
  FTM_CHECK_LAUNCH();
}

void check_align(uintptr_t ptr, int bytes, const char* what) {
  if (ptr % bytes) throw std::invalid_argument(std::string(what) + " is not " + std::to_string(bytes) + "-byte aligned");
}

}  // namespace

// Pipelined conv/GEMM entry point.  es = 2 (bf16 x/w) or 1 (e4m3 x/w with per-channel
// ``scale``); out_fp8 writes e4m3 with ``out_q`` = 1/sy.  KH = KW = 1, stride 1, no padding
// runs as a plain GEMM over the [M, Cin] pixel matrix.  bn = 64 | 128 output channels per tile.
void igemm_v2(uintptr_t x, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t res, uintptr_t y, int es, int N,
              int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw, int Ho,
              int Wo, int ldy, int y_coff, int ldr, int out_fp8, float out_q, int act, int bn, uintptr_t stream) {
  if (es != 1 && es != 2) throw std::invalid_argument("igemm_v2: es must be 1 (fp8) or 2 (bf16)");
  const int epc = 16 / es;
  const int oe = out_fp8 ? 16 : 8;
  if (Cin % epc) throw std::invalid_argument("igemm_v2: Cin must be a multiple of " + std::to_string(epc));
  if (Cout % oe || ldy % oe || y_coff % oe) throw std::invalid_argument("igemm_v2: Cout/ldy/y_coff alignment");
  if (Cout % 4) throw std::invalid_argument("igemm_v2: Cout % 4 != 0");
  if (bn != 64 && bn != 128 && bn != 256) throw std::invalid_argument("igemm_v2: bn must be 64, 128 or 256");
  if (res && (es != 2 || out_fp8 || ldr % 8)) throw std::invalid_argument("igemm_v2: bad residual");
  if (N <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0) throw std::invalid_argument("igemm_v2: empty problem");
  if ((long)N * H * W * Cin >= (1L << 31) || (long)N * Ho * Wo >= (1L << 31))
    throw std::invalid_argument("igemm_v2: tensor too large for 32-bit indexing");
  if (!bias || (es == 1 && !scale)) throw std::invalid_argument("igemm_v2: bias (and fp8 scale) required");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  check_align(bias, 16, "bias");
  if (scale) check_align(scale, 16, "scale");
  if (res) check_align(res, 16, "residual");
  V2Params p{};
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = reinterpret_cast<const float*>(scale);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const uint8_t*>(res);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.out_q = out_q;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.KH = KH; p.KW = KW; p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.M = N * Ho * Wo;
  p.K = KH * KW * Cin;
  p.ldx = Cin;
  p.ldy = ldy; p.y_coff = y_coff; p.ldr = ldr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool pointwise = KH == 1 && KW == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0;
  if (es == 2) {
    if (pointwise) launch_v2<2, false>(p, bn, out_fp8, act, s);
    else launch_v2<2, true>(p, bn, out_fp8, act, s);
  } else {
    if (pointwise) launch_v2<1, false>(p, bn, out_fp8, act, s);
    else launch_v2<1, true>(p, bn, out_fp8, act, s);
  }
}

// Diagnostic: times one ablated variant of the 3x3-conv kernel (es 2: bf16, BN 64, bf16
// out; es 1: fp8, BN 128, fp8 out; ReLU).  Outputs are meaningless.
template <int ES, int BN, bool OUT_FP8>
void launch_ablate(const V2Params& p0, int abl, hipStream_t s) {
  V2Params p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.Cout + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n), block(NT);
  switch (abl) {
    case 0: hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, true, OUT_FP8, ACT_RELU, false, 0>), grid, block, 0, s, p); break;
    case 1: hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, true, OUT_FP8, ACT_RELU, false, 1>), grid, block, 0, s, p); break;
    case 2: hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, true, OUT_FP8, ACT_RELU, false, 2>), grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, true, OUT_FP8, ACT_RELU, false, 4>), grid, block, 0, s, p); break;
    case 6: hipLaunchKernelGGL((igemm_v2_kernel<ES, BN, true, OUT_FP8, ACT_RELU, false, 6>), grid, block, 0, s, p); break;
    default: throw std::invalid_argument("ablation must be 0, 1, 2, 4 or 6");
  }
  FTM_CHECK_LAUNCH();
}

void igemm_v2_ablate(uintptr_t x, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t y, int es, int N, int H,
                     int W, int Cin, int Cout, int KH, int KW, int ph, int pw, int Ho, int Wo, int abl,
                     uintptr_t stream) {
  if (Cin % (16 / es) || Cout % 16) throw std::invalid_argument("igemm_v2_ablate: channel alignment");
  V2Params p{};
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = reinterpret_cast<const float*>(scale);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.out_q = 1.f;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.KH = KH; p.KW = KW; p.sh = 1; p.sw = 1; p.ph = ph; p.pw = pw; p.dh = 1; p.dw = 1;
  p.M = N * Ho * Wo;
  p.K = KH * KW * Cin;
  p.ldx = Cin;
  p.ldy = Cout;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (es == 2) launch_ablate<2, 64, false>(p, abl, s);
  else launch_ablate<1, 128, true>(p, abl, s);
}

void register_igemm_v2(pybind11::module_& m) {
  m.def("igemm_v2", &igemm_v2);
  m.def("igemm_v2_ablate", &igemm_v2_ablate);
}
