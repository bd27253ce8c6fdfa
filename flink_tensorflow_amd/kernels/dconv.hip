// Direct convolution for narrow layers (few input channels x taps): the whole reduction
// of one output tile runs out of LDS.
//
// The implicit-GEMM kernels re-read every input pixel once per filter tap (KH*KW x im2col
// traffic).  For layers whose weights and input halo fit on chip at once — the RGB stems
// (3 -> 32/64 channels), Inception's 147x147 / 73x73 / 35x35 3x3 layers (32..128 fp8 input
// channels) — that re-read traffic, not the MFMAs, bounds the layer.  Here one workgroup
//   1. DMAs its input patch ((TH-1)*S + KH) x ((TW-1)*S + KW) pixels x Cin (zero page for
//      padding) and the filter bank [BN][KH*KW*Cin (+pad)] into LDS (global_load_lds),
//   2. runs the K loop from LDS: an MFMA K-step covers 4 lane groups x KL bytes (KL = 16 B
//      bf16 / 32 B fp8); each lane group's KL-byte K segment lies inside ONE filter tap
//      (Cin*ES is a multiple of KL), so its B fragment is the tap-shifted patch row —
//      im2col happens in the LDS address, never in memory traffic,
//   3. stages the [256 px][BN] result through LDS and stores 16-B row segments (bf16 or
//      e4m3 with the successor's scale), channel-offset capable (concat slices).
// Output tile: 16 x 16 pixels of one image with 4 waves, 32 x 16 with 8 (wave w owns tile
// rows 4w..4w+3 = 4 fragments), BN = 32 or 64 channels.  Pooled (stem) tiles are 17 conv columns wide: 4 waves cover 7 x 8
// pooled pixels, 8 waves (pool_rows = 14) 14 x 8 — the filter bank DMA (34 KB for the
// ResNet s2d stem, an L2 hit but the largest per-workgroup transfer) is then paid once per
// 112 pooled pixels instead of 56: 181 -> 161 us for the B=256 stem (bench/stem_ab.py).  Weights are pre-arranged by the host: row pitch WP bytes =
// round_up(KH*KW*Cin*ES, 4*KL) + 16 (the +16 keeps the 16 rows of a fragment read on
// different banks).
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

typedef int i32x8 __attribute__((ext_vector_type(8)));

namespace {

__device__ __attribute__((aligned(16))) uint32_t g_zero16[4];

constexpr int TH = 16, TW = 16;  // 4-wave tile (8 waves: 32 x 16)

struct DconvParams {
  const uint8_t* x;    // [N, H, W, Cin] (bf16 or e4m3)
  const uint8_t* w;    // [Cout_pad][WP] bytes, K order (kh, kw, ci)
  const float* scale;  // fp8: per-channel sw[c]*sx (nullptr for bf16)
  const float* bias;
  uint8_t* y;
  float out_q;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, S, ph, pw;
  int RB;      // patch row bytes = Cin * ES
  int WP;      // weight row pitch (bytes)
  int ksteps;  // MFMA K-steps = (WP - 16) / (4 * KL)
  int PH, PW;  // patch rows / cols
  int ldy, y_coff;
  int tiles_h, tiles_w, tiles_n;
  int prio;  // s_setprio(1) around the K loop (ftm_mfma_prio)
  // POOL: fused 3x3 / stride-2 max pool of the (ReLU) conv output.  A workgroup owns a
  // 7 x 8 pooled tile, i.e. a 15 x 17 conv tile (255 of the 256 fragment pixels, rows
  // 14t - ppt.., cols 16t - ppl..); out-of-range conv positions enter the max as 0
  // (exact after a ReLU).
  int Hp, Wp, ppt, ppl;
  // U8: the input is the raw uint8 RGB batch [N, Hi, Wi, 3] and the patch is built as the
  // 2x2 space-to-depth bf16 rows the preprocess kernel would write ((v - mean) * istd at
  // channel (2a + b) * 3 + c of block (y, x) <- pixel (2y + a, 2x + b); 12..15 and pixels
  // past the image zero): the preprocess pass and its HBM round trip disappear
  const uint8_t* xu8;
  int Hi, Wi;
  float mean[3], istd[3];
  // byte offset into the patch of each (K-step, lane group) relative to the lane's pixel:
  // (dy * PW + dx) * RB + channel byte of the K segment's tap; host-built so the K loop has
  // no integer divisions (two runtime divides per step used to cost more than its MFMAs)
  int koff[4 * 64];
};

FTM_DEVICE int koff_of(const DconvParams& p, int s, int fq) {
  const int k0 = p.koff[s * 4], k1 = p.koff[s * 4 + 1], k2 = p.koff[s * 4 + 2], k3 = p.koff[s * 4 + 3];
  return fq == 0 ? k0 : fq == 1 ? k1 : fq == 2 ? k2 : k3;
}

FTM_DEVICE void glds16(const void* src, uint8_t* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

FTM_DEVICE uint32_t pack4_fp8(float a, float b, float c, float d) {
  const float M = 448.f;
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -M), M), fminf(fmaxf(b, -M), M), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -M), M), fminf(fmaxf(d, -M), M), w, true);
  return (uint32_t)w;
}

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));

// 3x3 max over bf16 rows of the LDS output tile.  The pooled convs are ReLU convs, so every
// value is +0 or positive (out-of-image positions enter as +0) and the bf16 bit patterns
// order like the values: the max is an unsigned 16-bit max, 4 v_pk_max_u16 per 8 channels
// (a float compare per element made this epilogue, not the MFMAs, bound the stem).
FTM_DEVICE u16x8 pool3x3_max(const uint8_t* base, int row_bytes, int px_bytes) {
  u16x8 m = *reinterpret_cast<const u16x8*>(base);
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
      if (dy | dx) m = __builtin_elementwise_max(m, *reinterpret_cast<const u16x8*>(base + dy * row_bytes + dx * px_bytes));
  return m;
}

// The same over e4m3 bytes (fp8 chains, e.g. Inception's Conv2d_2b -> MaxPool_3a): a ReLU
// output is +0 or positive and saturated below the NaN code, so the e4m3 bytes order like
// the values too: an unsigned byte max of the already-quantised tile (exactly the max pool
// of the fp8 values the unfused layers would store).
FTM_DEVICE u8x16 pool3x3_max_u8(const uint8_t* base, int row_bytes, int px_bytes) {
  u8x16 m = *reinterpret_cast<const u8x16*>(base);
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
      if (dy | dx) m = __builtin_elementwise_max(m, *reinterpret_cast<const u8x16*>(base + dy * row_bytes + dx * px_bytes));
  return m;
}

template <int ES, int BN, int ACT, bool OUT_FP8, bool POOL = false, int WAVES = 4, bool U8 = false>
__global__ __launch_bounds__(WAVES * 64) void dconv_kernel(DconvParams p) {
  static_assert(WAVES == 4 || WAVES == 8, "4 or 8 waves");
  constexpr int NTH = WAVES * 64;
  constexpr int PTH = WAVES == 8 ? 14 : 7;  // pooled rows per tile
  constexpr int THE = TH * WAVES / 4;       // conv rows per (unpooled) tile: 16 or 32
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int KL = ES == 2 ? 16 : 32;  // K bytes per lane per MFMA
  constexpr int I = BN / 16;             // channel fragments
  constexpr int J = 4;                   // pixel fragments (tile rows) per wave
  constexpr int OB = OUT_FP8 ? 1 : 2;
  constexpr int OLD = BN * OB + 16;

  // block -> (image, tile row, tile col, channel tile); channel tiles of one spatial tile
  // are adjacent so they share the patch through L2
  int b = blockIdx.x;
  const int tn = b % p.tiles_n; b /= p.tiles_n;
  const int tw = b % p.tiles_w; b /= p.tiles_w;
  const int th = b % p.tiles_h;
  const int n = b / p.tiles_h;
  constexpr int TPW = POOL ? 17 : TW;  // conv tile width (pixel p of the tile = row p / TPW, col p % TPW)
  const int oy0 = POOL ? th * (2 * PTH) - p.ppt : th * THE, ox0 = POOL ? tw * 16 - p.ppl : tw * TW, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int patch_bytes = p.PH * p.PW * p.RB;
  uint8_t* Ps = smem;                                     // patch [PH*PW][RB]
  uint8_t* Wsm = smem + ((patch_bytes + 1023) & ~1023);   // weights [BN][WP]

  // ---- 1. DMA the patch and the filter bank (lane-linear 16-B chunks)
  if constexpr (U8) {
    static_assert(ES == 2 && !POOL, "uint8 RGB input: bf16 s2d patch, no pool");
    const int iy0 = oy0 * p.S - p.ph, ix0 = ox0 * p.S - p.pw;
    const uint8_t* xb = p.xu8 + (size_t)n * p.Hi * p.Wi * 3;
    for (int q = tid; q < p.PH * p.PW; q += NTH) {
      const int py = q / p.PW, px = q - py * p.PW;
      const int by = iy0 + py, bx = ix0 + px;
      float v[12];
#pragma unroll
      for (int e = 0; e < 12; ++e) v[e] = 0.f;
      if ((unsigned)by < (unsigned)p.H && (unsigned)bx < (unsigned)p.W) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b2 = 0; b2 < 2; ++b2) {
            const int r = 2 * by + a, c = 2 * bx + b2;
            if (r < p.Hi && c < p.Wi) {
              const uint8_t* src = xb + ((size_t)r * p.Wi + c) * 3;
#pragma unroll
              for (int ch = 0; ch < 3; ++ch) v[(a * 2 + b2) * 3 + ch] = ((float)src[ch] - p.mean[ch]) * p.istd[ch];
            }
          }
      }
      bf16x8 lo, hi;
#pragma unroll
      for (int e = 0; e < 8; ++e) lo[e] = f2bf(v[e]);
#pragma unroll
      for (int e = 0; e < 8; ++e) hi[e] = f2bf(e < 4 ? v[8 + e] : 0.f);
      *reinterpret_cast<bf16x8*>(Ps + q * 32) = lo;
      *reinterpret_cast<bf16x8*>(Ps + q * 32 + 16) = hi;
    }
  }
  {
    const int cpr = p.RB >> 4;  // 16-B chunks per patch row
    const int nchunks = U8 ? 0 : p.PH * p.PW * cpr;
    const int iy0 = oy0 * p.S - p.ph, ix0 = ox0 * p.S - p.pw;
    const uint8_t* xb = p.x + (size_t)n * p.H * p.W * p.RB;
    for (int q0 = wave * 64; q0 < nchunks; q0 += NTH) {
      const int q = q0 + lane;
      const int r = q / cpr, c = q - r * cpr;
      const int py = r / p.PW, px = r - py * p.PW;
      const int iy = iy0 + py, ix = ix0 + px;
      const bool ok = q < nchunks && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const void* src = ok ? (const void*)(xb + ((size_t)iy * p.W + ix) * p.RB + c * 16) : (const void*)g_zero16;
      glds16(src, Ps + q0 * 16);  // a short last wave-instruction writes past nchunks: slack is reserved
    }
    const int wchunks = BN * (p.WP >> 4);
    const uint8_t* wb = p.w + (size_t)n0 * p.WP;
    for (int q0 = wave * 64; q0 < wchunks; q0 += NTH) {
      const int q = q0 + lane;
      const void* src = q < wchunks ? (const void*)(wb + (size_t)q * 16) : (const void*)g_zero16;
      glds16(src, Wsm + q0 * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- 2. K loop out of LDS
  const int frow = lane & 15, fq = lane >> 4;
  f32x4 acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // patch row of fragment j's pixel for this lane at tap offset 0
  int prow0[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int pix = (wave * J + j) * 16 + frow, r = pix / TPW, c = pix - r * TPW;
    prow0[j] = (r * p.S) * p.PW + c * p.S;
  }

  FTM_PRIO_HI(p.prio);
  for (int s = 0; s < p.ksteps; ++s) {
    const int kb = s * 4 * KL + fq * KL;  // this lane group's K byte offset
    const int bo = koff_of(p, s, fq);
    if constexpr (ES == 2) {
      bf16x8 a[I], bb[J];
#pragma unroll
      for (int i = 0; i < I; ++i) a[i] = *reinterpret_cast<const bf16x8*>(Wsm + (i * 16 + frow) * p.WP + kb);
#pragma unroll
      for (int j = 0; j < J; ++j) bb[j] = *reinterpret_cast<const bf16x8*>(Ps + prow0[j] * p.RB + bo);
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
    } else {
      i32x8 a[I], bb[J];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const uint8_t* src = Wsm + (i * 16 + frow) * p.WP + kb;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(src), hi = *reinterpret_cast<const u32x4*>(src + 16);
        a[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const uint8_t* src = Ps + prow0[j] * p.RB + bo;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(src), hi = *reinterpret_cast<const u32x4*>(src + 16);
        bb[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], bb[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    }
  }
  FTM_PRIO_LO(p.prio);
  __syncthreads();  // everyone done with the patch: reuse LDS for the output tile

  // ---- 3. epilogue: [dequant] + bias + act -> LDS [256 px][BN] -> 16-B row segments
  uint8_t* Os = smem;
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int cl = i * 16 + fq * 4;
    f32x4 sv = {1.f, 1.f, 1.f, 1.f}, bv = {0.f, 0.f, 0.f, 0.f};
    if (n0 + cl < p.Cout) {
      if constexpr (ES == 1) sv = *reinterpret_cast<const f32x4*>(p.scale + n0 + cl);
      bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int pl = (wave * J + j) * TW + frow;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act<ACT>(acc[i][j][r] * sv[r] + bv[r]);
      if constexpr (POOL) {  // conv positions outside the image must not win the max
        const int oy = oy0 + pl / TPW, ox = ox0 + pl % TPW;
        if ((unsigned)oy >= (unsigned)p.Ho || (unsigned)ox >= (unsigned)p.Wo) v[0] = v[1] = v[2] = v[3] = 0.f;
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
  constexpr int EPO = 16 / OB;
  constexpr int CPR = BN / EPO;
  if constexpr (POOL) {
    for (int q = tid; q < PTH * 8 * CPR; q += NTH) {
      const int pp = q / CPR, cc = q % CPR;
      const int pyl = pp >> 3, pxl = pp & 7;
      const int py = (oy0 + p.ppt) / 2 + pyl, px = (ox0 + p.ppl) / 2 + pxl;
      const int c = n0 + cc * EPO;
      if (py >= p.Hp || px >= p.Wp || c >= p.Cout) continue;
      const uint8_t* src = Os + ((2 * pyl) * TPW + 2 * pxl) * OLD + cc * 16;
      const size_t mo = ((size_t)n * p.Hp + py) * p.Wp + px;
      if constexpr (OUT_FP8)
        *reinterpret_cast<u8x16*>(p.y + mo * p.ldy + p.y_coff + c) = pool3x3_max_u8(src, TPW * OLD, OLD);
      else
        *reinterpret_cast<u16x8*>(p.y + (mo * p.ldy + p.y_coff + c) * 2) = pool3x3_max(src, TPW * OLD, OLD);
    }
    return;
  }
  for (int q = tid; q < THE * TW * CPR; q += NTH) {
    const int pl = q / CPR, cc = q % CPR;
    const int oy = oy0 + pl / TW, ox = ox0 + pl % TW;
    const int c = n0 + cc * EPO;
    if (oy >= p.Ho || ox >= p.Wo || c >= p.Cout) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(Os + pl * OLD + cc * 16);
    const size_t m = ((size_t)n * p.Ho + oy) * p.Wo + ox;
    *reinterpret_cast<u32x4*>(p.y + (m * p.ldy + p.y_coff + c) * OB) = v;
  }
}

template <int ES, int BN, bool OUT_FP8, int WAVES>
void launch_act(const DconvParams& p, int act, size_t lds, hipStream_t s) {
  dim3 grid(p.N * p.tiles_h * p.tiles_w * p.tiles_n), block(WAVES * 64);
  if constexpr ((ES == 2 && !OUT_FP8) || (ES == 1 && OUT_FP8)) {
    if (p.Hp > 0) {  // fused max pool (ReLU stems; fp8 -> fp8 chains)
      if (act != ACT_RELU) throw std::invalid_argument("dconv: fused pool needs a ReLU conv");
      static bool done = false;
      if (!done) {
        hipFuncSetAttribute((const void*)dconv_kernel<ES, BN, ACT_RELU, OUT_FP8, true, WAVES>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        done = true;
      }
      hipLaunchKernelGGL((dconv_kernel<ES, BN, ACT_RELU, OUT_FP8, true, WAVES>), grid, block, lds, s, p);
      return;
    }
  } else {
    if (p.Hp > 0) throw std::invalid_argument("dconv: fused pool needs bf16 -> bf16 or fp8 -> fp8");
  }
  switch (act) {
    case ACT_NONE:
      hipLaunchKernelGGL((dconv_kernel<ES, BN, ACT_NONE, OUT_FP8, false, WAVES>), grid, block, lds, s, p);
      break;
    case ACT_RELU:
      hipLaunchKernelGGL((dconv_kernel<ES, BN, ACT_RELU, OUT_FP8, false, WAVES>), grid, block, lds, s, p);
      break;
    default: throw std::invalid_argument("dconv: activation must be none/relu");
  }
}

template <int BN, bool OUT_FP8, int WAVES>
void launch_u8(const DconvParams& p, int act, size_t lds, hipStream_t s) {
  dim3 grid(p.N * p.tiles_h * p.tiles_w * p.tiles_n), block(WAVES * 64);
  static bool done = false;
  if (!done) {
    for (auto f : {(const void*)dconv_kernel<2, BN, ACT_NONE, OUT_FP8, false, WAVES, true>,
                   (const void*)dconv_kernel<2, BN, ACT_RELU, OUT_FP8, false, WAVES, true>})
      hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done = true;
  }
  if (act == ACT_RELU) hipLaunchKernelGGL((dconv_kernel<2, BN, ACT_RELU, OUT_FP8, false, WAVES, true>), grid, block, lds, s, p);
  else if (act == ACT_NONE) hipLaunchKernelGGL((dconv_kernel<2, BN, ACT_NONE, OUT_FP8, false, WAVES, true>), grid, block, lds, s, p);
  else throw std::invalid_argument("dconv: activation must be none/relu");
}

template <int ES, int BN, bool OUT_FP8, int WAVES>
void set_lds_limit() {
  static bool done = false;
  if (done) return;
  for (auto f : {(const void*)dconv_kernel<ES, BN, ACT_NONE, OUT_FP8, false, WAVES>,
                 (const void*)dconv_kernel<ES, BN, ACT_RELU, OUT_FP8, false, WAVES>})
    hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  done = true;
}

}  // namespace

// patch rows of a tile: pooled tiles are 17 conv columns wide and hold npx = 64 * waves
// fragment pixels (the last fragment row is (npx - 1) / 17)
int patch_rows(int KH, int S, bool pool, int npx) { return (pool ? (npx - 1) / 17 : npx / TW - 1) * S + KH; }

int lds_bytes(int es, int bn, int KH, int KW, int S, int Cin, int wp, bool pool, int npx = TH * TW) {
  const int PH = patch_rows(KH, S, pool, npx), PW = (pool ? TW : TW - 1) * S + KW;
  const int patch = PH * PW * Cin * es;
  const int ob = 2;  // bound by the bf16 output tile
  int need = ((patch + 1023) & ~1023) + bn * wp + 1024;  // + slack for a short last DMA
  const int epi = npx * (bn * ob + 16);
  return need > epi ? need : epi;
}

int dconv_lds_bytes(int es, int bn, int KH, int KW, int S, int Cin, int wp) {
  return lds_bytes(es, bn, KH, KW, S, Cin, wp, false);
}

// x: NHWC (bf16 es=2 / e4m3 es=1); w: host-arranged [Cout_pad][wp] bytes.
void dconv(uintptr_t x, uintptr_t w, uintptr_t scale, uintptr_t bias, uintptr_t y, int es, int N, int H, int W,
           int Cin, int Cout, int KH, int KW, int S, int ph, int pw, int Ho, int Wo, int wp, int ldy, int y_coff,
           int out_fp8, float out_q, int act, int bn, uintptr_t stream, int Hp, int Wp, int ppt, int ppl,
           int waves) {
  const int KL = es == 2 ? 16 : 32;
  if (es != 1 && es != 2) throw std::invalid_argument("dconv: es must be 1 or 2");
  if ((Cin * es) % KL) throw std::invalid_argument("dconv: Cin*es must be a multiple of " + std::to_string(KL));
  if (bn != 32 && bn != 64) throw std::invalid_argument("dconv: bn must be 32 or 64");
  const int kb = KH * KW * Cin * es;
  const int kpad = (kb + 4 * KL - 1) / (4 * KL) * (4 * KL);
  if (wp != kpad + 16) throw std::invalid_argument("dconv: weight pitch must be round_up(K bytes, 4*KL) + 16");
  const int oe = out_fp8 ? 16 : 8;
  if (Cout % oe || ldy % oe || y_coff % oe) throw std::invalid_argument("dconv: Cout/ldy/y_coff alignment");
  if (S != 1 && S != 2) throw std::invalid_argument("dconv: stride must be 1 or 2");
  if (!bias || (es == 1 && !scale)) throw std::invalid_argument("dconv: bias (and fp8 scale) required");
  if (x % 16 || w % 16 || y % 16 || bias % 16 || (scale && scale % 16)) throw std::invalid_argument("dconv: alignment");
  if (waves != 4 && waves != 8) throw std::invalid_argument("dconv: waves must be 4 or 8");
  if (waves == 8 && lds_bytes(es, bn, KH, KW, S, Cin, wp, Hp > 0, 512) > 160 * 1024) waves = 4;  // wide patches
  const int npx = waves * 64;                // fragment pixels per tile
  const int pool_rows = waves == 8 ? 14 : 7;  // pooled tiles: 7 or 14 x 8 pooled pixels
  const int lds = lds_bytes(es, bn, KH, KW, S, Cin, wp, Hp > 0, npx);
  if (lds > 160 * 1024) throw std::invalid_argument("dconv: tile does not fit LDS (" + std::to_string(lds) + " B)");
  DconvParams p{};
  p.x = reinterpret_cast<const uint8_t*>(x);
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = reinterpret_cast<const float*>(scale);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.out_q = out_q;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH; p.KW = KW; p.S = S;
  p.ph = ph; p.pw = pw;
  p.RB = Cin * es;
  p.WP = wp;
  p.ksteps = kpad / (4 * KL);
  if (p.ksteps > 64) throw std::invalid_argument("dconv: more than 64 K-steps");
  p.PH = patch_rows(KH, S, Hp > 0, npx);
  p.PW = (Hp > 0 ? TW : TW - 1) * S + KW;  // pooled tiles are 17 conv columns wide
  p.ldy = ldy; p.y_coff = y_coff;
  p.prio = ftm_mfma_prio();
  p.Hp = Hp; p.Wp = Wp; p.ppt = ppt; p.ppl = ppl;
  for (int st = 0; st < p.ksteps; ++st)
    for (int fq = 0; fq < 4; ++fq) {
      const int kb = st * 4 * KL + fq * KL;
      int tap = kb / p.RB;
      const int cb = kb - tap * p.RB;
      if (tap >= KH * KW) tap = 0;  // K padding: zero weights, any finite patch data
      const int dy = tap / KW, dx = tap - dy * KW;
      p.koff[st * 4 + fq] = (dy * p.PW + dx) * p.RB + cb;
    }
  if (Hp > 0) {  // pooled tiles of 7 x 8 (15 x 17 conv pixels) or 14 x 8 (29 x 17)
    if (ppt < 0 || ppt > 1 || ppl < 0 || ppl > 1) throw std::invalid_argument("dconv: pool padding must be 0/1");
    if ((Hp - 1) * 2 + 3 > Ho + ppt + 1 || (Wp - 1) * 2 + 3 > Wo + ppl + 1)
      throw std::invalid_argument("dconv: pooled shape inconsistent with conv output");
    p.tiles_h = (Hp + pool_rows - 1) / pool_rows;
    p.tiles_w = (Wp + 7) / 8;
  } else {
    p.tiles_h = (Ho + npx / TW - 1) / (npx / TW);
    p.tiles_w = (Wo + TW - 1) / TW;
  }
  p.tiles_n = (Cout + bn - 1) / bn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define FTM_DCONV(ES_, BN_, OF_)                                                   \
  do {                                                                             \
    if (waves == 8) {                                                              \
      set_lds_limit<ES_, BN_, OF_, 8>();                                           \
      launch_act<ES_, BN_, OF_, 8>(p, act, lds, s);                                \
    } else {                                                                       \
      set_lds_limit<ES_, BN_, OF_, 4>();                                           \
      launch_act<ES_, BN_, OF_, 4>(p, act, lds, s);                                \
    }                                                                              \
  } while (0)
  if (es == 2) {
    if (bn == 32) { if (out_fp8) FTM_DCONV(2, 32, true); else FTM_DCONV(2, 32, false); }
    else { if (out_fp8) FTM_DCONV(2, 64, true); else FTM_DCONV(2, 64, false); }
  } else {
    if (bn == 32) { if (out_fp8) FTM_DCONV(1, 32, true); else FTM_DCONV(1, 32, false); }
    else { if (out_fp8) FTM_DCONV(1, 64, true); else FTM_DCONV(1, 64, false); }
  }
#undef FTM_DCONV
  FTM_CHECK_LAUNCH();
}

// The RGB stem straight from the raw uint8 batch (the preprocess kernel fused away): a
// stride-2 conv already rewritten as a stride-1 conv over the 2x2 space-to-depth input
// (s2d_stem_weights: [Cout][KH][KW][16] bf16 rows), the patch built from uint8 pixels with
// the preprocess normalisation.  x: [N, Hi, Wi, 3] uint8; the conv input is [N, ceil(Hi/2),
// ceil(Wi/2), 16].
void dconv_u8s2d(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int Hi, int Wi, int Cout, int KH, int KW,
                 int ph, int pw, int Ho, int Wo, int wp, int ldy, int y_coff, int out_fp8, float out_q, int act, int bn,
                 float m0, float m1, float m2, float s0, float s1, float s2, uintptr_t stream, int waves) {
  const int Cin = 16, es = 2, KL = 16;
  if (bn != 32 && bn != 64) throw std::invalid_argument("dconv_u8s2d: bn must be 32 or 64");
  const int kb = KH * KW * Cin * es;
  const int kpad = (kb + 4 * KL - 1) / (4 * KL) * (4 * KL);
  if (wp != kpad + 16) throw std::invalid_argument("dconv_u8s2d: weight pitch must be round_up(K bytes, 64) + 16");
  const int oe = out_fp8 ? 16 : 8;
  if (Cout % oe || ldy % oe || y_coff % oe) throw std::invalid_argument("dconv_u8s2d: Cout/ldy/y_coff alignment");
  if (!bias || w % 16 || y % 16 || bias % 16) throw std::invalid_argument("dconv_u8s2d: bias / alignment");
  if (waves != 4 && waves != 8) throw std::invalid_argument("dconv_u8s2d: waves must be 4 or 8");
  if (waves == 8 && lds_bytes(es, bn, KH, KW, 1, Cin, wp, false, 512) > 160 * 1024) waves = 4;
  const int npx = waves * 64;
  const int lds = lds_bytes(es, bn, KH, KW, 1, Cin, wp, false, npx);
  if (lds > 160 * 1024) throw std::invalid_argument("dconv_u8s2d: tile does not fit LDS");
  DconvParams p{};
  p.x = nullptr;
  p.xu8 = reinterpret_cast<const uint8_t*>(x);
  p.Hi = Hi; p.Wi = Wi;
  p.mean[0] = m0; p.mean[1] = m1; p.mean[2] = m2;
  p.istd[0] = s0; p.istd[1] = s1; p.istd[2] = s2;
  p.w = reinterpret_cast<const uint8_t*>(w);
  p.scale = nullptr;
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<uint8_t*>(y);
  p.out_q = out_q;
  p.N = N; p.H = (Hi + 1) / 2; p.W = (Wi + 1) / 2; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout;
  p.KH = KH; p.KW = KW; p.S = 1; p.ph = ph; p.pw = pw;
  p.RB = Cin * es;
  p.WP = wp;
  p.ksteps = kpad / (4 * KL);
  if (p.ksteps > 64) throw std::invalid_argument("dconv_u8s2d: more than 64 K-steps");
  p.PH = patch_rows(KH, 1, false, npx);
  p.PW = (TW - 1) + KW;
  p.ldy = ldy; p.y_coff = y_coff;
  p.prio = ftm_mfma_prio();
  for (int st = 0; st < p.ksteps; ++st)
    for (int fq = 0; fq < 4; ++fq) {
      const int kb2 = st * 4 * KL + fq * KL;
      int tap = kb2 / p.RB;
      const int cb = kb2 - tap * p.RB;
      if (tap >= KH * KW) tap = 0;
      const int dy = tap / KW, dx = tap - dy * KW;
      p.koff[st * 4 + fq] = (dy * p.PW + dx) * p.RB + cb;
    }
  p.tiles_h = (Ho + npx / TW - 1) / (npx / TW);
  p.tiles_w = (Wo + TW - 1) / TW;
  p.tiles_n = (Cout + bn - 1) / bn;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define FTM_U8(BN_, OF_)                                              \
  do {                                                                \
    if (waves == 8) launch_u8<BN_, OF_, 8>(p, act, lds, s);            \
    else launch_u8<BN_, OF_, 4>(p, act, lds, s);                       \
  } while (0)
  if (bn == 32) { if (out_fp8) FTM_U8(32, true); else FTM_U8(32, false); }
  else { if (out_fp8) FTM_U8(64, true); else FTM_U8(64, false); }
#undef FTM_U8
  FTM_CHECK_LAUNCH();
}

void register_dconv(pybind11::module_& m) {
  m.def("dconv", &dconv);
  m.def("dconv_u8s2d", &dconv_u8s2d);
  m.def("dconv_lds_bytes", &dconv_lds_bytes);
}
