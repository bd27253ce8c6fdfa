// conv_lite: implicit-GEMM NHWC convolution on a 128 x 128 tile of four waves (gfx950).
//
//   y[p, yoff + co] = act( sum_src sum_(kh,kw,ci) x_src[n, oh*s-ph+kh*d, ow*s-pw+kw*d, ci]
//                          * w[co, k_src(kh,kw,ci)] + bias[co] (+ res[p, co]) )
//
// p = (n, oh, ow) is the output pixel (GEMM row), co the output channel (GEMM column) and
// k = (kh, kw, ci) the reduction index (OHWI filter rows are K-contiguous).  Up to two
// sources share one accumulator ("dual": a ResNet block's expand conv plus its strided 1x1
// projection shortcut — the K ranges are concatenated, so the projection never makes a
// round trip through HBM).
//
// * im2col happens in the DMA address: every lane keeps, per source, the byte offset of
//   its rows' receptive-field origin and the packed (ih0, iw0); the K walk (channel chunk,
//   filter column, filter row) advances in scalar registers (no divides in the K loop).
//   Taps that fall into the zero padding get an offset outside the buffer descriptor's
//   range, and the buffer load returns zeros — no branches, no clamping.
// * XOR-swizzled LDS images -> conflict-free ds_read_b128; XCD-aware bijective tile remap.
//
// (This file also held the 256x256 / 512x128 ping-pong conv_pp tiles, the 128x256 and
// 32-deep conv_lite tiles and the 8-wave DMA / MFMA-split tile; all measured slower than
// this tile in the two-lane plans and were removed: profiles/r02_conv_pp, r04_a, r04_ad,
// r04_u, r04_w.)
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>
#include <type_traits>

#include "common.h"

namespace {


struct CSrc {
  const bf16* x;
  int H, W, C;
  int sh, sw, ph, pw;
};

struct CPParams {
  CSrc s[2];
  const int2* ktab;  // per K-tile: {byte delta, src << 20 | dih << 10 | diw}
  const bf16* w;
  const float* bias;
  const bf16* res;
  void* y;
  int M, N, K;
  int OH, OW;
  int KW, dh, dw;  // source 0's filter width and dilation (conv_lite walks K without ktab)
  int ldw, ldy, y_coff, ldr;
  int tiles_m, tiles_n;
  int kt_per_split;
  long split_stride;
  int nk0;  // conv_lite with two sources: K-tiles of source 0 (source 1 follows, pointwise)
  unsigned long long* stamp;  // conv_lite STAMP diagnostics: [64 workgroups][64 K-tiles][5] clocks
};

// ---------------------------------------------------------------------------------------
// conv_lite: the same im2col-in-the-DMA-address loader for a 128x128 tile of FOUR waves
// (2 x 2, 64 x 64 outputs each) on two 32 KiB LDS stages — 64 KiB, so two workgroups (or
// one plus a sibling lane's kernel) share a CU, where conv_pp's 128-160 KiB tiles hold it
// alone.  Both operands stream global -> LDS by buffer_load ... lds (no VGPR staging, no
// ds_write: the register-staged igemm spends ~20 % of its wave cycles stalled on LDS issue,
// profiles/r03_conv); one barrier per K-tile: wait for this stage's DMA, barrier (which
// also retires every wave's reads of the other stage), issue the next K-tile's DMA into
// the other stage, then 2 x 16 MFMAs on this one — the DMA of tile t+1 overlaps the MFMAs
// of tile t.  Epilogue as igemm: + bias -> bf16 LDS tile -> coalesced 16-B row segments
// (+ residual, act).
// ---------------------------------------------------------------------------------------
// 16-B chunk slot of (row, chunk) in a conv_lite LDS image with CPR chunks per row
template <int CPR>
FTM_DEVICE int lite_slot(int row, int chunk) {
  if constexpr (CPR == 8) return chunk ^ (row & 7);
  else return chunk ^ ((row >> 2) & 3);
}

// DUAL: a second, pointwise and unpadded source (the strided projection input of a ResNet
// block's first expand: y = x W_e + x2[::s] W_p in one K loop); its K-tiles follow source
// 0's, the weight rows are [W_e | W_p].
// STAMP (diagnostics, bench/conv_stamp_probe.py): wave 0 of the first 64 workgroups records
// s_memtime before the vmcnt wait, after it, after the barrier, after the DMA issue and after
// the MFMA issue of each of the first 64 K-tiles (lane 0, vector stores).
// BN_ = 256 (tile 5, with BK = 32): a 128 x 256 tile — each wave 64 pixels x 128 channels —
// for Cout >= 256, so one workgroup stages the input tile once for 256 channels where two
// 128-wide tiles stage it twice: 24 KiB per 32-deep K-tile for 128 x 256 outputs, 25 % fewer
// bytes per MAC than the 128x128 / 64-deep tile (the fp8 192-wide tile's gain: r04_ac).
// MODE (diagnostics, bench/conv_layer_probe.py lite:4..6; outputs meaningless): 1 = no
// MFMA (the fragments are folded by one VALU op so the LDS reads stay), 2 = no DMA after
// the first K-tile, 3 = MFMAs only (fragments read once, no DMA or LDS reads in the loop).
// Measured on the stage-3 3x3 (profiles/r06_conv_probe): 68.7 µs whole, 45.0 µs MFMAs only
// (1.32 PF/s: the tile's ceiling at 784 tiles on 512 resident workgroups), 55.4 µs without
// the DMA.  Deeper DMA prefetch (32-deep K-tiles on four stages: 87 µs; 64-deep on three,
// one workgroup per CU: 110 µs) and a two-wave 128x64-per-wave tile (27 % fewer LDS
// fragment bytes per MFMA: 78 µs) were measured slower and removed.
template <int ACT, bool HAS_RES, int BK, bool DUAL = false, bool STAMP = false, int BN_ = 128, int MODE = 0>
__global__ __launch_bounds__(256, 2) void conv_lite_kernel(CPParams p) {
  // BK = 64: 128-B LDS rows, 2 x 32 KiB stages, 2 MFMA steps per K-tile.
  // BK = 32: 64-B rows, 2 x 16 KiB stages (the igemm's footprint: four workgroups per CU),
  //          1 MFMA step per K-tile; 16-B chunk slot = chunk ^ ((row >> 2) & 3) keeps the
  //          16-lane ds_read_b128 groups on distinct banks.
  constexpr int BM = 128, BN = BN_;
  constexpr int NT = 256;                  // threads
  constexpr int ROWB = BK * 2;             // LDS row bytes
  constexpr int CPR = ROWB / 16;           // 16-B chunks per row
  constexpr int RPI = 1024 / ROWB;         // rows per DMA wave-instruction
  constexpr int QX = BM / RPI / 4;         // DMA instructions per wave for the pixel image
  constexpr int QW = BN / RPI / 4;         // ... for the weight image
  constexpr int QM = QX > QW ? QX : QW;
  constexpr int NI = BN / 32;              // channel fragments per wave (BN / 2 channels)
  constexpr int PJ = 4;                    // pixel fragments per wave
  static_assert(QX <= 4 && QW <= 4 && (BN == 128 || BN == 256), "channel tile 128 or 256");
  constexpr int XB = BM * ROWB, WB = BN * ROWB, STG = XB + WB;
  constexpr int OPITCH = BN * 2 + 16;
  constexpr int LDS = 2 * STG > BM * OPITCH ? 2 * STG : BM * OPITCH;
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS];

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1;   // pixel half of the tile
  const int wn = wave >> 1;  // channel half

  // DMA roles: wave w stages image rows RPI * (QX w + q) + lane / CPR of both the X (pixel)
  // and W (channel) images; the lane's 16-B chunk is pre-swizzled on the source
  const int drow = lane / CPR;
  const int dchunk = lite_slot<CPR>(drow, lane % CPR);  // (row mod the swizzle period == drow's)
  const unsigned nimg = (unsigned)p.M / (unsigned)(p.OH * p.OW);
  const CSrc& S = p.s[0];
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)S.x, 0, (int)(nimg * (unsigned)(S.H * S.W) * (unsigned)S.C * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.w, 0, (int)((unsigned)p.N * (unsigned)p.ldw * 2u), 0x00020000);
  // fixed-size (QX <= 4): arrays sized by the template-dependent QX made hipcc's host pass
  // drop the kernel by SFINAE (an undefined device stub at load time)
  int pb[4], hw[4], pb1[4];
  unsigned offw[4];
  const CSrc& S1 = p.s[1];
  __amdgpu_buffer_rsrc_t rx1 = rx;
  if constexpr (DUAL)
    rx1 = __builtin_amdgcn_make_buffer_rsrc((void*)S1.x, 0, (int)(nimg * (unsigned)(S1.H * S1.W) * (unsigned)S1.C * 2u),
                                            0x00020000);
  const int ohw = p.OH * p.OW;
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    if (q < QW) {
      const unsigned co = n0 + RPI * (QW * wave + q) + drow;
      offw[q] = co < (unsigned)p.N ? (co * p.ldw + dchunk * 8) * 2u : 0x80000000u;
    }
    if (q >= QX) continue;
    const int r = RPI * (QX * wave + q) + drow;
    const int m = m0 + r;
    const bool live = m < p.M;
    const int n = live ? m / ohw : 0;
    const int rem = live ? m - n * ohw : 0;
    const int oh = rem / p.OW;
    const int ow = rem - oh * p.OW;
    const int ih0 = live ? oh * S.sh - S.ph : -16384;
    const int iw0 = ow * S.sw - S.pw;
    pb[q] = ((n * S.H + ih0) * S.W + iw0) * S.C * 2 + dchunk * 16;
    hw[q] = (ih0 << 16) | (iw0 & 0xFFFF);
    if constexpr (DUAL) pb1[q] = live ? ((n * S1.H + oh * S1.sh) * S1.W + ow * S1.sw) * S1.C * 2 + dchunk * 16 : -1;
  }
  // The K walk (channel chunk, filter column, filter row) advances incrementally in scalar
  // registers: no table read inside the loop (a ktab load there is a vector load — the
  // LDS-DMA in the loop defeats the scalar-load analysis — and stalled every K-tile).
  const int cpt = S.C / BK;  // K-tiles per filter tap
  int cc = 0, kw = 0, kh = 0, kt_dma = 0;
  auto dma = [&](int stage) {
    const unsigned woff = (unsigned)kt_dma * (unsigned)ROWB;
    if constexpr (DUAL) {
      if (kt_dma >= p.nk0) {  // source 1 (uniform branch: kt_dma is wave-uniform)
        const int delta1 = (kt_dma - p.nk0) * BK * 2;
        ++kt_dma;
        uint8_t* bx = smem + stage * STG + QX * wave * RPI * ROWB;
        uint8_t* bw = smem + stage * STG + XB + QW * wave * RPI * ROWB;
#pragma unroll
        for (int q = 0; q < QM; ++q) {
          if (q < QX)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rx1, (__attribute__((address_space(3))) void*)(bx + q * 1024), 16,
                                                     pb1[q] >= 0 ? (unsigned)(pb1[q] + delta1) : 0x80000000u, 0, 0, 0);
          if (q < QW)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(bw + q * 1024), 16,
                                                     offw[q], woff, 0, 0);
        }
        return;
      }
    }
    const int dih = kh * p.dh, diw = kw * p.dw;
    const int delta = ((dih * S.W + diw) * S.C + cc * BK) * 2;
    ++kt_dma;
    if (++cc == cpt) {
      cc = 0;
      if (++kw == p.KW) {
        kw = 0;
        ++kh;
      }
    }
    uint8_t* bx = smem + stage * STG + QX * wave * RPI * ROWB;
    uint8_t* bw = smem + stage * STG + XB + QW * wave * RPI * ROWB;
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      if (q < QX) {
        const int ih = (hw[q] >> 16) + dih;
        const int iw = ((hw[q] << 16) >> 16) + diw;
        const bool ok = (unsigned)ih < (unsigned)S.H && (unsigned)iw < (unsigned)S.W;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(bx + q * 1024), 16,
                                                 ok ? (unsigned)(pb[q] + delta) : 0x80000000u, 0, 0, 0);
      }
      if (q < QW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(bw + q * 1024), 16,
                                                 offw[q], woff, 0, 0);
    }
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  f32x4 acc[NI][PJ];  // [channel fragment i][pixel fragment j]
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < PJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  unsigned long long* sp = nullptr;
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  if constexpr (STAMP) {
    if (threadIdx.x == 0 && blockIdx.x < 64) sp = p.stamp + (size_t)blockIdx.x * 64 * 5;
  }
  // (address arithmetic moved out of the DMA phase into the MFMA phase measured slower:
  // the issue phase shrank 580 -> 392 clocks, the MFMA phase grew 800 -> 1128, profiles/r04_h)
  dma(0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if constexpr (STAMP) t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (STAMP) t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if constexpr (STAMP) t2 = __builtin_amdgcn_s_memtime();
    if (MODE < 2 && kt + 1 < nk) dma(st ^ 1);
    if constexpr (STAMP) t3 = __builtin_amdgcn_s_memtime();
    const uint8_t* xs = smem + st * STG;
    const uint8_t* ws = xs + XB;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int sl = lite_slot<CPR>(frow, ks * 4 + fq) << 4;
      bf16x8 a[NI], b[PJ];
      if (MODE < 3 || kt == 0) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(ws + (wn * (BN / 2) + i * 16 + frow) * ROWB + sl);
#pragma unroll
        for (int j = 0; j < PJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(xs + (wm * 64 + j * 16 + frow) * ROWB + sl);
      }
      if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < PJ; ++j) acc[i][j][0] += (float)a[i][0] * (float)b[j][1];
      } else {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < PJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
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
  __syncthreads();  // every wave is done with the stage images: the epilogue tile reuses them

#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int cl = wn * (BN / 2) + i * 16 + fq * 4;
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (p.bias && n0 + cl < p.N) bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const int pl = wm * 64 + j * 16 + frow;
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r] + bv[r];
        if constexpr (!HAS_RES) v = apply_act<ACT>(v);
        o[r] = f2bf(v);
      }
      *reinterpret_cast<bf16x4*>(smem + pl * OPITCH + cl * 2) = o;
    }
  }
  __syncthreads();
  bf16* y = reinterpret_cast<bf16*>(p.y);
  constexpr int SEGS = BN / 8;
#pragma unroll 4
  for (int q = threadIdx.x; q < BM * SEGS; q += NT) {
    const int ml = q / SEGS;
    const int ccol = q - ml * SEGS;
    const int m = m0 + ml;
    const int n = n0 + ccol * 8;
    if (m >= p.M || n >= p.N) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(smem + ml * OPITCH + ccol * 16);
    if constexpr (HAS_RES) {
      bf16x8 o = __builtin_bit_cast(bf16x8, v);
      const bf16x8 r = *reinterpret_cast<const bf16x8*>(p.res + (size_t)m * p.ldr + n);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(apply_act<ACT>((float)o[e] + (float)r[e]));
      v = __builtin_bit_cast(u32x4, o);
    }
    *reinterpret_cast<u32x4*>(y + (size_t)m * p.ldy + p.y_coff + n) = v;
  }
}

template <int ACT>
void launch_lite(const CPParams& p, hipStream_t s, bool dual, int tile) {
  const dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if (dual) {
    if (p.res) hipLaunchKernelGGL((conv_lite_kernel<ACT, true, 64, true>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((conv_lite_kernel<ACT, false, 64, true>), grid, block, 0, s, p);
    return;
  }
  if constexpr (ACT == ACT_RELU) {
    if (p.stamp && !p.res) {  // diagnostics only (conv_lite_stamp)
      hipLaunchKernelGGL((conv_lite_kernel<ACT, false, 64, false, true>), grid, block, 0, s, p);
      return;
    }
  }
  if (tile >= 4 && tile <= 6 && !p.res) {  // diagnostics (outputs meaningless)
    if (tile == 4) hipLaunchKernelGGL((conv_lite_kernel<ACT, false, 64, false, false, 128, 1>), grid, block, 0, s, p);
    if (tile == 5) hipLaunchKernelGGL((conv_lite_kernel<ACT, false, 64, false, false, 128, 2>), grid, block, 0, s, p);
    if (tile == 6) hipLaunchKernelGGL((conv_lite_kernel<ACT, false, 64, false, false, 128, 3>), grid, block, 0, s, p);
    return;
  }
  if (p.res) hipLaunchKernelGGL((conv_lite_kernel<ACT, true, 64>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((conv_lite_kernel<ACT, false, 64>), grid, block, 0, s, p);
}

void need(bool ok, const char* what) {
  if (!ok) throw std::invalid_argument(std::string("conv_pp: ") + what);
}

}  // namespace

// srcs: one or two (x, N, H, W, C, KH, KW, sh, sw, ph, pw, dh, dw) sources sharing the
// output grid (N, OH, OW); w [Cout, K] bf16 with K = sum KH*KW*C in (src, kh, kw, c) order;
// ktab: int32 [K/64, 2] built by the host (conv_pp_ktab); bias fp32 [Cout] or 0;
// res bf16 [N*OH*OW, ldr] or 0; y bf16 [N*OH*OW, ldy] at channel offset y_coff.
// conv_lite STAMP diagnostics target (0 = off): set by conv_lite_stamp, read by conv_pp
unsigned long long* g_lite_stamp = nullptr;

void conv_lite_stamp(uintptr_t buf) { g_lite_stamp = reinterpret_cast<unsigned long long*>(buf); }

void conv_pp(pybind11::list srcs, uintptr_t ktab, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int N,
             int OH, int OW, int Cout, int ldy, int y_coff, int ldr, int act, int tile, int splits, uintptr_t ws,
             uintptr_t stream) {
  const int ns = (int)pybind11::len(srcs);
  need(ns == 1 || ns == 2, "one or two sources");
  CPParams p{};
  long K = 0;
  for (int i = 0; i < ns; ++i) {
    pybind11::tuple t = srcs[i].cast<pybind11::tuple>();
    need(t.size() == 13, "source tuple (x, N, H, W, C, KH, KW, sh, sw, ph, pw, dh, dw)");
    CSrc& S = p.s[i];
    S.x = reinterpret_cast<const bf16*>(t[0].cast<uintptr_t>());
    const int n = t[1].cast<int>();
    S.H = t[2].cast<int>(); S.W = t[3].cast<int>(); S.C = t[4].cast<int>();
    const int KH = t[5].cast<int>(), KW = t[6].cast<int>();
    S.sh = t[7].cast<int>(); S.sw = t[8].cast<int>(); S.ph = t[9].cast<int>(); S.pw = t[10].cast<int>();
    const int dh = t[11].cast<int>(), dw = t[12].cast<int>();
    need(n == N, "source batch != output batch");
    need(S.C % 64 == 0, "input channels must be a multiple of 64");
    need(reinterpret_cast<uintptr_t>(S.x) % 16 == 0, "x alignment");
    need((long)N * S.H * S.W * S.C * 2 < (1L << 31), "input larger than 2 GiB");
    need(S.H < 16384 && S.W < 16384 && S.ph < 1024 && S.pw < 1024, "spatial size");
    need((KH - 1) * dh < 1024 && (KW - 1) * dw < 1024, "receptive field");
    K += (long)KH * KW * S.C;
    if (i == 0) {
      p.KW = KW;
      p.dh = dh;
      p.dw = dw;
      p.nk0 = (int)(K / 64);  // K-tiles of source 0
    } else {  // conv_lite's second source: pointwise, unpadded, in range
      need(KH == 1 && KW == 1 && S.ph == 0 && S.pw == 0, "the 4-wave tile's second source must be 1x1 unpadded");
      need((OH - 1) * S.sh < S.H && (OW - 1) * S.sw < S.W, "second source smaller than the output grid");
    }
  }
  for (int i = ns; i < 2; ++i) p.s[i] = p.s[0];
  need(Cout % 8 == 0 && ldy % 8 == 0 && y_coff % 8 == 0, "Cout / ldy / y_coff must be multiples of 8");
  need(!res || ldr % 8 == 0, "ldr alignment");
  need(w % 16 == 0 && y % 16 == 0 && (!bias || bias % 16 == 0) && (!res || res % 16 == 0), "alignment");
  need((long)Cout * K * 2 < (1L << 31), "weights larger than 2 GiB");
  p.ktab = reinterpret_cast<const int2*>(ktab);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const bf16*>(res);
  p.y = reinterpret_cast<void*>(y);
  p.M = N * OH * OW;
  p.N = Cout;
  p.K = (int)K;
  p.OH = OH; p.OW = OW;
  p.ldw = (int)K; p.ldy = ldy; p.y_coff = y_coff; p.ldr = ldr;
  p.stamp = g_lite_stamp;
  need(tile == 2 || (tile >= 4 && tile <= 6 && ns == 1),
       "tile must be 2 (conv_lite: 4 waves, K-tile 64, 2 stages); 4..6 are diagnostics");
  need(splits <= 1, "conv_lite takes no split-K");
  (void)ws;
  p.tiles_m = (p.M + 127) / 128;
  p.tiles_n = (Cout + 127) / 128;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (act == ACT_RELU) launch_lite<ACT_RELU>(p, s, ns == 2, tile);
  else if (act == ACT_NONE) launch_lite<ACT_NONE>(p, s, ns == 2, tile);
  else throw std::invalid_argument("conv_pp: unsupported activation");
  FTM_CHECK_LAUNCH();
}

void register_conv_pp(pybind11::module_& m) {
  m.def("conv_pp", &conv_pp);
  m.def("conv_lite_stamp", &conv_lite_stamp);
}
