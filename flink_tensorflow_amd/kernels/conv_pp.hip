// Implicit-GEMM NHWC convolution on the ping-pong MFMA pipeline of gemm_pp.hip (gfx950).
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
// Structure (same as gemm_pp, guide §5 "The 256² 8-phase template"):
// * BM x BN output tile with BM x BN in {256x256, 512x128}, BK = 64, 512 threads = 8 waves
//   as (BM/128) x (BN/64); every wave owns 128 x 64 outputs = 2 x 2 quadrants of 64 x 32
//   (32 v_mfma_f32_16x16x32_bf16 per K-tile, 128 accumulator registers).  The 512x128
//   tile serves 128-channel layers without wasting half of a 256-wide tile.
// * Both operands stream global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into two
//   stages of four half-tiles (X rows of quadrant-row 0/1, W rows of quadrant-column 0/1);
//   each half-tile is consumed inside one phase and restaged for the K-tile two ahead, so
//   three half-tiles stay in flight across every barrier (one counted vmcnt per K-tile).
// * im2col happens in the DMA address: every lane keeps, per source, the byte offset of
//   its rows' receptive-field origin and the packed (ih0, iw0); a host-built K-tile table
//   gives the tile's source, (kh*d, kw*d) and byte delta (no divides in the K loop).  Taps
//   that fall into the zero padding get an offset outside the buffer descriptor's range,
//   and the buffer load returns zeros — no branches, no clamping.
// * Ping-pong: the second wave group (one wave per SIMD) runs one barrier behind, so each
//   SIMD overlaps one wave's MFMA cluster with its partner's ds_reads and DMA issue.
// * XOR-swizzled LDS images (16-B chunk ^ (row & 7)) -> conflict-free ds_read_b128.
// * XCD-aware bijective tile remap.  M / N tails: rows past M read zeros and are not
//   stored; W rows past N clamp out of range.
// * Epilogue: + bias, act -> bf16 tile in LDS -> coalesced 16-B row segments (+ residual,
//   act) -> global (concat channel offset supported).  SPLIT mode writes fp32 partials per
//   K slice (blockIdx.y) and conv_pp_reduce finishes them.
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>
#include <type_traits>

#include "common.h"

namespace {

constexpr int NT = 512;

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

#define CP_FENCE() __builtin_amdgcn_sched_barrier(0)
#define CP_BARRIER()                              \
  do {                                            \
    CP_FENCE();                                   \
    asm volatile("s_barrier" ::: "memory");      \
    CP_FENCE();                                   \
  } while (0)

template <int BM, int BN>
struct Cfg {
  static constexpr int WC = BN / 64;          // wave columns
  static constexpr int WR = BM / 128;         // wave rows
  static_assert(WR * WC == 8, "8 waves");
  static constexpr int XH = BM * 64;          // X half-tile bytes (BM/2 rows x 128 B)
  static constexpr int WH = BN * 64;          // W half-tile bytes
  static constexpr int XL = BM / 128;         // 16-B DMA loads per lane per X half-tile
  static constexpr int WL = BN / 128;         // ... per W half-tile
  static constexpr int STG = 2 * XH + 2 * WH;
  static constexpr int OPITCH = BN * 2 + 16;  // epilogue LDS row pitch
  static constexpr int LDS_MAIN = 2 * STG;
  static constexpr int LDS_EPI = BM * OPITCH;
  static constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static constexpr int INFLIGHT = 2 * WL + XL;  // W_h0 + X_h0 + W_h1 of tile t+2
};

template <int BM, int BN, int ACT, bool HAS_RES, bool SPLIT, bool DUAL>
__global__ __launch_bounds__(NT, 1) void conv_pp_kernel(CPParams p) {
  using C = Cfg<BM, BN>;
  __shared__ __attribute__((aligned(1024))) uint8_t smem[C::LDS];

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave / C::WC;  // wave row
  const int wc = wave % C::WC; // wave column
  const int pp = wave >> 2;    // ping-pong group (one wave per SIMD in each)

  const int nk_all = p.K >> 6;
  int kt0 = 0, nk = nk_all;
  if constexpr (SPLIT) {
    kt0 = blockIdx.y * p.kt_per_split;
    nk = min(p.kt_per_split, nk_all - kt0);
  }

  // ---- DMA roles (see gemm_pp.hip): image rows 8 * (XL * wave + q) + (lane >> 3)
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;
  // (two scalars, not an array: the buffer-resource type is sizeless on the host side)
  const unsigned nimg = (unsigned)p.M / (unsigned)(p.OH * p.OW);
  const __amdgpu_buffer_rsrc_t rx0 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.s[0].x, 0, (int)(nimg * (unsigned)(p.s[0].H * p.s[0].W) * (unsigned)p.s[0].C * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.s[1].x, 0, (int)(nimg * (unsigned)(p.s[1].H * p.s[1].W) * (unsigned)p.s[1].C * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.w, 0, (int)((unsigned)p.N * (unsigned)p.ldw * 2u), 0x00020000);

  // per-lane row state: receptive-field origin byte offset and packed (ih0 << 16 | iw0)
  int pb[DUAL ? 2 : 1][2][C::XL];
  int hw[DUAL ? 2 : 1][2][C::XL];
  const int ohw = p.OH * p.OW;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int q = 0; q < C::XL; ++q) {
      const int r = 8 * (C::XL * wave + q) + drow;  // image row 0 .. BM/2-1
      const int m = m0 + (r >> 6) * 128 + h * 64 + (r & 63);
      const bool live = m < p.M;
      const int n = live ? m / ohw : 0;
      const int rem = live ? m - n * ohw : 0;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
#pragma unroll
      for (int s = 0; s < (DUAL ? 2 : 1); ++s) {
        const CSrc& S = p.s[s];
        const int ih0 = live ? oh * S.sh - S.ph : -16384;
        const int iw0 = ow * S.sw - S.pw;
        pb[s][h][q] = ((n * S.H + ih0) * S.W + iw0) * S.C * 2 + dchunk * 16;
        hw[s][h][q] = (ih0 << 16) | (iw0 & 0xFFFF);
      }
    }
  }
  unsigned offw[2][C::WL];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int q = 0; q < C::WL; ++q) {
      const int r = 8 * (C::WL * wave + q) + drow;  // image row 0 .. BN/2-1
      const unsigned n = n0 + (r >> 5) * 64 + h * 32 + (r & 31);
      offw[h][q] = n < (unsigned)p.N ? (n * p.ldw + dchunk * 8) * 2u : 0x80000000u;
    }
  }

  auto dma_x = [&](int h, int kt, int stage) {
    const int2 e = p.ktab[kt0 + kt];
    const int src = DUAL ? (e.y >> 20) : 0;
    const int dih = (e.y >> 10) & 1023;
    const int diw = e.y & 1023;
    uint8_t* base = smem + stage * C::STG + h * C::XH + C::XL * wave * 8 * 128;
#pragma unroll
    for (int q = 0; q < C::XL; ++q) {
      int pbv, hwv, Hs, Ws;
      if (DUAL && src) {
        pbv = pb[DUAL ? 1 : 0][h][q]; hwv = hw[DUAL ? 1 : 0][h][q]; Hs = p.s[1].H; Ws = p.s[1].W;
      } else {
        pbv = pb[0][h][q]; hwv = hw[0][h][q]; Hs = p.s[0].H; Ws = p.s[0].W;
      }
      const int ih = (hwv >> 16) + dih;
      const int iw = ((hwv << 16) >> 16) + diw;
      const bool ok = (unsigned)ih < (unsigned)Hs && (unsigned)iw < (unsigned)Ws;
      const unsigned off = ok ? (unsigned)(pbv + e.x) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(DUAL && src ? rx1 : rx0,
                                               (__attribute__((address_space(3))) void*)(base + q * 8 * 128), 16,
                                               off, 0, 0, 0);
    }
  };
  auto dma_w = [&](int h, int kt, int stage) {
    uint8_t* base = smem + stage * C::STG + 2 * C::XH + h * C::WH + C::WL * wave * 8 * 128;
    const unsigned soff = (unsigned)(kt0 + kt) * 128u;
#pragma unroll
    for (int q = 0; q < C::WL; ++q) {
      const unsigned o = offw[h][q];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(base + q * 8 * 128), 16,
                                               o, soff, 0, 0);
    }
  };

  // ---- fragment reads (bytes relative to a half-tile image), swizzled by (row & 7)
  const int frow = lane & 15;
  const int fx_row = (g * 64 + frow) * 128;
  const int fw_row = (wc * 32 + frow) * 128;
  const int fc0 = ((0 + (lane >> 4)) ^ (lane & 7)) << 4;
  const int fc1 = ((4 + (lane >> 4)) ^ (lane & 7)) << 4;

  f32x4 acc[2][4][2][2];  // [mh][i][nh][j]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][i][b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fx[2][4];
  bf16x8 fw[2][2][2];

  auto read_x = [&](int stage, int mh) {
    const uint8_t* b = smem + stage * C::STG + mh * C::XH + fx_row;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fx[0][i] = *reinterpret_cast<const bf16x8*>(b + i * 16 * 128 + fc0);
      fx[1][i] = *reinterpret_cast<const bf16x8*>(b + i * 16 * 128 + fc1);
    }
  };
  auto read_w = [&](int stage, int nh) {
    const uint8_t* b = smem + stage * C::STG + 2 * C::XH + nh * C::WH + fw_row;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fw[nh][0][j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * 128 + fc0);
      fw[nh][1][j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * 128 + fc1);
    }
  };
  auto mfma_q = [&](int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh][i][nh][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[nh][ks][j], fx[ks][i], acc[mh][i][nh][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  auto wait_inflight = [&]() {
    if constexpr (C::INFLIGHT == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (C::INFLIGHT == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  // One K-tile (local index t, stage S): P1 -> X_h1 of t+1 (other stage); P2..P4 -> W_h0,
  // X_h0, W_h1 of t+2 (this stage).
  // (stage S is a plain argument: called with literals and inlined, it folds the same as
  // a template constant; a generic lambda here trips host-side template substitution)
  auto ktile = [&](int t, const int S) {
    const bool pre1 = t + 1 < nk;
    const bool pre2 = t + 2 < nk;
    read_w(S, 0);
    CP_FENCE();
    read_x(S, 0);
    if (pre1) dma_x(1, t + 1, S ^ 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    CP_BARRIER();
    mfma_q(0, 0);
    CP_BARRIER();
    read_w(S, 1);
    if (pre2) dma_w(0, t + 2, S);
    CP_BARRIER();
    mfma_q(0, 1);
    CP_BARRIER();
    read_x(S, 1);
    if (pre2) dma_x(0, t + 2, S);
    CP_BARRIER();
    mfma_q(1, 1);
    CP_BARRIER();
    if (pre2) {
      dma_w(1, t + 2, S);
      wait_inflight();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    CP_BARRIER();
    mfma_q(1, 0);
    CP_BARRIER();
  };

  dma_w(0, 0, 0);
  dma_x(0, 0, 0);
  dma_w(1, 0, 0);
  dma_x(1, 0, 0);
  if (nk > 1) {
    dma_w(0, 1, 1);
    dma_x(0, 1, 1);
    dma_w(1, 1, 1);
    wait_inflight();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  CP_BARRIER();
  if (pp == 1) CP_BARRIER();

  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, 0);
    ktile(t + 1, 1);
  }
  if (t < nk) ktile(t, 0);
  if (pp == 0) CP_BARRIER();
  __syncthreads();

  const int fq = lane >> 4;
  if constexpr (SPLIT) {
    float* ys = reinterpret_cast<float*>(p.y) + (size_t)blockIdx.y * p.split_stride;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + g * 128 + mh * 64 + i * 16 + frow;
        if (m >= p.M) continue;
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = n0 + wc * 64 + nh * 32 + j * 16 + fq * 4;
            if (n < p.N) *reinterpret_cast<f32x4*>(ys + (size_t)m * p.N + n) = acc[mh][i][nh][j];
          }
      }
    return;
  } else {
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int nl = wc * 64 + nh * 32 + j * 16 + fq * 4;
        f32x4 bv = {0.f, 0.f, 0.f, 0.f};
        if (p.bias && n0 + nl < p.N) bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + nl);
#pragma unroll
        for (int mh = 0; mh < 2; ++mh)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int ml = g * 128 + mh * 64 + i * 16 + frow;
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc[mh][i][nh][j][r] + bv[r];
              if constexpr (!HAS_RES) v = apply_act<ACT>(v);
              o[r] = f2bf(v);
            }
            *reinterpret_cast<bf16x4*>(smem + ml * C::OPITCH + nl * 2) = o;
          }
      }
    __syncthreads();
    bf16* y = reinterpret_cast<bf16*>(p.y);
    constexpr int SEGS = BN / 8;
#pragma unroll 4
    for (int q = threadIdx.x; q < BM * SEGS; q += NT) {
      const int ml = q / SEGS;
      const int cc = q - ml * SEGS;
      const int m = m0 + ml;
      const int n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + ml * C::OPITCH + cc * 16);
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
}

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
template <int ACT, bool HAS_RES, int BK, bool DUAL = false, bool STAMP = false, int BN_ = 128>
__global__ __launch_bounds__(256, 2) void conv_lite_kernel(CPParams p) {
  // BK = 64: 128-B LDS rows, 2 x 32 KiB stages, 2 MFMA steps per K-tile.
  // BK = 32: 64-B rows, 2 x 16 KiB stages (the igemm's footprint: four workgroups per CU),
  //          1 MFMA step per K-tile; 16-B chunk slot = chunk ^ ((row >> 2) & 3) keeps the
  //          16-lane ds_read_b128 groups on distinct banks.
  constexpr int BM = 128, BN = BN_;
  constexpr int ROWB = BK * 2;             // LDS row bytes
  constexpr int CPR = ROWB / 16;           // 16-B chunks per row
  constexpr int RPI = 1024 / ROWB;         // rows per DMA wave-instruction
  constexpr int QX = BM / RPI / 4;         // DMA instructions per wave for the pixel image
  constexpr int QW = BN / RPI / 4;         // ... for the weight image
  constexpr int QM = QX > QW ? QX : QW;
  constexpr int NI = BN / 32;              // channel fragments per wave (BN / 2 channels)
  static_assert(QW <= 4 && (BN == 128 || BN == 256), "channel tile 128 or 256");
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
  f32x4 acc[NI][4];  // [channel fragment i][pixel fragment j]
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

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
    if (kt + 1 < nk) dma(st ^ 1);
    if constexpr (STAMP) t3 = __builtin_amdgcn_s_memtime();
    const uint8_t* xs = smem + st * STG;
    const uint8_t* ws = xs + XB;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int sl = lite_slot<CPR>(frow, ks * 4 + fq) << 4;
      bf16x8 a[NI], b[4];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(ws + (wn * (BN / 2) + i * 16 + frow) * ROWB + sl);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(xs + (wm * 64 + j * 16 + frow) * ROWB + sl);
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
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
    for (int j = 0; j < 4; ++j) {
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
  for (int q = threadIdx.x; q < BM * SEGS; q += 256) {
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

// conv_lite_ws (tile 4): conv_lite's 128x128 tile and LDS images with the roles split over
// EIGHT waves — waves 0-3 only run the MFMAs (2 x 2, 64 x 64 outputs each), waves 4-7 only
// issue the LDS-DMA (wave 4 + w stages what wave w stages in conv_lite).  In conv_lite each
// wave issues its eight 1 KiB DMA pieces (~50-100 cycles each) and then its 32 MFMAs, so a
// K-tile costs issue + MFMA per wave (in-kernel clocks: profiles/r04_g, r04_q); split, the
// DMA of K-tile t+1 is issued by other waves while the MFMA waves run K-tile t.  One
// barrier per K-tile for all eight waves: the DMA waves wait for their pieces (vmcnt), the
// barrier publishes the stage and retires every MFMA wave's reads of the other one.
// Measured: 7-14 % faster per 3x3 layer alone, neutral next to the second compute lane
// (profiles/r04_u, r04_w, r04_x) — opt-in (EngineConfig.conv_lite_ws, ConvPP tile 4).
template <int ACT, bool HAS_RES>
__global__ __launch_bounds__(512, 4) void conv_lite_ws_kernel(CPParams p) {  // 4 waves / SIMD: 2 workgroups per CU
  constexpr int BK = 64;
  constexpr int BM = 128, BN = 128;
  constexpr int ROWB = BK * 2;
  constexpr int CPR = ROWB / 16;
  constexpr int RPI = 1024 / ROWB;
  constexpr int QX = BM / RPI / 4;
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
  const bool mfma_wave = wave < 4;  // wave-uniform role
  const int role = wave & 3;
  const int nk = p.K / BK;

  if (!mfma_wave) {
    // ---------------- DMA waves
    const int drow = lane / CPR;
    const int dchunk = lite_slot<CPR>(drow, lane % CPR);
    const unsigned nimg = (unsigned)p.M / (unsigned)(p.OH * p.OW);
    const CSrc& S = p.s[0];
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)S.x, 0, (int)(nimg * (unsigned)(S.H * S.W) * (unsigned)S.C * 2u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.w, 0, (int)((unsigned)p.N * (unsigned)p.ldw * 2u), 0x00020000);
    int pb[4], hw[4];
    unsigned offw[4];
    const int ohw = p.OH * p.OW;
#pragma unroll
    for (int q = 0; q < QX; ++q) {
      const int r = RPI * (QX * role + q) + drow;
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
      const unsigned co = n0 + r;
      offw[q] = co < (unsigned)p.N ? (co * p.ldw + dchunk * 8) * 2u : 0x80000000u;
    }
    const int cpt = S.C / BK;
    int cc = 0, kw = 0, kh = 0, kt_dma = 0;
    auto dma = [&](int stage) {
      const unsigned woff = (unsigned)kt_dma * (unsigned)ROWB;
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
      uint8_t* bx = smem + stage * STG + QX * role * RPI * ROWB;
      uint8_t* bw = bx + XB;
#pragma unroll
      for (int q = 0; q < QX; ++q) {
        const int ih = (hw[q] >> 16) + dih;
        const int iw = ((hw[q] << 16) >> 16) + diw;
        const bool ok = (unsigned)ih < (unsigned)S.H && (unsigned)iw < (unsigned)S.W;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(bx + q * 1024), 16,
                                                 ok ? (unsigned)(pb[q] + delta) : 0x80000000u, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(bw + q * 1024), 16,
                                                 offw[q], woff, 0, 0);
      }
    };
    dma(0);
    for (int kt = 0; kt < nk; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kt + 1 < nk) dma((kt & 1) ^ 1);
    }
    __syncthreads();  // the MFMA waves' epilogue tile is written
  } else {
    // ---------------- MFMA waves
    const int wm = role & 1, wn = role >> 1;
    const int frow = lane & 15;
    const int fq = lane >> 4;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();
      const uint8_t* xs = smem + (kt & 1) * STG;
      const uint8_t* ws = xs + XB;
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        const int sl = lite_slot<CPR>(frow, ks * 4 + fq) << 4;
        bf16x8 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ws + (wn * 64 + i * 16 + frow) * ROWB + sl);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(xs + (wm * 64 + j * 16 + frow) * ROWB + sl);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done with the stage images: the epilogue tile reuses them
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cl = wn * 64 + i * 16 + fq * 4;
      f32x4 bv = {0.f, 0.f, 0.f, 0.f};
      if (p.bias && n0 + cl < p.N) bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
  }
  // (both branches pass the same number of barriers: nk + 1, and one more below)
  __syncthreads();
  bf16* y = reinterpret_cast<bf16*>(p.y);
  constexpr int SEGS = BN / 8;
#pragma unroll 4
  for (int q = threadIdx.x; q < BM * SEGS; q += 512) {
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
void launch_lite_ws(const CPParams& p, hipStream_t s) {
  const dim3 grid(p.tiles_m * p.tiles_n), block(512);
  if (p.res) hipLaunchKernelGGL((conv_lite_ws_kernel<ACT, true>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((conv_lite_ws_kernel<ACT, false>), grid, block, 0, s, p);
}

// lite_bk: 64 (tile 2) or 32 (tile 3; tile 5 with BN 256)
template <int ACT, int BK, int BN = 128>
void launch_lite(const CPParams& p, hipStream_t s, bool dual = false) {
  const dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if constexpr (BN == 256) {
    if (dual) {
      if (p.res) hipLaunchKernelGGL((conv_lite_kernel<ACT, true, BK, true, false, BN>), grid, block, 0, s, p);
      else hipLaunchKernelGGL((conv_lite_kernel<ACT, false, BK, true, false, BN>), grid, block, 0, s, p);
    } else {
      if (p.res) hipLaunchKernelGGL((conv_lite_kernel<ACT, true, BK, false, false, BN>), grid, block, 0, s, p);
      else hipLaunchKernelGGL((conv_lite_kernel<ACT, false, BK, false, false, BN>), grid, block, 0, s, p);
    }
    return;
  }
  if constexpr (BK == 64) {
    if (dual) {
      if (p.res) hipLaunchKernelGGL((conv_lite_kernel<ACT, true, BK, true>), grid, block, 0, s, p);
      else hipLaunchKernelGGL((conv_lite_kernel<ACT, false, BK, true>), grid, block, 0, s, p);
      return;
    }
  }
  if constexpr (BK == 64 && ACT == ACT_RELU) {
    if (p.stamp && !p.res) {  // diagnostics only (conv_lite_stamp)
      hipLaunchKernelGGL((conv_lite_kernel<ACT, false, BK, false, true>), grid, block, 0, s, p);
      return;
    }
  }
  if (p.res) hipLaunchKernelGGL((conv_lite_kernel<ACT, true, BK>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((conv_lite_kernel<ACT, false, BK>), grid, block, 0, s, p);
}

template <int ACT, bool HAS_RES>
__global__ __launch_bounds__(256) void conv_pp_reduce_kernel(const float* __restrict__ part, int splits,
                                                             long split_stride, const float* __restrict__ bias,
                                                             const bf16* __restrict__ res, int ldr,
                                                             bf16* __restrict__ y, int ldy, int y_coff, int M,
                                                             int N) {
  const int cpr = N >> 3;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * cpr) return;
  const int m = (int)(idx / cpr);
  const int n = (int)(idx - (long)m * cpr) * 8;
  const float* src = part + (size_t)m * N + n;
  f32x4 a0 = *reinterpret_cast<const f32x4*>(src);
  f32x4 a1 = *reinterpret_cast<const f32x4*>(src + 4);
  for (int s = 1; s < splits; ++s) {
    a0 += *reinterpret_cast<const f32x4*>(src + s * split_stride);
    a1 += *reinterpret_cast<const f32x4*>(src + s * split_stride + 4);
  }
  if (bias) {
    a0 += *reinterpret_cast<const f32x4*>(bias + n);
    a1 += *reinterpret_cast<const f32x4*>(bias + n + 4);
  }
  float v[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
  if constexpr (HAS_RES) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(res + (size_t)m * ldr + n);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += (float)r[e];
  }
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(apply_act<ACT>(v[e]));
  *reinterpret_cast<bf16x8*>(y + (size_t)m * ldy + y_coff + n) = o;
}

template <int BM, int BN, int ACT, bool HAS_RES, bool DUAL>
void launch_cp(const CPParams& p, int splits, float* ws, hipStream_t s) {
  dim3 block(NT);
  if (splits <= 1) {
    hipLaunchKernelGGL((conv_pp_kernel<BM, BN, ACT, HAS_RES, false, DUAL>), dim3(p.tiles_m * p.tiles_n), block, 0,
                       s, p);
    return;
  }
  CPParams q = p;
  q.y = ws;
  hipLaunchKernelGGL((conv_pp_kernel<BM, BN, ACT_NONE, false, true, DUAL>), dim3(p.tiles_m * p.tiles_n, splits),
                     block, 0, s, q);
  const long work = (long)p.M * (p.N >> 3);
  hipLaunchKernelGGL((conv_pp_reduce_kernel<ACT, HAS_RES>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                     ws, splits, p.split_stride, p.bias, p.res, p.ldr, reinterpret_cast<bf16*>(p.y), p.ldy, p.y_coff,
                     p.M, p.N);
}

template <int BM, int BN, int ACT>
void launch_act(const CPParams& p, int splits, float* ws, bool dual, hipStream_t s) {
  if (p.res) {
    if (dual) launch_cp<BM, BN, ACT, true, true>(p, splits, ws, s);
    else launch_cp<BM, BN, ACT, true, false>(p, splits, ws, s);
  } else {
    if (dual) launch_cp<BM, BN, ACT, false, true>(p, splits, ws, s);
    else launch_cp<BM, BN, ACT, false, false>(p, splits, ws, s);
  }
}

template <int BM, int BN>
void launch_tile(const CPParams& p, int splits, float* ws, bool dual, int act, hipStream_t s) {
  switch (act) {
    case ACT_NONE: launch_act<BM, BN, ACT_NONE>(p, splits, ws, dual, s); break;
    case ACT_RELU: launch_act<BM, BN, ACT_RELU>(p, splits, ws, dual, s); break;
    default: throw std::invalid_argument("conv_pp: unsupported activation");
  }
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
      p.nk0 = (int)(K / (tile == 5 ? 32 : 64));  // K-tiles of source 0 in the tile's K-tile depth
    } else if (tile == 2 || tile == 5) {  // conv_lite's second source: pointwise, unpadded, in range
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
  p.stamp = tile == 2 ? g_lite_stamp : nullptr;
  need(tile >= 0 && tile <= 5,
       "tile must be 0 (256x256), 1 (512x128), 2 / 3 (128x128, 4 waves, K-tile 64 / 32), 4 (128x128, DMA / MFMA "
       "waves), 5 (128x256, 4 waves, K-tile 32)");
  need(tile != 4 || ns == 1, "the wave-specialised tile takes one source");
  const bool lite = tile >= 2;
  need(!lite || ((ns == 1 || tile == 2 || tile == 5) && splits <= 1),
       "the 4-wave tiles take no split-K (two sources: tiles 2 and 5)");
  need(tile != 3 || p.s[0].C % 32 == 0, "the 32-deep 4-wave tile needs Cin % 32 == 0");
  const int BM = tile == 1 ? 512 : lite ? 128 : 256, BN = tile == 1 ? 128 : tile == 5 ? 256 : lite ? 128 : 256;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (Cout + BN - 1) / BN;
  const int nk = p.K / 64;
  if (splits < 1) splits = 1;
  if (splits > nk) splits = nk;
  if (splits > 1) {
    p.kt_per_split = (nk + splits - 1) / splits;
    splits = (nk + p.kt_per_split - 1) / p.kt_per_split;
    p.split_stride = (long)p.M * Cout;
    need(ws != 0 && ws % 16 == 0, "split-K needs an aligned workspace");
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* wsp = reinterpret_cast<float*>(ws);
  if (tile == 4) {
    if (act == ACT_RELU) launch_lite_ws<ACT_RELU>(p, s);
    else if (act == ACT_NONE) launch_lite_ws<ACT_NONE>(p, s);
    else throw std::invalid_argument("conv_pp: unsupported activation");
  } else if (tile == 5) {
    if (act == ACT_RELU) launch_lite<ACT_RELU, 32, 256>(p, s, ns == 2);
    else if (act == ACT_NONE) launch_lite<ACT_NONE, 32, 256>(p, s, ns == 2);
    else throw std::invalid_argument("conv_pp: unsupported activation");
  } else if (lite) {
    switch (act * 2 + (tile == 3)) {
      case ACT_NONE * 2: launch_lite<ACT_NONE, 64>(p, s, ns == 2); break;
      case ACT_NONE * 2 + 1: launch_lite<ACT_NONE, 32>(p, s); break;
      case ACT_RELU * 2: launch_lite<ACT_RELU, 64>(p, s, ns == 2); break;
      case ACT_RELU * 2 + 1: launch_lite<ACT_RELU, 32>(p, s); break;
      default: throw std::invalid_argument("conv_pp: unsupported activation");
    }
  } else if (tile == 1) launch_tile<512, 128>(p, splits, wsp, ns == 2, act, s);
  else launch_tile<256, 256>(p, splits, wsp, ns == 2, act, s);
  FTM_CHECK_LAUNCH();
}

void register_conv_pp(pybind11::module_& m) {
  m.def("conv_pp", &conv_pp);
  m.def("conv_lite_stamp", &conv_lite_stamp);
}
