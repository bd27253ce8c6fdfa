// Fused ResNet bottleneck boundary in the 64/256-channel stage (ResNet-50 stage 1):
//
//   y3  = relu(x2 . W3^T + b3 + r)        1x1 expand 64 -> 256 with residual (block k)
//   y1  = relu(y3 . W1^T + b1)            1x1 reduce 256 -> CN              (block k + 1)
//
// CN = 64 inside stage 1, CN = 128 where stage 1 hands over to stage 2 (ResNet v1.5 keeps
// stage 2's first 1x1 at stride 1).  The first block's expand conv, whose shortcut is a
// stride-1 projection of the block input, runs as the dual variant: K = 64 + 64 over
// [x2 | x] (the projection never reaches HBM) and no residual read.  Unfused, the 256-channel y3 (411 MB at micro-batch
// 256 x 56 x 56) is written by one kernel and read back whole by the next; here each tile
// of y3 is produced into LDS, stored once (it is still the next block's residual) and
// consumed from LDS by the reduce GEMM.  Persistent: one workgroup per CU keeps BOTH
// weight matrices resident in LDS and streams pixel tiles (TP = 128 for CN 64, 64 for
// CN 128):
//
//   LDS   W3 [256][64] 32 KB | W1 [CN][256] 32/64 KB | X tile (x2, then the y1 staging
//         tile) 16 KB | Y tile [TP][256] 64/32 KB  = 144 KB; 16-B chunks XOR-swizzled per
//         row so every ds_read_b128 fragment read is bank-conflict free
//   phase 1  8 waves x (32 channels x TP pixels), K = 64; acc + b3 -> bf16 into Y
//   pass     coalesced 16-B chunks: Y + r (16-B residual loads) -> relu -> y3 global store,
//            and back into Y
//   phase 2  8 waves over (TP pixels x CN channels), K = 256; + b1, relu -> X region ->
//            coalesced 16-B y1 stores
//   the next tile's x2 and residual rows are loaded into registers during phase 2.
#include <pybind11/pybind11.h>

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "common.h"

namespace {

constexpr int CX = 64;    // channels of each GEMM-1 source (x2, and the shortcut input xs)
constexpr int CO = 256;   // y3 channels
constexpr int NT = 512;   // threads (8 waves)

// 16-B chunk index in a row-major LDS tile, XOR-swizzled per row so 16 consecutive rows
// read at the same logical chunk land on distinct banks
template <int CPR>
FTM_DEVICE int swz(int row, int c) {
  if constexpr (CPR == 8) return row * 8 + (c ^ ((row >> 1) & 7));
  else return row * CPR + (c ^ (row & 15));
}

// TP pixels per tile, CN channels of the reduce output y1 (64 within stage 1, 128 for the
// stage-2 entry block).  DUAL: stage 1's first block, whose shortcut is a stride-1 1x1
// projection of the block input xs instead of an identity residual — GEMM 1 runs over
// K = 64 + 64 ([x2 | xs] . [W3 | Wsc]^T, bias summed) and there is no residual read.
template <int TP, int CN, bool DUAL>
__global__ __launch_bounds__(NT, 1) void bottleneck_tail_kernel(const bf16* __restrict__ x2, const bf16* __restrict__ xs,
                                                                const bf16* __restrict__ res,
                                                                const bf16* __restrict__ w3, const float* __restrict__ b3,
                                                                const bf16* __restrict__ w1, const float* __restrict__ b1,
                                                                bf16* __restrict__ y3, bf16* __restrict__ y1, int M,
                                                                int dec_h, int dec_w) {
  constexpr int CM = DUAL ? 2 * CX : CX;  // GEMM-1 depth
  constexpr int W3_BYTES = CO * CM * 2;
  constexpr int W1_BYTES = CN * CO * 2;
  constexpr int X_BYTES = TP * (CN > CM ? CN : CM) * 2;  // x2 tile, then the y1 staging tile
  constexpr int XCH = TP * CM / 8, OCH = TP * CN / 8, YCH = TP * CO / 8;
  constexpr int PF = TP / 16;        // 16-pixel fragments per tile
  constexpr int WPG = 8 / PF;        // phase-2 waves per pixel fragment
  constexpr int NF2 = CN / WPG / 16; // phase-2 16-channel fragments per wave
  static_assert(PF * WPG == 8 && NF2 >= 1 && XCH % NT == 0 && OCH % NT == 0 && YCH % NT == 0, "tile shape");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  u32x4* W3s = reinterpret_cast<u32x4*>(smem);
  u32x4* W1s = reinterpret_cast<u32x4*>(smem + W3_BYTES);
  u32x4* Xs = reinterpret_cast<u32x4*>(smem + W3_BYTES + W1_BYTES);
  u32x4* Ys = reinterpret_cast<u32x4*>(smem + W3_BYTES + W1_BYTES + X_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int prow = lane & 15, kg = lane >> 4;
  const int ntiles = (M + TP - 1) / TP;
  if ((int)blockIdx.x >= ntiles) return;  // block-uniform, before any barrier

  // ---- resident weights: w3 [256][CM], w1 [CN][256] (1x1 OHWI = row-major [co][ci])
  constexpr int XC = CM / 8;  // 16-B chunks per X / W3 row
  for (int q = tid; q < CO * CM / 8; q += NT) W3s[swz<XC>(q / XC, q % XC)] = reinterpret_cast<const u32x4*>(w3)[q];
  for (int q = tid; q < CN * CO / 8; q += NT) W1s[swz<32>(q >> 5, q & 31)] = reinterpret_cast<const u32x4*>(w1)[q];

  constexpr int XIT = XCH / NT;
  u32x4 xr[XIT];
  auto load_x = [&](int t) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int q = tid + it * NT;
      const int px = t * TP + q / XC, c = q % XC;
      const bf16* srcp = (!DUAL || c < 8) ? x2 : xs;
      xr[it] = px < M ? reinterpret_cast<const u32x4*>(srcp + (size_t)px * CX)[c & 7] : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int q = tid + it * NT;
      Xs[swz<XC>(q / XC, q % XC)] = xr[it];
    }
  };

  // residual rows of a tile, 16-B chunks in the pass's thread order; loaded one tile ahead
  // (during the previous tile's phase 2) so the pass never waits on HBM
  constexpr int YIT = YCH / NT;
  static_assert(NT / (CO / 8) == 16, "pass: 16 pixels per iteration");
  u32x4 rv[YIT];
  auto load_r = [&](int tt) {
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int q = tid + it * NT;
      const int px = tt * TP + (q >> 5);
      rv[it] = (!DUAL && px < M) ? reinterpret_cast<const u32x4*>(res + (size_t)px * CO)[q & 31]
                                 : u32x4{0u, 0u, 0u, 0u};
    }
  };

  int t = blockIdx.x;
  load_r(t);
  load_x(t);
  store_x();
  __syncthreads();
  while (true) {
    const int p0 = t * TP;
    // ---- phase 1: y3 tile = x2 tile . W3^T  (wave: channels 32*wave .. +32, all TP px)
    f32x4 acc[2][PF];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < PF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < CM / 32; ++ks) {
      const int c = ks * 4 + kg;
      bf16x8 a[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = __builtin_bit_cast(bf16x8, W3s[swz<XC>(wave * 32 + i * 16 + prow, c)]);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, Xs[swz<XC>(j * 16 + prow, c)]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
      }
    }
    // acc[i][j][r] = channel 32*wave + 16i + 4kg + r of pixel 16j + prow: + b3 -> bf16 into Y
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = wave * 32 + i * 16 + kg * 4;
      const f32x4 bv = *reinterpret_cast<const f32x4*>(b3 + co);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bv[r]);
        const int px = j * 16 + prow;
        bf16* chunk = reinterpret_cast<bf16*>(Ys + swz<32>(px, co >> 3));
        *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;  // 8-byte half of the chunk
      }
    }
    __syncthreads();
    // ---- pass: + residual, relu -> y3 (global) and back into Y (coalesced 16-B chunks)
    {
      // decimated y3: (n, h, w) of this thread's first pass pixel, advanced by 16 pixels per
      // iteration (one divide pair per tile, not per store)
      int dn = 0, dh = 0, dw = 0;
      if (dec_w) {
        const int o0 = p0 + (tid >> 5);
        dw = o0 % dec_w;
        const int tt = o0 / dec_w;
        dh = tt % dec_h;
        dn = tt / dec_h;
      }
#pragma unroll
      for (int it = 0; it < YIT; ++it) {
        const int q = tid + it * NT;
        const int pl = q >> 5, c = q & 31;
        const int si = swz<32>(pl, c);
        bf16x8 v = __builtin_bit_cast(bf16x8, Ys[si]);
        const bf16x8 r = __builtin_bit_cast(bf16x8, rv[it]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf((float)v[e] + (float)r[e], 0.f));
        Ys[si] = __builtin_bit_cast(u32x4, v);
        int o = p0 + pl;
        bool st = o < M;
        if (dec_w) {  // decimated y3: only the even (h, w) pixels, compact [N, H/2, W/2, 256]
          if (it) {
            dw += 16;
            while (dw >= dec_w) {
              dw -= dec_w;
              if (++dh == dec_h) { dh = 0; ++dn; }
            }
          }
          st = st && !((dh | dw) & 1);
          o = (dn * (dec_h >> 1) + (dh >> 1)) * (dec_w >> 1) + (dw >> 1);
        }
        if (st) reinterpret_cast<u32x4*>(y3 + (size_t)o * CO)[c] = __builtin_bit_cast(u32x4, v);
      }
    }
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    if (more) {  // next tile's x2 and residual in flight during phase 2
      load_x(tn);
      if constexpr (!DUAL) load_r(tn);
    }
    __syncthreads();
    // ---- phase 2: y1 tile = relu(Y . W1^T + b1)  (wave: one 16-pixel fragment, NF2 x 16 channels)
    const int pf = wave / WPG, cbase = (wave % WPG) * NF2 * 16;
    f32x4 acc2[NF2];
#pragma unroll
    for (int i = 0; i < NF2; ++i) acc2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < CO / 32; ++ks) {
      const int c = ks * 4 + kg;
      const bf16x8 b = __builtin_bit_cast(bf16x8, Ys[swz<32>(pf * 16 + prow, c)]);
#pragma unroll
      for (int i = 0; i < NF2; ++i) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, W1s[swz<32>(cbase + i * 16 + prow, c)]);
        acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc2[i], 0, 0, 0);
      }
    }
    // stage y1 in the X region: acc2[i][r] = channel cbase + 16i + 4kg + r of pixel 16*pf + prow
#pragma unroll
    for (int i = 0; i < NF2; ++i) {
      const int co = cbase + i * 16 + kg * 4;
      const f32x4 bv = *reinterpret_cast<const f32x4*>(b1 + co);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc2[i][r] + bv[r], 0.f));
      bf16* chunk = reinterpret_cast<bf16*>(Xs + swz<CN / 8>(pf * 16 + prow, co >> 3));
      *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < OCH / NT; ++it) {
      const int q = tid + it * NT;
      const int pl = q / (CN / 8), c = q % (CN / 8);
      if (p0 + pl < M) reinterpret_cast<u32x4*>(y1 + (size_t)(p0 + pl) * CN)[c] = Xs[swz<CN / 8>(pl, c)];
    }
    if (!more) break;
    __syncthreads();  // y1 staging read before the next tile's x2 overwrites it
    store_x();
    __syncthreads();
    t = tn;
  }
}

template <int TP, int CN, bool DUAL>
void launch_tail(const bf16* x2, const bf16* xs, const bf16* res, const bf16* w3, const float* b3, const bf16* w1,
                 const float* b1, bf16* y3, bf16* y1, int M, int num_cu, hipStream_t stream, int dec_h, int dec_w) {
  constexpr int CM = DUAL ? 2 * CX : CX;
  const int tiles = (M + TP - 1) / TP;
  const int grid = tiles < num_cu ? tiles : num_cu;
  const size_t lds = CO * CM * 2 + CN * CO * 2 + TP * (CN > CM ? CN : CM) * 2 + TP * CO * 2;
  static_assert(CO * CM * 2 + CN * CO * 2 + TP * (CN > CM ? CN : CM) * 2 + TP * CO * 2 <= 160 * 1024, "LDS");
  hipFuncSetAttribute((const void*)bottleneck_tail_kernel<TP, CN, DUAL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      lds);
  hipLaunchKernelGGL((bottleneck_tail_kernel<TP, CN, DUAL>), dim3(grid), dim3(NT), lds, stream, x2, xs, res, w3, b3, w1,
                     b1, y3, y1, M, dec_h, dec_w);
}


// ------------------------------------------------------------------------------------------
// The block's 3x3 conv fused in front of the tail (bottleneck3): per tile of 2 image rows x
// 28 columns (56 pixels in 64 MFMA slots: slot s = 32 i + j, j >= 28 dead),
//
//   x2  = relu(conv3x3(y1, W2) + b2)      3x3 64 -> 64 from a 4 x 34-pixel y1 patch in LDS
//   y3  = relu([x2 | xs] . W3^T + b3 [+ r])  and  y1' = relu(y3 . W1^T + b1)   (the tail)
//
// so x2 (103 MB per 256-image batch, written by the 3x3 and read back by the tail) never
// reaches HBM, and the 3x3's MFMA / LDS work overlaps the tail's HBM streams inside one
// persistent kernel instead of running as its own latency-bound launch.  LDS: the 3x3 bank
// W2 [64][576] (73.7 KB, resident) | y1 patch 17 KB | X (x2 [| xs], then the y1' staging)
// | Y [64][256] 32 KB.  The 1x1 banks live in registers: W3 rows of the wave's 32 phase-1
// channels (16 / 32 VGPRs) and W1 rows of its 16 phase-2 channels (32 VGPRs).
constexpr int F_TCV = 28;                 // valid columns per tile
constexpr int F_TP = 64;                  // MFMA slots per tile (2 rows x 32)
constexpr int F_PC = 34;                  // patch columns (32 slots + 2 halo)
constexpr int F_PCH = 4 * F_PC * 8;       // 16-B patch chunks (4 rows x 34 px x 8)
constexpr int F_PIT = (F_PCH + NT - 1) / NT;
constexpr int F_WCH = 64 * 72;            // W2 chunks: 72 per output channel

FTM_DEVICE int f_wchunk(int co, int k) { return co * 72 + (k ^ ((co >> 1) & 7)); }  // XOR stays in its group of 8
FTM_DEVICE int f_pchunk(int pix, int c) { return pix * 8 + (c ^ ((pix >> 1) & 7)); }

template <int CN, bool DUAL>
__global__ __launch_bounds__(NT, 1) void bottleneck3_kernel(const bf16* __restrict__ y1in, const bf16* __restrict__ xs,
                                                            const bf16* __restrict__ res,
                                                            const bf16* __restrict__ w2, const float* __restrict__ b2,
                                                            const bf16* __restrict__ w3, const float* __restrict__ b3,
                                                            const bf16* __restrict__ w1, const float* __restrict__ b1,
                                                            bf16* __restrict__ y3, bf16* __restrict__ y1out, int N, int H,
                                                            int W, int dec) {
  constexpr int CM = DUAL ? 2 * CX : CX;  // phase-1 depth
  constexpr int XC = CM / 8;
  constexpr int XW = CN > CM ? CN : CM;   // X row width
  constexpr int KS1 = CM / 32;
  constexpr int P2F = CN == 64 ? 2 : 4;   // phase-2 pixel fragments per wave
  static_assert(CN == 64 || (CN == 128 && !DUAL), "variants");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  u32x4* W2s = reinterpret_cast<u32x4*>(smem);
  u32x4* Ps = reinterpret_cast<u32x4*>(smem + F_WCH * 16);
  u32x4* Xs = reinterpret_cast<u32x4*>(smem + F_WCH * 16 + F_PCH * 16);
  u32x4* Ys = reinterpret_cast<u32x4*>(smem + F_WCH * 16 + F_PCH * 16 + F_TP * XW * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int prow = lane & 15, kg = lane >> 4;
  const int tiles_x = (W + F_TCV - 1) / F_TCV, tiles_y = (H + 1) / 2;
  const int ntiles = N * tiles_y * tiles_x;
  if ((int)blockIdx.x >= ntiles) return;  // block-uniform, before any barrier

  for (int q = tid; q < F_WCH; q += NT) W2s[f_wchunk(q / 72, q % 72)] = reinterpret_cast<const u32x4*>(w2)[q];
  bf16x8 a3[KS1][2], a1[8];
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      a3[ks][i] = *reinterpret_cast<const bf16x8*>(w3 + (size_t)(wave * 32 + i * 16 + prow) * CM + (ks * 4 + kg) * 8);
  const int cf2 = CN == 64 ? (wave & 3) : wave, pf2 = CN == 64 ? (wave >> 2) * 2 : 0;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    a1[ks] = *reinterpret_cast<const bf16x8*>(w1 + (size_t)(cf2 * 16 + prow) * CO + (ks * 4 + kg) * 8);

  // tile t -> image n, first row y0, first column x0; slot s -> pixel (valid: a real one)
  auto tile_of = [&](int t, int& n, int& y0, int& x0) {
    const int tx = t % tiles_x, r = t / tiles_x;
    y0 = (r % tiles_y) * 2;
    n = r / tiles_y;
    x0 = tx * F_TCV;
  };
  auto slot_px = [&](int n, int y0, int x0, int s, int& y, int& x) {
    y = y0 + (s >> 5);
    x = x0 + (s & 31);
    return (s & 31) < F_TCV && y < H && x < W;
  };

  u32x4 pr[F_PIT];
  auto load_p = [&](int t) {  // y1 patch rows y0-1 .. y0+2, columns x0-1 .. x0+32 (zero outside)
    int n, y0, x0;
    tile_of(t, n, y0, x0);
#pragma unroll
    for (int it = 0; it < F_PIT; ++it) {
      const int q = tid + it * NT;
      const int pix = q >> 3, c = q & 7;
      const int gy = y0 - 1 + pix / F_PC, gx = x0 - 1 + pix % F_PC;
      pr[it] = (q < F_PCH && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
                   ? reinterpret_cast<const u32x4*>(y1in + ((size_t)(n * H + gy) * W + gx) * CX)[c]
                   : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_p = [&]() {
#pragma unroll
    for (int it = 0; it < F_PIT; ++it) {
      const int q = tid + it * NT;
      if (q < F_PCH) Ps[f_pchunk(q >> 3, q & 7)] = pr[it];
    }
  };
  constexpr int YIT = F_TP * CO / 8 / NT;  // 4
  constexpr int NRV = DUAL ? 1 : YIT;
  u32x4 rv[NRV], rvn[NRV];  // this tile's residual / xs rows, and the next tile's (in flight)
  auto load_second = [&](int t, u32x4 (&rv)[NRV]) {  // residual rows (or, dual, the shortcut input xs) of a tile
    int n, y0, x0, y, x;
    tile_of(t, n, y0, x0);
    if constexpr (DUAL) {
      const int s = tid >> 3;
      rv[0] = slot_px(n, y0, x0, s, y, x) ? reinterpret_cast<const u32x4*>(xs + ((size_t)(n * H + y) * W + x) * CX)[tid & 7]
                                          : u32x4{0u, 0u, 0u, 0u};
    } else {
#pragma unroll
      for (int it = 0; it < YIT; ++it) {
        const int q = tid + it * NT;
        rv[it] = slot_px(n, y0, x0, q >> 5, y, x)
                     ? reinterpret_cast<const u32x4*>(res + ((size_t)(n * H + y) * W + x) * CO)[q & 31]
                     : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };

  int t = blockIdx.x;
  load_p(t);
  load_second(t, rv);
  store_p();
  __syncthreads();
  // 3x3 work split: wave = (K half kh) x (2 pixel fragments) x (2 channel fragments); the
  // two K halves of a quadrant meet in LDS (the Y region, free until phase 1)
  const int kh = wave >> 2, qp = (wave & 1) * 2, qc = (wave >> 1 & 1) * 2;
  f32x4* red = reinterpret_cast<f32x4*>(Ys);
  while (true) {
    int n, y0, x0;
    tile_of(t, n, y0, x0);
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    if (more) {  // the next tile's patch and residual / xs in flight for the whole tile
      load_p(tn);
      load_second(tn, rvn);
    }
    // ---- 3x3: x2 = relu(conv3x3(y1) + b2), quadrant (pixel fragments qp, qp+1) x
    // (channel fragments qc, qc+1), this wave's 9 of the 18 K-steps (tap-major, 32 channels)
    {
      f32x4 c3[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c3[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      int pb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int s = (qp + j) * 16 + prow;
        pb[j] = (s >> 5) * F_PC + (s & 31);
      }
#pragma unroll
      for (int kk = 0; kk < 9; ++kk) {
        const int ks = kh * 9 + kk, tap = ks >> 1;
        const int dy = tap >= 6 ? 2 : (tap >= 3 ? 1 : 0), dx = tap - 3 * dy;
        const int c = (ks & 1) * 4 + kg, po = dy * F_PC + dx;
        bf16x8 a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = __builtin_bit_cast(bf16x8, W2s[f_wchunk((qc + i) * 16 + prow, ks * 4 + kg)]);
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = __builtin_bit_cast(bf16x8, Ps[f_pchunk(pb[j] + po, c)]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) c3[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], c3[i][j], 0, 0, 0);
      }
      const int qi = wave & 3;
      if (kh) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) red[((qi * 2 + i) * 2 + j) * 64 + lane] = c3[i][j];
      }
      __syncthreads();
      if (!kh) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int co = (qc + i) * 16 + kg * 4;
          const f32x4 bv = *reinterpret_cast<const f32x4*>(b2 + co);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const f32x4 o2 = red[((qi * 2 + i) * 2 + j) * 64 + lane];
            bf16x4 o;
            // K half 0 + K half 1 in fp32: another association than conv3x3c64's single
            // 18-step chain, so x2 matches it up to bf16 rounding flips
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(c3[i][j][r] + o2[r] + bv[r], 0.f));
            const int s = (qp + j) * 16 + prow;
            bf16* chunk = reinterpret_cast<bf16*>(Xs + swz<XC>(s, co >> 3));
            *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
          }
        }
      }
      if constexpr (DUAL) Xs[swz<XC>(tid >> 3, 8 + (tid & 7))] = rv[0];
    }
    __syncthreads();
    // ---- phase 1: y3 tile = [x2 | xs] . W3^T + b3  (wave: channels 32 wave .. +32, all slots)
    {
      f32x4 acc[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8 b = __builtin_bit_cast(bf16x8, Xs[swz<XC>(j * 16 + prow, ks * 4 + kg)]);
#pragma unroll
          for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[ks][i], b, acc[i][j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int co = wave * 32 + i * 16 + kg * 4;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(b3 + co);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bv[r]);
          bf16* chunk = reinterpret_cast<bf16*>(Ys + swz<32>(j * 16 + prow, co >> 3));
          *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
        }
      }
    }
    __syncthreads();
    // ---- pass: (+ residual) relu -> y3 (global, real pixels; decimated: the even ones) and Y
#pragma unroll
    for (int it = 0; it < YIT; ++it) {
      const int q = tid + it * NT;
      const int pl = q >> 5, c = q & 31;
      const int si = swz<32>(pl, c);
      bf16x8 v = __builtin_bit_cast(bf16x8, Ys[si]);
      if constexpr (DUAL) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf((float)v[e], 0.f));
      } else {
        const bf16x8 r = __builtin_bit_cast(bf16x8, rv[it]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf((float)v[e] + (float)r[e], 0.f));
      }
      Ys[si] = __builtin_bit_cast(u32x4, v);
      int y, x;
      if (slot_px(n, y0, x0, pl, y, x)) {
        if (!dec)
          reinterpret_cast<u32x4*>(y3 + ((size_t)(n * H + y) * W + x) * CO)[c] = __builtin_bit_cast(u32x4, v);
        else if (!((y | x) & 1))
          reinterpret_cast<u32x4*>(y3 + ((size_t)(n * (H >> 1) + (y >> 1)) * (W >> 1) + (x >> 1)) * CO)[c] =
              __builtin_bit_cast(u32x4, v);
      }
    }
    __syncthreads();
    // ---- phase 2: y1' = relu(Y . W1^T + b1)  (wave: channels 16 cf2 .. +16, P2F pixel fragments)
    {
      f32x4 acc2[P2F];
#pragma unroll
      for (int f = 0; f < P2F; ++f) acc2[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int f = 0; f < P2F; ++f) {
          const bf16x8 b = __builtin_bit_cast(bf16x8, Ys[swz<32>((pf2 + f) * 16 + prow, ks * 4 + kg)]);
          acc2[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[ks], b, acc2[f], 0, 0, 0);
        }
      const int co = cf2 * 16 + kg * 4;
      const f32x4 bv = *reinterpret_cast<const f32x4*>(b1 + co);
#pragma unroll
      for (int f = 0; f < P2F; ++f) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc2[f][r] + bv[r], 0.f));
        bf16* chunk = reinterpret_cast<bf16*>(Xs + swz<CN / 8>((pf2 + f) * 16 + prow, co >> 3));
        *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < F_TP * CN / 8 / NT; ++it) {
      const int q = tid + it * NT;
      const int pl = q / (CN / 8), c = q % (CN / 8);
      int y, x;
      if (slot_px(n, y0, x0, pl, y, x))
        reinterpret_cast<u32x4*>(y1out + ((size_t)(n * H + y) * W + x) * CN)[c] = Xs[swz<CN / 8>(pl, c)];
    }
    if (!more) break;
    store_p();        // the patch region has been dead since the 3x3
#pragma unroll
    for (int k = 0; k < NRV; ++k) rv[k] = rvn[k];
    __syncthreads();  // patch in place; the y1' staging read before the next x2 overwrites it
    t = tn;
  }
}

template <int CN, bool DUAL>
void launch_b3(const bf16* y1in, const bf16* xs, const bf16* res, const bf16* w2, const float* b2, const bf16* w3,
               const float* b3, const bf16* w1, const float* b1, bf16* y3, bf16* y1, int N, int H, int W, int num_cu,
               hipStream_t stream, int dec) {
  constexpr int CM = DUAL ? 2 * CX : CX;
  constexpr int XW = CN > CM ? CN : CM;
  constexpr size_t lds = F_WCH * 16 + F_PCH * 16 + F_TP * XW * 2 + F_TP * CO * 2;
  static_assert(lds <= 160 * 1024, "LDS");
  const int tiles = N * ((H + 1) / 2) * ((W + F_TCV - 1) / F_TCV);
  const int grid = tiles < num_cu ? tiles : num_cu;
  hipFuncSetAttribute((const void*)bottleneck3_kernel<CN, DUAL>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL((bottleneck3_kernel<CN, DUAL>), dim3(grid), dim3(NT), lds, stream, y1in, xs, res, w2, b2, w3, b3,
                     w1, b1, y3, y1, N, H, W, dec);
}

}  // namespace

// x2 [M, 64], res [M, 256] (or, dual: xs [M, 64] and no residual), w3 [256, 64] (dual:
// [256, 128] = [W3 | Wsc]), b3 [256], w1 [cn, 256], b1 [cn] -> y3 [M, 256], y1 [M, cn]
// (all bf16 rows contiguous; biases fp32); cn = 64 or 128 (128: identity residual only).
void bottleneck_tail_bf16(uintptr_t x2, uintptr_t xs, uintptr_t res, uintptr_t w3, uintptr_t b3, uintptr_t w1,
                          uintptr_t b1, uintptr_t y3, uintptr_t y1, int M, int cn, int num_cu, uintptr_t stream,
                          int dec_h, int dec_w) {
  if (M <= 0) throw std::invalid_argument("bottleneck_tail: empty problem");
  if ((long)M * CO >= (1L << 31)) throw std::invalid_argument("bottleneck_tail: tensor too large for 32-bit indexing");
  const bool dual = xs != 0;
  if (dual == (res != 0)) throw std::invalid_argument("bottleneck_tail: pass exactly one of xs (dual) and res");
  for (uintptr_t p : {x2, dual ? xs : res, w3, w1, y3, y1, b3, b1})
    if (!p || p % 16) throw std::invalid_argument("bottleneck_tail: null or non-16-byte-aligned pointer");
  // dec_h x dec_w > 0: y3 is stored decimated (its only other reader is a stride-2 1x1
  // projection shortcut, ResNet's stage-1 -> stage-2 boundary): 1/4 of the y3 bytes
  if (dec_w < 0 || dec_h < 0 || (dec_w > 0) != (dec_h > 0) || dec_w % 2 || dec_h % 2 ||
      (dec_w > 0 && M % (dec_h * dec_w)))
    throw std::invalid_argument("bottleneck_tail: decimation needs even H, W dividing the pixel count");
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto bp = [](uintptr_t p) { return reinterpret_cast<bf16*>(p); };
  auto fp = [](uintptr_t p) { return reinterpret_cast<const float*>(p); };
  if (dual && cn == 64)
    launch_tail<64, 64, true>(bp(x2), bp(xs), nullptr, bp(w3), fp(b3), bp(w1), fp(b1), bp(y3), bp(y1), M, num_cu, s, dec_h, dec_w);
  else if (!dual && cn == 64)
    launch_tail<128, 64, false>(bp(x2), nullptr, bp(res), bp(w3), fp(b3), bp(w1), fp(b1), bp(y3), bp(y1), M, num_cu, s, dec_h, dec_w);
  else if (!dual && cn == 128)
    launch_tail<64, 128, false>(bp(x2), nullptr, bp(res), bp(w3), fp(b3), bp(w1), fp(b1), bp(y3), bp(y1), M, num_cu, s, dec_h, dec_w);
  else
    throw std::invalid_argument("bottleneck_tail: unsupported variant (dual " + std::to_string(dual) + ", cn " +
                                std::to_string(cn) + ")");
  FTM_CHECK_LAUNCH();
}

// The block's 3x3 + its tail (bottleneck3_kernel): y1in [N, H, W, 64] (the 3x3's input),
// w2 [64][3][3][64] OHWI + b2 (ReLU), then as bottleneck_tail_bf16 with x2 computed
// in-kernel; dec: y3 stored decimated [N, H/2, W/2, 256].
void bottleneck3_bf16(uintptr_t y1in, uintptr_t xs, uintptr_t res, uintptr_t w2, uintptr_t b2, uintptr_t w3,
                      uintptr_t b3, uintptr_t w1, uintptr_t b1, uintptr_t y3, uintptr_t y1, int N, int H, int W, int cn,
                      int num_cu, uintptr_t stream, int dec) {
  if (N <= 0 || H <= 0 || W <= 0) throw std::invalid_argument("bottleneck3: empty problem");
  if ((long)N * H * W * CO >= (1L << 31)) throw std::invalid_argument("bottleneck3: tensor too large for 32-bit indexing");
  const bool dual = xs != 0;
  if (dual == (res != 0)) throw std::invalid_argument("bottleneck3: pass exactly one of xs (dual) and res");
  for (uintptr_t p : {y1in, dual ? xs : res, w2, b2, w3, w1, y3, y1, b3, b1})
    if (!p || p % 16) throw std::invalid_argument("bottleneck3: null or non-16-byte-aligned pointer");
  if (dec && (H % 2 || W % 2)) throw std::invalid_argument("bottleneck3: decimated y3 needs even H, W");
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto bp = [](uintptr_t p) { return reinterpret_cast<bf16*>(p); };
  auto fp = [](uintptr_t p) { return reinterpret_cast<const float*>(p); };
  if (dual && cn == 64)
    launch_b3<64, true>(bp(y1in), bp(xs), nullptr, bp(w2), fp(b2), bp(w3), fp(b3), bp(w1), fp(b1), bp(y3), bp(y1), N, H, W,
                        num_cu, s, dec);
  else if (!dual && cn == 64)
    launch_b3<64, false>(bp(y1in), nullptr, bp(res), bp(w2), fp(b2), bp(w3), fp(b3), bp(w1), fp(b1), bp(y3), bp(y1), N, H,
                         W, num_cu, s, dec);
  else if (!dual && cn == 128)
    launch_b3<128, false>(bp(y1in), nullptr, bp(res), bp(w2), fp(b2), bp(w3), fp(b3), bp(w1), fp(b1), bp(y3), bp(y1), N,
                          H, W, num_cu, s, dec);
  else
    throw std::invalid_argument("bottleneck3: unsupported variant (dual " + std::to_string(dual) + ", cn " +
                                std::to_string(cn) + ")");
  FTM_CHECK_LAUNCH();
}

void register_bottleneck(pybind11::module_& m) {
  m.def("bottleneck_tail_bf16", &bottleneck_tail_bf16);
  m.def("bottleneck3_bf16", &bottleneck3_bf16);
}
