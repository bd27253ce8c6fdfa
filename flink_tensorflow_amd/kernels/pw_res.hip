// Persistent pointwise (1x1 / stride-1) expansion conv with residual for CDNA4 MFMA:
//
//   y[m, n] = relu(x[m, :] . W[n, :] + b[n] + r[m, n])      x [M, K], W [N, K], K = 128 / 256
//
// ResNet's stage-2/3 bottleneck expands (128 -> 512, 256 -> 1024, + identity residual) move
// ~4x more activation bytes than they do MACs per byte can hide: they are bound by how
// many bytes each CU keeps in flight, not by MFMA.  The tiled implicit-GEMM kernel
// (igemm_bf16.hip) exposes one HBM round trip per 128x128 tile at workgroup start (x, W)
// and another in the epilogue (r).  Here a workgroup stays resident:
//   * its 128-channel weight slice W[n0 .. n0+128, :] is loaded into LDS once;
//   * it walks 128-pixel tiles; the NEXT tile's x rows and the next tile's residual rows
//     are loaded into registers while the current tile computes / stores (the same
//     one-tile-ahead scheme that took the stage-1 -> 2 block tail from 248 to 200 µs,
//     profiles/r02_tail_prefetch);
//   * the S = N / 128 workgroups that share a pixel tile sit on one XCD and walk the same
//     tile sequence, so x is fetched into that XCD's L2 once, not S times.
// LDS: W slice [128][K] | x tile [128][K] (the bf16 output tile [128][128] reuses it);
// 16-B chunks XOR-swizzled per row (conflict-free ds_read_b128 fragment reads).
// 8 waves: wave (wp, wc) computes pixels 64 wp .. +64 x channels 32 wc .. +32 with
// v_mfma_f32_16x16x32_bf16 (4 x 2 fragments).
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int NT = 512;  // threads (8 waves)

template <int CPR>
FTM_DEVICE int swz(int row, int c) { return row * CPR + (c ^ (row & (CPR >= 16 ? 15 : CPR - 1))); }

// K = K1 + K2 input channels (K2 > 0: DUAL, a second [M, K2] source x2 — a 1x1 conv with its
// stride-1 projection shortcut, no residual; its host entry was removed: 0.2-0.4 % slower end
// to end, profiles/r02_pw_res2 — only K2 = 0 is instantiated), TP pixels per tile, BN output channels per
// workgroup (resident slice)
template <int K1, int K2, int TP, int BN>
__global__ __launch_bounds__(NT, 2) void pw_res_kernel(const bf16* __restrict__ x, const bf16* __restrict__ x2,
                                                       const bf16* __restrict__ w, const float* __restrict__ bias,
                                                       const bf16* __restrict__ res, bf16* __restrict__ y, int M,
                                                       int S, int ldy, int y_coff, int ldr, int prio) {
  constexpr int K = K1 + K2;
  constexpr bool DUAL = K2 > 0;
  constexpr int KC = K / 8;             // 16-B chunks per x / W row
  constexpr int KC1 = K1 / 8;
  constexpr int XIT = TP * KC / NT;     // x chunks per thread per tile
  constexpr int OC = BN / 8;            // 16-B chunks per output row
  constexpr int RIT = TP * OC / NT;     // output / residual chunks per thread per tile
  constexpr int I = BN / 64, J = TP / 32;  // per wave: I x 16 channels, J x 16 pixels
  static_assert(XIT * NT == TP * KC && RIT * NT == TP * OC && I >= 1 && J >= 1, "tile shape");
  static_assert((size_t)TP * K >= (size_t)TP * BN, "output tile must fit the x tile region");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  u32x4* Ws = reinterpret_cast<u32x4*>(smem);
  u32x4* Xs = reinterpret_cast<u32x4*>(smem + BN * K * 2);  // x tile, then the output tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int prow = lane & 15, kg = lane >> 4;
  const int wp = wave >> 2, wc = wave & 3;

  // workgroup -> (channel slice s, tile group g on XCD xcd); consecutive blocks alternate XCDs
  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int gpx = (int)(gridDim.x >> 3) / S;  // tile groups per XCD
  const int s = local % S, g = local / S;
  const int ngroups = 8 * gpx;
  const int tiles = (M + TP - 1) / TP;
  int t = xcd * gpx + g;
  if (t >= tiles) return;  // block-uniform, before any barrier
  const int n0 = s * BN;

  // ---- resident weight slice
  for (int q = tid; q < BN * KC; q += NT)
    Ws[swz<KC>(q / KC, q % KC)] = reinterpret_cast<const u32x4*>(w + (size_t)(n0 + q / KC) * K)[q % KC];

  u32x4 xr[XIT], rv[RIT];
  auto load_x = [&](int tt) {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int q = tid + it * NT, px = tt * TP + q / KC, c = q % KC;
      const u32x4* src = (!DUAL || c < KC1) ? reinterpret_cast<const u32x4*>(x + (size_t)px * K1) + c
                                            : reinterpret_cast<const u32x4*>(x2 + (size_t)px * K2) + (c - KC1);
      xr[it] = px < M ? *src : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int it = 0; it < XIT; ++it) {
      const int q = tid + it * NT;
      Xs[swz<KC>(q / KC, q % KC)] = xr[it];
    }
  };
  auto load_r = [&](int tt) {
    if constexpr (DUAL) return;  // no residual
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int q = tid + it * NT, px = tt * TP + q / OC;
      rv[it] = px < M ? reinterpret_cast<const u32x4*>(res + (size_t)px * ldr + n0)[q % OC] : u32x4{0u, 0u, 0u, 0u};
    }
  };

  load_x(t);
  load_r(t);
  store_x();
  int tn = t + ngroups;
  if (tn < tiles) load_x(tn);
  __syncthreads();
  f32x4 bv[I];
#pragma unroll
  for (int i = 0; i < I; ++i) bv[i] = *reinterpret_cast<const f32x4*>(bias + n0 + wc * (BN / 4) + i * 16 + kg * 4);

  while (true) {
    // ---- MFMA: acc[i][j] = channels BN/4 wc + 16 i + 4 kg .. +4 of pixel TP/2 wp + 16 j + prow
    f32x4 acc[I][J];
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    FTM_PRIO_HI(prio);
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
      const int c = ks * 4 + kg;
      bf16x8 a[I], bb[J];
#pragma unroll
      for (int i = 0; i < I; ++i) a[i] = __builtin_bit_cast(bf16x8, Ws[swz<KC>(wc * (BN / 4) + i * 16 + prow, c)]);
#pragma unroll
      for (int j = 0; j < J; ++j) bb[j] = __builtin_bit_cast(bf16x8, Xs[swz<KC>(wp * (TP / 2) + j * 16 + prow, c)]);
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    FTM_PRIO_LO(prio);
    __syncthreads();  // x tile fully read: its LDS becomes the output tile
    // ---- acc + bias -> bf16 output tile [TP][BN]
#pragma unroll
    for (int i = 0; i < I; ++i) {
      const int co = wc * (BN / 4) + i * 16 + kg * 4;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bv[i][r]);
        bf16* chunk = reinterpret_cast<bf16*>(Xs + swz<OC>(wp * (TP / 2) + j * 16 + prow, co >> 3));
        *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
      }
    }
    __syncthreads();
    // ---- + residual, relu -> y (coalesced 16-B chunks); then the next tile's residual
    const int p0 = t * TP;
#pragma unroll
    for (int it = 0; it < RIT; ++it) {
      const int q = tid + it * NT, pl = q / OC, c = q % OC;
      bf16x8 v = __builtin_bit_cast(bf16x8, Xs[swz<OC>(pl, c)]);
      if constexpr (DUAL) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf((float)v[e], 0.f));
      } else {
        const bf16x8 r = __builtin_bit_cast(bf16x8, rv[it]);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(fmaxf((float)v[e] + (float)r[e], 0.f));
      }
      if (p0 + pl < M)
        *reinterpret_cast<u32x4*>(y + (size_t)(p0 + pl) * ldy + y_coff + n0 + c * 8) = __builtin_bit_cast(u32x4, v);
    }
    const bool more = tn < tiles;
    if (more) load_r(tn);
    __syncthreads();  // output tile read: the LDS takes the next x tile
    if (!more) break;
    store_x();
    t = tn;
    tn = t + ngroups;
    if (tn < tiles) load_x(tn);
    __syncthreads();
  }
}

template <int K1, int K2, int TP, int BN>
void launch(const bf16* x, const bf16* x2, const bf16* w, const float* b, const bf16* r, bf16* y, int M, int N,
            int ldy, int y_coff, int ldr, int num_cu, hipStream_t s) {
  constexpr int K = K1 + K2;
  if (N % BN) throw std::invalid_argument("pw_res: N must be a multiple of " + std::to_string(BN));
  const int S = N / BN;
  constexpr int occ = 1;  // one 8-wave workgroup per CU (2 waves per SIMD: <= 256 VGPRs, no spills)
  const int G = (num_cu * occ) / (8 * S) * (8 * S);
  if (G <= 0) throw std::invalid_argument("pw_res: too few CUs for the channel slices");
  constexpr size_t lds = (size_t)BN * K * 2 + (size_t)TP * K * 2;
  static_assert(lds <= 160 * 1024, "LDS");
  (void)hipFuncSetAttribute((const void*)pw_res_kernel<K1, K2, TP, BN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds);
  hipLaunchKernelGGL((pw_res_kernel<K1, K2, TP, BN>), dim3(G), dim3(NT), lds, s, x, x2, w, b, r, y, M, S, ldy, y_coff,
                     ldr, ftm_mfma_prio());
}

}  // namespace

// x [M, K] (rows contiguous), w [N, K], bias [N] fp32, res [M, ldr] -> y [M, ldy] at channel
// offset y_coff: y = relu(x . w^T + bias + res).  Tiles of 128 output channels; pixels per
// tile (tp = 0: default): K 128 -> 128, K 256 -> 64 (tp = 128 selectable).  Measured
// (bench/pw_res_bench.py): K 256 at 64 px 47.4 µs vs 54.0 µs at 128 px (twice the tiles per
// workgroup: less tail imbalance); a K 512 / 64 x 64 variant lost to the igemm kernel
// (54 vs 48 µs: 32 channel slices re-read each x tile from L2) and was dropped.
void pw_res_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int M, int N, int K, int ldy,
                 int y_coff, int ldr, int num_cu, uintptr_t stream, int tp) {
  if (K != 128 && K != 256) throw std::invalid_argument("pw_res: K must be 128 or 256");
  if (M <= 0 || N <= 0) throw std::invalid_argument("pw_res: empty problem");
  if (ldy % 8 || y_coff % 8 || ldr % 8 || ldr < N || ldy < y_coff + N)
    throw std::invalid_argument("pw_res: output / residual strides");
  if ((long)M * (ldy > ldr ? ldy : ldr) >= (1L << 31) || (long)M * K >= (1L << 31))
    throw std::invalid_argument("pw_res: tensor too large for 32-bit indexing");
  for (uintptr_t p : {x, w, bias, res, y})
    if (!p || p % 16) throw std::invalid_argument("pw_res: null or non-16-byte-aligned pointer");
  auto bp = [](uintptr_t p) { return reinterpret_cast<bf16*>(p); };
  auto fb = reinterpret_cast<const float*>(bias);
  auto s = reinterpret_cast<hipStream_t>(stream);
  if (K == 128)
    launch<128, 0, 128, 128>(bp(x), nullptr, bp(w), fb, bp(res), bp(y), M, N, ldy, y_coff, ldr, num_cu, s);
  else if (tp == 128)
    launch<256, 0, 128, 128>(bp(x), nullptr, bp(w), fb, bp(res), bp(y), M, N, ldy, y_coff, ldr, num_cu, s);
  else
    launch<256, 0, 64, 128>(bp(x), nullptr, bp(w), fb, bp(res), bp(y), M, N, ldy, y_coff, ldr, num_cu, s);
  FTM_CHECK_LAUNCH();
}

// y = relu([x | x2] . w^T + bias): x [M, 128], x2 [M, 256] (rows contiguous), w [N, 384] —
// ResNet's stage-2 entry expand conv with its projection shortcut, whose input the stage-1
// tail stored already decimated (compiler._decimate_tails), so both sources are plain
// pixel matrices.  N % 128 == 0.
void register_pw_res(pybind11::module_& m) {
  m.def("pw_res_bf16", &pw_res_bf16);
}
