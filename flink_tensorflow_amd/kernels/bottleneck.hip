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

void register_bottleneck(pybind11::module_& m) {
  m.def("bottleneck_tail_bf16", &bottleneck_tail_bf16);
}
