// Persistent 3x3 / stride-1 / pad-1 convolution for 64 -> 64 channels (bf16 NHWC), the
// shape of ResNet-50's stage-1 bottleneck convs (56x56x64 at every micro-batch image).
//
// Why a dedicated kernel: as an implicit GEMM (N = Cout = 64, K = 576) every 256-pixel
// tile re-gathers its im2col rows nine times through L2 and reloads the 74 KB of weights,
// so the layer runs at ~460 TFLOP/s.  Here the whole filter bank stays RESIDENT in LDS
// for the life of the workgroup (gfx950: 160 KB of LDS per CU) and each input patch is
// staged once and read nine times (one per tap) from LDS:
//
//   grid  = one workgroup per CU (persistent), 8 waves; tiles = 8 output rows x 32 columns
//           of one image (the last row / column tile overlaps its neighbour when H % 8 or
//           W % 32 != 0 — recomputed pixels are written twice with identical values)
//   LDS   = weights [64 co][576 k] (73.7 KB, 16-B chunks XOR-swizzled by (co >> 1) & 7)
//           + input patch [10][34][64] (43.5 KB, chunks swizzled by (pixel >> 1) & 7):
//           every ds_read_b128 fragment read is bank-conflict free
//   wave  = one output row: 32 pixels x 64 channels = 2 x 4 fragments of
//           v_mfma_f32_16x16x32_bf16 (A = weights, B = pixels), 18 k-steps per tile
//   pipeline: the next tile's patch is loaded into registers while the current tile's
//           MFMAs run; epilogue (bias + act, 8-byte stores of 4 channels) from registers.
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int C = 64;            // in = out channels
constexpr int TR = 8;            // output rows per tile (one per wave)
constexpr int TC = 32;           // output columns per tile
constexpr int PR = TR + 2;       // patch rows
constexpr int PC = TC + 2;       // patch columns
constexpr int KC = 9 * C / 8;    // 16-B weight chunks per output channel (72)
constexpr int NT = 512;          // threads
constexpr int PCHUNKS = PR * PC * (C / 8);            // 2720 16-B chunks per patch
constexpr int PITER = (PCHUNKS + NT - 1) / NT;        // 6 loads per thread
constexpr int W_BYTES = C * KC * 16;                  // 73728
constexpr int P_BYTES = PR * PC * C * 2;              // 43520

FTM_DEVICE int wchunk(int co, int k) { return co * KC + (k ^ ((co >> 1) & 7)); }       // k < 72, XOR stays in its group of 8
FTM_DEVICE int pchunk(int pix, int c) { return pix * 8 + (c ^ ((pix >> 1) & 7)); }    // c < 8

struct Tile {
  int n, y0, x0;
};

FTM_DEVICE Tile tile_of(int t, int tiles_y, int tiles_x, int H, int W) {
  const int tx = t % tiles_x;
  const int r = t / tiles_x;
  const int ty = r % tiles_y;
  Tile o;
  o.n = r / tiles_y;
  o.y0 = min(ty * TR, H - TR);
  o.x0 = min(tx * TC, W - TC);
  return o;
}

template <int ACT>
__global__ __launch_bounds__(NT, 1) void conv3x3c64_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                          const float* __restrict__ bias, bf16* __restrict__ y,
                                                          int N, int H, int W, int ldy, int y_coff, int prio) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  u32x4* Ws = reinterpret_cast<u32x4*>(smem);
  u32x4* Ps = reinterpret_cast<u32x4*>(smem + W_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_y = (H + TR - 1) / TR, tiles_x = (W + TC - 1) / TC;
  const int ntiles = N * tiles_y * tiles_x;
  if ((int)blockIdx.x >= ntiles) return;  // block-uniform, before any barrier

  // ---- filter bank -> LDS once: w is OHWI [64][3][3][64] = [co][576] contiguous
  for (int q = tid; q < C * KC; q += NT) {
    const int co = q / KC, k = q - co * KC;
    Ws[wchunk(co, k)] = reinterpret_cast<const u32x4*>(w)[q];
  }
  float bv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[i][r] = bias[i * 16 + (lane >> 4) * 4 + r];

  u32x4 stage[PITER];
  // patch loads through a buffer descriptor: the zero padding and the chunks past the patch
  // read as zeros from an out-of-range offset — no branch around each load
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(x), 0, N * H * W * C * 2, 0x00020000);
  auto load_patch = [&](const Tile& t) {
#pragma unroll
    for (int it = 0; it < PITER; ++it) {
      const int q = tid + it * NT;
      const int pix = q >> 3, c = q & 7;
      const int py = pix / PC, px = pix - py * PC;
      const int gy = t.y0 - 1 + py, gx = t.x0 - 1 + px;
      const bool ok = q < PCHUNKS && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      const unsigned off = ok ? (unsigned)((((t.n * H + gy) * W + gx) * C) * 2 + c * 16) : 0x80000000u;
      stage[it] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int it = 0; it < PITER; ++it) {
      const int q = tid + it * NT;
      if (q < PCHUNKS) Ps[pchunk(q >> 3, q & 7)] = stage[it];
    }
  };

  int t = blockIdx.x;
  Tile cur = tile_of(t, tiles_y, tiles_x, H, W);
  load_patch(cur);
  store_patch();
  __syncthreads();

  const int prow = lane & 15;   // fragment row: pixel (B) / output channel (A)
  const int kg = lane >> 4;     // 8-element k group within a 32-deep step
  while (true) {
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    Tile nxt = cur;
    if (more) {
      nxt = tile_of(tn, tiles_y, tiles_x, H, W);
      load_patch(nxt);  // in flight while this tile's MFMAs run
    }
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    FTM_PRIO_HI(prio);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // 32 input channels per k-step
        const int c8 = h * 4 + kg;    // 16-B chunk of the pixel's 64 channels
        bf16x8 a[4], b[2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a[i] = __builtin_bit_cast(bf16x8, Ws[wchunk(i * 16 + prow, tap * 8 + c8)]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int pix = (wave + kh) * PC + j * 16 + prow + kw;
          b[j] = __builtin_bit_cast(bf16x8, Ps[pchunk(pix, c8)]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    FTM_PRIO_LO(prio);
    // ---- epilogue: lane holds channels 16i + 4*kg + r of pixel (wave, 16j + prow)
    {
      const int oy = cur.y0 + wave;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ox = cur.x0 + j * 16 + prow;
        bf16* dst = y + (((size_t)cur.n * H + oy) * W + ox) * ldy + y_coff;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(apply_act<ACT>(acc[i][j][r] + bv[i][r]));
          *reinterpret_cast<bf16x4*>(dst + i * 16 + kg * 4) = o;
        }
      }
    }
    if (!more) break;
    __syncthreads();  // every wave is done reading the current patch
    store_patch();
    __syncthreads();
    cur = nxt;
    t = tn;
  }
}

}  // namespace

// x [N, H, W, 64] bf16, w [64, 3, 3, 64] bf16 (OHWI, BN folded), bias [64] fp32,
// y [N, H, W, ldy] bf16 at channel offset y_coff.  SAME padding (1 each side), stride 1.
void conv3x3c64_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int H, int W, int ldy, int y_coff,
                     int act, int num_cu, uintptr_t stream) {
  if (H < TR || W < TC) throw std::invalid_argument("conv3x3c64: needs H >= 8 and W >= 32");
  if (ldy % 4 || y_coff % 4 || ldy < y_coff + C) throw std::invalid_argument("conv3x3c64: bad output stride/offset");
  if ((long)N * H * W * C * 2 >= (1L << 31) || (long)N * H * W * ldy >= (1L << 31))
    throw std::invalid_argument("conv3x3c64: tensor too large for 32-bit indexing");
  if (x % 16 || w % 16 || y % 8 || !bias) throw std::invalid_argument("conv3x3c64: misaligned pointers / no bias");
  const int tiles = N * ((H + TR - 1) / TR) * ((W + TC - 1) / TC);
  const int grid = tiles < num_cu ? tiles : num_cu;
  const size_t lds = W_BYTES + P_BYTES;
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto X = reinterpret_cast<const bf16*>(x);
  auto Wt = reinterpret_cast<const bf16*>(w);
  auto B = reinterpret_cast<const float*>(bias);
  auto Y = reinterpret_cast<bf16*>(y);
  if (act == ACT_RELU) {
    hipFuncSetAttribute((const void*)conv3x3c64_kernel<ACT_RELU>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(conv3x3c64_kernel<ACT_RELU>, dim3(grid), dim3(NT), lds, s, X, Wt, B, Y, N, H, W, ldy, y_coff,
                       ftm_mfma_prio());
  } else if (act == ACT_NONE) {
    hipFuncSetAttribute((const void*)conv3x3c64_kernel<ACT_NONE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(conv3x3c64_kernel<ACT_NONE>, dim3(grid), dim3(NT), lds, s, X, Wt, B, Y, N, H, W, ldy, y_coff,
                       ftm_mfma_prio());
  } else {
    throw std::invalid_argument("conv3x3c64: act must be none or relu");
  }
  FTM_CHECK_LAUNCH();
}

void register_conv3x3c64(pybind11::module_& m) { m.def("conv3x3c64_bf16", &conv3x3c64_bf16); }
