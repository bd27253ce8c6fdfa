// ResNet stage 1's residual stream by RECOMPUTATION instead of HBM round trips.
//
// Stage 1 at micro-batch 256 carries a 256-channel residual stream at 56 x 56: every block's
// y3 (411 MB) is written by its tail and read back whole by the next block's tail, while the
// sources it is computed from are four times narrower:
//
//   y3_1 = relu([c1 | x0] . [W3a | Wsc]^T + b_1)      (block 1: expand + projection shortcut)
//   y3_j = relu(c_j . W3_j^T + b_j + y3_{j-1})        (blocks 2, 3: identity shortcut)
//
// with c_j the 64-channel 3x3 outputs and x0 the 64-channel stem output.  A tail that needs
// y3_{j-1} can recompute it from (x0, c1, .., c_{j-1}) — 64 channels each — for a few K = 64
// GEMMs per pixel, instead of reading the 256-channel tensor; and a tail whose y3 has no
// other reader than the next tail need not store it at all.  For ResNet-50 (3 blocks) this
// takes the stage-1 tails from ~2.9 GB to ~1.4 GB of HBM traffic per 256 images for
// ~130 GFLOP of extra MFMA work (kernels are HBM-bound: bottleneck.hip's measured tails run
// at 4-5.8 TB/s).
//
// One persistent kernel per tail, J = 1..3 links, then the next block's 1x1 reduce:
//
//   per tile of TP = 64 pixels (one workgroup per CU, 8 waves):
//     LDS  X: two stages of S = J + 1 source tiles [64 px][64 ch] (16-B chunks XOR-swizzled
//          per row), filled by LDS-DMA one tile ahead; Y: [64][256] y3 tile; O: [64][CN]
//          y1 staging, stored at the top of the next tile (every wait is then a tile old)
//     phase 1  wave w owns y3 channels 32w .. 32w + 31 for all 64 pixels; the link weights
//              of those channels live in VGPRs for the whole kernel (K = 128 + 64 (J - 1)
//              bf16 per channel row: 16 VGPRs per 64-deep link); each link's accumulator
//              is rounded exactly as the unfused tail rounds it (acc + b -> bf16, + residual
//              -> relu -> bf16) and the previous link's y3 stays in registers as the
//              residual — only the last y3 goes to LDS
//     pass     (STORE) coalesced 16-B chunks of Y -> y3 in HBM, decimated or not
//     phase 2  y1 = relu(Y . W1^T + b1): wave w owns one 16-channel fragment of W1 (32 VGPRs)
//              and 64 / (CN / 16 / 8 * 16) pixel fragments; staged in O, coalesced stores
//     (a first version staged the sources through registers during phase 2: every tile
//     then waited one HBM latency, 130 / 183 / 303 µs for J = 1 / 2 / 3 at micro-batch 256
//     against 175 / 199 / 197 µs for the unfused tails: profiles/r06_f)
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int CX = 64;   // channels of every source
constexpr int CO = 256;  // y3 channels
constexpr int NT = 512;  // 8 waves
constexpr int TP = 64;   // pixels per tile
constexpr int PF = TP / 16;

struct Link {
  const bf16* x;   // [M, 64]
  const bf16* xs;  // link 0 only: the projection source [M, 64] (K = 128), else null
  const bf16* w;   // [256, K] row-major (1x1 OHWI squeezed; link 0: [W3 | Wsc])
  const float* b;  // [256]
};

struct ChainParams {
  Link l[3];
  const bf16* w1;  // [CN, 256]
  const float* b1;
  bf16* y3;  // last link's y3 [M, 256] (or decimated), null: not stored
  bf16* y1;  // [M, CN]
  int M, dec_h, dec_w;
};

template <int CPR>
FTM_DEVICE int swz(int row, int c) {
  if constexpr (CPR == 8) return row * 8 + (c ^ ((row >> 1) & 7));
  else return row * CPR + (c ^ (row & 15));
}

template <int J, int CN, bool STORE>
__global__ __launch_bounds__(NT, 1) void bottleneck_chain_kernel(ChainParams p) {
  constexpr int S = J + 1;                 // source tiles: link 0 is dual
  constexpr int XS = TP * CX * 2;          // 8 KB per source tile
  constexpr int XB = S * XS;               // one stage of sources
  constexpr int YB = TP * CO * 2;          // 32 KB
  constexpr int CF = CN / 16;              // phase-2 channel fragments (4 or 8)
  constexpr int WPC = 8 / CF;              // waves per channel fragment (2 or 1)
  constexpr int PPW = PF / WPC;            // pixel fragments per wave in phase 2 (2 or 4)
  constexpr int PIECES = S * XS / 1024;    // 1-KiB LDS-DMA pieces per stage (8 per source)
  static_assert(CF * WPC == 8 && PPW * WPC == PF && PIECES % 8 == 0, "tile split");
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem[];
  // two source stages (the next tile's sources land by LDS-DMA during this tile), Y, O
  u32x4* Ys = reinterpret_cast<u32x4*>(smem + 2 * XB);
  u32x4* Os = reinterpret_cast<u32x4*>(smem + 2 * XB + YB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int prow = lane & 15, kg = lane >> 4;
  const int M = p.M;
  const int ntiles = (M + TP - 1) / TP;
  if ((int)blockIdx.x >= ntiles) return;  // block-uniform, before any barrier

  // ---- resident weights in VGPRs: link j, channel fragment i, K-step ks
  bf16x8 wa0[2][4], wa1[2][2], wa2[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int co = wave * 32 + i * 16 + prow;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      wa0[i][ks] = *reinterpret_cast<const bf16x8*>(p.l[0].w + (size_t)co * 128 + ks * 32 + kg * 8);
    if constexpr (J >= 2)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        wa1[i][ks] = *reinterpret_cast<const bf16x8*>(p.l[1].w + (size_t)co * 64 + ks * 32 + kg * 8);
    if constexpr (J >= 3)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        wa2[i][ks] = *reinterpret_cast<const bf16x8*>(p.l[2].w + (size_t)co * 64 + ks * 32 + kg * 8);
  }
  const int cf = wave / WPC;                // phase-2 channel fragment
  const int pf0 = (wave % WPC) * PPW;       // phase-2 first pixel fragment
  bf16x8 wb[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    wb[ks] = *reinterpret_cast<const bf16x8*>(p.w1 + (size_t)(cf * 16 + prow) * CO + ks * 32 + kg * 8);

  // ---- source staging by LDS-DMA: piece k (1 KiB = 8 pixel rows x 8 chunks) of source
  // k / 8; lane l writes LDS slot l of the piece: row 8 (k % 8) + l / 8, slot l % 8, which
  // holds logical chunk slot ^ ((row >> 1) & 7) (the swz<8> image) — pre-swizzled on the
  // global side; rows past M read beyond the buffer range: zeros, no branch
  const unsigned nbytes = (unsigned)M * CX * 2u;
  __amdgpu_buffer_rsrc_t rs[4];
#pragma unroll
  for (int sidx = 0; sidx < S; ++sidx) {
    const bf16* sp = sidx == 0 ? p.l[0].x : sidx == 1 ? p.l[0].xs : sidx == 2 ? p.l[1].x : p.l[2].x;
    rs[sidx] = __builtin_amdgcn_make_buffer_rsrc((void*)sp, 0, (int)nbytes, 0x00020000);
  }
  const int drow = lane >> 3, dslot = lane & 7;
  auto dma = [&](int t, int stage) {
#pragma unroll
    for (int k0 = 0; k0 < PIECES / 8; ++k0) {
      const int k = wave * (PIECES / 8) + k0;  // wave-uniform
      const int sidx = k >> 3, q = k & 7;
      const int row = q * 8 + drow;
      const int c = dslot ^ ((row >> 1) & 7);
      const unsigned off = (unsigned)(t * TP + row) * (CX * 2u) + (unsigned)c * 16u;
      uint8_t* dst = smem + stage * XB + sidx * XS + q * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[sidx], (__attribute__((address_space(3))) void*)dst, 16,
                                               (unsigned)(t * TP + row) < (unsigned)M ? off : 0x80000000u, 0, 0, 0);
    }
  };

  // one 64-deep link of phase 1 from source tile X, pixel fragments j0 .. j0 + PF / 2 - 1
  auto mma64 = [&](f32x4 (&acc)[2][PF / 2], const bf16x8 (&wa)[2][2], const u32x4* X, int j0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + kg;
#pragma unroll
      for (int j = 0; j < PF / 2; ++j) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, X[swz<8>((j0 + j) * 16 + prow, c)]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks], b, acc[i][j], 0, 0, 0);
      }
    }
  };
  // acc + b -> bf16, + residual (the previous link's y3, bf16-exact floats), relu -> bf16
  auto finish = [&](f32x4 (&acc)[2][PF / 2], f32x4 (&res)[2][PF / 2], const float* b, bool first) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(b + wave * 32 + i * 16 + kg * 4);
#pragma unroll
      for (int j = 0; j < PF / 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = (float)f2bf(acc[i][j][r] + bv[r]);
          res[i][j][r] = (float)f2bf(fmaxf(first ? v : v + res[i][j][r], 0.f));
        }
    }
  };
  // y1 of the previous tile out of O (coalesced 16-B chunks)
  auto store_y1 = [&](int pt) {
#pragma unroll
    for (int it = 0; it < TP * CN / 8 / NT; ++it) {
      const int q = tid + it * NT;
      const int pl = q / (CN / 8), c = q % (CN / 8);
      if (pt * TP + pl < M) reinterpret_cast<u32x4*>(p.y1 + (size_t)(pt * TP + pl) * CN)[c] = Os[swz<CN / 8>(pl, c)];
    }
  };

  int t = blockIdx.x;
  int stage = 0;
  int prev = -1;  // tile whose y1 waits in O
  dma(t, 0);
  while (true) {
    const int p0 = t * TP;
    // this tile's sources (issued one tile ago) and every older store have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (prev >= 0) store_y1(prev);  // O is read before phase 2 rewrites it (a barrier between)
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    if (more) dma(tn, stage ^ 1);  // the next tile's sources, in flight during this whole tile
    const u32x4* X = reinterpret_cast<const u32x4*>(smem + stage * XB);
    // ---- phase 1: the chain, y3 of channels 32w .. 32w + 31 in registers, in two halves
    // of 32 pixels (the chain is per pixel: half the accumulators live at a time)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      constexpr int PH = PF / 2;
      f32x4 y[2][PH], acc[2][PH];
      auto zero = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < PH; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      };
      const int j0 = half * PH;
      zero();
      {
        const bf16x8 w0a[2][2] = {{wa0[0][0], wa0[0][1]}, {wa0[1][0], wa0[1][1]}};
        const bf16x8 w0b[2][2] = {{wa0[0][2], wa0[0][3]}, {wa0[1][2], wa0[1][3]}};
        mma64(acc, w0a, X, j0);  // [c1 | x0]: K 0..63 from c1, 64..127 from x0
        mma64(acc, w0b, X + TP * 8, j0);
      }
      finish(acc, y, p.l[0].b, true);
      if constexpr (J >= 2) {
        zero();
        mma64(acc, wa1, X + 2 * TP * 8, j0);
        finish(acc, y, p.l[1].b, false);
      }
      if constexpr (J >= 3) {
        zero();
        mma64(acc, wa2, X + 3 * TP * 8, j0);
        finish(acc, y, p.l[2].b, false);
      }
      // y3 into Y: y[i][j][r] = channel 32w + 16i + 4kg + r of pixel 16 (j0 + j) + prow
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int co = wave * 32 + i * 16 + kg * 4;
#pragma unroll
        for (int j = 0; j < PH; ++j) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(y[i][j][r]);
          bf16* chunk = reinterpret_cast<bf16*>(Ys + swz<32>((j0 + j) * 16 + prow, co >> 3));
          *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
        }
      }
    }
    __syncthreads();  // Y complete; this stage's sources read
    if constexpr (STORE) {  // y3 to HBM in coalesced 16-B chunks (decimated: even (h, w) only)
      int dn = 0, dh = 0, dw = 0;
      if (p.dec_w) {
        const int o0 = p0 + (tid >> 5);
        dw = o0 % p.dec_w;
        const int tt = o0 / p.dec_w;
        dh = tt % p.dec_h;
        dn = tt / p.dec_h;
      }
#pragma unroll
      for (int it = 0; it < TP * CO / 8 / NT; ++it) {
        const int q = tid + it * NT;
        const int pl = q >> 5, c = q & 31;
        int o = p0 + pl;
        bool st = o < M;
        if (p.dec_w) {
          if (it) {
            dw += 16;
            while (dw >= p.dec_w) {
              dw -= p.dec_w;
              if (++dh == p.dec_h) { dh = 0; ++dn; }
            }
          }
          st = st && !((dh | dw) & 1);
          o = (dn * (p.dec_h >> 1) + (dh >> 1)) * (p.dec_w >> 1) + (dw >> 1);
        }
        if (st) reinterpret_cast<u32x4*>(p.y3 + (size_t)o * CO)[c] = Ys[swz<32>(pl, c)];
      }
    }
    // ---- phase 2: y1 = relu(Y . W1^T + b1): channel fragment cf, pixel fragments pf0 ..
    f32x4 acc2[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) acc2[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int c = ks * 4 + kg;
#pragma unroll
      for (int q = 0; q < PPW; ++q) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, Ys[swz<32>((pf0 + q) * 16 + prow, c)]);
        acc2[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[ks], b, acc2[q], 0, 0, 0);
      }
    }
    {
      const int co = cf * 16 + kg * 4;
      const f32x4 bv = *reinterpret_cast<const f32x4*>(p.b1 + co);
#pragma unroll
      for (int q = 0; q < PPW; ++q) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc2[q][r] + bv[r], 0.f));
        bf16* chunk = reinterpret_cast<bf16*>(Os + swz<CN / 8>((pf0 + q) * 16 + prow, co >> 3));
        *reinterpret_cast<bf16x4*>(chunk + (co & 7)) = o;
      }
    }
    prev = t;
    if (!more) break;
    t = tn;
    stage ^= 1;
  }
  __syncthreads();  // the last tile's O
  store_y1(prev);
}

template <int J, int CN, bool STORE>
void launch_chain(const ChainParams& p, int num_cu, hipStream_t s) {
  constexpr int XB = (J + 1) * TP * CX * 2, YB = TP * CO * 2, OB = TP * CN * 2;
  constexpr int LDS = 2 * XB + YB + OB;
  static_assert(LDS <= 160 * 1024, "LDS");
  const int tiles = (p.M + TP - 1) / TP;
  const int grid = tiles < num_cu ? tiles : num_cu;
  hipFuncSetAttribute((const void*)bottleneck_chain_kernel<J, CN, STORE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      LDS);
  hipLaunchKernelGGL((bottleneck_chain_kernel<J, CN, STORE>), dim3(grid), dim3(NT), LDS, s, p);
}

template <int J>
void dispatch_cn(const ChainParams& p, int cn, bool store, int num_cu, hipStream_t s) {
  if (cn == 64) {
    if (store) launch_chain<J, 64, true>(p, num_cu, s);
    else launch_chain<J, 64, false>(p, num_cu, s);
  } else {
    if (store) launch_chain<J, 128, true>(p, num_cu, s);
    else launch_chain<J, 128, false>(p, num_cu, s);
  }
}

}  // namespace

// links: 1..3 tuples (x, xs, w, b) of device pointers — link 0 dual (xs != 0, w [256, 128]),
// the others identity-residual (xs == 0, w [256, 64]); w1 [cn, 256], b1 [cn]; y3 (0: not
// stored) [M, 256] or decimated; y1 [M, cn].  All bf16 rows contiguous, biases fp32.
void bottleneck_chain_bf16(pybind11::list links, uintptr_t w1, uintptr_t b1, uintptr_t y3, uintptr_t y1, int M, int cn,
                           int num_cu, uintptr_t stream, int dec_h, int dec_w) {
  const int J = (int)pybind11::len(links);
  if (J < 1 || J > 3) throw std::invalid_argument("bottleneck_chain: 1 to 3 links");
  if (M <= 0 || (long)M * CO >= (1L << 31)) throw std::invalid_argument("bottleneck_chain: bad pixel count");
  if (cn != 64 && cn != 128) throw std::invalid_argument("bottleneck_chain: reduce width 64 or 128");
  ChainParams p{};
  for (int j = 0; j < J; ++j) {
    pybind11::tuple t = links[j].cast<pybind11::tuple>();
    if (t.size() != 4) throw std::invalid_argument("bottleneck_chain: link tuple (x, xs, w, b)");
    const uintptr_t x = t[0].cast<uintptr_t>(), xs = t[1].cast<uintptr_t>(), w = t[2].cast<uintptr_t>(),
                    b = t[3].cast<uintptr_t>();
    if ((j == 0) != (xs != 0)) throw std::invalid_argument("bottleneck_chain: link 0 dual, the others plain");
    for (uintptr_t q : {x, w, b})
      if (!q || q % 16) throw std::invalid_argument("bottleneck_chain: null or non-16-byte-aligned pointer");
    if (xs % 16) throw std::invalid_argument("bottleneck_chain: xs alignment");
    p.l[j] = Link{reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(xs), reinterpret_cast<const bf16*>(w),
                  reinterpret_cast<const float*>(b)};
  }
  for (uintptr_t q : {w1, b1, y1})
    if (!q || q % 16) throw std::invalid_argument("bottleneck_chain: null or non-16-byte-aligned pointer");
  if (y3 % 16) throw std::invalid_argument("bottleneck_chain: y3 alignment");
  if (dec_w < 0 || dec_h < 0 || (dec_w > 0) != (dec_h > 0) || dec_w % 2 || dec_h % 2 ||
      (dec_w > 0 && M % (dec_h * dec_w)))
    throw std::invalid_argument("bottleneck_chain: decimation needs even H, W dividing the pixel count");
  if (dec_w && !y3) throw std::invalid_argument("bottleneck_chain: decimation without y3");
  p.w1 = reinterpret_cast<const bf16*>(w1);
  p.b1 = reinterpret_cast<const float*>(b1);
  p.y3 = reinterpret_cast<bf16*>(y3);
  p.y1 = reinterpret_cast<bf16*>(y1);
  p.M = M;
  p.dec_h = dec_h;
  p.dec_w = dec_w;
  auto s = reinterpret_cast<hipStream_t>(stream);
  const bool store = y3 != 0;
  if (J == 1) dispatch_cn<1>(p, cn, store, num_cu, s);
  else if (J == 2) dispatch_cn<2>(p, cn, store, num_cu, s);
  else dispatch_cn<3>(p, cn, store, num_cu, s);
  FTM_CHECK_LAUNCH();
}

void register_bottleneck_chain(pybind11::module_& m) { m.def("bottleneck_chain_bf16", &bottleneck_chain_bf16); }
