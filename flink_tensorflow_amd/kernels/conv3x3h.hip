// 3x3 / stride-1 / pad-1 convolution (bf16 NHWC, Cin % 64 == 0) whose input is staged ONCE
// per 64-channel chunk as a halo in LDS and read nine times (one per filter tap) from there:
// the shape of ResNet-50's stage 2-4 bottleneck 3x3 convs (28x28x128, 14x14x256, 7x7x512).
//
// Why: conv_pp.hip's conv_lite stages an im2col tile per K-tile — 128 pixels x 128 B of
// input plus 128 channels x 128 B of weights.  In-kernel clocks put its K-tile at ~1,850
// cycles for 64 KiB per CU (two workgroups), ~35 B/clk of L2/MALL -> LDS fill, the same rate
// the fp8 twin reaches with half the MFMA work (profiles/r04_g, r04_q, r04_r): the loop is
// bound by bytes filled per CU, not by issue or latency.  Nine taps re-read the same input
// pixels, so the input half of that fill is 9x redundant.  Here a K-tile fills only its
// weights (16 KiB); the input arrives once per 64 channels as the tile's halo.
//
//   tile  = 128 consecutive output pixels (flattened n, oh, ow) x 128 output channels,
//           4 waves as 2 x 2 (64 x 64 outputs each, 4 x 4 v_mfma_f32_16x16x32_bf16 fragments)
//   halo  = the tile's receptive field in PADDED flattened coordinates: with Hp = H + 2,
//           Wp = W + 2, output pixel (n, oh, ow) reads padded pixel P + kh Wp + kw,
//           P = (n Hp + oh) Wp + ow, so the tile's whole field is the contiguous padded
//           range [P(m0), P(m_last) + 2 Wp + 3) even across rows and images (HL <= 288
//           pixels: ResNet's 28x28 needs 260 at most, 14x14 214, 7x7 240; the host checks);
//           padding pixels read zeros through the buffer range check
//   LDS   = halo [288 px][128 B] (36 KiB, 16-B chunk ^ key(px), below) + 2 weight stages
//           [128 co][128 B] (LDS-DMA, swizzled on the source) = 68 KiB: two workgroups / CU
//   K loop= (chunk c, tap) pairs; the next weight stage's DMA overlaps this tap's MFMAs;
//           the next chunk's halo is loaded into registers at tap 0 (in flight for nine
//           taps) and written to LDS at the next chunk's first barrier
//   epilogue: + bias, act -> bf16 tile in LDS -> coalesced 16-B row segments.
//
// Measured (profiles/r04_s .. r04_u): 36 % less TA work and 33 % fewer L2 reads than
// conv_lite, yet 8-12 % slower per layer — its LDS waits stay at twice conv_lite's — so the
// compiler routes convs here only with EngineConfig.conv3x3_halo (default off).
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128;
constexpr int ROWB = 128;                 // 64 bf16 channels per LDS row
constexpr int HLMAX = 288;                // halo pixels
constexpr int HB = HLMAX * ROWB;          // 36864
constexpr int WB = BN * ROWB;             // 16384
constexpr int HIT = HLMAX * 8 / 256;      // halo 16-B chunks per thread (9)
constexpr int OPITCH = BN * 2 + 16;
constexpr int LDS_MAIN = HB + 2 * WB;
constexpr int LDS = LDS_MAIN > BM * OPITCH ? LDS_MAIN : BM * OPITCH;
static_assert(HLMAX * 8 % 256 == 0, "halo chunks split evenly over 256 threads");

struct H3Params {
  const bf16* x;
  const bf16* w;  // [Cout][9 * C], k = (kh * 3 + kw) * C + c
  const float* bias;
  bf16* y;
  int N, H, W, C, Cout;
  int M;
  int ldy, y_coff;
  int tiles_m, tiles_n;
};

FTM_DEVICE int padded_base(const H3Params& p, int m) {
  const int hw = p.H * p.W;
  const int n = m / hw;
  const int r = m - n * hw;
  const int oh = r / p.W;
  const int ow = r - oh * p.W;
  return (n * (p.H + 2) + oh) * (p.W + 2) + ow;
}

// LDS writes of this wave retired, then the workgroup barrier; outstanding global loads
// (vmcnt) are left in flight
#define H3_BARRIER()                                                   \
  do {                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                 \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);                                 \
  } while (0)

template <int ACT>
__global__ __launch_bounds__(256, 2) void conv3x3h_kernel(H3Params p) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS];
  uint8_t* hs = smem;       // halo
  uint8_t* wsb = smem + HB; // weight stages

  const int nwg = p.tiles_m * p.tiles_n;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int Hp = p.H + 2, Wp = p.W + 2;
  const int K = 9 * p.C;
  const int P0 = padded_base(p, m0);

  // ---- halo loader: thread owns halo chunks q = tid + 256 it (pixel q / 8, chunk q % 8)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(p.x), 0, (int)((unsigned)p.N * (unsigned)(p.H * p.W) * (unsigned)p.C * 2u), 0x00020000);
  unsigned hoff[HIT];
  {
    const int hp0 = tid >> 3, j = tid & 7;
    const int pimg = Hp * Wp;
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
      const int P = P0 + hp0 + 32 * it;
      const int n = P / pimg;
      const int r = P - n * pimg;
      const int ph = r / Wp;
      const int pw = r - ph * Wp;
      const bool ok = n < p.N && ph >= 1 && ph <= p.H && pw >= 1 && pw <= p.W;
      hoff[it] = ok ? (unsigned)((((n * p.H + ph - 1) * p.W + pw - 1) * p.C) * 2 + j * 16) : 0x80000000u;
    }
  }
  // LDS slot of this thread's chunks: pixel hp0 + 32 it -> (hp0 & 7) is the swizzle key
  // Swizzle key of halo pixel hp: (hp - 2 * padded_row(P0 + hp)) & 7.  It advances by one
  // from each output pixel to the next, across row ends too (the padded index jumps by 3
  // there, the row by 1), so the 16 pixels of a B fragment get 16 consecutive keys at every
  // tap and the ds_read_b128 lane groups stay conflict-free; a plain hp & 7 key collided
  // at every row end (13x the bank-conflict cycles of conv_lite: profiles/r04_t).
  int hslot[HIT];
#pragma unroll
  for (int it = 0; it < HIT; ++it) {
    const int hp = (tid >> 3) + 32 * it;
    const int key = (hp - 2 * ((P0 + hp) / Wp)) & 7;
    hslot[it] = hp * ROWB + (((tid & 7) ^ key) << 4);
  }
  u32x4 hreg[HIT];
  auto load_halo = [&](int c) {
#pragma unroll
    for (int it = 0; it < HIT; ++it)
      hreg[it] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, hoff[it], c * 128, 0));
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int it = 0; it < HIT; ++it) *reinterpret_cast<u32x4*>(hs + hslot[it]) = hreg[it];
  };

  // ---- weight DMA: wave w stages rows 8 (4 w + q) + lane / 8 of the [128 co][128 B] image;
  // the lane's 16-B chunk is pre-swizzled on the source
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(p.w), 0, (int)((unsigned)p.Cout * (unsigned)K * 2u), 0x00020000);
  unsigned offw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned co = n0 + 8 * (4 * wave + q) + drow;
    offw[q] = co < (unsigned)p.Cout ? (co * (unsigned)K + dchunk * 8) * 2u : 0x80000000u;
  }
  auto dma_w = [&](int stage, int kt) {
    const int c = kt / 9, tap = kt - c * 9;
    const unsigned woff = (unsigned)(tap * p.C + c * 64) * 2u;
    uint8_t* bw = wsb + stage * WB + 4 * wave * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(bw + q * 1024), 16,
                                               offw[q], woff, 0, 0);
  };

  // ---- fragment roles: A = weights (rows = output channels), B = halo pixels
  const int frow = lane & 15;
  const int fq = lane >> 4;
  int pbase[4];  // halo pixel of this lane's output pixel in fragment j, tap (0, 0)
  int pkey[4];   // its swizzle key minus the tap's part: key = (pkey + kh W + kw) & 7
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + frow;
    pbase[j] = m < p.M ? padded_base(p, m) - P0 : 0;  // tail rows read pixel 0 and are not stored
    pkey[j] = pbase[j] - 2 * ((P0 + pbase[j]) / Wp);
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nc = p.C / 64;
  const int nk = nc * 9;
  load_halo(0);
  dma_w(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  store_halo();
  int c = 0, tap = 0;
  bool halo_inflight = false;
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    // the halo loads issued at tap 0 went out after that tap's weight DMA: at tap 1 only the
    // weight stage must have landed
    // (raw barriers: __syncthreads would also drain vmcnt, i.e. wait for the halo loads)
    if (tap == 1 && halo_inflight) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    H3_BARRIER();
    if (tap == 0 && c > 0) {  // every wave is past the previous chunk's taps
      store_halo();
      H3_BARRIER();
      halo_inflight = false;
    }
    if (kt + 1 < nk) dma_w(st ^ 1, kt + 1);
    if (tap == 0 && c + 1 < nc) {
      load_halo(c + 1);
      halo_inflight = true;
    }
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = kh * Wp + kw;   // tap (kh, kw) reads padded row + kh, column + kw
    const int tkey = kh * p.W + kw;  // key advance: toff - 2 kh
    const uint8_t* ws = wsb + st * WB;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int lc = ks * 4 + fq;  // logical 16-B chunk (8 channels) of the 64
      const int sla = (lc ^ (frow & 7)) << 4;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ws + (wn * 64 + i * 16 + frow) * ROWB + sla);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int hp = pbase[j] + toff;
        b[j] = *reinterpret_cast<const bf16x8*>(hs + hp * ROWB + ((lc ^ ((pkey[j] + tkey) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (++tap == 9) {
      tap = 0;
      ++c;
    }
  }
  __syncthreads();  // the epilogue tile reuses the halo / weight images

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cl = wn * 64 + i * 16 + fq * 4;
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (n0 + cl < p.Cout) bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + cl);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pl = wm * 64 + j * 16 + frow;
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(apply_act<ACT>(acc[i][j][r] + bv[r]));
      *reinterpret_cast<bf16x4*>(smem + pl * OPITCH + cl * 2) = o;
    }
  }
  __syncthreads();
  constexpr int SEGS = BN / 8;
#pragma unroll 4
  for (int q = tid; q < BM * SEGS; q += 256) {
    const int ml = q / SEGS;
    const int ccol = q - ml * SEGS;
    const int m = m0 + ml;
    const int n = n0 + ccol * 8;
    if (m >= p.M || n >= p.Cout) continue;
    *reinterpret_cast<u32x4*>(p.y + (size_t)m * p.ldy + p.y_coff + n) =
        *reinterpret_cast<const u32x4*>(smem + ml * OPITCH + ccol * 16);
  }
}

// halo pixels the widest 128-pixel tile needs (host copy of padded_base)
int halo_len(int N, int H, int W) {
  const long M = (long)N * H * W;
  auto pb = [&](long m) {
    const long n = m / ((long)H * W), r = m - n * H * W, oh = r / W, ow = r - oh * W;
    return (n * (H + 2) + oh) * (W + 2) + ow;
  };
  long worst = 0;
  for (long m0 = 0; m0 < M; m0 += BM) {
    const long m1 = m0 + BM - 1 < M ? m0 + BM - 1 : M - 1;
    const long span = pb(m1) - pb(m0);
    if (span > worst) worst = span;
  }
  return (int)(worst + 2 * (W + 2) + 3);
}

}  // namespace

// x [N, H, W, C] bf16, w [Cout, 3, 3, C] bf16 (OHWI, BN folded), bias [Cout] fp32,
// y [N*H*W, ldy] bf16 at channel offset y_coff.  SAME padding (1 each side), stride 1.
int conv3x3h_halo(int N, int H, int W) { return halo_len(N, H, W); }

void conv3x3h_bf16(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int H, int W, int C, int Cout,
                   int ldy, int y_coff, int act, uintptr_t stream) {
  if (C % 64 || C <= 0) throw std::invalid_argument("conv3x3h: Cin must be a positive multiple of 64");
  if (Cout % 8 || ldy % 8 || y_coff % 8 || ldy < y_coff + Cout)
    throw std::invalid_argument("conv3x3h: Cout / ldy / y_coff must be multiples of 8 and fit");
  if ((long)N * H * W * C * 2 >= (1L << 31) || (long)N * H * W * ldy >= (1L << 31) ||
      (long)N * (H + 2) * (W + 2) >= (1L << 31) || (long)Cout * 9 * C * 2 >= (1L << 31))
    throw std::invalid_argument("conv3x3h: tensor too large for 32-bit indexing");
  if (x % 16 || w % 16 || y % 16 || !bias || bias % 16) throw std::invalid_argument("conv3x3h: misaligned pointers / no bias");
  if (N <= 0 || H <= 0 || W <= 0) throw std::invalid_argument("conv3x3h: empty input");
  if (halo_len(N, H, W) > HLMAX) throw std::invalid_argument("conv3x3h: a 128-pixel tile's halo exceeds 288 pixels");
  H3Params p{};
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.y = reinterpret_cast<bf16*>(y);
  p.N = N; p.H = H; p.W = W; p.C = C; p.Cout = Cout;
  p.M = N * H * W;
  p.ldy = ldy; p.y_coff = y_coff;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (Cout + BN - 1) / BN;
  auto s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if (act == ACT_RELU) hipLaunchKernelGGL(conv3x3h_kernel<ACT_RELU>, grid, block, 0, s, p);
  else if (act == ACT_NONE) hipLaunchKernelGGL(conv3x3h_kernel<ACT_NONE>, grid, block, 0, s, p);
  else throw std::invalid_argument("conv3x3h: act must be none or relu");
  FTM_CHECK_LAUNCH();
}

void register_conv3x3h(pybind11::module_& m) {
  m.def("conv3x3h_bf16", &conv3x3h_bf16);
  m.def("conv3x3h_halo", &conv3x3h_halo);
}
