// Winograd F(2x2, 3x3) convolution, stride 1, SAME padding, bf16 NHWC in / out, for the
// stride-1 3x3 convs of ResNet-50 (stages 1-4: 56x56x64 .. 7x7x512).
//
// Why: as a direct implicit GEMM a 3x3 conv runs 9 * Cin MACs per output value; F(2x2,3x3)
// computes a 2x2 output tile from its 4x4 input patch with 16 element-wise products per
// (input, output) channel pair instead of 36 — 2.25x fewer MFMA FLOPs.  (Lavin & Gray:
// Y = A^T [ (G g G^T) .* (B^T d B) ] A.)  The GEMM view: for each of the 16 transform
// positions xi, M_xi [tiles x Cout] = V_xi [tiles x Cin] . U_xi [Cin x Cout].
//
// Numerics: the transform domain is fp16 (10-bit mantissa, 3 more than bf16): the bf16
// input is converted once while it is staged into LDS, V = B^T d B is formed with packed
// fp16 adds (v_pk_add_f16 — gfx950 has no packed bf16 add), U = G g G^T is precomputed in
// fp32 and rounded to fp16 once; products accumulate in fp32 (v_mfma_f32_32x32x16_f16),
// and the output transform, bias and activation run in fp32.  Valid while |V| < 65504,
// i.e. |activation| < 16376 (ResNet activations are O(1..100)).
//
// Work split: one workgroup = 64 tiles (2x2 output blocks, flattened over N x TH x TW)
// x 64 output channels; 4 waves, one per SIMD, wave i owns transform ROW i (xi = 4i + j,
// j = 0..3), so every operand a wave touches is private to it:
//   * its B^T rows need only 2 of the patch's 4 input rows: per 16 input channels a lane
//     reads 8 pixels (one ds_read_b128 each = 8 channels) and forms its 4 V fragments with
//     32 v_pk_add_f16 — no V image in LDS, no second pass;
//   * U_xi for the wave's 4 xi comes straight from global (L2) into registers, laid out in
//     MFMA-fragment order at compile time (1 KiB contiguous per wave-instruction);
//   * 16 accumulators of 32x32 (4 xi x 2 channel blocks x 2 tile blocks) = 256 f32 / lane.
// MFMA: acc[cout][tile] += U_frag (A: rows = cout) . V_frag (B: cols = tile), so the
// accumulator has the tile on the lane and 4 consecutive output channels in 4 consecutive
// registers — which is what the epilogue's 16-byte LDS writes want.
// LDS: the input rows the 64 tiles touch, 32 channels per K-step, double buffered:
//   [row][column parity p][16-channel half s][column pair q][8-channel chunk h^z(q)]
// (columns de-interleaved by parity so lanes of consecutive tiles read consecutive 32-B
// pixel slots; z(q) = (q >> 3) & 1 makes a 16-lane ds_read_b128 group hit 16 distinct
// 16-B bank groups).  Epilogue: each wave applies the column half of A^T . A to its 4 xi
// (Z_i[c], c = 0, 1), writes Z into LDS [i][c][tile][cout] (f32, pitch 68), and then every
// thread combines the 4 rows for (tile, 8 channels): 2x2 outputs, + bias, act, 16-B stores.
#include <pybind11/pybind11.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

#include "common.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 256;   // 4 waves
constexpr int TB = 64;    // tiles per workgroup
constexpr int CB = 64;    // output channels per workgroup
constexpr int ZP = 68;    // f32 pitch of an epilogue exchange row [tile][cout]
constexpr int SMAX = 12;  // staged 16-B chunks per thread and K-step, at most
constexpr int Z_BYTES = 4 * 2 * TB * ZP * 4;
constexpr int U_LDS = 4 * 2 * 8 * 1024;  // per wave: 2 buffers x 8 U fragments of 1 KiB

// B^T rows (and A-side combination of t into V): row r = S0 * v[R0[r]] + S1 * v[R1[r]],
// S0 = +1:  0: v0 - v2 | 1: v1 + v2 | 2: v2 - v1 | 3: v1 - v3
constexpr int r0_of(int r) { return r == 3 ? 1 : r; }
constexpr int r1_of(int r) { return r == 0 ? 2 : r == 1 ? 2 : r == 2 ? 1 : 3; }
constexpr bool neg1_of(int r) { return r != 1; }

// V = t_a -/+ t_b as one v_pk_fma_f16 per dword: t_b * sign + t_a with the sign vector held
// in a register the compiler cannot see through (Params::neg_one = -1 at run time) — on a
// literal -1 (or a plain f16-vector subtraction) it emitted v_sub_f16 + v_sub_f16_sdwa +
// v_pack_b32_f16 per dword, 3x the VALU
template <int R>
FTM_DEVICE f16x8 bt_comb(const f16x8& v0, const f16x8& v1, const f16x8& neg) {
  if constexpr (neg1_of(R)) return __builtin_elementwise_fma(neg, v1, v0);
  else return v0 + v1;
}

FTM_DEVICE int chunk_of(int row, int p, int s, int q, int h, int Qp, int RS) {
  return row * RS + ((p * 2 + s) * 2 + h) * Qp + q;
}

FTM_DEVICE u32x4 bf16x8_to_f16x8(u32x4 v) {
  u32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = __builtin_bit_cast(float, v[e] << 16);
    const float hi = __builtin_bit_cast(float, v[e] & 0xffff0000u);
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    h2 pk = {(_Float16)lo, (_Float16)hi};
    o[e] = __builtin_bit_cast(uint32_t, pk);
  }
  return o;
}

// x / d for the kernel's non-constant divisors by a multiply-high with m = ceil(2^32 / d):
// exact while x * d < 2^32 (host-checked); an integer division is ~30 VALU on gfx950
struct FDiv {
  uint32_t m;
  int d;
};
FTM_DEVICE int fdiv(int x, FDiv f) { return (int)__umulhi((uint32_t)x, f.m); }

struct Params {
  const bf16* x;
  const _Float16* u;
  const float* bias;
  bf16* y;
  int N, H, W, C, Cout, T, TH, TW, HpL, Qp, RS, stage_chunks, ldy, y_coff;
  int nblk, ncb, xcd_k;  // tile blocks, channel blocks, XCD mapping (0: plain)
  float neg_one;
  FDiv d_per, d_tw, d_rs, d_hpl;
};

// One code path for the four waves (wave i = transform row I): the row's input-row pair
// and sign are data, not template arguments — four specialised bodies of ~16 KB each
// thrashed the instruction cache the two CUs of a WGP share (7-8x slower).
template <int N>
FTM_DEVICE void wait_vmcnt() {  // s_waitcnt vmcnt(N), expcnt / lgkmcnt untouched
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int NS>
FTM_DEVICE void wave_body(const Params& P, uint8_t* smem, const int (&soff)[SMAX], int chunks, int Ga, int t0,
                          int I, int cblk) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  const int Qp = P.Qp;
  const int KK = P.C / 32;
  const int stage_bytes = P.stage_chunks * 16;
  uint8_t* stages = smem + U_LDS;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(P.x), 0, P.N * P.H * P.W * P.C * 2, 0x00020000);

  // ---- per-lane patch addresses (byte offset of (row a, b) for s = 0), both tile blocks
  int rowslot[2], tx[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    int t = t0 + 32 * rb + r;
    if (t >= P.T) t = P.T - 1;  // clamped: valid reads, the output is not stored
    const int per = P.TH * P.TW;
    const int n = fdiv(t, P.d_per), rem = t - n * per;
    const int ty = fdiv(rem, P.d_tw);
    tx[rb] = rem - ty * P.TW;
    rowslot[rb] = n * P.HpL + 2 * ty - Ga;
  }
  int addr[2][2][4];  // [rb][row pick][b]
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int ai = 0; ai < 2; ++ai)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int a = ai ? (I == 3 ? 3 : I == 2 ? 1 : 2) : (I == 3 ? 1 : I);
        addr[rb][ai][b] = chunk_of(rowslot[rb] + a, b & 1, 0, tx[rb] + (b >> 1), h, Qp, P.RS) * 16;
      }
  const int s_stride = Qp * 2 * 16;  // bytes from the s = 0 planes to the s = 1 planes
  // sign of the second input row of B^T row I (rows 0, 2, 3 subtract, row 1 adds)
  const _Float16 m1 = (_Float16)P.neg_one;
  const f16x8 neg = {m1, m1, m1, m1, m1, m1, m1, m1};
  const f16x8 s1 = I == 1 ? -neg : neg;

  // ---- U fragments [Cout/32][C/16][16 xi][64 lanes][8] -> this wave's LDS region by DMA:
  // 2 buffers x 8 fragments (j, cb) x 1 KiB; no registers held while they are in flight
  const int ks_total = P.C / 16;
  const __amdgpu_buffer_rsrc_t urs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(P.u), 0, 16 * P.C * P.Cout * 2, 0x00020000);
  uint8_t* ulds = smem + I * 2 * 8 * 1024;
  const int cbg0 = cblk * 2;
  auto dma_u = [&](int ks, int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const unsigned base = (unsigned)((((cbg0 + cb) * ks_total + ks) * 16 + 4 * I + j) * 1024);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            urs, (__attribute__((address_space(3))) void*)(ulds + (buf * 8 + j * 2 + cb) * 1024), 16,
            (unsigned)lane * 16u, base, 0, 0);
      }
  };

  f32x16 acc[4][2][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][rb][cb][e] = 0.f;

  dma_u(0, 0);
  u32x4 st[NS];
  for (int kk = 0; kk < KK; ++kk) {
    const uint8_t* sb = stages + (kk & 1) * stage_bytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ks = 2 * kk + s;
      // next substep's U (one past the last reads zeros: every iteration issues the same
      // number of vector-memory ops, so the counted waits below hold)
      dma_u(ks + 1, (s + 1) & 1);
      if (s == 0) {  // next K-step's input chunks in flight during this one's MFMAs
        // (exactly NS loads on every K-step, the last one's unused, never under a branch: a
        // conditional issue made the compiler's vmcnt accounting fall back to vmcnt(0) before
        // the first MFMA, exposing the whole load latency once per K-step)
#pragma unroll
        for (int it = 0; it < NS; ++it)
          st[it] = __builtin_bit_cast(
              u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, (unsigned)soff[it] + (unsigned)(kk + 1) * 64u, 0, 0));
      }
      // this substep's U landed: everything younger (its successor's 8 DMAs + NS chunks) may fly
      wait_vmcnt<NS + 8>();
      f16x8 uf[4][2];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          uf[j][cb] = *reinterpret_cast<const f16x8*>(ulds + ((s & 1) * 8 + j * 2 + cb) * 1024 + lane * 16);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        f16x8 d0[4], d1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          d0[b] = *reinterpret_cast<const f16x8*>(sb + addr[rb][0][b] + s * s_stride);
          d1[b] = *reinterpret_cast<const f16x8*>(sb + addr[rb][1][b] + s * s_stride);
        }
        f16x8 t[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) t[b] = __builtin_elementwise_fma(s1, d1[b], d0[b]);
        f16x8 v[4];
        v[0] = bt_comb<0>(t[r0_of(0)], t[r1_of(0)], neg);
        v[1] = bt_comb<1>(t[r0_of(1)], t[r1_of(1)], neg);
        v[2] = bt_comb<2>(t[r0_of(2)], t[r1_of(2)], neg);
        v[3] = bt_comb<3>(t[r0_of(3)], t[r1_of(3)], neg);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            acc[j][rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(uf[j][cb], v[j], acc[j][rb][cb], 0, 0, 0);
      }
    }
    u32x4* dst = reinterpret_cast<u32x4*>(stages + ((kk + 1) & 1) * stage_bytes);
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int e = tid + it * NT;
      if (e < chunks && kk + 1 < KK) dst[e] = bf16x8_to_f16x8(st[it]);
    }
    __syncthreads();
  }
  wait_vmcnt<0>();  // the trailing (unused) U DMA lands before the epilogue reuses the LDS
  __syncthreads();

  // ---- epilogue 1: Z_I[c] = column half of A^T M A (c = 0: M0 + M1 + M2, c = 1: M1 - M2 - M3)
  float* Zs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 z0, z1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int reg = 4 * g + e;
          const float m0 = acc[0][rb][cb][reg], m1 = acc[1][rb][cb][reg], m2 = acc[2][rb][cb][reg],
                      m3 = acc[3][rb][cb][reg];
          z0[e] = m0 + m1 + m2;
          z1[e] = m1 - m2 - m3;
        }
        const int tile = 32 * rb + r, co = 32 * cb + 8 * g + 4 * h;
        *reinterpret_cast<f32x4*>(Zs + ((I * 2 + 0) * TB + tile) * ZP + co) = z0;
        *reinterpret_cast<f32x4*>(Zs + ((I * 2 + 1) * TB + tile) * ZP + co) = z1;
      }
}

template <int ACT, int NS>
__global__ __launch_bounds__(NT, 1) void wino_f23_kernel(Params P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, wave = tid >> 6;
  // XCD-aware block map (workgroup L runs on XCD L % 8): the workgroups of one XCD share
  // output-channel blocks, so the U slice they stream (1 MiB per 64 channels at Cin 512)
  // stays in that XCD's 4 MiB L2 instead of every XCD pulling every slice from the
  // Infinity Cache
  int tblk, cblk;
  {
    const int L = blockIdx.x, X = L & 7, Q = L >> 3;
    if (P.xcd_k > 0) {  // ncb divides 8: k = 8 / ncb XCDs per channel block
      cblk = X % P.ncb;
      tblk = Q * P.xcd_k + X / P.ncb;
    } else if (P.xcd_k < 0) {  // ncb a multiple of 8: m = ncb / 8 channel blocks per XCD
      const int m = -P.xcd_k;
      cblk = X + 8 * (Q % m);
      tblk = Q / m;
    } else {
      cblk = L % P.ncb;
      tblk = L / P.ncb;
    }
    if (tblk >= P.nblk) return;  // grid rounded up to whole XCD groups (before any barrier)
  }
  const int t0 = tblk * TB;
  // staged rows: padded rows G(n, yp) = n * HpL + yp (yp = input row + 1; rows past the
  // image's 2 TH + 2 are pitch padding, never read), from the first tile's top row to the
  // last tile's bottom row
  const int per = P.TH * P.TW;
  const int ta = t0, tb = min(t0 + TB - 1, P.T - 1);
  const int na = fdiv(ta, P.d_per), tya = fdiv(ta - na * per, P.d_tw);
  const int nb = fdiv(tb, P.d_per), tyb = fdiv(tb - nb * per, P.d_tw);
  const int Ga = na * P.HpL + 2 * tya;
  const int nrows = nb * P.HpL + 2 * tyb + 4 - Ga;
  const int chunks = nrows * P.RS;  // <= P.stage_chunks (host-checked)

  // per-thread staged chunk sources (byte offsets for K-step 0; out-of-image -> past the end)
  int soff[SMAX];
#pragma unroll
  for (int it = 0; it < SMAX; ++it) {
    const int e = tid + it * NT;
    unsigned off = 0x80000000u;
    if (e < chunks) {
      const int j = fdiv(e, P.d_rs), rem = e - j * P.RS;
      int plane = 0;  // rem / Qp without a divide (plane >= 8: the row's pad)
#pragma unroll
      for (int k = 1; k <= 8; ++k) plane += rem >= k * P.Qp;
      const int q = rem - plane * P.Qp;
      const int hh = plane & 1, s = (plane >> 1) & 1, p = plane >> 2;
      const int G = Ga + j;
      const int n = fdiv(G, P.d_hpl), yp = G - n * P.HpL;
      const int yy = yp - 1, xx = 2 * q + p - 1;
      if (plane < 8 && n < P.N && (unsigned)yy < (unsigned)P.H && (unsigned)xx < (unsigned)P.W)
        off = (unsigned)((((n * P.H + yy) * P.W + xx) * P.C + 16 * s + 8 * hh) * 2);
    }
    soff[it] = (int)off;
  }
  {  // stage 0
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(P.x), 0, P.N * P.H * P.W * P.C * 2, 0x00020000);
    u32x4* dst = reinterpret_cast<u32x4*>(smem + U_LDS);
#pragma unroll
    for (int it = 0; it < SMAX; ++it) {
      const int e = tid + it * NT;
      if (e < chunks)
        dst[e] = bf16x8_to_f16x8(
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, (unsigned)soff[it], 0, 0)));
    }
  }
  __syncthreads();
  wave_body<NS>(P, smem, soff, chunks, Ga, t0, __builtin_amdgcn_readfirstlane(wave), cblk);
  __syncthreads();

  // ---- epilogue 2: Y[rr][cc] = (rr = 0: Z0 + Z1 + Z2 | rr = 1: Z1 - Z2 - Z3)[cc]; + bias, act
  const float* Zs = reinterpret_cast<const float*>(smem);
  const int co_base = cblk * CB;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int uidx = tid + k * NT;
    const int T = uidx >> 3, c8 = (uidx & 7) * 8;
    const int t = t0 + T;
    if (t >= P.T) continue;
    float z[4][2][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float* src = Zs + ((i * 2 + c) * TB + T) * ZP + c8;
        const f32x4 a = *reinterpret_cast<const f32x4*>(src);
        const f32x4 b = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          z[i][c][e] = a[e];
          z[i][c][4 + e] = b[e];
        }
      }
    float bv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = P.bias[co_base + c8 + e];
    const int n = fdiv(t, P.d_per), rem = t - n * per;
    const int ty = fdiv(rem, P.d_tw), tx = rem - ty * P.TW;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int oy = 2 * ty + rr, ox = 2 * tx + cc;
        if (oy >= P.H || ox >= P.W) continue;
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = rr == 0 ? z[0][cc][e] + z[1][cc][e] + z[2][cc][e] : z[1][cc][e] - z[2][cc][e] - z[3][cc][e];
          o[e] = f2bf(apply_act<ACT>(v + bv[e]));
        }
        *reinterpret_cast<bf16x8*>(P.y + ((size_t)(n * P.H + oy) * P.W + ox) * P.ldy + P.y_coff + co_base + c8) = o;
      }
  }
}

template <int NS>
void launch_wino(const Params& P, int Cout, int act, size_t lds, uintptr_t stream) {
  int nb = P.nblk;
  if (P.xcd_k > 0) nb = (nb + P.xcd_k - 1) / P.xcd_k * P.xcd_k;
  dim3 grid(nb * P.ncb);
  auto s = reinterpret_cast<hipStream_t>(stream);
  if (act == ACT_RELU) {
    (void)hipFuncSetAttribute((const void*)wino_f23_kernel<ACT_RELU, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    hipLaunchKernelGGL((wino_f23_kernel<ACT_RELU, NS>), grid, dim3(NT), lds, s, P);
  } else {
    (void)hipFuncSetAttribute((const void*)wino_f23_kernel<ACT_NONE, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    hipLaunchKernelGGL((wino_f23_kernel<ACT_NONE, NS>), grid, dim3(NT), lds, s, P);
  }
}

struct Layout {
  int RS, HpL, rows;
};

// Rows of padded input (LDS image pitch HpL) the worst 64-tile block of a layer stages.
int max_rows(int N, int H, int W, int HpL) {
  const int TH = (H + 1) / 2, TW = (W + 1) / 2, per = TH * TW, T = N * per;
  int worst = 0;
  for (int t0 = 0; t0 < T; t0 += TB) {
    const int ta = t0, tb = t0 + TB - 1 < T - 1 ? t0 + TB - 1 : T - 1;
    const int na = ta / per, tya = (ta - na * per) / TW;
    const int nb = tb / per, tyb = (tb - nb * per) / TW;
    const int rows = nb * HpL + 2 * tyb + 4 - (na * HpL + 2 * tya);
    if (rows > worst) worst = rows;
  }
  return worst;
}

// Mean LDS cycles per ds_read_b128 lane group of the patch reads over a sample of blocks
// (1 = conflict-free): the 16-lane groups {0-3,12-15,20-27} / {4-11,16-19,28-31} of the
// 32 tile lanes, bank group = chunk mod 16.
double conflict_score(int N, int H, int W, int RS, int HpL) {
  static const int grp[2][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31}};
  const int TH = (H + 1) / 2, TW = (W + 1) / 2, per = TH * TW, T = N * per, Qp = TW + 1;
  const int nblk = (T + TB - 1) / TB, step = nblk > 48 ? nblk / 48 : 1;
  double cyc = 0;
  long cnt = 0;
  for (int blk = 0; blk < nblk; blk += step) {
    const int t0 = blk * TB;
    const int na = t0 / per, tya = (t0 - na * per) / TW, Ga = na * HpL + 2 * tya;
    for (int rb = 0; rb < 2; ++rb)
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b)
          for (int g = 0; g < 2; ++g) {
            int addr[16], bank[16];
            for (int i = 0; i < 16; ++i) {
              int t = t0 + 32 * rb + grp[g][i];
              if (t > T - 1) t = T - 1;
              const int n = t / per, rem = t - n * per, ty = rem / TW, tx = rem - ty * TW;
              addr[i] = (n * HpL + 2 * ty - Ga + a) * RS + (b & 1) * 4 * Qp + tx + (b >> 1);
              bank[i] = addr[i] & 15;
            }
            int worst = 1;
            for (int i = 0; i < 16; ++i) {
              int k = 0;
              for (int j = 0; j < 16; ++j) {
                bool dup = false;  // distinct addresses only (a broadcast is free)
                for (int m = 0; m < j; ++m) dup = dup || (addr[m] == addr[j] && bank[m] == bank[i]);
                k += bank[j] == bank[i] && !dup;
              }
              if (k > worst) worst = k;
            }
            cyc += worst;
            ++cnt;
          }
  }
  return cyc / cnt;
}

// Row pad e (RS = 8 Qp + e) and image row pitch HpL >= 2 TH + 2 with the fewest LDS bank
// conflicts whose stage fits the per-thread staging registers and the LDS left next to U.
Layout choose_layout(int N, int H, int W) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int>, Layout> memo;
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_tuple(N, H, W);
  auto it = memo.find(key);
  if (it != memo.end()) return it->second;
  const int TH = (H + 1) / 2, TW = (W + 1) / 2, Qp = TW + 1, Hp = 2 * TH + 2;
  const int max_chunks = std::min(SMAX * NT, (160 * 1024 - U_LDS) / 32);
  Layout best{-1, -1, -1};
  double best_score = 1e30;
  for (int HpL = Hp; HpL <= Hp + 16; ++HpL) {
    const int rows = max_rows(N, H, W, HpL);
    for (int e = 0; e < 16; ++e) {
      const int RS = 8 * Qp + e;
      if (rows * RS > max_chunks) continue;
      // small preference for compact stages at equal conflict levels
      const double sc = conflict_score(N, H, W, RS, HpL) + 1e-6 * rows * RS;
      if (sc < best_score) {
        best_score = sc;
        best = Layout{RS, HpL, rows};
      }
    }
  }
  return memo[key] = best;
}

}  // namespace

// staged rows and chunks per row of the chosen layout (-1: the layer does not fit)
pybind11::tuple wino_f23_layout(int N, int H, int W) {
  const Layout L = choose_layout(N, H, W);
  return pybind11::make_tuple(L.rows, L.RS, L.HpL);
}

// x [N, H, W, C] bf16, u = fp16 U fragments [Cout/32][C/16][16][64][8] (wino_f23_weights),
// bias [Cout] fp32, y [N, H, W, ldy] bf16 at channel offset y_coff.  3x3, stride 1, pad 1.
void wino_f23_bf16(uintptr_t x, uintptr_t u, uintptr_t bias, uintptr_t y, int N, int H, int W, int C, int Cout,
                   int ldy, int y_coff, int act, uintptr_t stream) {
  if (C % 32 || Cout % CB || C < 32) throw std::invalid_argument("wino_f23: needs C % 32 == 0 and Cout % 64 == 0");
  if (ldy % 8 || y_coff % 8 || ldy < y_coff + Cout) throw std::invalid_argument("wino_f23: bad output stride/offset");
  if ((long)N * H * W * C * 2 >= (1L << 31) - 4096 || (long)N * H * W * ldy >= (1L << 31))
    throw std::invalid_argument("wino_f23: tensor too large for 32-bit offsets");
  if (!x || !u || !bias || !y || x % 16 || u % 16 || y % 16 || bias % 16)
    throw std::invalid_argument("wino_f23: null or misaligned pointer");
  Params P;
  P.x = reinterpret_cast<const bf16*>(x);
  P.u = reinterpret_cast<const _Float16*>(u);
  P.bias = reinterpret_cast<const float*>(bias);
  P.y = reinterpret_cast<bf16*>(y);
  P.N = N;
  P.H = H;
  P.W = W;
  P.C = C;
  P.Cout = Cout;
  P.TH = (H + 1) / 2;
  P.TW = (W + 1) / 2;
  P.T = N * P.TH * P.TW;
  P.Qp = P.TW + 1;
  const Layout L = choose_layout(N, H, W);
  if (L.RS < 0)
    throw std::invalid_argument("wino_f23: a 64-tile block of a " + std::to_string(W) +
                                "-wide image stages more than the kernel's LDS / staging registers hold");
  P.RS = L.RS;
  P.HpL = L.HpL;
  P.stage_chunks = L.rows * L.RS;
  P.neg_one = -1.0f;
  P.nblk = (P.T + TB - 1) / TB;
  P.ncb = Cout / CB;
  P.xcd_k = 8 % P.ncb == 0 ? 8 / P.ncb : P.ncb % 8 == 0 ? -(P.ncb / 8) : 0;
  auto mk = [](int d, long xmax) {
    if (d <= 0 || xmax * (long)d >= (1L << 32)) throw std::invalid_argument("wino_f23: fast-divide range");
    return FDiv{(uint32_t)(((1ULL << 32) + d - 1) / d), d};
  };
  const int per = P.TH * P.TW;
  P.d_per = mk(per, P.T + TB);
  P.d_tw = mk(P.TW, per);
  P.d_rs = mk(P.RS, P.stage_chunks + SMAX * NT);
  P.d_hpl = mk(P.HpL, (long)(N + 1) * P.HpL + 8);
  P.ldy = ldy;
  P.y_coff = y_coff;
  const size_t lds = (size_t)U_LDS + 2 * P.stage_chunks * 16 > (size_t)Z_BYTES ? (size_t)U_LDS + 2 * P.stage_chunks * 16
                                                                              : (size_t)Z_BYTES;
  if (lds > 160 * 1024) throw std::invalid_argument("wino_f23: LDS stage too large");
  if (act != ACT_RELU && act != ACT_NONE) throw std::invalid_argument("wino_f23: act must be none or relu");
  const int need = (P.stage_chunks + NT - 1) / NT;  // staged chunks per thread, rounded up to 4 / 8 / 12
  if (need <= 4) launch_wino<4>(P, Cout, act, lds, stream);
  else if (need <= 8) launch_wino<8>(P, Cout, act, lds, stream);
  else launch_wino<12>(P, Cout, act, lds, stream);
  FTM_CHECK_LAUNCH();
}

void register_wino3x3(pybind11::module_& m) {
  m.def("wino_f23_bf16", &wino_f23_bf16);
  m.def("wino_f23_layout", &wino_f23_layout);
}
