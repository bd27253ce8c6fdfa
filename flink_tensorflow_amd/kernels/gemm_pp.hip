// Ping-pong 256x256 bf16 GEMM for CDNA4 (gfx950): the hot-path GEMM of the framework
// (transformer projections / FFN, deep-K 1x1 convolutions, classifier heads).
//
//   y[m, yoff + n] = act(x[m, :] . w[n, :] + bias[n] (+ res[m, n]))     bf16 in, fp32 acc
//
// Structure (guide §5 "The 256² 8-phase template", T1-T5):
// * 256 x 256 output tile, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns
//   128 x 64 outputs = 2 x 2 quadrants of 64 x 32, i.e. 32 v_mfma_f32_16x16x32_bf16 tiles
//   (128 accumulator registers).
// * Both operands stream global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into two
//   64 KiB stages.  A stage is split into four 16 KiB "half-tiles" (A rows of quadrant-row
//   0 / 1 of both wave rows, W rows of quadrant-column 0 / 1 of all four wave columns) so
//   that each half-tile is consumed inside ONE phase; it is restaged for the K-tile two
//   ahead as soon as that phase's reads retired.  One half-tile DMA per phase, counted
//   `vmcnt(6)` once per K-tile: three half-tiles stay in flight across every barrier.
// * Four phases per K-tile, one 64x32 quadrant x K=64 (16 MFMA) each:
//     P1 read W(nh0) + X(mh0) -> Q00 | P2 read W(nh1) -> Q01 | P3 read X(mh1) -> Q11 | P4 -> Q10
//   (W fragments of both column halves stay in registers through the K-tile).
// * Ping-pong: wave row 1 (waves 4-7, one per SIMD) starts one barrier late, so on every
//   SIMD one wave runs its MFMA cluster while its partner issues ds_reads and DMA.
// * LDS images are lane-linear per DMA instruction (8 rows x 128 B); the XOR swizzle
//   (16-B chunk ^ (row & 7)) is applied on the per-lane SOURCE address and on the
//   ds_read_b128 address (rule 21) -> conflict-free fragment reads.
// * XCD-aware bijective tile remap (T1).  M / N tails clamp the source row (the extra
//   rows / columns are computed and never stored); K must be a multiple of 64.
// * MFMA operand order is (W fragment, X fragment), so the accumulator holds D^T: each
//   lane owns 4 consecutive output columns of one row -> 8-B LDS writes in the epilogue
//   and 16-B fp32 stores in split-K mode.
// * Epilogue: + bias, act -> bf16 tile in LDS -> 16-B coalesced row segments (+ residual,
//   act) -> global.  SPLIT mode writes raw fp32 partial tiles instead (K range per
//   blockIdx.y); `gemm_pp_reduce` sums the slices and applies bias / residual / act.
#include <pybind11/pybind11.h>

#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <string>

#include "common.h"

namespace {

constexpr int NT = 512;
constexpr int HT = 128 * 128;        // half-tile: 128 image rows x 128 B
constexpr int STG = 4 * HT;          // one K-tile: X_h0 X_h1 W_h0 W_h1
constexpr int OPITCH = 512 + 16;     // epilogue LDS row pitch: 256 bf16 + 16 B pad
constexpr int LDS_MAIN = 2 * STG;
constexpr int LDS_EPI = 256 * OPITCH;
constexpr int LDS_BYTES = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

struct PPParams {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  void* y;
  int M, N, K;
  int ldx, ldw, ldy, y_coff, ldr;
  int tiles_m, tiles_n;
  int kt_per_split;   // K tiles per blockIdx.y slice (SPLIT mode)
  long split_stride;  // fp32 elements between partial slices (SPLIT mode)
};

#define PP_FENCE() __builtin_amdgcn_sched_barrier(0)
#define PP_BARRIER()                              \
  do {                                            \
    PP_FENCE();                                   \
    asm volatile("s_barrier" ::: "memory");      \
    PP_FENCE();                                   \
  } while (0)

// One 256x256 output tile (``tile`` = remapped tile index; SPLIT: K slice blockIdx.y).
template <int ACT, bool HAS_RES, bool SPLIT>
__device__ __forceinline__ void pp_tile(const PPParams& p, uint8_t* smem, const int tile) {
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * 256;
  const int n0 = tn * 256;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave >> 2;  // wave row: output rows g*128 .. +128 (also the ping-pong group)
  const int wc = wave & 3;  // wave column: output cols wc*64 .. +64

  // K range of this block (SPLIT: blockIdx.y selects a slice of K tiles)
  const int nk_all = p.K >> 6;
  int kt0 = 0, nk = nk_all;
  if constexpr (SPLIT) {
    kt0 = blockIdx.y * p.kt_per_split;
    nk = min(p.kt_per_split, nk_all - kt0);
  }

  // ---- DMA roles.  Per half-tile each wave writes image rows 16*wave + 8*q + (lane>>3),
  // q = 0, 1; the source chunk is pre-swizzled so LDS chunk c of row r holds global chunk
  // c ^ (r & 7).  Buffer loads (SRD in SGPRs, 32-bit per-lane offsets, the K step in the
  // scalar offset); rows past M / N fall outside the descriptor's range and read zeros.
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.x, 0, (int)((unsigned)p.M * (unsigned)p.ldx * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.w, 0, (int)((unsigned)p.N * (unsigned)p.ldw * 2u), 0x00020000);
  unsigned offx[2][2], offw[2][2];  // [half][q] byte offsets of this lane's source chunk
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = 16 * wave + 8 * q + drow;  // image row 0..127
      const unsigned m = m0 + (r >> 6) * 128 + h * 64 + (r & 63);
      offx[h][q] = m < (unsigned)p.M ? (m * p.ldx + dchunk * 8) * 2u : 0x80000000u;
      const unsigned n = n0 + (r >> 5) * 64 + h * 32 + (r & 31);
      offw[h][q] = n < (unsigned)p.N ? (n * p.ldw + dchunk * 8) * 2u : 0x80000000u;
    }
  }
  // kind: 0 = X_h0, 1 = X_h1, 2 = W_h0, 3 = W_h1
  auto dma = [&](int kind, int kt, int stage) {
    uint8_t* base = smem + stage * STG + kind * HT + 16 * wave * 128;
    const unsigned soff = (unsigned)(kt0 + kt) * 128u;
    const __amdgpu_buffer_rsrc_t r = kind < 2 ? rx : rw;
    const unsigned* o = kind < 2 ? offx[kind] : offw[kind - 2];
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)base, 16, o[0], soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(base + 8 * 128), 16, o[1],
                                             soff, 0, 0);
  };

  // ---- fragment read offsets (bytes, relative to a half-tile): row (lane & 15) of a
  // 16-row subtile, k chunk 4*ks + (lane >> 4), swizzled by (row & 7) == (lane & 7)
  const int frow = lane & 15;
  const int fx_row = (g * 64 + frow) * 128;    // X image: wave row g, quadrant row mh
  const int fw_row = (wc * 32 + frow) * 128;   // W image: wave col wc, quadrant col nh
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

  bf16x8 fx[2][4];     // [ks][i]   X fragments of the current quadrant row
  bf16x8 fw[2][2][2];  // [nh][ks][j] W fragments of both quadrant columns

  auto read_x = [&](int stage, int mh) {
    const uint8_t* b = smem + stage * STG + mh * HT + fx_row;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fx[0][i] = *reinterpret_cast<const bf16x8*>(b + i * 16 * 128 + fc0);
      fx[1][i] = *reinterpret_cast<const bf16x8*>(b + i * 16 * 128 + fc1);
    }
  };
  auto read_w = [&](int stage, int nh) {
    const uint8_t* b = smem + stage * STG + (2 + nh) * HT + fw_row;
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

  // One K-tile (local index t, LDS stage S) = four phases.  Loads: P1 -> X_h1 of tile t+1
  // (other stage); P2..P4 -> W_h0, X_h0, W_h1 of tile t+2 (this stage).
  auto ktile = [&](int t, auto S_) {
    constexpr int S = decltype(S_)::value;
    const bool pre1 = t + 1 < nk;
    const bool pre2 = t + 2 < nk;
    // P1
    read_w(S, 0);
    PP_FENCE();
    read_x(S, 0);
    if (pre1) dma(1, t + 1, S ^ 1);
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");  // W_h0 reads retired: restaged in P2
    PP_BARRIER();
    mfma_q(0, 0);
    PP_BARRIER();
    // P2
    read_w(S, 1);
    if (pre2) dma(2, t + 2, S);
    PP_BARRIER();
    mfma_q(0, 1);
    PP_BARRIER();
    // P3
    read_x(S, 1);
    if (pre2) dma(0, t + 2, S);
    PP_BARRIER();
    mfma_q(1, 1);
    PP_BARRIER();
    // P4: retire tile t+1 (all but the three half-tiles of tile t+2 just issued)
    if (pre2) {
      dma(3, t + 2, S);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    PP_BARRIER();
    mfma_q(1, 0);
    PP_BARRIER();
  };

  // ---- prologue: tile 0 whole, tile 1 except X_h1 (issued by tile 0's P1)
  dma(2, 0, 0);
  dma(0, 0, 0);
  dma(3, 0, 0);
  dma(1, 0, 0);
  if (nk > 1) {
    dma(2, 1, 1);
    dma(0, 1, 1);
    dma(3, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  PP_BARRIER();
  if (g == 1) PP_BARRIER();  // ping-pong: wave row 1 runs one barrier behind

  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  if (g == 0) PP_BARRIER();
  __syncthreads();  // every wave past its last LDS read and DMA wait: LDS is free

  const int fq = lane >> 4;
  if constexpr (SPLIT) {
    // raw fp32 partial tile: lane owns 4 consecutive columns of one row (16-B stores)
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
    // ---- epilogue 1: + bias, act (unless a residual follows) -> bf16 tile in LDS
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
            *reinterpret_cast<bf16x4*>(smem + ml * OPITCH + nl * 2) = o;
          }
      }
    __syncthreads();
    // ---- epilogue 2: 16-B row segments (+ residual, act) -> global
    bf16* y = reinterpret_cast<bf16*>(p.y);
#pragma unroll 4
    for (int q = threadIdx.x; q < 256 * 32; q += NT) {
      const int ml = q >> 5;
      const int cc = q & 31;
      const int m = m0 + ml;
      const int n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + ml * OPITCH + cc * 16);
      if constexpr (HAS_RES) {
        bf16x8 o = __builtin_bit_cast(bf16x8, v);
        const bf16x8 r = *reinterpret_cast<const bf16x8*>(p.res + (size_t)m * p.ldr + n);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if constexpr (ACT == ACT_DRELU) o[e] = (float)r[e] > 0.f ? o[e] : f2bf(0.f);
          else o[e] = f2bf(apply_act<ACT>((float)o[e] + (float)r[e]));
        }
        v = __builtin_bit_cast(u32x4, o);
      }
      *reinterpret_cast<u32x4*>(y + (size_t)m * p.ldy + p.y_coff + n) = v;
    }
  }
}

template <int ACT, bool HAS_RES, bool SPLIT>
__global__ __launch_bounds__(NT, 1) void gemm_pp_kernel(PPParams p) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS_BYTES];
  pp_tile<ACT, HAS_RES, SPLIT>(p, smem, xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n));
}

// Split-K reduction: y = act(sum_s part[s] + bias (+ res)), 8 columns per thread.
template <int ACT, bool HAS_RES>
__global__ __launch_bounds__(256) void gemm_pp_reduce_kernel(const float* __restrict__ part, int splits,
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
    for (int e = 0; e < 8; ++e) {
      if constexpr (ACT == ACT_DRELU) v[e] = (float)r[e] > 0.f ? v[e] : 0.f;
      else v[e] += (float)r[e];
    }
  }
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(apply_act<ACT>(v[e]));
  *reinterpret_cast<bf16x8*>(y + (size_t)m * ldy + y_coff + n) = o;
}

template <int ACT, bool HAS_RES>
void launch_pp(const PPParams& p, int splits, float* ws, hipStream_t s) {
  dim3 block(NT);
  const int tiles = p.tiles_m * p.tiles_n;
  if (splits <= 1) {
    hipLaunchKernelGGL((gemm_pp_kernel<ACT, HAS_RES, false>), dim3(tiles), block, 0, s, p);
    return;
  }
  PPParams q = p;
  q.y = ws;
  dim3 grid(tiles, splits);
  hipLaunchKernelGGL((gemm_pp_kernel<ACT_NONE, false, true>), grid, block, 0, s, q);
  const long work = (long)p.M * (p.N >> 3);
  hipLaunchKernelGGL((gemm_pp_reduce_kernel<ACT, HAS_RES>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                     ws, splits, p.split_stride, p.bias, p.res, p.ldr, reinterpret_cast<bf16*>(p.y), p.ldy, p.y_coff,
                     p.M, p.N);
}

template <int ACT>
void launch_res(const PPParams& p, int splits, float* ws, hipStream_t s) {
  if (p.res) launch_pp<ACT, true>(p, splits, ws, s);
  else launch_pp<ACT, false>(p, splits, ws, s);
}

void check_align(uintptr_t ptr, int bytes, const char* what) {
  if (ptr % bytes) throw std::invalid_argument(std::string("gemm_pp: ") + what + " is not " + std::to_string(bytes) + "-byte aligned");
}

}  // namespace

// y[:, y_coff:y_coff+N] = act(x @ w^T + bias (+ res)).  x [M, ldx] bf16, w [N, ldw] bf16
// (K-contiguous rows), bias fp32 [N] or 0, res bf16 [M, ldr] or 0, y bf16 [M, ldy].
// splits > 1: split-K over `splits` slices of K tiles into the fp32 workspace `ws`
// (splits * M * N floats), then one reduction kernel.
void gemm_pp(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int M, int N, int K, int ldx,
             int ldw, int ldy, int y_coff, int ldr, int act, int splits, uintptr_t ws, uintptr_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) throw std::invalid_argument("gemm_pp: empty problem");
  if (K % 64) throw std::invalid_argument("gemm_pp: K must be a multiple of 64");
  if (N % 8 || ldy % 8 || y_coff % 8 || ldx % 8 || ldw % 8) throw std::invalid_argument("gemm_pp: N/ld alignment (8)");
  if (res && ldr % 8) throw std::invalid_argument("gemm_pp: ldr alignment (8)");
  if ((long)M * ldx * 2 >= (1L << 31) || (long)N * ldw * 2 >= (1L << 31))
    throw std::invalid_argument("gemm_pp: operand larger than 2 GiB (split M on the host)");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  if (bias) check_align(bias, 16, "bias");
  if (res) check_align(res, 16, "res");
  const int nk = K / 64;
  if (splits < 1) splits = 1;
  if (splits > nk) splits = nk;
  PPParams p{};
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const bf16*>(res);
  p.y = reinterpret_cast<void*>(y);
  p.M = M; p.N = N; p.K = K;
  p.ldx = ldx; p.ldw = ldw; p.ldy = ldy; p.y_coff = y_coff; p.ldr = ldr;
  p.tiles_m = (M + 255) / 256;
  p.tiles_n = (N + 255) / 256;
  if (splits > 1) {
    // even split of the K tiles; the slice count is recomputed so none is empty
    p.kt_per_split = (nk + splits - 1) / splits;
    splits = (nk + p.kt_per_split - 1) / p.kt_per_split;
    p.split_stride = (long)M * N;
    if (!ws) throw std::invalid_argument("gemm_pp: split-K needs a workspace");
    check_align(ws, 16, "ws");
  }
  float* wsp = reinterpret_cast<float*>(ws);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (act) {
    case ACT_NONE: launch_res<ACT_NONE>(p, splits, wsp, s); break;
    case ACT_RELU: launch_res<ACT_RELU>(p, splits, wsp, s); break;
    case ACT_GELU_TANH: launch_res<ACT_GELU_TANH>(p, splits, wsp, s); break;
    case ACT_TANH: launch_res<ACT_TANH>(p, splits, wsp, s); break;
    case ACT_DRELU:
      if (!res) throw std::invalid_argument("gemm_pp: the drelu epilogue needs the mask operand (res)");
      launch_pp<ACT_DRELU, true>(p, splits, wsp, s);
      break;
    default: throw std::invalid_argument("gemm_pp: unsupported activation");
  }
  FTM_CHECK_LAUNCH();
}

// Number of K-slices `gemm_pp` would actually run for a requested split count.
int gemm_pp_splits(int K, int splits) {
  const int nk = K / 64;
  if (splits <= 1 || nk <= 1) return 1;
  if (splits > nk) splits = nk;
  const int per = (nk + splits - 1) / splits;
  return (nk + per - 1) / per;
}

void register_gemm_pp(pybind11::module_& m) {
  m.def("gemm_pp", &gemm_pp);
  m.def("gemm_pp_splits", &gemm_pp_splits);
}
