// Layout-general 128x128 bf16 MFMA GEMM for training steps (forward NT, backward NN / TN).
//
//   y[m, n] = epi( sum_k X(m, k) W(n, k) )         bf16 in, fp32 accumulate
//   X(m, k) = x[m*ldx + k]  (row)   or  x[k*ldx + m]  (x_t: K-major, e.g. dA^T of dW = dA^T H)
//   W(n, k) = w[n*ldw + k]  (row)   or  w[k*ldw + n]  (w_t: K-major, e.g. W of dX = dA W)
//
// The three GEMMs of a dense layer's training step read their operands in every layout:
// forward x W^T (both K-contiguous), dX = dA W (W K-major), dW = dA^T X (both K-major).
// gemm_pp (the 256x256 inference GEMM) needs K-contiguous operands; here a K-major
// operand is staged as a [k][128] LDS image and fed to the MFMA with the hardware
// transpose read ds_read_b64_tr_b16 (guide T10), so no transposed copy is ever made.
//
// * 128 x 128 tile, BK = 64, 256 threads = 4 waves as 2 (M) x 2 (N); each wave owns 64 x 64
//   outputs = 4 x 4 v_mfma_f32_16x16x32_bf16 tiles.  64 KiB of LDS (two stages of X + W
//   tiles): two workgroups per CU.  Training problems are small (4096 rows), so the small
//   tile is what fills 256 CUs; deep-K weight gradients add split-K.
// * Both operands stream global -> LDS by LDS-DMA (buffer_load ... lds, 16 B per lane),
//   lane-linear images with the swizzle applied on the per-lane SOURCE address (rule 21):
//   - K-contiguous: 128 rows x 128 B, chunk ^= row & 7, fragments by ds_read_b128;
//   - K-major:      64 k-rows x 256 B, 16-B chunk ^= 2*g(row), g = (row&3) | ((row>>3)&1)<<2
//     — each 32-lane half of a transposed read then covers 8 rows x 32 B on 8 distinct
//     chunk pairs: all 64 banks once, conflict-free.
// * 2-phase pipeline (guide T3 minimum form): the next K-tile's DMA is issued before the
//   current tile's fragment reads + 32 MFMAs, one vmcnt(0) + barrier per K-tile.
// * MFMA operand order (W fragment, X fragment): the accumulator holds D^T, so a lane owns 4
//   consecutive output columns of one row (16-B fp32 stores, 8-B bf16 LDS writes).
// * Epilogues: bf16 (+bias, act, or the ReLU-backward mask ACT_DRELU with `res` = the layer
//   input) through an LDS tile into 16-B row segments; fp32 (weight gradients) stored
//   directly; split-K writes fp32 slabs reduced by gemm_train_reduce (fixed order:
//   deterministic, no atomics).
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int TILE = 128 * 128;       // one operand tile: 128 x 64 bf16 (either image)
constexpr int STAGE = 2 * TILE;       // X tile + W tile
constexpr int OPITCH = 128 * 2 + 16;  // bf16 epilogue row pitch (bytes)
constexpr int LDS_EPI = 128 * OPITCH;
constexpr int LDS_RED = 4 * 16 * 8 * 4;  // column-sum partials after the epilogue tile
// STAGES = 2: 64 KiB, two workgroups per CU (grids wider than the chip); STAGES = 4: 128
// KiB, one workgroup per CU with three K tiles in flight across every barrier (small
// grids, where nothing else hides the DMA latency)
template <int STAGES>
constexpr int lds_bytes() {
  return STAGES * STAGE > LDS_EPI + LDS_RED ? STAGES * STAGE : LDS_EPI + LDS_RED;
}
static_assert(lds_bytes<2>() <= 64 * 1024, "two workgroups per CU");
static_assert(lds_bytes<4>() <= 160 * 1024, "LDS budget");

typedef short v4s __attribute__((ext_vector_type(4)));

struct TrParams {
  const bf16* x;
  const bf16* w;
  const float* bias;
  const bf16* res;
  void* y;
  float* colsum;      // bf16 epilogue: per-tile column sums [tiles_m][N] of the stored values
  int M, N, K;
  int ldx, ldw, ldy, ldr;
  int tiles_m, tiles_n;
  int kt_per_split;   // K tiles per blockIdx.y slice (split-K)
  long split_stride;  // fp32 elements between partial slabs
};

#define TR_BARRIER()                           \
  do {                                         \
    __builtin_amdgcn_sched_barrier(0);         \
    asm volatile("s_barrier" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);         \
  } while (0)

FTM_DEVICE bf16x8 tr_pair(const uint8_t* a0, const uint8_t* a1) {
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a1);
  const v4s v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v);
}

// One operand's staging + fragment reads.  ``T`` = K-major global layout.
template <bool T>
struct Operand {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned off[4];   // per-lane source byte offsets of this wave's 4 DMA instructions
  unsigned off_tail[4];  // K-contiguous: the same for the last, partial K tile (chunks >= K read 0)
  unsigned kstep;    // bytes per K-tile (scalar offset increment)
  int last_kt;       // index of a partial last K tile (K % 64 != 0), else -1

  FTM_DEVICE void init(const bf16* base, int rows_total, int ld, int mn0, int mn_total, int K, int wave, int lane) {
    if constexpr (!T) {
      // image row r (0..127) = operand row mn0 + r, 8 chunks of 16 B (64 k)
      rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)((unsigned)rows_total * (unsigned)ld * 2u),
                                               0x00020000);
      const int chunk = (lane & 7) ^ (lane >> 3);
      const int tail = (K & 63) >> 3;  // valid 16-B chunks of a partial last K tile
      last_kt = tail ? (K >> 6) : -1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned r = 32 * wave + 8 * q + (lane >> 3);
        const unsigned m = mn0 + r;
        off[q] = m < (unsigned)mn_total ? (m * ld + chunk * 8) * 2u : 0x80000000u;
        off_tail[q] = chunk < tail ? off[q] : 0x80000000u;
      }
      kstep = 128u;
    } else {
      // image row r (0..63) = k row, 16 chunks of 16 B (128 m / n)
      rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)((unsigned)K * (unsigned)ld * 2u), 0x00020000);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned r = 16 * wave + 4 * q + (lane >> 4);
        const int g = (lane >> 4) | ((q >> 1) << 2);  // (r & 3) | ((r >> 3) & 1) << 2
        const int chunk = (lane & 15) ^ (2 * g);
        off[q] = (r * ld + mn0 + chunk * 8) * 2u;
      }
      kstep = 64u * (unsigned)ld * 2u;
      last_kt = -1;  // k rows >= K lie past the descriptor's range: they read 0
    }
  }

  FTM_DEVICE void dma(uint8_t* tile, int wave, int kt) const {
    const unsigned soff = (unsigned)kt * kstep;
    constexpr int ROWB = T ? 4 * 256 : 8 * 128;  // image bytes per DMA instruction
    uint8_t* b = tile + wave * 4 * ROWB;
    const unsigned* o = off;
    if constexpr (!T) {
      if (kt == last_kt) o = off_tail;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(b + q * ROWB), 16, o[q],
                                               soff, 0, 0);
  }

  // fragment of subtile rows/cols [c0, c0+16) x k-slice ks (32 deep) for lane
  FTM_DEVICE bf16x8 frag(const uint8_t* tile, int c0, int ks, int lane) const {
    if constexpr (!T) {
      const int r = c0 + (lane & 15);
      const int chunk = 4 * ks + (lane >> 4);
      return *reinterpret_cast<const bf16x8*>(tile + r * 128 + ((chunk ^ (lane & 7)) << 4));
    } else {
      const int idx = lane & 15, q = idx >> 2, p = idx & 3, G = lane >> 4;
      const int g = q | ((G & 1) << 2);
      const int chunk = ((c0 >> 3) + (p >> 1)) ^ (2 * g);
      const int r0 = 32 * ks + 8 * G + q;
      const uint8_t* a0 = tile + r0 * 256 + (chunk << 4) + (p & 1) * 8;
      return tr_pair(a0, a0 + 4 * 256);  // rows r0 and r0 + 4: same g -> same chunk
    }
  }
};

template <bool XT, bool WT, int ACT, bool F32, bool HAS_RES, bool SPLIT, int STAGES>
__global__ __launch_bounds__(NT, STAGES == 2 ? 2 : 1) void gemm_train_kernel(TrParams p) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[lds_bytes<STAGES>()];
  const int tile = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int m0 = tm * 128, n0 = tn * 128;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int nk_all = (p.K + 63) >> 6;
  int kt0 = 0, nk = nk_all;
  if constexpr (SPLIT) {
    kt0 = blockIdx.y * p.kt_per_split;
    nk = min(p.kt_per_split, nk_all - kt0);
  }

  Operand<XT> ox;
  Operand<WT> ow;
  ox.init(p.x, p.M, p.ldx, m0, p.M, p.K, wave, lane);
  ow.init(p.w, p.N, p.ldw, n0, p.N, p.K, wave, lane);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int kt, int s) {
    ox.dma(smem + s * STAGE, wave, kt0 + kt);
    ow.dma(smem + s * STAGE + TILE, wave, kt0 + kt);
  };

  // K tiles t+1 .. t+STAGES-1 are in flight while tile t is consumed; 8 DMA instructions
  // per wave per K tile, so "tile t+1 has landed" is vmcnt(8 * tiles issued after it)
  auto wait_next = [&](int after) {  // after = tiles issued after the one waited for
    if (STAGES >= 4 && after >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (STAGES >= 3 && after >= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
#pragma unroll
  for (int j = 0; j < STAGES - 1; ++j)
    if (j < nk) stage(j, j);
  wait_next(min(STAGES - 2, nk - 1));
  TR_BARRIER();
  for (int t = 0; t < nk; ++t) {
    const int s = t % STAGES;
    if (t + STAGES - 1 < nk) stage(t + STAGES - 1, (t + STAGES - 1) % STAGES);  // buffer read in t-1
    const uint8_t* tx = smem + s * STAGE;
    const uint8_t* tw = tx + TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fx[4], fw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fx[i] = ox.frag(tx, wm * 64 + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fw[j] = ow.frag(tw, wn * 64 + 16 * j, ks, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fx[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    wait_next(min(STAGES - 2, nk - 2 - t));  // tile t+1 landed (tiles after it may fly on)
    TR_BARRIER();
  }

  // lane owns y[m][n .. n+3]: m = m0 + wm*64 + 16i + (lane & 15), n = n0 + wn*64 + 16j + 4*(lane >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (F32 || SPLIT) {
    float* y = reinterpret_cast<float*>(p.y);
    int ld = p.ldy;
    if constexpr (SPLIT) {
      y += (size_t)blockIdx.y * p.split_stride;
      ld = p.N;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + 16 * i + fr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + 4 * fq;
        if (n >= p.N) continue;
        f32x4 v = acc[i][j];
        if constexpr (!SPLIT) {
          if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + n);
        }
        *reinterpret_cast<f32x4*>(y + (size_t)m * ld + n) = v;
      }
    }
  } else {
    // bf16: + bias, act (unless a mask / residual follows) -> LDS tile -> 16-B row segments
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nl = wn * 64 + 16 * j + 4 * fq;
      f32x4 bv = {0.f, 0.f, 0.f, 0.f};
      if (p.bias && n0 + nl < p.N) bv = *reinterpret_cast<const f32x4*>(p.bias + n0 + nl);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ml = wm * 64 + 16 * i + fr;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bv[r];
          if constexpr (!HAS_RES) v = apply_act<ACT>(v);
          o[r] = f2bf(v);
        }
        *reinterpret_cast<bf16x4*>(smem + ml * OPITCH + nl * 2) = o;
      }
    }
    __syncthreads();
    bf16* y = reinterpret_cast<bf16*>(p.y);
    const int cc = threadIdx.x & 15;  // this thread's 8-column chunk (fixed: NT % 16 == 0)
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int q = threadIdx.x; q < 128 * 16; q += NT) {
      const int ml = q >> 4;
      const int m = m0 + ml, n = n0 + cc * 8;
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
      if (p.colsum) {
        const bf16x8 o = __builtin_bit_cast(bf16x8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += (float)o[e];
      }
      *reinterpret_cast<u32x4*>(y + (size_t)m * p.ldy + n) = v;
    }
    if (p.colsum) {  // block-uniform: this tile's column sums (bias gradient of the next layer)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], 16, 64);
        cs[e] += __shfl_xor(cs[e], 32, 64);
      }
      float* red = reinterpret_cast<float*>(smem + LDS_EPI);  // [wave][16 chunks][8]
      if (lane < 16) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(wave * 16 + lane) * 8 + e] = cs[e];
      }
      __syncthreads();
      if (threadIdx.x < 128) {
        const int c = threadIdx.x >> 3, e = threadIdx.x & 7;
        const int n = n0 + c * 8 + e;
        if (n < p.N)
          p.colsum[(size_t)tm * p.N + n] = red[c * 8 + e] + red[(16 + c) * 8 + e] + red[(32 + c) * 8 + e] + red[(48 + c) * 8 + e];
      }
    }
  }
}

// out[n] = sum_t part[t * ldp + n] in a fixed order (column-sum partials -> bias gradient):
// a block owns 64 columns, wave w sums rows t = w, w + 4, ... (8 independent loads in
// flight per lane), then the 4 wave partials are added in wave order.
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int T, int ldp, int N,
                                                            float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  float a = 0.f;
  if (n < N) {
    int t = w;
    for (; t + 28 < T; t += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(t + 4 * u) * ldp + n];
#pragma unroll
      for (int u = 0; u < 8; ++u) a += v[u];
    }
    for (; t < T; t += 4) a += part[(size_t)t * ldp + n];
  }
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && n < N) out[n] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// Split-K reduction: sum the fp32 slabs in slab order (deterministic), + bias, then fp32
// out, or bf16 out with act / residual / ReLU-backward mask.  4 columns per thread.
template <int ACT, bool F32, bool HAS_RES>
__global__ __launch_bounds__(256) void gemm_train_reduce_kernel(const float* __restrict__ part, int splits,
                                                                long split_stride, const float* __restrict__ bias,
                                                                const bf16* __restrict__ res, int ldr, void* y, int ldy,
                                                                int M, int N) {
  const int cpr = N >> 2;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * cpr) return;
  const int m = (int)(idx / cpr);
  const int n = (int)(idx - (long)m * cpr) * 4;
  const float* src = part + (size_t)m * N + n;
  f32x4 a = *reinterpret_cast<const f32x4*>(src);
  for (int s = 1; s < splits; ++s) a += *reinterpret_cast<const f32x4*>(src + s * split_stride);
  if (bias) a += *reinterpret_cast<const f32x4*>(bias + n);
  if constexpr (F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(y) + (size_t)m * ldy + n) = a;
  } else {
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = a[e];
      if constexpr (HAS_RES) {
        const float r = (float)res[(size_t)m * ldr + n + e];
        if constexpr (ACT == ACT_DRELU) v = r > 0.f ? v : 0.f;
        else v = apply_act<ACT>(v + r);
      } else {
        v = apply_act<ACT>(v);
      }
      o[e] = f2bf(v);
    }
    *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(y) + (size_t)m * ldy + n) = o;
  }
}

int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v;
  }();
  return n;
}

template <bool XT, bool WT, int ACT, bool F32, bool HAS_RES>
void launch_tr(const TrParams& p, int splits, float* ws, hipStream_t s) {
  const int tiles = p.tiles_m * p.tiles_n;
  const bool deep = tiles * (splits > 1 ? splits : 1) <= cu_count();  // one workgroup per CU
  if (splits <= 1) {
    if (deep) hipLaunchKernelGGL((gemm_train_kernel<XT, WT, ACT, F32, HAS_RES, false, 4>), dim3(tiles), dim3(NT), 0, s, p);
    else hipLaunchKernelGGL((gemm_train_kernel<XT, WT, ACT, F32, HAS_RES, false, 2>), dim3(tiles), dim3(NT), 0, s, p);
    return;
  }
  TrParams q = p;
  q.y = ws;
  if (deep)
    hipLaunchKernelGGL((gemm_train_kernel<XT, WT, ACT_NONE, true, false, true, 4>), dim3(tiles, splits), dim3(NT), 0, s, q);
  else
    hipLaunchKernelGGL((gemm_train_kernel<XT, WT, ACT_NONE, true, false, true, 2>), dim3(tiles, splits), dim3(NT), 0, s, q);
  const long work = (long)p.M * (p.N >> 2);
  hipLaunchKernelGGL((gemm_train_reduce_kernel<ACT, F32, HAS_RES>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                     s, ws, splits, p.split_stride, p.bias, p.res, p.ldr, p.y, p.ldy, p.M, p.N);
}

template <bool XT, bool WT>
void dispatch_epi(const TrParams& p, int act, bool f32, int splits, float* ws, hipStream_t s) {
  if (f32) {
    if (act != ACT_NONE || p.res) throw std::invalid_argument("gemm_train: fp32 output takes no activation / mask");
    launch_tr<XT, WT, ACT_NONE, true, false>(p, splits, ws, s);
    return;
  }
  switch (act) {
    case ACT_NONE:
      if (p.res) launch_tr<XT, WT, ACT_NONE, false, true>(p, splits, ws, s);
      else launch_tr<XT, WT, ACT_NONE, false, false>(p, splits, ws, s);
      break;
    case ACT_RELU:
      if (p.res) launch_tr<XT, WT, ACT_RELU, false, true>(p, splits, ws, s);
      else launch_tr<XT, WT, ACT_RELU, false, false>(p, splits, ws, s);
      break;
    case ACT_DRELU:
      if (!p.res) throw std::invalid_argument("gemm_train: the drelu epilogue needs the mask operand (res)");
      launch_tr<XT, WT, ACT_DRELU, false, true>(p, splits, ws, s);
      break;
    default:
      throw std::invalid_argument("gemm_train: unsupported activation");
  }
}

void check_align(uintptr_t ptr, int bytes, const char* what) {
  if (ptr % bytes)
    throw std::invalid_argument(std::string("gemm_train: ") + what + " is not " + std::to_string(bytes) + "-byte aligned");
}

}  // namespace

// y = epi(X . W^T) with X / W in row (K-contiguous) or K-major layout (x_t / w_t), see top.
// out_f32: y fp32 [M, ldy] (weight gradients), else bf16 with bias / act (relu, drelu with
// res = mask operand [M, ldr]).  splits > 1: split-K into ws (splits * M * N fp32) + reduce.
void gemm_train(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int M, int N, int K, int ldx,
                int ldw, int ldy, int ldr, bool x_t, bool w_t, int act, bool out_f32, int splits, uintptr_t ws,
                uintptr_t colsum, uintptr_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) throw std::invalid_argument("gemm_train: empty problem");
  if (K % 8) throw std::invalid_argument("gemm_train: K must be a multiple of 8");
  if (ldx % 8 || ldw % 8) throw std::invalid_argument("gemm_train: ldx / ldw must be multiples of 8");
  if (out_f32 ? (N % 4 || ldy % 4) : (N % 8 || ldy % 8)) throw std::invalid_argument("gemm_train: N / ldy alignment");
  if (x_t ? ldx < M : ldx < K) throw std::invalid_argument("gemm_train: ldx too small");
  if (w_t ? ldw < N : ldw < K) throw std::invalid_argument("gemm_train: ldw too small");
  if ((long)(x_t ? K : M) * ldx * 2 >= (1L << 31) || (long)(w_t ? K : N) * ldw * 2 >= (1L << 31))
    throw std::invalid_argument("gemm_train: operand larger than 2 GiB");
  if (res && (ldr % 8 || out_f32)) throw std::invalid_argument("gemm_train: res needs bf16 output and ldr % 8 == 0");
  check_align(x, 16, "x");
  check_align(w, 16, "w");
  check_align(y, 16, "y");
  if (bias) check_align(bias, 16, "bias");
  if (res) check_align(res, 16, "res");
  const int nk = (K + 63) / 64;
  if (splits < 1) splits = 1;
  if (splits > nk) splits = nk;
  TrParams p{};
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.bias = reinterpret_cast<const float*>(bias);
  p.res = reinterpret_cast<const bf16*>(res);
  p.y = reinterpret_cast<void*>(y);
  p.colsum = reinterpret_cast<float*>(colsum);
  p.M = M; p.N = N; p.K = K;
  p.ldx = ldx; p.ldw = ldw; p.ldy = ldy; p.ldr = ldr;
  p.tiles_m = (M + 127) / 128;
  p.tiles_n = (N + 127) / 128;
  if (splits > 1) {
    p.kt_per_split = (nk + splits - 1) / splits;
    splits = (nk + p.kt_per_split - 1) / p.kt_per_split;
    p.split_stride = (long)M * N;
    if (!ws) throw std::invalid_argument("gemm_train: split-K needs a workspace");
    if (N % 4) throw std::invalid_argument("gemm_train: split-K needs N % 4 == 0");
    check_align(ws, 16, "ws");
  }
  if (colsum && (out_f32 || splits > 1)) throw std::invalid_argument("gemm_train: colsum needs bf16 output, no split-K");
  float* wsp = reinterpret_cast<float*>(ws);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!x_t && !w_t) dispatch_epi<false, false>(p, act, out_f32, splits, wsp, s);
  else if (!x_t && w_t) dispatch_epi<false, true>(p, act, out_f32, splits, wsp, s);
  else if (x_t && w_t) dispatch_epi<true, true>(p, act, out_f32, splits, wsp, s);
  else dispatch_epi<true, false>(p, act, out_f32, splits, wsp, s);
  FTM_CHECK_LAUNCH();
}

// out[n] = sum over T rows of part (row stride ldp): the per-tile column sums -> bias gradient
void colsum_reduce(uintptr_t part, int T, int ldp, int N, uintptr_t out, uintptr_t stream) {
  if (T <= 0 || N <= 0) return;
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3((N + 63) / 64), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const float*>(part), T, ldp, N, reinterpret_cast<float*>(out));
  FTM_CHECK_LAUNCH();
}

// K-slices gemm_train would actually run for a requested split count.
int gemm_train_splits(int K, int splits) {
  const int nk = (K + 63) / 64;
  if (splits <= 1 || nk <= 1) return 1;
  if (splits > nk) splits = nk;
  const int per = (nk + splits - 1) / splits;
  return (nk + per - 1) / per;
}

void register_gemm_train(pybind11::module_& m) {
  m.def("gemm_train", &gemm_train);
  m.def("gemm_train_splits", &gemm_train_splits);
  m.def("colsum_reduce", &colsum_reduce);
}
