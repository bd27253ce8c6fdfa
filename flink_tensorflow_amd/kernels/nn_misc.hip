// Memory-bound CNN kernels for CDNA4: image preprocess, pooling, softmax+top-k.
// Every kernel moves bf16 as 16-byte vectors (8 channels per lane) — guide Guideline 13.
#include <pybind11/pybind11.h>

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"

namespace {

// ------------------------------------------------------------------------------------
// Fused preprocess: uint8 HWC image batch -> bilinear resize (TF ResizeBilinear
// semantics) -> (v - mean[c]) * inv_std[c] -> bf16 NHWC with C padded to 8 (zeros), the
// stem conv's input layout.  Replaces the reference's per-image
// DecodeJpeg->Cast->ExpandDims->ResizeBilinear->Sub->Div graph
// (EX/inception/ImageNormalization.scala:42-77) with one pass over the batch.
// One thread per output pixel; the 3 channels of each of the 4 taps are 3 byte loads.
// ------------------------------------------------------------------------------------
struct PreParams {
  int Hi, Wi, Ho, Wo;
  float sy, sx;
  int half_pixel;
  float m[3], s[3];
  int src_stride;
};

// One resized + normalized RGB pixel (TF ResizeBilinear coordinates).
FTM_DEVICE void resize_pixel(const uint8_t* img, const PreParams& q, int oy, int ox, float out[3]) {
  float fy = q.half_pixel ? (oy + 0.5f) * q.sy - 0.5f : oy * q.sy;
  float fx = q.half_pixel ? (ox + 0.5f) * q.sx - 0.5f : ox * q.sx;
  float fy0 = floorf(fy), fx0 = floorf(fx);
  int y0 = max((int)fy0, 0), x0 = max((int)fx0, 0);
  int y1 = min(y0 + 1, q.Hi - 1), x1 = min(x0 + 1, q.Wi - 1);
  float wy = fminf(fmaxf(fy - (q.half_pixel ? (float)y0 : fy0), 0.f), 1.f);
  float wx = fminf(fmaxf(fx - (q.half_pixel ? (float)x0 : fx0), 0.f), 1.f);
  const uint8_t* p00 = img + ((size_t)y0 * q.Wi + x0) * 3;
  const uint8_t* p01 = img + ((size_t)y0 * q.Wi + x1) * 3;
  const uint8_t* p10 = img + ((size_t)y1 * q.Wi + x0) * 3;
  const uint8_t* p11 = img + ((size_t)y1 * q.Wi + x1) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float top = (float)p00[c] + ((float)p01[c] - (float)p00[c]) * wx;
    float bot = (float)p10[c] + ((float)p11[c] - (float)p10[c]) * wx;
    out[c] = (top + (bot - top) * wy - q.m[c]) * q.s[c];
  }
}

// Layout 0: [B, Ho, Wo, 8] (RGB + 5 zero channels).
// Layout 1 (space-to-depth 2x2, for the stride-2 stem conv): [B, ceil(Ho/2), ceil(Wo/2), 16]
// with channel (dy*2+dx)*3 + c = pixel (2*oy2+dy, 2*ox2+dx) channel c, channels 12..15 zero;
// an odd size's last row / column block holds zeros for the pixels past the image (the
// stem weights of those taps are zero, e.g. Inception's 3x3 / s2 VALID stem on 299 x 299).
template <int S2D>
__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ src, bf16* __restrict__ dst,
                                                         int B, PreParams q) {
  const int Wo = S2D ? (q.Wo + 1) / 2 : q.Wo, Ho = S2D ? (q.Ho + 1) / 2 : q.Ho;
  const int total = B * Ho * Wo;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int ox = idx % Wo;
    const int t = idx / Wo;
    const int oy = t % Ho;
    const int b = t / Ho;
    const uint8_t* img = src + (size_t)b * q.src_stride;
    float v[3];
    if constexpr (S2D) {
      bf16x8 o0, o1;
      float pix[4][3];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int py = 2 * oy + (d >> 1), px = 2 * ox + (d & 1);
        if (py < q.Ho && px < q.Wo) resize_pixel(img, q, py, px, pix[d]);
        else pix[d][0] = pix[d][1] = pix[d][2] = 0.f;
      }
      o0[0] = f2bf(pix[0][0]); o0[1] = f2bf(pix[0][1]); o0[2] = f2bf(pix[0][2]);
      o0[3] = f2bf(pix[1][0]); o0[4] = f2bf(pix[1][1]); o0[5] = f2bf(pix[1][2]);
      o0[6] = f2bf(pix[2][0]); o0[7] = f2bf(pix[2][1]);
      o1[0] = f2bf(pix[2][2]);
      o1[1] = f2bf(pix[3][0]); o1[2] = f2bf(pix[3][1]); o1[3] = f2bf(pix[3][2]);
      o1[4] = o1[5] = o1[6] = o1[7] = f2bf(0.f);
      bf16x8* d = reinterpret_cast<bf16x8*>(dst + (size_t)idx * 16);
      d[0] = o0;
      d[1] = o1;
    } else {
      resize_pixel(img, q, oy, ox, v);
      bf16x8 o;
      o[0] = f2bf(v[0]);
      o[1] = f2bf(v[1]);
      o[2] = f2bf(v[2]);
      o[3] = o[4] = o[5] = o[6] = o[7] = f2bf(0.f);
      *reinterpret_cast<bf16x8*>(dst + (size_t)idx * 8) = o;
    }
  }
}

// Row-staged space-to-depth form (the ResNet stem input): one workgroup per output block
// row (2 output rows).  The <= 4 source rows its bilinear taps touch are copied into LDS
// with coalesced dword loads, then every thread interpolates its 2x2 output pixels from
// LDS.  The one-thread-per-pixel kernel above issues 48 scattered byte loads per thread
// (each wave instruction touching ~4 cache lines); here global traffic is the source rows
// once plus the 32-B output stores.  Same arithmetic as resize_pixel, so the results are
// identical.  Rows need not be dword-aligned (Inception's 299 x 3 = 897-byte rows): each
// slot keeps its row's misalignment and the copy starts at the dword below (reading at most
// 3 bytes past the last row, inside the allocation granule).  Needs Wi * 3 + 3 <= ROW_MAX.
constexpr int PRE_ROW_MAX = 4096;
constexpr int PRE_NT = 128;

// ROWB: LDS bytes per staged row (1024 for sources up to 340 pixels wide: 4 KiB per
// workgroup instead of 16 KiB, so LDS no longer caps the workgroups resident per CU).
template <int ROWB>
__global__ __launch_bounds__(PRE_NT) void preprocess_s2d_rows_kernel(const uint8_t* __restrict__ src,
                                                                     bf16* __restrict__ dst, PreParams q) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[4][ROWB];
  const int Wo2 = (q.Wo + 1) / 2, Ho2 = (q.Ho + 1) / 2;
  const int oy2 = blockIdx.x % Ho2, b = blockIdx.x / Ho2;
  const uint8_t* img = src + (size_t)b * q.src_stride;
  const int rb = q.Wi * 3;
  // source rows of output rows 2*oy2 + dy: slot 2*dy (y0) and 2*dy + 1 (y1), + their weights
  int ys[4];
  float wy[2];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    const int oy = min(2 * oy2 + dy, q.Ho - 1);  // a row past the image is zero-filled below
    const float fy = q.half_pixel ? (oy + 0.5f) * q.sy - 0.5f : oy * q.sy;
    const float fy0 = floorf(fy);
    const int y0 = max((int)fy0, 0);
    ys[2 * dy] = y0;
    ys[2 * dy + 1] = min(y0 + 1, q.Hi - 1);
    wy[dy] = fminf(fmaxf(fy - (q.half_pixel ? (float)y0 : fy0), 0.f), 1.f);
  }
  int sh[4];  // byte misalignment of each staged row
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint8_t* rowp = img + (size_t)ys[r] * rb;
    sh[r] = (int)(reinterpret_cast<uintptr_t>(rowp) & 3);
    const uint32_t* srow = reinterpret_cast<const uint32_t*>(rowp - sh[r]);
    uint32_t* drow = reinterpret_cast<uint32_t*>(rows[r]);
    const int rw = (sh[r] + rb + 3) >> 2;  // dwords covering the row
    for (int i = threadIdx.x; i < rw; i += PRE_NT) drow[i] = srow[i];
  }
  __syncthreads();
  for (int ox2 = threadIdx.x; ox2 < Wo2; ox2 += PRE_NT) {
    float pix[4][3];
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int ox = 2 * ox2 + dx;
      const float fx = q.half_pixel ? (ox + 0.5f) * q.sx - 0.5f : ox * q.sx;
      const float fx0 = floorf(fx);
      const int x0 = max((int)fx0, 0), x1 = min(x0 + 1, q.Wi - 1);
      const float wx = fminf(fmaxf(fx - (q.half_pixel ? (float)x0 : fx0), 0.f), 1.f);
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const uint8_t* r0 = rows[2 * dy] + sh[2 * dy];
        const uint8_t* r1 = rows[2 * dy + 1] + sh[2 * dy + 1];
        const bool live = 2 * oy2 + dy < q.Ho && ox < q.Wo;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float p00 = r0[x0 * 3 + c], p01 = r0[x1 * 3 + c], p10 = r1[x0 * 3 + c], p11 = r1[x1 * 3 + c];
          const float top = p00 + (p01 - p00) * wx;
          const float bot = p10 + (p11 - p10) * wx;
          pix[dy * 2 + dx][c] = live ? (top + (bot - top) * wy[dy] - q.m[c]) * q.s[c] : 0.f;
        }
      }
    }
    bf16x8 o0, o1;
    o0[0] = f2bf(pix[0][0]); o0[1] = f2bf(pix[0][1]); o0[2] = f2bf(pix[0][2]);
    o0[3] = f2bf(pix[1][0]); o0[4] = f2bf(pix[1][1]); o0[5] = f2bf(pix[1][2]);
    o0[6] = f2bf(pix[2][0]); o0[7] = f2bf(pix[2][1]);
    o1[0] = f2bf(pix[2][2]);
    o1[1] = f2bf(pix[3][0]); o1[2] = f2bf(pix[3][1]); o1[3] = f2bf(pix[3][2]);
    o1[4] = o1[5] = o1[6] = o1[7] = f2bf(0.f);
    bf16x8* d = reinterpret_cast<bf16x8*>(dst + ((size_t)blockIdx.x * Wo2 + ox2) * 16);
    d[0] = o0;
    d[1] = o1;
  }
}

// ------------------------------------------------------------------------------------
// 2-D pooling, NHWC bf16, TF semantics: MAX pads with -inf; AVG excludes padding from
// the divisor.  One thread per (output pixel, 8-channel chunk).
// ------------------------------------------------------------------------------------
template <bool MAX>
__global__ __launch_bounds__(256) void pool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H,
                                                   int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                                                   int ph, int pw, int ldy, int y_coff) {
  const int cchunks = C / 8;
  const long total = (long)N * Ho * Wo * cchunks;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int cc = idx % cchunks;
    long t = idx / cchunks;
    const int ox = t % Wo;
    t /= Wo;
    const int oy = t % Ho;
    const int n = t / Ho;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = MAX ? -INFINITY : 0.f;
    int cnt = 0;
    const int iy0 = oy * sh - ph, ix0 = ox * sw - pw;
    for (int dy = 0; dy < kh; ++dy) {
      const int iy = iy0 + dy;
      if ((unsigned)iy >= (unsigned)H) continue;
      for (int dx = 0; dx < kw; ++dx) {
        const int ix = ix0 + dx;
        if ((unsigned)ix >= (unsigned)W) continue;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (((size_t)n * H + iy) * W + ix) * C + cc * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = MAX ? fmaxf(acc[e], (float)v[e]) : acc[e] + (float)v[e];
        ++cnt;
      }
    }
    bf16x8 o;
    const float inv = MAX ? 1.f : 1.f / (float)max(cnt, 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e] * inv);
    *reinterpret_cast<bf16x8*>(y + (((size_t)n * Ho + oy) * Wo + ox) * ldy + y_coff + cc * 8) = o;
  }
}

// Global average pool [N, HW, C] -> [N, C] (fp32 accumulate).  One block per image,
// each thread owns 8 channels; loops over the HW positions with 16-B loads.
__global__ __launch_bounds__(256) void global_avgpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int HW,
                                                             int C) {
  const int n = blockIdx.x;
  const float inv = 1.f / (float)HW;
  for (int cc = threadIdx.x; cc < C / 8; cc += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bf16* p = x + (size_t)n * HW * C + cc * 8;
    // unrolled: 8 independent row loads in flight per thread (the rolled loop waited for
    // each of the HW loads in turn)
#pragma unroll 8
    for (int i = 0; i < HW; ++i) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(p + (size_t)i * C);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e] * inv);
    *reinterpret_cast<bf16x8*>(y + (size_t)n * C + cc * 8) = o;
  }
}

// ------------------------------------------------------------------------------------
// Row softmax fused with top-k (replaces the reference's host-side sort of the full
// [M, N] label matrix, EX/inception/InceptionModel.scala:76-90).  One wave per row; the
// row lives in registers (PER values per lane, strided by 64 for coalescing), so the
// logits are read exactly once.  Outputs top-k probabilities (fp32) and class indices;
// optionally the full probability row (bf16).
// ------------------------------------------------------------------------------------
template <int PER>
__global__ __launch_bounds__(256) void softmax_topk_kernel(const bf16* __restrict__ logits, int rows, int C, int ld,
                                                           int k, float* __restrict__ vals, int* __restrict__ idxs,
                                                           bf16* __restrict__ probs) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* p = logits + (size_t)row * ld;
  float v[PER];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? (float)p[c] : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_reduce_max(mx);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = (lane + 64 * i) < C ? __expf(v[i] - mx) : 0.f;
    s += v[i];
  }
  s = wave_reduce_sum(s);
  const float inv = 1.f / s;
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] *= inv;
  if (probs) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < C) probs[(size_t)row * C + c] = f2bf(v[i]);
    }
  }
  for (int t = 0; t < k; ++t) {
    float best = -1.f;
    int bi = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < C && (v[i] > best || (v[i] == best && c < bi))) {
        best = v[i];
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ob = __shfl_xor(best, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    if (lane == 0) {
      vals[(size_t)row * k + t] = best;
      idxs[(size_t)row * k + t] = bi;
    }
    // knock out the winner (owned by lane bi % 64, slot bi / 64)
    if ((bi & 63) == lane) {
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (i == (bi >> 6)) v[i] = -2.f;
    }
  }
}

int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 2048 * 8 ? 2048 * 8 : g));
}


}  // namespace

void preprocess_u8_to_bf16(uintptr_t src, uintptr_t dst, int B, int Hi, int Wi, int Ho, int Wo, int align_corners,
                           int half_pixel, float m0, float m1, float m2, float s0, float s1, float s2, int src_stride,
                           int s2d, uintptr_t stream) {
  if (B <= 0 || Hi <= 0 || Wi <= 0 || Ho <= 0 || Wo <= 0) throw std::invalid_argument("preprocess: bad shape");
  if (src_stride < Hi * Wi * 3) throw std::invalid_argument("preprocess: src_stride smaller than one image");
  if (dst % 16) throw std::invalid_argument("preprocess: dst not 16-byte aligned");
  PreParams q;
  q.Hi = Hi; q.Wi = Wi; q.Ho = Ho; q.Wo = Wo;
  q.sy = (align_corners && Ho > 1) ? (float)(Hi - 1) / (Ho - 1) : (float)Hi / Ho;
  q.sx = (align_corners && Wo > 1) ? (float)(Wi - 1) / (Wo - 1) : (float)Wi / Wo;
  q.half_pixel = half_pixel;
  q.m[0] = m0; q.m[1] = m1; q.m[2] = m2;
  q.s[0] = s0; q.s[1] = s1; q.s[2] = s2;
  q.src_stride = src_stride;
  long work = s2d ? (long)B * ((Ho + 1) / 2) * ((Wo + 1) / 2) : (long)B * Ho * Wo;
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto S = reinterpret_cast<const uint8_t*>(src);
  auto D = reinterpret_cast<bf16*>(dst);
  const bool rows_ok = s2d && Wi * 3 + 3 <= PRE_ROW_MAX;
  if (rows_ok && Wi * 3 + 3 <= 1024)
    hipLaunchKernelGGL(preprocess_s2d_rows_kernel<1024>, dim3(B * ((Ho + 1) / 2)), dim3(PRE_NT), 0, s, S, D, q);
  else if (rows_ok)
    hipLaunchKernelGGL(preprocess_s2d_rows_kernel<PRE_ROW_MAX>, dim3(B * ((Ho + 1) / 2)), dim3(PRE_NT), 0, s, S, D, q);
  else if (s2d) hipLaunchKernelGGL(preprocess_kernel<1>, dim3(grid_for(work, 256)), dim3(256), 0, s, S, D, B, q);
  else hipLaunchKernelGGL(preprocess_kernel<0>, dim3(grid_for(work, 256)), dim3(256), 0, s, S, D, B, q);
  FTM_CHECK_LAUNCH();
}

void pool2d_nhwc_bf16(uintptr_t x, uintptr_t y, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh,
                      int sw, int ph, int pw, int is_max, int ldy, int y_coff, uintptr_t stream) {
  if (C % 8 || ldy % 8 || y_coff % 8) throw std::invalid_argument("pool2d: C, ldy, y_coff must be multiples of 8");
  if (x % 16 || y % 16) throw std::invalid_argument("pool2d: pointers must be 16-byte aligned");
  long work = (long)N * Ho * Wo * (C / 8);
  auto s = reinterpret_cast<hipStream_t>(stream);
  if (is_max)
    hipLaunchKernelGGL(pool_kernel<true>, dim3(grid_for(work, 256)), dim3(256), 0, s, reinterpret_cast<const bf16*>(x),
                       reinterpret_cast<bf16*>(y), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, ldy, y_coff);
  else
    hipLaunchKernelGGL(pool_kernel<false>, dim3(grid_for(work, 256)), dim3(256), 0, s,
                       reinterpret_cast<const bf16*>(x), reinterpret_cast<bf16*>(y), N, H, W, C, Ho, Wo, kh, kw, sh, sw,
                       ph, pw, ldy, y_coff);
  FTM_CHECK_LAUNCH();
}

void global_avgpool_bf16(uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t stream) {
  if (C % 8) throw std::invalid_argument("global_avgpool: C must be a multiple of 8");
  if (x % 16 || y % 16) throw std::invalid_argument("global_avgpool: pointers must be 16-byte aligned");
  hipLaunchKernelGGL(global_avgpool_kernel, dim3(N), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16*>(x), reinterpret_cast<bf16*>(y), HW, C);
  FTM_CHECK_LAUNCH();
}

void softmax_topk_bf16(uintptr_t logits, int rows, int C, int ld, int k, uintptr_t vals, uintptr_t idxs,
                       uintptr_t probs, uintptr_t stream) {
  if (k < 1 || k > C) throw std::invalid_argument("softmax_topk: k out of range");
  if (C > 64 * 64) throw std::invalid_argument("softmax_topk: C > 4096 not supported");
  dim3 grid((rows + 3) / 4), block(256);
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto L = reinterpret_cast<const bf16*>(logits);
  auto V = reinterpret_cast<float*>(vals);
  auto I = reinterpret_cast<int*>(idxs);
  auto P = reinterpret_cast<bf16*>(probs);
  if (C <= 64 * 16) hipLaunchKernelGGL(softmax_topk_kernel<16>, grid, block, 0, s, L, rows, C, ld, k, V, I, P);
  else if (C <= 64 * 32) hipLaunchKernelGGL(softmax_topk_kernel<32>, grid, block, 0, s, L, rows, C, ld, k, V, I, P);
  else hipLaunchKernelGGL(softmax_topk_kernel<64>, grid, block, 0, s, L, rows, C, ld, k, V, I, P);
  FTM_CHECK_LAUNCH();
}

void register_nn_misc(pybind11::module_& m) {
  m.def("preprocess_u8_to_bf16", &preprocess_u8_to_bf16);
  m.def("pool2d_nhwc_bf16", &pool2d_nhwc_bf16);
  m.def("global_avgpool_bf16", &global_avgpool_bf16);
  m.def("softmax_topk_bf16", &softmax_topk_bf16);
}
