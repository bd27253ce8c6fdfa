// Fused Wide&Deep training-step kernels (models/zoo/wide_deep_fused.py).  Everything of the
// step that is not a GEMM, the sort or the segment sum runs here, replacing ~100 small
// framework kernels per step (casts, cat/pad, slices, BCE pieces, Adam, bf16 weight copies):
//
//   wd_gather     x[b] = [emb[cats[b,f] + f*V] for f | dense[b] | 0 pad]  (bf16 MLP input)
//                 wsum[b] = sum_c wide[cross[b,c], 0]; the sparse grouping keys of both tables
//   wd_loss       logit = deep[b] + wsum[b] + wide_bias, BCE-with-logits mean (block partials
//                 added in block order), dlogit = (sigmoid - y) / B, wide gradient rows, the
//                 scalar gradients (wide bias, head bias 0)
//   wd_head_bwd   dh[b, j] = (h[b, j] > 0) * dlogit[b] * w_head0[j]   (bf16)
//   wd_adam       Adam over the flat fp32 parameter buffer (device step counter, so a
//                 captured step replays correctly) + the bf16 copy of every weight segment
//   wd_mask_colsum  the ReLU backward mask of a layer input, in place on the library dX,
//                 and the bias gradient (column sums, fixed order) in the same pass
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

// G = D/8 lanes per (b, f) embedding row; rows r >= B*F are the per-record rows (dense, pad,
// wide sum) handled by the G lanes of row B*F + b.
// cats / dense / cross rows have their own strides (elements): they may be views of one
// packed record buffer.  keys [B*F + B*C]: the sparse-gradient grouping keys of BOTH
// tables in one key space — embedding rows as is, wide rows offset by F*V, invalid ids of
// either table -> F*V + WV (one dropped bucket) — so one radix sort groups both.
// The lookup keys of a micro-batch in the shared key space (embedding rows, then the wide
// table offset by F*V; F*V + WV = invalid) — exactly the keys wd_gather writes, but
// available BEFORE the gather: the data-parallel owner exchange refreshes those rows first.
__global__ __launch_bounds__(256) void wd_keys_kernel(const int* __restrict__ cats, int ldc, const int* __restrict__ cross,
                                                      int ldx, int* __restrict__ keys, int B, int F, int V, int C,
                                                      int WV) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long nemb = (long)B * F;
  const int FV = F * V, BAD = FV + WV;
  if (t < nemb) {
    const int b = (int)(t / F), f = (int)(t - (long)b * F);
    const int gid = cats[(size_t)b * ldc + f] + f * V;
    keys[t] = (gid >= 0 && gid < FV) ? gid : BAD;
  } else if (t < nemb + (long)B * C) {
    const long r = t - nemb;
    const int b = (int)(r / C), c = (int)(r - (long)b * C);
    const int id = cross[(size_t)b * ldx + c];
    keys[t] = (id >= 0 && id < WV) ? FV + id : BAD;
  }
}

__global__ __launch_bounds__(256) void wd_gather_kernel(const int* __restrict__ cats, int ldc,
                                                        const float* __restrict__ dense, int ldd,
                                                        const int* __restrict__ cross, int ldx,
                                                        const float* __restrict__ emb, const float* __restrict__ wide,
                                                        bf16* __restrict__ x, float* __restrict__ wsum,
                                                        int* __restrict__ keys, int B, int F,
                                                        int V, int D, int gshift, int ND, int XP, int C, int WV,
                                                        int WD) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long r = t >> gshift;
  const int g = (int)(t & ((1 << gshift) - 1));
  const long nemb = (long)B * F;
  if (r < nemb) {
    const int b = (int)(r / F), f = (int)(r - (long)b * F);
    const int gid = cats[(size_t)b * ldc + f] + f * V;  // field-local id -> row of the concatenated table
    const int FV = F * V, BAD = FV + WV;
    if (g == 0) keys[r] = (gid >= 0 && gid < FV) ? gid : BAD;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (gid >= 0 && gid < F * V) {
      const f32x4* src = reinterpret_cast<const f32x4*>(emb + (size_t)gid * D + g * 8);
      const f32x4 a = src[0], c = src[1];
      acc[0] = a[0]; acc[1] = a[1]; acc[2] = a[2]; acc[3] = a[3];
      acc[4] = c[0]; acc[5] = c[1]; acc[6] = c[2]; acc[7] = c[3];
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    *reinterpret_cast<bf16x8*>(x + (size_t)b * XP + f * D + g * 8) = o;
  } else if (r < nemb + B) {
    const int b = (int)(r - nemb);
    const int base = F * D;
    for (int c0 = g * 8; base + c0 < XP; c0 += 8 << gshift) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(c0 + e < ND ? dense[(size_t)b * ldd + c0 + e] : 0.f);
      *reinterpret_cast<bf16x8*>(x + (size_t)b * XP + base + c0) = o;
    }
    if (g == 0) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) {
        const int id = cross[(size_t)b * ldx + c];
        const bool ok = id >= 0 && id < WV;
        keys[nemb + (size_t)b * C + c] = ok ? F * V + id : F * V + WV;
        if (ok) s += wide[(size_t)id * WD];
      }
      wsum[b] = s;
    }
  }
}

// One thread per record; per-block partial sums of the loss and of dlogit go to part[2 * block]
// and wd_loss_final adds them in block order (deterministic).
__global__ __launch_bounds__(256) void wd_loss_kernel(const bf16* __restrict__ head, int ldh,
                                                      const float* __restrict__ wsum, const float* __restrict__ wbias,
                                                      const float* __restrict__ labels, int ldl, int B,
                                                      int nvalid, float norm, float* __restrict__ dlogit,
                                                      bf16* __restrict__ dlogit16, float* __restrict__ part,
                                                      float* __restrict__ wgrad, int C, int WD,
                                                      const int* __restrict__ args) {
  __shared__ float red[2][4];
  if (args) {  // device-resident {nvalid, norm bits}: one captured step serves every piece size
    nvalid = args[0];
    norm = __int_as_float(args[1]);
  }
  const int b = blockIdx.x * 256 + threadIdx.x;
  float lo = 0.f, d = 0.f;
  if (b >= nvalid && b < B) {  // padding rows of a batch rounded up to the GEMM granule: no loss, no gradient
    dlogit[b] = 0.f;
    dlogit16[b] = f2bf(0.f);
    for (int c = 0; c < C; ++c) {
      float* row = wgrad + ((size_t)b * C + c) * WD;
      for (int k = 0; k < WD; ++k) row[k] = 0.f;
    }
  } else if (b < B) {
    const float l = (float)head[(size_t)b * ldh] + wsum[b] + wbias[0];
    const float y = labels[(size_t)b * ldl];
    lo = fmaxf(l, 0.f) - l * y + log1pf(__expf(-fabsf(l)));
    d = (__builtin_amdgcn_rcpf(1.f + __expf(-l)) - y) / norm;
    dlogit[b] = d;
    dlogit16[b] = f2bf(d);
    for (int c = 0; c < C; ++c) {  // the wide part: every lookup's row gets d in column 0
      float* row = wgrad + ((size_t)b * C + c) * WD;
      if (WD % 4 == 0) {
        reinterpret_cast<f32x4*>(row)[0] = f32x4{d, 0.f, 0.f, 0.f};
        for (int k = 4; k < WD; k += 4) reinterpret_cast<f32x4*>(row + k)[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        row[0] = d;
        for (int k = 1; k < WD; ++k) row[k] = 0.f;
      }
    }
  }
  lo = wave_reduce_sum(lo);
  d = wave_reduce_sum(d);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = lo;
    red[1][threadIdx.x >> 6] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__global__ __launch_bounds__(64) void wd_loss_final_kernel(const float* __restrict__ part, int nb, float norm,
                                                           float* __restrict__ loss, float* __restrict__ g_wbias,
                                                           float* __restrict__ g_hb0, float* __restrict__ step,
                                                           const int* __restrict__ args) {
  if (args) norm = __int_as_float(args[1]);
  float a = 0.f, s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 64) {
    a += part[2 * i];
    s += part[2 * i + 1];
  }
  a = wave_reduce_sum(a);
  s = wave_reduce_sum(s);
  if (threadIdx.x == 0) {
    loss[0] = a / norm;
    g_wbias[0] = s;
    g_hb0[0] = s;
    if (step) step[0] += 1.f;  // Adam's step count (read by wd_adam later on the stream)
  }
}

__global__ __launch_bounds__(256) void wd_head_bwd_kernel(const bf16* __restrict__ h, const float* __restrict__ dlogit,
                                                          const float* __restrict__ wh0, bf16* __restrict__ dh, int B,
                                                          int H) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const int cpr = H >> 3;
  if (t >= (long)B * cpr) return;
  const int b = (int)(t / cpr), c = (int)(t - (long)b * cpr) * 8;
  const float d = dlogit[b];
  const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h + (size_t)b * H + c);
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf((float)hv[e] > 0.f ? d * wh0[c + e] : 0.f);
  *reinterpret_cast<bf16x8*>(dh + (size_t)b * H + c) = o;
}

// Head backward in one pass over the top hidden activations h [B, H] (only logit column 0
// of the 8-row head is used): dh = (h > 0) ? dlogit[b] * wh0 : 0 (bf16), plus this block's
// column partials of dh (-> the top layer's bias gradient) and of dlogit[b] * h (-> the head
// weight row): part[blk][0..H) and part[blk][H..2H), summed in fixed order by colsum_reduce.
// Thread t: 8-column chunk t % CH, row lane t / CH (CH = H / 8 chunks, 256 / CH row lanes).
__global__ __launch_bounds__(256) void wd_head_bwd2_kernel(const bf16* __restrict__ h, const float* __restrict__ dlogit,
                                                           const float* __restrict__ wh0, bf16* __restrict__ dh,
                                                           float* __restrict__ part, int B, int H, int rows_per_blk) {
  __shared__ float red[256 * 16];
  const int CH = H >> 3, RL = 256 / CH;
  const int c = threadIdx.x % CH, rl = threadIdx.x / CH;
  float db[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rl < RL) {
    f32x4 w0 = *reinterpret_cast<const f32x4*>(wh0 + c * 8), w1 = *reinterpret_cast<const f32x4*>(wh0 + c * 8 + 4);
    const float wv[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
    const int b0 = blockIdx.x * rows_per_blk, b1 = min(B, b0 + rows_per_blk);
    for (int b = b0 + rl; b < b1; b += RL) {
      const float d = dlogit[b];
      const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h + (size_t)b * H + c * 8);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = (float)hv[e];
        o[e] = f2bf(x > 0.f ? d * wv[e] : 0.f);
        db[e] += (float)o[e];
        dw[e] += d * x;
      }
      *reinterpret_cast<bf16x8*>(dh + (size_t)b * H + c * 8) = o;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[threadIdx.x * 16 + e] = db[e];
    red[threadIdx.x * 16 + 8 + e] = dw[e];
  }
  __syncthreads();
  float* out = part + (size_t)blockIdx.x * 2 * H;
  for (int j = threadIdx.x; j < 2 * H; j += 256) {
    const int col = j % H, kind = j / H;  // kind 0: bias, 1: weight
    const int cj = col >> 3, e = col & 7;
    float a = 0.f;
    for (int r = 0; r < RL; ++r) a += red[(r * CH + cj) * 16 + kind * 8 + e];
    out[j] = a;
  }
}

// seg: int64 [3, nseg] = (flat offset, element count, bf16 copy pointer) per weight segment
__global__ __launch_bounds__(256) void wd_adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, long n,
                                                      const float* __restrict__ step, float lr, float b1, float b2,
                                                      float eps, float gscale, const long long* __restrict__ seg,
                                                      int nseg) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float t = step[0];
  const float gi = g[i] * gscale;
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  // b^t = exp2(t log2 b): one v_exp_f32 each instead of powf
  const float bc1 = 1.f - __builtin_amdgcn_exp2f(t * __log2f(b1)), bc2 = 1.f - __builtin_amdgcn_exp2f(t * __log2f(b2));
  const float pi = p[i] - (lr / bc1) * mi / (sqrtf(vi) * __builtin_amdgcn_rsqf(bc2) + eps);
  p[i] = pi;
  for (int s = 0; s < nseg; ++s) {
    const long off = seg[s], cnt = seg[nseg + s];
    if (i >= off && i < off + cnt) reinterpret_cast<bf16*>(seg[2 * nseg + s])[i - off] = f2bf(pi);
  }
}

// db[j] = sum_b x[b, j] (fp32, fixed order), optionally after the ReLU backward mask of the
// layer input h (x[b, j] = 0 where h[b, j] <= 0, written back).  Block = 16 columns x 128
// row lanes; each lane sums every 128th row of its 8 columns, then a fixed LDS tree.
__global__ __launch_bounds__(256) void wd_mask_colsum_kernel(bf16* __restrict__ x, const bf16* __restrict__ h,
                                                             float* __restrict__ db, int B, int n) {
  __shared__ float red[128][17];
  const int chunk = threadIdx.x & 1;      // which 8 of the block's 16 columns
  const int rl = threadIdx.x >> 1;        // row lane 0..127
  const int c0 = blockIdx.x * 16 + chunk * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < n) {
    for (int b = rl; b < B; b += 128) {
      bf16x8* px = reinterpret_cast<bf16x8*>(x + (size_t)b * n + c0);
      bf16x8 xv = *px;
      if (h) {
        const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h + (size_t)b * n + c0);
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = (float)hv[e] > 0.f ? xv[e] : f2bf(0.f);
        *px = xv;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (float)xv[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][chunk * 8 + e] = acc[e];
  __syncthreads();
  for (int w = 64; w > 0; w >>= 1) {
    if (rl < w) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[rl][chunk * 8 + e] += red[rl + w][chunk * 8 + e];
    }
    __syncthreads();
  }
  if (rl == 0 && c0 < n) {
#pragma unroll
    for (int e = 0; e < 8; ++e) db[c0 + e] = red[0][chunk * 8 + e];
  }
}

int pow2_shift(int g) {
  for (int k = 0; k <= 6; ++k)
    if (g == (1 << k)) return k;
  return -1;
}

}  // namespace

void wd_gather(uintptr_t cats, int ldc, uintptr_t dense, int ldd, uintptr_t cross, int ldx, uintptr_t emb,
               uintptr_t wide, uintptr_t x, uintptr_t wsum, uintptr_t keys, int B, int F, int V, int D,
               int ND, int XP, int C, int WV, int WD, uintptr_t stream) {
  const int gs = pow2_shift(D / 8);
  if (D % 8 || gs < 0) throw std::invalid_argument("wd_gather: D / 8 must be a power of two <= 64");
  if (XP % 8 || XP < F * D + ND) throw std::invalid_argument("wd_gather: XP must be a multiple of 8 >= F*D + ND");
  if (emb % 16 || x % 16) throw std::invalid_argument("wd_gather: 16-byte alignment required");
  if ((long)F * V + WV >= (1L << 30)) throw std::invalid_argument("wd_gather: table rows must fit the key space");
  if (B <= 0) return;
  const long threads = ((long)B * F + B) << gs;
  hipLaunchKernelGGL(wd_gather_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const int*>(cats), ldc,
                     reinterpret_cast<const float*>(dense), ldd, reinterpret_cast<const int*>(cross), ldx,
                     reinterpret_cast<const float*>(emb), reinterpret_cast<const float*>(wide),
                     reinterpret_cast<bf16*>(x), reinterpret_cast<float*>(wsum), reinterpret_cast<int*>(keys), B, F,
                     V, D, gs, ND, XP, C, WV, WD);
  FTM_CHECK_LAUNCH();
}

void wd_keys(uintptr_t cats, int ldc, uintptr_t cross, int ldx, uintptr_t keys, int B, int F, int V, int C, int WV,
             uintptr_t stream) {
  const long n = (long)B * (F + C);
  if (n <= 0) return;
  hipLaunchKernelGGL(wd_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const int*>(cats), ldc,
                     reinterpret_cast<const int*>(cross), ldx, reinterpret_cast<int*>(keys), B, F, V, C, WV);
  FTM_CHECK_LAUNCH();
}

// part: >= 2 * ceil(B / 256) floats of workspace.  norm: the loss is sum / norm — B for the
// batch mean; the global record count of an agreed data-parallel step over uneven pieces
// (parallel/step_agreement.py), so the summed gradients are those of the union's mean.
// step (optional, 0 = none): Adam's step counter, incremented here so the captured step has
// no separate increment launch.
// nvalid <= B: rows [nvalid, B) are padding (a batch rounded up to the training GEMM's
// 8-row granule, or an agreed step's piece padded to the fixed micro-batch) and get zero
// loss and gradient.  args (0 = none): device int32 {nvalid, bits of float norm} read by the
// kernels instead of the host values — the agreed step of runtime/lockstep.py is captured
// once and replayed for every piece size (0 <= nvalid <= B, norm > 0 when the step runs).
void wd_loss(uintptr_t head, int ldh, uintptr_t wsum, uintptr_t wbias, uintptr_t labels, int ldl, int B, int nvalid,
             float norm, uintptr_t dlogit, uintptr_t dlogit16, uintptr_t loss, uintptr_t g_wbias, uintptr_t g_hb0,
             uintptr_t wgrad, int C, int WD, uintptr_t part, uintptr_t step, uintptr_t args, uintptr_t stream) {
  if (B <= 0 || (!args && (nvalid <= 0 || nvalid > B))) throw std::invalid_argument("wd_loss: empty batch or bad nvalid");
  if (!args && !(norm > 0.f)) throw std::invalid_argument("wd_loss: norm must be positive");
  if (args % 8) throw std::invalid_argument("wd_loss: args must be 8-byte aligned");
  if (wgrad % 16) throw std::invalid_argument("wd_loss: wgrad must be 16-byte aligned");
  auto s = reinterpret_cast<hipStream_t>(stream);
  const int nb = (B + 255) / 256;
  hipLaunchKernelGGL(wd_loss_kernel, dim3(nb), dim3(256), 0, s, reinterpret_cast<const bf16*>(head), ldh,
                     reinterpret_cast<const float*>(wsum), reinterpret_cast<const float*>(wbias),
                     reinterpret_cast<const float*>(labels), ldl, B, nvalid, norm, reinterpret_cast<float*>(dlogit),
                     reinterpret_cast<bf16*>(dlogit16), reinterpret_cast<float*>(part), reinterpret_cast<float*>(wgrad),
                     C, WD, reinterpret_cast<const int*>(args));
  hipLaunchKernelGGL(wd_loss_final_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<const float*>(part), nb, norm,
                     reinterpret_cast<float*>(loss), reinterpret_cast<float*>(g_wbias), reinterpret_cast<float*>(g_hb0),
                     reinterpret_cast<float*>(step), reinterpret_cast<const int*>(args));
  FTM_CHECK_LAUNCH();
}

void wd_head_bwd(uintptr_t h, uintptr_t dlogit, uintptr_t wh0, uintptr_t dh, int B, int H, uintptr_t stream) {
  if (H % 8 || h % 16 || dh % 16) throw std::invalid_argument("wd_head_bwd: H % 8 and 16-byte alignment");
  const long work = (long)B * (H / 8);
  if (work <= 0) return;
  hipLaunchKernelGGL(wd_head_bwd_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const bf16*>(h),
                     reinterpret_cast<const float*>(dlogit), reinterpret_cast<const float*>(wh0),
                     reinterpret_cast<bf16*>(dh), B, H);
  FTM_CHECK_LAUNCH();
}

void wd_head_bwd2(uintptr_t h, uintptr_t dlogit, uintptr_t wh0, uintptr_t dh, uintptr_t part, int B, int H, int blocks,
                  uintptr_t stream) {
  if (H % 8 || H > 2048 || 256 % (H / 8) || h % 16 || dh % 16 || wh0 % 16)
    throw std::invalid_argument("wd_head_bwd2: H / 8 must divide 256; 16-byte alignment");
  if (B <= 0 || blocks <= 0) return;
  const int rows = (B + blocks - 1) / blocks;
  hipLaunchKernelGGL(wd_head_bwd2_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16*>(h), reinterpret_cast<const float*>(dlogit),
                     reinterpret_cast<const float*>(wh0), reinterpret_cast<bf16*>(dh), reinterpret_cast<float*>(part),
                     B, H, rows);
  FTM_CHECK_LAUNCH();
}

void wd_adam(uintptr_t p, uintptr_t g, uintptr_t m, uintptr_t v, long n, uintptr_t step, float lr, float b1, float b2,
             float eps, float gscale, uintptr_t seg, int nseg, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(wd_adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<float*>(p),
                     reinterpret_cast<const float*>(g), reinterpret_cast<float*>(m), reinterpret_cast<float*>(v), n,
                     reinterpret_cast<const float*>(step), lr, b1, b2, eps, gscale,
                     reinterpret_cast<const long long*>(seg), nseg);
  FTM_CHECK_LAUNCH();
}

void wd_mask_colsum(uintptr_t x, uintptr_t h, uintptr_t db, int B, int n, uintptr_t stream) {
  if (n % 8 || x % 16 || h % 16) throw std::invalid_argument("wd_mask_colsum: n % 8 and 16-byte alignment");
  if (B <= 0 || n <= 0) return;
  hipLaunchKernelGGL(wd_mask_colsum_kernel, dim3((n + 15) / 16), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<bf16*>(x), reinterpret_cast<const bf16*>(h), reinterpret_cast<float*>(db), B, n);
  FTM_CHECK_LAUNCH();
}

void register_widedeep(pybind11::module_& m) {
  m.def("wd_gather", &wd_gather);
  m.def("wd_loss", &wd_loss);
  m.def("wd_keys", &wd_keys);
  m.def("wd_head_bwd", &wd_head_bwd);
  m.def("wd_head_bwd2", &wd_head_bwd2);
  m.def("wd_adam", &wd_adam);
  m.def("wd_mask_colsum", &wd_mask_colsum);
}
