// Fused multi-head attention forward (flash-style, online softmax) for the BERT path,
// plus the fused token-embedding + LayerNorm kernel.
//
// attention:  qkv [T = B*S, 3*H*D] bf16 straight from the fused QKV projection GEMM
// (Q | K | V column blocks, head h at columns h*D), key-padding mask from the token ids
// (id == pad_id -> masked), output ctx [T, H*D] bf16 — exactly the layout the output
// projection GEMM consumes, so no transposes exist anywhere in the layer.
//
// One workgroup = one (batch, head, 64-query block); 4 waves x 16 query rows.  Per 64-key
// block: K is staged row-major (d-contiguous, chunk-swizzled) and V transposed ([d][key])
// in LDS; S = Q K^T and O += P V run on v_mfma_f32_16x16x32_bf16 (D = 64: 2 k-steps for
// QK^T, 2 for PV); P goes through a per-wave LDS tile to become an A operand.  Softmax
// statistics are per-row, reduced across the 16-lane column groups with __shfl_xor.
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

constexpr int D = 64;     // head dim
constexpr int QB = 64;    // queries per workgroup
constexpr int KB = 64;    // keys per block

FTM_DEVICE int kswz(int row, int chunk) { return row * D + ((chunk ^ (row & 7)) << 3); }

__global__ __launch_bounds__(256) void attention_fwd_kernel(const bf16* __restrict__ qkv, const int* __restrict__ ids,
                                                            bf16* __restrict__ out, int B, int S, int H, int pad_id,
                                                            float scale_log2e) {
  __shared__ __attribute__((aligned(16))) bf16 Ks[KB * D];       // [key][d] swizzled
  __shared__ __attribute__((aligned(16))) bf16 Vt[D * (KB + 8)];  // [d][key] (+pad)
  __shared__ __attribute__((aligned(16))) bf16 Ps[4][16 * (KB + 8)];
  __shared__ float kmask[KB];

  const int qblocks = (S + QB - 1) / QB;
  const int bh = blockIdx.x / qblocks;
  const int qb = blockIdx.x % qblocks;
  const int b = bh / H, h = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ld = 3 * H * D;
  const size_t tok0 = (size_t)b * S;

  // Q fragments for this wave's 16 rows (A operand: row = lane&15, k = 8*(lane>>4) + j)
  const int qrow = qb * QB + wave * 16 + (lane & 15);
  bf16x8 qa[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (qrow < S)
      qa[ks] = *reinterpret_cast<const bf16x8*>(qkv + (tok0 + qrow) * ld + h * D + ks * 32 + (lane >> 4) * 8);
    else
      qa[ks] = bf16x8{};
  }

  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    mrow[r] = -INFINITY;
    lrow[r] = 0.f;
  }

  const int nkb = (S + KB - 1) / KB;
  for (int kb = 0; kb < nkb; ++kb) {
    // ---- stage K (row-major, swizzled) and V (transposed) for keys kb*64 .. +63
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int q = tid + it * 256;        // 512 chunks of 8 elements
      const int key = q >> 3, ch = q & 7;
      const int kg = kb * KB + key;
      u32x4 kv = {0u, 0u, 0u, 0u}, vv = {0u, 0u, 0u, 0u};
      if (kg < S) {
        const bf16* row = qkv + (tok0 + kg) * ld + h * D + ch * 8;
        kv = *reinterpret_cast<const u32x4*>(row + H * D);
        vv = *reinterpret_cast<const u32x4*>(row + 2 * H * D);
      }
      *reinterpret_cast<u32x4*>(Ks + kswz(key, ch)) = kv;
      const bf16x8 v8 = *reinterpret_cast<const bf16x8*>(&vv);
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(ch * 8 + e) * (KB + 8) + key] = v8[e];
    }
    if (tid < KB) {
      const int kg = kb * KB + tid;
      kmask[tid] = (kg < S && ids[tok0 + kg] != pad_id) ? 0.f : -INFINITY;
    }
    __syncthreads();

    // ---- S = Q K^T  (16 q x 64 keys per wave: 4 fragments)
    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + kswz(n * 16 + (lane & 15), ks * 4 + (lane >> 4)));
        s[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], kf, s[n], 0, 0, 0);
      }
    }
    // lane holds S[q = (lane>>4)*4 + r][key = n*16 + (lane&15)]
    float mnew[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        s[n][r] = s[n][r] * scale_log2e + kmask[n * 16 + (lane & 15)];
        mx = fmaxf(mx, s[n][r]);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      mnew[r] = fmaxf(mrow[r], mx);
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mref = mnew[r] == -INFINITY ? 0.f : mnew[r];
      alpha[r] = exp2f(mrow[r] - mref);
      float sum = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float pv = exp2f(s[n][r] - mref);
        s[n][r] = pv;
        sum += pv;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
      lrow[r] = lrow[r] * alpha[r] + sum;
      mrow[r] = mnew[r];
    }
    // rescale O (o[n][r] belongs to row (lane>>4)*4 + r)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[n][r] *= alpha[r];
    // ---- P -> per-wave LDS tile [16 q][64 keys] (bf16)
    bf16* ps = Ps[wave];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) ps[((lane >> 4) * 4 + r) * (KB + 8) + n * 16 + (lane & 15)] = f2bf(s[n][r]);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P writes landed
    __builtin_amdgcn_wave_barrier();
    // ---- O += P V  (A = P[q][key], B = V[key][d] read from Vt[d][key])
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(ps + (lane & 15) * (KB + 8) + ks * 32 + (lane >> 4) * 8);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 vb =
            *reinterpret_cast<const bf16x8*>(Vt + (n * 16 + (lane & 15)) * (KB + 8) + ks * 32 + (lane >> 4) * 8);
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[n], 0, 0, 0);
      }
    }
  }

  // ---- normalise and store: o[n][r] = O[q = (lane>>4)*4 + r][d = n*16 + (lane&15)]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = qb * QB + wave * 16 + (lane >> 4) * 4 + r;
    if (q >= S) continue;
    const float inv = lrow[r] > 0.f ? 1.f / lrow[r] : 0.f;
    bf16* dst = out + (tok0 + q) * (H * D) + h * D;
#pragma unroll
    for (int n = 0; n < 4; ++n) dst[n * 16 + (lane & 15)] = f2bf(o[n][r] * inv);
  }
}

// x[t] = LN(word[ids[t]] + pos[t % S] + type[tt[t]]) * gamma + beta   (D % 8 == 0, D <= 1024)
template <int MAXV>
__global__ __launch_bounds__(256) void embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ tt,
                                                       const bf16* __restrict__ word, const bf16* __restrict__ pos,
                                                       const bf16* __restrict__ type, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, bf16* __restrict__ y, int T,
                                                       int S, int D, int vocab, float eps) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const int ty = tt ? tt[t] : 0;
  const bf16* wp = word + (size_t)id * D;
  const bf16* pp = pos + (size_t)(t % S) * D;
  const bf16* tp = type + (size_t)ty * D;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < D) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(wp + c);
      const bf16x8 p = *reinterpret_cast<const bf16x8*>(pp + c);
      const bf16x8 q = *reinterpret_cast<const bf16x8*>(tp + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[i][e] = (float)a[e] + (float)p[e] + (float)q[e];
        s += v[i][e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  const float mean = wave_reduce_sum(s) / D;
  float qsum = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if ((lane + 64 * i) * 8 < D)
#pragma unroll
      for (int e = 0; e < 8; ++e) qsum += (v[i][e] - mean) * (v[i][e] - mean);
  const float rstd = rsqrtf(wave_reduce_sum(qsum) / D + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c >= D) continue;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf((v[i][e] - mean) * rstd * gamma[c + e] + beta[c + e]);
    *reinterpret_cast<bf16x8*>(y + (size_t)t * D + c) = o;
  }
}

}  // namespace

void attention_fwd_bf16(uintptr_t qkv, uintptr_t ids, uintptr_t out, int B, int S, int H, int Dh, int pad_id,
                        float scale, uintptr_t stream) {
  if (Dh != D) throw std::invalid_argument("attention_fwd: head dim must be 64");
  if (B <= 0 || S <= 0 || H <= 0) throw std::invalid_argument("attention_fwd: empty problem");
  if (qkv % 16 || out % 16) throw std::invalid_argument("attention_fwd: pointers must be 16-byte aligned");
  const int qblocks = (S + QB - 1) / QB;
  const float kLog2e = 1.4426950408889634f;
  hipLaunchKernelGGL(attention_fwd_kernel, dim3(B * H * qblocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16*>(qkv), reinterpret_cast<const int*>(ids), reinterpret_cast<bf16*>(out),
                     B, S, H, pad_id, scale * kLog2e);
  FTM_CHECK_LAUNCH();
}

void embed_ln_bf16(uintptr_t ids, uintptr_t tt, uintptr_t word, uintptr_t pos, uintptr_t type, uintptr_t gamma,
                   uintptr_t beta, uintptr_t y, int T, int S, int D, int vocab, float eps, uintptr_t stream) {
  if (D % 8 || D > 2048) throw std::invalid_argument("embed_ln: D must be a multiple of 8 and <= 2048");
  dim3 grid((T + 3) / 4), block(256);
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto I = reinterpret_cast<const int*>(ids);
  auto TT = reinterpret_cast<const int*>(tt);
  auto Wd = reinterpret_cast<const bf16*>(word);
  auto P = reinterpret_cast<const bf16*>(pos);
  auto Ty = reinterpret_cast<const bf16*>(type);
  auto G = reinterpret_cast<const float*>(gamma);
  auto Bt = reinterpret_cast<const float*>(beta);
  auto Y = reinterpret_cast<bf16*>(y);
  if (D <= 512) hipLaunchKernelGGL(embed_ln_kernel<1>, grid, block, 0, s, I, TT, Wd, P, Ty, G, Bt, Y, T, S, D, vocab, eps);
  else if (D <= 1024) hipLaunchKernelGGL(embed_ln_kernel<2>, grid, block, 0, s, I, TT, Wd, P, Ty, G, Bt, Y, T, S, D, vocab, eps);
  else hipLaunchKernelGGL(embed_ln_kernel<4>, grid, block, 0, s, I, TT, Wd, P, Ty, G, Bt, Y, T, S, D, vocab, eps);
  FTM_CHECK_LAUNCH();
}

void register_attention(pybind11::module_& m) {
  m.def("attention_fwd_bf16", &attention_fwd_bf16);
  m.def("embed_ln_bf16", &embed_ln_bf16);
}
