// Fused multi-head attention forward (flash-style, online softmax) for the BERT path,
// plus the fused token-embedding + LayerNorm kernel and the token-packing kernel of the
// padding-free encoder (attention then runs per packed sequence via cu_seqlens).
//
// attention:  qkv [T = B*S, 3*H*D] bf16 straight from the fused QKV projection GEMM
// (Q | K | V column blocks, head h at columns h*D), key-padding mask from the token ids
// (id == pad_id -> masked), output ctx [T, H*D] bf16 — exactly the layout the output
// projection GEMM consumes, so no transposes exist anywhere in the layer.
//
// One workgroup = one (batch, head, QB-query block); QB/16 waves x 16 query rows (QB = 128
// for BERT's S <= 128, so K/V of a head are staged once).  Per 64-key block: K is staged
// row-major with a chunk XOR swizzle (conflict-free b128 fragment reads), V row-major
// (coalesced 16-B writes) and consumed transposed by ds_read_b64_tr_b16 (the hardware
// transpose read, guide T10) as the PV B operand.  S = Q K^T and O += P V run on
// v_mfma_f32_16x16x32_bf16; P goes through a per-wave LDS tile to become an A operand;
// softmax statistics are per row, reduced across the 16-lane column groups with
// __shfl_xor; the normalised O tile is staged through LDS and stored as whole 128-B rows.
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

constexpr int D = 64;      // head dim
constexpr int VP = D + 8;  // V row pitch (elements): tr-read rows land on distinct banks
constexpr int OP = D + 8;   // output staging row pitch
constexpr int QP = 16 + 4;  // P^T row pitch: [key][16 q] tiles, 40-B rows (tr-read friendly)

typedef short v4s __attribute__((ext_vector_type(4)));

FTM_DEVICE int kswz(int row, int chunk) { return row * D + ((chunk ^ (row & 7)) << 3); }

// 4 consecutive keys x 1 d column per lane (a 16-lane group reads 4 keys x 16 d columns)
FTM_DEVICE v4s tr_read(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)p);
}

// QB queries x KB keys per step (KB = 128 covers BERT's S <= 128 in ONE staging round:
// no second K/V round trip and no online-softmax rescale)
template <int QB, int KB>
__global__ __launch_bounds__(QB * 4) void attention_fwd_kernel(const bf16* __restrict__ qkv, const int* __restrict__ ids,
                                                               const int* __restrict__ cu, bf16* __restrict__ out, int B,
                                                               int S, int H, int pad_id, float scale_log2e) {
  constexpr int NW = QB / 16;  // waves
  constexpr int NTH = NW * 64;
  constexpr int NF = KB / 16;  // key fragments of S per wave
  __shared__ __attribute__((aligned(16))) bf16 Ks[KB * D];   // [key][d] swizzled
  __shared__ __attribute__((aligned(16))) bf16 Vs[KB * VP];  // [key][d] (+pad)
  __shared__ __attribute__((aligned(16))) bf16 Ps[NW][KB * QP];  // per-wave P^T, reused for O staging
  __shared__ float kmask[KB];

  const int qblocks = (S + QB - 1) / QB;
  const int bh = blockIdx.x / qblocks;
  const int qb = blockIdx.x % qblocks;
  const int b = bh / H, h = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ld = 3 * H * D;
  // padded batch: sequence b is rows [b*S, b*S + S), padding keys masked by id; packed
  // (cu != null): sequence b is rows [cu[b], cu[b+1]) of the token-packed batch, no padding
  const size_t tok0 = cu ? (size_t)cu[b] : (size_t)b * S;
  const int Sb = cu ? cu[b + 1] - cu[b] : S;
  if (qb * QB >= Sb) return;  // block-uniform: this query block lies past the sequence

  // Q fragments for this wave's 16 rows (A operand: row = lane&15, k = 8*(lane>>4) + j)
  const int qrow = qb * QB + wave * 16 + (lane & 15);
  bf16x8 qa[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (qrow < Sb)
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
  // this lane's supplier address inside a 4-key x 16-d transposed-read block
  const int trq = (lane & 15) >> 2, trp = lane & 3;

  const int nkb = (Sb + KB - 1) / KB;
  for (int kb = 0; kb < nkb; ++kb) {
    // ---- stage K (row-major, swizzled) and V (row-major) for keys kb*64 .. +63
    __syncthreads();
#pragma unroll
    for (int it = 0; it < (KB * 8 + NTH - 1) / NTH; ++it) {
      const int q = tid + it * NTH;  // 512 chunks of 8 elements
      if (q < KB * 8) {
        const int key = q >> 3, ch = q & 7;
        const int kg = kb * KB + key;
        u32x4 kv = {0u, 0u, 0u, 0u}, vv = {0u, 0u, 0u, 0u};
        if (kg < Sb) {
          const bf16* row = qkv + (tok0 + kg) * ld + h * D + ch * 8;
          kv = *reinterpret_cast<const u32x4*>(row + H * D);
          vv = *reinterpret_cast<const u32x4*>(row + 2 * H * D);
        }
        *reinterpret_cast<u32x4*>(Ks + kswz(key, ch)) = kv;
        *reinterpret_cast<u32x4*>(Vs + key * VP + ch * 8) = vv;
      }
    }
    if (tid < KB) {
      const int kg = kb * KB + tid;
      kmask[tid] = (kg < Sb && (cu || ids[tok0 + kg] != pad_id)) ? 0.f : -INFINITY;
    }
    __syncthreads();

    // ---- S = Q K^T  (16 q x KB keys per wave: NF fragments)
    f32x4 s[NF];
#pragma unroll
    for (int n = 0; n < NF; ++n) {
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
      for (int n = 0; n < NF; ++n) {
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
      alpha[r] = __builtin_amdgcn_exp2f(mrow[r] - mref);
      float sum = 0.f;
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const float pv = __builtin_amdgcn_exp2f(s[n][r] - mref);
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
    // ---- P^T -> per-wave LDS tile [64 keys][16 q]: a lane's 4 rows r are 4 consecutive q
    // of one key, i.e. one 8-byte store per fragment (instead of 4 scalar 2-byte stores)
    bf16* ps = Ps[wave];
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      bf16x4 pk;
      pk[0] = f2bf(s[n][0]); pk[1] = f2bf(s[n][1]); pk[2] = f2bf(s[n][2]); pk[3] = f2bf(s[n][3]);
      *reinterpret_cast<bf16x4*>(ps + (n * 16 + (lane & 15)) * QP + (lane >> 4) * 4) = pk;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P writes landed
    __builtin_amdgcn_wave_barrier();
    // ---- O += P V  (A = P[q][key]; B[key][d] by transposed reads of row-major V)
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      const int key0 = ks * 32 + (lane >> 4) * 8;  // this lane group's 8 keys
      // A = P[q][keys]: transposed reads of P^T (lane i <- q = i, 4 keys per read)
      const bf16* psrc = ps + (key0 + trq) * QP + trp * 4;
      const v4s plo = tr_read(psrc), phi = tr_read(psrc + 4 * QP);
      const bf16x8 pa = __builtin_bit_cast(bf16x8, __builtin_shufflevector(plo, phi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16* src = Vs + (key0 + trq) * VP + n * 16 + trp * 4;
        const v4s lo = tr_read(src), hi = tr_read(src + 4 * VP);
        // whole-vector reinterpretation (element-wise short->bf16 inserts miscompile here)
        const bf16x8 vb = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[n], 0, 0, 0);
      }
    }
  }

  // ---- normalise, stage the wave's [16 q][64 d] tile in its P slot, store 128-B rows
  bf16* os = Ps[wave];
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = lrow[r] > 0.f ? 1.f / lrow[r] : 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n) os[((lane >> 4) * 4 + r) * OP + n * 16 + (lane & 15)] = f2bf(o[n][r] * inv);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = lane + it * 64;  // 16 rows x 8 chunks
    const int r = c >> 3, ch = c & 7;
    const int q = qb * QB + wave * 16 + r;
    if (q < Sb)
      *reinterpret_cast<u32x4*>(out + (tok0 + q) * (H * D) + h * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(os + r * OP + ch * 8);
  }
}

// x[t] = LN(word[ids[t]] + pos[t % S] + type[tt[t]]) * gamma + beta   (D % 8 == 0, D <= 1024)
template <int MAXV>
__global__ __launch_bounds__(256) void embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ tt,
                                                       const int* __restrict__ pos_ids,
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
  const bf16* pp = pos + (size_t)(pos_ids ? pos_ids[t] : t % S) * D;
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

// Token packing for padding-free encoders: the non-pad tokens of ids[B, S] (row order)
// -> packed[0, T_eff) with their in-row positions, cu[B + 1] row offsets and cls[B] (row
// starts, where each row's first token lands); rows [T_eff, T_cap) are zero-filled.  One
// 1024-thread workgroup (B <= 1024): per-row counts by wave ballots, an LDS scan, then a
// ballot-ranked scatter.  Writes past T_cap are dropped (the host sizes T_cap >= T_eff).
__global__ __launch_bounds__(1024) void pack_tokens_kernel(const int* __restrict__ ids, int B, int S, int pad_id,
                                                           int T_cap, int* __restrict__ packed,
                                                           int* __restrict__ pos, int* __restrict__ cu,
                                                           int* __restrict__ cls) {
  __shared__ int lens[1024];
  __shared__ int starts[1025];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int r = wave; r < B; r += 16) {
    int n = 0;
    for (int c = 0; c < S; c += 64) {
      const bool ok = c + lane < S && ids[(size_t)r * S + c + lane] != pad_id;
      n += __popcll(__ballot(ok));
    }
    if (lane == 0) lens[r] = n;
  }
  __syncthreads();
  if (tid == 0) {  // B <= 1024 row counts: a serial scan is ~1 us, below the launch cost
    int acc = 0;
    for (int r = 0; r < B; ++r) {
      starts[r] = acc;
      acc += lens[r];
    }
    starts[B] = acc;
  }
  __syncthreads();
  for (int r = tid; r <= B; r += 1024) cu[r] = starts[r];
  for (int r = tid; r < B; r += 1024) cls[r] = starts[r] < T_cap ? starts[r] : T_cap - 1;
  for (int r = wave; r < B; r += 16) {
    int dst = starts[r];
    for (int c = 0; c < S; c += 64) {
      const int tok = c + lane < S ? ids[(size_t)r * S + c + lane] : pad_id;
      const bool ok = c + lane < S && tok != pad_id;
      const unsigned long long m = __ballot(ok);
      const int d = dst + __popcll(m & below);
      if (ok && d < T_cap) {
        packed[d] = tok;
        pos[d] = c + lane;
      }
      dst += __popcll(m);
    }
  }
  for (int t = starts[B] + tid; t < T_cap; t += 1024) {
    packed[t] = pad_id;
    pos[t] = 0;
  }
}

// First-token ("CLS") attention of a packed batch: the final encoder layer of a sequence
// classifier only needs each sequence's first row, so its attention is one query per
// (sequence, head).  One wave per (b, h): lanes score keys (q . k_j, 64-d dot products from
// 16-B loads), the softmax is a wave reduction, then lane d accumulates sum_j p_j v_j[d]
// over coalesced 128-B V rows.  out [B, H*64] bf16.
__global__ __launch_bounds__(256) void cls_attention_kernel(const bf16* __restrict__ qkv, const int* __restrict__ cu,
                                                            bf16* __restrict__ out, int B, int H, float scale_log2e) {
  __shared__ float probs[4][512];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;  // wave-uniform; no block barrier below
  const int b = bh / H, h = bh % H;
  const int ld = 3 * H * D;
  const int t0 = cu[b];
  const int n = min(cu[b + 1] - t0, 512);
  const bf16* qrow = qkv + (size_t)t0 * ld + h * D;
  float q[D];
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[c * 8 + e] = (float)v[e];
  }
  float mx = -INFINITY;
  for (int j = lane; j < n; j += 64) {
    const bf16* krow = qkv + (size_t)(t0 + j) * ld + H * D + h * D;
    float sdot = 0.f;
#pragma unroll
    for (int c = 0; c < D / 8; ++c) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(krow + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) sdot += q[c * 8 + e] * (float)v[e];
    }
    sdot *= scale_log2e;
    probs[wave][j] = sdot;
    mx = fmaxf(mx, sdot);
  }
  mx = wave_reduce_max(mx);
  float sum = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float p = __builtin_amdgcn_exp2f(probs[wave][j] - mx);
    probs[wave][j] = p;
    sum += p;
  }
  sum = wave_reduce_sum(sum);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's probabilities are in LDS
  float acc = 0.f;
  const bf16* vcol = qkv + (size_t)t0 * ld + 2 * H * D + h * D + lane;
  for (int j = 0; j < n; ++j) acc += probs[wave][j] * (float)vcol[(size_t)j * ld];
  out[(size_t)b * H * D + h * D + lane] = f2bf(n > 0 ? acc / sum : 0.f);
}

}  // namespace

void pack_tokens(uintptr_t ids, int B, int S, int pad_id, int T_cap, uintptr_t packed, uintptr_t pos, uintptr_t cu,
                 uintptr_t cls, uintptr_t stream) {
  if (B <= 0 || B > 1024 || S <= 0 || T_cap <= 0) throw std::invalid_argument("pack_tokens: need 0 < B <= 1024");
  hipLaunchKernelGGL(pack_tokens_kernel, dim3(1), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const int*>(ids), B, S, pad_id, T_cap, reinterpret_cast<int*>(packed),
                     reinterpret_cast<int*>(pos), reinterpret_cast<int*>(cu), reinterpret_cast<int*>(cls));
  FTM_CHECK_LAUNCH();
}

void attention_fwd_bf16(uintptr_t qkv, uintptr_t ids, uintptr_t cu_seqlens, uintptr_t out, int B, int S, int H,
                        int Dh, int pad_id, float scale, uintptr_t stream) {
  if (Dh != D) throw std::invalid_argument("attention_fwd: head dim must be 64");
  if (B <= 0 || S <= 0 || H <= 0) throw std::invalid_argument("attention_fwd: empty problem");
  if (qkv % 16 || out % 16) throw std::invalid_argument("attention_fwd: pointers must be 16-byte aligned");
  const float kLog2e = 1.4426950408889634f;
  auto st = reinterpret_cast<hipStream_t>(stream);
  auto Q = reinterpret_cast<const bf16*>(qkv);
  auto I = reinterpret_cast<const int*>(ids);
  auto CU = reinterpret_cast<const int*>(cu_seqlens);
  if (!I && !CU) throw std::invalid_argument("attention_fwd: need token ids (padded) or cu_seqlens (packed)");
  auto O = reinterpret_cast<bf16*>(out);
  if (S > 64) {  // 128-query blocks: K/V of a head staged once for S <= 128
    const int qblocks = (S + 127) / 128;
    hipLaunchKernelGGL((attention_fwd_kernel<128, 128>), dim3(B * H * qblocks), dim3(512), 0, st, Q, I, CU, O, B, S,
                       H, pad_id, scale * kLog2e);
  } else {
    const int qblocks = (S + 63) / 64;
    hipLaunchKernelGGL((attention_fwd_kernel<64, 64>), dim3(B * H * qblocks), dim3(256), 0, st, Q, I, CU, O, B, S, H,
                       pad_id, scale * kLog2e);
  }
  FTM_CHECK_LAUNCH();
}

void embed_ln_bf16(uintptr_t ids, uintptr_t tt, uintptr_t pos_ids, uintptr_t word, uintptr_t pos, uintptr_t type,
                   uintptr_t gamma, uintptr_t beta, uintptr_t y, int T, int S, int D, int vocab, float eps,
                   uintptr_t stream) {
  if (D % 8 || D > 2048) throw std::invalid_argument("embed_ln: D must be a multiple of 8 and <= 2048");
  dim3 grid((T + 3) / 4), block(256);
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto I = reinterpret_cast<const int*>(ids);
  auto TT = reinterpret_cast<const int*>(tt);
  auto PI = reinterpret_cast<const int*>(pos_ids);
  auto Wd = reinterpret_cast<const bf16*>(word);
  auto P = reinterpret_cast<const bf16*>(pos);
  auto Ty = reinterpret_cast<const bf16*>(type);
  auto G = reinterpret_cast<const float*>(gamma);
  auto Bt = reinterpret_cast<const float*>(beta);
  auto Y = reinterpret_cast<bf16*>(y);
  if (D <= 512) hipLaunchKernelGGL(embed_ln_kernel<1>, grid, block, 0, s, I, TT, PI, Wd, P, Ty, G, Bt, Y, T, S, D, vocab, eps);
  else if (D <= 1024) hipLaunchKernelGGL(embed_ln_kernel<2>, grid, block, 0, s, I, TT, PI, Wd, P, Ty, G, Bt, Y, T, S, D, vocab, eps);
  else hipLaunchKernelGGL(embed_ln_kernel<4>, grid, block, 0, s, I, TT, PI, Wd, P, Ty, G, Bt, Y, T, S, D, vocab, eps);
  FTM_CHECK_LAUNCH();
}

// Diagnostic: LDS[r][c] = r * 256 + c (16-bit, 16 rows x 64 cols); every lane issues one
// transposed read at (row = 4*(lane>>4) + ((lane&15)>>2), col = 4*(lane&3) + 16*blk);
// out[lane][0..3] = the 4 returned elements.
__global__ void probe_tr_kernel(short* out, int blk) {
  __shared__ __attribute__((aligned(16))) short t[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) t[i] = (short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  const int lane = threadIdx.x;
  const int row = 4 * (lane >> 4) + ((lane & 15) >> 2), col = 4 * (lane & 3) + 16 * blk;
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(t + row * 64 + col));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}

void probe_tr_read(uintptr_t out, int blk, uintptr_t stream) {
  hipLaunchKernelGGL(probe_tr_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<short*>(out), blk);
  FTM_CHECK_LAUNCH();
}

void cls_attention_bf16(uintptr_t qkv, uintptr_t cu, uintptr_t out, int B, int H, int Dh, float scale,
                        uintptr_t stream) {
  if (Dh != D) throw std::invalid_argument("cls_attention: head dim must be 64");
  if (B <= 0 || H <= 0 || !cu) throw std::invalid_argument("cls_attention: empty problem / no cu_seqlens");
  if (qkv % 16 || out % 2) throw std::invalid_argument("cls_attention: misaligned pointers");
  const int waves = B * H;
  hipLaunchKernelGGL(cls_attention_kernel, dim3((waves + 3) / 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16*>(qkv), reinterpret_cast<const int*>(cu), reinterpret_cast<bf16*>(out),
                     B, H, scale * 1.4426950408889634f);
  FTM_CHECK_LAUNCH();
}

void register_attention(pybind11::module_& m) {
  m.def("cls_attention_bf16", &cls_attention_bf16);
  m.def("probe_tr_read", &probe_tr_read);
  m.def("attention_fwd_bf16", &attention_fwd_bf16);
  m.def("embed_ln_bf16", &embed_ln_bf16);
  m.def("pack_tokens", &pack_tokens);
}
