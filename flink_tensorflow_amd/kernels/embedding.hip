// Embedding kernels for the Wide&Deep online-training path (and BERT-style lookups).
//
//   embedding_bag_fwd   out[b, f*D + d] = sum_l table[ids[b, f, l], d]     (ids < 0 skipped)
//                       fp32 master table -> bf16 activations (16-B vector loads/stores)
//   segment_sum_rows    row-sparse backward: gradient rows are grouped by destination with a
//                       sort (done by the caller on the GPU), then every destination row is
//                       summed by ONE wave in a fixed order — deterministic, no float atomics
//                       (guide Appendix B "Scatter / gather / embedding": store-and-sum form)
//   sparse_adagrad      table[u] -= lr * g / (sqrt(acc[u] += g^2) + eps) on the touched rows
//
// D % 8 == 0 (D/8 a power of two); lane groups of D/8 lanes per row for the small rows of
// recommender tables, 8 elements per lane.
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

// One LANE GROUP of G = D/8 lanes per (bag, field) row (G a power of two <= 64; 64/G rows
// per wave), 8 consecutive elements per lane.  With the Wide&Deep shapes (D = 32 / 8) a
// whole wave per row left 60 / 63 of its lanes idle.
__global__ __launch_bounds__(256) void embedding_bag_fwd_kernel(const int* __restrict__ ids,
                                                                const float* __restrict__ table,
                                                                bf16* __restrict__ out, int rows, int L, int D,
                                                                int gshift, int V) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int r = t >> gshift;  // r = b * F + f
  if (r >= rows) return;
  const int c = (t & ((1 << gshift) - 1)) * 8;
  const int* idp = ids + (size_t)r * L;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int l = 0; l < L; ++l) {
    const int id = idp[l];
    if (id < 0 || id >= V) continue;
    const f32x4* src = reinterpret_cast<const f32x4*>(table + (size_t)id * D + c);
    const f32x4 a = src[0], b = src[1];
    acc[0] += a[0]; acc[1] += a[1]; acc[2] += a[2]; acc[3] += a[3];
    acc[4] += b[0]; acc[5] += b[1]; acc[6] += b[2]; acc[7] += b[3];
  }
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
  // out row b, field f -> column f*D (the F field blocks are contiguous per row)
  *reinterpret_cast<bf16x8*>(out + (size_t)r * D + c) = o;
}

// grad rows: grad_out[(b*F+f), :] (bf16 or fp32, pitch D); perm lists source rows sorted
// by destination; seg[u]..seg[u+1] is destination u's range in perm.
// One wave per destination row.  The wave's lanes are CW column chunks (8 elements each)
// x RG = 64 / CW row groups: row group g sums rows s0+g, s0+g+RG, ... (many independent
// loads in flight for hot ids), then the RG partials are combined by a fixed xor-shuffle
// tree — the summation order depends only on the segment, so results are bit-identical
// run to run.  D > 8 * 64 loops over 512-column blocks with RG = 1.
template <typename T, int CW>
__global__ __launch_bounds__(256) void segment_sum_rows_kernel(const T* __restrict__ grad, const int* __restrict__ perm,
                                                               const int* __restrict__ seg, float* __restrict__ out,
                                                               int U, int D, int L) {
  constexpr int RG = 64 / CW;
  const int lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U) return;
  const int s0 = seg[u], s1 = seg[u + 1];
  const int cl = lane % CW;
  const int rg = lane / CW;
  for (int c0 = 0; c0 < D; c0 += CW * 8) {
    const int c = c0 + cl * 8;
    const bool cv = c < D;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cv) {
      for (int i = s0 + rg; i < s1; i += RG) {
        const int src = perm[i] / L;  // bag element -> its (b, f) output row
        if constexpr (sizeof(T) == 2) {
          const bf16x8 g = *reinterpret_cast<const bf16x8*>(grad + (size_t)src * D + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += (float)g[e];
        } else {
          const f32x4* gp = reinterpret_cast<const f32x4*>(grad + (size_t)src * D + c);
          const f32x4 a = gp[0], b = gp[1];
          acc[0] += a[0]; acc[1] += a[1]; acc[2] += a[2]; acc[3] += a[3];
          acc[4] += b[0]; acc[5] += b[1]; acc[6] += b[2]; acc[7] += b[3];
        }
      }
    }
#pragma unroll
    for (int off = CW; off < 64; off <<= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], off, 64);
    }
    if (rg == 0 && cv) {
      f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)u * D + c);
      dst[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
      dst[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
    }
  }
}

// Lane-group variant: G = D/8 lanes per destination, 64/G destinations per wave.
// 1. every lane group whose segment is short (<= SHORT rows) sums it serially in perm order
//    with four interleaved accumulators (i mod 4) combined in a fixed order;
// 2. the wave then takes its long segments (hot ids: Zipf-distributed categorical data puts
//    ~1/4 of a field's lookups on one id) one at a time with all 64 lanes, lane = (row group
//    rg, column chunk), RG = 64/G row groups, fixed xor-tree combine.
// Each destination's path and summation order depend only on its own segment, so replicas
// given the same input agree bitwise (no float atomics).
template <typename T, int G>
__global__ __launch_bounds__(256) void segment_sum_rows_grp_kernel(const T* __restrict__ grad,
                                                                   const int* __restrict__ perm,
                                                                   const int* __restrict__ seg,
                                                                   float* __restrict__ out, int U, int D, int L) {
  constexpr int SHORT = 16;
  constexpr int PER_WAVE = 64 / G;
  constexpr int RG = 64 / G;
  const int lane = threadIdx.x & 63;
  const int u0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * PER_WAVE;
  if (u0 >= U) return;
  const int gi = lane / G;
  const int c = (lane % G) * 8;
  const int u = u0 + gi;
  const bool live = u < U;
  const int s0 = live ? seg[u] : 0, s1 = live ? seg[u + 1] : 0;
  auto load8 = [&](int i, float* a) {
    const int src = perm[i] / L;
    if constexpr (sizeof(T) == 2) {
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(grad + (size_t)src * D + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += (float)g[e];
    } else {
      const f32x4* gp = reinterpret_cast<const f32x4*>(grad + (size_t)src * D + c);
      const f32x4 x = gp[0], y = gp[1];
      a[0] += x[0]; a[1] += x[1]; a[2] += x[2]; a[3] += x[3];
      a[4] += y[0]; a[5] += y[1]; a[6] += y[2]; a[7] += y[3];
    }
  };
  auto store8 = [&](int uu, const float* o) {
    f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)uu * D + c);
    dst[0] = f32x4{o[0], o[1], o[2], o[3]};
    dst[1] = f32x4{o[4], o[5], o[6], o[7]};
  };
  const bool is_long = live && s1 - s0 > SHORT;
  if (live && !is_long) {
    float acc[4][8] = {};
    int i = s0;
    for (; i + 3 < s1; i += 4) {
      load8(i, acc[0]);
      load8(i + 1, acc[1]);
      load8(i + 2, acc[2]);
      load8(i + 3, acc[3]);
    }
    const int rem = s1 - i;  // static accumulator indices: no dynamic register indexing
    if (rem > 0) load8(i, acc[0]);
    if (rem > 1) load8(i + 1, acc[1]);
    if (rem > 2) load8(i + 2, acc[2]);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (acc[0][e] + acc[1][e]) + (acc[2][e] + acc[3][e]);
    store8(u, o);
  }
  // long segments of this wave, cooperatively (lane group gi of destination u is "long"
  // -> bit gi*G of the ballot; one destination per iteration, lowest first)
  unsigned long long longs = __ballot(is_long && (lane % G) == 0);
  const int rg = lane / G;
  while (longs) {
    const int k = __builtin_ctzll(longs) / G;
    longs &= longs - 1;
    const int uu = u0 + k;
    const int a0 = seg[uu], a1 = seg[uu + 1];
    // 8 rows in flight per lane (hot segments are latency-bound chains of perm -> row
    // loads), accumulators combined in a fixed tree
    float q[8][8] = {};
    for (int i = a0 + rg; i < a1; i += 8 * RG) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i + j * RG < a1) load8(i + j * RG, q[j]);
    }
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      acc[e] = ((q[0][e] + q[1][e]) + (q[2][e] + q[3][e])) + ((q[4][e] + q[5][e]) + (q[6][e] + q[7][e]));
#pragma unroll
    for (int off = G; off < 64; off <<= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], off, 64);
    }
    if (rg == 0) store8(uu, acc);
  }
}

// Reduce-by-key over the SORTED rows in fixed slices (static-shape pipeline): hot ids
// (Zipf-distributed categoricals put thousands of a batch's lookups on one id) no longer
// serialise on the one wave that owns their destination.
//  pass 1 (segsum_slices): lane group (G = D/8 lanes) k walks sorted rows [kS, kS + S)
//    in order, 8 rows in flight; a run wholly inside the slice is written to out[run]; the
//    part of a run that started before the slice goes to head[k], the part of a run that
//    continues past it to tail[k];
//  pass 2 (segsum_fixup): one wave per destination: runs spanning slices k0..k1 sum
//    tail[k0] + head[k0+1 .. k1] (RG row groups + fixed xor tree); empty (padding)
//    destinations get zero rows.
// Every sum has a fixed order: bit-identical across runs and replicas.
template <typename T, int G>
__global__ __launch_bounds__(256) void segsum_slices_kernel(const T* __restrict__ grad, const int* __restrict__ perm,
                                                            const int* __restrict__ seg_id,
                                                            const int* __restrict__ seg, float* __restrict__ out,
                                                            float* __restrict__ head, float* __restrict__ tail, int n,
                                                            int D, int L, int S, int lo, int hi) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long k = t / G;
  const int c = (int)(t % G) * 8;
  const long i0 = k * S;
  if (i0 >= n) return;
  const long i1 = i0 + S < n ? i0 + S : n;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int cur = seg_id[i0];
  auto flush = [&](int r) {
    const int rs = seg[r], re = seg[r + 1];
    float* dst = (rs >= i0 && re <= i1) ? out + (size_t)r * D : (rs < i0 ? head : tail) + (size_t)k * D;
    reinterpret_cast<f32x4*>(dst + c)[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    reinterpret_cast<f32x4*>(dst + c)[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
  };
  for (long b0 = i0; b0 < i1; b0 += 8) {
    float row[8][8];
    int rid[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // 8 independent perm -> row loads in flight
      const long i = b0 + j;
      rid[j] = i < i1 ? seg_id[i] : -1;
      const int pi = i < i1 ? perm[i] : lo - 1;
      if (pi >= lo && pi < hi) {  // rows of another table sharing the key space add nothing
        const int src = (pi - lo) / L;
        if constexpr (sizeof(T) == 2) {
          const bf16x8 gv = *reinterpret_cast<const bf16x8*>(grad + (size_t)src * D + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) row[j][e] = (float)gv[e];
        } else {
          const f32x4* gp = reinterpret_cast<const f32x4*>(grad + (size_t)src * D + c);
          const f32x4 x = gp[0], y = gp[1];
          row[j][0] = x[0]; row[j][1] = x[1]; row[j][2] = x[2]; row[j][3] = x[3];
          row[j][4] = y[0]; row[j][5] = y[1]; row[j][6] = y[2]; row[j][7] = y[3];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) row[j][e] = 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (rid[j] < 0) break;
      if (rid[j] != cur) {
        flush(cur);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
        cur = rid[j];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += row[j][e];
    }
  }
  flush(cur);
}

template <int G>
__global__ __launch_bounds__(256) void segsum_fixup_kernel(const int* __restrict__ seg, float* __restrict__ out,
                                                           const float* __restrict__ head,
                                                           const float* __restrict__ tail, int U, int D, int S) {
  constexpr int RG = 64 / G;
  const int lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= U) return;
  const int rs = seg[u], re = seg[u + 1];
  const int rg = lane / G;
  const int c = (lane % G) * 8;
  if (re <= rs) {  // empty (padding) destination
    if (rg == 0) {
      reinterpret_cast<f32x4*>(out + (size_t)u * D + c)[0] = f32x4{0.f, 0.f, 0.f, 0.f};
      reinterpret_cast<f32x4*>(out + (size_t)u * D + c)[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    return;
  }
  const int k0 = rs / S, k1 = (re - 1) / S;
  if (k0 == k1) return;  // written whole by its slice
  const int cnt = k1 - k0 + 1;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j = rg; j < cnt; j += RG) {
    const float* src = (j == 0 ? tail : head) + (size_t)(k0 + j) * D + c;
    const f32x4 x = reinterpret_cast<const f32x4*>(src)[0], y = reinterpret_cast<const f32x4*>(src)[1];
    acc[0] += x[0]; acc[1] += x[1]; acc[2] += x[2]; acc[3] += x[3];
    acc[4] += y[0]; acc[5] += y[1]; acc[6] += y[2]; acc[7] += y[3];
  }
#pragma unroll
  for (int off = G; off < 64; off <<= 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], off, 64);
  }
  if (rg == 0) {
    reinterpret_cast<f32x4*>(out + (size_t)u * D + c)[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    reinterpret_cast<f32x4*>(out + (size_t)u * D + c)[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
}

// Segment boundaries of a sorted key array, static shapes: for every i that starts a run
// (i == 0 or sorted[i] != sorted[i-1]) with run index s = seg_id[i]:  seg[s] = i and
// uids[s] = key (or -1 for the invalid bucket key == num_rows).  Each run is written by
// exactly one thread: deterministic, no atomics, no host round trip.
__global__ __launch_bounds__(256) void segment_starts_kernel(const int* __restrict__ sorted,
                                                             const int* __restrict__ seg_id, int* __restrict__ seg,
                                                             int* __restrict__ uids, int n, int num_rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = sorted[i];
  if (i == 0 || sorted[i - 1] != k) {
    const int sidx = seg_id[i];
    seg[sidx] = i;
    uids[sidx] = k >= num_rows ? -1 : (int)k;
  }
}

// G = D/4 lanes per touched row (a power of two <= 64), 4 elements per lane.
__global__ __launch_bounds__(256) void sparse_adagrad_kernel(float* __restrict__ table, float* __restrict__ accum,
                                                             const int* __restrict__ uids, const float* __restrict__ g,
                                                             int U, int D, int V, float lr, float eps, int gshift,
                                                             int off) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int u = t >> gshift;
  if (u >= U) return;
  const int id = uids[u] < 0 ? -1 : uids[u] - off;  // off: this table's base in a shared key space
  if (id < 0 || id >= V) return;  // padding of the static-shape sparse pipeline
  const int c = (t & ((1 << gshift) - 1)) * 4;
  const size_t row = (size_t)id * D;
  f32x4 gv = *reinterpret_cast<const f32x4*>(g + (size_t)u * D + c);
  f32x4 av = *reinterpret_cast<f32x4*>(accum + row + c);
  f32x4 tv = *reinterpret_cast<f32x4*>(table + row + c);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    av[e] += gv[e] * gv[e];
    tv[e] -= lr * gv[e] / (sqrtf(av[e]) + eps);
  }
  *reinterpret_cast<f32x4*>(accum + row + c) = av;
  *reinterpret_cast<f32x4*>(table + row + c) = tv;
}

// Row moves of the bucketed owner exchange (parallel/sparse_exchange.py): slot k carries
// table row ids[k] (ids outside [0, V) are padding).  gather: out[k] = table[ids[k]] (zeros
// for padding); scatter: table[ids[k]] = rows[k] (padding skipped; ids are unique).  One
// thread per 4 floats of a row.
__global__ __launch_bounds__(256) void rows_gather_kernel(const float* __restrict__ table, const int* __restrict__ ids,
                                                          float* __restrict__ out, long n, int D, int V, int gs) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long k = t >> gs;
  if (k >= n) return;
  const int c = (int)(t & ((1 << gs) - 1)) * 4;
  const int id = ids[k];
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (id >= 0 && id < V) v = *reinterpret_cast<const f32x4*>(table + (size_t)id * D + c);
  *reinterpret_cast<f32x4*>(out + k * D + c) = v;
}

__global__ __launch_bounds__(256) void rows_scatter_kernel(float* __restrict__ table, const int* __restrict__ ids,
                                                           const float* __restrict__ rows, long n, int D, int V,
                                                           int gs) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long k = t >> gs;
  if (k >= n) return;
  const int id = ids[k];
  if (id < 0 || id >= V) return;
  const int c = (int)(t & ((1 << gs) - 1)) * 4;
  *reinterpret_cast<f32x4*>(table + (size_t)id * D + c) = *reinterpret_cast<const f32x4*>(rows + k * D + c);
}

// Fixed-capacity owner buckets of the bucketed exchange (parallel/sparse_exchange.py).
// ids [n]: keys of a shared key space (-1 / outside [off, off + V) = none), distinct.  The
// ids whose table-local id (id - off) is owned by rank o (local % ws == o) go, in input
// order, to slots o * cap + k (send_ids: the local id, src: its input position); slots past
// the count get -1.  Two passes over SEG-id segments, grid (segments, owners): count, then
// place at the segment's offset (the sum of the earlier segments' counts, read by every
// placing block: the segment count is small).  Inside a segment, 1024 threads scan it in
// chunks: wave ballots + a 16-entry LDS prefix.  need / over: running maxima (global
// atomics) of the demand and of the demand beyond capacity.
constexpr int OB_SEG = 4096;

FTM_DEVICE bool owned_by(int id, int off, int V, int ws, int o, int& loc) {
  loc = id - off;
  return id >= 0 && loc >= 0 && loc < V && (loc % ws) == o;
}

__global__ __launch_bounds__(1024) void owner_count_kernel(const int* __restrict__ ids, int n, int off, int V, int ws,
                                                           int* __restrict__ counts) {
  __shared__ int cnt[16];
  const int s = blockIdx.x, o = blockIdx.y, nseg = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int total = 0;
  for (int b0 = s * OB_SEG; b0 < n && b0 < (s + 1) * OB_SEG; b0 += 1024) {
    const int i = b0 + t;
    int loc;
    const bool f = i < n && owned_by(ids[i], off, V, ws, o, loc);
    const unsigned long long m = __ballot(f);
    if (lane == 0) cnt[w] = __popcll(m);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) total += cnt[k];
    __syncthreads();
  }
  if (t == 0) counts[o * nseg + s] = total;
}

__global__ __launch_bounds__(1024) void owner_place_kernel(const int* __restrict__ ids, int n, int off, int V, int ws,
                                                           int cap, const int* __restrict__ counts,
                                                           int* __restrict__ send_ids, int* __restrict__ src,
                                                           int* __restrict__ need, int* __restrict__ over) {
  __shared__ int cnt[16];
  __shared__ int base_s;
  const int s = blockIdx.x, o = blockIdx.y, nseg = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) {
    int b = 0;
    for (int k = 0; k < s; ++k) b += counts[o * nseg + k];
    base_s = b;
  }
  __syncthreads();
  int run = base_s;
  for (int b0 = s * OB_SEG; b0 < n && b0 < (s + 1) * OB_SEG; b0 += 1024) {
    const int i = b0 + t;
    int loc = -1;
    const bool f = i < n && owned_by(ids[i], off, V, ws, o, loc);
    const unsigned long long m = __ballot(f);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) cnt[w] = __popcll(m);
    __syncthreads();
    int wbase = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = cnt[k];
      wbase += k < w ? c : 0;
      tot += c;
    }
    const int pos = run + wbase + before;
    if (f && pos < cap) {
      send_ids[(size_t)o * cap + pos] = loc;
      src[(size_t)o * cap + pos] = i;
    }
    run += tot;
    __syncthreads();
  }
  if (s == nseg - 1) {  // the last segment knows the owner's total: pad the bucket, record demand
    for (int p = (run < cap ? run : cap) + t; p < cap; p += 1024) {
      send_ids[(size_t)o * cap + p] = -1;
      src[(size_t)o * cap + p] = -1;
    }
    if (t == 0) {
      atomicMax(need, run);
      if (run > cap) atomicMax(over, run - cap);
    }
  }
}

}  // namespace

// log2 of a power of two in [1, 64], or -1
int pow2_shift(int g) {
  for (int k = 0; k <= 6; ++k)
    if (g == (1 << k)) return k;
  return -1;
}

void embedding_bag_fwd(uintptr_t ids, uintptr_t table, uintptr_t out, int rows, int L, int D, int V, uintptr_t stream) {
  if (D % 8) throw std::invalid_argument("embedding_bag_fwd: D % 8 != 0");
  const int gs = pow2_shift(D / 8);
  if (gs < 0) throw std::invalid_argument("embedding_bag_fwd: D / 8 must be a power of two <= 64");
  if (table % 16 || out % 16) throw std::invalid_argument("embedding_bag_fwd: 16-byte alignment required");
  if (rows <= 0) return;
  const long threads = (long)rows << gs;
  hipLaunchKernelGGL(embedding_bag_fwd_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const int*>(ids),
                     reinterpret_cast<const float*>(table), reinterpret_cast<bf16*>(out), rows, L, D, gs, V);
  FTM_CHECK_LAUNCH();
}

template <typename T>
void launch_segment_sum(const void* grad, const int* P, const int* S, float* O, int U, int D, int L, hipStream_t s) {
  const T* g = reinterpret_cast<const T*>(grad);
  const dim3 grid((U + 3) / 4), block(256);
  if (D / 8 <= 8) {  // small rows: lane groups, 64 / G destinations per wave
    const int G = D / 8, per_wave = 64 / G;
    const dim3 ggrid((unsigned)(((U + per_wave - 1) / per_wave + 3) / 4));
    switch (G) {
      case 1: hipLaunchKernelGGL((segment_sum_rows_grp_kernel<T, 1>), ggrid, block, 0, s, g, P, S, O, U, D, L); return;
      case 2: hipLaunchKernelGGL((segment_sum_rows_grp_kernel<T, 2>), ggrid, block, 0, s, g, P, S, O, U, D, L); return;
      case 4: hipLaunchKernelGGL((segment_sum_rows_grp_kernel<T, 4>), ggrid, block, 0, s, g, P, S, O, U, D, L); return;
      case 8: hipLaunchKernelGGL((segment_sum_rows_grp_kernel<T, 8>), ggrid, block, 0, s, g, P, S, O, U, D, L); return;
      default: break;
    }
  }
  switch (D / 8) {  // column chunks per row: pick the widest power of two that divides the work
    case 1: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 1>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 2: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 2>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 4: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 4>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 8: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 8>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 16: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 16>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    case 32: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 32>), grid, block, 0, s, g, P, S, O, U, D, L); break;
    default: hipLaunchKernelGGL((segment_sum_rows_kernel<T, 64>), grid, block, 0, s, g, P, S, O, U, D, L); break;
  }
}

void segment_sum_rows(uintptr_t grad, uintptr_t perm, uintptr_t seg, uintptr_t out, int U, int D, int L,
                      int grad_is_fp32, uintptr_t stream) {
  if (D % 8) throw std::invalid_argument("segment_sum_rows: D % 8 != 0");
  if (grad % 16 || out % 16) throw std::invalid_argument("segment_sum_rows: 16-byte alignment required");
  if (U <= 0) return;
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto P = reinterpret_cast<const int*>(perm);
  auto S = reinterpret_cast<const int*>(seg);
  auto O = reinterpret_cast<float*>(out);
  if (grad_is_fp32) launch_segment_sum<float>(reinterpret_cast<const void*>(grad), P, S, O, U, D, L, s);
  else launch_segment_sum<bf16>(reinterpret_cast<const void*>(grad), P, S, O, U, D, L, s);
  FTM_CHECK_LAUNCH();
}

void sparse_adagrad(uintptr_t table, uintptr_t accum, uintptr_t uids, uintptr_t g, int U, int D, int V, float lr,
                    float eps, int off, uintptr_t stream) {
  if (D % 4) throw std::invalid_argument("sparse_adagrad: D % 4 != 0");
  const int gs = pow2_shift(D / 4);
  if (gs < 0) throw std::invalid_argument("sparse_adagrad: D / 4 must be a power of two <= 64");
  if (table % 16 || accum % 16 || g % 16) throw std::invalid_argument("sparse_adagrad: 16-byte alignment required");
  if (U <= 0) return;
  const long threads = (long)U << gs;
  hipLaunchKernelGGL(sparse_adagrad_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<float*>(table),
                     reinterpret_cast<float*>(accum), reinterpret_cast<const int*>(uids),
                     reinterpret_cast<const float*>(g), U, D, V, lr, eps, gs, off);
  FTM_CHECK_LAUNCH();
}

// sorted: int32 keys (a 32-bit radix sort is half the passes of a 64-bit one)
template <typename T, int G>
void launch_segsum(const void* grad, const int* P, const int* SID, const int* SEG, float* O, float* ws, int n, int U,
                   int D, int L, int S, int lo, int hi, hipStream_t s) {
  const long slices = (n + S - 1) / S;
  float* head = ws;
  float* tail = ws + slices * D;
  const long threads = slices * G;
  hipLaunchKernelGGL((segsum_slices_kernel<T, G>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const T*>(grad), P, SID, SEG, O, head, tail, n, D, L, S, lo, hi);
  hipLaunchKernelGGL((segsum_fixup_kernel<G>), dim3((unsigned)((U + 3) / 4)), dim3(256), 0, s, SEG, O, head, tail, U,
                     D, S);
}

// Static-shape deterministic segment sum of sorted rows: seg_id[i] = destination of sorted
// position i, seg [U + 1] run starts; ws >= 2 * ceil(n / S) * D floats.  Only sorted
// positions whose perm lies in [lo, hi) contribute (rows (perm - lo) / L of grad): several
// tables can share one key space and one sort.
void segment_sum_sorted(uintptr_t grad, uintptr_t perm, uintptr_t seg_id, uintptr_t seg, uintptr_t out, uintptr_t ws,
                        int n, int U, int D, int L, int S, int grad_is_fp32, int lo, int hi, uintptr_t stream) {
  if (D % 8 || D / 8 > 64 || ((D / 8) & (D / 8 - 1))) throw std::invalid_argument("segment_sum_sorted: D/8 power of 2 <= 64");
  if (S <= 0 || S % 8) throw std::invalid_argument("segment_sum_sorted: slice length must be a positive multiple of 8");
  if (grad % 16 || out % 16 || ws % 16) throw std::invalid_argument("segment_sum_sorted: 16-byte alignment required");
  if (n <= 0 || U <= 0) return;
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto P = reinterpret_cast<const int*>(perm);
  auto SID = reinterpret_cast<const int*>(seg_id);
  auto SEG = reinterpret_cast<const int*>(seg);
  auto O = reinterpret_cast<float*>(out);
  auto W = reinterpret_cast<float*>(ws);
  const void* g = reinterpret_cast<const void*>(grad);
#define FTM_SEGSUM(T)                                                                      \
  switch (D / 8) {                                                                         \
    case 1: launch_segsum<T, 1>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;            \
    case 2: launch_segsum<T, 2>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;            \
    case 4: launch_segsum<T, 4>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;            \
    case 8: launch_segsum<T, 8>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;            \
    case 16: launch_segsum<T, 16>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;          \
    case 32: launch_segsum<T, 32>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;          \
    default: launch_segsum<T, 64>(g, P, SID, SEG, O, W, n, U, D, L, S, lo, hi, s); break;          \
  }
  if (grad_is_fp32) { FTM_SEGSUM(float) } else { FTM_SEGSUM(bf16) }
#undef FTM_SEGSUM
  FTM_CHECK_LAUNCH();
}

void segment_starts(uintptr_t sorted, uintptr_t seg_id, uintptr_t seg, uintptr_t uids, int n, long long num_rows,
                    uintptr_t stream) {
  if (n <= 0) return;
  if (num_rows >= (1LL << 31) - 1) throw std::invalid_argument("segment_starts: num_rows must fit int32");
  hipLaunchKernelGGL(segment_starts_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const int*>(sorted), reinterpret_cast<const int*>(seg_id),
                     reinterpret_cast<int*>(seg), reinterpret_cast<int*>(uids), n, (int)num_rows);
  FTM_CHECK_LAUNCH();
}

static void rows_move(bool gather, uintptr_t table, uintptr_t ids, uintptr_t rows, long long n, int D, int V,
                      uintptr_t stream) {
  if (D % 4) throw std::invalid_argument("rows_gather/scatter: D % 4 != 0");
  const int gs = pow2_shift(D / 4);
  if (gs < 0) throw std::invalid_argument("rows_gather/scatter: D / 4 must be a power of two <= 64");
  if (table % 16 || rows % 16) throw std::invalid_argument("rows_gather/scatter: 16-byte alignment required");
  if (n <= 0) return;
  const long long threads = n << gs;
  auto s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (gather)
    hipLaunchKernelGGL(rows_gather_kernel, grid, dim3(256), 0, s, reinterpret_cast<const float*>(table),
                       reinterpret_cast<const int*>(ids), reinterpret_cast<float*>(rows), (long)n, D, V, gs);
  else
    hipLaunchKernelGGL(rows_scatter_kernel, grid, dim3(256), 0, s, reinterpret_cast<float*>(table),
                       reinterpret_cast<const int*>(ids), reinterpret_cast<const float*>(rows), (long)n, D, V, gs);
  FTM_CHECK_LAUNCH();
}

void rows_gather(uintptr_t table, uintptr_t ids, uintptr_t out, long long n, int D, int V, uintptr_t stream) {
  rows_move(true, table, ids, out, n, D, V, stream);
}

void rows_scatter(uintptr_t table, uintptr_t ids, uintptr_t rows, long long n, int D, int V, uintptr_t stream) {
  rows_move(false, table, ids, rows, n, D, V, stream);
}

// counts: int32 workspace of ws * owner_buckets_segments(n) entries
int owner_buckets_segments(int n) { return n > 0 ? (n + OB_SEG - 1) / OB_SEG : 1; }

void owner_buckets(uintptr_t ids, int n, int off, int V, int ws, int cap, uintptr_t send_ids, uintptr_t src,
                   uintptr_t need, uintptr_t over, uintptr_t counts, uintptr_t stream) {
  if (ws < 1 || ws > 1024 || cap < 1) throw std::invalid_argument("owner_buckets: 1 <= ws <= 1024, cap >= 1");
  auto s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(owner_buckets_segments(n), ws), block(1024);
  hipLaunchKernelGGL(owner_count_kernel, grid, block, 0, s, reinterpret_cast<const int*>(ids), n, off, V, ws,
                     reinterpret_cast<int*>(counts));
  hipLaunchKernelGGL(owner_place_kernel, grid, block, 0, s, reinterpret_cast<const int*>(ids), n, off, V, ws, cap,
                     reinterpret_cast<const int*>(counts), reinterpret_cast<int*>(send_ids), reinterpret_cast<int*>(src),
                     reinterpret_cast<int*>(need), reinterpret_cast<int*>(over));
  FTM_CHECK_LAUNCH();
}

void register_embedding(pybind11::module_& m) {
  m.def("owner_buckets", &owner_buckets);
  m.def("owner_buckets_segments", &owner_buckets_segments);
  m.def("rows_gather", &rows_gather);
  m.def("rows_scatter", &rows_scatter);
  m.def("segment_starts", &segment_starts);
  m.def("embedding_bag_fwd", &embedding_bag_fwd);
  m.def("segment_sum_rows", &segment_sum_rows);
  m.def("segment_sum_sorted", &segment_sum_sorted);
  m.def("sparse_adagrad", &sparse_adagrad);
}
