// Static-shape key grouping for the row-sparse gradient pipeline (ops/embedding.py):
// keys -> (stable order, run boundaries, unique keys), no host sync, no library kernels.
//
// In-tree LSD radix sort over the key bits in use (ceil(log2(num_rows + 1)), 8-bit digits:
// 3 passes for the 3.6M-row Wide&Deep key space), 2048-key tiles of 256 threads:
//
//   count     per pass, per-tile digit counts [digit][tile] (LDS atomics; the first pass
//             clamps keys: ids outside [0, num_rows) form one bucket, num_rows, and sets
//             seg[] = n, uids[] = -1)
//   scatter   per pass: every tile derives its digit offsets itself from the pass's counts
//             (its predecessors' counts + the global digit totals: 256 threads x ntiles L2
//             reads, no scan launch), ranks its keys stably (per wave, 64-key rounds in tile
//             order: lanes with the same digit found by 9 ballots, the leader advances the
//             wave's LDS digit counter) and scatters (key, index)
//   runs      count of run starts per tile, then run index (tile prefix + block scan), run
//             starts and run keys (-1 for the invalid bucket)
//
// Stable: equal keys keep their input order (same result as a stable comparison sort), so
// every reduce-by-key downstream sums in a fixed order.  8 launches for 3 passes.  (Counting
// the next pass's digits inside the scatter with global atomics was tried: a hot id makes
// thousands of atomics on one counter, 150-330 us per pass.)
#include <pybind11/pybind11.h>

#include <stdexcept>

#include "common.h"

namespace {

constexpr int RT = 256;             // threads per tile
constexpr int KPT = 8;              // keys per thread
constexpr int TILE = RT * KPT;      // 2048 keys: wave w, round r, lane l -> key w*512 + r*64 + l
constexpr int RADIX = 256;
constexpr int MAXP = 4;             // num_rows < 2^30 -> at most 4 passes of 8 bits

int key_bits(int num_rows) {
  int b = 1;
  while (b < 31 && (1LL << b) <= (long long)num_rows) ++b;  // keys are 0..num_rows inclusive
  return b;
}

FTM_DEVICE int clamp_key(int k, int num_rows) { return (k >= 0 && k < num_rows) ? k : num_rows; }

// first: keys are the raw input (clamped here); also initialises the run outputs
__global__ __launch_bounds__(RT) void rs_count_kernel(const int* __restrict__ keys, int n, int num_rows, int shift,
                                                      bool first, int* __restrict__ hist, int* __restrict__ seg,
                                                      int* __restrict__ uids, int ntiles) {
  __shared__ int cnt[RADIX];
  const int t = blockIdx.x;
  cnt[threadIdx.x] = 0;
  if (first) {  // grid-stride init of the run outputs
    for (int i = t * RT + threadIdx.x; i <= n; i += ntiles * RT) {
      seg[i] = n;
      if (i < n) uids[i] = -1;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int i = t * TILE + j * RT + threadIdx.x;
    if (i < n) {
      const int k = first ? clamp_key(keys[i], num_rows) : keys[i];
      atomicAdd(&cnt[(k >> shift) & (RADIX - 1)], 1);
    }
  }
  __syncthreads();
  hist[threadIdx.x * ntiles + t] = cnt[threadIdx.x];
}

// One radix pass.  vin == nullptr: values are the input indices (first pass; keys clamped).
__global__ __launch_bounds__(RT) void rs_scatter_kernel(const int* __restrict__ kin, const int* __restrict__ vin,
                                                        int* __restrict__ kout, int* __restrict__ vout, int n,
                                                        int num_rows, int shift, const int* __restrict__ hist,
                                                        int ntiles) {
  __shared__ int goff[RADIX];
  __shared__ int tot[RADIX];
  __shared__ int wcnt[4][RADIX + 1];  // per-wave digit counters (+1: the out-of-range slot)
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  {  // this tile's offset for every digit: digits below it everywhere + this digit in earlier tiles
    const int d = threadIdx.x;
    int total = 0, pre = 0;
    for (int u = 0; u < ntiles; ++u) {
      const int c = hist[d * ntiles + u];
      total += c;
      pre += u < t ? c : 0;
    }
    tot[d] = total;
    goff[d] = pre;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) wcnt[ww][d] = 0;
    if (d < 4) wcnt[d][RADIX] = 0;
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the 256 digit totals by wave 0 (4 per lane)
    int v[4], s = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = s;
      s += tot[lane * 4 + e];
    }
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const int base = incl - s;
#pragma unroll
    for (int e = 0; e < 4; ++e) goff[lane * 4 + e] += base + v[e];
  }
  // stable ranks: wave w owns tile keys [w*512, w*512 + 512) in 8 rounds of 64
  int key[KPT], val[KPT], dig[KPT], rank[KPT];
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    const int i = t * TILE + w * 512 + r * 64 + lane;
    const bool ok = i < n;
    int k = ok ? kin[i] : 0;
    if (!vin) k = clamp_key(k, num_rows);
    key[r] = k;
    val[r] = ok ? (vin ? vin[i] : i) : 0;
    const int d = ok ? ((k >> shift) & (RADIX - 1)) : RADIX;  // 9-bit digit: RADIX = not a key
    dig[r] = d;
    unsigned long long m = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const unsigned long long bal = __ballot((d >> b) & 1);
      m &= ((d >> b) & 1) ? bal : ~bal;
    }
    const int leader = __ffsll((long long)m) - 1;
    int old = 0;
    if (lane == leader) {
      old = wcnt[w][d];
      wcnt[w][d] = old + __popcll(m);
    }
    old = __shfl(old, leader, 64);
    rank[r] = old + __popcll(m & lt);
  }
  __syncthreads();
  {  // exclusive prefix over waves per digit
    const int d = threadIdx.x;
    int s = 0;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const int c = wcnt[ww][d];
      wcnt[ww][d] = s;
      s += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    const int d = dig[r];
    if (d == RADIX) continue;
    const int pos = goff[d] + wcnt[w][d] + rank[r];
    kout[pos] = key[r];
    vout[pos] = val[r];
  }
}

// number of run starts (sorted[i] != sorted[i - 1]) per tile
__global__ __launch_bounds__(RT) void rs_runs_count_kernel(const int* __restrict__ s, int n, int* __restrict__ tcount) {
  __shared__ int red[RT / 64];
  const int t = blockIdx.x;
  int c = 0;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int i = t * TILE + threadIdx.x * KPT + j;
    if (i < n) c += (i == 0 || s[i] != s[i - 1]) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tcount[t] = red[0] + red[1] + red[2] + red[3];
}

// run index of every sorted position (earlier tiles' runs + block scan), run starts, run keys
__global__ __launch_bounds__(RT) void rs_runs_write_kernel(const int* __restrict__ s, int n, int num_rows,
                                                           const int* __restrict__ tcount, int* __restrict__ seg_id,
                                                           int* __restrict__ seg, int* __restrict__ uids) {
  __shared__ int wsum[RT / 64];
  __shared__ int base_s;
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    int b = 0;
    for (int u = 0; u < t; ++u) b += tcount[u];
    base_s = b;
  }
  int f[KPT], c = 0;
  const int i0 = t * TILE + threadIdx.x * KPT;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int i = i0 + j;
    f[j] = (i < n && (i == 0 || s[i] != s[i - 1])) ? 1 : 0;
    c += f[j];
  }
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int before = base_s;
  for (int ww = 0; ww < w; ++ww) before += wsum[ww];
  int run = before + incl - c;  // runs started before this thread's first position
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int i = i0 + j;
    if (i >= n) break;
    run += f[j];
    const int r = run - 1;
    seg_id[i] = r;
    if (f[j]) {
      const int k = s[i];
      seg[r] = i;
      uids[r] = k >= num_rows ? -1 : k;
    }
  }
}

int passes_for(int num_rows) { return (key_bits(num_rows) + 7) / 8; }

}  // namespace

// bytes of scratch (digit counters of every pass + per-tile run counts) for n keys
size_t sort_segments_temp_bytes(int n, int num_rows) {
  const size_t ntiles = (size_t)(n + TILE - 1) / TILE;
  return (size_t)passes_for(num_rows) * RADIX * ntiles * 4 + ntiles * 4 + 256;
}

// keys int32 [n] -> sorted int32 [n], perm int32 [n] (stable), seg_id int32 [n],
// seg int32 [n + 1] (run starts, n past the last run), uids int32 [n] (-1 past the runs / for
// the invalid bucket).  work: int32 [3 n] scratch; temp: sort_segments_temp_bytes bytes.
void sort_segments(uintptr_t keys, int n, int num_rows, uintptr_t sorted, uintptr_t perm, uintptr_t seg_id,
                   uintptr_t seg, uintptr_t uids, uintptr_t work, uintptr_t temp, size_t temp_bytes,
                   uintptr_t stream) {
  if (n <= 0) return;
  if (num_rows < 0 || num_rows >= (1 << 30)) throw std::invalid_argument("sort_segments: num_rows out of range");
  if (temp_bytes < sort_segments_temp_bytes(n, num_rows)) throw std::invalid_argument("sort_segments: temp too small");
  if (temp % 4) throw std::invalid_argument("sort_segments: temp alignment");
  auto s = reinterpret_cast<hipStream_t>(stream);
  const int ntiles = (n + TILE - 1) / TILE;
  const int P = passes_for(num_rows);
  int* hist = reinterpret_cast<int*>(temp);  // [P][RADIX][ntiles]
  int* tcount = hist + (size_t)P * RADIX * ntiles;
  const size_t hs = (size_t)RADIX * ntiles;
  int* wk = reinterpret_cast<int*>(work);
  int *ks = reinterpret_cast<int*>(sorted), *vs = reinterpret_cast<int*>(perm);
  // the last pass must land in (sorted, perm): alternate from there backwards
  int* kb[2] = {ks, wk};
  int* vb[2] = {vs, wk + n};
  const int* kin = reinterpret_cast<const int*>(keys);
  const int* vin = nullptr;
  for (int p = 0; p < P; ++p) {
    const int o = (P - 1 - p) & 1;  // pass P-1 writes buffer set 0 = (sorted, perm)
    int* hp = hist + (size_t)p * hs;
    hipLaunchKernelGGL(rs_count_kernel, dim3(ntiles), dim3(RT), 0, s, kin, n, num_rows, 8 * p, p == 0, hp,
                       reinterpret_cast<int*>(seg), reinterpret_cast<int*>(uids), ntiles);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3(ntiles), dim3(RT), 0, s, kin, vin, kb[o], vb[o], n, num_rows, 8 * p,
                       hp, ntiles);
    kin = kb[o];
    vin = vb[o];
  }
  hipLaunchKernelGGL(rs_runs_count_kernel, dim3(ntiles), dim3(RT), 0, s, ks, n, tcount);
  hipLaunchKernelGGL(rs_runs_write_kernel, dim3(ntiles), dim3(RT), 0, s, ks, n, num_rows, tcount,
                     reinterpret_cast<int*>(seg_id), reinterpret_cast<int*>(seg), reinterpret_cast<int*>(uids));
  FTM_CHECK_LAUNCH();
}

void register_sort_segments(pybind11::module_& m) {
  m.def("sort_segments_temp_bytes", &sort_segments_temp_bytes);
  m.def("sort_segments", &sort_segments);
}
