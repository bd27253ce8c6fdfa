// Baseline JPEG decoding straight into a micro-batch's staging slot.
//
// The reference decodes every image file in its source with TF's DecodeJpeg, one record
// per Session.run (ImageNormalization.scala:42-77, ImageInputFormat.scala:63-80).  Here the
// compressed bytes travel as the record (≈20 KB instead of 196 KB decoded), and the
// micro-batch's host stage decodes them with a GIL-free thread pool directly into the
// pinned rows the H2D copy reads (batching/engine.py PipelinedGpuRunner): no Python
// object per pixel row, no decoded image crossing a process boundary.
//
// Scope: ITU-T T.81 baseline and extended sequential Huffman JPEG, 8-bit samples, 1 or 3
// components (grayscale is replicated to RGB), any sampling factors up to 2x2 (4:4:4,
// 4:2:2, 4:2:0, 4:4:0), restart intervals; YCbCr -> RGB per JFIF.  Chroma is upsampled
// with the triangle filter ("fancy" upsampling).  Progressive / arithmetic / 12-bit
// files and images of another size than the slot's are reported back (status per image)
// and the caller decodes those with Pillow.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <immintrin.h>
#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "native.h"

namespace {

constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

enum Status : int { kOk = 0, kNotJpeg = 1, kUnsupported = 2, kCorrupt = 3, kSize = 4 };

struct Huff {
  // canonical table: lookup of the first 9 bits, then the classic maxcode walk
  uint16_t fast[512];  // (length << 8) | symbol, 0 = longer code
  // AC tables: when a 9-bit prefix holds a whole (code, magnitude bits) pair of a nonzero
  // coefficient, its run, value and total length in one lookup (0 length = not there)
  int16_t fast_val[512];
  uint8_t fast_run[512], fast_len[512];
  int32_t maxcode[18];
  int32_t valoff[17];
  uint8_t vals[256];
  bool ok = false;

  void build_fast_ac() {
    for (int p = 0; p < 512; ++p) {
      fast_len[p] = 0;
      const uint16_t f = fast[p];
      if (!f) continue;
      const int len = f >> 8, rs = f & 0xFF, r = rs >> 4, sz = rs & 15;
      if (sz == 0 || len + sz > 9) continue;
      const int v = (p >> (9 - len - sz)) & ((1 << sz) - 1);
      fast_val[p] = int16_t(v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v);
      fast_run[p] = uint8_t(r);
      fast_len[p] = uint8_t(len + sz);
    }
  }

  bool build(const uint8_t* counts, const uint8_t* symbols, int nsym) {
    std::memset(fast, 0, sizeof(fast));
    std::memcpy(vals, symbols, nsym);
    int code = 0, k = 0;
    for (int len = 1; len <= 16; ++len) {
      valoff[len] = k - code;
      for (int i = 0; i < counts[len - 1]; ++i, ++k, ++code) {
        if (len <= 9) {
          const int shift = 9 - len;
          for (int j = 0; j < (1 << shift); ++j) fast[(code << shift) | j] = uint16_t((len << 8) | symbols[k]);
        }
      }
      maxcode[len] = counts[len - 1] ? code - 1 : -1;
      if (code > (1 << len)) return false;
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
    ok = true;
    return true;
  }
};

struct Component {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int bw = 0, bh = 0;  // blocks per row / column in the padded plane
  int pred = 0;
  std::vector<uint8_t> plane;  // bw*8 x bh*8 samples
};

// 8x8 inverse DCT: the Loeffler-Ligtenberg-Moschytz factorisation of the 1-D 8-point
// transform (12 multiplies, 32 adds) applied to the rows, then the columns, in float; a
// block whose AC coefficients are all zero (most blocks of smooth content) is a constant.
// Output = IDCT / 8 + 128, rounded and clamped to [0, 255].
struct Idct {
  static inline void pass(const float* in, float* out, int is, int os) {
    // even part
    const float z2e = in[2 * is], z3e = in[6 * is];
    const float z1 = (z2e + z3e) * 0.541196100f;
    const float t2 = z1 - z3e * 1.847759065f;
    const float t3 = z1 + z2e * 0.765366865f;
    const float t0 = in[0] + in[4 * is], t1 = in[0] - in[4 * is];
    const float t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    // odd part
    float o0 = in[7 * is], o1 = in[5 * is], o2 = in[3 * is], o3 = in[is];
    const float q1 = o0 + o3, q2 = o1 + o2, q3 = o0 + o2, q4 = o1 + o3;
    const float q5 = (q3 + q4) * 1.175875602f;
    o0 *= 0.298631336f;
    o1 *= 2.053119869f;
    o2 *= 3.072711026f;
    o3 *= 1.501321110f;
    const float r1 = q1 * -0.899976223f, r2 = q2 * -2.562915447f;
    const float r3 = q3 * -1.961570560f + q5, r4 = q4 * -0.390180644f + q5;
    o0 += r1 + r3;
    o1 += r2 + r4;
    o2 += r2 + r3;
    o3 += r1 + r4;
    out[0] = t10 + o3;
    out[7 * os] = t10 - o3;
    out[os] = t11 + o2;
    out[6 * os] = t11 - o2;
    out[2 * os] = t12 + o1;
    out[5 * os] = t12 - o1;
    out[3 * os] = t13 + o0;
    out[4 * os] = t13 - o0;
  }
  static inline uint8_t clamp8(float v) {
    const int i = int(v + 128.5f);  // v + 128, rounded (v > -128.5 for the cast to floor)
    return uint8_t(i < 0 ? 0 : i > 255 ? 255 : i);
  }
#if defined(__AVX2__) && defined(__FMA__)
  static void run_avx2(const int32_t* F, uint8_t* out, int stride);
#endif
  // ac: whether the entropy decoder stored any AC coefficient (a zero one may still have
  // been coded: the DC-only shortcut then just does not fire)
  void run(const int32_t* F, uint8_t* out, int stride, bool ac) const {
    if (!ac) {  // DC only: IDCT = F[0] / 8 everywhere
      const uint8_t v = clamp8(float(F[0]) * 0.125f);
      for (int x = 0; x < 8; ++x) std::memset(out + x * stride, v, 8);
      return;
    }
#if defined(__AVX2__) && defined(__FMA__)
    run_avx2(F, out, stride);
    return;
#endif
    float f[64], g[64];
    for (int k = 0; k < 64; ++k) f[k] = float(F[k]);
    for (int u = 0; u < 8; ++u) {  // rows: f[u][v] over v -> g[u][y]
      const float* r = f + 8 * u;
      bool any = false;
      for (int v = 1; v < 8; ++v) any |= r[v] != 0.f;
      if (!any) {
        for (int y = 0; y < 8; ++y) g[8 * u + y] = r[0];
      } else {
        pass(r, g + 8 * u, 1, 1);
      }
    }
    float o[64];
    for (int y = 0; y < 8; ++y) pass(g + y, o + y, 8, 8);  // columns
    for (int x = 0; x < 8; ++x) {
      uint8_t* d = out + x * stride;
      for (int y = 0; y < 8; ++y) d[y] = clamp8(o[8 * x + y] * 0.125f);
    }
  }
};

#if defined(__AVX2__) && defined(__FMA__)
// The same factorisation on 8 lanes: a vector holds one coefficient index of 8 rows (or
// columns), the 1-D transform runs on 8 of them at once, and two 8x8 transposes put the
// row pass's outputs into the column pass's layout and its outputs back into rows.
static inline void transpose8(__m256* r) {
  const __m256 t0 = _mm256_unpacklo_ps(r[0], r[1]), t1 = _mm256_unpackhi_ps(r[0], r[1]);
  const __m256 t2 = _mm256_unpacklo_ps(r[2], r[3]), t3 = _mm256_unpackhi_ps(r[2], r[3]);
  const __m256 t4 = _mm256_unpacklo_ps(r[4], r[5]), t5 = _mm256_unpackhi_ps(r[4], r[5]);
  const __m256 t6 = _mm256_unpacklo_ps(r[6], r[7]), t7 = _mm256_unpackhi_ps(r[6], r[7]);
  const __m256 u0 = _mm256_shuffle_ps(t0, t2, 0x44), u1 = _mm256_shuffle_ps(t0, t2, 0xEE);
  const __m256 u2 = _mm256_shuffle_ps(t1, t3, 0x44), u3 = _mm256_shuffle_ps(t1, t3, 0xEE);
  const __m256 u4 = _mm256_shuffle_ps(t4, t6, 0x44), u5 = _mm256_shuffle_ps(t4, t6, 0xEE);
  const __m256 u6 = _mm256_shuffle_ps(t5, t7, 0x44), u7 = _mm256_shuffle_ps(t5, t7, 0xEE);
  r[0] = _mm256_permute2f128_ps(u0, u4, 0x20);
  r[1] = _mm256_permute2f128_ps(u1, u5, 0x20);
  r[2] = _mm256_permute2f128_ps(u2, u6, 0x20);
  r[3] = _mm256_permute2f128_ps(u3, u7, 0x20);
  r[4] = _mm256_permute2f128_ps(u0, u4, 0x31);
  r[5] = _mm256_permute2f128_ps(u1, u5, 0x31);
  r[6] = _mm256_permute2f128_ps(u2, u6, 0x31);
  r[7] = _mm256_permute2f128_ps(u3, u7, 0x31);
}

static inline void pass8(__m256* v) {
  const auto k = [](float c) { return _mm256_set1_ps(c); };
  const __m256 z1 = _mm256_mul_ps(_mm256_add_ps(v[2], v[6]), k(0.541196100f));
  const __m256 t2 = _mm256_fnmadd_ps(v[6], k(1.847759065f), z1);
  const __m256 t3 = _mm256_fmadd_ps(v[2], k(0.765366865f), z1);
  const __m256 t0 = _mm256_add_ps(v[0], v[4]), t1 = _mm256_sub_ps(v[0], v[4]);
  const __m256 t10 = _mm256_add_ps(t0, t3), t13 = _mm256_sub_ps(t0, t3);
  const __m256 t11 = _mm256_add_ps(t1, t2), t12 = _mm256_sub_ps(t1, t2);
  __m256 o0 = v[7], o1 = v[5], o2 = v[3], o3 = v[1];
  const __m256 q1 = _mm256_add_ps(o0, o3), q2 = _mm256_add_ps(o1, o2);
  const __m256 q3 = _mm256_add_ps(o0, o2), q4 = _mm256_add_ps(o1, o3);
  const __m256 q5 = _mm256_mul_ps(_mm256_add_ps(q3, q4), k(1.175875602f));
  const __m256 r1 = _mm256_mul_ps(q1, k(-0.899976223f)), r2 = _mm256_mul_ps(q2, k(-2.562915447f));
  const __m256 r3 = _mm256_fmadd_ps(q3, k(-1.961570560f), q5), r4 = _mm256_fmadd_ps(q4, k(-0.390180644f), q5);
  o0 = _mm256_fmadd_ps(o0, k(0.298631336f), _mm256_add_ps(r1, r3));
  o1 = _mm256_fmadd_ps(o1, k(2.053119869f), _mm256_add_ps(r2, r4));
  o2 = _mm256_fmadd_ps(o2, k(3.072711026f), _mm256_add_ps(r2, r3));
  o3 = _mm256_fmadd_ps(o3, k(1.501321110f), _mm256_add_ps(r1, r4));
  v[0] = _mm256_add_ps(t10, o3);
  v[7] = _mm256_sub_ps(t10, o3);
  v[1] = _mm256_add_ps(t11, o2);
  v[6] = _mm256_sub_ps(t11, o2);
  v[2] = _mm256_add_ps(t12, o1);
  v[5] = _mm256_sub_ps(t12, o1);
  v[3] = _mm256_add_ps(t13, o0);
  v[4] = _mm256_sub_ps(t13, o0);
}

void Idct::run_avx2(const int32_t* F, uint8_t* out, int stride) {
  __m256 v[8];
  for (int u = 0; u < 8; ++u) v[u] = _mm256_cvtepi32_ps(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(F + 8 * u)));
  transpose8(v);  // v[k]: coefficient k of every row u
  pass8(v);       // v[y]: row pass output y of every row u
  transpose8(v);  // v[u]: row u's outputs over y
  pass8(v);       // v[x]: output row x over y
  const __m256 sc = _mm256_set1_ps(0.125f), off = _mm256_set1_ps(128.5f);
  __m256i q[8];
  for (int x = 0; x < 8; ++x) {  // v / 8 + 128, rounded as the scalar path (truncation of v + 128.5)
    const __m256i i = _mm256_cvttps_epi32(_mm256_fmadd_ps(v[x], sc, off));
    q[x] = _mm256_min_epi32(_mm256_max_epi32(i, _mm256_setzero_si256()), _mm256_set1_epi32(255));
  }
  const __m256i perm = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
  for (int h = 0; h < 2; ++h) {  // rows 4h .. 4h + 3
    const __m256i p01 = _mm256_packus_epi32(q[4 * h], q[4 * h + 1]);
    const __m256i p23 = _mm256_packus_epi32(q[4 * h + 2], q[4 * h + 3]);
    const __m256i b = _mm256_permutevar8x32_epi32(_mm256_packus_epi16(p01, p23), perm);
    alignas(32) uint8_t rows[32];
    _mm256_store_si256(reinterpret_cast<__m256i*>(rows), b);
    for (int r = 0; r < 4; ++r) std::memcpy(out + (4 * h + r) * stride, rows + 8 * r, 8);
  }
}
#endif

const Idct& idct() {
  static const Idct k;
  return k;
}

class Decoder {
 public:
  Decoder(const uint8_t* data, size_t n) : p_(data), end_(data + n) {}

  // decodes into dst (H x W x 3, row stride W*3); returns a Status
  int decode(uint8_t* dst, int want_h, int want_w) {
    if (end_ - p_ < 4 || p_[0] != 0xFF || p_[1] != 0xD8) return kNotJpeg;
    p_ += 2;
    bool frame = false;
    while (p_ + 4 <= end_) {
      if (p_[0] != 0xFF) return kCorrupt;
      const uint8_t mk = p_[1];
      p_ += 2;
      if (mk == 0xD8 || (mk >= 0xD0 && mk <= 0xD7) || mk == 0x01 || mk == 0xFF) {
        if (mk == 0xFF) --p_;  // fill byte
        continue;
      }
      if (mk == 0xD9) break;
      if (p_ + 2 > end_) return kCorrupt;
      const int len = (p_[0] << 8) | p_[1];
      const uint8_t* seg = p_ + 2;
      const uint8_t* seg_end = p_ + len;
      if (len < 2 || seg_end > end_) return kCorrupt;
      int st = kOk;
      switch (mk) {
        case 0xDB: st = dqt(seg, seg_end); break;
        case 0xC4: st = dht(seg, seg_end); break;
        case 0xDD: if (len < 4) return kCorrupt; restart_ = (seg[0] << 8) | seg[1]; break;
        case 0xC0: case 0xC1:
          st = sof(seg, seg_end);
          if (st == kOk && (h_ != want_h || w_ != want_w)) return kSize;
          frame = true;
          break;
        case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
        case 0xCE: case 0xCF:
          return kUnsupported;  // progressive / lossless / arithmetic
        case 0xDA: {
          if (!frame) return kCorrupt;
          st = sos(seg, seg_end);
          if (st != kOk) return st;
          p_ = seg_end;
          st = scan();
          if (st != kOk) return st;
          return convert(dst);  // one interleaved scan carries every component (baseline)
        }
        default: break;  // APPn, COM, ...
      }
      if (st != kOk) return st;
      p_ = seg_end;
    }
    return kCorrupt;
  }

 private:
  int dqt(const uint8_t* s, const uint8_t* e) {
    while (s < e) {
      const int pq = s[0] >> 4, tq = s[0] & 15;
      ++s;
      if (tq > 3 || s + (pq ? 128 : 64) > e) return kCorrupt;
      for (int k = 0; k < 64; ++k) {
        qt_[tq][k] = pq ? ((s[2 * k] << 8) | s[2 * k + 1]) : s[k];
      }
      s += pq ? 128 : 64;
    }
    return kOk;
  }
  int dht(const uint8_t* s, const uint8_t* e) {
    while (s + 17 <= e) {
      const int tc = s[0] >> 4, th = s[0] & 15;
      if (tc > 1 || th > 3) return kCorrupt;
      int n = 0;
      for (int i = 1; i <= 16; ++i) n += s[i];
      if (n > 256 || s + 17 + n > e) return kCorrupt;
      Huff& h = tc ? ac_[th] : dc_[th];
      if (!h.build(s + 1, s + 17, n)) return kCorrupt;
      if (tc) h.build_fast_ac();
      s += 17 + n;
    }
    return kOk;
  }
  int sof(const uint8_t* s, const uint8_t* e) {
    if (e - s < 6) return kCorrupt;
    if (s[0] != 8) return kUnsupported;
    h_ = (s[1] << 8) | s[2];
    w_ = (s[3] << 8) | s[4];
    nc_ = s[5];
    if ((nc_ != 1 && nc_ != 3) || h_ <= 0 || w_ <= 0 || e - s < 6 + 3 * nc_) return kUnsupported;
    if (nc_ == 1) {  // a single-component scan is non-interleaved: one block per MCU whatever the factors
      c_[0].id = s[6];
      c_[0].h = c_[0].v = 1;
      c_[0].tq = s[8];
      if (c_[0].tq > 3) return kUnsupported;
      hmax_ = vmax_ = 1;
      mcux_ = (w_ + 7) / 8;
      mcuy_ = (h_ + 7) / 8;
      c_[0].bw = mcux_;
      c_[0].bh = mcuy_;
      c_[0].plane.assign(size_t(c_[0].bw) * 8 * c_[0].bh * 8, 0);
      return kOk;
    }
    hmax_ = vmax_ = 1;
    for (int i = 0; i < nc_; ++i) {
      Component& c = c_[i];
      c.id = s[6 + 3 * i];
      c.h = s[7 + 3 * i] >> 4;
      c.v = s[7 + 3 * i] & 15;
      c.tq = s[8 + 3 * i];
      if (c.h < 1 || c.h > 2 || c.v < 1 || c.v > 2 || c.tq > 3) return kUnsupported;
      hmax_ = c.h > hmax_ ? c.h : hmax_;
      vmax_ = c.v > vmax_ ? c.v : vmax_;
    }
    mcux_ = (w_ + 8 * hmax_ - 1) / (8 * hmax_);
    mcuy_ = (h_ + 8 * vmax_ - 1) / (8 * vmax_);
    for (int i = 0; i < nc_; ++i) {
      Component& c = c_[i];
      c.bw = mcux_ * c.h;
      c.bh = mcuy_ * c.v;
      c.plane.assign(size_t(c.bw) * 8 * c.bh * 8, 0);
    }
    return kOk;
  }
  int sos(const uint8_t* s, const uint8_t* e) {
    const int ns = s[0];
    if (ns != nc_ || e - s < 1 + 2 * ns + 3) return kUnsupported;  // one interleaved scan only
    for (int i = 0; i < ns; ++i) {
      const int id = s[1 + 2 * i];
      Component* c = nullptr;
      for (int j = 0; j < nc_; ++j)
        if (c_[j].id == id) c = &c_[j];
      if (!c) return kCorrupt;
      c->td = s[2 + 2 * i] >> 4;
      c->ta = s[2 + 2 * i] & 15;
      if (c->td > 3 || c->ta > 3 || !dc_[c->td].ok || !ac_[c->ta].ok) return kCorrupt;
    }
    return kOk;
  }

  // ---- entropy-coded segment: bit reader over the stuffed byte stream.  64-bit buffer,
  // MSB first; refill() tops it up to >= 32 valid bits — four bytes at once when none of
  // them is 0xFF (no stuffing, no marker), byte by byte otherwise — so one refill covers a
  // Huffman code (<= 16 bits) plus its magnitude bits (<= 15).
  static bool has_ff(uint32_t w) {
    const uint32_t v = ~w;
    return ((v - 0x01010101u) & ~v & 0x80808080u) != 0;
  }
  void refill() {
    if (nbits_ >= 32) return;
    if (!marker_ && end_ - p_ >= 4) {
      uint32_t w;
      std::memcpy(&w, p_, 4);
      if (!has_ff(w)) {
        bitbuf_ |= uint64_t(__builtin_bswap32(w)) << (32 - nbits_);
        nbits_ += 32;
        p_ += 4;
        return;
      }
    }
    while (nbits_ <= 56) {
      uint64_t byte = 0;
      if (!marker_ && p_ < end_) {
        byte = *p_;
        if (byte == 0xFF) {
          const uint8_t nx = p_ + 1 < end_ ? p_[1] : 0;
          if (nx == 0x00) {
            p_ += 2;
          } else {  // a marker (RSTn / EOI): stop, feed zeros
            marker_ = true;
            byte = 0;
          }
        } else {
          ++p_;
        }
      }
      bitbuf_ |= byte << (56 - nbits_);
      nbits_ += 8;
    }
  }
  // callers refill() first
  int getbits(int n) {
    if (n == 0) return 0;
    const int v = int(bitbuf_ >> (64 - n));
    bitbuf_ <<= n;
    nbits_ -= n;
    return v;
  }
  static int extend(int v, int t) { return v < (1 << (t - 1)) ? v - (1 << t) + 1 : v; }
  int huff(const Huff& h) {
    const uint16_t f = h.fast[bitbuf_ >> 55];
    if (f) {
      const int len = f >> 8;
      bitbuf_ <<= len;
      nbits_ -= len;
      return f & 0xFF;
    }
    int code = int(bitbuf_ >> 55);  // 9 bits
    int len = 9;
    uint64_t rest = bitbuf_ << 9;
    while (len < 16 && code > h.maxcode[len]) {
      code = (code << 1) | int(rest >> 63);
      rest <<= 1;
      ++len;
    }
    if (code > h.maxcode[len]) return -1;
    bitbuf_ <<= len;
    nbits_ -= len;
    return h.vals[h.valoff[len] + code];
  }
  bool block(Component& c, int32_t* F, bool& any_ac) {
    std::memset(F, 0, 64 * sizeof(int32_t));
    any_ac = false;
    const uint16_t* q = qt_[c.tq];
    refill();
    const int t = huff(dc_[c.td]);
    if (t < 0 || t > 11) return false;
    c.pred += t ? extend(getbits(t), t) : 0;
    F[0] = c.pred * q[0];
    const Huff& ac = ac_[c.ta];
    for (int k = 1; k < 64;) {
      refill();
      const int p9 = int(bitbuf_ >> 55);
      if (const int fl = ac.fast_len[p9]) {  // code + magnitude in the first 9 bits
        k += ac.fast_run[p9];
        if (k > 63) return false;
        F[kZigzag[k]] = ac.fast_val[p9] * q[k];
        any_ac = true;
        ++k;
        bitbuf_ <<= fl;
        nbits_ -= fl;
        continue;
      }
      const int rs = huff(ac);
      if (rs < 0) return false;
      const int r = rs >> 4, s = rs & 15;
      if (s) {
        k += r;
        if (k > 63) return false;
        F[kZigzag[k]] = extend(getbits(s), s) * q[k];
        any_ac = true;
        ++k;
      } else if (r == 15) {
        k += 16;
      } else {
        break;  // EOB
      }
    }
    return true;
  }
  void restart() {
    // skip to the RSTn marker the bit reader stopped at
    bitbuf_ = 0;
    nbits_ = 0;
    marker_ = false;
    while (p_ + 1 < end_ && !(p_[0] == 0xFF && p_[1] >= 0xD0 && p_[1] <= 0xD7)) ++p_;
    if (p_ + 1 < end_) p_ += 2;
    for (int i = 0; i < nc_; ++i) c_[i].pred = 0;
  }
  int scan() {
    alignas(16) int32_t F[64];
    const Idct& id = idct();
    int until = restart_;
    for (int my = 0; my < mcuy_; ++my)
      for (int mx = 0; mx < mcux_; ++mx) {
        if (restart_) {
          if (until == 0) {
            restart();
            until = restart_;
          }
          --until;
        }
        for (int i = 0; i < nc_; ++i) {
          Component& c = c_[i];
          const int stride = c.bw * 8;
          for (int by = 0; by < c.v; ++by)
            for (int bx = 0; bx < c.h; ++bx) {
              bool any_ac;
              if (!block(c, F, any_ac)) return kCorrupt;
              const int row = (my * c.v + by) * 8, col = (mx * c.h + bx) * 8;
              id.run(F, c.plane.data() + size_t(row) * stride + col, stride, any_ac);
            }
        }
      }
    return kOk;
  }

  // ---- upsampling (triangle filter) + colour conversion
  // sample of component c at full-resolution (y, x): c.h / hmax, c.v / vmax subsampling
  int convert(uint8_t* dst) {
    const int W = w_, H = h_;
    if (nc_ == 1) {
      const Component& c = c_[0];
      for (int y = 0; y < H; ++y) {
        const uint8_t* s = c.plane.data() + size_t(y) * c.bw * 8;
        uint8_t* d = dst + size_t(y) * W * 3;
        for (int x = 0; x < W; ++x) d[3 * x] = d[3 * x + 1] = d[3 * x + 2] = s[x];
      }
      return kOk;
    }
    std::vector<uint8_t> up[3];
    const uint8_t* pl[3];
    for (int i = 0; i < 3; ++i) {
      const Component& c = c_[i];
      const int sx = hmax_ / c.h, sy = vmax_ / c.v;
      if (sx == 1 && sy == 1) {
        pl[i] = nullptr;
        continue;
      }
      up[i].resize(size_t(W) * H);
      upsample(c, sx, sy, up[i].data(), W, H);
      pl[i] = up[i].data();
    }
    for (int y = 0; y < H; ++y) {
      const uint8_t* ys = pl[0] ? pl[0] + size_t(y) * W : c_[0].plane.data() + size_t(y) * c_[0].bw * 8;
      const uint8_t* cb = pl[1] ? pl[1] + size_t(y) * W : c_[1].plane.data() + size_t(y) * c_[1].bw * 8;
      const uint8_t* cr = pl[2] ? pl[2] + size_t(y) * W : c_[2].plane.data() + size_t(y) * c_[2].bw * 8;
      uint8_t* d = dst + size_t(y) * W * 3;
      int x0 = 0;
#if defined(__AVX2__)
      x0 = ycc_rgb16(ys, cb, cr, d, W);
#endif
      for (int x = x0; x < W; ++x) {  // JFIF YCbCr -> RGB in 16.16 fixed point
        const int Y = ys[x] << 16, B = cb[x] - 128, R = cr[x] - 128;
        const int r = (Y + 91881 * R + 32768) >> 16;
        const int g = (Y - 22554 * B - 46802 * R + 32768) >> 16;
        const int b = (Y + 116130 * B + 32768) >> 16;
        d[3 * x] = uint8_t(r < 0 ? 0 : r > 255 ? 255 : r);
        d[3 * x + 1] = uint8_t(g < 0 ? 0 : g > 255 ? 255 : g);
        d[3 * x + 2] = uint8_t(b < 0 ? 0 : b > 255 ? 255 : b);
      }
    }
    return kOk;
  }
#if defined(__AVX2__)
  // 16 pixels per step: YCbCr -> RGB in Q15 16-bit lanes (R = Y + Cr' + 0.402 Cr', G = Y -
  // 0.344 Cb' - 0.714 Cr', B = Y + Cb' + 0.772 Cb', each product rounded by mulhrs), packed
  // with saturation and interleaved to RGB by byte shuffles.  Returns the pixels done.
  static int ycc_rgb16(const uint8_t* ys, const uint8_t* cb, const uint8_t* cr, uint8_t* d, int W) {
    const __m256i c128 = _mm256_set1_epi16(128);
    const __m256i kr = _mm256_set1_epi16(13173), kgb = _mm256_set1_epi16(11277), kgr = _mm256_set1_epi16(23401),
                  kb = _mm256_set1_epi16(25297);
    const __m128i m_rg0 = _mm_setr_epi8(0, 8, -1, 1, 9, -1, 2, 10, -1, 3, 11, -1, 4, 12, -1, 5);
    const __m128i m_b0 = _mm_setr_epi8(-1, -1, 0, -1, -1, 1, -1, -1, 2, -1, -1, 3, -1, -1, 4, -1);
    const __m128i m_rg1 = _mm_setr_epi8(13, -1, 6, 14, -1, 7, 15, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const __m128i m_b1 = _mm_setr_epi8(-1, 5, -1, -1, 6, -1, -1, 7, -1, -1, -1, -1, -1, -1, -1, -1);
    int x = 0;
    for (; x + 16 <= W; x += 16) {
      const __m256i Y = _mm256_cvtepu8_epi16(_mm_loadu_si128(reinterpret_cast<const __m128i*>(ys + x)));
      const __m256i B_ = _mm256_sub_epi16(_mm256_cvtepu8_epi16(_mm_loadu_si128(reinterpret_cast<const __m128i*>(cb + x))), c128);
      const __m256i R_ = _mm256_sub_epi16(_mm256_cvtepu8_epi16(_mm_loadu_si128(reinterpret_cast<const __m128i*>(cr + x))), c128);
      const __m256i R = _mm256_add_epi16(_mm256_add_epi16(Y, R_), _mm256_mulhrs_epi16(R_, kr));
      const __m256i G = _mm256_sub_epi16(_mm256_sub_epi16(Y, _mm256_mulhrs_epi16(B_, kgb)), _mm256_mulhrs_epi16(R_, kgr));
      const __m256i B = _mm256_add_epi16(_mm256_add_epi16(Y, B_), _mm256_mulhrs_epi16(B_, kb));
      const __m256i rg = _mm256_packus_epi16(R, G);                         // lane h: r(8h..8h+7), g(..)
      const __m256i bb = _mm256_packus_epi16(B, _mm256_setzero_si256());   // lane h: b(8h..8h+7), 0
      for (int h = 0; h < 2; ++h) {
        const __m128i RG = h ? _mm256_extracti128_si256(rg, 1) : _mm256_castsi256_si128(rg);
        const __m128i BB = h ? _mm256_extracti128_si256(bb, 1) : _mm256_castsi256_si128(bb);
        uint8_t* o = d + 3 * (x + 8 * h);
        _mm_storeu_si128(reinterpret_cast<__m128i*>(o),
                         _mm_or_si128(_mm_shuffle_epi8(RG, m_rg0), _mm_shuffle_epi8(BB, m_b0)));
        _mm_storel_epi64(reinterpret_cast<__m128i*>(o + 16),
                         _mm_or_si128(_mm_shuffle_epi8(RG, m_rg1), _mm_shuffle_epi8(BB, m_b1)));
      }
    }
    return x;
  }
#endif
  // triangle ("fancy") upsampling by 2 in x and / or y: each output sample weighs its
  // nearer input sample 3/4 and the farther 1/4 per upsampled axis (edges replicate), in
  // integers: a vertical 3:1 column sum, then a horizontal 3:1 blend, one rounding
  void upsample(const Component& c, int sx, int sy, uint8_t* out, int W, int H) const {
    const int cw = c.bw * 8;
    const int vw = (W + sx - 1) / sx, vh = (H + sy - 1) / sy;  // valid source samples
    std::vector<int16_t> col(size_t(vw) + 18);  // + edge replicas and a 16-lane overrun
    for (int y = 0; y < H; ++y) {
      const uint8_t *r0, *r1;
      int wv;  // vertical weights (wv : 4 - wv), scale 4
      if (sy == 2) {
        const int yc = y >> 1;
        r0 = c.plane.data() + size_t(yc) * cw;
        const int yf = (y & 1) ? (yc + 1 < vh ? yc + 1 : yc) : (yc > 0 ? yc - 1 : 0);
        r1 = c.plane.data() + size_t(yf) * cw;
        wv = 3;
      } else {
        r0 = r1 = c.plane.data() + size_t(y) * cw;
        wv = 4;
      }
      int16_t* cs = col.data() + 1;  // cs[-1], cs[vw] replicate the edges
      for (int x = 0; x < vw; ++x) cs[x] = int16_t(wv * r0[x] + (4 - wv) * r1[x]);
      cs[-1] = cs[0];
      cs[vw] = cs[vw - 1];
      uint8_t* o = out + size_t(y) * W;
      if (sx == 2) {
        int x = 0;
#if defined(__AVX2__)
        // 16 source columns -> 32 outputs: even 3 cs[j] + cs[j-1], odd 3 cs[j] + cs[j+1]
        // (scale 16, + 8, >> 4), packed and interleaved byte-wise
        const __m256i eight = _mm256_set1_epi16(8);
        for (int j = 0; 2 * j + 32 <= W && j + 16 <= vw; j += 16, x += 32) {
          const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(cs + j));
          const __m256i cm = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(cs + j - 1));
          const __m256i cp = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(cs + j + 1));
          const __m256i c3 = _mm256_add_epi16(_mm256_add_epi16(c, c), c);
          const __m256i e = _mm256_srli_epi16(_mm256_add_epi16(_mm256_add_epi16(c3, cm), eight), 4);
          const __m256i od = _mm256_srli_epi16(_mm256_add_epi16(_mm256_add_epi16(c3, cp), eight), 4);
          // interleave e / od as 16-bit pairs, then pack to bytes: lane h holds j + 8h ..
          const __m256i lo = _mm256_unpacklo_epi16(e, od), hi = _mm256_unpackhi_epi16(e, od);
          const __m256i b = _mm256_packus_epi16(lo, hi);  // lane0: j0..3 pairs, j4..7 pairs; lane1: j8..
          _mm_storeu_si128(reinterpret_cast<__m128i*>(o + x), _mm256_castsi256_si128(b));
          _mm_storeu_si128(reinterpret_cast<__m128i*>(o + x + 16), _mm256_extracti128_si256(b, 1));
        }
#endif
        for (; x < W; ++x) {
          const int xc = x >> 1;
          const int v = 3 * cs[xc] + ((x & 1) ? cs[xc + 1] : cs[xc - 1]);  // scale 16
          o[x] = uint8_t((v + 8) >> 4);
        }
      } else {
        for (int x = 0; x < W; ++x) o[x] = uint8_t((cs[x] + 2) >> 2);
      }
    }
  }

  const uint8_t* p_;
  const uint8_t* end_;
  uint16_t qt_[4][64] = {};
  Huff dc_[4], ac_[4];
  Component c_[3];
  int h_ = 0, w_ = 0, nc_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0, restart_ = 0;
  uint64_t bitbuf_ = 0;
  int nbits_ = 0;
  bool marker_ = false;
};

// images[i] -> dst + i * stride (H x W x 3 uint8); per-image Status
std::vector<int> jpeg_decode_into(uintptr_t dst, size_t dst_bytes, const py::list& images, size_t stride, int H, int W,
                                  int nthreads) {
  const size_t n = images.size();
  if (size_t(H) * W * 3 > stride) throw std::invalid_argument("jpeg_decode_into: stride smaller than H*W*3");
  if (n * stride > dst_bytes) throw std::invalid_argument("jpeg_decode_into: slot too small for the batch");
  std::vector<Py_buffer> views(n);
  size_t held = 0;
  struct Release {
    std::vector<Py_buffer>& v;
    size_t& n;
    ~Release() {
      for (size_t i = 0; i < n; ++i) PyBuffer_Release(&v[i]);
    }
  } rel{views, held};
  for (size_t i = 0; i < n; ++i) {
    if (PyObject_GetBuffer(images[i].ptr(), &views[i], PyBUF_SIMPLE) != 0) throw py::error_already_set();
    ++held;
  }
  std::vector<int> status(n, kOk);
  uint8_t* d = reinterpret_cast<uint8_t*>(dst);
  {
    py::gil_scoped_release nogil;
    pool_run(int(n), std::max(1, nthreads), [&](int i) {
      Decoder dec(static_cast<const uint8_t*>(views[i].buf), size_t(views[i].len));
      try {
        status[i] = dec.decode(d + size_t(i) * stride, H, W);
      } catch (...) {
        status[i] = kCorrupt;
      }
    });
  }
  return status;
}

// A decode running in the background (jpeg_decode_start): a host thread drives the pool
// over the batch while the caller goes on (the model worker keeps reading and batching the
// next records); wait() joins it and returns the per-image statuses.  The job holds the
// byte strings (and their buffer views) until then.
struct DecodeJob {
  py::list keep;
  std::vector<Py_buffer> views;
  size_t held = 0;
  std::vector<int> status;
  std::thread th;
  std::atomic<bool> finished{false};
  bool joined = false;

  void release() {
    for (size_t i = 0; i < held; ++i) PyBuffer_Release(&views[i]);
    held = 0;
  }
  void join() {  // GIL held on entry
    if (joined) return;
    {
      py::gil_scoped_release nogil;
      th.join();
    }
    joined = true;
    release();
  }
  ~DecodeJob() {
    if (th.joinable()) join();
    release();
  }
};

std::shared_ptr<DecodeJob> jpeg_decode_start(uintptr_t dst, size_t dst_bytes, const py::list& images, size_t stride,
                                             int H, int W, int nthreads) {
  const size_t n = images.size();
  if (size_t(H) * W * 3 > stride) throw std::invalid_argument("jpeg_decode_start: stride smaller than H*W*3");
  if (n * stride > dst_bytes) throw std::invalid_argument("jpeg_decode_start: slot too small for the batch");
  auto job = std::make_shared<DecodeJob>();
  job->keep = images;
  job->views.resize(n);
  for (size_t i = 0; i < n; ++i) {
    if (PyObject_GetBuffer(images[i].ptr(), &job->views[i], PyBUF_SIMPLE) != 0) throw py::error_already_set();
    ++job->held;
  }
  job->status.assign(n, kOk);
  DecodeJob* j = job.get();
  uint8_t* d = reinterpret_cast<uint8_t*>(dst);
  job->th = std::thread([j, d, stride, H, W, nthreads, n]() {
    pool_run(int(n), std::max(1, nthreads), [&](int i) {
      Decoder dec(static_cast<const uint8_t*>(j->views[i].buf), size_t(j->views[i].len));
      try {
        j->status[i] = dec.decode(d + size_t(i) * stride, H, W);
      } catch (...) {
        j->status[i] = kCorrupt;
      }
    });
    j->finished.store(true, std::memory_order_release);
  });
  return job;
}

// (height, width, components, baseline) from the frame header, or (0, 0, 0, false) when
// the bytes are not a JPEG / carry no frame header
py::tuple jpeg_info(const py::bytes& b) {
  const std::string_view v(b);
  const uint8_t* p = reinterpret_cast<const uint8_t*>(v.data());
  const uint8_t* e = p + v.size();
  if (e - p < 4 || p[0] != 0xFF || p[1] != 0xD8) return py::make_tuple(0, 0, 0, false);
  p += 2;
  while (p + 4 <= e) {
    if (p[0] != 0xFF) break;
    const uint8_t mk = p[1];
    if (mk == 0xFF) {
      ++p;
      continue;
    }
    p += 2;
    if (mk == 0xD8 || (mk >= 0xD0 && mk <= 0xD7) || mk == 0x01) continue;
    if (mk == 0xD9 || mk == 0xDA) break;
    const int len = (p[0] << 8) | p[1];
    if (len < 2 || p + len > e) break;
    if (mk >= 0xC0 && mk <= 0xCF && mk != 0xC4 && mk != 0xC8 && mk != 0xCC) {
      if (len < 8) break;
      const int h = (p[3] << 8) | p[4], w = (p[5] << 8) | p[6], nc = p[7];
      return py::make_tuple(h, w, nc, (mk == 0xC0 || mk == 0xC1) && p[2] == 8);
    }
    p += len;
  }
  return py::make_tuple(0, 0, 0, false);
}

// Whole files -> bytes, read on the host pool with the GIL released (the file reader's
// bulk path: one Python call per run of paths instead of an open/read per record).  A file
// that cannot be read comes back as None.
py::list read_files(const py::list& paths, int nthreads) {
  const size_t n = paths.size();
  std::vector<std::string> names(n);
  for (size_t i = 0; i < n; ++i) names[i] = paths[i].cast<std::string>();
  std::vector<std::string> data(n);
  std::vector<char> ok(n, 0);
  {
    py::gil_scoped_release nogil;
    pool_run(int(n), std::max(1, nthreads), [&](int i) {
      FILE* f = std::fopen(names[i].c_str(), "rb");
      if (!f) return;
      std::string& d = data[i];
      if (std::fseek(f, 0, SEEK_END) == 0) {
        long len = std::ftell(f);
        if (len >= 0 && std::fseek(f, 0, SEEK_SET) == 0) {
          d.resize(size_t(len));
          size_t got = len ? std::fread(&d[0], 1, size_t(len), f) : 0;
          d.resize(got);
          ok[i] = got == size_t(len);
        }
      }
      std::fclose(f);
    });
  }
  py::list out(n);
  for (size_t i = 0; i < n; ++i) {
    if (ok[i]) {
      out[i] = py::bytes(data[i]);
    } else {
      out[i] = py::none();
    }
  }
  return out;
}

}  // namespace

void register_jpeg(py::module_& m) {
  m.def("jpeg_info", &jpeg_info, py::arg("data"),
        "(height, width, components, baseline) of a JPEG's frame header; zeros when there is none.");
  py::class_<DecodeJob, std::shared_ptr<DecodeJob>>(m, "DecodeJob")
      .def("done", [](DecodeJob& j) { return j.finished.load(std::memory_order_acquire); })
      .def("wait", [](DecodeJob& j) {
        j.join();
        return j.status;
      });
  m.def("jpeg_decode_start", &jpeg_decode_start, py::arg("dst"), py::arg("dst_bytes"), py::arg("images"),
        py::arg("stride"), py::arg("h"), py::arg("w"), py::arg("nthreads") = 8,
        "jpeg_decode_into in the background: returns a DecodeJob (done() / wait() -> statuses).");
  m.def("read_files", &read_files, py::arg("paths"), py::arg("nthreads") = 8,
        "Reads whole files on the host pool (GIL released); bytes per path, None for a file that cannot be read.");
  m.def("jpeg_decode_into", &jpeg_decode_into, py::arg("dst"), py::arg("dst_bytes"), py::arg("images"),
        py::arg("stride"), py::arg("h"), py::arg("w"), py::arg("nthreads") = 8,
        "Decodes baseline JPEG byte strings into rows of `stride` bytes at `dst` (H x W x 3 RGB); per-image status "
        "0 ok, 1 not a JPEG, 2 unsupported (progressive / arithmetic / 12-bit), 3 corrupt, 4 other size.");
}
