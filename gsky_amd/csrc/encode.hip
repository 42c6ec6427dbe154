// encode.hip -- output codecs: EncodePNG's png.Encode (utils/ogc_encoders.go:
// 139; Go 1.12 image/png) for batches of RGBA tiles in HBM.
//
// Go's encoder on the *image.RGBA canvas of EncodePNG (ogc_encoders.go:82):
//   * colour type: truecolour RGB (cbTC8) when every alpha is 0xff
//     (image.RGBA.Opaque), else RGBA (cbTCA8) whose bytes are the
//     color.NRGBAModel conversion of each premultiplied pixel (a = 0 ->
//     0,0,0,0; a = 0xffff -> the bytes; else r * 0xffff / a in 16 bits, high
//     byte, wrapping like Go's uint8()) -- image.RGBA stores the palette
//     colours as they are, so a palette entry with r > a wraps;
//   * per row the filter of writer.go filter(): the sums of |int8(byte)| of the
//     Up, Paeth, None, Sub and Average residuals, tried in that order, the
//     first strictly smaller sum wins (the early exits there never change the
//     choice); the previous row of the first row is zero;
//   * zlib at DefaultCompression (level 6) over the filtered rows, written
//     through a 32 KiB bufio.Writer: IDAT chunks of exactly 32768 bytes, the
//     last one shorter; IHDR / IDAT / IEND with their CRC-32.
// Here the colour-type test, the NRGBA conversion and the filter selection run
// on the GPU (one workgroup per row), the deflate of each tile on host threads
// (zlib 1.2.11, level 6, 32 KiB window, default strategy).  The filtered rows
// -- every byte zlib receives -- are Go's exactly; the compressed bytes are
// zlib's, not Go's compress/flate (both DEFLATE: the decoded image and the
// filter bytes are identical, byte identity with Go is parity unpinned).
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gskyhip.h"

namespace gsky {
namespace {

// ------------------------------------------------------------------ GPU pass
// tile t opaque (image.RGBA.Opaque over its w x h rectangle)?
__global__ __launch_bounds__(256) void png_opaque_kernel(const uint8_t *__restrict__ rgba, int64_t tile_stride,
                                                         int64_t row_stride, const int32_t *__restrict__ wh,
                                                         int32_t *__restrict__ opaque) {
  const int t = blockIdx.x;
  const int w = wh[2 * t], h = wh[2 * t + 1];
  const uint8_t *base = rgba + (int64_t)t * tile_stride;
  int bad = 0;
  for (int64_t i = threadIdx.x; i < (int64_t)w * h; i += blockDim.x) {
    const int y = (int)(i / w), x = (int)(i % w);
    bad |= base[(int64_t)y * row_stride + 4 * x + 3] != 0xFF;
  }
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) opaque[t] = bad ? 0 : 1;
}

// byte k of row y of the image data Go's writeImage feeds the filter: RGB of
// an opaque canvas, else NRGBA; the row above row 0 is zero
__device__ __forceinline__ uint32_t png_byte(const uint8_t *__restrict__ tile, int64_t row_stride, int y, int k,
                                             bool opq) {
  if (y < 0 || k < 0) return 0u;
  const int bpp = opq ? 3 : 4;
  const int x = k / bpp, c = k - x * bpp;
  const uint8_t *px = tile + (int64_t)y * row_stride + 4 * x;
  if (opq) return px[c];
  const uint32_t a = px[3];
  if (a == 0xFF) return px[c];
  if (a == 0) return 0u;
  if (c == 3) return a;
  const uint32_t a16 = a | (a << 8);
  const uint32_t v16 = (uint32_t)px[c] | ((uint32_t)px[c] << 8);
  return ((v16 * 0xFFFFu) / a16 >> 8) & 0xFFu;   // color.nrgbaModel, uint8() truncation
}

__device__ __forceinline__ uint32_t abs8(uint32_t d) { d &= 0xFFu; return d < 128u ? d : 256u - d; }

__device__ __forceinline__ uint32_t paeth(uint32_t a, uint32_t b, uint32_t c) {   // writer.go paeth()
  const int pc0 = (int)c;
  int pa = (int)b - pc0;
  int pb = (int)a - pc0;
  int pc = abs(pa + pb);
  pa = abs(pa);
  pb = abs(pb);
  if (pa <= pb && pa <= pc) return a;
  if (pb <= pc) return b;
  return c;
}

// One workgroup per (tile, row): out row = [filter byte][filtered bytes].
__global__ __launch_bounds__(256) void png_filter_kernel(const uint8_t *__restrict__ rgba, int64_t tile_stride,
                                                         int64_t row_stride, const int32_t *__restrict__ wh,
                                                         const int32_t *__restrict__ opaque, int max_h,
                                                         const int64_t *__restrict__ out_off,
                                                         uint8_t *__restrict__ out) {
  const int t = blockIdx.x / max_h, y = blockIdx.x % max_h;
  const int w = wh[2 * t], h = wh[2 * t + 1];
  if (y >= h) return;
  const bool opq = opaque[t] != 0;
  const int bpp = opq ? 3 : 4;
  const int n = bpp * w;
  const uint8_t *tile = rgba + (int64_t)t * tile_stride;
  __shared__ uint32_t s_sum[5][4];
  uint32_t sum[5] = {0, 0, 0, 0, 0};
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const uint32_t cur = png_byte(tile, row_stride, y, k, opq), up = png_byte(tile, row_stride, y - 1, k, opq);
    const uint32_t left = k >= bpp ? png_byte(tile, row_stride, y, k - bpp, opq) : 0u;
    const uint32_t ul = k >= bpp ? png_byte(tile, row_stride, y - 1, k - bpp, opq) : 0u;
    sum[0] += abs8(cur - up);                                        // Up
    sum[1] += abs8(k >= bpp ? cur - paeth(left, up, ul) : cur - up);   // Paeth (first bpp bytes: Up)
    sum[2] += abs8(cur);                                             // None
    sum[3] += abs8(cur - left);                                      // Sub
    sum[4] += abs8(k >= bpp ? cur - ((left + up) >> 1) : cur - (up >> 1));   // Average
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int f = 0; f < 5; f++) {
    uint32_t s = sum[f];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) s_sum[f][wv] = s;
  }
  __syncthreads();
  // tried in the order Up, Paeth, None, Sub, Average; a strictly smaller sum wins
  const int order[5] = {2, 4, 0, 1, 3};   // their PNG filter types
  uint32_t best = 0;
  int ft = 2;
#pragma unroll
  for (int f = 0; f < 5; f++) {
    const uint32_t s = s_sum[f][0] + s_sum[f][1] + s_sum[f][2] + s_sum[f][3];
    if (f == 0 || s < best) { best = s; ft = order[f]; }
  }
  uint8_t *row = out + out_off[t] + (int64_t)y * (1 + n);
  if (threadIdx.x == 0) row[0] = (uint8_t)ft;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const uint32_t cur = png_byte(tile, row_stride, y, k, opq), up = png_byte(tile, row_stride, y - 1, k, opq);
    const uint32_t left = k >= bpp ? png_byte(tile, row_stride, y, k - bpp, opq) : 0u;
    const uint32_t ul = k >= bpp ? png_byte(tile, row_stride, y - 1, k - bpp, opq) : 0u;
    uint32_t v;
    switch (ft) {
      case 0: v = cur; break;
      case 1: v = cur - left; break;
      case 2: v = cur - up; break;
      case 3: v = k >= bpp ? cur - ((left + up) >> 1) : cur - (up >> 1); break;
      default: v = k >= bpp ? cur - paeth(left, up, ul) : cur - up; break;
    }
    row[1 + k] = (uint8_t)v;
  }
}

// ------------------------------------------------------------------ GPU deflate
// The zlib stream of each tile's filtered rows built on the GPU: one final
// block -- Huffman codes built for the tile from its symbol frequencies
// (RFC 1951 3.2.7), or the fixed codes (3.2.6) where those come out shorter
// -- whose LZ77 matches are
// searched at the distances a PNG row offers -- runs, pixels to the left,
// rows above and the diagonals (deflate_tokens) -- within the row (so rows
// are encoded independently: a workgroup per tile, a thread per row, matches
// may reach back into earlier rows).  Pass 1 counts each row's bits; their prefix sums place every row
// in the tile's bit stream and every tile in one packed buffer (so only the
// compressed bytes cross PCIe); pass 2 writes the codes (the words two rows
// share by OR).  Adler-32 from per-row sums.  The stream is valid DEFLATE /
// zlib; its bytes are neither zlib's nor Go's compress/flate (parity
// unpinned; the tests inflate it and compare the rows).
__constant__ uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                      67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10,
                                       11, 11, 12, 12, 13, 13};

constexpr int kPngMaxRows = 4096;    // rows of a tile the deflate kernels handle (LDS scan)

struct BitSink {   // LSB-first bit writer over 32-bit words; first and last words by OR
  uint32_t *out;
  uint64_t acc;
  int nacc;
  int64_t word;
  bool first;
  __device__ void init(uint32_t *o, int64_t bitpos) {
    out = o; word = bitpos >> 5; nacc = (int)(bitpos & 31); acc = 0; first = true;
  }
  __device__ __forceinline__ void put(uint32_t bits, int n) {
    acc |= (uint64_t)bits << nacc;
    nacc += n;
    if (nacc >= 32) {
      if (first) { atomicOr(out + word, (uint32_t)acc); first = false; }
      else out[word] = (uint32_t)acc;
      acc >>= 32;
      nacc -= 32;
      word++;
    }
  }
  __device__ void finish() {
    if (nacc > 0) atomicOr(out + word, (uint32_t)acc);
  }
};

__device__ __forceinline__ uint32_t rev_bits(uint32_t code, int len) { return __brev(code) >> (32 - len); }

typedef uint32_t u32_unaligned __attribute__((aligned(1)));
__device__ __forceinline__ uint32_t ld_u32(const uint8_t *p) { return *(const u32_unaligned *)p; }

// fixed Huffman code of a literal / length symbol, bit-reversed for LSB-first output
__device__ __forceinline__ void lit_code(int v, uint32_t &code, int &len) {
  if (v < 144) { code = 0x30 + v; len = 8; }
  else if (v < 256) { code = 0x190 + (v - 144); len = 9; }
  else if (v < 280) { code = v - 256; len = 7; }
  else { code = 0xC0 + (v - 280); len = 8; }
  code = rev_bits(code, len);
}

// One row's LZ77 tokens, in order, to f(sym, len_extra, n_len_extra, dcode,
// dist_extra, n_dist_extra): dcode < 0 for a literal.  Candidates at the
// distances a PNG of upsampled tiles repeats at -- runs (1), the pixel to the
// left and 2-3 pixels back, the pixels above (1-3 rows) and the diagonals --
// the one saving the most bits by a static estimate (6.5 bits per literal
// byte against ~7 bits of length code plus the distance code and its extra
// bits), and one step of lazy matching (a match starting one byte later that
// is 2+ bytes longer wins, the byte going out as a literal).  A model of
// these tokens with dynamic Huffman costs: 461 -> 433 KB per C2 tile (zlib
// level 6: 409 KB).
__device__ __forceinline__ int dist_code(int d) {
  int dc = 0;
  while (dc < 29 && kDistBase[dc + 1] <= d) dc++;
  return dc;
}

__device__ __forceinline__ void best_match(const uint8_t *__restrict__ data, int64_t p, int64_t p1, int bpp,
                                           int stride, int &best, int &bd) {
  best = 0;
  bd = 0;
  int bscore = -(1 << 30);
  const int dists[11] = {1, bpp, stride, 2 * bpp, 3 * bpp, 2 * stride, stride - bpp, stride + bpp,
                         2 * stride - bpp, 2 * stride + bpp, 3 * stride};
  const int lim = (int)min((int64_t)258, p1 - p);
#pragma unroll
  for (int c = 0; c < 11; c++) {
    const int d = dists[c];
    if (p - d < 0 || d > 32768) continue;
    int l = 0;
    // 4 bytes per compare (unaligned dword loads), the first difference by ctz
    while (l + 4 <= lim) {
      const uint32_t x = ld_u32(data + p + l) ^ ld_u32(data + p + l - d);
      if (x) { l += __builtin_ctz(x) >> 3; goto done; }
      l += 4;
    }
    while (l < lim && data[p + l] == data[p + l - d]) l++;
  done:
    if (l < 3) continue;
    const int score = 13 * l - 2 * (7 + 5 + (int)kDistExtra[dist_code(d)]);   // 2x the bits saved
    if (score > bscore) { bscore = score; best = l; bd = d; }
  }
}

template <class F>
__device__ __forceinline__ void deflate_tokens(const uint8_t *__restrict__ data, int64_t p0, int64_t p1, int bpp,
                                               int stride, F &&f) {
  int64_t p = p0;
  while (p < p1) {
    int best, bd;
    best_match(data, p, p1, bpp, stride, best, bd);
    if (best >= 3 && p + 1 < p1) {   // lazy: a longer match one byte on
      int b2, d2;
      best_match(data, p + 1, p1, bpp, stride, b2, d2);
      if (b2 > best + 1) {
        f((int)data[p], 0u, 0, -1, 0u, 0);
        p++;
        best = b2;
        bd = d2;
      }
    }
    if (best >= 3) {
      int lc = 0;
      while (lc < 28 && kLenBase[lc + 1] <= best) lc++;
      const int dc = dist_code(bd);
      f(257 + lc, (uint32_t)(best - kLenBase[lc]), (int)kLenExtra[lc], dc, (uint32_t)(bd - kDistBase[dc]),
        (int)kDistExtra[dc]);
      p += best;
    } else {
      f((int)data[p], 0u, 0, -1, 0u, 0);
      p++;
    }
  }
}

// The tokens of a row are searched once (pass 1) and kept, packed one per
// dword -- symbol (9 bits) | distance code + 1 (5) | length extra (5) |
// distance extra (13) -- for the bit count and the write pass to replay.
__device__ __forceinline__ uint32_t tok_pack(int sym, uint32_t lx, int dc, uint32_t dx) {
  return (uint32_t)sym | ((uint32_t)(dc + 1) << 9) | (lx << 14) | (dx << 19);
}

template <class F>
__device__ __forceinline__ void tok_replay(const uint32_t *__restrict__ tk, int n, F &&f) {
  for (int i = 0; i < n; i++) {
    const uint32_t v = tk[i];
    const int sym = (int)(v & 511u), dc = (int)((v >> 9) & 31u) - 1;
    f(sym, (v >> 14) & 31u, sym >= 257 ? (int)kLenExtra[sym - 257] : 0, dc, v >> 19, dc >= 0 ? (int)kDistExtra[dc] : 0);
  }
}

// ---- per-tile Huffman codes (round 4: one dynamic block per tile, RFC 1951
// 3.2.7, or the fixed codes where those are shorter)
constexpr int kLitN = 286, kDistN = 30, kClN = 19, kSymN = kLitN + kDistN;
__constant__ uint8_t kClOrder[kClN] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct PngTab {   // a tile's codes (global, written by pass 1, read by pass 2)
  uint32_t hdr[160];        // the block header, LSB-first: BFINAL, BTYPE and (dynamic) the code lengths
  uint16_t code[kSymN];     // literal / length codes then distance codes, bit-reversed
  uint8_t len[kSymN];
  int32_t hdr_bits;
};

struct HuffLds {   // scratch of one code construction (thread 0 but the rank sort)
  uint32_t wf[kLitN];       // frequencies, at least two of them non-zero
  int16_t sorted[kLitN];    // symbols by ascending (frequency, symbol)
  uint32_t weight[2 * kLitN];
  int16_t parent[2 * kLitN];
  uint8_t depth[2 * kLitN];
  int32_t m, ok;
};

// Code lengths <= maxbits of the n symbols with frequencies `freq` (a
// Huffman tree by the two-queue merge over the sorted leaves; lengths past
// maxbits folded back as zlib's gen_bitlen does; least frequent symbols take
// the longest codes).  All threads call it; H.ok = 0 if the result is not a
// complete prefix code (the caller then uses the fixed codes).
__device__ void huff_lengths(const uint32_t *freq, int n, int maxbits, uint8_t *len, HuffLds &H) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    int m = 0;
    for (int s = 0; s < n; s++) { H.wf[s] = freq[s]; m += freq[s] ? 1 : 0; }
    for (int s = 0; m < 2 && s < n; s++)   // a code needs two leaves (zlib forces them too)
      if (!H.wf[s]) { H.wf[s] = 1; m++; }
    H.m = m;
  }
  __syncthreads();
  for (int s = tid; s < n; s += blockDim.x) {   // rank of (freq, symbol) among the used symbols
    len[s] = 0;
    if (!H.wf[s]) continue;
    const uint64_t key = ((uint64_t)H.wf[s] << 9) | (uint64_t)s;
    int r = 0;
    for (int q = 0; q < n; q++)
      if (H.wf[q] && (((uint64_t)H.wf[q] << 9) | (uint64_t)q) < key) r++;
    H.sorted[r] = (int16_t)s;
  }
  __syncthreads();
  if (tid == 0) {
    const int m = H.m;
    for (int i = 0; i < m; i++) H.weight[i] = H.wf[H.sorted[i]];
    int il = 0, in = m, nx = m;   // leaf queue, internal queue (ascending by construction)
    auto take = [&]() {
      if (il < m && (in >= nx || H.weight[il] <= H.weight[in])) return il++;
      return in++;
    };
    for (int k = 0; k < m - 1; k++) {
      const int a = take(), b = take();
      H.weight[nx] = H.weight[a] + H.weight[b];
      H.parent[a] = (int16_t)nx; H.parent[b] = (int16_t)nx;
      nx++;
    }
    const int root = nx - 1;
    int bl_count[16] = {0};
    int overflow = 0;
    H.depth[root] = 0;
    for (int i = root - 1; i >= 0; i--) {
      const int d = H.depth[H.parent[i]] + 1;
      H.depth[i] = (uint8_t)min(d, 255);
      if (i < m) {
        if (d > maxbits) overflow++;
        bl_count[min(d, maxbits)]++;
      }
    }
    while (overflow > 0) {   // zlib gen_bitlen: move leaves until the code fits
      int bits = maxbits - 1;
      while (bits > 0 && bl_count[bits] == 0) bits--;
      if (bits == 0) break;
      bl_count[bits]--;
      bl_count[bits + 1] += 2;
      bl_count[maxbits]--;
      overflow -= 2;
    }
    // longest codes to the least frequent symbols
    int i = 0;
    for (int bits = maxbits; bits >= 1; bits--)
      for (int c = bl_count[bits]; c > 0 && i < m; c--) len[H.sorted[i++]] = (uint8_t)bits;
    uint64_t kraft = 0;   // complete: sum 2^(maxbits - len) == 2^maxbits
    for (int s = 0; s < n; s++)
      if (len[s]) kraft += 1ull << (maxbits - len[s]);
    H.ok = (i == m && kraft == (1ull << maxbits)) ? 1 : 0;
  }
  __syncthreads();
}

// canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first output
__device__ void huff_codes(const uint8_t *len, int n, uint16_t *code) {
  int bl[16] = {0}, next[16];
  for (int s = 0; s < n; s++) bl[len[s]]++;
  bl[0] = 0;
  int c = 0;
  for (int b = 1; b < 16; b++) { c = (c + bl[b - 1]) << 1; next[b] = c; }
  for (int s = 0; s < n; s++)
    code[s] = len[s] ? (uint16_t)rev_bits((uint32_t)next[len[s]]++, len[s]) : 0;
}

__device__ void fixed_table(PngTab &T) {
  for (int v = 0; v < kLitN; v++) {
    uint32_t c;
    int l;
    lit_code(v, c, l);
    T.code[v] = (uint16_t)c; T.len[v] = (uint8_t)l;
  }
  for (int d = 0; d < kDistN; d++) { T.code[kLitN + d] = (uint16_t)rev_bits((uint32_t)d, 5); T.len[kLitN + d] = 5; }
  T.hdr[0] = 0x3u;   // BFINAL 1, BTYPE 01
  T.hdr_bits = 3;
}

// Pass 0, a thread per row (a wave per 64 rows of a tile, so every CU holds
// many rows in flight): the row's tokens, kept for pass 1's bit count and
// pass 2, and -- for a dynamic code -- their symbol frequencies, summed per
// workgroup in LDS and added to the tile's global histogram.
__global__ __launch_bounds__(64) void png_tokenize_kernel(const uint8_t *__restrict__ filt,
                                                          const int64_t *__restrict__ off,
                                                          const int32_t *__restrict__ wh,
                                                          const int32_t *__restrict__ opaque, int max_h,
                                                          uint32_t *__restrict__ tok, int32_t *__restrict__ ntok,
                                                          int64_t per, uint32_t *__restrict__ freq, int dynamic) {
  const int groups = (max_h + 63) / 64;
  const int t = (int)(blockIdx.x / groups), tid = threadIdx.x, y = (int)(blockIdx.x % groups) * 64 + tid;
  const int h = wh[2 * t + 1];
  const int bpp = opaque[t] ? 3 : 4;
  const int stride = 1 + bpp * wh[2 * t];
  const uint8_t *data = filt + off[t];
  __shared__ uint32_t s_freq[kSymN];
  for (int i = tid; i < kSymN; i += 64) s_freq[i] = 0;
  __syncthreads();
  if (y < h) {
    const int64_t p0 = (int64_t)y * stride;
    uint32_t *tk = tok + (int64_t)t * per + p0;   // a row has at most `stride` tokens
    int n = 0;
    deflate_tokens(data, p0, p0 + stride, bpp, stride, [&](int sym, uint32_t lx, int, int dc, uint32_t dx, int) {
      tk[n++] = tok_pack(sym, lx, dc, dx);
      if (dynamic) {
        atomicAdd(&s_freq[sym], 1u);
        if (dc >= 0) atomicAdd(&s_freq[kLitN + dc], 1u);
      }
    });
    ntok[(int64_t)t * max_h + y] = n;
  }
  __syncthreads();
  if (dynamic)
    for (int i = tid; i < kSymN; i += 64)
      if (s_freq[i]) atomicAdd(&freq[(int64_t)t * kSymN + i], s_freq[i]);
}

// Pass 1, a workgroup per tile: the rows' Adler-32 sums; the tile's dynamic
// code from pass 0's frequencies (or the fixed one where that is shorter,
// header included) into tab[t]; each row's bits under it; the stream length.
// Tile stream: zlib header (2 B), block header, rows, end of block, pad to a
// byte, Adler-32 (4 B).
__global__ __launch_bounds__(256) void png_deflate_count_kernel(const uint8_t *__restrict__ filt,
                                                                const int64_t *__restrict__ off,
                                                                const int32_t *__restrict__ wh,
                                                                const int32_t *__restrict__ opaque, int max_h,
                                                                int32_t *__restrict__ row_bits,
                                                                uint32_t *__restrict__ adler,
                                                                int64_t *__restrict__ zlen, PngTab *__restrict__ tab,
                                                                int dynamic, const uint32_t *__restrict__ tok,
                                                                const int32_t *__restrict__ ntok, int64_t per,
                                                                const uint32_t *__restrict__ freq) {
  const int t = blockIdx.x, tid = threadIdx.x;
  const int w = wh[2 * t], h = wh[2 * t + 1];
  const int bpp = opaque[t] ? 3 : 4;
  const int stride = 1 + bpp * w;
  const uint8_t *data = filt + off[t];
  __shared__ uint32_t s_a[kPngMaxRows], s_b[kPngMaxRows];
  __shared__ int64_t s_bits[256];
  __shared__ uint32_t s_freq[kSymN], s_clf[kClN];
  __shared__ uint8_t s_len[kSymN], s_cll[kClN];
  __shared__ uint16_t s_code[kSymN], s_clc[kClN];
  __shared__ uint8_t s_rs[kSymN];     // code-length RLE: symbols
  __shared__ uint8_t s_rx[kSymN];     // and their extra values
  __shared__ int32_t s_nr, s_hlit, s_hdist, s_use_fixed;
  __shared__ HuffLds H;
  PngTab &T = tab[t];
  for (int i = tid; i < kSymN; i += blockDim.x) s_freq[i] = dynamic ? freq[(int64_t)t * kSymN + i] : 0u;
  __syncthreads();
  for (int y = tid; y < h; y += blockDim.x) {
    const int64_t p0 = (int64_t)y * stride;
    uint64_t a = 0, bb = 0;   // sum of bytes, sum of (n - i) * byte (exact: < 2^40), then mod 65521
    int i = 0;
    for (; i + 4 <= stride; i += 4) {
      const uint32_t v = ld_u32(data + p0 + i);
      const uint32_t c0 = v & 0xFFu, c1 = (v >> 8) & 0xFFu, c2 = (v >> 16) & 0xFFu, c3 = v >> 24;
      a += c0 + c1 + c2 + c3;
      bb += (uint64_t)(stride - i) * c0 + (uint64_t)(stride - i - 1) * c1 + (uint64_t)(stride - i - 2) * c2 +
            (uint64_t)(stride - i - 3) * c3;
    }
    for (; i < stride; i++) {
      a += data[p0 + i];
      bb += (uint64_t)(stride - i) * data[p0 + i];
    }
    s_a[y] = (uint32_t)(a % 65521u);
    s_b[y] = (uint32_t)(bb % 65521u);
  }
  if (tid == 0) { s_freq[256] = 1; s_use_fixed = dynamic ? 0 : 1; }   // end of block
  __syncthreads();
  if (dynamic) {
    huff_lengths(s_freq, kLitN, 15, s_len, H);
    int ok = H.ok;
    huff_lengths(s_freq + kLitN, kDistN, 15, s_len + kLitN, H);
    ok &= H.ok;
    if (tid == 0) {   // HLIT / HDIST, then the run-length coded lengths (16 / 17 / 18)
      int hlit = kLitN, hdist = kDistN;
      while (hlit > 257 && !s_len[hlit - 1]) hlit--;
      while (hdist > 1 && !s_len[kLitN + hdist - 1]) hdist--;
      s_hlit = hlit; s_hdist = hdist;
      for (int k = 0; k < kClN; k++) s_clf[k] = 0;
      const int N = hlit + hdist;
      auto L = [&](int i) { return i < hlit ? s_len[i] : s_len[kLitN + i - hlit]; };
      int nr = 0;
      auto emit = [&](int sym, int x) { s_rs[nr] = (uint8_t)sym; s_rx[nr] = (uint8_t)x; nr++; s_clf[sym]++; };
      for (int i = 0; i < N;) {
        const int v = L(i);
        int run = 1;
        while (i + run < N && L(i + run) == v) run++;
        int r = run;
        if (v == 0) {
          while (r >= 11) { const int k = min(r, 138); emit(18, k - 11); r -= k; }
          if (r >= 3) { emit(17, r - 3); r = 0; }
          while (r > 0) { emit(0, 0); r--; }
        } else {
          emit(v, 0); r--;
          while (r >= 3) { const int k = min(r, 6); emit(16, k - 3); r -= k; }
          while (r > 0) { emit(v, 0); r--; }
        }
        i += run;
      }
      s_nr = nr;
    }
    __syncthreads();
    huff_lengths(s_clf, kClN, 7, s_cll, H);
    ok &= H.ok;
    if (tid == 0) {
      huff_codes(s_len, kLitN, s_code);
      huff_codes(s_len + kLitN, kDistN, s_code + kLitN);
      huff_codes(s_cll, kClN, s_clc);
      int hclen = kClN;
      while (hclen > 4 && !s_cll[kClOrder[hclen - 1]]) hclen--;
      int64_t hb = 3 + 5 + 5 + 4 + 3 * hclen;
      for (int k = 0; k < s_nr; k++) {
        const int sym = s_rs[k];
        hb += s_cll[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
      }
      // compare with the fixed codes (extra bits are the same under both)
      int64_t dyn = hb, fix = 3;
      for (int v = 0; v < kLitN; v++) {
        uint32_t c;
        int l;
        lit_code(v, c, l);
        dyn += (int64_t)s_freq[v] * s_len[v];
        fix += (int64_t)s_freq[v] * l;
      }
      for (int d = 0; d < kDistN; d++) {
        dyn += (int64_t)s_freq[kLitN + d] * s_len[kLitN + d];
        fix += (int64_t)s_freq[kLitN + d] * 5;
      }
      if (!ok || hb > 160 * 32 || fix <= dyn) {
        s_use_fixed = 1;
      } else {   // the header bits into tab[t].hdr
        uint64_t acc = 0;
        int nacc = 0, word = 0;
        auto put = [&](uint32_t bits, int nb) {
          acc |= (uint64_t)bits << nacc;
          nacc += nb;
          if (nacc >= 32) { T.hdr[word++] = (uint32_t)acc; acc >>= 32; nacc -= 32; }
        };
        put(0x5u, 3);   // BFINAL 1, BTYPE 10
        put((uint32_t)(s_hlit - 257), 5);
        put((uint32_t)(s_hdist - 1), 5);
        put((uint32_t)(hclen - 4), 4);
        for (int k = 0; k < hclen; k++) put(s_cll[kClOrder[k]], 3);
        for (int k = 0; k < s_nr; k++) {
          const int sym = s_rs[k];
          put(s_clc[sym], s_cll[sym]);
          if (sym == 16) put(s_rx[k], 2);
          else if (sym == 17) put(s_rx[k], 3);
          else if (sym == 18) put(s_rx[k], 7);
        }
        if (nacc > 0) T.hdr[word] = (uint32_t)acc;
        T.hdr_bits = (int32_t)hb;
      }
    }
    __syncthreads();
  }
  if (s_use_fixed) {
    if (tid == 0) fixed_table(T);
    __syncthreads();
    for (int i = tid; i < kSymN; i += blockDim.x) { s_len[i] = T.len[i]; s_code[i] = T.code[i]; }
  } else {
    for (int i = tid; i < kSymN; i += blockDim.x) { T.len[i] = s_len[i]; T.code[i] = s_code[i]; }
  }
  __syncthreads();
  int64_t mine = 0;
  for (int y = tid; y < h; y += blockDim.x) {
    uint32_t b = 0;
    tok_replay(tok + (int64_t)t * per + (int64_t)y * stride, ntok[(int64_t)t * max_h + y],
               [&](int sym, uint32_t, int le, int dc, uint32_t, int de) {
                 b += s_len[sym] + le + (dc >= 0 ? s_len[kLitN + dc] + de : 0);
               });
    row_bits[(int64_t)t * max_h + y] = (int32_t)b;
    mine += b;
  }
  s_bits[tid] = mine;
  __syncthreads();
  if (tid == 0) {
    int64_t total = 0;
    for (int k = 0; k < (int)blockDim.x; k++) total += s_bits[k];
    uint32_t A = 1, B = 0;   // adler32 of the rows in order
    for (int y = 0; y < h; y++) {
      B = (uint32_t)((B + (uint64_t)stride * A + s_b[y]) % 65521u);
      A = (A + s_a[y]) % 65521u;
    }
    adler[t] = (B << 16) | A;
    const int hdr_bits = s_use_fixed ? 3 : T.hdr_bits;
    zlen[t] = 2 + (hdr_bits + total + s_len[256] + 7) / 8 + 4;
  }
}

// Pass 2: the codes of every row at its bit offset in the tile's stream, at
// the tile's byte offset zoff[t] of the packed buffer (zeroed).
__global__ __launch_bounds__(256) void png_deflate_write_kernel(const uint8_t *__restrict__ filt,
                                                                const int64_t *__restrict__ off,
                                                                const int32_t *__restrict__ wh,
                                                                const int32_t *__restrict__ opaque, int max_h,
                                                                const int32_t *__restrict__ row_bits,
                                                                const uint32_t *__restrict__ adler,
                                                                const int64_t *__restrict__ zoff,
                                                                const int64_t *__restrict__ zlen,
                                                                uint8_t *__restrict__ packed,
                                                                const PngTab *__restrict__ tab,
                                                                const uint32_t *__restrict__ tok,
                                                                const int32_t *__restrict__ ntok, int64_t per) {
  const int t = blockIdx.x;
  const int w = wh[2 * t], h = wh[2 * t + 1];
  const int bpp = opaque[t] ? 3 : 4;
  const int stride = 1 + bpp * w;
  (void)filt;
  uint8_t *z = packed + zoff[t];
  // the tile's stream starts on a 4-byte boundary of the packed buffer
  uint32_t *words = (uint32_t *)z;
  __shared__ int64_t s_start[kPngMaxRows + 1];
  __shared__ uint16_t s_code[kSymN];
  __shared__ uint8_t s_len[kSymN];
  const PngTab &T = tab[t];
  for (int i = threadIdx.x; i < kSymN; i += blockDim.x) { s_code[i] = T.code[i]; s_len[i] = T.len[i]; }
  const int hdr_bits = T.hdr_bits;
  if (threadIdx.x == 0) {   // row bit offsets (serial: h <= 4096 adds)
    int64_t b = 16 + hdr_bits;
    for (int y = 0; y < h; y++) { s_start[y] = b; b += row_bits[(int64_t)t * max_h + y]; }
    s_start[h] = b;
  }
  __syncthreads();
  // every byte by OR into the zeroed buffer, so no write order matters
  auto or_byte = [&](int64_t pos, uint32_t v) { atomicOr(words + (pos >> 2), (v & 0xFFu) << (8 * (pos & 3))); };
  if (threadIdx.x == 0) {
    or_byte(0, 0x78);   // CMF: deflate, 32 KiB window
    or_byte(1, 0x01);   // FLG: (0x78 * 256 + 0x01) % 31 == 0
    BitSink bs;         // block header
    bs.init(words, 16);
    int k = 0;
    for (; k + 32 <= hdr_bits; k += 32) bs.put(T.hdr[k >> 5], 32);
    if (k < hdr_bits) bs.put(T.hdr[k >> 5] & ((1u << (hdr_bits - k)) - 1u), hdr_bits - k);
    bs.finish();
    bs.init(words, s_start[h]);   // end of block
    bs.put(s_code[256], s_len[256]);
    bs.finish();
    const int64_t end = (s_start[h] + s_len[256] + 7) / 8;   // Adler-32 after the byte padding
    const uint32_t ad = adler[t];
    or_byte(end, ad >> 24); or_byte(end + 1, ad >> 16); or_byte(end + 2, ad >> 8); or_byte(end + 3, ad);
  }
  for (int y = threadIdx.x; y < h; y += blockDim.x) {
    BitSink bs;
    bs.init(words, s_start[y]);
    tok_replay(tok + (int64_t)t * per + (int64_t)y * stride, ntok[(int64_t)t * max_h + y],
               [&](int sym, uint32_t lx, int le, int dc, uint32_t dx, int de) {
                     bs.put(s_code[sym], s_len[sym]);
                     if (dc >= 0) {
                       if (le) bs.put(lx, le);
                       bs.put(s_code[kLitN + dc], s_len[kLitN + dc]);
                       if (de) bs.put(dx, de);
                     }
                   });
    bs.finish();
  }
  (void)zlen;
}

// CRC-32 (PNG / zlib polynomial 0xEDB88320) of each 32 KiB IDAT chunk of
// every tile's stream, type bytes "IDAT" included: a thread per chunk,
// slicing by 4 over dword loads (the stream starts 4-byte aligned and so
// does every chunk), tables in LDS.
__global__ __launch_bounds__(256) void png_idat_crc_kernel(const uint8_t *__restrict__ packed,
                                                           const int64_t *__restrict__ zoff,
                                                           const int64_t *__restrict__ zlen, int n_tiles,
                                                           int max_chunks, uint32_t *__restrict__ crc) {
  __shared__ uint32_t T[4][256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    T[0][i] = c;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = T[0][i];
    for (int k = 1; k < 4; k++) { c = T[0][c & 0xFFu] ^ (c >> 8); T[k][i] = c; }
  }
  __syncthreads();
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)n_tiles * max_chunks) return;
  const int t = (int)(g / max_chunks), ch = (int)(g % max_chunks);
  const int64_t n_all = zlen[t], p0 = (int64_t)ch * 32768;
  if (p0 >= n_all) return;
  const int64_t n = min((int64_t)32768, n_all - p0);
  const uint8_t *d = packed + zoff[t] + p0;
  uint32_t c = 0xFFFFFFFFu;
  const uint8_t idat[4] = {'I', 'D', 'A', 'T'};
  for (int k = 0; k < 4; k++) c = T[0][(c ^ idat[k]) & 0xFFu] ^ (c >> 8);
  int64_t i = 0;
  for (; i + 4 <= n; i += 4) {
    c ^= *(const uint32_t *)(d + i);
    c = T[3][c & 0xFFu] ^ T[2][(c >> 8) & 0xFFu] ^ T[1][(c >> 16) & 0xFFu] ^ T[0][c >> 24];
  }
  for (; i < n; i++) c = T[0][(c ^ d[i]) & 0xFFu] ^ (c >> 8);
  crc[g] = c ^ 0xFFFFFFFFu;
}

// ------------------------------------------------------------------ GeoTIFF
// PackBits (TIFF 6.0 section 9) of one tile row (libtiff encodes tiled
// PackBits row by row): runs of 3+ equal bytes as replicate runs, the rest
// as literal runs, at most 128 bytes each.  Returns the encoded length.
__device__ int packbits_row(const uint8_t *in, int n, uint8_t *out) {
  int i = 0, o = 0;
  while (i < n) {
    int run = 1;
    while (i + run < n && run < 128 && in[i + run] == in[i]) run++;
    if (run >= 3) {
      out[o++] = (uint8_t)(257 - run);   // -(run - 1)
      out[o++] = in[i];
      i += run;
      continue;
    }
    // literal: up to the next run of 3 (or 128 bytes)
    int j = i, lit = 0;
    while (j < n && lit < 128) {
      if (j + 2 < n && in[j] == in[j + 1] && in[j] == in[j + 2]) break;
      j++;
      lit++;
    }
    out[o++] = (uint8_t)(lit - 1);
    for (int k = 0; k < lit; k++) out[o++] = in[i + k];
    i += lit;
  }
  return o;
}

// One thread per (band, tile, row of the tile): the row's samples (edge
// tiles padded with `pad`) PackBits-encoded into its slot.
__global__ __launch_bounds__(256) void tiff_rows_kernel(const uint8_t *const *__restrict__ bands, int ts, int width,
                                                        int height, int bx, int by, int ntx, int nty,
                                                        const uint8_t *__restrict__ pad, int64_t slot,
                                                        uint8_t *__restrict__ raw, uint8_t *__restrict__ enc,
                                                        int32_t *__restrict__ len, int64_t n_rows) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int row = (int)(r % by);
  const int64_t tb = r / by;
  const int tile = (int)(tb % ((int64_t)ntx * nty));
  const int b = (int)(tb / ((int64_t)ntx * nty));
  const int tx = tile % ntx, ty = tile / ntx;
  const int y = ty * by + row;
  const int rb = bx * ts;
  uint8_t *line = raw + r * (int64_t)rb;
  const uint8_t *src = bands[b];
  for (int x = 0; x < bx; x++) {
    const int gx = tx * bx + x;
    const bool in = src && gx < width && y < height;   // no source: an EmptyTile band, all `pad`
    for (int k = 0; k < ts; k++) line[x * ts + k] = in ? src[((int64_t)y * width + gx) * ts + k] : pad[b * 8 + k];
  }
  len[r] = packbits_row(line, rb, enc + r * slot);
}

// ------------------------------------------------------------------ host framing
void put32(std::vector<uint8_t> &o, uint32_t v) {
  o.push_back((uint8_t)(v >> 24)); o.push_back((uint8_t)(v >> 16));
  o.push_back((uint8_t)(v >> 8)); o.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t> &o, const char *type, const uint8_t *data, size_t n) {
  put32(o, (uint32_t)n);
  const size_t at = o.size();
  o.insert(o.end(), type, type + 4);
  if (n) o.insert(o.end(), data, data + n);
  put32(o, (uint32_t)crc32(0L, o.data() + at, (uInt)(n + 4)));
}

// PNG signature + IHDR of a w x h 8-bit truecolour (alpha) image.
void png_head(int w, int h, bool opq, std::vector<uint8_t> &o) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  o.assign(sig, sig + 8);
  uint8_t ihdr[13];
  const uint32_t ww = (uint32_t)w, hh = (uint32_t)h;
  ihdr[0] = ww >> 24; ihdr[1] = ww >> 16; ihdr[2] = ww >> 8; ihdr[3] = ww;
  ihdr[4] = hh >> 24; ihdr[5] = hh >> 16; ihdr[6] = hh >> 8; ihdr[7] = hh;
  ihdr[8] = 8;                 // bit depth
  ihdr[9] = opq ? 2 : 6;       // truecolour / truecolour + alpha
  ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
  chunk(o, "IHDR", ihdr, 13);
}

// A whole PNG around a finished zlib stream, written straight into dst
// (cap bytes): 32 KiB IDAT chunks (Go's bufio.Writer size), IEND; returns
// its size, 0 when it does not fit.
size_t png_frame(const uint8_t *z, size_t zn, int w, int h, bool opq, uint8_t *dst, size_t cap,
                 const uint32_t *idat_crc) {
  std::vector<uint8_t> head;
  png_head(w, h, opq, head);
  const size_t need = head.size() + (zn / 32768 + 1) * 12 + zn + 12;
  if (need > cap) return 0;
  uint8_t *o = dst;
  std::memcpy(o, head.data(), head.size());
  o += head.size();
  auto be32 = [&](uint32_t v) { o[0] = v >> 24; o[1] = v >> 16; o[2] = v >> 8; o[3] = v; o += 4; };
  const uLong crc_idat = crc32(0L, (const Bytef *)"IDAT", 4);
  for (size_t p = 0; p < zn; p += 32768) {
    const size_t n = std::min<size_t>(32768, zn - p);
    be32((uint32_t)n);
    std::memcpy(o, "IDAT", 4);
    o += 4;
    std::memcpy(o, z + p, n);
    o += n;
    be32(idat_crc ? idat_crc[p / 32768] : (uint32_t)crc32(crc_idat, z + p, (uInt)n));
  }
  be32(0);
  std::memcpy(o, "IEND", 4);
  o += 4;
  be32((uint32_t)crc32(0L, (const Bytef *)"IEND", 4));
  return (size_t)(o - dst);
}

// One tile through host zlib: PNG signature, IHDR, the zlib stream in 32 KiB
// IDAT chunks, IEND.
int png_tile(const uint8_t *filtered, size_t n_filtered, int w, int h, bool opq, std::vector<uint8_t> &o) {
  png_head(w, h, opq, o);
  std::vector<uint8_t> z(compressBound((uLong)n_filtered) + 64);
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  if (deflateInit2(&s, 6, Z_DEFLATED, 15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return GSKYHIP_E_ARG;
  s.next_in = (Bytef *)filtered;
  s.avail_in = (uInt)n_filtered;
  s.next_out = z.data();
  s.avail_out = (uInt)z.size();
  const int rc = deflate(&s, Z_FINISH);
  const size_t zn = z.size() - s.avail_out;
  deflateEnd(&s);
  if (rc != Z_STREAM_END) return GSKYHIP_E_ARG;
  for (size_t p = 0; p < zn; p += 32768) chunk(o, "IDAT", z.data() + p, std::min<size_t>(32768, zn - p));
  chunk(o, "IEND", nullptr, 0);
  return 0;
}

// BigTIFF writer state: IFD entries (sorted by tag on output) + out-of-line data.
struct TiffEntry {
  uint16_t tag, type;
  uint64_t count;
  std::vector<uint8_t> data;   // little-endian values
};

template <typename T> void put_le(std::vector<uint8_t> &o, T v) {
  for (size_t k = 0; k < sizeof(T); k++) o.push_back((uint8_t)((uint64_t)v >> (8 * k)));
}

TiffEntry tiff_shorts(uint16_t tag, const std::vector<uint16_t> &v) {
  TiffEntry e{tag, 3, v.size(), {}};
  for (uint16_t x : v) put_le(e.data, x);
  return e;
}
TiffEntry tiff_long(uint16_t tag, uint32_t v) {
  TiffEntry e{tag, 4, 1, {}};
  put_le(e.data, v);
  return e;
}
TiffEntry tiff_long8s(uint16_t tag, const std::vector<uint64_t> &v) {
  TiffEntry e{tag, 16, v.size(), {}};
  for (uint64_t x : v) put_le(e.data, x);
  return e;
}
TiffEntry tiff_doubles(uint16_t tag, const std::vector<double> &v) {
  TiffEntry e{tag, 12, v.size(), {}};
  for (double x : v) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    put_le(e.data, u);
  }
  return e;
}
TiffEntry tiff_ascii(uint16_t tag, const std::string &s) {
  TiffEntry e{tag, 2, s.size() + 1, {}};
  e.data.assign(s.begin(), s.end());
  e.data.push_back(0);
  return e;
}

bool epsg_geographic(int epsg) {
  return epsg == 4326 || epsg == 4283 || epsg == 4269 || epsg == 4258 || epsg == 4167 || epsg == 4674 ||
         epsg == 7844;
}

std::string xml_escape(const char *s) {
  std::string o;
  for (; s && *s; s++) {
    switch (*s) {
      case '&': o += "&amp;"; break;
      case '<': o += "&lt;"; break;
      case '>': o += "&gt;"; break;
      case '"': o += "&quot;"; break;
      default: o += *s;
    }
  }
  return o;
}

}  // namespace
}  // namespace gsky

using namespace gsky;

extern "C" {

// Workspace: filtered rows | per-tile offsets, sizes, opacity | per-row bit
// counts | Adler-32, zlib lengths and offsets | per-tile codes | the packed
// zlib streams (at most 9/8 of the filtered bytes + 16 per tile: a dynamic
// block is only used where it is shorter than the fixed one) | the rows'
// tokens (a dword per filtered byte at most) and token counts.
static int64_t png_deflate_cap(int64_t per) { return (per * 9 + 7) / 8 + 64 + (per / 32768 + 1) * 4 + 256; }

int64_t gskyhip_png_workspace_size(int n_tiles, int max_w, int max_h) {
  if (n_tiles <= 0 || max_w <= 0 || max_h <= 0) return 0;
  const int64_t per = (int64_t)max_h * (1 + 4 * (int64_t)max_w);
  const int64_t a = ((int64_t)n_tiles * per + 255) / 256 * 256 + (int64_t)n_tiles * (8 + 8 + 4) + 1024;
  const int64_t b = ((int64_t)n_tiles * max_h * 4 + 255) / 256 * 256 + (int64_t)n_tiles * (4 + 8 + 8) + 1024 +
                    (int64_t)n_tiles * (int64_t)sizeof(PngTab) + 256;
  const int64_t c = (int64_t)n_tiles * per * 4 + (int64_t)n_tiles * max_h * 4 + 1024 +   // tokens, counts,
                    (int64_t)n_tiles * kSymN * 4 + 256;                                  // symbol frequencies
  return a + b + (int64_t)n_tiles * png_deflate_cap(per) + 1024 + c;
}

int64_t gskyhip_png_bound(int width, int height) {
  if (width <= 0 || height <= 0) return 0;
  const uLong raw = (uLong)height * (1 + 4 * (uLong)width);
  const uLong z = std::max<uLong>(compressBound(raw) + 64, (uLong)png_deflate_cap((int64_t)raw));
  return 8 + 25 + (int64_t)(z / 32768 + 1) * 12 + (int64_t)z + 12;
}

int gskyhip_encode_png(const uint8_t *rgba, int n_tiles, int max_w, int max_h, int64_t tile_stride,
                       int64_t row_stride, const int32_t *sizes, void *workspace, int64_t workspace_bytes,
                       uint8_t *png_out, int64_t png_capacity, int64_t *png_sizes, int n_threads, void *stream) {
  if (n_tiles <= 0) return 0;
  if (!rgba || !sizes || !png_out || !png_sizes || max_w <= 0 || max_h <= 0 || row_stride < 4LL * max_w ||
      tile_stride < row_stride * max_h)
    return GSKYHIP_E_ARG;
  if (!workspace || workspace_bytes < gskyhip_png_workspace_size(n_tiles, max_w, max_h)) return GSKYHIP_E_ARG;
  for (int t = 0; t < n_tiles; t++) {
    const int w = sizes[2 * t], h = sizes[2 * t + 1];
    if (w <= 0 || h <= 0 || w > max_w || h > max_h || png_capacity < gskyhip_png_bound(w, h)) return GSKYHIP_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t per = (int64_t)max_h * (1 + 4 * (int64_t)max_w);
  char *ws = (char *)workspace;
  uint8_t *filt = (uint8_t *)ws;
  char *tail = ws + ((int64_t)n_tiles * per + 255) / 256 * 256;
  int64_t *d_off = (int64_t *)tail;
  int32_t *d_wh = (int32_t *)(d_off + n_tiles);
  int32_t *d_opq = d_wh + 2 * n_tiles;
  std::vector<int64_t> off(n_tiles);
  for (int t = 0; t < n_tiles; t++) off[t] = (int64_t)t * per;
  std::vector<char> meta((size_t)n_tiles * (8 + 8));
  std::memcpy(meta.data(), off.data(), (size_t)n_tiles * 8);
  std::memcpy(meta.data() + (size_t)n_tiles * 8, sizes, (size_t)n_tiles * 8);
  if (hipMemcpyAsync(d_off, meta.data(), meta.size(), hipMemcpyHostToDevice, s) != hipSuccess) return GSKYHIP_E_HIP;
  hipLaunchKernelGGL(png_opaque_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, rgba, tile_stride, row_stride, d_wh,
                     d_opq);
  hipLaunchKernelGGL(png_filter_kernel, dim3((unsigned)((int64_t)n_tiles * max_h)), dim3(256), 0, s, rgba,
                     tile_stride, row_stride, d_wh, d_opq, max_h, d_off, filt);
  if (hipGetLastError() != hipSuccess) return GSKYHIP_E_HIP;
  // GSKYHIP_PNG_ZLIB=1: deflate with zlib level 6 on host threads (round 3)
  const char *zl = std::getenv("GSKYHIP_PNG_ZLIB");
  const bool host_zlib = zl && std::atoi(zl) != 0;
  const bool trace = std::getenv("GSKYHIP_PNG_TRACE") != nullptr;
  auto now_us = [] {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  const double t_start = now_us();
  if (!host_zlib && max_h <= kPngMaxRows) {
    char *b = tail + (int64_t)n_tiles * (8 + 8 + 4) + 1024;
    b = (char *)(((uintptr_t)b + 255) & ~(uintptr_t)255);
    int32_t *d_rowbits = (int32_t *)b;
    b += ((int64_t)n_tiles * max_h * 4 + 255) / 256 * 256;
    uint32_t *d_adler = (uint32_t *)b;
    int64_t *d_zlen = (int64_t *)(b + (((int64_t)n_tiles * 4 + 7) & ~(int64_t)7));
    int64_t *d_zoff = d_zlen + n_tiles;
    PngTab *d_tab = (PngTab *)(((uintptr_t)(d_zoff + n_tiles) + 255) & ~(uintptr_t)255);
    uint8_t *d_packed = (uint8_t *)(((uintptr_t)(d_tab + n_tiles) + 255) & ~(uintptr_t)255);
    // per-tile dynamic Huffman codes where they are shorter (GSKYHIP_PNG_FIXED=1: fixed codes only)
    const char *fx = std::getenv("GSKYHIP_PNG_FIXED");
    const int dynamic = (fx && std::atoi(fx) != 0) ? 0 : 1;
    uint32_t *d_tok = (uint32_t *)(((uintptr_t)(d_packed + (int64_t)n_tiles * png_deflate_cap(per)) + 255) &
                                   ~(uintptr_t)255);
    int32_t *d_ntok = (int32_t *)(d_tok + (int64_t)n_tiles * per);
    uint32_t *d_freq = (uint32_t *)(((uintptr_t)(d_ntok + (int64_t)n_tiles * max_h) + 255) & ~(uintptr_t)255);
    if ((char *)(d_freq + (int64_t)n_tiles * kSymN) > ws + workspace_bytes) return GSKYHIP_E_ARG;
    if (hipMemsetAsync(d_freq, 0, (size_t)n_tiles * kSymN * 4, s) != hipSuccess) return GSKYHIP_E_HIP;
    hipLaunchKernelGGL(png_tokenize_kernel, dim3((unsigned)((int64_t)n_tiles * ((max_h + 63) / 64))), dim3(64), 0, s, filt,
                       d_off, d_wh, d_opq, max_h, d_tok, d_ntok, per, d_freq, dynamic);
    hipLaunchKernelGGL(png_deflate_count_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, filt, d_off, d_wh, d_opq,
                       max_h, d_rowbits, d_adler, d_zlen, d_tab, dynamic, d_tok, d_ntok, per, d_freq);
    std::vector<int64_t> zlen(n_tiles), zoff(n_tiles);
    std::vector<int32_t> opq(n_tiles);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(zlen.data(), d_zlen, (size_t)n_tiles * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(opq.data(), d_opq, (size_t)n_tiles * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return GSKYHIP_E_HIP;
    const double t_count = now_us();
    int64_t total = 0, max_zlen = 0;
    for (int t = 0; t < n_tiles; t++) {
      zoff[t] = total;
      total += (zlen[t] + 3) & ~(int64_t)3;
      max_zlen = std::max(max_zlen, zlen[t]);
    }
    const int max_chunks = (int)((max_zlen + 32767) / 32768);
    if (hipMemcpyAsync(d_zoff, zoff.data(), (size_t)n_tiles * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(d_packed, 0, (size_t)std::max<int64_t>(total, 4), s) != hipSuccess)
      return GSKYHIP_E_HIP;
    hipLaunchKernelGGL(png_deflate_write_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, filt, d_off, d_wh, d_opq,
                       max_h, d_rowbits, d_adler, d_zoff, d_zlen, d_packed, d_tab, d_tok, d_ntok, per);
    // IDAT CRCs behind the packed streams (the pinned read-back holds both)
    const int64_t crc_at = (total + 255) & ~(int64_t)255;
    const int64_t n_crc = (int64_t)n_tiles * max_chunks;
    if (crc_at + n_crc * 4 > (int64_t)n_tiles * png_deflate_cap(per)) return GSKYHIP_E_ARG;
    uint32_t *d_crc = (uint32_t *)(d_packed + crc_at);
    if (n_crc > 0)
      hipLaunchKernelGGL(png_idat_crc_kernel, dim3((unsigned)((n_crc + 255) / 256)), dim3(256), 0, s, d_packed, d_zoff,
                         d_zlen, n_tiles, max_chunks, d_crc);
    uint8_t *zhost = nullptr;
    const int64_t back = crc_at + n_crc * 4;
    if (hipGetLastError() != hipSuccess || hipHostMalloc((void **)&zhost, (size_t)std::max<int64_t>(back, 4),
                                                         hipHostMallocDefault) != hipSuccess)
      return GSKYHIP_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) { hipHostFree(zhost); return GSKYHIP_E_HIP; }
    const double t_write = now_us();
    if (hipMemcpyAsync(zhost, d_packed, (size_t)back, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      hipHostFree(zhost);
      return GSKYHIP_E_HIP;
    }
    const double t_copy = now_us();
    // PNG framing on host threads: IHDR, 32 KiB IDAT chunks with CRC-32, IEND
    std::atomic<int> next(0), err(0);
    auto frame = [&]() {
      for (;;) {
        const int t = next++;
        if (t >= n_tiles) return;
        const size_t n = png_frame(zhost + zoff[t], (size_t)zlen[t], sizes[2 * t], sizes[2 * t + 1], opq[t] != 0,
                                   png_out + (int64_t)t * png_capacity, (size_t)png_capacity,
                                   (const uint32_t *)(zhost + crc_at) + (int64_t)t * max_chunks);
        if (!n) err = GSKYHIP_E_ARG;
        png_sizes[t] = (int64_t)n;
      }
    };
    const int nt = std::max(1, std::min(n_threads > 0 ? n_threads : 1, n_tiles));
    std::vector<std::thread> pool;
    for (int i = 1; i < nt; i++) pool.emplace_back(frame);
    frame();
    for (auto &th : pool) th.join();
    hipHostFree(zhost);
    if (trace)
      std::fprintf(stderr, "png tiles=%d filter+count_us=%.0f write_us=%.0f d2h_us=%.0f (%.1f MB) frame_us=%.0f\n",
                   n_tiles, t_count - t_start, t_write - t_count, t_copy - t_write, total / 1e6, now_us() - t_copy);
    return err.load();
  }
  std::vector<uint8_t> host((size_t)n_tiles * per);
  std::vector<int32_t> opq(n_tiles);
  if (hipMemcpyAsync(host.data(), filt, host.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(opq.data(), d_opq, (size_t)n_tiles * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return GSKYHIP_E_HIP;
  // deflate + framing per tile on host threads
  std::atomic<int> next(0), err(0);
  auto work = [&]() {
    std::vector<uint8_t> o;
    for (;;) {
      const int t = next++;
      if (t >= n_tiles) return;
      const int w = sizes[2 * t], h = sizes[2 * t + 1];
      const size_t n = (size_t)h * (1 + (opq[t] ? 3 : 4) * (size_t)w);
      const int rc = png_tile(host.data() + off[t], n, w, h, opq[t] != 0, o);
      if (rc || (int64_t)o.size() > png_capacity) { err = rc ? rc : GSKYHIP_E_ARG; png_sizes[t] = 0; continue; }
      std::memcpy(png_out + (int64_t)t * png_capacity, o.data(), o.size());
      png_sizes[t] = (int64_t)o.size();
    }
  };
  const int nt = std::max(1, std::min(n_threads > 0 ? n_threads : 1, n_tiles));
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; i++) pool.emplace_back(work);
  work();
  for (auto &th : pool) th.join();
  return err.load();
}

// ---- GeoTIFF (EncodeGdalOpen / EncodeGdal, utils/ogc_encoders.go:277-450)
static int tiff_sample(int dtype, int &ts, uint16_t &fmt) {
  switch (dtype) {
    case GSKYHIP_BYTE: ts = 1; fmt = 1; return 0;
    case GSKYHIP_SIGNEDBYTE: ts = 1; fmt = 2; return 0;
    case GSKYHIP_INT16: ts = 2; fmt = 2; return 0;
    case GSKYHIP_UINT16: ts = 2; fmt = 1; return 0;
    case GSKYHIP_FLOAT32: ts = 4; fmt = 3; return 0;
    default: return GSKYHIP_E_TYPE;
  }
}

int64_t gskyhip_geotiff_workspace_size(int width, int height, int n_bands, int dtype, int block_x, int block_y) {
  int ts;
  uint16_t fmt;
  if (width <= 0 || height <= 0 || n_bands <= 0 || block_x <= 0 || block_y <= 0 || tiff_sample(dtype, ts, fmt))
    return 0;
  const int64_t ntx = (width + block_x - 1) / block_x, nty = (height + block_y - 1) / block_y;
  const int64_t rows = (int64_t)n_bands * ntx * nty * block_y;
  const int64_t rb = (int64_t)block_x * ts;
  const int64_t slot = rb + rb / 128 + 2;
  return rows * (rb + slot + 4) + 8 * (int64_t)n_bands + 64 * (int64_t)n_bands + 4096;
}

int64_t gskyhip_geotiff_bound(int width, int height, int n_bands, int dtype, int block_x, int block_y) {
  int ts;
  uint16_t fmt;
  if (width <= 0 || height <= 0 || n_bands <= 0 || block_x <= 0 || block_y <= 0 || tiff_sample(dtype, ts, fmt))
    return 0;
  const int64_t ntx = (width + block_x - 1) / block_x, nty = (height + block_y - 1) / block_y;
  const int64_t rows = (int64_t)n_bands * ntx * nty * block_y;
  const int64_t rb = (int64_t)block_x * ts;
  return rows * (rb + rb / 128 + 2) + (int64_t)n_bands * ntx * nty * 16 + 65536 + 512 * (int64_t)n_bands;
}

int gskyhip_encode_geotiff(const void *const *bands, int n_bands, int dtype, int width, int height,
                           const double *geot, int epsg, const double *nodata, const char *const *names,
                           int block_x, int block_y, void *workspace, int64_t workspace_bytes, uint8_t *out,
                           int64_t capacity, int64_t *size, void *stream) {
  int ts;
  uint16_t fmt;
  if (!bands || !geot || !out || !size || n_bands <= 0 || n_bands > 4096) return GSKYHIP_E_ARG;
  if (tiff_sample(dtype, ts, fmt)) return GSKYHIP_E_TYPE;
  if (width <= 0 || height <= 0 || block_x <= 0 || block_y <= 0 || block_x % 16 || block_y % 16) return GSKYHIP_E_ARG;
  if (!workspace || workspace_bytes < gskyhip_geotiff_workspace_size(width, height, n_bands, dtype, block_x, block_y))
    return GSKYHIP_E_ARG;
  if (capacity < gskyhip_geotiff_bound(width, height, n_bands, dtype, block_x, block_y)) return GSKYHIP_E_ARG;
  const int ntx = (width + block_x - 1) / block_x, nty = (height + block_y - 1) / block_y;
  const int64_t n_tiles = (int64_t)n_bands * ntx * nty;
  const int64_t n_rows = n_tiles * block_y;
  const int64_t rb = (int64_t)block_x * ts;
  const int64_t slot = rb + rb / 128 + 2;
  char *ws = (char *)workspace;
  uint8_t *raw = (uint8_t *)ws;
  uint8_t *enc = raw + n_rows * rb;
  int32_t *len = (int32_t *)(enc + n_rows * slot);
  const uint8_t **d_bands = (const uint8_t **)(((uintptr_t)(len + n_rows) + 15) & ~(uintptr_t)15);
  uint8_t *d_pad = (uint8_t *)(d_bands + n_bands);
  // EncodeGdal (ogc_encoders.go:357-436) skips EmptyTile bands: no nodata, no
  // long_name, no pixels -- GTiff fills their blocks at close with the
  // dataset nodata, the last value SetNoDataValue stored (one per GeoTIFF).
  std::vector<char> empty((size_t)n_bands, 0);
  int last_nd = -1;   // the band whose nodata the file keeps
  for (int b = 0; b < n_bands; b++) {
    empty[b] = names && names[b] && std::strncmp(names[b], "EmptyTile", 9) == 0;
    if (!empty[b] && nodata) last_nd = b;
  }
  // edge-tile padding: the band's nodata in the band type (0 without one);
  // an EmptyTile band is all the dataset nodata
  std::vector<char> meta((size_t)n_bands * 8 + (size_t)n_bands * 8, 0);
  std::memcpy(meta.data(), bands, (size_t)n_bands * 8);
  for (int b = 0; b < n_bands; b++) {
    uint8_t *pb = (uint8_t *)meta.data() + (size_t)n_bands * 8 + 8 * b;
    if (empty[b]) std::memset(meta.data() + 8 * (size_t)b, 0, 8);
    const double v = empty[b] ? (last_nd >= 0 ? nodata[last_nd] : 0.0) : nodata ? nodata[b] : 0.0;
    if (dtype == GSKYHIP_FLOAT32) { const float f = (float)v; std::memcpy(pb, &f, 4); }
    else if (ts == 2) { const int16_t h = (int16_t)(dtype == GSKYHIP_UINT16 ? (int32_t)(uint16_t)v : (int32_t)v); std::memcpy(pb, &h, 2); }
    else pb[0] = (uint8_t)(int)v;
  }
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(d_bands, meta.data(), meta.size(), hipMemcpyHostToDevice, s) != hipSuccess) return GSKYHIP_E_HIP;
  hipLaunchKernelGGL(tiff_rows_kernel, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, s, d_bands, ts, width,
                     height, block_x, block_y, ntx, nty, d_pad, slot, raw, enc, len, n_rows);
  if (hipGetLastError() != hipSuccess) return GSKYHIP_E_HIP;
  std::vector<int32_t> lens((size_t)n_rows);
  std::vector<uint8_t> encs((size_t)(n_rows * slot));
  if (hipMemcpyAsync(lens.data(), len, (size_t)n_rows * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(encs.data(), enc, encs.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return GSKYHIP_E_HIP;
  // file: header | tile data (band-major, tiles row-major) | IFD | out-of-line tag data
  std::vector<uint8_t> o;
  o.reserve((size_t)std::min<int64_t>(capacity, 1LL << 30));
  o.push_back('I'); o.push_back('I');
  put_le<uint16_t>(o, 43); put_le<uint16_t>(o, 8); put_le<uint16_t>(o, 0);
  put_le<uint64_t>(o, 0);   // first IFD offset, patched below
  std::vector<uint64_t> toff((size_t)n_tiles), tcnt((size_t)n_tiles);
  for (int64_t t = 0; t < n_tiles; t++) {
    toff[t] = o.size();
    for (int r = 0; r < block_y; r++) {
      const int64_t i = t * block_y + r;
      o.insert(o.end(), encs.begin() + i * slot, encs.begin() + i * slot + lens[i]);
    }
    tcnt[t] = o.size() - toff[t];
  }
  if (o.size() & 1) o.push_back(0);
  std::vector<TiffEntry> ents;
  ents.push_back(tiff_long(256, (uint32_t)width));
  ents.push_back(tiff_long(257, (uint32_t)height));
  ents.push_back(tiff_shorts(258, std::vector<uint16_t>((size_t)n_bands, (uint16_t)(8 * ts))));
  ents.push_back(tiff_shorts(259, {32773}));   // PackBits
  // GTiff Create's default photometric: RGB for 3 or 4 Byte bands (the 4th
  // an associated alpha extra sample), MinIsBlack otherwise
  const bool byte = dtype == GSKYHIP_BYTE || dtype == GSKYHIP_SIGNEDBYTE;
  const bool rgb = byte && (n_bands == 3 || n_bands == 4);
  ents.push_back(tiff_shorts(262, {(uint16_t)(rgb ? 2 : 1)}));
  ents.push_back(tiff_shorts(277, {(uint16_t)n_bands}));
  ents.push_back(tiff_shorts(284, {(uint16_t)(n_bands > 1 ? 2 : 1)}));   // INTERLEAVE=BAND
  ents.push_back(tiff_long(322, (uint32_t)block_x));
  ents.push_back(tiff_long(323, (uint32_t)block_y));
  ents.push_back(tiff_long8s(324, toff));
  ents.push_back(tiff_long8s(325, tcnt));
  if (rgb && n_bands == 4) ents.push_back(tiff_shorts(338, {1}));
  else if (!rgb && n_bands > 1) ents.push_back(tiff_shorts(338, std::vector<uint16_t>((size_t)n_bands - 1, 0)));
  ents.push_back(tiff_shorts(339, std::vector<uint16_t>((size_t)n_bands, fmt)));
  if (geot[2] == 0.0 && geot[4] == 0.0) {
    ents.push_back(tiff_doubles(33550, {geot[1], -geot[5], 0.0}));
    ents.push_back(tiff_doubles(33922, {0.0, 0.0, 0.0, geot[0], geot[3], 0.0}));
  } else {   // ModelTransformationTag for rotated grids
    ents.push_back(tiff_doubles(34264, {geot[1], geot[2], 0.0, geot[0], geot[4], geot[5], 0.0, geot[3],
                                        0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0}));
  }
  if (epsg > 0) {
    const bool geo = epsg_geographic(epsg);
    ents.push_back(tiff_shorts(34735, {1, 1, 0, 3, 1024, 0, 1, (uint16_t)(geo ? 2 : 1), 1025, 0, 1, 1,
                                       (uint16_t)(geo ? 2048 : 3072), 0, 1, (uint16_t)epsg}));
  }
  if (names) {   // GDALSetMetadataItem("long_name", NameSpace) per band
    std::string md = "<GDALMetadata>\n";
    for (int b = 0; b < n_bands; b++)
      if (names[b] && !empty[b])
        md += "  <Item name=\"long_name\" sample=\"" + std::to_string(b) + "\">" + xml_escape(names[b]) + "</Item>\n";
    md += "</GDALMetadata>";
    ents.push_back(tiff_ascii(42112, md));
  }
  if (last_nd >= 0) {   // GDAL_NODATA: a single dataset value, the last band's that set one
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%.18g", nodata[last_nd]);
    ents.push_back(tiff_ascii(42113, buf));
  }
  std::sort(ents.begin(), ents.end(), [](const TiffEntry &a, const TiffEntry &b) { return a.tag < b.tag; });
  const uint64_t ifd = o.size();
  const uint64_t ifd_bytes = 8 + 20 * ents.size() + 8;
  uint64_t extra = ifd + ifd_bytes;
  std::vector<uint8_t> tail;
  put_le<uint64_t>(o, ents.size());
  for (auto &e : ents) {
    put_le<uint16_t>(o, e.tag);
    put_le<uint16_t>(o, e.type);
    put_le<uint64_t>(o, e.count);
    if (e.data.size() <= 8) {
      std::vector<uint8_t> v = e.data;
      v.resize(8, 0);
      o.insert(o.end(), v.begin(), v.end());
    } else {
      put_le<uint64_t>(o, extra + tail.size());
      tail.insert(tail.end(), e.data.begin(), e.data.end());
      if (tail.size() & 1) tail.push_back(0);
    }
  }
  put_le<uint64_t>(o, 0);   // no next IFD
  o.insert(o.end(), tail.begin(), tail.end());
  for (int k = 0; k < 8; k++) o[8 + k] = (uint8_t)(ifd >> (8 * k));
  if ((int64_t)o.size() > capacity) return GSKYHIP_E_ARG;
  std::memcpy(out, o.data(), o.size());
  *size = (int64_t)o.size();
  return 0;
}

}  // extern "C"
