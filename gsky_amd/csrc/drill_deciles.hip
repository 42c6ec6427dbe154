// drill_deciles.hip -- computeDeciles (worker/gdalprocess/drill.go:229-273)
// for a batch of polygons over the HBM-resident time stack (SURVEY.md 8f
// row 3), by radix SELECTION of the order statistics the reference reads --
// no sort.
//
// Per (polygon, band) the reference collects the in-mask, non-nodata values
// (no clipping), sorts them ascending and reads decileCount order statistics:
// step = len / (dc + 1); if step > 0, decile i = buf[(i+1)*step], or the
// float32 mean of it and its successor when len % (dc + 1) == 0; otherwise
// the values are repeated in order to fill dc slots.  It runs only where the
// band's mean-pass total is > 0 (drill.go:179-191).
//
// Pipeline per chunk of bands (asynchronous, workspace from the caller):
//   drill_compact_kernel (drill.hip)  in-mask pixels of each window, compacted
//   decile_gather_kernel  one wave per (polygon, 64 bands of the chunk): tiles
//                         of 64 pixels x 64 bands read coalesced (a pixel's
//                         bands are contiguous in the time-innermost stack),
//                         transposed through LDS, compacted per band (ballot)
//                         and written as contiguous per-band segments -- each
//                         (polygon, band) gets a slot of count[p] values, so
//                         no count pass and no scan are needed
//   decile_select_kernel  one workgroup per (polygon, band) segment: the
//                         distinct ranks the picks need (<= 2 dc), found
//                         together by MSD radix selection on the order-
//                         preserving 32-bit keys of the floats -- the bits all
//                         keys share are skipped (one AND / OR reduction), then
//                         8-bit digits, one LDS histogram per distinct prefix
//                         of the pending ranks; the segment is re-read per
//                         digit (L2-resident) -- then the reference's picks.
// Keys order -0.0 before +0.0 where Go's sort may leave them in either order;
// the picked values are then equal as float32 (NaN-free stacks; with NaNs the
// reference's order is implementation-defined).
#include <algorithm>
#include <vector>

#include "drill.h"
#include "gsky_device.h"

namespace gsky {

namespace {

constexpr int kSelThreads = 256;
constexpr int kMaxRanks = 32;        // distinct ranks selected per pass set (2 x decile_count <= 32)
constexpr int kTilePad = 65;         // LDS tile row pitch (floats): conflict-free transposed reads

__device__ __forceinline__ uint32_t fkey(float f) {   // order-preserving key of a float
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fdecode(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// One wave per (polygon, group of 64 bands of the chunk).  Segment of band j
// of polygon p: vals[seg0 + j * count[p] ...), seg0 = mask_off[p] * n_chunk
// (the compacted pixel list of p holds count[p] <= its window bytes).
__global__ __launch_bounds__(64) void decile_gather_kernel(const float *__restrict__ stack, int t_stride,
                                                           const int32_t *__restrict__ idx,
                                                           const int64_t *__restrict__ mask_off,
                                                           const int32_t *__restrict__ count,
                                                           const int32_t *__restrict__ tsel, int n_chunk,
                                                           int n_groups, float nodata, float *__restrict__ vals,
                                                           int32_t *__restrict__ cnt) {
  __shared__ float tile[64 * kTilePad];
  const int p = blockIdx.x / n_groups;
  const int g = blockIdx.x % n_groups;
  const int lane = threadIdx.x;
  const int nb = min(64, n_chunk - g * 64);   // bands of this group
  const bool band_ok = lane < nb;
  const float *base = stack + (band_ok ? tsel[g * 64 + lane] : 0);
  const int32_t *ip = idx + mask_off[p];
  const int n = count[p];
  float *seg = vals + mask_off[p] * (int64_t)n_chunk + (int64_t)(g * 64) * n;
  int32_t mycnt = 0;   // lane j: values kept for band j so far
  for (int k0 = 0; k0 < n; k0 += 64) {
    const int m = min(64, n - k0);
    // 64 pixels x the group's bands: pixel kk's bands are 256 contiguous bytes
#pragma unroll 16
    for (int kk = 0; kk < 64; kk++) {
      if (kk < m) tile[kk * kTilePad + lane] = band_ok ? base[(int64_t)ip[k0 + kk] * t_stride] : 0.0f;
    }
    __syncthreads();
    for (int j = 0; j < nb; j++) {   // lane = pixel k0 + lane, band j
      const float v = tile[lane * kTilePad + j];
      const bool keep = lane < m && v != nodata;
      const unsigned long long bal = __ballot(keep);
      const int pos = __popcll(bal & ((1ull << lane) - 1ull));
      const int cj = __shfl(mycnt, j);
      if (keep) seg[(int64_t)j * n + cj + pos] = v;
      if (lane == j) mycnt += __popcll(bal);
    }
    __syncthreads();
  }
  if (band_ok) cnt[(int64_t)p * n_chunk + g * 64 + lane] = mycnt;
}

// Block-wide reduction helpers (256 threads).
__device__ __forceinline__ uint32_t block_and_or(uint32_t a, uint32_t o, uint32_t *red, uint32_t &or_out) {
  for (int s = 32; s > 0; s >>= 1) {
    a &= __shfl_xor(a, s);
    o |= __shfl_xor(o, s);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[w] = a; red[4 + w] = o; }
  __syncthreads();
  const uint32_t ra = red[0] & red[1] & red[2] & red[3];
  or_out = red[4] | red[5] | red[6] | red[7];
  __syncthreads();
  return ra;
}

// computeDeciles of one (polygon, band) segment; status 0, 1 (band total 0:
// zeros, Count 0 in the reference's TimeSeries) or GSKYHIP_E_RANGE (the
// reference indexes buf[len] and panics: len % (dc + 1) == 0 with step 1).
__global__ __launch_bounds__(kSelThreads) void decile_select_kernel(const float *__restrict__ vals,
                                                                    const int32_t *__restrict__ cnt,
                                                                    const int64_t *__restrict__ mask_off,
                                                                    const int32_t *__restrict__ count,
                                                                    const int32_t *__restrict__ totals, int n_chunk,
                                                                    int b0, int n_list, int dc,
                                                                    float *__restrict__ out,
                                                                    int32_t *__restrict__ status) {
  __shared__ uint32_t hist[kMaxRanks][256];
  __shared__ uint32_t s_pref[kMaxRanks];   // rank r: its key's bits above `pos`
  __shared__ uint32_t s_rem[kMaxRanks];    // rank r: its rank among the keys sharing that prefix
  __shared__ int32_t s_rank[kMaxRanks];    // the distinct ranks, ascending
  __shared__ int32_t s_slot[kMaxRanks];    // rank r -> histogram slot (distinct prefix)
  __shared__ uint32_t s_spref[kMaxRanks];  // slot -> prefix (ascending)
  __shared__ uint32_t red[8];
  __shared__ int32_t s_nr, s_ns;
  __shared__ float s_small[64];

  const int p = blockIdx.x / n_chunk, j = blockIdx.x % n_chunk;
  const int64_t o = (int64_t)p * n_list + b0 + j;
  float *dst = out + o * dc;
  const int tid = threadIdx.x;
  if (totals[o] <= 0) {   // drill.go:186-190
    for (int i = tid; i < dc; i += kSelThreads) dst[i] = 0.f;
    if (tid == 0) status[o] = 1;
    return;
  }
  const int len = cnt[(int64_t)p * n_chunk + j];
  const float *buf = vals + mask_off[p] * (int64_t)n_chunk + (int64_t)j * count[p];
  if (len <= 0) {   // total > 0 implies a non-nodata value; keep the slot defined anyway
    for (int i = tid; i < dc; i += kSelThreads) dst[i] = 0.f;
    if (tid == 0) status[o] = 0;
    return;
  }
  const int step = len / (dc + 1);
  if (step == 0) {   // len <= dc (<= 64): sort the few values, repeat them in order
    if (tid < len) s_small[tid] = buf[tid];
    __syncthreads();
    if (tid == 0) {
      for (int a = 1; a < len; a++) {
        const float v = s_small[a];
        int b = a - 1;
        while (b >= 0 && fkey(s_small[b]) > fkey(v)) { s_small[b + 1] = s_small[b]; b--; }
        s_small[b + 1] = v;
      }
      // padding[i % len]++ for i < dc, then each value repeated padding times, in order
      int idx = 0;
      for (int i = 0; i < len && idx < dc; i++) {
        const int pad = dc / len + (i < dc % len ? 1 : 0);
        for (int q = 0; q < pad && idx < dc; q++) dst[idx++] = s_small[i];
      }
      status[o] = 0;
    }
    return;
  }
  const bool isEven = len % (dc + 1) == 0;
  if (isEven && dc * step + 1 >= len) {   // buf[iStep + 1] past the end for the last pick
    for (int i = tid; i < dc; i += kSelThreads) dst[i] = 0.f;
    if (tid == 0) status[o] = GSKYHIP_E_RANGE;
    return;
  }
  if (tid == 0) {   // distinct ranks, ascending
    int nr = 0;
    for (int i = 0; i < dc; i++) {
      const int r = (i + 1) * step;
      if (nr == 0 || s_rank[nr - 1] != r) s_rank[nr++] = r;
      if (isEven && s_rank[nr - 1] != r + 1) s_rank[nr++] = r + 1;
    }
    s_nr = nr;
  }
  // common leading bits of every key
  uint32_t ka = 0xFFFFFFFFu, ko = 0u;
  for (int i = tid; i < len; i += kSelThreads) {
    const uint32_t k = fkey(buf[i]);
    ka &= k;
    ko |= k;
  }
  uint32_t kor;
  const uint32_t kand = block_and_or(ka, ko, red, kor);
  const int nr = s_nr;
  int pos = (kand == kor) ? 0 : 32 - __clz(kand ^ kor);   // bits below pos differ somewhere
  if (tid < nr) {
    s_pref[tid] = pos >= 32 ? 0u : (kand >> pos);
    s_rem[tid] = (uint32_t)s_rank[tid];
  }
  __syncthreads();
  while (pos > 0) {
    const int d = pos < 8 ? pos : 8;
    const int shift = pos - d;
    if (tid == 0) {   // slots: the distinct prefixes of the ranks (ascending with the ranks)
      int ns = 0;
      for (int r = 0; r < nr; r++) {
        if (ns == 0 || s_spref[ns - 1] != s_pref[r]) s_spref[ns++] = s_pref[r];
        s_slot[r] = ns - 1;
      }
      s_ns = ns;
    }
    __syncthreads();
    const int ns = s_ns;
    for (int i = tid; i < ns * 256; i += kSelThreads) hist[i >> 8][i & 255] = 0u;
    __syncthreads();
    for (int i = tid; i < len; i += kSelThreads) {
      const uint32_t k = fkey(buf[i]);
      const uint32_t hi = pos >= 32 ? 0u : (k >> pos);
      int lo = 0, hi_s = ns - 1;   // binary search of the slot with prefix hi
      while (lo < hi_s) {
        const int mid = (lo + hi_s) >> 1;
        if (s_spref[mid] < hi) lo = mid + 1; else hi_s = mid;
      }
      if (s_spref[lo] == hi) atomicAdd(&hist[lo][(k >> shift) & ((1u << d) - 1u)], 1u);
    }
    __syncthreads();
    if (tid < nr) {   // the digit bucket holding each rank
      const uint32_t *h = hist[s_slot[tid]];
      uint32_t rem = s_rem[tid], cum = 0;
      int dg = 0;
      for (; dg < (1 << d) - 1; dg++) {
        if (cum + h[dg] > rem) break;
        cum += h[dg];
      }
      s_pref[tid] = (s_pref[tid] << d) | (uint32_t)dg;
      s_rem[tid] = rem - cum;
    }
    __syncthreads();
    pos = shift;
  }
  // s_pref[r] is now the key of order statistic s_rank[r]
  if (tid < dc) {
    const int r = (tid + 1) * step;
    int a = 0;
    while (s_rank[a] != r) a++;
    float de = fdecode(s_pref[a]);
    if (isEven) de = (de + fdecode(s_pref[a + 1])) / 2.0f;
    dst[tid] = de;
  }
  if (tid == 0) status[o] = 0;
}

inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

struct DecWs {
  int32_t *idx, *count, *cnt, *tsel;
  float *vals;
  int64_t total;
};

DecWs decile_carve(void *base, int n_polys, int64_t mask_bytes, int chunk) {
  DecWs w;
  const int64_t n_seg = (int64_t)n_polys * chunk;
  const int64_t cap = mask_bytes * chunk;
  char *b = (char *)base;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { char *p = b ? b + o : nullptr; o += al256(bytes); return p; };
  w.idx = (int32_t *)take(mask_bytes * 4);
  w.count = (int32_t *)take((int64_t)n_polys * 4);
  w.cnt = (int32_t *)take(n_seg * 4);
  w.tsel = (int32_t *)take((int64_t)chunk * 4);
  w.vals = (float *)take(cap * 4);
  w.total = o;
  return w;
}

}  // namespace

int64_t drill_deciles_workspace_size(int n_polys, int64_t mask_bytes, int band_chunk) {
  if (n_polys <= 0 || band_chunk <= 0 || mask_bytes < 0) return 0;
  if (mask_bytes * band_chunk >= (1LL << 40) || (int64_t)n_polys * band_chunk >= 2147483647LL) return -1;
  return decile_carve(nullptr, n_polys, mask_bytes, band_chunk).total;
}

int launch_drill_deciles(const DecileCall &c) {
  const int n_list = c.bands ? c.n_list : c.n_bands;
  if (c.n_polys <= 0 || n_list <= 0) return 0;
  if (c.decile_count <= 0 || c.band_chunk <= 0) return GSKYHIP_E_ARG;
  if (2 * c.decile_count > kMaxRanks) return GSKYHIP_E_ARG;   // dc <= 16 (the reference's deciles: 9)
  if (c.t_stride < c.n_bands || (int64_t)c.xsize * c.ysize >= 2147483647LL) return GSKYHIP_E_ARG;
  const int64_t need = drill_deciles_workspace_size(c.n_polys, c.mask_bytes, c.band_chunk);
  if (need < 0 || !c.workspace || c.workspace_bytes < need) return GSKYHIP_E_ARG;
  std::vector<int32_t> sel(n_list);
  for (int i = 0; i < n_list; i++) {
    const int b = c.bands ? c.bands[i] : i + 1;
    if (b < 1 || b > c.n_bands) return GSKYHIP_E_RANGE;
    sel[i] = b - 1;
  }
  DecWs w = decile_carve(c.workspace, c.n_polys, c.mask_bytes, c.band_chunk);
  hipStream_t s = c.stream;
  hipLaunchKernelGGL(drill_compact_kernel, dim3(c.n_polys), dim3(256), 0, s, c.win, c.mask_off, c.masks, c.n_polys,
                     c.xsize, c.ysize, w.idx, w.count);
  for (int b0 = 0; b0 < n_list; b0 += c.band_chunk) {
    const int n_chunk = std::min(c.band_chunk, n_list - b0);
    const int n_groups = (n_chunk + 63) / 64;
    const int64_t n_seg = (int64_t)c.n_polys * n_chunk;
    if (hipMemcpyAsync(w.tsel, sel.data() + b0, sizeof(int32_t) * n_chunk, hipMemcpyHostToDevice, s) != hipSuccess)
      return GSKYHIP_E_HIP;
    hipLaunchKernelGGL(decile_gather_kernel, dim3((unsigned)((int64_t)c.n_polys * n_groups)), dim3(64), 0, s, c.stack,
                       c.t_stride, w.idx, c.mask_off, w.count, w.tsel, n_chunk, n_groups, c.nodata, w.vals, w.cnt);
    hipLaunchKernelGGL(decile_select_kernel, dim3((unsigned)n_seg), dim3(kSelThreads), 0, s, w.vals, w.cnt,
                       c.mask_off, w.count, c.totals, n_chunk, b0, n_list, c.decile_count, c.out, c.status);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
