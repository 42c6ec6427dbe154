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
//   decile_chunk_scan_kernel  64-pixel chunks per polygon (exclusive scan)
//   decile_transpose_kernel   one wave per (64-pixel chunk, 64 bands of the
//                         chunk): the [pixel][band] tile read coalesced (a
//                         pixel's bands are contiguous in the time-innermost
//                         stack), transposed through the wave's LDS tile and
//                         written band-major at the pixel's place in the
//                         compacted list -- every polygon is spread over all
//                         CUs (no largest-polygon bound), no counting, no
//                         compaction: nodata values are written too and
//                         skipped by the selection
//   decile_select_kernel  one workgroup per (polygon, band) segment: one pass
//                         over the segment counts its non-nodata values and
//                         finds the bits all their keys share (AND / OR), and
//                         keeps the keys in LDS when they fit; then the
//                         distinct ranks the picks need (<= 2 dc) on the
//                         order-preserving 32-bit keys: one 2048-bin
//                         histogram of the 11 bits below the shared ones,
//                         scanned once, places every rank in its bucket; the
//                         keys of those buckets (<= 64 each) are compacted
//                         into LDS and each rank is the rem-th of its
//                         bucket by a 64-lane counting compare.  Buckets
//                         holding more keys (heavy ties, skewed data)
//                         continue by MSD radix selection with 8-bit digits,
//                         one LDS histogram per distinct prefix of the
//                         pending ranks -- then the reference's picks.
// Keys order -0.0 before +0.0 where Go's sort may leave them in either order;
// the picked values are then equal as float32 (NaN-free stacks; with NaNs the
// reference's order is implementation-defined).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "drill.h"
#include "gsky_device.h"

namespace gsky {

namespace {

constexpr int kSelThreads = 512;
constexpr int kSelWaves = kSelThreads / 64;
constexpr int kMaxRanks = 32;        // distinct ranks selected per pass set (2 x decile_count <= 32)
constexpr int kBinsLog = 11;         // first selection pass: 2048 buckets
constexpr int kBins = 1 << kBinsLog;
constexpr int kCandMax = 64;         // keys of one bucket resolved by the counting compare
static_assert(kBins == 4 * kSelThreads, "the bucket scan gives each thread 4 bins");
static_assert(kMaxRanks * kCandMax <= kBins, "candidates reuse the bucket histogram");
constexpr int kTilePad = 65;         // LDS tile row pitch (floats): conflict-free transposed reads

__device__ __forceinline__ uint32_t fkey(float f) {   // order-preserving key of a float
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fdecode(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

constexpr int kDecChunk = 64;        // pixels per transpose item
constexpr int kSelLds = 36 * 1024;   // dynamic LDS of a select workgroup (histograms + key cache): 4 per CU
constexpr int kSelU = 16;            // segment values per thread in flight (a 6k-value segment: one round)
constexpr int kHistSlots = kBins / 256;  // radix histograms at once (the region also holds the 2048 buckets)

// Exclusive scan of 64-pixel chunks per polygon (one block; n_polys is modest).
__global__ __launch_bounds__(1024) void decile_chunk_scan_kernel(const int32_t *__restrict__ count, int n_polys,
                                                                 int32_t *__restrict__ base) {
  __shared__ int32_t s_sum[1024];
  const int tid = threadIdx.x;
  int carry = 0;
  for (int c0 = 0; c0 < n_polys; c0 += 1024) {
    const int i = c0 + tid;
    const int v = i < n_polys ? (count[i] + kDecChunk - 1) / kDecChunk : 0;
    s_sum[tid] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan
      const int add = tid >= o ? s_sum[tid - o] : 0;
      __syncthreads();
      s_sum[tid] += add;
      __syncthreads();
    }
    if (i < n_polys) base[i] = carry + s_sum[tid] - v;
    const int tot = s_sum[1023];
    __syncthreads();
    carry += tot;
  }
  if (tid == 0) base[n_polys] = carry;
}

// The 64 lanes of one wavefront see each other's LDS writes in program
// order: keep the compiler from moving LDS accesses across this point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave per (64-pixel chunk ch, group g of 32 bands of the pass); four
// independent waves per workgroup.  Band j of polygon p: vals[seg0 + j *
// count[p] + k] for its pixel k, seg0 = mask_off[p] * n_chunk (the compacted
// pixel list of p holds count[p] <= its window bytes).  A load instruction
// reads the 32 bands (128 contiguous bytes) of two pixels, a store
// instruction writes one band of the 64 pixels (256 contiguous bytes); the
// wave's 64 x 32 tile (8.4 KB of LDS) keeps 16 waves per CU.
constexpr int kTrBands = 32;
__global__ __launch_bounds__(256) void decile_transpose_kernel(const float *__restrict__ stack, int t_stride,
                                                               const int32_t *__restrict__ idx,
                                                               const int64_t *__restrict__ mask_off,
                                                               const int32_t *__restrict__ count,
                                                               const int32_t *__restrict__ chunk_base, int n_polys,
                                                               const int32_t *__restrict__ tsel, int n_chunk,
                                                               int n_groups, float *__restrict__ vals) {
  constexpr int kPad = kTrBands + 1;
  __shared__ float tile[4][64 * kPad];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;
  const int ch = (int)(item / n_groups), g = (int)(item % n_groups);
  if (ch >= chunk_base[n_polys]) return;   // whole waves; no workgroup barrier below
  int lo = 0, hi = n_polys - 1;            // polygon owning chunk ch
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (chunk_base[mid] <= ch) lo = mid; else hi = mid - 1;
  }
  const int p = lo;
  const int n = count[p];
  const int k0 = (ch - chunk_base[p]) * kDecChunk;
  const int m = min(kDecChunk, n - k0);
  const int nb = min(kTrBands, n_chunk - g * kTrBands);   // bands of this group
  const int bl = lane & (kTrBands - 1), half = lane / kTrBands;
  // every lane loads from a valid address (band 0 of the group, pixel 0 of
  // the chunk) so the loads are unconditional and all in flight
  const float *base = stack + tsel[g * kTrBands + (bl < nb ? bl : 0)];
  const int32_t my_px = idx[mask_off[p] + k0 + (lane < m ? lane : 0)];
  float *T = tile[wave];
  {   // all 64 pixels' loads in flight at once (lanes past m hold pixel 0 of the chunk;
      // their rows are never stored): 3 % faster than two rounds of 16
      // (profiles/r03u_kernel_stats_c4_tr*.csv)
    float v[32];
#pragma unroll
    for (int u = 0; u < 32; u++) {   // pixels 2u (lanes 0-31) and 2u + 1 (lanes 32-63)
      const int px0 = __builtin_amdgcn_readlane(my_px, 2 * u);
      const int px1 = __builtin_amdgcn_readlane(my_px, 2 * u + 1);
      v[u] = base[(int64_t)(half ? px1 : px0) * t_stride];
    }
#pragma unroll
    for (int u = 0; u < 32; u++) T[(2 * u + half) * kPad + bl] = v[u];
  }
  wave_lds_sync();
  float *seg = vals + mask_off[p] * (int64_t)n_chunk + (int64_t)(g * kTrBands) * n + k0;
  if (lane < m) {
    for (int j = 0; j < nb; j++) seg[(int64_t)j * n + lane] = T[lane * kPad + j];   // lane = pixel
  }
}

// computeDeciles of one (polygon, band) segment; status 0, 1 (band total 0:
// zeros, Count 0 in the reference's TimeSeries) or GSKYHIP_E_RANGE (the
// reference indexes buf[len] and panics: len % (dc + 1) == 0 with step 1).
// Dynamic LDS: n_slots histograms of 256 bins, then cache_keys keys (the
// segment as it is, nodata included: no compaction, skipped on every pass).
template <int kU>
__global__ __launch_bounds__(kSelThreads) void decile_select_kernel(const float *__restrict__ vals,
                                                                    const int64_t *__restrict__ mask_off,
                                                                    const int32_t *__restrict__ count,
                                                                    const int32_t *__restrict__ totals, int n_chunk,
                                                                    int b0, int n_list, int dc, float nodata,
                                                                    int n_slots, int cache_keys, float *__restrict__ out,
                                                                    int32_t *__restrict__ status) {
  extern __shared__ uint32_t dyn[];
  uint32_t (*hist)[256] = (uint32_t (*)[256])dyn;
  uint32_t *cache = dyn + n_slots * 256;
  __shared__ uint32_t s_pref[kMaxRanks];   // rank r: its key's bits above `pos`
  __shared__ uint32_t s_rem[kMaxRanks];    // rank r: its rank among the keys sharing that prefix
  __shared__ int32_t s_rank[kMaxRanks];    // the distinct ranks, ascending
  __shared__ int32_t s_slot[kMaxRanks];    // rank r -> histogram slot (distinct prefix)
  __shared__ uint32_t s_spref[kMaxRanks];  // slot -> prefix (ascending)
  __shared__ int32_t s_bkt[kMaxRanks];    // rank r: its bucket of the first pass
  __shared__ uint32_t s_bcnt[kMaxRanks];   // rank r: the keys in that bucket
  __shared__ int32_t s_soff[kMaxRanks];    // slot -> first candidate
  __shared__ uint32_t s_fill[kMaxRanks];   // slot -> candidates written
  __shared__ int8_t s_map[kBins];          // bucket -> slot, -1 when no rank needs it
  __shared__ uint32_t red[3 * kSelWaves];
  __shared__ uint32_t s_wsum[kSelWaves];
  __shared__ int32_t s_nr, s_ns, s_fast;
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
  const int n = count[p];
  const float *buf = vals + mask_off[p] * (int64_t)n_chunk + (int64_t)j * n;
  // pass 1: the non-nodata values (the reference's buf, drill.go:231-237):
  // their count, the bits all their keys share, and the segment's keys in
  // LDS while they fit (order is irrelevant to order statistics)
  const bool fits = n <= cache_keys;
  // keys of the values `v != nodata` rejects (-0.0 == 0.0; a NaN nodata rejects nothing)
  const bool skip_on = nodata == nodata;
  const uint32_t kn1 = fkey(nodata), kn2 = nodata == 0.0f ? fkey(-nodata) : kn1;
  auto skipk = [&](uint32_t k) { return skip_on && (k == kn1 || k == kn2); };
  uint32_t ka = 0xFFFFFFFFu, ko = 0u;
  int valid = 0;   // kU: values per thread in flight per round
  for (int i0 = 0; i0 < n; i0 += kSelThreads * kU) {
    float v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = i0 + u * kSelThreads + tid;
      v[u] = i < n ? buf[i] : nodata;
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = i0 + u * kSelThreads + tid;
      const bool keep = i < n && v[u] != nodata;
      const uint32_t k = fkey(v[u]);
      if (keep) { ka &= k; ko |= k; valid++; }
      if (fits && i < n) cache[i] = k;
    }
  }
  for (int sh = 32; sh > 0; sh >>= 1) {
    ka &= __shfl_xor(ka, sh);
    ko |= __shfl_xor(ko, sh);
    valid += __shfl_xor(valid, sh);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6] = ka; red[kSelWaves + (tid >> 6)] = ko; red[2 * kSelWaves + (tid >> 6)] = (uint32_t)valid;
  }
  __syncthreads();
  uint32_t kand = 0xFFFFFFFFu, kor = 0u;
  int len = 0;
#pragma unroll
  for (int w = 0; w < kSelWaves; w++) { kand &= red[w]; kor |= red[kSelWaves + w]; len += (int)red[2 * kSelWaves + w]; }
  if (len <= 0) {   // total > 0 implies a non-nodata value; keep the slot defined anyway
    for (int i = tid; i < dc; i += kSelThreads) dst[i] = 0.f;
    if (tid == 0) status[o] = 0;
    return;
  }
  const int step = len / (dc + 1);
  if (step == 0) {   // len <= dc (<= 16): sort the few values, repeat them in order
    if (tid == 0) {
      int m = 0;
      if (fits) {
        for (int i = 0; i < n && m < len; i++)
          if (!skipk(cache[i])) s_small[m++] = fdecode(cache[i]);
      } else {
        for (int i = 0; i < n && m < len; i++)
          if (buf[i] != nodata) s_small[m++] = buf[i];
      }
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
  if (tid < 64) {   // distinct ranks, ascending: the sequence r_0 (, r_0 + 1), r_1, ... is
    // non-decreasing, so a value is new where it differs from its predecessor
    const int nc = isEven ? 2 * dc : dc;
    const int i = isEven ? (tid >> 1) : tid;
    const int v = (i + 1) * step + (isEven ? (tid & 1) : 0);
    const int prev = __shfl_up(v, 1);
    const bool keep = tid < nc && (tid == 0 || v != prev);
    const uint64_t kb = __ballot(keep);
    if (keep) s_rank[__popcll(kb & ((1ull << tid) - 1ull))] = v;
    if (tid == 0) s_nr = __popcll(kb);
  }
  __syncthreads();
  const int nr = s_nr;
  int pos = (kand == kor) ? 0 : 32 - __clz(kand ^ kor);   // bits below pos differ somewhere
  if (tid < nr) {
    s_pref[tid] = pos >= 32 ? 0u : (kand >> pos);
    s_rem[tid] = (uint32_t)s_rank[tid];
  }
  // every valid key once, from the LDS copy or streamed from the segment
  auto for_keys = [&](auto &&f) {
    if (fits) {
      for (int i = tid; i < n; i += kSelThreads) {
        const uint32_t k = cache[i];
        if (!skipk(k)) f(k);
      }
    } else {
      for (int i0 = 0; i0 < n; i0 += kSelThreads * kU) {
        float v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const int i = i0 + u * kSelThreads + tid;
          v[u] = i < n ? buf[i] : nodata;
        }
#pragma unroll
        for (int u = 0; u < kU; u++)
          if (i0 + u * kSelThreads + tid < n && v[u] != nodata) f(fkey(v[u]));
      }
    }
  };
  const int wv = tid >> 6, ln = tid & 63;
  if (pos > 0) {
    // first pass: the 11 bits below the shared ones, one histogram
    const int bitsA = pos < kBinsLog ? pos : kBinsLog;
    const int shA = pos - bitsA;
    const uint32_t dmask = (1u << bitsA) - 1u;
    uint32_t *H = dyn;
    for (int i = tid; i < kBins; i += kSelThreads) { H[i] = 0u; s_map[i] = -1; }
    __syncthreads();
    for_keys([&](uint32_t k) { atomicAdd(&H[(k >> shA) & dmask], 1u); });
    __syncthreads();
    {   // inclusive scan of the buckets in place, 4 per thread
      const int b4 = 4 * tid;
      const uint32_t h0 = H[b4], h1 = H[b4 + 1], h2 = H[b4 + 2], h3 = H[b4 + 3];
      const uint32_t sum = h0 + h1 + h2 + h3;
      uint32_t incl = sum;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t up = __shfl_up(incl, o);
        if (ln >= o) incl += up;
      }
      if (ln == 63) s_wsum[wv] = incl;
      __syncthreads();
      uint32_t base = 0;
      for (int w = 0; w < wv; w++) base += s_wsum[w];
      const uint32_t ex = base + incl - sum;
      H[b4] = ex + h0; H[b4 + 1] = ex + h0 + h1; H[b4 + 2] = ex + h0 + h1 + h2; H[b4 + 3] = ex + sum;
    }
    __syncthreads();
    if (tid < 64) {   // wave 0, lane r < nr: the bucket of rank r (the first whose
      // cumulative count exceeds r), then the distinct buckets (ascending with
      // the ranks) -> slots and their candidate offsets
      const bool act = tid < nr;
      const uint32_t r = act ? (uint32_t)s_rank[tid] : 0u;
      int lo = 0, hi = (int)dmask;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (H[mid] > r) hi = mid; else lo = mid + 1;
      }
      const uint32_t before = lo ? H[lo - 1] : 0u;
      const uint32_t bcnt = H[lo] - before;
      const int prev = __shfl_up(lo, 1);
      const bool nw = act && (tid == 0 || lo != prev);
      const uint64_t nb = __ballot(nw);
      const int slot = __popcll(nb & ((2ull << tid) - 1ull)) - 1;
      uint32_t incl = nw ? bcnt : 0u;   // candidate offsets: exclusive scan over the new slots
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t up = __shfl_up(incl, o);
        if (tid >= o) incl += up;
      }
      const bool big = __ballot(act && bcnt > (uint32_t)kCandMax) != 0ull;
      if (act) {
        s_bkt[tid] = lo;
        s_rem[tid] = r - before;
        s_bcnt[tid] = bcnt;
        s_slot[tid] = slot;
      }
      if (nw) {
        s_spref[slot] = (uint32_t)lo;
        s_soff[slot] = (int)(incl - bcnt);
      }
      if (tid == 0) { s_ns = __popcll(nb); s_fast = big ? 0 : 1; }
    }
    __syncthreads();
    if (s_fast) {
      // the keys of the needed buckets, compacted per slot over the histogram
      if (tid < s_ns) { s_map[s_spref[tid]] = (int8_t)tid; s_fill[tid] = 0u; }
      __syncthreads();
      uint32_t *cand = dyn;
      for_keys([&](uint32_t k) {
        const int sl = s_map[(k >> shA) & dmask];
        if (sl >= 0) cand[s_soff[sl] + atomicAdd(&s_fill[sl], 1u)] = k;
      });
      __syncthreads();
      // rank r is the s_rem[r]-th key of its bucket (<= 64 keys, one per
      // lane): MSB-first selection over the bits below the bucket digit with
      // wave ballots -- lanes whose bit is 0 come first; equal keys end in
      // the same candidate set, any of them is the value
      for (int r = wv; r < nr; r += kSelWaves) {
        const int cnt = (int)s_bcnt[r];
        const uint32_t *c = cand + s_soff[s_slot[r]];
        const uint32_t ki = ln < cnt ? c[ln] : 0xFFFFFFFFu;
        uint64_t live = __ballot(ln < cnt);
        uint32_t rem = s_rem[r];
        for (int b = shA - 1; b >= 0; b--) {
          const uint64_t zero = __ballot(((ki >> b) & 1u) == 0u) & live;
          const uint32_t nz = (uint32_t)__popcll(zero);
          if (rem < nz) live = zero;
          else { rem -= nz; live &= ~zero; }
        }
        const int src = __ffsll((unsigned long long)live) - 1;
        const uint32_t key = __shfl(ki, src);
        if (ln == 0) s_pref[r] = key;
      }
      __syncthreads();
      pos = 0;
    } else {   // continue below the bucket digit by radix selection
      if (tid < nr) s_pref[tid] = ((pos >= 32 ? 0u : (kand >> pos)) << bitsA) | (uint32_t)s_bkt[tid];
      pos = shA;
    }
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
    // kHistSlots prefixes per pass over the keys
    for (int g0 = 0; g0 < ns; g0 += kHistSlots) {
      const int g1 = min(ns, g0 + kHistSlots);
      for (int i = tid; i < (g1 - g0) * 256; i += kSelThreads) hist[i >> 8][i & 255] = 0u;
      __syncthreads();
      auto bin = [&](uint32_t k) {
        const uint32_t hi = pos >= 32 ? 0u : (k >> pos);
        int lo = 0, hi_s = ns - 1;   // binary search of the slot with prefix hi
        while (lo < hi_s) {
          const int mid = (lo + hi_s) >> 1;
          if (s_spref[mid] < hi) lo = mid + 1; else hi_s = mid;
        }
        if (s_spref[lo] == hi && lo >= g0 && lo < g1) atomicAdd(&hist[lo - g0][(k >> shift) & ((1u << d) - 1u)], 1u);
      };
      for_keys(bin);
      __syncthreads();
      // the digit bucket holding each rank: a wave per rank, lane l sums bins
      // 4l..4l+3, an inclusive scan over the lanes finds the lane whose range
      // holds the rank, that lane walks its 4 bins (bins >= 2^d are empty)
      for (int r = wv; r < nr; r += kSelWaves) {
        if (s_slot[r] < g0 || s_slot[r] >= g1) continue;
        const uint32_t *h = hist[s_slot[r] - g0];
        const uint32_t rem = s_rem[r];
        const uint32_t b0 = h[4 * ln], b1 = h[4 * ln + 1], b2 = h[4 * ln + 2], b3 = h[4 * ln + 3];
        const uint32_t sum = b0 + b1 + b2 + b3;
        uint32_t incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t up = __shfl_up(incl, o);
          if (ln >= o) incl += up;
        }
        const uint32_t excl = incl - sum;
        if (excl <= rem && rem < incl) {   // exactly one lane (the counts of the slot exceed rem)
          uint32_t cum = excl;
          int dg = 4 * ln;
          if (cum + b0 <= rem) { cum += b0; dg++;
            if (cum + b1 <= rem) { cum += b1; dg++;
              if (cum + b2 <= rem) { cum += b2; dg++; } } }
          s_pref[r] = (s_pref[r] << d) | (uint32_t)dg;
          s_rem[r] = rem - cum;
        }
      }
      __syncthreads();
    }
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
  int32_t *idx, *count, *chunk_base, *tsel;
  float *vals;
  int64_t total;
};

DecWs decile_carve(void *base, int n_polys, int64_t mask_bytes, int chunk) {
  DecWs w;
  const int64_t cap = mask_bytes * chunk;
  char *b = (char *)base;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { char *p = b ? b + o : nullptr; o += al256(bytes); return p; };
  w.idx = (int32_t *)take(mask_bytes * 4);
  w.count = (int32_t *)take((int64_t)n_polys * 4);
  w.chunk_base = (int32_t *)take((mask_bytes / kDecChunk + n_polys + 1) * 4);
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
  hipLaunchKernelGGL(decile_chunk_scan_kernel, dim3(1), dim3(1024), 0, s, w.count, c.n_polys, w.chunk_base);
  const int64_t max_chunks = c.mask_bytes / kDecChunk + c.n_polys;   // >= sum of ceil(count / 64)
  const int n_slots = kHistSlots;
  int sel_lds = kSelLds, sel_u = kSelU;
#ifdef GSKYHIP_AB
  if (const char *e = getenv("GSKYHIP_DEC_LDS_KB")) sel_lds = std::max(12, std::min(60, atoi(e))) * 1024;
  if (const char *e = getenv("GSKYHIP_DEC_U")) sel_u = atoi(e);
#endif
  const int cache_keys = (sel_lds - n_slots * 256 * 4) / 4;
  const size_t dyn_lds = (size_t)sel_lds;
  for (int b0 = 0; b0 < n_list; b0 += c.band_chunk) {
    const int n_chunk = std::min(c.band_chunk, n_list - b0);
    const int n_groups = (n_chunk + kTrBands - 1) / kTrBands;
    const int64_t n_seg = (int64_t)c.n_polys * n_chunk;
    if (hipMemcpyAsync(w.tsel, sel.data() + b0, sizeof(int32_t) * n_chunk, hipMemcpyHostToDevice, s) != hipSuccess)
      return GSKYHIP_E_HIP;
    const int64_t items = max_chunks * n_groups;
    hipLaunchKernelGGL(decile_transpose_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, c.stack,
                       c.t_stride, w.idx, c.mask_off, w.count, w.chunk_base, c.n_polys, w.tsel, n_chunk, n_groups,
                       w.vals);
    if (sel_u == 8)
      hipLaunchKernelGGL(decile_select_kernel<8>, dim3((unsigned)n_seg), dim3(kSelThreads), dyn_lds, s, w.vals,
                         c.mask_off, w.count, c.totals, n_chunk, b0, n_list, c.decile_count, c.nodata, n_slots,
                         cache_keys, c.out, c.status);
    else
      hipLaunchKernelGGL(decile_select_kernel<kSelU>, dim3((unsigned)n_seg), dim3(kSelThreads), dyn_lds, s, w.vals,
                         c.mask_off, w.count, c.totals, n_chunk, b0, n_list, c.decile_count, c.nodata, n_slots,
                         cache_keys, c.out, c.status);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
