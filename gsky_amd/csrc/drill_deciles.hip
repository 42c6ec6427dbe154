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
//                         finds their smallest and largest order-preserving
//                         32-bit keys, and keeps the keys in LDS when they
//                         fit; then the distinct ranks the picks need
//                         (<= 2 dc): one 2048-bucket histogram of the key
//                         range [min, max] in buckets of 2^sh consecutive
//                         keys (>= 1024 buckets used, whatever bits the keys
//                         share), scanned once, places every rank in its
//                         bucket; the keys of those buckets (<= 64 each) are
//                         compacted into LDS and each rank is the rem-th of
//                         its bucket by a 64-lane counting select.  A rank
//                         whose bucket holds more keys (heavy ties, skew)
//                         continues on that bucket's key range, 11 bits
//                         finer per pass -- then the reference's picks.
//                         (Round 3 bucketed the 11 bits below the shared key
//                         prefix: where a band's values straddle a binary
//                         exponent most keys fell in a few buckets and 81 of
//                         the 365 C4 bands took the slow radix passes.)
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

constexpr int kSelThreads = 256;   // r04y sweep: 256 x 20 KB 14.9 ms vs 512 x 36 KB 19.1 ms (C4)
constexpr int kMaxRanks = 32;        // distinct ranks selected per pass set (2 x decile_count <= 32)
constexpr int kBinsLog = 11;         // first selection pass: 2048 buckets
constexpr int kBins = 1 << kBinsLog;
constexpr int kCandMax = 64;         // keys of one bucket resolved by the counting compare
static_assert(kBins % kSelThreads == 0, "the bucket scan gives each thread kBins / NT buckets");
static_assert(kMaxRanks * kCandMax <= kBins, "candidates reuse the bucket histogram");
constexpr int kTilePad = 65;         // LDS tile row pitch (floats): conflict-free transposed reads

__device__ __forceinline__ uint32_t fkey(float f) { return order_key(f); }
__device__ __forceinline__ float fdecode(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

constexpr int kDecChunk = 64;        // pixels per transpose item
constexpr int kSelLds = 16 * 1024;   // dynamic LDS of a select workgroup (histograms + key cache): 8 per CU
constexpr int kSelU = 8;             // segment values per thread in flight per round
constexpr int kSelWpe = 8;           // select compiled for 8 waves per SIMD (63 VGPRs): r04ab sweep 14.9 -> 13.5 ms
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

// One record per 64-pixel chunk, so a transpose wave finds its polygon's
// pixels with one load (round 3-4 waves binary-searched chunk_base: ten
// dependent loads before the first stack read).
struct ChunkRec {
  int64_t moff;   // mask_off[p]: the polygon's first compacted pixel
  int32_t n;      // count[p]
  int32_t cb;     // chunk_base[p]: the polygon's first chunk
};

__global__ __launch_bounds__(256) void decile_chunk_rec_kernel(const int32_t *__restrict__ count,
                                                               const int64_t *__restrict__ mask_off,
                                                               const int32_t *__restrict__ base,
                                                               ChunkRec *__restrict__ rec) {
  const int p = blockIdx.x;
  const int c0 = base[p], nc = base[p + 1] - c0;
  const int64_t mo = mask_off[p];
  const int n = count[p];
  for (int i = threadIdx.x; i < nc; i += 256) rec[c0 + i] = ChunkRec{mo, n, c0};
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
// npad + k] for its pixel k, seg0 = chunk_base[p] * 64 * n_chunk, npad =
// count[p] rounded up to 64 (rows start on 256-byte boundaries, so a chunk's
// store covers two whole lines: unaligned rows left partial lines that the
// L2s of two XCDs wrote back separately).  A load instruction
// reads the 32 bands (128 contiguous bytes) of two pixels, a store
// instruction writes one band of the 64 pixels (256 contiguous bytes); the
// wave's 64 x 32 tile (8.4 KB of LDS) keeps 16 waves per CU.
constexpr int kTrBands = 32;
__global__ __launch_bounds__(256) void decile_transpose_kernel(const float *__restrict__ stack, int t_stride,
                                                               const int32_t *__restrict__ idx,
                                                               const ChunkRec *__restrict__ rec,
                                                               const int32_t *__restrict__ chunk_base, int n_polys,
                                                               const int32_t *__restrict__ tsel, int n_chunk,
                                                               int n_groups, float *__restrict__ vals, float nodata,
                                                               uint4 *__restrict__ part) {
  constexpr int kPad = kTrBands + 1;
  __shared__ float tile[4][64 * kPad];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;
  const int ch = (int)(item / n_groups), g = (int)(item % n_groups);
  const int64_t n_ch = chunk_base[n_polys];
  if (item >= n_ch * n_groups) return;     // whole waves; no workgroup barrier below
  const ChunkRec r = rec[ch];
  const int n = r.n, k0 = (ch - r.cb) * kDecChunk;
  const int m = min(kDecChunk, n - k0);
  const int nb = min(kTrBands, n_chunk - g * kTrBands);   // bands of this group
  const int bl = lane & (kTrBands - 1), half = lane / kTrBands;
  // every lane loads from a valid address (band 0 of the group, pixel 0 of
  // the chunk) so the loads are unconditional and all in flight
  const float *base = stack + tsel[g * kTrBands + (bl < nb ? bl : 0)];
  const int32_t my_px = idx[r.moff + k0 + (lane < m ? lane : 0)];
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
    if (part) {   // the select's first pass, per (chunk, band): smallest / largest key, count of non-nodata values
      uint32_t pa = 0xFFFFFFFFu, po = 0u, pc = 0u;
#pragma unroll
      for (int u = 0; u < 32; u++) {
        const bool ok = 2 * u + half < m && v[u] != nodata;
        const uint32_t k = fkey(v[u]);
        if (ok) { pa = min(pa, k); po = max(po, k); pc++; }
      }
      pa = min(pa, (uint32_t)__shfl_xor(pa, 32));
      po = max(po, (uint32_t)__shfl_xor(po, 32));
      pc += (uint32_t)__shfl_xor(pc, 32);
      if (half == 0 && bl < nb) part[(int64_t)ch * n_chunk + g * kTrBands + bl] = make_uint4(pa, po, pc, 0u);
    }
  }
  wave_lds_sync();
  const int64_t npad = (int64_t)(n + kDecChunk - 1) / kDecChunk * kDecChunk;   // aligned band rows
  float *seg = vals + (int64_t)r.cb * kDecChunk * n_chunk + (int64_t)(g * kTrBands) * npad + k0;
  if (lane < m) {
    for (int j = 0; j < nb; j++) seg[(int64_t)j * npad + lane] = T[lane * kPad + j];   // lane = pixel
  }
}

// computeDeciles of one (polygon, band) segment; status 0, 1 (band total 0:
// zeros, Count 0 in the reference's TimeSeries) or GSKYHIP_E_RANGE (the
// reference indexes buf[len] and panics: len % (dc + 1) == 0 with step 1).
// Dynamic LDS: n_slots histograms of 256 bins, then cache_keys keys (the
// segment as it is, nodata included: no compaction, skipped on every pass).
template <int kU, int NT = kSelThreads, int WPE = 1>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void decile_select_kernel(const float *__restrict__ vals,
                                                                    const int32_t *__restrict__ chunk_base,
                                                                    const int32_t *__restrict__ count,
                                                                    const int32_t *__restrict__ totals, int n_chunk,
                                                                    int b0, int n_list, int dc, float nodata,
                                                                    int n_slots, int cache_keys, float *__restrict__ out,
                                                                    int32_t *__restrict__ status,
                                                                    const uint4 *__restrict__ part, int part_poly) {
  extern __shared__ uint32_t dyn[];
  uint32_t *cache = dyn + n_slots * 256;   // dyn[0, 2048): the buckets, then the candidates
  __shared__ uint32_t s_pref[kMaxRanks];   // rank r: its key, once resolved
  __shared__ uint32_t s_rem[kMaxRanks];    // rank r: its rank within its open range / bucket
  __shared__ int32_t s_rank[kMaxRanks];    // the distinct ranks, ascending
  __shared__ int32_t s_slot[kMaxRanks];    // rank r -> candidate slot (its bucket)
  __shared__ uint32_t s_spref[kMaxRanks];  // slot -> bucket (ascending)
  __shared__ uint32_t s_bcnt[kMaxRanks];   // rank r: the keys in that bucket
  __shared__ int32_t s_soff[kMaxRanks];    // slot -> first candidate
  __shared__ uint32_t s_fill[kMaxRanks];   // slot -> candidates written
  __shared__ int8_t s_map[kBins];          // bucket -> slot, -1 when no rank needs it
  __shared__ uint32_t red[3 * (NT / 64)];
  __shared__ uint32_t s_wsum[(NT / 64)];
  __shared__ int32_t s_nr, s_ns, s_nsl;
  __shared__ uint32_t s_lo[kMaxRanks], s_hi[kMaxRanks];   // rank r: its open key range
  __shared__ int32_t s_done[kMaxRanks], s_small_r[64];
  __shared__ float s_small[64];

  const int item = blockIdx.x;
  const int p = item / n_chunk, j = item % n_chunk;
  const int64_t o = (int64_t)p * n_list + b0 + j;
  float *dst = out + o * dc;
  const int tid = threadIdx.x;
  if (totals[o] <= 0) {   // drill.go:186-190
    for (int i = tid; i < dc; i += NT) dst[i] = 0.f;
    if (tid == 0) status[o] = 1;
    return;
  }
  const int n = count[p];
  const int64_t npad = (int64_t)(n + kDecChunk - 1) / kDecChunk * kDecChunk;
  const float *buf = vals + (int64_t)chunk_base[p] * kDecChunk * n_chunk + (int64_t)j * npad;
  auto ld = [&](int i) -> float { return buf[i]; };
  // pass 1: the non-nodata values (the reference's buf, drill.go:231-237):
  // their count, the bits all their keys share, and the segment's keys in
  // LDS while they fit (order is irrelevant to order statistics)
  const bool fits = n <= cache_keys;
  // with the transpose's per-chunk partials there is no first pass: the
  // first histogram pass streams the segment and fills the key cache
  bool filled = part == nullptr;
  // keys of the values `v != nodata` rejects (-0.0 == 0.0; a NaN nodata rejects nothing)
  const bool skip_on = nodata == nodata;
  const uint32_t kn1 = fkey(nodata), kn2 = nodata == 0.0f ? fkey(-nodata) : kn1;
  auto skipk = [&](uint32_t k) { return skip_on && (k == kn1 || k == kn2); };
  uint32_t ka = 0xFFFFFFFFu, ko = 0u;   // smallest / largest valid key
  int valid = 0;   // kU: values per thread in flight per round
  if (part && part_poly) {   // the fused mean pass's range and count of the whole segment
    if (tid == 0) {
      const uint4 q = part[o];
      ka = q.x; ko = q.y; valid = (int)q.z;
    }
  } else if (part) {         // the transpose's per-chunk partials
    const int cb = chunk_base[p], nc = (n + kDecChunk - 1) / kDecChunk;
    for (int i = tid; i < nc; i += NT) {
      const uint4 q = part[(int64_t)(cb + i) * n_chunk + j];
      ka = min(ka, q.x); ko = max(ko, q.y); valid += (int)q.z;
    }
  }
  for (int i0 = 0; i0 < (part ? 0 : n); i0 += NT * kU) {
    float v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = i0 + u * NT + tid;
      v[u] = i < n ? ld(i) : nodata;
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = i0 + u * NT + tid;
      const bool keep = i < n && v[u] != nodata;
      const uint32_t k = fkey(v[u]);
      if (keep) { ka = min(ka, k); ko = max(ko, k); valid++; }
      if (fits && i < n) cache[i] = k;
    }
  }
  for (int sh = 32; sh > 0; sh >>= 1) {
    ka = min(ka, (uint32_t)__shfl_xor(ka, sh));
    ko = max(ko, (uint32_t)__shfl_xor(ko, sh));
    valid += __shfl_xor(valid, sh);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6] = ka; red[(NT / 64) + (tid >> 6)] = ko; red[2 * (NT / 64) + (tid >> 6)] = (uint32_t)valid;
  }
  __syncthreads();
  uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;
  int len = 0;
#pragma unroll
  for (int w = 0; w < (NT / 64); w++) {
    kmn = min(kmn, red[w]); kmx = max(kmx, red[(NT / 64) + w]); len += (int)red[2 * (NT / 64) + w];
  }
  if (len <= 0) {   // total > 0 implies a non-nodata value; keep the slot defined anyway
    for (int i = tid; i < dc; i += NT) dst[i] = 0.f;
    if (tid == 0) status[o] = 0;
    return;
  }
  const int step = len / (dc + 1);
  if (step == 0) {   // len <= dc (<= 16): sort the few values, repeat them in order
    if (tid == 0) {
      int m = 0;
      if (fits && filled) {
        for (int i = 0; i < n && m < len; i++)
          if (!skipk(cache[i])) s_small[m++] = fdecode(cache[i]);
      } else {
        for (int i = 0; i < n && m < len; i++)
          if (ld(i) != nodata) s_small[m++] = ld(i);
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
    for (int i = tid; i < dc; i += NT) dst[i] = 0.f;
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
  // every valid key once, from the LDS copy or streamed from the segment
  auto for_keys = [&](auto &&f) {
    if (fits && filled) {
      for (int i = tid; i < n; i += NT) {
        const uint32_t k = cache[i];
        if (!skipk(k)) f(k);
      }
    } else {
      for (int i0 = 0; i0 < n; i0 += NT * kU) {
        float v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const int i = i0 + u * NT + tid;
          v[u] = i < n ? ld(i) : nodata;
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const int i = i0 + u * NT + tid;
          if (!filled && fits && i < n) cache[i] = fkey(v[u]);
          if (i < n && v[u] != nodata) f(fkey(v[u]));
        }
      }
    }
  };
  const int wv = tid >> 6, ln = tid & 63;
  // Range refinement: rank r is the s_rem[r]-th key in [s_lo[r], s_hi[r]].
  // A pass takes the ranks sharing the first open range [L, Hk], counts the
  // keys of the range in 2048 buckets of 2^sh consecutive keys from L (at
  // least 1024 of them used: the buckets follow the data, not a bit
  // prefix), and gives each rank its bucket; ranks whose bucket holds <= 64
  // keys are resolved by gathering those keys and a 64-lane counting select,
  // the others continue on their bucket's range (one more pass per 11 bits,
  // only under heavy ties or skew).
  if (tid < nr) { s_lo[tid] = kmn; s_hi[tid] = kmx; s_rem[tid] = (uint32_t)s_rank[tid]; s_done[tid] = 0; }
  __syncthreads();
  uint32_t *H = dyn;
  for (int guard = 0; guard < 4 * kMaxRanks; guard++) {
    if (tid == 0) {
      int f = -1;
      for (int r = 0; r < nr; r++)
        if (!s_done[r]) { f = r; break; }
      s_ns = f;
    }
    __syncthreads();
    const int f = s_ns;
    if (f < 0) break;
    const uint32_t L = s_lo[f], Hk = s_hi[f];
    const bool grp = tid < nr && !s_done[tid] && s_lo[tid] == L && s_hi[tid] == Hk;   // lane r of wave 0
    if (L == Hk) {   // one key value: every rank of the range is it
      if (grp) { s_pref[tid] = L; s_done[tid] = 1; }
      __syncthreads();
      continue;
    }
    const uint32_t span = Hk - L;                       // W - 1, W = keys in the range
    const int sh = max(0, 32 - __clz(span) - kBinsLog);  // bucket = (k - L) >> sh < 2048
    for (int i = tid; i < kBins; i += NT) { H[i] = 0u; s_map[i] = -1; }
    __syncthreads();
    for_keys([&](uint32_t k) {
      if (k >= L && k <= Hk) atomicAdd(&H[(k - L) >> sh], 1u);
    });
    __syncthreads();
    filled = true;
    {   // inclusive scan of the buckets in place, 4 per thread
      constexpr int BPT = kBins / NT;   // buckets per thread
      const int b4 = BPT * tid;
      uint32_t hb[BPT], sum = 0;
#pragma unroll
      for (int k = 0; k < BPT; k++) { hb[k] = H[b4 + k]; sum += hb[k]; }
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
      uint32_t run = ex;
#pragma unroll
      for (int k = 0; k < BPT; k++) { run += hb[k]; H[b4 + k] = run; }
    }
    __syncthreads();
    if (tid < 64) {   // wave 0, lane r of the group: its bucket, then the small
      // buckets (ascending with the ranks) -> slots and their candidate offsets
      const uint32_t r = grp ? s_rem[tid] : 0u;
      int lo = 0, hi = kBins - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (H[mid] > r) hi = mid; else lo = mid + 1;
      }
      const uint32_t before = lo ? H[lo - 1] : 0u;
      const uint32_t bcnt = H[lo] - before;
      const bool small = grp && bcnt <= (uint32_t)kCandMax;
      const uint64_t sm = __ballot(small);
      // consecutive small ranks of one bucket share its slot: a rank opens a
      // slot unless the previous small rank (same bucket) already did
      int last_small = -1;   // the nearest small rank below this lane
      {
        const uint64_t below = sm & ((1ull << tid) - 1ull);
        last_small = below ? 63 - __clzll(below) : -1;
      }
      const int last_b = __shfl(small ? lo : -1, last_small < 0 ? 0 : last_small);
      const bool nw = small && (last_small < 0 || last_b != lo);
      const uint64_t nb = __ballot(nw);
      const int slot = __popcll(nb & ((2ull << tid) - 1ull)) - 1;
      uint32_t incl = nw ? bcnt : 0u;   // candidate offsets: exclusive scan over the new slots
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t up = __shfl_up(incl, o);
        if (tid >= o) incl += up;
      }
      if (small) {
        s_rem[tid] = r - before;
        s_bcnt[tid] = bcnt;
        s_slot[tid] = slot;
      } else if (grp) {   // continue on the bucket's key range
        const uint32_t blo = L + ((uint32_t)lo << sh);
        const uint32_t bhi = (sh >= 32 || ((uint64_t)(lo + 1) << sh) - 1u >= (uint64_t)span)
                                 ? Hk : L + (uint32_t)(((uint64_t)(lo + 1) << sh) - 1u);
        s_lo[tid] = blo;
        s_hi[tid] = bhi;
        s_rem[tid] = r - before;
      }
      if (nw) {
        s_spref[slot] = (uint32_t)lo;
        s_soff[slot] = (int)(incl - bcnt);
      }
      if (tid == 0) s_nsl = __popcll(nb);
      s_small_r[tid] = small ? 1 : 0;
    }
    __syncthreads();
    const int nsl = s_nsl;
    if (nsl > 0) {
      if (tid < nsl) { s_map[s_spref[tid]] = (int8_t)tid; s_fill[tid] = 0u; }
      __syncthreads();
      uint32_t *cand = dyn;   // the bucket counts are no longer needed
      auto take = [&](uint32_t k) {
        if (k >= L && k <= Hk) {
          const int sl = s_map[(k - L) >> sh];
          if (sl >= 0) cand[s_soff[sl] + atomicAdd(&s_fill[sl], 1u)] = k;
        }
      };
      for_keys(take);
      __syncthreads();
      // rank r is the s_rem[r]-th key of its bucket (<= 64 keys, one per
      // lane): MSB-first selection with wave ballots over the bits where the
      // candidates differ -- lanes whose bit is 0 come first; equal keys end
      // in the same candidate set, any of them is the value
      for (int r = wv; r < nr; r += (NT / 64)) {
        if (!s_small_r[r]) continue;
        const int cnt = (int)s_bcnt[r];
        const uint32_t *c = cand + s_soff[s_slot[r]];
        const bool in = ln < cnt;
        const uint32_t ki = in ? c[ln] : 0u;
        uint32_t a = in ? ki : 0xFFFFFFFFu, o = in ? ki : 0u;
        for (int sft = 32; sft > 0; sft >>= 1) {
          a &= (uint32_t)__shfl_xor(a, sft);
          o |= (uint32_t)__shfl_xor(o, sft);
        }
        uint64_t live = __ballot(in);
        uint32_t rem = s_rem[r];
        for (int b = (a == o) ? -1 : 31 - __clz(a ^ o); b >= 0; b--) {
          const uint64_t zero = __ballot(((ki >> b) & 1u) == 0u) & live;
          const uint32_t nz = (uint32_t)__popcll(zero);
          if (rem < nz) live = zero;
          else { rem -= nz; live &= ~zero; }
        }
        const int src = __ffsll((unsigned long long)live) - 1;
        const uint32_t key = __shfl(ki, src);
        if (ln == 0) { s_pref[r] = key; s_done[r] = 1; }
      }
      __syncthreads();
    }
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
  ChunkRec *rec;
  uint4 *part;   // per (chunk, band of the pass): the transpose's key range and count
  float *vals;
  int64_t total;
};

DecWs decile_carve(void *base, int n_polys, int64_t mask_bytes, int chunk) {
  DecWs w;
  const int64_t cap = (mask_bytes + (int64_t)kDecChunk * n_polys) * chunk;   // rows padded to 64 values
  char *b = (char *)base;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { char *p = b ? b + o : nullptr; o += al256(bytes); return p; };
  w.idx = (int32_t *)take(mask_bytes * 4);
  w.count = (int32_t *)take((int64_t)n_polys * 4);
  w.chunk_base = (int32_t *)take((mask_bytes / kDecChunk + n_polys + 1) * 4);
  w.tsel = (int32_t *)take((int64_t)chunk * 4);
  w.rec = (ChunkRec *)take((mask_bytes / kDecChunk + n_polys) * (int64_t)sizeof(ChunkRec));
  w.part = (uint4 *)take((mask_bytes / kDecChunk + n_polys) * (int64_t)chunk * (int64_t)sizeof(uint4));
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
  hipLaunchKernelGGL(decile_chunk_rec_kernel, dim3(c.n_polys), dim3(256), 0, s, w.count, c.mask_off, w.chunk_base,
                     w.rec);
  const int64_t max_chunks = c.mask_bytes / kDecChunk + c.n_polys;   // >= sum of ceil(count / 64)
  const int n_slots = kHistSlots;
  const int cache_keys = (kSelLds - n_slots * 256 * 4) / 4;
  for (int b0 = 0; b0 < n_list; b0 += c.band_chunk) {
    const int n_chunk = std::min(c.band_chunk, n_list - b0);
    const int n_groups = (n_chunk + kTrBands - 1) / kTrBands;
    const int64_t n_seg = (int64_t)c.n_polys * n_chunk;
    if (hipMemcpyAsync(w.tsel, sel.data() + b0, sizeof(int32_t) * n_chunk, hipMemcpyHostToDevice, s) != hipSuccess)
      return GSKYHIP_E_HIP;
    const int64_t items = max_chunks * n_groups;
    hipLaunchKernelGGL(decile_transpose_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, c.stack,
                       c.t_stride, w.idx, w.rec, w.chunk_base, c.n_polys, w.tsel, n_chunk, n_groups,
                       w.vals, c.nodata, w.part);
    hipLaunchKernelGGL((decile_select_kernel<kSelU, kSelThreads, kSelWpe>), dim3((unsigned)n_seg), dim3(kSelThreads),
                       (size_t)kSelLds, s, w.vals, w.chunk_base, w.count, c.totals, n_chunk, b0, n_list,
                       c.decile_count, c.nodata, n_slots, cache_keys, c.out, c.status, (const uint4 *)w.part, 0);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

void launch_decile_chunk_scan(const int32_t *count, int n_polys, int32_t *chunk_base, hipStream_t s) {
  hipLaunchKernelGGL(decile_chunk_scan_kernel, dim3(1), dim3(1024), 0, s, count, n_polys, chunk_base);
}

int launch_decile_select_fused(const float *vals, const int32_t *chunk_base, const int32_t *count,
                               const int32_t *totals, int n_polys, int n_sel, int decile_count, float nodata,
                               const uint4 *stats, float *out, int32_t *status, hipStream_t s) {
  if (n_polys <= 0 || n_sel <= 0) return 0;
  if (decile_count < 1 || 2 * decile_count > kMaxRanks) return GSKYHIP_E_ARG;
  const int64_t n_seg = (int64_t)n_polys * n_sel;
  if (n_seg >= 2147483647LL) return GSKYHIP_E_ARG;
  const int n_slots = kHistSlots;
  const int cache_keys = (kSelLds - n_slots * 256 * 4) / 4;
  hipLaunchKernelGGL((decile_select_kernel<kSelU, kSelThreads, kSelWpe>), dim3((unsigned)n_seg), dim3(kSelThreads),
                     (size_t)kSelLds, s, vals, chunk_base, count, totals, n_sel, 0, n_sel, decile_count, nodata,
                     n_slots, cache_keys, out, status, stats, 1);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
