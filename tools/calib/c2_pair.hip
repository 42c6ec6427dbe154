// c2_pair.hip -- lane layouts for C2's single-entry gather + store at the
// real C2 rotation (round 6).  C2's Albers (EPSG:3577, lon0 132 E, standard
// parallels -18 / -36) granules sit at 147-152 E, where the grid convergence
// against EPSG:3857 is n (lon - lon0) ~ -0.45 x 17 deg ~ -8 deg: a 64-column
// gather slot spans ~30 source pixels across and ~4 source rows, and a quad
// of 4 lanes (4 columns, 1.9 source px) changes source row ~26 % of the time.
// Same synthetic C2 as c2_model.hip (4096 tiles x 512^2 RGBA, 16 int16
// 4000^2 granules, 0.47 px per column, block 4 waves x 8 rows x 512 columns),
// the rotation an argument.  Variants:
//   col64     the product's layout: lane pixels 64 columns apart, 16-bit gathers
//   pair_u4   lane owns column pairs (2 l + 128 h, + 1): one UNALIGNED 4-byte
//             gather at the pair's first source pixel serves both wherever
//             they share the source row and are <= 1 px apart; the other
//             lanes take a 16-bit gather for the second pixel (lane-masked,
//             issued when any lane needs it); 8-byte RGBA stores
//   pair_a4   lane owns column pairs with an ALIGNED dword gather (round 5's
//             lost variant): second gather where the pair straddles a dword
//   pair_u4s  pair_u4 with 4-byte stores (the store shape of col64)
// All variants write the same image (checksums agree).  One JSON line.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));    \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

constexpr int kG = 16, kB = 4000, kTiles = 4096, kW = 512, kRPW = 8;
constexpr int kBlkPerTile = kW / (4 * kRPW);
constexpr int kItems = kTiles * kBlkPerTile;
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

struct RowFix { int64_t x0, y0, dx, dy; };

// Slot-major variants: for each 64-column slot the wave's 8 rows back to back
// (the source footprint of one slot over 8 rows: ~31 px x ~8 rows at 7.6 deg).
//   P 4  colg    16-bit gathers per (row, slot)
//   P 5  boxlds  the slot's source box copied into a wave-private LDS window
//                by coalesced dword loads (16 dwords = 32 px per box row, 4
//                rows per load instruction), each pixel read with ds_read_u16
template <int P>
__device__ __forceinline__ void slot_major(const int16_t *src, __amdgpu_buffer_rsrc_t rs, const RowFix *fb, int r0,
                                           int lane, uint32_t *box, const uint32_t *tab, uint32_t *out_t) {
  const int16_t nd = -999;
  int64_t x0[kRPW], y0[kRPW];
  const int64_t dx = fb[r0].dx, dy = fb[r0].dy;
#pragma unroll
  for (int j = 0; j < kRPW; j++) { x0[j] = fb[r0 + j].x0; y0[j] = fb[r0 + j].y0; }
#pragma unroll 1
  for (int q = 0; q < 8; q++) {
    const int c = 64 * q + lane;
    uint32_t ix[kRPW], iy[kRPW];
#pragma unroll
    for (int j = 0; j < kRPW; j++) {
      ix[j] = (uint32_t)((uint64_t)(x0[j] + (int64_t)c * dx) >> 32);
      iy[j] = (uint32_t)((uint64_t)(y0[j] + (int64_t)c * dy) >> 32);
    }
    int16_t v[kRPW];
    bool done = false;
    if constexpr (P == 6) {   // 32-dword (64 px) box rows, 2 rows per load instruction, up to 12 rows
      const uint32_t a0 = __builtin_amdgcn_readlane(ix[0], 0), a1 = __builtin_amdgcn_readlane(ix[0], 63);
      const uint32_t a2 = __builtin_amdgcn_readlane(ix[kRPW - 1], 0), a3 = __builtin_amdgcn_readlane(ix[kRPW - 1], 63);
      const uint32_t b0 = __builtin_amdgcn_readlane(iy[0], 0), b1 = __builtin_amdgcn_readlane(iy[0], 63);
      const uint32_t b2 = __builtin_amdgcn_readlane(iy[kRPW - 1], 0), b3 = __builtin_amdgcn_readlane(iy[kRPW - 1], 63);
      const uint32_t bx0 = min(min(a0, a1), min(a2, a3)) & ~1u, bx1 = max(max(a0, a1), max(a2, a3));
      const uint32_t by0 = min(min(b0, b1), min(b2, b3)), by1 = max(max(b0, b1), max(b2, b3));
      const uint32_t h = by1 - by0 + 1;
      if (bx1 - bx0 < 64u && h <= 12u) {
        const uint32_t lr = (uint32_t)lane >> 5, ld = (uint32_t)lane & 31u;
        uint32_t w[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
          const uint32_t row = by0 + 2 * i + lr;
          w[i] = 0;
          if (2u * i < h) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (row * (uint32_t)kB + bx0) * 2u + ld * 4u, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 6; i++)
          if (2u * i < h) box[(2 * i + lr) * 32 + ld] = w[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint16_t *b16 = (const uint16_t *)box;
#pragma unroll
        for (int j = 0; j < kRPW; j++) v[j] = (int16_t)b16[(iy[j] - by0) * 64u + (ix[j] - bx0)];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        done = true;
      }
    }
    if constexpr (P == 5) {
      // the box: extremes at lanes 0 / 63 of rows 0 / 7 (linear in the column and the row)
      const uint32_t a0 = __builtin_amdgcn_readlane(ix[0], 0), a1 = __builtin_amdgcn_readlane(ix[0], 63);
      const uint32_t a2 = __builtin_amdgcn_readlane(ix[kRPW - 1], 0), a3 = __builtin_amdgcn_readlane(ix[kRPW - 1], 63);
      const uint32_t b0 = __builtin_amdgcn_readlane(iy[0], 0), b1 = __builtin_amdgcn_readlane(iy[0], 63);
      const uint32_t b2 = __builtin_amdgcn_readlane(iy[kRPW - 1], 0), b3 = __builtin_amdgcn_readlane(iy[kRPW - 1], 63);
      const uint32_t bx0 = min(min(a0, a1), min(a2, a3)) & ~1u, bx1 = max(max(a0, a1), max(a2, a3));
      const uint32_t by0 = min(min(b0, b1), min(b2, b3)), by1 = max(max(b0, b1), max(b2, b3));
      const uint32_t h = by1 - by0 + 1;
      if (bx1 - bx0 < 32u && h <= 16u) {
        const uint32_t lr = (uint32_t)lane >> 4, ld = (uint32_t)lane & 15u;
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t row = by0 + 4 * i + lr;
          w[i] = 0;
          if (4u * i < h) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (row * (uint32_t)kB + bx0) * 2u + ld * 4u, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (4u * i < h) box[(4 * i + lr) * 16 + ld] = w[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint16_t *b16 = (const uint16_t *)box;
#pragma unroll
        for (int j = 0; j < kRPW; j++) v[j] = (int16_t)b16[(iy[j] - by0) * 32u + (ix[j] - bx0)];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        done = true;
      }
    }
    if (!done) {
#pragma unroll
      for (int j = 0; j < kRPW; j++)
        v[j] = (int16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (__umul24(iy[j], (uint32_t)kB) + ix[j]) * 2u, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kRPW; j++) {
      const int16_t cc = v[j] != nd ? v[j] : nd;
      __builtin_nontemporal_store(tab[(uint32_t)cc & 0xFFu], out_t + (int64_t)(r0 + j) * kW + c);
    }
  }
}

// Pipelined slot-major variants: the loads of slot q + 1 are issued before
// the RGBA stores of slot q, so waiting for slot q + 1's data does not wait
// for slot q's stores (gfx9 counts loads and stores in one in-order vmcnt).
//   P 7  boxpipe   box of 32-dword (64 px) rows, 2 rows per load, <= 12 rows
//   P 8  colgpipe  16-bit gathers per (row, slot)
template <int P>
__device__ __forceinline__ void slot_pipe(__amdgpu_buffer_rsrc_t rs, const RowFix *fb, int r0, int lane,
                                          uint32_t *box, const uint32_t *tab, uint32_t *out_t) {
  const int16_t nd = -999;
  int64_t x0[kRPW], y0[kRPW];
  const int64_t dx = fb[r0].dx, dy = fb[r0].dy;
#pragma unroll
  for (int j = 0; j < kRPW; j++) { x0[j] = fb[r0 + j].x0; y0[j] = fb[r0 + j].y0; }
  auto coords = [&](int q, uint32_t (&ix)[kRPW], uint32_t (&iy)[kRPW]) {
    const int c = 64 * q + lane;
#pragma unroll
    for (int j = 0; j < kRPW; j++) {
      ix[j] = (uint32_t)((uint64_t)(x0[j] + (int64_t)c * dx) >> 32);
      iy[j] = (uint32_t)((uint64_t)(y0[j] + (int64_t)c * dy) >> 32);
    }
  };
  // box of slot q from the scalar row forms: corners (rows 0 / 7, columns 64 q / 64 q + 63)
  auto box_of = [&](int q, uint32_t &bx0, uint32_t &by0) {
    const int64_t ca = 64 * q, cb = 64 * q + 63;
    const uint32_t a0 = (uint32_t)((uint64_t)(x0[0] + ca * dx) >> 32), a1 = (uint32_t)((uint64_t)(x0[0] + cb * dx) >> 32);
    const uint32_t a2 = (uint32_t)((uint64_t)(x0[kRPW - 1] + ca * dx) >> 32), a3 = (uint32_t)((uint64_t)(x0[kRPW - 1] + cb * dx) >> 32);
    const uint32_t b0 = (uint32_t)((uint64_t)(y0[0] + ca * dy) >> 32), b1 = (uint32_t)((uint64_t)(y0[0] + cb * dy) >> 32);
    const uint32_t b2 = (uint32_t)((uint64_t)(y0[kRPW - 1] + ca * dy) >> 32), b3 = (uint32_t)((uint64_t)(y0[kRPW - 1] + cb * dy) >> 32);
    bx0 = min(min(a0, a1), min(a2, a3)) & ~1u;
    by0 = min(min(b0, b1), min(b2, b3));
  };
  const uint32_t lr = (uint32_t)lane >> 5, ld = (uint32_t)lane & 31u;
  uint32_t wn[6];
  int16_t vn[kRPW];
  uint32_t bxn = 0, byn = 0;
  auto issue = [&](int q) {
    if constexpr (P == 7) {
      box_of(q, bxn, byn);
#pragma unroll
      for (int i = 0; i < 5; i++)
        wn[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, ((byn + 2 * i + lr) * (uint32_t)kB + bxn) * 2u + ld * 4u, 0, 0);
    } else {
      uint32_t ix[kRPW], iy[kRPW];
      coords(q, ix, iy);
#pragma unroll
      for (int j = 0; j < kRPW; j++)
        vn[j] = (int16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (__umul24(iy[j], (uint32_t)kB) + ix[j]) * 2u, 0, 0);
    }
  };
  issue(0);
#pragma unroll 1
  for (int q = 0; q < 8; q++) {
    int16_t v[kRPW];
    uint32_t w[6], bx0 = bxn, by0 = byn;
    if constexpr (P == 7) {
#pragma unroll
      for (int i = 0; i < 5; i++) w[i] = wn[i];
    } else {
#pragma unroll
      for (int j = 0; j < kRPW; j++) v[j] = vn[j];
    }
    if (q + 1 < 8) issue(q + 1);
    if constexpr (P == 7) {
#pragma unroll
      for (int i = 0; i < 5; i++) box[(2 * i + lr) * 32 + ld] = w[i];
      asm volatile("" ::: "memory");
      uint32_t ix[kRPW], iy[kRPW];
      coords(q, ix, iy);
      const uint16_t *b16 = (const uint16_t *)box;
#pragma unroll
      for (int j = 0; j < kRPW; j++) v[j] = (int16_t)b16[(iy[j] - by0) * 64u + (ix[j] - bx0)];
      asm volatile("" ::: "memory");
    }
    const int c = 64 * q + lane;
#pragma unroll
    for (int j = 0; j < kRPW; j++) {
      const int16_t cc = v[j] != nd ? v[j] : nd;
      __builtin_nontemporal_store(tab[(uint32_t)cc & 0xFFu], out_t + (int64_t)(r0 + j) * kW + c);
    }
  }
}

template <int P>
__global__ __launch_bounds__(256, 8) void c2(const int16_t *__restrict__ src, const RowFix *__restrict__ fix,
                                             const int *__restrict__ gran, const uint32_t *__restrict__ ramp,
                                             uint32_t *__restrict__ out) {
  __shared__ uint32_t tab[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int item = blockIdx.x, t = item / kBlkPerTile;
  tab[tid] = tid != 255 ? ramp[tid] : 0u;
  __syncthreads();
  const int r0 = (item % kBlkPerTile) * 4 * kRPW + wave * kRPW;
  const int g = gran[t];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(src + (int64_t)g * kB * kB), (short)0, kB * kB * 2, 0x00020000);
  const int16_t nd = -999;
  const RowFix *fb = fix + (int64_t)t * kW;
  if constexpr (P >= 7) {
    __shared__ uint32_t s_boxp[4][12 * 32];
    slot_pipe<P>(rs, fb, r0, lane, s_boxp[wave], tab, out + (int64_t)t * kW * kW);
    return;
  }
  if constexpr (P >= 4) {
    __shared__ uint32_t s_box[4][12 * 32];
    slot_major<P>(src, rs, fb, r0, lane, s_box[wave], tab, out + (int64_t)t * kW * kW);
    return;
  }
#pragma unroll 1
  for (int j = 0; j < kRPW; j++) {
    const int r = r0 + j;
    const RowFix *p = fb + r;
    const int64_t f0 = p->x0, f1 = p->y0, f2 = p->dx, f3 = p->dy;
    uint32_t *dst = out + ((int64_t)t * kW + r) * kW;
    int16_t v[8];
    if constexpr (P == 0) {
      uint64_t X = (uint64_t)(f0 + (int64_t)lane * f2), Y = (uint64_t)(f1 + (int64_t)lane * f3);
      const uint64_t SX = (uint64_t)f2 << 6, SY = (uint64_t)f3 << 6;
      uint32_t offs[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        offs[q] = (__umul24((uint32_t)(Y >> 32), (uint32_t)kB) + (uint32_t)(X >> 32)) * 2u;
        X += SX;
        Y += SY;
      }
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = (int16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, offs[q], 0, 0);
    } else {
      // pairs: columns 2 lane + 128 h + {0, 1} -> v[2 h], v[2 h + 1]
      uint64_t X = (uint64_t)(f0 + (int64_t)(2 * lane) * f2), Y = (uint64_t)(f1 + (int64_t)(2 * lane) * f3);
      const uint64_t SX = (uint64_t)f2 << 7, SY = (uint64_t)f3 << 7;
      uint32_t e0[4], e1[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const uint64_t X1 = X + (uint64_t)f2, Y1 = Y + (uint64_t)f3;
        e0[h] = __umul24((uint32_t)(Y >> 32), (uint32_t)kB) + (uint32_t)(X >> 32);
        e1[h] = __umul24((uint32_t)(Y1 >> 32), (uint32_t)kB) + (uint32_t)(X1 >> 32);
        X += SX;
        Y += SY;
      }
      uint32_t w[4];
      bool two[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        if constexpr (P == 2) {   // aligned dword holding e0
          w[h] = __builtin_amdgcn_raw_buffer_load_b32(rs, (e0[h] * 2u) & ~3u, 0, 0);
          two[h] = (e1[h] >> 1) != (e0[h] >> 1);
        } else {                  // unaligned dword starting at e0
          w[h] = __builtin_amdgcn_raw_buffer_load_b32(rs, e0[h] * 2u, 0, 0);
          two[h] = e1[h] - e0[h] > 1u;
        }
      }
      uint32_t s1[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        s1[h] = 0;
        if (__builtin_amdgcn_ballot_w64(two[h]) != 0) {
          if (two[h]) s1[h] = __builtin_amdgcn_raw_buffer_load_b16(rs, e1[h] * 2u, 0, 0);
        }
      }
#pragma unroll
      for (int h = 0; h < 4; h++) {
        if constexpr (P == 2) {
          v[2 * h] = (int16_t)(uint16_t)(w[h] >> ((e0[h] & 1u) * 16u));
          v[2 * h + 1] = two[h] ? (int16_t)(uint16_t)s1[h] : (int16_t)(uint16_t)(w[h] >> ((e1[h] & 1u) * 16u));
        } else {
          v[2 * h] = (int16_t)(uint16_t)w[h];
          v[2 * h + 1] = two[h] ? (int16_t)(uint16_t)s1[h] : (int16_t)(uint16_t)(w[h] >> ((e1[h] - e0[h]) * 16u));
        }
      }
    }
    uint32_t px[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int16_t c = v[q] != nd ? v[q] : nd;
      px[q] = tab[(uint32_t)c & 0xFFu];
    }
    if constexpr (P == 0) {
#pragma unroll
      for (int q = 0; q < 8; q++) __builtin_nontemporal_store(px[q], dst + lane + 64 * q);
    } else if constexpr (P == 3) {
#pragma unroll
      for (int h = 0; h < 4; h++) {
        __builtin_nontemporal_store(px[2 * h], dst + 2 * lane + 128 * h);
        __builtin_nontemporal_store(px[2 * h + 1], dst + 2 * lane + 128 * h + 1);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 4; h++) __builtin_nontemporal_store(u2{px[2 * h], px[2 * h + 1]}, (u2 *)(dst + 2 * lane + 128 * h));
    }
  }
}

__global__ void checksum(const uint32_t *__restrict__ out, int64_t n, unsigned long long *acc) {
  uint64_t s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += (uint64_t)out[i] * (uint64_t)((i & 1023) + 1);
  atomicAdd(acc, (unsigned long long)s);
}

__global__ void fill_src(int16_t *s, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    s[i] = (int16_t)((h >> 8) % 10000);
    if (((i % kB) / 64 + (i / kB) / 64) % 10 == 3) s[i] = -999;
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  const double deg = argc > 2 ? std::atof(argv[2]) : -8.0;
  const int64_t nsrc = (int64_t)kG * kB * kB, nout = (int64_t)kTiles * kW * kW;
  int16_t *src;
  CHECK(hipMalloc(&src, nsrc * 2 + 64));
  hipLaunchKernelGGL(fill_src, dim3(4096), dim3(256), 0, 0, src, nsrc);
  uint32_t *out, *ramp;
  CHECK(hipMalloc(&out, nout * 4));
  CHECK(hipMalloc(&ramp, 1024));
  uint32_t hr[256];
  for (int i = 0; i < 256; i++) hr[i] = 0xFF000000u | (uint32_t)i * 0x10307u;
  CHECK(hipMemcpy(ramp, hr, 1024, hipMemcpyHostToDevice));
  const double sc = 0.47, ang = deg * M_PI / 180.0, two32 = 4294967296.0;
  RowFix *hf = (RowFix *)malloc(sizeof(RowFix) * kTiles * kW);
  int *hg = (int *)malloc(sizeof(int) * kTiles);
  for (int t = 0; t < kTiles; t++) {   // the real C2 layout: 64 x 64 tiles over 4 x 4 granules
    const int tx = t % 64, ty = t / 64;
    hg[t] = (ty / 16) * 4 + tx / 16;
    const double ox = 400.0 + (tx % 16) * 200.0 + 0.123, oy = 400.0 + (ty % 16) * 200.0 + 0.377;
    for (int r = 0; r < kW; r++) {
      const double x0 = ox - sc * std::sin(ang) * r, y0 = oy + sc * std::cos(ang) * r;
      RowFix &f = hf[(int64_t)t * kW + r];
      f.x0 = (int64_t)(x0 * two32);
      f.y0 = (int64_t)(y0 * two32);
      f.dx = (int64_t)(sc * std::cos(ang) * two32);
      f.dy = (int64_t)(sc * std::sin(ang) * two32);
    }
  }
  RowFix *fix;
  int *gran;
  CHECK(hipMalloc(&fix, sizeof(RowFix) * kTiles * kW));
  CHECK(hipMemcpy(fix, hf, sizeof(RowFix) * kTiles * kW, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&gran, sizeof(int) * kTiles));
  CHECK(hipMemcpy(gran, hg, sizeof(int) * kTiles, hipMemcpyHostToDevice));
  unsigned long long *acc;
  CHECK(hipMalloc(&acc, 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char *names[] = {"col64", "pair_u4", "pair_a4", "pair_u4s", "colg", "boxlds", "boxlds64", "boxpipe", "colgpipe"};
  std::printf("{\"deg\": %.2f, \"results\": {", deg);
  for (int p = 0; p < 9; p++) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; r++) {
      CHECK(hipEventRecord(e0));
      switch (p) {
        case 0: hipLaunchKernelGGL(c2<0>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 1: hipLaunchKernelGGL(c2<1>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 2: hipLaunchKernelGGL(c2<2>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 3: hipLaunchKernelGGL(c2<3>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 4: hipLaunchKernelGGL(c2<4>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 5: hipLaunchKernelGGL(c2<5>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 6: hipLaunchKernelGGL(c2<6>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        case 7: hipLaunchKernelGGL(c2<7>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
        default: hipLaunchKernelGGL(c2<8>, dim3(kItems), dim3(256), 0, 0, src, fix, gran, ramp, out); break;
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    CHECK(hipMemset(acc, 0, 8));
    hipLaunchKernelGGL(checksum, dim3(4096), dim3(256), 0, 0, out, nout, acc);
    unsigned long long h;
    CHECK(hipMemcpy(&h, acc, 8, hipMemcpyDeviceToHost));
    CHECK(hipMemset(out, 0, nout * 4));
    std::printf("%s\"%s\": {\"ms\": %.4f, \"checksum\": \"%016llx\"}", p ? ", " : "", names[p], best, h);
  }
  std::printf("}}\n");
  return 0;
}
