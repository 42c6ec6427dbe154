// quad_rate.hip -- the cost model of render_nn_kernel's single-entry C2 body
// (round 6), on a synthetic C2 of the same shape: 4096
// tiles of 512 x 512 RGBA from 16 int16 4000 x 4000 granules, source pixel
// 0.47 per output column under a 1-degree rotation (C2's Albers -> 3857
// convergence), 32.32 fixed-point row forms, nodata fold, LDS palette,
// non-temporal RGBA stores.  Variants of the lane layout:
//   col64   the product's: a lane's 8 pixels of a row 64 columns apart, one
//           16-bit gather per pixel (8 gathers / lane / row)
//   quad    a lane owns 2 runs of 4 adjacent columns; one UNALIGNED 8-byte
//           gather at the run's first source pixel serves the run wherever
//           the run stays on one source row within 4 pixels; lanes whose run
//           changes row take a second 8-byte gather (lane-masked), wider
//           spans 4 single gathers; one 16-B RGBA store per run
//   quad_b  quad with the second gather issued by every lane (no ballot)
//   quad4   quad with 4-B RGBA stores (the store shape of col64)
// Every variant writes the same image: the checksums must agree (this also
// checks that unaligned 8-byte buffer loads return the bytes at the address).
// Prints one JSON line: ms (best of reps), TB/s of algorithmic bytes, and
// gather / store instructions per 64 output pixels.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));    \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

constexpr int kG = 16, kB = 4000, kTiles = 4096, kW = 512, kRPW = 8;
constexpr int kItems = kTiles * (kW / (4 * kRPW));   // blocks of 4 waves x 8 rows x 512 columns
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

struct Map {   // per tile: source origin and the 32.32 steps per column / row
  int64_t x0, y0, dxc, dyc, dxr, dyr;
  int g, pad;
};

__device__ __forceinline__ uint32_t ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
}
__device__ __forceinline__ uint64_t ld64(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  const u2 v = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
  return ((uint64_t)v.y << 32) | v.x;
}

template <int P>
__global__ __launch_bounds__(256, 8) void c2(const int16_t *__restrict__ src, const Map *__restrict__ maps,
                                             const uint32_t *__restrict__ ramp, uint32_t *__restrict__ out) {
  __shared__ uint32_t tab[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  tab[tid] = ramp[tid];
  __syncthreads();
  const int item = blockIdx.x, t = item / (kW / (4 * kRPW));
  const int r0 = (item % (kW / (4 * kRPW))) * 4 * kRPW + wave * kRPW;
  const Map m = maps[t];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(src + (int64_t)m.g * kB * kB), (short)0, kB * kB * 2 + 8, 0x00020000);
  const int16_t nd = -999;
#pragma unroll 1
  for (int j = 0; j < kRPW; j++) {
    const int r = r0 + j;
    const uint64_t RX = (uint64_t)(m.x0 + (int64_t)r * m.dxr), RY = (uint64_t)(m.y0 + (int64_t)r * m.dyr);
    uint32_t *dst = out + ((int64_t)t * kW + r) * kW;
    if constexpr (P == 0) {
      uint32_t off[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int col = lane + 64 * q;
        const uint64_t X = RX + (uint64_t)col * (uint64_t)m.dxc, Y = RY + (uint64_t)col * (uint64_t)m.dyc;
        off[q] = (__umul24((uint32_t)(Y >> 32), (uint32_t)kB) + (uint32_t)(X >> 32)) * 2u;
      }
      int16_t v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = (int16_t)ld16(rs, off[q]);
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int16_t c = v[q] != nd ? v[q] : nd;
        __builtin_nontemporal_store(tab[(uint32_t)c & 0xFFu], dst + lane + 64 * q);
      }
    } else {
      int16_t v[8];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int col = 4 * lane + 256 * h;
        uint32_t ix[4], iy[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint64_t X = RX + (uint64_t)(col + k) * (uint64_t)m.dxc, Y = RY + (uint64_t)(col + k) * (uint64_t)m.dyc;
          ix[k] = (uint32_t)(X >> 32);
          iy[k] = (uint32_t)(Y >> 32);
        }
        const uint32_t lo = min(ix[0], ix[3]), span = max(ix[0], ix[3]) - lo;
        const uint64_t a = ld64(rs, (__umul24(iy[0], (uint32_t)kB) + lo) * 2u);
        uint64_t b = a;
        const bool two = iy[3] != iy[0];
        if constexpr (P == 2) {
          b = ld64(rs, (__umul24(iy[3], (uint32_t)kB) + lo) * 2u);
        } else {
          if (__builtin_amdgcn_ballot_w64(two) != 0) {
            if (two) b = ld64(rs, (__umul24(iy[3], (uint32_t)kB) + lo) * 2u);
          }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint64_t w = iy[k] == iy[0] ? a : b;
          v[4 * h + k] = (int16_t)(uint16_t)(w >> ((ix[k] - lo) * 16u));
        }
        // spans past 4 pixels or rows 2 apart (not on this map): single gathers
        if (__builtin_amdgcn_ballot_w64(span > 3u || iy[3] - iy[0] > 1u) != 0) {
          if (span > 3u || iy[3] - iy[0] > 1u) {
#pragma unroll
            for (int k = 0; k < 4; k++) v[4 * h + k] = (int16_t)ld16(rs, (__umul24(iy[k], (uint32_t)kB) + ix[k]) * 2u);
          }
        }
      }
      uint32_t px[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int16_t c = v[q] != nd ? v[q] : nd;
        px[q] = tab[(uint32_t)c & 0xFFu];
      }
      if constexpr (P == 3) {
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int k = 0; k < 4; k++) __builtin_nontemporal_store(px[4 * h + k], dst + 4 * lane + 256 * h + k);
      } else {
        __builtin_nontemporal_store(u4{px[0], px[1], px[2], px[3]}, (u4 *)(dst + 4 * lane));
        __builtin_nontemporal_store(u4{px[4], px[5], px[6], px[7]}, (u4 *)(dst + 4 * lane + 256));
      }
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
    s[i] = (int16_t)((h >> 8) % 251) - ((h & 0xF000) == 0 ? 1000 : 0);   // some -999 .. nodata-ish values
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  const int64_t nsrc = (int64_t)kG * kB * kB;
  int16_t *src;
  CHECK(hipMalloc(&src, nsrc * 2 + 64));
  hipLaunchKernelGGL(fill_src, dim3(4096), dim3(256), 0, 0, src, nsrc);
  uint32_t *out, *ramp;
  const int64_t nout = (int64_t)kTiles * kW * kW;
  CHECK(hipMalloc(&out, nout * 4));
  CHECK(hipMalloc(&ramp, 1024));
  uint32_t hr[256];
  for (int i = 0; i < 256; i++) hr[i] = 0xFF000000u | (uint32_t)i * 0x10307u;
  CHECK(hipMemcpy(ramp, hr, 1024, hipMemcpyHostToDevice));
  Map *hm = (Map *)malloc(sizeof(Map) * kTiles);
  const double sc = 0.47, ang = 1.0 * M_PI / 180.0, two32 = 4294967296.0;
  for (int t = 0; t < kTiles; t++) {
    const int g = t % kG, k = t / kG;   // 256 tiles per granule on a 16 x 16 grid
    const double ox = 60.0 + (k % 16) * 230.0 + 0.123, oy = 60.0 + (k / 16) * 230.0 + 0.377;
    hm[t].x0 = (int64_t)(ox * two32);
    hm[t].y0 = (int64_t)(oy * two32);
    hm[t].dxc = (int64_t)(sc * std::cos(ang) * two32);
    hm[t].dyc = (int64_t)(sc * std::sin(ang) * two32);
    hm[t].dxr = (int64_t)(-sc * std::sin(ang) * two32);
    hm[t].dyr = (int64_t)(sc * std::cos(ang) * two32);
    hm[t].g = g;
  }
  Map *maps;
  CHECK(hipMalloc(&maps, sizeof(Map) * kTiles));
  CHECK(hipMemcpy(maps, hm, sizeof(Map) * kTiles, hipMemcpyHostToDevice));
  unsigned long long *acc;
  CHECK(hipMalloc(&acc, 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char *names[] = {"col64", "quad", "quad_b", "quad4"};
  const double bytes = nout * 4.0 + nsrc * 2.0;
  std::printf("{\"bytes\": %.0f, \"results\": {", bytes);
  for (int p = 0; p < 4; p++) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; r++) {
      CHECK(hipMemset(out, 0, 4096));
      CHECK(hipEventRecord(e0));
      switch (p) {
        case 0: hipLaunchKernelGGL(c2<0>, dim3(kItems), dim3(256), 0, 0, src, maps, ramp, out); break;
        case 1: hipLaunchKernelGGL(c2<1>, dim3(kItems), dim3(256), 0, 0, src, maps, ramp, out); break;
        case 2: hipLaunchKernelGGL(c2<2>, dim3(kItems), dim3(256), 0, 0, src, maps, ramp, out); break;
        default: hipLaunchKernelGGL(c2<3>, dim3(kItems), dim3(256), 0, 0, src, maps, ramp, out); break;
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
    std::printf("%s\"%s\": {\"ms\": %.4f, \"tbps\": %.3f, \"checksum\": \"%016llx\"}", p ? ", " : "", names[p], best,
                bytes / (best * 1e-3) / 1e12, h);
  }
  std::printf("}}\n");
  return 0;
}
