// c2_model.hip -- what separates render_nn_kernel's single-entry C2 body
// from a bare gather + store kernel of the same shape (round 6, VERDICT r05
// item 2).  A synthetic C2: 4096 tiles of 512 x 512 RGBA from 16 int16
// 4000 x 4000 granules, 0.47 source px per output column under a 1-degree
// rotation, lane layout of the product (8 pixels of a row 64 columns apart,
// one 16-bit gather each, non-temporal 4-B RGBA stores), block = 4 waves x 8
// rows x 512 columns.  Each bit adds one piece of the product's body:
//   1  MARGIN  per-pixel fraction margin test + wave ballot (nn_fix_row)
//   2  ROWFIX  the row forms from a RowFix array in HBM (one vector load of
//              the wave's 8 records, v_readlane per row) instead of computed
//   4  SCALE   utils.Scale of int16 (offset wrap, clamp, float multiply,
//              Go uint8 conversion, nodata -> 0xFF) before the palette read
//   8  GRID    the real C2 geometry: a 64 x 64 tile grid over a 4 x 4 granule
//              grid (neighbouring tiles read neighbouring source footprints),
//              instead of consecutive tiles on different granules
//   16 PLAN    per-block tile plan loads (scalar) + the empty-tile test
// Prints one JSON line: ms (best of reps) per variant.
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
constexpr uint32_t kFixMargin = 1u << 13;

struct RowFix { int64_t x0, y0, dx, dy; };
struct Plan { int complex, n_entries, vt, e0; double nodata; int dtype, created; };

template <int F>
__global__ __launch_bounds__(256, 8) void c2(const int16_t *__restrict__ src, const RowFix *__restrict__ fix,
                                             const int *__restrict__ gran, const Plan *__restrict__ plans,
                                             const uint32_t *__restrict__ ramp, uint32_t *__restrict__ out,
                                             unsigned *__restrict__ amb_count, float scf, int off, int clip) {
  __shared__ uint32_t tab[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = blockIdx.x, t = item / kBlkPerTile;
  int16_t cnod = -999;
  if constexpr ((F & 16) != 0) {
    const Plan *p = plans + t;
    const int cx = p->complex, ne = p->n_entries, vt = p->vt;
    const double nd = p->nodata;
    asm volatile("" ::"s"(cx), "s"(ne), "s"(vt));
    if ((cx != 0) | ((ne > 0) & (vt != 3))) return;
    cnod = (int16_t)nd;
  }
  tab[tid] = tid != 255 ? ramp[tid] : 0u;
  __syncthreads();
  const int r0 = (item % kBlkPerTile) * 4 * kRPW + wave * kRPW;
  const int g = gran[t];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(src + (int64_t)g * kB * kB), (short)0, kB * kB * 2, 0x00020000);
  const int16_t nd = -999;
  const RowFix *fb = fix + (int64_t)t * kW;
  int64_t fv = 0;
  if constexpr ((F & 2) != 0) {
    if (lane < 4 * kRPW) fv = __builtin_nontemporal_load((const int64_t *)(fb + r0 + (lane >> 2)) + (lane & 3));
  }
  unsigned amb = 0;
#pragma unroll 1
  for (int j = 0; j < kRPW; j++) {
    const int r = r0 + j;
    int64_t f[4];
    if constexpr ((F & 2) != 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)fv, 4 * j + k);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)fv >> 32), 4 * j + k);
        f[k] = (int64_t)(((uint64_t)hi << 32) | lo);
      }
    } else {
      const RowFix *p = fb + r;   // uniform: scalar loads
      f[0] = p->x0; f[1] = p->y0; f[2] = p->dx; f[3] = p->dy;
    }
    uint64_t X = (uint64_t)(f[0] + (int64_t)lane * f[2]), Y = (uint64_t)(f[1] + (int64_t)lane * f[3]);
    const uint64_t SX = (uint64_t)f[2] << 6, SY = (uint64_t)f[3] << 6;
    uint32_t offs[8];
    uint32_t amin = 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      offs[q] = (__umul24((uint32_t)(Y >> 32), (uint32_t)kB) + (uint32_t)(X >> 32)) * 2u;
      if constexpr ((F & 1) != 0) {
        amin = min(amin, min((uint32_t)X + kFixMargin, (uint32_t)Y + kFixMargin));
        asm volatile("" : "+v"(offs[q]));
      }
      X += SX;
      Y += SY;
    }
    if constexpr ((F & 1) != 0) {
      if (__builtin_amdgcn_ballot_w64(amin < 2u * kFixMargin) != 0) { amb++; }   // the product redoes this row in fp64
    }
    int16_t v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = (int16_t)__builtin_amdgcn_raw_buffer_load_b16(rs, offs[q], 0, 0);
    uint32_t *dst = out + ((int64_t)t * kW + r) * kW;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int16_t c = v[q] != nd ? v[q] : cnod;
      uint32_t b;
      if constexpr ((F & 4) != 0) {
        int32_t value = (int16_t)(c + off);
        value = max(min(value, clip), 0);
        const float fl = (float)value * scf;
        b = c == nd ? 0xFFu : ((uint32_t)(int32_t)fl & 0xFFu);
      } else {
        b = (uint32_t)c & 0xFFu;
      }
      __builtin_nontemporal_store(tab[b], dst + lane + 64 * q);
    }
  }
  if ((F & 1) != 0 && lane == 0 && amb) atomicAdd(amb_count, amb);
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
    if (((i % kB) / 64 + (i / kB) / 64) % 10 == 3) s[i] = -999;   // nodata blocks
  }
}

template <int F>
float run(dim3 grid, const int16_t *src, const RowFix *fix, const int *gran, const Plan *plans, const uint32_t *ramp,
          uint32_t *out, unsigned *amb, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < reps + 1; r++) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(c2<F>, grid, dim3(256), 0, 0, src, fix, gran, plans, ramp, out, amb, 254.0f / 10000.0f, 0, 10000);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0 && ms < best) best = ms;
  }
  return best;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
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
  // two geometries: SCATTER (tile t on granule t % 16) and GRID (the real C2 layout)
  const double sc = 0.47, ang = 1.0 * M_PI / 180.0, two32 = 4294967296.0;
  RowFix *hf[2];
  int *hg[2];
  for (int geo = 0; geo < 2; geo++) {
    hf[geo] = (RowFix *)malloc(sizeof(RowFix) * kTiles * kW);
    hg[geo] = (int *)malloc(sizeof(int) * kTiles);
    for (int t = 0; t < kTiles; t++) {
      int g, px, py;
      if (geo == 0) {
        g = t % kG;
        const int k = t / kG;
        px = k % 16; py = k / 16;
      } else {
        const int tx = t % 64, ty = t / 64;
        g = (ty / 16) * 4 + tx / 16;
        px = tx % 16; py = ty % 16;
      }
      hg[geo][t] = g;
      const double ox = 60.0 + px * 240.7 + 0.123, oy = 60.0 + py * 240.7 + 0.377;
      for (int r = 0; r < kW; r++) {
        const double x0 = ox - sc * std::sin(ang) * r, y0 = oy + sc * std::cos(ang) * r;
        RowFix &f = hf[geo][(int64_t)t * kW + r];
        f.x0 = (int64_t)(x0 * two32);
        f.y0 = (int64_t)(y0 * two32);
        f.dx = (int64_t)(sc * std::cos(ang) * two32);
        f.dy = (int64_t)(sc * std::sin(ang) * two32);
      }
    }
  }
  RowFix *fix[2];
  int *gran[2];
  for (int geo = 0; geo < 2; geo++) {
    CHECK(hipMalloc(&fix[geo], sizeof(RowFix) * kTiles * kW));
    CHECK(hipMemcpy(fix[geo], hf[geo], sizeof(RowFix) * kTiles * kW, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&gran[geo], sizeof(int) * kTiles));
    CHECK(hipMemcpy(gran[geo], hg[geo], sizeof(int) * kTiles, hipMemcpyHostToDevice));
  }
  Plan *hp = (Plan *)malloc(sizeof(Plan) * kTiles);
  for (int t = 0; t < kTiles; t++) hp[t] = Plan{0, 1, 3, t, -999.0, 3, 1};
  Plan *plans;
  CHECK(hipMalloc(&plans, sizeof(Plan) * kTiles));
  CHECK(hipMemcpy(plans, hp, sizeof(Plan) * kTiles, hipMemcpyHostToDevice));
  unsigned *amb;
  CHECK(hipMalloc(&amb, 4));
  CHECK(hipMemset(amb, 0, 4));
  const dim3 grid(kItems);
  std::printf("{\"bytes\": %.0f, \"results\": {", nout * 4.0 + nsrc * 2.0);
#define V(F, NAME, GEO)                                                                                           \
  std::printf("%s\"%s\": %.4f", first ? "" : ", ", NAME,                                                          \
              run<F>(grid, src, fix[GEO], gran[GEO], plans, ramp, out, amb, reps));                               \
  first = false;
  bool first = true;
  V(0, "base", 0)
  V(1, "margin", 0)
  V(2, "rowfix", 0)
  V(4, "scale", 0)
  V(0, "grid", 1)
  V(16, "plan", 0)
  V(7, "margin+rowfix+scale", 0)
  V(7, "margin+rowfix+scale+grid", 1)
  V(23, "all", 1)
  std::printf("}}\n");
  return 0;
}
