// store_rate.hip -- write bandwidth of render_nn_kernel's output pattern
// without its gathers: 65536 workgroups of 4 waves, each workgroup 32 rows x
// 512 RGBA words of a 512-word-wide image (4.29 GB), a wave 8 rows, a row
// per lane 8 dwords 64 words apart (C2's layout, render_nn.h store_row).
//   nt_dword      __builtin_nontemporal_store, dword        (the product)
//   plain_dword   plain global_store_dword
//   nt_x4         16-B stores: lane i writes words 4i..4i+3 and 256+4i..
//   persist_nt    2048 workgroups looping over the same 65536 items
//   rows32_nt     16384 workgroups, 32 rows per wave
//   wg1024_nt     1024-thread workgroups (16 waves, 128 rows)
// Prints one JSON line (best of `reps`, TB/s of written bytes).
#include <hip/hip_runtime.h>

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

constexpr int kW = 512;          // words per row
constexpr int kItems = 65536;    // 32-row blocks
constexpr long kWords = (long)kItems * 32 * kW;

template <int P, int RPW, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void wr(uint32_t *__restrict__ out, int items) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int it = blockIdx.x; it < items; it += (P == 3 ? gridDim.x : items)) {
    const long row0 = (long)it * (RPW * WAVES) + wave * RPW;
#pragma unroll 1
    for (int j = 0; j < RPW; j++) {
      uint32_t *dst = out + (row0 + j) * kW;
      const uint32_t v = (uint32_t)(row0 + j) * 2654435761u + lane;
      if constexpr (P == 2) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 x = {v, v + 1, v + 2, v + 3};
        __builtin_nontemporal_store(x, (u4 *)(dst + 4 * lane));
        __builtin_nontemporal_store(x, (u4 *)(dst + 256 + 4 * lane));
      } else {
#pragma unroll
        for (int q = 0; q < 8; q++) {
          if constexpr (P == 1) dst[lane + 64 * q] = v + q;
          else __builtin_nontemporal_store(v + q, dst + lane + 64 * q);
        }
      }
    }
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  uint32_t *out = nullptr;
  CHECK(hipMalloc(&out, kWords * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char *names[] = {"nt_dword", "plain_dword", "nt_x4", "persist_nt", "rows32_nt", "wg1024_nt"};
  std::printf("{\"bytes\": %ld, \"results\": {", kWords * 4);
  for (int p = 0; p < 6; p++) {
    float best = 1e30f;
    for (int r = 0; r < reps + 1; r++) {
      CHECK(hipEventRecord(e0));
      switch (p) {
        case 0: hipLaunchKernelGGL((wr<0, 8, 4>), dim3(kItems), dim3(256), 0, 0, out, kItems); break;
        case 1: hipLaunchKernelGGL((wr<1, 8, 4>), dim3(kItems), dim3(256), 0, 0, out, kItems); break;
        case 2: hipLaunchKernelGGL((wr<2, 8, 4>), dim3(kItems), dim3(256), 0, 0, out, kItems); break;
        case 3: hipLaunchKernelGGL((wr<3, 8, 4>), dim3(2048), dim3(256), 0, 0, out, kItems); break;
        case 4: hipLaunchKernelGGL((wr<0, 32, 4>), dim3(kItems / 4), dim3(256), 0, 0, out, kItems / 4); break;
        default: hipLaunchKernelGGL((wr<0, 8, 16>), dim3(kItems / 4), dim3(1024), 0, 0, out, kItems / 4); break;
      }
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    std::printf("%s\"%s\": {\"ms\": %.4f, \"TBps\": %.3f}", p ? ", " : "", names[p], best,
                kWords * 4 / (best * 1e-3) / 1e12);
  }
  std::printf("}}\n");
  CHECK(hipFree(out));
  return 0;
}
