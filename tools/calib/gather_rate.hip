// gather_rate.hip -- issue rate of the vector-memory instruction shapes the
// NN band kernel could use (render_nn.h), from a 4 MiB L2-resident table so
// that HBM does not enter: cycles of one CU per wave-instruction.
//   u16_2x    buffer_load_ushort, lane i -> element base + i/2 (C2's 2x upsampling gather)
//   u16_1x    buffer_load_ushort, lane i -> element base + i
//   u16_rows  buffer_load_ushort, lane i -> row i (64 cache lines per instruction)
//   u32_1x    buffer_load_dword, lane i -> dword base + i (256 contiguous bytes)
//   u32_2x    buffer_load_dword, lane i -> dword base + i/2
//   g16_2x    global_load_ushort, the u16_2x addresses
//   bperm     ds_bpermute_b32 (no memory): the cross-lane pick of a cooperative load
// Each wave issues kIter x 8 instructions (8 independent loads per round,
// as render_nn_kernel's lane issues 8 gathers per row); the result of every
// load feeds an XOR so none is dead.  Prints one JSON line.
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

constexpr int kIter = 256;
constexpr int kRowElems = 4096;          // 8 KiB rows of uint16
constexpr int kRows = 256;               // 4 MiB table

template <int P>
__global__ __launch_bounds__(256) void rate(const uint16_t *__restrict__ tab, uint32_t *__restrict__ sink) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)tab, (short)0,
                                                                     kRowElems * kRows * 2, 0x00020000);
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
  uint32_t acc = 0;
  int row = wave % kRows, col = (wave * 64) % (kRowElems - 1024);
#pragma unroll 1
  for (int it = 0; it < kIter; it++) {
    uint32_t v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int c = col + 64 * q;
      const int r = (row + q) % kRows;
      if constexpr (P == 0) v[q] = __builtin_amdgcn_raw_buffer_load_b16(rs, (uint32_t)(r * kRowElems + c / 2 + lane / 2) * 2u, 0, 0);
      if constexpr (P == 1) v[q] = __builtin_amdgcn_raw_buffer_load_b16(rs, (uint32_t)(r * kRowElems + c + lane) * 2u, 0, 0);
      if constexpr (P == 2) v[q] = __builtin_amdgcn_raw_buffer_load_b16(rs, (uint32_t)(((r + lane) % kRows) * kRowElems + c) * 2u, 0, 0);
      if constexpr (P == 3) v[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(r * kRowElems + 2 * c + 2 * lane) * 2u, 0, 0);
      if constexpr (P == 4) v[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(r * kRowElems + c + 2 * (lane / 2)) * 2u, 0, 0);
      if constexpr (P == 5) v[q] = tab[r * kRowElems + c / 2 + lane / 2];
      if constexpr (P == 6) v[q] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane * 7 + q + it) & 63) * 4), (int)(acc + q));
    }
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= v[q];
    col = (col + 512) % (kRowElems - 1024);
    row = (row + 8) % kRows;
  }
  if (acc == 0x1234u) sink[0] = acc;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  uint16_t *tab = nullptr;
  uint32_t *sink = nullptr;
  CHECK(hipMalloc(&tab, (size_t)kRowElems * kRows * 2));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(tab, 1, (size_t)kRowElems * kRows * 2));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const dim3 grid(cus * 8), block(256);   // 8 workgroups (32 waves) per CU
  const char *names[] = {"u16_2x", "u16_1x", "u16_rows", "u32_1x", "u32_2x", "g16_2x", "bperm"};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("{\"cus\": %d, \"clock_ghz_assumed\": 2.4, \"waves_per_cu\": 32, \"insts_per_wave\": %d, \"results\": {",
              cus, kIter * 8);
  for (int p = 0; p < 7; p++) {
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
      CHECK(hipEventRecord(e0));
      switch (p) {
        case 0: hipLaunchKernelGGL(rate<0>, grid, block, 0, 0, tab, sink); break;
        case 1: hipLaunchKernelGGL(rate<1>, grid, block, 0, 0, tab, sink); break;
        case 2: hipLaunchKernelGGL(rate<2>, grid, block, 0, 0, tab, sink); break;
        case 3: hipLaunchKernelGGL(rate<3>, grid, block, 0, 0, tab, sink); break;
        case 4: hipLaunchKernelGGL(rate<4>, grid, block, 0, 0, tab, sink); break;
        case 5: hipLaunchKernelGGL(rate<5>, grid, block, 0, 0, tab, sink); break;
        default: hipLaunchKernelGGL(rate<6>, grid, block, 0, 0, tab, sink); break;
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    // per CU: 32 waves x kIter x 8 instructions
    const double insts_per_cu = 32.0 * kIter * 8;
    const double cyc = best * 1e-3 * 2.4e9 / insts_per_cu;
    std::printf("%s\"%s\": {\"ms\": %.4f, \"cu_cycles_per_inst\": %.2f}", p ? ", " : "", names[p], best, cyc);
  }
  std::printf("}}\n");
  CHECK(hipFree(tab));
  CHECK(hipFree(sink));
  return 0;
}
