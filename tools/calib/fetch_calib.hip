// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access widths of the render kernels (MI355X_MICROARCH.md: only
// 16-B streaming reads and stores are calibrated there).  Each kernel touches a
// known number of distinct bytes of a 1 GiB buffer (4x the Infinity Cache),
// every byte once:
//   read16   16 B per lane, streaming (the guide's known case: FETCH = 1/2)
//   gather2  2 B per lane, lane i of a row reads element i/2 (the NN 2x
//            upsampling pattern of render_nn_kernel over an int16 granule)
//   gather4  4 B per lane, the same pattern over a float32 granule
//   read2    2 B per lane, consecutive (1:1)
//   read8    8 B per lane, consecutive (the 2-tap loads of render_bil_kernel)
//   gather8  8 B per lane, lane i reads element i/2
//   store4   4 B per lane consecutive stores (the RGBA tile rows)
//   store16  16 B per lane streaming stores (the guide's known case: exact)
// Run: fetch_calib <launches>, under rocprofv3 --pmc FETCH_SIZE (one pass)
// and --pmc WRITE_SIZE (another); the factor is counter / bytes printed here.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

__global__ __launch_bounds__(256) void read16(const uint4 *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234u) sink[0] = acc;   // reachable for 16-bit values too (else the loop is dead code)
}

template <typename T>
__global__ __launch_bounds__(256) void gather_half(const T *__restrict__ in, size_t n_out, uint32_t *__restrict__ sink) {
  // output index o reads input o/2: every input element read by two lanes
  uint32_t acc = 0;
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < n_out; o += (size_t)gridDim.x * blockDim.x)
    acc ^= (uint32_t)in[o >> 1];
  if (acc == 0x1234u) sink[0] = acc;   // reachable for 16-bit values too (else the loop is dead code)
}

__global__ __launch_bounds__(256) void read2(const uint16_t *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= in[i];
  if (acc == 0x1234u) sink[0] = acc;   // reachable for 16-bit values too (else the loop is dead code)
}

__global__ __launch_bounds__(256) void read8(const uint2 *__restrict__ in, size_t n, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 v = in[i];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x1234u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void gather8(const uint2 *__restrict__ in, size_t n_out, uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < n_out; o += (size_t)gridDim.x * blockDim.x) {
    const uint2 v = in[o >> 1];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x1234u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void store4(uint32_t *__restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void store16(uint4 *__restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main(int argc, char **argv) {
  const int launches = argc > 1 ? std::atoi(argv[1]) : 3;
  const size_t bytes = (size_t)1 << 30;
  void *buf = nullptr;
  uint32_t *sink = nullptr;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(buf, 1, bytes));
  const dim3 grid(256 * 8 * 4), block(256);
  for (int l = 0; l < launches; l++) {
    hipLaunchKernelGGL(read16, grid, block, 0, 0, (const uint4 *)buf, bytes / 16, sink);
    hipLaunchKernelGGL(gather_half<uint16_t>, grid, block, 0, 0, (const uint16_t *)buf, bytes / 2 * 2, sink);
    hipLaunchKernelGGL(gather_half<float>, grid, block, 0, 0, (const float *)buf, bytes / 4 * 2, sink);
    hipLaunchKernelGGL(read2, grid, block, 0, 0, (const uint16_t *)buf, bytes / 2, sink);
    hipLaunchKernelGGL(read8, grid, block, 0, 0, (const uint2 *)buf, bytes / 8, sink);
    hipLaunchKernelGGL(gather8, grid, block, 0, 0, (const uint2 *)buf, bytes / 8 * 2, sink);
    hipLaunchKernelGGL(store4, grid, block, 0, 0, (uint32_t *)buf, bytes / 4);
    hipLaunchKernelGGL(store16, grid, block, 0, 0, (uint4 *)buf, bytes / 16);
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::printf("{\"distinct_bytes_per_launch\": %zu, \"kernels\": [\"read16\", \"gather_half<ushort>\", "
              "\"gather_half<float>\", \"read2\", \"read8\", \"gather8\", \"store4\", \"store16\"], \"launches\": %d}\n",
              bytes, launches);
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
