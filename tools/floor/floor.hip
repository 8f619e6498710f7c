// Calibration kernels (tools only, not part of the product): the time an ideal
// one-round-trip tile kernel needs to move the same bytes with the same grid.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(256) void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0xFFFFFFF) p[0] = 1;
}

// every workgroup reads in_per bytes and writes out_per bytes of its own tile
__global__ __launch_bounds__(256) void k_tile_copy(const uint4* __restrict__ in, int64_t in_per16,
                                                   uint4* __restrict__ out, int64_t out_per16, int64_t ntiles) {
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint4* s = in + t * in_per16;
    uint4* d = out + t * out_per16;
    uint4 acc = {0, 0, 0, 0};
    uint4 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = threadIdx.x + k * 256;
      r[k] = i < in_per16 ? s[i] : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { acc.x ^= r[k].x; acc.y ^= r[k].y; acc.z ^= r[k].z; acc.w ^= r[k].w; }
    for (int64_t i = threadIdx.x; i < out_per16; i += 256) d[i] = acc;
  }
}

extern "C" int floor_empty(int grid, void* stream) {
  hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, (hipStream_t)stream, nullptr);
  return hipGetLastError();
}
extern "C" int floor_tile_copy(const void* in, int64_t in_per16, void* out, int64_t out_per16, int64_t ntiles,
                               int grid, void* stream) {
  hipLaunchKernelGGL(k_tile_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)in, in_per16,
                     (uint4*)out, out_per16, ntiles);
  return hipGetLastError();
}
