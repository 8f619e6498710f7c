// Launch-floor probe (tools only): per-launch device time of back-to-back launches queued
// behind a spin kernel (host submission hidden), for an empty 512 x 448 grid, a 1-WG grid,
// and an 18.4 MB read+write copy (the B=4096 encode's bytes).
// Build: hipcc --offload-arch=gfx950 -O3 floor_launch.hip -o floor_launch
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}
__global__ void k_empty(float* out) {
  if (threadIdx.x == 1023) out[blockIdx.x] = 0.0f;   // never true: keeps the kernel non-trivial
}
__global__ void k_copy(float4* __restrict__ out, const float4* __restrict__ in, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = in[i];
}

template <class F>
float per_launch_us(F f, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 10; ++i) f();
  (void)hipDeviceSynchronize();
  k_spin<<<1, 64>>>(100LL * 1000 * 1000);   // ~40 ms at 2.4 GHz: the launches below queue up
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f / reps;
}

int main() {
  const long long n4 = 11468800LL / 16;   // 11.47 MB in, 6.9 MB out -> copy 9.2 MB each way
  float4 *a, *b;
  (void)hipMalloc(&a, n4 * 16);
  (void)hipMalloc(&b, n4 * 16);
  (void)hipMemset(a, 0, n4 * 16);
  const int reps = 500;
  printf("{\"empty_512x448_us\": %.3f, ", per_launch_us([&] { k_empty<<<512, 448>>>((float*)b); }, reps));
  printf("\"empty_1x64_us\": %.3f, ", per_launch_us([&] { k_empty<<<1, 64>>>((float*)b); }, reps));
  const long long half = n4 * 4 / 5;
  printf("\"copy_9MB_512x448_us\": %.3f}\n",
         per_launch_us([&] { k_copy<<<512, 448>>>(b, a, half); }, reps));
  return 0;
}
