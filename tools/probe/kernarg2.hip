// Kernel-argument latency probe, device-timed (tools only): back-to-back launches queued
// behind a spin kernel (host submission hidden) of a 512 x 448 tile-copy kernel moving the
// B=4096 encode's bytes (11.5 MB in, 6.9 MB out), with its pointers passed (a) inside a
// 256-byte by-value struct like EncArgs, (b) as leading scalar arguments.  Built twice:
// plain, and with -mllvm -amdgpu-kernarg-preload-count=8 (leading scalars preloaded into
// SGPRs by the dispatcher).
// Build: hipcc --offload-arch=gfx950 -O3 kernarg2.hip -o kernarg2
//        hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=8 kernarg2.hip -o kernarg2_pre
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { float4* out; const float4* in; long long n_in, n_out; int pad[56]; };

__global__ void k_spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}

__device__ __forceinline__ void tile_copy(float4* out, const float4* in, long long n_in, long long n_out) {
  // each workgroup: its contiguous slice of the input, then of the output (one round trip)
  const long long per_in = (n_in + gridDim.x - 1) / gridDim.x, per_out = (n_out + gridDim.x - 1) / gridDim.x;
  float4 v[4];
  const long long i0 = blockIdx.x * per_in;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = i0 + u * blockDim.x + threadIdx.x;
    v[u] = (i < min(i0 + per_in, n_in)) ? in[i] : make_float4(0, 0, 0, 0);
  }
  const long long o0 = blockIdx.x * per_out;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long o = o0 + u * blockDim.x + threadIdx.x;
    if (o < min(o0 + per_out, n_out)) out[o] = make_float4(v[u].x + v[(u + 1) & 3].y, v[u].y, v[u].z, v[u].w);
  }
}

__global__ __launch_bounds__(448) void k_struct(Big a) { tile_copy(a.out, a.in, a.n_in, a.n_out); }
__global__ __launch_bounds__(448) void k_scalar(float4* out, const float4* in, long long n_in, long long n_out) {
  tile_copy(out, in, n_in, n_out);
}
__global__ __launch_bounds__(448) void k_struct_store(Big a) {
  if (threadIdx.x == 0) a.out[blockIdx.x] = make_float4((float)a.n_in, 0, 0, 0);
}
__global__ __launch_bounds__(448) void k_scalar_store(float4* out, const float4* in, long long n_in, long long n_out) {
  if (threadIdx.x == 0) out[blockIdx.x] = make_float4((float)n_in, 0, 0, 0);
}

template <class F>
float per_launch_us(F f, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 10; ++i) f();
  (void)hipDeviceSynchronize();
  k_spin<<<1, 64>>>(100LL * 1000 * 1000);
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f / reps;
}

int main() {
  const long long n_in = 11468800LL / 16, n_out = 6881280LL / 16;
  float4 *a, *b;
  (void)hipMalloc(&a, n_in * 16);
  (void)hipMalloc(&b, n_in * 16);
  (void)hipMemset(a, 0, n_in * 16);
  Big s{b, a, n_in, n_out, {}};
  const int reps = 500;
  for (int r = 0; r < 2; ++r) {
    printf("{\"struct_store_us\": %.3f, ", per_launch_us([&] { k_struct_store<<<512, 448>>>(s); }, reps));
    printf("\"scalar_store_us\": %.3f, ", per_launch_us([&] { k_scalar_store<<<512, 448>>>(b, a, n_in, n_out); }, reps));
    printf("\"struct_copy_us\": %.3f, ", per_launch_us([&] { k_struct<<<512, 448>>>(s); }, reps));
    printf("\"scalar_copy_us\": %.3f}\n", per_launch_us([&] { k_scalar<<<512, 448>>>(b, a, n_in, n_out); }, reps));
  }
  return 0;
}
