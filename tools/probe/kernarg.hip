// Kernel-argument latency probe (tools only): per-launch duration of a 512-workgroup kernel
// that reads its arguments and stores one value per workgroup, with the arguments passed
// as a by-value struct, as leading scalars, and (built with -DPRELOAD) as leading scalars
// preloaded into SGPRs (-mllvm -amdgpu-kernarg-preload-count).  Also a 4 KB-per-workgroup
// copy kernel in both forms.  Build: hipcc --offload-arch=gfx950 -O3 kernarg.hip -o kernarg
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

struct Big { float* out; const float4* in; long long n; int pad[40]; };

__global__ void k_struct(Big a) {
  if (threadIdx.x == 0) a.out[blockIdx.x] = (float)a.n;
}
__global__ void k_scalar(float* out, long long n) {
  if (threadIdx.x == 0) out[blockIdx.x] = (float)n;
}
__global__ void k_copy_struct(Big a) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < a.n) reinterpret_cast<float4*>(a.out)[i] = a.in[i];
}
__global__ void k_copy_scalar(float* out, const float4* in, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) reinterpret_cast<float4*>(out)[i] = in[i];
}

template <class F>
float time_us(F f, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 20; ++i) f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f / reps;
}

int main() {
  const int nblk = 512;
  const long long n4 = (long long)nblk * 256;
  float* out; float4* in;
  hipMalloc(&out, n4 * 16); hipMalloc(&in, n4 * 16);
  hipMemset(in, 0, n4 * 16);
  Big b{out, in, n4, {}};
  const int reps = 2000;
  printf("{\"struct_store_us\": %.3f, ", time_us([&] { k_struct<<<nblk, 256>>>(b); }, reps));
  printf("\"scalar_store_us\": %.3f, ", time_us([&] { k_scalar<<<nblk, 256>>>(out, n4); }, reps));
  printf("\"struct_copy_us\": %.3f, ", time_us([&] { k_copy_struct<<<nblk, 256>>>(b); }, reps));
  printf("\"scalar_copy_us\": %.3f}\n", time_us([&] { k_copy_scalar<<<nblk, 256>>>(out, in, n4); }, reps));
  hipDeviceSynchronize();
  return 0;
}
