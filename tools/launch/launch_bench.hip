// Host cost of one kernel launch by different HIP entry points (tools only).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <vector>

struct Args { char pad[224]; };

__global__ void k_spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}

struct Args8 { long long p; };
struct Args64 { char pad[64]; };
__global__ void k_noop8(Args8 a) {
  if (a.p == 123 && threadIdx.x == 9999) __builtin_amdgcn_s_sleep(1);
}
__global__ void k_noop64(Args64 a) {
  if (a.pad[0] == 123 && threadIdx.x == 9999) a.pad[1] = 0;
}

__global__ void k_noop(Args a) {
  if (a.pad[0] == 123 && threadIdx.x == 9999) a.pad[1] = 0;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <class F>
double host_us(F f, int n) {
  for (int i = 0; i < 200; ++i) f();
  hipDeviceSynchronize();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Args a;
  memset(&a, 0, sizeof(a));
  const int n = 5000;
  hipFunction_t f;
  CK(hipGetFuncBySymbol(&f, (const void*)k_noop));
  size_t sz = sizeof(a);
  void* args[] = {&a};
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  // interleaved rounds: every entry point once per round, median over rounds
  const char* names[] = {"hipLaunchKernelGGL_512", "hipLaunchKernel", "hipModuleLaunchKernel_extra",
                         "hipModuleLaunchKernel_params", "hipExtLaunchKernel"};
  std::vector<double> t[5];
  for (int r = 0; r < 9; ++r) {
    t[0].push_back(host_us([&] { hipLaunchKernelGGL(k_noop, dim3(512), dim3(256), 0, s, a); }, n));
    t[1].push_back(host_us([&] { hipLaunchKernel((const void*)k_noop, dim3(512), dim3(256), args, 0, s); }, n));
    t[2].push_back(host_us([&] { hipModuleLaunchKernel(f, 512, 1, 1, 256, 1, 1, 0, s, nullptr, cfg); }, n));
    t[3].push_back(host_us([&] { hipModuleLaunchKernel(f, 512, 1, 1, 256, 1, 1, 0, s, args, nullptr); }, n));
    t[4].push_back(host_us([&] { hipExtLaunchKernel((const void*)k_noop, dim3(512), dim3(256), args, 0, s, nullptr, nullptr, 0); }, n));
  }
  printf("{");
  for (int i = 0; i < 5; ++i) {
    std::sort(t[i].begin(), t[i].end());
    printf("\"%s\": [%.3f, %.3f, %.3f], ", names[i], t[i][0], t[i][4], t[i][8]);
  }
  // null stream
  printf("\"GGL_null_stream\": %.3f, ", host_us([&] { hipLaunchKernelGGL(k_noop, dim3(512), dim3(256), 0, 0, a); }, n));
  // graph of 2 kernels
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(k_noop, dim3(512), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_noop, dim3(512), dim3(256), 0, s, a);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  printf("\"graph2_launch\": %.3f, ", host_us([&] { hipGraphLaunch(ge, s); }, n));
  // device-side throughput of back-to-back launches
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_noop, dim3(512), dim3(256), 0, s, a);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("\"gpu_us_per_noop_512\": %.3f, ", ms * 1000 / 2000);
  // queue pre-filled behind a spin: the GPU's own per-kernel cadence
  for (int grid : {1, 512, 2048}) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000000LL);
    hipEventRecord(e0, s);
    for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(k_noop, dim3(grid), dim3(256), 0, s, a);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("\"gpu_us_per_noop_queued_grid%d\": %.3f, ", grid, ms * 1000 / 1000);
  }
  // host cost alone: the stream held behind a long spin, so no launch can wait for the GPU
  {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 20000000LL);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 2000; ++i) hipModuleLaunchKernel(f, 512, 1, 1, 256, 1, 1, 0, s, args, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    printf("\"host_us_module_launch_blocked\": %.3f, ", std::chrono::duration<double, std::micro>(t1 - t0).count() / 2000);
    hipDeviceSynchronize();
    // the same with 8- and 64-byte argument blocks (host cost of the kernarg copy)
    hipFunction_t f8, f64;
    hipGetFuncBySymbol(&f8, (const void*)k_noop8);
    hipGetFuncBySymbol(&f64, (const void*)k_noop64);
    Args8 a8{0};
    Args64 a64;
    memset(&a64, 0, sizeof(a64));
    void* args8[] = {&a8};
    void* args64[] = {&a64};
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 20000000LL);
      t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 2000; ++i) hipModuleLaunchKernel(f8, 512, 1, 1, 256, 1, 1, 0, s, args8, nullptr);
      t1 = std::chrono::steady_clock::now();
      if (rep) printf("\"host_us_module_launch_blocked_8B\": %.3f, ", std::chrono::duration<double, std::micro>(t1 - t0).count() / 2000);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 20000000LL);
      t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 2000; ++i) hipModuleLaunchKernel(f64, 512, 1, 1, 256, 1, 1, 0, s, args64, nullptr);
      t1 = std::chrono::steady_clock::now();
      if (rep) printf("\"host_us_module_launch_blocked_64B\": %.3f, ", std::chrono::duration<double, std::micro>(t1 - t0).count() / 2000);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 20000000LL);
      t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 2000; ++i) hipModuleLaunchKernel(f, 512, 1, 1, 256, 1, 1, 0, s, args, nullptr);
      t1 = std::chrono::steady_clock::now();
      if (rep) printf("\"host_us_module_launch_blocked_224B\": %.3f, ", std::chrono::duration<double, std::micro>(t1 - t0).count() / 2000);
      hipDeviceSynchronize();
    }
    int dev = 0;
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 20000; ++i) hipStreamGetDevice(s, &dev);
    t1 = std::chrono::steady_clock::now();
    printf("\"host_us_stream_get_device\": %.4f, ", std::chrono::duration<double, std::micro>(t1 - t0).count() / 20000);
    hipDeviceSynchronize();
  }
  printf("\"end\": 0}\n");
  return 0;
}
