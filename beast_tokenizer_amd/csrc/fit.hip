// B-spline constants and small elementwise kernels for gfx950.
//
//   H1/H2  k_basis        Cox-de Boor basis at arbitrary times (bit-exact vs the
//                         reference's fp32 recursion, uni_bspline_basis.py:82-113)
//          k_projection   P = (Phi^T Phi + reg I)^-1 Phi^T in fp64 (one workgroup),
//                         written zero-padded as [16][Tp] for the encode kernel
//   H5     k_quantize     quantise-only epilogue (encode(update_bounds=True), continuous)
//   H13    k_colminmax_*  column min/max (update_weights_bounds*)
// The fused encode / reconstruct kernels live in codec.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {


// ------------------------------------------------------------------ basis --
template <int K>
__device__ float bfun(int i, float u, const float* __restrict__ kv, int nctrl) {
  if constexpr (K == 0) {
    const float a = kv[i], b = kv[i + 1];
    const bool in = (i == nctrl - 1) ? (u >= a && u <= b) : (u >= a && u < b);
    return in ? 1.0f : 0.0f;
  } else {
    const float d1 = __fsub_rn(kv[i + K], kv[i]);
    const float d2 = __fsub_rn(kv[i + K + 1], kv[i + 1]);
    float t1 = 0.0f, t2 = 0.0f;
    if (!(d1 == 0.0f)) t1 = __fmul_rn(__fdiv_rn(__fsub_rn(u, kv[i]), d1), bfun<K - 1>(i, u, kv, nctrl));
    if (!(d2 == 0.0f)) t2 = __fmul_rn(__fdiv_rn(__fsub_rn(kv[i + K + 1], u), d2), bfun<K - 1>(i + 1, u, kv, nctrl));
    return __fadd_rn(t1, t2);
  }
}

template <int K>
__global__ void k_basis(const float* __restrict__ times, int64_t n, float tau, float delay,
                        const float* __restrict__ kv, int nctrl, float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  // linear_phase.py:22-24: clip((t - delay) / tau, 0, 1)
  float u = __fdiv_rn(__fsub_rn(times[i], delay), tau);
  u = (u < 0.0f) ? 0.0f : u;
  u = (1.0f < u) ? 1.0f : u;
  for (int c = 0; c < nctrl; ++c) out[i * nctrl + c] = bfun<K>(c, u, kv, nctrl);
}

// ------------------------------------------------------------- projection --
// One workgroup.  G = Phi^T Phi + reg I (fp64), Gauss-Jordan with partial pivoting
// on [G | I], then P[n][t] = sum_k Ginv[n][k] Phi[t][k].
__global__ void k_projection(const float* __restrict__ basis, int T, int N, double reg,
                             double* __restrict__ P) {
  __shared__ double A[32][65];
  __shared__ double fac[32];
  __shared__ int piv;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < N * N; idx += blockDim.x) {
    const int r = idx / N, c = idx % N;
    double s = 0.0;
    for (int t = 0; t < T; ++t) s += (double)basis[t * N + r] * (double)basis[t * N + c];
    A[r][c] = s + (r == c ? reg : 0.0);
    A[r][N + c] = (r == c) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int k = 0; k < N; ++k) {
    if (tid == 0) {
      int p = k;
      double best = fabs(A[k][k]);
      for (int r = k + 1; r < N; ++r)
        if (fabs(A[r][k]) > best) { best = fabs(A[r][k]); p = r; }
      piv = p;
    }
    __syncthreads();
    const int p = piv;
    if (p != k)
      for (int c = tid; c < 2 * N; c += blockDim.x) { double t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t; }
    __syncthreads();
    const double inv = 1.0 / A[k][k];
    __syncthreads();
    for (int c = tid; c < 2 * N; c += blockDim.x) A[k][c] *= inv;
    __syncthreads();
    // eliminate with a per-row factor snapshot (column k is overwritten by the update)
    for (int r = tid; r < N; r += blockDim.x) fac[r] = (r == k) ? 0.0 : A[r][k];
    __syncthreads();
    for (int idx = tid; idx < N * 2 * N; idx += blockDim.x) {
      const int r = idx / (2 * N), c = idx % (2 * N);
      A[r][c] -= fac[r] * A[k][c];
    }
    __syncthreads();
  }
  // zero-padded [16][Tp] layout consumed directly by k_encode's MFMA A operand
  const int Tp = (T + 3) & ~3;
  for (int idx = tid; idx < 16 * Tp; idx += blockDim.x) {
    const int n = idx / Tp, t = idx % Tp;
    double s = 0.0;
    if (n < N && t < T)
      for (int k = 0; k < N; ++k) s += A[n][N + k] * (double)basis[t * N + k];
    P[idx] = s;
  }
}

// --------------------------------------------------------------- quantise --
// thread per output element (b, n, d): reads params (d n), writes (n d).
__global__ void k_quantize(const float* __restrict__ params, int64_t B, int D, int N, const float* __restrict__ w_min,
                           const float* __restrict__ w_max, int vocab, int64_t tok_offset, int mode,
                           long long* __restrict__ tok, float* __restrict__ ntok) {
  const int per = N * D;
  const int64_t total = B * per;
  const float vm1 = (float)(vocab - 1);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / per;
    const int r = (int)(e % per), n = r / D, d = r % D, k = d * N + n;
    const float p = params[b * per + k];
    if (mode == 0) tok[e] = beast::quantize_one(p, w_min[k], w_max[k], vm1) + tok_offset;
    else ntok[e] = beast::normalize_one(p, w_min[k], w_max[k]);
  }
}

// ------------------------------------------------------------ col min/max --
__device__ __forceinline__ float nanmin(float m, float v) {
  if (m != m) return m;
  if (v != v) return v;
  return (v < m) ? v : m;
}
__device__ __forceinline__ float nanmax(float m, float v) {
  if (m != m) return m;
  if (v != v) return v;
  return (m < v) ? v : m;
}

__global__ void k_colminmax_partial(const float* __restrict__ x, int64_t rows, int cols, int64_t rs,
                                    int64_t rows_per_block, float* __restrict__ pmin, float* __restrict__ pmax) {
  const int64_t r0 = blockIdx.x * rows_per_block;
  const int64_t r1 = min<int64_t>(rows, r0 + rows_per_block);
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    float mn = __builtin_inff(), mx = -__builtin_inff();
    for (int64_t r = r0; r < r1; ++r) {
      const float v = x[r * rs + c];
      mn = nanmin(mn, v);
      mx = nanmax(mx, v);
    }
    pmin[blockIdx.x * (int64_t)cols + c] = mn;
    pmax[blockIdx.x * (int64_t)cols + c] = mx;
  }
}

__global__ void k_colminmax_final(const float* __restrict__ pmin, const float* __restrict__ pmax, int nblk,
                                  int cols, float* __restrict__ omin, float* __restrict__ omax) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float mn = __builtin_inff(), mx = -__builtin_inff();
  for (int b = 0; b < nblk; ++b) {
    mn = nanmin(mn, pmin[(int64_t)b * cols + c]);
    mx = nanmax(mx, pmax[(int64_t)b * cols + c]);
  }
  omin[c] = mn;
  omax[c] = mx;
}

constexpr int MINMAX_BLOCKS = 512;

}  // namespace

// =================================================================== C-ABI ==
extern "C" int beast_bspline_basis_f32(const float* times, int64_t n_times, float tau, float delay,
                                       const float* knots, int n_knots, int degree, int num_basis,
                                       float* basis_out, void* stream) {
  BEAST_REQUIRE(times && knots && basis_out, "beast_bspline_basis_f32: null pointer");
  BEAST_REQUIRE(degree >= 0 && degree <= 8, "degree_p must be in [0, 8], got %d", degree);
  BEAST_REQUIRE(num_basis >= 1 && n_knots == degree + 1 + num_basis, "knot vector size %d != degree+1+num_basis",
                n_knots);
  if (n_times <= 0) return BEAST_OK;
  const int nthr = 256;
  const int64_t nblk = (n_times + nthr - 1) / nthr;
  hipStream_t s = beast::as_stream(stream);
#define BEAST_BASIS_CASE(K) \
  case K: hipLaunchKernelGGL(k_basis<K>, dim3(nblk), dim3(nthr), 0, s, times, n_times, tau, delay, knots, num_basis, basis_out); break;
  switch (degree) {
    BEAST_BASIS_CASE(0) BEAST_BASIS_CASE(1) BEAST_BASIS_CASE(2) BEAST_BASIS_CASE(3) BEAST_BASIS_CASE(4)
    BEAST_BASIS_CASE(5) BEAST_BASIS_CASE(6) BEAST_BASIS_CASE(7) BEAST_BASIS_CASE(8)
  }
#undef BEAST_BASIS_CASE
  BEAST_LAUNCHED("k_basis");
  return BEAST_OK;
}

extern "C" int beast_bspline_projection_f64(const float* basis, int T, int N, double reg, double* proj_out,
                                            void* stream) {
  BEAST_REQUIRE(basis && proj_out, "beast_bspline_projection_f64: null pointer");
  BEAST_REQUIRE(N >= 1 && N <= 16 && T >= 1, "projection: need 1 <= N <= 16, T >= 1 (N=%d T=%d)", N, T);
  hipLaunchKernelGGL(k_projection, dim3(1), dim3(256), 0, beast::as_stream(stream), basis, T, N, reg, proj_out);
  BEAST_LAUNCHED("k_projection");
  return BEAST_OK;
}

extern "C" int beast_quantize_f32(const float* params, int64_t B, int D, int N, const float* w_min,
                                  const float* w_max, int vocab, int64_t tok_offset, int mode, int64_t* tokens_out,
                                  float* ntok_out, void* stream) {
  BEAST_REQUIRE(params && w_min && w_max, "beast_quantize_f32: null input pointer");
  BEAST_REQUIRE((mode == 0 && tokens_out && vocab >= 2) || (mode == 1 && ntok_out), "beast_quantize_f32: bad mode");
  BEAST_REQUIRE(B >= 0, "batch size B=%lld must be >= 0", (long long)B);
  if (B == 0) return BEAST_OK;
  const int64_t total = B * (int64_t)N * D;
  const int64_t grid = std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(k_quantize, dim3(grid), dim3(256), 0, beast::as_stream(stream), params, B, D, N, w_min, w_max,
                     vocab, tok_offset, mode, reinterpret_cast<long long*>(tokens_out), ntok_out);
  BEAST_LAUNCHED("k_quantize");
  return BEAST_OK;
}

extern "C" size_t beast_colminmax_workspace_bytes(int64_t rows, int cols) {
  (void)rows;
  return (size_t)2 * MINMAX_BLOCKS * (size_t)cols * sizeof(float);
}

extern "C" int beast_colminmax_f32(const float* x, int64_t rows, int cols, int64_t row_stride, float* out_min,
                                   float* out_max, void* workspace, size_t ws_bytes, void* stream) {
  BEAST_REQUIRE(x && out_min && out_max && workspace, "beast_colminmax_f32: null pointer");
  BEAST_REQUIRE(rows >= 1 && cols >= 1, "colminmax needs rows >= 1, cols >= 1");
  BEAST_REQUIRE_CODE(ws_bytes >= beast_colminmax_workspace_bytes(rows, cols), BEAST_E_WORKSPACE,
                     "colminmax workspace too small");
  const int64_t rpb = std::max<int64_t>(1, (rows + MINMAX_BLOCKS - 1) / MINMAX_BLOCKS);
  const int nblk = (int)((rows + rpb - 1) / rpb);
  float* pmin = reinterpret_cast<float*>(workspace);
  float* pmax = pmin + (size_t)MINMAX_BLOCKS * cols;
  hipStream_t s = beast::as_stream(stream);
  hipLaunchKernelGGL(k_colminmax_partial, dim3(nblk), dim3(256), 0, s, x, rows, cols, row_stride, rpb, pmin, pmax);
  BEAST_LAUNCHED("k_colminmax_partial");
  hipLaunchKernelGGL(k_colminmax_final, dim3((cols + 255) / 256), dim3(256), 0, s, pmin, pmax, nblk, cols, out_min,
                     out_max);
  BEAST_LAUNCHED("k_colminmax_final");
  return BEAST_OK;
}
