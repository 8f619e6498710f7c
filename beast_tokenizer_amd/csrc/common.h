// Shared helpers for libbeast_hip.so (gfx950).  Error plumbing for the C-ABI and
// the bit-exact fp32 helpers the quantiser / dequantiser need.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "beast_hip.h"

namespace beast {

void set_error(const char* fmt, ...);
// BEAST_OPT_MERGE_LDS_MIN: pair count from which k_merge privatises its deltas in LDS
extern int64_t g_merge_lds_min;
// BEAST_OPT_BPE_ENCODE_MODE: bit 0 = heap merge, bit 1 = one workgroup per 4 rows
extern int g_bpe_encode_mode;
// BEAST_OPT_BPE_DEDUP_KEY_BITS: width of the dedup encode's word keys (tests force collisions)
extern int g_bpe_dedup_key_bits;
// BEAST_OPT_BPE_TRAIN_HOST_LOOP: beast_bpe_train's loop (tests: 1 host-driven, 2 rerun as after a
// string-hash collision of the batched loop)
extern int g_bpe_train_host;
int hip_fail(hipError_t e, const char* what);
// comm.hip: a rank's status agreed over the communicator (every rank must call it at the same
// point).  Returns rc when it failed locally, the failing rank's code (message: which rank) when
// another rank failed, BEAST_OK when all succeeded; comm == nullptr returns rc.
int comm_agree(beast_comm* comm, int rc, hipStream_t s);
// comm.hip: max over the ranks of a non-negative int (every rank calls it at the same point)
int comm_max_i32(beast_comm* comm, int v, int* out, hipStream_t s);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// torch.clamp(x, min=lo_tensor, max=hi_tensor): std::min(std::max(x, lo), hi) with
// NaN propagation (ATen clamp kernel; NaN bounds -> NaN).
__device__ __forceinline__ float clamp_t(float x, float lo, float hi) {
  if (lo != lo || hi != hi) return __builtin_nanf("");
  float r = (x < lo) ? lo : x;
  return (hi < r) ? hi : r;
}

// beast/utils.py:12-16, one element: sub, div, clamp, mul, rint -> int64.
// -ffp-contract=off is set for the whole library, and division is IEEE
// (correctly rounded), so every op rounds exactly like ATen's fp32 CPU kernels.
__device__ __forceinline__ long long quantize_one(float p, float lo, float hi, float vm1) {
  float x = clamp_t(p, lo, hi);                         // beast_bspline_tokenizer.py:419
  float s = __fsub_rn(hi, lo);
  s = (s < 1e-8f) ? 1e-8f : s;                          // clamp(max-min, min=1e-8), NaN kept
  float u = __fdiv_rn(__fsub_rn(x, lo), s);
  u = (u < 0.0f) ? 0.0f : u;                            // clamp(., 0, 1), NaN kept
  u = (1.0f < u) ? 1.0f : u;
  float r = rintf(__fmul_rn(u, vm1));                   // torch.round = half-to-even
  if (r != r) return (long long)0x8000000000000000ULL;  // x86 cvtt of NaN (ATen .to(long))
  return (long long)r;
}

// quantize_one with the per-column scale s = clamp(hi - lo, min=1e-8) precomputed.
__device__ __forceinline__ long long quantize_scaled(float p, float lo, float hi, float s, float vm1) {
  const float x = clamp_t(p, lo, hi);
  float u = __fdiv_rn(__fsub_rn(x, lo), s);
  u = (u < 0.0f) ? 0.0f : u;
  u = (1.0f < u) ? 1.0f : u;
  const float r = rintf(__fmul_rn(u, vm1));
  if (r != r) return (long long)0x8000000000000000ULL;
  return (long long)r;
}

// quantize_one as a bin index: the same ops, int32 result, INT32_MIN for NaN (widened
// to ATen's INT64_MIN by the caller).
__device__ __forceinline__ int quantize_bin(float p, float lo, float hi, float vm1) {
  const float x = clamp_t(p, lo, hi);
  float s = __fsub_rn(hi, lo);
  s = (s < 1e-8f) ? 1e-8f : s;
  float u = __fdiv_rn(__fsub_rn(x, lo), s);
  u = (u < 0.0f) ? 0.0f : u;
  u = (1.0f < u) ? 1.0f : u;
  const float r = rintf(__fmul_rn(u, vm1));
  return (r != r) ? (int)0x80000000 : (int)r;
}

// quantize_bin through a reciprocal: va = (x - lo) * (vm1 * rcp(s)) is within 3.6e-7 * vm1
// of the exactly-rounded chain's u * vm1, so whenever va is farther than 2^-20 * vm1 from
// a rounding boundary (k + 0.5) both round to the same bin; otherwise -- and for NaN /
// inf -- the exact chain decides.  Bit-identical to quantize_bin for every input.
__device__ __forceinline__ int quantize_bin_fast(float p, float lo, float hi, float vm1) {
  const float x = clamp_t(p, lo, hi);
  float s = __fsub_rn(hi, lo);
  s = (s < 1e-8f) ? 1e-8f : s;
  const float va = __fmul_rn(__fsub_rn(x, lo), __fmul_rn(vm1, __builtin_amdgcn_rcpf(s)));
  const float f = __fsub_rn(va, floorf(va));
  if (fabsf(__fsub_rn(f, 0.5f)) > 9.5367431640625e-7f * vm1) return (int)rintf(fminf(va, vm1));
  return quantize_bin(p, lo, hi, vm1);
}

// quantize_bin_fast with the scale precomputed per (DoF, basis) column,
// k = vm1 * rcp(max(hi - lo, 1e-8)) (NaN bounds give a NaN k): returns the fast bin and sets
// `exact` when quantize_bin must decide instead (within 2^-20 * vm1 of a rounding boundary,
// or a NaN / inf on the way).  med3 is clamp_t for lo <= hi; inverted bounds give va <= 0
// -> bin 0, as the exact chain's clamp of u to [0, 1] does.
__device__ __forceinline__ int quantize_bin_k(float p, float lo, float hi, float k, float vm1, bool& exact) {
  const float x = __builtin_amdgcn_fmed3f(p, lo, hi);
  const float va = __fmul_rn(__fsub_rn(x, lo), k);
  const float f = __builtin_amdgcn_fractf(va);
  exact = exact | !(fabsf(__fsub_rn(f, 0.5f)) > 9.5367431640625e-7f * vm1) | (p != p);   // branch-free
  return (int)rintf(fminf(fmaxf(va, 0.0f), vm1));
}

__device__ __forceinline__ float quantize_scale(float lo, float hi, float vm1) {
  float s = __fsub_rn(hi, lo);
  s = (s < 1e-8f) ? 1e-8f : s;
  return __fmul_rn(vm1, __builtin_amdgcn_rcpf(s));
}

__device__ __forceinline__ long long widen_bin(int bin, unsigned long long offset) {
  const unsigned long long v = (bin == (int)0x80000000) ? 0x8000000000000000ULL : (unsigned long long)(long long)bin;
  return (long long)(v + offset);   // two's-complement wrap, as ATen's int64 add
}

// beast/utils.py:23-25, one element: int64 -> fp32, div, mul, add, clamp.
__device__ __forceinline__ float dequantize_one(long long tok, float lo, float hi, float vm1) {
  float n = __fdiv_rn((float)tok, vm1);
  float c = __fadd_rn(__fmul_rn(n, __fsub_rn(hi, lo)), lo);
  return clamp_t(c, lo, hi);
}

// beast/utils.py:29-35 normalize_tensor, one element (norm range [-1, 1]).
__device__ __forceinline__ float normalize_one(float p, float lo, float hi) {
  const float x = clamp_t(p, lo, hi);
  float s = __fsub_rn(hi, lo);
  s = (s < 1e-8f) ? 1e-8f : s;
  const float u = __fdiv_rn(__fsub_rn(x, lo), s);
  return __fadd_rn(__fmul_rn(u, 2.0f), -1.0f);
}

// beast/utils.py:38-44 denormalize_tensor, one element.  The reference line 42
// calls torch.clamp on a Python float and raises TypeError; this implements the
// evident intent, (clip(x,-1,1) + 1) / 2 * (hi - lo) + lo (documented divergence).
__device__ __forceinline__ float denormalize_one(float x, float lo, float hi) {
  float c = (x < -1.0f) ? -1.0f : x;
  c = (1.0f < c) ? 1.0f : c;
  const float u = __fdiv_rn(__fsub_rn(c, -1.0f), 2.0f);
  return __fadd_rn(__fmul_rn(u, __fsub_rn(hi, lo)), lo);
}

}  // namespace beast

#define BEAST_REQUIRE(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      beast::set_error(__VA_ARGS__);             \
      return BEAST_E_INVALID;                    \
    }                                            \
  } while (0)

#define BEAST_REQUIRE_CODE(cond, code, ...)      \
  do {                                           \
    if (!(cond)) {                               \
      beast::set_error(__VA_ARGS__);             \
      return code;                               \
    }                                            \
  } while (0)

#define BEAST_HIP(call, what)                                     \
  do {                                                            \
    hipError_t _e = (call);                                       \
    if (_e != hipSuccess) return beast::hip_fail(_e, what);       \
  } while (0)

#define BEAST_LAUNCHED(what)                                      \
  do {                                                            \
    hipError_t _e = hipGetLastError();                            \
    if (_e != hipSuccess) return beast::hip_fail(_e, what);       \
  } while (0)
