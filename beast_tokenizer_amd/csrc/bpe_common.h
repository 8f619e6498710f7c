// Shared by the BPE training kernels (bpe_setup.hip, bpe_loop.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

// Bloom signature bits of symbol x: two of 64 (k = 2 keeps false positives of a 2-symbol query
// ~(2n/64)^4 for a word of n distinct symbols, vs (n/64)^2 with one bit)
__device__ __forceinline__ unsigned long long sig_bit(uint32_t x) {
  return (1ull << (x & 63u)) | (1ull << (((x * 0x9E3779B1u) >> 26) & 63u));
}

// workgroups for n items at per_block items each, at least 1 and at most cap
static inline int grid_for(int64_t n, int per_block, int cap) {
  const int64_t g = (n + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}
