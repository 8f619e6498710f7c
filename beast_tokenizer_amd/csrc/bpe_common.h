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

// Bloom bits of the adjacent pair (x, y): two of 64 from a multiplicative hash of both ids.
__device__ __forceinline__ unsigned long long pair_sig(uint32_t x, uint32_t y) {
  uint32_t h = x * 0x9E3779B1u + y * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  return (1ull << (h >> 26)) | (1ull << ((h >> 20) & 63u));
}

// A word's signature, the merge loop's candidate filter: the OR of sig_step(prev, y) over its
// symbols y (prev = the symbol before y, SIG_NONE for the first).  Pair-level (round 6, the
// default): the bits of every adjacent pair, so the test for a merge (a, b) admits only words
// holding a next to b (up to Bloom collisions).  Symbol-level (BPE_SIG_PAIR=0, rounds 1-5): the
// bits of every symbol, which admitted every word holding both a and b anywhere -- 80 % of the
// candidate visits at K5 were such false positives.
#ifndef BPE_SIG_PAIR
#define BPE_SIG_PAIR 1
#endif
constexpr uint32_t SIG_NONE = 0xFFFFFFFFu;
__device__ __forceinline__ unsigned long long sig_step(uint32_t prev, uint32_t y) {
#if BPE_SIG_PAIR
  return prev == SIG_NONE ? 0ull : pair_sig(prev, y);
#else
  (void)prev;
  return sig_bit(y);
#endif
}
// the bits a word's signature holds when it holds the pair (a, b)
__device__ __forceinline__ unsigned long long sig_need(uint32_t a, uint32_t b) {
#if BPE_SIG_PAIR
  return pair_sig(a, b);
#else
  return sig_bit(a) | sig_bit(b);
#endif
}

// workgroups for n items at per_block items each, at least 1 and at most cap
static inline int grid_for(int64_t n, int per_block, int cap) {
  const int64_t g = (n + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}
