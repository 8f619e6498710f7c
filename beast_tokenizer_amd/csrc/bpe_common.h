// Shared by the BPE training kernels (bpe_setup.hip, bpe_loop.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

// A word's 64-bit Bloom signature (the merge loop's candidate filter).  Round 6: the low 32 bits
// hold its symbols (two bits each), the high 32 its adjacent pairs (two bits each, from one
// multiplicative hash of the pair).  A query for pair (a, b) needs a's and b's symbol bits AND
// the pair's bits.  Round 5's form -- two bits per symbol over all 64 -- admits every word that
// holds a and b anywhere; most false candidates were of that kind (both symbols, not adjacent),
// which no symbol-only filter rejects.  Over the K5 merges (tools/sig_filter_sim.cpp, sampled
// every 75 merges) the false candidates fall from 302 k to 64 k against 100 k true ones, for the
// same 8 bytes a word in the scan.  BPE_SIG_PAIRS=0 builds round 5's form (A/B).
#ifndef BPE_SIG_PAIRS
#define BPE_SIG_PAIRS 1
#endif
#if BPE_SIG_PAIRS
__device__ __forceinline__ unsigned long long sig_sym(uint32_t x) {
  return (1ull << (x & 31u)) | (1ull << ((x * 0x9E3779B1u) >> 27));
}
__device__ __forceinline__ unsigned long long sig_pair(uint32_t a, uint32_t b) {
  const uint32_t q = (a * 0x9E3779B1u + b) * 0x85EBCA6Bu;
  return (1ull << (32u + (q >> 27))) | (1ull << (32u + ((q >> 22) & 31u)));
}
#else
__device__ __forceinline__ unsigned long long sig_sym(uint32_t x) {
  return (1ull << (x & 63u)) | (1ull << (((x * 0x9E3779B1u) >> 26) & 63u));
}
__device__ __forceinline__ unsigned long long sig_pair(uint32_t, uint32_t) { return 0ull; }
#endif
// the bits a word holding the adjacent pair (a, b) has set
__device__ __forceinline__ unsigned long long sig_need(uint32_t a, uint32_t b) {
  return sig_sym(a) | sig_sym(b) | sig_pair(a, b);
}
// the signature of a word's symbols s[0 .. L)
template <class Get>
__device__ __forceinline__ unsigned long long sig_of(Get s, uint32_t L) {
  unsigned long long g = 0;
  uint32_t prev = 0;
  for (uint32_t i = 0; i < L; ++i) {
    const uint32_t y = s(i);
    g |= sig_sym(y) | (i ? sig_pair(prev, y) : 0ull);
    prev = y;
  }
  return g;
}

// workgroups for n items at per_block items each, at least 1 and at most cap
static inline int grid_for(int64_t n, int per_block, int cap) {
  const int64_t g = (n + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}
