// Byte-level BPE training, setup kernels for gfx950: everything before the merge loop of HF
// tokenizers' BpeTrainer as driven by beast/beast_bpe_trainer.py:61-98.
//
//   k_minmax / k_presence    global min / max bin, occupied code points (alphabet)
//   k_pretok_wave<EMIT>      GPT-2 regex pre-tokeniser, one wave per sequence over a
//                            code-point class LUT; pass 1 counts words / byte symbols,
//                            pass 2 writes byte symbols as vocab ids
//   k_scan_*                 exclusive prefix sums (word / symbol offsets)
//   k_dedup_*                distinct words x counts (HF trains on word counts)
//   k_len_* / k_copy_words   distinct words repacked contiguously in length order
//   k_word_sig               64-bit Bloom signature of each word's symbols (merge loop filter)
//   k_count_pairs(_lds)      dense [Vt][Vt] uint32 pair table += word count
//   k_compact_words          drop words that can no longer merge (< 2 symbols)
// The merge loop itself is csrc/bpe_loop.hip.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bpe_common.h"
#include "common.h"
#include "pretok.h"

namespace {

[[maybe_unused]] constexpr int CLS_OTHER = 0, CLS_LETTER = 1, CLS_NUMBER = 2, CLS_WS = 3;

// ------------------------------------------------------------- min / max --
__global__ void k_minmax(const long long* __restrict__ x, int64_t n, long long* __restrict__ out) {
  long long mn = 0x7FFFFFFFFFFFFFFFLL, mx = (long long)0x8000000000000000ULL;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const long long v = x[i];
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  // one pair of device atomics per workgroup: the two result words are single addresses,
  // and atomics on one address serialise at the memory side
  __shared__ long long smn[16], smx[16];
  const int wv = threadIdx.x >> 6, nwv = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) { smn[wv] = mn; smx[wv] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < nwv; ++w) {
      mn = smn[w] < mn ? smn[w] : mn;
      mx = smx[w] > mx ? smx[w] : mx;
    }
    atomicMin(&out[0], mn);
    atomicMax(&out[1], mx);
  }
}

__global__ void k_minmax_init(long long* out) {
  out[0] = 0x7FFFFFFFFFFFFFFFLL;
  out[1] = (long long)0x8000000000000000ULL;
}

__global__ void k_presence(const long long* __restrict__ x, int64_t n, long long mn, uint8_t* __restrict__ pr,
                           int64_t ncp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const long long c = x[i] - mn;
    // every writer stores the same byte; the few distinct bytes are written once each instead
    // of once per token (the read hits the cache)
    if (c >= 0 && c < ncp && !pr[c]) pr[c] = 1;
  }
}

// ---------------------------------------------------------- pre-tokenise --
__device__ __forceinline__ int cls_of(long long cp, const uint8_t* __restrict__ lut, int64_t lut_n) {
  return (cp >= 0 && cp < lut_n) ? lut[cp] : CLS_OTHER;
}

__device__ __forceinline__ int utf8_len(long long cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

__device__ __forceinline__ void utf8_bytes(long long cp, uint8_t* b) {
  if (cp < 0x80) { b[0] = (uint8_t)cp; }
  else if (cp < 0x800) { b[0] = (uint8_t)(0xC0 | (cp >> 6)); b[1] = (uint8_t)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) {
    b[0] = (uint8_t)(0xE0 | (cp >> 12)); b[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); b[2] = (uint8_t)(0x80 | (cp & 0x3F));
  } else {
    b[0] = (uint8_t)(0xF0 | (cp >> 18)); b[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
    b[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); b[3] = (uint8_t)(0x80 | (cp & 0x3F));
  }
}

// Length of the GPT-2 contraction ('s|'t|'re|'ve|'m|'ll|'d) starting at s[i] == '\'', or 0.
__device__ __forceinline__ int contraction(const long long* __restrict__ s, int64_t i, int64_t n, long long mn) {
  if (i + 1 >= n) return 0;
  const long long c1 = s[i + 1] - mn;
  if (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd') return 2;
  if (i + 2 >= n) return 0;
  const long long c2 = s[i + 2] - mn;
  if ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l')) return 3;
  return 0;
}

// One sequence, serially.  Regex alternatives, leftmost first:
//   contraction | ' '?L+ | ' '?N+ | ' '?[^\s L N]+ | \s+(?!\S) | \s+
template <bool EMIT>
__device__ void pretok_serial(const long long* __restrict__ tok, const int64_t* __restrict__ seq_off, int64_t sidx,
                              long long mn, const uint8_t* __restrict__ lut, int64_t lut_n,
                              int64_t* __restrict__ words_per_seq, int64_t* __restrict__ syms_per_seq,
                              const int64_t* __restrict__ word_off, const int64_t* __restrict__ sym_off,
                              const uint16_t* __restrict__ byte2id, uint16_t* __restrict__ sym,
                              uint32_t* __restrict__ wstart, uint32_t* __restrict__ wlen) {
  const long long* s = tok + seq_off[sidx];
  const int64_t n = seq_off[sidx + 1] - seq_off[sidx];
  int64_t nw = 0, ns = 0;
  int64_t wo = EMIT ? word_off[sidx] : 0, so = EMIT ? sym_off[sidx] : 0;
  int64_t i = 0;
  while (i < n) {
    const long long c = s[i] - mn;
    int64_t j;
    int k = cls_of(c, lut, lut_n);
    const int con = (c == '\'') ? contraction(s, i, n, mn) : 0;
    if (con) {
      j = i + con;
    } else {
      int64_t st = i;
      if (c == ' ' && i + 1 < n) {
        const int k1 = cls_of(s[i + 1] - mn, lut, lut_n);
        if (k1 != CLS_WS) { k = k1; st = i + 1; }
      }
      if (k != CLS_WS) {
        j = st + 1;
        while (j < n && cls_of(s[j] - mn, lut, lut_n) == k) ++j;
      } else {
        j = i + 1;
        while (j < n && cls_of(s[j] - mn, lut, lut_n) == CLS_WS) ++j;
        if (j < n && j - i >= 2) --j;  // \s+(?!\S): leave the last blank for the next word
      }
    }
    // word = code points [i, j)
    int64_t wsyms = 0;
    for (int64_t p = i; p < j; ++p) wsyms += utf8_len(s[p] - mn);
    if (EMIT) {
      wstart[wo + nw] = (uint32_t)(so + ns);
      wlen[wo + nw] = (uint32_t)wsyms;
      int64_t o = so + ns;
      for (int64_t p = i; p < j; ++p) {
        uint8_t b[4];
        const long long cp = s[p] - mn;
        const int L = utf8_len(cp);
        utf8_bytes(cp, b);
        for (int q = 0; q < L; ++q) sym[o++] = byte2id[b[q]];
      }
    }
    ns += wsyms;
    ++nw;
    i = j;
  }
  if (!EMIT) {
    words_per_seq[sidx] = nw;
    syms_per_seq[sidx] = ns;
  }
}

// One wave per sequence.  A thread per sequence reads its row 8 B at a time at a 1 KiB
// stride (every load instruction touches 64 cache lines), branches on its own word
// structure, and scatters 2-byte stores the same way.  Here the lanes load the row coalesced
// into LDS, classify it, evaluate the regex from every position at once (end of the word
// that would start there), scan the UTF-8 lengths, and walk the word chain 0 -> end[0] -> ...
// together (csrc/pretok.h word_starts); the emission is lane-parallel over words and code points, so the
// stores of a wave land in one contiguous stretch.  Rows longer than PT_LC code points (or
// with code points outside [0, 2^31)) take pretok_serial on lane 0.
constexpr int PT_LC = 512;
constexpr int PT_WAVES = 4;
template <int LC>
struct PtLdsT {
  int32_t cp[LC];
  int32_t e[LC];         // end of the word starting at i
  int32_t wcp[LC + 1];   // first code point of word w
  int16_t so[LC + 1];    // byte-symbol offset of code point i
  uint8_t cls[LC];
  uint8_t vis[LC];       // word_starts' marks
  int32_t nw;
};
using PtLds = PtLdsT<PT_LC>;

__device__ __forceinline__ void pt_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool EMIT>
__global__ __launch_bounds__(64 * PT_WAVES) void k_pretok_wave(
    const long long* __restrict__ tok, const int64_t* __restrict__ seq_off, int64_t n_seq, long long mn,
    const uint8_t* __restrict__ lut, int64_t lut_n, int64_t* __restrict__ words_per_seq,
    int64_t* __restrict__ syms_per_seq, const int64_t* __restrict__ word_off, const int64_t* __restrict__ sym_off,
    const uint16_t* __restrict__ byte2id, uint16_t* __restrict__ sym, uint32_t* __restrict__ wstart,
    uint32_t* __restrict__ wlen) {
  __shared__ PtLds lds[PT_WAVES];
  __shared__ uint8_t s_lut[256];   // classes of code points < 256 (every BEAST bin of a 256 vocab)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lut[i] = i < lut_n ? lut[i] : (uint8_t)CLS_OTHER;
  __syncthreads();
  PtLds& L = lds[wv];
  constexpr int PF = PT_LC / 64;
  for (int64_t sidx = (int64_t)blockIdx.x * PT_WAVES + wv; sidx < n_seq; sidx += (int64_t)gridDim.x * PT_WAVES) {
    const int64_t r0 = seq_off[sidx], n64 = seq_off[sidx + 1] - r0;
    bool serial = n64 > PT_LC;
    const int n = serial ? 0 : (int)n64;
    // 1. code points and classes, then the UTF-8 symbol offsets.  Every load of the row is issued
    //    before the first is used (round 3 waited for each 64-code-point chunk, then for its class
    //    from the global LUT: two dependent round trips per chunk)
    long long tv[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) tv[k] = (lane + 64 * k < n) ? tok[r0 + lane + 64 * k] : 0;
    int carry = 0;
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      if (64 * k >= n) break;
      const int i = 64 * k + lane;
      int len = 0;
      if (i < n) {
        const long long c = tv[k] - mn;
        serial |= (c < 0) | (c > 0x7FFFFFFFLL);
        L.cp[i] = (int32_t)c;
        L.cls[i] = (c >= 0 && c < 256) ? s_lut[c] : (c >= 0 && c < lut_n) ? lut[c] : (uint8_t)CLS_OTHER;
        len = utf8_len(c);
      }
      int tot;
      const int ex = beast_pt::wave_excl_scan(len, lane, tot);
      if (i < n) L.so[i] = (int16_t)(carry + ex);
      carry += tot;
    }
    if (__any(serial)) {   // wave-uniform
      if (lane == 0)
        pretok_serial<EMIT>(tok, seq_off, sidx, mn, lut, lut_n, words_per_seq, syms_per_seq, word_off, sym_off,
                            byte2id, sym, wstart, wlen);
      continue;
    }
    if (lane == 0) L.so[n] = (int16_t)carry;
    pt_wave_sync();
    // 2. the end of the word that starts at every position (pretok_serial's rules), 3. the word
    //    chain 0 -> e[0] -> ... walked lane-parallel (csrc/pretok.h; round 3 walked it on lane 0)
    beast_pt::regex_ends(L.cp, L.cls, L.wcp, L.e, n, lane);   // wcp: scratch until word_starts
    beast_pt::word_starts(L.e, L.vis, L.wcp, nullptr, &L.nw, n, lane);
    const int nw = L.nw;
    if (!EMIT) {
      if (lane == 0) {
        words_per_seq[sidx] = nw;
        syms_per_seq[sidx] = carry;
      }
    } else {
      // 4. words (start, length) and byte symbols, lane-parallel
      const int64_t wo = word_off[sidx], so0 = sym_off[sidx];
      for (int w = lane; w < nw; w += 64) {
        const int s0 = L.so[L.wcp[w]], s1 = L.so[L.wcp[w + 1]];
        wstart[wo + w] = (uint32_t)(so0 + s0);
        wlen[wo + w] = (uint32_t)(s1 - s0);
      }
      for (int i = lane; i < n; i += 64) {
        uint8_t b[4];
        const long long cp = L.cp[i];
        const int Lb = utf8_len(cp);
        utf8_bytes(cp, b);
        uint16_t* o = sym + so0 + L.so[i];
        for (int q = 0; q < Lb; ++q) o[q] = byte2id[b[q]];
      }
    }
    pt_wave_sync();   // LDS is reused by the next sequence
  }
}

// ------------------------------------------------------------------ scan --
constexpr int SCAN_T = 256;
constexpr int SCAN_PER = 4;
constexpr int SCAN_TILE = SCAN_T * SCAN_PER;

__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int64_t off = 0;
  for (int k = 0; k < w; ++k) off += sh[k];
  total = 0;
  for (int k = 0; k < SCAN_T / 64; ++k) total += sh[k];
  __syncthreads();
  return off + x - v;
}

__global__ void k_scan_tiles(const int64_t* __restrict__ in, int64_t* __restrict__ out, int64_t n,
                             int64_t* __restrict__ tile_sums) {
  __shared__ int64_t sh[SCAN_T / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
  int64_t v[SCAN_PER], s = 0;
  for (int k = 0; k < SCAN_PER; ++k) {
    v[k] = (base + k < n) ? in[base + k] : 0;
    s += v[k];
  }
  int64_t total;
  int64_t pre = block_excl_scan(s, sh, total);
  for (int k = 0; k < SCAN_PER; ++k) {
    if (base + k < n) out[base + k] = pre;
    pre += v[k];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

__global__ void k_scan_add(int64_t* __restrict__ out, int64_t n, const int64_t* __restrict__ tile_off) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  const int64_t add = tile_off[blockIdx.x];
  for (int k = threadIdx.x; k < SCAN_TILE; k += SCAN_T)
    if (base + k < n) out[base + k] += add;
}

__global__ void k_scan_total(const int64_t* __restrict__ in, int64_t* __restrict__ out, int64_t n) {
  // out[n] = out[n-1] + in[n-1]
  if (threadIdx.x == 0 && blockIdx.x == 0) out[n] = (n > 0) ? out[n - 1] + in[n - 1] : 0;
}

int64_t scan_ws_elems(int64_t n) {
  int64_t total = 0;
  while (n > 1) {
    const int64_t t = (n + SCAN_TILE - 1) / SCAN_TILE;
    total += 2 * t + 1;
    n = t;
  }
  return total + 2;
}

int scan_rec(const int64_t* in, int64_t* out, int64_t n, int64_t* ws, hipStream_t s) {
  const int64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  int64_t* sums = ws;
  int64_t* offs = ws + tiles;
  hipLaunchKernelGGL(k_scan_tiles, dim3(tiles), dim3(SCAN_T), 0, s, in, out, n, sums);
  BEAST_LAUNCHED("k_scan_tiles");
  if (tiles > 1) {
    int rc = scan_rec(sums, offs, tiles, ws + 2 * tiles + 1, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add, dim3(tiles), dim3(SCAN_T), 0, s, out, n, offs);
    BEAST_LAUNCHED("k_scan_add");
  }
  return BEAST_OK;
}

// ----------------------------------------------------------- pair table --
__global__ void k_count_pairs(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                              const uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount, int64_t nw,
                              uint32_t* __restrict__ table, int Vt) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t st = wstart[w], L = wlen[w];
    const uint32_t cnt = wcount ? wcount[w] : 1u;
    if (L < 2) continue;
    uint32_t prev = sym[st];
    for (uint32_t i = 1; i < L; ++i) {
      const uint32_t cur = sym[st + i];
      atomicAdd(&table[(size_t)prev * Vt + cur], cnt);
      prev = cur;
    }
  }
}

// The same count with the table privatised in LDS: rows [r0, r0 + R) of the n_sym x n_sym
// block of the symbols present at setup (R * n_sym u32 <= 160 KiB), one row group per grid y.
// The workgroup takes 256-word chunks round-robin (words are stored in length order), counts
// its pairs with LDS atomics and flushes row segments to the table with contiguous global
// atomics: device-scope atomics execute at the memory side, so one per (pair, occurrence)
// was the bottleneck of k_count_pairs.
__global__ __launch_bounds__(256) void k_count_pairs_lds(const uint16_t* __restrict__ sym,
                                                         const uint32_t* __restrict__ wstart,
                                                         const uint32_t* __restrict__ wlen,
                                                         const uint32_t* __restrict__ wcount, int64_t nw,
                                                         uint32_t* __restrict__ table, int Vt, int n_sym, int R) {
  extern __shared__ uint32_t hs[];   // [R][n_sym]
  const int r0 = blockIdx.y * R;
  const int rr = min(R, n_sym - r0);
  for (int i = threadIdx.x; i < rr * n_sym; i += blockDim.x) hs[i] = 0;
  __syncthreads();
  const int64_t nchunks = (nw + 255) / 256;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t w = c * 256 + threadIdx.x;
    if (w >= nw) continue;
    const uint32_t L = wlen[w];
    if (L < 2) continue;
    const uint32_t cnt = wcount ? wcount[w] : 1u;
    const uint16_t* s = sym + wstart[w];
    uint32_t prev = s[0];
    for (uint32_t i = 1; i < L; ++i) {
      const uint32_t cur = s[i];
      const int p = (int)prev - r0;
      if (p >= 0 && p < rr && cur < (uint32_t)n_sym) atomicAdd(&hs[p * n_sym + cur], cnt);   // ids < n_sym
      prev = cur;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < rr * n_sym; i += blockDim.x) {
    const uint32_t v = hs[i];
    if (v) atomicAdd(&table[(size_t)(r0 + i / n_sym) * Vt + (i % n_sym)], v);
  }
}

// ------------------------------------------------------------ word dedup --
// HF trains on distinct words x their counts: words of >= 2 symbols are inserted into an
// open-addressing table keyed by (32-bit hash tag, representative index); a candidate
// whose tag matches is compared symbol by symbol with the representative, so collisions
// never merge different words.  The winner of an empty slot appends itself to the
// distinct list; every occurrence adds 1 to the slot's count.
__device__ __forceinline__ uint64_t word_hash(const uint16_t* s, uint32_t L) {
  uint64_t h = 0xcbf29ce484222325ull ^ (uint64_t)L;
  for (uint32_t i = 0; i < L; ++i) h = (h ^ s[i]) * 0x100000001b3ull;
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  return h;
}

struct DedupWs {
  unsigned long long* keys;   // [cap]
  uint32_t* cnt;              // [cap]
  uint32_t* rep;              // [n] distinct -> representative word
  uint32_t* slot;             // [n] distinct -> table slot
  unsigned long long* nu;     // distinct count; nu[1]: overflow flag
  uint64_t cap;
  uint32_t max_probe;         // DEDUP_MAX_PROBE, or unbounded when cap > n_words (never full)
};

// Table of the distinct words (keys + counts, 12 B a slot).  Round 4: sized for a quarter of the
// word occurrences, not twice them -- corpora of trajectories repeat their words (K5: 13 % distinct),
// and 2^24 slots (201 MB) stay in the 256 MB MALL where 2^27 (1.6 GB, round 3) made every probe an
// HBM round trip and took a 1.6 GB memset.  A table that fills up is detected (a probe run past
// DEDUP_MAX_PROBE slots sets the overflow flag, *out_n = -1) and the caller retries with a larger
// workspace: the capacity is the largest power of two the workspace holds.
constexpr int DEDUP_MAX_PROBE = 1024;
__host__ __device__ inline uint64_t dedup_cap(int64_t n) {
  uint64_t c = 1024;
  while (c < (uint64_t)n / 4) c <<= 1;
  return c;
}
__host__ __device__ inline size_t dedup_fixed_bytes(int64_t n) { return (size_t)(n > 0 ? n : 1) * 8 + 64; }

// One thread per word.  The table slot of the word's content is found as before; then the
// atomics that serialised at the memory side are aggregated.  New distinct words go to an LDS
// list (one LDS atomic per wave) that the workgroup appends to the global list with ONE device
// atomic when it is nearly full and at the end: the global list counter is a single address,
// and one atomic per wave on it (576 k at K5, each waiting on the previous at the memory side)
// took 7.2 ms of the 11.7 ms BPE setup.  Occurrence counts are summed per slot in an LDS hash
// (DEDUP_LDS entries, linear probing; a full probe falls back to the global atomic) and flushed
// once per workgroup -- the common words occur millions of times.
constexpr int DEDUP_LDS = 4096;
#ifndef DEDUP_NEW
#define DEDUP_NEW 1024            // LDS new-word list; flushed when a pass could overflow it
#endif
#ifndef DEDUP_T
// threads per workgroup: the LDS tables (41 KB) cap a CU at three workgroups, so 512 threads hold
// twice the waves of 256 for this chain of dependent loads (K5: 2.14 vs 2.83 ms per call;
// symbols loaded as aligned 16-byte blocks instead, 3.38 / 3.95 ms:
// profiles/r04/ab/bpe_dedup_ab_r04.txt)
#define DEDUP_T 512
#endif
__global__ __launch_bounds__(DEDUP_T) void k_dedup_insert(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                      const uint32_t* __restrict__ wlen, int64_t nw, DedupWs ws) {
  __shared__ uint32_t lkey[DEDUP_LDS];   // slot + 1, 0 = empty
  __shared__ uint32_t lcnt[DEDUP_LDS];
  __shared__ uint32_t nrep[DEDUP_NEW], nslot[DEDUP_NEW];
  __shared__ uint32_t ncnt;
  __shared__ unsigned long long nbase;
  for (int i = threadIdx.x; i < DEDUP_LDS; i += blockDim.x) { lkey[i] = 0; lcnt[i] = 0; }
  if (threadIdx.x == 0) ncnt = 0;
  __syncthreads();
  const uint64_t mask = ws.cap - 1;
  const int lane = threadIdx.x & 63;
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  // the workgroup's new words -> the global distinct list, one device atomic
  auto flush_new = [&]() {
    __syncthreads();
    const uint32_t n = ncnt;
    if (n) {
      if (threadIdx.x == 0) nbase = atomicAdd(ws.nu, (unsigned long long)n);
      __syncthreads();
      const unsigned long long b = nbase;
      for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        ws.rep[b + i] = nrep[i];
        ws.slot[b + i] = nslot[i];
      }
      __syncthreads();
      if (threadIdx.x == 0) ncnt = 0;
      __syncthreads();
    }
  };
  // workgroup-uniform trip count: every thread reaches the barriers of flush_new
  for (int64_t b0 = blockIdx.x * (int64_t)blockDim.x; b0 < nw; b0 += G) {
    const int64_t w = b0 + threadIdx.x;
    bool is_new = false;
    uint64_t k = 0;
    bool have = false;
    if (w < nw) {
      const uint32_t L = wlen[w];
      if (L >= 2) {
        have = true;
        const uint16_t* s = sym + wstart[w];
        const uint64_t h = word_hash(s, L);
        const unsigned long long mine = ((h >> 32) << 32) | (unsigned long long)(uint32_t)(w + 1);
        k = h & mask;
        for (int probe = 0;; ++probe) {
          if ((uint32_t)probe == ws.max_probe) {   // table too full: the caller retries with a larger one
            ws.nu[1] = 1ull;
            have = false;
            break;
          }
          unsigned long long v = ws.keys[k];
          if (v == 0ull) {
            v = atomicCAS(&ws.keys[k], 0ull, mine);
            if (v == 0ull) { is_new = true; break; }
          }
          if ((v >> 32) == (h >> 32)) {
            const uint32_t r = (uint32_t)(v & 0xFFFFFFFFull) - 1u;
            bool eq = wlen[r] == L;
            if (eq) {
              const uint16_t* t = sym + wstart[r];
              for (uint32_t i = 0; i < L && eq; ++i) eq = t[i] == s[i];
            }
            if (eq) break;
          }
          k = (k + 1) & mask;
        }
      }
    }
    // new distinct words -> the LDS list: one LDS atomic per wave
    const unsigned long long nb = __ballot(is_new);
    if (nb) {
      uint32_t base = 0;
      const int leader = __ffsll((long long)nb) - 1;
      if (lane == leader) base = atomicAdd(&ncnt, (uint32_t)__popcll(nb));
      base = __shfl(base, leader);
      if (is_new) {
        const uint32_t u = base + (uint32_t)__popcll(nb & ((1ull << lane) - 1ull));
        nrep[u] = (uint32_t)w;
        nslot[u] = (uint32_t)k;
      }
    }
    // occurrence count of slot k, aggregated in LDS
    if (have) {
      const uint32_t key = (uint32_t)k + 1u;
      uint32_t j = (key * 0x9E3779B1u) >> (32 - 12);
      bool done = false;
      for (int probe = 0; probe < 8 && !done; ++probe) {
        const uint32_t cur = atomicCAS(&lkey[j], 0u, key);
        if (cur == 0u || cur == key) { atomicAdd(&lcnt[j], 1u); done = true; }
        j = (j + 1) & (DEDUP_LDS - 1);
      }
      if (!done) atomicAdd(&ws.cnt[k], 1u);
    }
    __syncthreads();
    if (ncnt > (uint32_t)(DEDUP_NEW - DEDUP_T)) flush_new();   // the next pass adds <= DEDUP_T
  }
  flush_new();
  __syncthreads();
  for (int i = threadIdx.x; i < DEDUP_LDS; i += blockDim.x)
    if (lkey[i]) atomicAdd(&ws.cnt[lkey[i] - 1u], lcnt[i]);
}

__global__ __launch_bounds__(256) void k_dedup_gather(const uint32_t* __restrict__ wstart,
                                                      const uint32_t* __restrict__ wlen, DedupWs ws,
                                                      uint32_t* __restrict__ ow, uint32_t* __restrict__ ol,
                                                      uint32_t* __restrict__ oc, int64_t* __restrict__ out_n) {
  const int64_t nu = ws.nu[1] ? 0 : (int64_t)ws.nu[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_n = ws.nu[1] ? -1 : nu;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nu; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = ws.rep[i];
    ow[i] = wstart[r];
    ol[i] = wlen[r];
    oc[i] = ws.cnt[ws.slot[i]];
  }
}


// ---------------------------------------------- pre-tokenise + dedup, one pass --
// (round 5) HF's BpeTrainer trains on distinct words x counts, yet the pipeline above writes every
// word occurrence (K5: 36.9 M words, 210 MB of byte symbols and 295 MB of starts / lengths, after
// a counting pass and two scans) only for k_dedup_insert to read them back.  k_pretok_dedup
// pre-tokenises each sequence (one wave, k_pretok_wave's lane-parallel regex and word chain) and
// inserts its words straight into the distinct-word table.  A word is identified by its code
// points (UTF-8 and the byte -> symbol map are injective), so a table key is (22-bit hash tag,
// code-point length, token offset of the word's first occurrence) and a tag match is confirmed
// against that occurrence in the token array -- a read-only input, so no workgroup depends on
// bytes another one has just written.  Only the distinct words get byte symbols, in the repack
// (k_copy_words_cp).  Rows the lane-parallel pass does not take (over PT_LC code points, code
// points outside [0, 2^31), token offsets from 2^32) set a flag and the host runs the two-pass
// pipeline instead; a table that fills up sets another and the host retries with a larger one.
// (round 6) The distinct-word list is compacted from the table afterwards (k_pd_compact) instead
// of being flushed from per-wave LDS lists: 12 KB less LDS a workgroup, so three workgroups a CU
// (24 waves instead of 16) -- K5 setup kernels 2.95 -> 2.62 ms (profiles/r06/bpe_setup_ab_r06n.jsonl).
struct PdWs {
  unsigned long long* keys;   // [cap] tag << 42 | cp length << 32 | token offset; 0 = free
  uint32_t* cnt;              // [cap] occurrences per slot
  uint32_t* rep;              // [cap] distinct word -> token offset of its first occurrence
  uint32_t* lens;             // [cap] distinct word -> cp length << 16 | byte-symbol length
  uint32_t* slot;             // [cap] distinct word -> table slot
  uint32_t* slens;            // [cap] slot -> cp length << 16 | byte-symbol length
  unsigned long long* info;   // [4] distinct words, words, byte symbols, flags (PD_OVERFLOW | PD_UNSUPPORTED)
  uint64_t cap;
  uint32_t max_probe;
  int tag_bits;               // 22, or fewer (tests force tag collisions)
};
constexpr unsigned long long PD_OVERFLOW = 1, PD_UNSUPPORTED = 2, PD_LONG = 4;
constexpr int PD_LDS = 2048;    // per-workgroup LDS occurrence counts (slot -> count)
constexpr int PD_WAVES = 8;     // rows (waves) per workgroup
constexpr int PD_GRID = 3;      // workgroups a CU: all resident at once (49 KB of LDS each)

__device__ __forceinline__ uint64_t cp_hash(const int32_t* cps, int cs, int ce) {
  uint64_t h = 0xcbf29ce484222325ull ^ (uint64_t)(ce - cs);
  for (int i = cs; i < ce; ++i) h = (h ^ (uint32_t)cps[i]) * 0x100000001b3ull;
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
  return h;
}

// LC: the longest row the LDS image holds (256 first: three workgroups of 8 waves a CU for BEAST's
// rows of D * N bins; a longer row flags PD_LONG and the host reruns with 512)
template <int LC>
__global__ __launch_bounds__(64 * PD_WAVES) void k_pretok_dedup(const long long* __restrict__ tok,
                                                              const int64_t* __restrict__ seq_off, int64_t n_seq,
                                                              long long mn, const uint8_t* __restrict__ lut,
                                                              int64_t lut_n, PdWs ws) {
  __shared__ PtLdsT<LC> lds[PD_WAVES];
  __shared__ uint8_t s_lut[256];
  __shared__ uint32_t lkey[PD_LDS], lcnt[PD_LDS];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_lut[i] = i < lut_n ? lut[i] : (uint8_t)CLS_OTHER;
  for (int i = threadIdx.x; i < PD_LDS; i += blockDim.x) { lkey[i] = 0; lcnt[i] = 0; }
  __syncthreads();
  PtLdsT<LC>& L = lds[wv];
  const uint64_t mask = ws.cap - 1;
  const uint32_t tag_mask = (1u << ws.tag_bits) - 1u;
  unsigned long long nwords = 0, nsyms = 0;
  constexpr int PF = LC / 64;
  // the 512 kernel runs after the 256 one and takes only the rows that one left (257..512 code
  // points); it returns at once when there were none (the flag, a kernel boundary ago)
  if (LC > 256 && !(ws.info[3] & PD_LONG)) return;   // uniform: before any barrier
  for (int64_t sidx = (int64_t)blockIdx.x * PD_WAVES + wv; sidx < n_seq; sidx += (int64_t)gridDim.x * PD_WAVES) {
    const int64_t r0 = seq_off[sidx], n64 = seq_off[sidx + 1] - r0;
    if (LC > 256 && n64 <= 256) continue;   // the 256 kernel's
    if (LC == 256 && n64 > LC && n64 <= PT_LC) {   // wave-uniform: the 512-code-point kernel takes it
      if (lane == 0) atomicOr(&ws.info[3], PD_LONG);
      continue;
    }
    bool bad = n64 > LC || r0 + n64 > 0xFFFFFFFFll;
    const int n = bad ? 0 : (int)n64;
    // 1. code points, classes, UTF-8 symbol offsets (k_pretok_wave)
    long long tv[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) tv[k] = (lane + 64 * k < n) ? tok[r0 + lane + 64 * k] : 0;
    int carry = 0;
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      if (64 * k >= n) break;
      const int i = 64 * k + lane;
      int len = 0;
      if (i < n) {
        const long long c = tv[k] - mn;
        bad |= (c < 0) | (c > 0x7FFFFFFFLL);
        L.cp[i] = (int32_t)c;
        L.cls[i] = (c >= 0 && c < 256) ? s_lut[c] : (c >= 0 && c < lut_n) ? lut[c] : (uint8_t)CLS_OTHER;
        len = utf8_len(c);
      }
      int tot;
      const int ex = beast_pt::wave_excl_scan(len, lane, tot);
      if (i < n) L.so[i] = (int16_t)(carry + ex);
      carry += tot;
    }
    if (__any(bad)) {   // wave-uniform: the host takes the two-pass path
      if (lane == 0) atomicOr(&ws.info[3], PD_UNSUPPORTED);
      continue;
    }
    if (lane == 0) L.so[n] = (int16_t)carry;
    pt_wave_sync();
    // 2. word ends, 3. the word chain (csrc/pretok.h)
    beast_pt::regex_ends(L.cp, L.cls, L.wcp, L.e, n, lane);
    beast_pt::word_starts(L.e, L.vis, L.wcp, nullptr, &L.nw, n, lane);
    const int nw = L.nw;
    nwords += nw;
    nsyms += carry;
    // 4. the sequence's words into the distinct-word table, a lane per word
    for (int wb = 0; wb < nw; wb += 64) {
      const int w = wb + lane;
      bool have = false, is_new = false;
      uint64_t k = 0;
      uint32_t lens = 0;
      if (w < nw) {
        const int cs = L.wcp[w], ce = L.wcp[w + 1];
        const int blen = L.so[ce] - L.so[cs];
        if (blen >= 2) {
          have = true;
          const int cl = ce - cs;
          lens = ((uint32_t)cl << 16) | (uint32_t)blen;
          const uint64_t h = cp_hash(L.cp, cs, ce);
          const unsigned long long hi = ((unsigned long long)((uint32_t)(h >> 40) & tag_mask) << 42) |
                                        ((unsigned long long)cl << 32);
          const unsigned long long mine = hi | (unsigned long long)(uint32_t)(r0 + cs);
          k = h & mask;
          for (uint32_t probe = 0;; ++probe) {
            if (probe == ws.max_probe) {   // table too full: the host retries with a larger one
              atomicOr(&ws.info[3], PD_OVERFLOW);
              have = false;
              break;
            }
            unsigned long long v = ws.keys[k];
            if (v == 0ull) {
              v = atomicCAS(&ws.keys[k], 0ull, mine);
              if (v == 0ull) { is_new = true; break; }
            }
            if ((v >> 32) == (hi >> 32)) {   // same tag and length: compare the code points
              const long long* o = tok + (uint32_t)v;
              bool eq = true;
              for (int i = 0; i < cl && eq; ++i) eq = (o[i] - mn) == (long long)L.cp[cs + i];
              if (eq) break;
            }
            k = (k + 1) & mask;
          }
        }
      }
      if (is_new) ws.slens[k] = lens;   // the distinct-word list is compacted from the table afterwards
      // the occurrence, counted in LDS (the frequent words occur millions of times)
      if (have) {
        const uint32_t key = (uint32_t)k + 1u;
        uint32_t j = (key * 0x9E3779B1u) >> (32 - __builtin_ctz(PD_LDS));
        bool done = false;
        for (int probe = 0; probe < 8 && !done; ++probe) {
          const uint32_t cur = atomicCAS(&lkey[j], 0u, key);
          if (cur == 0u || cur == key) { atomicAdd(&lcnt[j], 1u); done = true; }
          j = (j + 1) & (PD_LDS - 1);
        }
        if (!done) atomicAdd(&ws.cnt[k], 1u);
      }
    }
    pt_wave_sync();   // LDS is reused by the next sequence
  }
  if (lane == 0) {
    atomicAdd(&ws.info[1], nwords);
    atomicAdd(&ws.info[2], nsyms);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < PD_LDS; i += blockDim.x)
    if (lkey[i]) atomicAdd(&ws.cnt[lkey[i] - 1u], lcnt[i]);
}

// the distinct-word list from the table: 4,096 slots a workgroup (16 a thread, coalesced), one
// atomic a workgroup for its place in the list
constexpr int PDC_PER = 16;
__global__ __launch_bounds__(256) void k_pd_compact(PdWs ws) {
  __shared__ uint32_t wtot[4];
  __shared__ unsigned long long gbase;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * (256 * PDC_PER);
  unsigned long long key[PDC_PER];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < PDC_PER; ++j) {
    const uint64_t sl = base + (uint64_t)j * 256 + threadIdx.x;
    key[j] = sl < ws.cap ? ws.keys[sl] : 0ull;
    cnt += (int)__popcll(__ballot(key[j] != 0ull));
  }
  if (lane == 0) wtot[wv] = (uint32_t)cnt;
  __syncthreads();
  if (threadIdx.x == 0) gbase = atomicAdd(&ws.info[0], (unsigned long long)(wtot[0] + wtot[1] + wtot[2] + wtot[3]));
  __syncthreads();
  unsigned long long o = gbase;
  for (int i = 0; i < wv; ++i) o += wtot[i];
#pragma unroll
  for (int j = 0; j < PDC_PER; ++j) {
    const uint64_t sl = base + (uint64_t)j * 256 + threadIdx.x;
    const unsigned long long m = __ballot(key[j] != 0ull);
    if (key[j] != 0ull) {
      const unsigned long long i = o + __popcll(m & ((1ull << lane) - 1ull));
      ws.rep[i] = (uint32_t)key[j];
      ws.lens[i] = ws.slens[sl];
      ws.slot[i] = (uint32_t)sl;
    }
    o += __popcll(m);
  }
}

// distinct word i -> (token offset, byte length, count) for the repack
__global__ __launch_bounds__(256) void k_pd_gather(PdWs ws, int64_t nu, uint32_t* __restrict__ ol,
                                                    uint32_t* __restrict__ oc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nu; i += (int64_t)gridDim.x * blockDim.x) {
    ol[i] = ws.lens[i] & 0xFFFFu;
    oc[i] = ws.cnt[ws.slot[i]];
  }
}

// keep the words that can still merge (>= 2 symbols); one atomic per wave
__global__ __launch_bounds__(256) void k_compact_words(const uint32_t* __restrict__ wstart,
                                                       const uint32_t* __restrict__ wlen,
                                                       const uint32_t* __restrict__ wcount, int64_t nw,
                                                       uint32_t* __restrict__ ow, uint32_t* __restrict__ ol,
                                                       uint32_t* __restrict__ oc, unsigned long long* __restrict__ n) {
  const int lane = threadIdx.x & 63;
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < nw; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = base + threadIdx.x;
    const bool keep = w < nw && wlen[w] >= 2;
    const unsigned long long m = __ballot(keep);
    unsigned long long off = 0;
    if (lane == 0 && m) off = atomicAdd(n, (unsigned long long)__popcll(m));
    off = __shfl(off, 0);
    if (keep) {
      const unsigned long long pos = off + __popcll(m & ((1ull << lane) - 1ull));
      ow[pos] = wstart[w];
      ol[pos] = wlen[w];
      oc[pos] = wcount ? wcount[w] : 1u;
    }
  }
}

// ------------------------------------------------------------ word repack --
// Distinct words copied into one contiguous symbol array ordered by length (bucket
// min(L, 255)): a wave's words are neighbours in memory and of similar length, so the
// merge scan is coalesced and its per-thread loops stay in step.  Each word starts at a
// multiple of 4 symbols and owns its span rounded up to 4: the merge loop reads and writes
// a word as 8-byte units that no other word shares.
constexpr int RP_WPB = 2048;   // words per workgroup in the bucket scatter

__global__ __launch_bounds__(256) void k_len_hist(const uint32_t* __restrict__ wlen, int64_t nw,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&h[min(wlen[w], 255u)], 1u);
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_bucket_scan(const uint32_t* __restrict__ hist, uint32_t* __restrict__ cursor) {
  __shared__ uint32_t v[256];
  v[threadIdx.x] = hist[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < 256; ++i) { const uint32_t c = v[i]; v[i] = acc; acc += c; }
  }
  __syncthreads();
  cursor[threadIdx.x] = v[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_len_scatter(const uint32_t* __restrict__ wlen, int64_t nw,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ order) {
  __shared__ uint32_t h[256], base[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t w0 = (int64_t)blockIdx.x * RP_WPB;
  uint32_t bk[RP_WPB / 256], rk[RP_WPB / 256];
#pragma unroll
  for (int k = 0; k < RP_WPB / 256; ++k) {
    const int64_t w = w0 + k * 256 + threadIdx.x;
    bk[k] = w < nw ? min(wlen[w], 255u) : 0u;
    rk[k] = w < nw ? atomicAdd(&h[bk[k]], 1u) : 0u;
  }
  __syncthreads();
  base[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], h[threadIdx.x]) : 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RP_WPB / 256; ++k) {
    const int64_t w = w0 + k * 256 + threadIdx.x;
    if (w < nw) order[base[bk[k]] + rk[k]] = (uint32_t)w;
  }
}

__global__ __launch_bounds__(256) void k_gather_lens(const uint32_t* __restrict__ order, const uint32_t* __restrict__ wlen,
                                                     const uint32_t* __restrict__ wcount, int64_t nw,
                                                     int64_t* __restrict__ lens, uint32_t* __restrict__ ol,
                                                     uint32_t* __restrict__ oc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = order[i];
    lens[i] = (wlen[w] + 3u) & ~3u;   // the word's span: 4-symbol (8-byte) units of its own
    ol[i] = wlen[w];
    oc[i] = wcount ? wcount[w] : 1u;
  }
}

__global__ __launch_bounds__(256) void k_copy_words(const uint32_t* __restrict__ order, const uint16_t* __restrict__ sym,
                                                    const uint32_t* __restrict__ wstart, const uint32_t* __restrict__ wlen,
                                                    const int64_t* __restrict__ offs, int64_t nw,
                                                    uint16_t* __restrict__ osym, uint32_t* __restrict__ ow,
                                                    int64_t* __restrict__ out_nsym) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = order[i], L = wlen[w];
    const uint16_t* src = sym + wstart[w];
    uint16_t* dst = osym + offs[i];
    for (uint32_t k = 0; k < L; ++k) dst[k] = src[k];
    for (uint32_t k = L; k & 3u; ++k) dst[k] = 0;   // the span's padding (never a symbol of the word)
    ow[i] = (uint32_t)offs[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_nsym = offs[nw];
}

// k_copy_words for the one-pass setup: a distinct word's byte symbols from its first occurrence's
// code points (UTF-8 bytes -> vocab ids), same layout (length order, spans of 4)
__global__ __launch_bounds__(256) void k_copy_words_cp(const uint32_t* __restrict__ order, const long long* __restrict__ tok,
                                                       long long mn, const uint16_t* __restrict__ byte2id,
                                                       const uint32_t* __restrict__ rep, const uint32_t* __restrict__ lens,
                                                       const int64_t* __restrict__ offs, int64_t nw,
                                                       uint16_t* __restrict__ osym, uint32_t* __restrict__ ow,
                                                       int64_t* __restrict__ out_nsym) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = order[i], cl = lens[w] >> 16;
    const long long* src = tok + rep[w];
    uint16_t* dst = osym + offs[i];
    uint32_t o = 0;
    auto emit = [&](long long t) {
      uint8_t b[4];
      const long long cp = t - mn;
      const int Lb = utf8_len(cp);
      utf8_bytes(cp, b);
      for (int q = 0; q < Lb; ++q) dst[o++] = byte2id[b[q]];
    };
    constexpr int CP_REG = 12;   // the first code points' loads all in flight (99.9 % of K5's words)
    long long c[CP_REG];
#pragma unroll
    for (int k = 0; k < CP_REG; ++k) c[k] = (uint32_t)k < cl ? src[k] : 0;
#pragma unroll
    for (int k = 0; k < CP_REG; ++k)
      if ((uint32_t)k < cl) emit(c[k]);
    for (uint32_t k = CP_REG; k < cl; ++k) emit(src[k]);
    for (; o & 3u; ++o) dst[o] = 0;   // the span's padding (never a symbol of the word)
    ow[i] = (uint32_t)offs[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_nsym = offs[nw];
}

__global__ __launch_bounds__(256) void k_word_sig(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                  const uint32_t* __restrict__ wlen, int64_t nw,
                                                  unsigned long long* __restrict__ sig) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const uint16_t* s = sym + wstart[w];
    sig[w] = sig_of([&](uint32_t i) { return (uint32_t)s[i]; }, wlen[w]);
  }
}

}  // namespace


// =================================================================== C-ABI ==
extern "C" int beast_i64_minmax(const int64_t* x, int64_t n, int64_t* out2, void* stream) {
  BEAST_REQUIRE(x && out2 && n >= 1, "beast_i64_minmax: bad args");
  hipStream_t s = beast::as_stream(stream);
  hipLaunchKernelGGL(k_minmax_init, dim3(1), dim3(1), 0, s, reinterpret_cast<long long*>(out2));
  hipLaunchKernelGGL(k_minmax, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, reinterpret_cast<const long long*>(x),
                     n, reinterpret_cast<long long*>(out2));
  BEAST_LAUNCHED("k_minmax");
  return BEAST_OK;
}

extern "C" int beast_bpe_cp_presence(const int64_t* tok, int64_t n, int64_t min_tok, uint8_t* present, int64_t n_cp,
                                     void* stream) {
  BEAST_REQUIRE(tok && present && n >= 0 && n_cp >= 1, "beast_bpe_cp_presence: bad args");
  hipStream_t s = beast::as_stream(stream);
  BEAST_HIP(hipMemsetAsync(present, 0, (size_t)n_cp, s), "presence memset");
  if (n == 0) return BEAST_OK;
  hipLaunchKernelGGL(k_presence, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s,
                     reinterpret_cast<const long long*>(tok), n, (long long)min_tok, present, n_cp);
  BEAST_LAUNCHED("k_presence");
  return BEAST_OK;
}

extern "C" int beast_bpe_pretok_count(const int64_t* tok, const int64_t* seq_off, int64_t n_seq, int64_t min_tok,
                                      const uint8_t* cls_lut, int64_t lut_n, int64_t* words_per_seq,
                                      int64_t* syms_per_seq, void* stream) {
  BEAST_REQUIRE(tok && seq_off && cls_lut && words_per_seq && syms_per_seq, "beast_bpe_pretok_count: null pointer");
  if (n_seq <= 0) return BEAST_OK;
  hipLaunchKernelGGL(k_pretok_wave<false>, dim3(grid_for(n_seq, PT_WAVES, 16384)), dim3(64 * PT_WAVES), 0,
                     beast::as_stream(stream),
                     reinterpret_cast<const long long*>(tok), seq_off, n_seq, (long long)min_tok, cls_lut, lut_n,
                     words_per_seq, syms_per_seq, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
  BEAST_LAUNCHED("k_pretok<count>");
  return BEAST_OK;
}

extern "C" size_t beast_scan_workspace_bytes(int64_t n) { return (size_t)scan_ws_elems(n) * sizeof(int64_t); }

extern "C" int beast_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* workspace, void* stream) {
  BEAST_REQUIRE(in && out && workspace && n >= 0, "beast_exclusive_scan_i64: bad args");
  hipStream_t s = beast::as_stream(stream);
  if (n > 0) {
    int rc = scan_rec(in, out, n, reinterpret_cast<int64_t*>(workspace), s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(64), 0, s, in, out, n);
  BEAST_LAUNCHED("k_scan_total");
  return BEAST_OK;
}

extern "C" int beast_bpe_pretok_emit(const int64_t* tok, const int64_t* seq_off, int64_t n_seq, int64_t min_tok,
                                     const uint8_t* cls_lut, int64_t lut_n, const int64_t* word_off,
                                     const int64_t* sym_off, const uint16_t* byte2id, uint16_t* sym,
                                     uint32_t* wstart, uint32_t* wlen, void* stream) {
  BEAST_REQUIRE(tok && seq_off && cls_lut && word_off && sym_off && byte2id && sym && wstart && wlen,
                "beast_bpe_pretok_emit: null pointer");
  if (n_seq <= 0) return BEAST_OK;
  hipLaunchKernelGGL(k_pretok_wave<true>, dim3(grid_for(n_seq, PT_WAVES, 16384)), dim3(64 * PT_WAVES), 0,
                     beast::as_stream(stream),
                     reinterpret_cast<const long long*>(tok), seq_off, n_seq, (long long)min_tok, cls_lut, lut_n,
                     nullptr, nullptr, word_off, sym_off, byte2id, sym, wstart, wlen);
  BEAST_LAUNCHED("k_pretok<emit>");
  return BEAST_OK;
}

extern "C" int beast_bpe_count_pairs(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen,
                                     const uint32_t* wcount, int64_t n_words, uint32_t* table, int Vt, int n_sym,
                                     void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && table && Vt >= 1 && Vt <= 65535, "beast_bpe_count_pairs: bad args");
  BEAST_REQUIRE(n_sym >= 0 && n_sym <= Vt, "beast_bpe_count_pairs: n_sym %d not in [0, Vt]", n_sym);
  if (n_words <= 0) return BEAST_OK;
  hipStream_t s = beast::as_stream(stream);
  const size_t budget = 160 * 1024;
  const int R = n_sym > 0 ? (int)std::min<size_t>((size_t)n_sym, budget / (4 * (size_t)n_sym)) : 0;
  const int groups = R > 0 ? (n_sym + R - 1) / R : 0;
  if (R > 0 && groups <= 16) {   // LDS-privatised (the words are read once per row group)
    const size_t lds = (size_t)R * n_sym * 4;
    if (lds > 65536)
      BEAST_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_count_pairs_lds),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                "hipFuncSetAttribute(k_count_pairs_lds)");
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    const int per_cu = std::max(1, (int)(budget / std::max<size_t>(lds, 1)));
    const int gx = std::max(1, std::min<int>(cus * per_cu / groups, (int)((n_words + 255) / 256)));
    hipLaunchKernelGGL(k_count_pairs_lds, dim3(gx, groups), dim3(256), lds, s, sym, wstart, wlen, wcount, n_words,
                       table, Vt, n_sym, R);
    BEAST_LAUNCHED("k_count_pairs_lds");
    return BEAST_OK;
  }
  hipLaunchKernelGGL(k_count_pairs, dim3(grid_for(n_words, 256, 8192)), dim3(256), 0, s, sym,
                     wstart, wlen, wcount, n_words, table, Vt);
  BEAST_LAUNCHED("k_count_pairs");
  return BEAST_OK;
}

extern "C" int beast_bpe_word_signatures(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen,
                                         int64_t n_words, uint64_t* sig, void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && sig && n_words >= 0, "beast_bpe_word_signatures: bad args");
  if (n_words == 0) return BEAST_OK;
  hipLaunchKernelGGL(k_word_sig, dim3(grid_for(n_words, 256, 8192)), dim3(256), 0, beast::as_stream(stream), sym,
                     wstart, wlen, n_words, reinterpret_cast<unsigned long long*>(sig));
  BEAST_LAUNCHED("k_word_sig");
  return BEAST_OK;
}

extern "C" size_t beast_bpe_dedup_workspace_bytes(int64_t n_words) {
  return (size_t)(dedup_cap(n_words > 0 ? n_words : 1) * 12) + dedup_fixed_bytes(n_words);
}
// a table of >= 2 n_words slots: it can never fill, so the probes are unbounded and *out_n is
// always the distinct count (no retry)
extern "C" size_t beast_bpe_dedup_workspace_bytes_safe(int64_t n_words) {
  uint64_t c = 1024;
  while (c < 2 * (uint64_t)(n_words > 0 ? n_words : 1)) c <<= 1;
  return (size_t)(c * 12) + dedup_fixed_bytes(n_words);
}
extern "C" int beast_bpe_dedup_words(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen,
                                     int64_t n_words, void* workspace, size_t ws_bytes, uint32_t* out_wstart,
                                     uint32_t* out_wlen, uint32_t* out_wcount, int64_t* out_n, void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && workspace && out_wstart && out_wlen && out_wcount && out_n,
                "beast_bpe_dedup_words: null pointer");
  BEAST_REQUIRE(n_words >= 0 && n_words < (int64_t(1) << 32) - 1, "beast_bpe_dedup_words: bad n_words");
  BEAST_REQUIRE_CODE(ws_bytes >= beast_bpe_dedup_workspace_bytes(n_words), BEAST_E_WORKSPACE,
                     "dedup workspace %zu < %zu", ws_bytes, beast_bpe_dedup_workspace_bytes(n_words));
  hipStream_t s = beast::as_stream(stream);
  const int64_t n = n_words > 0 ? n_words : 1;
  DedupWs ws;
  ws.cap = 1024;   // the largest power of two the workspace holds
  while ((ws.cap * 2) * 12 + dedup_fixed_bytes(n_words) <= ws_bytes) ws.cap *= 2;
  ws.max_probe = ws.cap > (uint64_t)n_words ? 0xFFFFFFFFu : (uint32_t)DEDUP_MAX_PROBE;
  char* p = static_cast<char*>(workspace);
  ws.keys = reinterpret_cast<unsigned long long*>(p);  p += ws.cap * 8;
  ws.cnt = reinterpret_cast<uint32_t*>(p);              p += ws.cap * 4;
  ws.rep = reinterpret_cast<uint32_t*>(p);              p += n * 4;
  ws.slot = reinterpret_cast<uint32_t*>(p);             p += n * 4;
  ws.nu = reinterpret_cast<unsigned long long*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
  BEAST_HIP(hipMemsetAsync(workspace, 0, ws.cap * 12, s), "dedup memset");
  BEAST_HIP(hipMemsetAsync(ws.nu, 0, 16, s), "dedup memset");
  if (n_words > 0) {
    hipLaunchKernelGGL(k_dedup_insert, dim3(grid_for(n_words, DEDUP_T, 16384 * 256 / DEDUP_T)), dim3(DEDUP_T), 0, s,
                       sym, wstart, wlen,
                       n_words, ws);
    BEAST_LAUNCHED("k_dedup_insert");
  }
  hipLaunchKernelGGL(k_dedup_gather, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, wstart, wlen, ws, out_wstart,
                     out_wlen, out_wcount, out_n);
  BEAST_LAUNCHED("k_dedup_gather");
  return BEAST_OK;
}

// ---- one-pass setup (k_pretok_dedup): the table and the distinct-word list in one workspace
static uint64_t pd_cap(int64_t n_tokens) {   // ~ n_tokens / 5 slots (K5: 4.85 M distinct words of 7e7 tokens)
  uint64_t c = 1024;
  while (c < (uint64_t)std::max<int64_t>(n_tokens, 1) / 5) c <<= 1;
  return c;
}
constexpr uint64_t PD_SLOT_BYTES = 28;   // keys 8, cnt 4, rep 4, lens 4, slot 4, slens 4
static PdWs pd_view(void* workspace, size_t ws_bytes) {
  PdWs w{};
  w.cap = 1024;   // the largest power of two the workspace holds (PD_SLOT_BYTES a slot)
  while ((w.cap * 2) * PD_SLOT_BYTES + 64 <= ws_bytes) w.cap *= 2;
  char* p = static_cast<char*>(workspace);
  w.keys = reinterpret_cast<unsigned long long*>(p);  p += w.cap * 8;
  w.cnt = reinterpret_cast<uint32_t*>(p);             p += w.cap * 4;
  w.rep = reinterpret_cast<uint32_t*>(p);             p += w.cap * 4;
  w.lens = reinterpret_cast<uint32_t*>(p);            p += w.cap * 4;
  w.slot = reinterpret_cast<uint32_t*>(p);            p += w.cap * 4;
  w.slens = reinterpret_cast<uint32_t*>(p);           p += w.cap * 4;
  w.info = reinterpret_cast<unsigned long long*>(p);
  w.max_probe = DEDUP_MAX_PROBE;
  w.tag_bits = std::min(22, std::max(1, beast::g_bpe_dedup_key_bits));
  return w;
}
extern "C" size_t beast_bpe_pretok_dedup_workspace_bytes(int64_t n_tokens) { return pd_cap(n_tokens) * PD_SLOT_BYTES + 64; }

extern "C" int beast_bpe_pretok_dedup(const int64_t* tok, const int64_t* seq_off, int64_t n_seq, int64_t min_tok,
                                      const uint8_t* cls_lut, int64_t lut_n, void* workspace, size_t ws_bytes,
                                      int64_t* out_info, void* stream) {
  BEAST_REQUIRE(tok && seq_off && cls_lut && workspace && out_info, "beast_bpe_pretok_dedup: null pointer");
  BEAST_REQUIRE(n_seq >= 0 && ws_bytes >= 1024 * PD_SLOT_BYTES + 64, "beast_bpe_pretok_dedup: bad sizes");
  hipStream_t s = beast::as_stream(stream);
  PdWs w = pd_view(workspace, ws_bytes);
  BEAST_HIP(hipMemsetAsync(w.keys, 0, w.cap * 12, s), "pretok_dedup memset");   // keys + counts
  BEAST_HIP(hipMemsetAsync(w.info, 0, 32, s), "pretok_dedup memset");
  if (n_seq > 0) {
    // the waves walk the sequences grid-stride; rows of <= 256 code points first (49 KB of LDS a
    // workgroup), rows of 257..512 by the 512 kernel only when some row needs it
    hipLaunchKernelGGL(k_pretok_dedup<256>, dim3(grid_for(n_seq, PD_WAVES, PD_GRID * 256)), dim3(64 * PD_WAVES), 0, s,
                       reinterpret_cast<const long long*>(tok), seq_off, n_seq, (long long)min_tok, cls_lut, lut_n, w);
    BEAST_LAUNCHED("k_pretok_dedup<256>");
    hipLaunchKernelGGL(k_pretok_dedup<PT_LC>, dim3(grid_for(n_seq, PD_WAVES, 2 * 256)), dim3(64 * PD_WAVES), 0, s,
                       reinterpret_cast<const long long*>(tok), seq_off, n_seq, (long long)min_tok, cls_lut, lut_n, w);
    BEAST_LAUNCHED("k_pretok_dedup<512>");
    hipLaunchKernelGGL(k_pd_compact, dim3((unsigned)((w.cap + 256 * PDC_PER - 1) / (256 * PDC_PER))), dim3(256), 0, s, w);
    BEAST_LAUNCHED("k_pd_compact");
  }
  BEAST_HIP(hipMemcpyAsync(out_info, w.info, 32, hipMemcpyDeviceToDevice, s), "pretok_dedup info");
  return BEAST_OK;
}

extern "C" int beast_bpe_pretok_dedup_repack(const int64_t* tok, int64_t min_tok, const uint16_t* byte2id,
                                             void* workspace, size_t ws_bytes, int64_t n_distinct, void* repack_ws,
                                             size_t repack_ws_bytes, uint16_t* out_sym, uint32_t* out_wstart,
                                             uint32_t* out_wlen, uint32_t* out_wcount, int64_t* out_nsym,
                                             void* stream) {
  BEAST_REQUIRE(tok && byte2id && workspace && repack_ws && out_sym && out_wstart && out_wlen && out_wcount && out_nsym,
                "beast_bpe_pretok_dedup_repack: null pointer");
  PdWs w = pd_view(workspace, ws_bytes);
  BEAST_REQUIRE(n_distinct >= 0 && (uint64_t)n_distinct <= w.cap, "beast_bpe_pretok_dedup_repack: bad n_distinct");
  BEAST_REQUIRE_CODE(repack_ws_bytes >= beast_bpe_repack_workspace_bytes(n_distinct) + 8 * (size_t)(n_distinct + 1),
                     BEAST_E_WORKSPACE, "repack workspace %zu too small", repack_ws_bytes);
  hipStream_t s = beast::as_stream(stream);
  const int64_t n = n_distinct > 0 ? n_distinct : 1;
  char* p = static_cast<char*>(repack_ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(p);   p += 256 * 4;
  uint32_t* cursor = reinterpret_cast<uint32_t*>(p); p += 256 * 4;
  uint32_t* order = reinterpret_cast<uint32_t*>(p);  p += n * 4;
  p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
  int64_t* lens = reinterpret_cast<int64_t*>(p);     p += n * 8;
  int64_t* offs = reinterpret_cast<int64_t*>(p);     p += (n + 1) * 8;
  int64_t* sws = reinterpret_cast<int64_t*>(p);      p += beast_scan_workspace_bytes(n);
  p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
  uint32_t* blen = reinterpret_cast<uint32_t*>(p);   p += n * 4;   // byte lengths / counts before the sort
  uint32_t* cnt = reinterpret_cast<uint32_t*>(p);
  BEAST_HIP(hipMemsetAsync(hist, 0, 256 * 4, s), "repack memset");
  if (n_distinct == 0) {
    BEAST_HIP(hipMemsetAsync(out_nsym, 0, 8, s), "repack memset");
    return BEAST_OK;
  }
  const int g = grid_for(n_distinct, 256, 8192);
  hipLaunchKernelGGL(k_pd_gather, dim3(g), dim3(256), 0, s, w, n_distinct, blen, cnt);
  hipLaunchKernelGGL(k_len_hist, dim3(g), dim3(256), 0, s, blen, n_distinct, hist);
  hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(256), 0, s, hist, cursor);
  hipLaunchKernelGGL(k_len_scatter, dim3((n_distinct + RP_WPB - 1) / RP_WPB), dim3(256), 0, s, blen, n_distinct, cursor,
                     order);
  hipLaunchKernelGGL(k_gather_lens, dim3(g), dim3(256), 0, s, order, blen, cnt, n_distinct, lens, out_wlen, out_wcount);
  BEAST_LAUNCHED("k_gather_lens");
  int rc = scan_rec(lens, offs, n_distinct, sws, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(64), 0, s, lens, offs, n_distinct);
  hipLaunchKernelGGL(k_copy_words_cp, dim3(g), dim3(256), 0, s, order, reinterpret_cast<const long long*>(tok),
                     (long long)min_tok, byte2id, w.rep, w.lens, offs, n_distinct, out_sym, out_wstart, out_nsym);
  BEAST_LAUNCHED("k_copy_words_cp");
  return BEAST_OK;
}

extern "C" int beast_bpe_compact_words(const uint32_t* wstart, const uint32_t* wlen, const uint32_t* wcount,
                                       int64_t n_words, uint32_t* out_wstart, uint32_t* out_wlen,
                                       uint32_t* out_wcount, int64_t* out_n, void* stream) {
  BEAST_REQUIRE(wstart && wlen && out_wstart && out_wlen && out_wcount && out_n,
                "beast_bpe_compact_words: null pointer");
  BEAST_REQUIRE(n_words >= 0, "beast_bpe_compact_words: bad n_words");
  hipStream_t s = beast::as_stream(stream);
  BEAST_HIP(hipMemsetAsync(out_n, 0, 8, s), "compact memset");
  if (n_words > 0) {
    hipLaunchKernelGGL(k_compact_words, dim3(grid_for(n_words, 256, 16384)), dim3(256), 0, s, wstart, wlen, wcount,
                       n_words, out_wstart, out_wlen, out_wcount, reinterpret_cast<unsigned long long*>(out_n));
    BEAST_LAUNCHED("k_compact_words");
  }
  return BEAST_OK;
}

extern "C" size_t beast_bpe_repack_workspace_bytes(int64_t n_words) {
  const int64_t n = n_words > 0 ? n_words : 1;
  return (size_t)(2 * 256 * 4 + n * 4 + n * 8 + (n + 1) * 8 + 64) + beast_scan_workspace_bytes(n);
}

extern "C" int beast_bpe_repack_words(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen,
                                      const uint32_t* wcount, int64_t n_words, void* workspace, size_t ws_bytes,
                                      uint16_t* out_sym, uint32_t* out_wstart, uint32_t* out_wlen,
                                      uint32_t* out_wcount, int64_t* out_nsym, void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && workspace && out_sym && out_wstart && out_wlen && out_wcount && out_nsym,
                "beast_bpe_repack_words: null pointer");
  BEAST_REQUIRE(n_words >= 0 && n_words < (int64_t(1) << 31), "beast_bpe_repack_words: bad n_words");
  BEAST_REQUIRE_CODE(ws_bytes >= beast_bpe_repack_workspace_bytes(n_words), BEAST_E_WORKSPACE,
                     "repack workspace %zu < %zu", ws_bytes, beast_bpe_repack_workspace_bytes(n_words));
  hipStream_t s = beast::as_stream(stream);
  const int64_t n = n_words > 0 ? n_words : 1;
  char* p = static_cast<char*>(workspace);
  uint32_t* hist = reinterpret_cast<uint32_t*>(p);   p += 256 * 4;
  uint32_t* cursor = reinterpret_cast<uint32_t*>(p); p += 256 * 4;
  uint32_t* order = reinterpret_cast<uint32_t*>(p);  p += n * 4;
  p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
  int64_t* lens = reinterpret_cast<int64_t*>(p);     p += n * 8;
  int64_t* offs = reinterpret_cast<int64_t*>(p);     p += (n + 1) * 8;
  int64_t* sws = reinterpret_cast<int64_t*>(p);
  BEAST_HIP(hipMemsetAsync(hist, 0, 256 * 4, s), "repack memset");
  if (n_words == 0) {
    BEAST_HIP(hipMemsetAsync(out_nsym, 0, 8, s), "repack memset");
    return BEAST_OK;
  }
  const int g = grid_for(n_words, 256, 8192);
  hipLaunchKernelGGL(k_len_hist, dim3(g), dim3(256), 0, s, wlen, n_words, hist);
  hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(256), 0, s, hist, cursor);
  hipLaunchKernelGGL(k_len_scatter, dim3((n_words + RP_WPB - 1) / RP_WPB), dim3(256), 0, s, wlen, n_words, cursor, order);
  hipLaunchKernelGGL(k_gather_lens, dim3(g), dim3(256), 0, s, order, wlen, wcount, n_words, lens, out_wlen,
                     out_wcount);
  BEAST_LAUNCHED("k_gather_lens");
  int rc = scan_rec(lens, offs, n_words, sws, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(64), 0, s, lens, offs, n_words);
  hipLaunchKernelGGL(k_copy_words, dim3(g), dim3(256), 0, s, order, sym, wstart, wlen, offs, n_words, out_sym,
                     out_wstart, out_nsym);
  BEAST_LAUNCHED("k_copy_words");
  return BEAST_OK;
}
