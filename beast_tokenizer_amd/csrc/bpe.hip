// Byte-level BPE training kernels for gfx950 (replaces HF tokenizers' BpeTrainer as
// driven by beast/beast_bpe_trainer.py:61-98; semantics in SURVEY.md §8a H9-H11).
//
//   k_minmax / k_bitmap      global min/max bin, occupied code points (alphabet)
//   k_pretok_wave<EMIT>      GPT-2 regex pre-tokeniser, one wave per sequence over a
//                            code-point class LUT; pass 1 counts words / byte symbols,
//                            pass 2 writes byte symbols as vocab ids
//   k_scan_*                 exclusive prefix sums (word / symbol offsets)
//   k_count_pairs            dense [Vt][Vt] uint32 pair table += word count
//   k_argmax                 (count, -pair) max over the live table -> one u64 key
//   k_merge                  one thread per word: HF Word::merge left-to-right,
//                            in place; HF's pair-count changes are accumulated in
//                            LDS-privatised delta vectors [4][Vt] and flushed once
//                            per workgroup
//   k_apply_argmax           table += deltas, retire the merged pair, then the argmax
//                            (incremental: only changed rows are rescanned)
//   k_dedup_*                distinct words x counts (HF trains on word counts)
//   k_compact_words          drop words that can no longer merge (< 2 symbols)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace {

constexpr int CLS_OTHER = 0, CLS_LETTER = 1, CLS_NUMBER = 2, CLS_WS = 3;

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

// One thread per sequence (tools A/B: -DBPE_SERIAL_PRETOK_TRAIN)
template <bool EMIT>
__global__ void k_pretok(const long long* __restrict__ tok, const int64_t* __restrict__ seq_off, int64_t n_seq,
                         long long mn, const uint8_t* __restrict__ lut, int64_t lut_n,
                         int64_t* __restrict__ words_per_seq, int64_t* __restrict__ syms_per_seq,
                         const int64_t* __restrict__ word_off, const int64_t* __restrict__ sym_off,
                         const uint16_t* __restrict__ byte2id, uint16_t* __restrict__ sym,
                         uint32_t* __restrict__ wstart, uint32_t* __restrict__ wlen) {
  const int64_t sidx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (sidx >= n_seq) return;
  pretok_serial<EMIT>(tok, seq_off, sidx, mn, lut, lut_n, words_per_seq, syms_per_seq, word_off, sym_off, byte2id, sym,
                      wstart, wlen);
}

// One wave per sequence.  A thread per sequence reads its row 8 B at a time at a 1 KiB
// stride (every load instruction touches 64 cache lines), branches on its own word
// structure, and scatters 2-byte stores the same way.  Here the lanes load the row coalesced
// into LDS, classify it, evaluate the regex from every position at once (end of the word
// that would start there), scan the UTF-8 lengths, and lane 0 only follows the word chain
// 0 -> end[0] -> ...; the emission is lane-parallel over words and code points, so the
// stores of a wave land in one contiguous stretch.  Rows longer than PT_LC code points (or
// with code points outside [0, 2^31)) take pretok_serial on lane 0.
constexpr int PT_LC = 512;
constexpr int PT_WAVES = 4;
struct PtLds {
  int32_t cp[PT_LC];
  int16_t nxt[PT_LC];       // end of the word starting at i
  int16_t so[PT_LC + 1];    // byte-symbol offset of code point i
  int16_t wcp[PT_LC + 1];   // first code point of word w
  uint8_t cls[PT_LC];
  int32_t nw;
};

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
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  PtLds& L = lds[wv];
  for (int64_t sidx = (int64_t)blockIdx.x * PT_WAVES + wv; sidx < n_seq; sidx += (int64_t)gridDim.x * PT_WAVES) {
    const int64_t r0 = seq_off[sidx], n64 = seq_off[sidx + 1] - r0;
    bool serial = n64 > PT_LC;
    const int n = serial ? 0 : (int)n64;
    // 1. code points and classes (coalesced), then the UTF-8 symbol offsets
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
      const int i = base + lane;
      int len = 0;
      if (i < n) {
        const long long c = tok[r0 + i] - mn;
        serial |= (c < 0) | (c > 0x7FFFFFFFLL);
        L.cp[i] = (int32_t)c;
        L.cls[i] = (c >= 0 && c < lut_n) ? lut[c] : (uint8_t)CLS_OTHER;
        len = utf8_len(c);
      }
      int x = len;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      if (i < n) L.so[i] = (int16_t)(carry + x - len);
      carry += __shfl(x, 63);
    }
    if (__any(serial)) {   // wave-uniform
      if (lane == 0)
        pretok_serial<EMIT>(tok, seq_off, sidx, mn, lut, lut_n, words_per_seq, syms_per_seq, word_off, sym_off,
                            byte2id, sym, wstart, wlen);
      continue;
    }
    if (lane == 0) L.so[n] = (int16_t)carry;
    pt_wave_sync();
    // 2. the end of the word that starts at every position (pretok_serial's rules)
    for (int i = lane; i < n; i += 64) {
      const int c = L.cp[i];
      int j = 0;
      if (c == '\'' && i + 1 < n) {
        const int c1 = L.cp[i + 1];
        if (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd') j = i + 2;
        else if (i + 2 < n) {
          const int c2 = L.cp[i + 2];
          if ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l')) j = i + 3;
        }
      }
      if (j == 0) {
        int k = L.cls[i], st = i;
        if (c == ' ' && i + 1 < n && L.cls[i + 1] != CLS_WS) { k = L.cls[i + 1]; st = i + 1; }
        if (k != CLS_WS) {
          j = st + 1;
          while (j < n && L.cls[j] == k) ++j;
        } else {
          j = i + 1;
          while (j < n && L.cls[j] == CLS_WS) ++j;
          if (j < n && j - i >= 2) --j;   // \s+(?!\S): leave the last blank for the next word
        }
      }
      L.nxt[i] = (int16_t)j;
    }
    pt_wave_sync();
    // 3. lane 0 follows the chain
    if (lane == 0) {
      int nw = 0, p = 0;
      while (p < n) {
        L.wcp[nw++] = (int16_t)p;
        p = L.nxt[p];
      }
      L.wcp[nw] = (int16_t)n;
      L.nw = nw;
    }
    pt_wave_sync();
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

__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }

// Only pairs with a positive count are candidates (the table holds int32 counts in u32 cells): a
// pair whose "+" was always blocked by max_token_length goes negative on its "-" updates, and HF
// never queues it (BpeTrainer pushes a pair only when its count is > 0), so neither do we.
// Incremental argmax.  ws layout (u64): [2 + parity] result slots, [4, 4+Vt) the best key of
// each row, then u32 clean[Vt] (0 = never scanned: the zero-filled workspace starts
// all-dirty).  Call k writes slot k & 1 and zeroes the other for call k + 1 (no memset).
struct ArgWs {
  unsigned long long* slot;   // [2]
  unsigned long long* rowbest;
  uint32_t* clean;
};
__host__ __device__ inline ArgWs argws_view(void* ws, int Vt) {
  ArgWs v;
  unsigned long long* p = static_cast<unsigned long long*>(ws);
  v.slot = p + 2;
  v.rowbest = p + 4;
  v.clean = reinterpret_cast<uint32_t*>(p + 4 + Vt);
  return v;
}

// Device-driven merge loop (beast_bpe_loop_*): each k_merge decides its merge ON the GPU from
// the previous argmax (workgroup 0 records the decision), the following k_apply_argmax applies
// it and commits it (vocabulary hash, log, vcur, parity), so the host enqueues merges without a
// round trip per merge.
struct LoopState {
  // loop state: written by k_apply_argmax's workgroup 0 (and init), read by k_merge
  int32_t active;        // 0 once the loop has stopped (later launches are no-ops)
  int32_t a, b, nid, reused;   // last committed merge
  int32_t vcur;          // vocabulary size
  int32_t parity;        // argmax slot holding the pair for the next merge
  int32_t n_merges;      // merges logged
  int32_t target;        // vocab_size
  int32_t min_freq;
  int32_t log2cap;       // token-string hash table
  int32_t max_merges;    // log capacity
  unsigned long long count;
  // the step k_merge decided for the following k_apply_argmax (written by its workgroup 0)
  int32_t r_active, r_a, r_b, r_nid, r_reused, r_vcur, r_parity;
  uint32_t r_len;
  unsigned long long r_count, r_h;
  // the batch k_merge_batch decided for the following k_apply_batch (written by its workgroup 0)
  int32_t bn, bvcur;
  int32_t maxtlen;       // longest token (bytes): k_apply_batch keeps it
  int32_t ba[8], bb[8], bnid[8], breused[8];
  uint32_t blen[8];
  unsigned long long bh[8];
};

// ------------------------------------------------------- device merge loop --
// Token strings are identified by (64-bit polynomial hash of their UTF-8 bytes, byte length):
// h(xy) = h(x) * P^len(y) + h(y), so a merge's string is hashed from its parts.  The table maps
// (h, len) -> id; equal strings always collide (HF reuses the id), different strings collide
// with probability ~2^-64 -- the host re-checks every logged merge against the real strings
// and reruns the loop on the host path if it ever finds one (beast_tokenizer_amd/bpe_train.py).
constexpr uint32_t LOOP_EMPTY = 0xFFFFFFFFu;
struct LoopHash {
  unsigned long long* key;   // [cap] h
  uint32_t* klen;            // [cap] byte length, LOOP_EMPTY = free slot
  int32_t* kid;              // [cap]
  unsigned long long* th;    // [Vt] token hash
  unsigned long long* tp;    // [Vt] P^len
  int32_t* log;              // [max_merges][4] a, b, nid, reused
};

__device__ __forceinline__ uint64_t loop_slot(unsigned long long h, uint32_t len, int log2cap) {
  return ((h ^ ((unsigned long long)len * 0x9E3779B97F4A7C15ull)) * 0xbf58476d1ce4e5b9ull) >> (64 - log2cap);
}

struct LoopStep {
  int active, a, b, nid, reused, vcur;
  uint32_t len;
  unsigned long long count, h;
};

// The merge after the previous argmax (read-only on the loop state: every k_merge workgroup
// computes the same answer).  HF's loop: stop at vocab_size, below min_frequency or an empty
// queue; the merged string's id is an existing one (HF id reuse) or the next free one.
__device__ LoopStep loop_decide(const LoopState* __restrict__ st, ArgWs aw, int Vt, const LoopHash& lh,
                                const uint32_t* __restrict__ tlen) {
  LoopStep r{};
  if (!st->active) return r;
  const unsigned long long key = aw.slot[st->parity];
  const unsigned long long count = key >> 32;
  if (st->vcur >= st->target || count < 1 || count < (unsigned long long)st->min_freq ||
      st->n_merges >= st->max_merges)
    return r;
  const uint32_t idx = 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull);
  r.a = (int)(idx / (uint32_t)Vt);
  r.b = (int)(idx % (uint32_t)Vt);
  r.h = lh.th[r.a] * lh.tp[r.b] + lh.th[r.b];
  r.len = tlen[r.a] + tlen[r.b];
  const uint64_t mask = (1ull << st->log2cap) - 1;
  uint64_t sl = loop_slot(r.h, r.len, st->log2cap);
  r.nid = -1;
  while (lh.klen[sl] != LOOP_EMPTY) {
    if (lh.key[sl] == r.h && lh.klen[sl] == r.len) { r.nid = lh.kid[sl]; break; }
    sl = (sl + 1) & mask;
  }
  r.reused = r.nid >= 0;
  if (!r.reused) r.nid = st->vcur;
  r.vcur = st->vcur + (r.reused ? 0 : 1);
  r.count = count;
  r.active = 1;
  return r;
}

// k_apply_argmax's workgroup 0, after the apply: the decided merge becomes part of the
// vocabulary (string hash -> id), the log and the loop state.
__device__ void loop_commit(LoopState* __restrict__ st, const LoopHash& lh) {
  const int a = st->r_a, b = st->r_b, nid = st->r_nid;
  if (!st->r_reused) {
    const uint64_t mask = (1ull << st->log2cap) - 1;
    uint64_t sl = loop_slot(st->r_h, st->r_len, st->log2cap);
    while (lh.klen[sl] != LOOP_EMPTY) sl = (sl + 1) & mask;
    lh.key[sl] = st->r_h;
    lh.klen[sl] = st->r_len;
    lh.kid[sl] = nid;
    lh.th[nid] = st->r_h;
    lh.tp[nid] = lh.tp[a] * lh.tp[b];
  }
  int32_t* lg = lh.log + 4 * (int64_t)st->n_merges;
  lg[0] = a; lg[1] = b; lg[2] = nid; lg[3] = st->r_reused;
  st->n_merges += 1;
  st->a = a; st->b = b; st->nid = nid; st->reused = st->r_reused; st->count = st->r_count;
  st->vcur = st->r_vcur;
  st->parity = st->r_parity ^ 1;
}

// ------------------------------------------------------------------ merge --
// Bloom signature bits of symbol x: two of 64 (k = 2 keeps false positives of a 2-symbol query
// ~(2n/64)^4 for a word of n distinct symbols, vs (n/64)^2 with one bit)
__device__ __forceinline__ unsigned long long sig_bit(uint32_t x) {
  return (1ull << (x & 63u)) | (1ull << (((x * 0x9E3779B1u) >> 26) & 63u));
}

// HF's merge of (a, b) -> new in one word (Word::merge: left to right, non-overlapping) with the
// pair-count changes ((prev, a) -1, (prev, new) +1, (b, next) -1, (new, next) +1, weighted by the
// word's count; the +1s only while the new string stays shorter than max_token_length).  Returns
// the new length (0: the word holds no (a, b)), the new Bloom signature in g and the occurrences
// merged in napp.  Words of <= MERGE_REG symbols are read once into registers (all loads in
// flight together) and rewritten there: the in-place loop over global memory made every symbol a
// dependent round trip, and a merge waits for its slowest word.
constexpr int MERGE_REG = 32;
struct MergeOp {
  int a, b, nid, max_len;
  uint32_t newlen;
  const uint32_t* __restrict__ tlen;
  int32_t* colA;
  int32_t* colN;
  int32_t* rowB;
  int32_t* rowN;
  __device__ __forceinline__ void left(uint32_t p, int32_t cnt) const {     // HF: ((prev, a), -1), ((prev, new), +1)
    atomicAdd(&colA[p], -cnt);
    // the left neighbour may be this merge's own new token ("a a a a" -> "n n"); its length is
    // not in tlen until the apply
    const uint32_t lp = p == (uint32_t)nid ? newlen : tlen[p];
    if ((int)(lp + newlen) < max_len) atomicAdd(&colN[p], cnt);
  }
  __device__ __forceinline__ void right(uint32_t nx, int32_t cnt) const {   // HF: ((b, next), -1), ((new, next), +1)
    atomicAdd(&rowB[nx], -cnt);
    if ((int)(tlen[nx] + newlen) < max_len) atomicAdd(&rowN[nx], cnt);
  }
};

template <class Op>
__device__ __forceinline__ uint32_t merge_global(uint16_t* __restrict__ s, uint32_t L, const uint32_t* __restrict__ wcount,
                                                 int64_t w, const Op& m, unsigned long long& g, uint32_t& napp) {
  const uint32_t a = (uint32_t)m.a, b = (uint32_t)m.b, nid = (uint32_t)m.nid;
  bool hit = false;
  uint32_t prev = s[0];
#pragma unroll 8
  for (uint32_t k = 1; k < L; ++k) {
    const uint32_t cur = s[k];
    hit |= (prev == a) & (cur == b);
    prev = cur;
  }
  if (!hit) return 0;
  const int32_t cnt = wcount ? (int32_t)wcount[w] : 1;
  uint32_t r = 0, o = 0;
  unsigned long long sg = 0;
  while (r < L) {
    uint32_t y = s[r];
    if (y == a && r + 1 < L && s[r + 1] == b) {
      if (o > 0) m.left(s[o - 1], cnt);
      if (r + 2 < L) m.right(s[r + 2], cnt);
      y = nid;
      r += 2;
      ++napp;
    } else {
      r += 1;
    }
    s[o++] = (uint16_t)y;
    sg |= sig_bit(y);
  }
  g = sg;
  return o;
}

// a word of L <= MERGE_REG symbols in registers (sentinels past the end)
__device__ __forceinline__ void load_word(const uint16_t* __restrict__ s, uint32_t L, uint32_t (&v)[MERGE_REG + 2]) {
#pragma unroll
  for (int i = 0; i < MERGE_REG; ++i) v[i] = (uint32_t)i < L ? (uint32_t)s[i] : 0xFFFFFFFFu;
  v[MERGE_REG] = v[MERGE_REG + 1] = 0xFFFFFFFFu;
}
__device__ __forceinline__ bool word_has_pair(const uint32_t (&v)[MERGE_REG + 2], uint32_t a, uint32_t b) {
  bool hit = false;
#pragma unroll
  for (int i = 0; i < MERGE_REG - 1; ++i) hit |= (v[i] == a) & (v[i + 1] == b);
  return hit;
}
// the merge of a word held in v (which holds the pair) written back to s
template <class Op>
__device__ __forceinline__ uint32_t merge_regs(const uint32_t (&v)[MERGE_REG + 2], uint32_t L, uint16_t* __restrict__ s,
                                               int32_t cnt, const Op& m, unsigned long long& g, uint32_t& napp) {
  const uint32_t a = (uint32_t)m.a, b = (uint32_t)m.b, nid = (uint32_t)m.nid;
  uint32_t o = 0, last = 0, skip = 0;
  unsigned long long sg = 0;
#pragma unroll
  for (int i = 0; i < MERGE_REG; ++i) {
    if ((uint32_t)i < L) {
      uint32_t y = v[i];
      if (skip) {
        skip = 0;
        continue;
      }
      if (v[i] == a && v[i + 1] == b) {   // v[i + 1] is the sentinel past the end
        if (o > 0) m.left(last, cnt);
        if (v[i + 2] != 0xFFFFFFFFu) m.right(v[i + 2], cnt);
        y = nid;
        skip = 1;
        ++napp;
      }
      s[o++] = (uint16_t)y;
      last = y;
      sg |= sig_bit(y);
    }
  }
  g = sg;
  return o;
}

template <class Op>
__device__ __forceinline__ uint32_t merge_symbols(uint16_t* __restrict__ s, uint32_t L, const uint32_t* __restrict__ wcount,
                                                  int64_t w, const Op& m, unsigned long long& g, uint32_t& napp) {
  const uint32_t a = (uint32_t)m.a, b = (uint32_t)m.b, nid = (uint32_t)m.nid;
  if (L <= (uint32_t)MERGE_REG) {
    uint32_t v[MERGE_REG + 2];
    load_word(s, L, v);
    if (!word_has_pair(v, a, b)) return 0;
    return merge_regs(v, L, s, wcount ? (int32_t)wcount[w] : 1, m, g, napp);
  }
  return merge_global(s, L, wcount, w, m, g, napp);
}

// Inverted index symbol -> distinct words that may contain it (HF's where_to_update, on
// the GPU).  Built once from the distinct words; the merge creating token `new` appends
// the words it rewrote to a pool and k_apply_argmax turns that range into new's list.
// A list that cannot be exact (pool full, or `new` re-used an existing id) is INEXACT and
// merges involving it fall back to scanning every word.  Stale entries (a word that no
// longer holds the symbol) are harmless: the probe finds no pair there.
constexpr uint32_t IDX_INEXACT = 0xFFFFFFFFu;


#ifdef BPE_MERGE_STATS
// tools only: [0] Bloom candidates, [1] words holding the pair, [2] their symbols, [3] symbols probed
__device__ unsigned long long g_merge_stats[4];
#endif
constexpr int MERGE_UNROLL = 4;
constexpr int MERGE_SCAN = 8;       // signature loads in flight per thread (two-phase scan)
constexpr int MERGE_CLIST = 2048;   // LDS candidate list per workgroup
constexpr int BATCH_CLIST = 2 * 256 * MERGE_SCAN;   // k_merge_batch's list: two scan rounds
// Per-workgroup phase stamps of the merge kernels (tools/ab builds with -DBPE_MERGE_STAMPS=<first
// merge>; the product library compiles them out): s_memrealtime (100 MHz) of thread 0 at
// entry, after the decision, after the candidate pass, before the delta flush and at exit,
// for 64 merges x the first 1024 workgroups.
#ifdef BPE_MERGE_STAMPS
__device__ unsigned long long g_bpe_stamps[64][1024][6];
__device__ unsigned long long g_bpe_dstamps[64][8];
__device__ unsigned long long g_apply_stamps[64][256][6];   // k_apply_batch phases (first 256 workgroups)   // k_merge_batch's decision phases (workgroup 0)
#define DSTAMP(mi, k)                                                                            \
  do {                                                                                           \
    if (blockIdx.x == 0 && lane == 0 && (mi) >= BPE_MERGE_STAMPS && (mi) < BPE_MERGE_STAMPS + 64)      \
      g_bpe_dstamps[(mi) - BPE_MERGE_STAMPS][k] = __builtin_amdgcn_s_memrealtime();                      \
  } while (0)
#define MSTAMP(mi, k)                                                                            \
  do {                                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && (mi) >= BPE_MERGE_STAMPS && (mi) < BPE_MERGE_STAMPS + 64)  \
      g_bpe_stamps[(mi) - BPE_MERGE_STAMPS][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#else
#define MSTAMP(mi, k) do { } while (0)
#define DSTAMP(mi, k) do { } while (0)
#endif
#ifndef BPE_MERGE_STAMPS
#define KM_MI 0
#endif
struct WordIndex {
  uint32_t* start;   // [Vt]
  uint32_t* len;     // [Vt]
  uint32_t* ctl;     // [0] pool top, [1] mark (top after the previous apply), [2] capacity
  uint32_t* pool;    // [capacity]
};

__host__ __device__ inline WordIndex index_view(void* ws, int Vt) {
  WordIndex ix;
  char* p = static_cast<char*>(ws);
  ix.start = reinterpret_cast<uint32_t*>(p);
  ix.len = ix.start + Vt;
  ix.ctl = ix.len + Vt;
  ix.pool = ix.ctl + 4;
  return ix;
}

// One thread per word; words are short, so the distinct-symbol test is a backward scan.
template <bool FILL>
__global__ __launch_bounds__(256) void k_index_words(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                     const uint32_t* __restrict__ wlen, int64_t nw, WordIndex ix,
                                                     uint32_t* __restrict__ cursor) {
  if (FILL && ix.ctl[3]) return;   // overflowed: the index is unused
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const uint16_t* s = sym + wstart[w];
    const uint32_t L = wlen[w];
    for (uint32_t i = 0; i < L; ++i) {
      const uint32_t x = s[i];
      bool seen = false;
      for (uint32_t k = 0; k < i && !seen; ++k) seen = s[k] == x;
      if (seen) continue;
      if (FILL) ix.pool[atomicAdd(&cursor[x], 1u)] = (uint32_t)w;
      else atomicAdd(&ix.len[x], 1u);
    }
  }
}

__global__ __launch_bounds__(1024) void k_index_scan(WordIndex ix, int Vt, uint32_t* __restrict__ cursor) {
  __shared__ uint32_t part[1024];
  const int per = (Vt + 1023) / 1024, t = threadIdx.x;
  uint32_t acc = 0;
  for (int k = 0; k < per; ++k) {
    const int x = t * per + k;
    if (x < Vt) acc += ix.len[x];
  }
  part[t] = acc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {   // inclusive Hillis-Steele scan of the partial sums
    const uint32_t v = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const uint32_t total = part[1023];
  const bool fits = (uint64_t)total + (uint64_t)Vt <= (uint64_t)ix.ctl[2];   // cursor scratch sits past the lists
  uint32_t run = t ? part[t - 1] : 0u;
  for (int k = 0; k < per; ++k) {
    const int x = t * per + k;
    if (x < Vt) {
      ix.start[x] = run;
      cursor[x] = run;
      run += ix.len[x];
      if (!fits) ix.len[x] = IDX_INEXACT;   // pool too small: no lists, merges scan every word
    }
  }
  if (t == 1023) {
    ix.ctl[0] = fits ? total : ix.ctl[2];
    ix.ctl[1] = ix.ctl[0];
    ix.ctl[3] = fits ? 0u : 1u;
  }
}


// Deltas go to LDS (LDS = true, 4*Vt int32 <= 64 KiB) and are flushed once per workgroup
// into deltas[] with contiguous atomics (multi-GPU: all-reduced, then k_apply_argmax).
// (A last-workgroup-applies variant was measured slower: every workgroup's device-scope
// fence writes back its XCD's L2.)  Candidate words: the shorter exact index list of a
// and b, else every word (pre-filtered by the Bloom signature).
// MODE 0: deltas by global atomics, 1: LDS-privatised, 2: (a, b, nid, count) from the device
// loop record, LDS-privatised when the pair is frequent (dynamic LDS always allocated)
template <int MODE>
__global__ __launch_bounds__(256) void k_merge(uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                               uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount,
                                               int64_t nw, int a, int b, int nid, uint32_t* __restrict__ tlen,
                                               int max_len, int32_t* __restrict__ deltas, int Vt,
                                               unsigned long long* __restrict__ sig, WordIndex ix, bool use_ix,
                                               LoopState* __restrict__ loop, long long lds_min, ArgWs aw,
                                               LoopHash lh) {
  extern __shared__ __attribute__((aligned(16))) int32_t dl[];
  __shared__ int touched;
  __shared__ LoopStep dec;
  bool LDS = (MODE == 1);
  // first signature batch of the two-phase scan: issued before the merge is known (MODE 2
  // decides it below; the loads overlap the decision's dependent reads)
  unsigned long long sgv[MERGE_SCAN];
  const bool two_phase = !use_ix && sig != nullptr;
  const int64_t nchunks = (nw + 255) / 256;
  if (two_phase) {
#pragma unroll
    for (int u = 0; u < MERGE_SCAN; ++u) {
      const int64_t w = (blockIdx.x + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
      sgv[u] = w < nw ? sig[w] : 0ull;
    }
  }
#ifdef BPE_MERGE_STAMPS
  __shared__ int st_mi;
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
  if (MODE != 2 && threadIdx.x == 0) st_mi = -1;
#define KM_MI st_mi
#endif
  if (MODE == 2) {
    if (threadIdx.x == 0) {
#ifdef BPE_MERGE_STAMPS
      st_mi = loop->n_merges;
#endif
      dec = loop_decide(loop, aw, Vt, lh, tlen);
      if (blockIdx.x == 0) {   // the record k_apply_argmax applies and commits
        loop->r_active = dec.active;
        loop->r_a = dec.a; loop->r_b = dec.b; loop->r_nid = dec.nid; loop->r_reused = dec.reused;
        loop->r_vcur = dec.vcur; loop->r_parity = loop->parity; loop->r_len = dec.len;
        loop->r_count = dec.count; loop->r_h = dec.h;
        if (!dec.active) loop->active = 0;
      }
    }
    __syncthreads();
    if (!dec.active) return;
    a = dec.a; b = dec.b; nid = dec.nid;
    LDS = dec.count >= (unsigned long long)lds_min;
#ifdef BPE_MERGE_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 1024 && st_mi >= BPE_MERGE_STAMPS && st_mi < BPE_MERGE_STAMPS + 64)
      g_bpe_stamps[st_mi - BPE_MERGE_STAMPS][blockIdx.x][0] = t_entry;
#endif
    MSTAMP(KM_MI, 1);
  }
  const uint32_t* cand = nullptr;
  int64_t ncand = nw;
  if (use_ix) {
    const uint32_t la = ix.len[a], lb = ix.len[b];
    if (la != IDX_INEXACT || lb != IDX_INEXACT) {
      const bool pa = la != IDX_INEXACT && (lb == IDX_INEXACT || la <= lb);
      const int64_t n = pa ? la : lb;
      if (n * 8 < nw) {   // indirect (uncoalesced) visits only pay for short lists
        ncand = n;
        cand = ix.pool + (pa ? ix.start[a] : ix.start[b]);
      }
    }
  }
  if ((int64_t)blockIdx.x * blockDim.x >= ncand) return;   // block-uniform: nothing to do
  int32_t* dv = LDS ? dl : deltas;
  if (LDS) {
    for (int i = threadIdx.x; i < 4 * Vt; i += blockDim.x) dl[i] = 0;
    if (threadIdx.x == 0) touched = 0;
    __syncthreads();
  }
  const uint32_t newlen = tlen[a] + tlen[b];
  int32_t* colA = dv;
  int32_t* colN = dv + Vt;
  int32_t* rowB = dv + 2 * Vt;
  int32_t* rowN = dv + 3 * Vt;
  bool any = false;
  const unsigned long long need = sig_bit(a) | sig_bit(b);
  const MergeOp mop{a, b, nid, max_len, newlen, tlen, colA, colN, rowB, rowN};
  auto merge_word = [&](int64_t w) {
    const uint32_t L = wlen[w];
    if (L < 2) return;
#ifdef BPE_MERGE_STATS
    atomicAdd(&g_merge_stats[3], (unsigned long long)L);
#endif
    unsigned long long g = 0;
    uint32_t napp = 0;
    const uint32_t o = merge_symbols(sym + wstart[w], L, wcount, w, mop, g, napp);
    if (!o) return;
    any = true;
#ifdef BPE_MERGE_STATS
    atomicAdd(&g_merge_stats[1], 1ull);
    atomicAdd(&g_merge_stats[2], (unsigned long long)L);
#endif
    wlen[w] = o;
    if (sig != nullptr) sig[w] = g;
    if (use_ix) {   // w now holds `new`: it goes on new's list
      const uint32_t pos = atomicAdd(&ix.ctl[0], 1u);
      if (pos < ix.ctl[2]) ix.pool[pos] = (uint32_t)w;
    }
  };
  if (cand == nullptr && two_phase) {
    // Two phases per workgroup over its contiguous range of words: (1) every thread issues all
    // its signature loads at once and pushes the words that pass the Bloom test onto an LDS
    // list; (2) the workgroup's threads take the listed words in parallel, so the dependent
    // wlen -> wstart -> symbols chains of the few candidates overlap instead of trailing the
    // scan of one thread.
    // Words are stored in length order, so the candidates (long words fail the Bloom test
    // more often) concentrate at the end: workgroups take 256-word chunks round-robin.
    __shared__ uint32_t clist[MERGE_CLIST];
    __shared__ int cn;
    if (threadIdx.x == 0) cn = 0;
    __syncthreads();
    // phase 1 over every chunk of this workgroup: only LDS appends between the load rounds
    for (int64_t c0 = blockIdx.x; c0 < nchunks; c0 += (int64_t)MERGE_SCAN * gridDim.x) {
      if (c0 != blockIdx.x) {
#pragma unroll
        for (int u = 0; u < MERGE_SCAN; ++u) {
          const int64_t w = (c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
          sgv[u] = w < nw ? sig[w] : 0ull;
        }
      }
#pragma unroll
      for (int u = 0; u < MERGE_SCAN; ++u) {
        if ((sgv[u] & need) == need) {
          const int64_t w = (c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
          const int slot = atomicAdd(&cn, 1);
          if (slot < MERGE_CLIST) clist[slot] = (uint32_t)w;
          else merge_word(w);            // list full: this thread handles it itself
        }
      }
    }
    __syncthreads();
    MSTAMP(KM_MI, 2);
    // phase 2: the listed candidates, one per thread
    const int n = min(cn, MERGE_CLIST);
#ifdef BPE_MERGE_STATS
    if (threadIdx.x == 0) atomicAdd(&g_merge_stats[0], (unsigned long long)cn);
#endif
    for (int k = threadIdx.x; k < n; k += blockDim.x) merge_word(clist[k]);
  } else {
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < ncand; i0 += MERGE_UNROLL * G) {
   // MERGE_UNROLL candidates per pass: their signature loads are all in flight together
   unsigned long long sg[MERGE_UNROLL];
   int64_t ws[MERGE_UNROLL];
#pragma unroll
   for (int u = 0; u < MERGE_UNROLL; ++u) {
     const int64_t i = min(i0 + u * G, ncand - 1);
     ws[u] = cand ? (int64_t)cand[i] : i;
   }
#pragma unroll
   for (int u = 0; u < MERGE_UNROLL; ++u) sg[u] = sig != nullptr ? sig[ws[u]] : need;
   for (int u = 0; u < MERGE_UNROLL; ++u) {
    if (i0 + u * G >= ncand) break;
    const int64_t w = ws[u];
    // the word's symbol signature (64-bit Bloom mask) rules out most words without
    // touching their symbols
    if ((sg[u] & need) != need) continue;
    merge_word(w);
   }
  }
  }
  MSTAMP(KM_MI, 3);
  if (LDS) {
    if (any) touched = 1;
    __syncthreads();
    if (touched)   // contiguous atomics (one cache line per 32 entries)
#pragma unroll 8
      for (int i = threadIdx.x; i < 4 * Vt; i += blockDim.x) {
        const int32_t v = dl[i];
        if (v) atomicAdd(&deltas[i], v);
      }
  }
  MSTAMP(KM_MI, 4);
}

// ------------------------------------------------------------ pair index --
// Exact candidate words per merge, without scanning every word's signature.  An adjacency
// (x, y) in a word is created either at setup (both ids < nb, the setup symbols) or by the
// merge that created the LATER of x and y (merged ids grow with creation: the larger id), at
// which moment the other was its left (y later) or right (x later) neighbour -- a merge only
// creates adjacencies with its own new token, and a token id made by one merge is never made
// again (an id re-used by a second merge marks its list INEXACT).  So:
//  * (setup, setup): the distinct words that held the pair at setup (CSR over nb x nb pairs);
//  * otherwise, t = max(x, y): the entries the merge creating t recorded -- per rewritten word,
//    the distinct LEFT neighbours of t and the distinct RIGHT neighbours of t -- filtered to
//    kind L and symbol x (t == y, x != y) or kind R and symbol y (t == x).
// Both are supersets (later merges may have consumed an adjacency: the probe then finds
// nothing) and list every word at most once.  Entries are 8 bytes {word, kind << 16 | sym} in
// the token index's pool, [start[t], start[t] + len[t]) per token (k_apply_argmax commits them).
constexpr uint32_t ENT_L = 0u, ENT_R = 1u;
struct PairIndex {
  const uint32_t* off;    // [nb * nb + 1]
  const uint32_t* list;   // [off[nb * nb]] word ids
  int nb;
};

// (p, q) = (s[i-1], s[i]) occurred earlier in the word (one list entry per distinct word)
__device__ __forceinline__ bool pair_seen_before(const uint16_t* s, uint32_t i, uint32_t p, uint32_t q) {
  for (uint32_t j = 1; j < i; ++j)
    if (s[j - 1] == p && s[j] == q) return true;
  return false;
}

// Count (FILL = false: LDS histogram of rows [r0, r0 + R) flushed into gcount) or fill (FILL:
// the workgroup reserves each pair's slots with one atomic on the pair's cursor, then writes
// its word ids at LDS cursors).  Workgroups take 256-word chunks round-robin (length-sorted
// words); a workgroup visits the same chunks in both walks.
template <bool FILL>
__global__ __launch_bounds__(256) void k_pair_lists(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                    const uint32_t* __restrict__ wlen, int64_t nw, int nb, int R,
                                                    uint32_t* __restrict__ gcount, uint32_t* __restrict__ list) {
  extern __shared__ uint32_t hs[];   // [R][nb]
  const int r0 = blockIdx.y * R;
  const int rr = min(R, nb - r0);
  for (int i = threadIdx.x; i < rr * nb; i += blockDim.x) hs[i] = 0;
  __syncthreads();
  const int64_t nchunks = (nw + 255) / 256;
  auto walk = [&](bool emit) {
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
      const int64_t w = c * 256 + threadIdx.x;
      if (w >= nw) continue;
      const uint32_t L = wlen[w];
      const uint16_t* s = sym + wstart[w];
      for (uint32_t i = 1; i < L; ++i) {
        const uint32_t p = s[i - 1], q = s[i];
        const int pr = (int)p - r0;
        if (pr < 0 || pr >= rr || q >= (uint32_t)nb || pair_seen_before(s, i, p, q)) continue;
        const uint32_t slot = atomicAdd(&hs[pr * nb + q], 1u);
        if (emit) list[slot] = (uint32_t)w;
      }
    }
  };
  walk(false);
  __syncthreads();
  for (int i = threadIdx.x; i < rr * nb; i += blockDim.x) {
    const uint32_t v = hs[i];
    if (!v) continue;
    const uint32_t g = (uint32_t)(r0 + i / nb) * (uint32_t)nb + (uint32_t)(i % nb);
    const uint32_t base = atomicAdd(&gcount[g], v);   // FILL: gcount holds the cursors
    if (FILL) hs[i] = base;
  }
  if (!FILL) return;
  __syncthreads();
  walk(true);
}

// off = exclusive scan of the per-pair counts, cursors = off (one workgroup; nb^2 is small)
__global__ __launch_bounds__(1024) void k_pair_scan(uint32_t* __restrict__ off, uint32_t* __restrict__ cursor, int64_t P) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (P + 1023) / 1024;
  uint32_t acc = 0;
  for (int64_t k = 0; k < per; ++k) {
    const int64_t i = t * per + k;
    if (i < P) acc += cursor[i];
  }
  part[t] = acc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = t ? part[t - 1] : 0u;
  for (int64_t k = 0; k < per; ++k) {
    const int64_t i = t * per + k;
    if (i < P) {
      const uint32_t c = cursor[i];
      off[i] = run;
      cursor[i] = run;
      run += c;
    }
  }
  if (t == 1023) off[P] = part[1023];
}

// The device-driven merge over the pair index: k_merge<2>'s decision, then the candidate words.
// A setup pair walks its CSR word list when it is shorter than nw / list_ratio (each entry a
// dependent random visit); a pair with a merged token streams its creator's entry list (8 B
// per entry, coalesced) and visits only the entries that match.  Otherwise -- a long setup
// list, an INEXACT token -- the merge runs k_merge's two-phase Bloom-signature scan.  Rounds:
// 256 * MIX_U candidates per workgroup (MIX_U in flight per thread); the rewritten words'
// entries are counted, reserved with one atomic per workgroup and round, then written.
// apps[m] = pair occurrences merge m rewrote (unweighted), apps[max_merges + m] = the list
// elements it read (word list, entry list, or every word for a scan) -- bench.py's accounting.
constexpr int MIX_U = 4;
constexpr int MIX_NEW = 256 * MIX_U;
// The neighbours of new in a rewritten word, as entries: an L entry per occurrence unless the
// previous occurrence had the same left neighbour, likewise R (O(L); a word may still be listed
// twice under one (kind, symbol) -- k_merge_ix claims every entry-list word once per merge).
template <bool WRITE>
__device__ __forceinline__ uint32_t word_entries(const uint16_t* __restrict__ s, uint32_t o, uint32_t nid, uint32_t w,
                                                 uint32_t* __restrict__ pool, uint32_t k, uint32_t cap) {
  uint32_t n = 0, pl = 0xFFFFFFFFu, pr = 0xFFFFFFFFu;
  auto emit = [&](uint32_t kind, uint32_t x) {
    if (WRITE) {
      if (k < cap) *reinterpret_cast<uint2*>(pool + 2 * (size_t)k) = make_uint2(w, (kind << 16) | x);
      ++k;
    } else {
      ++n;
    }
  };
  if (o <= (uint32_t)MERGE_REG) {   // the rewritten word in registers: one round trip, no chain
    uint32_t v[MERGE_REG + 1];
#pragma unroll
    for (int i = 0; i < MERGE_REG; ++i) v[i] = (uint32_t)i < o ? (uint32_t)s[i] : 0xFFFFFFFFu;
    v[MERGE_REG] = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < MERGE_REG; ++i)
      if (v[i] == nid) {
        if (i > 0 && v[i - 1] != pl) { emit(ENT_L, v[i - 1]); pl = v[i - 1]; }
        if (v[i + 1] != 0xFFFFFFFFu && v[i + 1] != pr) { emit(ENT_R, v[i + 1]); pr = v[i + 1]; }
      }
  } else {
    uint32_t prev = 0xFFFFFFFFu, cur = s[0];
    for (uint32_t i = 0; i < o; ++i) {
      const uint32_t next = i + 1 < o ? s[i + 1] : 0xFFFFFFFFu;
      if (cur == nid) {
        if (i > 0 && prev != pl) { emit(ENT_L, prev); pl = prev; }
        if (i + 1 < o && next != pr) { emit(ENT_R, next); pr = next; }
      }
      prev = cur;
      cur = next;
    }
  }
  return WRITE ? k : n;
}

__global__ __launch_bounds__(256) void k_merge_ix(uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                  uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount,
                                                  int64_t nw, uint32_t* __restrict__ tlen, int max_len,
                                                  int32_t* __restrict__ deltas, int Vt, WordIndex ix, PairIndex px,
                                                  uint32_t* __restrict__ claim, unsigned long long* __restrict__ sig,
                                                  int list_ratio, LoopState* __restrict__ loop, long long lds_min,
                                                  ArgWs aw, LoopHash lh, uint32_t* __restrict__ apps, int max_merges) {
  extern __shared__ __attribute__((aligned(16))) int32_t dl[];
  __shared__ LoopStep dec;
  __shared__ const uint32_t* s_cand;
  __shared__ long long s_n;
  __shared__ int s_mi, touched, s_mode;   // mode 0: signature scan, 1: word list, 2: entry list
  __shared__ uint32_t s_want;             // mode 2: kind << 16 | symbol of the entries to visit
  __shared__ uint32_t clist[MERGE_CLIST];
  __shared__ uint32_t ecnt, ebase, napps;
  __shared__ int cn;
#ifdef BPE_MERGE_STAMPS
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
#endif
  if (threadIdx.x == 0) {
    dec = loop_decide(loop, aw, Vt, lh, tlen);
    s_mi = loop->n_merges;
    // an id made a second time (HF id re-use) breaks "the later token's merge made the
    // adjacency": ctl[3] = 1 sends every merge after it to the signature scan
    const bool lists_valid = ix.ctl[3] == 0u;
    if (blockIdx.x == 0) {   // the record k_apply_argmax applies and commits
      loop->r_active = dec.active;
      loop->r_a = dec.a; loop->r_b = dec.b; loop->r_nid = dec.nid; loop->r_reused = dec.reused;
      loop->r_vcur = dec.vcur; loop->r_parity = loop->parity; loop->r_len = dec.len;
      loop->r_count = dec.count; loop->r_h = dec.h;
      if (!dec.active) loop->active = 0;
      if (dec.active && dec.reused) ix.ctl[3] = 1u;
    }
    int mode = 0;
    const uint32_t* cand = nullptr;
    long long n = nw;
    uint32_t want = 0;
    if (dec.active && px.off != nullptr && lists_valid) {
      const int a = dec.a, b = dec.b;
      if (a < px.nb && b < px.nb) {
        const uint32_t p = (uint32_t)a * (uint32_t)px.nb + (uint32_t)b;
        const uint32_t o0 = px.off[p], o1 = px.off[p + 1];
        if (sig == nullptr || (long long)(o1 - o0) * list_ratio < nw) {
          mode = 1;
          cand = px.list + o0;
          n = o1 - o0;
        }
      } else {
        const int t = a > b ? a : b;
        const uint32_t lt = ix.len[t];
        if (lt != IDX_INEXACT && (sig == nullptr || list_ratio == 0 || (long long)lt < nw)) {
          mode = 2;
          cand = ix.pool + 2 * (size_t)ix.start[t];
          n = lt;
          want = (t == b && a != b) ? (ENT_L << 16) | (uint32_t)a : (ENT_R << 16) | (uint32_t)b;
        }
      }
    }
    s_mode = mode;
    s_cand = cand;
    s_n = n;
    s_want = want;
    if (blockIdx.x == 0 && dec.active && apps != nullptr && s_mi < max_merges)
      apps[max_merges + s_mi] = (uint32_t)n;
    ecnt = 0;
    napps = 0;
    touched = 0;
    cn = 0;
  }
  __syncthreads();
  if (!dec.active) return;
#ifdef BPE_MERGE_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 1024 && s_mi >= BPE_MERGE_STAMPS && s_mi < BPE_MERGE_STAMPS + 64)
    g_bpe_stamps[s_mi - BPE_MERGE_STAMPS][blockIdx.x][0] = t_entry;
#endif
  MSTAMP(s_mi, 1);
  const int mode = s_mode;
  const long long ncand = s_n;
  const uint32_t* cand = s_cand;
  const uint32_t want = s_want;
  // candidates per thread and round: as few as fill the grid (a thread's words are merged one
  // after another, so a short list spreads over more workgroups)
  const int U = (int)max((int64_t)1, min((int64_t)MIX_U, (int64_t)((ncand + (int64_t)gridDim.x * 256 - 1) /
                                                                  ((int64_t)gridDim.x * 256))));
  const int64_t per_round = (int64_t)U * 256;
  const int64_t nchunks = (nw + 255) / 256;
  if (mode ? (int64_t)blockIdx.x * per_round >= ncand : (int64_t)blockIdx.x >= nchunks) return;   // uniform
  const int a = dec.a, b = dec.b, nid = dec.nid;
  const bool LDS = dec.count >= (unsigned long long)lds_min;
  int32_t* dv = LDS ? dl : deltas;
  if (LDS) {
    for (int i = threadIdx.x; i < 4 * Vt; i += blockDim.x) dl[i] = 0;
    __syncthreads();
  }
  const uint32_t newlen = tlen[a] + tlen[b];
  int32_t* colA = dv;
  int32_t* colN = dv + Vt;
  int32_t* rowB = dv + 2 * Vt;
  int32_t* rowN = dv + 3 * Vt;
  uint32_t my_apps = 0;
  const uint32_t cap = ix.ctl[2];
  const MergeOp mop{a, b, nid, max_len, newlen, tlen, colA, colN, rowB, rowN};
  // one round: every thread's (up to MIX_U) candidate words, then the block's entry appends
  auto round = [&](const int64_t (&wv)[MIX_U]) {
    uint32_t Lv[MIX_U], Sv[MIX_U], Ov[MIX_U];
#pragma unroll
    for (int u = 0; u < MIX_U; ++u) {
      Lv[u] = wv[u] >= 0 ? wlen[wv[u]] : 0u;
      Sv[u] = wv[u] >= 0 ? wstart[wv[u]] : 0u;
    }
    uint32_t my_ent = 0;
    for (int u = 0; u < MIX_U; ++u) {
      Ov[u] = 0;
      if (Lv[u] < 2) continue;
      unsigned long long g = 0;
      const uint32_t o = merge_symbols(sym + Sv[u], Lv[u], wcount, wv[u], mop, g, my_apps);
      if (!o) continue;
      wlen[wv[u]] = o;
      if (sig != nullptr) sig[wv[u]] = g;
      Ov[u] = o;
      my_ent += word_entries<false>(sym + Sv[u], o, (uint32_t)nid, 0u, nullptr, 0u, 0u);
    }
    const uint32_t my_off = my_ent ? atomicAdd(&ecnt, my_ent) : 0u;
    __syncthreads();
    const uint32_t c = ecnt;
    if (c) {
      if (threadIdx.x == 0) {
        ebase = atomicAdd(&ix.ctl[0], c);
        touched = 1;
      }
      __syncthreads();
      uint32_t k = ebase + my_off;
      for (int u = 0; u < MIX_U && my_ent; ++u)
        if (Ov[u]) k = word_entries<true>(sym + Sv[u], Ov[u], (uint32_t)nid, (uint32_t)wv[u], ix.pool, k, cap);
      __syncthreads();
      if (threadIdx.x == 0) ecnt = 0;
    }
    __syncthreads();
  };
  if (mode != 0) {
    for (int64_t r0 = (int64_t)blockIdx.x * per_round; r0 < ncand; r0 += (int64_t)gridDim.x * per_round) {
      int64_t wv[MIX_U];
      if (mode == 1) {
#pragma unroll
        for (int u = 0; u < MIX_U; ++u) {
          const int64_t i = r0 + u * 256 + threadIdx.x;
          wv[u] = (u < U && i < ncand) ? (int64_t)cand[i] : -1;
        }
      } else {
        uint2 e[MIX_U];
#pragma unroll
        for (int u = 0; u < MIX_U; ++u) {
          const int64_t i = r0 + u * 256 + threadIdx.x;
          e[u] = (u < U && i < ncand) ? reinterpret_cast<const uint2*>(cand)[i] : make_uint2(0u, 0xFFFFFFFFu);
        }
        const uint32_t stamp = (uint32_t)s_mi + 1u;   // a word listed twice is visited once
#pragma unroll
        for (int u = 0; u < MIX_U; ++u)
          wv[u] = (e[u].y == want && atomicMax(&claim[e[u].x], stamp) < stamp) ? (int64_t)e[u].x : -1;
      }
      round(wv);
    }
  } else {
    // k_merge's two-phase scan: MERGE_SCAN signature loads per thread over 256-word chunks taken
    // round-robin (length-sorted words), candidates listed in LDS (<= 8 per thread: they fit),
    // then visited in rounds of MIX_U per thread
    const unsigned long long need = sig_bit(a) | sig_bit(b);
    for (int64_t c0 = blockIdx.x; c0 < nchunks; c0 += (int64_t)MERGE_SCAN * gridDim.x) {
      unsigned long long sgv[MERGE_SCAN];
#pragma unroll
      for (int u = 0; u < MERGE_SCAN; ++u) {
        const int64_t w = (c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
        sgv[u] = (sig != nullptr && w < nw) ? sig[w] : (w < nw ? need : 0ull);
      }
#pragma unroll
      for (int u = 0; u < MERGE_SCAN; ++u)
        if ((sgv[u] & need) == need) clist[atomicAdd(&cn, 1)] = (uint32_t)((c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x);
      __syncthreads();
      const int n = cn;
      for (int k0 = 0; k0 < n; k0 += MIX_NEW) {
        int64_t wv[MIX_U];
#pragma unroll
        for (int u = 0; u < MIX_U; ++u) {
          const int k = k0 + u * 256 + threadIdx.x;
          wv[u] = k < n ? (int64_t)clist[k] : -1;
        }
        round(wv);
      }
      if (threadIdx.x == 0) cn = 0;
      __syncthreads();
    }
  }
  MSTAMP(s_mi, 2);
  if (my_apps) atomicAdd(&napps, my_apps);
  __syncthreads();
  MSTAMP(s_mi, 3);
  if (threadIdx.x == 0 && napps && apps != nullptr && s_mi < max_merges) atomicAdd(&apps[s_mi], napps);
  if (LDS && touched)   // contiguous atomics (one cache line per 32 entries)
#pragma unroll 8
    for (int i = threadIdx.x; i < 4 * Vt; i += blockDim.x) {
      const int32_t v = dl[i];
      if (v) atomicAdd(&deltas[i], v);
    }
  MSTAMP(s_mi, 4);
}

// Fused apply + argmax, one workgroup per row x (the apply touches only entries of rows it
// owns: (x, a) and (x, new) for every x, rows b and new entirely).  When `apply`:
// table += deltas for row x, deltas consumed are zeroed, row a's (a, b) is retired after its
// own adds (the only deltas that can reach (a, b) are row a's, when a == b), tlen[new] set.
// A row rescans only if it changed (or was never scanned); then each workgroup folds its
// row's best into the result slot.
__device__ __forceinline__ void wave_fence_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave per row x, four rows per workgroup (the apply touches only entries of rows it
// owns: (x, a) and (x, new) for every x, rows b and new entirely).  When `apply`:
// table += deltas for row x, deltas consumed are zeroed, row a's (a, b) is retired after its
// own adds (the only deltas that can reach (a, b) are row a's, when a == b), tlen[new] set.
// A row rescans only if it changed (or was never scanned); the workgroup folds its rows'
// bests and makes one atomicMax into the result slot.
#ifndef APPLY_ROWS_N
#define APPLY_ROWS_N 16
#endif
// rows (waves) per workgroup.  Each workgroup ends with one device-scope atomicMax on the result
// slot, a single address that serialises at the memory side: 16 rows per workgroup (128
// atomics for a 2,048-row table) instead of 4 (512) cut the merge loop 65.4 -> 61.6 ms at K5.
constexpr int APPLY_ROWS = APPLY_ROWS_N;
__global__ __launch_bounds__(64 * APPLY_ROWS) void k_apply_argmax(uint32_t* __restrict__ table,
                                                                 int32_t* __restrict__ deltas, int Vt, int vcur,
                                                                 ArgWs aw, int parity, int apply, int a, int b,
                                                                 int nid, uint32_t* __restrict__ tlen, WordIndex ix,
                                                                 bool use_ix, bool reused,
                                                                 LoopState* __restrict__ loop, LoopHash lh, int nrows) {
  __shared__ unsigned long long wbest[APPLY_ROWS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (loop != nullptr) {   // device-driven loop: the merge k_merge decided (record r_*)
    if (!loop->r_active) return;
    vcur = loop->r_vcur; parity = loop->r_parity ^ 1; a = loop->r_a; b = loop->r_b; nid = loop->r_nid;
    reused = loop->r_reused != 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) loop_commit(loop, lh);   // no other workgroup reads what it writes
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) aw.slot[parity ^ 1] = 0ull;
  const int x0 = blockIdx.x * APPLY_ROWS;
  const int x = x0 + wave;
  __shared__ int changed_w[APPLY_ROWS];
  unsigned long long best = 0;
  int changed = 0;
  if (apply) {
    // (1) each wave's single entries (x, a) and (x, new)
    if (lane == 0 && x < nrows) {
      uint32_t* row = table + (size_t)x * Vt;
      int32_t v;
      if ((v = deltas[x])) { row[a] += (uint32_t)v; deltas[x] = 0; changed = 1; }
      if ((v = deltas[Vt + x])) { row[nid] += (uint32_t)v; deltas[Vt + x] = 0; changed = 1; }
    }
    if (lane == 0) changed_w[wave] = changed;
    // (2) rows b and new entirely, by the whole workgroup that owns them (after (1): row[a] /
    //     row[new] of those rows may be among the entries)
    const bool own_b = b >= x0 && b < x0 + APPLY_ROWS && b < nrows;
    const bool own_n = nid >= x0 && nid < x0 + APPLY_ROWS && nid < nrows;
    __syncthreads();
    if (own_b || own_n) {
      for (int r = 0; r < 2; ++r) {
        const int xr = r == 0 ? b : nid;
        if (!(r == 0 ? own_b : own_n) || (r == 1 && nid == b)) continue;
        uint32_t* row = table + (size_t)xr * Vt;
        int any = 0;
        for (int y = threadIdx.x; y < Vt; y += 64 * APPLY_ROWS) {
          int32_t v;
          if (xr == b && (v = deltas[2 * Vt + y])) { row[y] += (uint32_t)v; deltas[2 * Vt + y] = 0; any = 1; }
          if (xr == nid && (v = deltas[3 * Vt + y])) { row[y] += (uint32_t)v; deltas[3 * Vt + y] = 0; any = 1; }
        }
        if (any) changed_w[xr - x0] = 1;
      }
      __syncthreads();
    }
    // (3) row a: the merged pair retired after its own adds
    if (x == a && lane == 0) {
      uint32_t* row = table + (size_t)x * Vt;
      row[b] = 0u;   // never re-picked
      tlen[nid] = tlen[a] + tlen[b];
      if (use_ix) {   // the pool range appended by the merge becomes new's word list
        const uint32_t top = ix.ctl[0], mark = ix.ctl[1], cap = ix.ctl[2];
        if (reused || top > cap) {
          ix.len[nid] = IDX_INEXACT;
        } else {
          ix.start[nid] = mark;
          ix.len[nid] = top - mark;
        }
        const uint32_t t = top > cap ? cap : top;
        ix.ctl[0] = t;
        ix.ctl[1] = t;
      }
      changed_w[wave] = 1;
    }
    if (a >= x0 && a < x0 + APPLY_ROWS) __syncthreads();
    changed = changed_w[wave];
  }
  if (x < nrows && x < vcur) {
    uint32_t* row = table + (size_t)x * Vt;
    if (aw.clean[x] && !changed) {
      best = aw.rowbest[x];
    } else {
      // all of a lane's loads of a 2,048-entry stretch in flight together
      for (int base = 0; base < vcur; base += 64 * 32) {
        uint32_t c[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int y0 = base + (k * 64 + lane) * 4;
          if (((Vt & 3) == 0) && y0 + 4 <= vcur) {
            const uint4 u = *reinterpret_cast<const uint4*>(row + y0);
            c[4 * k] = u.x; c[4 * k + 1] = u.y; c[4 * k + 2] = u.z; c[4 * k + 3] = u.w;
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) c[4 * k + q] = y0 + q < vcur ? row[y0 + q] : 0u;
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int y = base + (k * 64 + lane) * 4 + q;
            const uint32_t idx = (uint32_t)x * (uint32_t)Vt + (uint32_t)y;
            const uint32_t cv = c[4 * k + q];
            if ((int32_t)cv > 0) best = umax64(best, ((unsigned long long)cv << 32) | (unsigned long long)(~idx));
          }
      }
      for (int o = 32; o > 0; o >>= 1) best = umax64(best, __shfl_xor(best, o));
      if (lane == 0) {
        aw.rowbest[x] = best;
        aw.clean[x] = 1u;
      }
    }
  }
  if (lane == 0) wbest[wave] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0;
    for (int w = 0; w < APPLY_ROWS; ++w) m = umax64(m, wbest[w]);
    unsigned long long* slot = aw.slot + parity;
    if (m && m > __atomic_load_n(slot, __ATOMIC_RELAXED)) atomicMax(slot, m);
  }
}

// --------------------------------------------------------- batched merges --
// Several merges per (merge, apply) pass, exactly HF's sequence.  Let p1, p2, ... be the table's
// pairs in HF order (count, then smallest (a, b)).  After merging p1 -> n1 every old pair keeps
// or loses count; the only new pairs contain n1 and each is bounded by the old pair it grew
// from: count(x, n1) <= count(x, a1), count(n1, y) <= count(b1, y), count(n1, n1) <=
// count(b1, a1).  If p2 shares no symbol with p1 and p1 is not a self-pair (a1 == b1, where
// "a a a a" -> "n n" breaks the bound), those old pairs are neither p1 nor p2, so they rank
// below p2; a new pair at an equal count also ranks below (its new id exceeds every old one).
// So p2 is the argmax after p1 -- and by the same argument p3 after p1, p2 (its bounding pairs
// share a symbol with p1 or p2, so they are not batch members), and so on.  A batch therefore
// takes the top pairs in order while each is symbol-disjoint from the batch, the previous one
// was not a self-pair, its string is new (no HF id re-use; distinct within the batch), the
// count clears min_frequency and the vocabulary and log have room; the first pair that fails
// ends the batch (it is decided next pass, with the full rules, on the updated table).
//
// The order needs more than each row's best: the true next pair may be the second-best of a
// row already taken.  k_apply_batch keeps every row's best and second-best key and hands each
// workgroup's BK best rows (best, second) to the next k_merge_batch, whose wave 0 reduces them
// to the global BK best rows and stops the batch where an accepted row's second-best would
// come first.  Measured at K5: 1,724 merges in 627 passes (BK = 4) instead of 1,724.
constexpr int BK = 8;                 // merges per batch at most (LoopState holds 8)
constexpr int BATCH_LDS = 32768;      // bytes of LDS delta vectors per workgroup (k_merge's 4 * Vt int32 at Vt 2048)
constexpr int BATCH_WG_LANE = 4;      // apply-workgroup lists per lane of the deciding wave (Vt <= 4096)

struct BatchWs {
  unsigned long long* rowsecond;      // [Vt]
  unsigned long long* wgkey;          // [BK][nwg] each apply workgroup's BK best rows, best first (k-major:
  unsigned long long* wgsec;          // [BK][nwg]  the deciding wave reads them coalesced) and their second-best
};
__host__ __device__ inline int batch_nwg(int Vt) { return (Vt + APPLY_ROWS_N - 1) / APPLY_ROWS_N; }
__host__ __device__ inline size_t batch_ws_bytes(int Vt) {
  return ((size_t)Vt * 8 + (size_t)batch_nwg(Vt) * BK * 2 * 8 + 255) & ~size_t(255);
}
__host__ __device__ inline BatchWs batch_view(void* ws, int Vt) {
  BatchWs v;
  char* p = static_cast<char*>(ws);
  const size_t nt = (size_t)batch_nwg(Vt) * BK;
  v.rowsecond = reinterpret_cast<unsigned long long*>(p);
  v.wgkey = v.rowsecond + Vt;
  v.wgsec = v.wgkey + nt;
  return v;
}

// Pair-count changes of batch merge j go straight into the pair table (no delta vectors, so the
// apply has nothing to add): kind 0 (x, a_j) -1, 1 (x, new_j) +1, 2 (b_j, y) -1, 3 (new_j, y) +1.
// A row x touched through kinds 0 / 1 is marked for re-ranking (clean[x] = 0); rows b_j, new_j
// and a_j always are.  The first merges of the batch whose four vectors fit BATCH_LDS (symbols <
// stride = vcur + n, so several while the vocabulary is small) sum them in LDS first when their
// count is large (k_merge's rule).  A neighbour may be a token this batch creates: its length
// is in nlen (tlen is written by the apply).
struct BatchOp {
  int a, b, nid, max_len, Vt, vbase, nnew, stride;
  bool short_all;       // every token + the new one < max_len: no length lookups
  uint32_t newlen;
  const uint32_t* __restrict__ tlen;
  const uint32_t* nlen;
  int32_t* dl;          // LDS vectors of this merge, or null
  uint32_t* table;
  uint32_t* clean;
  __device__ __forceinline__ uint32_t len_of(uint32_t x) const {
    return (int)x >= vbase && (int)x < vbase + nnew ? nlen[x - vbase] : tlen[x];
  }
  __device__ __forceinline__ void table_add(int kind, uint32_t x, int32_t v) const {
    if (kind < 2) {
      atomicAdd(&table[(size_t)x * Vt + (kind == 0 ? a : nid)], (uint32_t)v);
      clean[x] = 0u;
    } else {
      atomicAdd(&table[(size_t)(kind == 2 ? b : nid) * Vt + x], (uint32_t)v);
    }
  }
  __device__ __forceinline__ void add(int kind, uint32_t x, int32_t v) const {
    if (dl != nullptr) atomicAdd(&dl[kind * stride + x], v);
    else table_add(kind, x, v);
  }
  __device__ __forceinline__ void left(uint32_t p, int32_t cnt) const {
    add(0, p, -cnt);
    if (short_all || (int)(len_of(p) + newlen) < max_len) add(1, p, cnt);
  }
  __device__ __forceinline__ void right(uint32_t nx, int32_t cnt) const {
    add(2, nx, -cnt);
    if (short_all || (int)(len_of(nx) + newlen) < max_len) add(3, nx, cnt);
  }
};

// 64-bit wave helpers: DPP row shifts and row broadcasts (gfx9) leave the wave max in lane 63
template <int CTRL, int ROW_MASK, bool BC>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK, 0xF, BC);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW_MASK, 0xF, BC);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  v = umax64(v, dpp_u64<0x111, 0xF, true>(v));    // row_shr:1
  v = umax64(v, dpp_u64<0x112, 0xF, true>(v));    // row_shr:2
  v = umax64(v, dpp_u64<0x114, 0xF, true>(v));    // row_shr:4
  v = umax64(v, dpp_u64<0x118, 0xF, true>(v));    // row_shr:8: lane 15 of a row holds its max
  v = umax64(v, dpp_u64<0x142, 0xA, false>(v));   // row_bcast:15 into rows 1, 3
  v = umax64(v, dpp_u64<0x143, 0xC, false>(v));   // row_bcast:31 into rows 2, 3
  return readlane_u64(v, 63);
}

// Two descending (key, second) lists of KM -> the top KM of both, descending: the elementwise
// max of one list against the other reversed is bitonic, and KM/2, KM/4, ... half-cleaners sort it.
template <int KM>
__device__ __forceinline__ void top_merge(unsigned long long (&K)[KM], unsigned long long (&S)[KM],
                                          const unsigned long long (&OK)[KM], const unsigned long long (&OS)[KM]) {
#pragma unroll
  for (int i = 0; i < KM; ++i) {
    const bool t = OK[KM - 1 - i] > K[i];
    K[i] = t ? OK[KM - 1 - i] : K[i];
    S[i] = t ? OS[KM - 1 - i] : S[i];
  }
#pragma unroll
  for (int d = KM / 2; d > 0; d >>= 1)
#pragma unroll
    for (int i = 0; i < KM; ++i)
      if ((i & d) == 0) {
        const bool t = K[i + d] > K[i];
        const unsigned long long k0 = K[i], s0 = S[i];
        K[i] = t ? K[i + d] : k0;
        S[i] = t ? S[i + d] : s0;
        K[i + d] = t ? k0 : K[i + d];
        S[i + d] = t ? s0 : S[i + d];
      }
}

template <int KM>
__global__ __launch_bounds__(256) void k_merge_batch(uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                     uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount,
                                                     int64_t nw, const uint32_t* __restrict__ tlen, int max_len,
                                                     int Vt, unsigned long long* __restrict__ sig,
                                                     LoopState* __restrict__ loop, LoopHash lh, BatchWs bw,
                                                     uint32_t* __restrict__ table, ArgWs aw, long long lds_min) {
  __shared__ __attribute__((aligned(16))) int32_t dl[BATCH_LDS / 4];
  __shared__ uint32_t clist[BATCH_CLIST];
  __shared__ int cn, touched, s_n, s_kd;
  __shared__ int s_a[BK], s_b[BK], s_nid[BK];
  __shared__ uint32_t s_len[BK];
  __shared__ unsigned long long s_need[BK];
  const int lane = threadIdx.x & 63;
  // first signature batch of the two-phase scan, issued before the batch is known
  unsigned long long sgv[MERGE_SCAN];
  const int64_t nchunks = (nw + 255) / 256;
#pragma unroll
  for (int u = 0; u < MERGE_SCAN; ++u) {
    const int64_t w = (blockIdx.x + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
    sgv[u] = w < nw ? sig[w] : 0ull;
  }
  const int vcur = loop->vcur;
  const int maxtlen = loop->maxtlen;
#ifdef BPE_MERGE_STAMPS
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
  const int st_mi = loop->n_merges;
#define KB_MI st_mi
#else
#define KB_MI 0
#endif
  if (threadIdx.x < 64) {
    // ---- the batch.  Lane l merges the sorted lists of apply workgroups l, l + 64, ... (top KM
    // rows each), then KM wave-max rounds hand the global order out.
    const int nwg = batch_nwg(Vt);
    unsigned long long K[KM], S[KM];
#pragma unroll
    for (int i = 0; i < KM; ++i) K[i] = S[i] = 0ull;
    unsigned long long LK[BATCH_WG_LANE][KM], LS[BATCH_WG_LANE][KM];
#pragma unroll
    for (int t = 0; t < BATCH_WG_LANE; ++t) {
      const int g = t * 64 + lane;
#pragma unroll
      for (int i = 0; i < KM; ++i) {
        LK[t][i] = g < nwg ? bw.wgkey[(size_t)i * nwg + g] : 0ull;
        LS[t][i] = g < nwg ? bw.wgsec[(size_t)i * nwg + g] : 0ull;
      }
    }
    DSTAMP(KB_MI, 0);
#pragma unroll
    for (int t = 0; t < BATCH_WG_LANE; ++t)
      if (t * 64 < nwg) top_merge<KM>(K, S, LK[t], LS[t]);
    DSTAMP(KB_MI, 1);
    // KM rounds: the wave max of the lanes' list heads (DPP, no LDS), its owner pops it; lane r
    // keeps the r-th (best, second)
    unsigned long long ckey = 0, csec = 0;
#pragma unroll
    for (int r = 0; r < KM; ++r) {
      const unsigned long long m = wave_max_u64(K[0]);
      const bool mine = m != 0ull && K[0] == m;   // keys are distinct: one owner
      const unsigned long long ball = __ballot(mine);
      const int src = ball ? (int)__builtin_ctzll(ball) : 0;
      const unsigned long long sec = readlane_u64(S[0], src);
      if (lane == r) { ckey = m; csec = ball ? sec : 0ull; }
      if (mine) {
#pragma unroll
        for (int i = 0; i < KM - 1; ++i) { K[i] = K[i + 1]; S[i] = S[i + 1]; }
        K[KM - 1] = S[KM - 1] = 0ull;
      }
    }
    DSTAMP(KB_MI, 2);
    // lanes j < KM: candidate j's string and its id if it exists (the probes run in parallel)
    int cand_a = 0, cand_b = 0, exist = -1;
    uint32_t clen = 0;
    unsigned long long ch = 0;
    if (lane < KM && ckey) {
      const uint32_t idx = 0xFFFFFFFFu - (uint32_t)(ckey & 0xFFFFFFFFull);
      cand_a = (int)(idx / (uint32_t)Vt);
      cand_b = (int)(idx % (uint32_t)Vt);
      ch = lh.th[cand_a] * lh.tp[cand_b] + lh.th[cand_b];
      clen = tlen[cand_a] + tlen[cand_b];
      const uint64_t mask = (1ull << loop->log2cap) - 1;
      uint64_t sl = loop_slot(ch, clen, loop->log2cap);
      while (lh.klen[sl] != LOOP_EMPTY) {
        if (lh.key[sl] == ch && lh.klen[sl] == clen) { exist = lh.kid[sl]; break; }
        sl = (sl + 1) & mask;
      }
    }
    DSTAMP(KB_MI, 3);
    // HF's stopping rules per merge and the batch rules (see above), every candidate on its own
    // lane against the ones before it; the batch is the leading run of lanes that pass
    const bool live = loop->active != 0;
    const int target = loop->target, nm = loop->n_merges, maxm = loop->max_merges;
    const unsigned long long minf = (unsigned long long)loop->min_freq;
    const unsigned long long count = ckey >> 32;
    bool ok = live && lane < KM && count >= 1 && count >= minf && vcur + lane < target && nm + lane < maxm;
    if (lane > 0) ok &= exist < 0;   // only the first may re-use an id
    unsigned long long sec = 0;
#pragma unroll
    for (int i = 0; i < KM - 1; ++i) {
      const int ai = __builtin_amdgcn_readlane(cand_a, i), bi = __builtin_amdgcn_readlane(cand_b, i);
      const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)clen, i);
      const unsigned long long hi = readlane_u64(ch, i), si = readlane_u64(csec, i);
      const bool ends = ai == bi || (i == 0 && __builtin_amdgcn_readlane(exist, 0) >= 0);   // self-pair / re-use
      if (i < lane)
        ok &= !ends && cand_a != ai && cand_a != bi && cand_b != ai && cand_b != bi && !(ch == hi && clen == li);
      if (i < lane) sec = umax64(sec, si);
    }
    ok &= sec < ckey;   // a taken row's second-best would come first
    const unsigned long long pass = __ballot(ok);
    const int n = (int)__builtin_ctzll(~pass);   // leading lanes that pass (<= KM)
    if (lane < n) {
      const bool reused = lane == 0 && exist >= 0;
      const int nid = reused ? exist : vcur + lane;
      s_a[lane] = cand_a;
      s_b[lane] = cand_b;
      s_nid[lane] = nid;
      s_len[lane] = clen;
      s_need[lane] = sig_bit((uint32_t)cand_a) | sig_bit((uint32_t)cand_b);
      if (blockIdx.x == 0) {   // the record k_apply_batch applies and commits
        loop->ba[lane] = cand_a; loop->bb[lane] = cand_b; loop->bnid[lane] = nid;
        loop->breused[lane] = reused ? 1 : 0; loop->blen[lane] = clen; loop->bh[lane] = ch;
      }
    }
    DSTAMP(KB_MI, 4);
    if (lane == 0) {
      s_n = n;
      // merges 0 .. kd-1 sum their changes in LDS: the frequent ones whose vectors fit
      const int stride = vcur + n;
      int kd = 0;
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (kd == j && j < n && (j + 1) * 16 * stride <= BATCH_LDS &&
            (long long)(readlane_u64(ckey, j) >> 32) >= lds_min)
          kd = j + 1;
      s_kd = kd;
      if (blockIdx.x == 0) {
        loop->bn = n;
        loop->bvcur = vcur + n - ((n > 0 && exist >= 0) ? 1 : 0);
        if (n == 0) loop->active = 0;
      }
    }
  }
  if (threadIdx.x == 0) { cn = 0; touched = 0; }
  __syncthreads();
  const int n = s_n;
  if (n == 0) return;
#ifdef BPE_MERGE_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 1024 && st_mi >= BPE_MERGE_STAMPS && st_mi < BPE_MERGE_STAMPS + 64) {
    g_bpe_stamps[st_mi - BPE_MERGE_STAMPS][blockIdx.x][0] = t_entry;
    g_bpe_stamps[st_mi - BPE_MERGE_STAMPS][blockIdx.x][5] = (unsigned long long)n;
  }
#endif
  MSTAMP(KB_MI, 1);
  const int kd = s_kd;
  const int stride = vcur + n;
  const int nl = kd * 4 * stride;   // LDS entries in use
  if (kd > 0) {
    for (int i = threadIdx.x; i < nl; i += 256) dl[i] = 0;
    __syncthreads();
  }
  int mt = maxtlen;   // longest token a word can hold now (this batch's new ones included)
  for (int j = 0; j < n; ++j) mt = max(mt, (int)s_len[j]);
  const int vbase = s_nid[0] == vcur ? vcur : vcur + 1;   // first new id (merge 0 may re-use one)
  const int nnew = n - (vbase == vcur ? 0 : 1);
  const uint32_t* nlen = vbase == vcur ? s_len : s_len + 1;
  unsigned long long need[KM];
#pragma unroll
  for (int j = 0; j < KM; ++j) need[j] = j < n ? s_need[j] : ~0ull;
  bool any = false;
  // the batch's merges in order on one word (one inlined merge_symbols: the op comes from LDS)
  // The batch's merges in order on one word.  Its symbols are read once: the merges it holds
  // are known up front (batch pairs are symbol-disjoint, so one merge neither makes nor breaks
  // another's pair), the first merges from the registers, a rare second re-reads the word.
  auto visit = [&](int64_t w, unsigned long long sgw) {
    uint32_t L = wlen[w];
    uint16_t* s = sym + wstart[w];
    const int32_t cnt = wcount ? (int32_t)wcount[w] : 1;
    unsigned long long g = 0;
    uint32_t napp = 0;
    bool changed = false;
#ifdef BPE_MERGE_STATS
    atomicAdd(&g_merge_stats[0], 1ull);
    atomicAdd(&g_merge_stats[3], (unsigned long long)L);
#endif
    if (L < 2) return;
    if (L <= (uint32_t)MERGE_REG) {
      uint32_t v[MERGE_REG + 2];
      load_word(s, L, v);
      uint32_t hits = 0;
#pragma unroll 1
      for (int j = 0; j < n; ++j) {
        const unsigned long long nd = s_need[j];
        if ((sgw & nd) == nd && word_has_pair(v, (uint32_t)s_a[j], (uint32_t)s_b[j])) hits |= 1u << j;
      }
      if (!hits) return;
      // one merge_regs pass per set bit: lanes of a wave holding different merges share it
      // (the op is per lane), so a wave runs as many passes as its lanes' most merges (~1)
      bool fresh = true;
      while (hits) {
        const int j = __builtin_ctz(hits);
        hits &= hits - 1;
        if (!fresh) load_word(s, L, v);
        const BatchOp op{s_a[j], s_b[j], s_nid[j], max_len, Vt, vbase, nnew, stride,
                         mt + (int)s_len[j] < max_len, s_len[j], tlen, nlen,
                         j < kd ? dl + j * 4 * stride : nullptr, table, aw.clean};
        L = merge_regs(v, L, s, cnt, op, g, napp);
        fresh = false;
      }
      changed = true;
    } else {
#pragma unroll 1
      for (int j = 0; j < n; ++j) {
        const unsigned long long nd = s_need[j];
        if (L < 2 || (sgw & nd) != nd) continue;
        const BatchOp op{s_a[j], s_b[j], s_nid[j], max_len, Vt, vbase, nnew, stride,
                         mt + (int)s_len[j] < max_len, s_len[j], tlen, nlen,
                         j < kd ? dl + j * 4 * stride : nullptr, table, aw.clean};
        unsigned long long gj = 0;
        const uint32_t o = merge_global(s, L, wcount, w, op, gj, napp);
        if (o) { L = o; g = gj; changed = true; }
      }
    }
    if (!changed) return;
#ifdef BPE_MERGE_STATS
    atomicAdd(&g_merge_stats[1], 1ull);
    atomicAdd(&g_merge_stats[2], (unsigned long long)napp);
#endif
    any = true;
    wlen[w] = L;
    sig[w] = g;
  };
  // two-phase scan (k_merge's): a word is a candidate if its signature holds some merge's pair.
  // Rounds of MERGE_SCAN signatures per thread append to the LDS list; it is processed once at
  // the end, or earlier when another round could overflow it (merge_symbols is inlined once).
  for (int64_t c0 = blockIdx.x;; c0 += (int64_t)MERGE_SCAN * gridDim.x) {
    const bool more = c0 < nchunks;   // uniform
    if (more) {
      if (c0 != blockIdx.x) {
#pragma unroll
        for (int u = 0; u < MERGE_SCAN; ++u) {
          const int64_t w = (c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
          sgv[u] = w < nw ? sig[w] : 0ull;
        }
      }
#pragma unroll
      for (int u = 0; u < MERGE_SCAN; ++u) {
        bool hit = false;
#pragma unroll
        for (int j = 0; j < KM; ++j) hit |= (sgv[u] & need[j]) == need[j];
        if (hit) clist[atomicAdd(&cn, 1)] = (uint32_t)((c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x);
      }
    }
    __syncthreads();
    const int nc = cn;
    if (!more || nc > BATCH_CLIST - 256 * MERGE_SCAN) {
      MSTAMP(KB_MI, 2);
#ifdef BPE_MERGE_STAMPS
      if (threadIdx.x == 0 && blockIdx.x < 1024 && st_mi >= BPE_MERGE_STAMPS && st_mi < BPE_MERGE_STAMPS + 64)
        g_bpe_stamps[st_mi - BPE_MERGE_STAMPS][blockIdx.x][5] += (unsigned long long)nc << 8;   // candidates
#endif
      for (int k = threadIdx.x; k < nc; k += 256) {
        const int64_t w = clist[k];
        visit(w, sig[w]);
      }
      __syncthreads();
      if (threadIdx.x == 0) cn = 0;
      __syncthreads();
    }
    if (!more) break;
  }
  MSTAMP(KB_MI, 3);
  if (kd == 0) { MSTAMP(KB_MI, 4); return; }
  if (any) touched = 1;
  __syncthreads();
  if (touched)   // LDS entry i = (j * 4 + kind) * stride + x -> the table
    for (int i = threadIdx.x; i < nl; i += 256) {
      const int32_t v = dl[i];
      if (v) {
        const int jk = i / stride;
        const int j = jk >> 2;
        const BatchOp op{s_a[j], s_b[j], s_nid[j], max_len, Vt, 0, 0, stride, true, 0u, tlen, nlen, nullptr, table,
                         aw.clean};
        op.table_add(jk & 3, (uint32_t)(i - jk * stride), v);
      }
    }
  MSTAMP(KB_MI, 4);
#undef KB_MI
}

// After a batch: retire the merged pairs, commit the batch (hash table, log, vcur) from
// workgroup 0, then every changed row's best and second-best and this workgroup's BK best rows
// for the next decision.  init: no batch, every row < vcur ranked.
__global__ __launch_bounds__(64 * APPLY_ROWS) void k_apply_batch(uint32_t* __restrict__ table, int Vt, ArgWs aw,
                                                                 BatchWs bw, uint32_t* __restrict__ tlen,
                                                                 LoopState* __restrict__ loop, LoopHash lh, int nrows,
                                                                 int init) {
  __shared__ unsigned long long wbest[APPLY_ROWS], wsec[APPLY_ROWS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = init ? 0 : loop->bn;
  if (!init && (n == 0 || !loop->active)) return;
#ifdef BPE_MERGE_STAMPS
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
  const int st_mi = loop->n_merges;
  const bool st_on = !init && threadIdx.x == 0 && blockIdx.x < 256 && st_mi >= BPE_MERGE_STAMPS &&
                     st_mi < BPE_MERGE_STAMPS + 64;
#define ASTAMP(k)                                                                                           \
  do {                                                                                                      \
    if (st_on) g_apply_stamps[st_mi - BPE_MERGE_STAMPS][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
  if (st_on) g_apply_stamps[st_mi - BPE_MERGE_STAMPS][blockIdx.x][0] = t_entry;
#else
#define ASTAMP(k) do { } while (0)
#endif
  int A[BK], B[BK], N[BK];
#pragma unroll
  for (int j = 0; j < BK; ++j) {
    A[j] = j < n ? loop->ba[j] : -1;
    B[j] = j < n ? loop->bb[j] : -1;
    N[j] = j < n ? loop->bnid[j] : -1;
  }
  const int vcur = init ? loop->vcur : loop->bvcur;
  const int x0 = blockIdx.x * APPLY_ROWS;
  const int x = x0 + wave;
  if (init && lane == 0 && x < vcur) atomicMax(&loop->maxtlen, (int)tlen[x]);
  // rows the merges changed: clean[x] == 0 (k_merge_batch's adds through (x, a_j), (x, new_j)),
  // and a_j, b_j, new_j
  int changed = 0;
#pragma unroll
  for (int j = 0; j < BK; ++j) changed |= x == A[j] || x == B[j] || x == N[j];   // -1 past n
  ASTAMP(1);
  ASTAMP(2);
  if (lane == 0 && x < nrows)     // the merged pairs (every add landed in the previous kernel)
#pragma unroll
    for (int j = 0; j < BK; ++j)
      if (x == A[j]) {
        table[(size_t)x * Vt + B[j]] = 0u;   // never re-picked
        tlen[N[j]] = tlen[A[j]] + tlen[B[j]];
      }
  if (blockIdx.x == 0 && threadIdx.x == 0 && n > 0) {   // commit the batch (no other workgroup reads it)
    const uint64_t mask = (1ull << loop->log2cap) - 1;
    int nm = loop->n_merges;
    for (int j = 0; j < n; ++j) {
      const int reused = loop->breused[j];
      if (!reused) {
        const unsigned long long h = loop->bh[j];
        const uint32_t len = loop->blen[j];
        uint64_t sl = loop_slot(h, len, loop->log2cap);
        while (lh.klen[sl] != LOOP_EMPTY) sl = (sl + 1) & mask;
        lh.key[sl] = h;
        lh.klen[sl] = len;
        lh.kid[sl] = N[j];
        lh.th[N[j]] = h;
        lh.tp[N[j]] = lh.tp[A[j]] * lh.tp[B[j]];
      }
      int32_t* lg = lh.log + 4 * (int64_t)nm;
      lg[0] = A[j]; lg[1] = B[j]; lg[2] = N[j]; lg[3] = reused;
      ++nm;
      loop->a = A[j]; loop->b = B[j]; loop->nid = N[j]; loop->reused = reused;
    }
    loop->n_merges = nm;
    loop->vcur = vcur;
    int mt = loop->maxtlen;
    for (int j = 0; j < n; ++j) mt = max(mt, (int)loop->blen[j]);
    loop->maxtlen = mt;
  }
  __syncthreads();
  ASTAMP(3);
  changed |= init;
  unsigned long long best = 0, second = 0;
  if (x < nrows && x < vcur) {
    if (aw.clean[x] && !changed) {
      best = aw.rowbest[x];
      second = bw.rowsecond[x];
    } else {
      const uint32_t* row = table + (size_t)x * Vt;
      for (int base = 0; base < vcur; base += 64 * 32) {
        uint32_t c[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int y0 = base + (k * 64 + lane) * 4;
          if (((Vt & 3) == 0) && y0 + 4 <= vcur) {
            const uint4 u = *reinterpret_cast<const uint4*>(row + y0);
            c[4 * k] = u.x; c[4 * k + 1] = u.y; c[4 * k + 2] = u.z; c[4 * k + 3] = u.w;
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) c[4 * k + q] = y0 + q < vcur ? row[y0 + q] : 0u;
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t cv = c[4 * k + q];
            const int y = base + (k * 64 + lane) * 4 + q;
            const unsigned long long key =
                (int32_t)cv > 0 ? ((unsigned long long)cv << 32) | (unsigned long long)(~((uint32_t)x * (uint32_t)Vt + (uint32_t)y))
                   : 0ull;
            const unsigned long long lo = umin64(key, best);
            best = umax64(key, best);
            second = umax64(second, lo);
          }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {   // the wave's top two
        const unsigned long long b2 = __shfl_xor(best, o), s2 = __shfl_xor(second, o);
        second = umax64(umax64(second, s2), umin64(best, b2));
        best = umax64(best, b2);
      }
      if (lane == 0) {
        aw.rowbest[x] = best;
        bw.rowsecond[x] = second;
        aw.clean[x] = 1u;
      }
    }
  }
  if (lane == 0) { wbest[wave] = best; wsec[wave] = second; }
  __syncthreads();
  ASTAMP(4);
  if (threadIdx.x < APPLY_ROWS) {   // this workgroup's BK best rows, best first: row w goes to its rank
    const int w = threadIdx.x;
    const unsigned long long kw = wbest[w];
    int rank = 0;   // rows above w (ties -- only empty rows -- by index)
#pragma unroll
    for (int v = 0; v < APPLY_ROWS; ++v) rank += wbest[v] > kw || (wbest[v] == kw && v < w);
    if (rank < BK) {
      bw.wgkey[(size_t)rank * batch_nwg(Vt) + blockIdx.x] = kw;   // the grid may cover fewer rows than Vt
      bw.wgsec[(size_t)rank * batch_nwg(Vt) + blockIdx.x] = kw ? wsec[w] : 0ull;
    }
  }
  ASTAMP(5);
#undef ASTAMP
}

// -------------------------------------------------- persistent merge loop --
// The whole device-driven loop in ONE launch (no kernel boundary per merge).  One workgroup of
// 1024 threads per CU, all resident; per merge:
//   D  every workgroup reduces the per-workgroup argmax keys of the previous phase A and makes
//      the same decision (HF's stop rules, id by the string hash table; loop_decide's logic);
//   M  the merge over the words: k_merge's two-phase Bloom-signature scan, LDS-privatised deltas
//      flushed to `deltas`;
//   -- grid barrier --
//   A  apply + argmax (k_apply_argmax): one wave per table row, rows split over the workgroups;
//      workgroup 0 also commits the merge (log, hash table, vcur) -- after every workgroup's
//      decision, so no workgroup's hash probe can see this merge's string;
//   -- grid barrier --
// The barrier is arrival counters per group of workgroups (blockIdx & 7) plus one top counter
// (a few dozen same-address atomics each, not one per workgroup), polled with an agent-scope
// acquire; every spin is bounded: a timeout raises `abort`, every workgroup leaves the loop and
// the host reruns the training on the launch-per-merge loop.
constexpr int PL_T = 1024;           // threads per workgroup
constexpr int PL_SCAN = 4;           // signature loads per thread and scan sub-batch
constexpr int PL_CLIST = PL_T * PL_SCAN;
constexpr int PL_GROUPS = 8;
constexpr unsigned PL_SPIN_LIMIT = 1u << 26;

struct PlBar {
  unsigned int* sub;                 // [PL_GROUPS]
  unsigned int* top;
  unsigned int* abort_flag;
  unsigned long long* bests;         // [grid] per-workgroup argmax key of the last phase A
};

__device__ __forceinline__ bool pl_barrier(const PlBar& pb, unsigned& epoch, int G) {
  __shared__ int s_ok;
  // every storing wave drains its stores (vmcnt(0); expcnt / lgkmcnt not waited), the
  // workgroup meets, then one agent-scope release before the arrival (MI355X_MICROARCH.md,
  // inter-workgroup visibility)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    ++epoch;
    const int ng = G < PL_GROUPS ? G : PL_GROUPS;
    const int grp = blockIdx.x % ng;
    const unsigned gsize = (unsigned)((G - grp + ng - 1) / ng);
    const unsigned old = __hip_atomic_fetch_add(&pb.sub[grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == epoch * gsize) __hip_atomic_fetch_add(pb.top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = epoch * (unsigned)ng;
    unsigned spins = 0;
    int ok = 1;
    while (__hip_atomic_load(pb.top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(pb.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > PL_SPIN_LIMIT) {
        __hip_atomic_store(pb.abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // other workgroups' writes, after it
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

__global__ __launch_bounds__(PL_T) void k_bpe_loop(uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                  uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount,
                                                  int64_t nw, uint32_t* __restrict__ tlen, int max_len,
                                                  int32_t* __restrict__ deltas, int Vt, int nrows,
                                                  unsigned long long* __restrict__ sig, uint32_t* __restrict__ table,
                                                  LoopState* __restrict__ loop, LoopHash lh, ArgWs aw, PlBar pb,
                                                  int n_steps, long long lds_min) {
  extern __shared__ __attribute__((aligned(16))) int32_t dl[];
  __shared__ uint32_t clist[PL_CLIST];
  __shared__ int cn, any_s, changed_w[PL_T / 64];
  __shared__ LoopStep dec;
  __shared__ unsigned long long wbest[PL_T / 64];
  const int G = gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rows_per = (nrows + G - 1) / G;   // <= 16 = waves per workgroup (host-checked)
  const int x0 = blockIdx.x * rows_per;
  unsigned epoch = 0;
  // argmax of the row x this wave owns (rescan unless its cached best is still valid)
  auto row_best = [&](int x, int vcur, bool changed) -> unsigned long long {
    unsigned long long best = 0;
    if (x >= nrows || x >= vcur) return 0;
    if (aw.clean[x] && !changed) return aw.rowbest[x];
    const uint32_t* row = table + (size_t)x * Vt;
    for (int base = 0; base < vcur; base += 64 * 32) {
      uint32_t c[32];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int y0 = base + (k * 64 + lane) * 4;
        if (((Vt & 3) == 0) && y0 + 4 <= vcur) {
          const uint4 u = *reinterpret_cast<const uint4*>(row + y0);
          c[4 * k] = u.x; c[4 * k + 1] = u.y; c[4 * k + 2] = u.z; c[4 * k + 3] = u.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) c[4 * k + q] = y0 + q < vcur ? row[y0 + q] : 0u;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int y = base + (k * 64 + lane) * 4 + q;
          const uint32_t idx = (uint32_t)x * (uint32_t)Vt + (uint32_t)y;
          const uint32_t cv = c[4 * k + q];
          if ((int32_t)cv > 0) best = umax64(best, ((unsigned long long)cv << 32) | (unsigned long long)(~idx));
        }
    }
    for (int o = 32; o > 0; o >>= 1) best = umax64(best, __shfl_xor(best, o));
    if (lane == 0) {
      aw.rowbest[x] = best;
      aw.clean[x] = 1u;
    }
    return best;
  };
  auto publish_best = [&](unsigned long long best) {
    if (lane == 0) wbest[wave] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long m = 0;
      for (int w = 0; w < PL_T / 64; ++w) m = umax64(m, wbest[w]);
      pb.bests[blockIdx.x] = m;
    }
  };
  // initial argmax (phase A without an apply)
  {
    const int x = x0 + wave;
    publish_best(wave < rows_per ? row_best(x, loop->vcur, false) : 0ull);
  }
  if (!pl_barrier(pb, epoch, G)) return;
  for (int step = 0; step < n_steps; ++step) {
#ifdef BPE_MERGE_STAMPS
    const int smi = loop->n_merges;
#else
    const int smi = 0;
#endif
    MSTAMP(smi, 0);
    // ---- D: the merge, decided identically by every workgroup
    if (threadIdx.x < 64) {
      unsigned long long m = 0;
      for (int g = threadIdx.x; g < G; g += 64) m = umax64(m, pb.bests[g]);
      for (int o = 32; o > 0; o >>= 1) m = umax64(m, __shfl_xor(m, o));
      if (threadIdx.x == 0) {
        aw.slot[loop->parity] = m;     // every workgroup writes the same value; loop_decide reads it
        dec = loop_decide(loop, aw, Vt, lh, tlen);
      }
    }
    __syncthreads();
    if (!dec.active) {
      if (blockIdx.x == 0 && threadIdx.x == 0) loop->active = 0;
      break;
    }
    MSTAMP(smi, 1);
    const int a = dec.a, b = dec.b, nid = dec.nid;
    const bool LDS = dec.count >= (unsigned long long)lds_min;
    // ---- M: merge (a, b) -> nid in every word holding the pair
    int32_t* dv = LDS ? dl : deltas;
    if (LDS)
      for (int i = threadIdx.x; i < 4 * Vt; i += PL_T) dl[i] = 0;
    if (threadIdx.x == 0) { cn = 0; any_s = 0; }
    __syncthreads();
    const uint32_t newlen = tlen[a] + tlen[b];
    const MergeOp mop{a, b, nid, max_len, newlen, tlen, dv, dv + Vt, dv + 2 * Vt, dv + 3 * Vt};
    const unsigned long long need = sig_bit(a) | sig_bit(b);
    const int64_t nchunks = (nw + 255) / 256;
    bool any = false;
    // chunks of 256 words taken round-robin: workgroup g, sub-batch r reads chunks
    // g + (r * PL_SCAN*4 + u*4 + t/256) * G (4 chunks per 1024 threads)
    for (int64_t c0 = blockIdx.x; c0 < nchunks; c0 += (int64_t)PL_SCAN * 4 * G) {
      unsigned long long sgv[PL_SCAN];
#pragma unroll
      for (int u = 0; u < PL_SCAN; ++u) {
        const int64_t c = c0 + ((int64_t)u * 4 + (threadIdx.x >> 8)) * G;
        const int64_t w = c * 256 + (threadIdx.x & 255);
        sgv[u] = (c < nchunks && w < nw) ? (sig != nullptr ? sig[w] : need) : 0ull;
      }
#pragma unroll
      for (int u = 0; u < PL_SCAN; ++u)
        if ((sgv[u] & need) == need) {
          const int64_t c = c0 + ((int64_t)u * 4 + (threadIdx.x >> 8)) * G;
          clist[atomicAdd(&cn, 1)] = (uint32_t)(c * 256 + (threadIdx.x & 255));
        }
      __syncthreads();
      const int n = cn;
      for (int k = threadIdx.x; k < n; k += PL_T) {
        const int64_t w = clist[k];
        const uint32_t L = wlen[w];
        if (L < 2) continue;
        unsigned long long g = 0;
        uint32_t napp = 0;
        const uint32_t o = merge_symbols(sym + wstart[w], L, wcount, w, mop, g, napp);
        if (!o) continue;
        any = true;
        wlen[w] = o;
        if (sig != nullptr) sig[w] = g;
      }
      __syncthreads();
      if (threadIdx.x == 0) cn = 0;
      __syncthreads();
    }
    if (LDS) {
      if (any) any_s = 1;
      __syncthreads();
      if (any_s)
        for (int i = threadIdx.x; i < 4 * Vt; i += PL_T) {
          const int32_t v = dl[i];
          if (v) atomicAdd(&deltas[i], v);
        }
    }
    MSTAMP(smi, 2);
    if (!pl_barrier(pb, epoch, G)) return;
    MSTAMP(smi, 3);
    // ---- A: apply the deltas, retire (a, b), commit, argmax
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // every workgroup has decided: commit
      loop->r_active = 1;
      loop->r_a = a; loop->r_b = b; loop->r_nid = nid; loop->r_reused = dec.reused;
      loop->r_vcur = dec.vcur; loop->r_parity = loop->parity; loop->r_len = dec.len;
      loop->r_count = dec.count; loop->r_h = dec.h;
      loop_commit(loop, lh);
    }
    const int x = x0 + wave;
    const bool mine = wave < rows_per && x < nrows;
    int changed = 0;
    if (mine && lane == 0) {
      uint32_t* row = table + (size_t)x * Vt;
      int32_t v;
      if ((v = deltas[x])) { row[a] += (uint32_t)v; deltas[x] = 0; changed = 1; }
      if ((v = deltas[Vt + x])) { row[nid] += (uint32_t)v; deltas[Vt + x] = 0; changed = 1; }
    }
    if (lane == 0) changed_w[wave] = changed;
    __syncthreads();
    const bool own_b = b >= x0 && b < x0 + rows_per && b < nrows;
    const bool own_n = nid >= x0 && nid < x0 + rows_per && nid < nrows;
    if (own_b || own_n) {
      for (int r = 0; r < 2; ++r) {
        const int xr = r == 0 ? b : nid;
        if (!(r == 0 ? own_b : own_n) || (r == 1 && nid == b)) continue;
        uint32_t* row = table + (size_t)xr * Vt;
        int anyr = 0;
        for (int y = threadIdx.x; y < Vt; y += PL_T) {
          int32_t v;
          if (xr == b && (v = deltas[2 * Vt + y])) { row[y] += (uint32_t)v; deltas[2 * Vt + y] = 0; anyr = 1; }
          if (xr == nid && (v = deltas[3 * Vt + y])) { row[y] += (uint32_t)v; deltas[3 * Vt + y] = 0; anyr = 1; }
        }
        if (anyr) changed_w[xr - x0] = 1;
      }
    }
    __syncthreads();
    if (x == a && mine && lane == 0) {
      table[(size_t)a * Vt + b] = 0u;   // never re-picked
      tlen[nid] = tlen[a] + tlen[b];
      changed_w[wave] = 1;
    }
    __syncthreads();
    publish_best(mine ? row_best(x, dec.vcur, changed_w[wave] != 0) : 0ull);
    MSTAMP(smi, 4);
    if (!pl_barrier(pb, epoch, G)) return;
    MSTAMP(smi, 5);
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
  unsigned long long* nu;     // distinct count
  uint64_t cap;
};

__host__ __device__ inline uint64_t dedup_cap(int64_t n) {
  uint64_t c = 1024;
  while (c < (uint64_t)n * 2) c <<= 1;
  return c;
}

// One thread per word.  The table slot of the word's content is found as before; then the
// atomics that serialised at the memory side are aggregated.  New distinct words go to an LDS
// list (one LDS atomic per wave) that the workgroup appends to the global list with ONE device
// atomic when it is nearly full and at the end: the global list counter is a single address,
// and one atomic per wave on it (576 k at K5, each waiting on the previous at the memory side)
// took 7.2 ms of the 11.7 ms BPE setup.  Occurrence counts are summed per slot in an LDS hash
// (DEDUP_LDS entries, linear probing; a full probe falls back to the global atomic) and flushed
// once per workgroup -- the common words occur millions of times.
constexpr int DEDUP_LDS = 4096;
constexpr int DEDUP_NEW = 1024;   // LDS new-word list; flushed when a pass could overflow it
__global__ __launch_bounds__(256) void k_dedup_insert(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
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
        while (true) {
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
    if (ncnt > (uint32_t)(DEDUP_NEW - 256)) flush_new();   // the next pass adds <= 256
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
  const int64_t nu = (int64_t)*ws.nu;
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_n = nu;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nu; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = ws.rep[i];
    ow[i] = wstart[r];
    ol[i] = wlen[r];
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
// merge scan is coalesced and its per-thread loops stay in step.
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
    lens[i] = wlen[w];
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
    ow[i] = (uint32_t)offs[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *out_nsym = offs[nw];
}

__global__ __launch_bounds__(256) void k_word_sig(const uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                  const uint32_t* __restrict__ wlen, int64_t nw,
                                                  unsigned long long* __restrict__ sig) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const uint16_t* s = sym + wstart[w];
    unsigned long long g = 0;
    for (uint32_t i = 0, L = wlen[w]; i < L; ++i) g |= sig_bit(s[i]);
    sig[w] = g;
  }
}

int grid_for(int64_t n, int per_block, int cap) {
  const int64_t g = (n + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// k_merge's grid: the workgroups the device holds at once (one pass over the words, each
// workgroup its contiguous range, MERGE_SCAN signature loads in flight per thread), not more
template <int MODE>
int merge_grid(int64_t nw, size_t lds) {
  static int resident[2] = {0, 0};   // [lds != 0]
  int& r = resident[lds != 0];
  if (r == 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_merge<MODE>, 256, lds) != hipSuccess || per <= 0)
      per = 4;
    r = cus * per;
  }
  return grid_for(nw, MERGE_SCAN * 256, r);
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
#ifdef BPE_SERIAL_PRETOK_TRAIN
  hipLaunchKernelGGL(k_pretok<false>, dim3((n_seq + 127) / 128), dim3(128), 0, beast::as_stream(stream),
#else
  hipLaunchKernelGGL(k_pretok_wave<false>, dim3(grid_for(n_seq, PT_WAVES, 16384)), dim3(64 * PT_WAVES), 0,
                     beast::as_stream(stream),
#endif
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
#ifdef BPE_SERIAL_PRETOK_TRAIN
  hipLaunchKernelGGL(k_pretok<true>, dim3((n_seq + 127) / 128), dim3(128), 0, beast::as_stream(stream),
#else
  hipLaunchKernelGGL(k_pretok_wave<true>, dim3(grid_for(n_seq, PT_WAVES, 16384)), dim3(64 * PT_WAVES), 0,
                     beast::as_stream(stream),
#endif
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

extern "C" size_t beast_bpe_argmax_workspace_bytes(int Vt) { return (size_t)(4 + (int64_t)Vt) * 8 + (size_t)Vt * 4; }

extern "C" int beast_bpe_argmax(const uint32_t* table, int Vt, int vcur, uint64_t* ws, int call, void* stream) {
  BEAST_REQUIRE(table && ws && vcur >= 1 && vcur <= Vt, "beast_bpe_argmax: bad args");
  BEAST_REQUIRE(call >= 0, "beast_bpe_argmax: call index must be >= 0");
  hipLaunchKernelGGL(k_apply_argmax, dim3((vcur + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0,
                     beast::as_stream(stream), const_cast<uint32_t*>(table), nullptr, Vt, vcur, argws_view(ws, Vt),
                     call & 1, 0, 0, 0, 0, nullptr, WordIndex{}, false, false, nullptr, LoopHash{}, vcur);
  BEAST_LAUNCHED("k_apply_argmax");
  return BEAST_OK;
}

extern "C" int beast_bpe_apply_argmax(uint32_t* table, int32_t* deltas, int Vt, int vcur, int a, int b, int new_id,
                                      uint32_t* tlen, void* index, int new_id_reused, uint64_t* ws, int call,
                                      void* stream) {
  BEAST_REQUIRE(table && deltas && tlen && ws && vcur >= 1 && vcur <= Vt && call >= 0,
                "beast_bpe_apply_argmax: bad args");
  BEAST_REQUIRE(a >= 0 && a < Vt && b >= 0 && b < Vt && new_id >= 0 && new_id < Vt,
                "beast_bpe_apply_argmax: ids out of range");
  const WordIndex ix = index ? index_view(index, Vt) : WordIndex{};
  // every row that can change must run: rows < vcur, and a / b / new_id
  const int rows = std::max(vcur, std::max(a, std::max(b, new_id)) + 1);
  hipLaunchKernelGGL(k_apply_argmax, dim3((rows + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0,
                     beast::as_stream(stream), table, deltas, Vt, vcur, argws_view(ws, Vt), call & 1, 1, a, b, new_id,
                     tlen, ix, index != nullptr, new_id_reused != 0, nullptr, LoopHash{}, rows);
  BEAST_LAUNCHED("k_apply_argmax");
  return BEAST_OK;
}

extern "C" size_t beast_bpe_index_workspace_bytes(int Vt, int64_t pool_capacity) {
  return (size_t)(2 * (int64_t)Vt + 4 + pool_capacity) * 4;
}

extern "C" int beast_bpe_build_index(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen, int64_t n_words,
                                     int Vt, void* index, size_t index_bytes, void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && index && n_words >= 0 && Vt >= 1 && Vt <= 65535,
                "beast_bpe_build_index: bad args");
  const size_t head = (size_t)(2 * (int64_t)Vt + 4) * 4;
  BEAST_REQUIRE_CODE(index_bytes >= head + 4, BEAST_E_WORKSPACE, "index workspace too small");
  const int64_t cap = (int64_t)(index_bytes - head) / 4;
  BEAST_REQUIRE(cap < (int64_t)IDX_INEXACT, "index pool too large");
  hipStream_t s = beast::as_stream(stream);
  WordIndex ix = index_view(index, Vt);
  uint32_t* cursor = ix.pool;   // scratch: the first Vt pool slots are rewritten by the fill
  BEAST_REQUIRE_CODE(cap >= Vt, BEAST_E_WORKSPACE, "index pool smaller than the vocabulary");
  BEAST_HIP(hipMemsetAsync(index, 0, head, s), "index memset");
  const uint32_t capv = (uint32_t)cap;
  BEAST_HIP(hipMemcpyAsync(ix.ctl + 2, &capv, 4, hipMemcpyHostToDevice, s), "index cap");
  if (n_words > 0) {
    hipLaunchKernelGGL(k_index_words<false>, dim3(grid_for(n_words, 256, 8192)), dim3(256), 0, s, sym, wstart, wlen,
                       n_words, ix, cursor);
    BEAST_LAUNCHED("k_index_words");
  }
  // cursor lives in a separate scratch region: reuse the (not yet filled) tail of the pool
  uint32_t* cur2 = ix.pool + (cap - Vt);
  hipLaunchKernelGGL(k_index_scan, dim3(1), dim3(1024), 0, s, ix, Vt, cur2);
  BEAST_LAUNCHED("k_index_scan");
  if (n_words > 0) {
    hipLaunchKernelGGL(k_index_words<true>, dim3(grid_for(n_words, 256, 8192)), dim3(256), 0, s, sym, wstart, wlen,
                       n_words, ix, cur2);
    BEAST_LAUNCHED("k_index_words");
  }
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

extern "C" int beast_bpe_merge(uint16_t* sym, const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount,
                               int64_t n_words, int a, int b, int new_id, const uint32_t* tlen, int max_token_length,
                               int32_t* deltas, int Vt, uint64_t* sig, void* index, int64_t pair_count,
                               void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && tlen && deltas, "beast_bpe_merge: null pointer");
  BEAST_REQUIRE(a >= 0 && a < Vt && b >= 0 && b < Vt && new_id >= 0 && new_id < Vt && Vt <= 65535,
                "beast_bpe_merge: ids out of range (a=%d b=%d new=%d Vt=%d)", a, b, new_id, Vt);
  if (n_words <= 0) return BEAST_OK;
  hipStream_t s = beast::as_stream(stream);
  const size_t lds = (size_t)4 * Vt * sizeof(int32_t);
  const bool use_lds = lds <= 64 * 1024 && pair_count >= beast::g_merge_lds_min;
  const int grid = use_lds ? merge_grid<1>(n_words, lds) : merge_grid<0>(n_words, 0);
  unsigned long long* sg = reinterpret_cast<unsigned long long*>(sig);
  const WordIndex ix = index ? index_view(index, Vt) : WordIndex{};
  // LDS-privatised deltas only for frequent pairs: a rare pair touches few words, and the
  // per-workgroup LDS clear / flush would dominate (global atomics then)
  if (use_lds)
    hipLaunchKernelGGL(k_merge<1>, dim3(grid), dim3(256), lds, s, sym, wstart, wlen, wcount, n_words, a, b, new_id,
                       const_cast<uint32_t*>(tlen), max_token_length, deltas, Vt, sg, ix, index != nullptr, nullptr, 0ll,
                       ArgWs{}, LoopHash{});
  else
    hipLaunchKernelGGL(k_merge<0>, dim3(grid), dim3(256), 0, s, sym, wstart, wlen, wcount, n_words, a, b, new_id,
                       const_cast<uint32_t*>(tlen), max_token_length, deltas, Vt, sg, ix, index != nullptr, nullptr, 0ll,
                       ArgWs{}, LoopHash{});
  BEAST_LAUNCHED("k_merge");
  return BEAST_OK;
}


// ---- device-driven loop: workspace = LoopState | hash table | token hashes | merge log
static int loop_log2cap(int Vt) {
  int l = 6;
  while ((1 << l) < 2 * Vt) ++l;
  return l;
}

static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

struct LoopLayout {
  size_t st, key, klen, kid, th, tp, log, total;
};

static LoopLayout loop_layout(int Vt, int max_merges) {
  const size_t cap = size_t(1) << loop_log2cap(Vt);
  LoopLayout L;
  size_t o = 0;
  L.st = o;   o += al256(sizeof(LoopState));
  L.key = o;  o += al256(cap * 8);
  L.klen = o; o += al256(cap * 4);
  L.kid = o;  o += al256(cap * 4);
  L.th = o;   o += al256((size_t)Vt * 8);
  L.tp = o;   o += al256((size_t)Vt * 8);
  L.log = o;  o += al256((size_t)max_merges * 16);
  L.total = o;
  return L;
}

static LoopHash loop_hash_view(void* ws, int Vt, int max_merges) {
  const LoopLayout L = loop_layout(Vt, max_merges);
  unsigned char* w = static_cast<unsigned char*>(ws);
  LoopHash lh;
  lh.key = reinterpret_cast<unsigned long long*>(w + L.key);
  lh.klen = reinterpret_cast<uint32_t*>(w + L.klen);
  lh.kid = reinterpret_cast<int32_t*>(w + L.kid);
  lh.th = reinterpret_cast<unsigned long long*>(w + L.th);
  lh.tp = reinterpret_cast<unsigned long long*>(w + L.tp);
  lh.log = reinterpret_cast<int32_t*>(w + L.log);
  return lh;
}

static __global__ void k_loop_init(LoopState* st, LoopState init, LoopHash lh, int n_tok, int log2cap,
                            const unsigned long long* __restrict__ h0, const unsigned long long* __restrict__ p0,
                            const uint32_t* __restrict__ tlen) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *st = init;
  if (i >= n_tok) return;
  const unsigned long long h = h0[i];
  lh.th[i] = h;
  lh.tp[i] = p0[i];
  const uint64_t mask = (1ull << log2cap) - 1;
  uint64_t sl = loop_slot(h, tlen[i], log2cap);
  while (true) {   // the initial tokens are distinct strings
    const uint32_t prev = atomicCAS(&lh.klen[sl], LOOP_EMPTY, tlen[i]);
    if (prev == LOOP_EMPTY) { lh.key[sl] = h; lh.kid[sl] = i; break; }
    sl = (sl + 1) & mask;
  }
}

#ifdef BPE_MERGE_STAMPS
extern "C" int beast_debug_merge_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_stamps), sizeof(g_bpe_stamps)) == hipSuccess ? 0 : -2;
}
extern "C" int beast_debug_apply_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_apply_stamps), sizeof(g_apply_stamps)) == hipSuccess ? 0 : -2;
}
extern "C" int beast_debug_decide_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_dstamps), sizeof(g_bpe_dstamps)) == hipSuccess ? 0 : -2;
}
#endif
#ifdef BPE_MERGE_STATS
extern "C" int beast_debug_merge_stats(unsigned long long* host4) {
  return hipMemcpyFromSymbol(host4, HIP_SYMBOL(g_merge_stats), sizeof(g_merge_stats)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" size_t beast_bpe_loop_workspace_bytes(int Vt, int max_merges) {
  return loop_layout(Vt, max_merges).total;
}

extern "C" int beast_bpe_loop_init(void* ws, size_t ws_bytes, int Vt, int max_merges, int n_tokens, int vocab_size,
                                   int min_frequency, int argmax_parity, const uint64_t* tok_hash,
                                   const uint64_t* tok_pow, const uint32_t* tlen, void* stream) {
  BEAST_REQUIRE(ws && tok_hash && tok_pow && tlen, "beast_bpe_loop_init: null pointer");
  BEAST_REQUIRE(Vt >= 1 && Vt <= 32768 && n_tokens >= 0 && n_tokens <= Vt && max_merges >= 1,
                "beast_bpe_loop_init: bad sizes");
  const LoopLayout L = loop_layout(Vt, max_merges);
  BEAST_REQUIRE_CODE(ws_bytes >= L.total, BEAST_E_WORKSPACE, "loop workspace %zu < %zu", ws_bytes, L.total);
  hipStream_t s = beast::as_stream(stream);
  unsigned char* w = static_cast<unsigned char*>(ws);
  BEAST_HIP(hipMemsetAsync(w + L.klen, 0xFF, L.kid - L.klen, s), "loop hash memset");
  LoopState init{};
  init.active = 1;
  init.vcur = n_tokens;
  init.parity = argmax_parity & 1;
  init.target = vocab_size;
  init.min_freq = min_frequency;
  init.log2cap = loop_log2cap(Vt);
  init.max_merges = max_merges;
  const int n = n_tokens > 0 ? n_tokens : 1;
  hipLaunchKernelGGL(k_loop_init, dim3((n + 255) / 256), dim3(256), 0, s, reinterpret_cast<LoopState*>(w + L.st), init,
                     loop_hash_view(ws, Vt, max_merges), n_tokens, init.log2cap,
                     reinterpret_cast<const unsigned long long*>(tok_hash),
                     reinterpret_cast<const unsigned long long*>(tok_pow), tlen);
  BEAST_LAUNCHED("k_loop_init");
  return BEAST_OK;
}

extern "C" int beast_bpe_loop_steps(void* ws, int Vt, int max_merges, int n_steps, uint16_t* sym,
                                    const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount, int64_t n_words,
                                    uint32_t* tlen, int max_token_length, int32_t* deltas, uint64_t* sig,
                                    void* index, uint32_t* table, uint64_t* argws, int vocab_size, void* stream) {
  BEAST_REQUIRE(ws && sym && wstart && wlen && tlen && deltas && table && argws, "beast_bpe_loop_steps: null pointer");
  BEAST_REQUIRE(Vt >= 1 && Vt <= 32768 && n_steps >= 0 && vocab_size >= 1, "beast_bpe_loop_steps: bad sizes");
  hipStream_t s = beast::as_stream(stream);
  const LoopLayout L = loop_layout(Vt, max_merges);
  LoopState* st = reinterpret_cast<LoopState*>(static_cast<unsigned char*>(ws) + L.st);
  const LoopHash lh = loop_hash_view(ws, Vt, max_merges);
  const ArgWs aw = argws_view(argws, Vt);
  const size_t lds = (size_t)4 * Vt * sizeof(int32_t);
  BEAST_REQUIRE_CODE(lds <= 64 * 1024, BEAST_E_UNSUPPORTED, "device loop needs 4*Vt int32 of LDS (Vt <= 4096)");
  const int grid = merge_grid<2>(n_words > 0 ? n_words : 1, lds);
  unsigned long long* sg = reinterpret_cast<unsigned long long*>(sig);
  const WordIndex ix = index ? index_view(index, Vt) : WordIndex{};
  // every row that can change: ids < vocab_size (and < Vt)
  const int rows = std::min(Vt, std::max(vocab_size, 1));
  for (int i = 0; i < n_steps; ++i) {   // k_merge decides the merge (even with no words left)
    hipLaunchKernelGGL(k_merge<2>, dim3(grid), dim3(256), lds, s, sym, wstart, wlen, wcount, n_words, 0, 0, 0, tlen,
                       max_token_length, deltas, Vt, sg, ix, index != nullptr, st, (long long)beast::g_merge_lds_min,
                       aw, lh);
    BEAST_LAUNCHED("k_merge");
    hipLaunchKernelGGL(k_apply_argmax, dim3((rows + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0, s,
                       table, deltas, Vt, 0, aw, 0, 1, 0, 0, 0, tlen, ix, index != nullptr, false, st, lh, rows);
    BEAST_LAUNCHED("k_apply_argmax");
  }
  return BEAST_OK;
}

extern "C" size_t beast_bpe_batch_workspace_bytes(int Vt) { return batch_ws_bytes(Vt > 0 ? Vt : 1); }

template <int KM>
static int batch_grid(int64_t nw) {
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_merge_batch<KM>, 256, 0) != hipSuccess || per <= 0)
      per = 2;
    resident = cus * per;
  }
  return grid_for(nw, MERGE_SCAN * 256, resident);
}

template <int KM>
static int loop_batch(LoopState* st, const LoopHash& lh, BatchWs bw, ArgWs aw, int Vt, int n_steps, uint16_t* sym,
                      const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount, int64_t n_words, uint32_t* tlen,
                      int max_token_length, uint64_t* sig, uint32_t* table, int rows, hipStream_t s) {
  const int grid = batch_grid<KM>(n_words > 0 ? n_words : 1);
  const int agrid = (rows + APPLY_ROWS - 1) / APPLY_ROWS;
  for (int i = 0; i < n_steps; ++i) {
    hipLaunchKernelGGL(k_merge_batch<KM>, dim3(grid), dim3(256), 0, s, sym, wstart, wlen, wcount, n_words, tlen,
                       max_token_length, Vt, reinterpret_cast<unsigned long long*>(sig), st, lh, bw, table, aw,
                       (long long)beast::g_merge_lds_min);
    BEAST_LAUNCHED("k_merge_batch");
    hipLaunchKernelGGL(k_apply_batch, dim3(agrid), dim3(64 * APPLY_ROWS), 0, s, table, Vt, aw, bw, tlen, st, lh, rows, 0);
    BEAST_LAUNCHED("k_apply_batch");
  }
  return BEAST_OK;
}

extern "C" int beast_bpe_loop_batch(void* ws, int Vt, int max_merges, int n_steps, int max_batch, uint16_t* sym,
                                    const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount, int64_t n_words,
                                    uint32_t* tlen, int max_token_length, uint64_t* sig, uint32_t* table,
                                    uint64_t* argws, void* batch_ws, size_t batch_ws_bytes_, int vocab_size, int init,
                                    void* stream) {
  BEAST_REQUIRE(ws && sym && wstart && wlen && tlen && sig && table && argws && batch_ws,
                "beast_bpe_loop_batch: null pointer");
  BEAST_REQUIRE(Vt >= 1 && n_steps >= 0 && vocab_size >= 1, "beast_bpe_loop_batch: bad sizes");
  BEAST_REQUIRE_CODE(Vt <= 4096, BEAST_E_UNSUPPORTED, "batched merge loop: Vt %d > 4096", Vt);
  BEAST_REQUIRE(max_batch == 2 || max_batch == 4 || max_batch == 8, "beast_bpe_loop_batch: max_batch must be 2, 4 or 8");
  BEAST_REQUIRE_CODE(batch_ws_bytes_ >= batch_ws_bytes(Vt), BEAST_E_WORKSPACE, "batch workspace %zu < %zu",
                     batch_ws_bytes_, batch_ws_bytes(Vt));
  hipStream_t s = beast::as_stream(stream);
  const LoopLayout L = loop_layout(Vt, max_merges);
  LoopState* st = reinterpret_cast<LoopState*>(static_cast<unsigned char*>(ws) + L.st);
  const LoopHash lh = loop_hash_view(ws, Vt, max_merges);
  const ArgWs aw = argws_view(argws, Vt);
  const BatchWs bw = batch_view(batch_ws, Vt);
  const int rows = std::min(Vt, std::max(vocab_size, 1));
  if (init) {   // every row's best and second-best, the workgroups' best rows
    BEAST_HIP(hipMemsetAsync(batch_ws, 0, batch_ws_bytes(Vt), s), "batch workspace memset");
    hipLaunchKernelGGL(k_apply_batch, dim3((rows + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0, s, table,
                       Vt, aw, bw, tlen, st, lh, rows, 1);
    BEAST_LAUNCHED("k_apply_batch(init)");
  }
  switch (max_batch) {
    case 2: return loop_batch<2>(st, lh, bw, aw, Vt, n_steps, sym, wstart, wlen, wcount, n_words, tlen,
                                 max_token_length, sig, table, rows, s);
    case 4: return loop_batch<4>(st, lh, bw, aw, Vt, n_steps, sym, wstart, wlen, wcount, n_words, tlen,
                                 max_token_length, sig, table, rows, s);
    default: return loop_batch<8>(st, lh, bw, aw, Vt, n_steps, sym, wstart, wlen, wcount, n_words, tlen,
                                  max_token_length, sig, table, rows, s);
  }
}

extern "C" size_t beast_bpe_pair_index_bytes(int n_sym, int64_t n_symbols) {
  const size_t P = (size_t)(n_sym > 0 ? n_sym : 1) * (size_t)(n_sym > 0 ? n_sym : 1);
  return al256((P + 1) * 4) + al256(P * 4) + al256((size_t)(n_symbols > 0 ? n_symbols : 1) * 4);
}

extern "C" int beast_bpe_build_pair_index(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen,
                                          int64_t n_words, int n_sym, int64_t n_symbols, void* ws, size_t ws_bytes,
                                          void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && ws && n_words >= 0 && n_symbols >= 0, "beast_bpe_build_pair_index: bad args");
  BEAST_REQUIRE(n_sym >= 1 && n_sym <= 4096, "beast_bpe_build_pair_index: n_sym %d not in [1, 4096]", n_sym);
  BEAST_REQUIRE(n_symbols < (int64_t)0xFFFFFFFF, "beast_bpe_build_pair_index: too many symbols");
  BEAST_REQUIRE_CODE(ws_bytes >= beast_bpe_pair_index_bytes(n_sym, n_symbols), BEAST_E_WORKSPACE,
                     "pair index workspace %zu < %zu", ws_bytes, beast_bpe_pair_index_bytes(n_sym, n_symbols));
  hipStream_t s = beast::as_stream(stream);
  const int64_t P = (int64_t)n_sym * n_sym;
  unsigned char* w = static_cast<unsigned char*>(ws);
  uint32_t* off = reinterpret_cast<uint32_t*>(w);
  uint32_t* cursor = reinterpret_cast<uint32_t*>(w + al256((P + 1) * 4));
  uint32_t* list = reinterpret_cast<uint32_t*>(w + al256((P + 1) * 4) + al256(P * 4));
  BEAST_HIP(hipMemsetAsync(cursor, 0, P * 4, s), "pair index memset");
  if (n_words > 0) {
    const size_t budget = 160 * 1024;
    const int R = (int)std::max<size_t>(1, std::min<size_t>((size_t)n_sym, budget / (4 * (size_t)n_sym)));
    const int groups = (n_sym + R - 1) / R;
    const size_t lds = (size_t)R * n_sym * 4;
    BEAST_REQUIRE_CODE(lds <= budget, BEAST_E_UNSUPPORTED, "pair index: one row needs %zu B of LDS", lds);
    if (lds > 65536) {
      BEAST_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pair_lists<false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "hipFuncSetAttribute");
      BEAST_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pair_lists<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "hipFuncSetAttribute");
    }
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    const int per_cu = std::max(1, (int)(budget / lds));
    const int gx = std::max(1, std::min<int>(std::max(1, cus * per_cu / groups), (int)((n_words + 255) / 256)));
    hipLaunchKernelGGL(k_pair_lists<false>, dim3(gx, groups), dim3(256), lds, s, sym, wstart, wlen, n_words, n_sym, R,
                       cursor, list);
    BEAST_LAUNCHED("k_pair_lists<count>");
    hipLaunchKernelGGL(k_pair_scan, dim3(1), dim3(1024), 0, s, off, cursor, P);
    BEAST_LAUNCHED("k_pair_scan");
    hipLaunchKernelGGL(k_pair_lists<true>, dim3(gx, groups), dim3(256), lds, s, sym, wstart, wlen, n_words, n_sym, R,
                       cursor, list);
    BEAST_LAUNCHED("k_pair_lists<fill>");
  } else {
    BEAST_HIP(hipMemsetAsync(off, 0, (P + 1) * 4, s), "pair index memset");
  }
  return BEAST_OK;
}

// Token index for the pair-index loop: no setup lists (the pair CSR serves setup symbols), every
// id INEXACT until a merge creates it; the pool (8-byte entries) receives k_merge_ix's appends.
extern "C" int beast_bpe_token_index_init(void* index, size_t index_bytes, int Vt, void* stream) {
  BEAST_REQUIRE(index && Vt >= 1 && Vt <= 65535, "beast_bpe_token_index_init: bad args");
  const size_t head = (size_t)(2 * (int64_t)Vt + 4) * 4;
  BEAST_REQUIRE_CODE(index_bytes >= head + 4, BEAST_E_WORKSPACE, "token index workspace too small");
  const int64_t cap = (int64_t)(index_bytes - head) / 8;   // 8-byte {word, kind << 16 | symbol} entries
  BEAST_REQUIRE(cap < (int64_t)IDX_INEXACT, "token index pool too large");
  hipStream_t s = beast::as_stream(stream);
  WordIndex ix = index_view(index, Vt);
  BEAST_HIP(hipMemsetAsync(ix.start, 0, (size_t)Vt * 4, s), "token index memset");
  BEAST_HIP(hipMemsetAsync(ix.len, 0xFF, (size_t)Vt * 4, s), "token index memset");
  const uint32_t ctl[4] = {0u, 0u, (uint32_t)cap, 0u};
  BEAST_HIP(hipMemcpyAsync(ix.ctl, ctl, sizeof(ctl), hipMemcpyHostToDevice, s), "token index ctl");
  return BEAST_OK;
}

extern "C" int beast_bpe_loop_steps_ix(void* ws, int Vt, int max_merges, int n_steps, uint16_t* sym,
                                       const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount,
                                       int64_t n_words, uint32_t* tlen, int max_token_length, int32_t* deltas,
                                       const void* pair_index, int n_sym, void* token_index, uint32_t* claim,
                                       uint64_t* sig, uint32_t* table, uint64_t* argws, int vocab_size,
                                       uint32_t* apps, void* stream) {
  BEAST_REQUIRE(ws && sym && wstart && wlen && tlen && deltas && table && argws && token_index && claim,
                "beast_bpe_loop_steps_ix: null pointer");
  BEAST_REQUIRE(Vt >= 1 && Vt <= 32768 && n_steps >= 0 && vocab_size >= 1, "beast_bpe_loop_steps_ix: bad sizes");
  BEAST_REQUIRE(pair_index == nullptr || (n_sym >= 1 && n_sym <= Vt), "beast_bpe_loop_steps_ix: bad n_sym");
  hipStream_t s = beast::as_stream(stream);
  const LoopLayout L = loop_layout(Vt, max_merges);
  LoopState* st = reinterpret_cast<LoopState*>(static_cast<unsigned char*>(ws) + L.st);
  const LoopHash lh = loop_hash_view(ws, Vt, max_merges);
  const ArgWs aw = argws_view(argws, Vt);
  const size_t lds = (size_t)4 * Vt * sizeof(int32_t);
  BEAST_REQUIRE_CODE(lds <= 64 * 1024, BEAST_E_UNSUPPORTED, "device loop needs 4*Vt int32 of LDS (Vt <= 4096)");
  PairIndex px{};
  if (pair_index != nullptr) {
    const int64_t P = (int64_t)n_sym * n_sym;
    const unsigned char* w = static_cast<const unsigned char*>(pair_index);
    px.off = reinterpret_cast<const uint32_t*>(w);
    px.list = reinterpret_cast<const uint32_t*>(w + al256((P + 1) * 4) + al256(P * 4));
    px.nb = n_sym;
  }
  const WordIndex ix = index_view(token_index, Vt);
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_merge_ix, 256, lds) != hipSuccess || per <= 0) per = 4;
    resident = cus * per;
  }
  // as many workgroups as are resident: a list round or a signature sweep per workgroup
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(resident, (n_words + 255) / 256));
  unsigned long long* sg = reinterpret_cast<unsigned long long*>(sig);
  const int rows = std::min(Vt, std::max(vocab_size, 1));
  for (int i = 0; i < n_steps; ++i) {
    hipLaunchKernelGGL(k_merge_ix, dim3(grid), dim3(256), lds, s, sym, wstart, wlen, wcount, n_words, tlen,
                       max_token_length, deltas, Vt, ix, px, claim, sg, beast::g_merge_list_ratio, st,
                       (long long)beast::g_merge_lds_min, aw, lh, apps, max_merges);
    BEAST_LAUNCHED("k_merge_ix");
    hipLaunchKernelGGL(k_apply_argmax, dim3((rows + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0, s,
                       table, deltas, Vt, 0, aw, 0, 1, 0, 0, 0, tlen, ix, true, false, st, lh, rows);
    BEAST_LAUNCHED("k_apply_argmax");
  }
  return BEAST_OK;
}

extern "C" size_t beast_bpe_loop_persistent_bytes(void) { return 4096 + 8 * 4096; }

extern "C" int beast_bpe_loop_persistent(void* ws, int Vt, int max_merges, int n_steps, uint16_t* sym,
                                         const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount,
                                         int64_t n_words, uint32_t* tlen, int max_token_length, int32_t* deltas,
                                         uint64_t* sig, uint32_t* table, uint64_t* argws, int vocab_size,
                                         void* bar_ws, size_t bar_bytes, void* stream) {
  BEAST_REQUIRE(ws && sym && wstart && wlen && tlen && deltas && table && argws && bar_ws,
                "beast_bpe_loop_persistent: null pointer");
  BEAST_REQUIRE(Vt >= 1 && Vt <= 4096 && n_steps >= 0 && vocab_size >= 1, "beast_bpe_loop_persistent: bad sizes");
  BEAST_REQUIRE_CODE(bar_bytes >= beast_bpe_loop_persistent_bytes(), BEAST_E_WORKSPACE,
                     "persistent loop workspace %zu < %zu", bar_bytes, beast_bpe_loop_persistent_bytes());
  hipStream_t s = beast::as_stream(stream);
  int dev = 0, cus = 0, per = 0;
  BEAST_HIP(hipGetDevice(&dev), "hipGetDevice");
  BEAST_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "CU count");
  const size_t lds = (size_t)4 * Vt * sizeof(int32_t);
  BEAST_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_bpe_loop, PL_T, lds), "occupancy");
  // one workgroup per CU, and only if the device holds at least that many at once: the barrier
  // needs every workgroup resident
  BEAST_REQUIRE_CODE(per >= 1 && cus >= 1 && cus <= 4096, BEAST_E_UNSUPPORTED,
                     "persistent loop: %d workgroups of %d threads per CU", per, PL_T);
  const int G = cus;
  const int rows = std::min(Vt, std::max(vocab_size, 1));
  BEAST_REQUIRE_CODE((rows + G - 1) / G <= PL_T / 64, BEAST_E_UNSUPPORTED,
                     "persistent loop: %d table rows over %d workgroups", rows, G);
  const LoopLayout L = loop_layout(Vt, max_merges);
  LoopState* st = reinterpret_cast<LoopState*>(static_cast<unsigned char*>(ws) + L.st);
  const LoopHash lh = loop_hash_view(ws, Vt, max_merges);
  const ArgWs aw = argws_view(argws, Vt);
  unsigned char* b = static_cast<unsigned char*>(bar_ws);
  PlBar pb;
  pb.sub = reinterpret_cast<unsigned int*>(b);
  pb.top = pb.sub + PL_GROUPS;
  pb.abort_flag = pb.top + 1;
  pb.bests = reinterpret_cast<unsigned long long*>(b + 4096);
  BEAST_HIP(hipMemsetAsync(bar_ws, 0, 4096, s), "persistent loop memset");
  hipLaunchKernelGGL(k_bpe_loop, dim3(G), dim3(PL_T), lds, s, sym, wstart, wlen, wcount, n_words, tlen,
                     max_token_length, deltas, Vt, rows, reinterpret_cast<unsigned long long*>(sig), table, st, lh,
                     aw, pb, n_steps, (long long)beast::g_merge_lds_min);
  BEAST_LAUNCHED("k_bpe_loop");
  return BEAST_OK;
}

extern "C" int beast_bpe_loop_state(const void* ws, int Vt, int max_merges, const void** state, const void** log) {
  BEAST_REQUIRE(ws && state && log, "beast_bpe_loop_state: null pointer");
  const LoopLayout L = loop_layout(Vt, max_merges);
  *state = static_cast<const unsigned char*>(ws) + L.st;
  *log = static_cast<const unsigned char*>(ws) + L.log;
  return BEAST_OK;
}

extern "C" size_t beast_bpe_dedup_workspace_bytes(int64_t n_words) {
  const uint64_t cap = dedup_cap(n_words > 0 ? n_words : 1);
  return (size_t)(cap * 12 + (uint64_t)(n_words > 0 ? n_words : 1) * 8 + 64);
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
  ws.cap = dedup_cap(n);
  char* p = static_cast<char*>(workspace);
  ws.keys = reinterpret_cast<unsigned long long*>(p);  p += ws.cap * 8;
  ws.cnt = reinterpret_cast<uint32_t*>(p);              p += ws.cap * 4;
  ws.rep = reinterpret_cast<uint32_t*>(p);              p += n * 4;
  ws.slot = reinterpret_cast<uint32_t*>(p);             p += n * 4;
  ws.nu = reinterpret_cast<unsigned long long*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
  BEAST_HIP(hipMemsetAsync(workspace, 0, ws.cap * 12, s), "dedup memset");
  BEAST_HIP(hipMemsetAsync(ws.nu, 0, 8, s), "dedup memset");
  if (n_words > 0) {
    hipLaunchKernelGGL(k_dedup_insert, dim3(grid_for(n_words, 256, 16384)), dim3(256), 0, s, sym, wstart, wlen,
                       n_words, ws);
    BEAST_LAUNCHED("k_dedup_insert");
  }
  hipLaunchKernelGGL(k_dedup_gather, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, wstart, wlen, ws, out_wstart,
                     out_wlen, out_wcount, out_n);
  BEAST_LAUNCHED("k_dedup_gather");
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
