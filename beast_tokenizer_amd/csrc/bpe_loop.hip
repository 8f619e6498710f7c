// Byte-level BPE training, the merge loop, for gfx950: HF tokenizers' BpeTrainer::do_train as
// driven by FIGBPE (beast/beast_bpe_trainer.py:61-98; semantics SURVEY.md §8a H11).
//
// Two loops over the same word layout (distinct words x counts, length-ordered, one 64-bit
// Bloom signature per word; csrc/bpe_setup.hip builds it):
//
//   batched device loop (the default)   k_merge_batch + k_apply_batch<KM> per pass: each pass
//       applies up to 8 merges that are provably HF's next ones (see "batched merges"); the
//       decision of the next pass is made by the last workgroup of k_apply_batch, so
//       k_merge_batch starts scanning at once.  No host round trip per pass.
//   host-driven loop (fallback: vocabularies above 4096, a string-hash collision, the CPU
//       model of the trainer)            k_merge + k_apply_argmax per merge, the host picks.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bpe_common.h"
#include "common.h"

namespace {

__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }

// agent-scope (L1-bypassing, sc1) loads and stores: the hand-off between the workgroups of one
// k_apply_batch launch (MI355X_MICROARCH.md, "Workgroup dispatch ... inter-workgroup visibility")
template <class T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Only pairs with a positive count are candidates (the table holds int32 counts in u32 cells): a
// pair whose "+" was always blocked by max_token_length goes negative on its "-" updates, and HF
// never queues it (BpeTrainer pushes a pair only when its count is > 0), so neither do we.
// Incremental argmax state.  ws layout (u64): [2 + parity] result slots of the host-driven
// loop, [4, 4+Vt) the best key of each row, then u32 clean[Vt] (0 = rescan the row; the
// zero-filled workspace starts all-dirty).
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

// ------------------------------------------------------------ host-driven merge --
// HF's merge of (a, b) -> new in one word (Word::merge: left to right, non-overlapping) with the
// pair-count changes ((prev, a) -1, (prev, new) +1, (b, next) -1, (new, next) +1, weighted by the
// word's count; the +1s only while the new string stays shorter than max_token_length).  Returns
// the new length (0: the word holds no (a, b)), the new Bloom signature in g and the occurrences
// merged in napp.  Words of <= MERGE_REG symbols are read once into registers (all loads in
// flight together) and rewritten there: the in-place loop over global memory made every symbol a
// dependent round trip, and a merge waits for its slowest word.  48 holds nearly every K5 word
// (1,050 of 4.85 M exceed 32 symbols, the longest 58; 99.9% <= 27); 64 would cost k_merge_batch
// a wave per SIMD (174 VGPRs) and measured slower.
#ifndef BPE_MERGE_REG
#define BPE_MERGE_REG 48
#endif
constexpr int MERGE_REG = BPE_MERGE_REG;
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
  uint32_t r = 0, o = 0, py = 0;
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
    sg |= sig_sym(y) | (o ? sig_pair(py, y) : 0ull);
    py = y;
    s[o++] = (uint16_t)y;
  }
  g = sg;
  return o;
}

// A word of L <= MERGE_REG symbols in registers (sentinels past the end).  Words start at a
// multiple of 4 symbols and own their span rounded up to 4 (beast_bpe_repack_words), so the word
// is read as 8-byte units -- at most 8 loads in flight, not 32 two-byte ones.
__device__ __forceinline__ void load_word(const uint16_t* __restrict__ s, uint32_t L, uint32_t (&v)[MERGE_REG + 2]) {
  const uint2* __restrict__ p = reinterpret_cast<const uint2*>(s);
#pragma unroll
  for (int i = 0; i < MERGE_REG + 2; ++i) v[i] = 0xFFFFFFFFu;   // the sentinel everywhere first
  // then the units some active lane's word reaches, its positions past L kept at the sentinel (the
  // padding of a word's last unit is zero, a valid id): no select over all MERGE_REG positions
#pragma unroll
  for (int q = 0; q < MERGE_REG / 4; ++q) {
    if (__builtin_amdgcn_ballot_w64((uint32_t)(4 * q) < L) == 0ull) break;
    uint2 u = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    if ((uint32_t)(4 * q) < L) u = p[q];
    v[4 * q] = (uint32_t)(4 * q) < L ? (u.x & 0xFFFFu) : 0xFFFFFFFFu;
    v[4 * q + 1] = (uint32_t)(4 * q + 1) < L ? (u.x >> 16) : 0xFFFFFFFFu;
    v[4 * q + 2] = (uint32_t)(4 * q + 2) < L ? (u.y & 0xFFFFu) : 0xFFFFFFFFu;
    v[4 * q + 3] = (uint32_t)(4 * q + 3) < L ? (u.y >> 16) : 0xFFFFFFFFu;
  }
}
// Wave-uniform exit from the unrolled sweeps once no active lane's word reaches position i.
#define WORD_SWEEP_EXIT(i, L)                                                                  \
  if (((i) & 7) == 0 && (i) > 0 && __builtin_amdgcn_ballot_w64((uint32_t)(i) < (L)) == 0ull) \
    break
__device__ __forceinline__ bool word_has_pair(const uint32_t (&v)[MERGE_REG + 2], uint32_t L, uint32_t a, uint32_t b) {
  bool hit = false;
#pragma unroll
  for (int i = 0; i < MERGE_REG - 1; ++i) {
    WORD_SWEEP_EXIT(i, L);
    hit |= (v[i] == a) & (v[i + 1] == b);
  }
  return hit;
}
// The merge of a word held in v (which holds the pair), written back to s as 8-byte units: the
// output symbols collect in a 64-bit accumulator that is stored whenever it holds four (the
// units past the new length are the word's own dead span).  The sweep is branch-free and marks
// the occurrences (HF's left-to-right, non-overlapping rule); the pair-count changes then go one
// occurrence at a time in a rolled loop -- the left neighbour is new when an occurrence starts
// two symbols before, else v[i - 1], the right one v[i + 2] -- so the code that adds them exists
// once, not once per position (the unrolled form overflowed the instruction cache).
template <class Op>
__device__ __forceinline__ uint32_t merge_regs(const uint32_t (&v)[MERGE_REG + 2], uint32_t L, uint16_t* __restrict__ s,
                                               int32_t cnt, const Op& m, unsigned long long& g, uint32_t& napp) {
  const uint32_t a = (uint32_t)m.a, b = (uint32_t)m.b, nid = (uint32_t)m.nid;
  uint2* __restrict__ out = reinterpret_cast<uint2*>(s);
  uint32_t o = 0, py = 0;
  bool skip = false;
  unsigned long long sg = 0, acc = 0, occ = 0;
#pragma unroll
  for (int i = 0; i < MERGE_REG; ++i) {
    WORD_SWEEP_EXIT(i, L);
    const bool emit = ((uint32_t)i < L) & !skip;
    const bool hit = emit & (v[i] == a) & (v[i + 1] == b);   // v[i + 1] is the sentinel past the end
    occ |= (unsigned long long)hit << i;
    skip = hit;
    const uint32_t y = hit ? nid : v[i];
    if (emit) {
      acc |= (unsigned long long)y << (16 * (o & 3u));
      sg |= sig_sym(y) | (o ? sig_pair(py, y) : 0ull);
      py = y;
      ++o;
      if ((o & 3u) == 0) {
        out[(o >> 2) - 1] = make_uint2((uint32_t)acc, (uint32_t)(acc >> 32));
        acc = 0;
      }
    }
  }
  if (o & 3u) out[o >> 2] = make_uint2((uint32_t)acc, (uint32_t)(acc >> 32));
  g = sg;
  napp += (uint32_t)__builtin_popcountll(occ);
  for (unsigned long long rest = occ; rest; rest &= rest - 1) {
    const int i = __builtin_ctzll(rest);
    uint32_t lv = nid, rv = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < MERGE_REG; ++k) {
      // past every active lane's word the registers hold the sentinel rv starts with: stop there
      // (round 5: the chains ran all MERGE_REG positions for words of ~8 symbols)
      WORD_SWEEP_EXIT(k, L);
      lv = k + 1 == i ? v[k] : lv;
      rv = k == i + 2 ? v[k] : rv;
    }
    if (i >= 2 && ((occ >> (i - 2)) & 1ull)) lv = nid;
    if (i > 0) m.left(lv, cnt);
    if (rv != 0xFFFFFFFFu) m.right(rv, cnt);
  }
  return o;
}

template <class Op>
__device__ __forceinline__ uint32_t merge_symbols(uint16_t* __restrict__ s, uint32_t L, const uint32_t* __restrict__ wcount,
                                                  int64_t w, const Op& m, unsigned long long& g, uint32_t& napp) {
  const uint32_t a = (uint32_t)m.a, b = (uint32_t)m.b;
  if (L <= (uint32_t)MERGE_REG) {
    uint32_t v[MERGE_REG + 2];
    load_word(s, L, v);
    if (!word_has_pair(v, L, a, b)) return 0;
    return merge_regs(v, L, s, wcount ? (int32_t)wcount[w] : 1, m, g, napp);
  }
  return merge_global(s, L, wcount, w, m, g, napp);
}

constexpr int MERGE_SCAN = 8;       // signature loads in flight per thread (two-phase scan)
constexpr int MERGE_CLIST = 2048;   // LDS candidate list per workgroup (k_merge)
constexpr int BATCH_CLIST = 2 * 256 * MERGE_SCAN;   // k_merge_batch's list: two scan rounds

__device__ const uint32_t k_one_u32 = 1u;   // the count of every word when wcount is null

// One merge (a, b) -> nid over every word (the host-driven loop).  Deltas go to LDS (LDS = true,
// 4*Vt int32 <= 64 KiB) and are flushed once per workgroup into deltas[] with contiguous
// atomics, or straight to deltas[] by global atomics (rare pairs: the per-workgroup LDS clear
// and flush would dominate).  Two phases per workgroup over 256-word chunks taken round-robin
// (the words are length-sorted, so the Bloom candidates concentrate in the long-word tail):
// (1) every thread issues its MERGE_SCAN signature loads at once and lists the words whose
// signature holds the pair; (2) the workgroup's threads take the listed words in parallel.
template <bool LDS>
__global__ __launch_bounds__(256) void k_merge(uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                               uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount,
                                               int64_t nw, int a, int b, int nid, const uint32_t* __restrict__ tlen,
                                               int max_len, int32_t* __restrict__ deltas, int Vt,
                                               unsigned long long* __restrict__ sig) {
  extern __shared__ __attribute__((aligned(16))) int32_t dl[];
  __shared__ int touched, cn;
  __shared__ uint32_t clist[MERGE_CLIST];
  const int64_t nchunks = (nw + 255) / 256;
  if ((int64_t)blockIdx.x >= nchunks) return;   // block-uniform
  int32_t* dv = LDS ? dl : deltas;
  if (LDS)
    for (int i = threadIdx.x; i < 4 * Vt; i += blockDim.x) dl[i] = 0;
  if (threadIdx.x == 0) { touched = 0; cn = 0; }
  __syncthreads();
  const uint32_t newlen = tlen[a] + tlen[b];
  const MergeOp mop{a, b, nid, max_len, newlen, tlen, dv, dv + Vt, dv + 2 * Vt, dv + 3 * Vt};
  const unsigned long long need = sig_need((uint32_t)a, (uint32_t)b);
  bool any = false;
  auto merge_word = [&](int64_t w) {
    const uint32_t L = wlen[w];
    if (L < 2) return;
    unsigned long long g = 0;
    uint32_t napp = 0;
    const uint32_t o = merge_symbols(sym + wstart[w], L, wcount, w, mop, g, napp);
    if (!o) return;
    any = true;
    wlen[w] = o;
    sig[w] = g;
  };
  for (int64_t c0 = blockIdx.x; c0 < nchunks; c0 += (int64_t)MERGE_SCAN * gridDim.x) {
    unsigned long long sgv[MERGE_SCAN];
#pragma unroll
    for (int u = 0; u < MERGE_SCAN; ++u) {
      const int64_t w = (c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
      sgv[u] = w < nw ? sig[w] : 0ull;
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
  const int n = min(cn, MERGE_CLIST);
  for (int k = threadIdx.x; k < n; k += blockDim.x) merge_word(clist[k]);
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
}

// One wave per row x, APPLY_ROWS rows per workgroup (the apply touches only entries of rows it
// owns: (x, a) and (x, new) for every x, rows b and new entirely).  When `apply`:
// table += deltas for row x, deltas consumed are zeroed, row a's (a, b) is retired after its
// own adds (the only deltas that can reach (a, b) are row a's, when a == b), tlen[new] set.
// A row rescans only if it changed (or was never scanned); the workgroup folds its rows'
// bests and makes one atomicMax of the packed (count << 32 | ~(a * Vt + b)) into the result
// slot (ties -> smallest (a, b), HF's order).  That slot is one address that serialises at the
// memory side: 16 rows per workgroup (128 atomics for a 2,048-row table) instead of 4 (512)
// cut the merge loop 65.4 -> 61.6 ms at K5 (round 1).
constexpr int APPLY_ROWS = 16;
// The row's best key (and second-best) over columns < vcur, by the whole wave: all of a lane's
// loads of a 2,048-entry stretch in flight together.
__device__ __forceinline__ void rank_row(const uint32_t* __restrict__ row, int x, int Vt, int vcur, int lane,
                                         unsigned long long& best, unsigned long long& second) {
  best = second = 0ull;
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
}

__global__ __launch_bounds__(64 * APPLY_ROWS) void k_apply_argmax(uint32_t* __restrict__ table,
                                                                 int32_t* __restrict__ deltas, int Vt, int vcur,
                                                                 ArgWs aw, int parity, int apply, int a, int b,
                                                                 int nid, uint32_t* __restrict__ tlen, int nrows) {
  __shared__ unsigned long long wbest[APPLY_ROWS];
  __shared__ int changed_w[APPLY_ROWS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (blockIdx.x == 0 && threadIdx.x == 0) aw.slot[parity ^ 1] = 0ull;
  const int x0 = blockIdx.x * APPLY_ROWS;
  const int x = x0 + wave;
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
      table[(size_t)x * Vt + b] = 0u;   // never re-picked
      tlen[nid] = tlen[a] + tlen[b];
      changed_w[wave] = 1;
    }
    if (a >= x0 && a < x0 + APPLY_ROWS) __syncthreads();
    changed = changed_w[wave];
  }
  if (x < nrows && x < vcur) {
    if (aw.clean[x] && !changed) {
      best = aw.rowbest[x];
    } else {
      unsigned long long second;
      rank_row(table + (size_t)x * Vt, x, Vt, vcur, lane, best, second);
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
// row already taken.  k_apply_batch keeps every row's best and second-best key and each
// workgroup's BK best rows (best, second); the workgroup that arrives last reduces them to the
// global BK best rows and stops the batch where an accepted row's second-best would come
// first.  Measured at K5: 1,724 merges in 514 passes (BK = 8), 627 (4), 965 (2).
constexpr int BK = 8;                 // merges per batch at most
constexpr int BATCH_LDS = 32768;      // bytes of LDS delta vectors per workgroup (k_merge's 4 * Vt int32 at Vt 2048)
constexpr int BATCH_WG_LANE = 4;      // apply-workgroup lists per lane of the deciding wave (Vt <= 4096)

// The loop's device state: counters, the string hash table's geometry and the batch the next
// k_merge_batch applies.  The batch record (b*) is written by the deciding wave of k_apply_batch
// (or k_loop_init); the counters (vcur, n_merges, maxtlen) by workgroup 0 of k_merge_batch when
// it commits the batch; every other reader is in a later kernel.
struct LoopState {
  int32_t active;        // 0 once the loop has stopped (later launches are no-ops)
  int32_t vcur;          // vocabulary size (committed merges)
  int32_t n_merges;      // merges logged
  int32_t target;        // vocab_size
  int32_t min_freq;
  int32_t log2cap;       // token-string hash table
  int32_t max_merges;    // log capacity
  int32_t maxtlen;       // longest committed token (HF length units)
  uint32_t ticket;       // k_apply_batch workgroups arrived in this launch
  int32_t passes;        // batches decided
  // the batch the next k_merge_batch applies (and commits: its workgroup 0)
  int32_t bn;            // merges (0: none; the loop has stopped)
  int32_t bv0, bnm0;     // vocabulary size and merges logged before the batch
  int32_t bvcur;         // vocabulary size after the batch
  int32_t bkd;           // merges 0 .. bkd-1 sum their pair-count changes in LDS first
  int32_t bmt;           // longest token a word can hold during the batch (its new ones included)
  int32_t ba[BK], bb[BK], bnid[BK], breused[BK];
  uint32_t blen[BK];
  unsigned long long bh[BK];
};

// Token strings are identified by (64-bit polynomial hash of their UTF-8 bytes, byte length):
// h(xy) = h(x) * P^len(y) + h(y), so a merge's string is hashed from its parts.  The table maps
// (h, len) -> id; equal strings always collide (HF reuses the id), different strings collide
// with probability ~2^-64 -- the host re-checks every logged merge against the real strings
// and reruns on the host-driven loop if it ever finds one (beast_tokenizer_amd/bpe_train.py).
// A slot is two 8-byte words loaded together (one round trip per probe step): the hash, and
// (length << 32 | id), all ones while the slot is free.
constexpr unsigned long long LOOP_EMPTY = ~0ull;
struct LoopHash {
  unsigned long long* key;   // [cap] h
  unsigned long long* lid;   // [cap] byte length << 32 | id, LOOP_EMPTY = free slot
  unsigned long long* th;    // [Vt] token hash
  unsigned long long* tp;    // [Vt] P^len
  int32_t* log;              // [max_merges][4] a, b, nid, reused
};
__device__ __forceinline__ unsigned long long lid_of(uint32_t len, int id) {
  return ((unsigned long long)len << 32) | (uint32_t)id;
}

__device__ __forceinline__ uint64_t loop_slot(unsigned long long h, uint32_t len, int log2cap) {
  return ((h ^ ((unsigned long long)len * 0x9E3779B97F4A7C15ull)) * 0xbf58476d1ce4e5b9ull) >> (64 - log2cap);
}

constexpr int KR = 4;   // candidate pairs per table row: its KR best, in HF order
// Each row's cached keys: rowtop[x][0 .. RT_K) descending (0 past them) are exactly the row's keys
// >= rowtop[x][RT_F] (the floor; 1 when they are all its positive keys).  RT_K = 8 (round 5): a
// full re-rank runs RT_K wave-max rounds, and 8 keys measured faster at K5 than 6, 10, 12 or 14
// (19.5 vs 19.5-20.2 ms, profiles/r05/bpe_loop_ab_rtk_r05k.txt) -- fewer rounds per re-rank
// against re-ranks a little more often.  A batch changes a row
// outside b_j / new_j only at known columns, so re-reading those keeps the invariant; the row is
// re-ranked in full only when fewer than KR + 1 keys stay above a floor > 1.
#ifndef BPE_RT_K
#define BPE_RT_K 8
#endif
constexpr int RT_K = BPE_RT_K, RT_F = 15, RT_STRIDE = 16;
static_assert(RT_K < RT_F, "the floor's slot follows the cached keys");
struct BatchWs {
  unsigned long long* rowtop;         // [Vt][RT_STRIDE]: the row caches above
  unsigned long long* wgkey;          // [BK][nwg] each apply workgroup's BK best candidates, best first (k-major:
  unsigned long long* wgsec;          // [BK][nwg]  the deciding wave reads them coalesced) and their rows' bounds
};
__host__ __device__ inline int batch_nwg(int Vt) { return (Vt + APPLY_ROWS - 1) / APPLY_ROWS; }
__host__ __device__ inline size_t batch_ws_bytes(int Vt) {
  return ((size_t)Vt * RT_STRIDE * 8 + (size_t)batch_nwg(Vt) * BK * 2 * 8 + 255) & ~size_t(255);
}
__host__ __device__ inline BatchWs batch_view(void* ws, int Vt) {
  BatchWs v;
  char* p = static_cast<char*>(ws);
  const size_t nt = (size_t)batch_nwg(Vt) * BK;
  v.rowtop = reinterpret_cast<unsigned long long*>(p);
  v.wgkey = v.rowtop + (size_t)Vt * RT_STRIDE;
  v.wgsec = v.wgkey + nt;
  return v;
}

// Pair-count changes of batch merge j: kind 0 (x, a_j) -1, 1 (x, new_j) +1, 2 (b_j, y) -1,
// 3 (new_j, y) +1.  One GPU: straight into the pair table (the apply has nothing to add); a row
// x touched through kinds 0 / 1 is marked for re-ranking (clean[x] = 0); rows a_j, b_j, new_j
// always are.  Sharded (dg != null): into this rank's delta vectors [BK][4][Vt], all-reduced
// before k_apply_batch adds them.  The first merges of the batch whose four vectors fit
// BATCH_LDS (symbols < stride = vcur + n) sum them in LDS first when their count is large
// (k_merge's rule).  A neighbour may be a token this batch creates: its length is in nlen (tlen
// is written when the batch is committed).
struct BatchOp {
  int a, b, nid, max_len, Vt, vbase, nnew, stride;
  bool short_all;       // every token + the new one < max_len: no length lookups
  uint32_t newlen;
  const uint32_t* __restrict__ tlen;
  const uint32_t* nlen;
  int32_t* dl;          // LDS vectors of this merge, or null
  int32_t* dg;          // sharded: this merge's global delta vectors [4][Vt], or null
  uint32_t* table;
  uint32_t* clean;
  __device__ __forceinline__ uint32_t len_of(uint32_t x) const {
    return (int)x >= vbase && (int)x < vbase + nnew ? nlen[x - vbase] : tlen[x];
  }
  __device__ __forceinline__ void table_add(int kind, uint32_t x, int32_t v) const {
    if (dg != nullptr) {
      atomicAdd(&dg[kind * Vt + x], v);
    } else if (kind < 2) {
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
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));    // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));    // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));    // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));    // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));   // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// The wave max of 64-bit keys (count << 32 | tie-break) as 32-bit DPP steps: the largest high word
// first, then the largest low word among the lanes holding it -- one lane in the common case (a
// readlane), a second 32-bit max only on ties.  Keys of count 0 are 0 in every caller.  K5 loop
// 19.8 vs 19.9-20.0 ms with the 64-bit DPP form (profiles/r05/bpe_loop_ab_r05f.txt).
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  const uint32_t hi = (uint32_t)(v >> 32);
  const uint32_t mh = wave_max_u32(hi);
  const bool cand = hi == mh;
  const unsigned long long b = __ballot(cand);
  const uint32_t lo = cand ? (uint32_t)v : 0u;
  const uint32_t ml = __popcll(b) == 1 ? (uint32_t)__builtin_amdgcn_readlane((int)lo, (int)__builtin_ctzll(b))
                                       : wave_max_u32(lo);
  return ((unsigned long long)mh << 32) | ml;
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

// The row's RT_K best keys (descending, 0 past its positive pairs) and its floor, by the whole
// wave, into out[RT_STRIDE] (LDS).  A key is count << 32 | ~(x * Vt + y): larger = earlier in HF
// order.  Lane `lane` holds columns i * 64 + lane of each 2,048-column stretch (neighbouring ids
// -- frequent tokens often are -- on different lanes); it keeps its best two by (count desc,
// column asc) -- its columns rise with i, so a strict '>' keeps the first of equal counts -- and
// wave-max rounds pop the owner's current one.  A lane popped past its second rescans its counts below the last one
// (registers for one stretch; Vt <= 4,096 is two).  RT_K rounds: the cache outlives many batches.
constexpr int ROW_STRETCH = 2048;
__device__ __forceinline__ void row_counts(const uint32_t* __restrict__ row, int Vt, int vcur, int lane, int base,
                                           int32_t (&c)[32]) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int y = base + i * 64 + lane;
    c[i] = y < vcur ? (int32_t)row[y] : 0;
  }
}
__device__ __forceinline__ int row_col(int idx, int lane) {   // idx = stretch * 32 + i
  return (idx >> 5) * ROW_STRETCH + (idx & 31) * 64 + lane;
}
__device__ __forceinline__ unsigned long long row_key(int32_t cnt, int x, int Vt, int y) {
  return cnt > 0 ? ((unsigned long long)(uint32_t)cnt << 32) | (unsigned long long)(~((uint32_t)x * (uint32_t)Vt + (uint32_t)y))
                 : 0ull;
}
__device__ __forceinline__ int key_col(unsigned long long k, int x, int Vt) {
  return (int)(~(uint32_t)k - (uint32_t)x * (uint32_t)Vt);
}

#ifndef BPE_RT_LANE
#define BPE_RT_LANE 2
#endif
constexpr int RT_LANE = BPE_RT_LANE;   // best counts kept per lane by the first pass over the row
__device__ __forceinline__ void rank_row_top(const uint32_t* __restrict__ row, int x, int Vt, int vcur, int lane,
                                             unsigned long long* __restrict__ out) {
  // Each lane keeps its RT_LANE best (count desc, column asc) from one pass; a lane owning more
  // of the row's top keys than it kept rescans its counts (a 32-step loop per extra pop).  Two
  // measured faster than four at K5 (20.1-20.3 vs 20.5-20.6 ms, profiles/r05/bpe_loop_ab_r05d.txt):
  // the sorted insert costs every element more than the rare rescans it saves.
  const int nst = (vcur + ROW_STRETCH - 1) / ROW_STRETCH;
  int32_t c[32];
  int32_t tc[RT_LANE];
  int ti[RT_LANE];
#pragma unroll
  for (int q = 0; q < RT_LANE; ++q) { tc[q] = 0; ti[q] = -1; }
  for (int st = 0; st < nst; ++st) {
    row_counts(row, Vt, vcur, lane, st * ROW_STRETCH, c);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int32_t v = c[i];
      const int idx = st * 32 + i;
      // insert into the sorted list; strict '>' keeps the earlier column first on equal counts
      bool g[RT_LANE];
#pragma unroll
      for (int q = 0; q < RT_LANE; ++q) g[q] = v > tc[q];
#pragma unroll
      for (int q = RT_LANE - 1; q > 0; --q) {
        tc[q] = g[q - 1] ? tc[q - 1] : (g[q] ? v : tc[q]);
        ti[q] = g[q - 1] ? ti[q - 1] : (g[q] ? idx : ti[q]);
      }
      tc[0] = g[0] ? v : tc[0];
      ti[0] = g[0] ? idx : ti[0];
    }
  }
  int32_t cc = tc[0];
  int ci = ti[0];
  int next = 1;   // (tc[next], ti[next]) is the lane's next while next < RT_LANE
  unsigned long long w = 0ull;
#pragma unroll 1
  for (int r = 0; r < RT_K; ++r) {   // rolled: one copy of the body stays in the instruction cache
    const unsigned long long k = row_key(cc, x, Vt, row_col(ci, lane));
    w = wave_max_u64(k);
    if (lane == 0) out[r] = w;
    if (r + 1 < RT_K && w != 0ull && k == w) {   // the owner (keys are distinct) moves to its next
      if (next < RT_LANE) {
        int32_t nc = tc[0];
        int ni = ti[0];
#pragma unroll
        for (int q = 1; q < RT_LANE; ++q) {
          nc = q == next ? tc[q] : nc;
          ni = q == next ? ti[q] : ni;
        }
        cc = nc;
        ci = ni;
        ++next;
      } else {   // rare: its best below (cc, ci)
        int32_t nc = 0;
        int ni = -1;
        for (int st = 0; st < nst; ++st) {
          if (nst > 1) row_counts(row, Vt, vcur, lane, st * ROW_STRETCH, c);
#pragma unroll
          for (int i = 0; i < 32; ++i) {
            const int32_t v = c[i];
            const int idx = st * 32 + i;
            const bool take = ((v < cc) | ((v == cc) & (idx > ci))) & (v > nc);   // no short-circuit branches
            nc = take ? v : nc;
            ni = take ? idx : ni;
          }
        }
        cc = nc;
        ci = ni;
      }
    }
  }
  if (lane == 0) out[RT_F] = w != 0ull ? w : 1ull;
}

// A row outside b_j / new_j after a batch: only its columns a_j (less), new_j (more) and, for
// x = a_j, b_j (retired) changed.  The cached keys at those columns are dropped, their current
// keys >= the floor added (lanes 32 + 8t + j: column t of merge j, a repeat column once), and the
// candidates ranked by one pass over them: still exactly the row's keys >= the floor.  The top
// RT_K are kept (the floor rises to the last kept when some are cut).  Returns false (a full
// re-rank is needed) when fewer than KR + 1 remain above a floor > 1.  The wave calls it together.
__device__ __forceinline__ bool row_top_update(const uint32_t* __restrict__ row, unsigned long long F,
                                               unsigned long long kc, int x, int Vt, int lane, int n,
                                               const int (&A)[BK], const int (&B)[BK], const int (&N)[BK],
                                               unsigned long long* __restrict__ out) {
  int col[3 * BK];   // uniform: the changed columns, -1 unused
#pragma unroll
  for (int j = 0; j < BK; ++j) {
    col[j] = j < n ? A[j] : -1;
    col[BK + j] = j < n ? N[j] : -1;
    col[2 * BK + j] = j < n && A[j] == x ? B[j] : -1;
  }
  // F = the cached floor, kc = the lane's cached key (lanes < RT_K), loaded by the caller
  unsigned long long k = 0ull;
  if (lane < RT_K) {
    k = kc;
    const int y = key_col(k, x, Vt);
    bool drop = false;
#pragma unroll
    for (int t = 0; t < 3 * BK; ++t) drop |= y == col[t];
    k = drop ? 0ull : k;
  } else if (lane >= 32 && lane < 32 + 3 * BK) {
    const int sl = lane - 32;
    int y = -1;
#pragma unroll
    for (int t = 0; t < 3 * BK; ++t) y = t == sl ? col[t] : y;
    bool rep = false;
#pragma unroll
    for (int t = 0; t < 3 * BK; ++t) rep |= t < sl && col[t] == y;
    if (y >= 0 && !rep) {
      k = row_key((int32_t)row[y], x, Vt, y);
      k = k >= F ? k : 0ull;
    }
  }
  unsigned long long m = __builtin_amdgcn_ballot_w64(k != 0ull);
  const int cnt = __builtin_popcountll(m);
  if (cnt < KR + 1 && F > 1ull) return false;
  int rank = 0;
  while (m) {   // uniform
    const int c = __builtin_ctzll(m);
    m &= m - 1;
    rank += readlane_u64(k, c) > k;
  }
  if (k != 0ull && rank < RT_K) out[rank] = k;
  if (lane >= cnt && lane < RT_K) out[lane] = 0ull;
  unsigned long long f = F;
  if (cnt > RT_K) {   // cut: the floor is the last kept key
    const unsigned long long last = __builtin_amdgcn_ballot_w64(k != 0ull && rank == RT_K - 1);
    f = readlane_u64(k, __builtin_ctzll(last));
  }
  if (lane == 0) out[RT_F] = f;
  return true;
}

// Per-pass phase stamps (tools builds with -DBPE_MERGE_STAMPS=<first pass>; the product library
// compiles them out): s_memrealtime (100 MHz) of thread 0 of the first 1024 merge workgroups at
// entry, after the record, after the scan, before the delta flush and at exit, and of the
// deciding apply workgroup at its phases, for 64 passes.
#ifdef BPE_MERGE_STAMPS
__device__ unsigned long long g_bpe_stamps[64][1024][12];
__device__ unsigned long long g_bpe_dstamps[64][16];
__device__ unsigned long long g_bpe_batch[1024][2];   // every pass: merges decided, why the batch ended
__device__ unsigned long long g_apply_stamps[64][256][12];
#define ASTAMP(pi, k)                                                                                     \
  do {                                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 256 && (pi) >= BPE_MERGE_STAMPS && (pi) < BPE_MERGE_STAMPS + 64)  \
      g_apply_stamps[(pi) - BPE_MERGE_STAMPS][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();           \
  } while (0)
#define MSTAMP(pi, k)                                                                                     \
  do {                                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && (pi) >= BPE_MERGE_STAMPS && (pi) < BPE_MERGE_STAMPS + 64) \
      g_bpe_stamps[(pi) - BPE_MERGE_STAMPS][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();             \
  } while (0)
#define DSTAMP(pi, k)                                                                                     \
  do {                                                                                                    \
    if (lane == 0 && (pi) >= BPE_MERGE_STAMPS && (pi) < BPE_MERGE_STAMPS + 64)                            \
      g_bpe_dstamps[(pi) - BPE_MERGE_STAMPS][k] = __builtin_amdgcn_s_memrealtime();                       \
  } while (0)
#else
#define MSTAMP(pi, k) do { } while (0)
#define DSTAMP(pi, k) do { } while (0)
#define ASTAMP(pi, k) do { } while (0)
#endif

// The merges of the batch the last k_apply_batch decided, over every word: one scan of the word
// signatures for the union of the batch's pairs, each candidate word read once into registers;
// the merges it holds are known up front (batch pairs are symbol-disjoint, so one merge neither
// makes nor breaks another's pair) and applied with the op per lane, so a wave whose lanes hold
// different merges runs one pass, not one per merge.  The first signature loads are in flight
// before the batch record arrives.  apps (nullable, tools / byte accounting): pair occurrences
// rewritten per merge, unweighted, at apps[n_merges + j].
__global__ __launch_bounds__(256) void k_merge_batch(uint16_t* __restrict__ sym, const uint32_t* __restrict__ wstart,
                                                     uint32_t* __restrict__ wlen, const uint32_t* __restrict__ wcount,
                                                     int64_t nw, uint32_t* __restrict__ tlen, int max_len,
                                                     int Vt, unsigned long long* __restrict__ sig,
                                                     LoopState* __restrict__ loop, LoopHash lh,
                                                     uint32_t* __restrict__ table, uint32_t* __restrict__ clean,
                                                     int32_t* __restrict__ deltas, uint32_t* __restrict__ apps) {
  __shared__ __attribute__((aligned(16))) int32_t dl[BATCH_LDS / 4];
  __shared__ uint32_t clist[BATCH_CLIST];
  __shared__ int cn, touched;
  __shared__ int s_a[BK], s_b[BK], s_nid[BK];
  __shared__ uint32_t s_len[BK], s_apps[BK];
  __shared__ unsigned long long s_need[BK];
#ifdef BPE_MERGE_STAMPS
  const int st_pi = loop->passes;
#define KB_PI st_pi
#else
#define KB_PI 0
#endif
  MSTAMP(KB_PI, 0);
  // the batch record (threads < BK), then the first signature batch of the two-phase scan
  int ra = 0, rb = 0, rn = 0;
  uint32_t rl = 0;
  if (threadIdx.x < BK) {
    ra = loop->ba[threadIdx.x];
    rb = loop->bb[threadIdx.x];
    rn = loop->bnid[threadIdx.x];
    rl = loop->blen[threadIdx.x];
  }
  // the record's fields all in one round trip (no load waits on the n == 0 test)
  const int n = loop->bn, vcur = loop->bv0, kd = loop->bkd, mt = loop->bmt, nm0 = loop->bnm0;
  unsigned long long sgv[MERGE_SCAN];
  const int64_t nchunks = (nw + 255) / 256;
#pragma unroll
  for (int u = 0; u < MERGE_SCAN; ++u) {
    const int64_t w = (blockIdx.x + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
    sgv[u] = w < nw ? sig[w] : 0ull;
  }
  // the LDS delta vectors cleared whole while the record is in flight (16-byte stores)
  for (int i = threadIdx.x; i < BATCH_LDS / 16; i += 256) reinterpret_cast<int4*>(dl)[i] = make_int4(0, 0, 0, 0);
  if (n == 0) return;   // the loop has stopped (uniform)
  if (threadIdx.x < BK) {
    s_a[threadIdx.x] = ra;
    s_b[threadIdx.x] = rb;
    s_nid[threadIdx.x] = rn;
    s_len[threadIdx.x] = rl;
    s_apps[threadIdx.x] = 0;
    s_need[threadIdx.x] = (int)threadIdx.x < n ? sig_need((uint32_t)ra, (uint32_t)rb) : ~0ull;
  }
  if (threadIdx.x == 0) { cn = 0; touched = 0; }
  const int stride = vcur + n;
  const int nl = kd * 4 * stride;   // LDS entries in use (<= BATCH_LDS / 4: the decider's rule)
  __syncthreads();
  MSTAMP(KB_PI, 1);
  const int vbase = s_nid[0] == vcur ? vcur : vcur + 1;   // first new id (merge 0 may re-use one)
  const int nnew = n - (vbase == vcur ? 0 : 1);
  const uint32_t* nlen = vbase == vcur ? s_len : s_len + 1;
  unsigned long long need[BK];
#pragma unroll
  for (int j = 0; j < BK; ++j) need[j] = s_need[j];
  bool any = false;
  auto op_of = [&](int j) {
    return BatchOp{s_a[j], s_b[j], s_nid[j], max_len, Vt, vbase, nnew, stride, mt + (int)s_len[j] < max_len,
                   s_len[j], tlen, nlen, j < kd ? dl + j * 4 * stride : nullptr,
                   deltas != nullptr ? deltas + (size_t)j * 4 * Vt : nullptr, table, clean};
  };
  // the batch's merges in order on one word; its symbols are read once (a rare second merge
  // in the same word re-reads them)
  auto visit = [&](int64_t w) {
    // the word's four metadata loads in one round trip: no branch between them (a null wcount
    // reads the constant 1)
    const uint32_t* wc = wcount != nullptr ? wcount + w : &k_one_u32;
    uint32_t L = wlen[w];
    const uint32_t st = wstart[w];
    const int32_t cnt = (int32_t)*wc;
    const unsigned long long sgw = sig[w];
    // used together here, so the compiler cannot sink three of the loads below the L < 2 exit
    asm volatile("" ::"v"(L), "v"(st), "v"(cnt), "v"((uint32_t)sgw), "v"((uint32_t)(sgw >> 32)));
    uint16_t* s = sym + st;
    unsigned long long g = 0;
    bool changed = false;
    if (L < 2) return;
#ifdef BPE_MERGE_STAMPS
    const bool vst = blockIdx.x < 1024 && KB_PI >= BPE_MERGE_STAMPS && KB_PI < BPE_MERGE_STAMPS + 64;
    if (vst && (sgw >> 63) != 2u)   // uses sgw and L: the metadata has arrived
      atomicMax(&g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][7], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
    if (L <= (uint32_t)MERGE_REG) {
      uint32_t v[MERGE_REG + 2];
      load_word(s, L, v);
#ifdef BPE_MERGE_STAMPS
      if (vst && v[0] != 0xFFFFFFFEu)   // the word has arrived
        atomicMax(&g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][8], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
      uint32_t cand = 0;   // the merges whose pair the signature admits (need[j] = ~0 past n)
#pragma unroll
      for (int j = 0; j < BK; ++j) cand |= (uint32_t)((sgw & need[j]) == need[j]) << j;
      // a saturated signature (all 64 bits: a long word of many distinct symbols) passes the ~0 of
      // the slots past n too, whose records are stale: only the batch's merges are candidates
      cand &= (1u << n) - 1u;
      uint32_t hits = 0;
      for (; cand; cand &= cand - 1) {
        const int j = __builtin_ctz(cand);
        if (word_has_pair(v, L, (uint32_t)s_a[j], (uint32_t)s_b[j])) hits |= 1u << j;
      }
      if (!hits) return;
      // one merge_regs pass per set bit: lanes of a wave holding different merges share it
      // (the op is per lane), so a wave runs as many passes as its lanes' most merges (~1)
      bool fresh = true;
      while (hits) {
        const int j = __builtin_ctz(hits);
        hits &= hits - 1;
        if (!fresh) load_word(s, L, v);
        uint32_t napp = 0;
        L = merge_regs(v, L, s, cnt, op_of(j), g, napp);
        if (apps != nullptr) atomicAdd(&s_apps[j], napp);
        fresh = false;
      }
      changed = true;
    } else {
#ifdef BPE_MERGE_STAMPS
      if (vst) atomicAdd(&g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][11], 1ull);   // long-word visits
#endif
#pragma unroll 1
      for (int j = 0; j < n; ++j) {
        const unsigned long long nd = s_need[j];
        if (L < 2 || (sgw & nd) != nd) continue;
        unsigned long long gj = 0;
        uint32_t napp = 0;
        const uint32_t o = merge_global(s, L, wcount, w, op_of(j), gj, napp);
        if (o) {
          L = o;
          g = gj;
          changed = true;
          if (apps != nullptr) atomicAdd(&s_apps[j], napp);
        }
      }
    }
    if (!changed) return;
#ifdef BPE_MERGE_STAMPS
    if (blockIdx.x < 1024 && KB_PI >= BPE_MERGE_STAMPS && KB_PI < BPE_MERGE_STAMPS + 64) {
      atomicAdd(&g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][6], 1ull);   // words rewritten
      atomicMax(&g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][9], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
#endif
    any = true;
    wlen[w] = L;
    sig[w] = g;
  };
  // two-phase scan: a word is a candidate if its signature holds some merge's pair.  Rounds of
  // MERGE_SCAN signatures per thread append to the LDS list, the next round's loads in flight
  // while this round is tested; the list is processed once at the end, or earlier when another
  // round could overflow it (visit is inlined once).
  const int64_t step = (int64_t)MERGE_SCAN * gridDim.x;
  for (int64_t c0 = blockIdx.x; c0 < nchunks; c0 += step) {   // uniform
    unsigned long long nxt[MERGE_SCAN];
    const bool ahead = c0 + step < nchunks;
    if (ahead) {
#pragma unroll
      for (int u = 0; u < MERGE_SCAN; ++u) {
        const int64_t w = (c0 + step + (int64_t)u * gridDim.x) * 256 + threadIdx.x;
        nxt[u] = w < nw ? sig[w] : 0ull;
      }
    }
#pragma unroll
    for (int u = 0; u < MERGE_SCAN; ++u) {
      bool hit = false;
#pragma unroll
      for (int j = 0; j < BK; ++j) hit |= (sgv[u] & need[j]) == need[j];
      if (hit) clist[atomicAdd(&cn, 1)] = (uint32_t)((c0 + (int64_t)u * gridDim.x) * 256 + threadIdx.x);
    }
    __syncthreads();
    const int nc = cn;
    if (!ahead || nc > BATCH_CLIST - 256 * MERGE_SCAN) {
      MSTAMP(KB_PI, 2);
#ifdef BPE_MERGE_STAMPS
      if (threadIdx.x == 0 && blockIdx.x < 1024 && KB_PI >= BPE_MERGE_STAMPS && KB_PI < BPE_MERGE_STAMPS + 64)
        g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][5] += nc;   // candidates visited
#endif
      for (int k = threadIdx.x; k < nc; k += 256) {
        visit(clist[k]);
#ifdef BPE_MERGE_STAMPS
        if (blockIdx.x < 1024 && KB_PI >= BPE_MERGE_STAMPS && KB_PI < BPE_MERGE_STAMPS + 64)
          atomicMax(&g_bpe_stamps[KB_PI - BPE_MERGE_STAMPS][blockIdx.x][10],
                    (unsigned long long)__builtin_amdgcn_s_memrealtime());   // any visit done
#endif
      }
      __syncthreads();
      if (threadIdx.x == 0) cn = 0;
      __syncthreads();
    }
    if (ahead) {
#pragma unroll
      for (int u = 0; u < MERGE_SCAN; ++u) sgv[u] = nxt[u];
    }
  }
  MSTAMP(KB_PI, 3);
  if (apps != nullptr && threadIdx.x < n && s_apps[threadIdx.x])
    atomicAdd(&apps[nm0 + threadIdx.x], s_apps[threadIdx.x]);
  if (kd > 0) {
    if (any) touched = 1;
    __syncthreads();
    if (touched)   // LDS entry i = (j * 4 + kind) * stride + x -> the table (or the delta vectors)
      for (int i = threadIdx.x; i < nl; i += 256) {
        const int32_t v = dl[i];
        if (v) {
          const int jk = i / stride;
          const int j = jk >> 2;
          BatchOp op = op_of(j);
          op.dl = nullptr;
          op.table_add(jk & 3, (uint32_t)(i - jk * stride), v);
        }
      }
  }
  MSTAMP(KB_PI, 4);
  // the commit last (round 5): its compare-and-swap round trips no longer hold workgroup 0's scan,
  // which made it one of the pass's last workgroups (profiles/r05/bpe_phases_r05a.json, raw; 19.8
  // vs 19.8-19.9 ms, profiles/r05/bpe_loop_ab_r05f.txt)
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    // commit the batch, merge j on lane j: its string into the hash table (distinct strings, so
    // concurrent inserts only race for free slots), the new token's hash / P^len / length, its log
    // entry; then the counters.  No other workgroup of this launch reads what this writes: they
    // take the vocabulary before the batch from bv0 and the new tokens' lengths from the record.
    const int j = threadIdx.x;
    if (j < n) {
      const int reused = loop->breused[j];
      if (!reused) {
        const unsigned long long h = loop->bh[j];
        const unsigned long long pa = lh.tp[ra], pb = lh.tp[rb];
        const uint64_t hmask = (1ull << loop->log2cap) - 1;
        uint64_t sl = loop_slot(h, rl, loop->log2cap);
        while (atomicCAS(&lh.lid[sl], LOOP_EMPTY, lid_of(rl, rn)) != LOOP_EMPTY) sl = (sl + 1) & hmask;
        lh.key[sl] = h;
        lh.th[rn] = h;
        lh.tp[rn] = pa * pb;
        tlen[rn] = rl;
      }
      int32_t* lg = lh.log + 4 * (int64_t)(nm0 + j);
      lg[0] = ra; lg[1] = rb; lg[2] = rn; lg[3] = reused;
    }
    if (j == 0) {
      loop->n_merges = nm0 + n;
      loop->vcur = loop->bvcur;
      loop->maxtlen = mt;
    }
  }

#undef KB_PI
}

// After a batch: (sharded: add the all-reduced delta vectors to the table,) retire the merged
// pairs, re-rank every changed row (best and second-best) and publish this workgroup's BK best
// rows.  The workgroup that arrives last then commits the batch (string hash table, token
// lengths, log, vcur) and decides the next one, so the next k_merge_batch reads a finished
// record.  init: no batch, every row < vcur ranked, then the first decision.
//
// The hand-off of the per-workgroup lists to the deciding workgroup: the lists are stored
// write-through (sc1) by wave 0, which waits for them (vmcnt(0)) before its lane 0 adds to the
// ticket; the workgroup whose add returns gridDim.x - 1 reads them with sc1 loads
// (MI355X_MICROARCH.md, hand-off table row 1).  Everything else the decision reads -- the hash
// table, tlen, th, tp, the loop state -- only the deciding lane writes.
template <int KM>
__global__ __launch_bounds__(64 * APPLY_ROWS) void k_apply_batch(uint32_t* __restrict__ table, int Vt, ArgWs aw,
                                                                 BatchWs bw, uint32_t* __restrict__ tlen,
                                                                 LoopState* __restrict__ loop, LoopHash lh, int nrows,
                                                                 int init, int32_t* __restrict__ deltas,
                                                                 long long lds_min) {
  __shared__ unsigned long long s_top[APPLY_ROWS][RT_STRIDE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#ifdef BPE_MERGE_STAMPS
  const int st_pi = loop->passes;
#define KA_PI st_pi
#else
#define KA_PI 0
#endif
  ASTAMP(KA_PI, 0);
  // rows interleaved over the workgroups (x = blockIdx + wave * grid): the rows a batch touches
  // -- neighbours of its pairs, often a run of early, frequent ids -- spread over the grid
  // instead of filling a few workgroups' waves (a workgroup re-ranking 14 of its 16 rows was the
  // pass's last ticket, 8.4 us against 4.4 for the median re-ranking one)
  const int x = (int)blockIdx.x + wave * (int)gridDim.x;
  // the row's clean flag and cached keys do not depend on the batch record: in flight with it
  uint32_t pre_clean = 0u;
  unsigned long long pre_k = 0ull, pre_F = 0ull;
  if (x < nrows) {
    const unsigned long long* g = bw.rowtop + (size_t)x * RT_STRIDE;
    pre_clean = aw.clean[x];
    pre_k = lane < RT_K ? g[lane] : 0ull;
    pre_F = g[RT_F];
  }
  const int n = init ? 0 : loop->bn;
  if (!init && (n == 0 || !loop->active)) return;   // uniform over the grid
  int A[BK], B[BK], N[BK];
#pragma unroll
  for (int j = 0; j < BK; ++j) {
    A[j] = j < n ? loop->ba[j] : -1;
    B[j] = j < n ? loop->bb[j] : -1;
    N[j] = j < n ? loop->bnid[j] : -1;
  }
  const int vcur = init ? loop->vcur : loop->bvcur;
  // rows the merges changed: b_j, new_j entirely (re-ranked); other rows x only at columns a_j,
  // new_j (k_merge_batch's adds: clean[x] == 0; or the sharded deltas: touched) and, for x = a_j,
  // b_j (retired below)
  int full = init, in_a = 0;
#pragma unroll
  for (int j = 0; j < BK; ++j) {   // -1 past n
    full |= x == B[j] || x == N[j];
    in_a |= x == A[j];
  }
  int touched = 0;
  if (deltas != nullptr && n > 0) {
    // sharded: the all-reduced changes.  (1) each wave's entries (x, a_j), (x, new_j)
    if (lane == 0 && x < nrows)
      for (int j = 0; j < n; ++j) {
        int32_t* d = deltas + (size_t)j * 4 * Vt;
        int32_t v;
        if ((v = d[x])) { atomicAdd(&table[(size_t)x * Vt + A[j]], (uint32_t)v); d[x] = 0; touched = 1; }
        if ((v = d[Vt + x])) { atomicAdd(&table[(size_t)x * Vt + N[j]], (uint32_t)v); d[Vt + x] = 0; touched = 1; }
      }
    touched = __builtin_amdgcn_readfirstlane(touched);   // the wave ranks its row together
    // (2) rows b_j and new_j entirely, by the workgroup that owns them (distinct rows: a batch
    //     of more than one merge has fresh ids and symbol-disjoint pairs)
    for (int j = 0; j < n; ++j)
      for (int r = 0; r < 2; ++r) {
        const int xr = r == 0 ? B[j] : N[j];
        if (xr < 0 || xr % (int)gridDim.x != (int)blockIdx.x || xr >= nrows || (r == 1 && N[j] == B[j])) continue;
        int32_t* d = deltas + ((size_t)j * 4 + 2 + r) * Vt;
        for (int y = threadIdx.x; y < Vt; y += 64 * APPLY_ROWS) {
          const int32_t v = d[y];
          if (v) { atomicAdd(&table[(size_t)xr * Vt + y], (uint32_t)v); d[y] = 0; }
        }
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
  }
  if (lane == 0 && x < nrows)     // the merged pairs (after every add to them)
#pragma unroll
    for (int j = 0; j < BK; ++j)
      if (x == A[j]) table[(size_t)x * Vt + B[j]] = 0u;   // never re-picked
  // every row's KR best keys and its bound, in LDS: cached when the row did not change
  unsigned long long* rt = s_top[wave];
  if (x < nrows && x < vcur) {
    unsigned long long* g = bw.rowtop + (size_t)x * RT_STRIDE;
    const uint32_t* row = table + (size_t)x * Vt;
    if (!full && !touched && !in_a && pre_clean) {
      if (lane <= KR) rt[lane] = pre_k;
    } else {
#ifdef BPE_MERGE_STAMPS
      const bool st_on = lane == 0 && blockIdx.x < 256 && KA_PI >= BPE_MERGE_STAMPS && KA_PI < BPE_MERGE_STAMPS + 64;
      unsigned long long* st_a = st_on ? g_apply_stamps[KA_PI - BPE_MERGE_STAMPS][blockIdx.x] : nullptr;
      if (st_on) atomicMax(&st_a[4], (unsigned long long)__builtin_amdgcn_s_memrealtime());
      const bool upd = !full && row_top_update(row, pre_F, pre_k, x, Vt, lane, n, A, B, N, rt);
      if (st_on) atomicMax(&st_a[5], (unsigned long long)__builtin_amdgcn_s_memrealtime());
      if (!upd) {   // the row's first stretch loaded and used, then the rank (cache hits)
        int32_t cw[32];
        row_counts(row, Vt, vcur, lane, 0, cw);
        int acc = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) acc += cw[i];
        asm volatile("" ::"v"(acc));   // keeps row_counts' loads (the timed stretch) alive
        if (st_on) atomicMax(&st_a[8], (unsigned long long)__builtin_amdgcn_s_memrealtime());
        rank_row_top(row, x, Vt, vcur, lane, rt);
      }
      if (st_on) {
        atomicMax(&st_a[6], (unsigned long long)__builtin_amdgcn_s_memrealtime());
        atomicAdd(&st_a[7], upd ? 1ull : 1ull << 32);
      }
#else
      if (full || !row_top_update(row, pre_F, pre_k, x, Vt, lane, n, A, B, N, rt)) rank_row_top(row, x, Vt, vcur, lane, rt);
#endif
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < RT_K || lane == RT_F) g[lane] = rt[lane];
      if (lane == 0) aw.clean[x] = 1u;
#ifdef BPE_MERGE_STAMPS
      if (lane == 0 && blockIdx.x < 256 && KA_PI >= BPE_MERGE_STAMPS && KA_PI < BPE_MERGE_STAMPS + 64)
        atomicAdd(&g_apply_stamps[KA_PI - BPE_MERGE_STAMPS][blockIdx.x][3], 1ull);   // rows re-ranked
#endif
    }
  } else if (lane <= KR) {
    rt[lane] = 0ull;
  }
  __syncthreads();
  ASTAMP(KA_PI, 1);
  if (wave != 0) return;
  const int nwg = batch_nwg(Vt);
  {   // this workgroup's BK best of its APPLY_ROWS x KR candidates, best first, with their rows' bounds
    static_assert(APPLY_ROWS * KR == 64, "one candidate per lane of the wave");
    const int w = lane / KR, r = lane % KR;   // 64 lanes = 16 rows x 4
    const unsigned long long kw = s_top[w][r];
    int rank = 0;   // candidates above this one (keys are distinct; empty ones by lane), in registers
#pragma unroll
    for (int v = 0; v < APPLY_ROWS * KR; ++v) {
      const unsigned long long kv = readlane_u64(kw, v);
      rank += (kv > kw) | ((kv == kw) & (v < lane));
    }
    if (rank < BK) {
      st_agent(&bw.wgkey[(size_t)rank * nwg + blockIdx.x], kw);   // the grid may cover fewer rows than Vt
      st_agent(&bw.wgsec[(size_t)rank * nwg + blockIdx.x], kw ? s_top[w][KR] : 0ull);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(&loop->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
  ASTAMP(KA_PI, 2);
  if (t != gridDim.x - 1) return;
  // ---- the last workgroup's wave 0: commit the batch just applied, decide the next one
  DSTAMP(KA_PI, 0);
  // the loop state in registers (uniform): this wave writes only the record below.  The batch
  // just applied was committed by k_merge_batch's workgroup 0 (a kernel boundary ago).
  const int log2cap = loop->log2cap, target = loop->target, maxm = loop->max_merges;
  const unsigned long long minf = (unsigned long long)loop->min_freq;
  const int nm = loop->n_merges;
  int mt = loop->maxtlen;
  const int vnow = loop->vcur;
  const uint64_t hmask = (1ull << log2cap) - 1;
  // the workgroups' lists (the first 128: the whole table up to Vt = 2,048) first: they do not
  // depend on the commit, so their round trip overlaps it
  unsigned long long LK[2][KM], LS[2][KM];
  auto load_lists = [&](int t0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int g = (t0 + t) * 64 + lane;
#pragma unroll
      for (int i = 0; i < KM; ++i) {
        LK[t][i] = g < nwg ? ld_agent(&bw.wgkey[(size_t)i * nwg + g]) : 0ull;
        LS[t][i] = g < nwg ? ld_agent(&bw.wgsec[(size_t)i * nwg + g]) : 0ull;
      }
    }
  };
  load_lists(0);
  if (lane == 0) st_agent(&loop->ticket, 0u);
  // the global order: lane l merges the sorted lists of apply workgroups l, l + 64, ... (top KM
  // rows each), then KM wave-max rounds hand it out
  unsigned long long K[KM], S[KM];
#pragma unroll
  for (int i = 0; i < KM; ++i) K[i] = S[i] = 0ull;
  for (int t0 = 0; t0 < BATCH_WG_LANE; t0 += 2) {
    if (t0 * 64 >= nwg) break;
    if (t0 > 0) load_lists(t0);
#pragma unroll
    for (int t = 0; t < 2; ++t) top_merge<KM>(K, S, LK[t], LS[t]);
  }
  DSTAMP(KA_PI, 1);
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
  DSTAMP(KA_PI, 2);
  // lanes j < KM: candidate j's string and its id if it exists (the probes run in parallel)
  int cand_a = 0, cand_b = 0, exist = -1;
  uint32_t clen = 0;
  unsigned long long ch = 0;
  if (lane < KM && ckey) {
    const uint32_t idx = 0xFFFFFFFFu - (uint32_t)(ckey & 0xFFFFFFFFull);
    cand_a = (int)(idx / (uint32_t)Vt);
    cand_b = (int)(idx % (uint32_t)Vt);
    ch = ld_agent(&lh.th[cand_a]) * ld_agent(&lh.tp[cand_b]) + ld_agent(&lh.th[cand_b]);
    clen = ld_agent(&tlen[cand_a]) + ld_agent(&tlen[cand_b]);
    uint64_t sl = loop_slot(ch, clen, log2cap);
    while (true) {
      const unsigned long long li = ld_agent(&lh.lid[sl]), ki = ld_agent(&lh.key[sl]);
      if (li == LOOP_EMPTY) break;
      if ((uint32_t)(li >> 32) == clen && ki == ch) { exist = (int)(uint32_t)li; break; }
      sl = (sl + 1) & hmask;
    }
  }
  DSTAMP(KA_PI, 3);
  // HF's stopping rules per merge and the batch rules (see above), every candidate on its own
  // lane against the ones before it; the batch is the leading run of lanes that pass
  const unsigned long long count = ckey >> 32;
  bool ok = lane < KM && count >= 1 && count >= minf && vnow + lane < target && nm + lane < maxm;
  if (lane > 0) ok &= exist < 0;   // only the first may re-use an id
  unsigned long long sec = 0;
#pragma unroll
  for (int i = 0; i < KM - 1; ++i) {
    const int ai = __builtin_amdgcn_readlane(cand_a, i), bi = __builtin_amdgcn_readlane(cand_b, i);
    const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)clen, i);
    const unsigned long long hi = readlane_u64(ch, i), si = readlane_u64(csec, i);
    const bool ends = ai == bi || (i == 0 && __builtin_amdgcn_readlane(exist, 0) >= 0);   // self-pair / re-use
    // a later pair must not chain onto an earlier one (b_j == a_i: (x, a_i) loses count; a_j ==
    // b_i: (b_i, y) does); sharing a_i as its left or b_i as its right symbol is fine
    if (i < lane) ok &= !ends && cand_b != ai && cand_a != bi && !(ch == hi && clen == li);
    if (i < lane) sec = umax64(sec, si);
  }
  ok &= sec < ckey;   // a taken row's second-best would come first
  const unsigned long long pass = __ballot(ok);
  const int nb = (int)__builtin_ctzll(~pass);   // leading lanes that pass (<= KM)
  DSTAMP(KA_PI, 5);   // rules and ballot done
  // a re-used id ends the batch at its first merge, so the new ids are vnow, vnow + 1, ...
  const int reused0 = nb > 0 && __builtin_amdgcn_readlane(exist, 0) >= 0;
  if (lane < nb) {
    const bool reused = lane == 0 && exist >= 0;
    loop->ba[lane] = cand_a;
    loop->bb[lane] = cand_b;
    loop->bnid[lane] = reused ? exist : vnow + lane;
    loop->breused[lane] = reused ? 1 : 0;
    loop->blen[lane] = clen;
    loop->bh[lane] = ch;
  }
  // merges 0 .. kd-1 sum their changes in LDS: the frequent ones whose vectors fit
  const int stride = vnow + nb;
  int kd = 0;
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    if (j < nb) mt = max(mt, (int)__builtin_amdgcn_readlane((int)clen, j));
    if (kd == j && j < nb && (j + 1) * 16 * stride <= BATCH_LDS &&
        (long long)(readlane_u64(ckey, j) >> 32) >= lds_min)
      kd = j + 1;
  }
  if (lane == 0) {
    loop->bn = nb;
    loop->bv0 = vnow;
    loop->bnm0 = nm;
    loop->bvcur = vnow + nb - (reused0 ? 1 : 0);
    loop->bkd = kd;
    loop->bmt = mt;
    loop->passes += 1;
    if (nb == 0) loop->active = 0;
  }
  DSTAMP(KA_PI, 4);
#ifdef BPE_MERGE_STAMPS
  {   // why the batch ended (after the last stamp: tools only): the first failing lane's rules (bit 0 list end, 1 HF stop, 2 re-use,
      // 3 after a self-pair / re-use, 4 chaining, 5 same string, 6 a taken row's bound)
    uint32_t why = lane >= KM ? 1u : 0u;
    why |= !(count >= 1 && count >= minf && vnow + lane < target && nm + lane < maxm) ? 2u : 0u;
    why |= lane > 0 && exist >= 0 ? 4u : 0u;
    for (int i = 0; i < KM - 1 && i < lane; ++i) {
      const int ai = __builtin_amdgcn_readlane(cand_a, i), bi = __builtin_amdgcn_readlane(cand_b, i);
      why |= ai == bi || (i == 0 && __builtin_amdgcn_readlane(exist, 0) >= 0) ? 8u : 0u;
      why |= cand_b == ai || cand_a == bi ? 16u : 0u;
      why |= ch == readlane_u64(ch, i) && clen == (uint32_t)__builtin_amdgcn_readlane((int)clen, i) ? 32u : 0u;
    }
    why |= !(sec < ckey) ? 64u : 0u;
    const uint32_t w_nb = (uint32_t)__builtin_amdgcn_readlane((int)why, nb < 64 ? nb : 63);
    if (lane == 0 && KA_PI < 1024) {
      g_bpe_batch[KA_PI][0] = (unsigned long long)nb;
      g_bpe_batch[KA_PI][1] = nb < KM ? w_nb : 1u;
    }
  }
#endif
#undef KA_PI
}

__global__ void k_loop_init(LoopState* st, LoopState init, LoopHash lh, int n_tok, int log2cap,
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
    const unsigned long long prev = atomicCAS(&lh.lid[sl], LOOP_EMPTY, lid_of(tlen[i], i));
    if (prev == LOOP_EMPTY) { lh.key[sl] = h; break; }
    sl = (sl + 1) & mask;
  }
}

// k_merge's grid: the workgroups the device holds at once (one pass over the words, each
// workgroup its chunks round-robin, MERGE_SCAN signature loads in flight per thread), not more
template <class K>
int resident_grid(K kernel, int threads, size_t lds, int per_default) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, lds) != hipSuccess || per <= 0)
    per = per_default;
  return cus * per;
}

}  // namespace

// =================================================================== C-ABI ==
extern "C" size_t beast_bpe_argmax_workspace_bytes(int Vt) { return (size_t)(4 + (int64_t)Vt) * 8 + (size_t)Vt * 4; }

extern "C" int beast_bpe_argmax(const uint32_t* table, int Vt, int vcur, uint64_t* ws, int call, void* stream) {
  BEAST_REQUIRE(table && ws && vcur >= 1 && vcur <= Vt, "beast_bpe_argmax: bad args");
  BEAST_REQUIRE(call >= 0, "beast_bpe_argmax: call index must be >= 0");
  hipLaunchKernelGGL(k_apply_argmax, dim3((vcur + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0,
                     beast::as_stream(stream), const_cast<uint32_t*>(table), nullptr, Vt, vcur, argws_view(ws, Vt),
                     call & 1, 0, 0, 0, 0, nullptr, vcur);
  BEAST_LAUNCHED("k_apply_argmax");
  return BEAST_OK;
}

extern "C" int beast_bpe_apply_argmax(uint32_t* table, int32_t* deltas, int Vt, int vcur, int a, int b, int new_id,
                                      uint32_t* tlen, uint64_t* ws, int call, void* stream) {
  BEAST_REQUIRE(table && deltas && tlen && ws && vcur >= 1 && vcur <= Vt && call >= 0,
                "beast_bpe_apply_argmax: bad args");
  BEAST_REQUIRE(a >= 0 && a < Vt && b >= 0 && b < Vt && new_id >= 0 && new_id < Vt,
                "beast_bpe_apply_argmax: ids out of range");
  // every row that can change must run: rows < vcur, and a / b / new_id
  const int rows = std::max(vcur, std::max(a, std::max(b, new_id)) + 1);
  hipLaunchKernelGGL(k_apply_argmax, dim3((rows + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0,
                     beast::as_stream(stream), table, deltas, Vt, vcur, argws_view(ws, Vt), call & 1, 1, a, b, new_id,
                     tlen, rows);
  BEAST_LAUNCHED("k_apply_argmax");
  return BEAST_OK;
}

extern "C" int beast_bpe_merge(uint16_t* sym, const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount,
                               int64_t n_words, int a, int b, int new_id, const uint32_t* tlen, int max_token_length,
                               int32_t* deltas, int Vt, uint64_t* sig, int64_t pair_count, void* stream) {
  BEAST_REQUIRE(sym && wstart && wlen && tlen && deltas && sig, "beast_bpe_merge: null pointer");
  BEAST_REQUIRE(a >= 0 && a < Vt && b >= 0 && b < Vt && new_id >= 0 && new_id < Vt && Vt <= 65535,
                "beast_bpe_merge: ids out of range (a=%d b=%d new=%d Vt=%d)", a, b, new_id, Vt);
  if (n_words <= 0) return BEAST_OK;
  hipStream_t s = beast::as_stream(stream);
  const size_t lds = (size_t)4 * Vt * sizeof(int32_t);
  const bool use_lds = lds <= 64 * 1024 && pair_count >= beast::g_merge_lds_min;
  static int resident[2] = {0, 0};
  int& r = resident[use_lds];
  if (r == 0) r = use_lds ? resident_grid(k_merge<true>, 256, 64 * 1024, 2) : resident_grid(k_merge<false>, 256, 0, 4);
  const int grid = grid_for(n_words, MERGE_SCAN * 256, r);
  unsigned long long* sg = reinterpret_cast<unsigned long long*>(sig);
  if (use_lds)
    hipLaunchKernelGGL(k_merge<true>, dim3(grid), dim3(256), lds, s, sym, wstart, wlen, wcount, n_words, a, b, new_id,
                       tlen, max_token_length, deltas, Vt, sg);
  else
    hipLaunchKernelGGL(k_merge<false>, dim3(grid), dim3(256), 0, s, sym, wstart, wlen, wcount, n_words, a, b, new_id,
                       tlen, max_token_length, deltas, Vt, sg);
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
  size_t st, key, lid, th, tp, log, total;
};

static LoopLayout loop_layout(int Vt, int max_merges) {
  const size_t cap = size_t(1) << loop_log2cap(Vt);
  LoopLayout L;
  size_t o = 0;
  L.st = o;   o += al256(sizeof(LoopState));
  L.key = o;  o += al256(cap * 8);
  L.lid = o;  o += al256(cap * 8);
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
  lh.lid = reinterpret_cast<unsigned long long*>(w + L.lid);
  lh.th = reinterpret_cast<unsigned long long*>(w + L.th);
  lh.tp = reinterpret_cast<unsigned long long*>(w + L.tp);
  lh.log = reinterpret_cast<int32_t*>(w + L.log);
  return lh;
}

#ifdef BPE_MERGE_STAMPS
extern "C" int beast_debug_merge_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_stamps), sizeof(g_bpe_stamps)) == hipSuccess ? 0 : -2;
}
extern "C" int beast_debug_decide_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_dstamps), sizeof(g_bpe_dstamps)) == hipSuccess ? 0 : -2;
}
extern "C" int beast_debug_batch_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_batch), sizeof(g_bpe_batch)) == hipSuccess ? 0 : -2;
}
extern "C" int beast_debug_apply_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_apply_stamps), sizeof(g_apply_stamps)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" size_t beast_bpe_loop_workspace_bytes(int Vt, int max_merges) {
  return loop_layout(Vt, max_merges).total;
}

extern "C" int beast_bpe_loop_init(void* ws, size_t ws_bytes, int Vt, int max_merges, int n_tokens, int vocab_size,
                                   int min_frequency, const uint64_t* tok_hash, const uint64_t* tok_pow,
                                   const uint32_t* tlen, int max_tlen, void* stream) {
  BEAST_REQUIRE(ws && tok_hash && tok_pow && tlen, "beast_bpe_loop_init: null pointer");
  BEAST_REQUIRE(Vt >= 1 && Vt <= 32768 && n_tokens >= 0 && n_tokens <= Vt && max_merges >= 1,
                "beast_bpe_loop_init: bad sizes");
  const LoopLayout L = loop_layout(Vt, max_merges);
  BEAST_REQUIRE_CODE(ws_bytes >= L.total, BEAST_E_WORKSPACE, "loop workspace %zu < %zu", ws_bytes, L.total);
  hipStream_t s = beast::as_stream(stream);
  unsigned char* w = static_cast<unsigned char*>(ws);
  BEAST_HIP(hipMemsetAsync(w + L.lid, 0xFF, L.th - L.lid, s), "loop hash memset");
  LoopState init{};
  init.active = 1;
  init.vcur = n_tokens;
  init.target = vocab_size;
  init.min_freq = min_frequency;
  init.log2cap = loop_log2cap(Vt);
  init.max_merges = max_merges;
  init.maxtlen = max_tlen;
  const int n = n_tokens > 0 ? n_tokens : 1;
  hipLaunchKernelGGL(k_loop_init, dim3((n + 255) / 256), dim3(256), 0, s, reinterpret_cast<LoopState*>(w + L.st), init,
                     loop_hash_view(ws, Vt, max_merges), n_tokens, init.log2cap,
                     reinterpret_cast<const unsigned long long*>(tok_hash),
                     reinterpret_cast<const unsigned long long*>(tok_pow), tlen);
  BEAST_LAUNCHED("k_loop_init");
  return BEAST_OK;
}

extern "C" int beast_bpe_loop_state(const void* ws, int Vt, int max_merges, const void** state, const void** log) {
  BEAST_REQUIRE(ws && state && log, "beast_bpe_loop_state: null pointer");
  const LoopLayout L = loop_layout(Vt, max_merges);
  *state = static_cast<const unsigned char*>(ws) + L.st;
  *log = static_cast<const unsigned char*>(ws) + L.log;
  return BEAST_OK;
}

extern "C" size_t beast_bpe_batch_workspace_bytes(int Vt) { return batch_ws_bytes(Vt > 0 ? Vt : 1); }

extern "C" size_t beast_bpe_batch_delta_count(int Vt) { return (size_t)BK * 4 * (size_t)(Vt > 0 ? Vt : 1); }

template <int KM>
static int launch_apply(LoopState* st, const LoopHash& lh, BatchWs bw, ArgWs aw, int Vt, uint32_t* tlen,
                        uint32_t* table, int rows, int init, int32_t* deltas, hipStream_t s) {
  hipLaunchKernelGGL(k_apply_batch<KM>, dim3((rows + APPLY_ROWS - 1) / APPLY_ROWS), dim3(64 * APPLY_ROWS), 0, s, table,
                     Vt, aw, bw, tlen, st, lh, rows, init, deltas, (long long)beast::g_merge_lds_min);
  BEAST_LAUNCHED("k_apply_batch");
  return BEAST_OK;
}

extern "C" int beast_bpe_loop_batch(void* ws, int Vt, int max_merges, int n_steps, int max_batch, int flags,
                                    uint16_t* sym, const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount,
                                    int64_t n_words, uint32_t* tlen, int max_token_length, uint64_t* sig,
                                    uint32_t* table, uint64_t* argws, void* batch_ws, size_t batch_ws_bytes_,
                                    int vocab_size, int32_t* deltas, uint32_t* apps, void* stream) {
  BEAST_REQUIRE(ws && sym && wstart && wlen && tlen && sig && table && argws && batch_ws,
                "beast_bpe_loop_batch: null pointer");
  BEAST_REQUIRE(Vt >= 1 && n_steps >= 0 && vocab_size >= 1, "beast_bpe_loop_batch: bad sizes");
  BEAST_REQUIRE(n_words >= 0 && n_words < (int64_t(1) << 32), "beast_bpe_loop_batch: bad n_words");
  BEAST_REQUIRE_CODE(Vt <= 4096, BEAST_E_UNSUPPORTED, "batched merge loop: Vt %d > 4096", Vt);
  BEAST_REQUIRE(max_batch == 2 || max_batch == 4 || max_batch == 8, "beast_bpe_loop_batch: max_batch must be 2, 4 or 8");
  BEAST_REQUIRE((flags & ~7) == 0, "beast_bpe_loop_batch: unknown flags %d", flags);
  BEAST_REQUIRE_CODE(batch_ws_bytes_ >= batch_ws_bytes(Vt), BEAST_E_WORKSPACE, "batch workspace %zu < %zu",
                     batch_ws_bytes_, batch_ws_bytes(Vt));
  hipStream_t s = beast::as_stream(stream);
  const LoopLayout L = loop_layout(Vt, max_merges);
  LoopState* st = reinterpret_cast<LoopState*>(static_cast<unsigned char*>(ws) + L.st);
  const LoopHash lh = loop_hash_view(ws, Vt, max_merges);
  const ArgWs aw = argws_view(argws, Vt);
  const BatchWs bw = batch_view(batch_ws, Vt);
  const int rows = std::min(Vt, std::max(vocab_size, 1));
  auto apply = [&](int init) {
    switch (max_batch) {
      case 2: return launch_apply<2>(st, lh, bw, aw, Vt, tlen, table, rows, init, deltas, s);
      case 4: return launch_apply<4>(st, lh, bw, aw, Vt, tlen, table, rows, init, deltas, s);
      default: return launch_apply<8>(st, lh, bw, aw, Vt, tlen, table, rows, init, deltas, s);
    }
  };
  if (flags & BEAST_BPE_BATCH_INIT) {   // every row's best and second-best, then the first batch
    BEAST_HIP(hipMemsetAsync(batch_ws, 0, batch_ws_bytes(Vt), s), "batch workspace memset");
    if (int rc = apply(1)) return rc;
  }
  static int resident = 0;
  if (resident == 0) resident = resident_grid(k_merge_batch, 256, 0, 2);
  const int grid = grid_for(n_words > 0 ? n_words : 1, MERGE_SCAN * 256, resident);
  for (int i = 0; i < n_steps; ++i) {
    if (!(flags & BEAST_BPE_BATCH_NO_MERGE)) {
      hipLaunchKernelGGL(k_merge_batch, dim3(grid), dim3(256), 0, s, sym, wstart, wlen, wcount, n_words, tlen,
                         max_token_length, Vt, reinterpret_cast<unsigned long long*>(sig), st, lh, table, aw.clean,
                         deltas, apps);
      BEAST_LAUNCHED("k_merge_batch");
    }
    if (!(flags & BEAST_BPE_BATCH_NO_APPLY))
      if (int rc = apply(0)) return rc;
  }
  return BEAST_OK;
}
