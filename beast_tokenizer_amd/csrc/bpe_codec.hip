// Byte-level BPE *inference* on gfx950: encode bin rows into BPE ids and decode BPE ids
// back into bins.  Replaces, per row,
//   tokenizer.encode("".join(map(chr, row - min)), add_special_tokens=False).ids
//   ord(c) + min for c in tokenizer.decode(ids, skip_special_tokens=True)
// of beast/beast_bspline_bpe_tokenizer.py:175-247 (HF tokenizers 0.22.2: AddedVocabulary
// split, ByteLevel pre-tokeniser, BPE::merge_word + Word::merge_all, ByteLevel decoder,
// String::from_utf8_lossy).
//
//   k_mergemap_build   open-addressing (a, b) -> (rank, new_id) table + rank -> new_id;
//                      a pair listed twice keeps its LAST rank (HF collects the merges
//                      into a HashMap)
//   k_bpe_encode       one wave per row, 4 rows per workgroup in flight, grid-stride over
//                      rows; the merge map is staged once per workgroup into LDS when it
//                      fits (<= 8192 slots, <= 4096 merges), so every lookup of the merge loop is an LDS
//                      probe, not a dependent HBM/L2 round trip.  Per row, all in LDS:
//                        lanes: code points, range checks, classes, UTF-8 symbol offsets
//                        lane 0: special-token split (leftmost-longest) + GPT-2 regex walk
//                        lanes: byte -> vocab id; one word per lane: HF's merge_all with
//                        its (rank, pos) min-heap (stale entries skipped exactly as HF
//                        does, so the result is HF's even when two merges share an id)
//                        lanes: scan of per-word counts, ids written to the padded output
//   k_bpe_decode       one wave per row: lanes gather their ids' bytes into LDS at
//                      scanned offsets; valid UTF-8 (the normal case) decodes lane-
//                      parallel (one lane per lead byte); anything else goes through
//                      Rust's lossy decoder (maximal-subpart U+FFFD) on lane 0
#include <hip/hip_runtime.h>

#include "common.h"
#include "pretok.h"

namespace {

constexpr uint32_t EMPTY_KEY = 0xFFFFFFFFu;
using beast_pt::CLS_OTHER;
using beast_pt::regex_word;
using beast_pt::wave_excl_scan;
using beast_pt::wave_sync;
using beast_pt::word_starts;
constexpr int WAVES = 4;            // rows in flight per workgroup (decode)
constexpr int ENC_MAX_WAVES = 16;   // encode: as many rows per workgroup as the LDS holds, up to 16
constexpr int BLOCK = 64 * WAVES;
constexpr int MAX_SPECIAL = 64, MAX_SPECIAL_LEN = 64;
constexpr int RM_PER = 8;           // symbol positions per lane of the round merge (rows <= 512 symbols)
constexpr int RM_NARROW = 6;        // ... in the narrow kernel (rows <= 384 symbols)
constexpr uint32_t RK_NONE = 0xFFFFFFFFu;
constexpr int LDS_MAP_MAX_LOG2 = 13;   // stage maps of <= 8192 slots (64 KiB + rank table)
constexpr size_t LDS_BUDGET = 160 * 1024;
constexpr size_t STATIC_LDS = 2048;         // k_bpe_encode's byte -> id table and LUT head   // gfx950: one workgroup may declare all 160 KiB

// encode status per row (host maps them to the reference's exceptions)
constexpr int ST_OK = 0, ST_BELOW_MIN = 1, ST_ABOVE_MAX = 2, ST_NOT_UNICODE = 3, ST_SURROGATE = 4,
              ST_NO_CLASS = 5, ST_TOO_LONG = 6;

#ifdef BPE_STAMPS
// tools/codec/bpe_encode_phases.py only (the product compiles these out): per row r < 4096,
// s_memrealtime (100 MHz) at each phase boundary [0, 7), then merge rounds, byte symbols, words
// and the workgroup's map-staging start / end -- plain stores by lane 0, one slot per row, so
// the stamps add no atomics and no shared address
constexpr int BPE_RS = 4096;
__device__ unsigned long long g_bpe_rs[BPE_RS][12];
// k_bpe_words' merge tasks per row wave: [0..3) time in mid / short / tiny tasks, [3..6) their counts
__device__ unsigned long long g_bpe_wt[BPE_RS][8];
#define BPE_STAMP(k)                                                                          \
  do {                                                                                        \
    if (lane == 0 && r < BPE_RS) g_bpe_rs[r][k] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#else
#define BPE_STAMP(k) do { } while (0)
#endif

__host__ __device__ inline size_t al16(size_t x) { return (x + 15) & ~size_t(15); }

// ------------------------------------------------------------- merge map --
// layout: kv uint2[cap] (key a << 16 | b, EMPTY_KEY = free; value (rank + 1) << 16 | new_id, 0 =
// unset) | rank2new u16[n].  Key and value side by side: a probe is one 8-byte load.
struct MergeMap {
  const uint2* kv;
  const uint16_t* rank2new;
  int log2cap;
};

__device__ __forceinline__ uint32_t mm_hash(uint32_t key, int log2cap) {
  return (key * 0x9E3779B1u) >> (32 - log2cap);
}

// k_bpe_words' merge map: two-choice bucketed cuckoo hashing, 1 << log2b buckets of two (key,
// value) slots (16 bytes), every key in one of its two buckets -- a lookup is exactly two 16-byte
// reads, one LDS round trip, where a linear-probe chain is a loop whose longest lane sets the
// wave's pace.  Built on the host (beast_bpe_wordmap_build_host); same key / value encoding as
// the merge map above.
struct WordMap {
  const uint4* b;
  int log2b;
};
__host__ __device__ __forceinline__ uint32_t wm_h1(uint32_t key, int log2b) { return (key * 0x9E3779B1u) >> (32 - log2b); }
__host__ __device__ __forceinline__ uint32_t wm_h2(uint32_t key, int log2b) {
  return ((key ^ 0x5BD1E995u) * 0x85EBCA77u) >> (32 - log2b);
}

__global__ void k_mergemap_clear(uint2* __restrict__ kv, int cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) kv[i] = make_uint2(EMPTY_KEY, 0u);
}

__global__ void k_mergemap_build(const int32_t* __restrict__ ma, const int32_t* __restrict__ mb,
                                 const int32_t* __restrict__ mnew, int n, uint2* __restrict__ kv,
                                 uint16_t* __restrict__ rank2new, int log2cap) {
  uint32_t* const w = reinterpret_cast<uint32_t*>(kv);   // slot h: key at 2h, value at 2h + 1
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = ((uint32_t)ma[i] << 16) | (uint32_t)mb[i];
  const uint32_t mask = (1u << log2cap) - 1u;
  uint32_t h = mm_hash(key, log2cap);
  while (true) {
    const uint32_t prev = atomicCAS(&w[2 * h], EMPTY_KEY, key);
    if (prev == EMPTY_KEY || prev == key) break;
    h = (h + 1) & mask;
  }
  atomicMax(&w[2 * h + 1], ((uint32_t)(i + 1) << 16) | (uint32_t)mnew[i]);   // later rank wins
  rank2new[i] = (uint16_t)mnew[i];
}

// rank of pair (a, b), or -1; *new_id set when found
template <class Map>
__device__ __forceinline__ int mm_find(const Map& m, int a, int b, int& new_id) {
  const uint32_t key = ((uint32_t)a << 16) | (uint32_t)b;
  const uint32_t mask = (1u << m.log2cap) - 1u;
  uint32_t h = mm_hash(key, m.log2cap);
  while (true) {
    const uint2 e = m.kv[h];
    if (e.x == key) {
      new_id = (int)(e.y & 0xFFFFu);
      return (int)(e.y >> 16) - 1;
    }
    if (e.x == EMPTY_KEY) return -1;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ int utf8_len(int cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

__device__ __forceinline__ int utf8_byte(int cp, int q) {
  const int L = utf8_len(cp);
  if (L == 1) return cp;
  if (q == 0) return (L == 2 ? 0xC0 : L == 3 ? 0xE0 : 0xF0) | (cp >> (6 * (L - 1)));
  return 0x80 | ((cp >> (6 * (L - 1 - q))) & 0x3F);
}

// ---------------------------------------------------------------- heap --
// min-heap of u32 keys (rank << 16 | pos) in LDS, one per word: HF's Merge order (rank, pos)
__device__ __forceinline__ void heap_push(uint32_t* h, int& n, uint32_t v) {
  int i = n++;
  while (i > 0) {
    const int p = (i - 1) >> 1;
    const uint32_t hp = h[p];
    if (hp <= v) break;
    h[i] = hp;
    i = p;
  }
  h[i] = v;
}

__device__ __forceinline__ uint32_t heap_pop(uint32_t* h, int& n) {
  const uint32_t top = h[0];
  const uint32_t v = h[--n];
  int i = 0;
  while (true) {
    int c = 2 * i + 1;
    if (c >= n) break;
    uint32_t hc = h[c];
    if (c + 1 < n) {
      const uint32_t h1 = h[c + 1];
      if (h1 < hc) { hc = h1; ++c; }
    }
    if (v <= hc) break;
    h[i] = hc;
    i = c;
  }
  if (n > 0) h[i] = v;
  return top;
}

// ------------------------------------------------------------- encode --
struct EncLds {
  uint32_t* heap;     // [3 S]
  int32_t* c;         // [S] symbol ids (-1: none)
  int32_t* cps;       // [Lc] shifted code points
  int32_t* symoff;    // [Lc + 1] first byte symbol of each code point
  int32_t* wcp;       // [Lc + 1] word boundaries (code point index)
  int32_t* wspec;     // [Lc] special-token id of a word, or -1
  int32_t* wcnt;      // [Lc] final symbols per word, then their output offsets
  int16_t* prv;       // [S]
  int16_t* nxt;       // [S]
  uint8_t* cls;       // [Lc]
  int32_t* misc;      // [4]: n_words
  uint32_t* rk;       // [S] round merge: (rank << 16 | new id) of the pair starting here, RK_NONE: none
  int16_t* wid;       // [S] word of each symbol
  uint8_t* cand;      // [S] this round's merge candidates
  uint8_t* dirty;     // [S] pair changed since its rank was read
  uint32_t* wmin;     // [Lc] this round's lowest pair per word
};

// the heap (long rows, or heap mode) and the round merge's arrays (rows <= 64 * RM_PER symbols)
// share a region; a launch that never takes the heap path sizes it for the rounds only.  The
// per-word counts (wcnt, live in steps 2 and 5) alias the round merge's wmin (live in step 4).
__host__ __device__ inline bool enc_needs_heap(int S, int heap_merge) { return heap_merge || S > 64 * RM_PER; }
__host__ __device__ inline size_t enc_merge_bytes(int Lc, int S, bool heap) {
  const size_t rounds = al16(sizeof(uint32_t) * S) + al16(sizeof(uint32_t) * Lc) + 2 * al16(S);
  const size_t hp = heap ? al16(sizeof(uint32_t) * 3 * (size_t)S) : 0;
  return hp > rounds ? hp : rounds;
}
__host__ __device__ inline size_t enc_row_bytes(int Lc, int S, bool heap) {
  return enc_merge_bytes(Lc, S, heap) + al16(sizeof(int32_t) * S) + al16(sizeof(int32_t) * Lc) +
         2 * al16(sizeof(int32_t) * (Lc + 1)) + al16(sizeof(int32_t) * Lc) + 2 * al16(sizeof(int16_t) * S) +
         al16(Lc) + 16 + al16(sizeof(int16_t) * S);
}

__device__ inline EncLds enc_carve(char* p, int Lc, int S, bool heap) {
  EncLds L;
  auto take = [&](size_t bytes) { char* r = p; p += al16(bytes); return r; };
  char* merge = take(enc_merge_bytes(Lc, S, heap));   // heap, or rk | wmin | cand | dirty
  L.heap = (uint32_t*)merge;
  L.rk = (uint32_t*)merge;
  L.wmin = (uint32_t*)(merge + al16(sizeof(uint32_t) * S));
  L.cand = (uint8_t*)(merge + al16(sizeof(uint32_t) * S) + al16(sizeof(uint32_t) * Lc));
  L.dirty = L.cand + al16(S);
  L.c = (int32_t*)take(sizeof(int32_t) * S);
  L.cps = (int32_t*)take(sizeof(int32_t) * Lc);
  L.symoff = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  L.wcp = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  L.wspec = (int32_t*)take(sizeof(int32_t) * Lc);
  L.wcnt = (int32_t*)L.wmin;
  L.prv = (int16_t*)take(sizeof(int16_t) * S);
  L.nxt = (int16_t*)take(sizeof(int16_t) * S);
  L.cls = (uint8_t*)take(Lc);
  L.misc = (int32_t*)take(16);
  L.wid = (int16_t*)take(sizeof(int16_t) * S);
  return L;
}

// bytes of the staged merge map (0 if it stays in HBM)
__host__ __device__ inline size_t map_lds_bytes(int log2cap, int n_merges) {
  if (log2cap > LDS_MAP_MAX_LOG2) return 0;
  return al16(sizeof(uint32_t) * 2 * ((size_t)1 << log2cap)) + al16(sizeof(uint16_t) * (size_t)n_merges);
}

struct EncArgs {
  const long long* tok;
  const int64_t* row_off;
  int64_t n_rows;
  long long min_tok;
  long long max_span;         // largest allowed shifted value, < 0: unbounded
  const uint8_t* lut;
  int lut_n;
  const int32_t* byte2id;     // [256], -1: byte-level char not in the vocab
  MergeMap map;               // in HBM
  int n_merges;
  int map_in_lds;             // host choice: k_bpe_encode<true> stages the map
  int heap_merge;             // BEAST_OPT_BPE_ENCODE_MODE bit 0: HF's heap per word instead of rounds
  const int32_t* spec_cps;    // [n_spec][MAX_SPECIAL_LEN]
  const int32_t* spec_len;
  const int32_t* spec_id;
  int n_spec;
  int unk_id;                 // model unk token id, -1: unknown chars are dropped
  int fuse_unk;
  int Lc, S;
  int32_t* out_ids;
  int64_t out_stride;
  int32_t* out_len;
  int32_t* status;
};

// 4b. (see encode_row) the round merge of a row of <= 64 * RMP byte symbols
template <int RMP, class Map>
__device__ __forceinline__ void round_merge(const Map& mm, EncLds& L, int npos, int nw, int lane) {
    // Each step reads all of a lane's positions first (addresses clamped, loads in flight
    // together) and then acts on them, so a step costs one LDS round trip, not one per position.
    const int kmax = (npos + 63) >> 6;   // positions per lane in use (<= RMP)
    for (int k = 0; k < kmax; ++k) {
      const int s = lane + 64 * k;
      if (s < npos) { L.dirty[s] = 1; L.cand[s] = 0; }
    }
    wave_sync();
    const int last = npos > 0 ? npos - 1 : 0;
    // every round with a live pair merges at least one (each word's lowest pair has a head), so
    // npos rounds bound the loop: a broken invariant ends it instead of hanging the wave
    for (int round = 0; round < npos; ++round) {
#ifdef BPE_STAMPS
      if (lane == 0) L.misc[1] += 1;
#endif
      for (int w = lane; w < nw; w += 64) L.wmin[w] = RK_NONE;
      // (a) ranks of the pairs next to last round's merges
      int ck[RMP], nk[RMP], dk[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) {
        const int s = min(lane + 64 * k, last);
        dk[k] = k < kmax && lane + 64 * k < npos ? L.dirty[s] : 0;
        ck[k] = L.c[s];
        nk[k] = L.nxt[s];
      }
      int cn[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) cn[k] = L.c[max(nk[k], 0)];
      // the dirty pairs' first probes all in flight together (one 8-byte load each), then the
      // rare collision chains per position
      const uint32_t mmask = (1u << mm.log2cap) - 1u;
      constexpr int PG = RMP < 4 ? RMP : 4;   // positions probed together (registers)
#pragma unroll
      for (int k0 = 0; k0 < RMP; k0 += PG) {
        uint32_t key[PG], hs[PG];
        uint2 e[PG];
        bool q[PG];   // a live pair to look up (a dead symbol's key may equal EMPTY_KEY)
#pragma unroll
        for (int i = 0; i < PG; ++i) {
          const int k = min(k0 + i, RMP - 1);   // RMP need not be a multiple of PG
          q[i] = k0 + i < RMP && dk[k] && ck[k] >= 0 && nk[k] >= 0;
          key[i] = ((uint32_t)ck[k] << 16) | (uint32_t)cn[k];
          hs[i] = mm_hash(key[i], mm.log2cap);
          e[i] = q[i] ? mm.kv[hs[i]] : make_uint2(EMPTY_KEY, 0u);
        }
#pragma unroll
        for (int i = 0; i < PG; ++i) {
          const int k = min(k0 + i, RMP - 1);
          if (k0 + i >= RMP || !dk[k]) continue;
          while (q[i] && e[i].x != key[i] && e[i].x != EMPTY_KEY) {
            hs[i] = (hs[i] + 1) & mmask;
            e[i] = mm.kv[hs[i]];
          }
          // (rank + 1) << 16 | new_id  ->  rank << 16 | new_id
          L.rk[lane + 64 * k] = (q[i] && e[i].x == key[i]) ? e[i].y - 0x10000u : RK_NONE;
          L.dirty[lane + 64 * k] = 0;
        }
      }
      wave_sync();
      // (b) every word's lowest pair
      bool live = false;
      uint32_t rv[RMP];
      int wv[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) {
        const int s = min(lane + 64 * k, last);
        rv[k] = (k < kmax && lane + 64 * k < npos) ? L.rk[s] : RK_NONE;
        wv[k] = L.wid[s];
        ck[k] = L.c[s];
      }
#pragma unroll
      for (int k = 0; k < RMP; ++k)
        if (ck[k] >= 0 && rv[k] != RK_NONE) {
          atomicMin(&L.wmin[wv[k]], rv[k]);
          live = true;
        }
      if (!__any(live)) break;
      wave_sync();
      // (c) candidates: the pairs equal to their word's lowest
      uint32_t mv[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) mv[k] = L.wmin[wv[k]];
      bool cd[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) {
        cd[k] = ck[k] >= 0 && rv[k] != RK_NONE && rv[k] == mv[k];
        if (k < kmax && lane + 64 * k < npos) L.cand[lane + 64 * k] = cd[k];
      }
      // links only (d) changes, read in this step's round trip: each position's left neighbour
      // and the symbol after its pair (its right one, nk, is from (a): nxt is unchanged since)
      int pk[RMP], nnk[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) {
        pk[k] = L.prv[min(lane + 64 * k, last)];
        nnk[k] = L.nxt[max(nk[k], 0)];
      }
      wave_sync();
      // (d) each run's head applies its run (one merge unless a self-pair repeats).  The heads'
      // first merges read everything in one round trip before any write (no head writes what
      // another head's first merge reads: nxt / cand of its own pair only, prv of the symbol after
      // it -- read here only as the head's own left neighbour, which marks the same live pair
      // dirty either way), then the rare self-pair runs one step at a time
      int cf[RMP];   // cand of the left neighbour (bit 0), of the pair's right symbol (1), of the one after (2)
#pragma unroll
      for (int k = 0; k < RMP; ++k)
        cf[k] = (int)L.cand[max(pk[k], 0)] | ((int)L.cand[max(nk[k], 0)] << 1) | ((int)L.cand[max(nnk[k], 0)] << 2);
      bool hd[RMP];
#pragma unroll
      for (int k = 0; k < RMP; ++k) hd[k] = cd[k] && !(pk[k] >= 0 && (cf[k] & 1));
#pragma unroll
      for (int k = 0; k < RMP; ++k) {
        if (!hd[k]) continue;
        const int nid = (int)(rv[k] & 0xFFFFu);
        const int t = lane + 64 * k, u = nk[k], nn = nnk[k];
        L.c[t] = nid;
        L.c[u] = -1;
        L.nxt[t] = (int16_t)nn;
        if (nn >= 0) L.prv[nn] = (int16_t)t;
        L.dirty[t] = 1;
        if (pk[k] >= 0) L.dirty[pk[k]] = 1;
      }
#pragma unroll
      for (int k = 0; k < RMP; ++k) {
        if (!hd[k] || !(cf[k] & 2) || nnk[k] < 0 || !(cf[k] & 4)) continue;
        const int nid = (int)(rv[k] & 0xFFFFu);
        int t = nnk[k];   // the run of a self-pair goes on
        while (true) {
          const int u = L.nxt[t], nn = L.nxt[u];
          L.c[t] = nid;
          L.c[u] = -1;
          L.nxt[t] = (int16_t)nn;
          if (nn >= 0) L.prv[nn] = (int16_t)t;
          L.dirty[t] = 1;
          const int pv = L.prv[t];
          if (pv >= 0) L.dirty[pv] = 1;
          if (!L.cand[u] || nn < 0 || !L.cand[nn]) break;
          t = nn;
        }
      }
      wave_sync();
    }
}

// RMX: the widest round merge compiled in.  RM_NARROW (rows of <= 384 byte symbols, e.g. 140 bins
// of 2-byte code points) keeps the kernel at ~109 VGPRs with nothing spilled; the RM_PER form
// needs 128 and spills ~16 to scratch.  The host launches the narrow kernel whenever every row fits.
template <int RMX, class Map>
__device__ void encode_row(const EncArgs& a, const Map& mm, EncLds& L, int64_t r, int lane, const int32_t* b2i,
                           const uint8_t* lut256) {
#ifdef BPE_STAMPS
  if (lane == 0) L.misc[1] = 0;
#endif
  BPE_STAMP(0);
  const int64_t r0 = a.row_off[r];
  const int n = (int)(a.row_off[r + 1] - r0);
  if (n > a.Lc) {
    if (lane == 0) { a.status[r] = ST_TOO_LONG; a.out_len[r] = 0; }
    return;
  }
  // 1. code points, range checks (reference :181-192 order: below-min first), classes.  The
  //    first 256 code points' loads are all in flight at once; classes of code points < 256
  //    come from the workgroup's LDS copy of the LUT.
  int below = 0, above = 0, notuni = 0, surr = 0, nocls = 0;
  auto code_point = [&](int i, long long t) {
    const long long v = t - a.min_tok;
    below |= v < 0;
    above |= (a.max_span >= 0 && v > a.max_span);
    notuni |= v > 0x10FFFF;
    surr |= (v >= 0xD800 && v <= 0xDFFF);
    nocls |= v >= a.lut_n;
    const int cp = (int)((v < 0 || v > 0x10FFFF) ? 0 : v);
    L.cps[i] = cp;
    L.cls[i] = cp < 256 ? lut256[cp] : (cp < a.lut_n) ? a.lut[cp] : CLS_OTHER;
  };
  constexpr int PF = 4;
  long long tv[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) tv[k] = lane + 64 * k < n ? a.tok[r0 + lane + 64 * k] : 0;
#pragma unroll
  for (int k = 0; k < PF; ++k)
    if (lane + 64 * k < n) code_point(lane + 64 * k, tv[k]);
  for (int i = lane + 64 * PF; i < n; i += 64) code_point(i, a.tok[r0 + i]);
  BPE_STAMP(1);
  int st = ST_OK;
  if (__any(below)) st = ST_BELOW_MIN;
  else if (__any(above)) st = ST_ABOVE_MAX;
  else if (__any(notuni)) st = ST_NOT_UNICODE;
  else if (__any(surr)) st = ST_SURROGATE;
  else if (__any(nocls)) st = ST_NO_CLASS;
  if (st != ST_OK) {
    if (lane == 0) { a.status[r] = st; a.out_len[r] = 0; }
    return;
  }
  // UTF-8 symbol offsets
  int carry = 0;
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    int tot;
    const int len = (i < n) ? utf8_len(L.cps[i]) : 0;
    const int ex = wave_excl_scan(len, lane, tot);
    if (i < n) L.symoff[i] = carry + ex;
    carry += tot;
  }
  if (lane == 0) L.symoff[n] = carry;
  if (carry > a.S) {   // host sizes S from the code-point bound; guard anyway
    if (lane == 0) { a.status[r] = ST_TOO_LONG; a.out_len[r] = 0; }
    return;
  }
  wave_sync();

  BPE_STAMP(2);
  // 2. word boundaries.  No special tokens: every lane evaluates the regex from each of its
  //    positions (end of a word starting there) in parallel, then lane 0 only follows the
  //    chain 0 -> e[0] -> ...  With special tokens: lane 0 runs AddedVocabulary's split
  //    (leftmost-longest) and the regex walk per segment.
  if (a.n_spec == 0) {
#ifndef BPE_SERIAL_PRETOK
    int32_t* e = L.wcnt;   // scratch until step 4
    for (int i = lane; i < n; i += 64) e[i] = regex_word(L.cps, L.cls, i, n);
    word_starts(e, L.cand, L.wcp, L.wspec, L.misc, n, lane);
#else
    if (lane == 0) {
      int nw = 0, p = 0;
      while (p < n) {
        L.wcp[nw] = p; L.wspec[nw] = -1; ++nw;
        p = regex_word(L.cps, L.cls, p, n);
      }
      L.wcp[nw] = n;
      L.misc[0] = nw;
    }
#endif
  } else if (lane == 0) {
    int nw = 0, seg = 0, i = 0;
    while (i <= n) {
      int mlen = 0, mid = -1;
      if (i < n) {
        for (int s = 0; s < a.n_spec; ++s) {
          const int sl = a.spec_len[s];
          if (sl <= mlen || i + sl > n) continue;
          const int32_t* sc = a.spec_cps + (size_t)s * MAX_SPECIAL_LEN;
          bool ok = true;
          for (int q = 0; q < sl && ok; ++q) ok = (L.cps[i + q] == sc[q]);
          if (ok) { mlen = sl; mid = a.spec_id[s]; }
        }
      }
      if (mlen > 0 || i == n) {
        int p = seg;
        while (p < i) {
          const int j = regex_word(L.cps, L.cls, p, i);
          L.wcp[nw] = p; L.wspec[nw] = -1; ++nw;
          p = j;
        }
        if (i == n) break;
        L.wcp[nw] = i; L.wspec[nw] = mid; ++nw;
        i += mlen;
        seg = i;
      } else {
        ++i;
      }
    }
    L.wcp[nw] = n;
    L.misc[0] = nw;
  }
  BPE_STAMP(3);
  // 3. byte symbols as vocab ids
  for (int i = lane; i < n; i += 64) {
    const int cp = L.cps[i], len = utf8_len(cp), o = L.symoff[i];
    for (int q = 0; q < len; ++q) L.c[o + q] = b2i[utf8_byte(cp, q)];
  }
  wave_sync();
  const int nw = L.misc[0];

  BPE_STAMP(4);
  // 4a. one word per lane: special words, unknown chars (HF's unk / fuse_unk), the symbol list
  const int npos = L.symoff[n];
  for (int w = lane; w < nw; w += 64) {
    const int sb = L.symoff[L.wcp[w]], se = L.symoff[L.wcp[w + 1]];
    for (int s = sb; s < se; ++s) L.wid[s] = (int16_t)w;
    if (L.wspec[w] >= 0) {
      L.c[sb] = L.wspec[w];
      L.nxt[sb] = -1;
      L.prv[sb] = -1;
      for (int s = sb + 1; s < se; ++s) L.c[s] = -1;
      continue;
    }
    bool pending_unk = false;
    int last = -1;
    for (int s = sb; s < se; ++s) {
      int id = L.c[s];
      if (id < 0) {
        if (a.unk_id >= 0 && !(a.fuse_unk && pending_unk)) { id = a.unk_id; pending_unk = true; }
        else id = -1;
      } else {
        pending_unk = false;
      }
      L.c[s] = id;
      if (id < 0) continue;
      L.prv[s] = (int16_t)last;
      L.nxt[s] = -1;
      if (last >= 0) L.nxt[last] = (int16_t)s;
      last = s;
    }
  }
  wave_sync();
#ifndef BPE_SKIP_MERGE
  if (npos <= 64 * RM_PER && !a.heap_merge) {
    // 4b. BPE::merge_word + Word::merge_all for every word of the row at once.  HF pops the
    //     lowest (rank, position) of the word's current pairs (stale heap entries skipped), so a
    //     word's result is: repeatedly merge its lowest-rank pair, leftmost first.  One round
    //     merges, in every word, all occurrences of that word's lowest pair (left to right in a
    //     run of a self-pair: each run's head walks it), so rounds = distinct ranks applied per
    //     word, and only pairs next to a merge are looked up again.
    if (npos <= 64 * 4) {
      round_merge<4>(mm, L, npos, nw, lane);
    } else {
      if constexpr (RMX == RM_NARROW) round_merge<RM_NARROW>(mm, L, npos, nw, lane);
      else round_merge<RM_PER>(mm, L, npos, nw, lane);
    }
  } else {
    // 4b'. long rows: one word per lane with HF's (rank, pos) min-heap
    for (int w = lane; w < nw; w += 64) {
      if (L.wspec[w] >= 0) continue;
      const int sb = L.symoff[L.wcp[w]], se = L.symoff[L.wcp[w + 1]];
      uint32_t* hp = L.heap + 3 * (size_t)sb;
      int hn = 0;
      for (int s = sb; s < se; ++s) {
        if (L.c[s] < 0 || L.nxt[s] < 0) continue;
        int nid;
        const int rk = mm_find(mm, L.c[s], L.c[L.nxt[s]], nid);
        if (rk >= 0) heap_push(hp, hn, ((uint32_t)rk << 16) | (uint32_t)(s - sb));
      }
      while (hn > 0) {
        const uint32_t top = heap_pop(hp, hn);
        const int pos = sb + (int)(top & 0xFFFFu);
        const int trank = (int)(top >> 16);
        if (L.c[pos] < 0) continue;             // merged into its left neighbour
        const int nx = L.nxt[pos];
        if (nx < 0) continue;                   // last symbol
        int new_id;
        const int rk = mm_find(mm, L.c[pos], L.c[nx], new_id);
        if (rk < 0) continue;
        if (rk != trank && mm.rank2new[trank] != new_id) continue;   // expired entry
        L.c[pos] = new_id;
        L.c[nx] = -1;
        const int nn = L.nxt[nx];
        L.nxt[pos] = (int16_t)nn;
        if (nn >= 0) L.prv[nn] = (int16_t)pos;
        const int pv = L.prv[pos];
        if (pv >= 0) {
          int nid;
          const int rp = mm_find(mm, L.c[pv], new_id, nid);
          if (rp >= 0) heap_push(hp, hn, ((uint32_t)rp << 16) | (uint32_t)(pv - sb));
        }
        if (nn >= 0) {
          int nid;
          const int rn = mm_find(mm, new_id, L.c[nn], nid);
          if (rn >= 0) heap_push(hp, hn, ((uint32_t)rn << 16) | (uint32_t)(pos - sb));
        }
      }
    }
    wave_sync();
  }
#endif
  // symbols left per word
  for (int w = lane; w < nw; w += 64) L.wcnt[w] = 0;
  wave_sync();
  for (int s = lane; s < npos; s += 64)
    if (L.c[s] >= 0) atomicAdd(&L.wcnt[L.wid[s]], 1);
  wave_sync();
  BPE_STAMP(5);
  // 5. word offsets (wave scan), ids in order
  carry = 0;
  for (int base = 0; base < nw; base += 64) {
    const int w = base + lane;
    int tot;
    const int v = (w < nw) ? L.wcnt[w] : 0;
    const int ex = wave_excl_scan(v, lane, tot);
    if (w < nw) L.wcnt[w] = carry + ex;
    carry += tot;
  }
  wave_sync();
  int32_t* out = a.out_ids + r * a.out_stride;
  for (int w = lane; w < nw; w += 64) {
    const int sb = L.symoff[L.wcp[w]], se = L.symoff[L.wcp[w + 1]];
    int o = L.wcnt[w];
    for (int s = sb; s < se; ++s)
      if (L.c[s] >= 0) out[o++] = L.c[s];
  }
  if (lane == 0) { a.out_len[r] = carry; a.status[r] = ST_OK; }
  BPE_STAMP(6);
#ifdef BPE_STAMPS
  if (lane == 0 && r < BPE_RS) {
    g_bpe_rs[r][7] = (unsigned long long)L.misc[1];
    g_bpe_rs[r][8] = (unsigned long long)npos;
    g_bpe_rs[r][9] = (unsigned long long)nw;
  }
#endif
}

// the merge map staged in LDS: offsets from the dynamic LDS base, so every probe is a ds_read
struct LdsMap {
  const uint2* kv;
  const uint16_t* rank2new;
  int log2cap;
};

template <bool MAP_LDS, int RMX>
__global__ __launch_bounds__(64 * ENC_MAX_WAVES) void k_bpe_encode(EncArgs a) {
  extern __shared__ __align__(16) char lds_raw[];
  __shared__ int32_t s_b2i[256];    // byte -> vocab id
  __shared__ uint8_t s_lut[256];    // classes of code points < 256
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
#ifdef BPE_STAMPS
  const unsigned long long t_stage = __builtin_amdgcn_s_memrealtime();
#endif
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    s_b2i[i] = a.byte2id[i];
    s_lut[i] = i < a.lut_n ? a.lut[i] : (uint8_t)CLS_OTHER;
  }
  if (!MAP_LDS) __syncthreads();
  size_t row_base = 0;
  LdsMap lm;
  if constexpr (MAP_LDS) {
    const int cap = 1 << a.map.log2cap;
    uint2* kv = reinterpret_cast<uint2*>(lds_raw);
    uint16_t* r2n = reinterpret_cast<uint16_t*>(lds_raw + al16(sizeof(uint32_t) * 2 * (size_t)cap));
    // 16-byte copies (cap >= 64 slots of 8 bytes, 16-byte aligned)
    const uint4* g = reinterpret_cast<const uint4*>(a.map.kv);
    for (int i = threadIdx.x; i < cap / 2; i += blockDim.x) reinterpret_cast<uint4*>(kv)[i] = g[i];
    for (int i = threadIdx.x; i < a.n_merges; i += blockDim.x) r2n[i] = a.map.rank2new[i];
    lm.kv = kv; lm.rank2new = r2n; lm.log2cap = a.map.log2cap;
    row_base = map_lds_bytes(a.map.log2cap, a.n_merges);
    __syncthreads();
  }
#ifdef BPE_STAMPS
  if (lane == 0) {
    const int64_t r0 = (int64_t)blockIdx.x * nwv + wave;
    if (r0 < BPE_RS) { g_bpe_rs[r0][10] = t_stage; g_bpe_rs[r0][11] = __builtin_amdgcn_s_memrealtime(); }
  }
#endif
  const bool heap = enc_needs_heap(a.S, a.heap_merge);
  EncLds L = enc_carve(lds_raw + row_base + (size_t)wave * enc_row_bytes(a.Lc, a.S, heap), a.Lc, a.S, heap);
  for (int64_t r = (int64_t)blockIdx.x * nwv + wave; r < a.n_rows; r += (int64_t)gridDim.x * nwv) {
    if constexpr (MAP_LDS) encode_row<RMX>(a, lm, L, r, lane, s_b2i, s_lut);
    else encode_row<RMX>(a, a.map, L, r, lane, s_b2i, s_lut);
    wave_sync();
  }
}

// ------------------------------------------------------ encode, by words --
// (round 4) HF's BPE merges each pre-tokenised word on its own, so a row's ids are the
// concatenation of its words' ids, and a word's ids are a function of the word alone (its code
// points).  A batch of BEAST rows holds few distinct words (K5's codec sample: 302 k words,
// 77 k distinct, 5.9 byte symbols on average, 47 at most), so k_bpe_words (below) merges each
// distinct word of a workgroup's rows once instead of every word of every row.
constexpr int DW_TINY = 8;         // byte symbols of a tiny word: half a DPP row
constexpr int DW_SHORT = 16;       // ... of a short word: one 16-lane DPP row
constexpr int DW_MID = 64;         // ... of a mid word: one wave; longer -> ST_FALLBACK
constexpr int ST_FALLBACK = 7;     // the row needs k_bpe_encode
constexpr int DW_WAVES = 16;       // rows per k_bpe_words workgroup (at most)
constexpr uint32_t SYM_NONE = 0xFFFFu;

// per-row LDS of k_bpe_words
__host__ __device__ inline size_t dw_row_bytes(int Lc, int S) {
  return 3 * al16(sizeof(int32_t) * (Lc + 1)) + al16(sizeof(int32_t) * Lc) + al16(sizeof(uint16_t) * S) +
         2 * al16(Lc) + 16;
}
// the workgroup's word table (32-bit hash, first occurrence): more slots than the rows can hold words
__host__ __device__ inline int dw_ltab_log2(int Lc, int nwv) {
  int l = 4;
  while ((1ll << l) <= (long long)nwv * Lc) ++l;
  return l;
}
__host__ __device__ inline size_t dw_ltab_bytes(int Lc, int nwv) { return (size_t)8 << dw_ltab_log2(Lc, nwv); }

struct DwRow {
  int32_t* cps;      // [Lc]
  int32_t* symoff;   // [Lc + 1]
  int32_t* wcp;      // [Lc + 1]
  int32_t* e;        // [Lc]
  uint16_t* c;       // [S] byte symbols as vocab ids (SYM_NONE: not in the vocab)
  uint8_t* cls;      // [Lc]
  uint8_t* vis;      // [Lc]
  int32_t* misc;     // [4]
};

__device__ inline DwRow dw_carve(char* p, int Lc, int S) {
  DwRow R;
  auto take = [&](size_t bytes) { char* r = p; p += al16(bytes); return r; };
  R.cps = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  R.symoff = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  R.wcp = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  R.e = (int32_t*)take(sizeof(int32_t) * Lc);
  R.c = (uint16_t*)take(sizeof(uint16_t) * S);
  R.cls = (uint8_t*)take(Lc);
  R.vis = (uint8_t*)take(Lc);
  R.misc = (int32_t*)take(16);
  return R;
}

// One row's pre-tokenisation into its LDS image (one wave): code points, the reference's range
// checks in its order (:181-192), classes, UTF-8 symbol offsets, the regex word starts (as
// k_bpe_encode, no special tokens), byte symbols as vocab ids; a word of more than 64 byte
// symbols makes the row ST_FALLBACK.  st / nw: the row's status and word count.
__device__ __forceinline__ void dw_pretok_row(const EncArgs& a, const DwRow& L, int64_t r, int lane,
                                              const int32_t* s_b2i, const uint8_t* s_lut, int S, int& st, int& nw) {
  BPE_STAMP(0);
  const int64_t r0 = a.row_off[r];
  const int n = (int)(a.row_off[r + 1] - r0);
  if (n > a.Lc) st = ST_TOO_LONG;
  // 1. code points, range checks (reference :181-192 order), classes
  int below = 0, above = 0, notuni = 0, surr = 0, nocls = 0;
  auto code_point = [&](int i, long long t) {
    const long long v = t - a.min_tok;
    below |= v < 0;
    above |= (a.max_span >= 0 && v > a.max_span);
    notuni |= v > 0x10FFFF;
    surr |= (v >= 0xD800 && v <= 0xDFFF);
    nocls |= v >= a.lut_n;
    const int cp = (int)((v < 0 || v > 0x10FFFF) ? 0 : v);
    L.cps[i] = cp;
    L.cls[i] = cp < 256 ? s_lut[cp] : (cp < a.lut_n) ? a.lut[cp] : CLS_OTHER;
  };
  if (st == ST_OK) {   // the first 256 code points' loads all in flight together
    constexpr int PF = 4;
    long long tv[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) tv[k] = lane + 64 * k < n ? a.tok[r0 + lane + 64 * k] : 0;
#pragma unroll
    for (int k = 0; k < PF; ++k)
      if (lane + 64 * k < n) code_point(lane + 64 * k, tv[k]);
    for (int i = lane + 64 * PF; i < n; i += 64) code_point(i, a.tok[r0 + i]);
  }
  if (st == ST_OK) {
    if (__any(below)) st = ST_BELOW_MIN;
    else if (__any(above)) st = ST_ABOVE_MAX;
    else if (__any(notuni)) st = ST_NOT_UNICODE;
    else if (__any(surr)) st = ST_SURROGATE;
    else if (__any(nocls)) st = ST_NO_CLASS;
  }
  BPE_STAMP(1);
  int carry = 0;
  if (st == ST_OK) {   // UTF-8 symbol offsets
    for (int base = 0; base < n; base += 64) {
      const int i = base + lane;
      int tot;
      const int len = (i < n) ? utf8_len(L.cps[i]) : 0;
      const int ex = wave_excl_scan(len, lane, tot);
      if (i < n) L.symoff[i] = carry + ex;
      carry += tot;
    }
    if (lane == 0) L.symoff[n] = carry;
    if (carry > S) st = ST_TOO_LONG;
  }
  wave_sync();
  BPE_STAMP(2);
  if (st == ST_OK) {
    // 2. word starts (as k_bpe_encode, no special tokens); 3. byte symbols as vocab ids
    beast_pt::regex_ends(L.cps, L.cls, L.wcp, L.e, n, lane);   // wcp: scratch until word_starts
    word_starts(L.e, L.vis, L.wcp, nullptr, L.misc, n, lane);
    BPE_STAMP(3);
    for (int i = lane; i < n; i += 64) {
      const int cp = L.cps[i], len = utf8_len(cp), o = L.symoff[i];
      for (int q = 0; q < len; ++q) L.c[o + q] = (uint16_t)s_b2i[utf8_byte(cp, q)];   // -1 -> SYM_NONE
    }
    wave_sync();
    nw = L.misc[0];
    bool fall = false;
    for (int k = lane; k < nw; k += 64) fall |= (L.symoff[L.wcp[k + 1]] - L.symoff[L.wcp[k]]) > DW_MID;
    if (__any(fall)) st = ST_FALLBACK;
  }
}

// lane gl of a GW-lane group reads lane gl + 1 (down) / gl - 1 (up) of its group; `fill` past the ends
template <int GW>
__device__ __forceinline__ uint32_t grp_down1(uint32_t v, uint32_t fill) {
  if constexpr (GW == 8) {   // row_shl:1, and the last lane of each half-row takes the fill
    const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x101, 0xF, 0xF, false);
    return (threadIdx.x & 7) == 7 ? fill : x;
  }
  if constexpr (GW == 16) return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x101, 0xF, 0xF, false);
  // wave_shl:1 (gfx9 DPP): lane 63 has no source and keeps `fill` -- no LDS permute on the round's chain
  else return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xF, 0xF, false);
}
template <int GW>
__device__ __forceinline__ uint32_t grp_up1(uint32_t v, uint32_t fill) {
  if constexpr (GW == 8) {   // row_shr:1, and the first lane of each half-row takes the fill
    const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x111, 0xF, 0xF, false);
    return (threadIdx.x & 7) == 0 ? fill : x;
  }
  if constexpr (GW == 16) return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x111, 0xF, 0xF, false);
  else return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xF, 0xF, false);   // wave_shr:1
}
template <int GW>
__device__ __forceinline__ uint32_t grp_min(uint32_t v) {   // every lane of the group gets the group's min
  if constexpr (GW == 8) {   // half-row mirror (lane i with 7 - i), then the quad's xor 2 and xor 1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    return min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
  }
  if constexpr (GW == 64) {   // row_shr 1, 2, 4, 8 then row_bcast 15 / 31: lane 63 holds the min (DPP only)
    constexpr int MX = (int)0xFFFFFFFFu;
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(MX, (int)v, 0x111, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(MX, (int)v, 0x112, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(MX, (int)v, 0x114, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(MX, (int)v, 0x118, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(MX, (int)v, 0x142, 0xA, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(MX, (int)v, 0x143, 0xC, 0xF, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  }
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false));   // row_ror:8
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false));   // row_ror:4
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xF, 0xF, false));   // row_ror:2
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, false));   // row_ror:1
  return v;
}

// The word's symbols move to the first n lanes of the group, in order (one forward permute).
template <int GW>
__device__ __forceinline__ uint32_t grp_compact(uint32_t sym, bool live, int gl, int gbase, int& n) {
  const unsigned long long bal = __ballot(live);
  const unsigned long long gm = GW == 64 ? bal : ((bal >> gbase) & ((1ull << GW) - 1ull));
  const unsigned long long below = gl == 0 ? 0ull : (gm & ((1ull << gl) - 1ull));
  n = __popcll(gm);
  const int dst = gbase + (live ? __popcll(below) : GW - 1);   // a dead lane only exists when n < GW
  const uint32_t got = (uint32_t)__builtin_amdgcn_ds_permute(dst * 4, (int)sym);
  return gl < n ? got : SYM_NONE;
}

// HF Word::merge_all of one word per GW-lane group: words of <= 16 byte symbols four to a wave
// (one 16-lane DPP row each), longer ones a wave each.  A round probes every adjacent pair's rank
// in the merge map, takes the word's lowest (DPP row rotations), merges its occurrences left to
// right (a self-pair run takes every other one) and compacts the word with one ds_permute.  For
// models whose merges only combine tokens made by earlier merges (the host checks) this is HF's
// merge_all.  raw: the lane's byte symbol
// (SYM_NONE: no vocab id), blen: the word's byte symbols (0: no word).  Returns the lane's final
// id (SYM_NONE past the end); n: the word's final length.
template <int GW>
__device__ __forceinline__ uint32_t dw_merge_word(const WordMap& mm, uint32_t raw, int blen, int unk_id, int fuse_unk,
                                                  int& n, int& rounds) {
  const int lane = threadIdx.x & 63, gl = lane & (GW - 1), gbase = lane - gl;
  // HF BPE::merge_word's unknown chars: unk_id (consecutive ones fused when fuse_unk), or dropped
  const bool in = gl < blen;
  const bool miss = in && raw == SYM_NONE;
  const bool pmiss = grp_up1<GW>(miss ? 1u : 0u, 0u) != 0u;
  const bool live = in && !(miss && (unk_id < 0 || (fuse_unk && pmiss)));
  const uint32_t id = miss ? (uint32_t)unk_id : raw;
  uint32_t sym = grp_compact<GW>(id, live, gl, gbase, n);
  for (int round = 0; round < DW_MID; ++round) {   // each round merges >= 1 pair: <= 63 rounds
    const uint32_t right = grp_down1<GW>(sym, SYM_NONE);
    const bool has = gl + 1 < n;
    uint32_t rk = RK_NONE;
    if (has) {
      const uint32_t key = (sym << 16) | right;
      const uint4 b1 = mm.b[wm_h1(key, mm.log2b)], b2 = mm.b[wm_h2(key, mm.log2b)];
      const uint32_t v = b1.x == key ? b1.y : b1.z == key ? b1.w : b2.x == key ? b2.y : b2.z == key ? b2.w : 0u;
      rk = v ? v - 0x10000u : RK_NONE;   // (rank + 1) << 16 | new_id -> rank << 16 | new_id
    }
    const uint32_t m = grp_min<GW>(rk);
    if (!__any(m != RK_NONE)) break;
    ++rounds;
    const bool match = has && m != RK_NONE && rk == m;
    const unsigned long long mb = __ballot(match);
    const unsigned long long M = GW == 64 ? mb : ((mb >> gbase) & ((1ull << GW) - 1ull));
    // a run of the same self-pair merges left to right: take a match when the matches right
    // before it are an even number (HF pops (rank, pos) in position order)
    const unsigned long long lowm = gl == 0 ? 0ull : ((1ull << gl) - 1ull);
    const unsigned long long z = ~M & lowm;
    const int hz = z ? 63 - __clzll(z) : -1;
    const bool take = match && !((gl - 1 - hz) & 1);
    const bool dies = grp_up1<GW>(take ? 1u : 0u, 0u) != 0u;
    if (take) sym = m & 0xFFFFu;
    sym = grp_compact<GW>(sym, gl < n && !dies, gl, gbase, n);
  }
  return sym;
}

// A word of <= ML byte symbols merged by ONE lane, in registers (round 5, the tiny words): HF's Word::merge_all
// exactly -- repeatedly the pair of lowest (rank, position) among the word's current pairs (the
// min-heap's order, without its stale entries), merged, and the two pairs it forms looked up --
// for any model (no rank-monotone requirement).  Every index into the register arrays is a
// compile-time one (select chains over the dynamic position), so nothing spills to scratch.  A
// wave merges 64 words at once: the cross-lane steps of dw_merge_word (DPP min, ballots, a
// ds_permute per round) are gone, and the map lookups of all lanes are in flight together.
// c: the word's byte symbols in the row image (SYM_NONE: no vocab id); the ids are written back
// over them.  Returns the word's final length.
__device__ __forceinline__ uint32_t wm_rank(const WordMap& mm, uint32_t a, uint32_t b) {   // rank << 16 | new id
  const uint32_t key = (a << 16) | b;
  const uint4 b1 = mm.b[wm_h1(key, mm.log2b)], b2 = mm.b[wm_h2(key, mm.log2b)];
  const uint32_t v = b1.x == key ? b1.y : b1.z == key ? b1.w : b2.x == key ? b2.y : b2.z == key ? b2.w : 0u;
  return v ? v - 0x10000u : RK_NONE;
}

template <int ML>
__device__ __forceinline__ int dw_merge_lane(const WordMap& mm, uint16_t* c, int blen, int unk_id, int fuse_unk,
                                             int& rounds) {
  uint32_t s[ML];
  bool miss_any = false;
#pragma unroll
  for (int i = 0; i < ML; ++i) {
    s[i] = i < blen ? (uint32_t)c[i] : SYM_NONE;
    miss_any |= i < blen && s[i] == SYM_NONE;
  }
  int n = blen;
  if (__any(miss_any)) {
    // HF BPE::merge_word's unknown chars (rare): unk_id, consecutive ones fused when fuse_unk, or
    // dropped without an unk token -- compacted by select chains
    uint32_t t[ML];
    bool pm = false;
    n = 0;
#pragma unroll
    for (int i = 0; i < ML; ++i) t[i] = SYM_NONE;
#pragma unroll
    for (int i = 0; i < ML; ++i) {
      if (i < blen) {
        const bool miss = s[i] == SYM_NONE;
        const bool live = !(miss && (unk_id < 0 || (fuse_unk && pm)));
        const uint32_t id = miss ? (uint32_t)unk_id : s[i];
#pragma unroll
        for (int k = 0; k <= i; ++k) t[k] = (live && k == n) ? id : t[k];
        n += live ? 1 : 0;
        pm = miss;
      }
    }
#pragma unroll
    for (int i = 0; i < ML; ++i) s[i] = t[i];
  }
  uint32_t rk[ML];   // rk[i]: the pair (s[i], s[i + 1]), RK_NONE when it is not a merge
#pragma unroll
  for (int i = 0; i < ML; ++i) rk[i] = i + 1 < n ? wm_rank(mm, s[i], s[i + 1]) : RK_NONE;
  for (int it = 0; it < ML - 1; ++it) {
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i + 1 < ML; ++i)
      best = min(best, rk[i] == RK_NONE ? 0xFFFFFFFFu : (((rk[i] >> 16) << 5) | (uint32_t)i));
    if (best == 0xFFFFFFFFu) break;
    ++rounds;
    const int p = (int)(best & 31u);
    uint32_t nid = 0, left = SYM_NONE, right = SYM_NONE;
#pragma unroll
    for (int i = 0; i < ML; ++i) {
      nid = i == p ? (rk[i] & 0xFFFFu) : nid;
      left = i + 1 == p ? s[i] : left;
      right = i == p + 2 ? s[i] : right;
    }
#pragma unroll
    for (int i = 0; i < ML; ++i) {   // s[p] <- the new id, the symbols after it move left by one
      const uint32_t nx = i + 1 < ML ? s[i + 1] : SYM_NONE;
      s[i] = i == p ? nid : (i > p ? nx : s[i]);
    }
    --n;
    const uint32_t rl = p > 0 ? wm_rank(mm, left, nid) : RK_NONE;
    const uint32_t rr = p + 1 < n ? wm_rank(mm, nid, right) : RK_NONE;
#pragma unroll
    for (int i = 0; i < ML; ++i) {
      const uint32_t nx = i + 1 < ML ? rk[i + 1] : RK_NONE;
      rk[i] = i + 1 == p ? rl : (i == p ? rr : (i > p ? nx : rk[i]));
    }
  }
#pragma unroll
  for (int i = 0; i < ML; ++i)
    if (i < n) c[i] = (uint16_t)s[i];
  return n;
}

// ------------------------------------------------------- encode by words, one launch --
// k_bpe_words: a workgroup takes nwv rows (one wave each) through the whole encode in LDS:
//   1. pre-tokenisation of each row (dw_pretok_row);
//   2. exact dedup of the workgroup's words: a table keyed by a 32-bit hash of the word's code
//      points, each entry (hash, first occurrence); a hash match is confirmed by comparing the
//      code points with the entry's occurrence, so equal hashes of different words only lengthen
//      the probe;
//   3. the distinct words counting-sorted by byte-symbol length, longest first, so the four
//      words of a 16-lane task have similar round counts;
//   4. every distinct word merged once (dw_merge_word), its ids written over its own byte
//      symbols in the row image, its id count beside it;
//   5. each row's ids gathered from its words' first occurrences.
// Nothing but the bins and the ids touches HBM (and the merge map when it is too large for LDS).
__device__ __forceinline__ uint32_t bw_hash(const int32_t* cps, int cs, int ce) {   // FNV-1a + murmur3 fmix
  uint32_t h = 0x811C9DC5u ^ (uint32_t)(ce - cs);
  for (int i = cs; i < ce; ++i) h = (h ^ (uint32_t)cps[i]) * 0x01000193u;
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

__host__ __device__ inline size_t bw_lds_bytes(int Lc, int S, int nwv, int wm_log2b /* < 0: map in HBM */) {
  size_t b = wm_log2b >= 0 ? sizeof(uint4) << wm_log2b : 0;
  b += dw_ltab_bytes(Lc, nwv);
  b += 2 * al16(sizeof(uint32_t) * (size_t)nwv * Lc);
  return b + (size_t)nwv * dw_row_bytes(Lc, S);
}

template <bool MAP_LDS>
__global__ __launch_bounds__(64 * DW_WAVES) void k_bpe_words(EncArgs a, WordMap wm, int ltab_log2, int hash_shift) {
  extern __shared__ __align__(16) char lds_raw[];
  __shared__ int32_t s_b2i[256];
  __shared__ uint8_t s_lut[256];
  __shared__ int s_nd, s_next;
  __shared__ int s_hist[DW_MID + 1];   // distinct words per byte-symbol length, then sort cursors
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  char* p = lds_raw;
  WordMap lm = wm;
  if constexpr (MAP_LDS) {
    uint4* kv = reinterpret_cast<uint4*>(p);
    for (int i = threadIdx.x; i < (1 << wm.log2b); i += blockDim.x) kv[i] = wm.b[i];
    lm.b = kv;
    p += sizeof(uint4) << wm.log2b;
  }
  const int lcap = 1 << ltab_log2;
  unsigned long long* ltab = reinterpret_cast<unsigned long long*>(p);
  p += sizeof(unsigned long long) * (size_t)lcap;
  const int capw = nwv * a.Lc;
  uint32_t* dl = reinterpret_cast<uint32_t*>(p);   // distinct words: wave << 22 | word << 7 | byte symbols
  p += al16(sizeof(uint32_t) * (size_t)capw);
  uint32_t* ds = reinterpret_cast<uint32_t*>(p);   // ... sorted, longest first
  p += al16(sizeof(uint32_t) * (size_t)capw);
  char* rows = p;
  const size_t rb = dw_row_bytes(a.Lc, a.S);
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    s_b2i[i] = a.byte2id[i];
    s_lut[i] = i < a.lut_n ? a.lut[i] : (uint8_t)CLS_OTHER;
  }
  for (int i = threadIdx.x; i < lcap; i += blockDim.x) ltab[i] = 0ull;
  for (int i = threadIdx.x; i <= DW_MID; i += blockDim.x) s_hist[i] = 0;   // 65 bins: one wave is 64 threads
  if (threadIdx.x == 0) { s_nd = 0; s_next = nwv; }
  __syncthreads();
  const DwRow L = dw_carve(rows + (size_t)wave * rb, a.Lc, a.S);
  const int64_t r = (int64_t)blockIdx.x * nwv + wave;
#ifdef BPE_STAMPS
  if (lane == 0 && r < BPE_RS) g_bpe_rs[r][10] = __builtin_amdgcn_s_memrealtime();
#endif
  int st = ST_OK, nw = 0;
  if (r < a.n_rows) dw_pretok_row(a, L, r, lane, s_b2i, s_lut, a.S, st, nw);
  __syncthreads();   // every row's code points, word starts and symbols are readable workgroup-wide
  if (r < a.n_rows) BPE_STAMP(4);
  // 2. exact dedup; L.e[k] = the word's first occurrence (wave << 16 | word)
#ifdef BPE_WORDS_SKIP_DEDUP   // counter attribution only (wrong ids): no dedup, sort or merges
  if (r < a.n_rows && st == ST_OK)
    for (int k = lane; k < nw; k += 64) { L.e[k] = (int32_t)(((uint32_t)wave << 16) | (uint32_t)k); L.vis[k] = 0; }
  if (false) {
#else
  if (r < a.n_rows && st == ST_OK) {
#endif
    const uint32_t lmask = (uint32_t)lcap - 1u;
    for (int k = lane; k < nw; k += 64) {
      const int cs = L.wcp[k], ce = L.wcp[k + 1], len = ce - cs;
      const uint32_t hk = (bw_hash(L.cps, cs, ce) >> hash_shift) | 1u;
      const uint32_t me = ((uint32_t)wave << 16) | (uint32_t)k;
      const unsigned long long mine = ((unsigned long long)hk << 32) | me;
      uint32_t ls = (hk * 0x9E3779B1u) >> (32 - ltab_log2), rep = me;
      while (true) {
        unsigned long long e = ltab[ls];
        if (e == 0ull) {
          e = atomicCAS(&ltab[ls], 0ull, mine);
          if (e == 0ull) break;
        }
        if ((uint32_t)(e >> 32) == hk) {
          const uint32_t o = (uint32_t)e;
          const DwRow Ro = dw_carve(rows + (size_t)(o >> 16) * rb, a.Lc, a.S);
          const int ocs = Ro.wcp[o & 0xFFFF];
          bool same = Ro.wcp[(o & 0xFFFF) + 1] - ocs == len;
          for (int i = 0; same && i < len; ++i) same = Ro.cps[ocs + i] == L.cps[cs + i];
          if (same) { rep = o; break; }
        }
        ls = (ls + 1) & lmask;
      }
      L.e[k] = (int32_t)rep;
      if (rep == me) {
        const int blen = L.symoff[ce] - L.symoff[cs];   // 1..64 (longer words made the row ST_FALLBACK)
        dl[atomicAdd(&s_nd, 1)] = ((uint32_t)wave << 22) | ((uint32_t)k << 7) | (uint32_t)blen;
        atomicAdd(&s_hist[blen], 1);
      }
    }
  }
  __syncthreads();
  // 3. counting sort, longest first: lane l holds length 64 - l
  if (wave == 0) {
    int tot;
    const int ex = wave_excl_scan(s_hist[DW_MID - lane], lane, tot);
    s_hist[DW_MID - lane] = ex;
  }
  __syncthreads();
  const int nd = s_nd;
  for (int i = threadIdx.x; i < nd; i += blockDim.x) {
    const uint32_t v = dl[i];
    ds[atomicAdd(&s_hist[v & 127u], 1)] = v;
  }
  __syncthreads();
  if (r < a.n_rows) BPE_STAMP(5);
  // 4. merges: a mid word (17..64 byte symbols) per wave and words of 9..16 four to a wave (16-lane
  // rows) by dw_merge_word's cooperative rounds; words of <= 8 one per lane, 64 to a task
  // (dw_merge_lane: its select chains stay short, and the tiny words are most of them)
  // the cursor of length 17 has passed every longer word, that of length 9 every word of 9 or
  // more.  Cursors out of order would be a corrupt sort: the workgroup's rows then report
  // ST_FALLBACK (the host re-encodes them with the per-row kernel) and no task runs, instead of a
  // clamp quietly merging whatever the cursors point at (round 5)
  const int c17 = s_hist[DW_SHORT + 1], c9 = s_hist[DW_TINY + 1];
  const bool sane = 0 <= c17 && c17 <= c9 && c9 <= nd;
  if (!sane && st == ST_OK) st = ST_FALLBACK;
  const int nmid = sane ? c17 : 0;
  const int n9 = sane ? c9 : 0;
  const int t16 = nmid + (n9 - nmid + 3) / 4;
  const int tasks = sane ? t16 + (nd - n9 + 63) / 64 : 0;
  int nrounds = 0;
#if defined(BPE_WORDS_SKIP_MERGES) || defined(BPE_WORDS_SKIP_DEDUP)   // counter attribution only (wrong ids)
  if (r < a.n_rows && st == ST_OK)
    for (int k = lane; k < nw; k += 64) L.vis[k] = 0;
  for (int t = tasks; t < tasks;) {
#else
  // tasks longest first, each wave taking the next one when it is done (an LDS counter): the
  // workgroup waits for its slowest wave at the barrier below (29.8 vs 33.0 us with tasks dealt
  // round-robin, profiles/r04/ab/encode_words_variants_r04d.txt)
  for (int t = wave; t < tasks;) {
#endif
#ifdef BPE_STAMPS
    const unsigned long long t_task0 = __builtin_amdgcn_s_memrealtime();
    const int kind_task = t < nmid ? 0 : (t < t16 ? 1 : 2);
#endif
    if (t < nmid) {
      const uint32_t v = ds[t];
      const DwRow Rw = dw_carve(rows + (size_t)(v >> 22) * rb, a.Lc, a.S);
      const int k = (v >> 7) & 0x7FFF, blen = v & 127u;
      const int bs = Rw.symoff[Rw.wcp[k]];
      const uint32_t raw = lane < blen ? (uint32_t)Rw.c[bs + lane] : SYM_NONE;
      int n;
      const uint32_t id = dw_merge_word<DW_MID>(lm, raw, blen, a.unk_id, a.fuse_unk, n, nrounds);
      if (lane < n) Rw.c[bs + lane] = (uint16_t)id;
      if (lane == 0) Rw.vis[k] = (uint8_t)n;
    } else if (t < t16) {
      const int j = nmid + 4 * (t - nmid) + (lane >> 4), gl = lane & 15;
      const bool valid = j < n9;
      const uint32_t v = valid ? ds[j] : 0u;
      const DwRow Rw = dw_carve(rows + (size_t)(v >> 22) * rb, a.Lc, a.S);
      const int k = (v >> 7) & 0x7FFF, blen = valid ? (int)(v & 127u) : 0;
      const int bs = valid ? Rw.symoff[Rw.wcp[k]] : 0;
      const uint32_t raw = gl < blen ? (uint32_t)Rw.c[bs + gl] : SYM_NONE;
      int n;
      const uint32_t id = dw_merge_word<DW_SHORT>(lm, raw, blen, a.unk_id, a.fuse_unk, n, nrounds);
      if (valid && gl < n) Rw.c[bs + gl] = (uint16_t)id;
      if (valid && gl == 0) Rw.vis[k] = (uint8_t)n;
    } else {
      const int j = n9 + 64 * (t - t16) + lane;
      const bool valid = j < nd;
      const uint32_t v = valid ? ds[j] : 0u;
      const DwRow Rw = dw_carve(rows + (size_t)(v >> 22) * rb, a.Lc, a.S);
      const int k = (v >> 7) & 0x7FFF, blen = valid ? (int)(v & 127u) : 0;
      uint16_t* c = Rw.c + (valid ? Rw.symoff[Rw.wcp[k]] : 0);
      const int n = dw_merge_lane<DW_TINY>(lm, c, blen, a.unk_id, a.fuse_unk, nrounds);
      if (valid) Rw.vis[k] = (uint8_t)n;
    }
#ifdef BPE_STAMPS
    if (lane == 0 && r < BPE_RS) {
      g_bpe_wt[r][kind_task] += __builtin_amdgcn_s_memrealtime() - t_task0;
      g_bpe_wt[r][3 + kind_task] += 1;
    }
#endif
    int nt = 0;
    if (lane == 0) nt = atomicAdd(&s_next, 1);
    t = __builtin_amdgcn_readfirstlane(nt);
  }
  __syncthreads();
  if (r < a.n_rows) BPE_STAMP(6);
  // 5. the row's ids from its words' first occurrences
  if (r < a.n_rows) {
    if (st != ST_OK) {
      if (lane == 0) { a.out_len[r] = 0; a.status[r] = st; }
    } else {
      int32_t* out = a.out_ids + r * a.out_stride;
      int carry = 0;
      for (int base = 0; base < nw; base += 64) {
        const int k = base + lane;
        int cnt = 0;
        const uint16_t* src = nullptr;
        if (k < nw) {
          const uint32_t o = (uint32_t)L.e[k];
          const DwRow Ro = dw_carve(rows + (size_t)(o >> 16) * rb, a.Lc, a.S);
          const int ko = o & 0xFFFF;
          cnt = Ro.vis[ko];
          src = Ro.c + Ro.symoff[Ro.wcp[ko]];
        }
        int tot;
        const int off = carry + wave_excl_scan(cnt, lane, tot);
        for (int q = 0; q < cnt; ++q) out[off + q] = (int32_t)src[q];
        carry += tot;
      }
      if (lane == 0) { a.out_len[r] = carry; a.status[r] = ST_OK; }
    }
#ifdef BPE_STAMPS
    if (lane == 0 && r < BPE_RS) { g_bpe_rs[r][7] = __builtin_amdgcn_s_memrealtime(); g_bpe_rs[r][8] = nd; g_bpe_rs[r][9] = nw; }
    if (lane == 0 && r < BPE_RS) g_bpe_rs[r][11] = (unsigned long long)nrounds;
#endif
  }
  (void)nrounds;
}

// ---------------------------------------------------------------- decode --
struct DecArgs {
  const int32_t* ids;
  const int64_t* row_off;
  int64_t n_rows;
  const int32_t* tok_off;     // [n_vocab + 1] byte ranges of each id's decoded bytes
  const uint8_t* tok_bytes;
  const uint8_t* tok_skip;    // [n_vocab] 1: special (skipped) or no such id
  int n_vocab;
  int unk_id;                 // id of "<unk>", -1: none
  long long min_tok;
  int L;                      // expected code points per row (output row width)
  int bcap;                   // LDS byte buffer per wave
  long long* out;             // [n_rows][L]
  int32_t* out_count;         // decoded code points per row
  int32_t* status;            // bit 0: the row holds the <unk> id; bit 1: an id < -1 (not a u32)
};

__device__ __forceinline__ bool cont(int b) { return (b & 0xC0) == 0x80; }

// One step of Rust's lossy UTF-8 decoder (core::str::lossy::Utf8Chunks) on b0 with the
// next bytes b1..b3 (0 past the end): code point (0xFFFD on error) and bytes consumed.
__device__ __forceinline__ int utf8_step(int b0, int b1, int b2, int b3, int& used) {
  if (b0 < 0x80) { used = 1; return b0; }
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (cont(b1)) { used = 2; return ((b0 & 0x1F) << 6) | (b1 & 0x3F); }
    used = 1; return 0xFFFD;
  }
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    const bool ok1 = (b0 == 0xE0) ? (b1 >= 0xA0 && b1 <= 0xBF) : (b0 == 0xED) ? (b1 >= 0x80 && b1 <= 0x9F)
                                                                              : (b1 >= 0x80 && b1 <= 0xBF);
    if (!ok1) { used = 1; return 0xFFFD; }
    if (!cont(b2)) { used = 2; return 0xFFFD; }
    used = 3; return ((b0 & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F);
  }
  if (b0 >= 0xF0 && b0 <= 0xF4) {
    const bool ok1 = (b0 == 0xF0) ? (b1 >= 0x90 && b1 <= 0xBF) : (b0 == 0xF4) ? (b1 >= 0x80 && b1 <= 0x8F)
                                                                              : (b1 >= 0x80 && b1 <= 0xBF);
    if (!ok1) { used = 1; return 0xFFFD; }
    if (!cont(b2)) { used = 2; return 0xFFFD; }
    if (!cont(b3)) { used = 3; return 0xFFFD; }
    used = 4; return ((b0 & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((b2 & 0x3F) << 6) | (b3 & 0x3F);
  }
  used = 1; return 0xFFFD;
}

// serial lossy decode of a byte source (get(i) for i < nb); returns the code point count
template <class Get>
__device__ int decode_serial(Get get, int64_t nb, long long* out, int L, long long min_tok) {
  int cnt = 0;
  int64_t i = 0;
  while (i < nb) {
    const int b0 = get(i);
    const int b1 = i + 1 < nb ? get(i + 1) : 0, b2 = i + 2 < nb ? get(i + 2) : 0, b3 = i + 3 < nb ? get(i + 3) : 0;
    int used;
    const int cp = utf8_step(b0, b1, b2, b3, used);
    if (cnt < L) out[cnt] = (long long)cp + min_tok;
    ++cnt;
    i += used;
  }
  return cnt;
}

__device__ __forceinline__ int tok_len(const DecArgs& a, int id) {
  if (id < 0 || id >= a.n_vocab || a.tok_skip[id]) return 0;
  return a.tok_off[id + 1] - a.tok_off[id];
}

__device__ void decode_row(const DecArgs& a, uint8_t* buf, int64_t r, int lane) {
  const int64_t i0 = a.row_off[r], i1 = a.row_off[r + 1];
  const int n = (int)(i1 - i0);
  long long* out = a.out + r * (int64_t)a.L;
  int unk = 0, ovf = 0;
  // gather bytes into LDS at scanned offsets
  int64_t nb = 0;
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const int id = (i < n) ? a.ids[i0 + i] : -1;
    unk |= (a.unk_id >= 0 && id == a.unk_id);
    ovf |= (id < -1);
    const int len = tok_len(a, id);
    int tot;
    const int ex = wave_excl_scan(len, lane, tot);
    const int64_t o = nb + ex;
    if (len > 0 && o + len <= a.bcap) {
      const uint8_t* src = a.tok_bytes + a.tok_off[id];
      for (int q = 0; q < len; ++q) buf[o + q] = src[q];
    }
    nb += tot;
  }
  const int flags = (__any(unk) ? 1 : 0) | (__any(ovf) ? 2 : 0);
  wave_sync();
  int cnt = -1;
  if (nb <= a.bcap) {
    // valid UTF-8 check and lane-parallel decode: every lead's sequence well-formed and
    // the continuation bytes exactly those the leads claim
    int bad = 0, claimed = 0, conts = 0;
    for (int i = lane; i < nb; i += 64) {
      const int b0 = buf[i];
      if (cont(b0)) { ++conts; continue; }
      const int b1 = i + 1 < nb ? buf[i + 1] : 0, b2 = i + 2 < nb ? buf[i + 2] : 0,
                b3 = i + 3 < nb ? buf[i + 3] : 0;
      int used;
      const int cp = utf8_step(b0, b1, b2, b3, used);
      bad |= (cp == 0xFFFD && !(b0 == 0xEF && b1 == 0xBF && b2 == 0xBD));   // a literal U+FFFD is valid
      claimed += used - 1;
    }
    for (int o = 32; o > 0; o >>= 1) {
      claimed += __shfl_xor(claimed, o);
      conts += __shfl_xor(conts, o);
    }
    if (!__any(bad) && claimed == conts) {
      int carry = 0;
      for (int base = 0; base < nb; base += 64) {
        const int i = base + lane;
        const bool lead = i < nb && !cont(buf[i]);
        int tot;
        const int ex = wave_excl_scan(lead ? 1 : 0, lane, tot);
        if (lead) {
          const int k = carry + ex;
          if (k < a.L) {
            const int b1 = i + 1 < nb ? buf[i + 1] : 0, b2 = i + 2 < nb ? buf[i + 2] : 0,
                      b3 = i + 3 < nb ? buf[i + 3] : 0;
            int used;
            out[k] = (long long)utf8_step(buf[i], b1, b2, b3, used) + a.min_tok;
          }
        }
        carry += tot;
      }
      cnt = carry;
    } else if (lane == 0) {
      cnt = decode_serial([&](int64_t i) { return (int)buf[i]; }, nb, out, a.L, a.min_tok);
    }
  } else if (lane == 0) {
    // more bytes than the LDS buffer holds (the row cannot decode to L code points anyway):
    // stream them from HBM to get HF's exact count for the error message
    const int32_t* ids = a.ids + i0;
    int64_t ti = 0;
    int32_t bo = 0, be = 0;
    auto next_byte = [&]() -> int {
      while (bo >= be) {
        if (ti >= n) return -1;
        const int id = ids[ti++];
        if (tok_len(a, id) == 0) continue;
        bo = a.tok_off[id];
        be = a.tok_off[id + 1];
      }
      return a.tok_bytes[bo++];
    };
    int bq[4], nq = 0, c = 0;
    while (true) {
      while (nq < 4) {
        const int b = next_byte();
        if (b < 0) break;
        bq[nq++] = b;
      }
      if (nq == 0) break;
      int used;
      const int cp = utf8_step(bq[0], nq > 1 ? bq[1] : 0, nq > 2 ? bq[2] : 0, nq > 3 ? bq[3] : 0, used);
      if (c < a.L) out[c] = (long long)cp + a.min_tok;
      ++c;
      for (int k = used; k < nq; ++k) bq[k - used] = bq[k];
      nq -= used;
    }
    cnt = c;
  }
  if (lane == 0) { a.out_count[r] = cnt; a.status[r] = flags; }
}

__global__ __launch_bounds__(BLOCK) void k_bpe_decode(DecArgs a) {
  extern __shared__ __align__(16) char lds_raw[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* buf = (uint8_t*)lds_raw + (size_t)wave * al16(a.bcap);
  for (int64_t r = (int64_t)blockIdx.x * WAVES + wave; r < a.n_rows; r += (int64_t)gridDim.x * WAVES) {
    decode_row(a, buf, r, lane);
    wave_sync();
  }
}

inline int log2_ceil(int64_t x) {
  int l = 0;
  while ((int64_t(1) << l) < x) ++l;
  return l;
}

// rows -> workgroups: at most the ones resident at once (per_cu from the occupancy of the launch:
// each workgroup stages the merge map once and then loops over rows)
int grid_for(int64_t n_rows, int per_cu = 4) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  const int64_t want = (n_rows + WAVES - 1) / WAVES;
  const int64_t cap = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
  return (int)(want < cap ? want : cap);
}

}  // namespace

#ifdef BPE_STAMPS
extern "C" int beast_debug_bpe_stamps(unsigned long long* host) {   // [4096][12]
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_rs), sizeof(g_bpe_rs)) == hipSuccess ? 0 : -2;
}
extern "C" int beast_debug_bpe_task_times(unsigned long long* host, int clear) {   // [4096][8]
  if (clear) {
    static unsigned long long zero[BPE_RS][8];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_bpe_wt), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bpe_wt), sizeof(g_bpe_wt)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int beast_bpe_mergemap_log2cap(int n_merges) {
  const int l = log2_ceil(2 * (int64_t)(n_merges > 0 ? n_merges : 1));
  return l < 6 ? 6 : l;
}

extern "C" size_t beast_bpe_mergemap_bytes(int n_merges) {
  const size_t cap = size_t(1) << beast_bpe_mergemap_log2cap(n_merges);
  return al16(cap * 2 * sizeof(uint32_t)) + al16((size_t)(n_merges > 0 ? n_merges : 1) * sizeof(uint16_t));
}

static MergeMap map_view(const void* map, int n_merges) {
  MergeMap m;
  m.log2cap = beast_bpe_mergemap_log2cap(n_merges);
  const size_t cap = size_t(1) << m.log2cap;
  m.kv = reinterpret_cast<const uint2*>(map);
  m.rank2new = reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(map) + al16(cap * 2 * sizeof(uint32_t)));
  return m;
}

extern "C" int beast_bpe_mergemap_build(const int32_t* merge_a, const int32_t* merge_b, const int32_t* merge_new,
                                        int n_merges, void* map, size_t map_bytes, void* stream) {
  BEAST_REQUIRE(n_merges >= 0 && n_merges < 65536, "n_merges out of range (0..65535): %d", n_merges);
  BEAST_REQUIRE(map != nullptr, "mergemap buffer is null");
  BEAST_REQUIRE_CODE(map_bytes >= beast_bpe_mergemap_bytes(n_merges), BEAST_E_WORKSPACE,
                     "mergemap buffer too small: %zu < %zu", map_bytes, beast_bpe_mergemap_bytes(n_merges));
  BEAST_REQUIRE(n_merges == 0 || (merge_a && merge_b && merge_new), "merge arrays are null");
  const MergeMap m = map_view(map, n_merges);
  const int cap = 1 << m.log2cap;
  hipStream_t s = beast::as_stream(stream);
  hipLaunchKernelGGL(k_mergemap_clear, dim3((cap + 255) / 256), dim3(256), 0, s, const_cast<uint2*>(m.kv), cap);
  BEAST_LAUNCHED("k_mergemap_clear");
  if (n_merges > 0) {
    hipLaunchKernelGGL(k_mergemap_build, dim3((n_merges + 255) / 256), dim3(256), 0, s, merge_a, merge_b, merge_new,
                       n_merges, const_cast<uint2*>(m.kv), const_cast<uint16_t*>(m.rank2new), m.log2cap);
    BEAST_LAUNCHED("k_mergemap_build");
  }
  return BEAST_OK;
}

extern "C" size_t beast_bpe_encode_lds_bytes(int max_row_cps, int max_row_syms) {   // per row (wave)
  return enc_row_bytes(max_row_cps, max_row_syms, enc_needs_heap(max_row_syms, beast::g_bpe_encode_mode & 1));
}

extern "C" int beast_bpe_encode_rows(const int64_t* tok, const int64_t* row_off, int64_t n_rows, int64_t min_tok,
                                     int64_t max_span, const uint8_t* cls_lut, int64_t lut_n, const int32_t* byte2id,
                                     const void* map, int n_merges, const int32_t* spec_cps, const int32_t* spec_len,
                                     const int32_t* spec_id, int n_spec, int unk_id, int fuse_unk, int max_row_cps,
                                     int max_row_syms, int32_t* out_ids, int64_t out_stride, int32_t* out_len,
                                     int32_t* status, void* stream) {
  BEAST_REQUIRE(n_rows >= 0, "n_rows must be >= 0");
  if (n_rows == 0) return BEAST_OK;
  BEAST_REQUIRE(tok && row_off && cls_lut && byte2id && map && out_ids && out_len && status, "null pointer argument");
  BEAST_REQUIRE(lut_n > 0 && lut_n <= 65536, "class LUT size %lld out of range", (long long)lut_n);
  BEAST_REQUIRE(n_merges >= 0 && n_merges < 65536, "n_merges out of range (0..65535): %d", n_merges);
  BEAST_REQUIRE(max_row_cps >= 0 && max_row_cps < 32768, "max_row_cps %d out of range", max_row_cps);
  BEAST_REQUIRE_CODE(max_row_syms >= 0 && max_row_syms <= 16384, BEAST_E_UNSUPPORTED,
                     "rows of %d byte symbols exceed the encoder's per-row LDS budget (16384)", max_row_syms);
  BEAST_REQUIRE(out_stride >= max_row_syms, "out_stride %lld < max_row_syms %d", (long long)out_stride, max_row_syms);
  BEAST_REQUIRE(n_spec >= 0 && n_spec <= MAX_SPECIAL, "at most %d special tokens are supported", MAX_SPECIAL);
  BEAST_REQUIRE(n_spec == 0 || (spec_cps && spec_len && spec_id), "special-token arrays are null");
  const size_t row_b = enc_row_bytes(max_row_cps, max_row_syms, enc_needs_heap(max_row_syms, beast::g_bpe_encode_mode & 1));
  BEAST_REQUIRE_CODE(row_b + STATIC_LDS <= LDS_BUDGET, BEAST_E_UNSUPPORTED,
                     "rows of %d code points / %d byte symbols need %zu B of LDS (> 160 KiB)", max_row_cps,
                     max_row_syms, row_b);
  EncArgs a;
  a.tok = reinterpret_cast<const long long*>(tok);
  a.row_off = row_off; a.n_rows = n_rows; a.min_tok = min_tok; a.max_span = max_span;
  a.lut = cls_lut; a.lut_n = (int)lut_n; a.byte2id = byte2id;
  a.map = map_view(map, n_merges);
  a.n_merges = n_merges;
  // one workgroup per CU holding the merge map once and as many rows (waves) as fit beside it
  // (BEAST_OPT_BPE_ENCODE_MODE bit 1: four waves per workgroup, as many workgroups as fit)
  const size_t map_lds = map_lds_bytes(a.map.log2cap, n_merges);
  const int want_w = (beast::g_bpe_encode_mode & 2) ? WAVES : ENC_MAX_WAVES;
  a.map_in_lds = (map_lds > 0 && map_lds + row_b + STATIC_LDS <= LDS_BUDGET) ? 1 : 0;
  const size_t room = LDS_BUDGET - STATIC_LDS - (a.map_in_lds ? map_lds : 0);
  const int nwv = (int)std::max<size_t>(1, std::min<size_t>((size_t)want_w, room / row_b));
  const size_t rows_lds = (size_t)nwv * row_b;
  a.spec_cps = spec_cps; a.spec_len = spec_len; a.spec_id = spec_id; a.n_spec = n_spec;
  a.unk_id = unk_id; a.fuse_unk = fuse_unk;
  a.heap_merge = beast::g_bpe_encode_mode & 1;
  a.Lc = max_row_cps; a.S = max_row_syms;
  a.out_ids = out_ids; a.out_stride = out_stride; a.out_len = out_len; a.status = status;
  const size_t lds = rows_lds + (a.map_in_lds ? map_lds : 0);
  const bool narrow = max_row_syms <= 64 * RM_NARROW;   // every row fits the narrow kernel's round merge
  const void* fn = a.map_in_lds ? (narrow ? reinterpret_cast<const void*>(&k_bpe_encode<true, RM_NARROW>)
                                          : reinterpret_cast<const void*>(&k_bpe_encode<true, RM_PER>))
                                : (narrow ? reinterpret_cast<const void*>(&k_bpe_encode<false, RM_NARROW>)
                                          : reinterpret_cast<const void*>(&k_bpe_encode<false, RM_PER>));
  if (lds > 65536)
    BEAST_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
              "hipFuncSetAttribute(k_bpe_encode)");
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * nwv, lds) != hipSuccess || per_cu <= 0) per_cu = 1;
  const int grid = (int)std::min<int64_t>((n_rows + nwv - 1) / nwv, (int64_t)grid_for(1 << 30, per_cu));
  if (a.map_in_lds && narrow)
    hipLaunchKernelGGL((k_bpe_encode<true, RM_NARROW>), dim3(grid), dim3(64 * nwv), lds, beast::as_stream(stream), a);
  else if (a.map_in_lds)
    hipLaunchKernelGGL((k_bpe_encode<true, RM_PER>), dim3(grid), dim3(64 * nwv), lds, beast::as_stream(stream), a);
  else if (narrow)
    hipLaunchKernelGGL((k_bpe_encode<false, RM_NARROW>), dim3(grid), dim3(64 * nwv), lds, beast::as_stream(stream), a);
  else
    hipLaunchKernelGGL((k_bpe_encode<false, RM_PER>), dim3(grid), dim3(64 * nwv), lds, beast::as_stream(stream), a);
  BEAST_LAUNCHED("k_bpe_encode");
  return BEAST_OK;
}


// ---- k_bpe_words' merge map (host build) ----
extern "C" int beast_bpe_wordmap_log2buckets(int n_merges) {   // buckets >= merges: at most half the slots used
  return std::max(4, log2_ceil(std::max(1, n_merges)));
}
extern "C" size_t beast_bpe_wordmap_bytes(int n_merges) {   // room for one doubling if an insertion fails
  return sizeof(uint32_t) * 4 * ((size_t)2 << beast_bpe_wordmap_log2buckets(n_merges));
}
static bool wordmap_try(const int32_t* ma, const int32_t* mb, const int32_t* mn, int n, uint32_t* t, int lb) {
  const size_t nb = (size_t)1 << lb;
  for (size_t i = 0; i < 4 * nb; i += 2) { t[i] = EMPTY_KEY; t[i + 1] = 0u; }
  auto slot_of = [&](uint32_t key) -> uint32_t* {   // the key's slot, if present
    for (uint32_t bk : {wm_h1(key, lb), wm_h2(key, lb)})
      for (int q = 0; q < 2; ++q)
        if (t[4 * bk + 2 * q] == key) return &t[4 * bk + 2 * q];
    return nullptr;
  };
  uint32_t rng = 0x2545F491u;
  for (int i = 0; i < n; ++i) {
    uint32_t key = ((uint32_t)ma[i] << 16) | (uint32_t)mb[i];
    uint32_t val = ((uint32_t)(i + 1) << 16) | (uint32_t)mn[i];
    if (uint32_t* e = slot_of(key)) { e[1] = val; continue; }   // a pair listed twice keeps its last rank
    uint32_t bk = wm_h1(key, lb);
    bool placed = false;
    for (int kick = 0; kick < 512 && !placed; ++kick) {
      for (uint32_t c : {wm_h1(key, lb), wm_h2(key, lb)})
        for (int q = 0; q < 2 && !placed; ++q)
          if (t[4 * c + 2 * q] == EMPTY_KEY) { t[4 * c + 2 * q] = key; t[4 * c + 2 * q + 1] = val; placed = true; }
      if (placed) break;
      // evict a pseudo-random slot of the bucket not just left, carry its key on
      rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5;
      bk = (bk == wm_h1(key, lb)) ? wm_h2(key, lb) : wm_h1(key, lb);
      const int q = rng & 1;
      std::swap(key, t[4 * bk + 2 * q]);
      std::swap(val, t[4 * bk + 2 * q + 1]);
    }
    if (!placed) return false;
  }
  return true;
}
extern "C" int beast_bpe_wordmap_build_host(const int32_t* merge_a, const int32_t* merge_b, const int32_t* merge_new,
                                            int n_merges, void* host_out, size_t bytes, int* log2b_out) {
  BEAST_REQUIRE(n_merges >= 0 && n_merges < 65536, "n_merges out of range (0..65535): %d", n_merges);
  BEAST_REQUIRE(host_out && log2b_out && (n_merges == 0 || (merge_a && merge_b && merge_new)), "null pointer argument");
  BEAST_REQUIRE_CODE(bytes >= beast_bpe_wordmap_bytes(n_merges), BEAST_E_WORKSPACE, "word map buffer %zu < %zu", bytes,
                     beast_bpe_wordmap_bytes(n_merges));
  uint32_t* t = static_cast<uint32_t*>(host_out);
  const int lb0 = beast_bpe_wordmap_log2buckets(n_merges);
  for (int lb = lb0; lb <= lb0 + 1; ++lb)
    if (wordmap_try(merge_a, merge_b, merge_new, n_merges, t, lb)) {
      *log2b_out = lb;
      return BEAST_OK;
    }
  BEAST_REQUIRE_CODE(false, BEAST_E_UNSUPPORTED, "word map: cuckoo insertion failed");
  return BEAST_E_UNSUPPORTED;
}

extern "C" int beast_bpe_encode_rows_words(const int64_t* tok, const int64_t* row_off, int64_t n_rows,
                                           int64_t min_tok, int64_t max_span, const uint8_t* cls_lut, int64_t lut_n,
                                           const int32_t* byte2id, const void* wordmap, int wordmap_log2b, int unk_id,
                                           int fuse_unk, int max_row_cps, int max_row_syms, int32_t* out_ids,
                                           int64_t out_stride, int32_t* out_len, int32_t* status, void* stream) {
  BEAST_REQUIRE(n_rows >= 0, "n_rows must be >= 0");
  if (n_rows == 0) return BEAST_OK;
  BEAST_REQUIRE(tok && row_off && cls_lut && byte2id && wordmap && out_ids && out_len && status, "null pointer argument");
  BEAST_REQUIRE(lut_n > 0 && lut_n <= 65536, "class LUT size %lld out of range", (long long)lut_n);
  BEAST_REQUIRE(wordmap_log2b >= 4 && wordmap_log2b <= 20, "wordmap_log2b %d out of range (4..20)", wordmap_log2b);
  BEAST_REQUIRE(max_row_cps >= 0 && max_row_cps < 32768, "max_row_cps %d out of range", max_row_cps);
  BEAST_REQUIRE(max_row_syms >= 0 && max_row_syms <= 16384, "max_row_syms %d out of range", max_row_syms);
  BEAST_REQUIRE(out_stride >= max_row_syms, "out_stride %lld < max_row_syms %d", (long long)out_stride, max_row_syms);
  EncArgs a{};
  a.tok = reinterpret_cast<const long long*>(tok);
  a.row_off = row_off; a.n_rows = n_rows; a.min_tok = min_tok; a.max_span = max_span;
  a.lut = cls_lut; a.lut_n = (int)lut_n; a.byte2id = byte2id;
  a.unk_id = unk_id; a.fuse_unk = fuse_unk;
  a.Lc = max_row_cps; a.S = max_row_syms;
  a.out_ids = out_ids; a.out_stride = out_stride; a.out_len = out_len; a.status = status;
  const WordMap wm{static_cast<const uint4*>(wordmap), wordmap_log2b};
  // as many rows per workgroup as the LDS holds (<= 16), the merge map staged when it fits beside them
  const size_t room = LDS_BUDGET - STATIC_LDS;
  int map_log2 = wordmap_log2b <= 13 ? wordmap_log2b : -1, nwv = 0;
  for (int pass = 0; pass < 2 && nwv == 0; ++pass) {
    for (int nv = DW_WAVES; nv > 0 && nwv == 0; --nv)
      if (bw_lds_bytes(a.Lc, a.S, nv, map_log2) <= room) nwv = nv;
    if (nwv == 0) map_log2 = -1;
  }
  BEAST_REQUIRE_CODE(nwv > 0, BEAST_E_UNSUPPORTED, "rows of %d code points exceed k_bpe_words' LDS budget", max_row_cps);
  const int ltab_log2 = dw_ltab_log2(a.Lc, nwv);
  const int hash_shift = 32 - std::min(32, std::max(1, beast::g_bpe_dedup_key_bits));
  const size_t lds = bw_lds_bytes(a.Lc, a.S, nwv, map_log2);
  hipStream_t s = beast::as_stream(stream);
  const dim3 grid((unsigned)((n_rows + nwv - 1) / nwv)), block(64 * nwv);
  if (map_log2 >= 0) {
    if (lds > 65536)
      BEAST_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bpe_words<true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "hipFuncSetAttribute(k_bpe_words)");
    hipLaunchKernelGGL(k_bpe_words<true>, grid, block, lds, s, a, wm, ltab_log2, hash_shift);
  } else {
    if (lds > 65536)
      BEAST_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bpe_words<false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "hipFuncSetAttribute(k_bpe_words)");
    hipLaunchKernelGGL(k_bpe_words<false>, grid, block, lds, s, a, wm, ltab_log2, hash_shift);
  }
  BEAST_LAUNCHED("k_bpe_words");
  return BEAST_OK;
}

extern "C" int beast_bpe_decode_rows(const int32_t* ids, const int64_t* row_off, int64_t n_rows,
                                     const int32_t* tok_off, const uint8_t* tok_bytes, const uint8_t* tok_skip,
                                     int n_vocab, int unk_id, int64_t min_tok, int L, int64_t* out,
                                     int32_t* out_count, int32_t* status, void* stream) {
  BEAST_REQUIRE(n_rows >= 0, "n_rows must be >= 0");
  if (n_rows == 0) return BEAST_OK;
  BEAST_REQUIRE(ids && row_off && tok_off && tok_bytes && tok_skip && out && out_count && status,
                "null pointer argument");
  BEAST_REQUIRE(n_vocab > 0 && L >= 0, "n_vocab must be > 0 and L >= 0");
  DecArgs a;
  a.ids = ids; a.row_off = row_off; a.n_rows = n_rows; a.tok_off = tok_off; a.tok_bytes = tok_bytes;
  a.tok_skip = tok_skip; a.n_vocab = n_vocab; a.unk_id = unk_id; a.min_tok = min_tok; a.L = L;
  // a row that decodes to L code points holds at most 4 L bytes; more -> streamed from HBM
  int64_t bcap = 4 * (int64_t)L + 16;
  if (bcap > (int64_t)(LDS_BUDGET / WAVES)) bcap = LDS_BUDGET / WAVES;
  a.bcap = (int)bcap;
  a.out = reinterpret_cast<long long*>(out); a.out_count = out_count; a.status = status;
  hipLaunchKernelGGL(k_bpe_decode, dim3(grid_for(n_rows)), dim3(BLOCK), (size_t)WAVES * al16(a.bcap),
                     beast::as_stream(stream), a);
  BEAST_LAUNCHED("k_bpe_decode");
  return BEAST_OK;
}
