// Byte-level BPE *inference* on gfx950: encode bin rows into BPE ids and decode BPE ids
// back into bins.  Replaces, per row,
//   tokenizer.encode("".join(map(chr, row - min)), add_special_tokens=False).ids
//   ord(c) + min for c in tokenizer.decode(ids, skip_special_tokens=True)
// of beast/beast_bspline_bpe_tokenizer.py:175-247 (HF tokenizers 0.22.2: AddedVocabulary
// split, ByteLevel pre-tokeniser, BPE::merge_word + Word::merge_all, ByteLevel decoder,
// String::from_utf8_lossy).
//
//   k_mergemap_build   open-addressing (a, b) -> (rank, new_id) table in HBM; a pair listed
//                      twice keeps its LAST rank (HF collects the merges into a HashMap)
//   k_bpe_encode       one 64-lane workgroup per row, everything of the row in LDS:
//                        lanes: code points, range checks, classes, UTF-8 symbol offsets
//                        lane 0: special-token split (leftmost-longest) + GPT-2 regex walk
//                        lanes: byte -> vocab id, one word per lane: HF's merge_all with
//                        its (rank, pos) min-heap in LDS (stale entries skipped exactly as
//                        HF does, so the result is HF's even when two merges share an id)
//                        lanes: scan of per-word counts, ids written to the padded output
//   k_bpe_decode       one thread per row: token bytes streamed through Rust's lossy UTF-8
//                      decoder (maximal-subpart U+FFFD), code points + min written out
#include <hip/hip_runtime.h>

#include "common.h"

namespace {

constexpr uint32_t EMPTY_KEY = 0xFFFFFFFFu;
constexpr int CLS_OTHER = 0, CLS_LETTER = 1, CLS_NUMBER = 2, CLS_WS = 3;
constexpr int ENC_T = 64;           // one wave per row
constexpr int MAX_SPECIAL = 64, MAX_SPECIAL_LEN = 64;

// encode status per row (host maps them to the reference's exceptions)
constexpr int ST_OK = 0, ST_BELOW_MIN = 1, ST_ABOVE_MAX = 2, ST_NOT_UNICODE = 3, ST_SURROGATE = 4,
              ST_NO_CLASS = 5, ST_TOO_LONG = 6;

__device__ __forceinline__ uint32_t mm_hash(uint32_t key, int log2cap) {
  return (key * 0x9E3779B1u) >> (32 - log2cap);
}

__global__ void k_mergemap_clear(uint32_t* __restrict__ keys, unsigned long long* __restrict__ vals, int cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) { keys[i] = EMPTY_KEY; vals[i] = 0ull; }
}

__global__ void k_mergemap_build(const int32_t* __restrict__ ma, const int32_t* __restrict__ mb,
                                 const int32_t* __restrict__ mnew, int n, uint32_t* __restrict__ keys,
                                 unsigned long long* __restrict__ vals, int log2cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = ((uint32_t)ma[i] << 16) | (uint32_t)mb[i];
  const uint32_t mask = (1u << log2cap) - 1u;
  uint32_t h = mm_hash(key, log2cap);
  while (true) {
    const uint32_t prev = atomicCAS(&keys[h], EMPTY_KEY, key);
    if (prev == EMPTY_KEY || prev == key) break;
    h = (h + 1) & mask;
  }
  // later rank wins; the value is (rank + 1) << 32 | new_id so that 0 means "unset"
  atomicMax(&vals[h], ((unsigned long long)(uint32_t)(i + 1) << 32) | (uint32_t)mnew[i]);
}

// (rank << 16 | new_id) of pair (a, b), or -1.  rank < 2^31, new_id < 2^16.
__device__ __forceinline__ long long mm_find(const uint32_t* __restrict__ keys,
                                             const unsigned long long* __restrict__ vals, int log2cap,
                                             int a, int b) {
  const uint32_t key = ((uint32_t)a << 16) | (uint32_t)b;
  const uint32_t mask = (1u << log2cap) - 1u;
  uint32_t h = mm_hash(key, log2cap);
  while (true) {
    const uint32_t k = keys[h];
    if (k == key) {
      const unsigned long long v = vals[h];
      return (long long)((((v >> 32) - 1ull) << 16) | (v & 0xFFFFull));
    }
    if (k == EMPTY_KEY) return -1;
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
// min-heap of u64 keys (rank << 32 | pos << 16 | new_id) in LDS, one per word
__device__ __forceinline__ void heap_push(unsigned long long* h, int& n, unsigned long long v) {
  int i = n++;
  while (i > 0) {
    const int p = (i - 1) >> 1;
    if (h[p] <= v) break;
    h[i] = h[p];
    i = p;
  }
  h[i] = v;
}

__device__ __forceinline__ unsigned long long heap_pop(unsigned long long* h, int& n) {
  const unsigned long long top = h[0];
  const unsigned long long v = h[--n];
  int i = 0;
  while (true) {
    int c = 2 * i + 1;
    if (c >= n) break;
    if (c + 1 < n && h[c + 1] < h[c]) ++c;
    if (v <= h[c]) break;
    h[i] = h[c];
    i = c;
  }
  if (n > 0) h[i] = v;
  return top;
}

struct EncLds {
  int32_t* cps;       // [Lc] shifted code points
  int32_t* symoff;    // [Lc + 1] first byte symbol of each code point
  int32_t* wcp;       // [Lc + 1] word boundaries (code point index)
  int32_t* wspec;     // [Lc] special-token id of a word, or -1
  int32_t* wcnt;      // [Lc] final symbols per word, then their output offsets
  uint8_t* cls;       // [Lc]
  int32_t* c;         // [S] symbol ids (-1: none)
  int16_t* prv;       // [S]
  int16_t* nxt;       // [S]
  unsigned long long* heap;  // [3 S]
  int32_t* misc;      // [4]: n_words
};

__host__ __device__ inline size_t enc_align(size_t x) { return (x + 15) & ~size_t(15); }

__host__ __device__ inline size_t enc_lds_bytes(int Lc, int S) {
  size_t b = 0;
  b += enc_align(sizeof(int32_t) * Lc);            // cps
  b += enc_align(sizeof(int32_t) * (Lc + 1)) * 2;  // symoff, wcp
  b += enc_align(sizeof(int32_t) * Lc) * 2;        // wspec, wcnt
  b += enc_align(Lc);                              // cls
  b += enc_align(sizeof(int32_t) * S);             // c
  b += enc_align(sizeof(int16_t) * S) * 2;         // prv, nxt
  b += enc_align(sizeof(unsigned long long) * 3 * (size_t)S);
  b += 16;                                         // misc
  return b;
}

__device__ inline EncLds enc_carve(char* p, int Lc, int S) {
  EncLds L;
  auto take = [&](size_t bytes) { char* r = p; p += enc_align(bytes); return r; };
  L.heap = (unsigned long long*)take(sizeof(unsigned long long) * 3 * (size_t)S);
  L.cps = (int32_t*)take(sizeof(int32_t) * Lc);
  L.symoff = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  L.wcp = (int32_t*)take(sizeof(int32_t) * (Lc + 1));
  L.wspec = (int32_t*)take(sizeof(int32_t) * Lc);
  L.wcnt = (int32_t*)take(sizeof(int32_t) * Lc);
  L.c = (int32_t*)take(sizeof(int32_t) * S);
  L.prv = (int16_t*)take(sizeof(int16_t) * S);
  L.nxt = (int16_t*)take(sizeof(int16_t) * S);
  L.cls = (uint8_t*)take(Lc);
  L.misc = (int32_t*)take(16);
  return L;
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
  const uint32_t* mm_keys;
  const unsigned long long* mm_vals;
  int mm_log2cap;
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

// GPT-2 regex from code point i of [.., n): returns the end of the word.
//   's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
__device__ __forceinline__ int regex_word(const int32_t* cps, const uint8_t* cls, int i, int n) {
  const int c = cps[i];
  if (c == '\'' && i + 1 < n) {
    const int c1 = cps[i + 1];
    if (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd') return i + 2;
    if (i + 2 < n) {
      const int c2 = cps[i + 2];
      if ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l')) return i + 3;
    }
  }
  int k = cls[i], st = i;
  if (c == ' ' && i + 1 < n && cls[i + 1] != CLS_WS) { k = cls[i + 1]; st = i + 1; }
  int j;
  if (k != CLS_WS) {
    j = st + 1;
    while (j < n && cls[j] == k) ++j;
  } else {
    j = i + 1;
    while (j < n && cls[j] == CLS_WS) ++j;
    if (j < n && j - i >= 2) --j;  // \s+(?!\S): the last blank starts the next word
  }
  return j;
}

__global__ __launch_bounds__(ENC_T) void k_bpe_encode(EncArgs a) {
  extern __shared__ __align__(16) char lds_raw[];
  const int64_t r = blockIdx.x;
  if (r >= a.n_rows) return;
  const int lane = threadIdx.x;
  EncLds L = enc_carve(lds_raw, a.Lc, a.S);
  const int64_t r0 = a.row_off[r];
  const int n = (int)(a.row_off[r + 1] - r0);
  if (n > a.Lc) {
    if (lane == 0) { a.status[r] = ST_TOO_LONG; a.out_len[r] = 0; }
    return;
  }

  // 1. code points, range checks (reference :181-192 order: below-min first), classes
  int below = 0, above = 0, notuni = 0, surr = 0, nocls = 0;
  for (int i = lane; i < n; i += ENC_T) {
    const long long v = a.tok[r0 + i] - a.min_tok;
    below |= v < 0;
    above |= (a.max_span >= 0 && v > a.max_span);
    notuni |= v > 0x10FFFF;
    surr |= (v >= 0xD800 && v <= 0xDFFF);
    nocls |= v >= a.lut_n;
    const int cp = (int)(v < 0 ? 0 : v > 0x10FFFF ? 0 : v);
    L.cps[i] = cp;
    L.cls[i] = (cp < a.lut_n) ? a.lut[cp] : CLS_OTHER;
  }
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
  // UTF-8 symbol offsets: wave scan in chunks of 64 code points
  int carry = 0;
  for (int base = 0; base < n; base += ENC_T) {
    const int i = base + lane;
    const int len = (i < n) ? utf8_len(L.cps[i]) : 0;
    int x = len;
    for (int o = 1; o < ENC_T; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (i < n) L.symoff[i] = carry + x - len;
    carry += __shfl(x, ENC_T - 1);
  }
  if (lane == 0) L.symoff[n] = carry;
  const int nsym = carry;
  if (nsym > a.S) {   // host sizes S from the code-point bound; guard anyway
    if (lane == 0) { a.status[r] = ST_TOO_LONG; a.out_len[r] = 0; }
    return;
  }
  __syncthreads();

  // 2. lane 0: AddedVocabulary split (leftmost-longest special token), then the regex walk
  if (lane == 0) {
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
        // pre-tokenise the plain segment [seg, i)
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
  // 3. byte symbols as vocab ids
  for (int i = lane; i < n; i += ENC_T) {
    const int cp = L.cps[i], len = utf8_len(cp), o = L.symoff[i];
    for (int q = 0; q < len; ++q) L.c[o + q] = a.byte2id[utf8_byte(cp, q)];
  }
  __syncthreads();
  const int nw = L.misc[0];

  // 4. one word per lane: BPE::merge_word + Word::merge_all
  for (int w = lane; w < nw; w += ENC_T) {
    const int sb = L.symoff[L.wcp[w]], se = L.symoff[L.wcp[w + 1]];
    if (L.wspec[w] >= 0) {
      L.c[sb] = L.wspec[w];
      for (int s = sb + 1; s < se; ++s) L.c[s] = -1;
      L.wcnt[w] = 1;
      continue;
    }
    // unknown chars: dropped (no unk token), or the unk id, fused if fuse_unk
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
    unsigned long long* hp = L.heap + 3 * (size_t)sb;
    int hn = 0;
    for (int s = sb; s < se; ++s) {
      if (L.c[s] < 0 || L.nxt[s] < 0) continue;
      const long long m = mm_find(a.mm_keys, a.mm_vals, a.mm_log2cap, L.c[s], L.c[L.nxt[s]]);
      if (m >= 0)
        heap_push(hp, hn, ((unsigned long long)(m >> 16) << 32) | ((unsigned long long)(s - sb) << 16) |
                              (unsigned long long)(m & 0xFFFF));
    }
    while (hn > 0) {
      const unsigned long long top = heap_pop(hp, hn);
      const int pos = sb + (int)((top >> 16) & 0xFFFF);
      const int new_id = (int)(top & 0xFFFF);
      if (L.c[pos] < 0) continue;             // merged into its left neighbour
      const int nx = L.nxt[pos];
      if (nx < 0) continue;                   // last symbol
      const long long m = mm_find(a.mm_keys, a.mm_vals, a.mm_log2cap, L.c[pos], L.c[nx]);
      if (m < 0 || (int)(m & 0xFFFF) != new_id) continue;  // expired entry
      L.c[pos] = new_id;
      L.c[nx] = -1;
      const int nn = L.nxt[nx];
      L.nxt[pos] = (int16_t)nn;
      if (nn >= 0) L.prv[nn] = (int16_t)pos;
      const int pv = L.prv[pos];
      if (pv >= 0) {
        const long long mp = mm_find(a.mm_keys, a.mm_vals, a.mm_log2cap, L.c[pv], new_id);
        if (mp >= 0)
          heap_push(hp, hn, ((unsigned long long)(mp >> 16) << 32) | ((unsigned long long)(pv - sb) << 16) |
                                (unsigned long long)(mp & 0xFFFF));
      }
      if (nn >= 0) {
        const long long mn = mm_find(a.mm_keys, a.mm_vals, a.mm_log2cap, new_id, L.c[nn]);
        if (mn >= 0)
          heap_push(hp, hn, ((unsigned long long)(mn >> 16) << 32) | ((unsigned long long)(pos - sb) << 16) |
                                (unsigned long long)(mn & 0xFFFF));
      }
    }
    int cnt = 0;
    for (int s = sb; s < se; ++s) cnt += (L.c[s] >= 0);
    L.wcnt[w] = cnt;
  }
  __syncthreads();
  // 5. word offsets (wave scan), ids in order
  carry = 0;
  for (int base = 0; base < nw; base += ENC_T) {
    const int w = base + lane;
    const int v = (w < nw) ? L.wcnt[w] : 0;
    int x = v;
    for (int o = 1; o < ENC_T; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (w < nw) L.wcnt[w] = carry + x - v;
    carry += __shfl(x, ENC_T - 1);
  }
  __syncthreads();
  int32_t* out = a.out_ids + r * a.out_stride;
  for (int w = lane; w < nw; w += ENC_T) {
    const int sb = L.symoff[L.wcp[w]], se = L.symoff[L.wcp[w + 1]];
    int o = L.wcnt[w];
    for (int s = sb; s < se; ++s)
      if (L.c[s] >= 0) out[o++] = L.c[s];
  }
  if (lane == 0) { a.out_len[r] = carry; a.status[r] = ST_OK; }
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
  long long* out;             // [n_rows][L]
  int32_t* out_count;         // decoded code points per row
  int32_t* status;            // bit 0: the row holds the <unk> id; bit 1: an id < -1 (not a u32)
};

struct ByteStream {
  const int32_t* ids;
  int64_t ni, ti;    // id index, byte index within that id
  int32_t bo, be;    // current id's byte range
  const DecArgs* a;
  __device__ bool next_token() {
    while (ti < ni) {
      const int id = ids[ti++];
      if (id < 0 || id >= a->n_vocab || a->tok_skip[id]) continue;
      bo = a->tok_off[id];
      be = a->tok_off[id + 1];
      if (bo < be) return true;
    }
    return false;
  }
  __device__ int get() {  // next byte or -1
    if (bo >= be && !next_token()) return -1;
    return a->tok_bytes[bo++];
  }
};

__global__ __launch_bounds__(256) void k_bpe_decode(DecArgs a) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= a.n_rows) return;
  const int64_t i0 = a.row_off[r], i1 = a.row_off[r + 1];
  int unk = 0, ovf = 0;
  for (int64_t i = i0; i < i1; ++i) {
    const int id = a.ids[i];
    unk |= (a.unk_id >= 0 && id == a.unk_id);
    ovf |= (id < -1);
  }
  a.status[r] = unk | (ovf << 1);
  ByteStream bs{a.ids + i0, i1 - i0, 0, 0, 0, &a};
  int buf[4], nb = 0, cnt = 0;
  long long* out = a.out + r * (int64_t)a.L;
  while (true) {
    while (nb < 4) {
      const int b = bs.get();
      if (b < 0) break;
      buf[nb++] = b;
    }
    if (nb == 0) break;
    const int b0 = buf[0];
    int cp, used;
    auto at = [&](int k) { return k < nb ? buf[k] : 0; };   // Rust's safe_get: 0 past the end
    auto cont = [](int b) { return (b & 0xC0) == 0x80; };
    if (b0 < 0x80) { cp = b0; used = 1; }
    else if (b0 >= 0xC2 && b0 <= 0xDF) {
      if (cont(at(1))) { cp = ((b0 & 0x1F) << 6) | (at(1) & 0x3F); used = 2; }
      else { cp = 0xFFFD; used = 1; }
    } else if (b0 >= 0xE0 && b0 <= 0xEF) {
      const int b1 = at(1);
      const bool ok1 = (b0 == 0xE0) ? (b1 >= 0xA0 && b1 <= 0xBF) : (b0 == 0xED) ? (b1 >= 0x80 && b1 <= 0x9F)
                                                                                : (b1 >= 0x80 && b1 <= 0xBF);
      if (!ok1) { cp = 0xFFFD; used = 1; }
      else if (!cont(at(2))) { cp = 0xFFFD; used = 2; }
      else { cp = ((b0 & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (at(2) & 0x3F); used = 3; }
    } else if (b0 >= 0xF0 && b0 <= 0xF4) {
      const int b1 = at(1);
      const bool ok1 = (b0 == 0xF0) ? (b1 >= 0x90 && b1 <= 0xBF) : (b0 == 0xF4) ? (b1 >= 0x80 && b1 <= 0x8F)
                                                                                : (b1 >= 0x80 && b1 <= 0xBF);
      if (!ok1) { cp = 0xFFFD; used = 1; }
      else if (!cont(at(2))) { cp = 0xFFFD; used = 2; }
      else if (!cont(at(3))) { cp = 0xFFFD; used = 3; }
      else { cp = ((b0 & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((at(2) & 0x3F) << 6) | (at(3) & 0x3F); used = 4; }
    } else { cp = 0xFFFD; used = 1; }
    if (cnt < a.L) out[cnt] = (long long)cp + a.min_tok;
    ++cnt;
    for (int k = used; k < nb; ++k) buf[k - used] = buf[k];
    nb -= used;
  }
  a.out_count[r] = cnt;
}

inline int log2_ceil(int64_t x) {
  int l = 0;
  while ((int64_t(1) << l) < x) ++l;
  return l;
}

}  // namespace

extern "C" int beast_bpe_mergemap_log2cap(int n_merges) {
  const int l = log2_ceil(2 * (int64_t)(n_merges > 0 ? n_merges : 1));
  return l < 6 ? 6 : l;
}

extern "C" size_t beast_bpe_mergemap_bytes(int n_merges) {
  const size_t cap = size_t(1) << beast_bpe_mergemap_log2cap(n_merges);
  return cap * sizeof(unsigned long long) + cap * sizeof(uint32_t);
}

extern "C" int beast_bpe_mergemap_build(const int32_t* merge_a, const int32_t* merge_b, const int32_t* merge_new,
                                        int n_merges, void* map, size_t map_bytes, void* stream) {
  BEAST_REQUIRE(n_merges >= 0 && n_merges < (1 << 30), "n_merges out of range: %d", n_merges);
  BEAST_REQUIRE(map != nullptr, "mergemap buffer is null");
  BEAST_REQUIRE_CODE(map_bytes >= beast_bpe_mergemap_bytes(n_merges), BEAST_E_WORKSPACE,
                     "mergemap buffer too small: %zu < %zu", map_bytes, beast_bpe_mergemap_bytes(n_merges));
  BEAST_REQUIRE(n_merges == 0 || (merge_a && merge_b && merge_new), "merge arrays are null");
  const int lg = beast_bpe_mergemap_log2cap(n_merges);
  const int cap = 1 << lg;
  auto* vals = reinterpret_cast<unsigned long long*>(map);
  auto* keys = reinterpret_cast<uint32_t*>(vals + cap);
  hipStream_t s = beast::as_stream(stream);
  hipLaunchKernelGGL(k_mergemap_clear, dim3((cap + 255) / 256), dim3(256), 0, s, keys, vals, cap);
  BEAST_LAUNCHED("k_mergemap_clear");
  if (n_merges > 0) {
    hipLaunchKernelGGL(k_mergemap_build, dim3((n_merges + 255) / 256), dim3(256), 0, s, merge_a, merge_b, merge_new,
                       n_merges, keys, vals, lg);
    BEAST_LAUNCHED("k_mergemap_build");
  }
  return BEAST_OK;
}

extern "C" size_t beast_bpe_encode_lds_bytes(int max_row_cps, int max_row_syms) {
  return enc_lds_bytes(max_row_cps, max_row_syms);
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
  BEAST_REQUIRE(max_row_cps >= 0 && max_row_cps < 32768, "max_row_cps %d out of range", max_row_cps);
  BEAST_REQUIRE_CODE(max_row_syms >= 0 && max_row_syms <= 16384, BEAST_E_UNSUPPORTED,
                     "rows of %d byte symbols exceed the encoder's per-row LDS budget (16384)", max_row_syms);
  BEAST_REQUIRE(out_stride >= max_row_syms, "out_stride %lld < max_row_syms %d", (long long)out_stride, max_row_syms);
  BEAST_REQUIRE(n_spec >= 0 && n_spec <= MAX_SPECIAL, "at most %d special tokens are supported", MAX_SPECIAL);
  BEAST_REQUIRE(n_spec == 0 || (spec_cps && spec_len && spec_id), "special-token arrays are null");
  const size_t lds = enc_lds_bytes(max_row_cps, max_row_syms);
  BEAST_REQUIRE_CODE(lds <= 65536, BEAST_E_UNSUPPORTED,
                     "rows of %d code points / %d byte symbols need %zu B of LDS (> 64 KiB)", max_row_cps,
                     max_row_syms, lds);
  const int lg = beast_bpe_mergemap_log2cap(n_merges);
  const int cap = 1 << lg;
  EncArgs a;
  a.tok = reinterpret_cast<const long long*>(tok);
  a.row_off = row_off; a.n_rows = n_rows; a.min_tok = min_tok; a.max_span = max_span;
  a.lut = cls_lut; a.lut_n = (int)lut_n; a.byte2id = byte2id;
  a.mm_vals = reinterpret_cast<const unsigned long long*>(map);
  a.mm_keys = reinterpret_cast<const uint32_t*>(a.mm_vals + cap);
  a.mm_log2cap = lg;
  a.spec_cps = spec_cps; a.spec_len = spec_len; a.spec_id = spec_id; a.n_spec = n_spec;
  a.unk_id = unk_id; a.fuse_unk = fuse_unk;
  a.Lc = max_row_cps; a.S = max_row_syms;
  a.out_ids = out_ids; a.out_stride = out_stride; a.out_len = out_len; a.status = status;
  hipLaunchKernelGGL(k_bpe_encode, dim3((unsigned)n_rows), dim3(ENC_T), lds, beast::as_stream(stream), a);
  BEAST_LAUNCHED("k_bpe_encode");
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
  a.out = reinterpret_cast<long long*>(out); a.out_count = out_count; a.status = status;
  hipLaunchKernelGGL(k_bpe_decode, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, beast::as_stream(stream), a);
  BEAST_LAUNCHED("k_bpe_decode");
  return BEAST_OK;
}
