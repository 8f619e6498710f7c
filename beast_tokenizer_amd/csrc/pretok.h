// Shared by the BPE kernels that pre-tokenise rows (bpe_codec.hip: inference, bpe_setup.hip:
// training): the GPT-2 / ByteLevel regex evaluated from every code point at once and the
// lane-parallel walk of its word chain.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace beast_pt {

constexpr int CLS_OTHER = 0, CLS_LETTER = 1, CLS_NUMBER = 2, CLS_WS = 3;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

// Exclusive prefix sum over the wave (all 64 lanes active) by DPP: row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast:15 / row_bcast:31 carry the rows' totals -- no LDS round trip (a
// __shfl_up ladder is six ds_bpermute round trips).
__device__ __forceinline__ int wave_excl_scan(int v, int lane, int& total) {
  int x = v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
  total = __builtin_amdgcn_readlane(x, 63);
  (void)lane;
  return x - v;
}

// e[i] = regex_word(cps, cls, i, n) for every i, without the per-position class-run loops: the
// end of each class run comes from one ballot per 64 positions (run[p] = one past the last
// position of p's run; scratch [n]), so every lane's regex end is a few independent reads.
__device__ __forceinline__ void regex_ends(const int32_t* cps, const uint8_t* cls, int32_t* run, int32_t* e, int n,
                                           int lane) {
  int carry = n;   // one past the first run end in the chunks after the current one
  for (int base = (n - 1) & ~63; base >= 0; base -= 64) {
    const int p = base + lane;
    const bool in = p < n;
    const int c0 = in ? (int)cls[p] : -1;
    const int c1 = p + 1 < n ? (int)cls[p + 1] : -2;
    const unsigned long long m = __ballot(in && c0 != c1);   // p ends its run
    const unsigned long long rest = m >> lane;
    if (in) run[p] = rest ? p + __builtin_ctzll(rest) + 1 : carry;
    if (m) carry = base + __builtin_ctzll(m) + 1;
  }
  wave_sync();
  for (int i = lane; i < n; i += 64) {
    const int c = cps[i];
    const int c1 = i + 1 < n ? cps[i + 1] : -1, c2 = i + 2 < n ? cps[i + 2] : -1;
    const int k0 = cls[i], k1 = i + 1 < n ? (int)cls[i + 1] : CLS_WS;
    int j;
    if (c == '\'' && (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd')) {
      j = i + 2;
    } else if (c == '\'' && ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l'))) {
      j = i + 3;
    } else if (c == ' ' && i + 1 < n && k1 != CLS_WS) {
      j = run[i + 1];                      // " ?" + the run of the next code point's class
    } else if (k0 != CLS_WS) {
      j = run[i];
    } else {
      j = run[i];                          // \s+, giving back the last blank before a non-blank
      if (j < n && j - i >= 2) --j;
    }
    e[i] = j;
  }
  wave_sync();
}

// The word starts of a row from e[i], the end of the regex word that would
// start at code point i: the chain 0 -> e[0] -> e[e[0]] -> ... < n.  Lane-parallel instead of one
// lane following ~n / 2 dependent links: lane s walks the chain from the start of its segment
// [s G, s G + G) (G = ceil(n / 64)), marking what it visits (vis, one byte per code point), and
// records where it leaves the segment.  The true chain enters segment s where it left segment
// s - 1; a marked entry means lane s's walk already is the true chain from there (the chain is a
// function of the position), an entry past the segment means the segment holds no start, and
// any other entry (rare: regex words self-synchronise within a word) makes the lane re-walk its
// segment from it -- repeated until no exit changes.  Starts = marked positions at or past
// their segment's entry, written in order by a wave scan.
// Invariant: the marks in [ws, se) are exactly the positions of the lane's latest walk, which
// started at ws and leaves the segment at wex.  The exit passed on, ex, is wex when the entry lies
// on that walk, or the entry itself when the chain jumps the segment.  A marked entry below ws is
// a mark of an older walk (e.g. "x!'tion": the walk from "'" marks "t" before the chain is known
// to enter at "t"), so only a marked entry at or past ws reuses the walk; anything else re-walks.
__device__ __forceinline__ void word_starts(const int32_t* e, uint8_t* vis, int32_t* wcp, int32_t* wspec,
                                            int32_t* nw_out, int n, int lane) {
  const int G = (n + 63) >> 6;
  const int sb = min(lane * G, n), se = min(sb + G, n);
  for (int i = lane; i < n; i += 64) vis[i] = 0;
  wave_sync();
  int ex = sb;    // exit passed to the next lane: the first chain position >= se (n past the end)
  int ws = sb;    // start of the walk the marks in [ws, se) belong to
  int wex = sb;   // that walk's exit
  if (sb < se) {
    int p = sb;
    while (p < se) { vis[p] = 1; p = e[p]; }
    wex = ex = p;
  }
  int entry = 0;
  while (true) {
    const int prev = __shfl_up(ex, 1);
    const int en = lane == 0 ? 0 : prev;
    int nex = ex;
    bool changed = false;
    if (sb < se) {
      if (en >= se) {
        nex = en;                 // the chain jumps this segment
      } else if (en >= sb && en >= ws && vis[en]) {
        nex = wex;                // the entry lies on the latest walk
      } else if (en >= sb) {
        for (int i = en; i < se; ++i) vis[i] = 0;   // re-walk from the true entry
        int p = en;
        while (p < se) { vis[p] = 1; p = e[p]; }
        nex = wex = p;
        ws = en;
        changed = true;
      }
    } else {
      nex = en > sb ? en : sb;   // empty segment (past n): pass the exit on
    }
    changed |= nex != ex || en != entry;
    ex = nex;
    entry = en;
    if (!__any(changed)) break;
  }
  wave_sync();
  int cnt = 0;
  for (int i = max(sb, entry); i < se; ++i) cnt += vis[i];
  int tot;
  int o = wave_excl_scan(cnt, lane, tot);
  for (int i = max(sb, entry); i < se; ++i)
    if (vis[i]) {
      wcp[o] = i;
      if (wspec) wspec[o] = -1;
      ++o;
    }
  if (lane == 0) { wcp[tot] = n; *nw_out = tot; }
  wave_sync();
}

}  // namespace beast_pt
