// beast_bpe_train: the whole byte-level BPE training in one C-ABI call (host code over the
// library's own entry points) -- what FIGBPE.fit_from_sequences does through HF
// (beast/beast_bpe_trainer.py:61-74, :76-98: BpeTrainer(vocab_size, min_frequency,
// special_tokens, initial_alphabet = chr(0 .. max - min), max_token_length) on the strings
// "".join(map(chr, seq - min))).  The same steps as beast_tokenizer_amd/bpe_train.py:train_bpe
// on one GPU: min / max, the code points present, the alphabet (special tokens, then byte-level
// chars by code point), pre-tokenisation (count, scan, emit), distinct words x counts, the
// length-ordered repack + word signatures, the pair table, then the device-driven batched
// merge loop with two chunks of passes in flight, and the host replay of its merge log against
// the real strings.  Vt <= 4,096 runs the batched loop; larger vocabularies (Vt <= 32,768, the
// dense pair table) the host-driven one (one merge per host round trip, bpe_train.py's loop
// below the device loop), as does a rerun after a 64-bit string-hash collision or a full merge
// log of the batched loop.  beast_bpe_train_comm is the same over several GPUs with the library's communicator
// (comm.hip): bpe_train.py's replicated form -- the range and presence all-reduced, the shards'
// distinct words all-gathered once, the loop run on the union on every rank.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace {

// GPT-2 bytes_to_unicode: bytes 33-126, 161-172, 174-255 map to themselves, the other 68 to
// U+0100 + k in ascending byte order
void bytes_to_unicode(uint32_t (&b2u)[256]) {
  int k = 0;
  for (int b = 0; b < 256; ++b) {
    const bool keep = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || (b >= 174 && b <= 255);
    b2u[b] = keep ? (uint32_t)b : (uint32_t)(256 + k++);
  }
}

void append_utf8(std::string& s, uint32_t cp) {
  if (cp < 0x80) {
    s += (char)cp;
  } else if (cp < 0x800) {
    s += (char)(0xC0 | (cp >> 6));
    s += (char)(0x80 | (cp & 63));
  } else if (cp < 0x10000) {
    s += (char)(0xE0 | (cp >> 12));
    s += (char)(0x80 | ((cp >> 6) & 63));
    s += (char)(0x80 | (cp & 63));
  } else {
    s += (char)(0xF0 | (cp >> 18));
    s += (char)(0x80 | ((cp >> 12) & 63));
    s += (char)(0x80 | ((cp >> 6) & 63));
    s += (char)(0x80 | (cp & 63));
  }
}

size_t utf8_chars(const std::string& s) {   // HF counts token lengths in characters
  size_t n = 0;
  for (unsigned char c : s) n += (c & 0xC0) != 0x80;
  return n;
}

// device allocations released on every return path
struct DevMem {
  std::vector<void*> ptrs;
  ~DevMem() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <class T>
  T* get(size_t count) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
};

struct HostPinned {
  void* p = nullptr;
  ~HostPinned() {
    if (p) (void)hipHostFree(p);
  }
};

constexpr uint64_t LOOP_P = 0x9E3779B97F4A7C15ull;   // bpe_train.py GpuBpeOps.LOOP_P
constexpr int ST_ACTIVE = 0, ST_VCUR = 1, ST_NMERGES = 2;
constexpr int KMAX = 8, CHUNK = 64;

}  // namespace

#define TRY(call)                  \
  do {                             \
    const int rc_ = (call);        \
    if (rc_ != BEAST_OK) return rc_; \
  } while (0)
#define ALLOC(var, T, n)                                                         \
  T* var = mem.get<T>(n);                                                        \
  BEAST_REQUIRE_CODE(var != nullptr, BEAST_E_HIP, "beast_bpe_train: hipMalloc of %zu x %zu bytes failed", \
                     (size_t)(n), sizeof(T))
#define ALLOC_TO(var, T, n)                                                                                \
  do {                                                                                                     \
    var = mem.get<T>(n);                                                                                   \
    BEAST_REQUIRE_CODE(var != nullptr, BEAST_E_HIP, "beast_bpe_train: hipMalloc of %zu x %zu bytes failed", \
                       (size_t)(n), sizeof(T));                                                            \
  } while (0)
// Every rank of a communicator must issue the same collectives in the same order.  A local phase
// that fails on one rank therefore still reaches the agreement that ends it (the status all-reduced
// with MAX, beast::comm_agree), where every rank learns of the failure and returns it together --
// a rank returning alone would leave the others blocked in the next collective.  Without a
// communicator AGREE is TRY.
#define AGREE(...)   /* variadic: a lambda argument may hold commas */ \
  do {                                                              \
    const int a_ = beast::comm_agree(comm, (__VA_ARGS__), s);       \
    if (a_ != BEAST_OK) return a_;                                  \
  } while (0)

namespace {

// rank r's word starts index its own symbols: shift them by where its symbols land in the union
__global__ void k_offset_starts(uint32_t* __restrict__ w, int64_t n, uint32_t off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w[i] += off;
}

// this shard's words: pre-tokenisation (count, scan, emit), the distinct words x counts (the
// table grows 4x while it overflows) and their length-ordered repack
int shard_words(DevMem& mem, const int64_t* tokens, const int64_t* seq_off, int64_t n_seq, int64_t mn,
                const uint8_t* cls_lut, int64_t lut_n, const uint16_t* byte2id, uint16_t*& sym2, uint32_t*& w2,
                uint32_t*& l2, uint32_t*& c2, int64_t& nu, int64_t& nsp, hipStream_t s) {
  void* stream = s;
  ALLOC(wps, int64_t, n_seq);
  ALLOC(sps, int64_t, n_seq);
  TRY(beast_bpe_pretok_count(tokens, seq_off, n_seq, mn, cls_lut, lut_n, wps, sps, stream));
  ALLOC(scan_ws, uint8_t, beast_scan_workspace_bytes(n_seq));
  ALLOC(woff, int64_t, n_seq + 1);
  ALLOC(soff, int64_t, n_seq + 1);
  TRY(beast_exclusive_scan_i64(wps, woff, n_seq, scan_ws, stream));
  TRY(beast_exclusive_scan_i64(sps, soff, n_seq, scan_ws, stream));
  int64_t nw = 0, ns = 0;
  BEAST_HIP(hipMemcpyAsync(&nw, woff + n_seq, sizeof(int64_t), hipMemcpyDeviceToHost, s), "word count read");
  BEAST_HIP(hipMemcpyAsync(&ns, soff + n_seq, sizeof(int64_t), hipMemcpyDeviceToHost, s), "symbol count read");
  BEAST_HIP(hipStreamSynchronize(s), "stream sync");
  BEAST_REQUIRE_CODE(ns < (int64_t(1) << 32), BEAST_E_UNSUPPORTED,
                     "BPE corpus has >= 2^32 byte symbols on one GPU; shard it over more ranks");
  ALLOC(b2i_d, uint16_t, 256);
  BEAST_HIP(hipMemcpyAsync(b2i_d, byte2id, 256 * sizeof(uint16_t), hipMemcpyHostToDevice, s), "byte2id upload");
  ALLOC(sym, uint16_t, ns);
  ALLOC(wstart, uint32_t, nw);
  ALLOC(wlen, uint32_t, nw);
  TRY(beast_bpe_pretok_emit(tokens, seq_off, n_seq, mn, cls_lut, lut_n, woff, soff, b2i_d, sym, wstart, wlen, stream));
  ALLOC(ow, uint32_t, nw);
  ALLOC(ol, uint32_t, nw);
  ALLOC(oc, uint32_t, nw);
  ALLOC(on, int64_t, 1);
  nu = -1;
  for (size_t nbytes = beast_bpe_dedup_workspace_bytes(nw); nu < 0; nbytes *= 4) {
    void* dws = nullptr;
    BEAST_HIP(hipMalloc(&dws, nbytes), "dedup workspace");
    const int rc = beast_bpe_dedup_words(sym, wstart, wlen, nw, dws, nbytes, ow, ol, oc, on, stream);
    if (rc == BEAST_OK) {
      const hipError_t e1 = hipMemcpyAsync(&nu, on, sizeof(int64_t), hipMemcpyDeviceToHost, s);
      const hipError_t e2 = hipStreamSynchronize(s);
      (void)hipFree(dws);
      BEAST_HIP(e1, "distinct count read");
      BEAST_HIP(e2, "stream sync");
    } else {
      (void)hipFree(dws);
      return rc;
    }
  }
  ALLOC(rp_ws, uint8_t, beast_bpe_repack_workspace_bytes(nu));
  sym2 = mem.get<uint16_t>(ns + 3 * nu);   // spans rounded up to 4
  w2 = mem.get<uint32_t>(nu);
  l2 = mem.get<uint32_t>(nu);
  c2 = mem.get<uint32_t>(nu);
  BEAST_REQUIRE_CODE(sym2 && w2 && l2 && c2, BEAST_E_HIP, "beast_bpe_train: hipMalloc of the repacked words failed");
  TRY(beast_bpe_repack_words(sym, ow, ol, oc, nu, rp_ws, beast_bpe_repack_workspace_bytes(nu), sym2, w2, l2, c2, on,
                             stream));
  BEAST_HIP(hipMemcpyAsync(&nsp, on, sizeof(int64_t), hipMemcpyDeviceToHost, s), "symbol count read");
  BEAST_HIP(hipStreamSynchronize(s), "stream sync");
  return BEAST_OK;
}

// every rank's distinct words x counts on every rank, in rank order, repacked for the loop
// (bpe_train.py GpuBpeOps.gather_words): one all-gather of the sizes, then one all-gather-v per
// array.  A word repeated across shards appears once per shard with its shard count, which
// leaves every pair count (and so every merge) unchanged.
int union_words(DevMem& mem, beast_comm* comm, uint16_t*& sym2, uint32_t*& w2, uint32_t*& l2, uint32_t*& c2,
                int64_t& nu, int64_t& nsp, hipStream_t s) {
  void* stream = s;
  int world = 0, rank = 0;
  TRY(beast_comm_info(comm, &world, &rank, nullptr));
  int64_t* sz = nullptr;
  const int64_t mine[2] = {nu, nsp};
  AGREE([&]() -> int {
    ALLOC_TO(sz, int64_t, 2 + 2 * (size_t)world);
    BEAST_HIP(hipMemcpyAsync(sz, mine, sizeof(mine), hipMemcpyHostToDevice, s), "size upload");
    return BEAST_OK;
  }());
  TRY(beast_comm_allgather(comm, sz, sz + 2, 2, BEAST_DT_I64, stream));
  std::vector<int64_t> all(2 * (size_t)world);
  BEAST_HIP(hipMemcpyAsync(all.data(), sz + 2, sizeof(int64_t) * all.size(), hipMemcpyDeviceToHost, s), "size read");
  BEAST_HIP(hipStreamSynchronize(s), "stream sync");
  std::vector<int64_t> wc(world), wd(world), bc(world), bd(world);   // words; symbol bytes
  int64_t NU = 0, NS = 0;
  for (int r = 0; r < world; ++r) {
    wc[r] = all[2 * r];
    wd[r] = NU;
    bc[r] = 2 * all[2 * r + 1];
    bd[r] = 2 * NS;
    NU += all[2 * r];
    NS += all[2 * r + 1];
  }
  // the sizes are every rank's alike: so is this check's outcome
  BEAST_REQUIRE_CODE(NS + 3 * NU < (int64_t(1) << 32), BEAST_E_UNSUPPORTED,
                     "beast_bpe_train: the shards' distinct words hold >= 2^32 symbols; the replicated loop keeps them on "
                     "every GPU");
  if (NU == 0) {
    sym2 = nullptr;
    nu = nsp = 0;
    return BEAST_OK;
  }
  uint16_t* gsym = nullptr;
  uint32_t *gw = nullptr, *gl = nullptr, *gc = nullptr;
  AGREE([&]() -> int {
    ALLOC_TO(gsym, uint16_t, NS);
    ALLOC_TO(gw, uint32_t, NU);
    ALLOC_TO(gl, uint32_t, NU);
    ALLOC_TO(gc, uint32_t, NU);
    return BEAST_OK;
  }());
  TRY(beast_comm_allgatherv(comm, sym2, gsym, bc.data(), bd.data(), BEAST_DT_U8, stream));
  TRY(beast_comm_allgatherv(comm, w2, gw, wc.data(), wd.data(), BEAST_DT_U32, stream));
  TRY(beast_comm_allgatherv(comm, l2, gl, wc.data(), wd.data(), BEAST_DT_U32, stream));
  TRY(beast_comm_allgatherv(comm, c2, gc, wc.data(), wd.data(), BEAST_DT_U32, stream));
  // local from here on: the caller agrees before its next collective
  for (int r = 0; r < world; ++r)
    if (wc[r] > 0 && bd[r] > 0) {
      hipLaunchKernelGGL(k_offset_starts, dim3((unsigned)((wc[r] + 255) / 256)), dim3(256), 0, s, gw + wd[r], wc[r],
                         (uint32_t)(bd[r] / 2));
      BEAST_LAUNCHED("k_offset_starts");
    }
  const size_t rp_bytes = beast_bpe_repack_workspace_bytes(NU);
  ALLOC(rp_ws, uint8_t, rp_bytes);
  ALLOC(on, int64_t, 1);
  sym2 = mem.get<uint16_t>(NS + 3 * NU);   // spans rounded up to 4
  w2 = mem.get<uint32_t>(NU);
  l2 = mem.get<uint32_t>(NU);
  c2 = mem.get<uint32_t>(NU);
  BEAST_REQUIRE_CODE(sym2 && w2 && l2 && c2, BEAST_E_HIP, "beast_bpe_train: hipMalloc of the union's words failed");
  TRY(beast_bpe_repack_words(gsym, gw, gl, gc, NU, rp_ws, rp_bytes, sym2, w2, l2, c2, on, stream));
  BEAST_HIP(hipMemcpyAsync(&nsp, on, sizeof(int64_t), hipMemcpyDeviceToHost, s), "symbol count read");
  BEAST_HIP(hipStreamSynchronize(s), "stream sync");
  nu = NU;
  return BEAST_OK;
}

}  // namespace

namespace beast {
int g_bpe_train_host = 0;
}

// the batched loop asks for the host-driven one (a 64-bit string-hash collision, or a full merge
// log): bpe_train_impl returns RERUN after releasing every device buffer of the attempt, and the
// entry points train again with host_loop set -- the peak memory stays one training's
constexpr int RERUN = 1;

static int bpe_train_impl(const int64_t* tokens, const int64_t* seq_off, int64_t n_seq, const uint8_t* cls_lut,
                          int64_t lut_n, int vocab_size, int min_frequency, int max_token_length,
                          const char* const* special_tokens, int n_special, int64_t* out_min_token,
                          int64_t* out_max_token, char* out_vocab_bytes, size_t vocab_bytes_cap,
                          int64_t* out_vocab_off, int max_vocab, int* out_n_vocab, int32_t* out_merges,
                          int max_merges_out, int* out_n_merges, beast_comm* comm, bool replicate,
                          bool host_loop, void* stream) {
  hipStream_t s = beast::as_stream(stream);
  DevMem mem;
  // ---- arguments, this shard's token count
  int64_t n_tok = 0;
  int64_t* red = nullptr;
  AGREE([&]() -> int {
    BEAST_REQUIRE(seq_off && cls_lut && out_min_token && out_max_token && out_vocab_bytes && out_vocab_off &&
                      out_n_vocab && out_merges && out_n_merges && (n_special == 0 || special_tokens),
                  "beast_bpe_train: null pointer argument");
    // with a communicator a rank may hold no sequences at all (its shard of the corpus is empty;
    // the total is checked below); alone, the reference's "no non-empty sequences" rule applies
    BEAST_REQUIRE(n_seq >= (comm != nullptr ? 0 : 1) && vocab_size >= 1 && n_special >= 0, "beast_bpe_train: bad sizes");
    BEAST_HIP(hipMemcpyAsync(&n_tok, seq_off + n_seq, sizeof(int64_t), hipMemcpyDeviceToHost, s), "seq_off read");
    BEAST_HIP(hipStreamSynchronize(s), "stream sync");
    BEAST_REQUIRE(n_tok >= 0 && (n_tok == 0 || tokens != nullptr), "beast_bpe_train: null pointer argument");
    ALLOC_TO(red, int64_t, 2);
    return BEAST_OK;
  }());
  // with a communicator: the shards' token count, range and code points are the corpus's
  if (comm != nullptr) {
    BEAST_HIP(hipMemcpyAsync(red, &n_tok, sizeof(int64_t), hipMemcpyHostToDevice, s), "token count upload");
    TRY(beast_comm_allreduce(comm, red, red, 1, BEAST_DT_I64, BEAST_OP_SUM, stream));
    int64_t total = 0;
    BEAST_HIP(hipMemcpyAsync(&total, red, sizeof(int64_t), hipMemcpyDeviceToHost, s), "token count read");
    BEAST_HIP(hipStreamSynchronize(s), "stream sync");
    BEAST_REQUIRE(total > 0, "No non-empty sequences provided for BPE training.");   // reference :84-85
  } else {
    BEAST_REQUIRE(n_tok > 0, "No non-empty sequences provided for BPE training.");   // reference :84-85
  }

  // ---- min / max (reference :86-87), the code points present
  constexpr int64_t NONE = int64_t(1) << 62;   // an empty shard's (min, -max)
  int64_t mmh[2] = {NONE, -NONE};
  AGREE([&]() -> int {
    if (n_tok > 0) {
      ALLOC(mm, int64_t, 2);
      TRY(beast_i64_minmax(tokens, n_tok, mm, stream));
      BEAST_HIP(hipMemcpyAsync(mmh, mm, sizeof(mmh), hipMemcpyDeviceToHost, s), "minmax read");
      BEAST_HIP(hipStreamSynchronize(s), "stream sync");
    }
    return BEAST_OK;
  }());
  if (comm != nullptr) {   // one MIN over (min, -max)
    int64_t lo_nhi[2] = {mmh[0], -mmh[1]};
    BEAST_HIP(hipMemcpyAsync(red, lo_nhi, sizeof(lo_nhi), hipMemcpyHostToDevice, s), "range upload");
    TRY(beast_comm_allreduce(comm, red, red, 2, BEAST_DT_I64, BEAST_OP_MIN, stream));
    BEAST_HIP(hipMemcpyAsync(lo_nhi, red, sizeof(lo_nhi), hipMemcpyDeviceToHost, s), "range read");
    BEAST_HIP(hipStreamSynchronize(s), "stream sync");
    mmh[0] = lo_nhi[0];
    mmh[1] = -lo_nhi[1];
  }
  const int64_t mn = mmh[0], mx = mmh[1], K = mx - mn;
  const int64_t n_cp = K + 1;
  uint8_t* pr = nullptr;
  AGREE([&]() -> int {
    BEAST_REQUIRE_CODE(K < 0xD800, BEAST_E_UNSUPPORTED,
                       "BPE alphabet reaches the UTF-16 surrogate range (max - min token >= 55296)");
    BEAST_REQUIRE(lut_n >= K + 1, "beast_bpe_train: class LUT covers %lld code points, the corpus needs %lld",
                  (long long)lut_n, (long long)(K + 1));
    ALLOC_TO(pr, uint8_t, n_cp);
    if (n_tok > 0) {
      TRY(beast_bpe_cp_presence(tokens, n_tok, mn, pr, n_cp, stream));
    } else {
      BEAST_HIP(hipMemsetAsync(pr, 0, n_cp, s), "presence memset");
    }
    return BEAST_OK;
  }());
  if (comm != nullptr) TRY(beast_comm_allreduce(comm, pr, pr, n_cp, BEAST_DT_U8, BEAST_OP_MAX, stream));
  std::vector<uint8_t> present(n_cp);
  BEAST_HIP(hipMemcpyAsync(present.data(), pr, n_cp, hipMemcpyDeviceToHost, s), "presence read");
  BEAST_HIP(hipStreamSynchronize(s), "stream sync");

  // ---- alphabet (HF BpeTrainer: special tokens, then compute_alphabet by code point)
  uint32_t b2u[256];
  bytes_to_unicode(b2u);
  bool seen[256] = {};
  for (int64_t cp = 0; cp < n_cp; ++cp)
    if (present[cp]) {
      std::string u;
      append_utf8(u, (uint32_t)cp);
      for (unsigned char c : u) seen[c] = true;
    }
  std::vector<uint32_t> chars;
  for (int b = 0; b < 256; ++b)
    if (seen[b]) chars.push_back(b2u[b]);
  for (int64_t cp = 0; cp < n_cp; ++cp) chars.push_back((uint32_t)cp);   // initial_alphabet = chr(0 .. K)
  std::sort(chars.begin(), chars.end());
  chars.erase(std::unique(chars.begin(), chars.end()), chars.end());
  std::vector<std::string> id2str;
  std::unordered_map<std::string, int> str2id;
  for (int i = 0; i < n_special; ++i) {
    const std::string t(special_tokens[i]);
    if (!str2id.count(t)) {
      str2id.emplace(t, (int)id2str.size());
      id2str.push_back(t);
    }
  }
  for (uint32_t c : chars) {
    std::string u;
    append_utf8(u, c);
    if (!str2id.count(u)) {
      str2id.emplace(u, (int)id2str.size());
      id2str.push_back(u);
    }
  }
  uint16_t byte2id[256];
  for (int b = 0; b < 256; ++b) {
    std::string u;
    append_utf8(u, b2u[b]);
    byte2id[b] = seen[b] ? (uint16_t)str2id.at(u) : (uint16_t)0xFFFF;
  }
  const int n_base = (int)id2str.size();
  const int Vt = std::max(vocab_size, n_base);

  // ---- this shard's distinct words x counts, length-ordered (sym2 / w2 / l2 / c2, nu words,
  // nsp padded symbols), then with a communicator the union of every rank's
  uint16_t* sym2 = nullptr;
  uint32_t *w2 = nullptr, *l2 = nullptr, *c2 = nullptr;
  int64_t nu = 0, nsp = 0;
  AGREE([&]() -> int {
    BEAST_REQUIRE_CODE(Vt <= 32768, BEAST_E_UNSUPPORTED, "beast_bpe_train: Vt %d > 32768 (the dense pair table)", Vt);
    if (max_vocab < Vt || max_merges_out < std::max(vocab_size - n_base, 0)) {
      // the sizes a retry needs (upper bounds until the training has run)
      *out_n_vocab = Vt;
      *out_n_merges = std::max(vocab_size - n_base, 0);
      BEAST_REQUIRE_CODE(false, BEAST_E_WORKSPACE,
                         "beast_bpe_train: output capacity (vocab %d, merges %d) below the vocabulary size %d; the "
                         "required sizes are in *out_n_vocab, *out_n_merges",
                         max_vocab, max_merges_out, Vt);
    }
    if (n_tok > 0) TRY(shard_words(mem, tokens, seq_off, n_seq, mn, cls_lut, lut_n, byte2id, sym2, w2, l2, c2, nu, nsp, s));
    return BEAST_OK;
  }());
  const bool sharded = comm != nullptr && !replicate;   // every rank keeps its shard of the words
  if (comm != nullptr && replicate) TRY(union_words(mem, comm, sym2, w2, l2, c2, nu, nsp, s));

  // ---- the pair table and the loop state
  uint64_t* sig = nullptr;
  uint32_t* table = nullptr;
  AGREE([&]() -> int {
    if (sym2 == nullptr) {   // no words anywhere: an empty table, the loop stops at once
      ALLOC(z16, uint16_t, 4);
      ALLOC(z32, uint32_t, 3);
      BEAST_HIP(hipMemsetAsync(z16, 0, 8, s), "empty words");
      BEAST_HIP(hipMemsetAsync(z32, 0, 12, s), "empty words");
      sym2 = z16, w2 = z32, l2 = z32 + 1, c2 = z32 + 2;
    }
    ALLOC_TO(sig, uint64_t, nu);
    if (nu > 0) TRY(beast_bpe_word_signatures(sym2, w2, l2, nu, sig, stream));
    ALLOC_TO(table, uint32_t, (size_t)Vt * Vt);
    BEAST_HIP(hipMemsetAsync(table, 0, sizeof(uint32_t) * (size_t)Vt * Vt, s), "pair table memset");
    TRY(beast_bpe_count_pairs(sym2, w2, l2, c2, nu, table, Vt, n_base, stream));
    return BEAST_OK;
  }());
  if (sharded) TRY(beast_comm_allreduce(comm, table, table, (int64_t)Vt * Vt, BEAST_DT_U32, BEAST_OP_SUM, stream));
  std::vector<uint64_t> hp(2 * (size_t)n_base);   // [0, n): string hash, [n, 2n): P^bytes
  std::vector<uint32_t> tlen(Vt, 0u);
  int max_tlen = 0;
  for (int i = 0; i < n_base; ++i) {
    uint64_t h = 0, pw = 1;
    for (unsigned char c : id2str[i]) {
      h = h * LOOP_P + c;
      pw *= LOOP_P;
    }
    hp[i] = h;
    hp[n_base + i] = pw;
    tlen[i] = (uint32_t)utf8_chars(id2str[i]);
    max_tlen = std::max(max_tlen, (int)tlen[i]);
  }
  const int max_len = max_token_length > 0 ? max_token_length : 0x7FFFFFFF;
  std::vector<int32_t> log;
  int n_log = 0;
  if (host_loop || Vt > 4096 || beast::g_bpe_train_host == 1) {
    // ---- host-driven loop (bpe_train.py train_bpe below the device loop): argmax, merge in
    // every word, apply + next argmax; one host read of the decided pair per merge
    uint64_t* hp_d = nullptr;
    uint32_t* tlen_d = nullptr;
    uint64_t* argws = nullptr;
    int32_t* deltas = nullptr;
    HostPinned kh;
    uint64_t key = 0;
    int call = 0;
    auto read_key = [&](int k, uint64_t& out) -> int {
      uint64_t* key_h = static_cast<uint64_t*>(kh.p);
      BEAST_HIP(hipMemcpyAsync(key_h, argws + 2 + (k & 1), sizeof(uint64_t), hipMemcpyDeviceToHost, s), "argmax read");
      BEAST_HIP(hipStreamSynchronize(s), "stream sync");
      out = *key_h;
      return BEAST_OK;
    };
    AGREE([&]() -> int {
      ALLOC_TO(hp_d, uint64_t, hp.size());
      ALLOC_TO(tlen_d, uint32_t, Vt);
      BEAST_HIP(hipMemcpyAsync(hp_d, hp.data(), sizeof(uint64_t) * hp.size(), hipMemcpyHostToDevice, s), "hash upload");
      BEAST_HIP(hipMemcpyAsync(tlen_d, tlen.data(), sizeof(uint32_t) * Vt, hipMemcpyHostToDevice, s), "tlen upload");
      const size_t aw_bytes = beast_bpe_argmax_workspace_bytes(Vt);
      ALLOC_TO(argws, uint64_t, (aw_bytes + 7) / 8);
      BEAST_HIP(hipMemsetAsync(argws, 0, ((aw_bytes + 7) / 8) * 8, s), "argmax workspace memset");
      ALLOC_TO(deltas, int32_t, 4 * (size_t)Vt);
      BEAST_HIP(hipMemsetAsync(deltas, 0, sizeof(int32_t) * 4 * (size_t)Vt, s), "deltas memset");
      BEAST_HIP(hipHostMalloc(&kh.p, 64, hipHostMallocDefault), "pinned key");
      TRY(beast_bpe_argmax(table, Vt, n_base, argws, call, stream));
      TRY(read_key(call++, key));
      return BEAST_OK;
    }());
    std::vector<std::string> ids = id2str;
    std::unordered_map<std::string, int> ix = str2id;
    int lrc = BEAST_OK;   // sharded: a failure is agreed at the top of the next merge, before its collective
    while (true) {
      AGREE(lrc);
      if ((int)ids.size() >= vocab_size) break;
      const uint64_t count = key >> 32;
      if (count < 1 || count < (uint64_t)std::max(min_frequency, 0)) break;
      const uint32_t idx = 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFu);
      const int a = (int)(idx / (uint32_t)Vt), b = (int)(idx % (uint32_t)Vt);
      BEAST_REQUIRE_CODE(a < (int)ids.size() && b < (int)ids.size(), BEAST_E_HIP,
                         "beast_bpe_train: argmax returned pair (%d, %d) outside the vocabulary", a, b);
      std::string t = ids[a] + ids[b];
      auto it = ix.find(t);
      const bool reused = it != ix.end();
      const int nid = reused ? it->second : (int)ids.size();
      if (!reused) {
        ix.emplace(t, nid);
        ids.push_back(std::move(t));
      }
      log.insert(log.end(), {a, b, nid, reused ? 1 : 0});
      ++n_log;
      lrc = beast_bpe_merge(sym2, w2, l2, c2, nu, a, b, nid, tlen_d, max_len, deltas, Vt, sig, (int64_t)count, stream);
      if (sharded) TRY(beast_comm_allreduce(comm, deltas, deltas, 4 * (int64_t)Vt, BEAST_DT_I32, BEAST_OP_SUM, stream));
      const int k = call++;
      if (lrc == BEAST_OK)
        lrc = beast_bpe_apply_argmax(table, deltas, Vt, (int)ids.size(), a, b, nid, tlen_d, argws, k, stream);
      if (lrc == BEAST_OK && (int)ids.size() < vocab_size) lrc = read_key(k, key);   // the last merge: no search
    }
    BEAST_HIP(hipStreamSynchronize(s), "stream sync");
  } else {
    const int max_merges = 4 * std::max(vocab_size - n_base, 0) + 1024;
    const size_t lws_bytes = beast_bpe_loop_workspace_bytes(Vt, max_merges);
    const size_t aw_bytes = beast_bpe_argmax_workspace_bytes(Vt);
    const size_t bw_bytes = beast_bpe_batch_workspace_bytes(Vt);
    const size_t nbd = beast_bpe_batch_delta_count(Vt);
    uint64_t* hp_d = nullptr;
    uint32_t* tlen_d = nullptr;
    uint8_t *lws = nullptr, *bws = nullptr;
    uint64_t* argws = nullptr;
    int32_t* bdeltas = nullptr;   // sharded: each pass's pair-count changes, summed over the ranks
    const void* st_p = nullptr;
    const void* log_p = nullptr;
    HostPinned stage;
    AGREE([&]() -> int {
      ALLOC_TO(hp_d, uint64_t, hp.size());
      ALLOC_TO(tlen_d, uint32_t, Vt);
      BEAST_HIP(hipMemcpyAsync(hp_d, hp.data(), sizeof(uint64_t) * hp.size(), hipMemcpyHostToDevice, s), "hash upload");
      BEAST_HIP(hipMemcpyAsync(tlen_d, tlen.data(), sizeof(uint32_t) * Vt, hipMemcpyHostToDevice, s), "tlen upload");
      ALLOC_TO(lws, uint8_t, lws_bytes);
      TRY(beast_bpe_loop_init(lws, lws_bytes, Vt, max_merges, n_base, vocab_size, min_frequency, hp_d, hp_d + n_base,
                              tlen_d, max_tlen, stream));
      TRY(beast_bpe_loop_state(lws, Vt, max_merges, &st_p, &log_p));
      ALLOC_TO(argws, uint64_t, (aw_bytes + 7) / 8);
      BEAST_HIP(hipMemsetAsync(argws, 0, ((aw_bytes + 7) / 8) * 8, s), "argmax workspace memset");
      ALLOC_TO(bws, uint8_t, bw_bytes);
      if (sharded) {
        ALLOC_TO(bdeltas, int32_t, nbd);
        BEAST_HIP(hipMemsetAsync(bdeltas, 0, sizeof(int32_t) * nbd, s), "pass deltas memset");
      }
      BEAST_HIP(hipHostMalloc(&stage.p, 2 * 64, hipHostMallocDefault), "pinned state");
      return BEAST_OK;
    }());
    auto run = [&](int steps, int flags) {
      return beast_bpe_loop_batch(lws, Vt, max_merges, steps, KMAX, flags, sym2, w2, l2, c2, nu, tlen_d, max_len, sig,
                                  table, argws, bws, bw_bytes, vocab_size, bdeltas, nullptr, stream);
    };

    // ---- the loop: two chunks of passes in flight, the host reads the state the older one left
    int32_t* st_host = static_cast<int32_t*>(stage.p);
    struct Inflight { hipEvent_t ev; int slot; int passes; };
    std::vector<Inflight> inflight;
    auto release = [&]() {
      for (auto& f : inflight) (void)hipEventDestroy(f.ev);
      inflight.clear();
    };
    auto launch = [&](int steps, int flags) -> int {
      if (int rc = run(steps, flags)) return rc;
      const int slot = inflight.empty() ? 0 : 1 - inflight.back().slot;
      if (hipMemcpyAsync(st_host + 16 * slot, st_p, 64, hipMemcpyDeviceToHost, s) != hipSuccess)
        return beast::hip_fail(hipGetLastError(), "loop state copy");
      hipEvent_t ev;
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return beast::hip_fail(hipGetLastError(), "event");
      (void)hipEventRecord(ev, s);
      inflight.push_back({ev, slot, steps});
      return BEAST_OK;
    };
    int vcur = n_base, rc = BEAST_OK;
    if (sharded) {
      // every rank holds the same table and takes the same decisions, so every rank runs the same
      // passes and collectives: merge on the shard, SUM of the pass's deltas, apply (bpe_train.py).
      // A launch that fails on one rank still joins every collective of its chunk; the chunk's end
      // agrees on the status before anyone reads the state.
      rc = run(0, 1 /* BATCH_INIT */);
      while (true) {
        const int steps = std::max(1, std::min(CHUNK, (vocab_size - vcur + 1) / 2));
        for (int i = 0; i < steps; ++i) {
          if (rc == BEAST_OK) rc = run(1, BEAST_BPE_BATCH_NO_APPLY);
          TRY(beast_comm_allreduce(comm, bdeltas, bdeltas, (int64_t)nbd, BEAST_DT_I32, BEAST_OP_SUM, stream));
          if (rc == BEAST_OK) rc = run(1, BEAST_BPE_BATCH_NO_MERGE);
        }
        AGREE(rc);
        int32_t st[16];
        BEAST_HIP(hipMemcpyAsync(st, st_p, sizeof(st), hipMemcpyDeviceToHost, s), "loop state read");
        BEAST_HIP(hipStreamSynchronize(s), "stream sync");
        vcur = st[ST_VCUR];
        if (!st[ST_ACTIVE] || vcur >= vocab_size) break;
      }
    }
    if (!sharded) rc = launch(std::max(1, std::min(CHUNK, (vocab_size - vcur + KMAX - 1) / KMAX)), 1 /* BATCH_INIT */);
    while (!sharded && rc == BEAST_OK) {
      int queued = 0;
      for (auto& f : inflight) queued += f.passes;
      const int left = vocab_size - vcur - 4 * queued;
      if (left > 0 && (rc = launch(std::min(CHUNK, (left + KMAX - 1) / KMAX), 0)) != BEAST_OK) break;
      Inflight f = inflight.front();
      inflight.erase(inflight.begin());
      const hipError_t e = hipEventSynchronize(f.ev);
      (void)hipEventDestroy(f.ev);
      if (e != hipSuccess) { rc = beast::hip_fail(e, "loop event"); break; }
      const int32_t* h = st_host + 16 * f.slot;
      const int active = h[ST_ACTIVE];
      vcur = h[ST_VCUR];
      if (!active || vcur >= vocab_size) break;
      if (inflight.empty() && (rc = launch(1, 0)) != BEAST_OK) break;
    }
    release();
    // the rerun decision below is a collective point too (replicated ranks ran the loop alone)
    AGREE([&]() -> int {
      if (rc != BEAST_OK) return rc;
      int32_t state[16];
      BEAST_HIP(hipMemcpyAsync(state, st_p, sizeof(state), hipMemcpyDeviceToHost, s), "loop state read");
      BEAST_HIP(hipStreamSynchronize(s), "stream sync");
      n_log = state[ST_NMERGES];
      if (n_log < max_merges) {
        log.resize(4 * (size_t)std::max(n_log, 1));
        if (n_log > 0) {
          BEAST_HIP(hipMemcpyAsync(log.data(), log_p, sizeof(int32_t) * 4 * n_log, hipMemcpyDeviceToHost, s), "log read");
          BEAST_HIP(hipStreamSynchronize(s), "stream sync");
        }
      }
      return BEAST_OK;
    }());
  }

  // ---- replay the log against the real strings (bpe_train.py replay_log); a disagreement of the
  // batched loop's log (a 64-bit string-hash collision) or its full log reruns on the host-driven
  // loop -- every rank together
  int n_merges = 0;
  std::vector<int32_t> merge_ids;
  bool rerun = !host_loop && (n_log >= 4 * std::max(vocab_size - n_base, 0) + 1024 || beast::g_bpe_train_host == 2);
  for (int i = 0; i < n_log && !rerun; ++i) {
    const int a = log[4 * i], b = log[4 * i + 1], nid = log[4 * i + 2], reused = log[4 * i + 3];
    BEAST_REQUIRE_CODE(a >= 0 && b >= 0 && a < (int)id2str.size() && b < (int)id2str.size(), BEAST_E_UNSUPPORTED,
                       "beast_bpe_train: merge log entry %d out of range", i);
    const std::string t = id2str[a] + id2str[b];
    auto it = str2id.find(t);
    const bool have = it != str2id.end();
    const bool agree = have == (reused != 0) && (!have || it->second == nid) && (have || nid == (int)id2str.size());
    if (!host_loop && !agree) {
      rerun = true;
      break;
    }
    BEAST_REQUIRE_CODE(agree, BEAST_E_HIP, "beast_bpe_train: merge %d disagrees with the strings", i);
    if (!have) {
      str2id.emplace(t, nid);
      id2str.push_back(t);
    }
    merge_ids.push_back(a);
    merge_ids.push_back(b);
    ++n_merges;
  }
  if (!host_loop) {
    int any = rerun ? 1 : 0;
    TRY(beast::comm_max_i32(comm, any, &any, s));
    if (any) return RERUN;
  }

  // ---- outputs: the vocabulary's strings in id order, the merges, the token range.  Capacities
  // are checked against the finished training: when one is short, the required sizes come back
  // (*out_n_vocab, *out_n_merges, out_vocab_off[0] = vocabulary bytes) with BEAST_E_WORKSPACE
  size_t need_bytes = 0;
  for (const std::string& t : id2str) need_bytes += t.size();
  if ((int)id2str.size() > max_vocab || n_merges > max_merges_out || need_bytes > vocab_bytes_cap) {
    *out_n_vocab = (int)id2str.size();
    *out_n_merges = n_merges;
    out_vocab_off[0] = (int64_t)need_bytes;
    BEAST_REQUIRE_CODE(false, BEAST_E_WORKSPACE,
                       "beast_bpe_train: output capacity (vocab %d, merges %d, bytes %zu) below the result's (%zu, %d, "
                       "%zu); the required sizes are in *out_n_vocab, *out_n_merges, out_vocab_off[0]",
                       max_vocab, max_merges_out, vocab_bytes_cap, id2str.size(), n_merges, need_bytes);
  }
  std::memcpy(out_merges, merge_ids.data(), merge_ids.size() * sizeof(int32_t));
  size_t off = 0;
  for (size_t i = 0; i < id2str.size(); ++i) {
    out_vocab_off[i] = (int64_t)off;
    std::memcpy(out_vocab_bytes + off, id2str[i].data(), id2str[i].size());
    off += id2str[i].size();
  }
  out_vocab_off[id2str.size()] = (int64_t)off;
  *out_n_vocab = (int)id2str.size();
  *out_n_merges = n_merges;
  *out_min_token = mn;
  *out_max_token = mx;
  return BEAST_OK;
}

// the batched attempt, then (RERUN) the host-driven one with the first attempt's memory released
static int bpe_train_entry(const int64_t* tokens, const int64_t* seq_off, int64_t n_seq, const uint8_t* cls_lut,
                           int64_t lut_n, int vocab_size, int min_frequency, int max_token_length,
                           const char* const* special_tokens, int n_special, int64_t* out_min_token,
                           int64_t* out_max_token, char* out_vocab_bytes, size_t vocab_bytes_cap,
                           int64_t* out_vocab_off, int max_vocab, int* out_n_vocab, int32_t* out_merges,
                           int max_merges_out, int* out_n_merges, beast_comm* comm, bool replicate, void* stream) {
  int rc = RERUN;
  for (int attempt = 0; attempt < 2 && rc == RERUN; ++attempt)
    rc = bpe_train_impl(tokens, seq_off, n_seq, cls_lut, lut_n, vocab_size, min_frequency, max_token_length,
                        special_tokens, n_special, out_min_token, out_max_token, out_vocab_bytes, vocab_bytes_cap,
                        out_vocab_off, max_vocab, out_n_vocab, out_merges, max_merges_out, out_n_merges, comm,
                        replicate, attempt == 1, stream);
  return rc;
}

extern "C" int beast_bpe_train(const int64_t* tokens, const int64_t* seq_off, int64_t n_seq, const uint8_t* cls_lut,
                               int64_t lut_n, int vocab_size, int min_frequency, int max_token_length,
                               const char* const* special_tokens, int n_special, int64_t* out_min_token,
                               int64_t* out_max_token, char* out_vocab_bytes, size_t vocab_bytes_cap,
                               int64_t* out_vocab_off, int max_vocab, int* out_n_vocab, int32_t* out_merges,
                               int max_merges_out, int* out_n_merges, void* stream) {
  return bpe_train_entry(tokens, seq_off, n_seq, cls_lut, lut_n, vocab_size, min_frequency, max_token_length,
                         special_tokens, n_special, out_min_token, out_max_token, out_vocab_bytes, vocab_bytes_cap,
                         out_vocab_off, max_vocab, out_n_vocab, out_merges, max_merges_out, out_n_merges, nullptr, true,
                         stream);
}

extern "C" int beast_bpe_train_comm(const int64_t* tokens, const int64_t* seq_off, int64_t n_seq,
                                    const uint8_t* cls_lut, int64_t lut_n, int vocab_size, int min_frequency,
                                    int max_token_length, const char* const* special_tokens, int n_special,
                                    int64_t* out_min_token, int64_t* out_max_token, char* out_vocab_bytes,
                                    size_t vocab_bytes_cap, int64_t* out_vocab_off, int max_vocab, int* out_n_vocab,
                                    int32_t* out_merges, int max_merges_out, int* out_n_merges, beast_comm* comm,
                                    int replicate, void* stream) {
  return bpe_train_entry(tokens, seq_off, n_seq, cls_lut, lut_n, vocab_size, min_frequency, max_token_length,
                         special_tokens, n_special, out_min_token, out_max_token, out_vocab_bytes, vocab_bytes_cap,
                         out_vocab_off, max_vocab, out_n_vocab, out_merges, max_merges_out, out_n_merges, comm,
                         replicate != 0, stream);
}
