// CPU oracle of the BPE merge loop -- TEST INFRASTRUCTURE ONLY.
// Restates HF tokenizers' BpeTrainer::do_train (word-level merge with HF's
// pair-count changes, lazy max-heap with stale-entry check, ties -> smallest
// (id_a, id_b), merged pair retired, new-token id reused when the concatenated
// string already exists).  Token identity = its sequence of alphabet ids.
// Built by oracle/Makefile into oracle/build/libbpe_oracle.so; driven by
// oracle/bpe_oracle.py.  Pinned against HF outputs in tests/golden/bpe_hf.json.
#include <algorithm>
#include <cstdint>
#include <map>
#include <queue>
#include <unordered_map>
#include <vector>

namespace {
inline uint64_t key(int a, int b) { return (uint64_t(uint32_t(a)) << 32) | uint32_t(b); }
}

extern "C" int bpe_oracle_train(const int32_t* flat, const int64_t* lens, const int64_t* cnt, int64_t nw, int n0,
                                int vocab_size, int64_t min_freq, int32_t* out_a, int32_t* out_b, int32_t* out_n,
                                int64_t cap) {
  std::vector<std::vector<int>> words(nw);
  int64_t o = 0;
  for (int64_t w = 0; w < nw; ++w) {
    words[w].assign(flat + o, flat + o + lens[w]);
    o += lens[w];
  }
  std::vector<std::vector<int>> comp(n0);
  std::map<std::vector<int>, int> comp2id;
  for (int i = 0; i < n0; ++i) { comp[i] = {i}; comp2id[comp[i]] = i; }
  std::unordered_map<uint64_t, int64_t> pc;
  std::unordered_map<uint64_t, std::vector<int64_t>> where;
  for (int64_t w = 0; w < nw; ++w)
    for (size_t i = 0; i + 1 < words[w].size(); ++i) {
      const uint64_t k = key(words[w][i], words[w][i + 1]);
      pc[k] += cnt[w];
      auto& v = where[k];
      if (v.empty() || v.back() != w) v.push_back(w);
    }
  // max-heap on (count, smallest pair first)
  typedef std::pair<int64_t, uint64_t> E;  // (count, ~key)
  std::priority_queue<E> heap;
  for (auto& kv : pc) if (kv.second > 0) heap.push(E(kv.second, ~kv.first));
  int vocab = n0, nm = 0;
  while (vocab < vocab_size && !heap.empty()) {
    E top = heap.top();
    heap.pop();
    const uint64_t k = ~top.second;
    const int64_t cur = pc[k];
    if (top.first != cur) {
      if (cur > 0) heap.push(E(cur, top.second));
      continue;
    }
    if (top.first < 1 || top.first < min_freq) break;
    const int a = int(k >> 32), b = int(k & 0xFFFFFFFFu);
    std::vector<int> c = comp[a];
    c.insert(c.end(), comp[b].begin(), comp[b].end());
    int nid;
    auto it = comp2id.find(c);
    if (it == comp2id.end()) {
      nid = int(comp.size());
      comp.push_back(c);
      comp2id[c] = nid;
      ++vocab;
    } else {
      nid = it->second;
    }
    if (nm >= cap) return -1;  // caller retries with a larger buffer
    out_a[nm] = a; out_b[nm] = b; out_n[nm] = nid; ++nm;
    std::vector<int64_t> ws = where[k];
    std::sort(ws.begin(), ws.end());
    ws.erase(std::unique(ws.begin(), ws.end()), ws.end());
    std::vector<uint64_t> grown;
    for (int64_t w : ws) {
      std::vector<int>& s = words[w];
      const int64_t n = cnt[w];
      for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == a && i + 1 < s.size() && s[i + 1] == b) {
          if (i > 0) {
            pc[key(s[i - 1], a)] -= n;
            const uint64_t g = key(s[i - 1], nid);
            pc[g] += n; grown.push_back(g); where[g].push_back(w);
          }
          s[i] = nid;
          s.erase(s.begin() + i + 1);
          if (i + 1 < s.size()) {
            pc[key(b, s[i + 1])] -= n;
            const uint64_t g = key(nid, s[i + 1]);
            pc[g] += n; grown.push_back(g); where[g].push_back(w);
          }
        }
      }
    }
    pc[k] = 0;
    std::sort(grown.begin(), grown.end());
    grown.erase(std::unique(grown.begin(), grown.end()), grown.end());
    for (uint64_t g : grown) if (pc[g] > 0) heap.push(E(pc[g], ~g));
  }
  return nm;
}
