// Exact per-column quantiles (fit_parameters' np.quantile(params, q, axis=0),
// beast/beast_bspline_tokenizer.py:211-214) by radix select on gfx950.
//
// 1. k_keys      transpose x[rows][cols] (row-major params) into order-preserving
//                uint32 keys [cols][rows] through a [KT_R][33] LDS tile (coalesced both ways)
// 2. k_hist      per pass (digits of 11, 11, 10 bits from the top, or 11, 7, 7, 7 -- the
//                radix the caller picks) and per target rank: LDS-privatised histograms
//                of the keys whose higher bits equal the target's prefix, flushed with
//                u32 atomics into a target-major [target][column][bins] array.
//                Multi-GPU: the caller all-reduces the pass's live slice of it between
//                hist and select (pass 0: target 0 only, every target shares the empty
//                prefix); every rank then selects the same bucket.  With ranks the 7-bit
//                digits keep the later slices small (1.15 MB, then 3 x 0.29 MB for 140
//                columns x 4 targets, against 3 x 9.2 MB of u64 [column][target] histograms
//                before) for one extra key pass; one GPU takes 11 bits (three passes).
// 3. k_select    one thread per (column, target): walk the histogram to the bucket
//                holding the remaining rank, extend the prefix.
// 4. k_finalize  numpy's float32 _lerp between ranks floor(vi) and floor(vi)+1.
// HBM traffic: rows*cols*4 (read x) + (1 + passes)*rows*cols*4 (write keys, 3 or 4 key passes).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "common.h"

namespace {

constexpr int MAXQ = 4;
constexpr int MAXTG = 2 * MAXQ;
constexpr int NBIN = 2048;   // bins of the widest digit (11 bits)
constexpr int HIST_THREADS = 256;
constexpr int64_t HIST_CHUNK = 32768;  // keys per workgroup per pass

struct QState {          // per (column, target)
  uint32_t prefix;       // selected high bits so far
  uint32_t pad;
  uint64_t rank;         // remaining rank inside the prefix bucket
};

struct QHeader {
  int64_t n_total;
  int32_t n_q, n_tg;
  int64_t ranks[MAXTG];
  float gamma[MAXQ];
};

struct WsLayout {
  size_t hdr, state, nan, hist, keys, total;
};

inline size_t al(size_t x) { return (x + 255) & ~size_t(255); }

inline WsLayout ws_layout(int64_t rows, int cols, int n_q) {
  WsLayout w;
  const int ntg = 2 * n_q;
  size_t o = 0;
  w.hdr = o;   o += al(sizeof(QHeader));
  w.state = o; o += al(sizeof(QState) * (size_t)cols * ntg);
  w.nan = o;   o += al(sizeof(uint32_t) * (size_t)cols);
  w.hist = o;  o += al(sizeof(uint32_t) * (size_t)cols * ntg * NBIN);
  w.keys = o;  o += al(sizeof(uint32_t) * (size_t)cols * (size_t)rows);
  w.total = o;
  return w;
}

__device__ __forceinline__ uint32_t f2key(float f) {
  if (f != f) return 0xFFFFFFFFu;  // every NaN sorts last (numpy sort order)
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(u);
}

// digits from the most significant end: radix 11 -> 11 + 11 + 10 bits, radix 7 -> 11 + 7 + 7 + 7
// (the first digit is 11 bits either way: its last bucket holds exactly the NaN keys)
__host__ __device__ inline int n_passes(int radix) { return radix == 11 ? 3 : 4; }
__host__ __device__ inline int hist_stride(int pass, int radix) { return (radix == 11 || pass == 0) ? NBIN : 128; }
__host__ __device__ inline void pass_geom(int pass, int radix, int& shift, int& bits) {
  if (radix == 11) {
    shift = (pass == 0) ? 21 : (pass == 1) ? 10 : 0;
    bits = (pass == 2) ? 10 : 11;
  } else {
    shift = (pass == 0) ? 21 : 21 - 7 * pass;
    bits = (pass == 0) ? 11 : 7;
  }
}

// A workgroup moves a KT_R x 32 tile (16 KiB in, 16 KiB out; 16 loads in flight per thread):
// a 32 x 32 tile kept too few bytes in flight per CU to cover HBM latency (3.2 TB/s at K4).
constexpr int KT_R = 128;
__device__ __forceinline__ void keys_tile(const float* __restrict__ src, int64_t stride, int nr, int c0, int cols,
                                          uint32_t* __restrict__ dst, int64_t rows) {
  __shared__ uint32_t tile[KT_R][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  const int c = c0 + tx;
  float v[KT_R / 8];
#pragma unroll
  for (int i = 0; i < KT_R / 8; ++i) {
    const int k = ty + 8 * i;
    v[i] = (k < nr && c < cols) ? src[(int64_t)k * stride + c] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < KT_R / 8; ++i) tile[ty + 8 * i][tx] = f2key(v[i]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cc = c0 + ty + 8 * j;
    if (cc >= cols) continue;
#pragma unroll
    for (int i = 0; i < KT_R / 32; ++i) {
      const int r = tx + 32 * i;
      if (r < nr) dst[(int64_t)cc * rows + r] = tile[r][ty + 8 * j];
    }
  }
}

__global__ __launch_bounds__(256) void k_keys(const float* __restrict__ x, int64_t rows, int cols, int64_t rs,
                                              uint32_t* __restrict__ keys) {
  const int64_t r0 = (int64_t)blockIdx.x * KT_R;
  const int nr = (int)min<int64_t>(KT_R, rows - r0);
  keys_tile(x + r0 * rs, rs, nr, blockIdx.y * 32, cols, keys + r0, rows);
}

// The same transpose over a list of row-major segments (fit_parameters' per-batch params,
// no torch.cat): seg[i] = {ptr, first row, row stride}, rows of segment i are
// [seg[i].first, seg[i + 1].first) of the concatenated space.  Grid x = nseg * tiles_per_seg
// KT_R-row tiles (tiles past a segment's end exit), so no tile straddles two segments.
struct QSeg {
  const float* ptr;
  int64_t first;
  int64_t stride;
};

__global__ __launch_bounds__(256) void k_keys_seg(const QSeg* __restrict__ seg, int nseg, int tiles_per_seg,
                                                  int64_t rows, int cols, uint32_t* __restrict__ keys) {
  const int si = blockIdx.x / tiles_per_seg;
  const int64_t t0 = (int64_t)(blockIdx.x % tiles_per_seg) * KT_R;
  const QSeg sg = seg[si];
  const int64_t seg_rows = ((si + 1 < nseg) ? seg[si + 1].first : rows) - sg.first;
  if (t0 >= seg_rows) return;   // workgroup-uniform: before the tile's barrier
  const int nr = (int)min<int64_t>(KT_R, seg_rows - t0);
  keys_tile(sg.ptr + t0 * sg.stride, sg.stride, nr, blockIdx.y * 32, cols, keys + sg.first + t0, rows);
}

__global__ void k_init(QState* __restrict__ st, uint32_t* __restrict__ nanf, QHeader* __restrict__ hdr, int cols,
                       QHeader h) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *hdr = h;
  if (i < cols * h.n_tg) {
    st[i].prefix = 0;
    st[i].pad = 0;
    st[i].rank = (uint64_t)h.ranks[i % h.n_tg];
  }
  if (i < cols) nanf[i] = 0;
}

// grid (chunks, cols).  Keys are read 16 B per lane; every thread keeps a run-length counter
// (bin, count) per histogram and only flushes it to the LDS histogram when the bin changes:
// parameter columns are narrow, so the top digits of most keys fall into a handful of bins,
// and one LDS atomic per key would serialise on them.
// LDS histograms hold 16-bit counts, two bins per word (a chunk has <= 32768 keys, so a bin
// never carries into its neighbour): 4 KiB per histogram keeps 8 workgroups per CU resident.
static_assert(HIST_CHUNK < 65536, "16-bit LDS bins");
__device__ __forceinline__ void bin_add(uint32_t* h, uint32_t bin, uint32_t cnt) {
  atomicAdd(&h[bin >> 1], cnt << ((bin & 1u) * 16));
}

__device__ __forceinline__ void run_add(uint32_t* h, uint32_t& bin, uint32_t& cnt, uint32_t b) {
  if (b == bin) { ++cnt; return; }
  if (cnt) bin_add(h, bin, cnt);
  bin = b;
  cnt = 1;
}

__global__ __launch_bounds__(HIST_THREADS) void k_hist(const uint32_t* __restrict__ keys, int64_t rows, int ntg,
                                                       int pass, int radix, const QState* __restrict__ st,
                                                       uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t h_raw[];   // [nh][nb / 2] packed 16-bit bins
  const int c = blockIdx.y, cols = gridDim.y;
  int shift, bits;
  pass_geom(pass, radix, shift, bits);
  const int nb = hist_stride(pass, radix), nb2 = nb / 2;
  auto h = [&](int t) { return h_raw + t * nb2; };
  const uint32_t mask = (1u << bits) - 1u;
  const int hi_shift = shift + bits;  // bits above the digit are known
  // targets that need their own histogram (pass 0: one shared histogram)
  const int nh = (pass == 0) ? 1 : ntg;
  uint32_t pref[MAXTG], rbin[MAXTG], rcnt[MAXTG];
  for (int t = 0; t < MAXTG; ++t) {
    pref[t] = (t < nh && hi_shift < 32) ? (st[c * ntg + t].prefix >> hi_shift) : 0u;
    rbin[t] = 0;
    rcnt[t] = 0;
  }
  for (int i = threadIdx.x; i < nh * nb2; i += HIST_THREADS) h_raw[i] = 0;
  __syncthreads();
  const uint32_t* kc = keys + (int64_t)c * rows;
  const int64_t chunk = HIST_CHUNK;
  const int64_t i0 = (int64_t)blockIdx.x * chunk;
  const int64_t i1 = min<int64_t>(rows, i0 + chunk);
  auto add = [&](uint32_t k) {
    const uint32_t dg = (k >> shift) & mask;
    if (pass == 0) {
      run_add(h(0), rbin[0], rcnt[0], dg);
    } else {
      const uint32_t hk = k >> hi_shift;
#pragma unroll
      for (int t = 0; t < MAXTG; ++t)
        if (t < nh && hk == pref[t]) run_add(h(t), rbin[t], rcnt[t], dg);
    }
  };
  // column c's keys start at c * rows: 16-B aligned only if rows % 4 == 0 -> scalar head
  const int64_t a0 = min<int64_t>(i1, (i0 + (int64_t)((4 - ((c * rows + i0) & 3)) & 3)));
  for (int64_t i = i0 + threadIdx.x; i < a0; i += HIST_THREADS) add(kc[i]);
  const int64_t nv = (i1 - a0) / 4;
  const uint4* kv = reinterpret_cast<const uint4*>(kc + a0);
  constexpr int UNR = 4;   // 64 B per lane in flight
  int64_t v = threadIdx.x;
  for (; v + (UNR - 1) * HIST_THREADS < nv; v += UNR * HIST_THREADS) {
    uint4 q[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) q[u] = kv[v + u * HIST_THREADS];
#pragma unroll
    for (int u = 0; u < UNR; ++u) { add(q[u].x); add(q[u].y); add(q[u].z); add(q[u].w); }
  }
  for (; v < nv; v += HIST_THREADS) {
    const uint4 q = kv[v];
    add(q.x); add(q.y); add(q.z); add(q.w);
  }
  for (int64_t i = a0 + 4 * nv + threadIdx.x; i < i1; i += HIST_THREADS) add(kc[i]);
#pragma unroll
  for (int t = 0; t < MAXTG; ++t)
    if (rcnt[t]) bin_add(h(t), rbin[t], rcnt[t]);
  __syncthreads();
  for (int i = threadIdx.x; i < nh * nb2; i += HIST_THREADS) {
    const uint32_t v = h_raw[i];
    const int t = i / nb2, b = 2 * (i - t * nb2);
    uint32_t* hc = hist + ((int64_t)t * cols + c) * nb;   // target-major: pass 0's live slice is contiguous
    if (v & 0xFFFFu) atomicAdd(hc + b, v & 0xFFFFu);
    if (v >> 16) atomicAdd(hc + b + 1, v >> 16);
  }
}

// One workgroup per (column, target): 256 threads x 8 bins, block-wide exclusive scan,
// the thread whose bins hold the remaining rank extends the prefix.
constexpr int SEL_T = 256;
__global__ __launch_bounds__(SEL_T) void k_select(QState* __restrict__ st, uint32_t* __restrict__ nanf,
                                                  const uint32_t* __restrict__ hist, int ntg, int pass, int radix,
                                                  int cols) {
  __shared__ uint64_t wsum[SEL_T / 64];
  const int i = blockIdx.x;  // (column, target)
  const int c = i / ntg, t = i % ntg;
  int shift, bits;
  pass_geom(pass, radix, shift, bits);
  const int nbins = 1 << bits;
  const uint32_t* h = hist + ((int64_t)(pass == 0 ? 0 : t) * cols + c) * hist_stride(pass, radix);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int PER = NBIN / SEL_T;  // 8
  uint64_t v[PER], sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int b = tid * PER + k;
    v[k] = (b < nbins) ? h[b] : 0;
    sum += v[k];
  }
  // inclusive scan of per-thread sums across the block
  uint64_t x = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint64_t off = 0;
  for (int k = 0; k < w; ++k) off += wsum[k];
  const uint64_t before = off + x - sum;  // exclusive prefix of this thread's first bin
  const uint64_t r = st[i].rank;
  if (r >= before && r < before + sum) {
    uint64_t cum = before;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (r < cum + v[k]) {
        st[i].prefix |= (uint32_t)(tid * PER + k) << shift;
        st[i].rank = r - cum;
        break;
      }
      cum += v[k];
    }
  }
  // the last bucket of pass 0 (11 bits) holds the NaN keys (0xFFFFFFFF) and no number's key
  if (pass == 0 && t == 0 && tid == SEL_T - 1 && v[PER - 1] != 0) nanf[c] = 1;
}

// numpy _lerp in float32 (lib/_function_base_impl.py): a + d*g, or b - d*(1-g) when g >= 0.5
__global__ void k_finalize(const QState* __restrict__ st, const uint32_t* __restrict__ nanf, int cols,
                           const QHeader* __restrict__ hp, float* __restrict__ out) {
  const QHeader& h = *hp;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cols * h.n_q) return;
  const int q = i / cols, c = i % cols;
  const float a = key2f(st[c * h.n_tg + 2 * q].prefix);
  const float b = key2f(st[c * h.n_tg + 2 * q + 1].prefix);
  const float g = h.gamma[q];
  const float d = __fsub_rn(b, a);
  float r;
  if (g >= 0.5f) r = __fsub_rn(b, __fmul_rn(d, __fsub_rn(1.0f, g)));
  else r = __fadd_rn(a, __fmul_rn(d, g));
  if (nanf[c]) r = __builtin_nanf("");
  out[q * cols + c] = r;
}

// host-side replica of numpy 2.x quantile index math in float32 (see oracle.quantile_ranks)
void numpy_ranks(int64_t n, float q, int64_t& lo, int64_t& hi, float& gamma) {
  const float vi = (float)(n - 1) * q;  // Python int weakly promoted to float32
  if (vi >= (float)(n - 1)) { lo = hi = n - 1; gamma = 0.0f; return; }
  if (vi < 0.0f) { lo = hi = 0; gamma = 0.0f; return; }
  const double fl = std::floor((double)vi);
  lo = (int64_t)fl;
  hi = lo + 1;
  gamma = (float)((double)vi - fl);
}

}  // namespace

extern "C" size_t beast_quantile_workspace_bytes(int64_t rows, int cols, int n_q) {
  return ws_layout(rows, cols, n_q).total;
}

extern "C" uint32_t* beast_quantile_hist_ptr(void* workspace, int cols, int n_q) {
  const WsLayout w = ws_layout(0, cols, n_q);
  return reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(workspace) + w.hist);
}

extern "C" int beast_quantile_passes(int radix_bits) { return radix_bits == 11 ? 3 : radix_bits == 7 ? 4 : 0; }

extern "C" int64_t beast_quantile_hist_count(int pass, int cols, int n_q, int radix_bits) {
  return (int64_t)(pass == 0 ? 1 : 2 * n_q) * cols * hist_stride(pass, radix_bits);
}

extern "C" int beast_quantile_prepare(const float* x, int64_t rows, int cols, int64_t row_stride, int64_t n_total,
                                      int n_q, const float* host_q, void* workspace, size_t ws_bytes, void* stream) {
  BEAST_REQUIRE(workspace && host_q, "beast_quantile_prepare: null pointer");
  BEAST_REQUIRE(n_q >= 1 && n_q <= MAXQ, "n_q must be in [1, %d]", MAXQ);
  BEAST_REQUIRE(cols >= 1 && rows >= 0 && n_total >= 1 && rows <= n_total, "bad quantile shape rows=%lld n=%lld",
                (long long)rows, (long long)n_total);
  BEAST_REQUIRE(rows == 0 || x, "beast_quantile_prepare: null x");
  BEAST_REQUIRE(rows < (int64_t(1) << 31), "rows per rank must be < 2^31");
  BEAST_REQUIRE(n_total < (int64_t(1) << 32), "n_total must be < 2^32 (uint32 histogram counts)");
  const WsLayout w = ws_layout(rows, cols, n_q);
  BEAST_REQUIRE_CODE(ws_bytes >= w.total, BEAST_E_WORKSPACE, "quantile workspace %zu < %zu", ws_bytes, w.total);
  QHeader h;
  std::memset(&h, 0, sizeof(h));
  h.n_total = n_total;
  h.n_q = n_q;
  h.n_tg = 2 * n_q;
  for (int q = 0; q < n_q; ++q) {
    BEAST_REQUIRE(host_q[q] >= 0.0f && host_q[q] <= 1.0f, "Quantiles must be in the range [0, 1]");
    int64_t lo, hi;
    float g;
    numpy_ranks(n_total, host_q[q], lo, hi, g);
    h.ranks[2 * q] = lo;
    h.ranks[2 * q + 1] = hi;
    h.gamma[q] = g;
  }
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  hipStream_t s = beast::as_stream(stream);
  auto* st = reinterpret_cast<QState*>(ws + w.state);
  auto* nanf = reinterpret_cast<uint32_t*>(ws + w.nan);
  const int ninit = cols * h.n_tg;
  hipLaunchKernelGGL(k_init, dim3((ninit + 255) / 256), dim3(256), 0, s, st, nanf,
                     reinterpret_cast<QHeader*>(ws + w.hdr), cols, h);
  BEAST_LAUNCHED("k_init");
  if (rows > 0) {
    dim3 grid((unsigned)((rows + KT_R - 1) / KT_R), (unsigned)((cols + 31) / 32));
    hipLaunchKernelGGL(k_keys, grid, dim3(256), 0, s, x, rows, cols, row_stride,
                       reinterpret_cast<uint32_t*>(ws + w.keys));
    BEAST_LAUNCHED("k_keys");
  }
  return BEAST_OK;
}

extern "C" int beast_quantile_prepare_segments(const void* seg_table, int nseg, int64_t max_seg_rows, int64_t rows,
                                               int cols, int64_t n_total, int n_q, const float* host_q,
                                               void* workspace, size_t ws_bytes, void* stream) {
  BEAST_REQUIRE(nseg >= 1 && seg_table, "beast_quantile_prepare_segments: need >= 1 segment");
  const int64_t tps = (max_seg_rows + KT_R - 1) / KT_R;
  BEAST_REQUIRE(max_seg_rows >= 0 && tps * nseg < (int64_t(1) << 31), "beast_quantile_prepare_segments: "
                "%d segments of up to %lld rows are too many tiles", nseg, (long long)max_seg_rows);
  // header, state and ranks as for one matrix; x is only dereferenced by k_keys
  int rc = beast_quantile_prepare(nullptr, 0, cols, cols, n_total, n_q, host_q, workspace, ws_bytes, stream);
  if (rc) return rc;
  BEAST_REQUIRE(rows >= 0 && rows <= n_total && rows < (int64_t(1) << 31), "bad segment rows %lld",
                (long long)rows);
  const WsLayout w = ws_layout(rows, cols, n_q);
  BEAST_REQUIRE_CODE(ws_bytes >= w.total, BEAST_E_WORKSPACE, "quantile workspace %zu < %zu", ws_bytes, w.total);
  if (rows > 0 && tps > 0) {
    dim3 grid((unsigned)(tps * nseg), (unsigned)((cols + 31) / 32));
    hipLaunchKernelGGL(k_keys_seg, grid, dim3(256), 0, beast::as_stream(stream), static_cast<const QSeg*>(seg_table),
                       nseg, (int)tps, rows, cols,
                       reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(workspace) + w.keys));
    BEAST_LAUNCHED("k_keys_seg");
  }
  return BEAST_OK;
}

extern "C" int beast_quantile_hist(int pass, int64_t rows, int cols, int n_q, int radix_bits, void* workspace,
                                   void* stream) {
  BEAST_REQUIRE(radix_bits == 11 || radix_bits == 7, "beast_quantile_hist: radix_bits must be 11 or 7");
  BEAST_REQUIRE(workspace && pass >= 0 && pass < n_passes(radix_bits) && n_q >= 1 && n_q <= MAXQ,
                "beast_quantile_hist: bad args");
  const WsLayout w = ws_layout(rows, cols, n_q);
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  hipStream_t s = beast::as_stream(stream);
  const int ntg = 2 * n_q;
  BEAST_HIP(hipMemsetAsync(ws + w.hist, 0, sizeof(uint32_t) * beast_quantile_hist_count(pass, cols, n_q, radix_bits),
                           s), "hist memset");
  if (rows > 0) {
    const int64_t chunk = HIST_CHUNK;
    dim3 grid((unsigned)((rows + chunk - 1) / chunk), (unsigned)cols);
    const size_t lds = sizeof(uint32_t) * (hist_stride(pass, radix_bits) / 2) * (pass == 0 ? 1 : ntg);
    hipLaunchKernelGGL(k_hist, grid, dim3(HIST_THREADS), lds, s, reinterpret_cast<const uint32_t*>(ws + w.keys), rows,
                       ntg, pass, radix_bits, reinterpret_cast<const QState*>(ws + w.state),
                       reinterpret_cast<uint32_t*>(ws + w.hist));
    BEAST_LAUNCHED("k_hist");
  }
  return BEAST_OK;
}

extern "C" int beast_quantile_select(int pass, int cols, int n_q, int radix_bits, void* workspace, void* stream) {
  BEAST_REQUIRE(radix_bits == 11 || radix_bits == 7, "beast_quantile_select: radix_bits must be 11 or 7");
  BEAST_REQUIRE(workspace && pass >= 0 && pass < n_passes(radix_bits) && n_q >= 1 && n_q <= MAXQ,
                "beast_quantile_select: bad args");
  const WsLayout w = ws_layout(0, cols, n_q);
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  const int n = cols * 2 * n_q;
  hipLaunchKernelGGL(k_select, dim3(n), dim3(SEL_T), 0, beast::as_stream(stream),
                     reinterpret_cast<QState*>(ws + w.state), reinterpret_cast<uint32_t*>(ws + w.nan),
                     reinterpret_cast<const uint32_t*>(ws + w.hist), 2 * n_q, pass, radix_bits, cols);
  BEAST_LAUNCHED("k_select");
  return BEAST_OK;
}

extern "C" int beast_quantile_finalize(int cols, int n_q, void* workspace, float* out, void* stream) {
  BEAST_REQUIRE(workspace && out && n_q >= 1 && n_q <= MAXQ, "beast_quantile_finalize: bad args");
  const WsLayout w = ws_layout(0, cols, n_q);
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  const int n = cols * n_q;
  hipLaunchKernelGGL(k_finalize, dim3((n + 127) / 128), dim3(128), 0, beast::as_stream(stream),
                     reinterpret_cast<const QState*>(ws + w.state), reinterpret_cast<const uint32_t*>(ws + w.nan),
                     cols, reinterpret_cast<const QHeader*>(ws + w.hdr), out);
  BEAST_LAUNCHED("k_finalize");
  return BEAST_OK;
}

extern "C" int beast_quantile_f32(const float* x, int64_t rows, int cols, int64_t row_stride, int n_q,
                                  const float* host_q, float* out, void* workspace, size_t ws_bytes, void* stream) {
  BEAST_REQUIRE(rows >= 1, "np.quantile of an empty array is undefined (rows=0)");
  int rc = beast_quantile_prepare(x, rows, cols, row_stride, rows, n_q, host_q, workspace, ws_bytes, stream);
  for (int p = 0; rc == BEAST_OK && p < n_passes(11); ++p) {
    rc = beast_quantile_hist(p, rows, cols, n_q, 11, workspace, stream);
    if (rc == BEAST_OK) rc = beast_quantile_select(p, cols, n_q, 11, workspace, stream);
  }
  if (rc == BEAST_OK) rc = beast_quantile_finalize(cols, n_q, workspace, out, stream);
  return rc;
}
