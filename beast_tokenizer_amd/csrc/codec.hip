// Fused BEAST encode / reconstruct kernels for gfx950.
//
//   k_encode       params = P . y on v_mfma_f32_16x16x4_f32 (P = fp32 rounding of the fp64
//                  ridge projection), fused with the clamp /
//                  quantise / (d n)->(n d) / LLM-offset epilogue (reference
//                  beast/beast_bspline_tokenizer.py:399-428, mp/uni_bspline.py:539-586)
//   k_reconstruct  dequantise + init_p + Phi . W on v_mfma_f32_16x16x4_f32 + scatter
//                  to the joint / gripper columns (reference :483-536, uni_bspline.py:114-177)
//
// Layout.  A workgroup (4 waves) walks tiles of TB consecutive trajectories (grid-stride,
// constants staged once per workgroup).  A tile's trajectories, params, tokens and
// positions are each contiguous in HBM, so every tile moves through LDS with 16-byte
// loads / stores; all of a thread's global loads of a stage are issued before its
// first LDS store (one HBM round trip per stage).  The MFMA column index enumerates
// (trajectory, DoF) pairs grouped by basis kind, so one 16-column tile never mixes the
// joint and gripper projections; the last tile of a kind may be partial (masked).
// Every operand the MFMA loops read is zero-padded in LDS (P to [16][Tp], Phi to
// [16*RT][Np], W to [Np]) so the loops are branch-free.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int NTHREADS = 256;
constexpr int NWAVES = NTHREADS / 64;
constexpr int MAX_T = 256;
constexpr int MAX_N = 16;
constexpr int MAX_D = 64;
constexpr int ECH = 4;    // encode: K-steps per LDS-operand chunk

typedef double double4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int round_up(int x, int m) { return (x + m - 1) / m * m; }

// x / d for x * d < 2^32 by multiply-high (d uniform, m = ceil(2^32 / d)).
struct FastDiv {
  uint32_t d, m;
};
inline FastDiv make_fd(uint32_t d) {
  FastDiv f;
  f.d = d;
  f.m = d <= 1 ? 0u : (uint32_t)((0x100000000ull + d - 1) / d);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t x, FastDiv f) { return f.d <= 1 ? x : __umulhi(x, f.m); }

// ------------------------------------------------------------- staging --
template <int MAXK>
__device__ __forceinline__ void burst16(uint4* __restrict__ dst, const uint4* __restrict__ src, int n16) {
  for (int base = 0; base < n16; base += MAXK * NTHREADS) {
    uint4 r[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) r[k] = src[min(base + k * NTHREADS + (int)threadIdx.x, n16 - 1)];
    // unconditional stores: a lane past the end rewrites element n16-1 with its own value,
    // so the compiler cannot sink the loads into per-element branches (one round trip)
#pragma unroll
    for (int k = 0; k < MAXK; ++k) dst[min(base + k * NTHREADS + (int)threadIdx.x, n16 - 1)] = r[k];
  }
}

template <int MAXK>
__device__ __forceinline__ void burst4(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int n) {
  for (int base = 0; base < n; base += MAXK * NTHREADS) {
    uint32_t r[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) r[k] = src[min(base + k * NTHREADS + (int)threadIdx.x, n - 1)];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) dst[min(base + k * NTHREADS + (int)threadIdx.x, n - 1)] = r[k];
  }
}

// global -> LDS, bytes % 4 == 0; 16-byte path when both ends are 16-byte aligned
template <int MAXK>
__device__ __forceinline__ void burst(void* __restrict__ dst, const void* __restrict__ src, int bytes) {
  if (bytes <= 0) return;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int n16 = bytes >> 4;
    if (n16) burst16<MAXK>(reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), n16);
    const int done = n16 << 4;
    if (done < bytes)
      burst4<1>(reinterpret_cast<uint32_t*>(static_cast<char*>(dst) + done),
                reinterpret_cast<const uint32_t*>(static_cast<const char*>(src) + done), (bytes - done) >> 2);
  } else {
    burst4<4 * MAXK>(reinterpret_cast<uint32_t*>(dst), reinterpret_cast<const uint32_t*>(src), bytes >> 2);
  }
}

// 16-byte output store with a cache policy SP: 0 plain (write-back L2), 1 nt, 2 sc1
// (write-through).  A dependent kernel boundary pays for the bytes its predecessor leaves
// dirty in L2 (MI355X_MICROARCH.md, "boundary": + B / 6 TB/s); in the latency regime (a tile or
// two per CU, the bench's B = 4,096) write-through stores move that write-back inside the
// kernel, under the other waves' work: encode -> reconstruct step 12.2 -> 10.5 us.  Bulk
// launches keep write-back stores (write-through encode at B = 262,144: 227 -> 311 us).
// BEAST_LAT_SP overrides the latency-regime policy (measurements).
#ifndef BEAST_LAT_SP
#define BEAST_LAT_SP 2
#endif
constexpr int LAT_SP = BEAST_LAT_SP;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
template <int SP>
__device__ __forceinline__ void st16(void* p, u32x4_t v) {
  if constexpr (SP == 1) {
    __builtin_nontemporal_store(v, static_cast<u32x4_t*>(p));
  } else if constexpr (SP == 2) {
    // vector store, write-through to memory (vmcnt counts it like any store; s_nop 1 covers
    // the store-data hazard of an inline-asm 128-bit store)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
  } else {
    *static_cast<u32x4_t*>(p) = v;
  }
}
template <int SP>
__device__ __forceinline__ void st4(float* p, float v) {
  if constexpr (SP == 2) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else *p = v;
}
template <int SP>
__device__ __forceinline__ void st16(void* p, float4 v) {
  st16<SP>(p, u32x4_t{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)});
}
template <int SP>
__device__ __forceinline__ void st16(void* p, long long a, long long b) {
  st16<SP>(p, u32x4_t{(unsigned)a, (unsigned)((unsigned long long)a >> 32), (unsigned)b,
                      (unsigned)((unsigned long long)b >> 32)});
}

// LDS -> global, float count
template <int NT = NTHREADS, int SP = 0>
__device__ __forceinline__ void store_out(float* __restrict__ dst, const float* __restrict__ src, int count) {
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int n4 = count >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i = threadIdx.x; i < n4; i += NT) st16<SP>(d4 + i, s4[i]);
    for (int i = (n4 << 2) + threadIdx.x; i < count; i += NT) dst[i] = src[i];
  } else {
    for (int i = threadIdx.x; i < count; i += NT) dst[i] = src[i];
  }
}

// LDS-DMA (global_load_lds): HBM -> LDS with no VGPR round trip, so every load of a stage
// is in flight at once and one vmcnt wait (the next __syncthreads) retires them all.  A
// wave-instruction writes 64 consecutive slots from a wave-uniform base: destinations are
// padded to whole wave-instructions, sources past the end are clamped to the last element.
typedef __attribute__((address_space(3))) void lds_void;

template <int NT = NTHREADS>
__device__ __forceinline__ void dma16(void* lds, const void* g, int n16) {
  const int tid = threadIdx.x, wb = tid & ~63;
  for (int base = 0; base < n16; base += NT) {
    if (base + wb < n16)
      __builtin_amdgcn_global_load_lds(static_cast<const uint4*>(g) + min(base + tid, n16 - 1),
                                       (lds_void*)(static_cast<uint4*>(lds) + base + wb), 16, 0, 0);
  }
}

template <int NT = NTHREADS>
__device__ __forceinline__ void dma4(void* lds, const void* g, int n) {
  const int tid = threadIdx.x, wb = tid & ~63;
  for (int base = 0; base < n; base += NT) {
    if (base + wb < n)
      __builtin_amdgcn_global_load_lds(static_cast<const uint32_t*>(g) + min(base + tid, n - 1),
                                       (lds_void*)(static_cast<uint32_t*>(lds) + base + wb), 4, 0, 0);
  }
}

// In-kernel cycle stamps (tools/stamps builds this file with -DBEAST_STAMPS; the product
// library compiles them out): s_memtime of lane 0 of every wave of workgroup 0 at the
// phase boundaries of its first tile.
#ifdef BEAST_STAMPS
__device__ unsigned long long g_stamps[2][8][16];
#define STAMP(k, i)                                                                              \
  do {                                                                                           \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_stamps[k][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// Per-workgroup lifetime (first 4096 workgroups): s_memrealtime (100 MHz, chip-wide) at
// entry and after the drain, and HW_ID / XCC_ID of the wave.
__device__ unsigned long long g_bstamps[2][4096][4];
#define BSTAMP(k, i)                                                                             \
  do {                                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                                 \
      g_bstamps[k][blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();                            \
      if (i == 0)                                                                                \
        g_bstamps[k][blockIdx.x][2] = ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32) | \
                                      (unsigned)__builtin_amdgcn_s_getreg(0xF804);               \
    }                                                                                            \
  } while (0)
#else
#define STAMP(k, i) do { } while (0)
#define BSTAMP(k, i) do { } while (0)
#endif

// -------------------------------------------------------------- geometry --
struct Geom {
  int D, nj, N, T, Tp, per;   // per = N * D
  int nq0, nq;                // column tiles of kind 0, of both kinds
  FastDiv fd_nj, fd_ng, fd_per, fd_N, fd_D, fd_nq;
};

template <int TBT>
inline Geom make_geom(int D, int nj, int N, int T) {
  Geom g;
  g.D = D; g.nj = nj; g.N = N; g.T = T; g.Tp = round_up(T, 4); g.per = N * D;
  const int ng = D - nj;
  g.nq0 = (TBT * nj + 15) / 16;
  g.nq = g.nq0 + (TBT * ng + 15) / 16;
  g.fd_nj = make_fd(std::max(nj, 1));
  g.fd_ng = make_fd(std::max(ng, 1));
  g.fd_per = make_fd(g.per);
  g.fd_N = make_fd(N);
  g.fd_D = make_fd(D);
  g.fd_nq = make_fd(std::max(g.nq, 1));
  return g;
}

// Compile-time problem shape.  A zero field is read from the runtime Geom instead; the
// BEAST defaults (N = 10 basis functions, T = 50 steps, 7 or 14 DoF with or without the
// two gripper DoF) get fully specialised kernels in which every index is a constant.
template <int SD, int SNJ, int SN, int ST, int SDL, int SW = NWAVES>
struct Shape {
  static constexpr int D = SD, NJ = SNJ, N = SN, T = ST, DL = SDL;
  static constexpr int W = SW;   // waves per workgroup: one per MFMA column tile of a full tile
  static constexpr bool fixed = SD > 0;
};
using DynShape = Shape<0, 0, 0, 0, 0>;

template <class S>
struct Dims {   // the shape, constant-folded where S fixes it
  int D, nj, ng, N, T, Tp, per;
  __device__ __forceinline__ Dims(const Geom& g)
      : D(S::D ? S::D : g.D), nj(S::fixed ? S::NJ : g.nj), ng(D - nj), N(S::N ? S::N : g.N),
        T(S::T ? S::T : g.T), Tp(S::T ? round_up(S::T, 4) : g.Tp), per(N * D) {}
};

template <class S>
__device__ __forceinline__ uint32_t div_by(uint32_t x, int dconst, const FastDiv& f) {
  return S::fixed ? x / (uint32_t)dconst : fdiv(x, f);
}

// MFMA column (trajectory j, DoF d) of tile q (wave-uniform) for lane column lc; valid =
// inside the tile set.
template <int TBT, class S>
__device__ __forceinline__ void tile_col(const Geom& g, const Dims<S>& m, int q, int lc, int& j, int& d, int& kind,
                                         bool& valid) {
  const int nq0 = (TBT * m.nj + 15) / 16;
  const int k0 = q < nq0 ? 0 : 1;
  const int dk = k0 ? m.ng : m.nj;
  const int c = (q - (k0 ? nq0 : 0)) * 16 + lc;
  valid = c < TBT * dk;
  const uint32_t cc = valid ? c : TBT * dk - 1;
  const uint32_t jj = k0 ? div_by<S>(cc, m.ng > 0 ? m.ng : 1, g.fd_ng) : div_by<S>(cc, m.nj > 0 ? m.nj : 1, g.fd_nj);
  j = (int)jj;
  d = (int)(cc - jj * dk) + (k0 ? m.nj : 0);
  kind = k0;
}

template <int TBT, class S>
__device__ __forceinline__ int n_coltiles(const Dims<S>& m) {
  return (TBT * m.nj + 15) / 16 + (TBT * m.ng + 15) / 16;
}

// ----------------------------------------------------------------- encode --
struct EncArgs {
  const float* traj;
  int64_t B, sb, st, sd, ntiles;
  int row_elems, vocab, phases;
  const int32_t* dof_src;
  const float* proj;   // [kinds][16][Tp] fp32 rounding of the fp64 ridge projection
  const float* w_min;
  const float* w_max;
  int64_t tok_offset;
  float* params_out;
  long long* tokens_out;
  Geom g;
  const float* const* traj_list;   // list mode: batch i at traj_list[i], list_rows rows each
  int64_t list_rows;               //   (a multiple of the tile, so no tile straddles two batches)
};

struct EncVArgs {
  const int32_t* dof_src;
  const float* proj;
  const float* w_min;
  const float* w_max;
  long long* tokens_out;
  float* params_out;
  int64_t tok_offset;
  int vocab, phases;
};
// First trajectory of tile row b0 (FAST path: contiguous rows of stride sb)
__device__ __forceinline__ const float* enc_tile_src(const EncArgs& a, int64_t b0) {
  if (a.traj_list == nullptr) return a.traj + b0 * a.sb;
  const uint64_t bi = (uint64_t)b0 / (uint64_t)a.list_rows;
  return a.traj_list[bi] + (b0 - (int64_t)bi * a.list_rows) * a.sb;
}

struct EncSmem {
  int P, Y, pb, kq, wlo, whi, lcol, total;
};

// Every buffer an LDS-DMA fills is padded to whole wave-instructions (64 lanes x 16 B).
template <int TBT>
__host__ __device__ inline EncSmem enc_smem(int T, int Tp, int Dl, int D, int N, int nkinds) {
  EncSmem s;
  int o = 0;
  // DMA destinations padded to whole wave-instructions, plus slack for the MFMA loop's
  // one-step-ahead operand reads past the last row (never used)
  s.P = o;    o += round_up(nkinds * 16 * Tp * 4 + 64 * ECH, 1024);   // fp32 [16][Tp] projection per kind
  s.Y = o;    o += round_up(TBT * T * Dl * 4, 1024);
  s.pb = o;   o += round_up(TBT * D * N * 4, 16);        // params, (d n) per trajectory
  s.kq = o;   o += round_up(D * N * 16, 16);             // {lo, hi, scale, 0} per (d n) column
  s.wlo = o;  o += round_up(D * N * 4, 256);
  s.whi = o;  o += round_up(D * N * 4, 256);
  s.lcol = o; o += round_up(D * 4, 256);
  s.total = o;
  return s;
}

template <int TBT, bool FAST, class S>
__global__ __launch_bounds__(S::W * 64) void k_encode(EncArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = S::W, NT = NW * 64;
  const Geom& g = a.g;
  const Dims<S> m(g);
  const int D = m.D, N = m.N, T = m.T, Tp = m.Tp, per = m.per, DN = D * N;
  const int Dl = FAST ? (S::DL ? S::DL : a.row_elems) : D;
  const int nkinds = (m.nj < D) ? 2 : 1;
  const int nq = n_coltiles<TBT>(m);
  const EncSmem L = enc_smem<TBT>(T, Tp, Dl, D, N, nkinds);
  float* P = reinterpret_cast<float*>(smem + L.P);
  float* Y = reinterpret_cast<float*>(smem + L.Y);
  float* pb = reinterpret_cast<float*>(smem + L.pb);
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  float4* kq = reinterpret_cast<float4*>(smem + L.kq);
  int* lcol = reinterpret_cast<int*>(smem + L.lcol);
  const int tid = threadIdx.x;
  const bool quant = a.tokens_out != nullptr;
  const int tile_elems = T * a.row_elems;   // FAST: one trajectory, contiguous, % 4 == 0

  STAMP(0, 0);
  BSTAMP(0, 0);
  // ---- prologue: the first tile and every constant go HBM -> LDS by DMA in one round trip
  if (FAST && (a.phases & 1) && blockIdx.x < a.ntiles) {
    const int64_t b0 = (int64_t)blockIdx.x * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);
    dma16<NT>(Y, enc_tile_src(a, b0), (nb * tile_elems) >> 2);
  }
  STAMP(0, 9);
  dma16<NT>(P, a.proj, nkinds * 4 * Tp);
  STAMP(0, 10);
  if (quant) {
    dma4<NT>(wlo, a.w_min, DN);
    dma4<NT>(whi, a.w_max, DN);
  }
  dma4<NT>(lcol, a.dof_src, D);
  STAMP(0, 11);

  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const float vm1 = (float)(a.vocab - 1);

  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);

    // ---- the trajectory tile lands in LDS (the first one is already in flight)
    if (a.phases & 1) {
      if (FAST) {
        if (tile != blockIdx.x) dma16<NT>(Y, enc_tile_src(a, b0), (nb * tile_elems) >> 2);
      } else {
        const int pt = T * D;
        for (int e = tid; e < nb * pt; e += NT) {
          const int j = e / pt, r = e - j * pt, t = r / D, d = r - t * D;
          const int col = a.dof_src[d];
          Y[e] = (col >= 0 && col < a.row_elems)
                     ? a.traj[(b0 + j) * a.sb + (int64_t)t * a.st + (int64_t)col * a.sd] : 0.0f;
        }
      }
    }
    if (tile == blockIdx.x) STAMP(0, 1);
    __syncthreads();   // waits for the DMA (vmcnt) and the LDS stores
    if (tile == blockIdx.x) STAMP(0, 2);
    if (tile == blockIdx.x + gridDim.x) STAMP(0, 12);
    if (quant && tile == blockIdx.x)   // bounds landed with the first tile; read after the next barrier
      for (int i = tid; i < DN; i += NT)
        kq[i] = make_float4(wlo[i], whi[i], beast::quantize_scale(wlo[i], whi[i], vm1), 0.0f);

    // ---- fit: params[j][d][n] = sum_t P_kind[n][t] y[j][t][d]  (f32 MFMA 16x16x4; A = P, B = y).
    //      A wave owns two column tiles per pass (two independent chains), operands
    //      pointer-stepped through LDS; rows t >= T (tail step) meet a zero A column.
    for (int q0 = wave; (a.phases & 2) && q0 < nq; q0 += NW * 2) {
      int j0, d0, k0, j1, d1, k1;
      bool ok0, ok1;
      tile_col<TBT>(g, m, q0, lr, j0, d0, k0, ok0);
      tile_col<TBT>(g, m, min(q0 + NW, nq - 1), lr, j1, d1, k1, ok1);
      ok0 = ok0 && j0 < nb;
      ok1 = ok1 && j1 < nb && (q0 + NW < nq);
      const int c0 = FAST ? min(max(lcol[d0], 0), Dl - 1) : d0;
      const int c1 = FAST ? min(max(lcol[d1], 0), Dl - 1) : d1;
      // K-steps in chunks of ECH: every LDS operand of a chunk is read before its MFMAs and
      // the next chunk's reads are issued before them too (one LDS round trip per chunk);
      // even / odd steps accumulate separately (two chains per tile).  Step s covers rows
      // t = 4s + lane/16, clamped to T - 1 (the zero-padded P columns meet them).
      const int nst = (T + 3) >> 2;
      const bool two = q0 + NW < nq;   // wave-uniform: a second column tile this pass
      const float* pa0 = P + (k0 * 16 + lr) * Tp + lk;
      const float* pa1 = P + (k1 * 16 + lr) * Tp + lk;
      const float* yc0 = Y + j0 * T * Dl + c0;
      const float* yc1 = Y + j1 * T * Dl + c1;
      float4_t acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
      float xa[ECH], ya[ECH], xb[ECH], yb[ECH];
#pragma unroll
      for (int i = 0; i < ECH; ++i) {
        const int row = min(4 * i + lk, T - 1) * Dl;
        xa[i] = pa0[4 * i]; ya[i] = yc0[row]; xb[i] = pa1[4 * i]; yb[i] = yc1[row];
      }
      for (int c = 0; c < nst; c += ECH) {
        float nxa[ECH], nya[ECH], nxb[ECH], nyb[ECH];
#pragma unroll
        for (int i = 0; i < ECH; ++i) {   // next chunk (reads past the end land in LDS slack, unused)
          const int st = c + ECH + i, row = min(4 * st + lk, T - 1) * Dl;
          nxa[i] = pa0[4 * st]; nya[i] = yc0[row]; nxb[i] = pa1[4 * st]; nyb[i] = yc1[row];
        }
#pragma unroll
        for (int i = 0; i < ECH; ++i) {
          if (c + i < nst) {   // wave-uniform
            if (i & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[i], ya[i], acc1, 0, 0, 0);
            else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[i], ya[i], acc0, 0, 0, 0);
            if (two) {
              if (i & 1) acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[i], yb[i], acc3, 0, 0, 0);
              else acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[i], yb[i], acc2, 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < ECH; ++i) { xa[i] = nxa[i]; ya[i] = nya[i]; xb[i] = nxb[i]; yb[i] = nyb[i]; }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc0[r] = __fadd_rn(acc0[r], acc1[r]);
        acc2[r] = __fadd_rn(acc2[r], acc3[r]);
      }
      // f32 C/D map: col = lane & 15, row = (lane >> 4) * 4 + r.  Each lane writes its params
      // into the (d n) image; quantisation happens in the epilogue, spread over every thread.
      if (tile == blockIdx.x && q0 == wave) STAMP(0, 8);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = lk * 4 + r;
        if (n < N) {
          if (ok0) pb[j0 * DN + d0 * N + n] = acc0[r];
          if (ok1) pb[j1 * DN + d1 * N + n] = acc2[r];
        }
      }
    }
    if (tile == blockIdx.x) STAMP(0, 3);
    if (tile == blockIdx.x + gridDim.x) STAMP(0, 13);
    __syncthreads();
    if (tile == blockIdx.x) STAMP(0, 4);

    // ---- epilogue: params (d n) and tokens (n d), both contiguous per tile
    constexpr int SP = (S::W == 7) ? LAT_SP : 0;   // the 7-wave shape is the latency regime's
    if (a.params_out != nullptr && (a.phases & 4)) store_out<NT, SP>(a.params_out + b0 * DN, pb, nb * DN);
    if (tile == blockIdx.x) STAMP(0, 5);
    if (quant && (a.phases & 8)) {
      // tokens in (n d) order: each thread quantises 4 consecutive tokens from the (d n)
      // params image (fast bins; the exactly-rounded chain only where one lies near a
      // rounding boundary), widens them to int64 + offset and stores 2 x 16 B.
      const int total = nb * per;
      long long* tout = a.tokens_out + b0 * per;
      const unsigned long long off = (unsigned long long)a.tok_offset;
      auto col_of = [&](int e, int& pj) {   // token e of the tile -> (d n) column, trajectory
        const int j = (int)div_by<S>((uint32_t)e, per, g.fd_per);
        const int r = e - j * per;
        const int n = (int)div_by<S>((uint32_t)r, D, g.fd_D);
        pj = j * DN;
        return (r - n * D) * N + n;
      };
      int done = 0;
      if ((((uintptr_t)tout) & 15) == 0) {
        const int n4 = total >> 2;
        for (int i = tid; i < n4; i += NT) {
          int bin[4], c[4], pj[4];
          float pv[4];
          float4 qv[4];
          bool ex = false;
          // every LDS operand of the 4 tokens is requested before any is used (one round trip)
#pragma unroll
          for (int u = 0; u < 4; ++u) c[u] = col_of(4 * i + u, pj[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) { pv[u] = pb[pj[u] + c[u]]; qv[u] = kq[c[u]]; }
#pragma unroll
          for (int u = 0; u < 4; ++u) bin[u] = beast::quantize_bin_k(pv[u], qv[u].x, qv[u].y, qv[u].z, vm1, ex);
          if (ex) {
#pragma unroll
            for (int u = 0; u < 4; ++u) bin[u] = beast::quantize_bin(pv[u], qv[u].x, qv[u].y, vm1);
          }
          st16<SP>(tout + 4 * i, beast::widen_bin(bin[0], off), beast::widen_bin(bin[1], off));
          st16<SP>(tout + 4 * i + 2, beast::widen_bin(bin[2], off), beast::widen_bin(bin[3], off));
        }
        done = n4 << 2;
      }
      for (int e = done + tid; e < total; e += NT) {
        int pj;
        const int c = col_of(e, pj);
        tout[e] = beast::widen_bin(beast::quantize_bin(pb[pj + c], wlo[c], whi[c], vm1), off);
      }
    }
    if (tile == blockIdx.x) STAMP(0, 6);
    if (tile == blockIdx.x + gridDim.x) STAMP(0, 14);
  }
#ifdef BEAST_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(0, 7);
  BSTAMP(0, 1);
#endif
}

// Fixed shapes of the per-trajectory kernels (k_encode_v): the MFMA K-steps over Tp.
template <class S>
struct VShape {
  static_assert(S::fixed && S::T > 0 && S::DL > 0 && ((S::T * S::DL) % 4) == 0, "per-trajectory encode: fixed shape");
  static constexpr int T = S::T, DL = S::DL, D = S::D, N = S::N, DN = S::D * S::N, Tp = round_up(S::T, 4);
  static constexpr int NST = Tp / 4;   // MFMA K-steps
};

// ------------------------------------------------------- encode, per-trajectory waves --
// waves = trajectories per tile of k_encode_v / k_reconstruct_v.  Round 6: 16 (one 1,024-thread
// workgroup per CU at B = 4,096) for both -- the encode -> reconstruct step is 2.4 % shorter than
// with 8-wave tiles (9.49-9.51 vs 9.70-9.75 us per step, outputs bitwise equal), although either
// kernel alone, launched back to back with itself, is 0.1 us slower; 16 / 8 mixed is slower than
// both (profiles/r06/codec_tile_width_ab_r06k.txt).  BEAST_RV_WE / _WR override (measurements).
// Bulk encode launches (more than one 16-trajectory tile per CU) keep 8-wave tiles: their 45 KB of
// LDS fit three workgroups -- 24 waves -- per CU, where a 16-wave tile's 84 KB fits one
// (B = 262,144: 232 vs 242 us, profiles/r06/).
#ifndef BEAST_RV_WE
#define BEAST_RV_WE 16
#endif
#ifndef BEAST_RV_WR
#define BEAST_RV_WR 16
#endif
constexpr int RV_WE = BEAST_RV_WE, RV_WR = BEAST_RV_WR, RV_WE_BULK = 8;
// Fixed shapes (the BEAST defaults), every batch size.  Wave j of the workgroup owns trajectory
// j of the 8-trajectory tile: C[n][d] = sum_t P_kind[n][t] y[j][t][lcol[d]] on
// v_mfma_f32_16x16x4_f32 (A = P, B = y[j]: the columns are the trajectory's DoFs), then the wave
// quantises its own accumulators, writes its trajectory's params (d n) and tokens (n d) into an
// LDS image of its own and copies both out with 16-byte write-through stores -- no workgroup
// barrier after the prologue, so one wave's stores overlap the others' MFMAs.  It replaced round 2's
// pipelined kernel (two sub-tiles, DMA / MFMA waves and store waves; 4.70 vs 4.44 us at B = 4,096,
// 209 vs 214 us at B = 262,144, profiles/r05/).  Same products in the same K order with the same
// even / odd accumulators as k_encode, and the same quantiser, so params and tokens are
// bit-identical.  With gripper DoFs each kind's chain sees zero B columns for the other kind.
struct EvSmem {
  int Y, P, wlo, whi, lcol, pimg, timg, total;
};
template <class S, int W>
__host__ __device__ constexpr EvSmem ev_smem(int nkinds) {
  using PS = VShape<S>;
  EvSmem s{};
  int o = 0;
  s.Y = o;    o += round_up(W * PS::T * PS::DL * 4, 1024);
  s.P = o;    o += round_up(nkinds * 16 * PS::Tp * 4, 1024);
  s.wlo = o;  o += round_up(PS::DN * 4, 256);
  s.whi = o;  o += round_up(PS::DN * 4, 256);
  s.lcol = o; o += round_up(PS::D * 4, 256);
  s.pimg = o; o += W * round_up(PS::DN * 4, 16);
  s.timg = o; o += W * round_up(PS::DN * 8, 16);
  s.total = o;
  return s;
}

template <class S, int SP, int W>
__global__ __launch_bounds__(W * 64) void k_encode_v(const float* __restrict__ traj, int64_t B, EncVArgs a) {
  using PS = VShape<S>;
  static_assert(PS::D <= 16 && PS::N <= 16 && PS::DL == PS::D, "per-trajectory encode: D, N <= 16, rows of D");
  constexpr int NT = W * 64, D = PS::D, N = PS::N, T = PS::T, Tp = PS::Tp, DN = PS::DN, NST = PS::NST;
  constexpr int NJ = S::NJ;
  constexpr int nkinds = NJ < D ? 2 : 1;
  constexpr EvSmem L = ev_smem<S, W>(nkinds);
  constexpr int PIMG = round_up(DN * 4, 16) / 4, TIMG = round_up(DN * 8, 16) / 8;
  static_assert((T * D) % 4 == 0 && (DN % 2) == 0, "per-trajectory encode: whole 16-byte rows");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* Y = reinterpret_cast<float*>(smem + L.Y);
  float* P = reinterpret_cast<float*>(smem + L.P);
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  int* lcol = reinterpret_cast<int*>(smem + L.lcol);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int64_t b0 = (int64_t)blockIdx.x * W;
  const int nb = (int)min<int64_t>(W, B - b0);
  const bool quant = a.tokens_out != nullptr;
  STAMP(0, 0);
  BSTAMP(0, 0);
  // ---- prologue: the tile and every constant HBM -> LDS by DMA, all in flight together
  constexpr int tile16 = T * D / 4;   // float4 per trajectory
  dma16<NT>(Y, reinterpret_cast<const float4*>(traj) + b0 * tile16, nb * tile16);
  STAMP(0, 9);
  dma16<NT>(P, a.proj, nkinds * 4 * Tp);
  if (quant) {
    dma4<NT>(wlo, a.w_min, DN);
    dma4<NT>(whi, a.w_max, DN);
  }
  dma4<NT>(lcol, a.dof_src, D);
  const float vm1 = (float)(a.vocab - 1);
  __syncthreads();
  STAMP(0, 2);
  const int j = wave;
  if (j >= nb) return;   // no barrier follows
  // ---- fit: lane (lr, lk): A = P_kind[n = lr][t = 4 st + lk], B = y[j][t][lcol[d = lr]] (t clamped
  //      to T - 1: the zero-padded P columns meet those rows), even / odd steps accumulate apart
  const int lr = lane & 15, lk = lane >> 4;
  const bool dok = lr < D;
  const int c = dok ? min(max(lcol[lr], 0), D - 1) : 0;
  const float* yc = Y + j * T * D + c;
  float4_t acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = acc0;
#pragma unroll
  for (int kd = 0; kd < nkinds; ++kd) {
    const bool mine = dok && (nkinds == 1 || ((lr < NJ) == (kd == 0)));
    const float* pa = P + (kd * 16 + lr) * Tp + lk;
    float xa[NST], ya[NST];
#pragma unroll
    for (int st = 0; st < NST; ++st) {   // every operand read before the chain (one LDS round trip)
      xa[st] = pa[4 * st];
      const float y = yc[min(4 * st + lk, T - 1) * D];
      ya[st] = mine ? y : 0.0f;
    }
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (st & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[st], ya[st], acc1, 0, 0, 0);
      else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[st], ya[st], acc0, 0, 0, 0);
    }
  }
  STAMP(0, 3);
  // ---- C/D map: row n = lk * 4 + r, column d = lr.  Params (d n) and tokens (n d) of the trajectory
  //      into this wave's images; the quantiser is k_encode's (fast bins, the exact chain near a
  //      rounding boundary or for NaN / inf)
  float* pimg = reinterpret_cast<float*>(smem + L.pimg) + j * PIMG;
  long long* timg = reinterpret_cast<long long*>(smem + L.timg) + j * TIMG;
  float pv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) pv[r] = __fadd_rn(acc0[r], acc1[r]);
  if (dok) {
    float* q = pimg + lr * N + 4 * lk;
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      if (4 * lk + r + 1 < N) *reinterpret_cast<float2*>(q + r) = make_float2(pv[r], pv[r + 1]);
      else if (4 * lk + r < N) q[r] = pv[r];
    }
  }
  if (quant) {
    const unsigned long long off = (unsigned long long)a.tok_offset;
    float lo[4], hi[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = lr * N + min(4 * lk + r, N - 1);
      lo[r] = wlo[min(k, DN - 1)];
      hi[r] = whi[min(k, DN - 1)];
    }
    int bin[4];
    bool ex = false;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bin[r] = beast::quantize_bin_k(pv[r], lo[r], hi[r], beast::quantize_scale(lo[r], hi[r], vm1), vm1, ex);
    if (ex) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bin[r] = beast::quantize_bin(pv[r], lo[r], hi[r], vm1);
    }
    if (dok) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * lk + r < N) timg[(4 * lk + r) * D + lr] = beast::widen_bin(bin[r], off);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  STAMP(0, 5);
  // ---- 16-byte write-through stores of the trajectory's params (DN floats) and tokens (DN int64)
  if (a.phases & 4) {
    if (a.params_out != nullptr) {
      float4* gp = reinterpret_cast<float4*>(a.params_out + (b0 + j) * DN);
#pragma unroll
      for (int u = 0; u < (DN / 4 + 63) / 64; ++u) {
        const int i = u * 64 + lane;
        if (i < DN / 4) st16<SP>(gp + i, reinterpret_cast<const float4*>(pimg)[i]);
      }
    }
    if (quant) {
      long long* gt = a.tokens_out + (b0 + j) * DN;
#pragma unroll
      for (int u = 0; u < (DN / 2 + 63) / 64; ++u) {
        const int i = u * 64 + lane;
        if (i < DN / 2) st16<SP>(gt + 2 * i, timg[2 * i], timg[2 * i + 1]);
      }
    }
  }
  STAMP(0, 7);
#ifdef BEAST_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(0, 8);
  BSTAMP(0, 1);
#endif
}

// ------------------------------------------------------------ reconstruct --
struct RecArgs {
  const long long* tokens;
  const float* ntokens;
  int64_t B, ntiles, tok_offset, basis_sb, init_p_sb;
  int vocab, Tout, ndo, phases, lut_n, tbt;
  const float* w_min;
  const float* w_max;
  const float* basis;      // [2][Tout][N] (shared) or per trajectory with stride basis_sb
  const int32_t* dof_dst;
  const float* init_p;
  const int32_t* init_p_src;
  float* params_out;
  float* pos_out;
  Geom g;
  FastDiv fd_row;          // Tout * ndo
};

// The per-trajectory kernels' argument blocks: only what k_encode_v / k_reconstruct_v read (their
// shapes are compile-time), 64 / 88 bytes instead of EncArgs' / RecArgs' ~260.  The runtime copies
// every launch's argument block into the kernarg ring, and a 224-byte block costs the host ~0.28 us
// more per launch than an 8- or 64-byte one (tools/launch/launch_bench.hip, profiles/r06/).
struct RecVArgs {
  const float* w_min;
  const float* w_max;
  const float* basis;
  const int32_t* dof_dst;
  const float* init_p;
  const int32_t* init_p_src;
  float* pos_out;
  int64_t tok_offset, init_p_sb;
  int vocab, lut_n, phases;
};

constexpr int LUT_MAX = 4096;   // dequantise LUT tok / (vocab - 1), IEEE-divided once
constexpr int RT_REG = 4;       // row tiles (64 output rows) whose basis operands live in registers

// token tile [nb][per] (int64, or fp32 normalised tokens) HBM -> LDS by DMA
// rows [b0, b0 + tbt) of a [B][per] array of esz-byte elements HBM -> LDS by DMA
template <int NT = NTHREADS>
__device__ __forceinline__ void stage_rows(void* lds, const void* base, int64_t B, int esz, int64_t b0, int per,
                                           int tbt) {
  const int nb = (int)min<int64_t>(B - b0, tbt);
  const char* src = static_cast<const char*>(base) + b0 * per * esz;
  const int bytes = nb * per * esz;
  if ((bytes & 15) == 0 && (((uintptr_t)src) & 15) == 0) dma16<NT>(lds, src, bytes >> 4);
  else dma4<NT>(lds, src, bytes >> 2);
}

template <int NT = NTHREADS>
__device__ __forceinline__ void stage_tokens(const RecArgs& a, void* lds, int64_t b0, int per) {
  const int nb = (int)min<int64_t>(a.B - b0, a.tbt);
  const void* src = a.ntokens ? static_cast<const void*>(a.ntokens + b0 * per)
                              : static_cast<const void*>(a.tokens + b0 * per);
  const int bytes = nb * per * (a.ntokens ? 4 : 8);
  if ((bytes & 15) == 0 && (((uintptr_t)src) & 15) == 0) dma16<NT>(lds, src, bytes >> 4);
  else dma4<NT>(lds, src, bytes >> 2);
}

// W[j][d][n] from the staged tile: bit-exact discrete_to_continuous (beast/utils.py:20-25)
// or, for normalised tokens, denormalize_tensor's intent (utils.py:38-44).
__device__ __forceinline__ float rec_weight(const RecArgs& a, const unsigned char* tokl, int e, int k,
                                            const float* wlo, const float* whi, const float* lut, float vm1) {
  const float lo = wlo[k], hi = whi[k];
  if (a.ntokens) return beast::denormalize_one(reinterpret_cast<const float*>(tokl)[e], lo, hi);
  const long long t = reinterpret_cast<const long long*>(tokl)[e] - a.tok_offset;
  const float nrm = (t >= 0 && t < a.lut_n) ? lut[t] : __fdiv_rn((float)t, vm1);
  return beast::clamp_t(__fadd_rn(__fmul_rn(nrm, __fsub_rn(hi, lo)), lo), lo, hi);
}

// B operand of one MFMA lane for KS K-steps: W[j][d][n], n = lk * KS + ks (clamped to N - 1
// for the read; the caller zeroes n >= N).  rec_weight's arithmetic, with every LDS read of
// the KS steps issued before any is used: tokens and bounds in one round trip, the LUT in
// a second; tokens outside the LUT (rare) take the IEEE division behind an exec branch.
template <int KS>
__device__ __forceinline__ void rec_weights(const RecArgs& a, const unsigned char* tokl, int j, int d, int lk,
                                            int N, int D, int per, const float* wlo, const float* whi,
                                            const float* lut, float vm1, float (&w)[KS]) {
  float lo[KS], hi[KS];
  int e[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int n = min(lk * KS + ks, N - 1), k = d * N + n;
    e[ks] = j * per + n * D + d;
    lo[ks] = wlo[k];
    hi[ks] = whi[k];
  }
  if (a.ntokens) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      w[ks] = beast::denormalize_one(reinterpret_cast<const float*>(tokl)[e[ks]], lo[ks], hi[ks]);
    return;
  }
  long long t[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) t[ks] = reinterpret_cast<const long long*>(tokl)[e[ks]] - a.tok_offset;
  float nrm[KS];
  bool far = false;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const bool in = (t[ks] >= 0) & (t[ks] < a.lut_n);
    far = far | !in;
    nrm[ks] = lut[in ? (int)t[ks] : 0];
  }
  if (far) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      if (!((t[ks] >= 0) & (t[ks] < a.lut_n))) nrm[ks] = __fdiv_rn((float)t[ks], vm1);
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    w[ks] = beast::clamp_t(__fadd_rn(__fmul_rn(nrm[ks], __fsub_rn(hi[ks], lo[ks])), lo[ks]), lo[ks], hi[ks]);
}

struct RecSmem {
  int phi, tok, wlo, whi, lut, dst, out, pb, pmap, col2d, total;
  int Np4, RTR;   // padded basis width, padded output rows
  bool stage;
};

// Shared basis (KS > 0, MFMA): the basis operands are in registers (RT = RT_REG, T_out <= 64)
// or in LDS (RT = 0).  Per-row basis (KS == 0, VALU): W in LDS, rows of the basis from HBM.
template <int TBT, int KS, int RT>
__host__ __device__ inline RecSmem rec_smem(int Tout, int D, int N, int ndo, int nkinds, int lut_n) {
  RecSmem s;
  const int per = N * D;
  s.Np4 = KS ? 4 * KS : round_up(N, 4);
  s.RTR = KS ? round_up(Tout, 64) : Tout;   // row tiles in groups of four
  int o = 0;
  // basis in LDS: RT == 0 the zero-padded [kinds][RTR][Np4] image; RT > 0 the raw [kinds][Tout][N] (DMA)
  s.phi = o;   o += KS ? (RT == 0 ? round_up(nkinds * s.RTR * s.Np4 * 4, 16) : round_up(nkinds * Tout * N * 4, 1024)) : 0;
  s.tok = o;   o += round_up(TBT * per * 8, 1024);   // DMA destinations: whole wave-instructions
  s.wlo = o;   o += round_up(per * 4, 256);
  s.whi = o;   o += round_up(per * 4, 256);
  s.lut = o;   o += round_up(lut_n * 4, 16);
  s.dst = o;   o += round_up(D * 4, 256);
  s.pb = o;    o += KS ? 0 : round_up(TBT * D * s.Np4 * 4, 16);
  s.pmap = o;  o += KS ? 0 : round_up(per * 2, 16);   // (n d) slot -> W offset d*Np4 + n
  s.col2d = o; o += KS ? 0 : round_up(ndo * 4, 16);
  const int outb = round_up(TBT * s.RTR * ndo * 4, 16);
  s.stage = KS ? true : (o + outb) <= 96 * 1024;
  s.out = o;   o += s.stage ? outb : 0;
  s.total = o;
  return s;
}

// decode-only output (params_out, (d n) order) straight from the staged tokens
template <int NT = NTHREADS>
__device__ __forceinline__ void rec_params_out(const RecArgs& a, const unsigned char* tokl, int64_t b0, int nb,
                                               const float* wlo, const float* whi, const float* lut, float vm1) {
  const Geom& g = a.g;
  const int per = g.per, D = g.D, N = g.N;
  float* pout = a.params_out + b0 * per;
  for (int e = threadIdx.x; e < nb * per; e += NT) {
    const uint32_t j = fdiv(e, g.fd_per);
    const int k = e - j * per;                 // (d n) index
    const uint32_t d = fdiv(k, g.fd_N);
    const int n = k - d * N;
    pout[e] = rec_weight(a, tokl, j * per + n * D + d, k, wlo, whi, lut, vm1);
  }
}

// ob rows [0, Tout) of each trajectory -> one contiguous HBM tile
template <class S>
__device__ __forceinline__ void rec_store(const RecArgs& a, float* gout, const float* ob, int nb, int RTR) {
  const int Tout = S::T ? S::T : a.Tout, ndo = S::DL ? S::DL : a.ndo;
  const int rowlen = Tout * ndo;
  if ((rowlen & 3) == 0 && ((RTR * ndo) & 3) == 0 && ((((uintptr_t)gout) & 15) == 0)) {
    const int n4 = nb * rowlen / 4;
    for (int i = threadIdx.x; i < n4; i += S::W * 64) {
      const uint32_t e = 4 * i;
      const uint32_t j = div_by<S>(e, rowlen, a.fd_row);
      st16<(S::W == 7) ? LAT_SP : 0>(reinterpret_cast<float4*>(gout) + i,
                                     *reinterpret_cast<const float4*>(ob + j * RTR * ndo + (e - j * rowlen)));
    }
  } else {
    for (int e = threadIdx.x; e < nb * rowlen; e += S::W * 64) {
      const uint32_t j = div_by<S>(e, rowlen, a.fd_row);
      gout[e] = ob[j * RTR * ndo + (e - j * rowlen)];
    }
  }
}

// tsrc (the token rows: a.tokens, or a.ntokens with esz 4), B and esz lead the argument list for
// kernarg preloading, as in k_encode_v: the first tile's DMA needs nothing else.
template <int TBT, int KS, int RT, class S>
__global__ __launch_bounds__(S::W * 64) void k_reconstruct(const void* __restrict__ tsrc, int64_t B, int esz,
                                                           RecArgs a) {
  static_assert(KS > 0, "shared-basis kernel");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = S::W, NT = NW * 64;
  const Geom& g = a.g;
  const Dims<S> m(g);
  const int D = m.D, N = m.N, nj = m.nj, per = m.per;
  const int Tout = S::T ? S::T : a.Tout, ndo = S::DL ? S::DL : a.ndo;
  const int nkinds = (nj < D) ? 2 : 1;
  const int nq = n_coltiles<TBT>(m);
  const RecSmem L = rec_smem<TBT, KS, RT>(Tout, D, N, ndo, nkinds, a.lut_n);
  constexpr int Np4 = 4 * KS;
  const int RTR = L.RTR;
  float* phi = reinterpret_cast<float*>(smem + L.phi);
  const unsigned char* tokl = smem + L.tok;
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  float* lut = reinterpret_cast<float*>(smem + L.lut);
  int* dst = reinterpret_cast<int*>(smem + L.dst);
  float* ob = reinterpret_cast<float*>(smem + L.out);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const float vm1 = (float)(a.vocab - 1);

  STAMP(1, 0);
  BSTAMP(1, 0);
  // ---- prologue: the first token tile, the bounds and the DoF map by DMA; the basis
  //      operands (registers or LDS) by clamped loads -- all in flight together
  // the first tile (the grid never exceeds the tile count); BEAST_DEBUG_PHASES does not skip it
  stage_rows<NT>(smem + L.tok, tsrc, B, esz, (int64_t)blockIdx.x * TBT, per, TBT);
  STAMP(1, 9);
  dma4<NT>(wlo, a.w_min, per);
  dma4<NT>(whi, a.w_max, per);
  dma4<NT>(dst, a.dof_dst, D);
  STAMP(1, 10);
  // A operand of MFMA row tile rt, K-step ks: Phi_kind[rt*16 + lr][n], n = lane/16 * KS + ks,
  // zero outside [Tout) x [N).  RT > 0: the raw basis [kinds][Tout][N] is DMA'd to LDS with
  // the first token tile and the operands are read into registers once, after it lands.
  float phr[2][RT > 0 ? RT : 1][KS];
  if constexpr (RT > 0) {
    const int pbytes = nkinds * Tout * N * 4;
    if ((pbytes & 15) == 0 && (((uintptr_t)a.basis) & 15) == 0) dma16<NT>(phi, a.basis, pbytes >> 4);
    else dma4<NT>(phi, a.basis, pbytes >> 2);
  } else {
    const int tot = nkinds * RTR * Np4, tn = RTR * Np4;
    for (int base = 0; base < tot; base += 8 * NT) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = min(base + u * NT + tid, tot - 1);
        const int k = i >= tn ? 1 : 0, r = i - k * tn, t = r / Np4, n = r - t * Np4;
        const float x = a.basis[(int64_t)k * Tout * N + min(t, Tout - 1) * N + min(n, N - 1)];
        const uint32_t keep = 0u - (uint32_t)((t < Tout) & (n < N));
        v[u] = __uint_as_float(__float_as_uint(x) & keep);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) phi[min(base + u * NT + tid, tot - 1)] = v[u];
    }
  }
  STAMP(1, 11);
  for (int t = tid; t < a.lut_n; t += NT) lut[t] = __fdiv_rn((float)t, vm1);
  STAMP(1, 12);

  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);

    if ((a.phases & 1) && tile != blockIdx.x) stage_tokens<NT>(a, smem + L.tok, b0, per);
    if (tile == blockIdx.x) STAMP(1, 1);
    __syncthreads();   // tokens (DMA), bounds, DoF map, LDS basis and LUT are in place
    if (tile == blockIdx.x) STAMP(1, 2);
    if constexpr (RT > 0) {
      if (tile == blockIdx.x) {
#pragma unroll
        for (int kd = 0; kd < 2; ++kd)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              const int t = rt * 16 + lr, n = lk * KS + ks;
              const float x = phi[(min(kd, nkinds - 1) * Tout + min(t, Tout - 1)) * N + min(n, N - 1)];
              phr[kd][rt][ks] = (t < Tout && n < N && kd < nkinds) ? x : 0.0f;
            }
      }
    }
    if (a.params_out != nullptr) rec_params_out<NT>(a, tokl, b0, nb, wlo, whi, lut, vm1);

    // ---- pos[j][t][dst(d)] = sum_n Phi_kind[t][n] W[j][d][n]  (f32 MFMA 16x16x4; A = Phi, B = W).
    //      A wave owns a column tile (j, d) and dequantises its own B operand (K-step ks
    //      holds n = 4*ks + lane/16) straight from the token tile; the basis operands
    //      are reused across the wave's column tiles; rows past Tout land in ob's padding.
    for (int q = wave; (a.phases & 2) && q < nq; q += NW) {
      int j, d, kind;
      bool ok;
      tile_col<TBT>(g, m, q, lr, j, d, kind, ok);
      ok = ok && j < nb;
      float w[KS];   // B operand, K-step ks: W[j][d][n], n = lane/16 * KS + ks
      rec_weights<KS>(a, tokl, j, d, lk, N, D, per, wlo, whi, lut, vm1, w);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) w[ks] = (ok && lk * KS + ks < N) ? w[ks] : 0.0f;
      if (a.init_p != nullptr && lk == 0 && ok && d < nj)   // coefficient n = 0 of the joint DoFs <- init_p
        w[0] = a.init_p[(b0 + j) * a.init_p_sb + a.init_p_src[d]];   // (reference :505-510)
      float* oc = ob + (j * RTR + lk * 4) * ndo + min(max(dst[d], 0), ndo - 1);
      if constexpr (RT > 0) {
        float4_t acc[RT];
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i] = float4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int i = 0; i < RT; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(kind ? phr[1][i][ks] : phr[0][i][ks], w[ks], acc[i], 0,
                                                          0, 0);
        // f32 C/D map: col = lane & 15, row = (lane >> 4) * 4 + r
        if (ok) {
#pragma unroll
          for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) oc[(i * 16 + r) * ndo] = acc[i][r];
        }
      } else {
        const float* Ph = phi + (kind * RTR + lr) * Np4 + lk * KS;
        for (int rt = 0; rt < RTR / 16; rt += 4) {   // four row tiles: four independent chains
          float av[4][KS];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) av[i][ks] = Ph[((rt + i) * 16) * Np4 + ks];
          float4_t acc[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = float4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][ks], w[ks], acc[i], 0, 0, 0);
          if (ok) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int r = 0; r < 4; ++r) oc[((rt + i) * 16 + r) * ndo] = acc[i][r];
          }
        }
      }
    }
    if (tile == blockIdx.x) STAMP(1, 5);
    __syncthreads();
    if (tile == blockIdx.x) STAMP(1, 6);
    if (a.phases & 4) rec_store<S>(a, a.pos_out + b0 * (int64_t)Tout * ndo, ob, nb, RTR);
    if (tile == blockIdx.x) STAMP(1, 7);
  }
#ifdef BEAST_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(1, 8);
  BSTAMP(1, 1);
#endif
}

// ------------------------------------------------ reconstruct, per-trajectory waves --
// Latency regime (<= 2 tiles per CU, e.g. the bench's B = 4,096), fixed shapes with
// num_dof_out == D.  k_reconstruct computes pos^T (rows t, columns (trajectory, DoF)), so a
// lane's accumulators are 4 rows of one output column, 4 * ndo bytes apart: they go through an
// LDS image, a workgroup barrier and a cooperative store, and HBM sits idle while the whole chip
// computes.  Here the MFMA computes pos[j] itself: wave j owns trajectory j of the tile, A = W
// (16 rows = output columns c, K = basis n), B = Phi^T (columns t), so a lane's accumulator
// holds columns c = 4 kk .. 4 kk + 3 of one row t -- contiguous bytes of pos[j][t][.] -- and each
// wave stores its trajectory straight from registers as soon as its own chain is done (no LDS
// image, no barrier): the stores of the first waves overlap the MFMAs of the others.
// Same K mapping (n = kk * KS + s) and the same products summed in the same order as
// k_reconstruct (a product's operands only swap roles), so positions are bit-identical.  With
// gripper DoFs the rows of the other kind are zero in each kind's chain: the joint chain then
// the gripper chain, each adding exact zeros to the other kind's rows.

struct RvSmem {
  int tok, wlo, whi, dst, phi, lut, wimg, img, total;
};
template <class S>
__host__ __device__ constexpr RvSmem rv_smem(int nkinds) {
  RvSmem s{};
  constexpr int per = S::D * S::N;
  int o = 0;
  s.tok = o;  o += round_up(RV_WR * per * 8, 1024);           // DMA: whole wave-instructions
  s.wlo = o;  o += round_up(per * 4, 256);
  s.whi = o;  o += round_up(per * 4, 256);
  s.dst = o;  o += round_up(S::D * 4, 256);
  s.phi = o;  o += round_up(nkinds * S::T * S::N * 4, 1024);
  s.lut = o;  o += round_up(LUT_MAX * 4, 16);
  s.wimg = o; o += round_up(RV_WR * per * 4, 16);              // W[j][d][n] (d n), one per wave
  s.img = o;  o += RV_WR * round_up(S::T * S::D * 4, 16);        // pos[j] [T][D], one per wave
  s.total = o;
  return s;
}

template <int KS, class S, int SP>
__global__ __launch_bounds__(RV_WR * 64) void k_reconstruct_v(const void* __restrict__ tsrc, int64_t B, int esz,
                                                             RecVArgs a) {
  static_assert(S::fixed && S::T > 0 && S::T <= 64 && S::D <= 16 && S::DL == S::D && 4 * KS >= S::N,
                "per-trajectory reconstruct: fixed shape, T <= 64, D <= 16, ndo == D");
  constexpr int NT = RV_WR * 64, D = S::D, N = S::N, T = S::T, per = D * N;
  constexpr int NJ = S::NJ;
  constexpr int nkinds = NJ < D ? 2 : 1;
  constexpr RvSmem L = rv_smem<S>(nkinds);
  constexpr int RV_IMG = round_up(T * D * 4, 16) / 4;   // floats per wave's output image
  static_assert((T * D) % 4 == 0, "per-trajectory reconstruct: whole 16-byte rows");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned char* tokl = smem + L.tok;
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  int* dst = reinterpret_cast<int*>(smem + L.dst);
  float* phi = reinterpret_cast<float*>(smem + L.phi);
  float* lut = reinterpret_cast<float*>(smem + L.lut);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int64_t b0 = (int64_t)blockIdx.x * RV_WR;
  STAMP(1, 0);
  BSTAMP(1, 0);
  // ---- prologue: the token tile, bounds, DoF map and raw basis by DMA, all in flight together
  stage_rows<NT>(smem + L.tok, tsrc, B, esz, b0, per, RV_WR);
  STAMP(1, 9);
  dma4<NT>(wlo, a.w_min, per);
  dma4<NT>(whi, a.w_max, per);
  dma4<NT>(dst, a.dof_dst, D);
  {
    constexpr int pbytes = nkinds * T * N * 4;
    if ((pbytes & 15) == 0 && (((uintptr_t)a.basis) & 15) == 0) dma16<NT>(phi, a.basis, pbytes >> 4);
    else dma4<NT>(phi, a.basis, pbytes >> 2);
  }
  const float vm1 = (float)(a.vocab - 1);
  for (int t = tid; t < a.lut_n; t += NT) lut[t] = __fdiv_rn((float)t, vm1);
  STAMP(1, 12);
  __syncthreads();   // every DMA and the LUT are in place
  STAMP(1, 2);
  const int j = wave;
  const int nb = (int)min<int64_t>(RV_WR, B - b0);
  if (j >= nb) return;   // no barrier follows
  // ---- W[j][d][n] of this wave's trajectory (bit-exact discrete_to_continuous, init_p for n = 0 of
  //      the joint DoFs: reference :505-510) into its LDS image
  float* wimg = reinterpret_cast<float*>(smem + L.wimg) + j * per;
  const long long* tk = reinterpret_cast<const long long*>(tokl) + j * per;
#pragma unroll
  for (int u = 0; u < (per + 63) / 64; ++u) {
    const int e = u * 64 + lane;   // (n d) order
    if (e < per) {
      const int n = e / D, d = e - n * D, k = d * N + n;
      const float lo = wlo[k], hi = whi[k];
      const long long t = tk[e] - a.tok_offset;
      const float nrm = (t >= 0 && t < a.lut_n) ? lut[(int)t] : __fdiv_rn((float)t, vm1);
      float w = beast::clamp_t(__fadd_rn(__fmul_rn(nrm, __fsub_rn(hi, lo)), lo), lo, hi);
      if (a.init_p != nullptr && n == 0 && d < NJ) w = a.init_p[(b0 + j) * a.init_p_sb + a.init_p_src[d]];
      wimg[k] = w;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  STAMP(1, 3);
  // ---- A = W: row c = lane & 15 is output column c, i.e. DoF d with dst[d] == c; K-step s holds
  //      n = kk * KS + s (k_reconstruct's mapping), zero past N, past D and for the other kind
  const int c = lane & 15, kk = lane >> 4;
  int dsrc = -1;
#pragma unroll
  for (int d = 0; d < D; ++d) dsrc = dst[d] == c ? d : dsrc;
  const bool row_ok = dsrc >= 0;
  const int dd = row_ok ? dsrc : 0;
  float av[KS];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) {
    const int n = kk * KS + s2;
    const float w = wimg[dd * N + min(n, N - 1)];
    av[s2] = (row_ok && n < N) ? w : 0.0f;
  }
  // ---- B = Phi_kind^T: column t = 16 tt + (lane & 15), K-step s: n = kk * KS + s
  float4_t acc[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) acc[tt] = float4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int kd = 0; kd < nkinds; ++kd) {
    float bv[4][KS];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        const int t = tt * 16 + c, n = kk * KS + s2;
        const float x = phi[(kd * T + min(t, T - 1)) * N + min(n, N - 1)];
        bv[tt][s2] = (t < T && n < N) ? x : 0.0f;
      }
    const bool mine = nkinds == 1 || ((dd < NJ) == (kd == 0));
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      const float ak = mine ? av[s2] : 0.0f;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
        if (tt * 16 < T) acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ak, bv[tt][s2], acc[tt], 0, 0, 0);
    }
  }
  STAMP(1, 5);
  // ---- f32 C/D map: row (column c of pos) = kk * 4 + r, column (t) = lane & 15: this lane holds
  //      pos[j][16 tt + (lane & 15)][4 kk .. 4 kk + 3].  Those are 8-byte aligned (t * D * 4 is a
  //      multiple of 16 only for even t), and 8-byte write-through stores are one fabric write each,
  //      so the wave puts its trajectory's [T][D] image into LDS (its own region: no workgroup
  //      barrier) and copies it out as 16-byte write-through stores.
  float* img = reinterpret_cast<float*>(smem + L.img) + j * RV_IMG;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    const int t = tt * 16 + c;
    if (tt * 16 < T && t < T) {
      float* q = img + t * D + 4 * kk;
      if (4 * kk + 1 < D) *reinterpret_cast<float2*>(q) = make_float2(acc[tt][0], acc[tt][1]);
      else if (4 * kk < D) q[0] = acc[tt][0];
      if (4 * kk + 3 < D) *reinterpret_cast<float2*>(q + 2) = make_float2(acc[tt][2], acc[tt][3]);
      else if (4 * kk + 2 < D) q[2] = acc[tt][2];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  STAMP(1, 6);
  if (a.phases & 4) {
    constexpr int n4 = T * D / 4;
    float4* gout = reinterpret_cast<float4*>(a.pos_out + (b0 + j) * (int64_t)T * D);
#pragma unroll
    for (int u = 0; u < (n4 + 63) / 64; ++u) {
      const int i = u * 64 + lane;
      if (i < n4) st16<SP>(gout + i, reinterpret_cast<const float4*>(img)[i]);
    }
  }
  STAMP(1, 7);
#ifdef BEAST_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(1, 8);
  BSTAMP(1, 1);
#endif
}

// Per-trajectory basis rows (custom times per row, KS == 0): decode W into LDS, then a
// sequential fma over n per output (the MFMA chain's order) on the VALU; also the
// decode-only path when no positions are requested.
template <int TBT>
__global__ __launch_bounds__(NTHREADS) void k_reconstruct_rows(RecArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Geom& g = a.g;
  const int D = g.D, N = g.N, nj = g.nj, per = g.per;
  const int Tout = a.Tout, ndo = a.ndo;
  const bool pos = a.pos_out != nullptr;
  const RecSmem L = rec_smem<TBT, 0, 0>(Tout, D, N, ndo, (nj < D) ? 2 : 1, a.lut_n);
  const int Np4 = L.Np4;
  const unsigned char* tokl = smem + L.tok;
  float* pb = reinterpret_cast<float*>(smem + L.pb);
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  float* lut = reinterpret_cast<float*>(smem + L.lut);
  uint16_t* pmap = reinterpret_cast<uint16_t*>(smem + L.pmap);
  int* dst = reinterpret_cast<int*>(smem + L.dst);
  int* col2d = reinterpret_cast<int*>(smem + L.col2d);
  float* ob = reinterpret_cast<float*>(smem + L.out);
  const int tid = threadIdx.x;
  const float vm1 = (float)(a.vocab - 1);

  if (blockIdx.x < a.ntiles) stage_tokens(a, smem + L.tok, (int64_t)blockIdx.x * TBT, per);
  dma4(wlo, a.w_min, per);
  dma4(whi, a.w_max, per);
  if (pos) dma4(dst, a.dof_dst, D);
  for (int t = tid; t < a.lut_n; t += NTHREADS) lut[t] = __fdiv_rn((float)t, vm1);
  for (int r = tid; r < per; r += NTHREADS) {
    const int n = r / D, d = r - n * D;
    pmap[r] = (uint16_t)(d * Np4 + n);
  }
  if (pos) {   // output column -> DoF (after the DMA of dst)
    __syncthreads();
    for (int c = tid; c < ndo; c += NTHREADS) col2d[c] = -1;
    __syncthreads();
    if (tid < D) {
      const int dd = dst[tid];
      if (dd >= 0 && dd < ndo) col2d[dd] = tid;
    }
  }

  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);
    if (tile != blockIdx.x) stage_tokens(a, smem + L.tok, b0, per);
    __syncthreads();
    if (a.params_out != nullptr) rec_params_out(a, tokl, b0, nb, wlo, whi, lut, vm1);
    if (!pos) continue;
    for (int e = tid; e < nb * per; e += NTHREADS) {   // (n d) tokens -> W[j][d][n]
      const uint32_t j = fdiv(e, g.fd_per);
      const int r = e - j * per;
      const uint32_t n = fdiv(r, g.fd_D);
      const int d = r - n * D;
      pb[j * D * Np4 + pmap[r]] = rec_weight(a, tokl, e, d * N + n, wlo, whi, lut, vm1);
    }
    __syncthreads();
    if (a.init_p != nullptr) {   // coefficient 0 of the joint DoFs <- init_p (reference :505-510)
      for (int e = tid; e < nb * nj; e += NTHREADS) {
        const int j = e / nj, d = e - j * nj;
        pb[(j * D + d) * Np4] = a.init_p[(b0 + j) * a.init_p_sb + a.init_p_src[d]];
      }
      __syncthreads();
    }
    float* gout = a.pos_out + b0 * (int64_t)Tout * ndo;
    for (int e = tid; e < nb * Tout * ndo; e += NTHREADS) {
      const int j = e / (Tout * ndo), r = e - j * Tout * ndo, t = r / ndo, c = r - t * ndo;
      const int d = col2d[c];
      float acc = 0.0f;
      if (d >= 0) {
        const int kind = (d < nj) ? 0 : 1;
        const float* Phr = a.basis + (b0 + j) * a.basis_sb + (int64_t)kind * Tout * N + (int64_t)t * N;
        const float* Wr = pb + (j * D + d) * Np4;
        for (int n = 0; n < N; ++n) acc = fmaf(Phr[n], Wr[n], acc);
      }
      if (L.stage) ob[e] = acc; else gout[e] = acc;
    }
    __syncthreads();
    if (L.stage) store_out(gout, ob, nb * Tout * ndo);   // (per-row path: DynShape)
  }
}

// ----------------------------------------------------------------- launch --
// Diagnostic knob: BEAST_DEBUG_PHASES=<bitmask> skips kernel phases (1 stage, 2 MFMA,
// 4 store, 8 quantise, 16 dequantise) to attribute time; default: all phases.
int debug_phases() {
  static const int v = [] {
    const char* e = getenv("BEAST_DEBUG_PHASES");
    return e ? atoi(e) : 0xFF;
  }();
  return v;
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// Diagnostic knob: BEAST_DEBUG_GRID_CAP=<n> caps the codec grids (tools/stamps uses it to
// give each workgroup a second tile, i.e. to time a tile with warm instruction cache).
int64_t debug_grid_cap() {
  static const int64_t v = [] {
    const char* e = getenv("BEAST_DEBUG_GRID_CAP");
    return e ? std::max<int64_t>(1, atoll(e)) : INT64_MAX;
  }();
  return v;
}

int64_t grid_for(int64_t ntiles, int lds_bytes) {
  const int per_cu = std::max(1, std::min(8, (160 * 1024) / std::max(lds_bytes, 1)));
  const int64_t g = std::min<int64_t>(ntiles, (int64_t)cu_count() * per_cu * 2);
  return std::max<int64_t>(1, std::min(g, debug_grid_cap()));
}

// Diagnostic / test knob (beast_set_option): run the runtime-shape kernels even where a
// specialised one exists.
bool g_generic_only = false;

// Specialised 14-DoF kernels come in two widths.  A batch that gives every CU at most two
// tiles is latency-bound: 7 waves, one MFMA column tile each, shorten a workgroup's critical
// path.  Larger batches want more tiles in flight per CU: 4 waves (two column tiles each)
// fit 4 workgroups per CU where 7-wave ones fit 2.  beast_set_option(BEAST_OPT_BLOCK_WAVES,
// 4 | 7) forces one (tests, measurements); 0 = by batch size.
int g_block_waves = 0;
bool wide_blocks(int64_t ntiles) {
  if (g_block_waves == 4 || g_block_waves == 7 || g_block_waves == 8) return g_block_waves != 4;
  return ntiles <= 2 * (int64_t)cu_count();
}
// The per-trajectory kernels (k_encode_v, k_reconstruct_v) for the fixed shapes: encode at every
// batch size, reconstruct in the latency regime (its 4-wave kernel is as fast for bulk launches,
// profiles/r05/).  BEAST_OPT_BLOCK_WAVES 4 / 7 forces the 4- / 7-wave k_encode / k_reconstruct, 8
// the per-trajectory kernels at any batch size.
bool enc_v() { return g_block_waves == 0 || g_block_waves == 8; }

// Host launch of a hot kernel through hipModuleLaunchKernel with a cached function handle (per
// device): the runtime skips hipLaunchKernel's host-function lookup and the GGL template's
// argument packing, ≈0.15 us of host time per launch (profiles/r02/launch_host_cost.json).
// The handle is the one of the STREAM's device: a tokenizer on cuda:1 may be called while another
// device is current (hipGetFuncBySymbol resolves for the current device, so it is looked up under
// a guard that makes the stream's device current).  Cache entries are atomics: the first launches
// on a device may race from several host threads, and every racer stores the same handle.
template <class... Args>
int launch_fn(const void* kernel, std::atomic<hipFunction_t> (&cache)[16], unsigned grid, unsigned block,
              unsigned lds, hipStream_t s, const char* what, Args... args) {
  int dev = 0;
  BEAST_HIP(hipStreamGetDevice(s, &dev), what);
  hipFunction_t f = (dev >= 0 && dev < 16) ? cache[dev].load(std::memory_order_acquire) : nullptr;
  if (f == nullptr) {
    int cur = 0;
    BEAST_HIP(hipGetDevice(&cur), what);
    if (cur != dev) BEAST_HIP(hipSetDevice(dev), what);
    const hipError_t e = hipGetFuncBySymbol(&f, kernel);
    if (cur != dev) BEAST_HIP(hipSetDevice(cur), what);
    BEAST_HIP(e, what);
    if (dev >= 0 && dev < 16) cache[dev].store(f, std::memory_order_release);
  }
  void* params[] = {static_cast<void*>(&args)...};
  BEAST_HIP(hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, lds, s, params, nullptr), what);
  return BEAST_OK;
}

template <class S, int W, int SP>
int launch_encode_vw(EncArgs a, hipStream_t s) {
  constexpr EvSmem L = ev_smem<S, W>(S::NJ < S::D ? 2 : 1);
  static_assert(L.total <= (W <= 8 ? 80 : 160) * 1024, "k_encode_v LDS");
  a.g = make_geom<W>(S::D, S::NJ, S::N, S::T);
  a.ntiles = (a.B + W - 1) / W;
  static std::atomic<hipFunction_t> fn[16] = {};
  return launch_fn(reinterpret_cast<const void*>(&k_encode_v<S, SP, W>), fn, (unsigned)a.ntiles, W * 64, L.total, s,
                   "k_encode_v", a.traj, a.B,
                   EncVArgs{a.dof_src, a.proj, a.w_min, a.w_max, a.tokens_out, a.params_out, a.tok_offset, a.vocab,
                            a.phases});
}

// write-through stores and RV_WE-wave tiles in the latency regime (at most one 16-trajectory tile
// per CU), write-back stores and 8-wave tiles for bulk launches
template <class S>
int launch_encode_v(EncArgs a, hipStream_t s) {
  const bool lat = a.B <= 16 * (int64_t)cu_count();
  return lat ? launch_encode_vw<S, RV_WE, LAT_SP>(a, s) : launch_encode_vw<S, RV_WE_BULK, 0>(a, s);
}

template <int TBT, class S>
int launch_encode_t(EncArgs a, int T, int D, int nj, int N, bool fast, hipStream_t s) {
  a.g = make_geom<TBT>(D, nj, N, T);
  a.ntiles = (a.B + TBT - 1) / TBT;
  const int Dl = fast ? a.row_elems : D;
  const EncSmem L = enc_smem<TBT>(T, a.g.Tp, Dl, D, N, nj < D ? 2 : 1);
  BEAST_REQUIRE_CODE(L.total <= 160 * 1024, BEAST_E_UNSUPPORTED, "encode tile needs %d B of LDS", L.total);
  const int64_t grid = grid_for(a.ntiles, L.total);
  if (fast) hipLaunchKernelGGL((k_encode<TBT, true, S>), dim3(grid), dim3(S::W * 64), L.total, s, a);
  else hipLaunchKernelGGL((k_encode<TBT, false, S>), dim3(grid), dim3(S::W * 64), L.total, s, a);
  BEAST_LAUNCHED("k_encode");
  return BEAST_OK;
}

// Tile size: the largest of 8/4/2/1 trajectories whose rows fit 32 KB of LDS
// (BEAST_ENC_TBT overrides, for measurements).  The BEAST default shapes (T = 50,
// N = 10, D = 14 with 0 or 2 gripper DoF, D = 7) run fully specialised kernels.
int launch_encode(EncArgs a, int T, int D, int nj, int N, hipStream_t s) {
  const int64_t traj_bytes = (int64_t)T * a.row_elems * 4;
  const bool contiguous = a.sd == 1 && a.st == a.row_elems && a.sb == (int64_t)T * a.row_elems &&
                          (((uintptr_t)a.traj) & 15) == 0 && ((int64_t)T * a.row_elems) % 4 == 0;
  static const int forced = [] {
    const char* e = getenv("BEAST_ENC_TBT");
    return e ? atoi(e) : 0;
  }();
  int tbt = 8;
  while (tbt > 1 && tbt * traj_bytes > 32 * 1024) tbt >>= 1;
  const bool fast = contiguous && tbt * traj_bytes <= 32 * 1024;
  if (!fast) tbt = 8;
  if (forced == 1 || forced == 2 || forced == 4 || (forced == 8 && fast)) tbt = std::min(tbt, forced);
  // list mode: the contiguous DMA path only, tiles of one batch each
  BEAST_REQUIRE(!a.traj_list || (fast && a.list_rows % tbt == 0),
                "encode list: rows must be contiguous and rows per batch a multiple of %d", tbt);
  if (fast && tbt == 8 && !g_generic_only && T == 50 && N == 10 && a.row_elems == D) {
    const bool wide = wide_blocks((a.B + 7) / 8);
    // k_encode_v stores its outputs with unconditional 16-byte stores: other alignments take k_encode
    const bool out16 = (((uintptr_t)a.params_out | (uintptr_t)a.tokens_out) & 15) == 0;
    if (!a.traj_list && enc_v() && out16) {
      if (D == 14 && nj == 14) return launch_encode_v<Shape<14, 14, 10, 50, 14>>(a, s);
      if (D == 14 && nj == 12) return launch_encode_v<Shape<14, 12, 10, 50, 14>>(a, s);
    }
    if (D == 14 && nj == 14)
      return wide ? launch_encode_t<8, Shape<14, 14, 10, 50, 14, 7>>(a, T, D, nj, N, true, s)
                  : launch_encode_t<8, Shape<14, 14, 10, 50, 14>>(a, T, D, nj, N, true, s);
    if (D == 14 && nj == 12)
      return wide ? launch_encode_t<8, Shape<14, 12, 10, 50, 14, 7>>(a, T, D, nj, N, true, s)
                  : launch_encode_t<8, Shape<14, 12, 10, 50, 14>>(a, T, D, nj, N, true, s);
    if (D == 7 && nj == 7) return launch_encode_t<8, Shape<7, 7, 10, 50, 7>>(a, T, D, nj, N, true, s);
  }
  switch (tbt) {
    case 1: return launch_encode_t<1, DynShape>(a, T, D, nj, N, fast, s);
    case 2: return launch_encode_t<2, DynShape>(a, T, D, nj, N, fast, s);
    case 4: return launch_encode_t<4, DynShape>(a, T, D, nj, N, fast, s);
    default: return launch_encode_t<8, DynShape>(a, T, D, nj, N, fast, s);
  }
}

template <int TBT, int KS, int RT, class S = DynShape>
int launch_rec_ks(RecArgs a, int D, int nj, hipStream_t s) {
  const RecSmem L = rec_smem<TBT, KS, RT>(a.Tout, D, a.g.N, a.ndo, nj < D ? 2 : 1, a.lut_n);
  BEAST_REQUIRE_CODE(L.total <= 160 * 1024, BEAST_E_UNSUPPORTED, "reconstruct tile needs %d B of LDS", L.total);
  const int64_t grid = grid_for(a.ntiles, L.total);
  if constexpr (KS == 0) hipLaunchKernelGGL((k_reconstruct_rows<TBT>), dim3(grid), dim3(NTHREADS), L.total, s, a);
  else {
    static std::atomic<hipFunction_t> fn[16] = {};
    return launch_fn(reinterpret_cast<const void*>(&k_reconstruct<TBT, KS, RT, S>), fn, (unsigned)grid, S::W * 64,
                     L.total, s, "k_reconstruct",
                     a.ntokens ? static_cast<const void*>(a.ntokens) : static_cast<const void*>(a.tokens), a.B,
                     a.ntokens ? 4 : 8, a);
  }
  BEAST_LAUNCHED("k_reconstruct");
  return BEAST_OK;
}

template <int TBT, int RT>
int launch_rec_mfma(RecArgs a, int D, int nj, int N, hipStream_t s) {
  switch ((N + 3) / 4) {
    case 1: return launch_rec_ks<TBT, 1, RT>(a, D, nj, s);
    case 2: return launch_rec_ks<TBT, 2, RT>(a, D, nj, s);
    case 3: return launch_rec_ks<TBT, 3, RT>(a, D, nj, s);
    default: return launch_rec_ks<TBT, 4, RT>(a, D, nj, s);
  }
}

// k_reconstruct_v takes the latency regime's fixed shapes unless BEAST_OPT_BLOCK_WAVES forces
// the 7-wave (or 4-wave) k_reconstruct; positions only (no params_out), int64 tokens, one tile
// per workgroup
bool rec_v(const RecArgs& a) {
  return (g_block_waves == 8 || (g_block_waves == 0 && a.ntiles <= 2 * (int64_t)cu_count())) &&
         a.params_out == nullptr && a.ntokens == nullptr && (((uintptr_t)a.pos_out) & 15) == 0;
}

template <class S>
int launch_rec_v(RecArgs a, hipStream_t s) {
  constexpr int KS = (S::N + 3) / 4;
  constexpr RvSmem L = rv_smem<S>(S::NJ < S::D ? 2 : 1);
  static_assert(L.total <= (RV_WR <= 8 ? 64 : 160) * 1024, "k_reconstruct_v LDS");
  a.tbt = RV_WR;
  a.ntiles = (a.B + RV_WR - 1) / RV_WR;
  static std::atomic<hipFunction_t> fn[2][16] = {};
  const bool lat = a.B <= 16 * (int64_t)cu_count();   // <= 2 eight-trajectory tiles per CU
  return launch_fn(lat ? reinterpret_cast<const void*>(&k_reconstruct_v<KS, S, LAT_SP>)
                       : reinterpret_cast<const void*>(&k_reconstruct_v<KS, S, 0>),
                   fn[lat ? 1 : 0], (unsigned)a.ntiles, RV_WR * 64, L.total, s, "k_reconstruct_v",
                   static_cast<const void*>(a.tokens), a.B, 8,
                   RecVArgs{a.w_min, a.w_max, a.basis, a.dof_dst, a.init_p, a.init_p_src, a.pos_out, a.tok_offset,
                            a.init_p_sb, a.vocab, a.lut_n, a.phases});
}

template <int TBT>
int launch_reconstruct(RecArgs a, int D, int nj, int N, bool shared, hipStream_t s) {
  a.g = make_geom<TBT>(D, nj, N, 1);
  a.ntiles = (a.B + TBT - 1) / TBT;
  a.tbt = TBT;
  a.fd_row = make_fd((uint32_t)(a.Tout * a.ndo));
  a.lut_n = (a.ntokens == nullptr && a.vocab <= LUT_MAX) ? a.vocab : 0;
  const bool pos = a.pos_out != nullptr;
  // MFMA path: shared basis, positions requested, the padded output tile fits LDS
  const bool mfma = shared && pos && rec_smem<TBT, 4, 0>(a.Tout, D, N, a.ndo, 2, a.lut_n).total <= 112 * 1024;
  if (!mfma) return launch_rec_ks<TBT, 0, 0>(a, D, nj, s);
  if (a.Tout <= 16 * RT_REG) {
    if (!g_generic_only && N == 10 && a.Tout == 50 && a.ndo == D) {
      const bool wide = wide_blocks(a.ntiles);
      if (wide && rec_v(a) && D == 14 && nj == 14) return launch_rec_v<Shape<14, 14, 10, 50, 14>>(a, s);
      if (wide && rec_v(a) && D == 14 && nj == 12) return launch_rec_v<Shape<14, 12, 10, 50, 14>>(a, s);
      if (D == 14 && nj == 14)
        return wide ? launch_rec_ks<TBT, 3, RT_REG, Shape<14, 14, 10, 50, 14, 7>>(a, D, nj, s)
                    : launch_rec_ks<TBT, 3, RT_REG, Shape<14, 14, 10, 50, 14>>(a, D, nj, s);
      if (D == 14 && nj == 12)
        return wide ? launch_rec_ks<TBT, 3, RT_REG, Shape<14, 12, 10, 50, 14, 7>>(a, D, nj, s)
                    : launch_rec_ks<TBT, 3, RT_REG, Shape<14, 12, 10, 50, 14>>(a, D, nj, s);
      if (D == 7 && nj == 7) return launch_rec_ks<TBT, 3, RT_REG, Shape<7, 7, 10, 50, 7>>(a, D, nj, s);
    }
    return launch_rec_mfma<TBT, RT_REG>(a, D, nj, N, s);
  }
  return launch_rec_mfma<TBT, 0>(a, D, nj, N, s);
}


}  // namespace

// =================================================================== C-ABI ==
extern "C" int beast_encode_f32(const float* traj, int64_t B, int T, int64_t sb, int64_t st, int64_t sd,
                                int row_elems, int D, int n_joint, const int32_t* dof_src, const float* proj,
                                int N, const float* w_min, const float* w_max, int vocab, int64_t tok_offset,
                                float* params_out, int64_t* tokens_out, void* stream) {
  BEAST_REQUIRE(traj && dof_src && proj, "beast_encode_f32: null input pointer");
  BEAST_REQUIRE(params_out || tokens_out, "beast_encode_f32: no output requested");
  BEAST_REQUIRE(T >= 1 && T <= MAX_T, "seq_len T=%d outside [1, %d]", T, MAX_T);
  BEAST_REQUIRE(N >= 1 && N <= MAX_N, "num_basis N=%d outside [1, %d]", N, MAX_N);
  BEAST_REQUIRE(D >= 1 && D <= MAX_D && n_joint >= 0 && n_joint <= D, "bad DoF split D=%d n_joint=%d", D, n_joint);
  BEAST_REQUIRE(row_elems >= 1, "row_elems must be >= 1");
  BEAST_REQUIRE(!tokens_out || (w_min && w_max && vocab >= 2), "quantisation needs w_min/w_max and vocab >= 2");
  BEAST_REQUIRE(B >= 0, "batch size B=%lld must be >= 0", (long long)B);
  if (B == 0) return BEAST_OK;
  EncArgs a{};
  a.traj = traj; a.B = B; a.sb = sb; a.st = st; a.sd = sd; a.row_elems = row_elems; a.vocab = vocab;
  a.phases = debug_phases(); a.dof_src = dof_src; a.proj = proj; a.w_min = w_min; a.w_max = w_max;
  a.tok_offset = tok_offset; a.params_out = params_out; a.tokens_out = reinterpret_cast<long long*>(tokens_out);
  return launch_encode(a, T, D, n_joint, N, beast::as_stream(stream));
}

extern "C" int beast_encode_list_f32(const float* const* traj_list, int nbatch, int64_t rows_per_batch, int T,
                                     int row_elems, int D, int n_joint, const int32_t* dof_src, const float* proj,
                                     int N, float* params_out, void* stream) {
  BEAST_REQUIRE(traj_list && dof_src && proj && params_out, "beast_encode_list_f32: null pointer");
  BEAST_REQUIRE(nbatch >= 0 && rows_per_batch >= 0, "beast_encode_list_f32: negative sizes");
  BEAST_REQUIRE(rows_per_batch % 8 == 0, "rows_per_batch=%lld is not a multiple of 8", (long long)rows_per_batch);
  BEAST_REQUIRE(T >= 1 && T <= MAX_T, "seq_len T=%d outside [1, %d]", T, MAX_T);
  BEAST_REQUIRE(N >= 1 && N <= MAX_N, "num_basis N=%d outside [1, %d]", N, MAX_N);
  BEAST_REQUIRE(D >= 1 && D <= MAX_D && n_joint >= 0 && n_joint <= D, "bad DoF split D=%d n_joint=%d", D, n_joint);
  BEAST_REQUIRE(row_elems >= 1 && ((int64_t)T * row_elems) % 4 == 0,
                "beast_encode_list_f32: T*row_elems must be a multiple of 4");
  if (nbatch == 0 || rows_per_batch == 0) return BEAST_OK;
  EncArgs a{};
  a.traj = nullptr; a.traj_list = traj_list; a.list_rows = rows_per_batch;
  a.B = (int64_t)nbatch * rows_per_batch; a.sb = (int64_t)T * row_elems; a.st = row_elems; a.sd = 1;
  a.row_elems = row_elems; a.vocab = 0; a.phases = debug_phases(); a.dof_src = dof_src; a.proj = proj;
  a.params_out = params_out;
  return launch_encode(a, T, D, n_joint, N, beast::as_stream(stream));
}

extern "C" int beast_reconstruct_f32(const int64_t* tokens, int64_t B, int D, int n_joint, int N, int vocab,
                                     int64_t tok_offset, const float* w_min, const float* w_max,
                                     const float* basis, int64_t basis_sb, int T_out, const int32_t* dof_dst,
                                     int num_dof_out, const float* init_p, int64_t init_p_sb,
                                     const int32_t* init_p_src, float* params_out, float* pos_out,
                                     const float* ntokens, void* stream) {
  BEAST_REQUIRE((tokens || ntokens) && w_min && w_max, "beast_reconstruct_f32: null input pointer");
  BEAST_REQUIRE(params_out || pos_out, "beast_reconstruct_f32: no output requested");
  BEAST_REQUIRE(N >= 1 && N <= MAX_N, "num_basis N=%d outside [1, %d]", N, MAX_N);
  BEAST_REQUIRE(D >= 1 && D <= MAX_D && n_joint >= 0 && n_joint <= D, "bad DoF split D=%d n_joint=%d", D, n_joint);
  BEAST_REQUIRE(vocab >= 2 || ntokens, "vocab must be >= 2");
  BEAST_REQUIRE(!pos_out || (basis && dof_dst && T_out >= 1 && T_out <= 4096 && num_dof_out >= D &&
                             num_dof_out <= 4096),
                "reconstruct: need basis, dof_dst, 1 <= T_out <= 4096, D <= num_dof_out <= 4096");
  BEAST_REQUIRE(!init_p || init_p_src, "init_p needs init_p_src");
  BEAST_REQUIRE(B >= 0, "batch size B=%lld must be >= 0", (long long)B);
  if (B == 0) return BEAST_OK;
  RecArgs a{};
  a.tokens = reinterpret_cast<const long long*>(tokens); a.ntokens = ntokens; a.B = B; a.tok_offset = tok_offset;
  a.basis_sb = basis_sb; a.init_p_sb = init_p_sb; a.vocab = vocab; a.Tout = pos_out ? T_out : 1;
  a.ndo = pos_out ? num_dof_out : 1; a.phases = debug_phases(); a.w_min = w_min; a.w_max = w_max; a.basis = basis;
  a.dof_dst = dof_dst; a.init_p = init_p; a.init_p_src = init_p_src; a.params_out = params_out; a.pos_out = pos_out;
  const bool shared = (basis_sb == 0);
  return launch_reconstruct<8>(a, D, n_joint, N, shared, beast::as_stream(stream));
}

#ifdef BEAST_STAMPS
extern "C" int beast_stamps_read(unsigned long long* out) {   // [2][8][16]
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) == hipSuccess ? 0 : -2;
}

extern "C" int beast_bstamps_read(unsigned long long* out) {   // [2][4096][4]
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bstamps), sizeof(g_bstamps)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int beast_set_option(int option, int value) {
  if (option == BEAST_OPT_GENERIC_KERNELS) {
    g_generic_only = value != 0;
    return BEAST_OK;
  }
  if (option == BEAST_OPT_BLOCK_WAVES) {
    BEAST_REQUIRE(value == 0 || value == 4 || value == 7 || value == 8,
                  "BEAST_OPT_BLOCK_WAVES: %d is not 0, 4, 7 or 8", value);
    g_block_waves = value;
    return BEAST_OK;
  }
  if (option == BEAST_OPT_MERGE_LDS_MIN) {
    BEAST_REQUIRE(value >= 0, "BEAST_OPT_MERGE_LDS_MIN: %d < 0", value);
    beast::g_merge_lds_min = value;
    return BEAST_OK;
  }
  if (option == BEAST_OPT_BPE_ENCODE_MODE) {
    BEAST_REQUIRE(value >= 0 && value <= 3, "BEAST_OPT_BPE_ENCODE_MODE: %d is not 0..3", value);
    beast::g_bpe_encode_mode = value;
    return BEAST_OK;
  }
  if (option == BEAST_OPT_BPE_DEDUP_KEY_BITS) {
    BEAST_REQUIRE(value >= 2 && value <= 64, "BEAST_OPT_BPE_DEDUP_KEY_BITS: %d is not 2..64", value);
    beast::g_bpe_dedup_key_bits = value;
    return BEAST_OK;
  }
  if (option == BEAST_OPT_BPE_TRAIN_HOST_LOOP) {
    BEAST_REQUIRE(value >= 0 && value <= 2, "BEAST_OPT_BPE_TRAIN_HOST_LOOP: %d is not 0..2", value);
    beast::g_bpe_train_host = value;
    return BEAST_OK;
  }
  BEAST_REQUIRE(false, "unknown option %d", option);
  return BEAST_E_INVALID;
}

extern "C" int beast_get_option(int option) {
  if (option == BEAST_OPT_GENERIC_KERNELS) return g_generic_only ? 1 : 0;
  if (option == BEAST_OPT_BLOCK_WAVES) return g_block_waves;
  if (option == BEAST_OPT_MERGE_LDS_MIN) return (int)beast::g_merge_lds_min;
  if (option == BEAST_OPT_BPE_ENCODE_MODE) return beast::g_bpe_encode_mode;
  if (option == BEAST_OPT_BPE_DEDUP_KEY_BITS) return beast::g_bpe_dedup_key_bits;
  if (option == BEAST_OPT_BPE_TRAIN_HOST_LOOP) return beast::g_bpe_train_host;
  beast::set_error("unknown option %d", option);
  return BEAST_E_INVALID;
}
