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

#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int NTHREADS = 256;
constexpr int NWAVES = NTHREADS / 64;
constexpr int MAX_T = 256;
constexpr int MAX_N = 16;
constexpr int MAX_D = 64;
constexpr int TILES = 4;  // independent MFMA accumulation chains per wave

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

// LDS -> global, float count
__device__ __forceinline__ void store_out(float* __restrict__ dst, const float* __restrict__ src, int count) {
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int n4 = count >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int i = threadIdx.x; i < n4; i += NTHREADS) d4[i] = s4[i];
    for (int i = (n4 << 2) + threadIdx.x; i < count; i += NTHREADS) dst[i] = src[i];
  } else {
    for (int i = threadIdx.x; i < count; i += NTHREADS) dst[i] = src[i];
  }
}

// LDS-DMA (global_load_lds): HBM -> LDS with no VGPR round trip, so every load of a stage
// is in flight at once and one vmcnt wait (the next __syncthreads) retires them all.  A
// wave-instruction writes 64 consecutive slots from a wave-uniform base: destinations are
// padded to whole wave-instructions, sources past the end are clamped to the last element.
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(void* lds, const void* g, int n16) {
  const int tid = threadIdx.x, wb = tid & ~63;
  for (int base = 0; base < n16; base += NTHREADS) {
    if (base + wb < n16)
      __builtin_amdgcn_global_load_lds(static_cast<const uint4*>(g) + min(base + tid, n16 - 1),
                                       (lds_void*)(static_cast<uint4*>(lds) + base + wb), 16, 0, 0);
  }
}

__device__ __forceinline__ void dma4(void* lds, const void* g, int n) {
  const int tid = threadIdx.x, wb = tid & ~63;
  for (int base = 0; base < n; base += NTHREADS) {
    if (base + wb < n)
      __builtin_amdgcn_global_load_lds(static_cast<const uint32_t*>(g) + min(base + tid, n - 1),
                                       (lds_void*)(static_cast<uint32_t*>(lds) + base + wb), 4, 0, 0);
  }
}

// -------------------------------------------------------------- geometry --
struct Geom {
  int D, nj, N, T, Tp, per;   // per = N * D
  int nq0, nq;                // column tiles of kind 0, of both kinds
  FastDiv fd_nj, fd_ng, fd_per, fd_N, fd_nq;
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
  g.fd_nq = make_fd(std::max(g.nq, 1));
  return g;
}

// MFMA column (trajectory j, DoF d) of tile q for lane column lc; valid = inside the tile set.
template <int TBT>
__device__ __forceinline__ void tile_col(const Geom& g, int q, int lc, int& j, int& d, int& kind, bool& valid) {
  const int k0 = q < g.nq0 ? 0 : 1;
  const int dk = k0 ? g.D - g.nj : g.nj;
  const int c = (q - (k0 ? g.nq0 : 0)) * 16 + lc;
  valid = c < TBT * dk;
  const uint32_t cc = valid ? c : TBT * dk - 1;
  const uint32_t jj = fdiv(cc, k0 ? g.fd_ng : g.fd_nj);
  j = (int)jj;
  d = (int)(cc - jj * dk) + (k0 ? g.nj : 0);
  kind = k0;
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
};

struct EncSmem {
  int P, Y, pb, wlo, whi, kmap, lcol, total;
};

// Every buffer an LDS-DMA fills is padded to whole wave-instructions (64 lanes x 16 B).
template <int TBT>
__host__ __device__ inline EncSmem enc_smem(int T, int Tp, int Dl, int D, int N, int nkinds) {
  EncSmem s;
  int o = 0;
  s.P = o;    o += round_up(nkinds * 16 * Tp * 4, 1024);   // fp32 [16][Tp] projection per kind
  s.Y = o;    o += round_up(TBT * T * Dl * 4, 1024);
  s.pb = o;   o += round_up(TBT * D * N * 4, 16);
  s.wlo = o;  o += round_up(D * N * 4, 256);
  s.whi = o;  o += round_up(D * N * 4, 256);
  s.kmap = o; o += round_up(D * N * 2, 16);
  s.lcol = o; o += round_up(D * 4, 256);
  s.total = o;
  return s;
}

template <int TBT, bool FAST>
__global__ __launch_bounds__(NTHREADS) void k_encode(EncArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Geom& g = a.g;
  const int D = g.D, N = g.N, T = g.T, Tp = g.Tp, per = g.per, DN = D * N;
  const int Dl = FAST ? a.row_elems : D;
  const int nkinds = (g.nj < D) ? 2 : 1;
  const EncSmem L = enc_smem<TBT>(T, Tp, Dl, D, N, nkinds);
  float* P = reinterpret_cast<float*>(smem + L.P);
  float* Y = reinterpret_cast<float*>(smem + L.Y);
  float* pb = reinterpret_cast<float*>(smem + L.pb);
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  uint16_t* kmap = reinterpret_cast<uint16_t*>(smem + L.kmap);
  int* lcol = reinterpret_cast<int*>(smem + L.lcol);
  const int tid = threadIdx.x;
  const bool quant = a.tokens_out != nullptr;
  const int tile_elems = T * a.row_elems;   // FAST: one trajectory, contiguous, % 4 == 0

  // ---- prologue: the first tile and every constant go HBM -> LDS by DMA in one round trip
  if (FAST && (a.phases & 1) && blockIdx.x < a.ntiles) {
    const int64_t b0 = (int64_t)blockIdx.x * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);
    dma16(Y, a.traj + b0 * a.sb, (nb * tile_elems) >> 2);
  }
  dma16(P, a.proj, nkinds * 4 * Tp);
  if (quant) {
    dma4(wlo, a.w_min, DN);
    dma4(whi, a.w_max, DN);
  }
  dma4(lcol, a.dof_src, D);
  for (int r = tid; r < per; r += NTHREADS) {   // (n d) slot -> (d n) index
    const int n = r / D, d = r - n * D;
    kmap[r] = (uint16_t)(d * N + n);
  }

  const int wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;
  const float vm1 = (float)(a.vocab - 1);

  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);

    // ---- the trajectory tile lands in LDS (the first one is already in flight)
    if (a.phases & 1) {
      if (FAST) {
        if (tile != blockIdx.x) dma16(Y, a.traj + b0 * a.sb, (nb * tile_elems) >> 2);
      } else {
        const int pt = T * D;
        for (int e = tid; e < nb * pt; e += NTHREADS) {
          const int j = e / pt, r = e - j * pt, t = r / D, d = r - t * D;
          const int col = a.dof_src[d];
          Y[e] = (col >= 0 && col < a.row_elems)
                     ? a.traj[(b0 + j) * a.sb + (int64_t)t * a.st + (int64_t)col * a.sd] : 0.0f;
        }
      }
    }
    __syncthreads();   // waits for the DMA (vmcnt) and the LDS stores

    // ---- fit: params[j][d][n] = sum_t P_kind[n][t] y[j][t][d]  (f32 MFMA 16x16x4; A = P, B = y).
    //      A wave owns two column tiles per pass (two independent chains), operands
    //      pointer-stepped through LDS; rows t >= T (tail step) meet a zero A column.
    for (int q0 = wave; (a.phases & 2) && q0 < g.nq; q0 += NWAVES * 2) {
      int j0, d0, k0, j1, d1, k1;
      bool ok0, ok1;
      tile_col<TBT>(g, q0, lr, j0, d0, k0, ok0);
      tile_col<TBT>(g, min(q0 + NWAVES, g.nq - 1), lr, j1, d1, k1, ok1);
      ok0 = ok0 && j0 < nb;
      ok1 = ok1 && j1 < nb && (q0 + NWAVES < g.nq);
      const int c0 = FAST ? min(max(lcol[d0], 0), Dl - 1) : d0;
      const int c1 = FAST ? min(max(lcol[d1], 0), Dl - 1) : d1;
      const float* pa0 = P + (k0 * 16 + lr) * Tp + lk;
      const float* pa1 = P + (k1 * 16 + lr) * Tp + lk;
      const float* yc0 = Y + j0 * T * Dl + c0;
      const float* yc1 = Y + j1 * T * Dl + c1;
      const float* yb0 = yc0 + lk * Dl;
      const float* yb1 = yc1 + lk * Dl;
      float4_t acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
      int s = 0;
#pragma unroll 4
      for (; s + 4 <= T; s += 4) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa0[s], *yb0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa1[s], *yb1, acc1, 0, 0, 0);
        yb0 += 4 * Dl;
        yb1 += 4 * Dl;
      }
      if (s < T) {   // wave-uniform tail (T % 4 != 0)
        const int row = min(s + lk, T - 1) * Dl;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa0[s], yc0[row], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa1[s], yc1[row], acc1, 0, 0, 0);
      }
      // f32 C/D map: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = lk * 4 + r;
        if (n < N) {
          if (ok0) pb[j0 * DN + d0 * N + n] = acc0[r];
          if (ok1) pb[j1 * DN + d1 * N + n] = acc1[r];
        }
      }
    }
    __syncthreads();

    // ---- epilogue: params (d n) and tokens (n d), both contiguous per tile
    if (a.params_out != nullptr && (a.phases & 4)) store_out(a.params_out + b0 * DN, pb, nb * DN);
    if (quant && (a.phases & 8)) {
      const int total = nb * per;
      long long* tout = a.tokens_out + b0 * per;
      const bool vec = ((((uintptr_t)tout) & 15) == 0);
      for (int e2 = tid; 2 * e2 < total; e2 += NTHREADS) {
        long long v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t e = min(2 * e2 + h, total - 1);
          const uint32_t j = fdiv(e, g.fd_per);
          const int k = kmap[e - j * per];
          const float lo = wlo[k], hi = whi[k];
          float sc = __fsub_rn(hi, lo);
          sc = (sc < 1e-8f) ? 1e-8f : sc;   // torch.clamp(max - min, min=1e-8), NaN kept
          v[h] = beast::quantize_scaled(pb[j * DN + k], lo, hi, sc, vm1) + a.tok_offset;
        }
        if (vec && 2 * e2 + 1 < total) {
          *reinterpret_cast<longlong2*>(tout + 2 * e2) = make_longlong2(v[0], v[1]);
        } else {
          tout[2 * e2] = v[0];
          if (2 * e2 + 1 < total) tout[2 * e2 + 1] = v[1];
        }
      }
    }
  }
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

constexpr int LUT_MAX = 4096;   // dequantise LUT tok / (vocab - 1), IEEE-divided once

struct RecSmem {
  int phi, pb, tok, wlo, whi, lut, pmap, kq, kpb, dst, col2d, out, total;
  int Np4, RTR;   // padded basis width, padded output rows
  bool stage;
};

// token tile [nb][per] (int64, or fp32 normalised tokens) HBM -> LDS by DMA
__device__ __forceinline__ void stage_tokens(const RecArgs& a, void* lds, int64_t b0, int per) {
  const int nb = (int)min<int64_t>(a.B - b0, 1 << 30);
  const void* src = a.ntokens ? static_cast<const void*>(a.ntokens + b0 * per)
                              : static_cast<const void*>(a.tokens + b0 * per);
  const int bytes = min(nb, a.tbt) * per * (a.ntokens ? 4 : 8);
  if ((bytes & 15) == 0 && (((uintptr_t)src) & 15) == 0) dma16(lds, src, bytes >> 4);
  else dma4(lds, src, bytes >> 2);
}

// KS > 0: shared basis on MFMA (K-steps of 4 basis functions); KS == 0: per-row basis on VALU
template <int TBT, int KS>
__host__ __device__ inline RecSmem rec_smem(int Tout, int D, int N, int ndo, int nkinds, int lut_n) {
  RecSmem s;
  const int per = N * D;
  s.Np4 = KS ? 4 * KS : round_up(N, 4);
  s.RTR = KS ? round_up(Tout, 32) : Tout;   // even number of 16-row tiles
  int o = 0;
  s.phi = o;   o += KS ? round_up(nkinds * s.RTR * s.Np4 * 4, 16) : 0;
  s.pb = o;    o += round_up(TBT * D * s.Np4 * 4, 16);
  s.tok = o;   o += round_up(TBT * per * 8, 1024);   // DMA destinations: whole wave-instructions
  s.wlo = o;   o += round_up(per * 4, 256);
  s.whi = o;   o += round_up(per * 4, 256);
  s.lut = o;   o += round_up(lut_n * 4, 16);
  s.pmap = o;  o += round_up(per * 2, 16);   // (n d) slot -> W offset d*Np4 + n
  s.kq = o;    o += round_up(per * 2, 16);   // (n d) slot -> (d n) index d*N + n
  s.kpb = o;   o += round_up(per * 2, 16);   // (d n) index -> W offset
  s.dst = o;   o += round_up(D * 4, 256);
  s.col2d = o; o += round_up(ndo * 4, 16);
  const int outb = round_up(TBT * s.RTR * ndo * 4, 16);
  s.stage = KS ? true : (o + outb) <= 96 * 1024;
  s.out = o;   o += s.stage ? outb : 0;
  s.total = o;
  return s;
}

template <int TBT, int KS>
__global__ __launch_bounds__(NTHREADS) void k_reconstruct(RecArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Geom& g = a.g;
  const int D = g.D, N = g.N, nj = g.nj, per = g.per;
  const int Tout = a.Tout, ndo = a.ndo;
  const int nkinds = (nj < D) ? 2 : 1;
  const bool pos = a.pos_out != nullptr;
  const RecSmem L = rec_smem<TBT, KS>(Tout, D, N, ndo, nkinds, a.lut_n);
  const int Np4 = L.Np4, RTR = L.RTR;
  float* phi = reinterpret_cast<float*>(smem + L.phi);
  float* pb = reinterpret_cast<float*>(smem + L.pb);
  float* wlo = reinterpret_cast<float*>(smem + L.wlo);
  float* whi = reinterpret_cast<float*>(smem + L.whi);
  float* lut = reinterpret_cast<float*>(smem + L.lut);
  uint16_t* pmap = reinterpret_cast<uint16_t*>(smem + L.pmap);
  uint16_t* kq = reinterpret_cast<uint16_t*>(smem + L.kq);
  uint16_t* kpb = reinterpret_cast<uint16_t*>(smem + L.kpb);
  int* dst = reinterpret_cast<int*>(smem + L.dst);
  int* col2d = reinterpret_cast<int*>(smem + L.col2d);
  float* ob = reinterpret_cast<float*>(smem + L.out);
  const int tid = threadIdx.x;
  const float vm1 = (float)(a.vocab - 1);

  // ---- prologue: the first token tile, the bounds and the DoF map by DMA, the
  //      padded basis by register staging -- all in flight together (one round trip)
  if ((a.phases & 1) && blockIdx.x < a.ntiles) stage_tokens(a, smem + L.tok, (int64_t)blockIdx.x * TBT, per);
  dma4(wlo, a.w_min, per);
  dma4(whi, a.w_max, per);
  if (pos) dma4(dst, a.dof_dst, D);
  if (KS && pos) {   // Phi zero-padded to [kinds][RTR][Np4]: clamped loads, then unconditional stores
    const int tot = nkinds * RTR * Np4;
    const int tn = RTR * Np4;
    for (int base = 0; base < tot; base += 8 * NTHREADS) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = min(base + u * NTHREADS + tid, tot - 1);
        const int k = i >= tn ? 1 : 0, r = i - k * tn, t = r / Np4, n = r - t * Np4;
        const float x = a.basis[(int64_t)k * Tout * N + min(t, Tout - 1) * N + min(n, N - 1)];
        // bit-mask select: x stays used on every path, so the load is not sunk into a branch
        const uint32_t keep = 0u - (uint32_t)((t < Tout) & (n < N));
        v[u] = __uint_as_float(__float_as_uint(x) & keep);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) phi[min(base + u * NTHREADS + tid, tot - 1)] = v[u];
    }
  }
  for (int t = tid; t < a.lut_n; t += NTHREADS) lut[t] = __fdiv_rn((float)t, vm1);
  for (int r = tid; r < per; r += NTHREADS) {
    const int n = r / D, d = r - n * D;
    pmap[r] = (uint16_t)(d * Np4 + n);
    kq[r] = (uint16_t)(d * N + n);
    const int d2 = r / N, n2 = r - d2 * N;
    kpb[r] = (uint16_t)(d2 * Np4 + n2);
  }
  for (int e = tid; e < TBT * D * (Np4 - N); e += NTHREADS) {   // zero W pad columns once
    const int row = e / (Np4 - N), n = N + (e - row * (Np4 - N));
    pb[row * Np4 + n] = 0.0f;
  }
  if (pos && KS == 0) {   // per-row basis path: output column -> DoF (after the DMA of dst)
    __syncthreads();
    for (int c = tid; c < ndo; c += NTHREADS) col2d[c] = -1;
    __syncthreads();
    if (tid < D) {
      const int dd = dst[tid];
      if (dd >= 0 && dd < ndo) col2d[dd] = tid;
    }
  }

  const int wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = lane >> 4;

  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * TBT;
    const int nb = (int)min<int64_t>(TBT, a.B - b0);

    // ---- the token tile lands in LDS (the first one is already in flight)
    if ((a.phases & 1) && tile != blockIdx.x) stage_tokens(a, smem + L.tok, b0, per);
    __syncthreads();

    // ---- decode (H6): (n d) tokens -> W[j][d][n], bit-exact discrete_to_continuous
    if (a.phases & 16) {
      const long long* tin = reinterpret_cast<const long long*>(smem + L.tok);
      const float* fin = reinterpret_cast<const float*>(smem + L.tok);
      for (int e = tid; e < nb * per; e += NTHREADS) {
        const uint32_t j = fdiv(e, g.fd_per);
        const int r = e - j * per;
        const int po = pmap[r], k = kq[r];
        float v;
        if (a.ntokens) {
          v = beast::denormalize_one(fin[e], wlo[k], whi[k]);
        } else {
          const long long t = tin[e] - a.tok_offset;
          const float nrm = (t >= 0 && t < a.lut_n) ? lut[t] : __fdiv_rn((float)t, vm1);
          const float lo = wlo[k], hi = whi[k];   // (max_val - min_val), beast/utils.py:24
          v = beast::clamp_t(__fadd_rn(__fmul_rn(nrm, __fsub_rn(hi, lo)), lo), lo, hi);
        }
        pb[j * D * Np4 + po] = v;
      }
    }
    __syncthreads();
    if (a.params_out != nullptr) {
      float* pout = a.params_out + b0 * per;
      for (int e = tid; e < nb * per; e += NTHREADS) {
        const uint32_t j = fdiv(e, g.fd_per);
        pout[e] = pb[j * D * Np4 + kpb[e - j * per]];
      }
    }
    if (!pos) continue;
    if (a.init_p != nullptr) {   // coefficient 0 of the joint DoFs <- init_p (reference :505-510)
      __syncthreads();
      for (int e = tid; e < nb * nj; e += NTHREADS) {
        const int j = e / nj, d = e - j * nj;
        pb[(j * D + d) * Np4] = a.init_p[(b0 + j) * a.init_p_sb + a.init_p_src[d]];
      }
      __syncthreads();
    }

    float* gout = a.pos_out + b0 * (int64_t)Tout * ndo;
    if constexpr (KS > 0) {
      // ---- pos[j][t][dst(d)] = sum_n Phi_kind[t][n] W[j][d][n]  (f32 MFMA 16x16x4; A = Phi, B = W).
      //      A wave owns a column tile: W stays in registers while it walks pairs of row
      //      tiles (two independent chains); rows past Tout land in ob's padding.
      for (int q = wave; (a.phases & 2) && q < g.nq; q += NWAVES) {
        int j, d, kind;
        bool ok;
        tile_col<TBT>(g, q, lr, j, d, kind, ok);
        ok = ok && j < nb;
        float w[KS];
        const float* Wc = pb + (j * D + d) * Np4 + lk;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) w[ks] = Wc[4 * ks];
        const float* Ph = phi + (kind * RTR + lr) * Np4 + lk;
        float* oc = ob + (j * RTR + lk * 4) * ndo + min(max(dst[d], 0), ndo - 1);
        for (int rt = 0; rt < RTR / 16; rt += 2) {
          float a0[KS], a1[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            a0[ks] = Ph[(rt * 16) * Np4 + 4 * ks];
            a1[ks] = Ph[(rt * 16 + 16) * Np4 + 4 * ks];
          }
          float4_t acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[ks], w[ks], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[ks], w[ks], acc1, 0, 0, 0);
          }
          // f32 C/D map: col = lane & 15, row = (lane >> 4) * 4 + r
          if (ok) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              oc[(rt * 16 + r) * ndo] = acc0[r];
              oc[(rt * 16 + 16 + r) * ndo] = acc1[r];
            }
          }
        }
      }
      __syncthreads();
      if (a.phases & 4) {   // ob rows [0, Tout) of each trajectory -> contiguous HBM tile
        const int rowlen = Tout * ndo;
        if ((rowlen & 3) == 0 && ((RTR * ndo) & 3) == 0 && ((((uintptr_t)gout) & 15) == 0)) {
          const int n4 = nb * rowlen / 4;
          for (int i = tid; i < n4; i += NTHREADS) {
            const uint32_t e = 4 * i;
            const uint32_t j = fdiv(e, a.fd_row);
            reinterpret_cast<float4*>(gout)[i] =
                *reinterpret_cast<const float4*>(ob + j * RTR * ndo + (e - j * rowlen));
          }
        } else {
          for (int e = tid; e < nb * rowlen; e += NTHREADS) {
            const uint32_t j = fdiv(e, a.fd_row);
            gout[e] = ob[j * RTR * ndo + (e - j * rowlen)];
          }
        }
      }
    } else {
      // per-trajectory basis (custom times per row): sequential fma over n, the MFMA chain's order
      for (int e = tid; (a.phases & 2) && e < nb * Tout * ndo; e += NTHREADS) {
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
      if (L.stage && (a.phases & 4)) {
        __syncthreads();
        store_out(gout, ob, nb * Tout * ndo);
      }
    }
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

int64_t grid_for(int64_t ntiles, int lds_bytes) {
  const int per_cu = std::max(1, std::min(8, (160 * 1024) / std::max(lds_bytes, 1)));
  return std::max<int64_t>(1, std::min<int64_t>(ntiles, (int64_t)cu_count() * per_cu * 2));
}

template <int TBT>
int launch_encode_t(EncArgs a, int T, int D, int nj, int N, bool fast, hipStream_t s) {
  a.g = make_geom<TBT>(D, nj, N, T);
  a.ntiles = (a.B + TBT - 1) / TBT;
  const int Dl = fast ? a.row_elems : D;
  const EncSmem L = enc_smem<TBT>(T, a.g.Tp, Dl, D, N, nj < D ? 2 : 1);
  BEAST_REQUIRE_CODE(L.total <= 160 * 1024, BEAST_E_UNSUPPORTED, "encode tile needs %d B of LDS", L.total);
  const int64_t grid = grid_for(a.ntiles, L.total);
  if (fast) hipLaunchKernelGGL((k_encode<TBT, true>), dim3(grid), dim3(NTHREADS), L.total, s, a);
  else hipLaunchKernelGGL((k_encode<TBT, false>), dim3(grid), dim3(NTHREADS), L.total, s, a);
  BEAST_LAUNCHED("k_encode");
  return BEAST_OK;
}

// Tile size: the largest of 8/4/2/1 trajectories whose rows fit 32 KB of LDS
// (BEAST_ENC_TBT overrides, for measurements).
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
  switch (tbt) {
    case 1: return launch_encode_t<1>(a, T, D, nj, N, fast, s);
    case 2: return launch_encode_t<2>(a, T, D, nj, N, fast, s);
    case 4: return launch_encode_t<4>(a, T, D, nj, N, fast, s);
    default: return launch_encode_t<8>(a, T, D, nj, N, fast, s);
  }
}

template <int TBT, int KS>
int launch_rec_ks(RecArgs a, int D, int nj, hipStream_t s) {
  const RecSmem L = rec_smem<TBT, KS>(a.Tout, D, a.g.N, a.ndo, nj < D ? 2 : 1, a.lut_n);
  BEAST_REQUIRE_CODE(L.total <= 160 * 1024, BEAST_E_UNSUPPORTED, "reconstruct tile needs %d B of LDS", L.total);
  const int64_t grid = grid_for(a.ntiles, L.total);
  hipLaunchKernelGGL((k_reconstruct<TBT, KS>), dim3(grid), dim3(NTHREADS), L.total, s, a);
  BEAST_LAUNCHED("k_reconstruct");
  return BEAST_OK;
}

template <int TBT>
int launch_reconstruct(RecArgs a, int D, int nj, int N, bool shared, hipStream_t s) {
  a.g = make_geom<TBT>(D, nj, N, 1);
  a.ntiles = (a.B + TBT - 1) / TBT;
  a.tbt = TBT;
  a.fd_row = make_fd((uint32_t)(a.Tout * a.ndo));
  a.lut_n = (a.ntokens == nullptr && a.vocab <= LUT_MAX) ? a.vocab : 0;
  const bool pos = a.pos_out != nullptr;
  // MFMA path needs the shared basis and the padded output tile in LDS
  const bool mfma = shared && pos && rec_smem<TBT, 4>(a.Tout, D, N, a.ndo, 2, a.lut_n).total <= 112 * 1024;
  if (!mfma) return launch_rec_ks<TBT, 0>(a, D, nj, s);
  switch ((N + 3) / 4) {
    case 1: return launch_rec_ks<TBT, 1>(a, D, nj, s);
    case 2: return launch_rec_ks<TBT, 2>(a, D, nj, s);
    case 3: return launch_rec_ks<TBT, 3>(a, D, nj, s);
    default: return launch_rec_ks<TBT, 4>(a, D, nj, s);
  }
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
