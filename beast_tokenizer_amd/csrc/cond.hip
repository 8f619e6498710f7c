// Boundary conditions of the joint spline (init_cond_order / end_cond_order != 0, SURVEY.md §8f
// rank 4) for gfx950: the per-call work around the fit / reconstruct kernels.
//
//   k_cond_fixed  encode side: each (trajectory, joint DoF)'s init / end conditions and the fixed
//                 control points from y[0], y[1], y[T-2], y[T-1] (compute_init_params /
//                 compute_end_params, MP_lite_PyTorch/mp_pytorch/basis_gn/uni_bspline_basis.py
//                 :192-301, as uni_bspline.py:499-550 calls them), in the reference's fp32 op order
//   k_cond_add    reconstruct side: pos[j][t][joint d] += sum_k Phi_full[t][k] ext[j][d][k]
//                 + init_pos[j][d] over the fixed columns k (get_traj_pos, uni_bspline.py:126-166,
//                 end order -1 subtracting the end term from column C-2)
// The fitted columns themselves run in the MFMA kernels of codec.hip with the conditioned
// projection (bspline.py:DeviceBasis); these replace about a dozen ATen launches per call.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace {

struct CondArgs {
  int ic, ec, p, C;
  float tau;
};

// one thread per (trajectory j, joint d)
__global__ void k_cond_fixed(const float* __restrict__ y, int64_t B, int T, int64_t sb, int64_t st, int64_t sd,
                             const int32_t* __restrict__ jidx, int dj, const float* __restrict__ times,
                             const float* __restrict__ knots, CondArgs c, float* __restrict__ init_pos,
                             float* __restrict__ init_vel, float* __restrict__ end_pos, float* __restrict__ end_vel,
                             float* __restrict__ p_init, float* __restrict__ p_end) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= B * dj) return;
  const int64_t j = i / dj;
  const int d = (int)(i - j * dj);
  const float* yr = y + j * sb + (int64_t)jidx[d] * sd;
  const float inv_dt = __fdiv_rn(1.0f, __fsub_rn(times[1], times[0]));   // 1 / (t[1] - t[0])
  const float pf = (float)c.p;
  float ip = 0.0f;
  if (c.ic) {
    const float y0 = yr[0], y1 = yr[st];
    ip = y0;
    const float iv = __fmul_rn(__fsub_rn(y1, y0), inv_dt);
    init_pos[i] = y0;
    init_vel[i] = iv;
    p_init[i * c.ic] = 0.0f;
    if (c.ic == 2) {   // init_vel * tau * dk0 / p + 0
      const float dk0 = __fsub_rn(knots[1 + c.p], knots[1]);
      p_init[i * c.ic + 1] = __fadd_rn(__fdiv_rn(__fmul_rn(__fmul_rn(iv, c.tau), dk0), pf), 0.0f);
    }
  }
  if (c.ec) {
    const float ya = yr[(int64_t)(T - 1) * st], yb = yr[(int64_t)(T - 2) * st];
    const float ev = __fmul_rn(__fsub_rn(ya, yb), inv_dt);
    const float e = c.ic ? __fsub_rn(ya, ip) : ya;   // relative to init_pos when it exists
    const int ne = c.ec < 0 ? -c.ec : c.ec;
    const float dke = __fsub_rn(knots[c.C - 1 + c.p], knots[c.C - 1]);
    const float slope = __fdiv_rn(__fmul_rn(__fmul_rn(ev, c.tau), dke), pf);   // end_vel * tau * dke / p
    if (c.ec == -1) {
      p_end[i] = slope;
    } else if (c.ec == 1) {
      p_end[i] = e;
    } else {
      p_end[i * ne] = __fsub_rn(e, slope);
      p_end[i * ne + 1] = e;
    }
    end_pos[i] = c.ic ? __fadd_rn(e, ip) : e;
    end_vel[i] = ev;
  }
}

// one thread per (trajectory j, time t, joint d); Phi_full [T][C] shared (full_sb = 0) or per
// trajectory [B][T][C].  The fixed columns in ascending order, as the einsum's sum over k (the
// other columns are zero), then + init_pos, then added to the fitted positions.
__global__ void k_cond_add(float* __restrict__ pos, int64_t B, int T, int D, const int32_t* __restrict__ jidx,
                           int dj, const float* __restrict__ full, int64_t full_sb, CondArgs c,
                           const float* __restrict__ p_init, const float* __restrict__ p_end,
                           const float* __restrict__ init_pos) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= B * T * dj) return;
  const int64_t jt = i / dj;
  const int d = (int)(i - jt * dj);
  const int64_t j = jt / T;
  const int t = (int)(jt - j * T);
  const float* ph = full + j * full_sb + (int64_t)t * c.C;
  const int64_t jd = j * dj + d;
  float acc = 0.0f;
  bool any = false;
  auto term = [&](int k, float w) {
    const float v = __fmul_rn(ph[k], w);
    acc = any ? __fadd_rn(acc, v) : v;
    any = true;
  };
  for (int k = 0; k < c.ic; ++k) term(k, p_init[jd * c.ic + k]);
  if (c.ec == -1) {
    term(c.C - 2, -p_end[jd]);
  } else if (c.ec > 0) {
    for (int q = 0; q < c.ec; ++q) term(c.C - c.ec + q, p_end[jd * c.ec + q]);
  }
  if (c.ic) acc = __fadd_rn(acc, init_pos[jd]);
  float* o = pos + jt * D + jidx[d];
  *o = __fadd_rn(*o, acc);
}

bool cond_orders_ok(int ic, int ec) { return ic >= 0 && ic <= 2 && ec >= -1 && ec <= 2 && (ic != 0 || ec != 0); }

}  // namespace

extern "C" int beast_cond_fixed_f32(const float* traj, int64_t B, int T, int64_t sb, int64_t st, int64_t sd,
                                    const int32_t* joint_idx, int dj, const float* times, const float* knots,
                                    int degree, int n_ctrl, float tau, int init_order, int end_order,
                                    float* init_pos, float* init_vel, float* end_pos, float* end_vel,
                                    float* params_init, float* params_end, void* stream) {
  BEAST_REQUIRE(cond_orders_ok(init_order, end_order), "beast_cond_fixed_f32: orders (%d, %d) out of range",
                init_order, end_order);
  BEAST_REQUIRE(B >= 0 && dj >= 0, "beast_cond_fixed_f32: B=%lld, dj=%d must be >= 0", (long long)B, dj);
  BEAST_REQUIRE(T >= 2, "index 1 is out of bounds for dimension 1 with size %d", T);
  BEAST_REQUIRE(degree >= 1 && n_ctrl >= 2, "beast_cond_fixed_f32: degree %d / control points %d", degree, n_ctrl);
  BEAST_REQUIRE(traj && joint_idx && times && knots, "beast_cond_fixed_f32: null input pointer");
  BEAST_REQUIRE(init_order == 0 || (init_pos && init_vel && params_init), "beast_cond_fixed_f32: null init output");
  BEAST_REQUIRE(end_order == 0 || (end_pos && end_vel && params_end), "beast_cond_fixed_f32: null end output");
  if (B == 0 || dj == 0) return BEAST_OK;
  const CondArgs c{init_order, end_order, degree, n_ctrl, tau};
  const int64_t n = B * dj;
  hipLaunchKernelGGL(k_cond_fixed, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, beast::as_stream(stream), traj, B,
                     T, sb, st, sd, joint_idx, dj, times, knots, c, init_pos, init_vel, end_pos, end_vel, params_init,
                     params_end);
  BEAST_LAUNCHED("k_cond_fixed");
  return BEAST_OK;
}

extern "C" int beast_cond_add_f32(float* pos, int64_t B, int T, int D, const int32_t* joint_idx, int dj,
                                  const float* full_basis, int64_t full_sb, int n_ctrl, int init_order, int end_order,
                                  const float* params_init, const float* params_end, const float* init_pos,
                                  void* stream) {
  BEAST_REQUIRE(cond_orders_ok(init_order, end_order), "beast_cond_add_f32: orders (%d, %d) out of range",
                init_order, end_order);
  BEAST_REQUIRE(B >= 0 && T >= 0 && dj >= 0 && D >= dj, "beast_cond_add_f32: bad shape B=%lld T=%d D=%d dj=%d",
                (long long)B, T, D, dj);
  BEAST_REQUIRE(n_ctrl >= 2 && full_sb >= 0, "beast_cond_add_f32: control points %d / basis stride", n_ctrl);
  BEAST_REQUIRE(pos && joint_idx && full_basis, "beast_cond_add_f32: null pointer");
  BEAST_REQUIRE(init_order == 0 || (params_init && init_pos), "beast_cond_add_f32: null init condition");
  BEAST_REQUIRE(end_order == 0 || params_end, "beast_cond_add_f32: null end condition");
  if (B == 0 || T == 0 || dj == 0) return BEAST_OK;
  const CondArgs c{init_order, end_order, 0, n_ctrl, 0.0f};
  const int64_t n = B * T * dj;
  hipLaunchKernelGGL(k_cond_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, beast::as_stream(stream), pos, B, T,
                     D, joint_idx, dj, full_basis, full_sb, c, params_init, params_end, init_pos);
  BEAST_LAUNCHED("k_cond_add");
  return BEAST_OK;
}
