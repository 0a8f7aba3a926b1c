// dcg-variants: bf16 f16 f32
// BatchNorm (TF batch_norm_with_global_normalization semantics) and
// activation kernels for gfx950, NHWC elem_t activations, fp32 statistics.
//
// Forward:  conv epilogue (igemm) or colstats -> per-tile partial sum / sum^2
//           -> bn_finalize (fp64 combine, biased variance, EMA update of the moving averages,
//              scale = gamma*rsqrt(var+eps), shift = beta - mean*scale)
//           -> bn_apply_act (y = act(x*scale + shift), 8 x elem_t per thread)
// Backward: colstats mode 1 (partials of sum g and sum g*xhat, g = dy*act'(y))
//           -> bn_bwd_finalize (d gamma, d beta into the flat fp32 gradient; per-group coefs)
//           -> bn_bwd_apply (dx = A*g + Bx*x + Cc, elem_t)
// Every reduction is two-stage with fixed order -> bitwise deterministic, no float atomics.
// "groups" split the rows into equal contiguous parts with independent statistics, which is
// how D(real) and D(fake) run as one 2B batch with the reference's per-call BN statistics.
// Elementwise kernels: 16-byte vector loads/stores, 32-bit index math with precomputed
// magic-number division, per-channel coefficients as float4 loads.
#include "kernels.h"

namespace dcg {

__device__ __forceinline__ void load8(const elem_t* p, float* f) {
  const elem8 b = ld8(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)b[i];
}

__device__ __forceinline__ void store8(elem_t* p, const float* f) {
  elem8 b;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (elem_t)f[i];
  st8(p, b);
}

__device__ __forceinline__ void load8f(const float* p, float* f) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}

// ---------------------------------------------------------------- column partial sums
// mode 0: (sum x, sum x^2)            -- BN forward statistics
// mode 1: (sum g, sum g*xhat)         -- BN backward, g = dy*act'(y), xhat = (x-mean)*rstd
// mode 2: (sum x, 0)                  -- plain column sums (bias gradients)
// Block: 256 threads = (C/8) channel vectors x LANES row lanes; each block covers
// rows_per_block rows and writes one partial row pair [2][C].
__global__ __launch_bounds__(256) void colstats_kernel(int mode, const elem_t* __restrict__ x,
                                                       const elem_t* __restrict__ dy, const elem_t* __restrict__ y,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       int act, float leak, int R, int C, int rows_per_block,
                                                       int rows_per_group, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int CV = C / 8;
  const int lanes = 256 / CV;  // row lanes (C <= 2048)
  const int cv = threadIdx.x % CV, rl = threadIdx.x / CV;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(R, r0 + rows_per_block);
  const int g = r0 / rows_per_group;
  float s[8], s2[8], mu[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; s2[i] = 0.f; mu[i] = 0.f; rs[i] = 0.f; }
  if (mode == 1) {
    load8f(mean + g * C + cv * 8, mu);
    load8f(rstd + g * C + cv * 8, rs);
  }
  if (rl < lanes) {
    for (int r = r0 + rl; r < r1; r += lanes) {
      float xv[8];
      load8(x + (size_t)r * C + cv * 8, xv);
      if (mode == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[i] += xv[i]; s2[i] += xv[i] * xv[i]; }
      } else if (mode == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += xv[i];
      } else {
        float dv[8], yv[8];
        load8(dy + (size_t)r * C + cv * 8, dv);
        load8(y + (size_t)r * C + cv * 8, yv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float gv = dv[i] * act_grad_from_out(yv[i], act, leak);
          s[i] += gv;
          s2[i] += gv * (xv[i] - mu[i]) * rs[i];
        }
      }
    }
  }
  // reduce over row lanes through LDS: red[lanes][C][2]
  if (rl < lanes) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(rl * C + cv * 8 + i) * 2 + 0] = s[i];
      red[(rl * C + cv * 8 + i) * 2 + 1] = s2[i];
    }
  }
  __syncthreads();
  int nl = lanes;
  if ((lanes & (lanes - 1)) == 0) {  // pairwise tree over the row lanes (fixed order)
    for (int h = lanes / 2; h > 0; h >>= 1) {
      for (int q = threadIdx.x; q < h * C * 2; q += 256) red[q] += red[q + h * C * 2];
      __syncthreads();
    }
    nl = 1;
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int l = 0; l < nl; ++l) { a += red[(l * C + c) * 2]; b += red[(l * C + c) * 2 + 1]; }
    part[(size_t)blockIdx.x * 2 * C + c] = a;
    part[(size_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

// ---------------------------------------------------------------- partial-row reduction
// Sum rows [p0, p1) of part (row stride `stride` floats) for the 16 channels of this block,
// two quantities per row (column offsets 0 and off1). 256 threads = 16 channels x 16 row lanes,
// each lane with 4 independent accumulators (latency hiding), fixed combine order ->
// deterministic. Result valid in lane 0 (threadIdx.x < 16).
template <typename T>
__device__ __forceinline__ void reduce_rows2(const float* __restrict__ part, int p0, int p1, size_t stride, int c,
                                             bool cok, int off1, T& s1, T& s2) {
  __shared__ T red[2][16][17];
  const int ch = threadIdx.x & 15, lane = threadIdx.x >> 4;
  // 8 independent loads per operand in flight per thread: the partial arrays are small and
  // freshly written by other CUs, so this loop is latency-bound, not bandwidth-bound
  T a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  if (cok) {
    int p = p0 + lane;
    for (; p + 112 < p1; p += 128) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        va[u] = part[(size_t)(p + 16 * u) * stride + c];
        vb[u] = off1 >= 0 ? part[(size_t)(p + 16 * u) * stride + off1 + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { a[u & 3] += (T)va[u]; b[u & 3] += (T)vb[u]; }
    }
    for (; p + 48 < p1; p += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] += (T)part[(size_t)(p + 16 * u) * stride + c];
        if (off1 >= 0) b[u] += (T)part[(size_t)(p + 16 * u) * stride + off1 + c];
      }
    }
    for (; p < p1; p += 16) {
      a[0] += (T)part[(size_t)p * stride + c];
      if (off1 >= 0) b[0] += (T)part[(size_t)p * stride + off1 + c];
    }
  }
  red[0][lane][ch] = (a[0] + a[1]) + (a[2] + a[3]);
  red[1][lane][ch] = (b[0] + b[1]) + (b[2] + b[3]);
  __syncthreads();
  T x = 0, y = 0;
  if (lane == 0) {
#pragma unroll
    for (int l = 0; l < 16; ++l) { x += red[0][l][ch]; y += red[1][l][ch]; }
  }
  __syncthreads();
  s1 = x;
  s2 = y;
}

// ---------------------------------------------------------------- BN forward finalize
// part: [P][2][C], partials of group g are [g*ppg, (g+1)*ppg). count = rows per group.
// grid (ceil(C/16), groups), block 256.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ part, int ppg, int groups, int C,
                                                          double count, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          float* __restrict__ scale_out, float* __restrict__ shift_out,
                                                          float* __restrict__ ema_mean, float* __restrict__ ema_var,
                                                          float decay) {
  const int g = blockIdx.y;
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  double s, s2;
  reduce_rows2<double>(part, g * ppg, (g + 1) * ppg, (size_t)2 * C, c, cok, C, s, s2);
  if ((threadIdx.x >> 4) != 0 || !cok) return;
  const int idx = g * C + c;
  const double m = s / count;
  double v = s2 / count - m * m;
  if (v < 0.0) v = 0.0;
  const float mf = (float)m, vf = (float)v;
  const float r = rsqrtf(vf + eps);
  mean_out[idx] = mf;
  rstd_out[idx] = r;
  const float sc = gamma[c] * r;
  scale_out[idx] = sc;
  shift_out[idx] = beta[c] - mf * sc;
  if (ema_mean) {
    // TF ExponentialMovingAverage: shadow -= (1 - decay) * (shadow - value), slot = group
    const float a = 1.f - decay;
    ema_mean[idx] -= a * (ema_mean[idx] - mf);
    ema_var[idx] -= a * (ema_var[idx] - vf);
  }
}

// inference-mode BN coefficients from moving averages (sampler, distriubted_model.py:46-47)
// debias_ptr (optional): TF zero-debiasing factor 1 / (1 - decay^t), written by the host before
// the sampler program runs (the recorded program keeps the pointer, not the value)
__global__ void bn_coef_eval_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                    float eps, const float* __restrict__ mean, const float* __restrict__ var,
                                    float debias, const float* __restrict__ debias_ptr, float* __restrict__ scale_out,
                                    float* __restrict__ shift_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (debias_ptr) debias = debias_ptr[0];
  const float m = mean[c] * debias, v = var[c] * debias;
  const float sc = gamma[c] * rsqrtf(v + eps);
  scale_out[c] = sc;
  shift_out[c] = beta[c] - m * sc;
}

// ---------------------------------------------------------------- BN apply + activation
// nv = R*C/8 vectors; vector v: row = v / C8, channel base = (v % C8) * 8, group = row / rpg
__global__ __launch_bounds__(256) void bn_apply_act_kernel(const elem_t* __restrict__ x, elem_t* __restrict__ y,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, uint32_t nv, int C,
                                                           FastDiv fd_c8, FastDiv fd_rpg, int act, float leak) {
  for (uint32_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += gridDim.x * 256) {
    const uint32_t r = fdiv(v, fd_c8);
    const int c = (int)(v - r * fd_c8.d) * 8;
    const int g = (int)fdiv(r, fd_rpg);
    float xv[8], sc[8], sh[8];
    load8(x + (size_t)v * 8, xv);
    load8f(scale + g * C + c, sc);
    load8f(shift + g * C + c, sh);
#pragma unroll
    for (int i = 0; i < 8; ++i) xv[i] = apply_act(__builtin_fmaf(xv[i], sc[i], sh[i]), act, leak);
    store8(y + (size_t)v * 8, xv);
  }
}

// ---------------------------------------------------------------- BN backward finalize
// part: [P][2][C] (sum g, sum g*xhat). Writes dgamma/dbeta (sum over groups) when non-null and
// per-(group, channel) coefficients of dx = A*g + Bx*x + Cc, layout coef[g][3][C].
// grid ceil(C/16), block 256.
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int ppg, int groups,
                                                              int C, float count, const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ coef) {
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  const bool lead = (threadIdx.x >> 4) == 0 && cok;
  float dg = 0.f, db = 0.f;
  for (int g = 0; g < groups; ++g) {
    float s1, s2;
    reduce_rows2<float>(part, g * ppg, (g + 1) * ppg, (size_t)2 * C, c, cok, C, s1, s2);
    if (lead) {
      dg += s2;
      db += s1;
      const float r = rstd[g * C + c], mu = mean[g * C + c];
      const float a = gamma[c] * r;
      const float c2 = -a * s2 / count;  // multiplies xhat
      const float b = -a * s1 / count;
      coef[(g * 3 + 0) * C + c] = a;
      coef[(g * 3 + 1) * C + c] = c2 * r;            // * x
      coef[(g * 3 + 2) * C + c] = b - c2 * mu * r;   // constant
    }
  }
  if (lead) {
    if (dgamma) dgamma[c] = dg;
    if (dbeta) dbeta[c] = db;
  }
}

// dx = (a * dy * act'(y) + b * x + c) per group (a, b, c: bn_bwd_finalize's coefficients)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const elem_t* __restrict__ dy, const elem_t* __restrict__ y,
                                                           const elem_t* __restrict__ x,
                                                           const float* __restrict__ coef, elem_t* __restrict__ dx,
                                                           uint32_t nv, int C, FastDiv fd_c8, FastDiv fd_rpg, int act,
                                                           float leak) {
  for (uint32_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += gridDim.x * 256) {
    const uint32_t r = fdiv(v, fd_c8);
    const int c = (int)(v - r * fd_c8.d) * 8;
    const int g = (int)fdiv(r, fd_rpg);
    float dv[8], ag[8], xv[8], yv[8], ca[8], cb[8], cc[8];
    load8(dy + (size_t)v * 8, dv);
    load8(x + (size_t)v * 8, xv);
    load8(y + (size_t)v * 8, yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) ag[i] = act_grad_from_out(yv[i], act, leak);
    load8f(coef + (g * 3 + 0) * C + c, ca);
    load8f(coef + (g * 3 + 1) * C + c, cb);
    load8f(coef + (g * 3 + 2) * C + c, cc);
#pragma unroll
    for (int i = 0; i < 8; ++i) dv[i] = __builtin_fmaf(ca[i], dv[i] * ag[i], __builtin_fmaf(cb[i], xv[i], cc[i]));
    store8(dx + (size_t)v * 8, dv);
  }
}

// ---------------------------------------------------------------- split finalizes
// The partial arrays come from the conv epilogues: one row per output tile, up to ~2k rows for
// a 64-channel layer. A handful of workgroups walking them serially was latency-bound (up to
// 40 us); here grid.z = PS slices each reduce ~64 rows of 16 channels, write their (double)
// sums with `sc1` stores, and the workgroup that arrives last (agent-scope counter, reset for
// the next launch / graph replay) combines the PS slices in slice order -- deterministic -- and
// runs the finalize. ws: [groups][PS][2][C] doubles; counters: zero-initialised.
// sum of the PS slice rows of group g, column c (and C + c), in slice order; 8 slices' loads in
// flight at a time (a plain loop waited on every `sc1` load: ~60 dependent L2 round trips)
__device__ __forceinline__ void slice_sums(__amdgpu_buffer_rsrc_t rw, int g, int PS, int C, int c, double& a,
                                           double& b) {
  for (int q = 0; q < PS; q += 8) {  // guarded rounds of 8: no serial tail
    double va[8], vb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = q + u < PS;
      va[u] = ok ? ld_sc1_f64(rw, (uint32_t)((((size_t)g * PS + q + u) * 2 + 0) * C + c) * 8u) : 0.0;
      vb[u] = ok ? ld_sc1_f64(rw, (uint32_t)((((size_t)g * PS + q + u) * 2 + 1) * C + c) * 8u) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a += va[u];
      b += vb[u];
    }
  }
}

__global__ __launch_bounds__(256) void bn_finalize_split_kernel(
    const float* __restrict__ part, int ppg, int groups, int C, double count, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    float* __restrict__ scale_out, float* __restrict__ shift_out, float* __restrict__ ema_mean,
    float* __restrict__ ema_var, float decay, double* ws, unsigned* counters, int PS) {
  __shared__ int flag;
  const int cg = blockIdx.x, g = blockIdx.y, ps = blockIdx.z;
  const int c = cg * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  const int chunk = (ppg + PS - 1) / PS;
  const int p0 = g * ppg + ps * chunk, p1 = min(g * ppg + ppg, p0 + chunk);
  double s1, s2;
  reduce_rows2<double>(part, p0, max(p0, p1), (size_t)2 * C, c, cok, C, s1, s2);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(ws, (uint32_t)((size_t)groups * PS * 2 * C * 8));
  if (threadIdx.x < 16 && cok) {
    st_sc1_f64(rw, (uint32_t)((((size_t)g * PS + ps) * 2 + 0) * C + c) * 8u, s1);
    st_sc1_f64(rw, (uint32_t)((((size_t)g * PS + ps) * 2 + 1) * C + c) * 8u, s2);
  }
  if (!last_arrival(counters + g * gridDim.x + cg, (unsigned)PS, &flag)) return;
  if (threadIdx.x >= 16 || !cok) return;
  double a = 0.0, b = 0.0;
  slice_sums(rw, g, PS, C, c, a, b);
  const int idx = g * C + c;
  const double m = a / count;
  double v = b / count - m * m;
  if (v < 0.0) v = 0.0;
  const float mf = (float)m, vf = (float)v;
  const float r = rsqrtf(vf + eps);
  mean_out[idx] = mf;
  rstd_out[idx] = r;
  const float sc = gamma[c] * r;
  scale_out[idx] = sc;
  shift_out[idx] = beta[c] - mf * sc;
  if (ema_mean) {
    const float al = 1.f - decay;
    ema_mean[idx] -= al * (ema_mean[idx] - mf);
    ema_var[idx] -= al * (ema_var[idx] - vf);
  }
}

// backward: slices over (group, rows); the last arrival per 16-channel group (over all groups x
// slices) forms each group's coefficients and the group-summed dgamma / dbeta.
__global__ __launch_bounds__(256) void bn_bwd_finalize_split_kernel(
    const float* __restrict__ part, int ppg, int groups, int C, float count, const float* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ coef, double* ws, unsigned* counters, int PS) {
  __shared__ int flag;
  const int cg = blockIdx.x, g = blockIdx.y, ps = blockIdx.z;
  const int c = cg * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  const int chunk = (ppg + PS - 1) / PS;
  const int p0 = g * ppg + ps * chunk, p1 = min(g * ppg + ppg, p0 + chunk);
  double s1, s2;
  reduce_rows2<double>(part, p0, max(p0, p1), (size_t)2 * C, c, cok, C, s1, s2);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(ws, (uint32_t)((size_t)groups * PS * 2 * C * 8));
  if (threadIdx.x < 16 && cok) {
    st_sc1_f64(rw, (uint32_t)((((size_t)g * PS + ps) * 2 + 0) * C + c) * 8u, s1);
    st_sc1_f64(rw, (uint32_t)((((size_t)g * PS + ps) * 2 + 1) * C + c) * 8u, s2);
  }
  if (!last_arrival(counters + cg, (unsigned)(PS * groups), &flag)) return;
  if (threadIdx.x >= 16 || !cok) return;
  float dg = 0.f, db = 0.f;
  for (int gg = 0; gg < groups; ++gg) {
    double a = 0.0, b = 0.0;
    slice_sums(rw, gg, PS, C, c, a, b);
    const float sg1 = (float)a, sg2 = (float)b;
    dg += sg2;
    db += sg1;
    const float r = rstd[gg * C + c], mu = mean[gg * C + c];
    const float A = gamma[c] * r;
    const float c2 = -A * sg2 / count;
    const float bb = -A * sg1 / count;
    coef[(gg * 3 + 0) * C + c] = A;
    coef[(gg * 3 + 1) * C + c] = c2 * r;
    coef[(gg * 3 + 2) * C + c] = bb - c2 * mu * r;
  }
  if (dgamma) dgamma[c] = dg;
  if (dbeta) dbeta[c] = db;
}

// ---------------------------------------------------------------- sliced partial-row sums
// sum_partials over many rows (e.g. the bias-gradient partials of a dgrad GEMM's store pass:
// ~2k tile rows): grid (ceil(C/16), PS) slices reduce ~64 rows each, `sc1`-store their sums,
// the last slice per 16-channel group (agent counter, re-armed) adds the slices in slice order.
__global__ __launch_bounds__(256) void sum_partials_split_kernel(const float* __restrict__ part, int P, int stride,
                                                                 int C, float* __restrict__ dst, float* ws,
                                                                 unsigned* counters) {
  __shared__ int flag;
  const int cg = blockIdx.x, ps = blockIdx.y, PS = gridDim.y;
  const int c = cg * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  const int chunk = (P + PS - 1) / PS;
  const int p0 = ps * chunk, p1 = min(P, p0 + chunk);
  float s1, unused;
  reduce_rows2<float>(part, p0, max(p0, p1), (size_t)stride, c, cok, -1, s1, unused);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(ws, (uint32_t)((size_t)PS * C * 4));
  if (threadIdx.x < 16 && cok) st_sc1_f32(rw, (uint32_t)(ps * C + c) * 4u, s1);
  if (!last_arrival(counters + cg, (unsigned)PS, &flag)) return;
  if (threadIdx.x >= 16 || !cok) return;
  float a = 0.f;
  for (int q = 0; q < PS; q += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = q + u < PS ? ld_sc1_f32(rw, (uint32_t)((q + u) * C + c) * 4u) : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  dst[c] = a;
}

// ---------------------------------------------------------------- activation backward (no BN)
// dx = dy * act'(y); 8 per thread + scalar tail
__global__ __launch_bounds__(256) void act_bwd_kernel(const elem_t* __restrict__ dy, const elem_t* __restrict__ y,
                                                      elem_t* __restrict__ dx, size_t n, int act, float leak) {
  const size_t nv = n / 8;
  for (size_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (size_t)gridDim.x * 256) {
    float dv[8], yv[8];
    load8(dy + v * 8, dv);
    load8(y + v * 8, yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) dv[i] *= act_grad_from_out(yv[i], act, leak);
    store8(dx + v * 8, dv);
  }
  for (size_t i = nv * 8 + blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dx[i] = (elem_t)((float)dy[i] * act_grad_from_out((float)y[i], act, leak));
}

// sum over partial rows -> dst[C]; grid ceil(C/16), block 256
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part, int P, int stride, int C,
                                                           float* __restrict__ dst) {
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  float s, unused;
  reduce_rows2<float>(part, 0, P, (size_t)stride, c, c < C, -1, s, unused);
  if ((threadIdx.x >> 4) == 0 && c < C) dst[c] = s;
}

// column sums for a small channel count (C <= 16), e.g. dbias of a 3-channel image gradient
__global__ __launch_bounds__(256) void colsum_small_kernel(const elem_t* __restrict__ x, int R, int C,
                                                           float* __restrict__ part) {
  __shared__ float red[256][17];
  float s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = 0.f;
  for (int r = blockIdx.x * 256 + threadIdx.x; r < R; r += gridDim.x * 256)
    for (int c = 0; c < C; ++c) s[c] += (float)x[(size_t)r * C + c];
  for (int c = 0; c < C; ++c) red[threadIdx.x][c] = s[c];
  __syncthreads();
  if (threadIdx.x < C) {
    float a = 0.f;
    for (int t = 0; t < 256; ++t) a += red[t][threadIdx.x];
    part[blockIdx.x * C + threadIdx.x] = a;
  }
}

// ---------------------------------------------------------------- activation backward + bias gradient
// dx = dy * act'(y) over [R][C] and db[c] = sum_r dx[r][c] (of the stored, rounded dx) in ONE
// launch, replacing act_bwd + a column-sum pass + a partials pass: every block writes its
// partial column sums, the last block to arrive (counter) reduces them in block order
// (deterministic) and re-arms the counter for the next replay.
//   CC = 0: C % 8 == 0; thread = (row lane, 8-channel chunk), 16-byte loads / stores.
//   CC = 1 / 3: image tensors; thread = 8 consecutive elements, channel = element index % CC.
template <int CC>
__global__ __launch_bounds__(256) void act_bwd_dbias_kernel(const elem_t* __restrict__ dy,
                                                            const elem_t* __restrict__ y, elem_t* __restrict__ dx,
                                                            int R, int C, int per_block, int act, float leak,
                                                            float* __restrict__ part, unsigned* __restrict__ counter,
                                                            float* __restrict__ db) {
  __shared__ float red[2048];
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t prs = make_rsrc(part, (uint32_t)(gridDim.x * C * 4));
  if constexpr (CC == 0) {
    const int C8 = C >> 3, RL = 256 / C8, c = tid % C8, rl = tid / C8;
    const int r0 = blockIdx.x * per_block, r1 = min(R, r0 + per_block);
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = 0.f;
    if (rl < RL) {
      // 4 rows per iteration, all loads issued before any use (memory-level parallelism)
      for (int rb = r0 + rl; rb < r1; rb += 4 * RL) {
        elem8 dvv[4], yvv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rb + u * RL;
          const size_t o = (size_t)(r < r1 ? r : r0) * C + 8 * c;
          dvv[u] = ld8(dy + o);
          yvv[u] = ld8(y + o);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = rb + u * RL;
          if (r >= r1) break;
          const elem8 dv = dvv[u], yv = yvv[u];
          elem8 out;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            out[i] = f2bf((float)dv[i] * act_grad_from_out((float)yv[i], act, leak));
            s[i] += (float)out[i];
          }
          st8(dx + (size_t)r * C + 8 * c, out);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) red[rl * C + 8 * c + i] = s[i];
    }
    __syncthreads();
    // pairwise tree over the RL row lanes (fixed order, log2(RL) LDS rounds)
    for (int h = RL / 2; h > 0; h >>= 1) {
      for (int q = tid; q < h * C; q += 256) red[q] += red[q + h * C];
      __syncthreads();
    }
    for (int cc = tid; cc < C; cc += 256) st_sc1_f32(prs, (uint32_t)(blockIdx.x * C + cc) * 4u, red[cc]);
  } else {
    const size_t n = (size_t)R * CC;
    const size_t e0 = (size_t)blockIdx.x * per_block, e1 = min(n, e0 + per_block);  // per_block % 8 == 0
    float s[CC];
#pragma unroll
    for (int i = 0; i < CC; ++i) s[i] = 0.f;
    // full 8-element chunks: 2 per iteration, loads first; the scalar tail after
    const uint32_t nfull = (uint32_t)((min(e1, n & ~(size_t)7) - min(e0, n & ~(size_t)7)) / 8);
    for (uint32_t q0 = tid; q0 < nfull; q0 += 2 * 256) {
      elem8 dvv[2], yvv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t q = q0 + u * 256 < nfull ? q0 + u * 256 : q0;
        dvv[u] = ld8(dy + e0 + 8 * (size_t)q);
        yvv[u] = ld8(y + e0 + 8 * (size_t)q);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t q = q0 + u * 256;
        if (q >= nfull) break;
        const size_t e = e0 + 8 * (size_t)q;
        int ch = (int)((uint32_t)(e % CC));
        const elem8 dv = dvv[u], yv = yvv[u];
        elem8 out;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          out[i] = f2bf((float)dv[i] * act_grad_from_out((float)yv[i], act, leak));
          const float v = (float)out[i];
#pragma unroll
          for (int k = 0; k < CC; ++k) s[k] += ch == k ? v : 0.f;
          ch = ch == CC - 1 ? 0 : ch + 1;
        }
        st8(dx + e, out);
      }
    }
    for (size_t e = e0 + 8 * (size_t)nfull + tid; e < e1; e += 256) {  // tail (< 8 elements)
      const int ch = (int)(e % CC);
      const elem_t o = f2bf((float)dy[e] * act_grad_from_out((float)y[e], act, leak));
      dx[e] = o;
#pragma unroll
      for (int k = 0; k < CC; ++k) s[k] += ch == k ? (float)o : 0.f;
    }
#pragma unroll
    for (int q = 0; q < CC; ++q) {  // butterfly within each wave, then the 4 waves in order
      const float w = wave_sum(s[q]);
      if ((tid & 63) == 0) red[(tid >> 6) * CC + q] = w;
    }
    __syncthreads();
    if (tid < CC)
      st_sc1_f32(prs, (uint32_t)(blockIdx.x * CC + tid) * 4u, red[tid] + red[CC + tid] + red[2 * CC + tid] + red[3 * CC + tid]);
  }
  // ---- last-arrival reduction of the partials [gridDim.x][C]: the partials were written with
  // plain stores; a device-scope __threadfence() here would write back the whole XCD L2 in
  // every block (measured: 30 us for this kernel). Instead: vmcnt(0) + relaxed agent-scope
  // counter (last_arrival) and the partials re-read with `sc1` loads that bypass the
  // (non-coherent) L1 of this CU; the writers' L2 lines are written through by the sc1 store
  // policy below (partials are stored with st_sc1 in the two paths above).
  __shared__ int flag_s;
  if (!last_arrival(counter, gridDim.x, &flag_s)) return;
  const int nb = gridDim.x;
  int G = 1;  // power-of-two block groups summed in parallel, then a fixed-order tree
  while (G * 2 * C <= 256) G *= 2;
  const int c = tid % C, g = tid / C;
  float a = 0.f;
  if (g < G) {
    // 8 partial loads in flight per round, guarded (no serial tail: every `sc1` load is a full
    // memory round trip, ~1-2 us)
    for (int b0 = g; b0 < nb; b0 += 8 * G) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + u * G;
        v[u] = b < nb ? ld_sc1_f32(prs, (uint32_t)(b * C + c) * 4u) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) a += v[u];
    }
  }
  __syncthreads();
  if (g < G) red[g * C + c] = a;
  __syncthreads();
  for (int h = G / 2; h > 0; h >>= 1) {
    if (tid < h * C) red[tid] += red[tid + h * C];
    __syncthreads();
  }
  if (tid < C) db[tid] = red[tid];
  if (tid == 0) *counter = 0u;
}

}  // namespace dcg

using namespace dcg;

static inline unsigned ew_blocks(size_t nvec) {
  size_t b = (nvec + 255) / 256;
  if (b > 8192) b = 8192;
  return (unsigned)(b ? b : 1);
}

extern "C" int DCG_API(dcg_colstats)(int mode, const elem_t* x, const elem_t* dy, const elem_t* y, const float* mean,
                            const float* rstd, int act, float leak, int R, int C, int rows_per_block,
                            int rows_per_group, float* part, hipStream_t s) {
  if (C % 8 || C > 2048) return -2;
  const int P = (R + rows_per_block - 1) / rows_per_block;
  const int lanes = 256 / (C / 8);
  const size_t shm = (size_t)lanes * C * 2 * sizeof(float);
  hipLaunchKernelGGL(colstats_kernel, dim3(P), dim3(256), shm, s, mode, x, dy, y, mean, rstd, act, leak, R, C,
                     rows_per_block, rows_per_group, part);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_finalize)(const float* part, int ppg, int groups, int C, double count, const float* gamma,
                               const float* beta, float eps, float* mean, float* rstd, float* scale, float* shift,
                               float* ema_mean, float* ema_var, float decay, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 15) / 16, groups), dim3(256), 0, s, part, ppg, groups, C, count,
                     gamma, beta, eps, mean, rstd, scale, shift, ema_mean, ema_var, decay);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_coef_eval)(int C, const float* gamma, const float* beta, float eps, const float* mean,
                                const float* var, float debias, const float* debias_ptr, float* scale, float* shift,
                                hipStream_t s) {
  hipLaunchKernelGGL(bn_coef_eval_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, eps, mean, var,
                     debias, debias_ptr, scale, shift);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_apply_act)(const elem_t* x, elem_t* y, const float* scale, const float* shift, int R, int C,
                                int rows_per_group, int act, float leak, hipStream_t s) {
  if (C % 8) return -2;
  const size_t nv = (size_t)R * C / 8;
  if (nv >= 0x80000000ull) return -3;
  hipLaunchKernelGGL(bn_apply_act_kernel, dim3(ew_blocks(nv)), dim3(256), 0, s, x, y, scale, shift, (uint32_t)nv, C,
                     fastdiv_make(C / 8), fastdiv_make(rows_per_group), act, leak);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_bwd_finalize)(const float* part, int ppg, int groups, int C, float count, const float* gamma,
                                   const float* mean, const float* rstd, float* dgamma, float* dbeta, float* coef,
                                   hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, s, part, ppg, groups, C, count,
                     gamma, mean, rstd, dgamma, dbeta, coef);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_bwd_apply)(const elem_t* dy, const elem_t* y, const elem_t* x, const float* coef, elem_t* dx, int R,
                                int C, int rows_per_group, int act, float leak, hipStream_t s) {
  if (C % 8) return -2;
  const size_t nv = (size_t)R * C / 8;
  if (nv >= 0x80000000ull) return -3;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_blocks(nv)), dim3(256), 0, s, dy, y, x, coef, dx, (uint32_t)nv, C,
                     fastdiv_make(C / 8), fastdiv_make(rows_per_group), act, leak);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_act_bwd)(const elem_t* dy, const elem_t* y, elem_t* dx, size_t n, int act, float leak, hipStream_t s) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(ew_blocks(n / 8 + 1)), dim3(256), 0, s, dy, y, dx, n, act, leak);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_sum_partials)(const float* part, int P, int stride, int C, float* dst, hipStream_t s) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3((C + 15) / 16), dim3(256), 0, s, part, P, stride, C, dst);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_colsum_small)(const elem_t* x, int R, int C, float* part, int blocks, hipStream_t s) {
  if (C > 16) return -2;
  hipLaunchKernelGGL(colsum_small_kernel, dim3(blocks), dim3(256), 0, s, x, R, C, part);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_finalize_split)(const float* part, int ppg, int groups, int C, double count,
                                              const float* gamma, const float* beta, float eps, float* mean,
                                              float* rstd, float* scale, float* shift, float* ema_mean, float* ema_var,
                                              float decay, double* ws, unsigned* counters, int PS, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_split_kernel, dim3((C + 15) / 16, groups, PS), dim3(256), 0, s, part, ppg, groups, C,
                     count, gamma, beta, eps, mean, rstd, scale, shift, ema_mean, ema_var, decay, ws, counters, PS);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bn_bwd_finalize_split)(const float* part, int ppg, int groups, int C, float count,
                                                  const float* gamma, const float* mean, const float* rstd,
                                                  float* dgamma, float* dbeta, float* coef, double* ws,
                                                  unsigned* counters, int PS, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_split_kernel, dim3((C + 15) / 16, groups, PS), dim3(256), 0, s, part, ppg,
                     groups, C, count, gamma, mean, rstd, dgamma, dbeta, coef, ws, counters, PS);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_act_bwd_dbias)(const elem_t* dy, const elem_t* y, elem_t* dx, int R, int C, int act,
                                          float leak, float* part, int max_blocks, unsigned* counter, float* db,
                                          hipStream_t s) {
  int per_block = 0, blocks = 0;
  if (C % 8 == 0) {
    if (C > 256 || 256 % (C / 8)) return -2;
    const int RL = 256 / (C / 8);
    per_block = RL * 16;  // 16 rows per thread (<= max_blocks: one same-address atomic per block)
    blocks = (R + per_block - 1) / per_block;
    if (blocks > max_blocks) { per_block = (R + max_blocks - 1) / max_blocks; blocks = (R + per_block - 1) / per_block; }
    hipLaunchKernelGGL(act_bwd_dbias_kernel<0>, dim3(blocks), dim3(256), 0, s, dy, y, dx, R, C, per_block, act, leak,
                       part, counter, db);
  } else if (C == 1 || C == 3) {
    const size_t n = (size_t)R * C;
    per_block = 8 * 256 * 2;  // 2 chunks of 8 per thread
    blocks = (int)((n + per_block - 1) / per_block);
    if (blocks > max_blocks) {
      per_block = (int)(((n + max_blocks - 1) / max_blocks + 7) / 8 * 8);
      blocks = (int)((n + per_block - 1) / per_block);
    }
    if (C == 1)
      hipLaunchKernelGGL(act_bwd_dbias_kernel<1>, dim3(blocks), dim3(256), 0, s, dy, y, dx, R, C, per_block, act,
                         leak, part, counter, db);
    else
      hipLaunchKernelGGL(act_bwd_dbias_kernel<3>, dim3(blocks), dim3(256), 0, s, dy, y, dx, R, C, per_block, act,
                         leak, part, counter, db);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_sum_partials_split)(const float* part, int P, int stride, int C, float* dst, float* ws,
                                               unsigned* counters, int PS, hipStream_t s) {
  hipLaunchKernelGGL(sum_partials_split_kernel, dim3((C + 15) / 16, PS), dim3(256), 0, s, part, P, stride, C, dst, ws,
                     counters);
  return (int)hipGetLastError();
}
