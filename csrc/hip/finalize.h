// BN finalize fused into the GEMM that produces the statistics (igemm3.hip epilogue).
//
// A conv GEMM with BN after it writes one partial row per output tile: (sum, sum of squares) per
// channel for the forward, (sum g, sum g*xhat) for the backward (epilogue.h vec_store_bnb), or
// (sum g, 0) for the bias gradient of an activation-only backward. Round 1 reduced those rows
// in a separate finalize kernel (bn.hip: bn_finalize / bn_bwd_finalize / sum_partials), one more
// dependent launch on the critical chain per BN layer and direction (~5-11 us each in the
// round-1 step profile, profiles/r1_step_profile_v12_1.29ms.txt).
//
// Here the GEMM's own workgroups finish the job with two levels of last-arrival reduction
// (the split-K hand-off of igemm3.hip: `sc1` stores, s_waitcnt vmcnt(0), barrier, one agent-scope
// counter bump; the last arrival re-arms the counter and reads the rows with `sc1` loads):
//   level 1: the F consecutive partial rows of a row group (all inside one BN group) -- the
//            workgroup that completes the group sums them IN ROW ORDER (double) into an L1 row;
//   level 2: the workgroup that completes the last L1 group of a column tile sums, per BN group,
//            its L1 rows in order and evaluates the finalize for that tile's channels.
// Deterministic (fixed association), no float atomics, and the counters are zero again after
// every launch, so graph replays need no reset kernel.
#pragma once
#include "kernels.h"

namespace dcg {

// sum of the `n` fp32 rows [r0, r0 + n) (stride `row_floats`) of column `col`, in row order;
// eight loads in flight at a time
__device__ __forceinline__ double sum_rows_sc1_f32(__amdgpu_buffer_rsrc_t r, int r0, int n, int row_floats, int col) {
  double s = 0.0;
  for (int q = 0; q < n; q += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = q + u < n ? ld_sc1_f32(r, (uint32_t)((size_t)(r0 + q + u) * row_floats + col) * 4u) : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u];
  }
  return s;
}

__device__ __forceinline__ double sum_rows_sc1_f64(__amdgpu_buffer_rsrc_t r, int r0, int n, int row_doubles, int col) {
  double s = 0.0;
  for (int q = 0; q < n; q += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = q + u < n ? ld_sc1_f64(r, (uint32_t)((size_t)(r0 + q + u) * row_doubles + col) * 8u) : 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  return s;
}

// Called by every thread of a workgroup right after the workgroup stored (sc1) its partial row
// `row` (channels [n0, n0 + BN) of both halves) into f.part. flag: an LDS int.
template <int BN, int NT>
__device__ __forceinline__ void tile_bn_finalize(const BnFin& f, int row, int nt, int n0, int* flag) {
  const int C = f.C;
  const int l1 = row / f.F;
  const int nl1 = f.groups * (f.ppg / f.F);
  if (!last_arrival(f.ctr + (size_t)l1 * f.ntn + nt, (unsigned)f.F, flag)) return;
  const __amdgpu_buffer_rsrc_t rp = make_rsrc(f.part, (uint32_t)((size_t)f.groups * f.ppg * 2 * C * 4));
  const __amdgpu_buffer_rsrc_t rl = make_rsrc(f.l1, (uint32_t)((size_t)nl1 * 2 * C * 8));
  for (int q = threadIdx.x; q < 2 * BN; q += NT) {
    const int h = q / BN, n = n0 + (q - h * BN);
    if (n >= C) continue;
    st_sc1_f64(rl, (uint32_t)(((size_t)l1 * 2 + h) * C + n) * 8u, sum_rows_sc1_f32(rp, l1 * f.F, f.F, 2 * C, h * C + n));
  }
  if (!last_arrival(f.ctr + (size_t)nl1 * f.ntn + nt, (unsigned)nl1, flag)) return;
  const int lpg = f.ppg / f.F;  // L1 rows per BN group
  for (int c = n0 + (int)threadIdx.x; c < min(C, n0 + BN); c += NT) {
    if (f.mode == 1) {          // forward: mean / rstd / scale / shift (+ EMA) per group
      for (int g = 0; g < f.groups; ++g) {
        const double a = sum_rows_sc1_f64(rl, g * lpg, lpg, 2 * C, c);
        const double b = sum_rows_sc1_f64(rl, g * lpg, lpg, 2 * C, C + c);
        const int idx = g * C + c;
        const double m = a / f.count;
        double v = b / f.count - m * m;
        if (v < 0.0) v = 0.0;
        const float mf = (float)m, vf = (float)v;
        const float r = rsqrtf(vf + f.eps);
        f.mean[idx] = mf;
        f.rstd[idx] = r;
        const float sc = f.gamma[c] * r;
        f.scale[idx] = sc;
        f.shift[idx] = f.beta[c] - mf * sc;
        if (f.ema_mean) {
          const float al = 1.f - f.decay;
          f.ema_mean[idx] -= al * (f.ema_mean[idx] - mf);
          f.ema_var[idx] -= al * (f.ema_var[idx] - vf);
        }
      }
    } else if (f.mode == 2) {   // backward: dx coefficients per group, group-summed dgamma / dbeta
      float dg = 0.f, db = 0.f;
      for (int g = 0; g < f.groups; ++g) {
        const float s1 = (float)sum_rows_sc1_f64(rl, g * lpg, lpg, 2 * C, c);
        const float s2 = (float)sum_rows_sc1_f64(rl, g * lpg, lpg, 2 * C, C + c);
        dg += s2;
        db += s1;
        const float r = f.rstd_in[g * C + c], mu = f.mean_in[g * C + c];
        const float A = f.gamma[c] * r;
        const float c2 = -A * s2 / (float)f.count;
        const float bb = -A * s1 / (float)f.count;
        f.coef[(g * 3 + 0) * C + c] = A;
        f.coef[(g * 3 + 1) * C + c] = c2 * r;
        f.coef[(g * 3 + 2) * C + c] = bb - c2 * mu * r;
      }
      if (f.dgamma) f.dgamma[c] = dg;
      if (f.dbeta) f.dbeta[c] = db;
    } else {                    // 3: bias gradient = column sum over every group
      double s = 0.0;
      for (int g = 0; g < f.groups; ++g) s += sum_rows_sc1_f64(rl, g * lpg, lpg, 2 * C, c);
      f.dbeta[c] = (float)s;
    }
  }
}

}  // namespace dcg
