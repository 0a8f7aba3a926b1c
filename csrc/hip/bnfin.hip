// dcg-variants: bf16 f16 f32
// BatchNorm finalize, round 2: one launch, one level, every lane of the workgroup on the partial
// rows (bn.hip's bn_finalize_split: 16 channels x 16 row lanes per workgroup, then a second
// level through a workspace and a last-arrival counter -- two dependent memory round trips and an
// atomic on the forward's critical path, 5-6 us per BN layer in profiles/r2/step_profile_r2_1.15ms.txt).
//
// Workgroup = 4 channels of one BN group (forward) / of all groups (backward); its 256 lanes take
// the partial rows r = lane, lane + 256, ... (16-byte loads: the 4 channels of both statistics of a
// row), accumulate in double, then a fixed-order reduction (xor butterfly inside each wave, the 4
// waves in order through LDS) -- deterministic, no atomics, no counters to re-arm.
#include "kernels.h"

namespace dcg {

// sum over the partial rows [p0, p1) of (stat 0, stat 1) for channels c0..c0+3; valid in tid < 8:
// out[st * 4 + i]
__device__ __forceinline__ void bnfin_rows(const float* __restrict__ part, int p0, int p1, int C, int c0, bool cok,
                                           double* red, double (&out)[8]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.0;
  if (cok) {
    int r = p0 + tid;
    for (; r + 256 < p1; r += 512) {  // two rows in flight per lane
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(part + (size_t)r * 2 * C + c0);
      const f32x4 q0 = *reinterpret_cast<const f32x4*>(part + (size_t)r * 2 * C + C + c0);
      const f32x4 s1 = *reinterpret_cast<const f32x4*>(part + (size_t)(r + 256) * 2 * C + c0);
      const f32x4 q1 = *reinterpret_cast<const f32x4*>(part + (size_t)(r + 256) * 2 * C + C + c0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] += (double)s0[i];
        a[4 + i] += (double)q0[i];
        a[i] += (double)s1[i];
        a[4 + i] += (double)q1[i];
      }
    }
    if (r < p1) {
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(part + (size_t)r * 2 * C + c0);
      const f32x4 q0 = *reinterpret_cast<const f32x4*>(part + (size_t)r * 2 * C + C + c0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] += (double)s0[i];
        a[4 + i] += (double)q0[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a[i] += __shfl_xor(a[i], o, 64);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wave * 8 + i] = a[i];
  }
  __syncthreads();
  if (tid < 8) {
    const double v = ((red[tid] + red[8 + tid]) + red[16 + tid]) + red[24 + tid];
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = 0.0;
    out[0] = v;  // thread tid owns statistic tid / 4 of channel c0 + tid % 4
  }
  __syncthreads();
}

// forward: grid (ceil(C / 4), groups); part [groups * ppg][2][C] (sum, sum of squares)
__global__ __launch_bounds__(256) void bnfin_fwd_kernel(const float* __restrict__ part, int ppg, int C, double count,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                        float* __restrict__ scale_out, float* __restrict__ shift_out,
                                                        float* __restrict__ ema_mean, float* __restrict__ ema_var,
                                                        float decay) {
  __shared__ double red[32];
  __shared__ double tot[8];
  const int g = blockIdx.y, c0 = blockIdx.x * 4, tid = threadIdx.x;
  double o[8];
  bnfin_rows(part, g * ppg, (g + 1) * ppg, C, c0, c0 < C, red, o);
  if (tid < 8) tot[tid] = o[0];
  __syncthreads();
  if (tid < 4 && c0 + tid < C) {
    const int c = c0 + tid, idx = g * C + c;
    const double m = tot[tid] / count;
    double v = tot[4 + tid] / count - m * m;
    if (v < 0.0) v = 0.0;
    const float mf = (float)m, vf = (float)v;
    const float r = rsqrtf(vf + eps);
    mean_out[idx] = mf;
    rstd_out[idx] = r;
    const float sc = gamma[c] * r;
    scale_out[idx] = sc;
    shift_out[idx] = __builtin_fmaf(-mf, sc, beta[c]);  // explicit fma: bnfold.hip computes the same bits
    if (ema_mean) {  // TF ExponentialMovingAverage, slot = group
      const float al = 1.f - decay;
      ema_mean[idx] = __builtin_fmaf(-al, ema_mean[idx] - mf, ema_mean[idx]);
      ema_var[idx] = __builtin_fmaf(-al, ema_var[idx] - vf, ema_var[idx]);
    }
  }
}

// backward: grid ceil(C / 4); part [groups * ppg][2][C] (sum g, sum g*xhat); per group the dx
// coefficients coef[g][3][C], group-summed dgamma / dbeta
__global__ __launch_bounds__(256) void bnfin_bwd_kernel(const float* __restrict__ part, int ppg, int groups, int C,
                                                        float count, const float* __restrict__ gamma,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta, float* __restrict__ coef) {
  __shared__ double red[32];
  __shared__ double tot[8];
  const int c0 = blockIdx.x * 4, tid = threadIdx.x;
  float dg = 0.f, db = 0.f;
  for (int g = 0; g < groups; ++g) {
    double o[8];
    bnfin_rows(part, g * ppg, (g + 1) * ppg, C, c0, c0 < C, red, o);
    if (tid < 8) tot[tid] = o[0];
    __syncthreads();
    if (tid < 4 && c0 + tid < C) {
      const int c = c0 + tid;
      const float s1 = (float)tot[tid], s2 = (float)tot[4 + tid];
      dg += s2;
      db += s1;
      const float r = rstd[g * C + c], mu = mean[g * C + c];
      const float A = gamma[c] * r;
      const float c2 = -A * s2 / count;
      const float bb = -A * s1 / count;
      coef[(g * 3 + 0) * C + c] = A;
      coef[(g * 3 + 1) * C + c] = c2 * r;
      coef[(g * 3 + 2) * C + c] = __builtin_fmaf(-(c2 * mu), r, bb);
    }
    __syncthreads();
  }
  if (tid < 4 && c0 + tid < C) {
    if (dgamma) dgamma[c0 + tid] = dg;
    if (dbeta) dbeta[c0 + tid] = db;
  }
}

}  // namespace dcg

using namespace dcg;

extern "C" int DCG_API(dcg_bnfin_fwd)(const float* part, int ppg, int groups, int C, double count, const float* gamma,
                                      const float* beta, float eps, float* mean, float* rstd, float* scale,
                                      float* shift, float* ema_mean, float* ema_var, float decay, hipStream_t s) {
  if (C % 4 || ppg < 1 || groups < 1) return -2;
  hipLaunchKernelGGL(bnfin_fwd_kernel, dim3(C / 4, groups), dim3(256), 0, s, part, ppg, C, count, gamma, beta, eps,
                     mean, rstd, scale, shift, ema_mean, ema_var, decay);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bnfin_bwd)(const float* part, int ppg, int groups, int C, float count, const float* gamma,
                                      const float* mean, const float* rstd, float* dgamma, float* dbeta, float* coef,
                                      hipStream_t s) {
  if (C % 4 || ppg < 1 || groups < 1) return -2;
  hipLaunchKernelGGL(bnfin_bwd_kernel, dim3(C / 4), dim3(256), 0, s, part, ppg, groups, C, count, gamma, mean, rstd,
                     dgamma, dbeta, coef);
  return (int)hipGetLastError();
}
