// dcg-variants: bf16 f16 f32
// BatchNorm finalize folded into the apply pass, for layers with few partial-statistics rows
// (<= 256 per BN group: the small 8x8 / 4x4 layers of the 64x64 step). One launch replaces
// bnfin_fwd + bn_apply_act (forward) or bnfin_bwd + bn_bwd_apply (backward): every workgroup owns
// 64 channels x a chunk of rows of ONE BN group, reduces that group's partial rows for its 64
// channels itself (no cross-workgroup hand-off: the round-2 one-launch form with claimed finalize
// jobs lost to the two launches, profiles/r2/ab_bn_fin_apply_one_launch_r2.txt), then applies.
// The first chunk of each group writes mean / rstd / scale / shift (+ the EMA update) or the dx
// coefficients + dgamma / dbeta, which later kernels and the sampler read.
//
// The reduction order is bnfin.hip's (partial row 64 w + l on lane l of slot w, an xor butterfly
// per slot in double, slots added in order), so the statistics are bit-identical to the
// two-launch path, and every multiply-add is an explicit fma in both (bn.hip / bnfin.hip too), so
// the outputs are bit-identical as well. Reference op: batch_norm + moments + EMA, /root/reference/distriubted_model.py:37-50.
#include "kernels.h"

namespace dcg {

constexpr int BNF_CW = 64;     // channels per workgroup (8 vectors of 8)
constexpr int BNF_ITERS = 4;   // apply rows per thread (chunk <= 32 x 4 = 128 rows), prefetched

__device__ __forceinline__ void bnf_load8(const elem_t* p, float* f) {
  const elem8 b = ld8(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)b[i];
}

__device__ __forceinline__ void bnf_store8(elem_t* p, const float* f) {
  elem8 b;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (elem_t)f[i];
  st8(p, b);
}

// sums of the partial rows [p0, p0 + n) (n <= 256) of both statistics for channels c0..c0+63 into
// tot[2][64] (LDS, double). Lane group (16 lanes) q = threadIdx.x / 16 owns channel quad q; its
// lane l (0..15) adds rows l, l+16, l+32, l+48 of each 64-row slot as (r0 + r32) + (r16 + r48) --
// exactly what lane l holds after the xor-32 and xor-16 steps of bnfin.hip's 64-lane butterfly --
// then runs that butterfly's xor 8 / 4 / 2 / 1 steps; slots are added in order. So the sums are
// bnfin's bit for bit, with a quarter of its shuffles and every quad reduced at once.
__device__ __forceinline__ void bnf_sums(const float* __restrict__ part, int p0, int n, int C, int c0, double* tot) {
  const int l = threadIdx.x & 15, q = threadIdx.x >> 4, c = c0 + 4 * q;
  const int nslot = (n + 63) >> 6;
  double acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (w < nslot) {  // workgroup-uniform
      double v[4][8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 64 * w + l + 16 * j;
        if (r < n) {
          const float* row = part + (size_t)(p0 + r) * 2 * C + c;
          const f32x4 s = *reinterpret_cast<const f32x4*>(row);
          const f32x4 t = *reinterpret_cast<const f32x4*>(row + C);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[j][i] = (double)s[i];
            v[j][4 + i] = (double)t[i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[j][i] = 0.0;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        double a = (v[0][i] + v[2][i]) + (v[1][i] + v[3][i]);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        acc[i] = w == 0 ? a : acc[i] + a;
      }
    }
  }
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      tot[4 * q + i] = acc[i];
      tot[BNF_CW + 4 * q + i] = acc[4 + i];
    }
  }
}

// forward: grid (C / 64, groups * chunks); y = act(x * scale + shift)
__global__ __launch_bounds__(256) void bnfold_fwd_kernel(
    const float* __restrict__ part, int ppg, int C, int rpg, int rch, int chunks, double count,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, float* __restrict__ scale_out, float* __restrict__ shift_out,
    float* __restrict__ ema_mean, float* __restrict__ ema_var, float decay, const elem_t* __restrict__ x,
    elem_t* __restrict__ y, int act, float leak) {
  __shared__ double tot[2 * BNF_CW];
  __shared__ float sc_s[BNF_CW], sh_s[BNF_CW];
  const int tid = threadIdx.x, c0 = blockIdx.x * BNF_CW;
  const int g = blockIdx.y / chunks, ch = blockIdx.y - g * chunks;
  const int r0 = g * rpg + ch * rch, r1 = min(r0 + rch, (g + 1) * rpg);
  const int vc = c0 + 8 * (tid & 7), rt = tid >> 3;
  // the chunk's activations first: their loads overlap the statistics reduction
  elem8 xr[BNF_ITERS];
#pragma unroll
  for (int it = 0; it < BNF_ITERS; ++it) {
    const int r = r0 + rt + 32 * it;
    if (r < r1) xr[it] = ld8(x + (size_t)r * C + vc);
  }
  bnf_sums(part, g * ppg, ppg, C, c0, tot);
  __syncthreads();
  if (tid < BNF_CW) {
    const int c = c0 + tid, idx = g * C + c;
    const double m = tot[tid] / count;
    double v = tot[BNF_CW + tid] / count - m * m;
    if (v < 0.0) v = 0.0;
    const float mf = (float)m, vf = (float)v;
    const float r = rsqrtf(vf + eps);
    const float sc = gamma[c] * r, sh = __builtin_fmaf(-mf, sc, beta[c]);
    sc_s[tid] = sc;
    sh_s[tid] = sh;
    if (ch == 0) {
      mean_out[idx] = mf;
      rstd_out[idx] = r;
      scale_out[idx] = sc;
      shift_out[idx] = sh;
      if (ema_mean) {  // TF ExponentialMovingAverage, slot = group
        const float al = 1.f - decay;
        ema_mean[idx] = __builtin_fmaf(-al, ema_mean[idx] - mf, ema_mean[idx]);
        ema_var[idx] = __builtin_fmaf(-al, ema_var[idx] - vf, ema_var[idx]);
      }
    }
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = sc_s[8 * (tid & 7) + i];
    sh[i] = sh_s[8 * (tid & 7) + i];
  }
#pragma unroll
  for (int it = 0; it < BNF_ITERS; ++it) {
    const int r = r0 + rt + 32 * it;
    if (r < r1) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = apply_act(__builtin_fmaf((float)xr[it][i], sc[i], sh[i]), act, leak);
      bnf_store8(y + (size_t)r * C + vc, v);
    }
  }
}

// backward: grid (C / 64, groups * chunks); dx = A * dy * act'(y) + Bx * x + Cc with the group's
// coefficients. The first chunk of group 0 also sums dgamma / dbeta over every group (the order
// of bnfin_bwd: group 0 first).
__global__ __launch_bounds__(256) void bnfold_bwd_kernel(
    const float* __restrict__ part, int ppg, int groups, int C, int rpg, int rch, int chunks, float count,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ rstd,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ coef, const elem_t* __restrict__ dy,
    const elem_t* __restrict__ y, const elem_t* __restrict__ x, elem_t* __restrict__ dx, int act, float leak) {
  __shared__ double tot[2 * BNF_CW];
  __shared__ float ca_s[BNF_CW], cb_s[BNF_CW], cc_s[BNF_CW];
  const int tid = threadIdx.x, c0 = blockIdx.x * BNF_CW;
  const int g = blockIdx.y / chunks, ch = blockIdx.y - g * chunks;
  const int r0 = g * rpg + ch * rch, r1 = min(r0 + rch, (g + 1) * rpg);
  const int vc = c0 + 8 * (tid & 7), rt = tid >> 3;
  elem8 dr[BNF_ITERS], yr[BNF_ITERS], xr[BNF_ITERS];
#pragma unroll
  for (int it = 0; it < BNF_ITERS; ++it) {
    const int r = r0 + rt + 32 * it;
    if (r < r1) {
      const size_t o = (size_t)r * C + vc;
      dr[it] = ld8(dy + o);
      yr[it] = ld8(y + o);
      xr[it] = ld8(x + o);
    }
  }
  const bool writer = blockIdx.y == 0;            // dgamma / dbeta: every group, in order
  const int gb = writer ? 0 : g, ge = writer ? groups : g + 1;
  float dg = 0.f, db = 0.f;
  for (int gg = gb; gg < ge; ++gg) {               // workgroup-uniform
    bnf_sums(part, gg * ppg, ppg, C, c0, tot);
    __syncthreads();
    if (tid < BNF_CW) {
      const int c = c0 + tid;
      const float s1 = (float)tot[tid], s2 = (float)tot[BNF_CW + tid];
      dg += s2;
      db += s1;
      const float r = rstd[gg * C + c], mu = mean[gg * C + c];
      const float A = gamma[c] * r;
      const float c2 = -A * s2 / count;
      const float bb = -A * s1 / count;
      const float cb = c2 * r, cc = __builtin_fmaf(-(c2 * mu), r, bb);
      if (gg == g) {
        ca_s[tid] = A;
        cb_s[tid] = cb;
        cc_s[tid] = cc;
      }
      if (ch == 0 && gg == g) {
        coef[(gg * 3 + 0) * C + c] = A;
        coef[(gg * 3 + 1) * C + c] = cb;
        coef[(gg * 3 + 2) * C + c] = cc;
      }
    }
    __syncthreads();
  }
  if (writer && tid < BNF_CW) {
    if (dgamma) dgamma[c0 + tid] = dg;
    if (dbeta) dbeta[c0 + tid] = db;
  }
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ca[i] = ca_s[8 * (tid & 7) + i];
    cb[i] = cb_s[8 * (tid & 7) + i];
    cc[i] = cc_s[8 * (tid & 7) + i];
  }
#pragma unroll
  for (int it = 0; it < BNF_ITERS; ++it) {
    const int r = r0 + rt + 32 * it;
    if (r < r1) {
      float dv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float ag = act_grad_from_out((float)yr[it][i], act, leak);
        dv[i] = __builtin_fmaf(ca[i], (float)dr[it][i] * ag, __builtin_fmaf(cb[i], (float)xr[it][i], cc[i]));
      }
      bnf_store8(dx + (size_t)r * C + vc, dv);
    }
  }
}

// rows per chunk (32..128, a multiple of 32): the largest that still gives >= 256 workgroups
inline int bnfold_rch(int C, int rows) {
  int rch = 32 * BNF_ITERS;
  while (rch > 32 && (long long)(C / BNF_CW) * ((rows + rch - 1) / rch) < 256) rch >>= 1;
  return rch;
}

}  // namespace dcg

using namespace dcg;

extern "C" int DCG_API(dcg_bnfold_ok)(int ppg, int groups, int C, int rows_per_group) {
  return ppg >= 1 && ppg <= 256 && groups >= 1 && C % BNF_CW == 0 && rows_per_group >= 1 ? 1 : 0;
}

extern "C" int DCG_API(dcg_bnfold_fwd)(const float* part, int ppg, int groups, int C, int rpg, double count,
                                       const float* gamma, const float* beta, float eps, float* mean, float* rstd,
                                       float* scale, float* shift, float* ema_mean, float* ema_var, float decay,
                                       const elem_t* x, elem_t* y, int act, float leak, hipStream_t s) {
  if (!DCG_API(dcg_bnfold_ok)(ppg, groups, C, rpg)) return -2;
  const int rch = bnfold_rch(C, groups * rpg), chunks = (rpg + rch - 1) / rch;
  if ((long long)groups * chunks >= 65536) return -3;
  hipLaunchKernelGGL(bnfold_fwd_kernel, dim3(C / BNF_CW, groups * chunks), dim3(256), 0, s, part, ppg, C, rpg, rch,
                     chunks, count, gamma, beta, eps, mean, rstd, scale, shift, ema_mean, ema_var, decay, x, y, act,
                     leak);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_bnfold_bwd)(const float* part, int ppg, int groups, int C, int rpg, float count,
                                       const float* gamma, const float* mean, const float* rstd, float* dgamma,
                                       float* dbeta, float* coef, const elem_t* dy, const elem_t* y, const elem_t* x,
                                       elem_t* dx, int act, float leak, hipStream_t s) {
  if (!DCG_API(dcg_bnfold_ok)(ppg, groups, C, rpg)) return -2;
  const int rch = bnfold_rch(C, groups * rpg), chunks = (rpg + rch - 1) / rch;
  if ((long long)groups * chunks >= 65536) return -3;
  hipLaunchKernelGGL(bnfold_bwd_kernel, dim3(C / BNF_CW, groups * chunks), dim3(256), 0, s, part, ppg, groups, C, rpg,
                     rch, chunks, count, gamma, mean, rstd, dgamma, dbeta, coef, dy, y, x, dx, act, leak);
  return (int)hipGetLastError();
}
