// dcg-variants: bf16 f16 f32
// Device-side TensorBoard summary statistics: the reference computes
// `zero_fraction` and histograms as graph ops next to the data (`_activation_summary`,
// distriubted_model.py:75-80; per-variable histograms, image_train.py:86-89,114-115). Here one
// launch per tensor reduces it ON THE DEVICE to min / max / count / sum / sum of squares /
// zero count and the bucket counts over TF's default histogram edges (obs/events.py), so a
// summary step copies a few KB to the host instead of every activation and weight.
//
// Bucketing = numpy.searchsorted(edges, v, side="left"): bucket = number of edges < v (binary
// search in a double copy of the edges in LDS; values are exact in double). Counts are integer
// LDS atomics (order-independent), the float sums a fixed-order tree per block, and the blocks'
// partial rows [min, max, n, sum, sumsq, zeros, counts...] are combined in block order by the
// last-arriving block (agent-scope counter, re-armed) -- bitwise deterministic.
#include "kernels.h"

namespace dcg {

constexpr int SUMMARY_MAX_BINS = 2048;

__global__ __launch_bounds__(256) void tensor_summary_kernel(const void* __restrict__ x, int x_dtype, size_t n,
                                                             const double* __restrict__ edges, int nbins,
                                                             double* __restrict__ out, double* part,
                                                             unsigned* counter) {
  __shared__ double e_s[SUMMARY_MAX_BINS];
  __shared__ unsigned cnt[SUMMARY_MAX_BINS];
  __shared__ double red[5][4];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int E = nbins - 1;
  for (int i = tid; i < E; i += 256) e_s[i] = edges[i];
  for (int i = tid; i < nbins; i += 256) cnt[i] = 0u;
  __syncthreads();
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t e0 = (size_t)blockIdx.x * per, e1 = e0 + per < n ? e0 + per : n;
  double mn = __builtin_inf(), mx = -__builtin_inf(), sm = 0.0, sq = 0.0, zr = 0.0;
  for (size_t i = e0 + tid; i < e1; i += 256) {
    const float v = x_dtype == 0 ? reinterpret_cast<const float*>(x)[i] : (float)reinterpret_cast<const elem_t*>(x)[i];
    const double d = (double)v;
    mn = fmin(mn, d);
    mx = fmax(mx, d);
    sm += d;
    sq += d * d;
    zr += v == 0.f ? 1.0 : 0.0;
    int lo = 0, hi = E;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (e_s[mid] < d) lo = mid + 1;
      else hi = mid;
    }
    atomicAdd(&cnt[lo], 1u);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_xor(mn, o, 64));
    mx = fmax(mx, __shfl_xor(mx, o, 64));
    sm += __shfl_xor(sm, o, 64);
    sq += __shfl_xor(sq, o, 64);
    zr += __shfl_xor(zr, o, 64);
  }
  if (lane == 0) {
    red[0][wave] = mn; red[1][wave] = mx; red[2][wave] = sm; red[3][wave] = sq; red[4][wave] = zr;
  }
  __syncthreads();
  const int W = nbins + 6;
  const __amdgpu_buffer_rsrc_t rp = make_rsrc(part, (uint32_t)((size_t)gridDim.x * W * 8));
  const uint32_t row = (uint32_t)blockIdx.x * (uint32_t)W;
  if (tid == 0) {
    st_sc1_f64(rp, (row + 0) * 8u, fmin(fmin(red[0][0], red[0][1]), fmin(red[0][2], red[0][3])));
    st_sc1_f64(rp, (row + 1) * 8u, fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3])));
    st_sc1_f64(rp, (row + 2) * 8u, (double)(e1 > e0 ? e1 - e0 : 0));
    st_sc1_f64(rp, (row + 3) * 8u, (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]));
    st_sc1_f64(rp, (row + 4) * 8u, (red[3][0] + red[3][1]) + (red[3][2] + red[3][3]));
    st_sc1_f64(rp, (row + 5) * 8u, (red[4][0] + red[4][1]) + (red[4][2] + red[4][3]));
  }
  for (int b = tid; b < nbins; b += 256) st_sc1_f64(rp, (row + 6 + (uint32_t)b) * 8u, (double)cnt[b]);
  if (!last_arrival(counter, gridDim.x, &flag)) return;
  const int nb = (int)gridDim.x;
  for (int col = tid; col < W; col += 256) {
    double a = col == 0 ? __builtin_inf() : (col == 1 ? -__builtin_inf() : 0.0);
    for (int b0 = 0; b0 < nb; b0 += 8) {  // 8 partial loads in flight per round
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = b0 + u < nb ? ld_sc1_f64(rp, ((uint32_t)(b0 + u) * (uint32_t)W + (uint32_t)col) * 8u)
                           : (col == 0 ? __builtin_inf() : (col == 1 ? -__builtin_inf() : 0.0));
#pragma unroll
      for (int u = 0; u < 8; ++u) a = col == 0 ? fmin(a, v[u]) : (col == 1 ? fmax(a, v[u]) : a + v[u]);
    }
    out[col] = a;
  }
}

}  // namespace dcg

extern "C" int DCG_API(dcg_tensor_summary)(const void* x, int x_dtype, size_t n, const double* edges, int nbins,
                                           double* out, double* part, unsigned* counter, int blocks, hipStream_t s) {
  if (nbins < 2 || nbins > dcg::SUMMARY_MAX_BINS || blocks < 1 || (x_dtype != 0 && x_dtype != 1)) return -2;
  hipLaunchKernelGGL(dcg::tensor_summary_kernel, dim3(blocks), dim3(256), 0, s, x, x_dtype, n, edges, nbins, out, part,
                     counter);
  return (int)hipGetLastError();
}
