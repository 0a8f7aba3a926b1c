// dcg-variants: bf16 f16 f32
// Small fused kernels of the DCGAN step for gfx950:
//   * BCE-with-logits, all 3 reference losses + both logit gradients in ONE kernel (K15/K16)
//   * linear layers: G projection z->h0 (K1), its weight gradient (K2), D's 1-output head
//     (GEMV) and its gradients
//   * TF-form Adam over a flat fp32 buffer + device-side beta powers (K17, graph-capturable)
//   * elem_t weight packing (natural + per-tap transposed / im2col-ordered copies)
//   * Philox-4x32-10 z ~ U(-1,1) keyed by a device step counter (K19, graph-capturable)
//   * stride-2 TF-SAME im2col for 3-channel tensors, dtype casts
#include <algorithm>

#include "kernels.h"

namespace dcg {

// ---------------------------------------------------------------- losses
// logits: [2B] (real rows first). out[0..3] = d_loss_real, d_loss_fake, g_loss, d_loss;
// dl_d[2B] = d d_loss / d logit; dl_g[B] = d g_loss / d logit_fake; prob[2B] = sigmoid.
// The block-wide body, shared by the standalone kernel and the head GEMV's last-arriving block;
// logit(i) fetches logit i.
template <typename F>
__device__ __forceinline__ void gan_loss_block(F logit, int B, float* __restrict__ out, float* __restrict__ dl_d,
                                               float* __restrict__ dl_g, float* __restrict__ prob,
                                               const float* __restrict__ ls) {
  __shared__ float red[3][256];
  float lr = 0.f, lf = 0.f, lg = 0.f;
  const float invB = 1.f / (float)B;
  // fp16 training: the gradient seeds carry the dynamic loss scale ls[0] (the losses do not)
  const float gB = ls ? ls[0] * invB : invB;
  for (int i = threadIdx.x; i < 2 * B; i += 256) {
    const float x = logit(i);
    const float sp = log1pf(expf(-fabsf(x)));
    const float sg = 1.f / (1.f + expf(-x));
    if (prob) prob[i] = sg;
    if (i < B) {
      lr += fmaxf(x, 0.f) - x + sp;          // target 1
      dl_d[i] = (sg - 1.f) * gB;
    } else {
      lf += fmaxf(x, 0.f) + sp;              // target 0
      lg += fmaxf(x, 0.f) - x + sp;          // target 1 (non-saturating G loss)
      dl_d[i] = sg * gB;
      dl_g[i - B] = (sg - 1.f) * gB;
    }
  }
  red[0][threadIdx.x] = lr;
  red[1][threadIdx.x] = lf;
  red[2][threadIdx.x] = lg;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float a = red[0][0] * invB, b = red[1][0] * invB, c = red[2][0] * invB;
    out[0] = a; out[1] = b; out[2] = c; out[3] = a + b;
  }
}

__global__ __launch_bounds__(256) void gan_loss_kernel(const float* __restrict__ logits, int B,
                                                       float* __restrict__ out, float* __restrict__ dl_d,
                                                       float* __restrict__ dl_g, float* __restrict__ prob,
                                                       const float* __restrict__ ls) {
  gan_loss_block([&](int i) { return logits[i]; }, B, out, dl_d, dl_g, prob, ls);
}

// ---------------------------------------------------------------- Philox z ~ U(-1, 1)
__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                             uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
  const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
  const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
  c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
}

// 4 uniforms of counter i4 (Philox-4x32-10 keyed by seed, counter = (i4, step, stream)) in [lo, hi)
__device__ __forceinline__ float philox_uniform_at(size_t idx, uint64_t seed, uint64_t st, uint64_t stream_id,
                                                   float lo, float hi) {
  const size_t i4 = idx >> 2;
  uint32_t c0 = (uint32_t)i4, c1 = (uint32_t)(i4 >> 32), c2 = (uint32_t)st, c3 = (uint32_t)(st >> 32) ^ (uint32_t)stream_id;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const int j = (int)(idx & 3);
  const uint32_t cj = j == 0 ? c0 : (j == 1 ? c1 : (j == 2 ? c2 : c3));
  return lo + (hi - lo) * ((float)(cj >> 8) * (1.0f / 16777216.0f));
}

// ---------------------------------------------------------------- linear: out = z @ W + b
// z fp32 [B][K], W fp32 [K][N], out elem_t [B][N]; block = 256 columns x RB rows.
// Latency-bound (each thread walks K = 100 W rows): 20 independent W loads in flight.
// stats != nullptr: also the BN partial statistics of the stored (rounded) output, channel =
// column % C, one partial row per (row block, column / C) -> part[P][2][C] (no colstats pass).
// gen_step != nullptr: z is not read but generated here -- z ~ U(-1,1) by Philox keyed by
// (gen_seed, *gen_step), bit-identical to philox_uniform_kernel -- and written to z by the
// column-0 blocks (the backward and the summaries read it): one launch less per step.
template <int RB>
__global__ __launch_bounds__(256) void linear_fwd_kernel(float* __restrict__ z, const float* __restrict__ W,
                                                         const float* __restrict__ bias, elem_t* __restrict__ out,
                                                         int B, int K, int N, float* __restrict__ stats, int C,
                                                         const unsigned long long* __restrict__ gen_step,
                                                         uint64_t gen_seed) {
  extern __shared__ __attribute__((aligned(16))) float zs[];  // [RB][K]
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int r0 = blockIdx.y * RB;
  const uint64_t st = gen_step ? gen_step[0] : 0ull;
  for (int i = threadIdx.x; i < RB * K; i += 256) {
    const int r = i / K, k = i - r * K;
    float v = 0.f;
    if (r0 + r < B) {
      const size_t idx = (size_t)(r0 + r) * K + k;
      if (gen_step) {
        v = philox_uniform_at(idx, gen_seed, st, 0, -1.f, 1.f);
        if (blockIdx.x == 0) z[idx] = v;
      } else {
        v = z[idx];
      }
    }
    zs[i] = v;
  }
  __syncthreads();
  if (n >= N) return;
  float acc[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc[r] = 0.f;
  // z is read from LDS as float4 (4 k per ds_read_b128, broadcast): with scalar reads the loop
  // was LDS-instruction bound (8 rows x 100 k reads per thread)
  constexpr int KU = 20;
  int k = 0;
  if ((K & 3) == 0) {
    for (; k + KU <= K; k += KU) {
      float w[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) w[u] = W[(size_t)(k + u) * N + n];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int u4 = 0; u4 < KU / 4; ++u4) {
          const f32x4 zv = *reinterpret_cast<const f32x4*>(zs + r * K + k + 4 * u4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[r] += zv[e] * w[4 * u4 + e];
        }
    }
  }
  for (; k < K; ++k) {
    const float w = W[(size_t)k * N + n];
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] += zs[r * K + k] * w;
  }
  const float b = bias ? bias[n] : 0.f;
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int r = 0; r < RB; ++r)
    if (r0 + r < B) {
      const elem_t o = (elem_t)(acc[r] + b);
      out[(size_t)(r0 + r) * N + n] = o;
      const float v = (float)o;
      s += v;
      s2 += v * v;
    }
  if (stats) {
    const int sp = n / C, c = n - sp * C;
    const size_t prow = (size_t)blockIdx.y * (N / C) + sp;
    stats[(prow * 2 + 0) * C + c] = s;
    stats[(prow * 2 + 1) * C + c] = s2;
  }
}

// dW[K][N] = z^T @ dh (fp32 out), db[N] = sum_b dh; block = 256 columns x KC k-rows
template <int KC>  // KC % 4 == 0
__global__ __launch_bounds__(256) void linear_wgrad_kernel(const float* __restrict__ z, const elem_t* __restrict__ dh,
                                                           float* __restrict__ dW, float* __restrict__ db, int B,
                                                           int K, int N) {
  extern __shared__ __attribute__((aligned(16))) float zs[];  // [B][KC]
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int k0 = blockIdx.y * KC;
  for (int i = threadIdx.x; i < B * KC; i += 256) {
    const int b = i / KC, k = i - b * KC;
    zs[i] = (k0 + k < K) ? z[(size_t)b * K + k0 + k] : 0.f;
  }
  __syncthreads();
  if (n >= N) return;
  float acc[KC];
  float sb = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) acc[k] = 0.f;
  int b = 0;
  for (; b + 8 <= B; b += 8) {  // 8 dh loads in flight, z rows as float4 LDS reads
    float g[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) g[u] = (float)dh[(size_t)(b + u) * N + n];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sb += g[u];
#pragma unroll
      for (int k4 = 0; k4 < KC / 4; ++k4) {
        const f32x4 zv = *reinterpret_cast<const f32x4*>(zs + (b + u) * KC + 4 * k4);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[4 * k4 + e] += zv[e] * g[u];
      }
    }
  }
  for (; b < B; ++b) {
    const float g = (float)dh[(size_t)b * N + n];
    sb += g;
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[k] += zs[b * KC + k] * g;
  }
#pragma unroll
  for (int k = 0; k < KC; ++k)
    if (k0 + k < K) dW[(size_t)(k0 + k) * N + n] = acc[k];
  if (db && blockIdx.y == 0) db[n] = sb;
}

// D head: logits[r] = sum_k x[r][k] * w[k] + b ; one wave per row, x elem_t [R][K], K % 512 == 0
struct HeadLossArgs {  // fused gan loss (counter == nullptr: plain GEMV)
  unsigned* counter;
  float* out;
  float* dl_d;
  float* dl_g;
  float* prob;
  const float* ls;
};

// BNA (optional): x is the top BN layer's PRE-BN input; the head applies that BN + activation on
// the fly (y = act(x * scale[g][c] + shift[g][c]), c = k % C, g = row / rpg), writes y (the layer's
// activation, which the backward reads) and dots the stored (rounded) y -- the layer's separate
// BN-apply launch folded into the head.
struct HeadBnArgs {
  const float* scale; const float* shift; int C, rpg, act; float leak; elem_t* y;
};

template <bool BNA>
__global__ __launch_bounds__(256) void gemv_head_kernel(const elem_t* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ b, float* __restrict__ out, int R,
                                                        int K, HeadLossArgs L, HeadBnArgs bn) {
  // one workgroup per row, each of the 4 waves a quarter of K with all its loads issued up
  // front (one wave per row walked K serially: latency-bound, 9 us for 256 x 8192)
  __shared__ float part[4];
  const int row = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = K / 4;  // K % 32 == 0 (launcher): 16-byte chunks per quarter
  const elem_t* xr = x + (size_t)row * K + wave * kq;
  const float* wr = w + wave * kq;
  const int grp = BNA ? row / bn.rpg : 0;
  float bsc[BNA ? 8 : 1], bsh[BNA ? 8 : 1];  // BNA: channel (k % C) = lane * 8 % C for every chunk (512 % C == 0)
  if constexpr (BNA) {
    const int c = (lane * 8) % bn.C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsc[e] = bn.scale[grp * bn.C + c + e];
      bsh[e] = bn.shift[grp * bn.C + c + e];
    }
  }
  float s = 0.f;
  for (int k0 = lane * 8; k0 < kq; k0 += 4 * 512) {
    elem8 xv[4];
    f32x4 w0[4], w1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * 512 < kq ? k0 + u * 512 : k0;
      xv[u] = ld8(xr + k);
      w0[u] = *reinterpret_cast<const f32x4*>(wr + k);
      w1[u] = *reinterpret_cast<const f32x4*>(wr + k + 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + u * 512 >= kq) break;
      elem8 xb = xv[u];
      if constexpr (BNA) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xb[e] = (elem_t)apply_act((float)xb[e] * bsc[e] + bsh[e], bn.act, bn.leak);
        st8(bn.y + (size_t)row * K + wave * kq + k0 + u * 512, xb);
      }
      s += (float)xb[0] * w0[u][0] + (float)xb[1] * w0[u][1] + (float)xb[2] * w0[u][2] + (float)xb[3] * w0[u][3] +
           (float)xb[4] * w1[u][0] + (float)xb[5] * w1[u][1] + (float)xb[6] * w1[u][2] + (float)xb[7] * w1[u][3];
    }
  }
  s = wave_sum(s);
  if (lane == 0) part[wave] = s;
  __syncthreads();
  const float logit = ((part[0] + part[1]) + (part[2] + part[3])) + b[0];
  if (!L.counter) {
    if (threadIdx.x == 0) out[row] = logit;
    return;
  }
  // fused 3-loss BCE: the logit is written through (sc1), the last row's block computes the
  // losses and seeds from `sc1` loads of all 2B logits (one launch less per step)
  const __amdgpu_buffer_rsrc_t rl = make_rsrc(out, (uint32_t)(R * 4));
  if (threadIdx.x == 0)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, logit), rl, (uint32_t)row * 4u, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(L.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
    if (last) __hip_atomic_store(L.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  gan_loss_block([&](int i) { return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rl, (uint32_t)i * 4u, 0, 16)); },
                 R / 2, L.out, L.dl_d, L.dl_g, L.prob, L.ls);
}

// dx[r][k] = dl[r] * w[k] (elem_t), 8 per thread
__global__ __launch_bounds__(256) void head_dgrad_kernel(const float* __restrict__ dl, const float* __restrict__ w,
                                                         elem_t* __restrict__ dx, int R, int K) {
  const size_t nv = (size_t)R * K / 8;
  for (size_t v = blockIdx.x * 256 + threadIdx.x; v < nv; v += (size_t)gridDim.x * 256) {
    const size_t e = v * 8;
    const int r = (int)(e / K), k = (int)(e - (size_t)r * K);
    const float g = dl[r];
    elem8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (elem_t)(g * w[k + i]);
    st8(dx + e, o);
  }
}

// head weight-grad partials: part[split][K] = sum_{r in split} x[r][k] * dl[r]
__global__ __launch_bounds__(256) void head_wgrad_kernel(const elem_t* __restrict__ x, const float* __restrict__ dl,
                                                         float* __restrict__ part, int R, int K, int rows_per_split) {
  const int k8 = blockIdx.x * 256 + threadIdx.x;
  const int split = blockIdx.y;
  if (k8 * 8 >= K) return;
  float s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = 0.f;
  const int r0 = split * rows_per_split, r1 = min(R, r0 + rows_per_split);
  for (int r = r0; r < r1; ++r) {
    const float g = dl[r];
    const elem8 xb = ld8(x + (size_t)r * K + k8 * 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] += (float)xb[i] * g;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) part[(size_t)split * K + k8 * 8 + i] = s[i];
}

// db = sum dl (single block)
__global__ void sum_vec_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// D head backward in ONE launch (was: partial wgrad + split reduce + bias sum + dgrad + a
// column-statistics pass of the BN backward below the head):
//   dx[r][k] = dl[r] * w[k] (elem_t);  optional  dW[k] = sum_r xa[r][k] * dl[r], db = sum_r dl[r]
//   optional BN-backward partial statistics of the top BN layer (x = its pre-BN input, y = its
//   activation, both [R][K] = NHWC-flattened [R][K/C][C]): per group of rows_per_group rows and
//   per spatial position s = k / C, part[g * (K/C) + s][0|1][c] = (sum g, sum g * xhat),
//   g = dx * act'(y), xhat = (x - mean[g][c]) * rstd[g][c] -- of the STORED (rounded) dx.
// block = 64 columns (8 chunks of 8, inside one spatial position) x 32 row lanes; row lanes
// reduce through LDS in a fixed order (deterministic). Block 0's second wave sums dl for db.
// Row splits (gridDim.y = RS > 1): workgroup (x, y) takes rows [y R/RS, (y+1) R/RS) of column block
// x -- RS times the workgroups for the same bytes. The BN-statistics partial rows become
// [(g RS + y) S + sp] (zeros for a group the split does not touch); dW partials go to dw_ws[y][K]
// (write-through) and the last of the RS arrivals per column block (counter dw_ctr[x], re-armed)
// sums them in split order -- deterministic.
__global__ __launch_bounds__(256) void head_bwd_kernel(const elem_t* __restrict__ xa, const float* __restrict__ dl,
                                                       const float* __restrict__ w, elem_t* __restrict__ dx,
                                                       float* __restrict__ dW, float* __restrict__ db, int R, int K,
                                                       const elem_t* __restrict__ bx, const elem_t* __restrict__ by,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       int C, int rpg, int act, float leak, float* __restrict__ part,
                                                       float* __restrict__ dw_ws, unsigned* __restrict__ dw_ctr) {
  __shared__ float red[32][65];
  __shared__ float bred[2][2][32][65];  // [group][stat][lane][col]
  const int tid = threadIdx.x, c = tid & 7, rl = tid >> 3;
  const int k = blockIdx.x * 64 + c * 8;
  const bool kok = k < K;  // K % 64 == 0 when stats are requested (launcher); K % 8 otherwise
  const bool stats = bx != nullptr;
  const int ch = stats ? k % C : 0;
  float s[8], wv[8], mu[2][8], rs[2][8], t1[2][8], t2[2][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s[i] = 0.f;
    wv[i] = kok ? w[k + i] : 0.f;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      mu[g][i] = (stats && kok && g * rpg < R) ? mean[g * C + ch + i] : 0.f;
      rs[g][i] = (stats && kok && g * rpg < R) ? rstd[g * C + ch + i] : 0.f;
      t1[g][i] = 0.f;
      t2[g][i] = 0.f;
    }
  }
  const float slope = act == ACT_LRELU ? leak : 0.f;
  const int RS = gridDim.y, rsp = blockIdx.y;
  const int r_lo = rsp * (R / RS), r_hi = RS > 1 ? r_lo + R / RS : R;
  if (kok) {
    for (int rb = r_lo + rl; rb < r_hi; rb += 4 * 32) {  // 4 rows per iteration, loads first
      elem8 xv[4], yv[4], xb[4];
      float gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 32 * u < r_hi ? rb + 32 * u : rb;
        const size_t o = (size_t)r * K + k;
        xv[u] = xa ? ld8(xa + o) : (elem8)(elem_t)0.f;
        if (stats) {
          yv[u] = ld8(by + o);
          xb[u] = ld8(bx + o);
        }
        gv[u] = dl[r];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 32 * u;
        if (r >= r_hi) break;
        const int grp = r >= rpg ? 1 : 0;
        const elem8 xe = xv[u];
        elem8 ob;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s[i] += (float)xe[i] * gv[u];
          ob[i] = (elem_t)(gv[u] * wv[i]);
        }
        st8(dx + (size_t)r * K + k, ob);
        if (stats) {
          const elem8 ye = yv[u], be = xb[u];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float g = (float)ob[i] * ((float)ye[i] > 0.f ? 1.f : slope);
            const float xh = ((float)be[i] - mu[grp][i]) * rs[grp][i];
            t1[grp][i] += g;
            t2[grp][i] += g * xh;
          }
        }
      }
    }
  }
  if (dW) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[rl][c * 8 + i] = s[i];
  }
  if (stats) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bred[g][0][rl][c * 8 + i] = t1[g][i];
        bred[g][1][rl][c * 8 + i] = t2[g][i];
      }
  }
  __syncthreads();
  if (dW && RS == 1 && tid < 64 && blockIdx.x * 64 + tid < K) {
    float a = 0.f;
    for (int l = 0; l < 32; ++l) a += red[l][tid];
    dW[blockIdx.x * 64 + tid] = a;
  }
  if (dW && RS > 1) {  // split partial, then the last arrival of the column block sums the splits in order
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(dw_ws, (uint32_t)((size_t)RS * K * 4));
    const int col = blockIdx.x * 64 + tid;
    if (tid < 64 && col < K) {
      float a = 0.f;
      for (int l = 0; l < 32; ++l) a += red[l][tid];
      st_sc1_f32(rw, (uint32_t)((size_t)rsp * K + col) * 4u, a);
    }
    __shared__ int last_s;
    if (last_arrival(dw_ctr + blockIdx.x, (unsigned)RS, &last_s) && tid < 64 && col < K) {
      float a = 0.f;
      for (int q = 0; q < RS; ++q) a += ld_sc1_f32(rw, (uint32_t)((size_t)q * K + col) * 4u);
      dW[col] = a;
    }
  }
  if (stats) {
    for (int h = 16; h > 0; h >>= 1) {  // fixed-order tree over the 32 row lanes
      for (int q = tid; q < 2 * 2 * h * 64; q += 256) {
        const int col = q & 63, l = (q >> 6) % h, gs = q / (64 * h);
        float* base = &bred[gs >> 1][gs & 1][0][0];
        base[l * 65 + col] += base[(l + h) * 65 + col];
      }
      __syncthreads();
    }
    const int groups = (R + rpg - 1) / rpg, S = K / C;
    const int k0 = blockIdx.x * 64, sp = k0 / C, c0 = k0 % C;
    for (int q = tid; q < groups * 2 * 64; q += 256) {
      const int col = q & 63, st = (q >> 6) & 1, g = q >> 7;
      part[((size_t)((g * RS + rsp) * S + sp) * 2 + st) * C + c0 + col] = bred[g][st][0][col];
    }
  }
  if (db && blockIdx.x == 0 && blockIdx.y == 0 && tid >= 64 && tid < 128) {
    const int lane = tid - 64;
    float a = 0.f;
    for (int r = lane; r < R; r += 64) a += dl[r];
    a = wave_sum(a);
    if (lane == 0) db[0] = a;
  }
}

// ---------------------------------------------------------------- TF Adam
// lr_t = lr*sqrt(1-b2^t)/(1-b1^t) from device powers (= b^t); w -= lr_t*m/(sqrt(v)+eps)
// GW = bf16: the gradient is read from the all-reduced bf16 wire buffer (DDP with a bf16 wire:
// no bf16 -> fp32 copy-back after the collective; the values are the same)
template <typename GW>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ w, elem_t* __restrict__ wbf,
                                                   const GW* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, const float* __restrict__ powers, size_t n,
                                                   float lr, float b1, float b2, float eps, float gscale,
                                                   const float* __restrict__ ls) {
  // dynamic loss scaling (fp16): ls = [scale, overflow flag, good steps]; an overflowed step
  // is skipped entirely (weights, slots and the bf16/fp16 mirror untouched), else unscale
  if (ls) {
    if (ls[1] != 0.f) return;
    gscale /= ls[0];
  }
  // wbf (optional): elem_t mirror of the updated weights in the SAME flat layout -- the only
  // weight copy the conv kernels read (they take either operand layout), so no repack pass
  const float lr_t = lr * sqrtf(1.f - powers[1]) / (1.f - powers[0]);
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 gv;
    if constexpr (sizeof(GW) == 4) {
      gv = reinterpret_cast<const f32x4*>(g)[i] * gscale;
    } else {
      typedef GW gw4 __attribute__((ext_vector_type(4)));
      const gw4 gb = reinterpret_cast<const gw4*>(g)[i];
      gv = (f32x4){(float)gb[0], (float)gb[1], (float)gb[2], (float)gb[3]} * gscale;
    }
    f32x4 mv = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    f32x4 wv = reinterpret_cast<f32x4*>(w)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // explicit fma: the same rounding as every other TF-Adam path
      mv[k] = __builtin_fmaf(b1, mv[k], (1.f - b1) * gv[k]);
      vv[k] = __builtin_fmaf(b2, vv[k], (1.f - b2) * gv[k] * gv[k]);
      wv[k] -= lr_t * mv[k] / (sqrtf(vv[k]) + eps);
    }
    reinterpret_cast<f32x4*>(m)[i] = mv;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    reinterpret_cast<f32x4*>(w)[i] = wv;
    if (wbf) {
      elem4 o = {(elem_t)wv[0], (elem_t)wv[1], (elem_t)wv[2], (elem_t)wv[3]};
      reinterpret_cast<elem4*>(wbf)[i] = o;
    }
  }
  for (size_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float gv = (float)g[i] * gscale;
    m[i] = __builtin_fmaf(b1, m[i], (1.f - b1) * gv);
    v[i] = __builtin_fmaf(b2, v[i], (1.f - b2) * gv * gv);
    w[i] -= lr_t * m[i] / (sqrtf(v[i]) + eps);
    if (wbf) wbf[i] = (elem_t)w[i];
  }
}

// Both TF-Adams (G then D, each with its own lr_t from its own device beta powers) + the
// step-end update in ONE launch (single-process bf16 path): the blocks walk the two flat
// buffers' float4s as one index space; the last block to finish (agent counter) advances both
// beta-power pairs and the global step -- after every block has read the powers (at its start).
struct Adam2Set {
  float* w;
  elem_t* wbf;
  const float* g;
  float* m;
  float* v;
  float* powers;
  size_t n;  // % 4 == 0 (64-aligned ParamSet padding)
  float lr, b1, b2, eps;
};

__global__ __launch_bounds__(256) void adam2_kernel(Adam2Set A, Adam2Set D, float gscale,
                                                    unsigned long long* __restrict__ step,
                                                    unsigned* __restrict__ counter, unsigned blocksA) {
  __shared__ int flag;
  // block-uniform split of the grid between the two sets (per-lane selection of the kernarg
  // structs made the compiler spill them to scratch: 116 us instead of ~52)
  const unsigned gA = blocksA;
  const bool inA = blockIdx.x < gA;
  f32x4* __restrict__ w = reinterpret_cast<f32x4*>(inA ? A.w : D.w);
  elem4* __restrict__ wbf = reinterpret_cast<elem4*>(inA ? A.wbf : D.wbf);
  const f32x4* __restrict__ g = reinterpret_cast<const f32x4*>(inA ? A.g : D.g);
  f32x4* __restrict__ m = reinterpret_cast<f32x4*>(inA ? A.m : D.m);
  f32x4* __restrict__ v = reinterpret_cast<f32x4*>(inA ? A.v : D.v);
  const float* pw = inA ? A.powers : D.powers;
  const float b1 = inA ? A.b1 : D.b1, b2 = inA ? A.b2 : D.b2, eps = inA ? A.eps : D.eps;
  const float lr_t = (inA ? A.lr : D.lr) * sqrtf(1.f - pw[1]) / (1.f - pw[0]);
  const size_t n4 = (inA ? A.n : D.n) / 4;
  const unsigned b0 = inA ? blockIdx.x : blockIdx.x - gA, nb = inA ? gA : gridDim.x - gA;
  for (size_t i = (size_t)b0 * 256 + threadIdx.x; i < n4; i += (size_t)nb * 256) {
    const f32x4 gv = g[i] * gscale;
    f32x4 mv = m[i];
    f32x4 vv = v[i];
    f32x4 wv = w[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mv[k] = __builtin_fmaf(b1, mv[k], (1.f - b1) * gv[k]);
      vv[k] = __builtin_fmaf(b2, vv[k], (1.f - b2) * gv[k] * gv[k]);
      wv[k] -= lr_t * mv[k] / (sqrtf(vv[k]) + eps);
    }
    m[i] = mv;
    v[i] = vv;
    w[i] = wv;
    const elem4 o = {(elem_t)wv[0], (elem_t)wv[1], (elem_t)wv[2], (elem_t)wv[3]};
    wbf[i] = o;
  }
  // counter == nullptr: a first part of the update (the beta powers and the step are advanced
  // by a later adam2 launch over the remaining ranges)
  if (!counter) return;
  // last arrival: every block has read the powers above before it increments the counter
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = old == gridDim.x - 1;
    if (flag) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (flag && threadIdx.x == 0) {
    A.powers[0] *= A.b1;
    A.powers[1] *= A.b2;
    D.powers[0] *= D.b1;
    D.powers[1] *= D.b2;
    if (step) step[0] += 1ull;
  }
}

// after both Adams: beta powers *= beta (TF variable update) and the global step counter
__global__ void step_end_kernel(float* __restrict__ pd, float* __restrict__ pg, float b1d, float b2d, float b1g,
                                float b2g, unsigned long long* __restrict__ step, float* __restrict__ ls,
                                int growth_interval) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    bool skipped = false;
    if (ls) {  // dynamic loss scale: halve on overflow, double after growth_interval good steps
      skipped = ls[1] != 0.f;
      if (skipped) {
        ls[0] = fmaxf(ls[0] * 0.5f, 1.f);
        ls[2] = 0.f;
      } else if ((ls[2] += 1.f) >= (float)growth_interval) {
        ls[0] = fminf(ls[0] * 2.f, 16777216.f);
        ls[2] = 0.f;
      }
      ls[1] = 0.f;
    }
    if (!skipped) {  // a skipped step does not advance the Adam beta powers
      if (pd) { pd[0] *= b1d; pd[1] *= b2d; }
      if (pg) { pg[0] *= b1g; pg[1] *= b2g; }
    }
    if (step) step[0] += 1ull;
  }
}

// overflow detection for dynamic loss scaling: any non-finite gradient sets ls[1]
__global__ __launch_bounds__(256) void nonfinite_check_kernel(const float* __restrict__ g, size_t n,
                                                              float* __restrict__ ls) {
  bool bad = false;
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const f32x4 v = reinterpret_cast<const f32x4*>(g)[i];
    bad |= !(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]) && isfinite(v[3]));
  }
  for (size_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) ls[1] = 1.f;  // benign race: every writer stores 1
}

// ---------------------------------------------------------------- weight packing
// src fp32 [T][A][Bd] -> nat elem_t (same order, optional) and tr elem_t at t*st + b*sb + a*sa
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ src, uint32_t n, FastDiv fd_b,
                                                   FastDiv fd_a, elem_t* __restrict__ nat, elem_t* __restrict__ tr,
                                                   int st, int sb, int sa) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float v = src[i];
    const uint32_t ta = fdiv(i, fd_b);
    const uint32_t b = i - ta * fd_b.d;
    const uint32_t t = fdiv(ta, fd_a);
    const uint32_t a = ta - t * fd_a.d;
    if (nat) nat[i] = (elem_t)v;
    if (tr) tr[t * st + b * sb + a * sa] = (elem_t)v;
  }
}

__global__ __launch_bounds__(256) void philox_uniform_kernel(float* __restrict__ out, size_t n, uint64_t seed,
                                                             const unsigned long long* __restrict__ step,
                                                             uint64_t stream_id, float lo, float hi) {
  const size_t i4 = blockIdx.x * 256 + threadIdx.x;
  if (i4 * 4 >= n) return;
  const uint64_t st = step ? step[0] : 0ull;
  uint32_t c0 = (uint32_t)i4, c1 = (uint32_t)(i4 >> 32), c2 = (uint32_t)st, c3 = (uint32_t)(st >> 32) ^ (uint32_t)stream_id;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const uint32_t c[4] = {c0, c1, c2, c3};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t idx = i4 * 4 + j;
    if (idx < n) {
      const float u = (float)(c[j] >> 8) * (1.0f / 16777216.0f);  // [0, 1)
      out[idx] = lo + (hi - lo) * u;
    }
  }
}

// ---------------------------------------------------------------- im2col (stride 2, TF SAME)
// src elem_t [B][H][W][C] -> dst elem_t [B*Ho*Wo][Kpad], k = tap*C + c (tap = ky*5 + kx), zero pad.
// One workgroup per IM_ROWS output rows of one image: the 2*IM_ROWS+3 input rows they read
// (zero-padded to 2*Wo+3 columns) are staged in LDS once (no 5/2x re-read of shared rows; ~9
// independent loads per thread), then every thread writes several 16-byte chunks of the output
// rows (consecutive threads -> consecutive chunks). Channel count fixed at compile time (CC > 0)
// so k -> (ky, kx, c) is multiply-shift arithmetic.
constexpr int IM_ROWS = 4;
template <int CC>
__global__ __launch_bounds__(256) void im2col_s2_kernel(const elem_t* __restrict__ src, elem_t* __restrict__ dst,
                                                        int Crt, int H, int W, int Ho, int Wo, int pl_y, int pl_x,
                                                        int Kpad, int row_blocks) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  elem_t* band = reinterpret_cast<elem_t*>(smem);  // [2*IM_ROWS+3][Wp][C]
  const int C = CC > 0 ? CC : Crt;
  const int Wp = 2 * Wo + 3, WpC = Wp * C;
  const int b = blockIdx.x / row_blocks, oy0 = (blockIdx.x - b * row_blocks) * IM_ROWS;
  const int nrows = min(IM_ROWS, Ho - oy0);
  const int iy0 = 2 * oy0 - pl_y, ix0 = -pl_x;
  const elem_t* img = src + (size_t)b * H * W * C;
  const int band_n = (2 * nrows + 3) * WpC;
  for (int i = threadIdx.x; i < band_n; i += 256) {
    const int row = i / WpC, rem = i - row * WpC;
    const int col = rem / C, c = rem - col * C;
    const int iy = iy0 + row, ix = ix0 + col;
    elem_t v = (elem_t)0.f;
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) v = img[((size_t)iy * W + ix) * C + c];
    band[i] = v;
  }
  __syncthreads();
  const int KV = Kpad >> 3;
  const int per_row = Wo * KV;
  elem_t* drow = dst + ((size_t)b * Ho + oy0) * Wo * Kpad;
  for (int q = threadIdx.x; q < nrows * per_row; q += 256) {
    const int r = q / per_row, qq = q - r * per_row;
    const int ox = qq / KV, v = qq - ox * KV;
    const elem_t* bp = band + (2 * r * Wp + 2 * ox) * C;
    elem8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = v * 8 + j;
      elem_t val = (elem_t)0.f;
      if (k < 25 * C) {
        const int tap = k / C, c = k - tap * C;
        const int ky = tap / 5, kx = tap - 5 * ky;
        val = bp[(ky * Wp + kx) * C + c];
      }
      o[j] = val;
    }
    st8(drow + (size_t)q * 8, o);
  }
}

// ---------------------------------------------------------------- casts
__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ s, elem_t* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = (elem_t)s[i];
}
__global__ __launch_bounds__(256) void cast_f64_bf16_kernel(const double* __restrict__ s, elem_t* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = (elem_t)(float)s[i];
}
__global__ __launch_bounds__(256) void cast_u8_bf16_kernel(const uint8_t* __restrict__ s, elem_t* __restrict__ d, size_t n,
                                                           float scale, float shift) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    d[i] = (elem_t)((float)s[i] * scale + shift);
}
__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const elem_t* __restrict__ s, float* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = (float)s[i];
}

// sum of `splits` fp32 slabs of `n` elements -> dst (scaled). Block = (256/L) float4 columns x L
// split lanes; each lane sums every L-th slab, then the L partial sums are combined in LDS in a
// fixed order (deterministic). Handles the few-elements / many-slabs shape of small wgrads.
template <int L>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* src, int splits, size_t n,
                                                            float* dst, float scale) {
  constexpr int COLS = 256 / L;
  __shared__ f32x4 red[L][COLS];
  const int col = threadIdx.x % COLS, lane = threadIdx.x / COLS;
  const size_t n4 = n / 4;
  const size_t i = (size_t)blockIdx.x * COLS + col;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    auto slab = [&](int k) { return reinterpret_cast<const f32x4*>(src + (size_t)k * n)[i]; };
    int k = lane;
    for (; k + 3 * L < splits; k += 4 * L) {  // 4 slabs in flight per lane, summed in slab order
      const f32x4 a = slab(k), b = slab(k + L), c = slab(k + 2 * L), d = slab(k + 3 * L);
      s += a;
      s += b;
      s += c;
      s += d;
    }
    for (; k < splits; k += L) s += slab(k);
  }
  red[lane][col] = s;
  __syncthreads();
  if (lane == 0 && i < n4) {
    f32x4 t = red[0][col];
#pragma unroll
    for (int l = 1; l < L; ++l) t += red[l][col];
    reinterpret_cast<f32x4*>(dst)[i] = t * scale;
  }
  // scalar tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (int)(n - n4 * 4)) {
    const size_t j = n4 * 4 + threadIdx.x;
    float t = 0.f;
    for (int k = 0; k < splits; ++k) t += src[(size_t)k * n + j];
    dst[j] = t * scale;
  }
}

}  // namespace dcg

using namespace dcg;

static inline unsigned grid_for(size_t n, size_t per = 256) {
  size_t b = (n + per - 1) / per;
  if (b > 16384) b = 16384;
  return (unsigned)(b ? b : 1);
}

extern "C" int DCG_API(dcg_gan_loss)(const float* logits, int B, float* out, float* dl_d, float* dl_g, float* prob,
                                      const float* ls, hipStream_t s) {
  hipLaunchKernelGGL(gan_loss_kernel, dim3(1), dim3(256), 0, s, logits, B, out, dl_d, dl_g, prob, ls);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_linear_fwd)(float* z, const float* W, const float* b, elem_t* out, int B, int K, int N,
                              float* stats, int C, const unsigned long long* gen_step, uint64_t gen_seed,
                              hipStream_t s) {
  if (stats && (C <= 0 || N % C)) return -2;
  constexpr int RB = 8;  // (N/256) x (B/8) = 512 blocks for the 64x64 model at B=128
  dim3 grid((N + 255) / 256, (B + RB - 1) / RB);
  hipLaunchKernelGGL((linear_fwd_kernel<RB>), grid, dim3(256), RB * K * sizeof(float), s, z, W, b, out, B, K, N,
                     stats, C, gen_step, gen_seed);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_linear_wgrad)(const float* z, const elem_t* dh, float* dW, float* db, int B, int K, int N,
                                hipStream_t s) {
  constexpr int KC = 8;  // 8 k-rows per block: (N/256) x (K/8) = 416 blocks for the 64x64 model
  if ((size_t)B * KC * sizeof(float) > 65536) return -2;
  dim3 grid((N + 255) / 256, (K + KC - 1) / KC);
  hipLaunchKernelGGL((linear_wgrad_kernel<KC>), grid, dim3(256), B * KC * sizeof(float), s, z, dh, dW, db, B, K, N);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_gemv_head)(const elem_t* x, const float* w, const float* b, float* out, int R, int K,
                                      unsigned* counter, float* loss_out, float* dl_d, float* dl_g, float* prob,
                                      const float* ls, hipStream_t s) {
  if (K % 32 || (counter && (R % 2 || !loss_out || !dl_d || !dl_g))) return -2;
  const dcg::HeadLossArgs L{counter, loss_out, dl_d, dl_g, prob, ls};
  hipLaunchKernelGGL(gemv_head_kernel<false>, dim3(R), dim3(256), 0, s, x, w, b, out, R, K, L, dcg::HeadBnArgs{});
  return (int)hipGetLastError();
}

// the head with the top BN layer's apply + activation fused (x = pre-BN input, y = activation out)
extern "C" int DCG_API(dcg_gemv_head_bn)(const elem_t* x, const float* w, const float* b, float* out, int R, int K,
                                         unsigned* counter, float* loss_out, float* dl_d, float* dl_g, float* prob,
                                         const float* ls, const float* scale, const float* shift, int C, int rpg,
                                         int act, float leak, elem_t* y, hipStream_t s) {
  if (K % 2048 || C % 8 || 512 % C || (counter && (R % 2 || !loss_out || !dl_d || !dl_g)) || !scale || !shift || !y)
    return -2;  // (every 8-element chunk of a lane then holds channels lane * 8 % C ..: loaded once)
  const dcg::HeadLossArgs L{counter, loss_out, dl_d, dl_g, prob, ls};
  const dcg::HeadBnArgs bn{scale, shift, C, rpg, act, leak, y};
  hipLaunchKernelGGL(gemv_head_kernel<true>, dim3(R), dim3(256), 0, s, x, w, b, out, R, K, L, bn);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_head_dgrad)(const float* dl, const float* w, elem_t* dx, int R, int K, hipStream_t s) {
  if (K % 8) return -2;
  hipLaunchKernelGGL(head_dgrad_kernel, dim3(grid_for((size_t)R * K / 8)), dim3(256), 0, s, dl, w, dx, R, K);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_head_wgrad)(const elem_t* x, const float* dl, float* part, int R, int K, int splits,
                              hipStream_t s) {
  if (K % 8) return -2;
  const int rps = (R + splits - 1) / splits;
  dim3 grid((K / 8 + 255) / 256, splits);
  hipLaunchKernelGGL(head_wgrad_kernel, grid, dim3(256), 0, s, x, dl, part, R, K, rps);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_sum_vec)(const float* v, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_vec_kernel, dim3(1), dim3(256), 0, s, v, n, out);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_adam)(float* w, elem_t* wbf, const float* g, float* m, float* v, const float* powers,
                                  size_t n, float lr, float b1, float b2, float eps, float gscale, const float* ls,
                                  const void* g_bf16, hipStream_t s) {
  if (g_bf16)
    hipLaunchKernelGGL(adam_kernel<__bf16>, dim3(grid_for(n / 4 + 1)), dim3(256), 0, s, w, wbf,
                       static_cast<const __bf16*>(g_bf16), m, v, powers, n, lr, b1, b2, eps, gscale, ls);
  else
    hipLaunchKernelGGL(adam_kernel<float>, dim3(grid_for(n / 4 + 1)), dim3(256), 0, s, w, wbf, g, m, v, powers, n, lr,
                       b1, b2, eps, gscale, ls);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_step_end)(float* pd, float* pg, float b1d, float b2d, float b1g, float b2g,
                                      unsigned long long* step, float* ls, int growth_interval, hipStream_t s) {
  hipLaunchKernelGGL(step_end_kernel, dim3(1), dim3(64), 0, s, pd, pg, b1d, b2d, b1g, b2g, step, ls,
                     growth_interval);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_nonfinite_check)(const float* g, size_t n, float* ls, hipStream_t s) {
  hipLaunchKernelGGL(nonfinite_check_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, s, g, n, ls);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_pack)(const float* src, int T, int A, int Bd, elem_t* nat, elem_t* tr, int st, int sb, int sa,
                        hipStream_t s) {
  const size_t n = (size_t)T * A * Bd;
  if (n >= 0x80000000ull) return -3;
  hipLaunchKernelGGL(pack_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, (uint32_t)n, fastdiv_make(Bd),
                     fastdiv_make(A), nat, tr, st, sb, sa);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_philox_uniform)(float* out, size_t n, uint64_t seed, const unsigned long long* step,
                                  uint64_t stream_id, float lo, float hi, hipStream_t s) {
  hipLaunchKernelGGL(philox_uniform_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, out, n, seed, step,
                     stream_id, lo, hi);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_im2col_s2)(const elem_t* src, elem_t* dst, int B, int H, int W, int C, int Ho, int Wo, int pl_y,
                             int pl_x, int Kpad, hipStream_t s) {
  if (Kpad % 8 || Kpad < 25 * C) return -2;
  const size_t shm = (size_t)(2 * dcg::IM_ROWS + 3) * (2 * Wo + 3) * C * sizeof(elem_t);
  if (shm > 64 * 1024) return -2;
  const int row_blocks = (Ho + dcg::IM_ROWS - 1) / dcg::IM_ROWS;
  const dim3 grid((unsigned)(B * row_blocks));
  if (C == 3)
    hipLaunchKernelGGL(im2col_s2_kernel<3>, grid, dim3(256), shm, s, src, dst, C, H, W, Ho, Wo, pl_y, pl_x, Kpad,
                       row_blocks);
  else if (C == 1)
    hipLaunchKernelGGL(im2col_s2_kernel<1>, grid, dim3(256), shm, s, src, dst, C, H, W, Ho, Wo, pl_y, pl_x, Kpad,
                       row_blocks);
  else
    hipLaunchKernelGGL(im2col_s2_kernel<0>, grid, dim3(256), shm, s, src, dst, C, H, W, Ho, Wo, pl_y, pl_x, Kpad,
                       row_blocks);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_cast_to_bf16)(const void* src, int src_dtype, elem_t* dst, size_t n, float scale, float shift,
                                hipStream_t s) {
  // src_dtype: 0 f32, 1 f64, 2 u8 (x*scale+shift)
  if (src_dtype == 0)
    hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const float*)src, dst, n);
  else if (src_dtype == 1)
    hipLaunchKernelGGL(cast_f64_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const double*)src, dst, n);
  else if (src_dtype == 2)
    hipLaunchKernelGGL(cast_u8_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const uint8_t*)src, dst, n, scale,
                       shift);
  else
    return -2;
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_cast_bf16_f32)(const elem_t* src, float* dst, size_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, dst, n);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_head_bwd)(const elem_t* x, const float* dl, const float* w, elem_t* dx, float* dW, float* db,
                                     int R, int K, const elem_t* bx, const elem_t* by, const float* mean,
                                     const float* rstd, int C, int rpg, int act, float leak, float* part,
                                     hipStream_t s) {
  if (K % 8) return -2;
  if (bx && (C <= 0 || C % 64 || K % C || rpg <= 0 || (R + rpg - 1) / rpg > 2 || !by || !mean || !rstd || !part))
    return -2;
  hipLaunchKernelGGL(head_bwd_kernel, dim3((K + 63) / 64), dim3(256), 0, s, x, dl, w, dx, dW, db, R, K, bx, by, mean,
                     rstd, C, rpg > 0 ? rpg : R, act, leak, part, (float*)nullptr, (unsigned*)nullptr);
  return (int)hipGetLastError();
}

// the head backward with RS row splits (R % RS == 0; with statistics, R / RS must divide rpg):
// dw_ws [RS][K] and dw_ctr [ceil(K / 64)] (zero-initialised) when dW != nullptr and RS > 1
extern "C" int DCG_API(dcg_head_bwd_rs)(const elem_t* x, const float* dl, const float* w, elem_t* dx, float* dW,
                                        float* db, int R, int K, const elem_t* bx, const elem_t* by,
                                        const float* mean, const float* rstd, int C, int rpg, int act, float leak,
                                        float* part, int RS, float* dw_ws, unsigned* dw_ctr, hipStream_t s) {
  if (K % 8 || RS < 1 || R % RS) return -2;
  if (bx && (C <= 0 || C % 64 || K % C || rpg <= 0 || (R + rpg - 1) / rpg > 2 || !by || !mean || !rstd || !part ||
             (RS > 1 && rpg % (R / RS))))
    return -2;
  if (dW && RS > 1 && (!dw_ws || !dw_ctr)) return -2;
  hipLaunchKernelGGL(head_bwd_kernel, dim3((K + 63) / 64, RS), dim3(256), 0, s, x, dl, w, dx, dW, db, R, K, bx, by,
                     mean, rstd, C, rpg > 0 ? rpg : R, act, leak, part, dw_ws, dw_ctr);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_adam2)(float* wA, elem_t* wbfA, const float* gA, float* mA, float* vA, float* pA, size_t nA,
                                  float lrA, float b1A, float b2A, float epsA, float* wD, elem_t* wbfD, const float* gD,
                                  float* mD, float* vD, float* pD, size_t nD, float lrD, float b1D, float b2D,
                                  float epsD, float gscale, unsigned long long* step, unsigned* counter,
                                  hipStream_t s) {
  if (nA % 4 || nD % 4 || !wbfA || !wbfD) return -2;
  const dcg::Adam2Set A{wA, wbfA, gA, mA, vA, pA, nA, lrA, b1A, b2A, epsA};
  const dcg::Adam2Set D{wD, wbfD, gD, mD, vD, pD, nD, lrD, b1D, b2D, epsD};
  // ~512 blocks in total (grid-stride loops): every block bumps ONE arrival counter, and a
  // same-address atomic per block serialises (9k blocks: +60 us)
  const size_t q = (nA + nD) / 4;
  unsigned blocksA = (unsigned)std::max<size_t>(1, (512 * (nA / 4) + q - 1) / q);
  unsigned blocksD = (unsigned)std::max<size_t>(1, 512 - std::min<size_t>(511, blocksA));
  hipLaunchKernelGGL(dcg::adam2_kernel, dim3(blocksA + blocksD), dim3(256), 0, s, A, D, gscale, step, counter,
                     blocksA);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_splitk_reduce)(const float* src, int splits, size_t n, float* dst, float scale, hipStream_t s) {
  const size_t n4 = n / 4;
  if (splits >= 256) {  // many slabs of a small result (narrow2 nwgrad partials): 64 lanes per column
    hipLaunchKernelGGL(dcg::splitk_reduce_kernel<64>, dim3((unsigned)((n4 + 3) / 4 + 1)), dim3(256), 0, s, src,
                       splits, n, dst, scale);
  } else if (splits >= 64) {
    hipLaunchKernelGGL(dcg::splitk_reduce_kernel<16>, dim3((unsigned)((n4 + 15) / 16 + 1)), dim3(256), 0, s, src,
                       splits, n, dst, scale);
  } else if (splits >= 8) {
    hipLaunchKernelGGL(dcg::splitk_reduce_kernel<4>, dim3((unsigned)((n4 + 63) / 64 + 1)), dim3(256), 0, s, src,
                       splits, n, dst, scale);
  } else {
    hipLaunchKernelGGL(dcg::splitk_reduce_kernel<1>, dim3((unsigned)((n4 + 255) / 256 + 1)), dim3(256), 0, s, src,
                       splits, n, dst, scale);
  }
  return (int)hipGetLastError();
}
