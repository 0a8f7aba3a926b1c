// Fused conv-GEMM epilogue shared by igemm.hip and igemm3.hip: + bias, per-channel BN partial
// statistics of the stored value, activation, pixel scatter (rowoff), output staged through
// LDS for 16-byte row stores.
//
// Compile-time activation / store mode: a runtime `switch (act)` inside the 64-element loop was
// expanded per element by hipcc (incl. an inlined tanh) into ~200 scalar branches per thread --
// measured 16k cycles per 128x128 workgroup, a quarter of its lifetime. The caller dispatches
// ONCE on (act, vec) and every variant below is straight-line code (validity by selects).
#pragma once
#include "kernels.h"

namespace dcg {

template <int ACT>
__device__ __forceinline__ float act_ct(float v, float leak) {
  if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == ACT_LRELU) return fmaxf(v, leak * v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}

// acc[FM][FN] of a (WM x WN)-wave tile, wave (wm, wn), lane (fr, fq). rowoff[BM] (LDS) holds each
// tile row's output element offset or -1; red[WM][BN][2] and ctile[BM][BN + 8] are LDS scratch.
template <int ACT, bool VEC, int FM, int FN, int TM, int TN, int BN, bool BNB = false>
__device__ __forceinline__ void frag_epilogue(const f32x4 (&acc)[FM][FN], const IGemmArgs& p, const int* rowoff,
                                              float* red, elem_t* ctile, int wm, int wn, int fr, int fq, int n0,
                                              bool do_stats, int m0 = 0) {
  constexpr int CPAD = BN + 8;
  const int N = p.N;
  // the 4 consecutive rows of each M fragment: one 16-byte LDS read per fragment
  int ro[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int4 v = *reinterpret_cast<const int4*>(rowoff + wm * TM + i * 16 + fq * 4);
    ro[i][0] = v.x; ro[i][1] = v.y; ro[i][2] = v.z; ro[i][3] = v.w;
  }
  const bool f32out = p.out_f32 != 0;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * TN + j * 16 + fr;
    const int n = n0 + nl;
    const bool nok = n < N;
    const float bv = (p.bias && nok) ? p.bias[n] : 0.f;
    float s = 0.f, s2 = 0.f;
    float bmu = 0.f, brs = 0.f;
    const float bslope = p.bnb_act == ACT_LRELU ? p.bnb_leak : 0.f;  // relu / lrelu derivative below 0
    if constexpr (BNB) {
      const int g = m0 / p.bnb_rpg;
      bmu = nok ? p.bnb_mean[g * N + n] : 0.f;
      brs = nok ? p.bnb_rstd[g * N + n] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int off = ro[i][r];
        const bool valid = off >= 0 && nok;
        const float v = acc[i][j][r] + bv;
        // statistics of exactly the stored (rounded) tensor: BN forward and backward see one x
        const float vs = f32out ? v : (float)f2bf(v);
        if constexpr (BNB) {
          const int idx = valid ? off + p.cofs + n : 0;
          const float ya = (float)p.bnb_y[idx], xa = (float)p.bnb_x[idx];
          const float gv = vs * (ya > 0.f ? 1.f : bslope);
          s += valid ? gv : 0.f;
          s2 += valid ? gv * (xa - bmu) * brs : 0.f;
        } else {
          s += valid ? vs : 0.f;
          s2 += valid ? vs * vs : 0.f;
        }
        const float o = act_ct<ACT>(v, p.leak);
        if constexpr (VEC) {
          ctile[(wm * TM + i * 16 + fq * 4 + r) * CPAD + nl] = f2bf(o);
        } else if (valid) {
          if (f32out) reinterpret_cast<float*>(p.C)[off + p.cofs + n] = o;
          else reinterpret_cast<elem_t*>(p.C)[off + p.cofs + n] = f2bf(o);
        }
      }
    }
    if (do_stats) {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (fq == 0) {
        red[(wm * BN + nl) * 2 + 0] = s;
        red[(wm * BN + nl) * 2 + 1] = s2;
      }
    }
  }
}

// one uniform dispatch on (act, vec) around the straight-line variants
template <int FM, int FN, int TM, int TN, int BN>
__device__ __forceinline__ void frag_epilogue_dispatch(const f32x4 (&acc)[FM][FN], const IGemmArgs& p,
                                                       const int* rowoff, float* red, elem_t* ctile, int wm, int wn,
                                                       int fr, int fq, int n0, bool do_stats, bool vec, int m0) {
  if (p.bnb_x) {  // data-gradient GEMM feeding a BN backward: C tile only; stats in vec_store_bnb
    frag_epilogue<ACT_NONE, true, FM, FN, TM, TN, BN>(acc, p, rowoff, red, ctile, wm, wn, fr, fq, n0, false);
    return;
  }
#define DCG_EPI(A)                                                                                         \
  if (vec) frag_epilogue<A, true, FM, FN, TM, TN, BN>(acc, p, rowoff, red, ctile, wm, wn, fr, fq, n0, do_stats); \
  else frag_epilogue<A, false, FM, FN, TM, TN, BN>(acc, p, rowoff, red, ctile, wm, wn, fr, fq, n0, do_stats);
  switch (p.act) {
    case ACT_RELU: DCG_EPI(ACT_RELU) break;
    case ACT_LRELU: DCG_EPI(ACT_LRELU) break;
    case ACT_TANH: DCG_EPI(ACT_TANH) break;
    default: DCG_EPI(ACT_NONE) break;
  }
#undef DCG_EPI
}

// Pairwise tree over the RL row lanes of red2[RL][BN][2] (fixed order: deterministic; log2(RL)
// LDS rounds instead of an RL-long dependent chain of LDS reads). Result in red2[0][BN][2].
template <int RL, int BN, int NT = 256>
__device__ __forceinline__ void lane_tree(float* red2) {
#pragma unroll
  for (int h = RL / 2; h > 0; h >>= 1) {
    for (int q = threadIdx.x; q < h * BN * 2; q += NT) red2[q] += red2[q + h * BN * 2];
    __syncthreads();
  }
}

// Store pass of a data-gradient GEMM that feeds a BN + activation backward: 16-byte row stores
// of the C tile (LDS) and, in the same pass, 16-byte loads of the layer's x and y at the same
// offsets -> per-channel partial sums (sum g, sum g*xhat), g = dL/da * act'(y) -- the statistics
// the BN backward needs, without a separate pass over three tensors. Each thread owns one fixed
// 8-channel chunk; row lanes are reduced through LDS scratch (red2, 16 KiB) in a fixed order.
// Requires elem_t output with N % 8 == 0 (the caller checks) and a tile inside one BN group.
// NT threads per workgroup; red2 holds 64 * NT bytes. ALIAS: red2 overlaps ctile (a barrier
// separates the last ctile read from the first red2 write).
template <int BM, int BN, int NT = 256, bool ALIAS = false>
__device__ __forceinline__ void vec_store_bnb(const IGemmArgs& p, const int* rowoff, const elem_t* ctile,
                                              float* red2, int n0, int m0, float* dst) {
  constexpr int CPAD = BN + 8, CPR = BN / 8, RL = NT / CPR;
  static_assert(NT % CPR == 0, "chunks per row");
  const int tid = threadIdx.x, c = tid % CPR, rl = tid / CPR;
  const int N = p.N, n = n0 + 8 * c;
  const bool nok = n < N;
  const int g = m0 / p.bnb_rpg;
  const float slope = p.bnb_act == ACT_LRELU ? p.bnb_leak : 0.f;
  // Every x / y row this thread needs is loaded BEFORE the first store: interleaved with the C
  // stores, each row's loads waited a full memory round trip (the compiler cannot move a load of
  // bnb_x / bnb_y above a store to C, they may alias), IT of them back to back per thread.
  constexpr int IT = (BM + RL - 1) / RL;
  int offs[IT];
  elem8 yv_[IT], xv_[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int r = rl + it * RL;
    const int off = (r < BM && nok) ? rowoff[r] : -1;
    offs[it] = off;
    const size_t o = off >= 0 ? (size_t)off + p.cofs + n : 0;
    if (off >= 0) {
      yv_[it] = *reinterpret_cast<const elem8*>(p.bnb_y + o);
      if (!p.bnb_store_g) xv_[it] = *reinterpret_cast<const elem8*>(p.bnb_x + o);
    }
  }
  if (p.bnb_store_g) {  // activation backward only: store g, partial sums of the stored g
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = 0.f;
    elem_t* C = reinterpret_cast<elem_t*>(p.C);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int r = rl + it * RL;
      const int off = offs[it];
      if (off < 0) continue;
      const size_t o = (size_t)off + p.cofs + n;
      const elem8 dv = __builtin_bit_cast(elem8, *reinterpret_cast<const u32x4*>(ctile + r * CPAD + 8 * c));
      const elem8 yv = yv_[it];
      elem8 gv;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float yy = (float)yv[i];
        gv[i] = f2bf((float)dv[i] * (p.bnb_act == ACT_TANH ? 1.f - yy * yy : (yy > 0.f ? 1.f : slope)));
        s[i] += (float)gv[i];
      }
      *reinterpret_cast<u32x4*>(C + o) = __builtin_bit_cast(u32x4, gv);
    }
    if constexpr (ALIAS) __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) red2[(rl * BN + 8 * c + i) * 2 + 0] = s[i];
    __syncthreads();
    lane_tree<RL, BN, NT>(red2);
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(dst, (uint32_t)(2 * N * 4));
    for (int nl = tid; nl < BN; nl += NT) {  // write-through (sc1): a fused finalize may read it on another CU
      if (n0 + nl >= N) continue;
      st_sc1_f32(rd, (uint32_t)(n0 + nl) * 4u, red2[nl * 2 + 0]);
      st_sc1_f32(rd, (uint32_t)(N + n0 + nl) * 4u, 0.f);
    }
    return;
  }
  float mu[8], rs[8], s[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = nok ? p.bnb_mean[g * N + n + i] : 0.f;
    rs[i] = nok ? p.bnb_rstd[g * N + n + i] : 0.f;
    s[i] = 0.f;
    s2[i] = 0.f;
  }
  elem_t* C = reinterpret_cast<elem_t*>(p.C);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int r = rl + it * RL;
    const int off = offs[it];
    if (off < 0) continue;
    const size_t o = (size_t)off + p.cofs + n;
    const u32x4 v = *reinterpret_cast<const u32x4*>(ctile + r * CPAD + 8 * c);
    *reinterpret_cast<u32x4*>(C + o) = v;
    const elem8 dv = __builtin_bit_cast(elem8, v);
    const elem8 yv = yv_[it], xv = xv_[it];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float gv = (float)dv[i] * ((float)yv[i] > 0.f ? 1.f : slope);
      s[i] += gv;
      s2[i] += gv * ((float)xv[i] - mu[i]) * rs[i];
    }
  }
  if constexpr (ALIAS) __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red2[(rl * BN + 8 * c + i) * 2 + 0] = s[i];
    red2[(rl * BN + 8 * c + i) * 2 + 1] = s2[i];
  }
  __syncthreads();
  lane_tree<RL, BN, NT>(red2);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(dst, (uint32_t)(2 * N * 4));
  for (int nl = tid; nl < BN; nl += NT) {
    if (n0 + nl >= N) continue;
    st_sc1_f32(rd, (uint32_t)(n0 + nl) * 4u, red2[nl * 2 + 0]);
    st_sc1_f32(rd, (uint32_t)(N + n0 + nl) * 4u, red2[nl * 2 + 1]);
  }
}

}  // namespace dcg
