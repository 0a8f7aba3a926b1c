// dcg-variants: f32
// Reference-precision (fp32) convolution GEMMs for gfx950: the same implicit-GEMM semantics as
// igemm3.hip (mode 0 TF-SAME stride-2 conv, mode 1 conv_transpose as 4 sub-pixel phases, mode 2
// plain GEMM; either weight layout) and as wgrad.hip (25-tap gather / plain weight gradient into
// split-K fp32 slabs), on the fp32-input MFMA v_mfma_f32_16x16x4_f32 -- exact fp32 products
// accumulated in fp32, the reference's precision (distriubted_model.py:165-197 runs all of it in
// fp32). gfx950 has no xf32 / TF32 shortcut; the f32 MFMA runs at the fp32 vector rate, 1/16 of
// bf16 MFMA, so this path is about numerics, not speed.
//
// Tile core: LDS tiles are [rows][BK + 4] floats (BK = 16); lane l of a wave reads ONE float4
// per 16x16 fragment: row l & 15, k = 4 (l >> 4) .. +3, i.e. the k values that the four
// 16x16x4 MFMAs e = 0..3 take in their k slot l >> 4 (A[row][4g + e] pairs with B[4g + e][col]
// for lane group g): four MFMAs consume a whole 16-deep k-tile from one ds_read_b128 per
// operand fragment. Operands are staged global -> registers -> LDS (double buffered); operands
// that are k-major in memory (the BKN weight layout, both wgrad operands) are transposed on the
// LDS write, with chunk -> thread maps that keep those scalar writes bank-conflict free.
//
// The 16-bit-only kernels of the library (igemm v1, wgrad3, narrow_deconv) have no
// fp32 build: their fp32 entry points report "unsupported" and the engine takes the im2col /
// implicit-GEMM paths instead.
#include "kernels.h"

namespace dcg {

constexpr int F_BK = 16;        // k per LDS tile
constexpr int F_LDK = F_BK + 4; // LDS row stride in floats (16-byte aligned fragment reads)

template <int FM, int FN>
__device__ __forceinline__ void f32_tile_mma(const float* sa, const float* sb, int arow0, int brow0, int lane,
                                             f32x4 (&acc)[FM][FN]) {
  const int r = lane & 15, kq = (lane >> 4) * 4;
  f32x4 a[FM], b[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const f32x4*>(sa + (arow0 + i * 16 + r) * F_LDK + kq);
#pragma unroll
  for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const f32x4*>(sb + (brow0 + j * 16 + r) * F_LDK + kq);
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
}

__device__ __forceinline__ f32x4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4, buf_load16(r, off));
}

template <int ACT>
__device__ __forceinline__ float f_act(float v, float leak) {
  if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == ACT_LRELU) return fmaxf(v, leak * v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}

// + bias, BN partial statistics of the stored value, activation, scatter to the output pixels
template <int ACT, int FM, int FN, int TM, int TN, int BN, int WM>
__device__ __forceinline__ void f32_epilogue(const f32x4 (&acc)[FM][FN], const IGemmArgs& p, const int* rowoff,
                                             float* red, int wm, int wn, int lane, int n0) {
  const int fr = lane & 15, fq = lane >> 4;
  float* C = reinterpret_cast<float*>(p.C);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * TN + j * 16 + fr, n = n0 + nl;
    const bool nok = n < p.N;
    const float bv = (p.bias && nok) ? p.bias[n] : 0.f;
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int off = rowoff[wm * TM + i * 16 + fq * 4 + q];
        const bool valid = off >= 0 && nok;
        const float v = acc[i][j][q] + bv;
        s += valid ? v : 0.f;
        s2 += valid ? v * v : 0.f;
        if (valid) C[off + p.cofs + n] = f_act<ACT>(v, p.leak);
      }
    if (p.stats) {
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

template <int BM, int BN, int WM, int WN, int BKN>
__global__ __launch_bounds__(256) void igemm_f32_kernel(IGemmArgs p) {
  constexpr int BK = F_BK, LDK = F_LDK;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_CH = BM * BK / 4, B_CH = BN * BK / 4;  // float4 chunks per tile
  constexpr int A_PT = (A_CH + 255) / 256, B_PT = (B_CH + 255) / 256;
  constexpr int STAGE = (BM + BN) * LDK;
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1, "4 waves of 16x16 fragments");
  static_assert(BM + 2 * WM * BN <= 2 * STAGE, "epilogue scratch");
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntn = (p.N + BN - 1) / BN;
  const int total = p.mtiles * ntn * p.nphases;
  int t = blockIdx.x;
  {  // bijective XCD remap (as igemm3): one XCD gets a contiguous run of tiles
    const int q = total >> 3, rr = total & 7, xcd = t & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  const int phase = t % p.nphases;
  const int r_ = t / p.nphases;
  const int nt = r_ % ntn, mt = r_ / ntn;
  const IGemmPhaseK& ph = p.phk[phase];
  const int M = ph.M, m0 = mt * BM, n0 = nt * BN;
  if (m0 >= M) {  // shorter phase: its statistics slot must still be defined
    if (p.stats) {
      float* dst = p.stats + (size_t)(mt * p.nphases + phase) * 2 * p.N;
      for (int nl = tid; nl < BN; nl += 256)
        if (n0 + nl < p.N) { dst[n0 + nl] = 0.f; dst[p.N + n0 + nl] = 0.f; }
    }
    return;
  }
  const int Kc = p.Kc, N = p.N;
  const int ntaps = p.plain ? 1 : ph.ntaps;
  const int kt_per_tap = (Kc + BK - 1) / BK;
  const int nk = ntaps * kt_per_tap;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.Bw, p.b_bytes);

  // A chunk q: row q >> 2, k offset 4 (q & 3) (k contiguous in memory and in LDS)
  int a_base[A_PT], a_iy[A_PT], a_ix[A_PT];
  bool a_ok[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int q = tid + 256 * i, m = m0 + (q >> 2);
    a_ok[i] = q < A_CH && m < M;
    a_base[i] = 0; a_iy[i] = 0; a_ix[i] = 0;
    if (!a_ok[i]) continue;
    if (p.plain) {
      a_base[i] = m * Kc;
    } else {
      const uint32_t b = fdiv((uint32_t)m, ph.fd_hw);
      const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph.Hq * ph.Wq);
      const uint32_t qy = fdiv(rem, ph.fd_w);
      const uint32_t qx = rem - qy * (uint32_t)ph.Wq;
      a_iy[i] = (int)qy * p.sstride + ph.iy0_off;
      a_ix[i] = (int)qx * p.sstride + ph.ix0_off;
      a_base[i] = (((int)b * p.H + a_iy[i]) * p.W + a_ix[i]) * Kc;
    }
  }
  f32x4 ra_reg[A_PT], rb_reg[B_PT];

  auto load = [&](int kt) {
    const int ti = kt / kt_per_tap, c0 = (kt - ti * kt_per_tap) * BK;
    int dy = 0, dx = 0, wt = 0;
    if (!p.plain) {
      const int tp = ph.tap[ti];
      dy = (int)(signed char)(tp & 0xff);
      dx = (int)(signed char)((tp >> 8) & 0xff);
      wt = tp >> 16;
    }
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int q = tid + 256 * i, cc = c0 + 4 * (q & 3);
      uint32_t off = OOB;
      if (a_ok[i] && cc < Kc) {
        if (p.plain) {
          off = (uint32_t)(a_base[i] + cc) * 4u;
        } else {
          const int iy = a_iy[i] + dy, ix = a_ix[i] + dx;
          if ((unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W)
            off = (uint32_t)(a_base[i] + (dy * p.W + dx) * Kc + cc) * 4u;
        }
      }
      ra_reg[i] = ld4(ra, off);
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int q = tid + 256 * i;
      uint32_t off = OOB;
      if (q < B_CH) {
        if constexpr (BKN) {  // Bw[tap][Kc][N]: chunk = 4 n of one k row; k varies fastest over q
          const int k = c0 + (q % BK), n = n0 + 4 * (q / BK);
          if (k < Kc && k < p.kb_valid && n < N) off = (uint32_t)((wt * Kc + k) * N + n) * 4u;
        } else {              // Bw[tap][N][Kc]: chunk = 4 k of one n row
          const int n = n0 + (q >> 2), c = c0 + 4 * (q & 3);
          if (n < N && c < Kc && c < p.kb_valid) off = (uint32_t)((wt * N + n) * Kc + c) * 4u;
        }
      }
      rb_reg[i] = ld4(rb, off);
    }
  };
  auto store = [&](int buf) {
    float* sa = lds + buf * STAGE;
    float* sb = sa + BM * LDK;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int q = tid + 256 * i;
      if (q < A_CH) *reinterpret_cast<f32x4*>(sa + (q >> 2) * LDK + 4 * (q & 3)) = ra_reg[i];
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int q = tid + 256 * i;
      if (q >= B_CH) continue;
      if constexpr (BKN) {
        const int k = q % BK, nl = 4 * (q / BK);
#pragma unroll
        for (int e = 0; e < 4; ++e) sb[(nl + e) * LDK + k] = rb_reg[i][e];
      } else {
        *reinterpret_cast<f32x4*>(sb + (q >> 2) * LDK + 4 * (q & 3)) = rb_reg[i];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
    f32_tile_mma<FM, FN>(lds + buf * STAGE, lds + buf * STAGE + BM * LDK, wm * TM, wn * TN, lane, acc);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: per-row output offsets (pixel scatter of conv / deconv phases)
  int* rowoff = reinterpret_cast<int*>(lds);
  float* red = lds + BM;
  for (int r = tid; r < BM; r += 256) {
    const int m = m0 + r;
    int off = -1;
    if (m < M) {
      if (p.plain) {
        off = m * p.ldc;
      } else {
        const uint32_t b = fdiv((uint32_t)m, ph.fd_hw);
        const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph.Hq * ph.Wq);
        const uint32_t qy = fdiv(rem, ph.fd_w);
        const uint32_t qx = rem - qy * (uint32_t)ph.Wq;
        const int y = (int)qy * p.ostride + ph.oy_off, x = (int)qx * p.ostride + ph.ox_off;
        off = (((int)b * p.outH + y) * p.outW + x) * p.ldc;
      }
    }
    rowoff[r] = off;
  }
  __syncthreads();
  switch (p.act) {
    case ACT_RELU: f32_epilogue<ACT_RELU, FM, FN, TM, TN, BN, WM>(acc, p, rowoff, red, wm, wn, lane, n0); break;
    case ACT_LRELU: f32_epilogue<ACT_LRELU, FM, FN, TM, TN, BN, WM>(acc, p, rowoff, red, wm, wn, lane, n0); break;
    case ACT_TANH: f32_epilogue<ACT_TANH, FM, FN, TM, TN, BN, WM>(acc, p, rowoff, red, wm, wn, lane, n0); break;
    default: f32_epilogue<ACT_NONE, FM, FN, TM, TN, BN, WM>(acc, p, rowoff, red, wm, wn, lane, n0); break;
  }
  if (p.stats) {
    __syncthreads();
    float* dst = p.stats + (size_t)(mt * p.nphases + phase) * 2 * N;
    for (int nl = tid; nl < BN; nl += 256) {
      if (n0 + nl >= N) continue;
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s += red[(w * BN + nl) * 2 + 0];
        s2 += red[(w * BN + nl) * 2 + 1];
      }
      dst[n0 + nl] = s;
      dst[N + n0 + nl] = s2;
    }
  }
}

// ---------------------------------------------------------------- weight gradient (fp32)
// out[split][tap][m][n] = sum over the split's pixels k of G(k, tap)[m] * Dm[k][n] (see wgrad.hip).
// Both operands are channel-contiguous per pixel (k-major): chunk q = 4 channels of pixel row
// q % 16 (pixel fastest over the threads), transposed into the [channel][k] LDS tiles.
template <int BM, int BN>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(WGradArgs p) {
  constexpr int BK = F_BK, LDK = F_LDK, WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_CH = BM * BK / 4, B_CH = BN * BK / 4;
  constexpr int A_PT = (A_CH + 255) / 256, B_PT = (B_CH + 255) / 256;
  constexpr int STAGE = (BM + BN) * LDK;
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = (p.Mc + BM - 1) / BM;
  const int mt = blockIdx.x % ntm, nt = blockIdx.x / ntm;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tap = blockIdx.y, split = blockIdx.z;
  const int ky = tap / 5, kx = tap - 5 * (tap / 5);
  const int kb = split * p.kt_per_split * 64;  // split ranges are 64-pixel granular (host)
  const int ke = min(p.K, kb + p.kt_per_split * 64);
  const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.G, p.g_bytes);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(p.Dm, p.d_bytes);
  f32x4 ga[A_PT], db[B_PT];

  auto load = [&](int kt) {
    const int k0 = kb + kt * BK;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int q = tid + 256 * i;
      const int k = k0 + (q % BK), m = m0 + 4 * (q / BK);
      uint32_t off = OOB;
      if (q < A_CH && k < ke && m < p.Mc) {
        if (p.plain) {
          off = (uint32_t)(k * p.Mc + m) * 4u;
        } else {
          const uint32_t b = fdiv((uint32_t)k, p.fd_hw);
          const uint32_t rem = (uint32_t)k - b * (uint32_t)(p.Hd * p.Wd);
          const uint32_t y = fdiv(rem, p.fd_w);
          const uint32_t x = rem - y * (uint32_t)p.Wd;
          const int iy = 2 * (int)y + ky - p.pl, ix = 2 * (int)x + kx - p.pl;
          if ((unsigned)iy < (unsigned)p.Hg && (unsigned)ix < (unsigned)p.Wg)
            off = (uint32_t)((((int)b * p.Hg + iy) * p.Wg + ix) * p.Mc + m) * 4u;
        }
      }
      ga[i] = ld4(rg, off);
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int q = tid + 256 * i;
      const int k = k0 + (q % BK), n = n0 + 4 * (q / BK);
      uint32_t off = OOB;
      if (q < B_CH && k < ke && n < p.Nc) off = (uint32_t)(k * p.Nc + n) * 4u;
      db[i] = ld4(rd, off);
    }
  };
  auto store = [&](int buf) {
    float* sa = lds + buf * STAGE;
    float* sb = sa + BM * LDK;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int q = tid + 256 * i;
      if (q >= A_CH) continue;
      const int k = q % BK, ml = 4 * (q / BK);
#pragma unroll
      for (int e = 0; e < 4; ++e) sa[(ml + e) * LDK + k] = ga[i][e];
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int q = tid + 256 * i;
      if (q >= B_CH) continue;
      const int k = q % BK, nl = 4 * (q / BK);
#pragma unroll
      for (int e = 0; e < 4; ++e) sb[(nl + e) * LDK + k] = db[i][e];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
    f32_tile_mma<FM, FN>(lds + buf * STAGE, lds + buf * STAGE + BM * LDK, wm * TM, wn * TN, lane, acc);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  float* out = p.out + ((size_t)split * p.ntaps + tap) * (size_t)p.Mc * p.Nc;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + wm * TM + i * 16 + fq * 4 + q;
        if (m < p.Mc && n < p.Nc) out[(size_t)m * p.Nc + n] = acc[i][j][q];
      }
    }
}

}  // namespace dcg

// ---------------------------------------------------------------------------- host launch
// fp32 tiles behind the igemm3 cfg numbering: 200 64x64, 201 128x64, 202 64x16, 203 128x128
#define DCG_IGEMM_F32_TILES(X) X(0, 64, 64, 2, 2) X(1, 128, 64, 2, 2) X(2, 64, 16, 4, 1) X(3, 128, 128, 2, 2)

extern "C" int DCG_API(dcg_igemm3_tile)(int cfg, int* bm, int* bn, int* ns) {
  if (cfg < 200 || cfg >= 210) return -1;
  const int id = cfg - 200;
  *ns = 2;
#define X(id_, BM_, BN_, WM_, WN_) if (id == id_) { *bm = BM_; *bn = BN_; return 0; }
  DCG_IGEMM_F32_TILES(X)
#undef X
  return -1;
}

extern "C" int DCG_API(dcg_igemm3_launch)(const dcg::IGemmArgs* a, int cfg, int bkn, unsigned blocks, hipStream_t s) {
  if (a->splits != 1 || a->bnb_x) return -2;  // fp32 build: no split-K, no fused BN-backward statistics
  const int id = cfg - 200;
#define X(id_, BM_, BN_, WM_, WN_)                                                                             \
  if (id == id_) {                                                                                             \
    if (bkn) hipLaunchKernelGGL((dcg::igemm_f32_kernel<BM_, BN_, WM_, WN_, 1>), dim3(blocks), dim3(256), 0, s, *a); \
    else hipLaunchKernelGGL((dcg::igemm_f32_kernel<BM_, BN_, WM_, WN_, 0>), dim3(blocks), dim3(256), 0, s, *a);     \
    return (int)hipGetLastError();                                                                             \
  }
  DCG_IGEMM_F32_TILES(X)
#undef X
  return -1;
}

extern "C" int DCG_API(dcg_wgrad_tile)(int cfg, int* bm, int* bn) {
  if (cfg < 0 || cfg > 6) return -1;
  *bm = 64;  // one fp32 tile for every wgrad cfg
  *bn = 64;
  return 0;
}

extern "C" int DCG_API(dcg_wgrad_launch)(const dcg::WGradArgs* a, int cfg, int splits, hipStream_t s) {
  if (cfg < 0 || cfg > 6 || a->Mc % 4 || a->Nc % 4) return -2;
  const int ntm = (a->Mc + 63) / 64, ntn = (a->Nc + 63) / 64;
  hipLaunchKernelGGL((dcg::wgrad_f32_kernel<64, 64>), dim3(ntm * ntn, a->ntaps, splits), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

// 16-bit-only kernels: no fp32 build (the engine does not select them for fp32)
extern "C" int DCG_API(dcg_igemm_tile)(int, int*, int*) { return -1; }
extern "C" int DCG_API(dcg_igemm_launch)(const dcg::IGemmArgs*, int, int, int, hipStream_t) { return -2; }
extern "C" int DCG_API(dcg_igemm3_threads)(int) { return 256; }
extern "C" int DCG_API(dcg_wgrad3_tile)(int, int*, int*, int*) { return -1; }
extern "C" int DCG_API(dcg_wgrad3_launch)(const dcg::WGrad3Args*, int, hipStream_t) { return -2; }
extern "C" int DCG_API(dcg_narrow_deconv)(const elem_t*, const elem_t*, const float*, elem_t*, int, int, int, int, int,
                                          int, int, int, int, float, hipStream_t) {
  return -2;
}
