// dcg-variants: bf16 f16
// Weight-gradient ("wgrad") for the TF-'SAME' stride-2 5x5 conv and
// conv_transpose on CDNA4 MFMA, NHWC, elem_t in / fp32 out.
//
// Both cases have the same form (G = the operand read at stride-2 shifted pixels, Dm = the
// operand read at its own pixels, k = pixels of Dm):
//   out[tap][m][n] = sum_k G[b, 2y+ky-pl, 2x+kx-pl, m] * Dm[b, y, x, n]
//   conv  (D layers): G = layer input X,  Dm = dL/d(conv out)  -> dW [kh,kw,ci,co] (HWIO)
//   deconv(G layers): G = dL/d(deconv out), Dm = layer input X  -> dW [kh,kw,co,ci]
// so the result lands directly in the TF variable layout (no transposes).
// "plain" mode (1 tap, G already a [K][Mc] matrix) serves the im2col'd 3-channel layers.
//
// GEMM view per tap: M = G channels, N = Dm channels, K = B*Hd*Wd (up to 262,144) -> split-K
// over blockIdx.z into fp32 slabs, summed by a deterministic reduce kernel (no float atomics).
// Both operands are k-major in memory (channels contiguous), so tiles are staged k-major in
// LDS and the MFMA fragments (which need 8 consecutive k per lane) are read with the gfx950
// transposing LDS read ds_read_b64_tr_b16 (2 per fragment). LDS rows use an 8-byte-chunk XOR
// swizzle chosen so each 32-lane half of a transposed read hits 32 distinct bank slots.
#include "kernels.h"

namespace dcg {

// XOR (in 8-byte chunks) applied to LDS row r of a k-major tile with row stride S bytes
template <int S>
__device__ __forceinline__ int wg_swz(int r) {
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void wgrad_kernel(WGradArgs p) {
  constexpr int BK = 64, WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int GC = BM / 8, DC = BN / 8;          // 16-byte chunks per k-row
  constexpr int G_PT = (BK * GC + 255) / 256, D_PT = (BK * DC + 255) / 256;
  constexpr int SG = BM * 2, SD = BN * 2;          // LDS row strides (bytes)
  constexpr int STAGE = BK * (SG + SD);            // bytes per stage
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = (p.Mc + BM - 1) / BM;
  const int mt = blockIdx.x % ntm, nt = blockIdx.x / ntm;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tap = blockIdx.y, split = blockIdx.z;
  const int ky = tap / 5, kx = tap - 5 * (tap / 5);
  const int KT_total = (p.K + BK - 1) / BK;
  const int kt0 = split * p.kt_per_split;
  const int kt1 = min(KT_total, kt0 + p.kt_per_split);

  const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.G, p.g_bytes);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(p.Dm, p.d_bytes);

  u32x4 rg_reg[G_PT], rd_reg[D_PT];

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < G_PT; ++i) {
      const int q = tid + 256 * i;
      const int r = q / GC, c = q - r * GC;
      const int k = k0 + r;
      const int m = m0 + c * 8;
      uint32_t off = OOB;
      if (r < BK && k < p.K && m < p.Mc) {
        if (p.plain) {
          off = (uint32_t)(k * p.Mc + m) * 2u;
        } else {
          const uint32_t b = fdiv((uint32_t)k, p.fd_hw);
          const uint32_t rem = (uint32_t)k - b * (uint32_t)(p.Hd * p.Wd);
          const uint32_t y = fdiv(rem, p.fd_w);
          const uint32_t x = rem - y * (uint32_t)p.Wd;
          const int iy = 2 * (int)y + ky - p.pl, ix = 2 * (int)x + kx - p.pl;
          if ((unsigned)iy < (unsigned)p.Hg && (unsigned)ix < (unsigned)p.Wg)
            off = (uint32_t)((((int)b * p.Hg + iy) * p.Wg + ix) * p.Mc + m) * 2u;
        }
      }
      rg_reg[i] = buf_load16(rg, off);
    }
#pragma unroll
    for (int i = 0; i < D_PT; ++i) {
      const int q = tid + 256 * i;
      const int r = q / DC, c = q - r * DC;
      const int k = k0 + r;
      const int n = n0 + c * 8;
      uint32_t off = OOB;
      if (r < BK && k < p.K && n < p.Nc) off = (uint32_t)(k * p.Nc + n) * 2u;
      rd_reg[i] = buf_load16(rd, off);
    }
  };

  auto store_tile = [&](int buf) {
    char* sg = lds + buf * STAGE;
    char* sd = sg + BK * SG;
#pragma unroll
    for (int i = 0; i < G_PT; ++i) {
      const int q = tid + 256 * i;
      const int r = q / GC, c = q - r * GC;
      if ((BK * GC) % 256 == 0 || r < BK)
        *reinterpret_cast<u32x4*>(sg + r * SG + (((2 * c) ^ wg_swz<SG>(r)) * 8)) = rg_reg[i];
    }
#pragma unroll
    for (int i = 0; i < D_PT; ++i) {
      const int q = tid + 256 * i;
      const int r = q / DC, c = q - r * DC;
      if ((BK * DC) % 256 == 0 || r < BK)
        *reinterpret_cast<u32x4*>(sd + r * SD + (((2 * c) ^ wg_swz<SD>(r)) * 8)) = rd_reg[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;

  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    if (kt + 1 < kt1) load_tile(kt + 1);
    const char* sg = lds + buf * STAGE;
    const char* sd = sg + BK * SG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      elem8 af[FM], bfr[FN];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = ks * 32 + 8 * g4 + 4 * h + q4;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int c8 = (wm * TM + i * 16) / 4 + p4;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, sg + r * SG + ((c8 ^ wg_swz<SG>(r)) * 8)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][4 * h + e] = vb[e];
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c8 = (wn * TN + j * 16) / 4 + p4;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, sd + r * SD + ((c8 ^ wg_swz<SD>(r)) * 8)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[j][4 * h + e] = vb[e];
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = DCG_MFMA_16x16x32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < kt1) store_tile(buf ^ 1);
    __syncthreads();
  }

  float* out = p.out + ((size_t)split * p.ntaps + tap) * (size_t)p.Mc * p.Nc;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + g4 * 4 + r;
        if (m < p.Mc && n < p.Nc) out[(size_t)m * p.Nc + n] = acc[i][j][r];
      }
    }
}

}  // namespace dcg

#define DCG_WGRAD_CONFIGS(X) \
  X(0, 128, 128) X(1, 64, 128) X(2, 128, 64) X(3, 64, 64) X(4, 32, 64) X(5, 64, 32) X(6, 32, 32)

extern "C" int DCG_API(dcg_wgrad_tile)(int cfg, int* bm, int* bn) {
#define X(id, BM_, BN_) if (cfg == id) { *bm = BM_; *bn = BN_; return 0; }
  DCG_WGRAD_CONFIGS(X)
#undef X
  return -1;
}

extern "C" int DCG_API(dcg_wgrad_launch)(const dcg::WGradArgs* a, int cfg, int splits, hipStream_t s) {
  int bm = 0, bn = 0;
  if (DCG_API(dcg_wgrad_tile)(cfg, &bm, &bn)) return -1;
  const int ntm = (a->Mc + bm - 1) / bm, ntn = (a->Nc + bn - 1) / bn;
  dim3 grid(ntm * ntn, a->ntaps, splits);
#define X(id, BM_, BN_) \
  if (cfg == id) { hipLaunchKernelGGL((dcg::wgrad_kernel<BM_, BN_>), grid, dim3(256), 0, s, *a); \
                   return (int)hipGetLastError(); }
  DCG_WGRAD_CONFIGS(X)
#undef X
  return -1;
}

