// dcg-variants: bf16 f16 f32
// The 3-channel image layers of the step without column matrices (round 2):
//
//   nconv  : TF-SAME stride-2 5x5 conv, 1..4 input -> 64 output channels. D layer 0's forward
//            (+ bias + LeakyReLU) and the data gradient of G's RGB deconv (the adjoint of a
//            stride-2 deconv is this conv; optional fused BN-backward statistics of the BN layer
//            below, as igemm's bnb epilogue). Replaces conv3.hip (forward) and im2col + a plain
//            GEMM (G chain).
//   nwgrad : the weight gradient of those two layers, dW[tap][c][n] = sum over output pixels of
//            X[2y+ky-pl, 2x+kx-pl, c] * D[y, x, n] (X = the 3-channel image / image gradient,
//            D = the 64-channel side). Replaces im2col + wgrad.hip slabs; the per-workgroup
//            partials are summed by splitk_reduce in workgroup order (deterministic).
//
// Why new kernels: the round-1 forms of these layers were latency-bound launches at 2-5x their
// memory floor (profiles/r2/step_profile_r2_1.21ms.txt: conv3 35 us, G-chain RGB backward 70 us
// for ~25 MB of traffic) -- 2-byte global loads, per-workgroup weight re-staging, column matrices
// written and re-read.
//
// nconv: persistent workgroups; the 64x(4 tap x 4 ch) weight matrix is staged ONCE per workgroup
// and held as MFMA A fragments (W^T: 16 x elem8 in VGPRs). Tile = 4 output rows x 32 columns of
// one image; wave w owns output row w (two 16-pixel blocks). The 11 x 67 input window is held in
// LDS as 4-channel (8 B) pixels; the next tile's window is loaded into registers while the current
// one is computed. Swapped operands (C^T = W^T X^T): each lane ends with 4 consecutive channels of
// one pixel; the 4x32-pixel C tile goes through LDS so the store pass writes whole 16-byte chunks
// of contiguous 4 KiB rows, with the BN-backward operands (x, y) of its pixels loaded before any
// store (round 6: the fused-statistics variant went from 39.7 to 27.9 us, the forward from 19.0
// to 16.9 us; round 5's 8-byte stores interleaved with dependent loads waited a memory round
// trip per 16 pixels).
//
// nwgrad: one workgroup = a band of output rows of one image, processed in chunks of <= 256
// pixels; both MFMA operands are "k = pixel" fragments read with the gfx950 transposing read
// ds_read_b64_tr_b16: the D tile (rows = pixels, 64 channels, XOR-swizzled 128 B rows) and the
// image window, where lane 4q+p's address is the 4-channel pixel of tap 4*mb + p at its pixel --
// the im2col row never exists (k' = 4 tap + c, taps >= 25 read a zero pixel).
#include "kernels.h"

#if defined(DCG_F32)
// the fp32 (reference-precision) engine runs these layers on igemm_f32.hip: stubs only
extern "C" int DCG_API(dcg_nconv)(const elem_t*, const elem_t*, const float*, elem_t*, int, int, int, int, int, int,
                                  int, int, int, float, int, const elem_t*, const elem_t*, const float*, const float*,
                                  int, float, float*, hipStream_t) { return -2; }
extern "C" int DCG_API(dcg_nconv_tiles)(int, int, int) { return -1; }
extern "C" int DCG_API(dcg_nwgrad_plan)(int, int, int, int, int*, int*, int*) { return -1; }
extern "C" int DCG_API(dcg_nwgrad)(const elem_t*, int, int, int, int, const elem_t*, int, int, int, int, float*,
                                   hipStream_t) { return -2; }
extern "C" int DCG_API(dcg_narrow_deconv_dact)(const elem_t*, const elem_t*, elem_t*, const elem_t*, int, int, int, int,
                                               int, int, int, int, int, float, float*, hipStream_t) { return -2; }
extern "C" int DCG_API(dcg_narrow_deconv_tiles)(int, int, int) { return -1; }
extern "C" int DCG_API(dcg_wgrad3_taps_per_tile)(int) { return 1; }
extern "C" int DCG_API(dcg_narrow_deconv_bnin)(const elem_t*, const elem_t*, const float*, elem_t*, int, int, int, int,
                                               int, int, int, int, int, float, const float*, const float*, int, float,
                                               elem_t*, hipStream_t) { return -2; }
#else

namespace dcg {

// ------------------------------------------------------------------------------------ nconv
constexpr int NC_TY = 4;                    // output rows per tile (= waves)
constexpr int NC_TX = 32;                   // output columns per tile
constexpr int NC_WR = 2 * NC_TY + 3;        // 11 window rows
constexpr int NC_WC = 2 * NC_TX + 3;        // 67 window columns
constexpr int NC_WP = NC_WC + 1;            // window pixel pitch per row
constexpr int NC_WPIX = NC_WR * NC_WC;      // 737 staged pixels
constexpr int NC_PPT = (NC_WPIX + 255) / 256;
constexpr int NC_KS = 136;                  // transposed-weight row stride (elements; 272 B = 17 x 16 B)
constexpr int NC_CS = 72;                   // C-tile pixel stride (elements; 144 B = 9 x 16 B)
constexpr int NC_SP = NC_TY * NC_TX * 8 / 256;  // 16-byte chunks per thread in the store pass

struct NConvArgs {
  const elem_t* x; const elem_t* w; const float* bias; elem_t* y;
  int H, W, Ho, Wo, pad_y, pad_x, act; float leak;
  int tiles_x, tiles_per_img, ntiles;
  // fused BN-backward statistics (data gradient feeding a BN + activation layer)
  const elem_t* bx; const elem_t* by; const float* mean; const float* rstd; int bact; float bleak;
  float* part;  // [gridDim.x][2][64]
};

template <int ACT>
__device__ __forceinline__ float nc_act(float v, float leak) {
  if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == ACT_LRELU) return fmaxf(v, leak * v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}

template <int CIN, bool BNB, int ACT>
__global__ __launch_bounds__(256) void nconv_kernel(NConvArgs p) {
  __shared__ __attribute__((aligned(16))) elem_t wt[64 * NC_KS];
  __shared__ __attribute__((aligned(16))) elem_t xs[NC_WR * NC_WP * 4];
  __shared__ float red[4][2][64];
  __shared__ __attribute__((aligned(16))) elem_t ct[NC_TY * NC_TX * NC_CS];  // C tile (store pass)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  int t = blockIdx.x;
  if (t >= p.ntiles) return;  // the host sizes the grid to <= ntiles (every partial row written)

  // ---- weights, once: wt[n][k = 4 tap + c] (taps 25..31 and c >= CIN zero) -> A fragments W^T
  for (int q = tid; q < 64 * NC_KS / 8; q += 256) reinterpret_cast<u32x4*>(wt)[q] = (u32x4){0u, 0u, 0u, 0u};
  __syncthreads();
  for (int q = tid; q < 25 * CIN * 64; q += 256) {
    const int n = q & 63, kk = q >> 6, tap = kk / CIN, c = kk - tap * CIN;
    wt[n * NC_KS + 4 * tap + c] = p.w[q];
  }
  __syncthreads();
  elem8 wf[4][4];  // [nb][kb]: lane holds W^T[n = 16 nb + li][k = 32 kb + 8 g + j]
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
      wf[nb][kb] = *reinterpret_cast<const elem8*>(wt + (16 * nb + li) * NC_KS + 32 * kb + 8 * g);
  float bias_r[4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias_r[nb][e] = p.bias ? p.bias[16 * nb + 4 * g + e] : 0.f;
  // store pass: this thread's fixed 8-channel chunk
  const int c8 = tid & 7;
  float mu[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = BNB ? p.mean[8 * c8 + e] : 0.f;
    rs[e] = BNB ? p.rstd[8 * c8 + e] : 0.f;
    s1[e] = 0.f;
    s2[e] = 0.f;
  }
  const float bslope = p.bact == ACT_LRELU ? p.bleak : 0.f;

  // ---- window staging: registers (next tile) -> LDS
  elem_t pv[NC_PPT][CIN];
  auto fetch = [&](int tt) {
    const int b = tt / p.tiles_per_img, rem = tt - b * p.tiles_per_img;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    const int iy0 = 2 * ty * NC_TY - p.pad_y, ix0 = 2 * tx * NC_TX - p.pad_x;
#pragma unroll
    for (int i = 0; i < NC_PPT; ++i) {
      const int q = tid + 256 * i;
      const int r = q / NC_WC, c = q - r * NC_WC;
      const int iy = iy0 + r, ix = ix0 + c;
      const bool ok = q < NC_WPIX && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const elem_t* src = p.x + (((size_t)b * p.H + (ok ? iy : 0)) * p.W + (ok ? ix : 0)) * CIN;
#pragma unroll
      for (int cc = 0; cc < CIN; ++cc) pv[i][cc] = ok ? src[cc] : (elem_t)0.f;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < NC_PPT; ++i) {
      const int q = tid + 256 * i;
      if (q < NC_WPIX) {
        const int r = q / NC_WC, c = q - r * NC_WC;
        elem4 v = {(elem_t)0.f, (elem_t)0.f, (elem_t)0.f, (elem_t)0.f};
#pragma unroll
        for (int cc = 0; cc < CIN; ++cc) v[cc] = pv[i][cc];
        *reinterpret_cast<elem4*>(xs + (r * NC_WP + c) * 4) = v;
      }
    }
  };
  fetch(t);
  commit();
  __syncthreads();
  for (; t < p.ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    const int b = t / p.tiles_per_img, rem = t - b * p.tiles_per_img;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    f32x4 acc[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[h][nb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      // this lane's two taps of the k-block (taps >= 25 carry zero weights: clamp the address)
      const int t0 = min(8 * kb + 2 * g, 24), t1 = min(8 * kb + 2 * g + 1, 24);
      const int off0 = (t0 / 5) * NC_WP + (t0 % 5), off1 = (t1 / 5) * NC_WP + (t1 % 5);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int base = 2 * wave * NC_WP + 2 * (16 * h + li);  // window pixel of tap (0, 0)
        const elem4 a0 = *reinterpret_cast<const elem4*>(xs + (base + off0) * 4);
        const elem4 a1 = *reinterpret_cast<const elem4*>(xs + (base + off1) * 4);
        const elem8 xf = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[h][nb] = DCG_MFMA_16x16x32(wf[nb][kb], xf, acc[h][nb], 0, 0, 0);
      }
    }
    // next window in flight under this tile's store pass (issued after the MFMAs: issued before
    // them, the compiler's register reuse drained it at the first LDS read)
    if (tn < p.ntiles) fetch(tn);
    // ---- C tile -> LDS: lane = pixel 16 h + li of output row `wave`, channels 16 nb + 4 g + e
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int px = wave * NC_TX + 16 * h + li;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        elem4 ov;
#pragma unroll
        for (int e = 0; e < 4; ++e) ov[e] = f2bf(nc_act<ACT>(acc[h][nb][e] + bias_r[nb][e], p.leak));
        *reinterpret_cast<elem4*>(ct + px * NC_CS + 16 * nb + 4 * g) = ov;
      }
    }
    __syncthreads();  // the C tile is complete; every wave is done with this window
    // ---- store pass: thread = one 8-channel chunk (c8) of 4 pixels, 16-byte coalesced rows
    //      (a tile row is 32 contiguous pixels = 4 KiB); BN operands loaded before the stores
    size_t o[NC_SP];
    bool ok[NC_SP];
#pragma unroll
    for (int i = 0; i < NC_SP; ++i) {
      const int px = (tid >> 3) + 32 * i;  // pixel of the tile: row px / 32, column px % 32
      const int oy = ty * NC_TY + (px >> 5), ox = tx * NC_TX + (px & 31);
      ok[i] = oy < p.Ho && ox < p.Wo;
      o[i] = ok[i] ? (((size_t)b * p.Ho + oy) * p.Wo + ox) * 64 + 8 * c8 : 0;
    }
    elem8 bxv[NC_SP], byv[NC_SP];
    if constexpr (BNB) {
#pragma unroll
      for (int i = 0; i < NC_SP; ++i) {
        bxv[i] = *reinterpret_cast<const elem8*>(p.bx + o[i]);
        byv[i] = *reinterpret_cast<const elem8*>(p.by + o[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < NC_SP; ++i) {
      const int px = (tid >> 3) + 32 * i;
      const u32x4 v = *reinterpret_cast<const u32x4*>(ct + px * NC_CS + 8 * c8);
      if (ok[i]) {
        *reinterpret_cast<u32x4*>(p.y + o[i]) = v;
        if constexpr (BNB) {  // statistics of exactly the stored (rounded) gradient
          const elem8 dv = __builtin_bit_cast(elem8, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gv = (float)dv[e] * ((float)byv[i][e] > 0.f ? 1.f : bslope);
            s1[e] += gv;
            s2[e] += gv * ((float)bxv[i][e] - mu[e]) * rs[e];
          }
        }
      }
    }
    if (tn < p.ntiles) {
      commit();         // (every wave finished its window reads before the barrier above)
      __syncthreads();  // the window is staged; every wave is done with this C tile
    }
  }
  if constexpr (BNB) {
    // fixed-order reduction: the 8 lanes of a wave with the same chunk (xor 8, 16, 32), then
    // the 4 waves in order
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float a = s1[e], c = s2[e];
#pragma unroll
      for (int sh = 8; sh < 64; sh <<= 1) {
        a += __shfl_xor(a, sh, 64);
        c += __shfl_xor(c, sh, 64);
      }
      if (lane < 8) {
        red[wave][0][8 * c8 + e] = a;
        red[wave][1][8 * c8 + e] = c;
      }
    }
    __syncthreads();
    if (tid < 128) {
      const int st = tid >> 6, n = tid & 63;
      p.part[(size_t)blockIdx.x * 128 + tid] = ((red[0][st][n] + red[1][st][n]) + red[2][st][n]) + red[3][st][n];
    }
  }
}

// ------------------------------------------------------------------------------------ nwgrad
constexpr int NWG_PX = 256;         // pixels per chunk (D tile rows)
// max staged window pixels (+1 zero pixel after them): 2 rows of a 128-wide D side (the 256x256
// ladder's RGB layers) stage 7 x 259 = 1813 window pixels
constexpr int NWG_WIN = 2048;
constexpr int NWG_WPT = NWG_WIN / 256;

struct NWGradArgs {
  const elem_t* x; int H, W;          // image side [B][H][W][CIN]
  const elem_t* d; int Hd, Wd;        // 64-channel side [B][Hd][Wd][64]
  int pl;                             // top / left padding of the stride-2 window
  int tyc, np, nks;                   // rows per chunk, pixels per chunk (tyc * Wd), k-steps of 32
  int wrows, wcols;                   // window rows / columns of a chunk
  int chunks_per_wg, wg_per_img;
  float* part;                        // [gridDim.x][25][CIN][64]
};

__device__ __forceinline__ int nwg_swz(int r) {  // 8-byte-chunk XOR of 128-byte D-tile row r
  return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
}

template <int CIN>
__global__ __launch_bounds__(256) void nwgrad_kernel(NWGradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* dt = smem;                          // [NWG_PX][128 B] D tile, swizzled
  char* win = smem + NWG_PX * 128;          // [wrows * wcols + 1][8 B] window (+ zero pixel)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const int b = blockIdx.x / p.wg_per_img;
  const int yb = (blockIdx.x - b * p.wg_per_img) * p.chunks_per_wg * p.tyc;
  const int zero_pix = p.wrows * p.wcols;
  if (tid == 0) *reinterpret_cast<elem4*>(win + zero_pix * 8) = (elem4){(elem_t)0.f, (elem_t)0.f, (elem_t)0.f, (elem_t)0.f};

  // per-lane A addresses (chunk-invariant): pixel part and tap part
  // pixel of k-step ks, half h: px = 32 ks + 8 g + 4 h + q (clamped into the chunk)
  int pxoff[8][2];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int px = min(32 * ks + 8 * g + 4 * h + q, p.np - 1);
      const int yy = px / p.Wd, xx = px - yy * p.Wd;
      pxoff[ks][h] = 2 * yy * p.wcols + 2 * xx;
    }
  // M-blocks of this wave: k' = 4 tap + c, tap = 4 mb + (lane's p); mb 7 (taps 28..31) is all zero
  const int mb0 = 2 * wave, nmb = wave < 3 ? 2 : 1;
  int tapoff[2];
  bool tapok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tap = 4 * (mb0 + i) + pp;
    tapok[i] = tap < 25;
    tapoff[i] = tapok[i] ? (tap / 5) * p.wcols + (tap % 5) : 0;
  }

  u32x4 dv[NWG_PX * 8 / 256];  // 8 x 16 B of the next D tile
  elem_t xv[NWG_WPT][CIN];
  // chunk-invariant addressing, computed once (round 6: the per-chunk divisions by Wd / wcols and
  // bounds selects were most of the kernel's VALU, 13.8 VALU per MFMA in profiles/pmc/step_pmc_r5b.txt):
  // a chunk's D tile is tyc full rows = one contiguous block; window pixel s sits at row wr(s),
  // column wc(s) of every chunk's window, only the window's first input row changes per chunk
  int w_off[NWG_WPT], w_row[NWG_WPT];
#pragma unroll
  for (int i = 0; i < NWG_WPT; ++i) {
    const int s_ = tid + 256 * i;
    const int wr = s_ / p.wcols, wc = s_ - wr * p.wcols, ix = wc - p.pl;
    const bool col_ok = s_ < zero_pix && (unsigned)ix < (unsigned)p.W;
    w_row[i] = col_ok ? wr : -(1 << 20);  // an invalid column fails every row test below
    w_off[i] = (wr * p.W + ix) * CIN;
  }
  auto fetch = [&](int y0) {
    const elem_t* dsrc = p.d + ((size_t)b * p.Hd + y0) * p.Wd * 64;
    const int lim = min(p.tyc, p.Hd - y0) * p.Wd * 64;  // elements of the chunk inside the image
#pragma unroll
    for (int i = 0; i < NWG_PX * 8 / 256; ++i) {
      const int e0 = (tid + 256 * i) * 8;
      dv[i] = e0 < lim ? *reinterpret_cast<const u32x4*>(dsrc + e0) : (u32x4){0u, 0u, 0u, 0u};
    }
    const int iy0 = 2 * y0 - p.pl;
    const long long xbase = ((long long)b * p.H + iy0) * p.W * CIN;  // (row iy0 may be -1 / -2: only
#pragma unroll                                                          //  valid rows are read)
    for (int i = 0; i < NWG_WPT; ++i) {
      const bool ok = (unsigned)(iy0 + w_row[i]) < (unsigned)p.H;
#pragma unroll
      for (int cc = 0; cc < CIN; ++cc) xv[i][cc] = ok ? p.x[xbase + w_off[i] + cc] : (elem_t)0.f;
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < NWG_PX * 8 / 256; ++i) {
      const int qd = tid + 256 * i, px = qd >> 3, j = qd & 7;
      *reinterpret_cast<u32x4*>(dt + px * 128 + ((j ^ (nwg_swz(px) >> 1)) << 4)) = dv[i];
    }
#pragma unroll
    for (int i = 0; i < NWG_WPT; ++i) {
      const int s = tid + 256 * i;
      if (s < zero_pix) {
        elem4 v = {(elem_t)0.f, (elem_t)0.f, (elem_t)0.f, (elem_t)0.f};
#pragma unroll
        for (int cc = 0; cc < CIN; ++cc) v[cc] = xv[i][cc];
        *reinterpret_cast<elem4*>(win + s * 8) = v;
      }
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[i][nb] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const lds_char* dt3 = (const lds_char*)dt;
  const lds_char* win3 = (const lds_char*)win;
  int nch = 0;  // chunks of this workgroup that start inside the image
  for (int c = 0; c < p.chunks_per_wg; ++c) nch += (yb + c * p.tyc < p.Hd) ? 1 : 0;
  if (nch > 0) {
    fetch(yb);
    commit();
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) fetch(yb + (c + 1) * p.tyc);  // next chunk in flight during this one
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks >= p.nks) break;  // wave-uniform: EXEC stays full for the tr reads
      elem8 bfr[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 32 * ks + 8 * g + 4 * h + q;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, dt3 + r * 128 + (((4 * nb + pp) ^ nwg_swz(r)) << 3)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[nb][4 * h + e] = vb[e];
        }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i < nmb) {  // wave-uniform
          elem8 af;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int pix = tapok[i] ? pxoff[ks][h] + tapoff[i] : zero_pix;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, win3 + pix * 8));
            const elem4 va = __builtin_bit_cast(elem4, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) af[4 * h + e] = va[e];
          }
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) acc[i][nb] = DCG_MFMA_16x16x32(af, bfr[nb], acc[i][nb], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // every wave is done with this chunk's tiles
    if (c + 1 < nch) {
      commit();
      __syncthreads();
    }
  }
  // ---- partial: lane holds C[k' = 16 mb + 4 g + e][n = 16 nb + li] -> tap 4 mb + g, channel e
  float* dst = p.part + (size_t)blockIdx.x * 25 * CIN * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i < nmb) {
      const int tap = 4 * (mb0 + i) + g;
      if (tap < 25) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int e = 0; e < CIN; ++e) dst[(tap * CIN + e) * 64 + 16 * nb + li] = acc[i][nb][e];
      }
    }
  }
}

}  // namespace dcg

using namespace dcg;

// grid = persistent workgroup count (<= tiles); part / bx.. only with bnb != 0
extern "C" int DCG_API(dcg_nconv)(const elem_t* x, const elem_t* w, const float* bias, elem_t* y, int B, int H, int W,
                                  int Cin, int Ho, int Wo, int pad_y, int pad_x, int act, float leak, int grid,
                                  const elem_t* bx, const elem_t* by, const float* mean, const float* rstd, int bact,
                                  float bleak, float* part, hipStream_t s) {
  if (Cin < 1 || Cin > 4 || pad_y < 0 || pad_y > 2 || pad_x < 0 || pad_x > 2) return -2;
  if (Ho != (H + 1) / 2 || Wo != (W + 1) / 2) return -2;
  NConvArgs a{};
  a.x = x; a.w = w; a.bias = bias; a.y = y;
  a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.pad_y = pad_y; a.pad_x = pad_x; a.act = act; a.leak = leak;
  a.tiles_x = (Wo + NC_TX - 1) / NC_TX;
  a.tiles_per_img = a.tiles_x * ((Ho + NC_TY - 1) / NC_TY);
  a.ntiles = B * a.tiles_per_img;
  if (grid < 1 || grid > a.ntiles) return -2;
  a.bx = bx; a.by = by; a.mean = mean; a.rstd = rstd; a.bact = bact; a.bleak = bleak; a.part = part;
  const bool bnb = bx != nullptr;
  if (bnb && (!by || !mean || !rstd || !part)) return -2;
#define NC_ACT(CI, BB)                                                                              \
  switch (act) {                                                                                    \
    case ACT_RELU: hipLaunchKernelGGL((nconv_kernel<CI, BB, ACT_RELU>), dim3(grid), dim3(256), 0, s, a); break;   \
    case ACT_LRELU: hipLaunchKernelGGL((nconv_kernel<CI, BB, ACT_LRELU>), dim3(grid), dim3(256), 0, s, a); break; \
    case ACT_TANH: hipLaunchKernelGGL((nconv_kernel<CI, BB, ACT_TANH>), dim3(grid), dim3(256), 0, s, a); break;   \
    default: hipLaunchKernelGGL((nconv_kernel<CI, BB, ACT_NONE>), dim3(grid), dim3(256), 0, s, a); break;         \
  }
#define NC_LAUNCH(CI)    \
  if (bnb) {             \
    NC_ACT(CI, true)     \
  } else {               \
    NC_ACT(CI, false)    \
  }
  switch (Cin) {
    case 1: NC_LAUNCH(1) break;
    case 2: NC_LAUNCH(2) break;
    case 3: NC_LAUNCH(3) break;
    default: NC_LAUNCH(4) break;
  }
#undef NC_LAUNCH
#undef NC_ACT
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_nconv_tiles)(int B, int Ho, int Wo) {
  return B * ((Wo + NC_TX - 1) / NC_TX) * ((Ho + NC_TY - 1) / NC_TY);
}

// nwgrad geometry for (Hd, Wd): rows per chunk, window shape; -1 when unsupported
extern "C" int DCG_API(dcg_nwgrad_plan)(int H, int W, int Hd, int Wd, int* tyc, int* wrows, int* wcols) {
  if (Wd < 1 || Wd > NWG_PX || Hd < 1 || W > 2 * Wd + 1 || H > 2 * Hd + 1) return -1;
  const int t = NWG_PX / Wd;
  const int wr = 2 * t + 3, wc = 2 * Wd + 3;
  if (wr * wc > NWG_WIN) return -1;
  *tyc = t; *wrows = wr; *wcols = wc;
  return 0;
}

extern "C" int DCG_API(dcg_nwgrad)(const elem_t* x, int B, int H, int W, int Cin, const elem_t* d, int Hd, int Wd,
                                   int pl, int chunks_per_wg, float* part, hipStream_t s) {
  NWGradArgs a{};
  if (Cin < 1 || Cin > 4 || pl < 0 || pl > 2 || chunks_per_wg < 1) return -2;
  if (DCG_API(dcg_nwgrad_plan)(H, W, Hd, Wd, &a.tyc, &a.wrows, &a.wcols)) return -2;
  a.x = x; a.H = H; a.W = W; a.d = d; a.Hd = Hd; a.Wd = Wd; a.pl = pl;
  a.np = a.tyc * Wd;
  a.nks = (a.np + 31) / 32;
  a.chunks_per_wg = chunks_per_wg;
  const int chunks_per_img = (Hd + a.tyc - 1) / a.tyc;
  a.wg_per_img = (chunks_per_img + chunks_per_wg - 1) / chunks_per_wg;
  a.part = part;
  const size_t shm = (size_t)NWG_PX * 128 + (size_t)(a.wrows * a.wcols + 1) * 8;
  const unsigned grid = (unsigned)(B * a.wg_per_img);
#define NW_LAUNCH(CI)                                                                                       \
  {                                                                                                         \
    static bool attr = false;                                                                               \
    if (!attr) {                                                                                            \
      hipError_t e = hipFuncSetAttribute((const void*)nwgrad_kernel<CI>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                         (int)(NWG_PX * 128 + (NWG_WIN + 1) * 8));                          \
      if (e != hipSuccess) return (int)e;                                                                   \
      attr = true;                                                                                          \
    }                                                                                                       \
    hipLaunchKernelGGL(nwgrad_kernel<CI>, dim3(grid), dim3(256), shm, s, a);                                \
  }
  switch (Cin) {
    case 1: NW_LAUNCH(1) break;
    case 2: NW_LAUNCH(2) break;
    case 3: NW_LAUNCH(3) break;
    default: NW_LAUNCH(4) break;
  }
#undef NW_LAUNCH
  return (int)hipGetLastError();
}
#endif  // DCG_F32
