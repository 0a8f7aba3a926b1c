// dcg-variants: bf16 f16
// Direct MFMA convolution for the narrow-INPUT stride-2 5x5 TF-SAME conv: D layer 0 (RGB / gray
// image -> 64 channels, + bias + LeakyReLU). The im2col + GEMM pair it replaces on the forward
// path wrote and re-read a [rows][80] column matrix (2 x 42 MB at 64x64, 2B = 256) for a GEMM
// with K = 75; here the image tile is staged once in LDS and the A fragments are built from it.
//
// Workgroup = 16x16 output pixels of one image; LDS holds the 35x35 input region (stride 2,
// 5 taps, pad_lo rows/cols before) as 4-channel pixels (8 B; channel 3 and out-of-image pixels
// zero) and the weights transposed to [N][K=128] with k = 4 * tap + c (taps 25..31 and c = 3
// are zero), so each 16x16x32 MFMA k-block covers 8 taps. A fragment (lane l: pixel l & 15 of
// the M-block, k = 8 (l >> 4) + j) = two taps x 4 channels = two ds_read_b64 of the staged
// tile; B fragments (N = 64 = 4 blocks x 4 k-blocks) stay in 64 VGPRs for the whole tile.
// Wave w computes output rows 4w..4w+3 of the tile (one M-block per row). Epilogue: bias +
// activation, bf16 through LDS, 16-byte coalesced stores.
#include "kernels.h"

namespace dcg {

constexpr int C3_TILE = 16;
constexpr int C3_IN = 2 * C3_TILE + 3;  // 35 input rows/cols per 16 output rows/cols (k=5, s=2)
constexpr int C3_N = 64;
constexpr int C3_K = 128;
constexpr int C3_KS = C3_K + 8;  // LDS row stride of the transposed weights: the n-strided scatter
                                 // walks the banks 4 dwords apart instead of hitting one bank

template <int Cin>
__global__ __launch_bounds__(256) void conv3_direct_kernel(const elem_t* __restrict__ x, const elem_t* __restrict__ w,
                                                           const float* __restrict__ bias, elem_t* __restrict__ y,
                                                           int H, int W, int Ho, int Wo, int pad_y,
                                                           int pad_x, int act, float leak, int tiles_x,
                                                           int tiles_per_img) {
  constexpr int OS = C3_N + 8;  // output staging pixel stride: the 4 pixel rows of a ds_write_b16 half-wave
                               // land 16 dwords apart (conflict-free)
  __shared__ __attribute__((aligned(16))) char smem[C3_TILE * C3_TILE * OS * 2];  // 36 KB (output staging)
  elem_t* xs = reinterpret_cast<elem_t*>(smem);                                 // [35*35][4]  9800 B
  elem_t* wt = reinterpret_cast<elem_t*>(smem + 10240);                         // [64][136]  17 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / tiles_per_img;
  const int trem = blockIdx.x - b * tiles_per_img;
  const int ty0 = (trem / tiles_x) * C3_TILE, tx0 = (trem % tiles_x) * C3_TILE;
  const int iy0 = 2 * ty0 - pad_y, ix0 = 2 * tx0 - pad_x;

  // ---- stage the input region (4-channel pixels, zero padded) and the transposed weights.
  // Both loops walk their source in memory order (coalesced 2-byte loads): the image region
  // element by element, the HWIO weights [25][Cin][64] with the output channel fastest.
  uint2* wz = reinterpret_cast<uint2*>(wt);
  for (int q = tid; q < C3_N * C3_KS / 4; q += 256) wz[q] = make_uint2(0u, 0u);  // pad taps / channel 3
  // all loads of a thread are issued before the first LDS store (fixed trip counts, unrolled):
  // one load latency per workgroup instead of one per loop iteration
  const int nel = C3_IN * C3_IN * Cin;  // <= 4900 = 20 x 256 (Cin <= 4)
  elem_t xv[20];
#pragma unroll
  for (int it = 0; it < 20; ++it) {
    const int q = tid + it * 256;
    xv[it] = (elem_t)0.f;
    if (q < nel) {
      const int pq = q / Cin, c = q - pq * Cin;
      const int ry = pq / C3_IN, rx = pq - ry * C3_IN;
      const int iy = iy0 + ry, ix = ix0 + rx;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) xv[it] = x[(((size_t)b * H + iy) * W + ix) * Cin + c];
    }
  }
  const int nw = 25 * Cin * C3_N;  // <= 6400 = 25 x 256
  elem_t wv[25];
#pragma unroll
  for (int it = 0; it < 25; ++it) {
    const int q = tid + it * 256;
    wv[it] = q < nw ? w[q] : (elem_t)0.f;
  }
#pragma unroll
  for (int it = 0; it < 20; ++it) {
    const int q = tid + it * 256;
    if (q < nel) {
      const int pq = q / Cin, c = q - pq * Cin;
      xs[pq * 4 + c] = xv[it];
      if (c == Cin - 1)
        for (int cc = Cin; cc < 4; ++cc) xs[pq * 4 + cc] = (elem_t)0.f;
    }
  }
  __syncthreads();  // the zero fill of wt precedes the weight scatter below
#pragma unroll
  for (int it = 0; it < 25; ++it) {
    const int q = tid + it * 256;
    if (q < nw) {
      const int n = q & (C3_N - 1), kk = q >> 6;  // kk = tap * Cin + c
      const int tap = kk / Cin, c = kk - tap * Cin;
      wt[n * C3_KS + 4 * tap + c] = wv[it];
    }
  }
  __syncthreads();

  const int r = lane & 15, qq = lane >> 4;
  elem8 bfr[4][4];  // [n-block][k-block]: lane holds B[k = 32 kb + 8 qq + j][n = 16 nb + r]
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
      bfr[nb][kb] = *reinterpret_cast<const elem8*>(wt + (16 * nb + r) * C3_KS + 32 * kb + 8 * qq);

  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[m][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    // this lane's two taps of the k-block (taps >= 25 have zero weights: clamp the address)
    const int t0 = min(8 * kb + 2 * qq, 24), t1 = min(8 * kb + 2 * qq + 1, 24);
    const int off0 = (t0 / 5) * C3_IN + (t0 % 5), off1 = (t1 / 5) * C3_IN + (t1 % 5);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int oyl = 4 * wave + m;                  // output row within the tile (M-block m)
      const int base = (2 * oyl) * C3_IN + 2 * r;    // input pixel of tap (0, 0)
      const elem4 a0 = *reinterpret_cast<const elem4*>(xs + (base + off0) * 4);
      const elem4 a1 = *reinterpret_cast<const elem4*>(xs + (base + off1) * 4);
      const elem8 af = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[m][nb] = DCG_MFMA_16x16x32(af, bfr[nb][kb], acc[m][nb], 0, 0, 0);
    }
  }
  __syncthreads();  // everyone is done with xs / wt: reuse the LDS for the output tile
  elem_t* os = reinterpret_cast<elem_t*>(smem);  // [16 rows][16 px][64 ch]
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int n = 16 * nb + r;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = 4 * qq + i;  // C row = pixel within the M-block
        os[((4 * wave + m) * C3_TILE + px) * OS + n] = f2bf(apply_act(acc[m][nb][i] + bv, act, leak));
      }
  }
  __syncthreads();
  // 16 rows x 16 px x 64 ch = 16 rows of 2 KB contiguous in NHWC (one output row segment each)
  for (int q = tid; q < C3_TILE * C3_TILE * C3_N / 8; q += 256) {
    const int row = q >> 7, rem = q & 127;  // 128 chunks of 8 channels per row (16 px x 8 chunks)
    const int oy = ty0 + row;
    const int px = rem >> 3, ch = rem & 7;
    const int ox = tx0 + px;
    if (oy < Ho && ox < Wo)
      *reinterpret_cast<elem8*>(y + (((size_t)b * Ho + oy) * Wo + ox) * C3_N + ch * 8) =
          *reinterpret_cast<const elem8*>(os + (row * C3_TILE + px) * OS + ch * 8);
  }
}

}  // namespace dcg

extern "C" int DCG_API(dcg_conv3_direct)(const elem_t* x, const elem_t* w, const float* bias, elem_t* y, int B, int H,
                                         int W, int Cin, int Ho, int Wo, int Cout, int pad_y, int pad_x, int act,
                                         float leak, hipStream_t s) {
  // stride 2, 5x5, Cin <= 4, Cout = 64; the 35x35 staged region covers a 16x16 output tile
  if (Cin < 1 || Cin > 4 || Cout != dcg::C3_N || pad_y < 0 || pad_y > 2 || pad_x < 0 || pad_x > 2) return -2;
  if (Ho != (H + 1) / 2 || Wo != (W + 1) / 2) return -2;
  const int tiles_x = (Wo + dcg::C3_TILE - 1) / dcg::C3_TILE, tiles_y = (Ho + dcg::C3_TILE - 1) / dcg::C3_TILE;
#define C3_LAUNCH(CI)                                                                                          \
  hipLaunchKernelGGL(dcg::conv3_direct_kernel<CI>, dim3(B * tiles_x * tiles_y), dim3(256), 0, s, x, w, bias, y, H, W, \
                     Ho, Wo, pad_y, pad_x, act, leak, tiles_x, tiles_x * tiles_y)
  switch (Cin) {
    case 1: C3_LAUNCH(1); break;
    case 2: C3_LAUNCH(2); break;
    case 3: C3_LAUNCH(3); break;
    default: C3_LAUNCH(4); break;
  }
#undef C3_LAUNCH
  return (int)hipGetLastError();
}
