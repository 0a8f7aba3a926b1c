// dcg-variants: bf16 f16
// Narrow-output TF-SAME stride-2 5x5 conv_transpose (N = 1..4 output channels), direct on VALU:
// the two 3-channel GEMMs of the step -- G's last layer (64 -> 3, + bias + tanh) and D layer 0's
// data gradient for the fake half (64 -> 3) -- where an MFMA tile pads N=3 to 16 (5x waste;
// measured 29 TF/s, 43 us each at B=128).
//
// Workgroup = one output tile of 16x16 pixels of one image = the 4 sub-pixel phases x an 8x8
// grid; wave w computes phase w (so every lane of a wave walks the same tap list and the weight
// reads are LDS broadcasts). The input halo (<= 12x12 pixels x C channels) and all 25 x N x C
// weights are staged once in LDS; each lane accumulates its pixel's N outputs in fp32 with
// v_dot2_f32_bf16 (2 MACs / instruction) over 8-channel 16-byte chunks.
#include "kernels.h"

namespace dcg {

constexpr int NW_TILE = 16;   // output tile edge
constexpr int NW_HALO = 12;   // input tile edge (covers the taps of all 4 phases, pad <= 2)

template <int K>
__device__ __forceinline__ float dot2k(const elem8 a, const elem8 b, float acc) {
#ifdef DCG_F16
  return __builtin_amdgcn_fdot2(__builtin_shufflevector(a, a, K, K + 1), __builtin_shufflevector(b, b, K, K + 1), acc,
                                false);
#else
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, K, K + 1),
                                         __builtin_shufflevector(b, b, K, K + 1), acc, false);
#endif
}

__device__ __forceinline__ float dot8(const elem8 a, const elem8 b, float acc) {
  acc = dot2k<0>(a, b, acc);
  acc = dot2k<2>(a, b, acc);
  acc = dot2k<4>(a, b, acc);
  return dot2k<6>(a, b, acc);
}

template <int N, int CT8>  // CT8 = C / 8 when fixed at compile time (0 = runtime C)
__global__ __launch_bounds__(256) void narrow_deconv_kernel(const elem_t* __restrict__ x, const elem_t* __restrict__ w,
                                                            const float* __restrict__ bias, elem_t* __restrict__ y,
                                                            int Hi, int Wi, int C, int Ho, int Wo, int pad, int act,
                                                            float leak, int tiles_x, int tiles_per_img) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int C8 = CT8 > 0 ? CT8 : (C >> 3);
  const int swz = ((C8 & (C8 - 1)) == 0) ? ((C8 - 1) & 7) : 0;  // chunk XOR (power-of-2 chunk counts)
  elem8* xs = reinterpret_cast<elem8*>(smem);                         // [HALO*HALO][C8] (chunk-swizzled)
  elem8* ws = xs + NW_HALO * NW_HALO * C8;                            // [25][N][C8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / tiles_per_img;
  const int trem = blockIdx.x - b * tiles_per_img;
  const int ty0 = (trem / tiles_x) * NW_TILE, tx0 = (trem % tiles_x) * NW_TILE;
  // input rows/cols needed: iy = (oy + pad - ky) / 2 for oy in [ty0, ty0 + 16), ky in [0, 5)
  const int iy_lo = (ty0 + pad - 4) >> 1, ix_lo = (tx0 + pad - 4) >> 1;  // floor division (>> on negatives)

  // ---- stage input halo (zero outside the image) and weights
  const elem8 zero8 = {};
  for (int q = tid; q < NW_HALO * NW_HALO * C8; q += 256) {
    const int pix = q / C8, c = q - pix * C8;
    const int iy = iy_lo + pix / NW_HALO, ix = ix_lo + pix % NW_HALO;
    elem8 v = zero8;
    if ((unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi)
      v = *reinterpret_cast<const elem8*>(x + (((size_t)b * Hi + iy) * Wi + ix) * C + c * 8);
    xs[pix * C8 + (c ^ (pix & swz))] = v;
  }
  for (int q = tid; q < 25 * N * C8; q += 256) ws[q] = reinterpret_cast<const elem8*>(w)[q];
  __syncthreads();

  // ---- this lane's output pixel: phase (py, px) = wave, grid position = lane
  const int py = wave >> 1, px = wave & 1;
  const int oy = ty0 + 2 * (lane >> 3) + py, ox = tx0 + 2 * (lane & 7) + px;
  const int kys = (oy + pad) & 1, kxs = (ox + pad) & 1;  // tap parities of this phase
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
  for (int ky = kys; ky < 5; ky += 2) {
    const int iy = ((oy + pad - ky) >> 1) - iy_lo;
    for (int kx = kxs; kx < 5; kx += 2) {
      const int ix = ((ox + pad - kx) >> 1) - ix_lo;
      const int pix = iy * NW_HALO + ix;
      const elem8* xr = xs + pix * C8;
      const elem8* wr = ws + (ky * 5 + kx) * N * C8;
      if constexpr (CT8 > 0) {
        // fixed channel count: the tap's N x C weights in registers (one broadcast read each),
        // then one input read + 4N dot2 per 8-channel chunk
        elem8 wv[N][CT8];
#pragma unroll
        for (int n = 0; n < N; ++n)
#pragma unroll
          for (int c = 0; c < CT8; ++c) wv[n][c] = wr[n * CT8 + c];
#pragma unroll
        for (int c = 0; c < CT8; ++c) {
          const elem8 xv = xr[c ^ (pix & swz)];
#pragma unroll
          for (int n = 0; n < N; ++n) acc[n] = dot8(xv, wv[n][c], acc[n]);
        }
      } else {
        for (int c = 0; c < C8; ++c) {
          const elem8 xv = xr[c ^ (pix & swz)];
#pragma unroll
          for (int n = 0; n < N; ++n) acc[n] = dot8(xv, wr[n * C8 + c], acc[n]);
        }
      }
    }
  }
  if (oy < Ho && ox < Wo) {
    elem_t* dst = y + (((size_t)b * Ho + oy) * Wo + ox) * N;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float v = acc[n] + (bias ? bias[n] : 0.f);
      dst[n] = f2bf(apply_act(v, act, leak));
    }
  }
}

// MFMA form of the same operation (C a multiple of 32): identical tile, halo and weight
// staging, but each wave computes its phase's 8x8 = 64 output pixels as 4 M-blocks of a
// v_mfma_f32_16x16x32 GEMM: A = 16 pixels x 32 channels read straight from the staged halo at
// the tap's shift (lane l: pixel l&15, 8-channel chunk l>>4 -- one ds_read_b128), B = 32
// channels x 16 outputs of the tap's weights (outputs >= N are zero lanes). N=3 pads to 16
// (5.3x the useful MACs), but one MFMA replaces 64 lanes x 32 MACs of v_dot2 work at 4x the
// per-SIMD rate of the VALU kernel above (measured: see BASELINE.md / profiles).
// DACT: the output is multiplied by act'(ya) (ya = the activation output at the same pixel: the
// tanh backward of G's RGB layer fused into the image-gradient kernel) and every workgroup writes
// its per-channel partial sum of the stored values (the bias gradient) to part[blockIdx][N].
// BNIN: x is the PRE-BN input of the layer below; the halo staging applies that BN + activation
// (scale / shift [C], one group) and the workgroup writes the activation of the 8x8 input pixels
// it owns (the ones under its 16x16 output tile) to a_out -- the layer's separate BN-apply launch
// folded into this one (the backward reads a_out).
struct NarrowBnIn {
  const float* scale; const float* shift; int act; float leak; elem_t* a_out;
};

template <int N, int C8, bool WG, bool DACT = false, bool BNIN = false>  // WG: B fragments from global/L1
__global__ __launch_bounds__(256) void narrow_deconv_mfma_kernel(const elem_t* __restrict__ x,
                                                                 const elem_t* __restrict__ w,
                                                                 const float* __restrict__ bias,
                                                                 elem_t* __restrict__ y, int Hi, int Wi, int Ho,
                                                                 int Wo, int pad, int act, float leak, int tiles_x,
                                                                 int tiles_per_img, const elem_t* __restrict__ ya,
                                                                 float* __restrict__ part, NarrowBnIn bnin) {
  static_assert(C8 == 8, "the bank swizzle below assumes 8 chunks (64 channels) per pixel");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  elem8* xs = reinterpret_cast<elem8*>(smem);  // [HALO*HALO][C8], chunk c of pixel (row, col) at c ^ sw(col)
  elem8* ws = xs + NW_HALO * NW_HALO * C8;     // [25][N][C8]
  // sw(col) = 2 * ((col >> 1) & 3): an A-fragment read (ds_read_b128, 4 lane groups of 16) takes 8
  // consecutive halo columns (any shift) for each of two chunk quarters qq, qq+1 of one k-block;
  // bank slot = (col & 1) * 8 + (chunk ^ sw): the 8 columns fill 8 distinct slots and the two
  // chunks land on opposite chunk parities -> conflict-free for every tap.
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / tiles_per_img;
  const int trem = blockIdx.x - b * tiles_per_img;
  const int ty0 = (trem / tiles_x) * NW_TILE, tx0 = (trem % tiles_x) * NW_TILE;
  const int iy_lo = (ty0 + pad - 4) >> 1, ix_lo = (tx0 + pad - 4) >> 1;
  const elem8 zero8 = {};
  float bsc[BNIN ? 8 : 1], bsh[BNIN ? 8 : 1];  // BNIN: this thread's chunk is always tid & 7
  if constexpr (BNIN) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bsc[i] = bnin.scale[(tid & 7) * 8 + i];
      bsh[i] = bnin.shift[(tid & 7) * 8 + i];
    }
  }
  for (int q = tid; q < NW_HALO * NW_HALO * C8; q += 256) {
    const int pix = q >> 3, c = q & 7;
    const int row = pix / NW_HALO, col = pix - row * NW_HALO;
    const int iy = iy_lo + row, ix = ix_lo + col;
    elem8 v = zero8;
    if ((unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi) {
      const size_t o = (((size_t)b * Hi + iy) * Wi + ix) * (C8 * 8) + c * 8;
      v = *reinterpret_cast<const elem8*>(x + o);
      if constexpr (BNIN) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (elem_t)apply_act((float)v[i] * bsc[i] + bsh[i], bnin.act, bnin.leak);
        if ((iy >> 3) == (ty0 >> 4) && (ix >> 3) == (tx0 >> 4))  // this tile's own 8x8 input pixels
          *reinterpret_cast<elem8*>(bnin.a_out + o) = v;
      }
    }
    xs[pix * C8 + (c ^ (((col >> 1) & 3) << 1))] = v;
  }
  if (!WG)
    for (int q = tid; q < 25 * N * C8; q += 256) ws[q] = reinterpret_cast<const elem8*>(w)[q];
  __syncthreads();

  const int py = wave >> 1, px = wave & 1;  // this wave's sub-pixel phase
  const int r = lane & 15, qq = lane >> 4;
  // A rows of M-block m: phase pixel p = 16 m + r of the 8x8 grid -> (gy, gx) = (2 m + (r >> 3), r & 7);
  // its input pixel for tap (ky, kx) is (gy + oyk, gx + oxk), oyk = ((ty0 + py + pad - ky) >> 1) - iy_lo
  // (ty0 even: the shift is exact per tap)
  const int gy0 = r >> 3, gx = r & 7;
  const int kys = (ty0 + py + pad) & 1, kxs = (tx0 + px + pad) & 1;
  f32x4 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ky = kys; ky < 5; ky += 2) {
    const int oyk = ((ty0 + py + pad - ky) >> 1) - iy_lo;
    for (int kx = kxs; kx < 5; kx += 2) {
      const int col = gx + (((tx0 + px + pad - kx) >> 1) - ix_lo);
      const int sw = ((col >> 1) & 3) << 1;
      const elem8* wr = (WG ? reinterpret_cast<const elem8*>(w) : ws) + (ky * 5 + kx) * N * C8;
      const elem8* xr = xs + ((gy0 + oyk) * NW_HALO + col) * C8;  // M-block m adds 2 m halo rows
      elem8 bfs[C8 / 4];
#pragma unroll
      for (int kb = 0; kb < C8 / 4; ++kb) bfs[kb] = r < N ? wr[r * C8 + 4 * kb + qq] : zero8;
#pragma unroll
      for (int kb = 0; kb < C8 / 4; ++kb) {
        const int ch = 4 * kb + qq;
        const elem8 bf = bfs[kb];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const elem8 af = xr[2 * m * NW_HALO * C8 + (ch ^ sw)];
          acc[m] = DCG_MFMA_16x16x32(af, bf, acc[m], 0, 0, 0);
        }
      }
    }
  }
  // epilogue through LDS: the N useful accumulator columns (lanes r < N) -> [64 pixels][N] fp32 per
  // wave, then one lane per pixel applies bias + activation and stores its N outputs
  __syncthreads();  // every wave is done reading the halo
  float* ob = reinterpret_cast<float*>(smem) + wave * 64 * N;
  if (r < N) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) ob[(16 * m + 4 * qq + i) * N + r] = acc[m][i];
  }
  __syncthreads();
  const int oy = ty0 + 2 * (lane >> 3) + py, ox = tx0 + 2 * (lane & 7) + px;
  if constexpr (DACT) {
    float ps[N];
    const bool ok = oy < Ho && ox < Wo;
    const size_t o = (((size_t)b * Ho + (ok ? oy : 0)) * Wo + (ok ? ox : 0)) * N;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float v = ob[lane * N + n] + (bias ? bias[n] : 0.f);
      const elem_t r = f2bf(v * act_grad_from_out((float)ya[o + n], act, leak));
      if (ok) y[o + n] = r;
      ps[n] = wave_sum(ok ? (float)r : 0.f);
    }
    __syncthreads();  // every wave has read its ob rows: reuse the LDS for the wave partials
    float* wsum = reinterpret_cast<float*>(smem);
    if (lane == 0) {
#pragma unroll
      for (int n = 0; n < N; ++n) wsum[wave * N + n] = ps[n];
    }
    __syncthreads();
    if (tid < N) part[(size_t)blockIdx.x * N + tid] = ((wsum[tid] + wsum[N + tid]) + wsum[2 * N + tid]) + wsum[3 * N + tid];
  } else if (oy < Ho && ox < Wo) {
    elem_t* dst = y + (((size_t)b * Ho + oy) * Wo + ox) * N;
#pragma unroll
    for (int n = 0; n < N; ++n) dst[n] = f2bf(apply_act(ob[lane * N + n] + (bias ? bias[n] : 0.f), act, leak));
  }
}

}  // namespace dcg

extern "C" int DCG_API(dcg_narrow_deconv)(const elem_t* x, const elem_t* w, const float* bias, elem_t* y, int B,
                                          int Hi, int Wi, int C, int Ho, int Wo, int N, int pad, int act, float leak,
                                          hipStream_t s) {
  // the 12x12 halo covers oy in [ty0, ty0+16) for pad <= 2; C a multiple of 8 up to 256
  if (pad < 0 || pad > 2 || C % 8 || C > 256 || N < 1 || N > 4) return -2;
  const int tiles_x = (Wo + dcg::NW_TILE - 1) / dcg::NW_TILE, tiles_y = (Ho + dcg::NW_TILE - 1) / dcg::NW_TILE;
  const size_t shm = (size_t)(dcg::NW_HALO * dcg::NW_HALO + 25 * N) * C * sizeof(elem_t);
  if (shm > 160 * 1024) return -2;
  dim3 grid(B * tiles_x * tiles_y);
  static const bool valu_only = getenv("DCGAN_NARROW_VALU") != nullptr;  // A/B: the v_dot2 kernel
  static const bool w_lds = getenv("DCGAN_NARROW_WLDS") != nullptr;       // A/B: weights staged in LDS
  if (C == 64 && !valu_only) {
    const size_t shm_m = w_lds ? shm : (size_t)dcg::NW_HALO * dcg::NW_HALO * C * sizeof(elem_t);
#define NW_MFMA(NN)                                                                                            \
  {                                                                                                            \
    auto k = w_lds ? dcg::narrow_deconv_mfma_kernel<NN, 8, false> : dcg::narrow_deconv_mfma_kernel<NN, 8, true>; \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      if (e != hipSuccess) return (int)e;                                                                      \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL(k, grid, dim3(256), shm_m, s, x, w, bias, y, Hi, Wi, Ho, Wo, pad, act, leak, tiles_x,   \
                       tiles_x * tiles_y, (const elem_t*)nullptr, (float*)nullptr, dcg::NarrowBnIn{});         \
  }
    switch (N) {
      case 1: NW_MFMA(1) break;
      case 2: NW_MFMA(2) break;
      case 3: NW_MFMA(3) break;
      default: NW_MFMA(4) break;
    }
#undef NW_MFMA
    return (int)hipGetLastError();
  }
#define NW_LAUNCH(NN)                                                                                          \
  {                                                                                                            \
    auto k = C == 64 ? dcg::narrow_deconv_kernel<NN, 8> : dcg::narrow_deconv_kernel<NN, 0>;                    \
    static bool attr[2] = {false, false};                                                                      \
    if (!attr[C == 64]) {                                                                                      \
      hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      if (e != hipSuccess) return (int)e;                                                                      \
      attr[C == 64] = true;                                                                                    \
    }                                                                                                          \
    hipLaunchKernelGGL(k, grid, dim3(256), shm, s, x, w, bias, y, Hi, Wi, C, Ho, Wo, pad, act, leak, tiles_x,  \
                       tiles_x * tiles_y);                                                                     \
  }
  switch (N) {
    case 1: NW_LAUNCH(1) break;
    case 2: NW_LAUNCH(2) break;
    case 3: NW_LAUNCH(3) break;
    default: NW_LAUNCH(4) break;
  }
#undef NW_LAUNCH
  return (int)hipGetLastError();
}

// image gradient of G's RGB layer with its activation backward fused (narrow_deconv_mfma_kernel
// DACT): y = conv_transpose(x, w) * act'(ya); part[tiles][N] = per-workgroup column sums of y
extern "C" int DCG_API(dcg_narrow_deconv_dact)(const elem_t* x, const elem_t* w, elem_t* y, const elem_t* ya, int B,
                                               int Hi, int Wi, int C, int Ho, int Wo, int N, int pad, int act,
                                               float leak, float* part, hipStream_t s) {
  if (pad < 0 || pad > 2 || C != 64 || N < 1 || N > 4 || !ya || !part) return -2;
  const int tiles_x = (Wo + dcg::NW_TILE - 1) / dcg::NW_TILE, tiles_y = (Ho + dcg::NW_TILE - 1) / dcg::NW_TILE;
  const size_t shm = (size_t)dcg::NW_HALO * dcg::NW_HALO * C * sizeof(elem_t);
  dim3 grid(B * tiles_x * tiles_y);
#define NWD(NN)                                                                                                \
  {                                                                                                            \
    auto k = dcg::narrow_deconv_mfma_kernel<NN, 8, true, true>;                                                \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      if (e != hipSuccess) return (int)e;                                                                      \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL(k, grid, dim3(256), shm, s, x, w, (const float*)nullptr, y, Hi, Wi, Ho, Wo, pad, act, leak, \
                       tiles_x, tiles_x * tiles_y, ya, part, dcg::NarrowBnIn{});                               \
  }
  switch (N) {
    case 1: NWD(1) break;
    case 2: NWD(2) break;
    case 3: NWD(3) break;
    default: NWD(4) break;
  }
#undef NWD
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_narrow_deconv_tiles)(int B, int Ho, int Wo) {
  return B * ((Wo + dcg::NW_TILE - 1) / dcg::NW_TILE) * ((Ho + dcg::NW_TILE - 1) / dcg::NW_TILE);
}

// G's RGB layer forward with the BN apply + activation of the layer below fused into the halo
// staging (x = that layer's pre-BN output, a_out = its activation, written by the owning tiles)
extern "C" int DCG_API(dcg_narrow_deconv_bnin)(const elem_t* x, const elem_t* w, const float* bias, elem_t* y, int B,
                                               int Hi, int Wi, int C, int Ho, int Wo, int N, int pad, int act,
                                               float leak, const float* scale, const float* shift, int bn_act,
                                               float bn_leak, elem_t* a_out, hipStream_t s) {
  // every input pixel must sit under exactly one 16x16 output tile: Ho = 2 Hi, Wo = 2 Wi
  if (pad < 0 || pad > 2 || C != 64 || N < 1 || N > 4 || Ho != 2 * Hi || Wo != 2 * Wi || !scale || !shift || !a_out)
    return -2;
  const int tiles_x = (Wo + dcg::NW_TILE - 1) / dcg::NW_TILE, tiles_y = (Ho + dcg::NW_TILE - 1) / dcg::NW_TILE;
  const size_t shm = (size_t)dcg::NW_HALO * dcg::NW_HALO * C * sizeof(elem_t);
  dim3 grid(B * tiles_x * tiles_y);
  const dcg::NarrowBnIn bn{scale, shift, bn_act, bn_leak, a_out};
#define NWB(NN)                                                                                                \
  {                                                                                                            \
    auto k = dcg::narrow_deconv_mfma_kernel<NN, 8, true, false, true>;                                         \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      if (e != hipSuccess) return (int)e;                                                                      \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL(k, grid, dim3(256), shm, s, x, w, bias, y, Hi, Wi, Ho, Wo, pad, act, leak, tiles_x,     \
                       tiles_x * tiles_y, (const elem_t*)nullptr, (float*)nullptr, bn);                        \
  }
  switch (N) {
    case 1: NWB(1) break;
    case 2: NWB(2) break;
    case 3: NWB(3) break;
    default: NWB(4) break;
  }
#undef NWB
  return (int)hipGetLastError();
}
