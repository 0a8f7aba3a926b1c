// dcg-variants: bf16 f16
// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), NHWC, elem_t in / fp32 acc.
//
// One kernel family covers every conv-shaped op of the DCGAN step:
//   * TF-'SAME' stride-2 5x5 conv (D forward, G dgrad)          mode "conv":   25 taps, sstride 2
//   * TF-'SAME' stride-2 5x5 conv_transpose (G forward, D dgrad) mode "deconv": sub-pixel phase
//     decomposition -> 4 dense convs with 3x3 / 3x2 / 2x3 / 2x2 taps (no zero-insertion, no 4x
//     wasted MACs); the phase is blockIdx.z and each phase scatters to its output pixels.
//   * plain GEMM C[M][N] = A[M][K] . Bt[N][K]                    mode "plain" (im2col'd 3-channel
//     layers, 1 tap).
// GEMM view: rows m = output pixels of one phase, cols n = output channels, k = (tap, channel).
// Weights are pre-packed elem_t [25][N][Kc] (k contiguous per output channel), so both operands
// are "K-contiguous rows" and every fragment is one 16-byte ds_read_b128.
//
// Block = 256 threads (4 waves, WM x WN wave grid), tile BM x BN x 64, two LDS stages, one
// barrier per K-tile. Two staging variants (template STAGING):
//   0: register staging -- next tile's 16-byte global loads issued before the current tile's
//      MFMAs, written to the other LDS stage after them (ds_write_b128).
//   1: LDS-DMA staging -- `buffer_load_dwordx4 ... lds` writes each 1 KiB wave piece (8 rows x
//      128 B) straight into LDS: no VGPR staging, no ds_write. The LDS image is lane-linear, so
//      the XOR swizzle is applied to the per-lane SOURCE chunk (rule: linear dest + swizzled
//      source + the same XOR on the read).
// LDS rows are 128 B with a chunk ^= (row & 7) swizzle: conflict-free ds_read_b128 for the
// 16x16x32 A/B fragment maps. A-operand gathers use buffer loads whose out-of-range offset
// returns zeros, which implements the conv zero padding with no branches.
//
// Fused epilogue: + bias, per-channel BN partial statistics (sum, sum^2 of the stored elem_t
// value over the tile's rows, per (M-tile, phase) for a deterministic finalize), activation
// (relu / lrelu / tanh), pixel scatter of the phase, output staged through LDS and written as
// 16-byte row segments (elem_t, N % 8 == 0) or element-wise (fp32 / narrow N).
#include "epilogue.h"

namespace dcg {

template <int BM, int BN, int WM, int WN, int STAGING>
__global__ __launch_bounds__(256) void igemm_kernel(IGemmArgs p) {
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_CH = BM * 8, B_CH = BN * 8;
  constexpr int A_PT = (A_CH + 255) / 256, B_PT = (B_CH + 255) / 256;
  constexpr int STAGE = (BM + BN) * 8;  // 16-byte units per stage
  constexpr int NPA = BM / 8, NPB = BN / 8;  // 1 KiB LDS-DMA pieces per stage
  constexpr int PPW_A = (NPA + 3) / 4, PPW_B = (NPB + 3) / 4;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) u32x4 lds[2 * STAGE];
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_char*)lds;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int phase = blockIdx.z;
  const IGemmPhase* ph = p.ph + phase;
  const int M = ph->M;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  if (m0 >= M) {  // phase with fewer rows (odd output sizes): its stats slot must still be defined
    if (p.stats) {
      const int row = blockIdx.x * p.nphases + phase;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.stats + (size_t)row * 2 * p.N, (uint32_t)(2 * p.N * 4));
      for (int nl = threadIdx.x; nl < BN; nl += 256)
        if (n0 + nl < p.N) { st_sc1_f32(rs, (uint32_t)(n0 + nl) * 4u, 0.f); st_sc1_f32(rs, (uint32_t)(p.N + n0 + nl) * 4u, 0.f); }
    }
    return;
  }
  const int Kc = p.Kc, N = p.N;
  const int ntaps = p.plain ? 1 : ph->ntaps;
  const int kt_per_tap = (Kc + BK - 1) / BK;
  const int KT = ntaps * kt_per_tap;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.Bw, p.b_bytes);

  // ---- the A rows this thread loads (fixed for the whole K loop)
  constexpr int AR = STAGING ? PPW_A : A_PT;
  int a_bh[AR], a_iy[AR], a_ix[AR], a_row[AR];
  bool a_ok[AR];
  // register staging: row = (tid + 256 i) / 8, chunk = tid & 7
  // LDS-DMA: piece q = wave + 4 i, row = 8 q + lane / 8, LDS slot = lane & 7,
  //          global chunk = slot ^ (row & 7) = (lane & 7) ^ (lane >> 3)
  const int chunk = STAGING ? ((lane & 7) ^ (lane >> 3)) : (tid & 7);
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int r = STAGING ? (8 * (wave + 4 * i) + (lane >> 3)) : ((tid + 256 * i) >> 3);
    a_row[i] = r;
    const int m = m0 + r;
    a_ok[i] = (r < BM) && (m < M);
    if (p.plain) {
      a_bh[i] = m; a_iy[i] = 0; a_ix[i] = 0;
    } else {
      const uint32_t b = fdiv((uint32_t)m, ph->fd_hw);
      const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph->Hq * ph->Wq);
      const uint32_t qy = fdiv(rem, ph->fd_w);
      const uint32_t qx = rem - qy * (uint32_t)ph->Wq;
      a_bh[i] = (int)b * p.H;
      a_iy[i] = (int)qy * p.sstride + ph->iy0_off;
      a_ix[i] = (int)qx * p.sstride + ph->ix0_off;
    }
  }

  auto a_offset = [&](int i, int dy, int dx, int cc, bool kval) -> uint32_t {
    if (p.plain) return oob_unless(a_ok[i] && kval, (uint32_t)(a_bh[i] * Kc + cc) * 2u);
    const int iy = a_iy[i] + dy, ix = a_ix[i] + dx;
    return oob_unless(a_ok[i] && kval && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W,
                      (uint32_t)(((a_bh[i] + iy) * p.W + ix) * Kc + cc) * 2u);
  };

  u32x4 ra_reg[STAGING ? 1 : A_PT], rb_reg[STAGING ? 1 : B_PT];

  auto load_tile = [&](int kt, int buf) {
    const int ti = kt / kt_per_tap;
    const int c0 = (kt - ti * kt_per_tap) * BK;
    const int cc = c0 + chunk * 8;
    const bool kval = cc < Kc;
    int dy = 0, dx = 0, wt = 0;
    if (!p.plain) { dy = ph->dy[ti]; dx = ph->dx[ti]; wt = ph->wtap[ti]; }
    if constexpr (STAGING) {
      // asm LDS-DMA (common.h dma16_asm): the compiler-visible builtin made hipcc wait
      // vmcnt before every further DMA (measured: s_waitcnt vmcnt(3) between pieces)
      const uint32_t sa = lds_base + buf * STAGE * 16;
      const uint32_t sb = sa + BM * 128;
#pragma unroll
      for (int i = 0; i < PPW_A; ++i) {
        const int q = wave + 4 * i;
        if (NPA % 4 == 0 || q < NPA)
          dma16_asm_la(ra, sa + q * 1024, a_offset(i, dy, dx, cc, kval));
      }
#pragma unroll
      for (int i = 0; i < PPW_B; ++i) {
        const int q = wave + 4 * i;
        if (NPB % 4 == 0 || q < NPB) {
          const int n = n0 + 8 * q + (lane >> 3);
          dma16_asm_la(rb, sb + q * 1024, oob_unless(n < N && kval, (uint32_t)((wt * N + n) * Kc + cc) * 2u));
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_PT; ++i) ra_reg[i] = buf_load16(ra, a_offset(i, dy, dx, cc, kval));
#pragma unroll
      for (int i = 0; i < B_PT; ++i) {
        const int r = (tid + 256 * i) >> 3;
        const int n = n0 + r;
        uint32_t off = OOB;
        if (r < BN && n < N && kval) off = (uint32_t)((wt * N + n) * Kc + cc) * 2u;
        rb_reg[i] = buf_load16(rb, off);
      }
    }
  };

  auto store_tile = [&](int buf) {  // register staging only
    if constexpr (!STAGING) {
      u32x4* sa = lds + buf * STAGE;
      u32x4* sb = sa + BM * 8;
#pragma unroll
      for (int i = 0; i < A_PT; ++i) {
        const int r = (tid + 256 * i) >> 3;
        if (A_CH % 256 == 0 || r < BM) sa[r * 8 + (chunk ^ (r & 7))] = ra_reg[i];
      }
#pragma unroll
      for (int i = 0; i < B_PT; ++i) {
        const int r = (tid + 256 * i) >> 3;
        if (B_CH % 256 == 0 || r < BN) sb[r * 8 + (chunk ^ (r & 7))] = rb_reg[i];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  load_tile(0, 0);
  store_tile(0);
  if constexpr (STAGING) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tile(kt + 1, buf ^ 1);
    const u32x4* sa = lds + buf * STAGE;
    const u32x4* sb = sa + BM * 8;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      elem8 af[FM], bfr[FN];
      const int c = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * TM + i * 16 + fr;
        af[i] = __builtin_bit_cast(elem8, sa[r * 8 + (c ^ (r & 7))]);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * TN + j * 16 + fr;
        bfr[j] = __builtin_bit_cast(elem8, sb[r * 8 + (c ^ (r & 7))]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = DCG_MFMA_16x16x32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store_tile(buf ^ 1);
    if constexpr (STAGING) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // LDS reuse: rowoff[BM] ints | red[WM][BN][2] floats | C tile [BM][BN + 8] elem_t
  int* rowoff = reinterpret_cast<int*>(lds);
  float* red = reinterpret_cast<float*>(lds) + BM;
  constexpr int CPAD = BN + 8;
  elem_t* ctile = reinterpret_cast<elem_t*>(reinterpret_cast<float*>(lds) + BM + 2 * WM * BN);
  static_assert((BM + 2 * WM * BN) * 4 + BM * CPAD * 2 <= 2 * STAGE * 16, "epilogue LDS");
  for (int r = tid; r < BM; r += 256) {
    const int m = m0 + r;
    int off = -1;
    if (m < M) {
      if (p.plain) {
        off = m * p.ldc;
      } else {
        const uint32_t b = fdiv((uint32_t)m, ph->fd_hw);
        const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph->Hq * ph->Wq);
        const uint32_t qy = fdiv(rem, ph->fd_w);
        const uint32_t qx = rem - qy * (uint32_t)ph->Wq;
        const int y = (int)qy * p.ostride + ph->oy_off, x = (int)qx * p.ostride + ph->ox_off;
        off = (((int)b * p.outH + y) * p.outW + x) * p.ldc;
      }
    }
    rowoff[r] = off;
  }
  __syncthreads();

  const bool do_stats = p.stats != nullptr;
  // vector store path: elem_t output, whole 8-channel groups, aligned destination
  const bool vec = !p.out_f32 && (BN % 8 == 0) && (N % 8 == 0) && (p.ldc % 8 == 0) && (p.cofs % 8 == 0);
  frag_epilogue_dispatch<FM, FN, TM, TN, BN>(acc, p, rowoff, red, ctile, wm, wn, fr, fq, n0, do_stats, vec, m0);
  if (p.bnb_x) {  // BN-backward statistics fused into the store pass (epilogue.h)
    constexpr bool kFits = (BM + 2 * WM * BN) * 4 + BM * CPAD * 2 + 16384 <= 2 * STAGE * 16;
    if constexpr (kFits) {
      __syncthreads();
      float* red2 = reinterpret_cast<float*>(reinterpret_cast<char*>(ctile) + BM * CPAD * 2);
      vec_store_bnb<BM, BN>(p, rowoff, ctile, red2, n0, m0, p.stats + (size_t)(blockIdx.x * p.nphases + phase) * 2 * N);
    } else {
      __builtin_trap();  // the host only requests fused statistics on tiles with the LDS for them
    }
    return;
  }
  if (do_stats || vec) __syncthreads();
  if (vec) {
    constexpr int CPR = BN / 8;  // 16-byte chunks per row
    elem_t* C = reinterpret_cast<elem_t*>(p.C);
    for (int q = tid; q < BM * CPR; q += 256) {
      const int r = q / CPR, c = q - r * CPR;
      const int off = rowoff[r];
      const int n = n0 + 8 * c;
      if (off >= 0 && n < N)
        *reinterpret_cast<u32x4*>(C + off + p.cofs + n) = *reinterpret_cast<const u32x4*>(ctile + r * CPAD + 8 * c);
    }
  }
  if (do_stats) {
    for (int nl = tid; nl < BN; nl += 256) {
      const int n = n0 + nl;
      if (n >= N) continue;
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s += red[(w * BN + nl) * 2 + 0];
        s2 += red[(w * BN + nl) * 2 + 1];
      }
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.stats + (size_t)(blockIdx.x * p.nphases + phase) * 2 * N,
                                                  (uint32_t)(2 * N * 4));
      st_sc1_f32(rs, (uint32_t)n * 4u, s);  // write-through (read by the finalize kernel)
      st_sc1_f32(rs, (uint32_t)(N + n) * 4u, s2);
    }
  }
}

}  // namespace dcg

// ---------------------------------------------------------------------------- host launch
// Tile configurations (BM, BN, WM, WN); the engine picks one per layer. cfg + 100 selects the
// LDS-DMA staging variant of the same tile.
#define DCG_IGEMM_CONFIGS(X) \
  X(0, 128, 128, 2, 2) X(1, 128, 64, 2, 2) X(2, 64, 128, 2, 2) X(3, 64, 64, 2, 2) \
  X(4, 32, 64, 2, 2) X(5, 64, 32, 2, 2) X(6, 32, 32, 2, 2) X(7, 128, 16, 4, 1) \
  X(8, 64, 16, 4, 1) X(9, 256, 64, 4, 1)

extern "C" int DCG_API(dcg_igemm_tile)(int cfg, int* bm, int* bn) {
  const int c = cfg % 100;
#define X(id, BM_, BN_, WM_, WN_) if (c == id) { *bm = BM_; *bn = BN_; return 0; }
  DCG_IGEMM_CONFIGS(X)
#undef X
  return -1;
}

extern "C" int DCG_API(dcg_igemm_launch)(const dcg::IGemmArgs* a, int cfg, int mtiles, int ntiles, hipStream_t s) {
  dim3 grid(mtiles, ntiles, a->nphases);
  const int c = cfg % 100;
  const bool glds = cfg >= 100;
#define X(id, BM_, BN_, WM_, WN_)                                                                    \
  if (c == id) {                                                                                    \
    if (glds) hipLaunchKernelGGL((dcg::igemm_kernel<BM_, BN_, WM_, WN_, 1>), grid, dim3(256), 0, s, *a); \
    else hipLaunchKernelGGL((dcg::igemm_kernel<BM_, BN_, WM_, WN_, 0>), grid, dim3(256), 0, s, *a);      \
    return (int)hipGetLastError();                                                                  \
  }
  DCG_IGEMM_CONFIGS(X)
#undef X
  return -1;
}
