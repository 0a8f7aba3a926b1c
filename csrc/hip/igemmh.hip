// dcg-variants: bf16 f16
// Implicit-GEMM convolution, "halo" version: the whole input window of a tile stays in LDS.
//
// igemm3.hip streams BOTH operands through its LDS ring: for every (tap, 64-channel chunk)
// k-tile it gathers BM input rows (the A tile) and BN weight rows (the B tile) with LDS-DMA.
// A tile of BM output pixels, though, only ever reads a small window of the input -- its rows
// plus a halo of (kernel - 1) rows / columns -- and the 9 / 6 / 4 (deconv phases) or 25
// (stride-2 conv) taps re-read that window over and over. Measured on igemm3 (profiles/r2/
// igemm3_ablations_r2.txt): the K loop is bound by the ISSUE of the 1 KiB LDS-DMA pieces
// (~100 cycles each next to the fragment reads), not by HBM or the MFMAs.
//
// Here each workgroup loads its input window ONCE (all Kc channels, pixel-major, in the
// prologue), then its K loop streams only the B tiles through an NS-stage LDS-DMA ring exactly
// like igemm3 (a constant DMA count per step, so a counted `s_waitcnt vmcnt` + raw s_barrier
// keeps NS-2 younger B tiles in flight). A fragments are read straight out of the window: the
// tap is a uniform pixel offset (host-computed), so the per-step A address is one add + the slot
// swizzle. Per k-step the DMA pieces per wave drop from (BM + BN) / 32 to BN / 32.
//
// Tiles are contiguous runs of BM rows of one phase, where a row is an output pixel (b, qy, qx)
// of that phase's grid: BM is a multiple of the grid width (a band of whole rows of one image)
// or of the whole grid (whole images). So the row -> (rowoff, stats slot) bookkeeping and the
// fused epilogue (epilogue.h) are igemm3's unchanged. No split-K: the layers this kernel serves
// have M >= 8K rows per phase.
//
// Window image in LDS (Kc = 64 -> 128-byte pixels, Kc >= 128 -> pixel pitch multiple of 256 B):
// the 16-byte slot j of window pixel P lives at
//   Kc = 64 : pixel slot P ^ ((P >> 4) & 1), slot j ^ ((P >> 1) & 7)
//   Kc >= 128: pixel slot P,                  slot j ^ ((P >> (sstride - 1)) & 15)
// so the 16 lanes of a fragment read (16 output pixels of a row, stride 1 or 2 apart in the
// window, one 16-byte k slot) hit 16 different bank groups. The LDS-DMA writes lane-linear 1 KiB
// pieces, so the swizzle is applied on the SOURCE side (an involution: same formula both ways).
#include "epilogue.h"

namespace dcg {

namespace {

template <int S>
__device__ __forceinline__ int knh_swz(int r) {  // as igemm3's kn_swz (k-major B rows of S bytes)
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// byte offset of 16-byte slot j of window pixel P (see the header)
__device__ __forceinline__ uint32_t win_off(int P, int j, int kc8, int sh) {
  if (kc8 == 8) return (uint32_t)(((P ^ ((P >> 4) & 1)) << 7) + ((j ^ ((P >> 1) & 7)) << 4));
  return (uint32_t)((P * kc8 + (j ^ ((P >> sh) & 15))) << 4);
}

}  // namespace

template <int BM, int BN, int WM, int WN, int BKN, int NS>
__global__ __launch_bounds__(256) void igemmh_kernel(IGemmArgs p) {
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int NPB = B_BYTES / 1024;
  constexpr int PPW_B = NPB / 4;  // B pieces per wave per k-step
  constexpr int SB = BN * 2;      // k-major B row stride (bytes)
  constexpr int B_ROWS_PER_PIECE = BKN ? 1024 / SB : 8;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(NPB % 4 == 0, "every wave issues the same B DMA count");
  static_assert(FM >= 1 && FN >= 1, "tile");
  static_assert(!BKN || (SB <= 1024 && 1024 % SB == 0), "k-major B rows");
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // ---- tile decode (XCD-aware bijective remap as igemm3): t -> (phase, nt, mt), phase fastest
  const int ntn = (p.N + BN - 1) / BN;
  const int total = p.mtiles * ntn * p.nphases;
  int t = blockIdx.x;
  {
    const int q = total >> 3, rr = total & 7, xcd = t & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  const int phase = t % p.nphases;
  int r_ = t / p.nphases;
  const int nt = r_ % ntn;
  const int mt = r_ / ntn;

  const IGemmPhaseK& ph = p.phk[phase];
  const int M = ph.M;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= M) {
    if (p.stats) {
      float* dst = p.stats + (size_t)(mt * p.nphases + phase) * 2 * p.N;
      for (int nl = tid; nl < BN; nl += 256)
        if (n0 + nl < p.N) { dst[n0 + nl] = 0.f; dst[p.N + n0 + nl] = 0.f; }
    }
    return;
  }
  const int Kc = p.Kc, N = p.N;
  const int kc8 = Kc >> 3;                     // 16-byte slots per pixel (power of two >= 8)
  const int lkc8 = 31 - __builtin_clz(kc8);
  const int sh = p.sstride - 1;
  const int nch = Kc >> 6;                     // 64-channel chunks per tap
  const int KT = ph.ntaps * nch;
  const int HW = ph.Hq * ph.Wq;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, (p.ablate & 1) ? 0u : p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.Bw, (p.ablate & 2) ? 0u : p.b_bytes);

  // ---- tile origin: first image b0 and first grid row y0 (tiles never straddle a band)
  const int b0 = (int)fdiv((uint32_t)m0, ph.fd_hw);
  const int y0 = (int)fdiv((uint32_t)(m0 - b0 * HW), ph.fd_w);
  const int WW = ph.win_w, WHW = ph.win_h * ph.win_w;
  char* win = lds;
  char* ring = lds + p.h_wbytes;

  // ---- window: h_tb x win_h x win_w pixels x kc8 slots, 64 slots (1 KiB) per DMA piece, pieces round-robin
  //      over the waves (issued first: the first B wait of the K loop covers them)
  if (!(p.ablate & 8)) {
    const int nslots = (p.h_tb * WHW) << lkc8;
    const int npieces = (nslots + 63) >> 6;
    const int oy = y0 * p.sstride + ph.win_oy, ox = ph.win_ox;
    for (int q = wave; q < npieces; q += 4) {
      const int s = (q << 6) + lane;  // LDS slot
      uint32_t off = OOB;
      if (s < nslots) {
        // invert win_off: LDS slot -> (P, j)
        int P, j;
        if (kc8 == 8) {
          const int Ps = s >> 3;
          P = Ps ^ ((Ps >> 4) & 1);
          j = (s & 7) ^ ((P >> 1) & 7);
        } else {
          P = s >> lkc8;
          j = (s & (kc8 - 1)) ^ ((P >> sh) & 15);
        }
        const int bl = (int)fdiv((uint32_t)P, ph.fd_whw);
        const int rem = P - bl * WHW;
        const int wy = (int)fdiv((uint32_t)rem, ph.fd_ww);
        const int wx = rem - wy * WW;
        const int b = b0 + bl, iy = oy + wy, ix = ox + wx;
        if (b < p.Bn && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W)
          off = (uint32_t)((((b * p.H + iy) * p.W + ix) * Kc + j * 8) * 2);
      }
      dma16_asm(ra, win + (q << 10), off);
    }
  }

  // ---- B ring: step s = (tap ti, chunk c) in tap-major order
  const int a_chunk = (lane & 7) ^ (lane >> 3);
  int cur_ti = 0, cur_c0 = 0;
  auto issue_b = [&](int slot) {
    char* sb = ring + slot * B_BYTES;
    const int wt = ph.tap[cur_ti] >> 16;  // scalar (kernarg)
#pragma unroll
    for (int i = 0; i < PPW_B; ++i) {
      const int q = wave + 4 * i;
      uint32_t off = OOB;
      if constexpr (BKN) {
        const int rr = q * B_ROWS_PER_PIECE + lane / (SB / 16);
        const int k = cur_c0 + rr;
        const int n = n0 + ((lane % (SB / 16)) ^ (knh_swz<SB>(rr) >> 1)) * 8;
        if (n < N) off = (uint32_t)((wt * Kc + k) * N + n) * 2u;
      } else {
        const int n = n0 + 8 * q + (lane >> 3);
        const int c = cur_c0 + a_chunk * 8;
        if (n < N) off = (uint32_t)((wt * N + n) * Kc + c) * 2u;
      }
      dma16_asm(rb, sb + q * 1024, off);
    }
    cur_c0 += BK;
    if (cur_c0 >= Kc) { cur_c0 = 0; ++cur_ti; }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KT && !(p.ablate & 8)) issue_b(s);

  const int fr = lane & 15, fq = lane >> 4;
  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;

  // window pixel of each A fragment row of this lane at tap offset 0
  int pb[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = min(m0 + wm * TM + i * 16 + fr, M - 1);  // rows past M: any in-window pixel
    const int b = (int)fdiv((uint32_t)m, ph.fd_hw);
    const int rem = m - b * HW;
    const int qy = (int)fdiv((uint32_t)rem, ph.fd_w);
    const int qx = rem - qy * ph.Wq;
    pb[i] = (b - b0) * WHW + (qy - y0) * p.sstride * WW + qx * p.sstride;
  }

  int con_ti = 0, con_ch = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if constexpr (NS >= 3) {
      if (kt + 1 < KT) wait_vm<PPW_B * (NS - 2)>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_barrier" ::: "memory");
    if (kt + NS - 1 < KT && !(p.ablate & 8)) issue_b((kt + NS - 1) % NS);
    const int T = ph.tap[con_ti] & 0xffff;
    const int jb = con_ch * 8 + fq;
    if (++con_ch == nch) { con_ch = 0; ++con_ti; }
    if (p.ablate & 4) continue;
    const char* sb = ring + (kt % NS) * B_BYTES;
    elem8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const uint32_t o = win_off(pb[i] + T, jb, kc8, sh);
      af[0][i] = *reinterpret_cast<const elem8*>(win + o);
      af[1][i] = *reinterpret_cast<const elem8*>(win + (o ^ 64u));  // slot j + 4 (bit 2 of j is 0)
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      if constexpr (BKN) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = ks * 32 + 8 * g4 + 4 * h + q4;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int c8 = (wn * TN + j * 16) / 4 + p4;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                LDS_PTR(s16x4, sb + r * SB + ((c8 ^ knh_swz<SB>(r)) * 8)));
            const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) bfr[ks][j][4 * h + e] = vb[e];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wn * TN + j * 16 + fr;
          bfr[ks][j] = *reinterpret_cast<const elem8*>(sb + r * 128 + ((c ^ (r & 7)) << 4));
        }
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = DCG_MFMA_16x16x32(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  if (KT == 0) wait_vm<0>();

  // ------------------------------------------------------------------ epilogue (as igemm3)
  __syncthreads();
  int* rowoff = reinterpret_cast<int*>(lds);
  float* red = reinterpret_cast<float*>(lds) + BM;
  constexpr int CPAD = BN + 8;
  elem_t* ctile = reinterpret_cast<elem_t*>(reinterpret_cast<float*>(lds) + BM + 2 * WM * BN);
  for (int r = tid; r < BM; r += 256) {
    const int m = m0 + r;
    int off = -1;
    if (m < M) {
      const uint32_t b = fdiv((uint32_t)m, ph.fd_hw);
      const uint32_t rem = (uint32_t)m - b * (uint32_t)HW;
      const uint32_t qy = fdiv(rem, ph.fd_w);
      const uint32_t qx = rem - qy * (uint32_t)ph.Wq;
      const int y = (int)qy * p.ostride + ph.oy_off, x = (int)qx * p.ostride + ph.ox_off;
      off = (((int)b * p.outH + y) * p.outW + x) * p.ldc;
    }
    rowoff[r] = off;
  }
  __syncthreads();

  const bool do_stats = p.stats != nullptr;
  const bool vec = !p.out_f32 && (N % 8 == 0) && (p.ldc % 8 == 0) && (p.cofs % 8 == 0);
  frag_epilogue_dispatch<FM, FN, TM, TN, BN>(acc, p, rowoff, red, ctile, wm, wn, fr, fq, n0, do_stats, vec, m0);
  if (p.bnb_x) {  // the host checked that the dynamic LDS holds the fused-statistics scratch
    __syncthreads();
    float* red2 = reinterpret_cast<float*>(reinterpret_cast<char*>(ctile) + BM * CPAD * 2);
    vec_store_bnb<BM, BN>(p, rowoff, ctile, red2, n0, m0, p.stats + (size_t)(mt * p.nphases + phase) * 2 * N);
    return;
  }
  if (do_stats || vec) __syncthreads();
  if (vec) {
    constexpr int CPR = BN / 8;
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
      float* dst = p.stats + (size_t)(mt * p.nphases + phase) * 2 * N;
      dst[n] = s;
      dst[N + n] = s2;
    }
  }
}

}  // namespace dcg

// ---------------------------------------------------------------------------- host launch
// halo configs: cfg = 400 + 10 * k + id, B ring stages NS = {3, 2, 4}[k]. The dynamic LDS
// (window + ring, at least the epilogue scratch) is computed per op by the host.
#define DCG_IGEMMH_TILES(X) \
  X(0, 128, 128, 2, 2) X(1, 128, 64, 2, 2) X(2, 256, 64, 4, 1) X(3, 64, 128, 2, 2) X(4, 64, 64, 2, 2)

static constexpr int kIgemmhStages[3] = {3, 2, 4};

extern "C" int DCG_API(dcg_igemmh_tile)(int cfg, int* bm, int* bn, int* ns) {
  if (cfg < 400 || cfg >= 430) return -1;
  const int id = cfg % 10;
  *ns = kIgemmhStages[(cfg - 400) / 10];
#define X(id_, BM_, BN_, WM_, WN_) \
  if (id == id_) { *bm = BM_; *bn = BN_; return 0; }
  DCG_IGEMMH_TILES(X)
#undef X
  return -1;
}

template <int BM, int BN, int WM, int WN, int BKN, int NS>
static int launchh(const dcg::IGemmArgs* a, unsigned blocks, size_t shm, hipStream_t s) {
  auto k = dcg::igemmh_kernel<BM, BN, WM, WN, BKN, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), shm, s, *a);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_igemmh_launch)(const dcg::IGemmArgs* a, int cfg, int bkn, unsigned blocks, size_t shm,
                                          hipStream_t s) {
  int bm, bn, ns;
  if (DCG_API(dcg_igemmh_tile)(cfg, &bm, &bn, &ns) || shm > 160 * 1024) return -1;
  const int id = cfg % 10;
#define X(id_, BM_, BN_, WM_, WN_)                                                             \
  if (id == id_) {                                                                             \
    if (ns == 3) return bkn ? launchh<BM_, BN_, WM_, WN_, 1, 3>(a, blocks, shm, s)             \
                            : launchh<BM_, BN_, WM_, WN_, 0, 3>(a, blocks, shm, s);            \
    if (ns == 4) return bkn ? launchh<BM_, BN_, WM_, WN_, 1, 4>(a, blocks, shm, s)             \
                            : launchh<BM_, BN_, WM_, WN_, 0, 4>(a, blocks, shm, s);            \
    return bkn ? launchh<BM_, BN_, WM_, WN_, 1, 2>(a, blocks, shm, s)                          \
               : launchh<BM_, BN_, WM_, WN_, 0, 2>(a, blocks, shm, s);                         \
  }
  DCG_IGEMMH_TILES(X)
#undef X
  return -1;
}
