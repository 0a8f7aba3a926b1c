// dcg-variants: bf16 f16 f32
// Weight gradient, version 5: halo-row tiles for the stride-2 5x5 layers. Same problem and output
// as wgrad3.hip --
//
//   out[ky*5+kx][m][n] = scale * sum_{b,y,x} G[b, 2y+ky-pl, 2x+kx-pl, m] * Dm[b, y, x, n]
//
// (reference ops: the conv2d / conv2d_transpose weight gradients of
// /root/reference/distriubted_model.py:109-111,118, computed by TF's Conv2DBackpropFilter) -- but a
// workgroup owns one kernel ROW ky (all five kx taps) of one MC x BN channel block, and a
// k-tile is R = 64 / Wd whole output rows of one image. For those 64 pixels the five taps read the
// SAME R input rows 2y+ky-pl at columns 2x+kx-pl, so the A operand is staged once per k-tile as an
// R x (2 Wd + 4)-pixel window (every tap's pixels inside it, stride 2) instead of five 64-pixel
// gathers, and the Dm tile feeds five MFMA groups instead of one. Within a window row the even
// columns are stored first, then the odd ones: a tap's 16 fragment rows are then consecutive LDS
// rows (column stride 2 would put them all on one parity, half the banks). Per 16x16x32 MFMA that is ~3x
// fewer LDS-DMA bytes and ~40 % fewer LDS fragment reads than a one-tap wgrad3 tile of the same
// channels (round-4 review: the 64-channel wgrad3 tiles ran at 15 % of peak, bound by operand fill).
//
// Everything else is wgrad3's: LDS-DMA (buffer_load ... lds) with the 8-byte-chunk XOR swizzle
// applied on the source side, NS stages, one bare s_barrier per k-tile, counted vmcnt, fragments
// read with ds_read_b64_tr_b16, XCD-aware tile order, in-kernel split-K summed in split order by
// the last-arriving workgroup (bitwise deterministic).
#include "kernels.h"

#if defined(DCG_F32)
// the fp32 (reference-precision) engine keeps its weight gradients on igemm_f32.hip: stubs only
extern "C" int DCG_API(dcg_wgrad5_tile)(int, int*, int*, int*, int*) { return -1; }
extern "C" int DCG_API(dcg_wgrad5_launch)(const dcg::WGrad3Args*, int, hipStream_t) { return -2; }
#else

namespace dcg {

template <int S>
__device__ __forceinline__ int w5_swz(int r) {  // 8-byte-chunk XOR of k-major row r (stride S bytes)
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

// the window (A operand) swizzle. One ds_read_tr16_b64 half-wave reads the pixels q4 + 20 g4'
// (g4' = 0, 1) apart for WD = 8 (window rows of W2 = 20) and q4 + 8 g4' for WD = 16: the rows of
// one parity must take four distinct 8-byte-chunk groups of their 32-bank half. Bits 1 + 3 do
// that for the +8 spacing; for +20 (= 4 mod 8) bits 1 + 2 do (the rows are then four distinct
// residues mod 8 of one parity). Round 6: 64x8 tiles measured a 0.43 LDS bank-conflict ratio.
template <int S, int WD>
__device__ __forceinline__ int w5_swz_a(int r) {
  if constexpr (S == 128 && WD == 8) return 4 * (((r >> 1) & 1) | (((r >> 2) & 1) << 1));
  else return w5_swz<S>(r);
}

template <int N_>
__device__ __forceinline__ void w5_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

template <int L, int NMAX>
__device__ __forceinline__ void w5_wait_vmcnt_n(int n) {
  if constexpr (NMAX >= 2) { if (n >= 2) { w5_wait_vmcnt<2 * L>(); return; } }
  if constexpr (NMAX >= 1) { if (n >= 1) { w5_wait_vmcnt<L>(); return; } }
  w5_wait_vmcnt<0>();
}

template <int MC, int BN, int WD, int NS>
__global__ __launch_bounds__(256) void wgrad5_kernel(WGrad3Args p) {
  constexpr int BK = 64, R = BK / WD;                  // output rows per k-tile
  constexpr int W2 = 2 * WD + 4;                       // window columns: ix = c - pl
  constexpr int NPIX = (R * W2 + 31) / 32 * 32;        // window pixels, whole 1 KiB pieces per wave
  constexpr int SA = MC * 2, SB = BN * 2;              // k-major LDS row strides (bytes)
  constexpr int A_BYTES = NPIX * SA, B_BYTES = BK * SB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PPW_A = A_BYTES / 4096, PPW_B = B_BYTES / 4096;
  constexpr int LPT = PPW_A + PPW_B;
  constexpr int RPA = 1024 / SA, RPB = 1024 / SB, CA = SA / 16, CB = SB / 16;
  constexpr int TM = MC / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16;  // 2 x 2 waves
  static_assert(R * WD == BK, "whole output rows per k-tile");
  static_assert(A_BYTES % 4096 == 0 && B_BYTES % 4096 == 0, "every wave issues the same DMA count");
  static_assert(SA <= 1024 && SB <= 1024 && FM >= 1 && FN >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  lds_char* const lds3 = (lds_char*)lds;
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds3;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile decode: XCD remap, then (ky, n block) fastest and the k split slowest, so one XCD's
  //      run of workgroups shares its pixel range (its G rows and Dm tile) in that XCD's L2
  const int S = p.splits;
  const int ntn = (p.Nc + BN - 1) / BN, ntm = p.Mc / MC;  // MC = the tile's channel block (host: Mc % MC == 0)
  const int total = 5 * ntn * ntm * S;
  int t = blockIdx.x;
  {
    const int q = total >> 3, rr = total & 7, xcd = t & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  const int ky = t % 5;
  int r_ = t / 5;
  const int nt = r_ % ntn;
  r_ /= ntn;
  const int mt = r_ % ntm;
  const int split = r_ / ntm;
  const int tile_id = (mt * ntn + nt) * 5 + ky;
  const int n0 = nt * BN, m0 = mt * MC;

  const int KT = p.K / BK;                 // host: whole output rows per k-tile, K a multiple of 64
  const int kt0 = split * p.kt_per_split;
  const int nk = max(0, min(KT, kt0 + p.kt_per_split) - kt0);

  const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.G, p.g_bytes);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(p.Dm, p.d_bytes);

  // per-lane fixed parts of the DMA addresses
  int a_ry[PPW_A], a_ix[PPW_A], a_m[PPW_A];
  bool a_ok[PPW_A];
#pragma unroll
  for (int i = 0; i < PPW_A; ++i) {
    const int wp = (wave + 4 * i) * RPA + lane / CA;  // window pixel (LDS row) this lane's chunk lands in
    const int ry = wp / W2, jj = wp - ry * W2;
    const int c = jj < W2 / 2 ? 2 * jj : 2 * (jj - W2 / 2) + 1;  // its column: even ones first, then odd
    a_ry[i] = ry;
    a_ix[i] = c - p.pl;
    a_m[i] = m0 + ((lane % CA) ^ (w5_swz_a<SA, WD>(wp) >> 1)) * 8;
    a_ok[i] = ry < R && c < 2 * WD + 3 && (unsigned)(c - p.pl) < (unsigned)p.Wg;
  }
  int b_row[PPW_B], b_n[PPW_B];
#pragma unroll
  for (int i = 0; i < PPW_B; ++i) {
    const int rr = (wave + 4 * i) * RPB + lane / CB;
    b_row[i] = rr;
    b_n[i] = n0 + ((lane % CB) ^ (w5_swz<SB>(rr) >> 1)) * 8;
  }

  int cur_kt = kt0;
  auto issue = [&](int slot) {
    const uint32_t sa = lds_base + slot * STAGE;
    const uint32_t sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < PPW_A; ++i) {
      // output row gy of the whole batch (a k-tile may span several small images: Hd < R)
      const uint32_t gy = (uint32_t)(cur_kt * R + a_ry[i]);
      const int b = (int)fdiv(gy * (uint32_t)WD, p.fd_hw), y = (int)gy - b * p.Hd;
      const int iy = 2 * y + ky - p.pl;
      const bool ok = a_ok[i] && (unsigned)iy < (unsigned)p.Hg;
      dma16_asm_la(rg, sa + (wave + 4 * i) * 1024,
                   oob_unless(ok, (uint32_t)(((b * p.Hg + iy) * p.Wg + a_ix[i]) * p.Mc + a_m[i]) * 2u));
    }
#pragma unroll
    for (int i = 0; i < PPW_B; ++i) {
      const int k = cur_kt * BK + b_row[i];
      dma16_asm_la(rd, sb + (wave + 4 * i) * 1024, oob_unless(b_n[i] < p.Nc, (uint32_t)(k * p.Nc + b_n[i]) * 2u));
    }
    ++cur_kt;
  };

  f32x4 acc[5][FM][FN];
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[x][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);

  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  for (int kt = 0; kt < nk; ++kt) {
    w5_wait_vmcnt_n<LPT, NS - 2>(min(NS - 2, nk - 1 - kt));
    asm volatile("s_barrier" ::: "memory");
    if (kt + NS - 1 < nk) issue((kt + NS - 1) % NS);
    const lds_char* sa = lds3 + (kt % NS) * STAGE;
    const lds_char* sb = sa + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      elem8 bfr[FN], af[5][FM];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = ks * 32 + 8 * g4 + 4 * h + q4;  // pixel of the k-tile
        const int wr0 = (r / WD) * W2 + (r % WD);      // its window row for kx = 0 (even columns)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c8 = (wn * TN + j * 16) / 4 + p4;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, sb + r * SB + ((c8 ^ w5_swz<SB>(r)) * 8)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[j][4 * h + e] = vb[e];
        }
#pragma unroll
        for (int x = 0; x < 5; ++x) {
          // column 2 (r % WD) + x: even columns are window rows [0, W2/2), odd ones [W2/2, W2)
          const int wr = wr0 + ((x & 1) ? W2 / 2 + (x >> 1) : (x >> 1));
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const int c8 = (wm * TM + i * 16) / 4 + p4;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                LDS_PTR(s16x4, sa + wr * SA + ((c8 ^ w5_swz_a<SA, WD>(wr)) * 8)));
            const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) af[x][i][4 * h + e] = vb[e];
          }
        }
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int x = 0; x < 5; ++x)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[x][i][j] = DCG_MFMA_16x16x32(af[x][i], bfr[j], acc[x][i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // ---- split-K hand-off (as wgrad3.hip): sc1 slab stores, drain, agent-scope counter; the last
  //      arrival sums the S slabs in split order and re-arms the counter
  constexpr int NF = 5 * FM * FN;
  if (S > 1 && p.counters == nullptr) {
    // separate reduction (cfg 41x): store this split's slab (accumulator-register order, one 4 KiB
    // block per fragment) and leave the sum to wgrad5_reduce_kernel, which spreads it over the GPU
    float* wsl = p.ws + ((size_t)tile_id * S + split) * (5 * MC * BN);
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          *reinterpret_cast<f32x4*>(wsl + (size_t)(((x * FM + i) * FN + j) * 256 + tid) * 4) = acc[x][i][j];
    return;
  }
  if (S > 1) {
    int& last_flag = *reinterpret_cast<int*>(lds);
    const __amdgpu_buffer_rsrc_t rw =
        make_rsrc(p.ws + (size_t)tile_id * S * (5 * MC * BN), (uint32_t)(S * 5 * MC * BN * 4));
    const uint32_t own = (uint32_t)split * (5 * MC * BN * 4);
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[x][i][j]), rw,
                                                 own + (uint32_t)((((x * FM + i) * FN + j) * 256 + tid) * 16), 0, 16);
    w5_wait_vmcnt<0>();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = (old == (unsigned)(S - 1));
      if (last_flag) __hip_atomic_store(p.counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_flag) return;
    for (int x = 0; x < 5; ++x) {  // one tap at a time: FM x FN running sums in registers
      f32x4 tot[FM][FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) tot[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      constexpr int U = 4;  // four slabs' loads in flight per round trip, summed in split order
      for (int s0 = 0; s0 < S; s0 += U) {
        f32x4 v[U][FM][FN];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int s = s0 + u;
          const uint32_t base = (uint32_t)s * (5 * MC * BN * 4);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              v[u][i][j] = (s < S && s != split)
                               ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                     rw, base + (uint32_t)((((x * FM + i) * FN + j) * 256 + tid) * 16), 0, 16))
                               : acc[x][i][j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (s0 + u < S) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
              for (int j = 0; j < FN; ++j) tot[i][j] += v[u][i][j];
          }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[x][i][j] = tot[i][j];
    }
  }
  (void)NF;

  // ---- scaled store into the fp32 gradient, TF layout [tap][Mc][Nc]
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + j * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + i * 16 + g4 * 4 + r;
          if (n < p.Nc) p.out[((size_t)(ky * 5 + x) * p.Mc + m) * p.Nc + n] = acc[x][i][j][r] * p.scale;
        }
      }
}

// the split sum of the separate-reduction variant: one thread per f32x4 of one tile's slab (the same
// thread -> (m, n) map as the producing kernel), splits added in order (8 loads in flight)
template <int MC, int BN>
__global__ __launch_bounds__(256) void wgrad5_reduce_kernel(const float* __restrict__ ws, int S, int Mc, int Nc,
                                                            float scale, float* __restrict__ out) {
  constexpr int TM = MC / 2, TN = BN / 2, FM = TM / 16, FN = TN / 16, NF = 5 * FM * FN;
  const int tile_id = blockIdx.x / NF, f = blockIdx.x - tile_id * NF, tid = threadIdx.x;
  const int x = f / (FM * FN), i = (f / FN) % FM, j = f % FN;
  const int ntn = (Nc + BN - 1) / BN, ky = tile_id % 5, nt = (tile_id / 5) % ntn, mt = tile_id / 5 / ntn;
  const int n0 = nt * BN, m0 = mt * MC;
  const int lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1, g4 = lane >> 4, li = lane & 15;
  const float* src = ws + (size_t)tile_id * S * (5 * MC * BN) + (size_t)(f * 256 + tid) * 4;
  f32x4 tot = (f32x4){0.f, 0.f, 0.f, 0.f};
  constexpr int U = 8;
  for (int s0 = 0; s0 < S; s0 += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = s0 + u < S ? *reinterpret_cast<const f32x4*>(src + (size_t)(s0 + u) * (5 * MC * BN)) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s0 + u < S) tot += v[u];
  }
  const int n = n0 + wn * TN + j * 16 + li;
  if (n < Nc) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * TM + i * 16 + g4 * 4 + r;
      out[((size_t)(ky * 5 + x) * Mc + m) * Nc + n] = tot[r] * scale;
    }
  }
}

}  // namespace dcg

// cfg 400 + id: (MC channel block, BN, Wd, NS); 410 + id: the same with the split sum in a second,
// GPU-wide kernel
#define DCG_WGRAD5_CFGS(X) \
  X(0, 64, 64, 16, 2) X(1, 64, 64, 16, 3) X(2, 64, 64, 8, 2) X(3, 64, 64, 32, 2) X(4, 128, 64, 8, 2) \
  X(5, 128, 64, 16, 2) X(6, 128, 32, 8, 2) X(7, 128, 32, 16, 2) X(8, 64, 64, 64, 2) X(9, 64, 64, 4, 2)

extern "C" int DCG_API(dcg_wgrad5_tile)(int cfg, int* mc, int* bn, int* wd, int* ns) {
  if (cfg < 400 || cfg >= 420) return -1;
  const int id = cfg % 10;
#define X(id_, MC_, BN_, WD_, NS_) if (id == id_) { *mc = MC_; *bn = BN_; *wd = WD_; *ns = NS_; return 0; }
  DCG_WGRAD5_CFGS(X)
#undef X
  return -1;
}

template <int MC, int BN, int WD, int NS>
static int w5launch(const dcg::WGrad3Args* a, unsigned blocks, hipStream_t s) {
  constexpr int R = 64 / WD, W2 = 2 * WD + 4, NPIX = (R * W2 + 31) / 32 * 32;
  constexpr size_t shm = (size_t)NS * ((size_t)NPIX * MC * 2 + (size_t)64 * BN * 2);
  auto k = dcg::wgrad5_kernel<MC, BN, WD, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), shm, s, *a);
  return (int)hipGetLastError();
}

template <int MC, int BN>
static int w5reduce(const dcg::WGrad3Args* a, unsigned tiles, hipStream_t s) {
  constexpr int NF = 5 * (MC / 32) * (BN / 32);  // f32x4 blocks of 256 threads per tile
  auto k = dcg::wgrad5_reduce_kernel<MC, BN>;
  hipLaunchKernelGGL(k, dim3(tiles * NF), dim3(256), 0, s, a->ws, a->splits, a->Mc, a->Nc, a->scale, a->out);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_wgrad5_launch)(const dcg::WGrad3Args* a, int cfg, hipStream_t s) {
  int mc, bn, wd, ns;
  if (DCG_API(dcg_wgrad5_tile)(cfg, &mc, &bn, &wd, &ns)) return -1;
  // shapes the kernel assumes (the host binding checks them too)
  const int R = 64 / wd;  // output rows per k-tile: whole images or whole-image fractions, K in whole tiles
  if (a->Mc % mc || a->Wd != wd || (a->Hd % R && R % a->Hd) || a->K % 64) return -2;
  const unsigned tiles = 5u * (unsigned)((a->Nc + bn - 1) / bn) * (unsigned)(a->Mc / mc);
  const unsigned blocks = tiles * (unsigned)a->splits;
  const bool sep = cfg >= 410 && a->splits > 1;  // (the binding allocates no counters for 41x)
  if ((cfg >= 410) != (a->counters == nullptr) && a->splits > 1) return -3;
  const int id = cfg % 10;
#define X(id_, MC_, BN_, WD_, NS_)                                 \
  if (id == id_) {                                                 \
    const int e = w5launch<MC_, BN_, WD_, NS_>(a, blocks, s);      \
    return (e || !sep) ? e : w5reduce<MC_, BN_>(a, tiles, s);      \
  }
  DCG_WGRAD5_CFGS(X)
#undef X
  return -1;
}

#endif  // DCG_F32
