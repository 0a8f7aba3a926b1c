// dcg-variants: bf16 f16
// Weight gradient, version 3: the igemm3.hip recipe (LDS-DMA multi-stage pipeline, 64x64 wave
// tiles, XCD-aware tile order, in-kernel deterministic split-K) applied to wgrad.hip's problem.
//
//   out[tap][m][n] = scale * sum_k G[b, 2y+ky-pl, 2x+kx-pl, m] * Dm[b, y, x, n],  k = (b, y, x)
//
// (conv: G = layer input, Dm = dL/d(conv out) -> HWIO dW; deconv: G = dL/d(deconv out), Dm = layer
// input -> [kh,kw,co,ci] dW -- the TF layouts, no transposes). Per tap it is an Mc x Nc GEMM over
// K = B*Hd*Wd pixels, and BOTH operands are k-major (channels contiguous per pixel): both LDS
// tiles are k-major rows of BM / BN channels, written by 16-byte LDS-DMA whose lane -> chunk map
// realises the 8-byte-chunk XOR swizzle, and every MFMA fragment is read with the gfx950
// transposing read ds_read_b64_tr_b16 (as igemm3's BKN path and wgrad.hip).
//
// Differences from wgrad.hip (register-staged double buffer, slabs + a separate reduce kernel):
//   * global -> LDS by DMA, NS stages in flight, one bare s_barrier per k-tile;
//   * split-K partials are summed in-kernel by the last-arriving workgroup of each output tile
//     in split order (bitwise deterministic) and written scaled into the fp32 gradient directly;
//   * tile order: tap fastest, then n, m and split slowest, so each XCD's contiguous run of
//     workgroups covers all 25 taps of ONE pixel range -- the 25 shifted reads of G and the 25
//     reads of Dm then hit that XCD's L2.
#include "kernels.h"

namespace dcg {

template <int S>
__device__ __forceinline__ int w3_swz(int r) {  // 8-byte-chunk XOR of k-major row r (stride S bytes)
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

template <int N_>
__device__ __forceinline__ void w3_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// vmcnt(n * L) for a runtime n in [0, NMAX]
template <int L, int NMAX>
__device__ __forceinline__ void w3_wait_vmcnt_n(int n) {
  if constexpr (NMAX >= 2) { if (n >= 2) { w3_wait_vmcnt<2 * L>(); return; } }
  if constexpr (NMAX >= 1) { if (n >= 1) { w3_wait_vmcnt<L>(); return; } }
  w3_wait_vmcnt<0>();
}

// TT taps per tile (1 or 2): with TT = 2 the tile's BM rows are [tap 2 tg: Mc channels][tap 2 tg + 1:
// Mc channels] (BM = 2 Mc): both taps share the B (Dm) tile -- half the DMA per MFMA of the 64-row
// single-tap tile for the 64-channel layers (tap 25 of group 12 reads zeros and is not stored).
template <int BM, int BN, int WM, int WN, int NS, int P2, int TT>
__global__ __launch_bounds__(256) void wgrad3_kernel(WGrad3Args p) {
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int SA = BM * 2, SB = BN * 2;             // k-major LDS row strides (bytes)
  constexpr int A_BYTES = BK * SA, B_BYTES = BK * SB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PPW_A = A_BYTES / 4096, PPW_B = B_BYTES / 4096;  // 1 KiB DMA pieces per wave
  constexpr int LPT = PPW_A + PPW_B;                  // DMA instructions per lane per k-tile
  constexpr int RPA = 1024 / SA, RPB = 1024 / SB;     // k rows per piece
  constexpr int CA = SA / 16, CB = SB / 16;           // 16-byte chunks per row
  static_assert(WM * WN == 4, "4 waves");
  static_assert(A_BYTES % 4096 == 0 && B_BYTES % 4096 == 0, "every wave issues the same DMA count");
  static_assert(SA <= 1024 && SB <= 1024 && FM >= 1 && FN >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  lds_char* const lds3 = (lds_char*)lds;  // 32-bit LDS addressing
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds3;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // ---- tile decode: XCD remap (each XCD gets a contiguous run of t), then tap fastest
  const int S = p.splits;
  constexpr int NTG = (25 + TT - 1) / TT;             // tap groups
  const int ntm = TT == 1 ? (p.Mc + BM - 1) / BM : 1, ntn = (p.Nc + BN - 1) / BN;
  const int total = ntm * ntn * NTG * S;
  int t = blockIdx.x;
  {
    const int q = total >> 3, rr = total & 7, xcd = t & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  const int tap = t % NTG;  // TT = 2: the tap group
  int r_ = t / NTG;
  const int nt = r_ % ntn;
  r_ /= ntn;
  const int mt = r_ % ntm;
  const int split = r_ / ntm;
  const int tile_id = (tap * ntm + mt) * ntn + nt;
  const int m0 = mt * BM, n0 = nt * BN;
  constexpr int MCT = BM / TT;  // channels per tap in the tile (TT = 2: = Mc)

  const int KT = (p.K + BK - 1) / BK;
  const int kt0 = split * p.kt_per_split;
  const int nk = max(0, min(KT, kt0 + p.kt_per_split) - kt0);

  const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.G, p.g_bytes);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(p.Dm, p.d_bytes);

  // per-lane fixed parts of the DMA addresses: row within the tile and the swizzled chunk
  int a_row[PPW_A], a_m[PPW_A], a_ky[PPW_A], a_kx[PPW_A], b_row[PPW_B], b_n[PPW_B];
  bool a_tok[PPW_A];
#pragma unroll
  for (int i = 0; i < PPW_A; ++i) {
    const int rr = (wave + 4 * i) * RPA + lane / CA;
    a_row[i] = rr;
    const int ml = ((lane % CA) ^ (w3_swz<SA>(rr) >> 1)) * 8;  // row of the tile this lane's chunk feeds
    const int tp = TT == 1 ? tap : TT * tap + ml / MCT;          // its tap
    a_m[i] = TT == 1 ? m0 + ml : ml % MCT;                       // its channel
    a_tok[i] = tp < 25;
    a_ky[i] = tp / 5;
    a_kx[i] = tp - 5 * (tp / 5);
  }
#pragma unroll
  for (int i = 0; i < PPW_B; ++i) {
    const int rr = (wave + 4 * i) * RPB + lane / CB;
    b_row[i] = rr;
    b_n[i] = n0 + ((lane % CB) ^ (w3_swz<SB>(rr) >> 1)) * 8;
  }

  int cur_k0 = kt0 * BK;  // first pixel of the next tile to issue
  auto issue = [&](int slot) {
    const uint32_t sa = lds_base + slot * STAGE;
    const uint32_t sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < PPW_A; ++i) {  // branch-free: invalid lanes get an out-of-range offset
      const int k = cur_k0 + a_row[i];
      uint32_t b, y, x;
      if constexpr (P2) {  // power-of-two images: shifts and masks (every DCGAN resolution but 28)
        b = (uint32_t)k >> p.lhw;
        const uint32_t rem = (uint32_t)k & ((1u << p.lhw) - 1u);
        y = rem >> p.lw;
        x = rem & ((1u << p.lw) - 1u);
      } else {
        b = fdiv((uint32_t)k, p.fd_hw);
        const uint32_t rem = (uint32_t)k - b * (uint32_t)(p.Hd * p.Wd);
        y = fdiv(rem, p.fd_w);
        x = rem - y * (uint32_t)p.Wd;
      }
      const int iy = 2 * (int)y + a_ky[i] - p.pl, ix = 2 * (int)x + a_kx[i] - p.pl;
      const bool ok = k < p.K && a_tok[i] && a_m[i] < p.Mc && (unsigned)iy < (unsigned)p.Hg &&
                      (unsigned)ix < (unsigned)p.Wg;
      dma16_asm_la(rg, sa + (wave + 4 * i) * 1024,
                   oob_unless(ok, (uint32_t)((((int)b * p.Hg + iy) * p.Wg + ix) * p.Mc + a_m[i]) * 2u));
    }
#pragma unroll
    for (int i = 0; i < PPW_B; ++i) {
      const int k = cur_k0 + b_row[i];
      dma16_asm_la(rd, sb + (wave + 4 * i) * 1024,
                   oob_unless(k < p.K && b_n[i] < p.Nc, (uint32_t)(k * p.Nc + b_n[i]) * 2u));
    }
    cur_k0 += BK;
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);

  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed; the younger tiles issued so far (at most NS - 2, fewer at the loop's end) may
    // stay in flight
    w3_wait_vmcnt_n<LPT, NS - 2>(min(NS - 2, nk - 1 - kt));
    // all waves' DMA of tile kt landed; all waves are done reading slot (kt-1) % NS
    asm volatile("s_barrier" ::: "memory");
    if (kt + NS - 1 < nk) issue((kt + NS - 1) % NS);
    const lds_char* sa = lds3 + (kt % NS) * STAGE;
    const lds_char* sb = sa + A_BYTES;
    elem8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = ks * 32 + 8 * g4 + 4 * h + q4;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int c8 = (wm * TM + i * 16) / 4 + p4;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, sa + r * SA + ((c8 ^ w3_swz<SA>(r)) * 8)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[ks][i][4 * h + e] = vb[e];
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c8 = (wn * TN + j * 16) / 4 + p4;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, sb + r * SB + ((c8 ^ w3_swz<SB>(r)) * 8)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[ks][j][4 * h + e] = vb[e];
        }
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = DCG_MFMA_16x16x32(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }

  // ---- split-K hand-off (as igemm3.hip): sc1 slab stores, drain, agent-scope counter; the last
  //      arrival sums the S slabs in split order with sc1 loads and re-arms the counter
  if (S > 1) {
    int& last_flag = *reinterpret_cast<int*>(lds);
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.ws + (size_t)tile_id * S * (BM * BN), (uint32_t)(S * BM * BN * 4));
    const uint32_t own = (uint32_t)split * (BM * BN * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rw,
                                               own + (uint32_t)(((i * FN + j) * 256 + tid) * 16), 0, 16);
    w3_wait_vmcnt<0>();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = (old == (unsigned)(S - 1));
      if (last_flag) __hip_atomic_store(p.counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_flag) return;
    f32x4 tot[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) tot[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // several slabs' loads in flight per round trip (a round per slab left the small tiles' reduction
    // latency-bound: one L2/HBM round trip per split at the kernel's tail); summed in split order
    constexpr int U = FM * FN >= 16 ? 1 : 16 / (FM * FN);  // <= 16 loads in flight per thread
    for (int s0 = 0; s0 < S; s0 += U) {
      f32x4 v[U][FM][FN];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int s = s0 + u;
        const uint32_t base = (uint32_t)s * (BM * BN * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            v[u][i][j] = (s < S && s != split)
                             ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             rw, base + (uint32_t)(((i * FN + j) * 256 + tid) * 16), 0, 16))
                             : acc[i][j];
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
      for (int j = 0; j < FN; ++j) acc[i][j] = tot[i][j];
  }

  // ---- scaled store into the fp32 gradient (TF layout [tap][Mc][Nc])
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ml = wm * TM + i * 16 + g4 * 4 + r;
        const int tp = TT == 1 ? tap : TT * tap + ml / MCT;
        const int m = TT == 1 ? m0 + ml : ml % MCT;
        if (tp < 25 && m < p.Mc && n < p.Nc) p.out[((size_t)tp * p.Mc + m) * p.Nc + n] = acc[i][j][r] * p.scale;
      }
    }
}

}  // namespace dcg

// cfg = 300 + 10 * (3 - NS) + id   (NS = 3 -> 300..303, NS = 2 -> 310..313); two taps per tile
// (TT = 2, BM = 2 Mc): 320..323 with NS = 2, 330..333 with NS = 3
#define DCG_WGRAD3_TILES(X) X(0, 128, 128, 2, 2) X(1, 64, 128, 2, 2) X(2, 128, 64, 2, 2) X(3, 64, 64, 2, 2)

extern "C" int DCG_API(dcg_wgrad3_tile)(int cfg, int* bm, int* bn, int* ns) {
  if (cfg < 300 || cfg >= 340 || cfg % 10 > 3) return -1;
  const int id = cfg % 10;
  *ns = (cfg < 310 || cfg >= 330) ? 3 : 2;
#define X(id_, BM_, BN_, WM_, WN_) if (id == id_) { *bm = BM_; *bn = BN_; return 0; }
  DCG_WGRAD3_TILES(X)
#undef X
  return -1;
}

template <int BM, int BN, int WM, int WN, int NS, int P2, int TT>
static int wlaunch3p(const dcg::WGrad3Args* a, unsigned blocks, hipStream_t s) {
  constexpr size_t shm = (size_t)NS * (BM + BN) * 64 * 2;
  auto k = dcg::wgrad3_kernel<BM, BN, WM, WN, NS, P2, TT>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), shm, s, *a);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int NS, int TT>
static int wlaunch3(const dcg::WGrad3Args* a, unsigned blocks, hipStream_t s) {
  return a->lhw >= 0 ? wlaunch3p<BM, BN, WM, WN, NS, 1, TT>(a, blocks, s)
                     : wlaunch3p<BM, BN, WM, WN, NS, 0, TT>(a, blocks, s);
}

extern "C" int DCG_API(dcg_wgrad3_taps_per_tile)(int cfg) { return cfg >= 320 ? 2 : 1; }

extern "C" int DCG_API(dcg_wgrad3_launch)(const dcg::WGrad3Args* a, int cfg, hipStream_t s) {
  int bm, bn, ns;
  if (DCG_API(dcg_wgrad3_tile)(cfg, &bm, &bn, &ns)) return -1;
  const int tt = DCG_API(dcg_wgrad3_taps_per_tile)(cfg);
  if (tt == 2 && 2 * a->Mc != bm) return -2;  // two-tap tiles hold exactly two taps of every channel
  const unsigned mt = tt == 2 ? 1u : (unsigned)((a->Mc + bm - 1) / bm);
  const unsigned blocks = mt * (unsigned)((a->Nc + bn - 1) / bn) * (unsigned)((25 + tt - 1) / tt) * a->splits;
  const int id = cfg % 10;
#define X(id_, BM_, BN_, WM_, WN_)                                                               \
  if (id == id_) {                                                                               \
    if (tt == 2) return ns == 3 ? wlaunch3<BM_, BN_, WM_, WN_, 3, 2>(a, blocks, s)               \
                                : wlaunch3<BM_, BN_, WM_, WN_, 2, 2>(a, blocks, s);              \
    return ns == 3 ? wlaunch3<BM_, BN_, WM_, WN_, 3, 1>(a, blocks, s)                            \
                   : wlaunch3<BM_, BN_, WM_, WN_, 2, 1>(a, blocks, s);                           \
  }
  DCG_WGRAD3_TILES(X)
#undef X
  return -1;
}
