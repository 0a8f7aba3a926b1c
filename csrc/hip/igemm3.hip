// dcg-variants: bf16 f16
// Implicit-GEMM convolution, version 3: big wave tiles + deep LDS-DMA pipeline + in-kernel
// deterministic split-K + either weight layout. Same conv/deconv/plain semantics and fused
// epilogue as igemm.hip (read that header first); what changes is how the K loop is fed.
//
// Why: a 16x16x32 elem_t MFMA takes 16 cycles/SIMD and a ds_read_b128 costs 4 LDS cycles/CU
// (256 B/clk). With 4 waves of TMxTN wave tiles, LDS time / MFMA time = 16 (TM + TN) / (TM TN):
// 1.0 for 32x32 wave tiles (igemm.hip's 64x64 blocks -> LDS-bound), 0.5 for 64x64. So the
// main tiles here are 128x128 (2x2 waves), 256x64 (4x1) and 64x256 (1x4), all 64x64 per wave.
// Those tiles give too few workgroups for the small-M layers (4x4 / 8x8 outputs), so K is
// split over workgroups: every split writes its fp32 accumulators to a workspace slab with
// `sc1` stores, one lane bumps a per-tile counter (agent atomic), and the workgroup whose add
// comes last sums the slabs IN SPLIT ORDER (deterministic; `sc1` loads bypass the stale L1),
// resets the counter for the next launch / graph replay and runs the fused epilogue.
//
// Pipeline: NS LDS stages, LDS-DMA (buffer_load_dwordx4 ... lds) for both operands, tile
// kt + NS - 1 issued right after the single per-tile barrier, `s_waitcnt vmcnt(LPT * (NS-2))`
// keeps the younger tiles in flight while tile kt is consumed.
//
// Weight layouts (BKN template flag):
//   BKN = 0: Bw[tap][N][Kc] (k contiguous) -> fragments via ds_read_b128, like igemm.hip;
//   BKN = 1: Bw[tap][Kc][N] (n contiguous) -> the LDS tile is k-major and fragments are read
//            with the gfx950 transposing read ds_read_b64_tr_b16 (as in wgrad.hip).
// With both layouts available, every GEMM of the step reads the ONE elem_t mirror of the TF
// weight layout (HWIO conv / [kh,kw,out,in] deconv) that Adam writes: no repack kernels.
//
// Workgroup -> tile mapping is XCD-aware: workgroups are dispatched round-robin over the 8
// XCDs, so workgroup b works on tile (b % 8) * (T / 8) + b / 8, which gives every XCD a
// contiguous run of tiles (neighbouring output pixels share input rows in that XCD's L2).
#include "epilogue.h"

namespace dcg {

template <int S>
__device__ __forceinline__ int kn_swz(int r) {  // 8-byte-chunk XOR of k-major row r (stride S bytes)
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

// 16-byte stores / loads with the `sc1` cache policy (aux bit 16 on gfx94x/gfx950): stores
// write through and drop the line from this XCD's L2, loads bypass L1 -- the cross-workgroup
// hand-off of the split-K slabs. Builtins (not inline asm) so the compiler keeps tracking the
// waitcnts and the store-data hazards.
constexpr int CPOL_SC1 = 16;

__device__ __forceinline__ void store16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, CPOL_SC1);
}

__device__ __forceinline__ f32x4 load16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, CPOL_SC1));
}

// Timing studies (DCGAN_IGEMM_ABLATE / DCGAN_IGEMM_STAMPS) need a build with
// -DDCG_IGEMM_STUDY=1; production kernels carry no runtime study branches.
#ifndef DCG_IGEMM_STUDY
#define DCG_IGEMM_STUDY 0
#endif

template <int N_>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// vmcnt(n * L) for a runtime n in [0, NMAX]
template <int L, int NMAX>
__device__ __forceinline__ void wait_vmcnt_n(int n) {
  if constexpr (NMAX >= 3) { if (n >= 3) { wait_vmcnt<3 * L>(); return; } }
  if constexpr (NMAX >= 2) { if (n >= 2) { wait_vmcnt<2 * L>(); return; } }
  if constexpr (NMAX >= 1) { if (n >= 1) { wait_vmcnt<L>(); return; } }
  wait_vmcnt<0>();
}

// vmcnt(n * L + X): the younger weight tiles plus the next chunk's X window pieces (halo K loop)
template <int L, int NMAX, int X>
__device__ __forceinline__ void wait_vmcnt_win(int n) {
  if constexpr (NMAX >= 3) { if (n >= 3) { wait_vmcnt<3 * L + X>(); return; } }
  if constexpr (NMAX >= 2) { if (n >= 2) { wait_vmcnt<2 * L + X>(); return; } }
  if constexpr (NMAX >= 1) { if (n >= 1) { wait_vmcnt<L + X>(); return; } }
  wait_vmcnt<X>();
}

__device__ __forceinline__ void pp_barrier() {
  // a raw s_barrier pinned in place: no MFMA / ds_read may be scheduled across it (hipcc moves
  // register-only MFMAs past an asm statement otherwise), and no vmcnt drain (the LDS-DMA of
  // younger tiles stays in flight across it)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// dynamic LDS of a tile: the NS-stage operand ring, or the epilogue's row offsets + statistics +
// C tile when that is larger (the 256x256 tile at NS = 2)
template <int BM, int BN, int WM, int NS>
constexpr int igemm3_lds_bytes() {
  constexpr int ring = NS * (BM + BN) * 128, epi = (BM + 2 * WM * BN) * 4 + BM * (BN + 8) * 2;
  return ring > epi ? ring : epi;
}

// HALO K loop (PP == 2; deconv phases, k-contiguous weights): the window of input pixels under a
// phase tile (every tap's rows) is staged ONCE per 64-channel chunk, double-buffered, and each tap
// reads its A fragments from it at the tap's (dy, dx) shift; only the weight tile is loaded per
// tap. Window capacity: HALO_WPW 1 KiB pieces (8 pixels) per wave.
constexpr int HALO_WPW = 7;

template <int BM, int BN, int WM, int WN, int NS>
constexpr int igemm3_halo_lds() {
  constexpr int win = HALO_WPW * WM * WN * 8 * 128;  // one window buffer
  constexpr int ops = 2 * win + NS * BN * 128;
  constexpr int epi = (BM + 2 * WM * BN) * 4 + BM * (BN + 8) * 2;
  return ops > epi ? ops : epi;
}

template <int BM, int BN, int WM, int WN, int BKN, int NS, int PL, int PP = 0>
__global__ __launch_bounds__(64 * WM * WN) void igemm3_kernel(IGemmArgs p) {
  constexpr bool kStudy = DCG_IGEMM_STUDY != 0;
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NW = WM * WN, NT = 64 * NW;                   // 4 or 8 waves
  constexpr int NPA = A_BYTES / 1024, NPB = B_BYTES / 1024;  // 1 KiB DMA pieces per stage
  constexpr int PPW_A = NPA / NW, PPW_B = NPB / NW;           // per wave
  constexpr int LPT = PPW_A + PPW_B;                          // DMA instructions per wave per tile
  constexpr int SB = BN * 2;                                  // k-major B row stride (bytes)
  constexpr int B_ROWS_PER_PIECE = BKN ? 1024 / SB : 8;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(NPA % NW == 0 && NPB % NW == 0, "every wave issues the same DMA count");
  static_assert(FM >= 1 && FN >= 1, "tile");
  static_assert(!BKN || (SB <= 1024 && 1024 % SB == 0), "k-major B rows");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  lds_char* const lds3 = (lds_char*)lds;            // LDS address space: 32-bit ds_* addressing
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds3;

  // wave index as a scalar: every per-wave LDS / DMA address below stays in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // diagnostics: [start, K loop start, K loop end, end] per workgroup (study builds only)
  unsigned long long* stamp = (kStudy && p.stamps) ? p.stamps + (size_t)blockIdx.x * 8 : nullptr;
  if (stamp && tid == 0) stamp[0] = __builtin_amdgcn_s_memtime();

  // ---- tile decode (XCD-aware): t -> (phase, mt, nt, split), split fastest
  const int S = p.splits;
  const int ntn = (p.N + BN - 1) / BN;
  const int total = p.mtiles * ntn * p.nphases * S;
  int t = blockIdx.x;
  int split, phase, nt, mt;
  if (p.lpt && p.nphases > 1) {
    // longest processing time first: the phases (host-sorted, most taps first) are dispatched one
    // after the other, so the short phases fill in at the end; within a phase the same bijective
    // remap over the phase-local index u. The hardware XCD is blockIdx.x & 7, which equals u & 7
    // only when T1 is a multiple of 8; otherwise a phase >= 1 sees its runs on rotated XCDs (still
    // one contiguous run per residue class, so per-XCD L2 locality holds only approximately there)
    const int T1 = p.mtiles * ntn * S;
    phase = t / T1;
    int u = t - phase * T1;
    const int q = T1 >> 3, rr = T1 & 7, f = u & 7;
    u = (f < rr ? f * (q + 1) : rr * (q + 1) + (f - rr) * q) + (u >> 3);
    split = u % S;
    const int r2 = u / S;
    if (p.nmajor) {
      mt = r2 % p.mtiles;
      nt = r2 / p.mtiles;
    } else {
      nt = r2 % ntn;
      mt = r2 / ntn;
    }
  } else {
    {  // bijective XCD remap: workgroups b, b+8, b+16, ... (one XCD) get a contiguous run of t
      const int q = total >> 3, rr = total & 7, xcd = t & 7;
      t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
    }
    // split fastest (a tile's slabs on one XCD), then PHASE (deconv phases have 9/6/6/4 taps: a
    // phase-slowest order would give whole XCDs the 9-tap phase), then n, then m
    split = t % S;
    int r_ = t / S;
    phase = r_ % p.nphases;
    r_ /= p.nphases;
    if (p.nmajor) {
      mt = r_ % p.mtiles;
      nt = r_ / p.mtiles;
    } else {
      nt = r_ % ntn;
      mt = r_ / ntn;
    }
  }
  const int tile_id = (phase * p.mtiles + mt) * ntn + nt;

  const IGemmPhaseK& ph = p.phk[phase];  // kernarg segment: scalar loads
  const int M = ph.M;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= M) {  // phase with fewer rows (odd output sizes): its stats slot must still be defined
    if (p.stats && split == 0) {
      const int row = mt * p.nphases + phase;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.stats + (size_t)row * 2 * p.N, (uint32_t)(2 * p.N * 4));
      for (int nl = tid; nl < BN; nl += NT)
        if (n0 + nl < p.N) { st_sc1_f32(rs, (uint32_t)(n0 + nl) * 4u, 0.f); st_sc1_f32(rs, (uint32_t)(p.N + n0 + nl) * 4u, 0.f); }
    }
    return;
  }
  const int Kc = p.Kc, N = p.N;
  const int ntaps = PL ? 1 : ph.ntaps;
  const int kt_per_tap = (Kc + BK - 1) / BK;
  const int KT = ntaps * kt_per_tap;
  const int kps = (KT + S - 1) / S;  // per phase: deconv phases have 9 / 6 / 6 / 4 taps
  if (stamp && tid == 0) stamp[7] = __builtin_amdgcn_s_memtime();
  const int kt0 = split * kps;
  const int kt1 = min(KT, kt0 + kps);
  const int nk = max(0, kt1 - kt0);

  // ablation (timing only, outputs wrong): bit 0 / 1 a zero-size descriptor drops every A / B
  // fetch (the LDS-DMA still writes zeros), bit 2 skips fragment reads + MFMAs, bit 3 skips the
  // LDS-DMA issue altogether
  const int ablate = kStudy ? p.ablate : 0;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, (ablate & 1) ? 0u : p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.Bw, (ablate & 2) ? 0u : p.b_bytes);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int a_chunk = (lane & 7) ^ (lane >> 3);
  const int fr = lane & 15, fq = lane >> 4;

  // fragments of one k-tile (both k32 halves) from LDS stage `slot` into registers
  elem8 af[2][FM], bfr[2][FN];
  auto read_frags = [&](int slot) {
    const lds_char* sa = lds3 + slot * STAGE;
    const lds_char* sb = sa + A_BYTES;
    const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * TM + i * 16 + fr;
        af[ks][i] = *reinterpret_cast<const __attribute__((address_space(3))) elem8*>(sa + r * 128 + ((c ^ (r & 7)) << 4));
      }
      if constexpr (BKN) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = ks * 32 + 8 * g4 + 4 * h + q4;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int c8 = (wn * TN + j * 16) / 4 + p4;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                LDS_PTR(s16x4, sb + r * SB + ((c8 ^ kn_swz<SB>(r)) * 8)));
            const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) bfr[ks][j][4 * h + e] = vb[e];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wn * TN + j * 16 + fr;
          bfr[ks][j] = *reinterpret_cast<const __attribute__((address_space(3))) elem8*>(sb + r * 128 + ((c ^ (r & 7)) << 4));
        }
      }
    }
  };
  auto mfma_half = [&](int ks) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = DCG_MFMA_16x16x32(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
  };

  if constexpr (PP == 2) {
    // ================================================================ halo K loop (deconv phases)
    static_assert(!BKN && !PL, "halo: k-contiguous weights, conv / deconv modes");
    constexpr int WPIX = HALO_WPW * NW * 8;              // window capacity (pixels)
    constexpr int WBUF = WPIX * 128;                     // bytes per window buffer
    const uint32_t ring_base = lds_base + 2 * WBUF;      // B ring after the two window buffers
    // tile geometry (host-checked): whole images (BM % (Hq Wq) == 0) or whole rows of one image
    const int Hq = ph.Hq, Wq = ph.Wq, HW = Hq * Wq, WC = Wq + 2;
    const int nimg = BM >= HW ? BM / HW : 1, R = BM >= HW ? Hq : BM / Wq, WR = R + 2;
    const int b0 = m0 / HW, qy0 = BM >= HW ? 0 : (m0 - b0 * HW) / Wq;
    const int npix = nimg * WR * WC;
    // per-lane window pieces (chunk-invariant byte offsets; invalid pixels -> zero fill)
    uint32_t w_off[HALO_WPW];
#pragma unroll
    for (int j = 0; j < HALO_WPW; ++j) {
      const int px = 8 * (wave + NW * j) + (lane >> 3);
      const int img = px / (WR * WC), rem = px - img * (WR * WC);
      const int wr = rem / WC, wc = rem - wr * WC;
      const int iy = qy0 + wr - 2 + ph.iy0_off, ix = wc - 2 + ph.ix0_off;
      const bool ok = px < npix && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && b0 + img < p.Bn;
      const int gch = (lane & 7) ^ (px & 7);  // 16-byte slot lane&7 of the LDS row holds chunk gch
      w_off[j] = oob_unless(ok, (uint32_t)((((b0 + img) * p.H + iy) * p.W + ix) * Kc + gch * 8) * 2u);
    }
    // A fragment rows of this lane: window pixel of tap (0, 0)
    int pb[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * TM + i * 16 + fr;
      const int img = BM >= HW ? r / HW : 0, rem = r - img * HW;
      const int rr = rem / Wq, cc = rem - rr * Wq;
      pb[i] = img * WR * WC + (rr + 2) * WC + cc + 2;
    }
    // k-steps: (chunk c, tap t), chunk-major; this split's chunks [c_lo, c_hi)
    const int nch = Kc / BK, ntp = ph.ntaps;
    const int cps = (nch + S - 1) / S;
    const int c_lo = split * cps, c_hi = min(nch, c_lo + cps);
    const int nsteps = max(0, c_hi - c_lo) * ntp;
    auto issue_win = [&](int c) {
      const uint32_t wb = lds_base + (c & 1) * WBUF;
#pragma unroll
      for (int j = 0; j < HALO_WPW; ++j) dma16_asm_la(ra, wb + (wave + NW * j) * 1024, w_off[j] + (uint32_t)(c * BK) * 2u);
    };
    auto issue_b = [&](int st) {  // weight tile of step st (local index) into ring slot st % NS
      const int c = c_lo + st / ntp, t = st - (st / ntp) * ntp;
      const int wt = ph.tap[t] >> 16;
      const uint32_t sb = ring_base + (st % NS) * B_BYTES;
#pragma unroll
      for (int i = 0; i < PPW_B; ++i) {
        const int q = wave + NW * i;
        const int n = n0 + 8 * q + (lane >> 3);
        const int cch = c * BK + a_chunk * 8;
        dma16_asm_la(rb, sb + q * 1024, oob_unless(n < N, (uint32_t)((wt * N + n) * Kc + cch) * 2u));
      }
    };
    if (nsteps > 0) {
      issue_win(c_lo);
#pragma unroll
      for (int st = 0; st < NS - 1; ++st)
        if (st < nsteps) issue_b(st);
    }
    for (int st = 0; st < nsteps; ++st) {
      const int cl = st / ntp, t = st - cl * ntp, c = c_lo + cl;
      // B(st) landed: the younger B tiles stay in flight, and -- on the last NS - 2 taps of a chunk
      // -- the next chunk's window, issued right before the next chunk's first weight tile
      const int ny = min(NS - 2, nsteps - 1 - st);
      const bool wy = NS > 2 && t >= ntp - NS + 2 && c + 1 < c_hi;
      if (wy) wait_vmcnt_win<PPW_B, NS - 2, HALO_WPW>(ny);
      else wait_vmcnt_n<PPW_B, NS - 2>(ny);
      asm volatile("s_barrier" ::: "memory");
      if (st + NS - 1 < nsteps) {
        // the next chunk's window goes out just before that chunk's first weight tile (its buffer
        // was last read in chunk c - 1: every wave is past this step's barrier)
        if ((st + NS - 1) % ntp == 0) issue_win(c + 1);
        issue_b(st + NS - 1);
      }
      const int ti = ph.tap[t];
      const int dy = (int)(signed char)(ti & 0xff), dx = (int)(signed char)((ti >> 8) & 0xff);
      const lds_char* wbuf = lds3 + (c & 1) * WBUF;
      const lds_char* sb = lds3 + 2 * WBUF + (st % NS) * B_BYTES;
      const int sh = dy * WC + dx;
      elem8 af[2][FM], bfr[2][FN];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cq = ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int px = pb[i] + sh;
          af[ks][i] = *reinterpret_cast<const __attribute__((address_space(3))) elem8*>(wbuf + px * 128 + ((cq ^ (px & 7)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wn * TN + j * 16 + fr;
          bfr[ks][j] = *reinterpret_cast<const __attribute__((address_space(3))) elem8*>(sb + r * 128 + ((cq ^ (r & 7)) << 4));
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
  } else if constexpr (PP == 1) {
    // ================================================================ ping-pong K loop
    // 8 waves in two groups of 4 (G0 = waves 0-3 = the tile's first BM/2 rows, G1 = the rest);
    // waves w and w + 4 share a SIMD. Every k-tile t is two barrier-separated phases:
    //   P0(t): G0 runs its MFMAs of tile t (fragments already in registers) while G1 issues its
    //          half of the LDS-DMA of tile t + NS - 1 and reads its fragments of tile t;
    //   P1(t): G1 runs its MFMAs of tile t while G0 issues its half of tile t + NS and reads its
    //          fragments of tile t + 1.
    // So each SIMD's matrix pipe alternates between its two waves while the partner loads
    // (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_programming.md §5 8-phase template).
    // Each group DMAs its own A rows and half of the shared B tile. Tile u lands in slot u % NS;
    // that slot was last read by G1 in P0(u - NS) and by G0 in P1(u - NS - 1), so G0 may refill it
    // from P1(u - NS) on, G1 from its next load phase P0(u - NS + 1) (NS = 2: G1 refills it in its
    // compute phase P1(u - NS), between its two MFMA halves). Every wave waits for its own pieces
    // of tile t + 1 at the end of P0(t) with a counted vmcnt (younger tiles stay in flight); the
    // barrier then publishes the tile to G0's reads in P1(t) and G1's in P0(t + 1).
    // Addressing is hoisted: per-piece byte offsets (with bounds folded in) are computed once per
    // tap; a k-tile adds one scalar term per piece.
    static_assert(NW == 8 && NPA % 8 == 0 && NPB % 8 == 0, "ping-pong: 8 waves, whole pieces per group wave");
    static_assert(!PL, "ping-pong: conv / deconv modes only (Kc % 64 == 0, host-checked)");
    constexpr int PA = NPA / 8, PB = NPB / 8;  // pieces per wave per tile (its group's half)
    constexpr int L = PA + PB;
    constexpr uint32_t BAD = 0xFFF00000u;      // invalid piece: past every descriptor, + <1 MiB per tile
    const int grp = wave >> 2, lw = wave & 3;
    int a_base[PA], a_iy[PA], a_ix[PA];
    bool a_ok[PA];
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int q = grp * (NPA / 2) + lw + 4 * i;
      const int m = m0 + 8 * q + (lane >> 3);
      a_ok[i] = m < M;
      const uint32_t b = fdiv((uint32_t)m, ph.fd_hw);
      const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph.Hq * ph.Wq);
      const uint32_t qy = fdiv(rem, ph.fd_w);
      const uint32_t qx = rem - qy * (uint32_t)ph.Wq;
      a_iy[i] = (int)qy * p.sstride + ph.iy0_off;
      a_ix[i] = (int)qx * p.sstride + ph.ix0_off;
      a_base[i] = (((int)b * p.H + a_iy[i]) * p.W + a_ix[i]) * Kc + a_chunk * 8;
    }
    uint32_t a_off[PA], b_off[PB];
    int tap_ti = -1;
    int cur_ti = kt0 / kt_per_tap;
    int cur_c0 = (kt0 - cur_ti * kt_per_tap) * BK;
    auto set_tap = [&]() {
      const int ti = ph.tap[cur_ti];
      const int dy = (int)(signed char)(ti & 0xff), dx = (int)(signed char)((ti >> 8) & 0xff), wt = ti >> 16;
      const int delta = (dy * p.W + dx) * Kc;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int iy = a_iy[i] + dy, ix = a_ix[i] + dx;
        const bool ok = a_ok[i] && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        a_off[i] = ok ? (uint32_t)(a_base[i] + delta) * 2u : BAD;
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int q = grp * (NPB / 2) + lw + 4 * i;
        if constexpr (BKN) {
          const int rr = q * B_ROWS_PER_PIECE + lane / (SB / 16);
          const int n = n0 + ((lane % (SB / 16)) ^ (kn_swz<SB>(rr) >> 1)) * 8;
          b_off[i] = n < N ? (uint32_t)((wt * Kc + rr) * N + n) * 2u : BAD;
        } else {
          const int n = n0 + 8 * q + (lane >> 3);
          b_off[i] = n < N ? (uint32_t)((wt * N + n) * Kc + a_chunk * 8) * 2u : BAD;
        }
      }
      tap_ti = cur_ti;
    };
    auto issue = [&](int slot) {
      if (tap_ti != cur_ti) set_tap();
      const uint32_t sa = lds_base + slot * STAGE;
      const uint32_t sb = sa + A_BYTES;
      const uint32_t ca = (uint32_t)cur_c0 * 2u, cb = BKN ? (uint32_t)(cur_c0 * N) * 2u : ca;
#pragma unroll
      for (int i = 0; i < PA; ++i) dma16_asm_la(ra, sa + (grp * (NPA / 2) + lw + 4 * i) * 1024, a_off[i] + ca);
#pragma unroll
      for (int i = 0; i < PB; ++i) dma16_asm_la(rb, sb + (grp * (NPB / 2) + lw + 4 * i) * 1024, b_off[i] + cb);
      cur_c0 += BK;
      if (cur_c0 >= Kc) { cur_c0 = 0; ++cur_ti; }
    };
    auto mfma_all = [&]() {
      __builtin_amdgcn_s_setprio(1);
      mfma_half(0);
      mfma_half(1);
      __builtin_amdgcn_s_setprio(0);
    };

    // prologue: G0 issues tiles 0..NS-1, G1 tiles 0..NS-2 (0..NS-1 at NS = 2)
    const int pre = (grp == 0 || NS == 2) ? NS : NS - 1;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (s < pre && s < nk) issue(s);
    if (nk > 0) {
      wait_vmcnt_n<L, NS - 1>(min(min(nk, pre) - 1, NS - 1));  // tile 0 landed (this wave's pieces)
      pp_barrier();
      if (grp == 0) read_frags(0);
    }
    for (int kt = 0; kt < nk; ++kt) {
      // ---- P0(kt)
      if (grp == 0) {
        mfma_all();
      } else {
        if (NS > 2 && kt + NS - 1 < nk) issue((kt + NS - 1) % NS);
        read_frags(kt % NS);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      // tile kt+1 landed for this wave; the younger tiles issued so far stay in flight
      if (kt + 1 < nk) wait_vmcnt_n<L, NS - 2>(min(NS - 2, nk - 2 - kt));
      pp_barrier();
      // ---- P1(kt)
      if (grp == 1) {
        __builtin_amdgcn_s_setprio(1);
        mfma_half(0);
        if (NS == 2 && kt + NS < nk) issue((kt + NS) % NS);
        mfma_half(1);
        __builtin_amdgcn_s_setprio(0);
      } else {
        if (kt + NS < nk) issue((kt + NS) % NS);
        if (kt + 1 < nk) read_frags((kt + 1) % NS);
      }
      pp_barrier();
    }
  } else {
  // ---- A rows of this lane: piece q = wave + 4 i, row = 8 q + lane / 8, slot = lane & 7,
  //      global 16-byte chunk = slot ^ (row & 7)
  int a_base[PPW_A], a_iy[PPW_A], a_ix[PPW_A];
  bool a_ok[PPW_A];
#pragma unroll
  for (int i = 0; i < PPW_A; ++i) {
    const int r = 8 * (wave + NW * i) + (lane >> 3);
    const int m = m0 + r;
    a_ok[i] = m < M;
    if constexpr (PL) {
      a_base[i] = m * Kc; a_iy[i] = 0; a_ix[i] = 0;
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
  // ---- B: BKN=0 rows n (8 per piece, chunk like A); BKN=1 rows k (1024/SB per piece, the
  //      16-byte slot of lane L holds global chunk slot ^ (swizzle(row) / 2))

  // issue cursor: (tap index, channel offset) of the next tile to load
  int cur_ti = kt0 / kt_per_tap;
  int cur_c0 = (kt0 - cur_ti * kt_per_tap) * BK;

  auto issue = [&](int slot) {
    const uint32_t sa = lds_base + slot * STAGE;
    const uint32_t sb = sa + A_BYTES;
    int dy = 0, dx = 0, wt = 0;
    if constexpr (!PL) {
      const int ti = ph.tap[cur_ti];  // scalar load (kernarg): no vector load inside the pipelined loop
      dy = (int)(signed char)(ti & 0xff);
      dx = (int)(signed char)((ti >> 8) & 0xff);
      wt = ti >> 16;
    }
    const int cc = cur_c0 + a_chunk * 8;
    const bool kval = cc < Kc;
    const int tap_delta = (dy * p.W + dx) * Kc + cc;
    // branch-free: every lane computes its offset, a select turns invalid ones into OOB (zero fill)
#pragma unroll
    for (int i = 0; i < PPW_A; ++i) {
      bool ok = a_ok[i] && kval;
      if constexpr (!PL) {
        const int iy = a_iy[i] + dy, ix = a_ix[i] + dx;
        ok = ok && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      }
      const uint32_t off = oob_unless(ok, (uint32_t)(a_base[i] + (PL ? cc : tap_delta)) * 2u);
      dma16_asm_la(ra, sa + (wave + NW * i) * 1024, off);
    }
#pragma unroll
    for (int i = 0; i < PPW_B; ++i) {
      const int q = wave + NW * i;
      uint32_t off;
      if constexpr (BKN) {
        const int rr = q * B_ROWS_PER_PIECE + lane / (SB / 16);
        const int k = cur_c0 + rr;
        const int n = n0 + ((lane % (SB / 16)) ^ (kn_swz<SB>(rr) >> 1)) * 8;
        off = oob_unless(k < p.kb_valid && n < N, (uint32_t)((wt * Kc + k) * N + n) * 2u);
      } else {
        const int n = n0 + 8 * q + (lane >> 3);
        const int c = cur_c0 + a_chunk * 8;
        off = oob_unless(n < N && c < Kc && c < p.kb_valid, (uint32_t)((wt * N + n) * Kc + c) * 2u);
      }
      dma16_asm_la(rb, sb + q * 1024, off);
    }
    cur_c0 += BK;
    if (cur_c0 >= Kc) { cur_c0 = 0; ++cur_ti; }
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk && !(ablate & 8)) issue(s);

  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  if (stamp && tid == 0) stamp[1] = __builtin_amdgcn_s_memtime();
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed for this wave; the younger tiles issued so far (up to NS-2 of them) may stay
    // in flight -- fewer near the end of the loop, where no new tile was issued (a fixed
    // vmcnt(LPT * (NS-2)) would not cover tile nk-2 at NS >= 4)
    wait_vmcnt_n<LPT, NS - 2>(min(NS - 2, nk - 1 - kt));
    // every wave's tile kt landed; every wave is done with slot (kt-1) % NS. A bare s_barrier:
    // __syncthreads() would add the workgroup release, i.e. a vmcnt(0) that also waits for the
    // younger DMA tiles and flattens the pipeline (LDS reads of the previous tile have all
    // returned: their values fed the MFMAs already).
    asm volatile("s_barrier" ::: "memory");
    if (kt + NS - 1 < nk && !(ablate & 8)) issue((kt + NS - 1) % NS);
    if (ablate & 4) continue;  // timing study: no fragment reads / MFMAs
    const lds_char* sa = lds3 + (kt % NS) * STAGE;
    const lds_char* sb = sa + A_BYTES;
    // all fragments of the k-tile first (both k32 halves: the second half's LDS reads are in
    // flight while the first half's MFMAs run), then one prioritised MFMA cluster
    elem8 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * TM + i * 16 + fr;
        af[ks][i] = *reinterpret_cast<const __attribute__((address_space(3))) elem8*>(sa + r * 128 + ((c ^ (r & 7)) << 4));
      }
      if constexpr (BKN) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = ks * 32 + 8 * g4 + 4 * h + q4;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int c8 = (wn * TN + j * 16) / 4 + p4;
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                LDS_PTR(s16x4, sb + r * SB + ((c8 ^ kn_swz<SB>(r)) * 8)));
            const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) bfr[ks][j][4 * h + e] = vb[e];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wn * TN + j * 16 + fr;
          bfr[ks][j] = *reinterpret_cast<const __attribute__((address_space(3))) elem8*>(sb + r * 128 + ((c ^ (r & 7)) << 4));
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
  }  // classic K loop

  if (stamp && tid == 0) stamp[2] = __builtin_amdgcn_s_memtime();
  // ------------------------------------------------------------------ split-K hand-off
  if (S > 1) {
    // flag word in the (now idle) dynamic LDS: a static __shared__ would shift the 16-byte
    // alignment of the dynamic base the ds_read_b128 / tr reads rely on
    int& last_flag = *reinterpret_cast<int*>(lds);
    // this tile's S slabs [S][BM*BN] fp32; lane layout = accumulator-register order, so each
    // (i, j) fragment is one fully coalesced 4 KiB block per workgroup
    const __amdgpu_buffer_rsrc_t rw =
        make_rsrc(p.ws + (size_t)tile_id * S * (BM * BN), (uint32_t)(S * BM * BN * 4));
    const uint32_t own_base = (uint32_t)split * (BM * BN * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) store16_sc1(rw, own_base + (uint32_t)(((i * FN + j) * NT + tid) * 16), acc[i][j]);
    wait_vmcnt<0>();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.counters + tile_id, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      last_flag = (old == (unsigned)(S - 1));
      if (last_flag) __hip_atomic_store(p.counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_flag) return;
    // deterministic: sum slabs in split order, independent of which split arrived last
    f32x4 tot[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) tot[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      if (s == split) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) tot[i][j] += acc[i][j];
      } else {
        const uint32_t base = (uint32_t)s * (BM * BN * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            tot[i][j] += load16_sc1(rw, base + (uint32_t)(((i * FN + j) * NT + tid) * 16));
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = tot[i][j];
  }

  // ------------------------------------------------------------------ epilogue (as igemm.hip)
  __syncthreads();
  int* rowoff = reinterpret_cast<int*>(lds);
  float* red = reinterpret_cast<float*>(lds) + BM;
  constexpr int CPAD = BN + 8;
  elem_t* ctile = reinterpret_cast<elem_t*>(reinterpret_cast<float*>(lds) + BM + 2 * WM * BN);
  constexpr int LDS_TOTAL = PP == 2 ? igemm3_halo_lds<BM, BN, WM, WN, NS>() : igemm3_lds_bytes<BM, BN, WM, NS>();
  static_assert((BM + 2 * WM * BN) * 4 + BM * CPAD * 2 <= LDS_TOTAL, "epilogue LDS");
  for (int r = tid; r < BM; r += NT) {
    const int m = m0 + r;
    int off = -1;
    if (m < M) {
      if constexpr (PL) {
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
  if (stamp && tid == 0) stamp[4] = __builtin_amdgcn_s_memtime();

  const bool do_stats = p.stats != nullptr;
  const bool vec = !p.out_f32 && (N % 8 == 0) && (p.ldc % 8 == 0) && (p.cofs % 8 == 0);
  frag_epilogue_dispatch<FM, FN, TM, TN, BN>(acc, p, rowoff, red, ctile, wm, wn, fr, fq, n0, do_stats, vec, m0);
  if (stamp && tid == 0) stamp[5] = __builtin_amdgcn_s_memtime();
  if (p.bnb_x) {  // BN-backward statistics fused into the store pass (epilogue.h)
    // row-lane scratch (64 * NT bytes) after the C tile, or -- when that does not fit (8-wave
    // tiles at NS = 2) -- over the C tile, written after a barrier once the store pass read it
    constexpr int kEpi = (BM + 2 * WM * BN) * 4, kCt = BM * CPAD * 2, kRed2 = 64 * NT;
    constexpr bool kSep = kEpi + kCt + kRed2 <= LDS_TOTAL;
    constexpr bool kAlias = !kSep && kEpi + (kCt > kRed2 ? kCt : kRed2) <= LDS_TOTAL;
    if constexpr (kSep || kAlias) {
      __syncthreads();
      float* red2 = reinterpret_cast<float*>(reinterpret_cast<char*>(ctile) + (kSep ? kCt : 0));
      vec_store_bnb<BM, BN, NT, kAlias>(p, rowoff, ctile, red2, n0, m0,
                                        p.stats + (size_t)(mt * p.nphases + phase) * 2 * N);
    } else {
      __builtin_trap();  // the host only requests fused statistics on tiles with the LDS for them
    }
    return;
  }
  if (do_stats || vec) __syncthreads();
  if (stamp && tid == 0) stamp[6] = __builtin_amdgcn_s_memtime();
  if (vec) {
    constexpr int CPR = BN / 8;
    elem_t* C = reinterpret_cast<elem_t*>(p.C);
    for (int q = tid; q < BM * CPR; q += NT) {
      const int r = q / CPR, c = q - r * CPR;
      const int off = rowoff[r];
      const int n = n0 + 8 * c;
      if (off >= 0 && n < N)
        *reinterpret_cast<u32x4*>(C + off + p.cofs + n) = *reinterpret_cast<const u32x4*>(ctile + r * CPAD + 8 * c);
    }
  }
  if (do_stats) {
    for (int nl = tid; nl < BN; nl += NT) {
      const int n = n0 + nl;
      if (n >= N) continue;
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s += red[(w * BN + nl) * 2 + 0];
        s2 += red[(w * BN + nl) * 2 + 1];
      }
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.stats + (size_t)(mt * p.nphases + phase) * 2 * N,
                                                  (uint32_t)(2 * N * 4));
      st_sc1_f32(rs, (uint32_t)n * 4u, s);  // write-through (read by the finalize kernel)
      st_sc1_f32(rs, (uint32_t)(N + n) * 4u, s2);
    }
  }
  if (stamp && tid == 0) stamp[3] = __builtin_amdgcn_s_memtime();
}

}  // namespace dcg

// ---------------------------------------------------------------------------- host launch
// v3 configs: cfg = 200 + 10 * k + id, LDS stages NS = {3, 2, 4, 5}[k]  (NS = 3 -> 200..209,
// NS = 2 -> 210..219, NS = 4 -> 220..229, NS = 5 -> 230..239). Deeper rings keep more k-tiles of
// LDS-DMA in flight (issue -> landed is ~1.1 us, several k-tiles of MFMA work), at the cost of
// workgroups per CU (160 KiB of LDS per CU).
// ids 6..9: 8-wave workgroups (512 threads): bigger tiles load fewer operand bytes per MFMA (the
// K loop is bound by the LDS-DMA fill rate, profiles/r2/igemm3_ablations_r2.txt).
// cfg 240..259: the ping-pong K loop (PP) on the 8-wave tiles, NS = 3 (240..249) or 2 (250..259).
#define DCG_IGEMM3_TILES(X) \
  X(0, 128, 128, 2, 2) X(1, 256, 64, 4, 1) X(2, 64, 256, 1, 4) X(3, 128, 64, 2, 2) \
  X(4, 64, 128, 2, 2) X(5, 64, 64, 2, 2) X(6, 256, 128, 4, 2) X(7, 128, 256, 2, 4) X(8, 512, 64, 8, 1) \
  X(9, 256, 256, 4, 2)

static constexpr int kIgemm3Stages[6] = {3, 2, 4, 5, 3, 2};

// halo K loop configs (deconv phases, k-contiguous weights): cfg 300 + 10 k + id, NS = {3, 2}[k],
// 4-wave tiles only (id 0 / 3 / 4 / 5: 128x128, 128x64, 64x128, 64x64)
static bool igemm3_halo_cfg(int cfg) { return cfg >= 300 && cfg < 320 && (cfg % 10 == 0 || (cfg % 10 >= 3 && cfg % 10 <= 5)); }

extern "C" int DCG_API(dcg_igemm3_tile)(int cfg, int* bm, int* bn, int* ns) {
  if (igemm3_halo_cfg(cfg)) {
    const int id = cfg % 10;
    *ns = cfg < 310 ? 3 : 2;
    *bm = (id == 0 || id == 3) ? 128 : 64;
    *bn = (id == 0 || id == 4) ? 128 : 64;
    const size_t win = (size_t)dcg::HALO_WPW * 4 * 8 * 128, epi = (*bm + 2 * 2 * *bn) * 4 + *bm * (*bn + 8) * 2;
    return std::max(2 * win + (size_t)*ns * *bn * 128, epi) <= 160 * 1024 ? 0 : -1;
  }
  if (cfg < 200 || cfg >= 260) return -1;
  const int id = cfg % 10;
  if (cfg >= 240 && id < 6) return -1;  // ping-pong: 8-wave tiles only
  *ns = kIgemm3Stages[(cfg - 200) / 10];
#define X(id_, BM_, BN_, WM_, WN_) \
  if (id == id_) {                                                                                 \
    *bm = BM_; *bn = BN_;                                                                          \
    const size_t epi = (BM_ + 2 * WM_ * BN_) * 4 + BM_ * (BN_ + 8) * 2;                            \
    return (size_t)*ns * (BM_ + BN_) * 128 <= 160 * 1024 && epi <= 160 * 1024 ? 0 : -1;           \
  }
  DCG_IGEMM3_TILES(X)
#undef X
  return -1;
}

template <typename K>
static int launch_k(K k, size_t shm, unsigned blocks, unsigned threads, const dcg::IGemmArgs* a, hipStream_t s) {
  // one attribute call per instantiation (the maximum dynamic LDS of the kernel)
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), shm, s, *a);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int BKN, int NS, int PP>
static int launch3(const dcg::IGemmArgs* a, unsigned blocks, hipStream_t s) {
  constexpr size_t shm = PP == 2 ? (size_t)dcg::igemm3_halo_lds<BM, BN, WM, WN, NS>()
                                 : (size_t)dcg::igemm3_lds_bytes<BM, BN, WM, NS>();
  constexpr unsigned nt = 64 * WM * WN;
  if constexpr (PP == 2) {
    if constexpr (WM * WN == 4 && !BKN && shm <= 160 * 1024) {
      if (a->plain || a->Kc % 64) return -1;
      return launch_k(dcg::igemm3_kernel<BM, BN, WM, WN, 0, NS, 0, 2>, shm, blocks, nt, a, s);
    }
    return -1;
  } else if constexpr (PP) {
    if constexpr (WM * WN == 8) {
      if (a->plain || a->Kc % 64) return -1;  // conv / deconv with whole 64-channel k-tiles only
      return launch_k(dcg::igemm3_kernel<BM, BN, WM, WN, BKN, NS, 0, 1>, shm, blocks, nt, a, s);
    }
    return -1;
  } else {
    // plain (im2col'd) GEMMs read their weight k-major only (the host never asks otherwise)
    if constexpr (BKN) {
      if (a->plain) return launch_k(dcg::igemm3_kernel<BM, BN, WM, WN, 1, NS, 1>, shm, blocks, nt, a, s);
    } else {
      if (a->plain) return -1;
    }
    return launch_k(dcg::igemm3_kernel<BM, BN, WM, WN, BKN, NS, 0>, shm, blocks, nt, a, s);
  }
}

extern "C" int DCG_API(dcg_igemm3_threads)(int cfg) {
  const int id = cfg % 10;
#define X(id_, BM_, BN_, WM_, WN_) if (id == id_) return 64 * WM_ * WN_;
  DCG_IGEMM3_TILES(X)
#undef X
  return 256;
}

template <int BM, int BN, int WM, int WN, int NS, int PP>
static int launch3_ns(const dcg::IGemmArgs* a, int bkn, unsigned blocks, hipStream_t s) {
  if constexpr ((size_t)NS * (BM + BN) * 128 <= 160 * 1024)
    return bkn ? launch3<BM, BN, WM, WN, 1, NS, PP>(a, blocks, s) : launch3<BM, BN, WM, WN, 0, NS, PP>(a, blocks, s);
  return -1;
}

extern "C" int DCG_API(dcg_igemm3_launch)(const dcg::IGemmArgs* a, int cfg, int bkn, unsigned blocks, hipStream_t s) {
  int bm, bn, ns;
  if (DCG_API(dcg_igemm3_tile)(cfg, &bm, &bn, &ns)) return -1;
  const int id = cfg % 10;
  if (igemm3_halo_cfg(cfg)) {
    if (bkn) return -1;
#define XH(id_, BM_, BN_)                                                                          \
    if (id == id_) return ns == 3 ? launch3<BM_, BN_, 2, 2, 0, 3, 2>(a, blocks, s)                  \
                                  : launch3<BM_, BN_, 2, 2, 0, 2, 2>(a, blocks, s);
    XH(0, 128, 128) XH(3, 128, 64) XH(4, 64, 128) XH(5, 64, 64)
#undef XH
    return -1;
  }
  const bool pp = cfg >= 240;
#define X(id_, BM_, BN_, WM_, WN_)                                                              \
  if (id == id_) {                                                                              \
    if (pp) {                                                                                   \
      if constexpr (WM_ * WN_ == 8) {                                                           \
        if (ns == 3) return launch3_ns<BM_, BN_, WM_, WN_, 3, 1>(a, bkn, blocks, s);            \
        return launch3_ns<BM_, BN_, WM_, WN_, 2, 1>(a, bkn, blocks, s);                         \
      }                                                                                         \
      return -1;                                                                                \
    }                                                                                           \
    if (ns == 3) return launch3_ns<BM_, BN_, WM_, WN_, 3, 0>(a, bkn, blocks, s);                \
    if (ns == 4) return launch3_ns<BM_, BN_, WM_, WN_, 4, 0>(a, bkn, blocks, s);                \
    if (ns == 5) return launch3_ns<BM_, BN_, WM_, WN_, 5, 0>(a, bkn, blocks, s);                \
    return launch3_ns<BM_, BN_, WM_, WN_, 2, 0>(a, bkn, blocks, s);                             \
  }
  DCG_IGEMM3_TILES(X)
#undef X
  return -1;
}
