// dcg-variants: bf16 f16
// Implicit-GEMM convolution, version 5: two ping-pong wave groups per workgroup, a 3-4 stage
// LDS-DMA ring that stays in flight across barriers, and a register-direct epilogue.
// Same conv / deconv semantics, tile decode, split-K protocol and IGemmArgs as igemm3.hip (read
// its header first); what changes is how the K loop overlaps loads with MFMAs.
//
// Why (profiles/r2/igemm3_ablations_r2.txt): in igemm3 every wave of a workgroup waits for its
// k-tile's LDS-DMA (`vmcnt(0)` at two stages), passes the barrier, issues the next tile's DMA,
// reads fragments and only then runs its MFMAs, so the DMA issue, the fragment reads and the
// MFMAs of a workgroup are serial: on the D1 forward GEMM the K loop with MFMAs alone takes
// 13.7 us, with DMA alone 22.6 us and with both 32 us. Here:
//  * 8 waves = 2 groups of 4. Group g owns rows [g*GM, (g+1)*GM) of the BM = 2 GM row tile (2x2
//    waves of (GM/2) x (BN/2)); both groups share the weight tile. Waves w and w+4 share a SIMD,
//    so every SIMD hosts one wave of each group.
//  * Each k-tile is two phases separated by s_barrier: in phase 1 group 0 runs its 32 MFMAs while
//    group 1 reads its fragments of the same k-tile and issues its half of the LDS-DMA for a
//    stage NS-1 tiles ahead; in phase 2 the roles swap (group 0 reads the NEXT k-tile's
//    fragments and issues the stage NS tiles ahead). Every SIMD's matrix pipe stays busy while
//    its partner wave does the loads (MI355X_MICROARCH.md, "Two waves per SIMD").
//  * The DMA of a stage is waited for with a counted `s_waitcnt vmcnt((NS-2) * L)` at the end of
//    phase 1 (L = DMA instructions per wave per stage), never vmcnt(0) inside the loop: up to
//    NS-2 stages stay in flight across the barriers.
//  * Transposed MFMA: acc = mfma(weights, activations), so each lane holds 4 consecutive output
//    channels of one pixel: bias, activation, BN statistics (DPP row sums) and 8-byte stores run
//    straight from the accumulators; no C tile in LDS (the igemm3 epilogue wrote 256 2-byte LDS
//    values per lane).
//
// LDS protocol (slot s = tile % NS; G0 / G1 = the groups; P1(t) / P2(t) = the phases of tile t):
//   G1 issues stage t+NS-1 in P1(t), G0 issues stage t+NS in P2(t) (stages 0..NS-2 / 0..NS-1 in
//   the prologue). Tile t is read by G0 in P2(t-1) and by G1 in P1(t). Write-after-read: the slot
//   a group refills was last read in an earlier phase that ended with `lgkmcnt(0)` + barrier.
//   Read-after-DMA: every wave waits for its own share of stage t+1 at the end of P1(t), before
//   the barrier after which G0 reads it.
#include "kernels.h"

namespace dcg {
namespace ig5 {

template <int N_>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n that is a multiple of L (0..3 L); waiting for more than
// needed is always safe, so unsupported values round down
template <int L>
__device__ __forceinline__ void vmcnt_mul(int k) {
  if (k >= 3) vmcnt<3 * L>();
  else if (k == 2) vmcnt<2 * L>();
  else if (k == 1) vmcnt<L>();
  else vmcnt<0>();
}

__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

template <int S>
__device__ __forceinline__ int kn_swz(int r) {  // 8-byte-chunk XOR of k-major row r (stride S bytes), as igemm3
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

template <int ACT>
__device__ __forceinline__ float act_f(float v, float leak) {
  if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == ACT_LRELU) return fmaxf(v, leak * v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}

__device__ __forceinline__ u32x2 pack4(float a, float b, float c, float d) {
  const elem4 v = {f2bf(a), f2bf(b), f2bf(c), f2bf(d)};
  return __builtin_bit_cast(u32x2, v);
}

__device__ __forceinline__ f32x4 unpack4(u32x2 u) {
  const elem4 v = __builtin_bit_cast(elem4, u);
  return (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// sum over the 16 lanes of a DPP row (lane & 15); every lane of the row gets it
__device__ __forceinline__ float red16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

}  // namespace ig5

// Register epilogue of one wave: acc[i][j] holds C[m = mrow0 + 16 i + fr][n = nl0(j) + r], r = 0..3
// (nl0(j) = wn * TN + 16 j + 4 fq). EPI: 0 plain (+bias, statistics of the stored value, act),
// 1 BN-backward statistics (sum g, sum g * xhat) of the layer whose dL/da this GEMM produces,
// 2 activation backward only (store g = dL/da * act'(y), sum g). The per-wave column sums go to
// part[wrow][BN][2] (LDS).
template <int FM, int FN, int TN, int BN, int ACT, int EPI>
__device__ __forceinline__ void ig5_epilogue(const f32x4 (&acc)[FM][FN], const IGemmArgs& p, const int (&off)[FM],
                                             int wrow, int wn, int fr, int fq, int n0, int m0, float* part) {
  const bool do_stats = p.stats != nullptr;
  const float slope = p.bnb_act == ACT_LRELU ? p.bnb_leak : 0.f;
  const int g = EPI == 1 ? m0 / p.bnb_rpg : 0;
  const int N = p.N;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl0 = wn * TN + 16 * j + 4 * fq;
    const int n = n0 + nl0;
    const bool nok = n < N;  // N % 4 == 0 (host): all 4 channels or none
    f32x4 bv = (f32x4){0.f, 0.f, 0.f, 0.f}, mu = bv, rs = bv;
    if (EPI == 0 && p.bias && nok) bv = *reinterpret_cast<const f32x4*>(p.bias + n);
    if constexpr (EPI == 1) {
      if (nok) {
        mu = *reinterpret_cast<const f32x4*>(p.bnb_mean + g * N + n);
        rs = *reinterpret_cast<const f32x4*>(p.bnb_rstd + g * N + n);
      }
    }
    f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f}, s2 = s;
    // the backward variants' y / x operands of this column block, all issued before any is used
    u32x2 yall[EPI != 0 ? FM : 1], xall[EPI == 1 ? FM : 1];
    if constexpr (EPI != 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const bool ok = nok && off[i] >= 0;
        yall[i] = ok ? *reinterpret_cast<const u32x2*>(p.bnb_y + off[i] + n) : (u32x2){0u, 0u};
        if constexpr (EPI == 1) xall[i] = ok ? *reinterpret_cast<const u32x2*>(p.bnb_x + off[i] + n) : (u32x2){0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bool ok = nok && off[i] >= 0;
      const f32x4 v = acc[i][j] + bv;
      const u32x2 pv = ig5::pack4(v[0], v[1], v[2], v[3]);
      const f32x4 vs = p.out_f32 ? v : ig5::unpack4(pv);  // statistics of exactly the stored tensor
      if constexpr (EPI == 0) {
        if (ok) {
          s += vs;
          s2 += vs * vs;
        }
        if (p.out_f32) {
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = ig5::act_f<ACT>(v[r], p.leak);
          if (ok) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.C) + off[i] + n) = o;
        } else {
          const u32x2 o = ACT == ACT_NONE ? pv
                                          : ig5::pack4(ig5::act_f<ACT>(v[0], p.leak), ig5::act_f<ACT>(v[1], p.leak),
                                                       ig5::act_f<ACT>(v[2], p.leak), ig5::act_f<ACT>(v[3], p.leak));
          if (ok) *reinterpret_cast<u32x2*>(reinterpret_cast<elem_t*>(p.C) + off[i] + n) = o;
        }
      } else if constexpr (EPI == 1) {
        const f32x4 yv = ig5::unpack4(yall[i]), xv = ig5::unpack4(xall[i]);
        f32x4 gv;
#pragma unroll
        for (int r = 0; r < 4; ++r) gv[r] = vs[r] * (yv[r] > 0.f ? 1.f : slope);
        if (ok) {
          s += gv;
          s2 += gv * (xv - mu) * rs;
          *reinterpret_cast<u32x2*>(reinterpret_cast<elem_t*>(p.C) + off[i] + n) = pv;
        }
      } else {
        const f32x4 yv = ig5::unpack4(yall[i]);
        f32x4 d;
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] = p.bnb_act == ACT_TANH ? 1.f - yv[r] * yv[r] : (yv[r] > 0.f ? 1.f : slope);
        const u32x2 pg = ig5::pack4(vs[0] * d[0], vs[1] * d[1], vs[2] * d[2], vs[3] * d[3]);
        if (ok) {
          s += ig5::unpack4(pg);
          *reinterpret_cast<u32x2*>(reinterpret_cast<elem_t*>(p.C) + off[i] + n) = pg;
        }
      }
    }
    if (do_stats) {
      // over the wave's rows: registers over i (above), then the 16 pixel lanes of the DPP row;
      // lane fr == 0 of each row writes its 4 channels
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[r] = ig5::red16(s[r]);
        s2[r] = EPI == 2 ? 0.f : ig5::red16(s2[r]);
      }
      if (fr == 0) {
        float* q = part + (wrow * BN + nl0) * 2;
#pragma unroll
        for (int r = 0; r < 4; ++r) { q[2 * r] = s[r]; q[2 * r + 1] = s2[r]; }
      }
    }
  }
}

template <int GM, int BN, int BKN, int NS>
__global__ __launch_bounds__(512) void igemm5_kernel(IGemmArgs p) {
  constexpr int BK = 64;
  constexpr int BM = 2 * GM;                 // two groups of GM rows
  constexpr int TM = GM / 2, TN = BN / 2;    // wave tile (2 x 2 waves per group)
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NPB = B_BYTES / 1024;                 // B pieces per stage (each group loads half)
  constexpr int PA = GM / 32, PB = NPB / 8;           // DMA pieces per wave per stage
  constexpr int L = PA + PB;                          // DMA instructions per wave per stage
  constexpr int SB = BN * 2;                          // k-major B row stride (bytes)
  constexpr int B_ROWS_PER_PIECE = BKN ? 1024 / SB : 8;
  constexpr int NT = 512;
  static_assert(PA >= 1 && PB >= 1 && FM >= 1 && FN >= 1, "tile");
  static_assert(!BKN || (SB <= 1024 && 1024 % SB == 0), "k-major B rows");
  static_assert(NS >= 3 && NS <= 5, "ring depth");
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  lds_char* const lds3 = (lds_char*)lds;
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds3;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wg = wave & 3;
  const int wm = wg >> 1, wn = wg & 1;

  // ---- tile decode (as igemm3): XCD-aware remap, then split fastest, phase, n, m
  const int S = p.splits;
  const int ntn = (p.N + BN - 1) / BN;
  const int total = p.mtiles * ntn * p.nphases * S;
  int t = blockIdx.x;
  {
    const int q = total >> 3, rr = total & 7, xcd = t & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  const int split = t % S;
  int r_ = t / S;
  const int phase = r_ % p.nphases;
  r_ /= p.nphases;
  const int nt = r_ % ntn;
  const int mt = r_ / ntn;
  const int tile_id = (phase * p.mtiles + mt) * ntn + nt;

  const IGemmPhaseK& ph = p.phk[phase];
  const int M = ph.M;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= M) {  // phase with fewer rows (odd output sizes): its stats slot must still be defined
    if (p.stats && split == 0) {
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.stats + (size_t)(mt * p.nphases + phase) * 2 * p.N,
                                                  (uint32_t)(2 * p.N * 4));
      for (int nl = tid; nl < BN; nl += NT)
        if (n0 + nl < p.N) { st_sc1_f32(rs, (uint32_t)(n0 + nl) * 4u, 0.f); st_sc1_f32(rs, (uint32_t)(p.N + n0 + nl) * 4u, 0.f); }
    }
    return;
  }
  const int Kc = p.Kc, N = p.N;
  const int ntaps = ph.ntaps;
  const int kt_per_tap = (Kc + BK - 1) / BK;
  const int KT = ntaps * kt_per_tap;
  const int kps = (KT + S - 1) / S;
  const int kt0 = split * kps;
  const int kt1 = min(KT, kt0 + kps);
  const int nk = max(0, kt1 - kt0);

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.Bw, p.b_bytes);

  // ---- this lane's A rows: piece q = grp * GM/8 + wg + 4 i (rows 8q .. 8q+7 of the stage),
  //      row = 8 q + lane / 8, LDS slot lane & 7 holds global 16-byte chunk slot ^ (row & 7)
  const int a_chunk = (lane & 7) ^ (lane >> 3);
  int a_base[PA], a_iy[PA], a_ix[PA];
  bool a_ok[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int q = grp * (GM / 8) + wg + 4 * i;
    const int r = 8 * q + (lane >> 3);
    const int m = m0 + r;
    a_ok[i] = m < M;
    const uint32_t b = fdiv((uint32_t)m, ph.fd_hw);
    const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph.Hq * ph.Wq);
    const uint32_t qy = fdiv(rem, ph.fd_w);
    const uint32_t qx = rem - qy * (uint32_t)ph.Wq;
    a_iy[i] = (int)qy * p.sstride + ph.iy0_off;
    a_ix[i] = (int)qx * p.sstride + ph.ix0_off;
    a_base[i] = (((int)b * p.H + a_iy[i]) * p.W + a_ix[i]) * Kc;
  }

  int cur_ti = kt0 / kt_per_tap;  // issue cursor: (tap index, channel offset) of the next stage
  int cur_c0 = (kt0 - cur_ti * kt_per_tap) * BK;

  // this wave's share of one stage: its group's A rows and half of the B tile
  auto issue = [&](int slot) {
    const uint32_t sa = lds_base + slot * STAGE;
    const uint32_t sb = sa + A_BYTES;
    const int ti = ph.tap[cur_ti];
    const int dy = (int)(signed char)(ti & 0xff);
    const int dx = (int)(signed char)((ti >> 8) & 0xff);
    const int wt = ti >> 16;
    const int cc = cur_c0 + a_chunk * 8;
    const bool kval = cc < Kc;
    const int tap_delta = (dy * p.W + dx) * Kc + cc;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int iy = a_iy[i] + dy, ix = a_ix[i] + dx;
      const bool ok = a_ok[i] && kval && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const uint32_t off = oob_unless(ok, (uint32_t)(a_base[i] + tap_delta) * 2u);
      dma16_asm_la(ra, sa + (grp * (GM / 8) + wg + 4 * i) * 1024, off);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int q = grp * (NPB / 2) + wg + 4 * i;
      uint32_t off;
      if constexpr (BKN) {
        const int rr = q * B_ROWS_PER_PIECE + lane / (SB / 16);
        const int k = cur_c0 + rr;
        const int n = n0 + ((lane % (SB / 16)) ^ (ig5::kn_swz<SB>(rr) >> 1)) * 8;
        off = oob_unless(k < p.kb_valid && n < N, (uint32_t)((wt * Kc + k) * N + n) * 2u);
      } else {
        const int n = n0 + 8 * q + (lane >> 3);
        off = oob_unless(n < N && cc < Kc && cc < p.kb_valid, (uint32_t)((wt * N + n) * Kc + cc) * 2u);
      }
      dma16_asm_la(rb, sb + q * 1024, off);
    }
    cur_c0 += BK;
    if (cur_c0 >= Kc) { cur_c0 = 0; ++cur_ti; }
  };

  const int fr = lane & 15, fq = lane >> 4;
  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  elem8 af[2][FM], bfr[2][FN];
  auto read_frags = [&](int slot) {
    const lds_char* sa = lds3 + slot * STAGE;
    const lds_char* sb = sa + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = grp * GM + wm * TM + i * 16 + fr;
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
                LDS_PTR(s16x4, sb + r * SB + ((c8 ^ ig5::kn_swz<SB>(r)) * 8)));
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

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = DCG_MFMA_16x16x32(bfr[ks][j], af[ks][i], acc[i][j], 0, 0, 0);  // transposed: C^T
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: G0 issues stages 0..NS-1, G1 stages 0..NS-2; stage 0 landed -> G0 reads it
  if (nk > 0) {
    const int pre = min(nk, grp == 0 ? NS : NS - 1);
    for (int s = 0; s < pre; ++s) issue(s);
    ig5::vmcnt_mul<L>(pre - 1);
    ig5::barrier();
    if (grp == 0) read_frags(0);
  }

  // The two groups run separate loops (wave-uniform branch): each body is straight-line code
  // with the same two barriers per k-tile, so the groups stay in lockstep. Fragment reads are
  // unconditional (the last G0 read is of a slot nobody refills any more: harmless), so the
  // reads land directly in the MFMA operand registers.
  if (grp == 0) {
    for (int kt = 0; kt < nk; ++kt) {
      mfma();                                           // P1: tile kt (fragments read in P2(kt-1))
      // own share of stage kt+1 landed; stages kt+2 .. min(kt+NS-1, nk-1) may stay in flight
      ig5::vmcnt_mul<L>(min(NS - 2, nk - 2 - kt));
      ig5::barrier();
      read_frags((kt + 1) % NS);                        // P2: tile kt+1, then stage kt+NS
      if (kt + NS < nk) issue((kt + NS) % NS);
      ig5::lgkm0();
      ig5::barrier();
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      read_frags(kt % NS);                              // P1: tile kt, then stage kt+NS-1
      if (kt + NS - 1 < nk) issue((kt + NS - 1) % NS);
      ig5::lgkm0();
      ig5::vmcnt_mul<L>(min(NS - 2, nk - 2 - kt));
      ig5::barrier();
      mfma();                                           // P2: tile kt
      ig5::barrier();
    }
  }
  ig5::vmcnt<0>();

  // ------------------------------------------------------------------ split-K hand-off (igemm3)
  if (S > 1) {
    int& last_flag = *reinterpret_cast<int*>(lds);
    const __amdgpu_buffer_rsrc_t rw =
        make_rsrc(p.ws + (size_t)tile_id * S * (BM * BN), (uint32_t)(S * BM * BN * 4));
    const uint32_t own_base = (uint32_t)split * (BM * BN * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rw,
                                               own_base + (uint32_t)(((i * FN + j) * NT + tid) * 16), 0, 16);
    ig5::vmcnt<0>();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.counters + tile_id, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
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
    for (int s = 0; s < S; ++s) {  // split order: deterministic
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
            tot[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rw, base + (uint32_t)(((i * FN + j) * NT + tid) * 16), 0, 16));
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = tot[i][j];
  }

  // ------------------------------------------------------------------ register epilogue
  __syncthreads();  // every wave is out of the K loop: the ring is free for the statistics rows
  float* part = reinterpret_cast<float*>(lds);  // [4 wave rows][BN][2]
  const int wrow = grp * 2 + wm;
  const int mrow0 = m0 + grp * GM + wm * TM + fr;
  int off[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = mrow0 + 16 * i;
    int o = -1;
    if (m < M) {
      const uint32_t b = fdiv((uint32_t)m, ph.fd_hw);
      const uint32_t rem = (uint32_t)m - b * (uint32_t)(ph.Hq * ph.Wq);
      const uint32_t qy = fdiv(rem, ph.fd_w);
      const uint32_t qx = rem - qy * (uint32_t)ph.Wq;
      const int y = (int)qy * p.ostride + ph.oy_off, x = (int)qx * p.ostride + ph.ox_off;
      o = (((int)b * p.outH + y) * p.outW + x) * p.ldc + p.cofs;
    }
    off[i] = o;
  }
  if (p.bnb_x) {
    if (p.bnb_store_g) {  // EPI 2 reads the activation from bnb_act at run time
      ig5_epilogue<FM, FN, TN, BN, ACT_NONE, 2>(acc, p, off, wrow, wn, fr, fq, n0, m0, part);
    } else {
      ig5_epilogue<FM, FN, TN, BN, ACT_NONE, 1>(acc, p, off, wrow, wn, fr, fq, n0, m0, part);
    }
  } else {
    switch (p.act) {
      case ACT_RELU: ig5_epilogue<FM, FN, TN, BN, ACT_RELU, 0>(acc, p, off, wrow, wn, fr, fq, n0, m0, part); break;
      case ACT_LRELU: ig5_epilogue<FM, FN, TN, BN, ACT_LRELU, 0>(acc, p, off, wrow, wn, fr, fq, n0, m0, part); break;
      case ACT_TANH: ig5_epilogue<FM, FN, TN, BN, ACT_TANH, 0>(acc, p, off, wrow, wn, fr, fq, n0, m0, part); break;
      default: ig5_epilogue<FM, FN, TN, BN, ACT_NONE, 0>(acc, p, off, wrow, wn, fr, fq, n0, m0, part); break;
    }
  }
  if (!p.stats) return;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.stats + (size_t)(mt * p.nphases + phase) * 2 * N, (uint32_t)(2 * N * 4));
  for (int nl = tid; nl < BN; nl += NT) {
    if (n0 + nl >= N) continue;
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {  // fixed order over the 4 wave rows: deterministic
      s += part[(w * BN + nl) * 2];
      s2 += part[(w * BN + nl) * 2 + 1];
    }
    st_sc1_f32(rs, (uint32_t)(n0 + nl) * 4u, s);  // write-through: the finalize kernel reads it
    st_sc1_f32(rs, (uint32_t)(N + n0 + nl) * 4u, s2);
  }
}

}  // namespace dcg

// ---------------------------------------------------------------------------- host launch
// igemm5 configs: cfg = 400 + 10 * k + id, ring depth NS = {3, 4}[k]; tile id -> (GM, BN):
// the workgroup tile is (2 GM) x BN on 8 waves (2 groups x 2 x 2 waves of (GM/2) x (BN/2)).
#define DCG_IGEMM5_TILES(X) X(0, 128, 128) X(1, 128, 64) X(2, 64, 128) X(3, 64, 64)

static constexpr int kIgemm5Stages[2] = {3, 4};

extern "C" int DCG_API(dcg_igemm5_tile)(int cfg, int* bm, int* bn, int* ns) {
  if (cfg < 400 || cfg >= 420) return -1;
  const int id = cfg % 10;
  *ns = kIgemm5Stages[(cfg - 400) / 10];
#define X(id_, GM_, BN_) \
  if (id == id_) { *bm = 2 * GM_; *bn = BN_; return (size_t)*ns * (2 * GM_ + BN_) * 128 <= 160 * 1024 ? 0 : -1; }
  DCG_IGEMM5_TILES(X)
#undef X
  return -1;
}

template <int GM, int BN, int BKN, int NS>
static int launch5(const dcg::IGemmArgs* a, unsigned blocks, hipStream_t s) {
  constexpr size_t shm = (size_t)NS * (2 * GM + BN) * 128;
  auto k = dcg::igemm5_kernel<GM, BN, BKN, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), shm, s, *a);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_igemm5_launch)(const dcg::IGemmArgs* a, int cfg, int bkn, unsigned blocks, hipStream_t s) {
  int bm, bn, ns;
  if (DCG_API(dcg_igemm5_tile)(cfg, &bm, &bn, &ns)) return -1;
  if (a->plain) return -1;  // conv / deconv only
  const int id = cfg % 10;
#define X(id_, GM_, BN_)                                                                          \
  if (id == id_) {                                                                                \
    if (ns == 4) {                                                                                \
      if constexpr ((size_t)4 * (2 * GM_ + BN_) * 128 <= 160 * 1024)                              \
        return bkn ? launch5<GM_, BN_, 1, 4>(a, blocks, s) : launch5<GM_, BN_, 0, 4>(a, blocks, s); \
      return -1;                                                                                  \
    }                                                                                             \
    return bkn ? launch5<GM_, BN_, 1, 3>(a, blocks, s) : launch5<GM_, BN_, 0, 3>(a, blocks, s);   \
  }
  DCG_IGEMM5_TILES(X)
#undef X
  return -1;
}
