// dcg-variants: bf16 f16
// Implicit-GEMM convolution, version 4: input window in LDS ("halo"), loader waves, and a
// transposed accumulator layout with a register-direct epilogue.
//
// Why (profiles/r3/dma_bw_r3.txt, profiles/r2/igemm3_ablations_r2.txt): igemm3's K loop is bound by
// LDS-DMA issue. A buffer_load ... lds of 1 KiB costs its wave ~60-110 issue cycles, and a CU
// moves at most ~75 GB/s from L2 into LDS with 4 issuing waves (~115 GB/s with 16). igemm3
// gathers every operand byte once per tap: a 128x128 tile moves 32 KiB per 64-deep k-step for
// 2 MFLOP, i.e. 64 FLOP per byte, below the ~75 FLOP/B the MFMA rate needs.
//
// Here:
//  * A (activations): a workgroup's output tile is NI images x TR grid rows x Wq columns, so the
//    input pixels all its taps read form a small window (halo). The window of one 64-channel
//    chunk is staged ONCE (full 128-byte lines) and all 25 taps (conv) / 9+6+6+4 taps (the four
//    sub-pixel phases of a deconv, run one after the other) read their fragments out of it at a
//    constant pixel offset. Stride-2 convs store the window column-split by parity
//    (space-to-depth), so 16 lanes reading 16 consecutive output columns read 16 consecutive
//    LDS pixels; a 16-byte chunk XOR (bits 1..3 of the pixel) makes those reads conflict-free.
//  * B (weights): one 64-deep k-step of BN columns per ring stage (NSB stages), as igemm3.
//  * Loader waves: 4 extra waves (one per SIMD) issue every LDS-DMA; the compute waves only
//    ds_read fragments and run MFMAs. One s_barrier per k-step; the loaders keep stage s+1
//    landed at barrier s, so compute waves prefetch the next step's first fragments before it.
//    The next chunk's window streams into the second window buffer in slices behind the B stages
//    (nwb = 2), or -- when two windows do not fit -- after NSB-1 empty steps (nwb = 1).
//  * Transposed MFMA: acc = mfma(weights, activations), so a lane holds 4 consecutive output
//    channels of one pixel: bias / activation / BN statistics / BN-backward statistics and an
//    8-byte packed store straight from registers. Per-channel sums are reduced over the 16
//    pixel lanes with shuffles, and across the compute waves of a column in LDS by the last of
//    them to arrive (LDS counter; in wave order: deterministic) -- no barrier, so the loader
//    waves keep streaming while a deconv phase's epilogue runs.
// Statistics rows: one per (m tile, phase), as igemm3 (engine-compatible).
#include "ig4.h"

namespace dcg {
namespace ig4 {

constexpr int NL = 4;  // loader waves

template <int N_>
__device__ __forceinline__ void wvm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (rounded down above 15: waiting longer is safe)
__device__ __forceinline__ void wvm_dyn(int n) {
  if (n >= 16) {
    if (n >= 48) wvm<48>();
    else if (n >= 32) wvm<32>();
    else if (n >= 24) wvm<24>();
    else wvm<16>();
    return;
  }
  switch (n) {
    case 15: wvm<15>(); break;
    case 14: wvm<14>(); break;
    case 13: wvm<13>(); break;
    case 12: wvm<12>(); break;
    case 11: wvm<11>(); break;
    case 10: wvm<10>(); break;
    case 9: wvm<9>(); break;
    case 8: wvm<8>(); break;
    case 7: wvm<7>(); break;
    case 6: wvm<6>(); break;
    case 5: wvm<5>(); break;
    case 4: wvm<4>(); break;
    case 3: wvm<3>(); break;
    case 2: wvm<2>(); break;
    case 1: wvm<1>(); break;
    default: wvm<0>(); break;
  }
}

__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ void barrier_study(int ablate) {  // ablate bit 8: no barriers (timing only)
  if (!(ablate & 8)) barrier();
}

// 16-byte chunk XOR of a 128-byte LDS row r (window pixel or B row): rows r, r+1 share a 256-byte
// bank row, so XOR bits 1..3 of r -> 16 consecutive rows x one chunk = 16 distinct bank slots
__device__ __forceinline__ int sw8(int r) { return (r >> 1) & 7; }

// Window pixels are 160 bytes apart in LDS (the 128 bytes of a 64-channel chunk + 32 bytes of
// padding): 16 lanes reading 16 consecutive pixels then hit 16 distinct bank slots for ANY first
// pixel (a pure XOR swizzle of 128-byte pixels is 2-way conflicted when the run starts at an odd
// or 2 mod 4 pixel), and a fragment address is one add: lane base + the tap's pixel offset x 160.
constexpr int PIXS = 10;          // 16-byte slots per window pixel
constexpr int PIXB = PIXS * 16;

template <int S>
__device__ __forceinline__ int kn_swz(int r) {  // as igemm3.hip (k-major B rows of S bytes)
  if constexpr (S >= 256) return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (S == 128) return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 4 * ((r >> 3) & 1);
}

// descriptor loads through the constant address space: uniform, so scalar loads (s_load), which
// the compiler may use only when the kernel's own stores cannot alias the table -- through a
// generic pointer it emitted a vector load and waited for it (vmcnt) on every step
__device__ __forceinline__ IG4CDesc ld_desc(const IG4CDesc* p, int i) {
  typedef __attribute__((address_space(4))) const uint32_t cu32;
  cu32* q = (cu32*)p + 2 * i;
  IG4CDesc d;
  d.uoff = q[0];
  d.soff = q[1];
  return d;
}
__device__ __forceinline__ IG4LDesc ld_desc(const IG4LDesc* p, int i) {
  typedef __attribute__((address_space(4))) const uint32_t cu32;
  cu32* q = (cu32*)p + 4 * i;
  IG4LDesc d;
  d.boff = q[0];
  d.soff = q[1];
  d.win = q[2];
  d.pad = 0;
  return d;
}

// scheduling recipe of an MFMA cluster (NM MFMAs) and NR fragment reads for the next one:
// read / MFMA alternate until the reads are out, then the remaining MFMAs
template <int NM, int NR>
__device__ __forceinline__ void interleave() {
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
  }
  __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
}

template <int ACT>
__device__ __forceinline__ float act_f(float v, float leak) {
  if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else if constexpr (ACT == ACT_LRELU) return fmaxf(v, leak * v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  const elem4 v = {f2bf(a), f2bf(b), f2bf(c), f2bf(d)};
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ f32x4 unpack4(uint2 u) {
  const elem4 v = __builtin_bit_cast(elem4, u);
  return (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// sum over the 16 lanes of a DPP row (lane & 15), every lane gets it: quad_perm xor 1 / xor 2,
// then row_half_mirror and row_mirror -- VALU only (__shfl_xor lowers to LDS permutes here)
__device__ __forceinline__ float red16(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}

// B stage row -> channel (n-major B): inside each 32-row group, row bits (h, f1, f0, r1, r0) hold
// channel bits (f1, f0, h, r1, r0) -- MFMA blocks 2P / 2P+1 then give lane group f the channels
// P*32 + 8f + [0, 8), contiguous for one 16-byte store
__device__ __forceinline__ int pair_perm(int r) {
  return (r & ~31) | (((r >> 2) & 3) << 3) | (((r >> 4) & 1) << 2) | (r & 3);
}

}  // namespace ig4

// EPI: 0 plain (+bias, statistics of the stored value, activation), 1 BN-backward statistics of
// the layer whose dL/da this GEMM produces, 2 activation backward only (store g, sums of g).
// PAIR (B in n-major rows): the loader permuted the weight rows inside every 32-row group so that
// MFMA blocks 2P and 2P+1 hold channels P*32 + fq*8 + [0,4) and + [4,8) in lane group fq: one
// 16-byte store per (pixel, 8 channels) instead of two 8-byte ones -- the epilogue is store-issue
// bound (MI355X_MICROARCH.md, epilogue store tail), so half the store instructions.
template <int FM, int FN, int TM, int TN, int WMC, int BN, int ACT, int EPI, bool PAIR>
__device__ __forceinline__ void ig4_epilogue(f32x4 (&acc)[FN][FM], const IG4Args& a, int p, int mt, int m0, int n0,
                                             int b0, int y0, int wm, int wn, int fr, int fq, lds_f32* part,
                                             lds_i32* ctr) {
  constexpr int NPJ = PAIR ? 2 : 1;  // MFMA column blocks per store
  static_assert(FN % NPJ == 0, "pairs of column blocks");
  const int lane = threadIdx.x & 63;
  // laundered: nothing below is loop-invariant to the compiler, so none of it is hoisted out of
  // the phase loop to sit in registers (and spill) across the K loop
  int mlb = wm * TM + fr, nlb = wn * TN + fq * (PAIR ? 8 : 4);
  asm volatile("" : "+v"(mlb), "+v"(nlb));
  int off[FM];
#pragma unroll
  for (int im = 0; im < FM; ++im) {
    const int ml = mlb + im * 16;
    const int bl = (int)fdiv((uint32_t)ml, a.fd_tw);
    const int rem = ml - bl * a.TR * a.Wq;
    const int ty = (int)fdiv((uint32_t)rem, a.fd_wq);
    const int x = rem - ty * a.Wq;
    off[im] = (((b0 + bl) * a.outH + (y0 + ty) * a.ostride + a.oy_off[p]) * a.outW + x * a.ostride + a.ox_off[p]) *
                  a.ldc + a.cofs;
  }
  const bool do_stats = a.stats != nullptr;
  const float slope = a.bnb_act == ACT_LRELU ? a.bnb_leak : 0.f;
  const int g = EPI == 1 ? m0 / a.bnb_rpg : 0;
  using vst = std::conditional_t<PAIR, uint4, uint2>;
#pragma unroll
  for (int jp = 0; jp < FN / NPJ; ++jp) {
    // this lane's first channel of the block group (local to the workgroup's BN columns)
    const int nl0 = nlb + (PAIR ? jp * 32 : jp * 16);
    const int n = n0 + nl0;
    f32x4 bv[NPJ], mu[NPJ], rs[NPJ], s[NPJ], s2[NPJ];
#pragma unroll
    for (int h = 0; h < NPJ; ++h) {
      bv[h] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (EPI == 0 && a.bias) bv[h] = *reinterpret_cast<const f32x4*>(a.bias + n + 4 * h);
      mu[h] = bv[h];
      rs[h] = bv[h];
      if constexpr (EPI == 1) {
        mu[h] = *reinterpret_cast<const f32x4*>(a.bnb_mean + g * a.N + n + 4 * h);
        rs[h] = *reinterpret_cast<const f32x4*>(a.bnb_rstd + g * a.N + n + 4 * h);
      }
      s[h] = (f32x4){0.f, 0.f, 0.f, 0.f};
      s2[h] = s[h];
    }
    // the backward epilogues' y / x tiles of this block group, all issued before any is used
    // (one memory round trip per group; the group barrier below keeps the next group's loads
    // from being hoisted here, which would double the live registers and spill)
    vst yall[EPI != 0 ? FM : 1], xall[EPI == 1 ? FM : 1];
    if constexpr (EPI != 0) {
#pragma unroll
      for (int im = 0; im < FM; ++im) yall[im] = *reinterpret_cast<const vst*>(a.bnb_y + off[im] + n);
    }
    if constexpr (EPI == 1) {
#pragma unroll
      for (int im = 0; im < FM; ++im) xall[im] = *reinterpret_cast<const vst*>(a.bnb_x + off[im] + n);
    }
#pragma unroll
    for (int im = 0; im < FM; ++im) {
      elem_t* dst = a.C + off[im] + n;
      uint2 out[NPJ];
      uint2 yin[NPJ], xin[NPJ];
      if constexpr (EPI != 0) {
        const vst yy = yall[im];
        if constexpr (PAIR) { yin[0] = make_uint2(yy.x, yy.y); yin[NPJ - 1] = make_uint2(yy.z, yy.w); }
        else yin[0] = *reinterpret_cast<const uint2*>(&yy);
      }
      if constexpr (EPI == 1) {
        const vst xx = xall[im];
        if constexpr (PAIR) { xin[0] = make_uint2(xx.x, xx.y); xin[NPJ - 1] = make_uint2(xx.z, xx.w); }
        else xin[0] = *reinterpret_cast<const uint2*>(&xx);
      }
#pragma unroll
      for (int h = 0; h < NPJ; ++h) {
        const f32x4 v = acc[jp * NPJ + h][im] + bv[h];
        // the stored (rounded) values; statistics are of exactly the stored tensor
        const uint2 pv = ig4::pack4(v[0], v[1], v[2], v[3]);
        const f32x4 vs = ig4::unpack4(pv);
        if constexpr (EPI == 0) {
          s[h] += vs;
          s2[h] += vs * vs;
          if constexpr (ACT == ACT_NONE) out[h] = pv;
          else
            out[h] = ig4::pack4(ig4::act_f<ACT>(v[0], a.leak), ig4::act_f<ACT>(v[1], a.leak),
                                ig4::act_f<ACT>(v[2], a.leak), ig4::act_f<ACT>(v[3], a.leak));
        } else if constexpr (EPI == 1) {
          const f32x4 yv = ig4::unpack4(yin[h]), xv = ig4::unpack4(xin[h]);
          f32x4 gv;
#pragma unroll
          for (int r = 0; r < 4; ++r) gv[r] = vs[r] * (yv[r] > 0.f ? 1.f : slope);
          s[h] += gv;
          s2[h] += gv * (xv - mu[h]) * rs[h];
          out[h] = pv;
        } else {
          const f32x4 yv = ig4::unpack4(yin[h]);
          f32x4 d;
#pragma unroll
          for (int r = 0; r < 4; ++r) d[r] = a.bnb_act == ACT_TANH ? 1.f - yv[r] * yv[r] : (yv[r] > 0.f ? 1.f : slope);
          const uint2 pg = ig4::pack4(vs[0] * d[0], vs[1] * d[1], vs[2] * d[2], vs[3] * d[3]);
          s[h] += ig4::unpack4(pg);
          out[h] = pg;
        }
      }
      if constexpr (PAIR) *reinterpret_cast<uint4*>(dst) = make_uint4(out[0].x, out[0].y, out[NPJ - 1].x, out[NPJ - 1].y);
      else *reinterpret_cast<uint2*>(dst) = out[0];
    }
    if (do_stats) {
      // sums over the wave's TM rows: in registers over im, then over the 16 pixel lanes; lanes
      // 0, 16, 32, 48 put 4 * NPJ channels each into this wave's partial row part[wm][BN][2]
#pragma unroll
      for (int h = 0; h < NPJ; ++h) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[h][r] = ig4::red16(s[h][r]);
          s2[h][r] = EPI == 2 ? 0.f : ig4::red16(s2[h][r]);
        }
        if (fr == 0) {
          lds_f32* q = part + (wm * BN + nl0 + 4 * h) * 2;
#pragma unroll
          for (int r = 0; r < 4; ++r) { q[2 * r] = s[h][r]; q[2 * r + 1] = s2[h][r]; }
        }
      }
    }
    if constexpr (EPI != 0) __builtin_amdgcn_sched_barrier(0);
  }
  if (!do_stats) return;
  // the last compute wave of column wn to arrive sums the partial rows in wave order
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(ctr + wn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0, 64);
  if (old != WMC - 1) return;
  if (lane == 0) __hip_atomic_store(ctr + wn, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  float* dst = a.stats + (size_t)(mt * a.nphases + p) * 2 * a.N;
  for (int c = lane; c < TN; c += 64) {
    const int nl = wn * TN + c;
    float t0 = 0.f, t1 = 0.f;
#pragma unroll
    for (int w = 0; w < WMC; ++w) {
      t0 += part[(w * BN + nl) * 2];
      t1 += part[(w * BN + nl) * 2 + 1];
    }
    dst[n0 + nl] = t0;
    dst[a.N + n0 + nl] = t1;
  }
}

template <int BM, int BN, int WMC, int WNC, int NSB, int BKN>
__global__ __launch_bounds__(64 * (WMC * WNC + ig4::NL)) void igemm4_kernel(IG4Args a) {
  using namespace ig4;
  constexpr int NC = WMC * WNC;
  constexpr int TM = BM / WMC, TN = BN / WNC;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int BSTAGE = BN * 128;  // 64 k-rows x BN columns x 2 bytes
  constexpr int NPB = BSTAGE / 1024;
  constexpr int PBL = NPB / NL;     // B pieces per loader wave per stage
  constexpr int SB = BN * 2;        // k-major (BKN) B row bytes
  static_assert(NPB % NL == 0 && PBL >= 1, "B stage pieces split evenly over the loader waves");
  static_assert(FM >= 1 && FN >= 1 && TM % 16 == 0 && TN % 16 == 0, "wave tile");
  static_assert(!BKN || (SB <= 1024 && 1024 % SB == 0), "k-major B rows");
  static_assert(NSB == 3 || NSB == 4, "ring depth");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  lds_char* const l3 = (lds_char*)lds;
  const uint32_t lbase = (uint32_t)(uintptr_t)l3;
  const uint32_t win0 = (uint32_t)a.ring_bytes;  // window buffers after the ring
  lds_f32* part = reinterpret_cast<lds_f32*>(l3 + a.part_off);
  lds_i32* ctr = reinterpret_cast<lds_i32*>(part + WMC * BN * 2);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // diagnostics: 12 s_memtime stamps per workgroup (8 kernel entry, 9 tile decoded,
  // 0-3 compute wave 0, 4-7 loader wave 0)
  unsigned long long* const stw = a.stamps ? a.stamps + (size_t)blockIdx.x * 12 : nullptr;
  if (stw && wave == 0 && lane == 0) stw[8] = __builtin_amdgcn_s_memtime();

  // ---- tile: n fastest (tiles of one window on one XCD), XCD-aware bijective remap
  int t = blockIdx.x;
  {
    const int total = a.mtiles * a.ntiles;
    const int q = total >> 3, rr = total & 7, xcd = t & 7;
    t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (t >> 3);
  }
  const int nt = t % a.ntiles, mt = t / a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int b0 = (int)fdiv((uint32_t)m0, a.fd_hw);
  const int y0 = (int)fdiv((uint32_t)(m0 - b0 * a.Hq * a.Wq), a.fd_wq);
  const int S_ = a.steps;
  if (stw && wave == 0 && lane == 0) stw[9] = __builtin_amdgcn_s_memtime();

  if (tid < 64 && lane < WNC) ctr[lane] = 0;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.A, a.a_bytes);
// window pieces [q0, q1) of chunk `ch` into window buffer `buf`: wave `wid` of `nw` takes q = wid mod nw
  auto issue_win_w = [&](int q0, int q1, int buf, int ch, int wid, int nw) -> int {
    int n = 0;
    const uint32_t dst0 = lbase + win0 + (uint32_t)buf * a.win_bytes;
    for (int q = q0 + wid; q < q1; q += nw, ++n) {
      const int L = q * 64 + lane;
      const int P = L / PIXS;
      const int j = L - P * PIXS;  // 8, 9: padding slots (zero-filled)
      uint32_t off = OOB;
      if (P < a.wpix && j < 8) {
        const int bl = (int)fdiv((uint32_t)P, a.fd_wimg);
        const int rem = P - bl * a.WY * a.WXP;
        const int wy = (int)fdiv((uint32_t)rem, a.fd_wxp);
        const int X = rem - wy * a.WXP;
        const int wx = a.S == 2 ? (X < a.HX ? 2 * X : 2 * (X - a.HX) + 1) : X;
        const int iy = y0 * a.S + a.win_oy + wy, ix = a.win_ox + wx;
        const int b = b0 + bl;
        if (wx < a.WX && b < a.Bn && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
          off = (uint32_t)((((b * a.H + iy) * a.W + ix) * a.Kc + ch * 64 + j * 8) * 2);
      }
      dma16_asm_la(ra, dst0 + q * 1024, off);
    }
    return n;
  };
  if (wave >= NC) {
    // =============================================================== loader waves
    const int lid = wave - NC;
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(a.Bw, a.b_bytes);
    const int Kc = a.Kc, N = a.N;
    // per-lane part of each B piece's global byte offset (the step's (tap, k0) part is uniform:
    // IG4LDesc::boff)
    uint32_t boff_l[PBL];
#pragma unroll
    for (int i = 0; i < PBL; ++i) {
      const int q = lid * PBL + i;
      if constexpr (BKN) {
        const int rr = q * (1024 / SB) + lane / (SB / 16);
        const int n = n0 + ((lane % (SB / 16)) ^ (kn_swz<SB>(rr) >> 1)) * 8;
        boff_l[i] = (uint32_t)((rr * N + n) * 2);
      } else {
        const int r = q * 8 + (lane >> 3);
        const int j = (lane & 7) ^ sw8(r);
        // stage row r holds channel n0 + ig4::pair_perm(r) (the epilogue's 16-byte stores)
        boff_l[i] = (uint32_t)(((n0 + ig4::pair_perm(r)) * Kc + j * 8) * 2);
      }
    }
    // everything stage x carries for this loader; returns its DMA count
    auto issue_stage = [&](int x) -> int {
      if (a.ablate & 2) return 0;  // timing study: no DMA at all
      const IG4LDesc d = ig4::ld_desc(a.ldesc, x);
      int n = 0;
      if (!(d.boff & IG4_EMPTY)) {
        const uint32_t dst0 = lbase + d.soff;
#pragma unroll
        for (int i = 0; i < PBL; ++i) dma16_asm_la(rb, dst0 + (lid * PBL + i) * 1024, d.boff + boff_l[i]);
        n = PBL;
      }
      const int q0 = d.win & 255, q1 = (d.win >> 8) & 255;
      if (q0 < q1) n += issue_win_w(q0, q1, (d.win >> 16) & 1, d.win >> 17, lid, NL);
      return n;
    };

    unsigned long long* st = (lid == 0 && lane == 0) ? stw : nullptr;
    if (st) st[4] = __builtin_amdgcn_s_memtime();
    int cnt[NSB];
    if (!(a.ablate & 2)) issue_win_w(0, a.npw, 0, 0, wave, NC + NL);  // window 0: every wave issues a share
#pragma unroll
    for (int x = 0; x < NSB - 1; ++x) cnt[x] = x < S_ ? issue_stage(x) : 0;
    // stages 0 and 1 (and window 0) landed at barrier 0
    if constexpr (NSB == 4) wvm_dyn(cnt[2]);
    else wvm<0>();
    if (st) st[5] = __builtin_amdgcn_s_memtime();
    barrier_study(a.ablate);
    if (st) st[6] = __builtin_amdgcn_s_memtime();
    for (int s = 0; s + 1 < S_; ++s) {
      const int x = s + NSB - 1;
      const int cx = x < S_ ? issue_stage(x) : 0;
      // stage s+2 landed at barrier s+1 (stage s+3 = x may stay in flight when NSB = 4)
      if constexpr (NSB == 4) wvm_dyn(cx);
      else wvm<0>();
      barrier_study(a.ablate);
    }
    if (st) st[7] = __builtin_amdgcn_s_memtime();
    wvm<0>();
    return;
  }

  // ================================================================= compute waves
  const int wm = wave / WNC, wn = wave % WNC;
  const int fr = lane & 15, fq = lane >> 4;
  const int g4 = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  // LDS byte offset (in a window buffer, tap offset 0) of each activation fragment of this lane:
  // window pixel of the fragment row x 160 + the lane's 16-byte k chunk
  int pb[FM];
#pragma unroll
  for (int im = 0; im < FM; ++im) {
    const int ml = wm * TM + im * 16 + fr;
    const int bl = (int)fdiv((uint32_t)ml, a.fd_tw);
    const int rem = ml - bl * a.TR * a.Wq;
    const int ty = (int)fdiv((uint32_t)rem, a.fd_wq);
    const int x = rem - ty * a.Wq;
    pb[im] = ((bl * a.WY + a.S * ty) * a.WXP + x) * PIXB + fq * 16;
  }
  // BKN = 0: weight-fragment row byte offsets in a stage (chunk fq of row r, XOR-swizzled)
  int wrow[FN];
#pragma unroll
  for (int jn = 0; jn < FN; ++jn) {
    const int r = wn * TN + jn * 16 + fr;
    wrow[jn] = r * 128 + ((fq ^ sw8(r)) << 4);
  }

  f32x4 acc[FN][FM];
#pragma unroll
  for (int jn = 0; jn < FN; ++jn)
#pragma unroll
    for (int im = 0; im < FM; ++im) acc[jn][im] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragments of k-half h (32 of the 64 k rows) of the step with descriptor d (uoff, soff in SGPRs)
  auto read_frags = [&](int h, uint32_t uoff, uint32_t soff, elem8 (&af)[FM], elem8 (&wf)[FN]) {
    const lds_char* wb = l3 + (uoff + h * 64);
#pragma unroll
    for (int im = 0; im < FM; ++im) af[im] = *LDS_PTR(const elem8, wb + pb[im]);
    const lds_char* sb = l3 + (soff & ~IG4_EMPTY);
    if constexpr (BKN) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = h * 32 + 8 * g4 + 4 * hh + q4;
#pragma unroll
        for (int jn = 0; jn < FN; ++jn) {
          const int c8 = (wn * TN + jn * 16) / 4 + p4;
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, sb + r * SB + ((c8 ^ kn_swz<SB>(r)) * 8)));
          const elem4 vb = __builtin_bit_cast(elem4, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) wf[jn][4 * hh + e] = vb[e];
        }
      }
    } else {
#pragma unroll
      for (int jn = 0; jn < FN; ++jn) wf[jn] = *LDS_PTR(const elem8, sb + (wrow[jn] ^ (h * 64)));
    }
  };
  // (no s_setprio around the MFMAs: with one compute wave per SIMD the cluster form serialises
  // the fragment reads / address adds behind the matrix pipe; left free, hipcc interleaves them)
  auto mfmas = [&](const elem8 (&af)[FM], const elem8 (&wf)[FN]) {
#pragma unroll
    for (int jn = 0; jn < FN; ++jn)
#pragma unroll
      for (int im = 0; im < FM; ++im) acc[jn][im] = DCG_MFMA_16x16x32(wf[jn], af[im], acc[jn][im], 0, 0, 0);
  };
  auto epilogue = [&](int p) {
    if (a.ablate & 4) {  // timing study: no epilogue (keep the accumulators live)
#pragma unroll
      for (int jn = 0; jn < FN; ++jn)
#pragma unroll
        for (int im = 0; im < FM; ++im) asm volatile("" ::"v"(acc[jn][im]));
      return;
    }
#define DCG_IG4_EPI(ACT_, EPI_) \
  ig4_epilogue<FM, FN, TM, TN, WMC, BN, ACT_, EPI_, BKN == 0>(acc, a, p, mt, m0, n0, b0, y0, wm, wn, fr, fq, part, ctr)
    if (a.bnb_x) {
      if (a.bnb_store_g) DCG_IG4_EPI(ACT_NONE, 2);
      else DCG_IG4_EPI(ACT_NONE, 1);
    } else {
      switch (a.act) {
        case ACT_RELU: DCG_IG4_EPI(ACT_RELU, 0); break;
        case ACT_LRELU: DCG_IG4_EPI(ACT_LRELU, 0); break;
        case ACT_TANH: DCG_IG4_EPI(ACT_TANH, 0); break;
        default: DCG_IG4_EPI(ACT_NONE, 0); break;
      }
    }
#undef DCG_IG4_EPI
#pragma unroll
    for (int jn = 0; jn < FN; ++jn)
#pragma unroll
      for (int im = 0; im < FM; ++im) acc[jn][im] = (f32x4){0.f, 0.f, 0.f, 0.f};
  };

  unsigned long long* stc = (wave == 0 && lane == 0) ? stw : nullptr;
  if (stc) stc[0] = __builtin_amdgcn_s_memtime();
  // the compute waves' share of window 0 (they are idle until barrier 0 anyway) and the copy of
  // the step descriptors into LDS (landed before barrier 0)
  if (!(a.ablate & 2)) issue_win_w(0, a.npw, 0, 0, wave, NC + NL);
  for (int i = tid; i < S_ + 1; i += 64 * NC) {
    const IG4CDesc d = ig4::ld_desc(a.cdesc, i);
    *LDS_PTR(unsigned long long, l3 + a.desc_off + i * 8) = (unsigned long long)d.uoff | ((unsigned long long)d.soff << 32);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // The step descriptors: copied into LDS in the prologue, and 64 at a time from there into two
  // VGPRs (lane i = step base + i); a step takes its successor's with two v_readlane -- no memory
  // access, so no wait, in the step loop (a scalar load there turned every LDS wait in its
  // shadow into lgkmcnt(0): SMEM returns out of order; an LDS read of it forced a drain at the
  // register hand-over). The 64-step window is refilled once every 64 steps.
  const lds_char* cdl = l3 + a.desc_off;
  uint32_t vdu = 0, vds = 0;
  auto fill_cd = [&](int base) {
    const unsigned long long v = *LDS_PTR(const unsigned long long, cdl + min(base + lane, S_) * 8);
    vdu = (uint32_t)v;
    vds = (uint32_t)(v >> 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto cd_at = [&](int i) -> IG4CDesc {  // i - (the window base) in [0, 64)
    IG4CDesc d;
    d.uoff = __builtin_amdgcn_readlane(vdu, i);
    d.soff = __builtin_amdgcn_readlane(vds, i);
    return d;
  };
  elem8 a0[FM], w0[FN], a1[FM], w1[FN];
  barrier_study(a.ablate);  // B_0: stages 0, 1 and window 0 landed
  if (stc) stc[1] = __builtin_amdgcn_s_memtime();
  fill_cd(0);
  IG4CDesc d0 = cd_at(0);
  const bool study_nomfma = (a.ablate & 1) != 0;
  // every step ends by reading the first k-half of the NEXT step (stage s+1 landed at B_s); an
  // empty step's descriptor points at valid LDS, so its reads need no clamping (data unused), and
  // the last empty step's prefetch is the first real step's first half.
  if (!study_nomfma) read_frags(0, d0.uoff, d0.soff, a0, w0);
  // phases outer, steps inner: the epilogue code sits between the loops, so the hot loop body
  // stays a few hundred bytes of code (inlined into the step loop, the epilogue variants spread
  // every iteration over tens of KiB: instruction-cache misses cost more than the MFMAs)
  int s = 0;
  for (int p = 0; p < a.nphases; ++p) {
    const int send = a.send[p];
    for (; s < send; ++s) {
      if (s > 0) barrier_study(a.ablate);  // B_s: stage s+1 landed, every compute wave done with step s-1
      if (__builtin_expect(((s + 1) & 63) == 0, 0)) fill_cd(s + 1);
      const IG4CDesc d1 = cd_at((s + 1) & 63);
      if (!study_nomfma) {
        // the k-half-1 fragment reads are interleaved with the first MFMA cluster (they land
        // long before the second needs them): one compute wave per SIMD, so an un-interleaved
        // read / address block would leave the matrix core idle. The next step's k-half-0 reads
        // run on every path: one definition of a0 / w0, so no register copies at the join.
        const bool real = !(d0.soff & IG4_EMPTY);
        if (real) {
          read_frags(1, d0.uoff, d0.soff, a1, w1);
          mfmas(a0, w0);
          ig4::interleave<FM * FN, FM + FN>();
        } else {
          // an empty step consumes its (unused) first-half fragments too: both paths reach the
          // next reads with nothing in flight into a0 / w0, so no waits for them there
#pragma unroll
          for (int im = 0; im < FM; ++im) asm volatile("" ::"v"(a0[im]));
#pragma unroll
          for (int jn = 0; jn < FN; ++jn) asm volatile("" ::"v"(w0[jn]));
        }
        read_frags(0, d1.uoff, d1.soff, a0, w0);
        if (real) mfmas(a1, w1);
      }
      d0 = d1;
    }
    if (stc) stc[2] = __builtin_amdgcn_s_memtime();
    epilogue(p);
    if (stc) stc[3] = __builtin_amdgcn_s_memtime();
  }
}

}  // namespace dcg

// ---------------------------------------------------------------------------- host launch
// cfg = 500 + 10 * k + id, B ring stages NSB = {4, 3}[k]; tile id -> (BM, BN, compute waves WMC x WNC),
// 64x64 per compute wave, + 4 loader waves
#define DCG_IGEMM4_TILES(X)                                                                  \
  X(0, 128, 128, 2, 2) X(1, 256, 64, 4, 1) X(2, 256, 128, 4, 2) X(3, 128, 256, 2, 4) X(4, 512, 64, 8, 1) \
  X(5, 64, 256, 1, 4) X(6, 128, 64, 2, 1) X(7, 64, 128, 1, 2)

#ifdef DCG_ONE_CFG  // kernel studies: compile one tile only
#define DCG_IGEMM4_TILES_SEL(X) X(0, 128, 128, 2, 2)
#else
#define DCG_IGEMM4_TILES_SEL(X) DCG_IGEMM4_TILES(X)
#endif

static constexpr int kIgemm4Stages[2] = {4, 3};

extern "C" int DCG_API(dcg_igemm4_tile)(int cfg, int* bm, int* bn, int* nsb, int* wm, int* wn) {
  if (cfg < 500 || cfg >= 520) return -1;
  const int id = cfg % 10;
  *nsb = kIgemm4Stages[(cfg - 500) / 10];
#define X(id_, BM_, BN_, WM_, WN_) \
  if (id == id_) { *bm = BM_; *bn = BN_; *wm = WM_; *wn = WN_; return 0; }
  DCG_IGEMM4_TILES_SEL(X)
#undef X
  return -1;
}

template <int BM, int BN, int WM, int WN, int NSB, int BKN>
static int launch4(const dcg::IG4Args* a, unsigned blocks, size_t shm, hipStream_t s) {
  auto k = dcg::igemm4_kernel<BM, BN, WM, WN, NSB, BKN>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * (WM * WN + dcg::ig4::NL)), shm, s, *a);
  return (int)hipGetLastError();
}

extern "C" int DCG_API(dcg_igemm4_launch)(const dcg::IG4Args* a, int cfg, int bkn, unsigned blocks, size_t shm,
                                          hipStream_t s) {
  int bm, bn, nsb, wm, wn;
  if (DCG_API(dcg_igemm4_tile)(cfg, &bm, &bn, &nsb, &wm, &wn) || shm > 160 * 1024) return -1;
  const int id = cfg % 10;
#define X(id_, BM_, BN_, WM_, WN_)                                                         \
  if (id == id_) {                                                                         \
    if (nsb == 3) return bkn ? launch4<BM_, BN_, WM_, WN_, 3, 1>(a, blocks, shm, s)        \
                             : launch4<BM_, BN_, WM_, WN_, 3, 0>(a, blocks, shm, s);       \
    return bkn ? launch4<BM_, BN_, WM_, WN_, 4, 1>(a, blocks, shm, s)                      \
               : launch4<BM_, BN_, WM_, WN_, 4, 0>(a, blocks, shm, s);                     \
  }
  DCG_IGEMM4_TILES_SEL(X)
#undef X
  return -1;
}
