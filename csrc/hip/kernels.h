// Argument structs and host launchers of the gfx950 kernel library (csrc/hip/*.hip).
#pragma once
#include "common.h"

namespace dcg {

struct IGemmPhase {
  int Hq, Wq, M;            // row grid of this phase: m -> (b, qy, qx)
  int iy0_off, ix0_off;     // source pixel base: iy0 = qy * sstride + iy0_off
  int oy_off, ox_off;       // output pixel:      y   = qy * ostride + oy_off
  int ntaps;
  FastDiv fd_hw, fd_w;      // division by Hq*Wq and by Wq
  signed char dy[25], dx[25];
  short wtap[25];
  short pad_;
  int tap[25];              // packed (dy & 0xff) | (dx & 0xff) << 8 | wtap << 16 (igemm3: staged in LDS)
};

// Compact per-phase table passed BY VALUE in the kernel arguments (igemm3): uniform reads of it
// are scalar loads from the kernarg segment, instead of dependent vector loads from a device
// table (which cost ~1-2k cycles each in a workgroup's prologue / epilogue).
struct IGemmPhaseK {
  int Hq, Wq, M, iy0_off, ix0_off, oy_off, ox_off, ntaps;
  FastDiv fd_hw, fd_w;
  int tap[25];              // packed (dy & 0xff) | (dx & 0xff) << 8 | wtap << 16
};

struct IGemmArgs {
  const elem_t* A; int Bn, H, W, Kc, sstride, plain;
  const elem_t* Bw; int N;
  void* C; int out_f32, outH, outW, ldc, ostride, cofs;
  const float* bias; int act; float leak;
  float* stats;             // [mtiles * nphases][2][N] or nullptr
  int nphases, mtiles;
  uint32_t a_bytes, b_bytes;
  const IGemmPhase* ph;     // device table [nphases]
  // igemm3 only
  int kb_valid;             // B rows (k) that exist; larger k reads zeros (im2col'd K padding)
  int splits;               // split-K over workgroups (k tiles split evenly per phase)
  float* ws;                // [tiles][splits][BM*BN] fp32 slabs (splits > 1)
  unsigned* counters;       // [tiles] arrival counters, zero between launches
  int ablate;               // timing-only builds: bit0 drops A loads, bit1 drops B loads (0 = normal)
  unsigned long long* stamps;  // diagnostics: per-workgroup s_memtime at 4 points (nullptr = off)
  IGemmPhaseK phk[4];       // igemm3: the phase table by value
  // fused BN-backward statistics (epilogue of the data-gradient GEMM that produces dL/da for a
  // BN + activation layer): stats become (sum g, sum g*xhat), g = da * act'(y), xhat = (x-mean)*rstd,
  // instead of (sum v, sum v^2). x / y share C's layout. Tile group = tile row0 / bnb_rpg.
  const elem_t* bnb_x;
  const elem_t* bnb_y;
  const float* bnb_mean;    // [groups][N]
  const float* bnb_rstd;
  int bnb_rpg, bnb_act;
  float bnb_leak;
  // activation-only backward (layer without BN): store g = dL/da * act'(y) instead of dL/da and
  // emit (sum g, 0) per channel -- the bias gradient partials. bnb_x aliases y, mean/rstd unused.
  int bnb_store_g;
  // igemm3: longest phase first (mode 1: phases host-sorted by decreasing tap count, dispatched
  // phase by phase, each phase's tiles XCD-contiguous) instead of the phases interleaved
  int lpt;
  // igemm3: tile order with N slowest (each XCD's contiguous run of tiles shares weight columns)
  // instead of M slowest (shares activation rows); the host picks the smaller per-XCD footprint
  int nmajor;
};


struct WGradArgs {
  const elem_t* G; int Hg, Wg, Mc;     // gathered operand [B][Hg][Wg][Mc] (plain: [K][Mc])
  const elem_t* Dm; int Nc;            // direct operand [K][Nc]
  int K, plain, pl, ntaps;
  float* out;                        // [splits][ntaps][Mc][Nc]
  int kt_per_split;
  uint32_t g_bytes, d_bytes;
  FastDiv fd_hw, fd_w;               // of Hd*Wd, Wd (pixel decode of k)
  int Hd, Wd;
};

struct WGrad3Args {                 // wgrad3.hip: 25-tap gather GEMM, in-kernel split-K
  const elem_t* G; int Hg, Wg, Mc;     // gathered operand [B][Hg][Wg][Mc]
  const elem_t* Dm; int Nc;            // direct operand [K][Nc]
  int K, pl, splits, kt_per_split;
  uint32_t g_bytes, d_bytes;
  FastDiv fd_hw, fd_w;                 // of Hd*Wd, Wd (pixel decode of k)
  int Hd, Wd;
  float* out;                          // final fp32 gradient [25][Mc][Nc] (TF layout), scaled
  float scale;
  float* ws;                           // [tiles][splits][BM*BN] fp32 slabs (splits > 1)
  unsigned* counters;                  // [tiles] arrival counters, zero between launches
  int lhw, lw;                         // log2(Hd*Wd), log2(Wd) when both are powers of two, else -1
};

}  // namespace dcg

extern "C" {
#include "launchers.inc"
}
