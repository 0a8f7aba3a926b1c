// Arguments of csrc/hip/igemm4.hip (own header: kernel studies of igemm4 rebuild two objects, not
// the whole library).
#pragma once
#include "kernels.h"

namespace dcg {

// igemm4.hip: halo-window implicit GEMM (conv mode 0 / 4-phase deconv mode 1) with loader waves.
// A tile = NI images x TR phase-grid rows x Wq columns (all phases of a deconv in one workgroup,
// one after the other); its input window (per 64-channel chunk) is staged once in LDS and every
// tap reads its fragments from it at a constant pixel offset.
//
// The K schedule (phase, 64-channel chunk, tap, window buffer, ring slot, empty steps) is the
// same for every workgroup, so the host unrolls it into per-step descriptor tables (built in
// csrc/bindings.cpp igemm4_ex) and the kernel's step loop only loads the next descriptor: no
// cursor arithmetic, no tap-table lookups, no branches on the schedule.
struct IG4CDesc {  // compute waves, per step s (steps + 1 entries: the last step's prefetch reads one more)
  uint32_t uoff;   // LDS byte offset of the step's tap in its window buffer (k-half 0)
  uint32_t soff;   // LDS byte offset of the step's B ring slot | IG4_EMPTY (an empty step)
};
struct IG4LDesc {  // loader waves, per stage x
  uint32_t boff;   // uniform part of the B global byte offset ((tap, k0) of the step), IG4_EMPTY = none
  uint32_t soff;   // LDS byte offset of the ring slot
  uint32_t win;    // window pieces [q0, q1) = bits 0-7 / 8-15, buffer bit 16, 64-channel chunk bits 17-26
  uint32_t pad;
};
constexpr uint32_t IG4_EMPTY = 0x80000000u;

struct IG4Args {
  const elem_t* A; int Bn, H, W, Kc;
  const elem_t* Bw; int N;
  elem_t* C; int outH, outW, ldc, cofs, ostride;
  const float* bias; int act; float leak;
  float* stats;                 // [mtiles * nphases][2][N] or nullptr
  int nphases, mtiles, ntiles, steps;
  int Hq, Wq, TR, NI, S;        // phase grid, tile rows per image, images per tile, input stride in the window
  int WY, WX, WXP, HX;          // window rows / cols per image (input pixels), LDS pixels per window row, s2d split
  int win_oy, win_ox;           // input row of window row 0 = y0 * S + win_oy; input col of window col 0 = win_ox
  int wpix, npw;                // window pixels (NI * WY * WXP) and 1 KiB DMA pieces per window
  int ring_bytes, win_bytes, part_off, desc_off;  // LDS layout: [B ring][windows][stats scratch][step descriptors]
  FastDiv fd_hw, fd_tw, fd_wq, fd_wimg, fd_wxp;  // Hq*Wq, TR*Wq, Wq, WY*WXP, WXP
  uint32_t a_bytes, b_bytes;
  const elem_t* bnb_x; const elem_t* bnb_y; const float* bnb_mean; const float* bnb_rstd;
  int bnb_rpg, bnb_act; float bnb_leak; int bnb_store_g;
  int oy_off[4], ox_off[4];
  int send[4];                  // first step after phase p (the epilogue of phase p runs there)
  const IG4CDesc* cdesc;        // [steps + 1]
  const IG4LDesc* ldesc;        // [steps]
  unsigned long long* stamps;   // timing studies (DCGAN_IGEMM_STAMPS): s_memtime per workgroup, 12 slots
  int ablate;                   // timing studies (DCGAN_IGEMM_ABLATE): 1 no fragment reads / MFMAs, 2 no DMA,
                                // 4 no epilogue, 8 no barriers
};

}  // namespace dcg
