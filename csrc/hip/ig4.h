// Arguments of csrc/hip/igemm4.hip (own header: kernel studies of igemm4 rebuild two objects, not
// the whole library).
#pragma once
#include "kernels.h"

namespace dcg {

// igemm4.hip: halo-window implicit GEMM (conv mode 0 / 4-phase deconv mode 1) with loader waves.
// A tile = NI images x TR phase-grid rows x Wq columns (all phases of a deconv in one workgroup,
// one after the other); its input window (per 64-channel chunk) is staged once in LDS and every
// tap reads its fragments from it at a constant pixel offset.
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
  int nwb, shared_win, nch;     // window buffers (1|2), one window for all phases, 64-channel chunks
  int ring_bytes, win_bytes;    // LDS layout: [B ring][windows][stats scratch]
  FastDiv fd_hw, fd_tw, fd_wq, fd_wimg, fd_wxp;  // Hq*Wq, TR*Wq, Wq, WY*WXP, WXP
  uint32_t a_bytes, b_bytes;
  const elem_t* bnb_x; const elem_t* bnb_y; const float* bnb_mean; const float* bnb_rstd;
  int bnb_rpg, bnb_act; float bnb_leak; int bnb_store_g;
  int ntaps[4], oy_off[4], ox_off[4];
  int tap[4][25];               // window pixel offset | weight tap << 16
  unsigned long long* stamps;   // timing studies (DCGAN_IGEMM_STAMPS): s_memtime per workgroup, 8 slots
  int ablate;                   // timing studies (DCGAN_IGEMM_ABLATE): 1 no fragment reads / MFMAs, 2 no DMA,
                                // 4 no epilogue, 8 no barriers
};

}  // namespace dcg
