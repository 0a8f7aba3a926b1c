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
};

struct IGemmArgs {
  const bf16* A; int Bn, H, W, Kc, sstride, plain;
  const bf16* Bw; int N;
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
};

struct WGradArgs {
  const bf16* G; int Hg, Wg, Mc;     // gathered operand [B][Hg][Wg][Mc] (plain: [K][Mc])
  const bf16* Dm; int Nc;            // direct operand [K][Nc]
  int K, plain, pl, ntaps;
  float* out;                        // [splits][ntaps][Mc][Nc]
  int kt_per_split;
  uint32_t g_bytes, d_bytes;
  FastDiv fd_hw, fd_w;               // of Hd*Wd, Wd (pixel decode of k)
  int Hd, Wd;
};

}  // namespace dcg

extern "C" {
int dcg_igemm_tile(int cfg, int* bm, int* bn);
int dcg_igemm_launch(const dcg::IGemmArgs* a, int cfg, int mtiles, int ntiles, hipStream_t s);
int dcg_igemm3_tile(int cfg, int* bm, int* bn, int* ns);
int dcg_igemm3_launch(const dcg::IGemmArgs* a, int cfg, int bkn, unsigned blocks, hipStream_t s);
int dcg_wgrad_tile(int cfg, int* bm, int* bn);
int dcg_wgrad_launch(const dcg::WGradArgs* a, int cfg, int splits, hipStream_t s);
int dcg_splitk_reduce(const float* src, int splits, size_t n, float* dst, float scale, hipStream_t s);

int dcg_colstats(int mode, const bf16* x, const bf16* dy, const bf16* y, const float* mean, const float* rstd,
                 int act, float leak, int R, int C, int rows_per_block, int rows_per_group, float* part,
                 hipStream_t s);
int dcg_bn_finalize(const float* part, int ppg, int groups, int C, double count, const float* gamma,
                    const float* beta, float eps, float* mean, float* rstd, float* scale, float* shift,
                    float* ema_mean, float* ema_var, float decay, hipStream_t s);
int dcg_bn_coef_eval(int C, const float* gamma, const float* beta, float eps, const float* mean, const float* var,
                     float debias, float* scale, float* shift, hipStream_t s);
int dcg_bn_apply_act(const bf16* x, bf16* y, const float* scale, const float* shift, int R, int C,
                     int rows_per_group, int act, float leak, hipStream_t s);
int dcg_bn_bwd_finalize(const float* part, int ppg, int groups, int C, float count, const float* gamma,
                        const float* mean, const float* rstd, float* dgamma, float* dbeta, float* coef,
                        hipStream_t s);
int dcg_bn_bwd_apply(const bf16* dy, const bf16* y, const bf16* x, const float* coef, bf16* dx, int R, int C,
                     int rows_per_group, int act, float leak, hipStream_t s);
int dcg_act_bwd(const bf16* dy, const bf16* y, bf16* dx, size_t n, int act, float leak, hipStream_t s);
int dcg_sum_partials(const float* part, int P, int stride, int C, float* dst, hipStream_t s);
int dcg_colsum_small(const bf16* x, int R, int C, float* part, int blocks, hipStream_t s);

int dcg_gan_loss(const float* logits, int B, float* out, float* dl_d, float* dl_g, float* prob, hipStream_t s);
int dcg_linear_fwd(const float* z, const float* W, const float* b, bf16* out, int B, int K, int N, hipStream_t s);
int dcg_linear_wgrad(const float* z, const bf16* dh, float* dW, float* db, int B, int K, int N, hipStream_t s);
int dcg_gemv_head(const bf16* x, const float* w, const float* b, float* out, int R, int K, hipStream_t s);
int dcg_head_dgrad(const float* dl, const float* w, bf16* dx, int R, int K, hipStream_t s);
int dcg_head_wgrad(const bf16* x, const float* dl, float* part, int R, int K, int splits, hipStream_t s);
int dcg_sum_vec(const float* v, int n, float* out, hipStream_t s);
int dcg_adam(float* w, bf16* wbf, const float* g, float* m, float* v, const float* powers, size_t n, float lr,
             float b1, float b2, float eps, float gscale, hipStream_t s);
int dcg_step_end(float* pd, float* pg, float b1d, float b2d, float b1g, float b2g, unsigned long long* step,
                 hipStream_t s);
int dcg_pack(const float* src, int T, int A, int Bd, bf16* nat, bf16* tr, int st, int sb, int sa, hipStream_t s);
int dcg_philox_uniform(float* out, size_t n, uint64_t seed, const unsigned long long* step, uint64_t stream_id,
                       float lo, float hi, hipStream_t s);
int dcg_im2col_s2(const bf16* src, bf16* dst, int B, int H, int W, int C, int Ho, int Wo, int pl_y, int pl_x,
                  int Kpad, hipStream_t s);
int dcg_cast_to_bf16(const void* src, int src_dtype, bf16* dst, size_t n, float scale, float shift, hipStream_t s);
int dcg_cast_bf16_f32(const bf16* src, float* dst, size_t n, hipStream_t s);
}
