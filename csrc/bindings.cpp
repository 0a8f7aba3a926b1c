// Python bindings of the native runtime: a recorded "Program" of kernel launches.
//
// The training step is static (fixed shapes, fixed buffers), so the Python engine records it
// ONCE as a list of fully-bound launch closures (pointers, grids, phase tables resolved at
// build time) and then replays ranges of it with one Python->C++ call per range. A range can be
// captured into a hipGraph by the caller (torch.cuda.graph) or replayed eagerly; either way
// there is no per-launch Python work in the steady state. Each op carries a stream slot (0 =
// compute, 1.. = side streams) and event ops express cross-stream dependencies, so
// gradient all-reduces can overlap backward compute.
//
// No torch headers: pointers are passed as integers (tensor.data_ptr()), streams as the raw
// hipStream_t integer (torch.cuda.Stream.cuda_stream). Built with hipcc for gfx950.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "hip/kernels.h"

// The fp16 build of the same kernels (csrc/build.py compiles every .hip twice): identical C
// signatures -- element pointers are 16-bit either way -- with a `_f16` suffix.
#undef DCG_API
#define DCG_API(name) name##_f16
extern "C" {
#include "hip/launchers.inc"
}
#undef DCG_API
#define DCG_API(name) name

// launcher of the Program's element type (bf16 or fp16)
#define KF(fn) (f16_ ? fn##_f16 : fn)

namespace py = pybind11;
using namespace dcg;

#define HIPCHECK(x)                                                                             \
  do {                                                                                          \
    hipError_t e__ = (x);                                                                       \
    if (e__ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e__)); \
  } while (0)

template <class T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

struct Op {
  std::string name;
  int stream;  // slot
  std::function<int(hipStream_t)> fn;
};

class Program {
 public:
  explicit Program(bool f16 = false) : f16_(f16) {}
  bool f16() const { return f16_; }

  ~Program() {
    for (void* p : dev_allocs_) (void)hipFree(p);
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  }

  int size() const { return (int)ops_.size(); }
  std::string name(int i) const { return ops_.at(i).name; }

  void run(std::vector<uintptr_t> streams, int begin, int end) {
    if (end < 0 || end > (int)ops_.size()) end = (int)ops_.size();
    for (int i = begin; i < end; ++i) {
      const Op& op = ops_[i];
      if (op.stream >= (int)streams.size()) throw std::runtime_error("op " + op.name + ": missing stream slot");
      const int rc = op.fn(reinterpret_cast<hipStream_t>(streams[op.stream]));
      if (rc != 0) throw std::runtime_error("op " + std::to_string(i) + " (" + op.name + ") failed: rc=" +
                                            std::to_string(rc) + " " + hipGetErrorString((hipError_t)rc));
    }
  }

  // ------------------------------------------------------------------ events
  int new_event() {
    hipEvent_t e;
    HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    events_.push_back(e);
    return (int)events_.size() - 1;
  }
  int record(int ev, int stream) {
    hipEvent_t e = events_.at(ev);
    return add("record", stream, [e](hipStream_t s) { return (int)hipEventRecord(e, s); });
  }
  int wait(int ev, int stream) {
    hipEvent_t e = events_.at(ev);
    return add("wait", stream, [e](hipStream_t s) { return (int)hipStreamWaitEvent(s, e, 0); });
  }
  int memset(uintptr_t ptr, size_t bytes, int stream) {
    void* p = reinterpret_cast<void*>(ptr);
    return add("memset", stream, [p, bytes](hipStream_t s) { return (int)hipMemsetAsync(p, 0, bytes, s); });
  }
  int copy(uintptr_t dst, uintptr_t src, size_t bytes, int stream) {
    void* d = reinterpret_cast<void*>(dst);
    const void* sp = reinterpret_cast<const void*>(src);
    return add("copy", stream, [d, sp, bytes](hipStream_t s) {
      return (int)hipMemcpyAsync(d, sp, bytes, hipMemcpyDeviceToDevice, s);
    });
  }

  // ------------------------------------------------------------------ implicit GEMM conv
  // mode 0 conv (stride-2 TF SAME), 1 deconv (conv_transpose, 4 sub-pixel phases), 2 plain GEMM
  int igemm(std::string name, int mode, uintptr_t A, uintptr_t Bw, uintptr_t C, int Bn, int Hin, int Win, int Kc,
            int Hout, int Wout, int N, int pad_y, int pad_x, int cfg, int out_f32, int ldc, int cofs,
            uintptr_t bias, int act, float leak, uintptr_t stats, int stream) {
    return igemm_ex(name, mode, A, Bw, C, Bn, Hin, Win, Kc, Hout, Wout, N, pad_y, pad_x, cfg, out_f32, ldc, cofs, bias,
                    act, leak, stats, stream, 0, -1, 1);
  }

  // cfg < 200: igemm.hip tiles (Bw k-contiguous only, no split-K); cfg 200..219: igemm3.hip
  // (bkn = 1 reads Bw as [tap][Kc][N]; kb_valid = number of real B k-rows; splits = split-K).
  int igemm_ex(std::string name, int mode, uintptr_t A, uintptr_t Bw, uintptr_t C, int Bn, int Hin, int Win, int Kc,
               int Hout, int Wout, int N, int pad_y, int pad_x, int cfg, int out_f32, int ldc, int cofs,
               uintptr_t bias, int act, float leak, uintptr_t stats, int stream, int bkn, int kb_valid, int splits,
               uintptr_t bnb_x = 0, uintptr_t bnb_y = 0, uintptr_t bnb_mean = 0, uintptr_t bnb_rstd = 0,
               int bnb_rpg = 0, int bnb_act = 0, float bnb_leak = 0.f, int bnb_store_g = 0) {
    int bm = 0, bn = 0, ns = 0;
    const bool v3 = cfg >= 200;
    if (v3 ? dcg_igemm3_tile(cfg, &bm, &bn, &ns) : dcg_igemm_tile(cfg, &bm, &bn))
      throw std::runtime_error("bad igemm cfg " + std::to_string(cfg));
    if (!v3 && (bkn || splits != 1)) throw std::runtime_error("igemm cfg < 200 supports neither bkn nor split-K");
    if (splits < 1) throw std::runtime_error("splits must be >= 1");
    if (Kc % 8) throw std::runtime_error("igemm needs Kc % 8 == 0 (16-byte A rows)");
    if (bkn && N % 8) throw std::runtime_error("igemm bkn needs N % 8 == 0");
    if (kb_valid < 0) kb_valid = Kc;
    if (kb_valid > Kc) throw std::runtime_error("kb_valid > Kc");
    std::vector<IGemmPhase> ph;
    IGemmArgs a{};
    a.A = P<const elem_t>(A); a.Bn = Bn; a.H = Hin; a.W = Win; a.Kc = Kc;
    a.Bw = P<const elem_t>(Bw); a.N = N;
    a.C = P<void>(C); a.out_f32 = out_f32; a.outH = Hout; a.outW = Wout; a.ldc = ldc; a.cofs = cofs;
    a.bias = P<const float>(bias); a.act = act; a.leak = leak; a.stats = P<float>(stats);
    size_t a_elems, b_elems;
    if (mode == 0) {
      a.sstride = 2; a.plain = 0; a.ostride = 1;
      IGemmPhase p{};
      p.Hq = Hout; p.Wq = Wout; p.M = Bn * Hout * Wout;
      p.iy0_off = -pad_y; p.ix0_off = -pad_x; p.oy_off = 0; p.ox_off = 0;
      p.ntaps = 25;
      for (int t = 0; t < 25; ++t) { p.dy[t] = (signed char)(t / 5); p.dx[t] = (signed char)(t % 5); p.wtap[t] = (short)t; }
      p.fd_hw = fastdiv_make(Hout * Wout); p.fd_w = fastdiv_make(Wout);
      ph.push_back(p);
      a_elems = (size_t)Bn * Hin * Win * Kc; b_elems = (size_t)25 * N * Kc;
    } else if (mode == 1) {
      a.sstride = 1; a.plain = 0; a.ostride = 2;
      for (int py = 0; py < 2; ++py)
        for (int px = 0; px < 2; ++px) {
          IGemmPhase p{};
          p.Hq = (Hout - py + 1) / 2; p.Wq = (Wout - px + 1) / 2; p.M = Bn * p.Hq * p.Wq;
          const int kys = (py + pad_y) & 1, kxs = (px + pad_x) & 1;
          p.iy0_off = (py + pad_y - kys) / 2; p.ix0_off = (px + pad_x - kxs) / 2;
          p.oy_off = py; p.ox_off = px;
          int n = 0;
          for (int ty = 0; kys + 2 * ty < 5; ++ty)
            for (int tx = 0; kxs + 2 * tx < 5; ++tx) {
              p.dy[n] = (signed char)(-ty); p.dx[n] = (signed char)(-tx);
              p.wtap[n] = (short)((kys + 2 * ty) * 5 + kxs + 2 * tx);
              ++n;
            }
          p.ntaps = n;
          p.fd_hw = fastdiv_make(p.Hq * p.Wq); p.fd_w = fastdiv_make(p.Wq);
          if (p.M > 0) ph.push_back(p);
        }
      a_elems = (size_t)Bn * Hin * Win * Kc; b_elems = (size_t)25 * N * Kc;
    } else if (mode == 2) {
      a.sstride = 1; a.plain = 1; a.ostride = 1;
      IGemmPhase p{};
      p.Hq = 1; p.Wq = 1; p.M = Bn * Hout * Wout; p.ntaps = 1;
      p.fd_hw = fastdiv_make(1); p.fd_w = fastdiv_make(1);
      ph.push_back(p);
      a_elems = (size_t)p.M * Kc; b_elems = bkn ? (size_t)kb_valid * N : (size_t)N * Kc;
    } else {
      throw std::runtime_error("bad igemm mode");
    }
    if (a_elems * 2 >= OOB || b_elems * 2 >= OOB)
      throw std::runtime_error("igemm operand exceeds the 3.875 GiB buffer-descriptor range");
    a.a_bytes = (uint32_t)(a_elems * 2); a.b_bytes = (uint32_t)(b_elems * 2);
    for (auto& q : ph)
      for (int t = 0; t < q.ntaps; ++t)
        q.tap[t] = (q.dy[t] & 0xff) | ((q.dx[t] & 0xff) << 8) | ((int)q.wtap[t] << 16);
    a.nphases = (int)ph.size();
    if (a.nphases > 4) throw std::runtime_error("igemm: more than 4 phases");
    for (int i = 0; i < a.nphases; ++i) {
      const IGemmPhase& q = ph[i];
      IGemmPhaseK& k = a.phk[i];
      k.Hq = q.Hq; k.Wq = q.Wq; k.M = q.M; k.iy0_off = q.iy0_off; k.ix0_off = q.ix0_off;
      k.oy_off = q.oy_off; k.ox_off = q.ox_off; k.ntaps = q.ntaps; k.fd_hw = q.fd_hw; k.fd_w = q.fd_w;
      for (int t = 0; t < 25; ++t) k.tap[t] = q.tap[t];
    }
    int maxM = 0;
    for (auto& p : ph) maxM = std::max(maxM, p.M);
    const int mtiles = (maxM + bm - 1) / bm, ntiles = (N + bn - 1) / bn;
    a.mtiles = mtiles;
    void* dph = nullptr;
    HIPCHECK(hipMalloc(&dph, ph.size() * sizeof(IGemmPhase)));
    HIPCHECK(hipMemcpy(dph, ph.data(), ph.size() * sizeof(IGemmPhase), hipMemcpyHostToDevice));
    dev_allocs_.push_back(dph);
    a.ph = reinterpret_cast<const IGemmPhase*>(dph);
    last_mtiles_ = mtiles;
    last_nphases_ = a.nphases;
    a.kb_valid = kb_valid;
    a.splits = splits;
    if (bnb_x) {
      const size_t lds = (size_t)(v3 ? ns : 2) * (bm + bn) * 128;
      if ((size_t)(bm + 8 * bn) * 4 + (size_t)bm * (bn + 8) * 2 + 16384 > lds || out_f32 || N % 8 || ldc % 8 || cofs % 8)
        throw std::runtime_error("igemm bnb: tile has no LDS for the fused statistics or output is not vectorizable");
      if (bnb_store_g) {  // activation backward only (no BN): x, mean, rstd and groups unused
        if (!stats || !bnb_y) throw std::runtime_error("igemm act-backward store: needs stats and y");
        a.bnb_x = P<const elem_t>(bnb_y); a.bnb_y = P<const elem_t>(bnb_y);
        a.bnb_rpg = 1 << 30; a.bnb_act = bnb_act; a.bnb_leak = bnb_leak; a.bnb_store_g = 1;
      } else {
        if (!stats || bnb_rpg <= 0 || !bnb_y || !bnb_mean || !bnb_rstd)
          throw std::runtime_error("igemm bnb: needs stats, rows-per-group, y, mean, rstd");
        for (auto& q : ph)  // tiles must not straddle a BN group (a phase's rows are (b, qy, qx))
          if (bnb_rpg % bm || q.M % bnb_rpg) throw std::runtime_error("igemm bnb: tile rows must divide the group");
        a.bnb_x = P<const elem_t>(bnb_x); a.bnb_y = P<const elem_t>(bnb_y);
        a.bnb_mean = P<const float>(bnb_mean); a.bnb_rstd = P<const float>(bnb_rstd);
        a.bnb_rpg = bnb_rpg; a.bnb_act = bnb_act; a.bnb_leak = bnb_leak;
      }
    }
    if (const char* ab = getenv("DCGAN_IGEMM_ABLATE")) a.ablate = atoi(ab);  // kernel studies only
    if (const char* st = getenv("DCGAN_IGEMM_STAMPS")) a.stamps = reinterpret_cast<unsigned long long*>(strtoull(st, nullptr, 0));
    if (!v3)
      return add(name, stream, [this, a, cfg, mtiles, ntiles](hipStream_t s) {
        return KF(dcg_igemm_launch)(&a, cfg, mtiles, ntiles, s);
      });
    const size_t tiles = (size_t)mtiles * ntiles * a.nphases;
    if (splits > 1) {  // per-op workspace + zeroed arrival counters (reset by the kernel itself)
      void* ws = nullptr;
      void* ctr = nullptr;
      HIPCHECK(hipMalloc(&ws, tiles * splits * (size_t)bm * bn * sizeof(float)));
      HIPCHECK(hipMalloc(&ctr, tiles * sizeof(unsigned)));
      HIPCHECK(hipMemset(ctr, 0, tiles * sizeof(unsigned)));
      dev_allocs_.push_back(ws);
      dev_allocs_.push_back(ctr);
      a.ws = reinterpret_cast<float*>(ws);
      a.counters = reinterpret_cast<unsigned*>(ctr);
    }
    const unsigned blocks = (unsigned)(tiles * splits);
    return add(name, stream, [this, a, cfg, bkn, blocks](hipStream_t s) { return KF(dcg_igemm3_launch)(&a, cfg, bkn, blocks, s); });
  }
  int last_mtiles() const { return last_mtiles_; }
  int last_nphases() const { return last_nphases_; }

  // ------------------------------------------------------------------ weight gradient
  // mode 0 conv/deconv gather (25 taps), 2 plain (1 tap). out: [splits][taps][Mc][Nc] fp32 slabs,
  // then reduced into dst (fp32, scaled) by a fused split-K reduce op.
  int wgrad(std::string name, int mode, uintptr_t G, int Hg, int Wg, int Mc, uintptr_t Dm, int Bn, int Hd, int Wd,
            int Nc, int pad, int cfg, int splits, uintptr_t slabs, uintptr_t dst, size_t dst_elems, float scale,
            int stream) {
    WGradArgs a{};
    a.G = P<const elem_t>(G); a.Hg = Hg; a.Wg = Wg; a.Mc = Mc;
    a.Dm = P<const elem_t>(Dm); a.Nc = Nc;
    a.K = Bn * Hd * Wd; a.plain = mode == 2; a.pl = pad; a.ntaps = mode == 2 ? 1 : 25;
    a.out = P<float>(slabs);
    const int KT = (a.K + 63) / 64;
    a.kt_per_split = (KT + splits - 1) / splits;
    const size_t g_elems = mode == 2 ? (size_t)a.K * Mc : (size_t)Bn * Hg * Wg * Mc;
    const size_t d_elems = (size_t)a.K * Nc;
    if (g_elems * 2 >= OOB || d_elems * 2 >= OOB)
      throw std::runtime_error("wgrad operand exceeds the 3.875 GiB buffer-descriptor range");
    a.g_bytes = (uint32_t)(g_elems * 2); a.d_bytes = (uint32_t)(d_elems * 2);
    a.fd_hw = fastdiv_make(Hd * Wd); a.fd_w = fastdiv_make(Wd); a.Hd = Hd; a.Wd = Wd;
    const size_t n = (size_t)a.ntaps * Mc * Nc;
    if (dst_elems > n) throw std::runtime_error("wgrad dst larger than result");
    float* slab = P<float>(slabs);
    float* d = P<float>(dst);
    add(name, stream, [this, a, cfg, splits](hipStream_t s) { return KF(dcg_wgrad_launch)(&a, cfg, splits, s); });
    // plain mode may carry padded rows (im2col K padding): reduce only the first dst_elems of
    // each slab's leading part -- rows are m-major so the valid prefix is contiguous.
    return add(name + ".reduce", stream, [this, slab, splits, n, d, dst_elems, scale](hipStream_t s) {
      if (dst_elems == n) return KF(dcg_splitk_reduce)(slab, splits, n, d, scale, s);
      // strided variant: reduce the whole slab into itself (slab 0) then copy the valid prefix
      int rc = KF(dcg_splitk_reduce)(slab, splits, n, slab, scale, s);
      if (rc) return rc;
      return (int)hipMemcpyAsync(d, slab, dst_elems * sizeof(float), hipMemcpyDeviceToDevice, s);
    });
  }

  // weight gradient v3 (wgrad3.hip): the 25-tap gather GEMM with the split-K reduction in-kernel,
  // written scaled straight into the fp32 gradient dst [25][Mc][Nc] -- one launch, no slabs pass
  int wgrad3(std::string name, uintptr_t G, int Hg, int Wg, int Mc, uintptr_t Dm, int Bn, int Hd, int Wd, int Nc,
             int pad, int cfg, int splits, uintptr_t dst, float scale, int stream) {
    int bm = 0, bn = 0, ns = 0;
    if (dcg_wgrad3_tile(cfg, &bm, &bn, &ns)) throw std::runtime_error("bad wgrad3 cfg " + std::to_string(cfg));
    if (Mc % 8 || Nc % 8) throw std::runtime_error("wgrad3 needs Mc % 8 == 0 and Nc % 8 == 0 (16-byte DMA chunks)");
    if (splits < 1) throw std::runtime_error("splits must be >= 1");
    WGrad3Args a{};
    a.G = P<const elem_t>(G); a.Hg = Hg; a.Wg = Wg; a.Mc = Mc;
    a.Dm = P<const elem_t>(Dm); a.Nc = Nc;
    a.K = Bn * Hd * Wd; a.pl = pad; a.splits = splits;
    const int KT = (a.K + 63) / 64;
    a.kt_per_split = (KT + splits - 1) / splits;
    const size_t g_elems = (size_t)Bn * Hg * Wg * Mc, d_elems = (size_t)a.K * Nc;
    if (g_elems * 2 >= OOB || d_elems * 2 >= OOB)
      throw std::runtime_error("wgrad3 operand exceeds the 3.875 GiB buffer-descriptor range");
    a.g_bytes = (uint32_t)(g_elems * 2); a.d_bytes = (uint32_t)(d_elems * 2);
    a.fd_hw = fastdiv_make(Hd * Wd); a.fd_w = fastdiv_make(Wd); a.Hd = Hd; a.Wd = Wd;
    a.out = P<float>(dst); a.scale = scale;
    const size_t tiles = (size_t)((Mc + bm - 1) / bm) * ((Nc + bn - 1) / bn) * 25;
    if (splits > 1) {
      if ((size_t)splits * bm * bn * 4 >= OOB) throw std::runtime_error("wgrad3: split slabs too large");
      void* ws = nullptr;
      void* ctr = nullptr;
      HIPCHECK(hipMalloc(&ws, tiles * splits * (size_t)bm * bn * sizeof(float)));
      HIPCHECK(hipMalloc(&ctr, tiles * sizeof(unsigned)));
      HIPCHECK(hipMemset(ctr, 0, tiles * sizeof(unsigned)));
      dev_allocs_.push_back(ws);
      dev_allocs_.push_back(ctr);
      a.ws = reinterpret_cast<float*>(ws);
      a.counters = reinterpret_cast<unsigned*>(ctr);
    }
    return add(name, stream, [this, a, cfg](hipStream_t s) { return KF(dcg_wgrad3_launch)(&a, cfg, s); });
  }

  // ------------------------------------------------------------------ BN / activations
  int colstats(std::string name, int mode, uintptr_t x, uintptr_t dy, uintptr_t y, uintptr_t mean, uintptr_t rstd,
               int act, float leak, int R, int C, int rows_per_block, int rows_per_group, uintptr_t part,
               int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_colstats)(mode, P<const elem_t>(x), P<const elem_t>(dy), P<const elem_t>(y), P<const float>(mean),
                          P<const float>(rstd), act, leak, R, C, rows_per_block, rows_per_group, P<float>(part), s);
    });
  }
  int bn_finalize(std::string name, uintptr_t part, int ppg, int groups, int C, double count, uintptr_t gamma,
                  uintptr_t beta, float eps, uintptr_t mean, uintptr_t rstd, uintptr_t scale, uintptr_t shift,
                  uintptr_t ema_mean, uintptr_t ema_var, float decay, int stream) {
    if (use_rows_fin()) {
      const int PS = rows_slices(ppg, C);
      double* ws = nullptr;
      unsigned* ctr = nullptr;
      alloc_split(&ws, &ctr, (size_t)groups * PS * 2 * C, (size_t)groups);
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bn_finalize_rows)(0, P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                        P<const float>(beta), eps, P<float>(mean), P<float>(rstd), P<float>(scale),
                                        P<float>(shift), P<float>(ema_mean), P<float>(ema_var), decay, nullptr,
                                        nullptr, nullptr, ws, ctr, PS, s);
      });
    }
    int PS = split_slices(ppg);
    if (PS > 1) {  // many partial rows: sliced reduction + last-arrival finalize
      double* ws = nullptr;
      unsigned* ctr = nullptr;
      alloc_split(&ws, &ctr, (size_t)groups * PS * 2 * C, (size_t)groups * ((C + 15) / 16));
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bn_finalize_split)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                         P<const float>(beta), eps, P<float>(mean), P<float>(rstd), P<float>(scale),
                                         P<float>(shift), P<float>(ema_mean), P<float>(ema_var), decay, ws, ctr, PS, s);
      });
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_finalize)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                             P<const float>(beta), eps, P<float>(mean), P<float>(rstd), P<float>(scale),
                             P<float>(shift), P<float>(ema_mean), P<float>(ema_var), decay, s);
    });
  }
  static int split_slices(int ppg) { return ppg > 64 ? std::min(32, (ppg + 63) / 64) : 1; }
  // row-wide finalize (bn_finalize_rows_kernel): ~8 partial rows per row lane per slice
  // measured slower than the 16-channel split finalize on the 64x64 step (+85 us): opt-in only
  static bool use_rows_fin() {
    const char* e = getenv("DCGAN_BN_FIN_V2");
    return e && e[0] == '1';
  }
  static int rows_slices(int ppg, int C) {
    const int lanes = C <= 512 ? std::max(1, 512 / C) : 1;
    return std::max(1, std::min(64, (ppg + lanes * 8 - 1) / (lanes * 8)));
  }
  void alloc_split(double** ws, unsigned** ctr, size_t ws_elems, size_t counters) {
    void* w = nullptr;
    void* c = nullptr;
    HIPCHECK(hipMalloc(&w, ws_elems * sizeof(double)));
    HIPCHECK(hipMalloc(&c, counters * sizeof(unsigned)));
    HIPCHECK(hipMemset(c, 0, counters * sizeof(unsigned)));
    dev_allocs_.push_back(w);
    dev_allocs_.push_back(c);
    *ws = reinterpret_cast<double*>(w);
    *ctr = reinterpret_cast<unsigned*>(c);
  }
  int bn_coef_eval(std::string name, int C, uintptr_t gamma, uintptr_t beta, float eps, uintptr_t mean,
                   uintptr_t var, float debias, uintptr_t scale, uintptr_t shift, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_coef_eval)(C, P<const float>(gamma), P<const float>(beta), eps, P<const float>(mean),
                              P<const float>(var), debias, P<float>(scale), P<float>(shift), s);
    });
  }
  int bn_apply_act(std::string name, uintptr_t x, uintptr_t y, uintptr_t scale, uintptr_t shift, int R, int C,
                   int rows_per_group, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_apply_act)(P<const elem_t>(x), P<elem_t>(y), P<const float>(scale), P<const float>(shift), R, C,
                              rows_per_group, act, leak, s);
    });
  }
  int bn_bwd_finalize(std::string name, uintptr_t part, int ppg, int groups, int C, float count, uintptr_t gamma,
                      uintptr_t mean, uintptr_t rstd, uintptr_t dgamma, uintptr_t dbeta, uintptr_t coef,
                      int stream) {
    if (use_rows_fin()) {
      const int PS = rows_slices(ppg, C);
      double* ws = nullptr;
      unsigned* ctr = nullptr;
      alloc_split(&ws, &ctr, (size_t)groups * PS * 2 * C, 1);
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bn_finalize_rows)(1, P<const float>(part), ppg, groups, C, (double)count, P<const float>(gamma),
                                        nullptr, 0.f, P<float>(mean), P<float>(rstd), nullptr, nullptr, nullptr,
                                        nullptr, 0.f, P<float>(dgamma), P<float>(dbeta), P<float>(coef), ws, ctr, PS,
                                        s);
      });
    }
    int PS = split_slices(ppg);
    if (PS > 1) {
      double* ws = nullptr;
      unsigned* ctr = nullptr;
      alloc_split(&ws, &ctr, (size_t)groups * PS * 2 * C, (size_t)((C + 15) / 16));
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bn_bwd_finalize_split)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                             P<const float>(mean), P<const float>(rstd), P<float>(dgamma),
                                             P<float>(dbeta), P<float>(coef), ws, ctr, PS, s);
      });
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_bwd_finalize)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                 P<const float>(mean), P<const float>(rstd), P<float>(dgamma), P<float>(dbeta),
                                 P<float>(coef), s);
    });
  }
  int bn_bwd_apply(std::string name, uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t coef, uintptr_t dx, int R,
                   int C, int rows_per_group, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_bwd_apply)(P<const elem_t>(dy), P<const elem_t>(y), P<const elem_t>(x), P<const float>(coef),
                              P<elem_t>(dx), R, C, rows_per_group, act, leak, s);
    });
  }
  int act_bwd(std::string name, uintptr_t dy, uintptr_t y, uintptr_t dx, size_t n, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_act_bwd)(P<const elem_t>(dy), P<const elem_t>(y), P<elem_t>(dx), n, act, leak, s);
    });
  }
  // dx = dy * act'(y) and db = column sums of dx in one launch (last-arrival reduction)
  int act_bwd_dbias(std::string name, uintptr_t dy, uintptr_t y, uintptr_t dx, int R, int C, int act, float leak,
                    uintptr_t db, int stream) {
    const int max_blocks = 256;  // every block bumps one arrival counter: keep the atomics few
    void* part = nullptr;
    void* ctr = nullptr;
    HIPCHECK(hipMalloc(&part, (size_t)max_blocks * C * sizeof(float)));
    HIPCHECK(hipMalloc(&ctr, sizeof(unsigned)));
    HIPCHECK(hipMemset(ctr, 0, sizeof(unsigned)));
    dev_allocs_.push_back(part);
    dev_allocs_.push_back(ctr);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_act_bwd_dbias)(P<const elem_t>(dy), P<const elem_t>(y), P<elem_t>(dx), R, C, act, leak,
                                   reinterpret_cast<float*>(part), max_blocks, reinterpret_cast<unsigned*>(ctr),
                                   P<float>(db), s);
    });
  }

  // D head backward (weight + bias + data gradient) in one launch
  // bx != 0: also the BN-backward partial statistics of the top BN layer -> part
  // [groups * (K / C)][2][C] (see head_bwd_kernel); dW / db / x may be 0 (g_loss chain: dgrad only)
  int head_bwd(std::string name, uintptr_t x, uintptr_t dl, uintptr_t w, uintptr_t dx, uintptr_t dW, uintptr_t db,
               int R, int K, int stream, uintptr_t bx, uintptr_t by, uintptr_t mean, uintptr_t rstd, int C, int rpg,
               int act, float leak, uintptr_t part) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_bwd)(P<const elem_t>(x), P<const float>(dl), P<const float>(w), P<elem_t>(dx), P<float>(dW),
                              P<float>(db), R, K, P<const elem_t>(bx), P<const elem_t>(by), P<const float>(mean),
                              P<const float>(rstd), C, rpg, act, leak, P<float>(part), s);
    });
  }

  int sum_partials(std::string name, uintptr_t part, int Pn, int stride, int C, uintptr_t dst, int stream) {
    const int PS = split_slices(Pn);
    if (PS > 1) {  // many rows: sliced + last-arrival combine
      void* ws = nullptr;
      void* ctr = nullptr;
      HIPCHECK(hipMalloc(&ws, (size_t)PS * C * sizeof(float)));
      HIPCHECK(hipMalloc(&ctr, (size_t)((C + 15) / 16) * sizeof(unsigned)));
      HIPCHECK(hipMemset(ctr, 0, (size_t)((C + 15) / 16) * sizeof(unsigned)));
      dev_allocs_.push_back(ws);
      dev_allocs_.push_back(ctr);
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_sum_partials_split)(P<const float>(part), Pn, stride, C, P<float>(dst),
                                          reinterpret_cast<float*>(ws), reinterpret_cast<unsigned*>(ctr), PS, s);
      });
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_sum_partials)(P<const float>(part), Pn, stride, C, P<float>(dst), s);
    });
  }
  int colsum_small(std::string name, uintptr_t x, int R, int C, uintptr_t part, int blocks, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_colsum_small)(P<const elem_t>(x), R, C, P<float>(part), blocks, s);
    });
  }

  // ------------------------------------------------------------------ heads, losses, optimiser
  int gan_loss(std::string name, uintptr_t logits, int B, uintptr_t out, uintptr_t dl_d, uintptr_t dl_g,
               uintptr_t prob, int stream, uintptr_t ls) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_gan_loss)(P<const float>(logits), B, P<float>(out), P<float>(dl_d), P<float>(dl_g),
                          P<float>(prob), P<const float>(ls), s);
    });
  }
  // stats (optional): BN partial statistics of the output, channel = column % C ->
  // [(B / 8) * (N / C)][2][C] partial rows (the row block of the kernel is 8)
  // gen_step != 0: z ~ U(-1,1) generated in-kernel (Philox keyed by gen_seed and the device
  // step counter, identical to philox_uniform) and written to z
  int linear_fwd(std::string name, uintptr_t z, uintptr_t W, uintptr_t b, uintptr_t out, int B, int K, int N,
                 int stream, uintptr_t stats = 0, int C = 0, uintptr_t gen_step = 0, uint64_t gen_seed = 0) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_linear_fwd)(P<float>(z), P<const float>(W), P<const float>(b), P<elem_t>(out), B, K, N,
                                P<float>(stats), C, P<const unsigned long long>(gen_step), gen_seed, s);
    });
  }
  int linear_wgrad(std::string name, uintptr_t z, uintptr_t dh, uintptr_t dW, uintptr_t db, int B, int K, int N,
                   int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_linear_wgrad)(P<const float>(z), P<const elem_t>(dh), P<float>(dW), P<float>(db), B, K, N, s);
    });
  }
  // loss_out != 0: the 3-loss BCE (gan_loss) runs in the GEMV's last-arriving block
  int gemv_head(std::string name, uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t out, int R, int K, int stream,
                uintptr_t loss_out, uintptr_t dl_d, uintptr_t dl_g, uintptr_t prob, uintptr_t ls) {
    unsigned* ctr = nullptr;
    if (loss_out) {
      void* c = nullptr;
      HIPCHECK(hipMalloc(&c, sizeof(unsigned)));
      HIPCHECK(hipMemset(c, 0, sizeof(unsigned)));
      dev_allocs_.push_back(c);
      ctr = reinterpret_cast<unsigned*>(c);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_gemv_head)(P<const elem_t>(x), P<const float>(w), P<const float>(b), P<float>(out), R, K, ctr,
                               P<float>(loss_out), P<float>(dl_d), P<float>(dl_g), P<float>(prob), P<const float>(ls),
                               s);
    });
  }
  int head_dgrad(std::string name, uintptr_t dl, uintptr_t w, uintptr_t dx, int R, int K, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_dgrad)(P<const float>(dl), P<const float>(w), P<elem_t>(dx), R, K, s);
    });
  }
  int head_wgrad(std::string name, uintptr_t x, uintptr_t dl, uintptr_t part, int R, int K, int splits,
                 uintptr_t dW, uintptr_t db, int stream) {
    add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_wgrad)(P<const elem_t>(x), P<const float>(dl), P<float>(part), R, K, splits, s);
    });
    add(name + ".reduce", stream, [=](hipStream_t s) {
      return KF(dcg_splitk_reduce)(P<const float>(part), splits, (size_t)K, P<float>(dW), 1.f, s);
    });
    return add(name + ".bias", stream, [=](hipStream_t s) { return KF(dcg_sum_vec)(P<const float>(dl), R, P<float>(db), s); });
  }
  int adam(std::string name, uintptr_t w, uintptr_t g, uintptr_t m, uintptr_t v, uintptr_t powers, size_t n, float lr,
           float b1, float b2, float eps, float gscale, int stream) {
    return adam_bf(name, w, 0, g, m, v, powers, n, lr, b1, b2, eps, gscale, stream, 0);
  }
  // + elem_t mirror of the updated weights (same flat layout)
  int adam_bf(std::string name, uintptr_t w, uintptr_t wbf, uintptr_t g, uintptr_t m, uintptr_t v, uintptr_t powers,
              size_t n, float lr, float b1, float b2, float eps, float gscale, int stream, uintptr_t ls) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_adam)(P<float>(w), P<elem_t>(wbf), P<const float>(g), P<float>(m), P<float>(v), P<const float>(powers),
                      n, lr, b1, b2, eps, gscale, P<const float>(ls), s);
    });
  }
  // both TF-Adams (A first) + beta powers / step counter in one launch (see adam2_kernel)
  int adam2(std::string name, uintptr_t wA, uintptr_t wbfA, uintptr_t gA, uintptr_t mA, uintptr_t vA, uintptr_t pA,
            size_t nA, float lrA, float b1A, float b2A, float epsA, uintptr_t wD, uintptr_t wbfD, uintptr_t gD,
            uintptr_t mD, uintptr_t vD, uintptr_t pD, size_t nD, float lrD, float b1D, float b2D, float epsD,
            float gscale, uintptr_t step, int stream) {
    void* ctr = nullptr;
    HIPCHECK(hipMalloc(&ctr, sizeof(unsigned)));
    HIPCHECK(hipMemset(ctr, 0, sizeof(unsigned)));
    dev_allocs_.push_back(ctr);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_adam2)(P<float>(wA), P<elem_t>(wbfA), P<const float>(gA), P<float>(mA), P<float>(vA), P<float>(pA),
                           nA, lrA, b1A, b2A, epsA, P<float>(wD), P<elem_t>(wbfD), P<const float>(gD), P<float>(mD),
                           P<float>(vD), P<float>(pD), nD, lrD, b1D, b2D, epsD, gscale,
                           P<unsigned long long>(step), reinterpret_cast<unsigned*>(ctr), s);
    });
  }
  // TF-SAME stride-2 5x5 conv with 1..4 input and 64 output channels (direct MFMA kernel, conv3.hip)
  int conv3_direct(std::string name, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int H, int W,
                   int Cin, int Ho, int Wo, int Cout, int pad_y, int pad_x, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_conv3_direct)(P<const elem_t>(x), P<const elem_t>(w), P<const float>(bias), P<elem_t>(y), B, H,
                                  W, Cin, Ho, Wo, Cout, pad_y, pad_x, act, leak, s);
    });
  }
  // TF-SAME stride-2 5x5 conv_transpose with 1..4 output channels (direct VALU kernel)
  int narrow_deconv(std::string name, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int Hi, int Wi,
                    int C, int Ho, int Wo, int N, int pad, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_narrow_deconv)(P<const elem_t>(x), P<const elem_t>(w), P<const float>(bias), P<elem_t>(y), B, Hi,
                                   Wi, C, Ho, Wo, N, pad, act, leak, s);
    });
  }
  // dynamic loss scaling: flag ls[1] if any gradient is non-finite
  int nonfinite_check(std::string name, uintptr_t g, size_t n, uintptr_t ls, int stream) {
    return add(name, stream, [=](hipStream_t s) { return KF(dcg_nonfinite_check)(P<const float>(g), n, P<float>(ls), s); });
  }
  int step_end(std::string name, uintptr_t pd, uintptr_t pg, float b1d, float b2d, float b1g, float b2g,
               uintptr_t step, int stream, uintptr_t ls, int growth_interval) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_step_end)(P<float>(pd), P<float>(pg), b1d, b2d, b1g, b2g, P<unsigned long long>(step), P<float>(ls),
                          growth_interval, s);
    });
  }
  int pack(std::string name, uintptr_t src, int T, int A, int Bd, uintptr_t nat, uintptr_t tr, int st, int sb, int sa,
           int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_pack)(P<const float>(src), T, A, Bd, P<elem_t>(nat), P<elem_t>(tr), st, sb, sa, s);
    });
  }
  int philox_uniform(std::string name, uintptr_t out, size_t n, uint64_t seed, uintptr_t step, uint64_t stream_id,
                     float lo, float hi, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_philox_uniform)(P<float>(out), n, seed, P<const unsigned long long>(step), stream_id, lo, hi, s);
    });
  }
  int im2col_s2(std::string name, uintptr_t src, uintptr_t dst, int Bn, int H, int W, int C, int Ho, int Wo, int pl_y,
                int pl_x, int Kpad, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_im2col_s2)(P<const elem_t>(src), P<elem_t>(dst), Bn, H, W, C, Ho, Wo, pl_y, pl_x, Kpad, s);
    });
  }
  int cast_to_bf16(std::string name, uintptr_t src, int src_dtype, uintptr_t dst, size_t n, float scale, float shift,
                   int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_cast_to_bf16)(P<const void>(src), src_dtype, P<elem_t>(dst), n, scale, shift, s);
    });
  }
  int cast_bf16_f32(std::string name, uintptr_t src, uintptr_t dst, size_t n, int stream) {
    return add(name, stream, [=](hipStream_t s) { return KF(dcg_cast_bf16_f32)(P<const elem_t>(src), P<float>(dst), n, s); });
  }
  int splitk_reduce(std::string name, uintptr_t src, int splits, size_t n, uintptr_t dst, float scale, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_splitk_reduce)(P<const float>(src), splits, n, P<float>(dst), scale, s);
    });
  }

 private:
  int add(const std::string& name, int stream, std::function<int(hipStream_t)> fn) {
    ops_.push_back(Op{name, stream, std::move(fn)});
    return (int)ops_.size() - 1;
  }
  std::vector<Op> ops_;
  std::vector<void*> dev_allocs_;
  std::vector<hipEvent_t> events_;
  int last_mtiles_ = 0, last_nphases_ = 0;
  bool f16_ = false;  // element type of every activation / weight-mirror pointer: fp16, else bf16
};

static py::tuple igemm_tile(int cfg) {
  if (cfg >= 200) {
    int bm, bn, ns;
    if (dcg_igemm3_tile(cfg, &bm, &bn, &ns)) throw std::runtime_error("bad cfg");
    return py::make_tuple(bm, bn);
  }
  int bm = 0, bn = 0;
  if (dcg_igemm_tile(cfg, &bm, &bn)) throw std::runtime_error("bad cfg");
  return py::make_tuple(bm, bn);
}
static py::tuple wgrad_tile(int cfg) {
  int bm = 0, bn = 0, ns = 0;
  if (cfg >= 300) {
    if (dcg_wgrad3_tile(cfg, &bm, &bn, &ns)) throw std::runtime_error("bad cfg");
    return py::make_tuple(bm, bn);
  }
  if (dcg_wgrad_tile(cfg, &bm, &bn)) throw std::runtime_error("bad cfg");
  return py::make_tuple(bm, bn);
}

static std::string device_arch() {
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess) return "";
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return "";
  return std::string(prop.gcnArchName);
}

PYBIND11_MODULE(_dcgan_hip, m) {
  m.doc() = "gfx950 (MI355X) kernel library + recorded launch programs for the DCGAN framework";
  m.def("igemm_tile", &igemm_tile);
  m.def("wgrad_tile", &wgrad_tile);
  m.def("device_arch", &device_arch);
  m.attr("built_for") = "gfx950";
  py::class_<Program>(m, "Program")
      .def(py::init<bool>(), py::arg("f16") = false)
      .def_property_readonly("f16", &Program::f16)
      .def("size", &Program::size)
      .def("name", &Program::name)
      .def("run", &Program::run, py::arg("streams"), py::arg("begin") = 0, py::arg("end") = -1)
      .def("new_event", &Program::new_event)
      .def("record", &Program::record)
      .def("wait", &Program::wait)
      .def("memset", &Program::memset)
      .def("copy", &Program::copy)
      .def("igemm", &Program::igemm)
      .def("igemm_ex", &Program::igemm_ex, py::arg("name"), py::arg("mode"), py::arg("A"), py::arg("Bw"), py::arg("C"),
           py::arg("Bn"), py::arg("Hin"), py::arg("Win"), py::arg("Kc"), py::arg("Hout"), py::arg("Wout"), py::arg("N"),
           py::arg("pad_y"), py::arg("pad_x"), py::arg("cfg"), py::arg("out_f32"), py::arg("ldc"), py::arg("cofs"),
           py::arg("bias"), py::arg("act"), py::arg("leak"), py::arg("stats"), py::arg("stream"), py::arg("bkn"),
           py::arg("kb_valid"), py::arg("splits"), py::arg("bnb_x") = 0, py::arg("bnb_y") = 0,
           py::arg("bnb_mean") = 0, py::arg("bnb_rstd") = 0, py::arg("bnb_rpg") = 0, py::arg("bnb_act") = 0,
           py::arg("bnb_leak") = 0.f, py::arg("bnb_store_g") = 0)
      .def("last_mtiles", &Program::last_mtiles)
      .def("last_nphases", &Program::last_nphases)
      .def("wgrad", &Program::wgrad)
      .def("wgrad3", &Program::wgrad3)
      .def("colstats", &Program::colstats)
      .def("bn_finalize", &Program::bn_finalize)
      .def("bn_coef_eval", &Program::bn_coef_eval)
      .def("bn_apply_act", &Program::bn_apply_act)
      .def("bn_bwd_finalize", &Program::bn_bwd_finalize)
      .def("bn_bwd_apply", &Program::bn_bwd_apply)
      .def("act_bwd", &Program::act_bwd)
      .def("sum_partials", &Program::sum_partials)
      .def("act_bwd_dbias", &Program::act_bwd_dbias)
      .def("head_bwd", &Program::head_bwd, py::arg("name"), py::arg("x"), py::arg("dl"), py::arg("w"), py::arg("dx"),
           py::arg("dW"), py::arg("db"), py::arg("R"), py::arg("K"), py::arg("stream"), py::arg("bx") = 0,
           py::arg("by") = 0, py::arg("mean") = 0, py::arg("rstd") = 0, py::arg("C") = 0, py::arg("rpg") = 0,
           py::arg("act") = 0, py::arg("leak") = 0.f, py::arg("part") = 0)
      .def("colsum_small", &Program::colsum_small)
      .def("gan_loss", &Program::gan_loss, py::arg("name"), py::arg("logits"), py::arg("B"), py::arg("out"),
           py::arg("dl_d"), py::arg("dl_g"), py::arg("prob"), py::arg("stream"), py::arg("ls") = 0)
      .def("linear_fwd", &Program::linear_fwd, py::arg("name"), py::arg("z"), py::arg("W"), py::arg("b"),
           py::arg("out"), py::arg("B"), py::arg("K"), py::arg("N"), py::arg("stream"), py::arg("stats") = 0,
           py::arg("C") = 0, py::arg("gen_step") = 0, py::arg("gen_seed") = 0)
      .def("linear_wgrad", &Program::linear_wgrad)
      .def("gemv_head", &Program::gemv_head, py::arg("name"), py::arg("x"), py::arg("w"), py::arg("b"), py::arg("out"),
           py::arg("R"), py::arg("K"), py::arg("stream"), py::arg("loss_out") = 0, py::arg("dl_d") = 0,
           py::arg("dl_g") = 0, py::arg("prob") = 0, py::arg("ls") = 0)
      .def("head_dgrad", &Program::head_dgrad)
      .def("head_wgrad", &Program::head_wgrad)
      .def("adam", &Program::adam)
      .def("adam_bf", &Program::adam_bf, py::arg("name"), py::arg("w"), py::arg("wbf"), py::arg("g"), py::arg("m"),
           py::arg("v"), py::arg("powers"), py::arg("n"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
           py::arg("gscale"), py::arg("stream"), py::arg("ls") = 0)
      .def("step_end", &Program::step_end, py::arg("name"), py::arg("pd"), py::arg("pg"), py::arg("b1d"),
           py::arg("b2d"), py::arg("b1g"), py::arg("b2g"), py::arg("step"), py::arg("stream"), py::arg("ls") = 0,
           py::arg("growth_interval") = 2000)
      .def("adam2", &Program::adam2)
      .def("nonfinite_check", &Program::nonfinite_check)
      .def("narrow_deconv", &Program::narrow_deconv)
      .def("conv3_direct", &Program::conv3_direct)
      .def("pack", &Program::pack)
      .def("philox_uniform", &Program::philox_uniform)
      .def("im2col_s2", &Program::im2col_s2)
      .def("cast_to_bf16", &Program::cast_to_bf16)
      .def("cast_bf16_f32", &Program::cast_bf16_f32)
      .def("splitk_reduce", &Program::splitk_reduce);
}
