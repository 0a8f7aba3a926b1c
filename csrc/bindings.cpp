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
// Every op also records the device byte ranges it reads and writes (`accesses`). The schedule
// checker (engine/schedule_check.py) walks a whole training step -- programs, cross-stream
// events, collectives -- and proves that no two ops on unordered streams touch overlapping
// bytes with at least one write. A Program built with dry=true records ops and accesses but
// allocates nothing on the device (workspaces get disjoint fake addresses) and cannot run:
// that is how the checker runs on a CPU-only machine.
//
// Element type per Program: 0 = bf16, 1 = fp16, 2 = fp32 (the reference-precision build).
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
#include <tuple>
#include <vector>

#include "hip/kernels.h"
#include "comm.h"
extern "C" {
#include "hip/narrow2.inc"
}

// The fp16 and fp32 builds of the same kernels (csrc/build.py compiles every .hip three times):
// identical C signatures (element pointers are void-compatible at the ABI level) with `_f16` /
// `_f32` suffixes.
#undef DCG_API
#define DCG_API(name) name##_f16
extern "C" {
#include "hip/launchers.inc"
#include "hip/narrow2.inc"
}
#undef DCG_API
#define DCG_API(name) name##_f32
extern "C" {
#include "hip/launchers.inc"
#include "hip/narrow2.inc"
}
#undef DCG_API
#define DCG_API(name) name

// launcher of the Program's element type (bf16, fp16 or fp32)
#define KF(fn) (dt_ == 2 ? fn##_f32 : dt_ == 1 ? fn##_f16 : fn)

extern "C" int dcg_comm_emulate(const void* src, void* dst, size_t bytes, double us, int nwg, hipStream_t s);

namespace py = pybind11;
using namespace dcg;

#define HIPCHECK(x)                                                                             \
  do {                                                                                          \
    hipError_t e__ = (x);                                                                       \
    if (e__ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e__)); \
  } while (0)

template <class T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

struct Acc {
  uintptr_t p;
  size_t n;
  bool w;
};

enum OpKind { OP_LAUNCH = 0, OP_RECORD = 1, OP_WAIT = 2 };

struct Op {
  std::string name;
  int stream;  // slot
  int kind;
  int event;
  std::vector<Acc> acc;
  std::function<int(hipStream_t)> fn;
};

// access-list builder: null pointers / empty ranges are dropped
struct AccList {
  std::vector<Acc> v;
  AccList& r(uintptr_t p, size_t n) { if (p && n) v.push_back({p, n, false}); return *this; }
  AccList& w(uintptr_t p, size_t n) { if (p && n) v.push_back({p, n, true}); return *this; }
};

class Program {
 public:
  explicit Program(int dtype = 0, bool dry = false) : dt_(dtype), dry_(dry) {
    if (dtype < 0 || dtype > 2) throw std::runtime_error("Program dtype must be 0 (bf16), 1 (fp16) or 2 (fp32)");
    es_ = dtype == 2 ? 4 : 2;
  }
  int dtype() const { return dt_; }
  bool f16() const { return dt_ == 1; }
  bool dry() const { return dry_; }
  int elem_size() const { return (int)es_; }

  ~Program() {
    if (dry_) return;
    for (void* p : dev_allocs_) (void)hipFree(p);
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  }

  int size() const { return (int)ops_.size(); }
  std::string name(int i) const { return ops_.at(i).name; }

  // (name, stream slot, kind, event, [(ptr, bytes, is_write), ...]) of op i
  py::tuple op_info(int i) const {
    const Op& o = ops_.at(i);
    py::list acc;
    for (const Acc& a : o.acc) acc.append(py::make_tuple(a.p, a.n, a.w));
    return py::make_tuple(o.name, o.stream, o.kind, o.event, acc);
  }

  void run(std::vector<uintptr_t> streams, int begin, int end) {
    if (dry_) throw std::runtime_error("a dry Program records only; it cannot run");
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
    hipEvent_t e = nullptr;
    if (!dry_) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    events_.push_back(e);
    return (int)events_.size() - 1;
  }
  int record(int ev, int stream) {
    hipEvent_t e = events_.at(ev);
    return add("record", stream, [e](hipStream_t s) { return (int)hipEventRecord(e, s); }, {}, OP_RECORD, ev);
  }
  int wait(int ev, int stream) {
    hipEvent_t e = events_.at(ev);
    return add("wait", stream, [e](hipStream_t s) { return (int)hipStreamWaitEvent(s, e, 0); }, {}, OP_WAIT, ev);
  }
  int memset(uintptr_t ptr, size_t bytes, int stream) {
    void* p = reinterpret_cast<void*>(ptr);
    return add("memset", stream, [p, bytes](hipStream_t s) { return (int)hipMemsetAsync(p, 0, bytes, s); },
               AccList().w(ptr, bytes).v);
  }
  int copy(uintptr_t dst, uintptr_t src, size_t bytes, int stream) {
    void* d = reinterpret_cast<void*>(dst);
    const void* sp = reinterpret_cast<const void*>(src);
    return add("copy", stream, [d, sp, bytes](hipStream_t s) {
      return (int)hipMemcpyAsync(d, sp, bytes, hipMemcpyDeviceToDevice, s);
    }, AccList().r(src, bytes).w(dst, bytes).v);
  }

  // in-place SUM all-reduce of `count` elements (dtype 0 fp32 / 1 bf16 / 2 fp16) over a native
  // RCCL communicator (comm.h), enqueued on the op's stream: a collective the C++ replay (and a
  // hipGraph capture) issues in program order with the kernels, no Python in between
  int allreduce(const std::string& name, std::shared_ptr<dcg_comm::Comm> comm, uintptr_t ptr, size_t count, int dtype,
                int stream) {
    const size_t es = dtype == 0 ? 4 : 2;
    dcg_comm::Comm* c = comm.get();
    comms_.push_back(comm);  // keep the communicator alive as long as the program
    return add(name, stream, [c, ptr, count, dtype](hipStream_t s) {
      c->all_reduce(ptr, count, dtype, reinterpret_cast<uintptr_t>(s));
      return 0;
    }, AccList().w(ptr, count * es).v);
  }

  // RCCL stand-in for schedule studies (csrc/hip/comm_emu.hip): nwg workgroups copy `bytes` from
  // src to dst through HBM, paced to take `us` microseconds
  int comm_emulate(const std::string& name, uintptr_t src, uintptr_t dst, size_t bytes, double us, int nwg,
                   int stream) {
    const void* sp = reinterpret_cast<const void*>(src);
    void* d = reinterpret_cast<void*>(dst);
    return add(name, stream, [sp, d, bytes, us, nwg](hipStream_t s) { return dcg_comm_emulate(sp, d, bytes, us, nwg, s); },
               AccList().r(src, bytes).w(dst, bytes).v);
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
  // The fp32 build has one tile family (igemm_f32.hip) behind the same entry points.
  int igemm_ex(std::string name, int mode, uintptr_t A, uintptr_t Bw, uintptr_t C, int Bn, int Hin, int Win, int Kc,
               int Hout, int Wout, int N, int pad_y, int pad_x, int cfg, int out_f32, int ldc, int cofs,
               uintptr_t bias, int act, float leak, uintptr_t stats, int stream, int bkn, int kb_valid, int splits,
               uintptr_t bnb_x = 0, uintptr_t bnb_y = 0, uintptr_t bnb_mean = 0, uintptr_t bnb_rstd = 0,
               int bnb_rpg = 0, int bnb_act = 0, float bnb_leak = 0.f, int bnb_store_g = 0) {
    int bm = 0, bn = 0, ns = 0;
    const bool v3 = cfg >= 200;
    if (cfg >= 400) throw std::runtime_error("bad igemm cfg " + std::to_string(cfg));
    if (v3 ? KF(dcg_igemm3_tile)(cfg, &bm, &bn, &ns) : KF(dcg_igemm_tile)(cfg, &bm, &bn))
      throw std::runtime_error("bad igemm cfg " + std::to_string(cfg) + " for this element type");
    if (!v3 && (bkn || splits != 1)) throw std::runtime_error("igemm cfg < 200 supports neither bkn nor split-K");
    if (splits < 1) throw std::runtime_error("splits must be >= 1");
    const int kal = (int)(16 / es_);  // 16-byte A rows
    if (Kc % kal) throw std::runtime_error("igemm needs 16-byte A rows (Kc % " + std::to_string(kal) + " == 0)");
    if (bkn && N % kal) throw std::runtime_error("igemm bkn needs 16-byte B rows");
    if (kb_valid < 0) kb_valid = Kc;
    if (kb_valid > Kc) throw std::runtime_error("kb_valid > Kc");
    std::vector<IGemmPhase> ph;
    IGemmArgs a{};
    a.A = P<const elem_t>(A); a.Bn = Bn; a.H = Hin; a.W = Win; a.Kc = Kc;
    a.Bw = P<const elem_t>(Bw); a.N = N;
    a.C = P<void>(C); a.out_f32 = out_f32; a.outH = Hout; a.outW = Wout; a.ldc = ldc; a.cofs = cofs;
    a.bias = P<const float>(bias); a.act = act; a.leak = leak; a.stats = P<float>(stats);
    size_t a_elems, b_elems, c_rows;
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
      c_rows = (size_t)Bn * Hout * Wout;
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
      c_rows = (size_t)Bn * Hout * Wout;
    } else if (mode == 2) {
      a.sstride = 1; a.plain = 1; a.ostride = 1;
      IGemmPhase p{};
      p.Hq = 1; p.Wq = 1; p.M = Bn * Hout * Wout; p.ntaps = 1;
      p.fd_hw = fastdiv_make(1); p.fd_w = fastdiv_make(1);
      ph.push_back(p);
      a_elems = (size_t)p.M * Kc; b_elems = bkn ? (size_t)kb_valid * N : (size_t)N * Kc;
      c_rows = (size_t)p.M;
    } else {
      throw std::runtime_error("bad igemm mode");
    }
    if (a_elems * es_ >= OOB || b_elems * es_ >= OOB)
      throw std::runtime_error("igemm operand exceeds the 3.875 GiB buffer-descriptor range");
    a.a_bytes = (uint32_t)(a_elems * es_); a.b_bytes = (uint32_t)(b_elems * es_);
    for (auto& q : ph)
      for (int t = 0; t < q.ntaps; ++t)
        q.tap[t] = (q.dy[t] & 0xff) | ((q.dx[t] & 0xff) << 8) | ((int)q.wtap[t] << 16);
    // deconv phases by decreasing tap count (9 / 6 / 6 / 4): the longest-first dispatch order then
    // runs the long phases first; the phase order is otherwise free (each phase carries its own
    // output offsets; the BN partial rows are summed over all of them)
    std::stable_sort(ph.begin(), ph.end(), [](const IGemmPhase& x, const IGemmPhase& y) { return x.ntaps > y.ntaps; });
    a.nphases = (int)ph.size();
    if (a.nphases > 4) throw std::runtime_error("igemm: more than 4 phases");
    {
      // longest phase first (igemm3, mode 1): +0.7 % at 64x64, +5.3 % at 256x256 fp16 over the
      // interleaved phase order (profiles/r5/ab_igemm_lpt_r5.txt); DCGAN_IGEMM_LPT=0 restores it
      const char* e = std::getenv("DCGAN_IGEMM_LPT");
      a.lpt = (e && e[0] == '0') ? 0 : 1;
    }
    for (int i = 0; i < a.nphases; ++i) {
      const IGemmPhase& q = ph[i];
      IGemmPhaseK& k = a.phk[i];
      k.Hq = q.Hq; k.Wq = q.Wq; k.M = q.M; k.iy0_off = q.iy0_off; k.ix0_off = q.ix0_off;
      k.oy_off = q.oy_off; k.ox_off = q.ox_off; k.ntaps = q.ntaps; k.fd_hw = q.fd_hw; k.fd_w = q.fd_w;
      for (int t = 0; t < 25; ++t) k.tap[t] = q.tap[t];
    }
    if (cfg >= 300) {
      // halo K loop (igemm3.hip PP == 2): deconv phases, k-contiguous weights, whole 64-channel
      // chunks (split-K over chunks); every phase tile covers whole images or whole rows of one
      // image, and its input window (every tap's rows) fits the 224-pixel buffer (HALO_WPW x 4 x 8)
      if (mode != 1 || bkn || Kc % 64 || splits > Kc / 64)
        throw std::runtime_error("igemm halo cfg: deconv mode, k-contiguous weights, Kc % 64, splits <= Kc / 64");
      for (auto& q : ph) {
        const int hw = q.Hq * q.Wq;
        const bool whole = bm % hw == 0, rows = hw % bm == 0 && bm % q.Wq == 0;
        const int nimg = whole ? bm / hw : 1, R = whole ? q.Hq : bm / std::max(1, q.Wq);
        if ((!whole && !rows) || nimg * (R + 2) * (q.Wq + 2) > 224)
          throw std::runtime_error("igemm halo cfg: phase tile is not whole images / rows, or its window exceeds 224 pixels");
      }
    }
    int maxM = 0;
    for (auto& p : ph) maxM = std::max(maxM, p.M);
    const int mtiles = (maxM + bm - 1) / bm, ntiles = (N + bn - 1) / bn;
    a.mtiles = mtiles;
    a.ph = reinterpret_cast<const IGemmPhase*>(dev_alloc(ph.size() * sizeof(IGemmPhase), ph.data()));
    last_mtiles_ = mtiles;
    last_nphases_ = a.nphases;
    a.kb_valid = kb_valid;
    a.splits = splits;
    {
      // XCD locality (igemm3): each of the 8 XCDs runs a contiguous eighth of the tiles. M slowest
      // (default): a run spans whole tile rows -- 1/8 of the activations, all weight columns; N
      // slowest: the reverse. Per-XCD footprint of a run of T/8 tiles (T = mtiles x ntiles):
      //   M slowest: A/8 + B        (T/8 >= ntiles), else A/mtiles + B*mtiles/8
      //   N slowest: A + B/8        (T/8 >= mtiles), else A*ntiles/8 + B/ntiles
      // N slowest when that is clearly smaller (weight-heavy layers: G's 4x4 -> 8x8 deconv reads
      // 6.5 MB of weights against 2 MB of input). DCGAN_IGEMM_NMAJOR=0 / 1 forces the order.
      const double A_ = (double)a.a_bytes, B_ = (double)a.b_bytes, T8 = (double)mtiles * ntiles / 8.0;
      const double fm = T8 >= ntiles ? A_ / 8 + B_ : A_ / mtiles + B_ * mtiles / 8.0;
      const double fn = T8 >= mtiles ? A_ + B_ / 8 : A_ * ntiles / 8.0 + B_ / ntiles;
      a.nmajor = fn < 0.8 * fm ? 1 : 0;
      if (const char* e = std::getenv("DCGAN_IGEMM_NMAJOR")) a.nmajor = e[0] == '1' ? 1 : (e[0] == '0' ? 0 : a.nmajor);
    }
    const size_t out_es = out_f32 ? 4 : es_;
    AccList acc;
    acc.r(A, a_elems * es_).r(Bw, b_elems * es_).r(bias, (size_t)N * 4)
        .w(C, (c_rows - 1) * ldc * out_es + (size_t)(cofs + N) * out_es)
        .w(stats, (size_t)mtiles * a.nphases * 2 * N * 4);
    if (bnb_x) {
      size_t lds = (size_t)(v3 ? ns : 2) * (bm + bn) * 128;
      if (dt_ == 2) throw std::runtime_error("igemm bnb: not available in the fp32 build");
      const size_t nt = v3 ? (size_t)KF(dcg_igemm3_threads)(cfg) : 256;
      // igemm3 (waves along M per tile id, igemm3.hip DCG_IGEMM3_TILES): the row-lane scratch may
      // alias the C tile; v1 keeps them apart
      static const int kWM3[10] = {2, 4, 1, 2, 2, 2, 4, 2, 8, 4};
      const size_t wm = v3 ? (size_t)kWM3[cfg % 10] : 4;
      const size_t ct = (size_t)bm * (bn + 8) * 2, r2 = 64 * nt;
      if (v3) lds = std::max(lds, (bm + 2 * wm * bn) * 4 + ct);  // igemm3_lds_bytes
      const size_t need = (bm + 2 * wm * bn) * 4 + (v3 ? std::max(ct, r2) : ct + r2);
      if (need > lds || out_f32 || N % 8 || ldc % 8 || cofs % 8)
        throw std::runtime_error("igemm bnb: tile has no LDS for the fused statistics or output is not vectorizable");
      const size_t xy_bytes = (c_rows - 1) * ldc * es_ + (size_t)(cofs + N) * es_;
      if (bnb_store_g) {  // activation backward only (no BN): x, mean, rstd and groups unused
        if (!stats || !bnb_y) throw std::runtime_error("igemm act-backward store: needs stats and y");
        a.bnb_x = P<const elem_t>(bnb_y); a.bnb_y = P<const elem_t>(bnb_y);
        a.bnb_rpg = 1 << 30; a.bnb_act = bnb_act; a.bnb_leak = bnb_leak; a.bnb_store_g = 1;
        acc.r(bnb_y, xy_bytes);
      } else {
        if (!stats || bnb_rpg <= 0 || !bnb_y || !bnb_mean || !bnb_rstd)
          throw std::runtime_error("igemm bnb: needs stats, rows-per-group, y, mean, rstd");
        for (auto& q : ph)  // tiles must not straddle a BN group (a phase's rows are (b, qy, qx))
          if (bnb_rpg % bm || q.M % bnb_rpg) throw std::runtime_error("igemm bnb: tile rows must divide the group");
        a.bnb_x = P<const elem_t>(bnb_x); a.bnb_y = P<const elem_t>(bnb_y);
        a.bnb_mean = P<const float>(bnb_mean); a.bnb_rstd = P<const float>(bnb_rstd);
        a.bnb_rpg = bnb_rpg; a.bnb_act = bnb_act; a.bnb_leak = bnb_leak;
        const size_t groups = (size_t)(maxM / bnb_rpg);
        acc.r(bnb_x, xy_bytes).r(bnb_y, xy_bytes).r(bnb_mean, groups * N * 4).r(bnb_rstd, groups * N * 4);
      }
    }
    if (const char* ab = getenv("DCGAN_IGEMM_ABLATE")) a.ablate = atoi(ab);  // kernel studies only
    if (const char* st = getenv("DCGAN_IGEMM_STAMPS")) a.stamps = reinterpret_cast<unsigned long long*>(strtoull(st, nullptr, 0));
    if (!v3) {
      return add(name, stream, [this, a, cfg, mtiles, ntiles](hipStream_t s) {
        return KF(dcg_igemm_launch)(&a, cfg, mtiles, ntiles, s);
      }, acc.v);
    }
    const size_t tiles = (size_t)mtiles * ntiles * a.nphases;
    if (splits > 1) {  // per-op workspace + zeroed arrival counters (reset by the kernel itself)
      a.ws = reinterpret_cast<float*>(dev_alloc(tiles * splits * (size_t)bm * bn * sizeof(float)));
      a.counters = reinterpret_cast<unsigned*>(dev_alloc(tiles * sizeof(unsigned), nullptr, true));
      acc.w((uintptr_t)a.ws, tiles * splits * (size_t)bm * bn * sizeof(float)).w((uintptr_t)a.counters, tiles * 4);
    }
    const unsigned blocks = (unsigned)(tiles * splits);
    return add(name, stream, [this, a, cfg, bkn, blocks](hipStream_t s) { return KF(dcg_igemm3_launch)(&a, cfg, bkn, blocks, s); },
               acc.v);
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
    if (g_elems * es_ >= OOB || d_elems * es_ >= OOB)
      throw std::runtime_error("wgrad operand exceeds the 3.875 GiB buffer-descriptor range");
    a.g_bytes = (uint32_t)(g_elems * es_); a.d_bytes = (uint32_t)(d_elems * es_);
    a.fd_hw = fastdiv_make(Hd * Wd); a.fd_w = fastdiv_make(Wd); a.Hd = Hd; a.Wd = Wd;
    const size_t n = (size_t)a.ntaps * Mc * Nc;
    if (dst_elems > n) throw std::runtime_error("wgrad dst larger than result");
    float* slab = P<float>(slabs);
    float* d = P<float>(dst);
    add(name, stream, [this, a, cfg, splits](hipStream_t s) { return KF(dcg_wgrad_launch)(&a, cfg, splits, s); },
        AccList().r(G, g_elems * es_).r(Dm, d_elems * es_).w(slabs, (size_t)splits * n * 4).v);
    // plain mode may carry padded rows (im2col K padding): reduce only the first dst_elems of
    // each slab's leading part -- rows are m-major so the valid prefix is contiguous.
    return add(name + ".reduce", stream, [this, slab, splits, n, d, dst_elems, scale](hipStream_t s) {
      if (dst_elems == n) return KF(dcg_splitk_reduce)(slab, splits, n, d, scale, s);
      // strided variant: reduce the whole slab into itself (slab 0) then copy the valid prefix
      int rc = KF(dcg_splitk_reduce)(slab, splits, n, slab, scale, s);
      if (rc) return rc;
      return (int)hipMemcpyAsync(d, slab, dst_elems * sizeof(float), hipMemcpyDeviceToDevice, s);
    }, AccList().w(slabs, (size_t)splits * n * 4).w(dst, dst_elems * 4).v);
  }

  // weight gradient v3 (wgrad3.hip): the 25-tap gather GEMM with the split-K reduction in-kernel,
  // written scaled straight into the fp32 gradient dst [25][Mc][Nc] -- one launch, no slabs pass
  int wgrad3(std::string name, uintptr_t G, int Hg, int Wg, int Mc, uintptr_t Dm, int Bn, int Hd, int Wd, int Nc,
             int pad, int cfg, int splits, uintptr_t dst, float scale, int stream) {
    int bm = 0, bn = 0, ns = 0, w5_wd = 0;
    const bool w5 = cfg >= 400;  // wgrad5.hip: one kernel row (5 taps) x all Mc x bn per workgroup
    if (w5) {
      if (KF(dcg_wgrad5_tile)(cfg, &bm, &bn, &w5_wd, &ns)) throw std::runtime_error("bad wgrad5 cfg " + std::to_string(cfg));
      if (Mc % bm || Wd != w5_wd || (Hd % (64 / w5_wd) && (64 / w5_wd) % Hd) || (Bn * Hd * Wd) % 64)
        throw std::runtime_error("wgrad5 cfg " + std::to_string(cfg) + " does not fit Mc=" + std::to_string(Mc) +
                                 " Hd=" + std::to_string(Hd) + " Wd=" + std::to_string(Wd));
    } else if (KF(dcg_wgrad3_tile)(cfg, &bm, &bn, &ns)) {
      throw std::runtime_error("bad wgrad3 cfg " + std::to_string(cfg));
    }
    const int al = (int)(16 / es_);
    if (Mc % al || Nc % al) throw std::runtime_error("wgrad3 needs 16-byte channel rows (Mc, Nc multiples of 16 bytes)");
    if (splits < 1) throw std::runtime_error("splits must be >= 1");
    WGrad3Args a{};
    a.G = P<const elem_t>(G); a.Hg = Hg; a.Wg = Wg; a.Mc = Mc;
    a.Dm = P<const elem_t>(Dm); a.Nc = Nc;
    a.K = Bn * Hd * Wd; a.pl = pad; a.splits = splits;
    const int KT = (a.K + 63) / 64;
    a.kt_per_split = (KT + splits - 1) / splits;
    const size_t g_elems = (size_t)Bn * Hg * Wg * Mc, d_elems = (size_t)a.K * Nc;
    if (g_elems * es_ >= OOB || d_elems * es_ >= OOB)
      throw std::runtime_error("wgrad3 operand exceeds the 3.875 GiB buffer-descriptor range");
    a.g_bytes = (uint32_t)(g_elems * es_); a.d_bytes = (uint32_t)(d_elems * es_);
    a.fd_hw = fastdiv_make(Hd * Wd); a.fd_w = fastdiv_make(Wd); a.Hd = Hd; a.Wd = Wd;
    auto lg2 = [](int v) { int l = 0; while ((1 << l) < v) ++l; return (1 << l) == v ? l : -1; };
    a.lhw = lg2(Hd * Wd); a.lw = lg2(Wd);
    if (a.lhw < 0 || a.lw < 0) a.lhw = a.lw = -1;  // pixel decode by shifts only for power-of-two images
    a.out = P<float>(dst); a.scale = scale;
    AccList acc;
    acc.r(G, g_elems * es_).r(Dm, d_elems * es_).w(dst, (size_t)25 * Mc * Nc * 4);
    const int tt = w5 ? 1 : KF(dcg_wgrad3_taps_per_tile)(cfg);
    if (tt == 2 && 2 * Mc != bm) throw std::runtime_error("wgrad3: two-tap tiles need BM = 2 Mc");
    // wgrad5: 5 * ceil(Nc / bn) tiles of 5 taps x Mc x bn; wgrad3: tap (group) x m x n tiles of bm x bn
    const size_t tiles = w5 ? (size_t)5 * ((Nc + bn - 1) / bn) * (Mc / bm)
                            : (size_t)(tt == 2 ? 1 : (Mc + bm - 1) / bm) * ((Nc + bn - 1) / bn) * ((25 + tt - 1) / tt);
    const size_t slab = (size_t)(w5 ? 5 : 1) * bm * bn;
    if (splits > 1) {
      if ((size_t)splits * slab * 4 >= OOB) throw std::runtime_error("wgrad3: split slabs too large");
      a.ws = reinterpret_cast<float*>(dev_alloc(tiles * splits * slab * sizeof(float)));
      acc.w((uintptr_t)a.ws, tiles * splits * slab * 4);
      if (!(w5 && cfg >= 410)) {  // wgrad5 cfg 41x: the split sum is a second kernel, no counters
        a.counters = reinterpret_cast<unsigned*>(dev_alloc(tiles * sizeof(unsigned), nullptr, true));
        acc.w((uintptr_t)a.counters, tiles * 4);
      }
    }
    if (w5) return add(name, stream, [this, a, cfg](hipStream_t s) { return KF(dcg_wgrad5_launch)(&a, cfg, s); }, acc.v);
    return add(name, stream, [this, a, cfg](hipStream_t s) { return KF(dcg_wgrad3_launch)(&a, cfg, s); }, acc.v);
  }

  // ------------------------------------------------------------------ BN / activations
  int colstats(std::string name, int mode, uintptr_t x, uintptr_t dy, uintptr_t y, uintptr_t mean, uintptr_t rstd,
               int act, float leak, int R, int C, int rows_per_block, int rows_per_group, uintptr_t part,
               int stream) {
    const size_t t = (size_t)R * C * es_;
    const int Pn = (R + rows_per_block - 1) / rows_per_block;
    const size_t groups = (size_t)((R + rows_per_group - 1) / rows_per_group);
    AccList acc;
    acc.r(x, t).w(part, (size_t)Pn * 2 * C * 4);
    if (mode == 1) acc.r(dy, t).r(y, t).r(mean, groups * C * 4).r(rstd, groups * C * 4);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_colstats)(mode, P<const elem_t>(x), P<const elem_t>(dy), P<const elem_t>(y), P<const float>(mean),
                          P<const float>(rstd), act, leak, R, C, rows_per_block, rows_per_group, P<float>(part), s);
    }, acc.v);
  }
  int bn_finalize(std::string name, uintptr_t part, int ppg, int groups, int C, double count, uintptr_t gamma,
                  uintptr_t beta, float eps, uintptr_t mean, uintptr_t rstd, uintptr_t scale, uintptr_t shift,
                  uintptr_t ema_mean, uintptr_t ema_var, float decay, int stream) {
    const size_t gc = (size_t)groups * C * 4;
    AccList acc;
    acc.r(part, (size_t)groups * ppg * 2 * C * 4).r(gamma, (size_t)C * 4).r(beta, (size_t)C * 4)
        .w(mean, gc).w(rstd, gc).w(scale, gc).w(shift, gc).w(ema_mean, gc).w(ema_var, gc);
    if (C % 4 == 0) {  // one level, all lanes on the rows (bnfin.hip; measured 1.151 vs 1.156 ms/step)
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bnfin_fwd)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                 P<const float>(beta), eps, P<float>(mean), P<float>(rstd), P<float>(scale),
                                 P<float>(shift), P<float>(ema_mean), P<float>(ema_var), decay, s);
      }, acc.v);
    }
    int PS = split_slices(ppg);
    if (PS > 1) {  // many partial rows: sliced reduction + last-arrival finalize
      double* ws = nullptr;
      unsigned* ctr = nullptr;
      alloc_split(&ws, &ctr, (size_t)groups * PS * 2 * C, (size_t)groups * ((C + 15) / 16), acc);
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bn_finalize_split)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                         P<const float>(beta), eps, P<float>(mean), P<float>(rstd), P<float>(scale),
                                         P<float>(shift), P<float>(ema_mean), P<float>(ema_var), decay, ws, ctr, PS, s);
      }, acc.v);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_finalize)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                             P<const float>(beta), eps, P<float>(mean), P<float>(rstd), P<float>(scale),
                             P<float>(shift), P<float>(ema_mean), P<float>(ema_var), decay, s);
    }, acc.v);
  }
  static int split_slices(int ppg) { return ppg > 64 ? std::min(32, (ppg + 63) / 64) : 1; }
  void alloc_split(double** ws, unsigned** ctr, size_t ws_elems, size_t counters, AccList& acc) {
    *ws = reinterpret_cast<double*>(dev_alloc(ws_elems * sizeof(double)));
    *ctr = reinterpret_cast<unsigned*>(dev_alloc(counters * sizeof(unsigned), nullptr, true));
    acc.w((uintptr_t)*ws, ws_elems * 8).w((uintptr_t)*ctr, counters * 4);
  }
  // debias_ptr (optional): device scalar multiplying the moving averages (TF zero-debiasing,
  // 1 / (1 - decay^t) written by the host before the sampler runs); else the constant debias
  int bn_coef_eval(std::string name, int C, uintptr_t gamma, uintptr_t beta, float eps, uintptr_t mean,
                   uintptr_t var, float debias, uintptr_t scale, uintptr_t shift, int stream, uintptr_t debias_ptr) {
    const size_t c4 = (size_t)C * 4;
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_coef_eval)(C, P<const float>(gamma), P<const float>(beta), eps, P<const float>(mean),
                              P<const float>(var), debias, P<const float>(debias_ptr), P<float>(scale),
                              P<float>(shift), s);
    }, AccList().r(gamma, c4).r(beta, c4).r(mean, c4).r(var, c4).r(debias_ptr, 4).w(scale, c4).w(shift, c4).v);
  }
  int bn_apply_act(std::string name, uintptr_t x, uintptr_t y, uintptr_t scale, uintptr_t shift, int R, int C,
                   int rows_per_group, int act, float leak, int stream) {
    const size_t t = (size_t)R * C * es_, gc = (size_t)((R + rows_per_group - 1) / rows_per_group) * C * 4;
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_apply_act)(P<const elem_t>(x), P<elem_t>(y), P<const float>(scale), P<const float>(shift), R, C,
                              rows_per_group, act, leak, s);
    }, AccList().r(x, t).w(y, t).r(scale, gc).r(shift, gc).v);
  }
  int bn_bwd_finalize(std::string name, uintptr_t part, int ppg, int groups, int C, float count, uintptr_t gamma,
                      uintptr_t mean, uintptr_t rstd, uintptr_t dgamma, uintptr_t dbeta, uintptr_t coef,
                      int stream) {
    const size_t gc = (size_t)groups * C * 4;
    AccList acc;
    acc.r(part, (size_t)groups * ppg * 2 * C * 4).r(gamma, (size_t)C * 4).r(mean, gc).r(rstd, gc)
        .w(dgamma, (size_t)C * 4).w(dbeta, (size_t)C * 4).w(coef, 3 * gc);
    if (C % 4 == 0) {  // one level, all lanes on the rows (bnfin.hip; measured 1.151 vs 1.156 ms/step)
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bnfin_bwd)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                 P<const float>(mean), P<const float>(rstd), P<float>(dgamma), P<float>(dbeta),
                                 P<float>(coef), s);
      }, acc.v);
    }
    int PS = split_slices(ppg);
    if (PS > 1) {
      double* ws = nullptr;
      unsigned* ctr = nullptr;
      alloc_split(&ws, &ctr, (size_t)groups * PS * 2 * C, (size_t)((C + 15) / 16), acc);
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_bn_bwd_finalize_split)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                             P<const float>(mean), P<const float>(rstd), P<float>(dgamma),
                                             P<float>(dbeta), P<float>(coef), ws, ctr, PS, s);
      }, acc.v);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_bwd_finalize)(P<const float>(part), ppg, groups, C, count, P<const float>(gamma),
                                 P<const float>(mean), P<const float>(rstd), P<float>(dgamma), P<float>(dbeta),
                                 P<float>(coef), s);
    }, acc.v);
  }
  int bn_bwd_apply(std::string name, uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t coef, uintptr_t dx, int R,
                   int C, int rows_per_group, int act, float leak, int stream) {
    const size_t t = (size_t)R * C * es_, gc = (size_t)((R + rows_per_group - 1) / rows_per_group) * C * 4;
    AccList acc;
    acc.r(dy, t).r(x, t).r(y, t).r(coef, 3 * gc).w(dx, t);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_bn_bwd_apply)(P<const elem_t>(dy), P<const elem_t>(y), P<const elem_t>(x), P<const float>(coef),
                              P<elem_t>(dx), R, C, rows_per_group, act, leak, s);
    }, acc.v);
  }
  int act_bwd(std::string name, uintptr_t dy, uintptr_t y, uintptr_t dx, size_t n, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_act_bwd)(P<const elem_t>(dy), P<const elem_t>(y), P<elem_t>(dx), n, act, leak, s);
    }, AccList().r(dy, n * es_).r(y, n * es_).w(dx, n * es_).v);
  }
  // dx = dy * act'(y) and db = column sums of dx in one launch (last-arrival reduction)
  int act_bwd_dbias(std::string name, uintptr_t dy, uintptr_t y, uintptr_t dx, int R, int C, int act, float leak,
                    uintptr_t db, int stream) {
    const int max_blocks = 256;  // every block bumps one arrival counter: keep the atomics few
    AccList acc;
    const size_t t = (size_t)R * C * es_;
    acc.r(dy, t).r(y, t).w(dx, t).w(db, (size_t)C * 4);
    void* part = dev_alloc((size_t)max_blocks * C * sizeof(float));
    void* ctr = dev_alloc(sizeof(unsigned), nullptr, true);
    acc.w((uintptr_t)part, (size_t)max_blocks * C * 4).w((uintptr_t)ctr, 4);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_act_bwd_dbias)(P<const elem_t>(dy), P<const elem_t>(y), P<elem_t>(dx), R, C, act, leak,
                                   reinterpret_cast<float*>(part), max_blocks, reinterpret_cast<unsigned*>(ctr),
                                   P<float>(db), s);
    }, acc.v);
  }

  // D head backward (weight + bias + data gradient) in one launch
  // bx != 0: also the BN-backward partial statistics of the top BN layer -> part
  // [groups * (K / C)][2][C] (see head_bwd_kernel); dW / db / x may be 0 (g_loss chain: dgrad only)
  int head_bwd(std::string name, uintptr_t x, uintptr_t dl, uintptr_t w, uintptr_t dx, uintptr_t dW, uintptr_t db,
               int R, int K, int stream, uintptr_t bx, uintptr_t by, uintptr_t mean, uintptr_t rstd, int C, int rpg,
               int act, float leak, uintptr_t part) {
    const size_t t = (size_t)R * K * es_;
    AccList acc;
    acc.r(x, t).r(dl, (size_t)R * 4).r(w, (size_t)K * 4).w(dx, t).w(dW, (size_t)K * 4).w(db, 4);
    if (bx) {
      const size_t groups = (size_t)((R + rpg - 1) / rpg);
      acc.r(bx, t).r(by, t).r(mean, groups * C * 4).r(rstd, groups * C * 4).w(part, groups * (K / C) * 2 * C * 4);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_bwd)(P<const elem_t>(x), P<const float>(dl), P<const float>(w), P<elem_t>(dx), P<float>(dW),
                              P<float>(db), R, K, P<const elem_t>(bx), P<const elem_t>(by), P<const float>(mean),
                              P<const float>(rstd), C, rpg, act, leak, P<float>(part), s);
    }, acc.v);
  }
  // the head backward with RS row splits: BN partial rows [(g RS + y) S + sp] (ppg = RS S);
  // dW partials in a workspace summed by the last split of each column block (in-kernel)
  int head_bwd_rs(std::string name, uintptr_t x, uintptr_t dl, uintptr_t w, uintptr_t dx, uintptr_t dW, uintptr_t db,
                  int R, int K, int stream, uintptr_t bx, uintptr_t by, uintptr_t mean, uintptr_t rstd, int C, int rpg,
                  int act, float leak, uintptr_t part, int RS) {
    const size_t t = (size_t)R * K * es_;
    AccList acc;
    acc.r(x, t).r(dl, (size_t)R * 4).r(w, (size_t)K * 4).w(dx, t).w(dW, (size_t)K * 4).w(db, 4);
    if (bx) {
      const size_t groups = (size_t)((R + rpg - 1) / rpg);
      acc.r(bx, t).r(by, t).r(mean, groups * C * 4).r(rstd, groups * C * 4)
          .w(part, groups * RS * (K / C) * 2 * C * 4);
    }
    float* ws = nullptr;
    unsigned* ctr = nullptr;
    if (dW && RS > 1) {
      ws = reinterpret_cast<float*>(dev_alloc((size_t)RS * K * sizeof(float)));
      ctr = reinterpret_cast<unsigned*>(dev_alloc((size_t)((K + 63) / 64) * sizeof(unsigned), nullptr, true));
      acc.w((uintptr_t)ws, (size_t)RS * K * 4).w((uintptr_t)ctr, (size_t)((K + 63) / 64) * 4);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_bwd_rs)(P<const elem_t>(x), P<const float>(dl), P<const float>(w), P<elem_t>(dx),
                                 P<float>(dW), P<float>(db), R, K, P<const elem_t>(bx), P<const elem_t>(by),
                                 P<const float>(mean), P<const float>(rstd), C, rpg, act, leak, P<float>(part), RS, ws,
                                 ctr, s);
    }, acc.v);
  }

  int sum_partials(std::string name, uintptr_t part, int Pn, int stride, int C, uintptr_t dst, int stream) {
    AccList acc;
    acc.r(part, ((size_t)(Pn - 1) * stride + C) * 4).w(dst, (size_t)C * 4);
    const int PS = split_slices(Pn);
    if (PS > 1) {  // many rows: sliced + last-arrival combine
      void* ws = dev_alloc((size_t)PS * C * sizeof(float));
      void* ctr = dev_alloc((size_t)((C + 15) / 16) * sizeof(unsigned), nullptr, true);
      acc.w((uintptr_t)ws, (size_t)PS * C * 4).w((uintptr_t)ctr, (size_t)((C + 15) / 16) * 4);
      return add(name, stream, [=](hipStream_t s) {
        return KF(dcg_sum_partials_split)(P<const float>(part), Pn, stride, C, P<float>(dst),
                                          reinterpret_cast<float*>(ws), reinterpret_cast<unsigned*>(ctr), PS, s);
      }, acc.v);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_sum_partials)(P<const float>(part), Pn, stride, C, P<float>(dst), s);
    }, acc.v);
  }
  int colsum_small(std::string name, uintptr_t x, int R, int C, uintptr_t part, int blocks, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_colsum_small)(P<const elem_t>(x), R, C, P<float>(part), blocks, s);
    }, AccList().r(x, (size_t)R * C * es_).w(part, (size_t)blocks * C * 4).v);
  }

  // ------------------------------------------------------------------ heads, losses, optimiser
  int gan_loss(std::string name, uintptr_t logits, int B, uintptr_t out, uintptr_t dl_d, uintptr_t dl_g,
               uintptr_t prob, int stream, uintptr_t ls) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_gan_loss)(P<const float>(logits), B, P<float>(out), P<float>(dl_d), P<float>(dl_g),
                          P<float>(prob), P<const float>(ls), s);
    }, AccList().r(logits, (size_t)B * 8).w(out, 16).w(dl_d, (size_t)B * 8).w(dl_g, (size_t)B * 4)
           .w(prob, (size_t)B * 8).r(ls, 12).v);
  }
  // stats (optional): BN partial statistics of the output, channel = column % C ->
  // [(B / 8) * (N / C)][2][C] partial rows (the row block of the kernel is 8)
  // gen_step != 0: z ~ U(-1,1) generated in-kernel (Philox keyed by gen_seed and the device
  // step counter, identical to philox_uniform) and written to z
  int linear_fwd(std::string name, uintptr_t z, uintptr_t W, uintptr_t b, uintptr_t out, int B, int K, int N,
                 int stream, uintptr_t stats = 0, int C = 0, uintptr_t gen_step = 0, uint64_t gen_seed = 0) {
    AccList acc;
    if (gen_step) acc.w(z, (size_t)B * K * 4).r(gen_step, 8);
    else acc.r(z, (size_t)B * K * 4);
    acc.r(W, (size_t)K * N * 4).r(b, (size_t)N * 4).w(out, (size_t)B * N * es_);
    if (stats) acc.w(stats, (size_t)((B + 7) / 8) * (N / C) * 2 * C * 4);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_linear_fwd)(P<float>(z), P<const float>(W), P<const float>(b), P<elem_t>(out), B, K, N,
                                P<float>(stats), C, P<const unsigned long long>(gen_step), gen_seed, s);
    }, acc.v);
  }
  int linear_wgrad(std::string name, uintptr_t z, uintptr_t dh, uintptr_t dW, uintptr_t db, int B, int K, int N,
                   int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_linear_wgrad)(P<const float>(z), P<const elem_t>(dh), P<float>(dW), P<float>(db), B, K, N, s);
    }, AccList().r(z, (size_t)B * K * 4).r(dh, (size_t)B * N * es_).w(dW, (size_t)K * N * 4).w(db, (size_t)N * 4).v);
  }
  // loss_out != 0: the 3-loss BCE (gan_loss) runs in the GEMV's last-arriving block
  int gemv_head(std::string name, uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t out, int R, int K, int stream,
                uintptr_t loss_out, uintptr_t dl_d, uintptr_t dl_g, uintptr_t prob, uintptr_t ls) {
    unsigned* ctr = nullptr;
    AccList acc;
    acc.r(x, (size_t)R * K * es_).r(w, (size_t)K * 4).r(b, 4).w(out, (size_t)R * 4);
    if (loss_out) {
      ctr = reinterpret_cast<unsigned*>(dev_alloc(sizeof(unsigned), nullptr, true));
      acc.w((uintptr_t)ctr, 4).w(loss_out, 16).w(dl_d, (size_t)R * 4).w(dl_g, (size_t)R * 2).w(prob, (size_t)R * 4)
          .r(ls, 12);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_gemv_head)(P<const elem_t>(x), P<const float>(w), P<const float>(b), P<float>(out), R, K, ctr,
                               P<float>(loss_out), P<float>(dl_d), P<float>(dl_g), P<float>(prob), P<const float>(ls),
                               s);
    }, acc.v);
  }
  // the head with the top BN layer's apply + activation fused: x = that layer's pre-BN input,
  // y = its activation (written here), scale / shift [groups][C] from its BN finalize
  int gemv_head_bn(std::string name, uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t out, int R, int K, int stream,
                   uintptr_t loss_out, uintptr_t dl_d, uintptr_t dl_g, uintptr_t prob, uintptr_t ls, uintptr_t scale,
                   uintptr_t shift, int C, int rpg, int act, float leak, uintptr_t y) {
    if (dt_ == 2) throw std::runtime_error("gemv_head_bn: 16-bit builds only");
    unsigned* ctr = nullptr;
    AccList acc;
    const size_t groups = (size_t)((R + rpg - 1) / rpg);
    acc.r(x, (size_t)R * K * es_).r(w, (size_t)K * 4).r(b, 4).w(out, (size_t)R * 4).r(scale, groups * C * 4)
        .r(shift, groups * C * 4).w(y, (size_t)R * K * es_);
    if (loss_out) {
      ctr = reinterpret_cast<unsigned*>(dev_alloc(sizeof(unsigned), nullptr, true));
      acc.w((uintptr_t)ctr, 4).w(loss_out, 16).w(dl_d, (size_t)R * 4).w(dl_g, (size_t)R * 2).w(prob, (size_t)R * 4)
          .r(ls, 12);
    }
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_gemv_head_bn)(P<const elem_t>(x), P<const float>(w), P<const float>(b), P<float>(out), R, K, ctr,
                                  P<float>(loss_out), P<float>(dl_d), P<float>(dl_g), P<float>(prob),
                                  P<const float>(ls), P<const float>(scale), P<const float>(shift), C, rpg, act, leak,
                                  P<elem_t>(y), s);
    }, acc.v);
  }
  int head_dgrad(std::string name, uintptr_t dl, uintptr_t w, uintptr_t dx, int R, int K, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_dgrad)(P<const float>(dl), P<const float>(w), P<elem_t>(dx), R, K, s);
    }, AccList().r(dl, (size_t)R * 4).r(w, (size_t)K * 4).w(dx, (size_t)R * K * es_).v);
  }
  int head_wgrad(std::string name, uintptr_t x, uintptr_t dl, uintptr_t part, int R, int K, int splits,
                 uintptr_t dW, uintptr_t db, int stream) {
    add(name, stream, [=](hipStream_t s) {
      return KF(dcg_head_wgrad)(P<const elem_t>(x), P<const float>(dl), P<float>(part), R, K, splits, s);
    }, AccList().r(x, (size_t)R * K * es_).r(dl, (size_t)R * 4).w(part, (size_t)splits * K * 4).v);
    add(name + ".reduce", stream, [=](hipStream_t s) {
      return KF(dcg_splitk_reduce)(P<const float>(part), splits, (size_t)K, P<float>(dW), 1.f, s);
    }, AccList().r(part, (size_t)splits * K * 4).w(dW, (size_t)K * 4).v);
    return add(name + ".bias", stream, [=](hipStream_t s) { return KF(dcg_sum_vec)(P<const float>(dl), R, P<float>(db), s); },
               AccList().r(dl, (size_t)R * 4).w(db, 4).v);
  }
  int adam(std::string name, uintptr_t w, uintptr_t g, uintptr_t m, uintptr_t v, uintptr_t powers, size_t n, float lr,
           float b1, float b2, float eps, float gscale, int stream) {
    return adam_bf(name, w, 0, g, m, v, powers, n, lr, b1, b2, eps, gscale, stream, 0, 0);
  }
  // + elem_t mirror of the updated weights (same flat layout); gbf: read the gradient from this
  // bf16 buffer (the all-reduced bf16 wire of the DDP step) instead of g
  int adam_bf(std::string name, uintptr_t w, uintptr_t wbf, uintptr_t g, uintptr_t m, uintptr_t v, uintptr_t powers,
              size_t n, float lr, float b1, float b2, float eps, float gscale, int stream, uintptr_t ls, uintptr_t gbf) {
    AccList acc;
    acc.w(w, n * 4).w(wbf, n * es_).w(m, n * 4).w(v, n * 4).r(powers, 8).r(ls, 12);
    if (gbf) acc.r(gbf, n * 2);
    else acc.r(g, n * 4);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_adam)(P<float>(w), P<elem_t>(wbf), P<const float>(g), P<float>(m), P<float>(v), P<const float>(powers),
                      n, lr, b1, b2, eps, gscale, P<const float>(ls), P<const void>(gbf), s);
    }, acc.v);
  }
  // both TF-Adams (A first) + beta powers / step counter in one launch (see adam2_kernel)
  int adam2(std::string name, uintptr_t wA, uintptr_t wbfA, uintptr_t gA, uintptr_t mA, uintptr_t vA, uintptr_t pA,
            size_t nA, float lrA, float b1A, float b2A, float epsA, uintptr_t wD, uintptr_t wbfD, uintptr_t gD,
            uintptr_t mD, uintptr_t vD, uintptr_t pD, size_t nD, float lrD, float b1D, float b2D, float epsD,
            float gscale, uintptr_t step, int stream) {
    void* ctr = dev_alloc(sizeof(unsigned), nullptr, true);
    AccList acc;
    acc.w(wA, nA * 4).w(wbfA, nA * es_).r(gA, nA * 4).w(mA, nA * 4).w(vA, nA * 4).w(pA, 8)
        .w(wD, nD * 4).w(wbfD, nD * es_).r(gD, nD * 4).w(mD, nD * 4).w(vD, nD * 4).w(pD, 8).w(step, 8)
        .w((uintptr_t)ctr, 4);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_adam2)(P<float>(wA), P<elem_t>(wbfA), P<const float>(gA), P<float>(mA), P<float>(vA), P<float>(pA),
                           nA, lrA, b1A, b2A, epsA, P<float>(wD), P<elem_t>(wbfD), P<const float>(gD), P<float>(mD),
                           P<float>(vD), P<float>(pD), nD, lrD, b1D, b2D, epsD, gscale,
                           P<unsigned long long>(step), reinterpret_cast<unsigned*>(ctr), s);
    }, acc.v);
  }
  // narrow2.hip: TF-SAME stride-2 5x5 conv, 1..4 input -> 64 output channels, persistent `grid`
  // workgroups (<= tiles: nconv_tiles). bx != 0: fused BN-backward statistics of the layer below
  // (x = bx, y = by, one BN group), one partial row [2][64] per workgroup into part.
  int nconv(std::string name, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int H, int W, int Cin,
            int Ho, int Wo, int pad_y, int pad_x, int act, float leak, int grid, uintptr_t bx, uintptr_t by,
            uintptr_t mean, uintptr_t rstd, int bact, float bleak, uintptr_t part, int stream) {
    if (dt_ == 2) throw std::runtime_error("nconv: 16-bit builds only");
    const int tiles = KF(dcg_nconv_tiles)(B, Ho, Wo);
    if (grid < 1 || grid > tiles) throw std::runtime_error("nconv: grid must be in [1, tiles]");
    const size_t out = (size_t)B * Ho * Wo * 64 * es_;
    AccList acc;
    acc.r(x, (size_t)B * H * W * Cin * es_).r(w, (size_t)25 * Cin * 64 * es_).r(bias, 64 * 4).w(y, out);
    if (bx) acc.r(bx, out).r(by, out).r(mean, 64 * 4).r(rstd, 64 * 4).w(part, (size_t)grid * 128 * 4);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_nconv)(P<const elem_t>(x), P<const elem_t>(w), P<const float>(bias), P<elem_t>(y), B, H, W, Cin,
                           Ho, Wo, pad_y, pad_x, act, leak, grid, P<const elem_t>(bx), P<const elem_t>(by),
                           P<const float>(mean), P<const float>(rstd), bact, bleak, P<float>(part), s);
    }, acc.v);
  }
  int nconv_tiles(int B, int Ho, int Wo) const { return KF(dcg_nconv_tiles)(B, Ho, Wo); }
  // G's RGB layer forward with the BN apply + activation of the layer below fused into its halo
  // staging: x = that layer's pre-BN output, a_out = its activation (written by the owning tiles)
  int narrow_deconv_bnin(std::string name, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int Hi,
                         int Wi, int C, int Ho, int Wo, int N, int pad, int act, float leak, uintptr_t scale,
                         uintptr_t shift, int bn_act, float bn_leak, uintptr_t a_out, int stream) {
    if (dt_ == 2) throw std::runtime_error("narrow_deconv_bnin: 16-bit builds only");
    const size_t in = (size_t)B * Hi * Wi * C * es_;
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_narrow_deconv_bnin)(P<const elem_t>(x), P<const elem_t>(w), P<const float>(bias), P<elem_t>(y), B,
                                        Hi, Wi, C, Ho, Wo, N, pad, act, leak, P<const float>(scale),
                                        P<const float>(shift), bn_act, bn_leak, P<elem_t>(a_out), s);
    }, AccList().r(x, in).r(w, (size_t)25 * N * C * es_).r(bias, (size_t)N * 4).r(scale, (size_t)C * 4)
           .r(shift, (size_t)C * 4).w(a_out, in).w(y, (size_t)B * Ho * Wo * N * es_).v);
  }
  // G's RGB-layer image gradient with its activation backward fused (narrow.hip DACT variant):
  // y = conv_transpose(x, w) * act'(ya), db[N] = column sums of y (per-workgroup partials + a
  // sliced fixed-order sum) -- replaces narrow_deconv + act_bwd_dbias.
  int narrow_deconv_dact(std::string name, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ya, int B, int Hi, int Wi,
                         int C, int Ho, int Wo, int N, int pad, int act, float leak, uintptr_t db, int stream) {
    if (dt_ == 2) throw std::runtime_error("narrow_deconv_dact: 16-bit builds only");
    const int tiles = KF(dcg_narrow_deconv_tiles)(B, Ho, Wo);
    float* part = reinterpret_cast<float*>(dev_alloc((size_t)tiles * N * sizeof(float)));
    const size_t out = (size_t)B * Ho * Wo * N * es_;
    add(name, stream, [=](hipStream_t s) {
      return KF(dcg_narrow_deconv_dact)(P<const elem_t>(x), P<const elem_t>(w), P<elem_t>(y), P<const elem_t>(ya), B,
                                        Hi, Wi, C, Ho, Wo, N, pad, act, leak, part, s);
    }, AccList().r(x, (size_t)B * Hi * Wi * C * es_).r(w, (size_t)25 * N * C * es_).r(ya, out).w(y, out)
           .w((uintptr_t)part, (size_t)tiles * N * 4).v);
    return sum_partials(name + ".dbias", (uintptr_t)part, tiles, N, N, db, stream);
  }
  bool nwgrad_ok(int H, int W, int Hd, int Wd) const {
    int t, r, c;
    return dt_ != 2 && KF(dcg_nwgrad_plan)(H, W, Hd, Wd, &t, &r, &c) == 0;
  }
  // narrow2.hip weight gradient of a 1..4-channel image layer: dst[25][Cin][64] (fp32, TF layout)
  // = sum over output pixels of the stride-2 window of x times d; per-workgroup partials
  // (workspace) summed in workgroup order by splitk_reduce -- deterministic.
  int nwgrad(std::string name, uintptr_t x, int B, int H, int W, int Cin, uintptr_t d, int Hd, int Wd, int pad,
             uintptr_t dst, int stream, int chunks_per_wg) {
    int tyc, wr, wc;
    if (dt_ == 2 || KF(dcg_nwgrad_plan)(H, W, Hd, Wd, &tyc, &wr, &wc))
      throw std::runtime_error("nwgrad: unsupported shape / dtype");
    const int chunks_img = (Hd + tyc - 1) / tyc;
    const int total = B * chunks_img;
    // auto: chunks per workgroup (<= 8) so that about NWG_TARGET workgroups run -- fewer
    // workgroups = fewer partial slabs for the reduce, more = more latency hiding
    int cpw = chunks_per_wg > 0 ? chunks_per_wg : total / 256;
    cpw = cpw < 1 ? 1 : (cpw > 8 ? 8 : cpw);
    const int wg = B * ((chunks_img + cpw - 1) / cpw);
    const size_t n = (size_t)25 * Cin * 64;
    float* part = reinterpret_cast<float*>(dev_alloc((size_t)wg * n * sizeof(float)));
    add(name, stream, [=](hipStream_t s) {
      return KF(dcg_nwgrad)(P<const elem_t>(x), B, H, W, Cin, P<const elem_t>(d), Hd, Wd, pad, cpw, part, s);
    }, AccList().r(x, (size_t)B * H * W * Cin * es_).r(d, (size_t)B * Hd * Wd * 64 * es_)
           .w((uintptr_t)part, (size_t)wg * n * 4).v);
    return add(name + ".reduce", stream, [=](hipStream_t s) {
      return KF(dcg_splitk_reduce)(part, wg, n, P<float>(dst), 1.f, s);
    }, AccList().r((uintptr_t)part, (size_t)wg * n * 4).w(dst, n * 4).v);
  }
  // TF-SAME stride-2 5x5 conv_transpose with 1..4 output channels (direct VALU kernel)
  int narrow_deconv(std::string name, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int B, int Hi, int Wi,
                    int C, int Ho, int Wo, int N, int pad, int act, float leak, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_narrow_deconv)(P<const elem_t>(x), P<const elem_t>(w), P<const float>(bias), P<elem_t>(y), B, Hi,
                                   Wi, C, Ho, Wo, N, pad, act, leak, s);
    }, AccList().r(x, (size_t)B * Hi * Wi * C * es_).r(w, (size_t)25 * N * C * es_).r(bias, (size_t)N * 4)
           .w(y, (size_t)B * Ho * Wo * N * es_).v);
  }
  // dynamic loss scaling: flag ls[1] if any gradient is non-finite
  int nonfinite_check(std::string name, uintptr_t g, size_t n, uintptr_t ls, int stream) {
    return add(name, stream, [=](hipStream_t s) { return KF(dcg_nonfinite_check)(P<const float>(g), n, P<float>(ls), s); },
               AccList().r(g, n * 4).w(ls, 12).v);
  }
  int step_end(std::string name, uintptr_t pd, uintptr_t pg, float b1d, float b2d, float b1g, float b2g,
               uintptr_t step, int stream, uintptr_t ls, int growth_interval) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_step_end)(P<float>(pd), P<float>(pg), b1d, b2d, b1g, b2g, P<unsigned long long>(step), P<float>(ls),
                          growth_interval, s);
    }, AccList().w(pd, 8).w(pg, 8).w(step, 8).w(ls, 12).v);
  }
  int pack(std::string name, uintptr_t src, int T, int A, int Bd, uintptr_t nat, uintptr_t tr, int st, int sb, int sa,
           int stream) {
    const size_t n = (size_t)T * A * Bd;
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_pack)(P<const float>(src), T, A, Bd, P<elem_t>(nat), P<elem_t>(tr), st, sb, sa, s);
    }, AccList().r(src, n * 4).w(nat, n * es_).w(tr, n * es_).v);
  }
  int philox_uniform(std::string name, uintptr_t out, size_t n, uint64_t seed, uintptr_t step, uint64_t stream_id,
                     float lo, float hi, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_philox_uniform)(P<float>(out), n, seed, P<const unsigned long long>(step), stream_id, lo, hi, s);
    }, AccList().w(out, n * 4).r(step, 8).v);
  }
  int im2col_s2(std::string name, uintptr_t src, uintptr_t dst, int Bn, int H, int W, int C, int Ho, int Wo, int pl_y,
                int pl_x, int Kpad, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_im2col_s2)(P<const elem_t>(src), P<elem_t>(dst), Bn, H, W, C, Ho, Wo, pl_y, pl_x, Kpad, s);
    }, AccList().r(src, (size_t)Bn * H * W * C * es_).w(dst, (size_t)Bn * Ho * Wo * Kpad * es_).v);
  }
  int cast_to_bf16(std::string name, uintptr_t src, int src_dtype, uintptr_t dst, size_t n, float scale, float shift,
                   int stream) {
    const size_t ss = src_dtype == 1 ? 8 : src_dtype == 2 ? 1 : 4;
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_cast_to_bf16)(P<const void>(src), src_dtype, P<elem_t>(dst), n, scale, shift, s);
    }, AccList().r(src, n * ss).w(dst, n * es_).v);
  }
  int cast_bf16_f32(std::string name, uintptr_t src, uintptr_t dst, size_t n, int stream) {
    return add(name, stream, [=](hipStream_t s) { return KF(dcg_cast_bf16_f32)(P<const elem_t>(src), P<float>(dst), n, s); },
               AccList().r(src, n * es_).w(dst, n * 4).v);
  }
  int splitk_reduce(std::string name, uintptr_t src, int splits, size_t n, uintptr_t dst, float scale, int stream) {
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_splitk_reduce)(P<const float>(src), splits, n, P<float>(dst), scale, s);
    }, AccList().r(src, (size_t)splits * n * 4).w(dst, n * 4).v);
  }
  // summary statistics of one tensor (zero fraction + fixed-bucket histogram), see summary.hip
  int tensor_summary(std::string name, uintptr_t x, int x_dtype, size_t n, uintptr_t edges, int nbins, uintptr_t out,
                     int stream) {
    const int blocks = summary_blocks(n);
    void* part = dev_alloc((size_t)blocks * (nbins + 6) * sizeof(double));
    void* ctr = dev_alloc(sizeof(unsigned), nullptr, true);
    const size_t xs = x_dtype == 0 ? 4 : (x_dtype == 3 ? 4 : (size_t)es_);
    return add(name, stream, [=](hipStream_t s) {
      return KF(dcg_tensor_summary)(P<const void>(x), x_dtype, n, P<const double>(edges), nbins, P<double>(out),
                                    reinterpret_cast<double*>(part), reinterpret_cast<unsigned*>(ctr), blocks, s);
    }, AccList().r(x, n * xs).r(edges, (size_t)(nbins - 1) * 8).w(out, (size_t)(nbins + 6) * 8)
           .w((uintptr_t)part, (size_t)blocks * (nbins + 6) * 8).w((uintptr_t)ctr, 4).v);
  }
  static int summary_blocks(size_t n) { return (int)std::max<size_t>(1, std::min<size_t>(256, (n + 8191) / 8192)); }

 private:
  int add(const std::string& name, int stream, std::function<int(hipStream_t)> fn, std::vector<Acc> acc,
          int kind = OP_LAUNCH, int ev = -1) {
    ops_.push_back(Op{name, stream, kind, ev, std::move(acc), std::move(fn)});
    return (int)ops_.size() - 1;
  }
  // device allocation owned by the program (optionally initialised from host / zeroed); a dry
  // program hands out disjoint fake addresses above any real one
  void* dev_alloc(size_t bytes, const void* init = nullptr, bool zero = false) {
    if (dry_) {  // process-wide counter: fake ranges of different programs never overlap
      static uintptr_t fake_next = (uintptr_t)1 << 60;
      const uintptr_t p = fake_next;
      fake_next += (bytes + 255) / 256 * 256 + 256;
      return reinterpret_cast<void*>(p);
    }
    void* p = nullptr;
    HIPCHECK(hipMalloc(&p, bytes));
    if (init) HIPCHECK(hipMemcpy(p, init, bytes, hipMemcpyHostToDevice));
    if (zero) HIPCHECK(hipMemset(p, 0, bytes));
    dev_allocs_.push_back(p);
    return p;
  }
  std::vector<Op> ops_;
  std::vector<void*> dev_allocs_;
  std::vector<hipEvent_t> events_;
  std::vector<std::shared_ptr<dcg_comm::Comm>> comms_;
  int last_mtiles_ = 0, last_nphases_ = 0;
  int dt_ = 0;       // element type of every activation / weight-mirror pointer
  size_t es_ = 2;    // its size in bytes
  bool dry_ = false;
};

static py::tuple igemm_tile(int cfg, int dtype) {
  int bm = 0, bn = 0, ns = 0;
  int rc;
#define DT(fn) (dtype == 2 ? fn##_f32 : dtype == 1 ? fn##_f16 : fn)
  if (cfg >= 400) rc = -1;
  else if (cfg >= 200) rc = DT(dcg_igemm3_tile)(cfg, &bm, &bn, &ns);
  else rc = DT(dcg_igemm_tile)(cfg, &bm, &bn);
#undef DT
  if (rc) throw std::runtime_error("bad cfg");
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
  m.def("igemm_tile", &igemm_tile, py::arg("cfg"), py::arg("dtype") = 0);
  m.def("wgrad_tile", &wgrad_tile);
  m.def("device_arch", &device_arch);
  m.attr("built_for") = "gfx950";
  m.attr("OP_LAUNCH") = (int)OP_LAUNCH;
  m.attr("OP_RECORD") = (int)OP_RECORD;
  m.attr("OP_WAIT") = (int)OP_WAIT;
  py::class_<dcg_comm::Comm, std::shared_ptr<dcg_comm::Comm>>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, const std::string&, int>(), py::arg("lib_path"), py::arg("nranks"),
           py::arg("rank"), py::arg("unique_id"), py::arg("device"))
      .def_static("unique_id", [](const std::string& lib) { return py::bytes(dcg_comm::Comm::unique_id(lib)); })
      .def("all_reduce", &dcg_comm::Comm::all_reduce, py::arg("ptr"), py::arg("count"), py::arg("dtype"),
           py::arg("stream"))
      .def("destroy", &dcg_comm::Comm::destroy)
      .def_property_readonly("nranks", &dcg_comm::Comm::nranks)
      .def_property_readonly("rank", &dcg_comm::Comm::rank);
  py::class_<Program>(m, "Program")
      .def(py::init<int, bool>(), py::arg("dtype") = 0, py::arg("dry") = false)
      .def_property_readonly("f16", &Program::f16)
      .def_property_readonly("dtype", &Program::dtype)
      .def_property_readonly("dry", &Program::dry)
      .def_property_readonly("elem_size", &Program::elem_size)
      .def("size", &Program::size)
      .def("name", &Program::name)
      .def("op_info", &Program::op_info)
      .def("run", &Program::run, py::arg("streams"), py::arg("begin") = 0, py::arg("end") = -1)
      .def("new_event", &Program::new_event)
      .def("record", &Program::record)
      .def("wait", &Program::wait)
      .def("memset", &Program::memset)
      .def("copy", &Program::copy)
      .def("comm_emulate", &Program::comm_emulate)
      .def("allreduce", &Program::allreduce)
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
      .def("wgrad3", &Program::wgrad3, py::arg("name"), py::arg("G"), py::arg("Hg"), py::arg("Wg"), py::arg("Mc"),
           py::arg("Dm"), py::arg("Bn"), py::arg("Hd"), py::arg("Wd"), py::arg("Nc"), py::arg("pad"), py::arg("cfg"),
           py::arg("splits"), py::arg("dst"), py::arg("scale"), py::arg("stream"))
      .def("colstats", &Program::colstats)
      .def("bn_finalize", &Program::bn_finalize)
      .def("bn_coef_eval", &Program::bn_coef_eval, py::arg("name"), py::arg("C"), py::arg("gamma"), py::arg("beta"),
           py::arg("eps"), py::arg("mean"), py::arg("var"), py::arg("debias"), py::arg("scale"), py::arg("shift"),
           py::arg("stream"), py::arg("debias_ptr") = 0)
      .def("bn_apply_act", &Program::bn_apply_act)
      .def("bn_bwd_finalize", &Program::bn_bwd_finalize)
      .def("bn_bwd_apply", &Program::bn_bwd_apply, py::arg("name"), py::arg("dy"), py::arg("y"), py::arg("x"),
           py::arg("coef"), py::arg("dx"), py::arg("R"), py::arg("C"), py::arg("rows_per_group"), py::arg("act"),
           py::arg("leak"), py::arg("stream"))
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
           py::arg("gscale"), py::arg("stream"), py::arg("ls") = 0, py::arg("gbf") = 0)
      .def("step_end", &Program::step_end, py::arg("name"), py::arg("pd"), py::arg("pg"), py::arg("b1d"),
           py::arg("b2d"), py::arg("b1g"), py::arg("b2g"), py::arg("step"), py::arg("stream"), py::arg("ls") = 0,
           py::arg("growth_interval") = 2000)
      .def("adam2", &Program::adam2)
      .def("nonfinite_check", &Program::nonfinite_check)
      .def("narrow_deconv", &Program::narrow_deconv)
      .def("nconv", &Program::nconv)
      .def("nconv_tiles", &Program::nconv_tiles)
      .def("narrow_deconv_dact", &Program::narrow_deconv_dact)
      .def("gemv_head_bn", &Program::gemv_head_bn)
      .def("head_bwd_rs", &Program::head_bwd_rs)
      .def("narrow_deconv_bnin", &Program::narrow_deconv_bnin)
      .def("nwgrad_ok", &Program::nwgrad_ok)
      .def("nwgrad", &Program::nwgrad, py::arg("name"), py::arg("x"), py::arg("B"), py::arg("H"), py::arg("W"),
           py::arg("Cin"), py::arg("d"), py::arg("Hd"), py::arg("Wd"), py::arg("pad"), py::arg("dst"), py::arg("stream"),
           py::arg("chunks_per_wg") = 0)
      .def("pack", &Program::pack)
      .def("philox_uniform", &Program::philox_uniform)
      .def("im2col_s2", &Program::im2col_s2)
      .def("cast_to_bf16", &Program::cast_to_bf16)
      .def("cast_bf16_f32", &Program::cast_bf16_f32)
      .def("splitk_reduce", &Program::splitk_reduce)
      .def("tensor_summary", &Program::tensor_summary);
}
