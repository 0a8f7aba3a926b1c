// Study (not part of the product .so): global -> LDS fill throughput on gfx950, the operand-fill
// path of the implicit-GEMM K loops (igemm3.hip / wgrad3.hip / wgrad5.hip stage their tiles with
// LDS-DMA, `buffer_load_dwordx4 ... lds`). Two fill paths, same bytes:
//   dma  16-byte LDS-DMA pieces (no VGPR round trip), NS-deep ring, counted vmcnt + barrier
//   reg  16-byte buffer loads into VGPRs, then ds_write_b128 (the classic register-staged fill)
// Each workgroup (4 waves) streams 16 KiB per iteration (one GEMM stage of a 128x64 tile) from
// its own slice of a working set sized to sit in L2 (a few MiB) or not (HBM / MALL).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o ldsdma_bw benchmarks/study/ldsdma_bw.hip
//   ./ldsdma_bw            -> one line per (path, working set, workgroups per CU, stages)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../csrc/hip/common.h"
using namespace dcg;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr int STAGE = 16384;  // bytes per workgroup per iteration (16 pieces of 1 KiB, 4 per wave)

template <int N_>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }

template <int NS>
__global__ __launch_bounds__(256) void dma_kernel(const char* src, uint32_t slice, int iters, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(src) + (size_t)blockIdx.x * slice, (short)0, (int)slice, 0x00020000);
  const uint32_t lbase = (uint32_t)(uintptr_t)(lds_char*)lds;
  const uint32_t nst = slice / STAGE;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    const uint32_t goff = (uint32_t)(it % nst) * STAGE;
    const uint32_t la = lbase + (uint32_t)(it % NS) * STAGE;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t piece = wave * 4 + p;  // 1 KiB pieces: wave w fills [4w, 4w + 4)
      dma16_asm_la(r, la + piece * 1024, goff + piece * 1024 + lane * 16);
    }
    wait_vm<4 * (NS - 1)>();  // the stage issued NS-1 iterations ago has landed
    __syncthreads();
    acc += reinterpret_cast<const lds_f32*>((lds_char*)lds)[((it + 1) % NS) * (STAGE / 4) + tid];
    __syncthreads();
  }
  wait_vm<0>();
  if (acc == 12345.f) out[blockIdx.x] = acc;  // keep the reads
}

__global__ __launch_bounds__(256) void reg_kernel(const char* src, uint32_t slice, int iters, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(src) + (size_t)blockIdx.x * slice, (short)0, (int)slice, 0x00020000);
  const uint32_t nst = slice / STAGE;
  float acc = 0.f;
  u32x4 v[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) v[p] = buf_load16(r, p * 4096 + tid * 16);
  for (int it = 0; it < iters; ++it) {
    u32x4* st = reinterpret_cast<u32x4*>(lds + (it & 1) * STAGE);
#pragma unroll
    for (int p = 0; p < 4; ++p) st[p * 256 + tid] = v[p];  // 16-byte LDS writes
    const uint32_t goff = (uint32_t)((it + 1) % nst) * STAGE;
#pragma unroll
    for (int p = 0; p < 4; ++p) v[p] = buf_load16(r, goff + p * 4096 + tid * 16);  // next stage in flight
    __syncthreads();
    acc += reinterpret_cast<const float*>(lds + (it & 1) * STAGE)[(tid * 4 + 1) & (STAGE / 4 - 1)];
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

int main() {
  int dev = 0, cus = 0, clk_khz = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CHECK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
  const size_t max_bytes = (size_t)1 << 30;
  char* src = nullptr;
  float* out = nullptr;
  CHECK(hipMalloc(&src, max_bytes));
  CHECK(hipMemset(src, 1, max_bytes));
  CHECK(hipMalloc(&out, 65536 * sizeof(float)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("# %d CUs, clock %.2f GHz (attribute); B/clk/CU at that clock\n", cus, clk_khz / 1e6);
  std::printf("%-4s %10s %6s %3s %10s %9s\n", "path", "set_MiB", "wg/CU", "NS", "TB/s", "B/clk/CU");
  // per-workgroup slice: 64 KiB (past L1; 256 / 512 workgroups = 2 / 4 MiB per XCD's L2) or
  // 1 GiB / grid (streams from HBM / MALL)
  for (int regime = 0; regime < 2; ++regime) {
    for (int per_cu : {1, 2, 4}) {
      const int grid = cus * per_cu;
      const uint32_t slice = regime == 0 ? 65536u : (uint32_t)(max_bytes / grid) / STAGE * STAGE;
      const size_t set = (size_t)grid * slice;
      const int iters = 2000;
      for (int variant = 0; variant < 4; ++variant) {  // dma NS=2,3,4; reg
        const int ns = variant < 3 ? variant + 2 : 2;
        const size_t shm = (size_t)ns * STAGE;
        auto launch = [&]() {
          if (variant == 0) hipLaunchKernelGGL(dma_kernel<2>, dim3(grid), dim3(256), shm, 0, src, slice, iters, out);
          else if (variant == 1) hipLaunchKernelGGL(dma_kernel<3>, dim3(grid), dim3(256), shm, 0, src, slice, iters, out);
          else if (variant == 2) hipLaunchKernelGGL(dma_kernel<4>, dim3(grid), dim3(256), shm, 0, src, slice, iters, out);
          else hipLaunchKernelGGL(reg_kernel, dim3(grid), dim3(256), shm, 0, src, slice, iters, out);
        };
        launch();
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int rep = 0; rep < 5; ++rep) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double bytes = 5.0 * grid * (double)iters * STAGE;
        const double tbs = bytes / (ms * 1e-3) / 1e12;
        std::printf("%-4s %10.0f %6d %3d %10.2f %9.1f\n", variant < 3 ? "dma" : "reg", set / 1048576.0, per_cu, ns, tbs,
                    tbs * 1e12 / cus / (clk_khz * 1e3));
        std::fflush(stdout);
      }
    }
  }
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
