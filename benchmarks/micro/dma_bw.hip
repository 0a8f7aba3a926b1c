// LDS-DMA (buffer_load_dwordx4 ... lds) throughput per CU on gfx950, by access pattern and depth.
// Decides the operand-staging design of the conv GEMMs: how many bytes per clock a CU can pull
// from L2 into LDS, and what partial-line (32 / 64 B of a 128 B line) reads cost.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dma_bw benchmarks/micro/dma_bw.hip && /tmp/dma_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(const void* b, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(b), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t la_in, uint32_t off) {
  const uint32_t la = __builtin_amdgcn_readfirstlane(la_in);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" :: "s"(la), "v"(off), "s"(r) : "memory", "m0");
}
template <int N_> __device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N_) : "memory"); }

// PAT 0: 1 KiB contiguous per piece; 1: 64 B of each of 16 lines (stride 128); 2: 32 B of 32 lines;
// 3: like 2 but 4 consecutive pieces cover the 4 quarters of the same 32 lines (L1 reuse)
// 4: lockstep -- every block walks the SAME piece sequence (all CUs streaming one weight matrix
//    in the same K order, as a conv GEMM's B operand does); 5: like 4 with the sequence rotated
//    by a per-block offset (the K-step order staggered over workgroups)
template <int PAT, int DEPTH>
__global__ void dma_kernel(const char* src, uint32_t span, int iters, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds + wave * DEPTH * 1024;
  const __amdgpu_buffer_rsrc_t r = mk(src, span);
  const uint32_t gid = (blockIdx.x * nw + wave);
  for (int i = 0; i < iters; ++i) {
    uint32_t q = gid * 7919u + (uint32_t)i * 131u;  // piece id (pseudo-random walk)
    uint32_t off;
    if (PAT == 0) off = (q * 1024u) % span + lane * 16;
    else if (PAT == 1) off = (q * 2048u) % span + (lane >> 2) * 128 + (lane & 3) * 16;
    else if (PAT == 2) off = (q * 4096u) % span + (lane >> 1) * 128 + (lane & 1) * 16;
    else if (PAT == 4) off = (((uint32_t)i * nw + wave) * 1024u) % span + lane * 16;
    else if (PAT == 5) off = (((uint32_t)i * nw + wave + blockIdx.x * 16u) * 1024u) % span + lane * 16;
    else { const uint32_t g = gid * 7919u + (uint32_t)(i >> 2) * 131u; off = (g * 4096u) % span + (lane >> 1) * 128 + (lane & 1) * 16 + (i & 3) * 32; }
    dma16(r, lbase + (i % DEPTH) * 1024, off);
    wvm<DEPTH - 1>();
  }
  wvm<0>();
  __syncthreads();
  if (threadIdx.x == 0 && lds[5] == 123) sink[0] = 1;
}

template <int PAT, int DEPTH>
int run(const char* src, uint32_t span, int waves, int blocks, const char* tag) {
  const int iters = 2048;
  int* sink; CK(hipMalloc(&sink, 4));
  const size_t shm = (size_t)waves * DEPTH * 1024;
  if (shm > 160 * 1024) return 0;
  CK(hipFuncSetAttribute((const void*)dma_kernel<PAT, DEPTH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((dma_kernel<PAT, DEPTH>), dim3(blocks), dim3(64 * waves), shm, 0, src, span, iters, sink);
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((dma_kernel<PAT, DEPTH>), dim3(blocks), dim3(64 * waves), shm, 0, src, span, iters, sink);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)reps * blocks * waves * iters * 1024.0;
  const double gbs = bytes / (ms * 1e-3) / 1e9;
  printf("%-6s pat %d depth %2d waves %d blocks %4d span %8u KiB : %8.1f GB/s chip  %6.1f GB/s/CU  %5.1f B/clk/CU@2.1GHz\n", tag, PAT, DEPTH,
         waves, blocks, span >> 10, gbs, gbs / 256, gbs / 256 / 2.1);
  CK(hipFree(sink));
  return 0;
}

int main(int argc, char** argv) {
  char* src; const size_t big = (size_t)1 << 30;
  CK(hipMalloc(&src, big)); CK(hipMemset(src, 1, big));
  const uint32_t l2 = 2u << 20, hbm = (uint32_t)big;
  if (argc > 1) {  // lockstep study: one 400 KiB weight matrix streamed by every CU
    const uint32_t w = 400u << 10;
    run<0, 8>(src, w, 4, 256, "W400"); run<4, 8>(src, w, 4, 256, "W400"); run<5, 8>(src, w, 4, 256, "W400");
    run<0, 8>(src, w, 4, 512, "W400"); run<4, 8>(src, w, 4, 512, "W400"); run<5, 8>(src, w, 4, 512, "W400");
    run<4, 16>(src, w, 4, 256, "W400"); run<5, 16>(src, w, 4, 256, "W400");
    return 0;
  }
  for (uint32_t span : {l2, hbm}) {
    const char* tag = span == l2 ? "L2" : "HBM";
    run<0, 4>(src, span, 4, 256, tag); run<0, 8>(src, span, 4, 256, tag); run<0, 16>(src, span, 4, 256, tag);
    run<0, 8>(src, span, 8, 256, tag); run<0, 16>(src, span, 8, 256, tag); run<0, 8>(src, span, 4, 512, tag);
    run<0, 16>(src, span, 4, 512, tag); run<0, 8>(src, span, 8, 512, tag);
    run<1, 8>(src, span, 8, 256, tag); run<1, 16>(src, span, 8, 256, tag);
    run<2, 8>(src, span, 8, 256, tag); run<2, 16>(src, span, 8, 256, tag);
    run<3, 8>(src, span, 8, 256, tag); run<3, 16>(src, span, 8, 256, tag);
  }
  return 0;
}
