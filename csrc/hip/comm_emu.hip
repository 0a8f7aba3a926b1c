// dcg-variants: bf16
// Stand-in for an RCCL ring all-reduce on ONE GPU (DDP schedule studies, benchmarks/phase_timing.py).
//
// A real RCCL all-reduce is not a timer: its kernel holds `nchannels` workgroups (one CU each) for
// the whole collective and streams about 2 (W-1)/W x the payload through this GPU's HBM (read the
// local chunk, write the received one). `torch.cuda._sleep` (round 3's stand-in) took one thread
// and no bandwidth, so it could not show compute slowing down beside a collective. This kernel
// does what the collective costs the GPU: `nwg` persistent workgroups copy `bytes` (read src, write
// dst) and pace themselves with the constant 100 MHz real-time counter so that the copy ends
// no earlier than `ticks` after it started (the modelled ring time: latency + wire bytes / bus
// bandwidth). Every workgroup exits after its last chunk: no cross-workgroup waits.
#include "kernels.h"

namespace dcg {

__global__ __launch_bounds__(256) void comm_emu_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       uint64_t n16, uint64_t ticks, int chunks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t per_wg = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = (uint64_t)blockIdx.x * per_wg;
  const uint64_t hi = lo + per_wg < n16 ? lo + per_wg : n16;
  const uint64_t per_chunk = (per_wg + chunks - 1) / chunks;
  for (int c = 0; c < chunks; ++c) {
    const uint64_t a = lo + (uint64_t)c * per_chunk;
    const uint64_t b = a + per_chunk < hi ? a + per_chunk : hi;
    for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x) dst[i] = src[i];
    // pace: chunk c may not finish before t0 + (c+1)/chunks of the modelled time
    const uint64_t due = t0 + ticks * (uint64_t)(c + 1) / (uint64_t)chunks;
    while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(2);
  }
}

}  // namespace dcg

extern "C" int dcg_comm_emulate(const void* src, void* dst, size_t bytes, double us, int nwg, hipStream_t s) {
  if (nwg < 1 || nwg > 1024) return -1;
  const uint64_t n16 = bytes / 16;
  const uint64_t ticks = (uint64_t)(us * 100.0);  // s_memrealtime: 100 MHz
  const int chunks = 16;
  hipLaunchKernelGGL(dcg::comm_emu_kernel, dim3(nwg), dim3(256), 0, s, reinterpret_cast<const u32x4*>(src),
                     reinterpret_cast<u32x4*>(dst), n16, ticks, chunks);
  return (int)hipGetLastError();
}
