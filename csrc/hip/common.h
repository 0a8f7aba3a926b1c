// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels of this framework.
//
// Element type: every kernel file is compiled once per element type it declares
// (`// dcg-variants:` line, csrc/build.py): elem_t = bf16 (the default training dtype), fp16
// (-DDCG_F16: the 256x256 fp16 config, dynamic loss scaling in the engine) and fp32 (-DDCG_F32:
// the reference precision). Each build lives in its own namespace (dcg, dcg_f16, dcg_f32) and
// its C launchers carry a suffix (DCG_API: none, `_f16`, `_f32`), so all coexist in one .so and
// the Program picks one set per engine. 16-bit MFMA: v_mfma_f32_16x16x32_{bf16,f16} (same lane
// maps, same cycles); fp32: v_mfma_f32_16x16x4_f32 (igemm_f32.hip).
// Wave = 64 lanes. 16x16x32 MFMA fragment lane maps:
//   A: lane l holds A[row l&15][k = 8*(l>>4) + j], j = 0..7
//   B: lane l holds B[k = 8*(l>>4) + j][col l&15]
//   C: lane l holds C[row 4*(l>>4) + r][col l&15], r = 0..3
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#if defined(DCG_F32)
// reference-precision build: fp32 activations / weight mirrors, fp32-input MFMA
// (v_mfma_f32_16x16x4_f32, exact f32 fma chains) in igemm_f32.hip
typedef float elem_t;
typedef float elem8 __attribute__((ext_vector_type(8)));
typedef float elem4 __attribute__((ext_vector_type(4)));
typedef float elem2 __attribute__((ext_vector_type(2)));
#define DCG_API(name) name##_f32
#define dcg dcg_f32
#elif defined(DCG_F16)
typedef _Float16 elem_t;
typedef _Float16 elem8 __attribute__((ext_vector_type(8)));
typedef _Float16 elem4 __attribute__((ext_vector_type(4)));
typedef _Float16 elem2 __attribute__((ext_vector_type(2)));
#define DCG_MFMA_16x16x32 __builtin_amdgcn_mfma_f32_16x16x32_f16
#define DCG_API(name) name##_f16
#define dcg dcg_f16
#else
typedef __bf16 elem_t;
typedef __bf16 elem8 __attribute__((ext_vector_type(8)));
typedef __bf16 elem4 __attribute__((ext_vector_type(4)));
typedef __bf16 elem2 __attribute__((ext_vector_type(2)));
#define DCG_MFMA_16x16x32 __builtin_amdgcn_mfma_f32_16x16x32_bf16
#define DCG_API(name) name
#endif
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

namespace dcg {

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_TANH = 3 };

__device__ __forceinline__ float bf2f(elem_t x) { return (float)x; }

// 8 consecutive elements (16 bytes for 16-bit types, 32 for fp32: two 16-byte accesses)
__device__ __forceinline__ elem8 ld8(const elem_t* p) {
#if defined(DCG_F32)
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  return (elem8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#else
  return __builtin_bit_cast(elem8, *reinterpret_cast<const u32x4*>(p));
#endif
}
__device__ __forceinline__ void st8(elem_t* p, elem8 v) {
#if defined(DCG_F32)
  *reinterpret_cast<f32x4*>(p) = (f32x4){v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = (f32x4){v[4], v[5], v[6], v[7]};
#else
  *reinterpret_cast<u32x4*>(p) = __builtin_bit_cast(u32x4, v);
#endif
}
__device__ __forceinline__ elem_t f2bf(float x) { return (elem_t)x; }

__device__ __forceinline__ float apply_act(float v, int act, float leak) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_LRELU: return fmaxf(v, leak * v);
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// derivative of the activation expressed through its OUTPUT y (valid for relu, lrelu, tanh)
__device__ __forceinline__ float act_grad_from_out(float y, int act, float leak) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_LRELU: return y > 0.f ? 1.f : leak;
    case ACT_TANH: return 1.f - y * y;
    default: return 1.f;
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// 16-byte buffer load; an offset >= the descriptor's byte count returns zeros (HW range check).
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

constexpr uint32_t OOB = 0xF8000000u;  // any offset past the descriptor size (operands < OOB bytes)

// offset, or past the descriptor's range when !ok (a buffer load then returns zeros): arithmetic,
// not a select, so hipcc emits no exec-mask branch per load (valid offsets < OOB by host checks)
__device__ __forceinline__ uint32_t oob_unless(bool ok, uint32_t off) {
  return off | (((uint32_t)ok - 1u) & OOB);
}

// 16-byte LDS-DMA: buffer_load_dwordx4 ... lds. The wave's 64 lanes write 1 KiB contiguously at
// `lds` (wave-uniform) + 16 * lane; the global offset is per lane (out of range -> zeros).
__device__ __forceinline__ void buf_load16_lds(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
#endif
}

// 32-bit LDS address space (ds_* addressing: no generic-pointer null checks)
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) int lds_i32;

// The same 16-byte LDS-DMA as inline asm. hipcc cannot tell which LDS bytes a DMA writes, so
// after the builtin form it waits vmcnt(0) before the next ds_read of ANY LDS address -- which
// drains the tile just issued for the NEXT k-step and serialises load and compute. Hidden in
// asm, the DMA is invisible to its waitcnt pass; the caller orders it with explicit counted
// `s_waitcnt vmcnt(N)` + barrier (and must not mix it with compiler-visible vector loads in
// the same pipelined span). M0 write -> LDS-DMA needs one wait state (s_nop 0).
// variant taking the wave-uniform LDS byte address directly (keeps per-piece addressing in SGPRs)
__device__ __forceinline__ void dma16_asm_la(__amdgpu_buffer_rsrc_t r, uint32_t la_in, uint32_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t la = __builtin_amdgcn_readfirstlane(la_in);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(la), "v"(off), "s"(r) : "memory", "m0");
#pragma clang diagnostic pop
#endif
}

__device__ __forceinline__ void dma16_asm(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(la), "v"(off), "s"(r) : "memory", "m0");
#pragma clang diagnostic pop
#endif
}

// Unsigned division by a runtime-invariant divisor (round-up multiply method, exact for all
// 32-bit n). Host computes {mul, shift} with fastdiv_make().
struct FastDiv {
  uint32_t d, mul, shr;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  if (f.d == 1) return n;
  uint32_t t = __umulhi(n, f.mul);
  return (t + ((n - t) >> 1)) >> f.shr;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- cross-workgroup hand-off helpers (sc1 = write-through / L1-bypassing buffer accesses)
__device__ __forceinline__ void st_sc1_f64(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 16);
}
__device__ __forceinline__ double ld_sc1_f64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16));
}
__device__ __forceinline__ void st_sc1_f32(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 16);
}
__device__ __forceinline__ float ld_sc1_f32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}

// returns true in the last-arriving workgroup of `expected`; every thread of the block agrees
__device__ __forceinline__ bool last_arrival(unsigned* counter, unsigned expected, int* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_lds = old == expected - 1;
    if (*flag_lds) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return *flag_lds != 0;
}

}  // namespace dcg

// host helper
static inline dcg::FastDiv fastdiv_make(uint32_t d) {
  dcg::FastDiv f;
  f.d = d;
  if (d <= 1) { f.mul = 0; f.shr = 0; f.d = 1; return f; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  // mul = floor(2^32 * (2^l - d) / d) + 1
  uint64_t m = ((((uint64_t)1 << l) - d) << 32) / d + 1;
  f.mul = (uint32_t)m;
  f.shr = l - 1;
  return f;
}
