// Common helpers for mdtf HIP/CDNA4 kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MDTF_EXPORT extern "C" __attribute__((visibility("default")))

// Error codes returned by every launcher (0 = ok, >0 = hipError_t, <0 = argument errors).
enum MdtfStatus { MDTF_OK = 0, MDTF_EINVAL = -1, MDTF_EUNSUPPORTED = -2 };

#define MDTF_LAUNCH_CHECK()                            \
  do {                                                 \
    hipError_t e_ = hipGetLastError();                 \
    if (e_ != hipSuccess) return static_cast<int>(e_); \
  } while (0)

namespace mdtf {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // raw bf16 bits
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

// round-to-nearest-even f32 -> bf16 on the gfx950 conversion unit (v_cvt_pk_bf16_f32: one VALU
// instruction per two values, where a software rounding sequence costs ~6 per value)
__device__ __forceinline__ bf16_t f2bf(float f) {
  const __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, h);
}

// two floats -> packed bf16x2 (lo in bits 0-15), one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const bf2_t v = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 8 x bf16 <-> 8 x f32 through one 16-byte vector access
struct alignas(16) BF8 {
  bf16_t v[8];
};

__device__ __forceinline__ void load_bf8(const bf16_t* p, float (&f)[8]) {
  uint4 raw = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ void store_bf8(bf16_t* p, const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pack_bf2(f[2 * i], f[2 * i + 1]);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

__host__ __device__ __forceinline__ int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// 16 B per lane global -> LDS (buffer_load_dwordx4 ... lds): LDS destination = wave-uniform
// `lds` + 16 * lane; offsets at or past `nbytes` read zeros
__device__ __forceinline__ void dma16(const void* base, int nbytes, char* lds, unsigned voff, int soff) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nbytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// Same transfer, issued from inline asm so the compiler does not see an LDS write: it then
// inserts no vmcnt(0) in front of later LDS reads (it cannot prove they miss the DMA target).
// The caller owns the ordering: a counted wait_vmcnt<N>() plus an asm s_barrier with a "memory"
// clobber (which LDS reads cannot move across) before any wave reads the target.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4_t buffer_rsrc(const void* base, int nbytes) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  i32x4_t r;
  r.x = static_cast<int>(p & 0xffffffffu);
  r.y = static_cast<int>((p >> 32) & 0xffffu);
  r.z = nbytes;
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ void dma16_asm(i32x4_t rsrc, const char* lds, unsigned voff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      static_cast<unsigned>(reinterpret_cast<unsigned long long>((__attribute__((address_space(3))) const char*)lds)));
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc), "{m0}"(m0) : "memory");
}

// s_waitcnt vmcnt(N) leaving lgkm/exp counters alone (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// s_waitcnt vmcnt(min(n, N)) for a wave-uniform runtime n (a ladder of scalar compares; n <= N expected)
template <int N>
__device__ __forceinline__ void wait_vmcnt_le(int n) {
  if constexpr (N <= 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N)
      wait_vmcnt<N>();
    else
      wait_vmcnt_le<N - 1>(n);
  }
}

}  // namespace mdtf
