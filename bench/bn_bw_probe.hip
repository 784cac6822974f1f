// Bandwidth probe for the BN backward elementwise pass (bn_dx_kernel shape: dx = k1*(dy*mask) + k2*x + k3, two
// bf16 streams + a 1-bit mask in, one bf16 stream out) at the ResNet-50 stage-1 size, in several structures, next
// to copy / 2-in-1-out baselines of the same byte counts.  Which structure reaches the HBM rate decides how the
// BN kernels (csrc/bn.hip) are written.
// Build: hipcc -O3 --offload-arch=gfx950 bench/bn_bw_probe.hip -o bench/bn_bw_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned short bf16_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf(uint32_t w, int hi) { return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)); }
__device__ __forceinline__ uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

template <bool NT>
__device__ __forceinline__ u32x4 ld(const bf16_t* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(bf16_t* p, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else
    *reinterpret_cast<u32x4*>(p) = v;
}

__device__ __forceinline__ u32x4 body(u32x4 g, u32x4 x, uint32_t m, const float* A, const float* B, const float* E) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float g0 = ((m >> (2 * k)) & 1u) ? bf(g[k], 0) : 0.f, g1 = ((m >> (2 * k + 1)) & 1u) ? bf(g[k], 1) : 0.f;
    float a = A[2 * k] * g0 + B[2 * k] * bf(x[k], 0) + E[2 * k];
    float b = A[2 * k + 1] * g1 + B[2 * k + 1] * bf(x[k], 1) + E[2 * k + 1];
    o[k] = f2bf(a) | (f2bf(b) << 16);
  }
  return o;
}

// chunked (the current kernel): block = VPT*256 contiguous vectors, thread t: base + u*256
template <int VPT, bool NTL, bool NTS, int TH>
__global__ void __launch_bounds__(TH) k_dx(const bf16_t* dy, const bf16_t* x, const uint8_t* mk, bf16_t* dx,
                                           long long n8, int C, const float* k1, const float* k2, const float* k3) {
  const long long base = (long long)blockIdx.x * TH * VPT + threadIdx.x;
  u32x4 g[VPT], xv[VPT];
  uint32_t m[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const long long i = base + u * TH;
    const bool ok = i < n8;
    g[u] = ok ? ld<NTL>(dy + i * 8) : u32x4{0, 0, 0, 0};
    xv[u] = ok ? ld<NTL>(x + i * 8) : u32x4{0, 0, 0, 0};
    m[u] = ok ? mk[i] : 0u;
  }
  const int c = (int)((base * 8) % C);
  float A[8], B[8], E[8];
  for (int k = 0; k < 8; ++k) A[k] = k1[c + k], B[k] = k2[c + k], E[k] = k3[c + k];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const long long i = base + u * TH;
    if (i < n8) st<NTS>(dx + i * 8, body(g[u], xv[u], m[u], A, B, E));
  }
}

// mask as one dword per thread: thread t of a block owns 4 CONSECUTIVE vectors (mask bytes 4t..4t+3)
template <bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_dx_q(const bf16_t* dy, const bf16_t* x, const uint8_t* mk, bf16_t* dx,
                                              long long n8, int C, const float* k1, const float* k2, const float* k3) {
  const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= n8) return;
  u32x4 g[4], xv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    g[u] = ld<NTL>(dy + (i0 + u) * 8);
    xv[u] = ld<NTL>(x + (i0 + u) * 8);
  }
  const uint32_t m4 = *reinterpret_cast<const uint32_t*>(mk + i0);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = (int)(((i0 + u) * 8) % C);
    float A[8], B[8], E[8];
    for (int k = 0; k < 8; ++k) A[k] = k1[c + k], B[k] = k2[c + k], E[k] = k3[c + k];
    st<NTS>(dx + (i0 + u) * 8, body(g[u], xv[u], (m4 >> (8 * u)) & 0xffu, A, B, E));
  }
}

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const bf16_t* x, bf16_t* y, long long n8) {
  const long long base = (long long)blockIdx.x * 1024 + threadIdx.x;
  u32x4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = base + u * 256 < n8 ? ld<NT>(x + (base + u * 256) * 8) : u32x4{0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * 256 < n8) st<NT>(y + (base + u * 256) * 8, v[u]);
}

template <bool NT>
__global__ void __launch_bounds__(256) k_add(const bf16_t* x, const bf16_t* r, bf16_t* y, long long n8) {
  const long long base = (long long)blockIdx.x * 1024 + threadIdx.x;
  u32x4 v[4], w[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = base + u * 256;
    v[u] = i < n8 ? ld<NT>(x + i * 8) : u32x4{0, 0, 0, 0};
    w[u] = i < n8 ? ld<NT>(r + i * 8) : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * 256 < n8) st<NT>(y + (base + u * 256) * 8, v[u] ^ w[u]);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const long long M = 256LL * 56 * 56;
  const int C = 256;
  const long long n = M * C, n8 = n / 8;
  bf16_t *dy, *x, *dx;
  uint8_t* mk;
  float *k1, *k2, *k3;
  CK(hipMalloc(&dy, n * 2));
  CK(hipMalloc(&x, n * 2));
  CK(hipMalloc(&dx, n * 2));
  CK(hipMalloc(&mk, n8));
  CK(hipMalloc(&k1, C * 4));
  CK(hipMalloc(&k2, C * 4));
  CK(hipMalloc(&k3, C * 4));
  CK(hipMemset(dy, 0x3f, n * 2));
  CK(hipMemset(x, 0x3e, n * 2));
  CK(hipMemset(mk, 0x5a, n8));
  CK(hipMemset(k1, 0, C * 4));
  CK(hipMemset(k2, 0, C * 4));
  CK(hipMemset(k3, 0, C * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bdx = 3.0 * n * 2 + n8, bcopy = 2.0 * n * 2, badd = 3.0 * n * 2;
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int rep = 0; rep < 15; ++rep) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"kernel\": \"%s\", \"us\": %.1f, \"TBs\": %.2f}\n", name, 1000.0 * ts[ts.size() / 2],
           bytes / ts[ts.size() / 2] / 1e9);
    fflush(stdout);
    return 0;
  };
  for (int rnd = 0; rnd < 2; ++rnd) {
    run("copy", bcopy, [&] { hipLaunchKernelGGL(k_copy<false>, dim3((n8 + 1023) / 1024), dim3(256), 0, 0, x, dx, n8); });
    run("copy_nt", bcopy, [&] { hipLaunchKernelGGL(k_copy<true>, dim3((n8 + 1023) / 1024), dim3(256), 0, 0, x, dx, n8); });
    run("add2in1out", badd, [&] { hipLaunchKernelGGL(k_add<false>, dim3((n8 + 1023) / 1024), dim3(256), 0, 0, x, dy, dx, n8); });
    run("add2in1out_nt", badd, [&] { hipLaunchKernelGGL(k_add<true>, dim3((n8 + 1023) / 1024), dim3(256), 0, 0, x, dy, dx, n8); });
    run("dx_vpt4 (current)", bdx, [&] {
      hipLaunchKernelGGL((k_dx<4, false, false, 256>), dim3((n8 + 1023) / 1024), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_vpt8", bdx, [&] {
      hipLaunchKernelGGL((k_dx<8, false, false, 256>), dim3((n8 + 2047) / 2048), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_vpt2", bdx, [&] {
      hipLaunchKernelGGL((k_dx<2, false, false, 256>), dim3((n8 + 511) / 512), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_vpt4_ntload", bdx, [&] {
      hipLaunchKernelGGL((k_dx<4, true, false, 256>), dim3((n8 + 1023) / 1024), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_vpt4_ntstore", bdx, [&] {
      hipLaunchKernelGGL((k_dx<4, false, true, 256>), dim3((n8 + 1023) / 1024), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_vpt4_ntboth", bdx, [&] {
      hipLaunchKernelGGL((k_dx<4, true, true, 256>), dim3((n8 + 1023) / 1024), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_vpt4_512thr", bdx, [&] {
      hipLaunchKernelGGL((k_dx<4, false, false, 512>), dim3((n8 + 2047) / 2048), dim3(512), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_quad_mask32", bdx, [&] {
      hipLaunchKernelGGL((k_dx_q<false, false>), dim3((n8 + 1023) / 1024), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
    run("dx_quad_mask32_nt", bdx, [&] {
      hipLaunchKernelGGL((k_dx_q<true, true>), dim3((n8 + 1023) / 1024), dim3(256), 0, 0, dy, x, mk, dx, n8, C, k1, k2, k3);
    });
  }
  return 0;
}
