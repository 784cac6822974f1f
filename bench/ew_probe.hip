// Elementwise streaming probe: BN-apply-shaped kernels (y = x*s + h + r, ReLU, 1-bit mask) at the
// ResNet-50 stage-1 size, in several loop/launch structures, to find what reaches HBM rate.
// Build: hipcc -O3 --offload-arch=gfx950 bench/ew_probe.hip -o bench/ew_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef unsigned short bf16_t;

__device__ __forceinline__ float bf(uint32_t w, int hi) { return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)); }
__device__ __forceinline__ uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

template <bool MASK>
__device__ __forceinline__ void body(const uint4& xr, const uint4& rr, const float* sc, const float* sh, bf16_t* y,
                                     uint8_t* mask, long long i) {
  const uint32_t xw[4] = {xr.x, xr.y, xr.z, xr.w}, rw[4] = {rr.x, rr.y, rr.z, rr.w};
  uint32_t o[4], bits = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float a = fmaxf(bf(xw[k], 0) * sc[2 * k] + sh[2 * k] + bf(rw[k], 0), 0.f);
    float b = fmaxf(bf(xw[k], 1) * sc[2 * k + 1] + sh[2 * k + 1] + bf(rw[k], 1), 0.f);
    bits |= (a > 0.f ? 1u : 0u) << (2 * k);
    bits |= (b > 0.f ? 1u : 0u) << (2 * k + 1);
    o[k] = f2bf(a) | (f2bf(b) << 16);
  }
  *reinterpret_cast<uint4*>(y + i * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  if (MASK) mask[i] = (uint8_t)bits;
}

// A: grid-stride, 4 vectors in flight, channel-invariant coefficients (the current kernel)
template <bool MASK>
__global__ void __launch_bounds__(256) k_stride4(const bf16_t* x, const bf16_t* r, bf16_t* y, uint8_t* mask,
                                                 long long n8, int C, const float* scale, const float* shift) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const int c = (int)((i * 8) % C);
  float sc[8], sh[8];
  for (int k = 0; k < 8; ++k) sc[k] = scale[c + k], sh[k] = shift[c + k];
  for (; i + 3 * stride < n8; i += 4 * stride) {
    uint4 xr[4], rr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xr[u] = *reinterpret_cast<const uint4*>(x + (i + u * stride) * 8);
      rr[u] = *reinterpret_cast<const uint4*>(r + (i + u * stride) * 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body<MASK>(xr[u], rr[u], sc, sh, y, mask, i + u * stride);
  }
  for (; i < n8; i += stride)
    body<MASK>(*reinterpret_cast<const uint4*>(x + i * 8), *reinterpret_cast<const uint4*>(r + i * 8), sc, sh, y,
               mask, i);
}

// B: one block per contiguous chunk of VPT*256 vectors (torch-style), no grid-stride loop
template <bool MASK, int VPT>
__global__ void __launch_bounds__(256) k_chunk(const bf16_t* x, const bf16_t* r, bf16_t* y, uint8_t* mask,
                                               long long n8, int C, const float* scale, const float* shift) {
  const long long base = (long long)blockIdx.x * 256 * VPT + threadIdx.x;
  uint4 xr[VPT], rr[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const long long i = base + u * 256;
    if (i < n8) {
      xr[u] = *reinterpret_cast<const uint4*>(x + i * 8);
      rr[u] = *reinterpret_cast<const uint4*>(r + i * 8);
    }
  }
  // with C | 2048 and 256 threads, a thread's channel group is fixed across u
  const int c = (int)((base * 8) % C);
  float sc[8], sh[8];
  for (int k = 0; k < 8; ++k) sc[k] = scale[c + k], sh[k] = shift[c + k];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const long long i = base + u * 256;
    if (i < n8) body<MASK>(xr[u], rr[u], sc, sh, y, mask, i);
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const long long M = 256LL * 56 * 56;
  const int C = 256;
  const long long n = M * C, n8 = n / 8;
  bf16_t *x, *r, *y;
  uint8_t* mask;
  float *sc, *sh;
  CK(hipMalloc(&x, n * 2));
  CK(hipMalloc(&r, n * 2));
  CK(hipMalloc(&y, n * 2));
  CK(hipMalloc(&mask, n8));
  CK(hipMalloc(&sc, C * 4));
  CK(hipMalloc(&sh, C * 4));
  CK(hipMemset(x, 0x3f, n * 2));
  CK(hipMemset(r, 0x3e, n * 2));
  CK(hipMemset(sc, 0, C * 4));
  CK(hipMemset(sh, 0, C * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes_mask = 3.0 * n * 2 + n8, bytes_nomask = 3.0 * n * 2;
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
    printf("%-34s %.3f ms  %.2f TB/s\n", name, ts[ts.size() / 2], bytes / ts[ts.size() / 2] / 1e9);
    return 0;
  };
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "stride4 mask grid %d", g);
    run(nm, bytes_mask, [&] { hipLaunchKernelGGL(k_stride4<true>, dim3(g), dim3(256), 0, 0, x, r, y, mask, n8, C, sc, sh); });
    snprintf(nm, 64, "stride4 nomask grid %d", g);
    run(nm, bytes_nomask, [&] { hipLaunchKernelGGL(k_stride4<false>, dim3(g), dim3(256), 0, 0, x, r, y, mask, n8, C, sc, sh); });
  }
  long long g1 = (n8 + 255) / 256, g4 = (n8 + 1023) / 1024, g8 = (n8 + 2047) / 2048;
  run("chunk1 mask", bytes_mask, [&] { hipLaunchKernelGGL((k_chunk<true, 1>), dim3(g1), dim3(256), 0, 0, x, r, y, mask, n8, C, sc, sh); });
  run("chunk4 mask", bytes_mask, [&] { hipLaunchKernelGGL((k_chunk<true, 4>), dim3(g4), dim3(256), 0, 0, x, r, y, mask, n8, C, sc, sh); });
  run("chunk8 mask", bytes_mask, [&] { hipLaunchKernelGGL((k_chunk<true, 8>), dim3(g8), dim3(256), 0, 0, x, r, y, mask, n8, C, sc, sh); });
  run("chunk4 nomask", bytes_nomask, [&] { hipLaunchKernelGGL((k_chunk<false, 4>), dim3(g4), dim3(256), 0, 0, x, r, y, mask, n8, C, sc, sh); });
  return 0;
}
