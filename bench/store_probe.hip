// Output-tile store probe: how fast can a GEMM epilogue write a [M][N] bf16 output tile by tile?
// Mimics the conv v2 epilogue's copy-out (16 B per lane along full tile rows) for a 128x128 tile per
// 256-thread block, with and without the XCD-aware block remap, plus the direct MFMA-layout store
// (8 B per lane, 16 rows x 32 B per instruction).  M = 50176, N = 1024 (ResNet-50 stage-3 1x1 expand).
// Build: hipcc -O3 --offload-arch=gfx950 bench/store_probe.hip -o bench/store_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int BM, int BN, bool REMAP>
__global__ void __launch_bounds__(256) tile_rows(unsigned short* out, int M, int N, int ntiles) {
  const int t = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int mt = t / ntiles, nt = t % ntiles;
  const uint4 v = make_uint4(threadIdx.x, 1, 2, 3);
  constexpr int ITER = BM * (BN / 8) / 256;
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int idx = threadIdx.x + it * 256;
    const int row = idx / (BN / 8), c8 = idx % (BN / 8);
    const long long m = (long long)mt * BM + row;
    if (m < M) *reinterpret_cast<uint4*>(out + m * N + nt * BN + c8 * 8) = v;
  }
}

// MFMA 16x16 accumulator layout written straight from registers: lane (li, g) holds 4 channels of one row
template <int BM, int BN, bool REMAP>
__global__ void __launch_bounds__(256) tile_mfma(unsigned short* out, int M, int N, int ntiles) {
  const int t = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int mt = t / ntiles, nt = t % ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave / 2, wn = wave % 2;
  const int li = lane & 15, g = lane >> 4;
  const uint2 v = make_uint2(lane, 7);
  constexpr int TM = BM / 2 / 16, TN = BN / 2 / 16;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const long long m = (long long)mt * BM + wm * (TM * 16) + i * 16 + li;
      const int c = nt * BN + wn * (TN * 16) + j * 16 + 4 * g;
      if (m < M) *reinterpret_cast<uint2*>(out + m * N + c) = v;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const int M = 50176, N = 1024;
  unsigned short* out;
  CK(hipMalloc(&out, (size_t)M * N * 2));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 15; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float ms = ts[ts.size() / 2];
    printf("%-32s %.4f ms  %.2f TB/s\n", name, ms, (double)M * N * 2 / ms / 1e9);
    return 0;
  };
  const int nt128 = N / 128, mt128 = (M + 127) / 128;
  const int nt256 = N / 256;
  run("rows 128x128 remap", [&] { hipLaunchKernelGGL((tile_rows<128, 128, true>), dim3(mt128 * nt128), dim3(256), 0, 0, out, M, N, nt128); });
  run("rows 128x128 linear", [&] { hipLaunchKernelGGL((tile_rows<128, 128, false>), dim3(mt128 * nt128), dim3(256), 0, 0, out, M, N, nt128); });
  run("rows 128x256 remap", [&] { hipLaunchKernelGGL((tile_rows<128, 256, true>), dim3(mt128 * nt256), dim3(256), 0, 0, out, M, N, nt256); });
  run("mfma 128x128 remap", [&] { hipLaunchKernelGGL((tile_mfma<128, 128, true>), dim3(mt128 * nt128), dim3(256), 0, 0, out, M, N, nt128); });
  run("mfma 128x128 linear", [&] { hipLaunchKernelGGL((tile_mfma<128, 128, false>), dim3(mt128 * nt128), dim3(256), 0, 0, out, M, N, nt128); });
  CK(hipMemset(out, 0, (size_t)M * N * 2));
  run("hipMemset", [&] { (void)hipMemsetAsync(out, 0, (size_t)M * N * 2, 0); });
  return 0;
}
