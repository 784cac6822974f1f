// Main-loop probe for the conv / GEMM cores: a 256 x 256 block tile (8 waves, 128 x 64 per wave, two waves per
// SIMD) fed from LDS by ds_read_b128 over 64-deep K steps, operands resident (random bf16 in [-1, 1)), so it
// measures the LDS -> MFMA loop alone.  Two questions the round-4 review asked to be measured, not argued:
//   1. MFMA shape: v_mfma_f32_16x16x32_bf16 (what every mdtf core uses) vs v_mfma_f32_32x32x16_bf16 at the same
//      wave tile, the same LDS image and the same bytes read per K step;
//   2. the price of applying a BatchNorm (per-input-channel scale / shift + ReLU) to the A operand inside the
//      consumer conv's main loop, the fusion that would remove bn_apply before a 1x1 conv:
//        XF 0: plain;  XF 1: transform every A fragment in registers after its LDS read (per wave, so an A element
//        is transformed by each of the 4 waves that read it);  XF 2: transform the block's A tile once per K step
//        (LDS raw -> registers -> LDS operand image, double-buffered, one barrier per K step), the MFMAs read the
//        transformed image.
// Timing: alternating variants in one process, several rounds, median (cdna_hip_programming.md rule 24); wave cycles
// from clock64 give the held clock.
// Build: hipcc -O3 --offload-arch=gfx950 bench/mfma_loop_probe.hip -o bench/mfma_loop_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short bf16_t;

constexpr int kRows = 256;           // block tile rows (A) and columns (B)
constexpr int kRowBytes = 128;       // 64 k of bf16 per row
constexpr int kImg = kRows * kRowBytes;  // 32 KiB per operand image

// 16-B chunk c of row r; conflict-free for ds_read_b128 of 16 consecutive rows at one logical chunk
__device__ __forceinline__ int off(int r, int c) { return r * kRowBytes + ((c ^ ((r >> 1) & 7)) << 4); }

__device__ __forceinline__ bf16x8 rd(const char* lds, int r, int c) {
  return *reinterpret_cast<const bf16x8*>(lds + off(r, c));
}

__device__ __forceinline__ bf16x8 xf8(bf16x8 a, const float* s, const float* t) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)fmaxf(fmaf((float)a[j], s[j], t[j]), 0.f);
  return o;
}

template <int SHAPE, int XF>
__global__ void __launch_bounds__(512, 1)
    loop_kernel(const bf16_t* ga, const bf16_t* gb, const float* gst, int iters, float* out, long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* la = smem;             // A operand image (XF 2: two transformed images)
  char* lb = smem + 2 * kImg;  // B operand image
  char* lr = smem + 3 * kImg;  // XF 2: raw A image
  float* lst = reinterpret_cast<float*>(smem + 4 * kImg);  // 64 scales, 64 shifts
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // fill: 256 rows x 8 chunks per image, 4 chunks per thread
  for (int q = tid; q < kRows * 8; q += 512) {
    const int r = q >> 3, c = q & 7;
    const uint4 va = reinterpret_cast<const uint4*>(ga)[q], vb = reinterpret_cast<const uint4*>(gb)[q];
    *reinterpret_cast<uint4*>(lb + off(r, c)) = vb;
    *reinterpret_cast<uint4*>(la + off(r, c)) = va;
    *reinterpret_cast<uint4*>(la + kImg + off(r, c)) = va;
    *reinterpret_cast<uint4*>(lr + off(r, c)) = va;
  }
  if (tid < 128) lst[tid] = gst[tid];
  __syncthreads();
  const int wm = w >> 2, wn = w & 3;  // 2 x 4 waves: rows 128 wm.., cols 64 wn..
  const long long t0 = clock64();
  constexpr int NI = SHAPE == 16 ? 8 : 4, NJ = SHAPE == 16 ? 4 : 2, NK = SHAPE == 16 ? 2 : 4;
  typedef typename std::conditional<SHAPE == 16, f32x4, f32x16>::type acc_t;
  acc_t acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = acc_t{};
  const int fr = SHAPE == 16 ? (lane & 15) : (lane & 31), fh = SHAPE == 16 ? (lane >> 4) : (lane >> 5);
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");  // the operands are re-read from LDS every K step, as in the cores
    const char* A = la;
    if (XF == 2) {
      // transform the raw tile into image (it + 1) & 1 while the MFMAs below read image it & 1
      char* dst = la + ((it + 1) & 1) * kImg;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = tid + u * 512, r = q >> 3, c = q & 7;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(lr + off(r, c));
        float s[8], t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = lst[c * 8 + j], t[j] = lst[64 + c * 8 + j];
        *reinterpret_cast<bf16x8*>(dst + off(r, c)) = xf8(v, s, t);
      }
      A = la + (it & 1) * kImg;
    }
#pragma unroll
    for (int ks = 0; ks < NK; ++ks) {
      const int c = ks * (SHAPE == 16 ? 4 : 2) + fh;  // this lane's 8-k chunk
      float s[8], t[8];
      if (XF == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = lst[c * 8 + j], t[j] = lst[64 + c * 8 + j];
      }
      bf16x8 fb[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = rd(lb, 64 * wn + SHAPE * j + fr, c);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        bf16x8 fa = rd(A, 128 * wm + SHAPE * i + fr, c);
        if (XF == 1) fa = xf8(fa, s, t);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (SHAPE == 16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    if (XF == 2) __syncthreads();
  }
  const long long t1 = clock64();
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < (SHAPE == 16 ? 4 : 16); ++e) sum += acc[i][j][e];
  out[(long long)blockIdx.x * 512 + tid] = sum;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

struct Variant {
  const char* name;
  void (*k)(const bf16_t*, const bf16_t*, const float*, int, float*, long long*);
  int shape, xf;
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 256;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = cus * 4;
  std::vector<uint16_t> ha(kRows * 64), hb(kRows * 64);
  std::vector<float> hst(128);
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0f / 16777216.0f); };
  for (auto& v : ha) v = f2bf(rnd() * 2.f - 1.f);
  for (auto& v : hb) v = f2bf(rnd() * 2.f - 1.f);
  for (int i = 0; i < 64; ++i) hst[i] = 0.5f + rnd(), hst[64 + i] = rnd() - 0.5f;
  bf16_t *da, *db;
  float *dst, *dout;
  long long* dcyc;
  CK(hipMalloc(&da, ha.size() * 2));
  CK(hipMalloc(&db, hb.size() * 2));
  CK(hipMalloc(&dst, 128 * 4));
  CK(hipMalloc(&dout, (size_t)grid * 512 * 4));
  CK(hipMalloc(&dcyc, (size_t)grid * 8));
  CK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dst, hst.data(), 128 * 4, hipMemcpyHostToDevice));
  Variant vs[] = {
      {"16x16x32", loop_kernel<16, 0>, 16, 0},         {"32x32x16", loop_kernel<32, 0>, 32, 0},
      {"16x16x32+xf_reg", loop_kernel<16, 1>, 16, 1},  {"32x32x16+xf_reg", loop_kernel<32, 1>, 32, 1},
      {"16x16x32+xf_lds", loop_kernel<16, 2>, 16, 2},  {"32x32x16+xf_lds", loop_kernel<32, 2>, 32, 2},
  };
  const int nv = sizeof(vs) / sizeof(vs[0]);
  const size_t lds = 4 * kImg + 512;
  for (auto& v : vs) CK(hipFuncSetAttribute((const void*)v.k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(nv), cyc(nv);
  std::vector<long long> hc(grid);
  printf("{\"cus\": %d, \"grid\": %d, \"iters\": %d}\n", cus, grid, iters);
  for (int r = -1; r < rounds; ++r) {
    for (int v = 0; v < nv; ++v) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(512), lds, 0, da, db, dst, iters, dout, dcyc);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      CK(hipMemcpy(hc.data(), dcyc, (size_t)grid * 8, hipMemcpyDeviceToHost));
      double cs = 0;
      for (long long c : hc) cs += (double)c;
      if (r >= 0) ms[v].push_back(t), cyc[v].push_back(cs / grid);
    }
  }
  const double flop = 2.0 * kRows * kRows * 64.0 * iters * grid;
  for (int v = 0; v < nv; ++v) {
    std::vector<double> a = ms[v], c = cyc[v];
    std::sort(a.begin(), a.end());
    std::sort(c.begin(), c.end());
    const double t = a[a.size() / 2], cy = c[c.size() / 2];
    // blocks run in grid / cus waves of one block per CU, so per-CU busy cycles = cy * grid / cus
    const double ghz = cy * grid / cus / (t * 1e6);
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"min_ms\": %.3f, \"tflops\": %.1f, \"block_cycles\": %.0f, "
           "\"cycles_per_kstep\": %.1f, \"clock_ghz\": %.3f}\n",
           vs[v].name, t, a[0], flop / (t * 1e-3) / 1e12, cy, cy / iters, ghz);
  }
  return 0;
}
