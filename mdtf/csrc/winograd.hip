// Non-fused Winograd F(2x2, 3x3) convolution: the MI355X implementation of the
// reference's Winograd toggle (TF_ENABLE_WINOGRAD_NONFUSED).
//
//   V[p][t][c]  = (B^T d_t B)[p]     input transform, one 4x4 patch d_t per 2x2 output tile t
//   U[p][c][k]  = (G g G^T)[p]       filter transform (per step: the weights change)
//   M[p][t][k]  = sum_c V[p][t][c] U[p][c][k]     16 independent GEMMs (hipBLASLt batched bf16)
//   Y[t][k]     = A^T M_t A          output transform
//
// Layouts are NHWC / HWIO with channel-contiguous 16-B vectors (8 x bf16) per
// thread: every global access is a full 16-B lane access.  Transforms run in
// fp32 and round to bf16 once.  The dgrad of a stride-1 3x3 conv is the same
// algorithm on DY with the 180-degree-rotated, in/out-transposed filter
// (`flip` of the filter transform).
#include "mdtf_common.h"

using namespace mdtf;

namespace {

constexpr int kT = 256;

// input transform: thread = (tile, 8-channel chunk)
__global__ void __launch_bounds__(kT)
    wino_input_tf(const bf16_t* __restrict__ x, bf16_t* __restrict__ v, int N, int H, int W, int C, int TH, int TW,
                  int PH, int PW) {
  const int cv = C / 8;
  const long long T = (long long)N * TH * TW;
  const long long gid = (long long)blockIdx.x * kT + threadIdx.x;
  if (gid >= T * cv) return;
  const int c0 = static_cast<int>(gid % cv) * 8;
  const long long t = gid / cv;
  const int tw = static_cast<int>(t % TW);
  const int th = static_cast<int>((t / TW) % TH);
  const int n = static_cast<int>(t / ((long long)TW * TH));
  const int y0 = th * 2 - PH, x0 = tw * 2 - PW;
  float d[4][4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int yy = y0 + i, xx = x0 + j;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        load_bf8(x + (((long long)n * H + yy) * W + xx) * C + c0, d[i][j]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) d[i][j][e] = 0.f;
      }
    }
  // B^T d: rows  r0 = d0 - d2, r1 = d1 + d2, r2 = d2 - d1, r3 = d1 - d3
  float b[4][4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b[0][j][e] = d[0][j][e] - d[2][j][e];
      b[1][j][e] = d[1][j][e] + d[2][j][e];
      b[2][j][e] = d[2][j][e] - d[1][j][e];
      b[3][j][e] = d[1][j][e] - d[3][j][e];
    }
  const long long stride_p = T * C;
  bf16_t* out = v + t * C + c0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float r[4][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      r[0][e] = b[i][0][e] - b[i][2][e];
      r[1][e] = b[i][1][e] + b[i][2][e];
      r[2][e] = b[i][2][e] - b[i][1][e];
      r[3][e] = b[i][1][e] - b[i][3][e];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) store_bf8(out + (i * 4 + j) * stride_p, r[j]);
  }
}

// filter transform: g = w[kh][kw][c][k] (flip: g = w[2-kh][2-kw][k][c], the dgrad filter)
// U[p][a][b] with (a, b) = (c, k), or (k, c) when flipped; thread = (a, 8 consecutive b)
__global__ void __launch_bounds__(kT)
    wino_filter_tf(const bf16_t* __restrict__ w, bf16_t* __restrict__ u, int C, int K, int flip) {
  const int A = flip ? K : C, B = flip ? C : K;
  const int bv = B / 8;
  const long long gid = (long long)blockIdx.x * kT + threadIdx.x;
  if (gid >= (long long)A * bv) return;
  const int b0 = static_cast<int>(gid % bv) * 8;
  const int a = static_cast<int>(gid / bv);
  float g[3][3][8];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (!flip) {
        load_bf8(w + ((long long)(i * 3 + j) * C + a) * K + b0, g[i][j]);
      } else {
        // dgrad filter g'[i][j][k=a][c=b] = w[2-i][2-j][c][k]: 8 channels c are K apart
        const bf16_t* p = w + ((long long)((2 - i) * 3 + (2 - j)) * C + b0) * K + a;
#pragma unroll
        for (int e = 0; e < 8; ++e) g[i][j][e] = bf2f(p[(long long)e * K]);
      }
    }
  // G g: rows  q0 = g0, q1 = (g0+g1+g2)/2, q2 = (g0-g1+g2)/2, q3 = g2
  float q[4][3][8];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      q[0][j][e] = g[0][j][e];
      q[1][j][e] = 0.5f * (g[0][j][e] + g[1][j][e] + g[2][j][e]);
      q[2][j][e] = 0.5f * (g[0][j][e] - g[1][j][e] + g[2][j][e]);
      q[3][j][e] = g[2][j][e];
    }
  const long long stride_p = (long long)A * B;
  bf16_t* out = u + (long long)a * B + b0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float r[4][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      r[0][e] = q[i][0][e];
      r[1][e] = 0.5f * (q[i][0][e] + q[i][1][e] + q[i][2][e]);
      r[2][e] = 0.5f * (q[i][0][e] - q[i][1][e] + q[i][2][e]);
      r[3][e] = q[i][2][e];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) store_bf8(out + (i * 4 + j) * stride_p, r[j]);
  }
}

// output transform: thread = (tile, 8-channel chunk); A^T m: r0 = m0 + m1 + m2, r1 = m1 - m2 - m3
__global__ void __launch_bounds__(kT)
    wino_output_tf(const bf16_t* __restrict__ m, bf16_t* __restrict__ y, int N, int OH, int OW, int K, int TH,
                   int TW) {
  const int kv = K / 8;
  const long long T = (long long)N * TH * TW;
  const long long gid = (long long)blockIdx.x * kT + threadIdx.x;
  if (gid >= T * kv) return;
  const int k0 = static_cast<int>(gid % kv) * 8;
  const long long t = gid / kv;
  const int tw = static_cast<int>(t % TW);
  const int th = static_cast<int>((t / TW) % TH);
  const int n = static_cast<int>(t / ((long long)TW * TH));
  const long long stride_p = T * K;
  const bf16_t* in = m + t * K + k0;
  float s[2][4][8];                // A^T applied over the rows
  {
    float mm[4][4][8];
#pragma unroll
    for (int p = 0; p < 16; ++p) load_bf8(in + p * stride_p, mm[p / 4][p % 4]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[0][j][e] = mm[0][j][e] + mm[1][j][e] + mm[2][j][e];
        s[1][j][e] = mm[1][j][e] - mm[2][j][e] - mm[3][j][e];
      }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oy = th * 2 + i;
    if (oy >= OH) continue;
    float r[2][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      r[0][e] = s[i][0][e] + s[i][1][e] + s[i][2][e];
      r[1][e] = s[i][1][e] - s[i][2][e] - s[i][3][e];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ox = tw * 2 + j;
      if (ox < OW) store_bf8(y + (((long long)n * OH + oy) * OW + ox) * K + k0, r[j]);
    }
  }
}

inline unsigned grid_for(long long threads) { return static_cast<unsigned>(ceil_div(threads, kT)); }

}  // namespace

// V: [16][N*TH*TW][C] bf16, TH = ceil(OH/2), TW = ceil(OW/2)
MDTF_EXPORT int mdtf_wino_input(const void* x, void* v, int N, int H, int W, int C, int OH, int OW, int PH, int PW,
                                hipStream_t st) {
  if (C % 8) return MDTF_EINVAL;
  const int TH = (OH + 1) / 2, TW = (OW + 1) / 2;
  const long long thr = (long long)N * TH * TW * (C / 8);
  if (thr == 0) return 0;
  hipLaunchKernelGGL(wino_input_tf, dim3(grid_for(thr)), dim3(kT), 0, st, (const bf16_t*)x, (bf16_t*)v, N, H, W, C,
                     TH, TW, PH, PW);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// U: [16][C][K] (flip = 0) or [16][K][C] (flip = 1: the dgrad filter)
MDTF_EXPORT int mdtf_wino_filter(const void* w, void* u, int C, int K, int flip, hipStream_t st) {
  if (C % 8 || K % 8) return MDTF_EINVAL;
  const long long thr = (long long)(flip ? K : C) * ((flip ? C : K) / 8);
  hipLaunchKernelGGL(wino_filter_tf, dim3(grid_for(thr)), dim3(kT), 0, st, (const bf16_t*)w, (bf16_t*)u, C, K, flip);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// M: [16][N*TH*TW][K] -> Y [N][OH][OW][K]
MDTF_EXPORT int mdtf_wino_output(const void* m, void* y, int N, int OH, int OW, int K, hipStream_t st) {
  if (K % 8) return MDTF_EINVAL;
  const int TH = (OH + 1) / 2, TW = (OW + 1) / 2;
  const long long thr = (long long)N * TH * TW * (K / 8);
  if (thr == 0) return 0;
  hipLaunchKernelGGL(wino_output_tf, dim3(grid_for(thr)), dim3(kT), 0, st, (const bf16_t*)m, (bf16_t*)y, N, OH, OW, K,
                     TH, TW);
  MDTF_LAUNCH_CHECK();
  return 0;
}
