// Weight gradient of the few-channel stem convolution (ResNet's 7x7/2 on RGB) on bf16 MFMA (gfx950).
//
// The forward (conv_ws.hip, mdtf_conv_ws_stem) repacks the image into a zero-haloed 4-channel layout
// x4[N][H4][W4][4], in which the KW(<=8) taps x 4 channels of one filter row are 32 contiguous elements
// for every output pixel.  The weight gradient is then a GEMM
//     dW^T-ish  C[r][co] = sum_p X[p][r] * DY[p][co],   r = kh*32 + kw*4 + c  (KHP*32 rows, 64 columns)
// reduced over the output pixels p.  Both operands are pixel-major in memory, so a block stages 32 pixels
// per k-step in LDS by LDS-DMA -- X as 4 [32 px][64 r] sub-images (the 64-B row segments of two filter rows
// per 128-B image row), DY as one [32 px][64 co] image -- and reads both MFMA operands with
// ds_read_b64_tr_b16 (hardware transpose) under one key permutation; 8 waves own 32 r x 64 co each.  Blocks
// split the pixels; each adds its C tile into the fp32 weight-gradient slot with one atomic per element of
// the real filter.  Replaces MIOpen's stem weight gradient (reference distribute_tools.py:76).
#include "mdtf_common.h"

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr unsigned kOOB = 0x80000000u;

struct SwzV {    // 128-B rows read transposed, rows {4g+q} / {16+4g+q}
  __device__ static int f(int r, int c) { return c ^ (((r >> 1) & 3) << 1); }
};

__device__ __forceinline__ float4v mfma(const bf16x8_t& a, const bf16x8_t& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ v4s tr4(const char* img, int r, int col) {
  const char* p = img + r * 128 + (SwzV::f(r, col >> 3) << 4) + (col & 7) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p);
}

// operand X^T[col][k] (or B[k][col]: the same register layout) from a [32 k][64 col] image, k order
// {4g..4g+3, 16+4g..16+4g+3} -- identical for both operands, which the k reduction does not see
__device__ __forceinline__ bf16x8_t trp_frag(const char* img, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
  const v4s lo = tr4(img, 4 * g + q4, col0 + 4 * p4);
  const v4s hi = tr4(img, 16 + 4 * g + q4, col0 + 4 * p4);
  const short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, f);
}

constexpr int kX = 4 * 32 * 128;        // 4 X sub-images
constexpr int kStage = kX + 32 * 128;   // + the DY image

__global__ void __launch_bounds__(512) stem_wgrad_kernel(const bf16_t* __restrict__ x4, const bf16_t* __restrict__ dy,
                                                          float* __restrict__ dw, int N, int H4, int W4, int OH, int OW,
                                                          int SH, int SW, int KH, int KW, int CI, unsigned m_ow,
                                                          int s_ow, unsigned m_oh, int s_oh, int steps_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long M = (long long)N * OH * OW;
  const int xbytes = (int)((long long)N * H4 * W4 * 4 * 2);
  const int dbytes = (int)(M * 64 * 2);
  const long long ks_total = (M + 31) / 32;
  const long long ks0 = (long long)blockIdx.x * steps_per_block;
  long long ks1 = ks0 + steps_per_block;
  if (ks1 > ks_total) ks1 = ks_total;

  // this lane's DMA piece: X instructions j = wave, wave + 8 (16 per stage), DY instruction j = wave (< 4)
  auto stage = [&](long long ks, int buf) {
    char* base = smem + buf * kStage;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wave + 8 * jj;               // 0..15
      const int s = j >> 2;                      // sub-image: filter rows 2s, 2s+1
      const int px = (j & 3) * 8 + (lane >> 3);
      const int c = SwzV::f(px, lane & 7);       // logical 16-B chunk of the 128-B image row
      const long long p = ks * 32 + px;
      unsigned voff = kOOB;
      if (p < M) {
        const unsigned pu = (unsigned)p;
        const unsigned q = (__umulhi(pu, m_ow) + pu) >> s_ow;
        const int ow = (int)(pu - q * (unsigned)OW);
        const unsigned n = (__umulhi(q, m_oh) + q) >> s_oh;
        const int oh = (int)(q - n * (unsigned)OH);
        const int kh = 2 * s + (c >> 2);
        const long long e = (((long long)n * H4 + oh * SH + kh) * W4 + ow * SW) * 4 + (c & 3) * 8;
        voff = (unsigned)(e * 2);
      }
      dma16(x4, xbytes, base + j * 1024, voff, 0);
    }
    if (wave < 4) {
      const int px = wave * 8 + (lane >> 3);
      const int c = SwzV::f(px, lane & 7);
      const long long p = ks * 32 + px;
      const unsigned voff = p < M ? (unsigned)((p * 64 + c * 8) * 2) : kOOB;
      dma16(dy, dbytes, base + kX + wave * 1024, voff, 0);
    }
  };

  float4v acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[i][c] = float4v{0.f, 0.f, 0.f, 0.f};
  if (ks0 < ks1) stage(ks0, 0);
  for (long long ks = ks0; ks < ks1; ++ks) {
    const int buf = (int)((ks - ks0) & 1);
    wait_vmcnt<0>();
    __syncthreads();                             // stage ks landed; the other buffer is free
    if (ks + 1 < ks1) stage(ks + 1, buf ^ 1);
    const char* base = smem + buf * kStage;
    bf16x8_t bf[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) bf[c] = trp_frag(base + kX, c * 16, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rt = 2 * wave + i;               // 16-row r tile: sub-image rt / 4, columns (rt % 4) * 16
      const bf16x8_t af = trp_frag(base + (rt >> 2) * 4096, (rt & 3) * 16, lane);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[i][c] = mfma(af, bf[c], acc[i][c]);
    }
  }
  // C[r][co]: lane holds r = 16 rt + 4g + e, co = 16 c + li
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rt = 2 * wave + i;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 16 * rt + 4 * g + e;
      const int kh = r >> 5, kw = (r >> 2) & 7, ci = r & 3;
      if (kh >= KH || kw >= KW || ci >= CI) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        atomicAdd(dw + (((long long)kh * KW + kw) * CI + ci) * 64 + 16 * c + li, acc[i][c][e]);
    }
  }
}

void magic(unsigned d, unsigned& m, int& l) {
  l = 0;
  while ((1ull << l) < d) ++l;
  m = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
}

}  // namespace

// dw (fp32 HWIO [KH][KW][CI][64], accumulated) += weight gradient of the stem conv whose forward read x4
// (mdtf_stem_pack4 layout [N][H4][W4][4]) with output gradient dy [N][OH][OW][64].  KH <= 8, KW <= 8, CI <= 4.
MDTF_EXPORT int mdtf_stem_wgrad(const void* x4, const void* dy, float* dw, int N, int H4, int W4, int OH, int OW,
                                int SH, int SW, int KH, int KW, int CI, int blocks, hipStream_t st) {
  if (KH > 8 || KW > 8 || CI > 4 || CI < 1) return MDTF_EINVAL;
  // rows / taps past the image (kh >= KH, kw >= KW) only feed discarded rows of C, and every read is
  // range-checked by the buffer descriptor: no geometry constraint beyond the real filter's
  const long long M = (long long)N * OH * OW;
  if (M * 64 * 2 >= 0x80000000LL || (long long)N * H4 * W4 * 8 >= 0x80000000LL) return MDTF_EUNSUPPORTED;
  const long long ks_total = (M + 31) / 32;
  if (blocks <= 0) blocks = 512;
  const int per = (int)ceil_div(ks_total, (long long)blocks);
  const int nblk = (int)ceil_div(ks_total, (long long)per);
  unsigned mo, mh;
  int so, sh;
  magic((unsigned)OW, mo, so);
  magic((unsigned)OH, mh, sh);
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(nblk), dim3(512), 2 * kStage, st, (const bf16_t*)x4,
                     (const bf16_t*)dy, dw, N, H4, W4, OH, OW, SH, SW, KH, KW, CI, mo, so, mh, sh, per);
  MDTF_LAUNCH_CHECK();
  return 0;
}
