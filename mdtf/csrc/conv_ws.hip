// Weight-stationary streamed convolution / GEMM (gfx950, bf16 MFMA): the kernel for the
// short-reduction, bandwidth-bound passes of ResNet (1x1 convolutions with K <= 256, the
// 64/128-channel 3x3 convolutions of the first two stages) in forward and stride-1 dgrad.
//
// Why a second conv design (conv_igemm.hip stays for the long-K / strided-dgrad shapes):
// on those passes the LDS-ring kernels spend a tile's life in first-stage fill latency and
// an LDS-staged copy-out with ~1.7 blocks per CU (profiles/conv_small_k_investigation.md),
// so HBM sits at a third of its rate.  Here
//   * the block's filter slice (<= 64 KiB per 64 output channels) is loaded ONCE into LDS in
//     MFMA fragment order (lane l reads bytes 16l..16l+15 of a 1 KiB fragment: no bank
//     conflicts, no swizzle) and the block stays resident over many pixel tiles (persistent);
//   * the activation operand never touches LDS: each lane loads its MFMA B fragment (8
//     consecutive channels of one pixel/tap = 16 B) straight to VGPRs with bounds-checked
//     buffer loads (out-of-image taps and pixels past M read as zero), double-buffered across
//     k-steps AND across tile boundaries, so the next tile's loads overlap this tile's MFMAs and
//     stores; waves run free of barriers;
//   * the MFMA is oriented C[channel][pixel] and the filter rows are permuted so that a lane's
//     16 accumulators of a pixel are two runs of 8 consecutive output channels: the epilogue
//     stores 2 x 16 B per pixel straight from registers (each store instruction writes 64
//     contiguous bytes of 16 output rows), no LDS staging of C;
//   * BatchNorm statistics (fwd: sum y, sum y^2; dgrad: sum g*mask, sum g*mask*x of the BN this
//     gradient completes) accumulate per lane across all of a wave's tiles and are reduced once
//     per wave (16-lane xor shuffles + one atomic per channel), instead of once per tile.
//
// GEMM view: out[p][n] = sum_k src_gather(p, k) * A[n][k],  k = (tap, c), c fastest.
//   wmode 0 (fwd):   A = Wt[n][k], the filter pre-transposed to [co][(kh,kw,ci)].
//   wmode 1 (dgrad): A[n = ci][k = (tap', co)] = W[KH*KW-1-tap'][ci][co] (HWIO, both filter axes
//                    flipped); with src = DY, pads (KH-1)*DH-PH, stride 1 this is the data gradient.
// Replaces the cuDNN conv2d the reference reaches through tf.nn.conv2d (distribute_tools.py:76,88)
// and its autodiff backward (distribute_tower.py:27); SURVEY §2.5 K1.
#include "conv_ws_kernel.inc"

using namespace mdtf;

namespace mdtf {
namespace ws {
// one epilogue mode per translation unit (conv_ws_e<N>.hip)
extern template int dispatch_ws<0>(WsArgs&, int, int, int, int, int, hipStream_t);
extern template int dispatch_ws<1>(WsArgs&, int, int, int, int, int, hipStream_t);
extern template int dispatch_ws<2>(WsArgs&, int, int, int, int, int, hipStream_t);
extern template int dispatch_ws<3>(WsArgs&, int, int, int, int, int, hipStream_t);
extern template int dispatch_ws<4>(WsArgs&, int, int, int, int, int, hipStream_t);
extern template int dispatch_ws<5>(WsArgs&, int, int, int, int, int, hipStream_t);
template int dispatch_ws_dual<0>(WsArgs&, int, int, int, hipStream_t);
template int dispatch_ws_dual<3>(WsArgs&, int, int, int, hipStream_t);
}  // namespace ws
}  // namespace mdtf

using namespace mdtf::ws;

namespace {
int ws_debug = 0;

// magic multiplier for q = n / d, n < 2^31: l = ceil(log2 d), m = 2^32 (2^l - d) / d + 1,
// q = (umulhi(n, m) + n) >> l
void magic_div(unsigned d, unsigned& m, int& l) {
  l = 0;
  while ((1ull << l) < d) ++l;
  m = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
}

}  // namespace

MDTF_EXPORT void mdtf_conv_ws_debug(int mode) { ws_debug = mode; }

namespace {
// MDTF_WS_EPF=1: the epilogue's global reads are issued before the tile's MFMAs (2-subtile tiles); measured
// neutral in the ResNet-50 step (profiles/ab_r5.md), so off by default
int ws_epf() {
  static const int on = [] {
    const char* e = getenv("MDTF_WS_EPF");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return on;
}
}  // namespace

// out = conv(src, filter) on the weight-stationary kernel (see the header comment).
// wmode 0: wgt = Wt[Ncol][K] (K = KH*KW*C); wmode 1: wgt = W HWIO [KH][KW][Ncol][C] used flipped
// (the stride-1 data gradient; pass the DX pads (KH-1)*DH-PH, (KW-1)*DW-PW).
// tile = tp (16-pixel subtiles per wave) + 10 * nw (waves per block) + 100 * cg (64-channel groups
// per block) + 1000 * d (load-ring depth in k-steps), e.g. 4184 = 4 pixel subtiles, 8 waves, 1 group,
// 4 k-steps of loads in flight.  grid_cap: persistent blocks (0: 256 x
// blocks per CU).  ssum/ssq: forward BN statistics ([sslots][Ncol] partial rows, or null);
// bx/bmask/bsum/bsq: BN-backward statistics of the stored gradient (dgrad); accumulate: out += conv.
namespace {
int conv_ws_impl(const void* src, const void* wgt, void* out, int N, int H, int W, int C, int cs, int OH, int OW,
                 int Ncol, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW, int wmode, int tile,
                 int grid_cap, float* ssum, float* ssq, int sslots, const void* bx, const void* bmask, float* bsum,
                 float* bsq, int bslots, int accumulate, const void* acc_src, const void* acc_mask,
                 hipStream_t st, const float* bn_ss = nullptr, void* bn_y = nullptr, void* bn_mask = nullptr) {
  WsArgs a{};
  a.cs = cs;
  a.src = (const bf16_t*)src;
  a.wgt = (const bf16_t*)wgt;
  a.out = (bf16_t*)out;
  a.N = N; a.H = H; a.W = W; a.C = C;
  a.OH = OH; a.OW = OW; a.Ncol = Ncol;
  a.KH = KH; a.KW = KW; a.SH = SH; a.SW = SW; a.PH = PH; a.PW = PW; a.DH = DH; a.DW = DW;
  a.wmode = wmode;
  a.Cw = C;
  a.K = KH * KW * C;
  a.M = (long long)N * OH * OW;
  a.ssum = ssum; a.ssq = ssq; a.sslots = sslots > 0 ? sslots : 1;
  a.bx = (const bf16_t*)bx; a.bmask = (const uint8_t*)bmask; a.bsum = bsum; a.bsq = bsq;
  a.bslots = bslots > 0 ? bslots : 1;
  a.accumulate = accumulate;
  if ((acc_src || acc_mask) && !accumulate) return MDTF_EINVAL;
  a.acc_src = (const bf16_t*)acc_src;
  a.acc_mask = (const uint8_t*)acc_mask;
  a.direct = (KH == 1 && KW == 1 && SH == 1 && SW == 1 && PH == 0 && PW == 0 && OH == H && OW == W && cs == C) ? 1 : 0;
  magic_div((unsigned)OW, a.mow, a.sow);
  magic_div((unsigned)OH, a.mohh, a.sohh);
  const int tp = tile % 10, nw = (tile / 10) % 10, cg = (tile / 100) % 10, d = tile / 1000;
  if (C % 32 || cg < 1 || Ncol % (64 * cg) || KH * KW > 32 || a.M <= 0) return MDTF_EINVAL;
  if (wmode == 1 && (SH != 1 || SW != 1)) return MDTF_EINVAL;
  if ((long long)N * H * W * cs * 2 >= 0x80000000LL) return MDTF_EUNSUPPORTED;  // 32-bit buffer offsets
  if (a.M + 16LL * 8 * 64 >= 0x7fffffffLL) return MDTF_EUNSUPPORTED;           // 32-bit pixel indices
  if (nw % cg) return MDTF_EINVAL;
  a.dbg = ws_debug;
  a.epf = ws_epf();
  const bool stats = ssum != nullptr, bstat = bsum != nullptr;
  if (stats && bstat) return MDTF_EINVAL;
  if (bn_ss) {                           // BN + ReLU applied to the operand (epilogue mode 5)
    if (!stats || accumulate || !a.direct || wmode != 0 || !bn_y || !bn_mask || a.K > 128) return MDTF_EINVAL;
    a.bn_ss = bn_ss;
    a.bn_y = (bf16_t*)bn_y;
    a.bn_mask = (uint8_t*)bn_mask;
    return dispatch_ws<5>(a, tp, nw, cg, d, grid_cap, st);
  }
  if (stats) return accumulate ? MDTF_EINVAL : dispatch_ws<1>(a, tp, nw, cg, d, grid_cap, st);
  if (bstat) return accumulate ? dispatch_ws<4>(a, tp, nw, cg, d, grid_cap, st)
                               : dispatch_ws<3>(a, tp, nw, cg, d, grid_cap, st);
  return accumulate ? dispatch_ws<2>(a, tp, nw, cg, d, grid_cap, st) : dispatch_ws<0>(a, tp, nw, cg, d, grid_cap, st);
}
}  // namespace

MDTF_EXPORT int mdtf_conv_ws(const void* src, const void* wgt, void* out, int N, int H, int W, int C, int OH, int OW,
                             int Ncol, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW, int wmode,
                             int tile, int grid_cap, float* ssum, float* ssq, int sslots, const void* bx,
                             const void* bmask, float* bsum, float* bsq, int bslots, int accumulate,
                             const void* acc_src, const void* acc_mask, hipStream_t st) {
  return conv_ws_impl(src, wgt, out, N, H, W, C, C, OH, OW, Ncol, KH, KW, SH, SW, PH, PW, DH, DW, wmode, tile,
                      grid_cap, ssum, ssq, sslots, bx, bmask, bsum, bsq, bslots, accumulate, acc_src, acc_mask, st);
}

// 1x1 / stride-1 forward (with forward BN statistics) whose operand is a = relu(x * scale + shift), the output of a
// training BatchNorm + ReLU applied on the fly: ss = scale[C] then shift[C] (the BN's finalize), a and its ReLU
// mask (1 bit per element, as mdtf_bn_fwd_stats writes them) are written once for the backward.  C <= 128.
MDTF_EXPORT int mdtf_conv_ws_bna(const void* x, const void* wgt, void* out, int N, int H, int W, int C, int Ncol,
                                 int tile, int grid_cap, float* ssum, float* ssq, int sslots, const float* ss,
                                 void* a_out, void* mask, hipStream_t st) {
  return conv_ws_impl(x, wgt, out, N, H, W, C, C, H, W, Ncol, 1, 1, 1, 1, 0, 0, 1, 1, 0, tile, grid_cap, ssum, ssq,
                      sslots, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, st, ss, a_out, mask);
}

// Fused fan-out data gradient of a block input x that feeds a 1x1 / stride-1 convolution (gradient dy1
// [N][H][W][C1], HWIO filter w1 [1][1][Ncol][C1]) and a 1x1 / stride-S2 projection (dy2 [N][H2][W2][C2], w2
// [1][1][Ncol][C2]): out = dgrad1 + dgrad2 in ONE pass over out, as a single GEMM with K = C1 + C2 whose second
// k-range runs only over the output pixels the projection sampled (the kernel's pixel order puts them first).
// C1, C2 multiples of 128 (the 4-deep load ring), stride 2.  Replaces the projection's
// strided dgrad (GEMM + zero classes, writing out) followed by the 1x1 dgrad accumulating into it.
// bsum non-null: BN-backward statistics of out against bx / bmask (as mdtf_conv_ws).
MDTF_EXPORT int mdtf_conv_ws_dual(const void* dy1, const void* w1, const void* dy2, const void* w2, void* out, int N,
                                  int H, int W, int Ncol, int C1, int H2, int W2, int C2, int S2, int tile,
                                  const void* bx, const void* bmask, float* bsum, float* bsq, int bslots,
                                  hipStream_t st) {
  if (C1 % 128 || C2 % 128 || Ncol % 64 || S2 != 2 || H2 != (H + 1) / 2 || W2 != (W + 1) / 2) return MDTF_EINVAL;
  if (64LL * (C1 + C2) * 2 > 160 * 1024) return MDTF_EUNSUPPORTED;
  if ((long long)N * H * W * C1 * 2 >= 0x80000000LL || (long long)N * H2 * W2 * C2 * 2 >= 0x80000000LL)
    return MDTF_EUNSUPPORTED;
  WsArgs a{};
  a.src = (const bf16_t*)dy1;
  a.wgt = (const bf16_t*)w1;
  a.out = (bf16_t*)out;
  a.N = N; a.H = H; a.W = W; a.C = C1; a.cs = C1;
  a.OH = H; a.OW = W; a.Ncol = Ncol;
  a.KH = a.KW = a.SH = a.SW = a.DH = a.DW = 1;
  a.PH = a.PW = 0;
  a.wmode = 1;
  a.Cw = C1;
  a.K = C1 + C2;
  a.M = (long long)N * H * W;
  if (a.M + 16LL * 8 * 64 >= 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  a.sslots = 1;
  a.bx = (const bf16_t*)bx; a.bmask = (const uint8_t*)bmask; a.bsum = bsum; a.bsq = bsq;
  a.bslots = bslots > 0 ? bslots : 1;
  a.direct = 1;
  a.src2 = (const bf16_t*)dy2;
  a.wgt2 = (const bf16_t*)w2;
  a.K1 = C1; a.C2 = C2; a.H2 = H2; a.W2 = W2; a.S2 = S2;
  a.Mee = N * H2 * W2;
  a.Cimg = H * W - H2 * W2;
  a.G = 2 * W - W2;
  a.wodd = W - W2;
  magic_div((unsigned)W2, a.mw2, a.sw2);
  magic_div((unsigned)H2, a.mh2, a.sh2);
  magic_div((unsigned)a.Cimg, a.mci, a.sci);
  magic_div((unsigned)a.G, a.mpr, a.spr);
  magic_div((unsigned)W, a.mow, a.sow);
  magic_div((unsigned)H, a.mohh, a.sohh);
  a.dbg = ws_debug;
  a.epf = ws_epf();
  const int tp = tile % 10, nw = (tile / 10) % 10, cg = (tile / 100) % 10;
  if (bsum) {
    if (!bx) return MDTF_EINVAL;
    return dispatch_ws_dual<3>(a, tp, nw, cg, st);
  }
  return dispatch_ws_dual<0>(a, tp, nw, cg, st);
}

// ---------------------------------------------------------------------------------------------
// Stem convolution (Cin <= 4, KW <= 8: ResNet's 7x7/2 on RGB).  The input is repacked once into a
// zero-haloed 4-channel image x4[N][H+pt+pb][W+pl+pr][4] (8 B per pixel), so the KW taps x 4
// channels of one filter row are 32 contiguous, 16-B aligned elements for every output pixel
// (stride 2 keeps 2*ow*8 B aligned).  The forward is then the weight-stationary GEMM with one
// 32-deep k-step per filter row (rows padded to a multiple of 4 with zero weights), reading its B
// fragments straight from x4: no im2col, no library call.
// ---------------------------------------------------------------------------------------------
namespace {
// One 128-thread block per x4 image row: the source row (W * C bf16) is staged through LDS with 16-byte loads
// when it is 16-byte aligned, then written out two pixels (16 bytes) per thread; the blocks past the rows repack
// the HWIO filter into wt[co][KHp][32] (tap kw, channel c at element 4 kw + c; zero past KH / KW / C), so the
// stem's operands are ready after a single launch.
constexpr int kPackThreads = 128;
constexpr int kStemRowMax = 16384;            // W * C bf16 staged per row (32 KB of LDS)

__device__ __forceinline__ uint2 stem_pixel(const bf16_t* row, int iw, int W, int C) {
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  if (iw >= 0 && iw < W)
    for (int c = 0; c < C; ++c) v[c] = row[iw * C + c];
  return make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
}

template <bool VEC>
__global__ void __launch_bounds__(kPackThreads) stem_pack4(const bf16_t* __restrict__ x, uint2* __restrict__ x4,
                                                           int N, int H, int W, int C, int pt, int pl, int H4,
                                                           int W4, const bf16_t* __restrict__ w,
                                                           bf16_t* __restrict__ wt, int KH, int KW, int CO, int KHP) {
  extern __shared__ __align__(16) bf16_t row_s[];
  const int rows = N * H4;
  const int b = blockIdx.x, t = threadIdx.x;
  if (b >= rows) {
    const int i = (b - rows) * kPackThreads + t;
    if (i >= CO * KHP * 32) return;
    const int co = i / (KHP * 32), r = i % (KHP * 32);
    const int kh = r >> 5, kw = (r & 31) >> 2, c = r & 3;
    wt[i] = (kh < KH && kw < KW && c < C) ? w[((kh * KW + kw) * C + c) * CO + co] : bf16_t(0);
    return;
  }
  const int n = b / H4, ih = b - n * H4 - pt;
  const bool live = ih >= 0 && ih < H;                 // block-uniform
  if (live) {
    const bf16_t* src = x + ((long long)n * H + ih) * W * C;
    if (VEC) {
      const uint4* s4 = reinterpret_cast<const uint4*>(src);
      uint4* d4 = reinterpret_cast<uint4*>(row_s);
      for (int i = t; i < W * C / 8; i += kPackThreads) d4[i] = s4[i];
    } else {
      for (int i = t; i < W * C; i += kPackThreads) row_s[i] = src[i];
    }
    __syncthreads();
  }
  uint2* dst = x4 + (long long)b * W4;
  if ((W4 & 1) == 0) {
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (int p = t; p < W4 / 2; p += kPackThreads) {
      uint2 a = make_uint2(0u, 0u), c = a;
      if (live) {
        a = stem_pixel(row_s, 2 * p - pl, W, C);
        c = stem_pixel(row_s, 2 * p + 1 - pl, W, C);
      }
      d4[p] = make_uint4(a.x, a.y, c.x, c.y);
    }
  } else {
    for (int p = t; p < W4; p += kPackThreads) dst[p] = live ? stem_pixel(row_s, p - pl, W, C) : make_uint2(0u, 0u);
  }
}
}  // namespace

// x -> zero-haloed x4 [N][H4][W4][4]; with w non-null also the filter rows wt (see stem_pack4).
MDTF_EXPORT int mdtf_stem_pack4(const void* x, void* x4, int N, int H, int W, int C, int pt, int pl, int H4, int W4,
                                const void* w, void* wt, int KH, int KW, int CO, int KHP, hipStream_t st) {
  if (C < 1 || C > 4 || KH > KHP || KW > 8 || W * C > kStemRowMax) return MDTF_EINVAL;
  const long long rows = (long long)N * H4;
  const long long wblocks = w ? ceil_div((long long)CO * KHP * 32, (long long)kPackThreads) : 0;
  if (rows + wblocks >= (1LL << 31)) return MDTF_EINVAL;
  const bool vec = (W * C) % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const size_t lds = (size_t)W * C * sizeof(bf16_t);
  auto k = vec ? stem_pack4<true> : stem_pack4<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)(rows + wblocks)), dim3(kPackThreads), lds, st, (const bf16_t*)x,
                     (uint2*)x4, N, H, W, C, pt, pl, H4, W4, (const bf16_t*)w, (bf16_t*)wt, KH, KW, CO, KHP);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// y = conv(x, W) for the stem: x4 from mdtf_stem_pack4 ([N][H4][W4][4]), wt = [Ncol][KHp][32] filter rows
// (tap kw, channel c at element 4 kw + c; zero rows/taps past KH / KW), KHp % 4 == 0.
MDTF_EXPORT int mdtf_conv_ws_stem(const void* x4, const void* wt, void* out, int N, int H4, int W4, int OH, int OW,
                                  int Ncol, int KHp, int SH, int SW, int tile, float* ssum, float* ssq, int sslots,
                                  hipStream_t st) {
  if ((OH - 1) * SH + KHp > H4 + 3 || (OW - 1) * SW + 8 > W4) return MDTF_EINVAL;   // rows / taps stay in x4
  return conv_ws_impl(x4, wt, out, N, H4, W4, 32, 4, OH, OW, Ncol, KHp, 1, SH, SW, 0, 0, 1, 1, 0, tile, 0, ssum,
                      ssq, sslots, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, st);
}

// ---------------------------------------------------------------------------------------------
// Row-staged stem convolution.  The streamed kernel above reads each B fragment from x4 in global
// memory with only a 4-k-step ring in flight at two waves per SIMD: the stem's 8 KB-per-output-row
// reads are latency bound there (259 us for ResNet's 7x7/2, against ~45 us of MFMA work).  Here a
// 4-wave block owns kStemRows consecutive output rows of one image (one row per wave, all 64
// channels of its channel group): it stages the KH filter rows (fragment order, 1 KiB per fragment)
// and the (kStemRows-1)*SH + KH input rows it reads into LDS with every load issued before the
// first wait, then each wave runs KH k-steps of 4 x TP MFMAs with both operands from LDS and stores
// its row.  Three blocks fit a CU (52 KB of LDS at W4 = 230), so one block's staging overlaps the
// others' MFMAs.  Forward BN statistics are reduced per wave and added to [sslots][Ncol] slots.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int kStemRows = 4;
constexpr int kStemStage = 8;          // 16-B staging loads in flight per thread per batch

// Σ over the 16 lanes of a DPP row (lane & 15), valid in the row's lane 15: four v_add_f32 with row_shr
// operands -- no LDS crossbar traffic (the __shfl_xor version cost ~45 us in this kernel's 28k waves).
__device__ __forceinline__ float row_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// AL16: SW even, so every B fragment (16 B at pixel ow*SW + 2g) is 16-B aligned: one ds_read_b128
// (two 8-B reads per lane at a 16-B lane stride conflict 2-way)
// PF: the next group's input rows are loaded into registers before this group's MFMAs and written to LDS after
// them (2 blocks per CU with the registers that takes, instead of 3 blocks staging in turn)
template <int TP, bool AL16, bool PF>
__global__ void __launch_bounds__(256, PF ? 2 : 3) stem_conv_rows(const bf16_t* __restrict__ x4, const bf16_t* __restrict__ wt,
                                                         bf16_t* __restrict__ out, int H4, int W4, int OH, int OW,
                                                         int Ncol, int KH, int KHP, int SH, int SW, int rblocks,
                                                         int ngroups, float* __restrict__ ssum,
                                                         float* __restrict__ ssq, int sslots) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int cgroups = Ncol / 64;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cblk = bid % cgroups;                          // fixed per block: gridDim.x % cgroups == 0
  const int nrows = (kStemRows - 1) * SH + KH;
  const int pitch = W4 * 8;                                // bytes per staged row (W4 even: 16-B aligned)
  const int chunks_w = KH * 4 * 64, chunks_r = nrows * (W4 / 2);
  char* rows_s = lds + chunks_w * 16;
  float* stat_s = reinterpret_cast<float*>(rows_s + chunks_r * 16);   // [2][64] block partials (LDS atomics)
  const int n0 = cblk * 64;
  if (threadIdx.x < 128) stat_s[threadIdx.x] = 0.f;

  // ---- filter fragments once per block (f = ks*4 + i: lane l holds channel chan_of(i, l&15), k = 32 ks + 8 (l>>4))
  for (int q = threadIdx.x; q < chunks_w; q += 256) {
    const int f = q >> 6, l = q & 63;
    const int ch = n0 + chan_of(f & 3, l & 15);
    reinterpret_cast<uint4*>(lds)[q] =
        *reinterpret_cast<const uint4*>(wt + (long long)ch * (KHP * 32) + (f >> 2) * 32 + 8 * (l >> 4));
  }

  // row layout as conv_ws_kernel's epilogue: pixel rp = (lane & 31) >> 1, chunk rc = (lane & 1) | (lane >> 5) << 1,
  // so the ds_bpermute sources of each 32-lane half are distinct mod 32 (conflict-free)
  const int rp = (lane & 31) >> 1, rc = (lane & 1) | ((lane >> 5) << 1);
  const int xsrc = (16 * rc + rp) * 4;
  auto xpose = [&](const uint4& v) {
    return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.x),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.y),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.z),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.w));
  };

  auto load_rows = [&](int grp, uint4 (&v)[kStemStage], int base) {
    const int rb = grp / cgroups;
    const int n = rb / rblocks, oh0 = (rb - n * rblocks) * kStemRows;
    const uint4* src4 = reinterpret_cast<const uint4*>(x4) + ((long long)n * H4 + (long long)oh0 * SH) * (W4 / 2);
    const int avail = (H4 - oh0 * SH) * (W4 / 2);          // chunks of the staged rows that exist in x4
#pragma unroll
    for (int u = 0; u < kStemStage; ++u) {
      const int q = base + u * 256 + threadIdx.x;
      v[u] = grp < ngroups && q < chunks_r && q < avail ? src4[q] : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store_rows = [&](const uint4 (&v)[kStemStage], int base) {
#pragma unroll
    for (int u = 0; u < kStemStage; ++u) {
      const int q = base + u * 256 + threadIdx.x;
      if (q < chunks_r) reinterpret_cast<uint4*>(rows_s)[q] = v[u];
    }
  };
  auto run_group = [&](int grp) {
    const int rb = grp / cgroups;
    const int n = rb / rblocks, oh0 = (rb - n * rblocks) * kStemRows;
    const int oh = oh0 + wave;
    if (oh >= OH) return;                                  // wave-uniform
    float4v acc[4][TP];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < KH; ++ks) {
      bf16x8_t af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(lds + (ks * 4 + i) * 1024 + lane * 16));
      const char* row = rows_s + (wave * SH + ks) * pitch;
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int ow = 16 * j + li;
        uint4 bv = make_uint4(0u, 0u, 0u, 0u);
        if (ow < OW) {
          if (AL16) {
            bv = *reinterpret_cast<const uint4*>(row + (ow * SW + 2 * g) * 8);
          } else {
            const uint2* p = reinterpret_cast<const uint2*>(row + (ow * SW + 2 * g) * 8);
            const uint2 lo = p[0], hi = p[1];
            bv = make_uint4(lo.x, lo.y, hi.x, hi.y);
          }
        }
        const bf16x8_t b = __builtin_bit_cast(bf16x8_t, bv);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = mfma(af[i], b, acc[i][j]);
      }
    }

    // ---- epilogue: fragment layout (channel chunk g, pixel li) -> row layout (pixel rp, chunk rc) and
    // 2 x 16-B stores per pixel (a full 128-B output row); statistics from the fp32 accumulators (pixels
    // past OW hold zeros), row-reduced and added to the block's LDS partials
    float s0[16], s1[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) s0[e] = s1[e] = 0.f;
    const long long prow = ((long long)n * OH + oh) * OW;
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      float v0[8], v1[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v0[r] = acc[0][j][r];
        v0[4 + r] = acc[1][j][r];
        v1[r] = acc[2][j][r];
        v1[4 + r] = acc[3][j][r];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s0[e] += v0[e];
        s1[e] += v0[e] * v0[e];
        s0[8 + e] += v1[e];
        s1[8 + e] += v1[e] * v1[e];
      }
      const uint4 w0 = xpose(pack8(v0)), w1 = xpose(pack8(v1));
      const int ow = 16 * j + rp;
      if (ow < OW) {
        bf16_t* o = out + (prow + ow) * Ncol + n0 + 8 * rc;
        *reinterpret_cast<uint4*>(o) = w0;
        *reinterpret_cast<uint4*>(o + 32) = w1;
      }
    }
    if (ssum) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        s0[e] = row_sum16(s0[e]);
        s1[e] = row_sum16(s1[e]);
      }
      if (li == 15) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int c = e < 8 ? 8 * g + e : 32 + 8 * g + (e - 8);
          atomicAdd(stat_s + c, s0[e]);                    // LDS atomics: the block's partials
          atomicAdd(stat_s + 64 + c, s1[e]);
        }
      }
    }
    };

  if constexpr (PF) {
    // chunks_r <= kStemStage * 256 (host-checked): one register batch holds a group's rows
    uint4 pv[kStemStage];
    load_rows(bid, pv, 0);
    store_rows(pv, 0);
    for (int grp = bid; grp < ngroups; grp += gridDim.x) {
      __syncthreads();                                     // this group's rows (and the filter) are in LDS
      const int nxt = grp + gridDim.x;
      load_rows(nxt, pv, 0);                               // in flight during this group's MFMAs
      run_group(grp);
      __syncthreads();                                     // every wave is done with this group's rows
      if (nxt < ngroups) store_rows(pv, 0);
    }
  } else {
    for (int grp = bid; grp < ngroups; grp += gridDim.x) {
      __syncthreads();                                     // the previous group's rows are consumed
      // ---- input rows oh0*SH .. + nrows-1 (zero past H4): a batch of loads before its LDS writes
      for (int base = 0; base < chunks_r; base += kStemStage * 256) {
        uint4 v[kStemStage];
        load_rows(grp, v, base);
        store_rows(v, base);
      }
      __syncthreads();
      run_group(grp);
    }
  }
  if (ssum) {
    __syncthreads();
    if (threadIdx.x < 128) {
      const int c = threadIdx.x & 63;
      float* dst = (threadIdx.x < 64 ? ssum : ssq) + (long long)(blockIdx.x % sslots) * Ncol + n0 + c;
      atomicAdd(dst, stat_s[threadIdx.x]);
    }
  }
}

bool stem_rows_prefetch() {   // MDTF_STEM_PREFETCH=0: stage each group's rows in turn (3 blocks per CU)
  static const bool on = [] {
    const char* e = getenv("MDTF_STEM_PREFETCH");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int TP>
void launch_stem_rows(const void* x4, const void* wt, void* out, int N, int H4, int W4, int OH, int OW, int Ncol,
                      int KH, int KHP, int SH, int SW, float* ssum, float* ssq, int sslots, size_t lds, hipStream_t st) {
  const int rblocks = (OH + kStemRows - 1) / kStemRows;
  const int cgroups = Ncol / 64;
  const long long ngroups = (long long)N * rblocks * cgroups;
  // persistent: as many blocks as fit (LDS-bound, <= 3 per CU; 2 with the register prefetch), a multiple of the
  // channel groups
  const int nrows = (kStemRows - 1) * SH + KH;
  const bool pf = stem_rows_prefetch() && nrows * (W4 / 2) <= kStemStage * 256;
  long long per_cu = (160 * 1024) / (long long)lds;
  if (per_cu > (pf ? 2 : 3)) per_cu = pf ? 2 : 3;
  long long nblk = 256 * per_cu / cgroups * cgroups;
  if (nblk < cgroups) nblk = cgroups;
  if (nblk > ngroups) nblk = ngroups;
  auto k = (SW & 1) ? (pf ? stem_conv_rows<TP, false, true> : stem_conv_rows<TP, false, false>)
                     : (pf ? stem_conv_rows<TP, true, true> : stem_conv_rows<TP, true, false>);
  hipLaunchKernelGGL(k, dim3((unsigned)nblk), dim3(256), lds, st, (const bf16_t*)x4, (const bf16_t*)wt,
                     (bf16_t*)out, H4, W4, OH, OW, Ncol, KH, KHP, SH, SW, rblocks, (int)ngroups, ssum, ssq,
                     sslots > 0 ? sslots : 1);
}
}  // namespace

// Row-staged stem forward (see above): same operands as mdtf_conv_ws_stem plus KH, the filter rows actually
// used (rows KH..KHp-1 of wt are zero and skipped).  Needs W4 even, OW <= 128, Ncol % 64 == 0.
MDTF_EXPORT int mdtf_stem_conv_rows(const void* x4, const void* wt, void* out, int N, int H4, int W4, int OH, int OW,
                                    int Ncol, int KH, int KHp, int SH, int SW, float* ssum, float* ssq, int sslots,
                                    hipStream_t st) {
  if ((W4 & 1) || OW < 1 || OW > 128 || Ncol % 64 || KH < 1 || KH > KHp || (OW - 1) * SW + 8 > W4 ||
      (OH - 1) * SH + KH > H4)
    return MDTF_EINVAL;
  const size_t lds = (size_t)KH * 4 * 1024 + (size_t)((kStemRows - 1) * SH + KH) * W4 * 8 + 128 * sizeof(float);
  if (lds > 160 * 1024) return MDTF_EUNSUPPORTED;
  if ((long long)N * ((OH + kStemRows - 1) / kStemRows) * (Ncol / 64) >= (1LL << 31)) return MDTF_EUNSUPPORTED;
  switch ((OW + 15) / 16) {
    case 1: launch_stem_rows<1>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    case 2: launch_stem_rows<2>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    case 3: launch_stem_rows<3>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    case 4: launch_stem_rows<4>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    case 5: launch_stem_rows<5>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    case 6: launch_stem_rows<6>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    case 7: launch_stem_rows<7>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
    default: launch_stem_rows<8>(x4, wt, out, N, H4, W4, OH, OW, Ncol, KH, KHp, SH, SW, ssum, ssq, sslots, lds, st); break;
  }
  MDTF_LAUNCH_CHECK();
  return 0;
}
