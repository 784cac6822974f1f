// Implicit-GEMM convolution on bf16 MFMA (gfx950), NHWC activations, HWIO filters.
//
// Replaces the cuDNN conv2d the reference reaches through tf.nn.conv2d
// (distribute_tools.py:76,88,104,119) and its autodiff backward
// (distribute_tower.py:27), SURVEY §2.5 K1/K4.  Three passes share one MFMA
// core (v_mfma_f32_16x16x32_bf16, 4 waves per 256-thread block, register-staged
// double-buffered LDS, one barrier per 32-deep K step):
//
//   fwd   : Y[m=(n,oh,ow)][co]   = Σ_{k=(kh,kw,ci)} X[n,ih,iw,ci] · W[k][co]
//   dgrad : DX[m=(n,h,w)][ci]    = Σ_{k=(kh,kw,co)} DY[n,oh,ow,co] · W[kh][kw][ci][co]
//           (oh = (h+ph-kh·dh)/sh, only where divisible — strided convs included)
//   wgrad : DW[r=(kh,kw,ci)][co] = Σ_{m=(n,oh,ow)} X[n,ih,iw,ci] · DY[m][co]
//           (split over the pixel dimension, fp32 atomics into DW)
//
// Operand staging: a tile whose reduction index is contiguous in memory
// ("K-contiguous": the im2col gather of X/DY, and W^T for dgrad) is stored in
// LDS as [rows][32 + 8 pad] and read with ds_read_b128; a tile whose reduction
// index is the memory row ("N-contiguous": W for fwd, X and DY for wgrad) is
// stored as [32][cols + 16 pad] and read transposed with two
// ds_read_b64_tr_b16 per fragment (CDNA4 hardware transpose).  The pad makes
// both reads conflict-free (row stride ≡ 8 dwords mod 64 for the transposed
// reads; see frag_ncontig for the lane/row pairing).  Blocks are XCD-remapped
// so the N-tiles of one M-tile share an L2.  Forward can emit per-channel
// Σy / Σy² partials for the following BatchNorm (bn.hip consumes them).
#include "mdtf_common.h"

#ifndef FD_PF16
#define FD_PF16 1
#endif

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int BK = 32;
constexpr int PADK = 8;    // K-contiguous rows: 32 + 8 elements = 80 B
constexpr int PADN = 16;   // N-contiguous rows: cols + 16 elements
constexpr int NT = 256;
constexpr int kStatSlots = 64;   // BN-statistics partial rows written by the fwd epilogue

struct ConvArgs {
  const bf16_t* src;   // gathered activation: X (fwd, wgrad) or DY (dgrad)
  const bf16_t* wgt;   // W (fwd, dgrad)
  const bf16_t* dy;    // DY (wgrad)
  bf16_t* out;         // Y (fwd) / DX (dgrad)
  float* dw;           // DW (wgrad, fp32, pre-zeroed)
  float* stat_sum;     // fwd: per-channel partials [gridM][Cout] (optional)
  float* stat_sq;
  int N, H, W, Cin;    // X dims
  int OH, OW, Cout;    // Y dims
  int KH, KW, SH, SW, PH, PW, DH, DW;
  long long M;         // GEMM rows
  int Ncol;            // GEMM cols
  int K;               // GEMM reduction length (fwd/dgrad)
  int mtiles, ntiles;  // tile grid
  int ksplit_steps;    // wgrad: K steps per split
  int stat_slots;      // fwd: BN-statistics partial rows (power of two: atomics spread; = mtiles: deterministic)
  int ld_dy, ld_dw;    // wgrad v2: row strides of DY and DW in elements (Cout for convolutions)
  int accumulate;      // fwd/dgrad v2: out += result (fan-out gradient accumulation) instead of out = result
  // accumulate source (default: out itself): out = result + acc_src * [acc_mask bit] -- a ReLU-masked
  // gradient another consumer left unmaterialised (1 mask bit per element, null: no mask)
  const bf16_t* acc_src;
  const uint8_t* acc_mask;
  // strided dgrad (MODE 2), one stride-parity class of DX pixels per launch: pixels
  // (h0 + SH i, w0 + SW j), i < Hc, j < Wc; their taps kh = kh0 + SH t (t < th), kw = kw0 + SW u (u < tw)
  // read DY at (q0h + i - t, q0w + j - u)
  int cls_h0, cls_w0, cls_q0h, cls_q0w, cls_kh0, cls_kw0, cls_Hc, cls_Wc, cls_th, cls_tw;
  // dgrad v2 writing the COMPLETE gradient g of a BatchNorm output (its last contribution):
  // also emit that BN's backward statistics  Σ g·relu_mask, Σ g·relu_mask·x  per channel into
  // bslots atomic partial rows (saves the BN backward's separate reduction pass over g and x)
  const bf16_t* bx;      // the BN's input x  [M][Ncol]
  const uint8_t* bmask;  // its forward ReLU bitmask (1 bit / element) or null
  float* bsum;           // [bslots][Ncol] (null: off)
  float* bsq;
  int bslots;
  // wgrad (4-wave tiles): also add the column sums of DY (a dense layer's bias gradient) into
  // dbias[Cout]; the first row-tile's blocks sum their B fragments with an all-ones MFMA (null: off)
  float* dbias;
  // wgrad v2 split-K: per-split partial tiles stored to slab[split][R][Cout] (plain stores) and summed
  // into DW by one reduction pass, instead of fp32 atomics into DW (null: atomics)
  float* slab;
  int slab_cap;          // splits the slab has room for
  int slab_nt;           // partials with nontemporal stores, summed with nontemporal loads (MDTF_SLAB_NT=0: cached)
  int* cnt;              // non-null: split-K partials summed in the kernel by each tile's last arriving workgroup
                         // (slab = [tiles][splits][BM * BN], write-through; cnt = per-tile tickets, left zeroed)
  int wg_xcd;            // wgrad v2: XCD-aware block order (the row/col tiles of one pixel split share an L2)
  // dense forward (fd v2 MODE 3): Y[M][Ncol] = act(X[M][K] W + bias), W N-contiguous [K][ld_b] read as
  // [64 k][64 col] half-images by transposed fragment reads (no transposed weight copy).  The columns are
  // nseg segments of seg_cols, each its own matrix wseg[s] (q | k | v without a concatenated copy).
  const bf16_t* wseg[4];
  int seg_cols, ld_b;
  const bf16_t* bias;    // bf16 [Ncol], added to the fp32 accumulators (null: none)
  bf16_t* pre_out;       // act != 0: the bf16 pre-activation is also stored here (null: not kept)
  int act;               // 0 none, 1 relu, 2 gelu (tanh form)
  // v2 fwd/dgrad: the row index -> pixel decomposition divides by the row grid's width and height (RW, RH);
  // n / d = (n * mg) >> sh for n < 2^31 (Granlund-Montgomery, set by launch_fd_v2): the 64-bit divisions of
  // the per-row setup were ~1,000 VALU instructions per wave before the first DMA of every tile
  unsigned mg_rw, mg_rh;
  int sh_rw, sh_rh;
  // v2 fwd / dgrad: first GEMM row of this launch (a tile-count tail split runs the last rows as a second launch
  // with smaller tiles, launch_fd_v2); rows [m_base, M)
  long long m_base;
  // wgrad v2: fin_blocks extra workgroups (the first blocks of the grid, or the last) run the backward finalize of the BatchNorm
  // whose output gradient the conv's data gradient just completed (fin_*; see fin_bwd_block)
  int fin_blocks, fin_first;
  // v2 forward / data gradient, BN = 128: the copy-out's bank-aligned lane order (copyout_rc; MDTF_FD_COREMAP=1; default
  // row-major)
  int co_remap;
  const float* fin_psum;
  const float* fin_psq;
  int fin_P, fin_C;
  long long fin_M;
  const float* fin_gamma;
  const float* fin_mean;
  const float* fin_invstd;
  float* fin_ws;
};

// BatchNorm backward finalize of one 32-channel group, run by an extra workgroup of a weight-gradient launch: the
// conv's data gradient (the previous launch) completed the BN's statistics Σ g·mask, Σ g·mask·x in fin_P partial
// rows; this sums them (fp64 across the thread groups), writes k1 | k2 | k3 | dgamma | dbeta into fin_ws[5][C]
// (dgamma / dbeta written, not accumulated: csrc/bn.hip mdtf_bn_dx_ws adds them into the slots) and re-zeroes the
// partial rows -- the math of bn.hip finalize_bwd with zero_after = 3.  The finalize then costs no launch of its
// own: it runs beside the weight gradient, which does not depend on it (ops.conv MDTF_BN_WG_FIN).
// (the fields are passed by value: a reference to the kernel's ConvArgs would take its address and turn the GEMM
// path's uniform buffer descriptors into per-lane values)
__device__ __noinline__ void fin_bwd_block(float* psum, float* psq, int P, int C, long long M, const float* gamma,
                                           const float* meanp, const float* invstdp, float* ws, int blk, char* smem) {
  const int G = blockDim.x / 32;
  const int lc = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int c = blk * 32 + lc;
  const bool own = grp == 0 && c < C;
  const float mu = own ? meanp[c] : 0.f, inv = own ? invstdp[c] : 0.f;
  const float gm = own && gamma ? gamma[c] : 1.f;
  float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int r = grp;
    for (; r + 3 * G < P; r += 4 * G) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s[u] += psum[(long long)(r + u * G) * C + c];
        q[u] += psq[(long long)(r + u * G) * C + c];
      }
    }
    for (; r < P; r += G) {
      s[0] += psum[(long long)r * C + c];
      q[0] += psq[(long long)r * C + c];
    }
    // re-zero the rows this thread read (no other thread reads them): the persistent statistics pool's next user
    // accumulates into zeros
    for (r = grp; r < P; r += G) {
      psum[(long long)r * C + c] = 0.f;
      psq[(long long)r * C + c] = 0.f;
    }
  }
  double* L0 = reinterpret_cast<double*>(smem);
  double* L1 = L0 + G * 32;
  L0[grp * 32 + lc] = (double)s[0] + (double)s[1] + (double)s[2] + (double)s[3];
  L1[grp * 32 + lc] = (double)q[0] + (double)q[1] + (double)q[2] + (double)q[3];
  __syncthreads();
  if (!own) return;
  double sdz = 0.0, sdzx = 0.0;
  for (int g = 0; g < G; ++g) {
    sdz += L0[g * 32 + lc];
    sdzx += L1[g * 32 + lc];
  }
  const float db = (float)sdz;
  const float dg = (float)((sdzx - (double)mu * sdz) * inv);
  ws[3 * C + c] = dg;
  ws[4 * C + c] = db;
  const float ak = gm * inv, invM = 1.f / (float)M;
  ws[c] = ak;
  ws[C + c] = -ak * inv * dg * invM;
  ws[2 * C + c] = ak * (-db * invM + mu * inv * dg * invM);
}

// m, sh with floor(n / d) = (n * m) >> sh for every 0 <= n < 2^31: l = ceil(log2 d), m = ceil(2^(31+l) / d)
// (m * d - 2^(31+l) < d <= 2^l; m < 2^32 for d >= 1)
inline void magic31(unsigned d, unsigned* m, int* sh) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  *m = static_cast<unsigned>(((1ull << (31 + l)) + d - 1) / d);
  *sh = 31 + l;
}

__device__ __forceinline__ unsigned fdiv31(unsigned n, unsigned m, int sh) {
  return static_cast<unsigned>((static_cast<unsigned long long>(n) * m) >> sh);
}

// zero the bf16 elements of an 8-element vector whose mask bit (element k: bit k) is clear
__device__ __forceinline__ uint4 mask_bf8(const uint4& v, uint32_t m8) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    o[k] = (w[k] & (((m8 >> (2 * k)) & 1u) ? 0x0000ffffu : 0u)) | (w[k] & (((m8 >> (2 * k + 1)) & 1u) ? 0xffff0000u : 0u));
  return make_uint4(o[0], o[1], o[2], o[3]);
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// 8 packed bf16 -> floats
__device__ __forceinline__ void unpack8(const uint4& raw, float (&f)[8]) {
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 ld16(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ void st16(bf16_t* lds, const uint4& v) { *reinterpret_cast<uint4*>(lds) = v; }

// fragment of a K-contiguous LDS tile: lane l -> row (l&15), k = 8*(l>>4) .. +7
__device__ __forceinline__ bf16x8_t frag_kcontig(const bf16_t* tile, int row0, int lane) {
  const bf16_t* p = tile + (row0 + (lane & 15)) * (BK + PADK) + 8 * (lane >> 4);
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return __builtin_bit_cast(bf16x8_t, v);
}

// fragment of an N-contiguous LDS tile [BK][ld]: lane l -> col (l&15), k = 8*(l>>4) .. +7.
// Two transposed reads; odd 16-lane groups fetch their upper k-half in the FIRST
// instruction so each 32-lane half touches rows {0-3,12-15} then {4-7,8-11}
// (conflict-free with row stride ≡ 8 dwords mod 64).
__device__ __forceinline__ bf16x8_t frag_ncontig(const bf16_t* tile, int ld, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int odd = g & 1;
  const int rfirst = 8 * g + (odd ? 4 : 0) + q;
  const int rsecond = 8 * g + (odd ? 0 : 4) + q;
  const bf16_t* a1 = tile + rfirst * ld + col0 + 4 * p;
  const bf16_t* a2 = tile + rsecond * ld + col0 + 4 * p;
  v4s r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a1);
  v4s r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a2);
  v4s lo = odd ? r2 : r1;
  v4s hi = odd ? r1 : r2;
  short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, f);
}

// dense-layer activation epilogue: 1 relu, 2 gelu (tanh form, as kernels.hip's act_f).  0.5 (1 + tanh u) is
// sigmoid(2u): one v_exp_f32 and one v_rcp_f32 per element instead of a libm tanhf in the GEMM's epilogue
__device__ __forceinline__ float dense_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) {
    const float u2 = 1.5957691216f * (v + 0.044715f * v * v * v);     // 2u
    return v * __builtin_amdgcn_rcpf(1.f + __expf(-u2));
  }
  return v;
}

// its derivative at the pre-activation x: relu [x > 0]; gelu s + 2 x s (1 - s) u'(x), s = sigmoid(2u)
// (= kernels.hip act_grad's tanh form: 0.5 (1 + t) = s, 1 - t^2 = 4 s (1 - s))
__device__ __forceinline__ float dense_act_grad(float x, int act) {
  if (act == 1) return x > 0.f ? 1.f : 0.f;
  if (act == 2) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-1.5957691216f * (x + 0.044715f * x * x * x)));
    return s + 2.f * x * s * (1.f - s) * 0.7978845608f * (1.f + 0.134145f * x * x);
  }
  return 1.f;
}

// chunk swizzle of the [64 k][64 col] half-images read by transposed fragment reads (see the v2 wgrad)
__device__ __forceinline__ int trswz(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }

// fragment (16 cols x 32 k) of a [64 k][64 col] half-image: lane l -> col (l&15), k = 8*(l>>4) .. +7
__device__ __forceinline__ bf16x8_t frag_tr(const char* img, int col0, int kbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c = col0 + 4 * p;                       // first of this lane's 4 columns
  const int k1 = kbase + 8 * g + q, k2 = k1 + 4;
  const char* a1 = img + k1 * 128 + (((c >> 3) ^ trswz(k1)) << 4) + (c & 7) * 2;
  const char* a2 = img + k2 * 128 + (((c >> 3) ^ trswz(k2)) << 4) + (c & 7) * 2;
  v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a1);
  v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a2);
  short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, f);
}

__device__ __forceinline__ float4v mfma(const bf16x8_t& a, const bf16x8_t& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// bijective XCD-aware remap of a 1-D block index (cdna_hip_programming.md §5 T1)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// ============================================================================
// forward / dgrad: rows = output pixels (K-contiguous gather), cols = channels
// MODE 0 = fwd (B = W as N-contiguous [k][co]); MODE 1 = dgrad (B = W^T K-contiguous)
// ============================================================================
template <int BM, int BN, int MODE, bool STATS>
__global__ void __launch_bounds__(NT) conv_fd_kernel(ConvArgs a) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_CHUNKS = BM * BK / 8 / NT;                 // 16-B chunks per thread
  constexpr int B_CHUNKS = BN * BK / 8 / NT;
  constexpr int LDA = BK + PADK;
  constexpr int LDB_N = BN + PADN;                           // fwd (N-contiguous)
  constexpr int A_ELEMS = BM * LDA;
  constexpr int B_ELEMS = MODE == 0 ? BK * LDB_N : BN * LDA;
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small for 256 threads");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* As[2] = {smem, smem + A_ELEMS};
  bf16_t* Bs[2] = {smem + 2 * A_ELEMS, smem + 2 * A_ELEMS + B_ELEMS};

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / a.ntiles, nt = tile % a.ntiles;
  const long long m0 = (long long)mt * BM;
  const int n0 = nt * BN;

  // ---- A (gather) per-thread setup: rows fixed across K, chunk column kc fixed
  const int kc = tid & 3;
  int a_n[A_CHUNKS], a_y[A_CHUNKS], a_x[A_CHUNKS];
  bool a_ok[A_CHUNKS];
  const int GH = MODE == 0 ? a.H : a.OH;          // gathered tensor (X or DY) dims
  const int GW = MODE == 0 ? a.W : a.OW;
  const int GC = MODE == 0 ? a.Cin : a.Cout;
  const int RH = MODE == 0 ? a.OH : a.H;          // pixel grid of the GEMM rows
  const int RW = MODE == 0 ? a.OW : a.W;
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    const int row = (tid >> 2) + i * (NT / 4);
    const long long m = m0 + row;
    a_ok[i] = m < a.M;
    const long long mm = a_ok[i] ? m : 0;
    const int ow = static_cast<int>(mm % RW);
    const long long t = mm / RW;
    const int oh = static_cast<int>(t % RH);
    a_n[i] = static_cast<int>(t / RH);
    if (MODE == 0) {
      a_y[i] = oh * a.SH - a.PH;
      a_x[i] = ow * a.SW - a.PW;
    } else {
      a_y[i] = oh + a.PH;   // dgrad: DY row = (h + ph - kh*dh) / sh where divisible
      a_x[i] = ow + a.PW;
    }
  }
  // incremental decomposition of this thread's k = kt*BK + kc*8 -> (kh, kw, c)
  int g_c = kc * 8, g_kw = 0, g_kh = 0;
  while (g_c >= GC) { g_c -= GC; if (++g_kw == a.KW) { g_kw = 0; ++g_kh; } }
  // dgrad B: k = kt*BK + kcc*8 -> (tt = kh*KW+kw, co); kcc == kc for every chunk of this thread
  int b_co = kc * 8, b_tt = 0;
  if (MODE == 1) while (b_co >= a.Cout) { b_co -= a.Cout; ++b_tt; }

  uint4 ra[A_CHUNKS], rb[B_CHUNKS];

  // loads tile kt (called with kt = 0, 1, 2, ... in order) and advances the counters
  auto load_tiles = [&](int kt) {
    const bool kok = g_kh < a.KH;
    const int c = g_c, kw = g_kw, kh = g_kh;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      int iy, ix;
      bool ok = kok && a_ok[i];
      if (MODE == 0) {
        iy = a_y[i] + kh * a.DH;
        ix = a_x[i] + kw * a.DW;
      } else {
        const int ny = a_y[i] - kh * a.DH, nx = a_x[i] - kw * a.DW;
        iy = ny / a.SH;
        ix = nx / a.SW;
        ok = ok && ny >= 0 && nx >= 0 && (ny - iy * a.SH) == 0 && (nx - ix * a.SW) == 0;
      }
      ok = ok && iy >= 0 && iy < GH && ix >= 0 && ix < GW;
      const bf16_t* p = a.src + (((long long)a_n[i] * GH + (ok ? iy : 0)) * GW + (ok ? ix : 0)) * GC + c;
      ra[i] = ld16(p, ok);
    }
    g_c += BK;
    while (g_c >= GC) { g_c -= GC; if (++g_kw == a.KW) { g_kw = 0; ++g_kh; } }
    if (MODE == 0) {
      // W [K][Cout], tile rows = k, cols = n (N-contiguous)
#pragma unroll
      for (int i = 0; i < B_CHUNKS; ++i) {
        const int cidx = tid + i * NT;
        const int krow = cidx / (BN / 8), c8 = cidx % (BN / 8);
        const int kg = kt * BK + krow, ng = n0 + c8 * 8;
        const bool ok = kg < a.K && ng < a.Ncol;
        rb[i] = ld16(a.wgt + (long long)(ok ? kg : 0) * a.Ncol + (ok ? ng : 0), ok);
      }
    } else {
      // dgrad: B^T[n = ci][k = (kh,kw,co)] = W[kh][kw][ci][co]  (K-contiguous)
      const bool bok = b_tt < a.KH * a.KW;
#pragma unroll
      for (int i = 0; i < B_CHUNKS; ++i) {
        const int cidx = tid + i * NT;
        const int ng = n0 + (cidx >> 2);
        const bool ok = bok && ng < a.Ncol;
        rb[i] = ld16(a.wgt + ((long long)(ok ? b_tt : 0) * a.Cin + (ok ? ng : 0)) * a.Cout + b_co, ok);
      }
      b_co += BK;
      while (b_co >= a.Cout) { b_co -= a.Cout; ++b_tt; }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int row = (tid >> 2) + i * (NT / 4);
      st16(As[buf] + row * LDA + kc * 8, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const int cidx = tid + i * NT;
      if (MODE == 0) {
        const int krow = cidx / (BN / 8), c8 = cidx % (BN / 8);
        st16(Bs[buf] + krow * LDB_N + c8 * 8, rb[i]);
      } else {
        const int nrow = cidx >> 2, kcc = cidx & 3;
        st16(Bs[buf] + nrow * LDA + kcc * 8, rb[i]);
      }
    }
  };

  float4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  const int KT = (a.K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 1 < KT) load_tiles(kt + 1);
    bf16x8_t fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = frag_kcontig(As[cur], wm * (TM * 16) + i * 16, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (MODE == 0)
        fb[j] = frag_ncontig(Bs[cur], LDB_N, wn * (TN * 16) + j * 16, lane);
      else
        fb[j] = frag_kcontig(Bs[cur], wn * (TN * 16) + j * 16, lane);
    }
    // D[n][m] = W^T · X^T  -> lane owns 4 consecutive channels of one pixel
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fb[j], fa[i], acc[i][j]);
    if (kt + 1 < KT) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: bf16 stores (8 B per lane per tile) + optional BN statistics
  const int g = lane >> 4, li = lane & 15;
  float ssum[TN][4], ssq[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[j][r] = ssq[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const long long m = m0 + wm * (TM * 16) + i * 16 + li;
    const bool mok = m < a.M;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (TN * 16) + j * 16 + 4 * g;
      if (mok && n < a.Ncol) {
        float4v v = acc[i][j];
        uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(a.out + m * a.Ncol + n) = make_uint2(lo, hi);
        if (STATS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ssum[j][r] += v[r];
            ssq[j][r] += v[r] * v[r];
          }
        }
      }
    }
  }
  if (STATS) {
    // reduce over the 16 pixel lanes of each 16-lane group
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ssum[j][r] += __shfl_xor(ssum[j][r], o, 64);
          ssq[j][r] += __shfl_xor(ssq[j][r], o, 64);
        }
      }
    __syncthreads();  // LDS tiles are free now
    float* red = reinterpret_cast<float*>(smem_raw);   // [WM][BN] sums then [WM][BN] squares
    if (li == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = wn * (TN * 16) + j * 16 + 4 * g + r;
          red[wm * BN + nl] = ssum[j][r];
          red[WM * BN + wm * BN + nl] = ssq[j][r];
        }
    }
    __syncthreads();
    for (int nl = tid; nl < BN; nl += NT) {
      const int n = n0 + nl;
      if (n < a.Ncol) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          s += red[w * BN + nl];
          q += red[WM * BN + w * BN + nl];
        }
        // 64 atomic slots (zeroed by the caller) spread the M-tiles' partials
        const long long slot = (long long)(mt % a.stat_slots) * a.Ncol + n;
        atomicAdd(a.stat_sum + slot, s);
        atomicAdd(a.stat_sq + slot, q);
      }
    }
  }
}

// ============================================================================
// wgrad: rows r = (kh,kw,ci), cols co, reduction over output pixels m (split-K)
// A' = X gathered, staged [BK(m)][BM(r)] (r contiguous); B' = DY [BK(m)][BN(co)]
// ============================================================================
template <int BM, int BN>
__global__ void __launch_bounds__(NT) conv_wgrad_kernel(ConvArgs a) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int A_CHUNKS = BM * BK / 8 / NT;
  constexpr int B_CHUNKS = BN * BK / 8 / NT;
  constexpr int LDA = BM + PADN, LDB = BN + PADN;
  constexpr int A_ELEMS = BK * LDA, B_ELEMS = BK * LDB;
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small for 256 threads");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* As[2] = {smem, smem + A_ELEMS};
  bf16_t* Bs[2] = {smem + 2 * A_ELEMS, smem + 2 * A_ELEMS + B_ELEMS};

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_mn = a.mtiles * a.ntiles;
  const int tile = blockIdx.x % tiles_mn;
  const int split = blockIdx.x / tiles_mn;
  const int mt = tile / a.ntiles, nt = tile % a.ntiles;
  const int r0 = mt * BM, n0 = nt * BN;
  const int R = a.KH * a.KW * a.Cin;

  // per-thread A columns (r) fixed: decompose once
  int a_kh[A_CHUNKS], a_kw[A_CHUNKS], a_c[A_CHUNKS], a_mrow[A_CHUNKS], a_rc[A_CHUNKS];
  bool a_rok[A_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    const int cidx = tid + i * NT;
    a_mrow[i] = cidx / (BM / 8);
    a_rc[i] = cidx % (BM / 8);
    const int r = r0 + a_rc[i] * 8;
    a_rok[i] = r < R;
    const int rr = a_rok[i] ? r : 0;
    a_c[i] = rr % a.Cin;
    const int t = rr / a.Cin;
    a_kw[i] = t % a.KW;
    a_kh[i] = t / a.KW;
  }
  const long long Mpix = a.M;  // reduction length (pixels of DY)
  const int KT_total = static_cast<int>((Mpix + BK - 1) / BK);
  const int kt_begin = split * a.ksplit_steps;
  const int kt_end = min(KT_total, kt_begin + a.ksplit_steps);
  if (kt_begin >= kt_end) return;

  // incremental pixel decomposition of m = kt*BK + mrow for each A chunk
  int p_ow[A_CHUNKS], p_oh[A_CHUNKS], p_n[A_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    const long long m = (long long)kt_begin * BK + a_mrow[i];
    p_ow[i] = static_cast<int>(m % a.OW);
    const long long t = m / a.OW;
    p_oh[i] = static_cast<int>(t % a.OH);
    p_n[i] = static_cast<int>(t / a.OH);
  }
  uint4 ra[A_CHUNKS], rb[B_CHUNKS];
  // loads tile kt (called in order kt_begin, kt_begin+1, ...) and advances the pixel counters
  auto load_tiles = [&](int kt) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const long long m = (long long)kt * BK + a_mrow[i];
      const int iy = p_oh[i] * a.SH - a.PH + a_kh[i] * a.DH, ix = p_ow[i] * a.SW - a.PW + a_kw[i] * a.DW;
      const bool ok = a_rok[i] && m < Mpix && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      ra[i] = ld16(a.src + (((long long)p_n[i] * a.H + (ok ? iy : 0)) * a.W + (ok ? ix : 0)) * a.Cin + a_c[i], ok);
      p_ow[i] += BK;
      while (p_ow[i] >= a.OW) { p_ow[i] -= a.OW; if (++p_oh[i] == a.OH) { p_oh[i] = 0; ++p_n[i]; } }
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const int cidx = tid + i * NT;
      const int mrow = cidx / (BN / 8), c8 = cidx % (BN / 8);
      const long long m = (long long)kt * BK + mrow;
      const int n = n0 + c8 * 8;
      const bool ok = m < Mpix && n < a.Cout;
      rb[i] = ld16(a.dy + (ok ? m : 0) * a.Cout + (ok ? n : 0), ok);
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) st16(As[buf] + a_mrow[i] * LDA + a_rc[i] * 8, ra[i]);
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const int cidx = tid + i * NT;
      st16(Bs[buf] + (cidx / (BN / 8)) * LDB + (cidx % (BN / 8)) * 8, rb[i]);
    }
  };

  float4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  load_tiles(kt_begin);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    if (kt + 1 < kt_end) load_tiles(kt + 1);
    bf16x8_t fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = frag_ncontig(As[cur], LDA, wm * (TM * 16) + i * 16, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = frag_ncontig(Bs[cur], LDB, wn * (TN * 16) + j * 16, lane);
    // D[r][co]: lane owns 4 consecutive r of one co -> row-contiguous atomics
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
    if (kt + 1 < kt_end) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = n0 + wn * (TN * 16) + j * 16 + li;
      if (co >= a.Cout) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = r0 + wm * (TM * 16) + i * 16 + 4 * g + rr;
        if (r < R) atomicAdd(a.dw + (long long)r * a.Cout + co, acc[i][j][rr]);
      }
    }
}

// ============================================================================
// v2 forward / dgrad for C % 64 == 0: BK = 64, both operands K-contiguous in
// LDS (fwd takes the filter pre-transposed to Wt[co][(kh,kw,ci)]), staged by
// LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB = 8 rows x 128 B per wave
// instruction, no VGPR round trip) into a STAGES-deep ring with counted
// vmcnt waits and one raw barrier per K step.  Address generation is nearly
// free: per A row a 32-bit base offset and a bitmask of the taps that stay
// inside the image are computed once; each K step adds a wave-uniform tap
// offset and tests one bit; padding taps and rows past M/N get an offset
// beyond the buffer's num_records, which the hardware returns as zeros.
// LDS rows are 128 B; 16-B chunk c of row r lives at chunk c ^ ((r >> 1) & 7)
// (the swizzle is applied to the per-lane SOURCE address, the LDS image
// stays lane-linear), which makes the ds_read_b128 fragment reads of 16 rows
// conflict-free.  MODE 0 = forward, 1 = stride-1 dgrad, 2 = strided dgrad
// by stride-parity class: within one class of DX pixels the set of filter
// taps that reach DY is fixed and the DY offsets are affine again, so each
// class is a dense implicit GEMM over only its own taps (no zero-tap waste).
// ============================================================================
// Copy-out element idx (= tid + k * NT) of a BM x BN C tile staged in LDS -> (row, 16-B chunk).  ds_read_b128 serves
// a wave in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32): for BN = 128 each group
// gets one whole 256-B row of the tile (all 64 banks once).  The row-major order (lanes 0-15 row r, 16-31 row r + 1)
// gave every group parts of two rows whose 272-B pitch overlaps 4 banks: 2-way on every copy-out read.  Each 64-lane
// block still covers the same 4 rows, so only the lanes' assignment within them changes.
template <int BN>
__device__ __forceinline__ void copyout_rc(int idx, int& row, int& c8, bool remap) {
  if (BN == 128 && remap) {
    const int l = idx & 31, hh = (idx >> 5) & 1;
    const bool ga = l < 4 || (l >= 12 && l < 16) || (l >= 20 && l < 28);
    c8 = ga ? (l < 4 ? l : (l < 16 ? l - 8 : l - 12)) : (l < 12 ? l - 4 : (l < 20 ? l - 8 : l - 16));
    row = ((idx >> 6) << 2) + 2 * hh + (ga ? 0 : 1);
  } else {
    row = idx / (BN / 8);
    c8 = idx - row * (BN / 8);
  }
}

template <int BM, int BN, int MODE, bool STATS, int STAGES, int NW>
__global__ void __launch_bounds__(64 * NW) conv_fd_v2(ConvArgs a) {
  // NW = 4 waves (2x2) or 8 waves (one 256-row block per CU: 2 waves per SIMD, half the
  // operand traffic per FLOP of a 128x128 tile; 4x2 or 2x4 waves by the tile's aspect)
  constexpr int NT = 64 * NW;
  constexpr int WM = NW == 4 ? 2 : (BM > BN ? 4 : 2), WN = NW / WM;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int RA = BM / (8 * NW), RB = BN / (8 * NW);   // DMA instructions per wave per K step
  constexpr int ROWB = 128;                       // bytes per LDS row (64 bf16)
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int PER_STAGE = RA + RB;               // LDS-DMA wave-instructions per stage
  constexpr unsigned OOB = 0x80000000u;            // buffer offset past num_records -> zero fill
  // STAGES >= 10: split ring, SA = STAGES / 10 A stages and SB = STAGES % 10 B stages (SA > SB >= 2).  The A
  // operand (the gathered activation / output gradient) streams from HBM or the Infinity Cache and is read by one
  // tile only when the N grid is a single column; the B operand (filter) is shared by every tile and L2-resident.
  // One 64-KiB stage in flight left the 8-wave tiles latency-bound on A (32 KiB in flight per CU vs ~25-33 GB/s
  // per CU at ~1-2 us loaded latency); the split ring keeps SA - 1 A stages in flight in the same 160 KiB.
  constexpr bool SPLIT = STAGES >= 10;
  constexpr int SA = SPLIT ? STAGES / 10 : STAGES, SB = SPLIT ? STAGES % 10 : STAGES;
  static_assert(RA >= 1 && RB >= 1, "tile too small");
  static_assert(STAGES >= 1 && (STAGES < 2 || SPLIT || (STAGES - 2) * PER_STAGE < 64), "pipeline depth");  // 1: K == 64 only
  static_assert(!SPLIT || (SA > SB && SB >= 2 && (SA - 1) * PER_STAGE < 64), "split ring");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / a.ntiles, nt = tile % a.ntiles;
  const long long m0 = a.m_base + (long long)mt * BM;
  const int n0 = nt * BN;

  // MODE 3 (dense forward) gathers A like a 1x1 forward convolution; MODE 4 (dense data gradient with the
  // producer's activation backward in the epilogue) like a stride-1 dgrad
  constexpr int AM = MODE == 3 ? 0 : MODE == 4 ? 1 : MODE;
  const int GH = AM == 0 ? a.H : a.OH;
  const int GW = AM == 0 ? a.W : a.OW;
  const int GC = AM == 0 ? a.Cin : a.Cout;
  const int RH = AM == 0 ? a.OH : AM == 1 ? a.H : a.cls_Hc;
  const int RW = AM == 0 ? a.OW : AM == 1 ? a.W : a.cls_Wc;
  const int lrow = lane >> 3;
  const int TKW = MODE == 2 ? a.cls_tw : a.KW;      // taps per filter row of the K walk
  const int ntaps = MODE == 2 ? a.cls_th * a.cls_tw : a.KH * a.KW;   // <= 32 (host-checked)
  const int DHe = MODE == 2 ? 1 : a.DH, DWe = MODE == 2 ? 1 : a.DW;

  // buffer ranges: bounds-checked loads, out-of-range offsets read as zero (host checks < 2 GiB)
  const int bytes_a = (int)((long long)a.N * GH * GW * GC * 2);
  // (MODE 2 walks a subset of the filter taps: the range is the whole filter)
  const int bytes_b = MODE == 3 ? (int)((long long)a.K * a.ld_b * 2)
                                : (int)((long long)(MODE == 2 ? a.KH * a.KW * a.Cout : a.K) * a.Ncol * 2);
  // MODE 3: this block's column segment (seg_cols % BN == 0, host-checked)
  const int seg = MODE == 3 ? n0 / a.seg_cols : 0;
  const bf16_t* wbase = MODE == 3 ? a.wseg[seg] : a.wgt;
  const int nl0 = MODE == 3 ? n0 - seg * a.seg_cols : n0;

  // per A row: element offset of tap (0,0) (may be "negative", wraps) + valid-tap bitmask
  unsigned a_off[RA], a_mask[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int row = 8 * (wave + NW * i) + lrow;
    const long long m = m0 + row;
    const bool ok = m < a.M;
    // 32-bit index math: every tensor is < 2 GiB (host-checked), so rows and element offsets fit 31 bits
    const unsigned mm = ok ? static_cast<unsigned>(m) : 0u;
    const unsigned t = fdiv31(mm, a.mg_rw, a.sh_rw);
    const int ow = static_cast<int>(mm - t * static_cast<unsigned>(RW));
    const unsigned nq = fdiv31(t, a.mg_rh, a.sh_rh);
    const int oh = static_cast<int>(t - nq * static_cast<unsigned>(RH));
    const int n = static_cast<int>(nq);
    const int y0 = AM == 0 ? oh * a.SH - a.PH : AM == 1 ? oh + a.PH : a.cls_q0h + oh;
    const int x0 = AM == 0 ? ow * a.SW - a.PW : AM == 1 ? ow + a.PW : a.cls_q0w + ow;
    const int ch = 8 * ((lane & 7) ^ ((row >> 1) & 7));
    a_off[i] = static_cast<unsigned>(((n * GH + y0) * GW + x0) * GC + ch);
    unsigned mask = 0;
    if (ok) {
      for (int tt = 0; tt < ntaps; ++tt) {
        const int kh = tt / TKW, kw = tt - kh * TKW;
        const int iy = AM == 0 ? y0 + kh * DHe : y0 - kh * DHe;
        const int ix = AM == 0 ? x0 + kw * DWe : x0 - kw * DWe;
        if (iy >= 0 && iy < GH && ix >= 0 && ix < GW) mask |= 1u << tt;
      }
    }
    a_mask[i] = mask;
  }
  // per B row: byte offset of k = 0 (OOB for rows past Ncol)
  unsigned b_off[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    if (MODE == 3) {
      // 1 KiB block (wave + NW i) = rows 8 (blk & 7) .. +7 of half-image blk >> 3; each lane fetches the
      // 16-B column chunk that the transposed reads expect at its LDS slot
      const int blk = wave + NW * i;
      const int krow = 8 * (blk & 7) + lrow;
      const int col = nl0 + 64 * (blk >> 3) + 8 * ((lane & 7) ^ trswz(krow));
      b_off[i] = (unsigned)(((long long)krow * a.ld_b + col) * 2);
      continue;
    }
    const int row = 8 * (wave + NW * i) + lrow;
    const int n = n0 + row;
    const int ch = 8 * ((lane & 7) ^ ((row >> 1) & 7));
    const long long e = MODE == 0 ? (long long)n * a.K + ch : (long long)n * a.Cout + ch;
    b_off[i] = n < a.Ncol ? (unsigned)(e * 2) : OOB;
  }

  // scalar K-walk state: tap index, (kh, kw), channel offset c0 within the tap
  int s_t = 0, s_kh = 0, s_kw = 0, s_c0 = 0, s_k0 = 0;
  auto stage = [&](int buf) {
    const int tap_e = (AM == 0 ? (s_kh * DHe * GW + s_kw * DWe) : -(s_kh * DHe * GW + s_kw * DWe)) * GC + s_c0;
    char* lds = smem_raw + buf * STAGE;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const bool ok = (a_mask[i] >> s_t) & 1u;
      const unsigned voff = ok ? (a_off[i] + (unsigned)tap_e) * 2u : OOB;
      dma16(a.src, bytes_a, lds + (wave + NW * i) * 1024, voff, 0);
    }
    char* ldsb = lds + BM * ROWB;
    const int wtap = MODE == 2 ? (a.cls_kh0 + a.SH * s_kh) * a.KW + a.cls_kw0 + a.SW * s_kw : s_t;
    const int sb = MODE == 3 ? s_k0 * a.ld_b * 2 : MODE == 0 ? s_k0 * 2 : (wtap * a.Cin * a.Cout + s_c0) * 2;
#pragma unroll
    for (int i = 0; i < RB; ++i)
      dma16(wbase, bytes_b, ldsb + (wave + NW * i) * 1024, b_off[i], sb);
    // advance the K walk by 64 (scalar selects)
    s_k0 += 64;
    s_c0 += 64;
    const int wrap = s_c0 == GC ? 1 : 0;
    s_c0 = wrap ? 0 : s_c0;
    s_t += wrap;
    s_kw += wrap;
    const int wrap2 = s_kw == TKW ? 1 : 0;
    s_kw = wrap2 ? 0 : s_kw;
    s_kh += wrap2;
  };

  float4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // MODE 4: this thread's pre-activation vectors of the copy-out, loaded before the first stage so their HBM
  // latency hides under the main loop (the copy-out's row mapping: idx = tid + it * NT, 8 columns per idx)
  constexpr int PITER = MODE == 4 ? BM * (BN / 8) / (64 * NW) : 1;
  uint4 prepf[PITER];
  if constexpr (MODE == 4) {
#pragma unroll
    for (int it = 0; it < PITER; ++it) {
      const int idx = tid + it * 64 * NW;
      int row, c8;
      copyout_rc<BN>(idx, row, c8, a.co_remap != 0);
      const long long m = m0 + row;
      const int n = n0 + c8 * 8;
      prepf[it] = (m < a.M && n < a.Ncol) ? *reinterpret_cast<const uint4*>(a.pre_out + m * a.Ncol + n)
                                          : make_uint4(0, 0, 0, 0);
    }
  }

  const int KT = a.K / 64;
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (SPLIT) {
    // separate K walks for the A ring (SA - 1 steps ahead) and the B ring (SB - 1 steps ahead)
    struct Walk { int t, kh, kw, c0, k0; };
    Walk wa{0, 0, 0, 0, 0}, wb{0, 0, 0, 0, 0};
    auto advance = [&](Walk& w) {
      w.k0 += 64;
      w.c0 += 64;
      const int wrap = w.c0 == GC ? 1 : 0;
      w.c0 = wrap ? 0 : w.c0;
      w.t += wrap;
      w.kw += wrap;
      const int wrap2 = w.kw == TKW ? 1 : 0;
      w.kw = wrap2 ? 0 : w.kw;
      w.kh += wrap2;
    };
    char* const ringB = smem_raw + SA * BM * ROWB;
    auto stage_a = [&](int buf) {
      const int tap_e = (AM == 0 ? (wa.kh * DHe * GW + wa.kw * DWe) : -(wa.kh * DHe * GW + wa.kw * DWe)) * GC + wa.c0;
      char* lds = smem_raw + buf * (BM * ROWB);
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const bool ok = (a_mask[i] >> wa.t) & 1u;
        const unsigned voff = ok ? (a_off[i] + (unsigned)tap_e) * 2u : OOB;
        dma16(a.src, bytes_a, lds + (wave + NW * i) * 1024, voff, 0);
      }
      advance(wa);
    };
    auto stage_b = [&](int buf) {
      char* ldsb = ringB + buf * (BN * ROWB);
      const int wtap = MODE == 2 ? (a.cls_kh0 + a.SH * wb.kh) * a.KW + a.cls_kw0 + a.SW * wb.kw : wb.t;
      const int sb = MODE == 3 ? wb.k0 * a.ld_b * 2 : MODE == 0 ? wb.k0 * 2 : (wtap * a.Cin * a.Cout + wb.c0) * 2;
#pragma unroll
      for (int i = 0; i < RB; ++i)
        dma16(wbase, bytes_b, ldsb + (wave + NW * i) * 1024, b_off[i], sb);
      advance(wb);
    };
    // issue order: prologue group s = [B(s) if s <= SB-2, A(s)]; loop group j = [B(j+SB-1), A(j+SA-1)]
    // (each only while < KT).  vmcnt retires in issue order, so "A(kt) and B(kt) landed" = at most `younger`
    // operations issued after the later of the two are still outstanding.
    auto nb_of = [&](int j) { return (j + SB - 1 < KT ? RB : 0); };
    auto na_of = [&](int j) { return (j + SA - 1 < KT ? RA : 0); };
#pragma unroll
    for (int s = 0; s < SA - 1; ++s) {
      if (s <= SB - 2 && s < KT) stage_b(s);
      if (s < KT) stage_a(s);
    }
    int ca = 0, cb = 0;
    for (int kt = 0; kt < KT; ++kt) {
      int younger = 0;
      if (kt <= SB - 2) {                    // A(kt) last, in prologue group kt
        for (int s = kt + 1; s <= SA - 2; ++s) younger += (s <= SB - 2 && s < KT ? RB : 0) + (s < KT ? RA : 0);
        for (int j = 0; j < kt; ++j) younger += nb_of(j) + na_of(j);
      } else {                               // B(kt) last, first of loop group kt - SB + 1
        const int g0 = kt - SB + 1;
        younger = na_of(g0);
        for (int j = g0 + 1; j < kt; ++j) younger += nb_of(j) + na_of(j);
      }
      wait_vmcnt_le<(SA - 1) * PER_STAGE>(younger);
      __builtin_amdgcn_s_barrier();          // every wave's DMA of step kt is in; A(kt-1), B(kt-1) are free
      if (kt + SB - 1 < KT) stage_b(cb == 0 ? SB - 1 : cb - 1);      // buffer (kt + SB - 1) % SB
      if (kt + SA - 1 < KT) stage_a(ca == 0 ? SA - 1 : ca - 1);      // buffer (kt + SA - 1) % SA
      const char* As = smem_raw + ca * (BM * ROWB);
      const char* Bs = ringB + cb * (BN * ROWB);
      ca = ca + 1 == SA ? 0 : ca + 1;
      cb = cb + 1 == SB ? 0 : cb + 1;
      bf16x8_t fa[2][TM], fb[2][TN];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * (TM * 16) + i * 16 + fr;
          const int pc = (h * 4 + fq) ^ ((row >> 1) & 7);
          fa[h][i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(As + row * ROWB + pc * 16));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (MODE == 3) {
            const int col = wn * (TN * 16) + j * 16;
            fb[h][j] = frag_tr(Bs + (col >> 6) * 8192, col & 63, 32 * h, lane);
            continue;
          }
          const int row = wn * (TN * 16) + j * 16 + fr;
          const int pc = (h * 4 + fq) ^ ((row >> 1) & 7);
          fb[h][j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(Bs + row * ROWB + pc * 16));
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fb[h][j], fa[h][i], acc[i][j]);
      {
        constexpr int R = TM + TN, MF = TM * TN, PER = MF / R > 0 ? MF / R : 1;
        __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
#pragma unroll
        for (int i = 0; i < R; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * MF, 0);
      }
    }
  } else {
  // prologue: stages 0 .. STAGES-2 in flight
#pragma unroll
  for (int s = 0; s < (STAGES > 1 ? STAGES - 1 : 1); ++s)
    if (s < KT) stage(s);
  int cur = 0;
  for (int kt = 0; kt < KT; ++kt) {
    // stage kt must have landed: leave the (STAGES-2) younger stages in flight
    if (STAGES >= 2 && kt + STAGES - 2 < KT)
      wait_vmcnt<(STAGES >= 2 ? (STAGES - 2) * PER_STAGE : 0)>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();          // every wave's DMA for stage kt is in; buffer (kt-1) is free
    if (STAGES >= 2) {
      const int nk = kt + STAGES - 1;
      if (nk < KT) stage(nk % STAGES);
    }
    const char* As = smem_raw + cur * STAGE;
    cur = cur + 1 == STAGES ? 0 : cur + 1;
    const char* Bs = As + BM * ROWB;
    // both K halves' fragments in registers; the scheduling groups below issue the first
    // half's reads, then interleave the second half's reads with the first half's MFMAs
    bf16x8_t fa[2][TM], fb[2][TN];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (TM * 16) + i * 16 + fr;
        const int pc = (h * 4 + fq) ^ ((row >> 1) & 7);
        fa[h][i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(As + row * ROWB + pc * 16));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (MODE == 3) {
          const int col = wn * (TN * 16) + j * 16;
          fb[h][j] = frag_tr(Bs + (col >> 6) * 8192, col & 63, 32 * h, lane);
          continue;
        }
        const int row = wn * (TN * 16) + j * 16 + fr;
        const int pc = (h * 4 + fq) ^ ((row >> 1) & 7);
        fb[h][j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(Bs + row * ROWB + pc * 16));
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fb[h][j], fa[h][i], acc[i][j]);
    {
      constexpr int R = TM + TN, MF = TM * TN, PER = MF / R > 0 ? MF / R : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, R, 0);      // half 0 reads
#pragma unroll
      for (int i = 0; i < R; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // half 0 MFMAs ...
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // ... with one half 1 read each
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MF, 0); // the rest
    }
  }
  }

  // ---- epilogue: the C tile goes through LDS ([px][ch], rows padded by 16 B) so the
  // global stores are 16 B per lane along full output rows; BN statistics from the
  // fp32 accumulators (16-lane shuffles, then one atomic per channel per block)
  constexpr int LDC = BN * 2 + 16;
  // (the launcher sizes the LDS as max(stages, C tile))
  const int g = lane >> 4, li = lane & 15;
  __syncthreads();                           // every wave is done reading the stage buffers
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int pl = wm * (TM * 16) + i * 16 + li;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wn * (TN * 16) + j * 16 + 4 * g;
      float4v v = acc[i][j];
      if (MODE == 3 && a.bias) {                 // bias on the fp32 accumulators (one rounding)
        const uint2 b4 = *reinterpret_cast<const uint2*>(a.bias + n0 + cl);
        v[0] += __uint_as_float(b4.x << 16);
        v[1] += __uint_as_float(b4.x & 0xffff0000u);
        v[2] += __uint_as_float(b4.y << 16);
        v[3] += __uint_as_float(b4.y & 0xffff0000u);
      }
      uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      // 8-B half swap on rows 8..15 of every 16: rows li and li+8 would otherwise share
      // banks ((LDC/4) % 32 == 4) and the ds_write_b64 would be 2-way
      *reinterpret_cast<uint2*>(smem_raw + pl * LDC + ((cl * 2) ^ (((pl >> 3) & 1) << 3))) = make_uint2(lo, hi);
    }
  }
  __syncthreads();
  const bool bstat = (MODE == 1 || MODE == 2) && a.bsum != nullptr;
  float bs0[8], bs1[8];                        // this thread's BN-backward partials (fixed c8 per thread)
#pragma unroll
  for (int k = 0; k < 8; ++k) bs0[k] = bs1[k] = 0.f;
  // every global read of the copy-out (old DX when accumulating, BN input x and ReLU mask for the
  // statistics) is issued for all of this thread's rows before the first store: one latency, not ITER
  constexpr int ITER = BM * (BN / 8) / NT;
  static_assert(ITER * NT == BM * (BN / 8), "copy-out rows per thread");
  // rows in flight (register budget of the 256-row tiles; the 448-row tile's 14 rows per thread go in pairs)
  // (data gradients: the accumulators are dead once the C tile is in LDS, so up to 16 rows' reads go out at once
  // -- one latency per tile instead of ITER / 4; MDTF_FD_PF16=0 builds keep groups of 4)
  constexpr int PF = (FD_PF16 && (MODE == 1 || MODE == 2) && ITER <= 16) ? ITER
                                                                        : (ITER < 4 ? ITER : (ITER % 4 == 0 ? 4 : 2));
  static_assert(ITER % PF == 0, "prefetch groups");
#pragma unroll
  for (int g0 = 0; g0 < ITER; g0 += PF) {
  long long off[PF];
  uint4 old4[PF], x4[PF];
  uint32_t mb[PF];
#pragma unroll
  for (int it = 0; it < PF; ++it) {
    const int idx = tid + (g0 + it) * NT;
    int row, c8;
    copyout_rc<BN>(idx, row, c8, a.co_remap != 0);
    const long long m = m0 + row;
    const int n = n0 + c8 * 8;
    off[it] = -1;
    if (m < a.M && n < a.Ncol) {
      long long pix = m;
      if (MODE == 2) {          // class pixel (n, i, j) -> DX pixel (n, h0 + SH i, w0 + SW j)
        const unsigned mu = static_cast<unsigned>(m);
        const unsigned t = fdiv31(mu, a.mg_rw, a.sh_rw);          // RW = cls_Wc, RH = cls_Hc in MODE 2
        const int j = static_cast<int>(mu - t * static_cast<unsigned>(a.cls_Wc));
        const unsigned nb = fdiv31(t, a.mg_rh, a.sh_rh);
        const int i = static_cast<int>(t - nb * static_cast<unsigned>(a.cls_Hc));
        pix = (static_cast<long long>(nb) * a.H + a.cls_h0 + a.SH * i) * a.W + a.cls_w0 + a.SW * j;
      }
      off[it] = pix * a.Ncol + n;
      if (a.accumulate) {
        old4[it] = *reinterpret_cast<const uint4*>((a.acc_src ? a.acc_src : a.out) + off[it]);
        if (a.acc_mask) old4[it] = mask_bf8(old4[it], a.acc_mask[off[it] >> 3]);
      }
      if (bstat) {
        x4[it] = *reinterpret_cast<const uint4*>(a.bx + off[it]);
        mb[it] = a.bmask ? a.bmask[off[it] >> 3] : 0xffu;
      }
    }
  }
#pragma unroll
  for (int it = 0; it < PF; ++it) {
    if (off[it] < 0) continue;
    const int idx = tid + (g0 + it) * NT;
    int row, c8;
    copyout_rc<BN>(idx, row, c8, a.co_remap != 0);
    uint4 v = *reinterpret_cast<const uint4*>(smem_raw + row * LDC + c8 * 16);
    if ((row >> 3) & 1) v = make_uint4(v.z, v.w, v.x, v.y);
    bf16_t* dst = a.out + off[it];
    if (MODE == 3 && a.act) {                    // activation epilogue on the rounded pre-activation
      if (a.pre_out) *reinterpret_cast<uint4*>(a.pre_out + off[it]) = v;
      float c[8];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c[2 * k] = dense_act(__uint_as_float(w4[k] << 16), a.act);
        c[2 * k + 1] = dense_act(__uint_as_float(w4[k] & 0xffff0000u), a.act);
      }
      store_bf8(dst, c);
    } else if (MODE == 4) {                      // the producer's activation backward: dx = (dy W^T) act'(pre)
      float c[8];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      const uint4 pv = prepf[(g0 + it) % PITER];
      const uint32_t p4[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c[2 * k] = __uint_as_float(w4[k] << 16) * dense_act_grad(__uint_as_float(p4[k] << 16), a.act);
        c[2 * k + 1] = __uint_as_float(w4[k] & 0xffff0000u) * dense_act_grad(__uint_as_float(p4[k] & 0xffff0000u), a.act);
      }
      store_bf8(dst, c);
    } else if (a.accumulate || bstat) {
      float c[8];
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c[2 * k] = __uint_as_float(w4[k] << 16);
        c[2 * k + 1] = __uint_as_float(w4[k] & 0xffff0000u);
      }
      if (a.accumulate) {        // second contribution to a fanned-out activation gradient
        const uint32_t o4[4] = {old4[it].x, old4[it].y, old4[it].z, old4[it].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = __uint_as_float(o4[k] << 16) + c[2 * k];
          const float hi = __uint_as_float(o4[k] & 0xffff0000u) + c[2 * k + 1];
          c[2 * k] = __uint_as_float((uint32_t)f2bf(lo) << 16);      // as stored
          c[2 * k + 1] = __uint_as_float((uint32_t)f2bf(hi) << 16);
        }
        store_bf8(dst, c);
      } else {
        *reinterpret_cast<uint4*>(dst) = v;
      }
      if (bstat) {
        const uint32_t xw[4] = {x4[it].x, x4[it].y, x4[it].z, x4[it].w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xk = (k & 1) ? __uint_as_float(xw[k >> 1] & 0xffff0000u) : __uint_as_float(xw[k >> 1] << 16);
          const float gk = ((mb[it] >> k) & 1u) ? c[k] : 0.f;
          bs0[k] += gk;
          bs1[k] += gk * xk;
        }
      }
    } else {
      *reinterpret_cast<uint4*>(dst) = v;
    }
  }
  }
  if (bstat) {
    static_assert(NT % (BN / 8) == 0, "one channel chunk per thread");
    __syncthreads();                           // the C tile copy-out is done with the LDS
    // [16][NT + 4] floats: the per-k rows are written lane-contiguously; the reads (ds_read_b32: two 32-lane groups,
    // bank = dword mod 32) of lanes (k = lane & 7, c8 = lane >> 3) hit dword 4k + c8 mod 32 -- distinct within a
    // group (an NT + 8 pad put k and k + 4 on one bank: 2-way on every read)
    constexpr int LDR = NT + 4;
    float* red = reinterpret_cast<float*>(smem_raw);
    // this thread's slot: slot % (BN / 8) == its chunk c8 (the reads below walk t2 = c8 + j BN / 8); with the
    // BN = 128 copy-out remap the chunk is not tid % 16: slot = (wave, row within the wave's 4, c8)
    int slot = tid;
    if (BN == 128 && a.co_remap) {
      int r0_, c0_;
      copyout_rc<BN>(tid, r0_, c0_, true);
      slot = (tid & ~63) | ((r0_ & 3) << 4) | c0_;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[k * LDR + slot] = bs0[k];
      red[(8 + k) * LDR + slot] = bs1[k];
    }
    __syncthreads();
    for (int nl = tid; nl < BN; nl += NT) {
      const int n = n0 + nl, c8 = nl >> 3, k = nl & 7;
      if (n < a.Ncol) {
        float sv = 0.f, q = 0.f;
        for (int t2 = c8; t2 < NT; t2 += BN / 8) {
          sv += red[k * LDR + t2];
          q += red[(8 + k) * LDR + t2];
        }
        const long long slot = (long long)(mt % a.bslots) * a.Ncol + n;
        atomicAdd(a.bsum + slot, sv);
        atomicAdd(a.bsq + slot, q);
      }
    }
  }
  if (STATS) {
    float ssum[TN][4], ssq[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ssum[j][r] = ssq[j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bool mok = m0 + wm * (TM * 16) + i * 16 + li < a.M;
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if (mok) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ssum[j][r] += acc[i][j][r];
            ssq[j][r] += acc[i][j][r] * acc[i][j][r];
          }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ssum[j][r] += __shfl_xor(ssum[j][r], o, 64);
          ssq[j][r] += __shfl_xor(ssq[j][r], o, 64);
        }
      }
    __syncthreads();                         // the C tile copy-out is done with the LDS
    float* red = reinterpret_cast<float*>(smem_raw);
    if (li == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int nl = wn * (TN * 16) + j * 16 + 4 * g + r;
          red[wm * BN + nl] = ssum[j][r];
          red[WM * BN + wm * BN + nl] = ssq[j][r];
        }
    }
    __syncthreads();
    for (int nl = tid; nl < BN; nl += NT) {
      const int n = n0 + nl;
      if (n < a.Ncol) {
        float sv = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          sv += red[w * BN + nl];
          q += red[WM * BN + w * BN + nl];
        }
        const long long slot = (long long)(mt % a.stat_slots) * a.Ncol + n;
        atomicAdd(a.stat_sum + slot, sv);
        atomicAdd(a.stat_sq + slot, q);
      }
    }
  }
}

// ============================================================================
// Persistent v2 forward / data gradient (MODE 0..2), register epilogue.
// One workgroup per (CU x occupancy) walks tiles w = blockIdx.x + i * gridDim.x in XCD-contiguous order
// (tile = xcd_remap(w, tiles): the tiles an XCD runs at once are consecutive, sharing A rows in its L2).
// The epilogue stores straight from the accumulators: v_permlane16_swap of fragment pairs (j, j+1) gives every
// lane 8 consecutive channels of one pixel (16-B buffer stores; out-of-range rows / columns get an offset past
// num_records, so every wave issues the same number of memory instructions), so the C tile never goes through
// LDS.  With a plain (or forward BN-statistics) epilogue the NEXT tile's row setup and prologue LDS-DMA are issued
// before the stores: its first operands land while this tile's output drains, and the tiles on different CUs
// drift out of lockstep, spreading the HBM write bursts over the main loops.  Epilogues that read (accumulate
// source, BN-backward statistics) issue the next prologue after their loads are consumed (an early DMA would be
// waited for by every load behind it: vmcnt retires in issue order).
// ============================================================================
template <int BM, int BN, int MODE, bool STATS, int STAGES, int NW, bool HEAVY>
__global__ void __launch_bounds__(64 * NW) conv_fd_p(ConvArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int WM = NW == 4 ? 2 : (BM > BN ? 4 : 2), WN = NW / WM;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int RA = BM / (8 * NW), RB = BN / (8 * NW);
  constexpr int ROWB = 128;
  constexpr int PER_STAGE = RA + RB;
  constexpr unsigned OOB = 0x80000000u;
  constexpr bool SPLIT = STAGES >= 10;
  constexpr int SA = SPLIT ? STAGES / 10 : STAGES, SB = SPLIT ? STAGES % 10 : STAGES;
  constexpr int RING = (SA * BM + SB * BN) * ROWB;
  static_assert(MODE <= 2 && TN % 2 == 0 && RA >= 1 && RB >= 1, "persistent tile");
  constexpr int EMAX = TM * (TN / 2);             // epilogue stores per wave (the E of the first waits)
  static_assert(SA >= SB && SB >= 2 && (SA - 1) * PER_STAGE + EMAX < 64, "persistent ring");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* red = reinterpret_cast<float*>(smem_raw + RING);        // STATS: [2][WM][BN] (outside the ring)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int total = a.mtiles * a.ntiles;
  const int GH = MODE == 0 ? a.H : a.OH;
  const int GW = MODE == 0 ? a.W : a.OW;
  const int GC = MODE == 0 ? a.Cin : a.Cout;
  const int RH = MODE == 0 ? a.OH : MODE == 1 ? a.H : a.cls_Hc;
  const int RW = MODE == 0 ? a.OW : MODE == 1 ? a.W : a.cls_Wc;
  const int lrow = lane >> 3;
  const int TKW = MODE == 2 ? a.cls_tw : a.KW;
  const int ntaps = MODE == 2 ? a.cls_th * a.cls_tw : a.KH * a.KW;
  const int DHe = MODE == 2 ? 1 : a.DH, DWe = MODE == 2 ? 1 : a.DW;
  const int bytes_a = (int)((long long)a.N * GH * GW * GC * 2);
  const int bytes_b = (int)((long long)(MODE == 2 ? a.KH * a.KW * a.Cout : a.K) * a.Ncol * 2);
  const int bytes_o = (int)((long long)a.N * (MODE == 0 ? a.OH * a.OW : a.H * a.W) * a.Ncol * 2);
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, bytes_o, 0x00020000);
  // HEAVY (template): an epilogue that reads (accumulate source / BN-backward statistics); the plain instantiation
  // carries none of its registers (the 256 x 256 tile fits 2 waves per SIMD without spilling only then)
  constexpr bool heavy = HEAVY && (MODE == 1 || MODE == 2);
  const bool bstat = heavy && a.bsum != nullptr;
  const int KT = a.K / 64;

  // ---- per-tile state
  int mt = 0, nt = 0;
  long long m0 = 0;
  int n0 = 0;
  unsigned a_off[RA], a_mask[RA], b_off[RB];
  auto setup = [&](int w) {
    const int tile = xcd_remap(w, total);
    mt = tile / a.ntiles;
    nt = tile - mt * a.ntiles;
    m0 = a.m_base + (long long)mt * BM;
    n0 = nt * BN;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int row = 8 * (wave + NW * i) + lrow;
      const long long m = m0 + row;
      const bool ok = m < a.M;
      const unsigned mm = ok ? static_cast<unsigned>(m) : 0u;
      const unsigned t = fdiv31(mm, a.mg_rw, a.sh_rw);
      const int ow = static_cast<int>(mm - t * static_cast<unsigned>(RW));
      const unsigned nq = fdiv31(t, a.mg_rh, a.sh_rh);
      const int oh = static_cast<int>(t - nq * static_cast<unsigned>(RH));
      const int n = static_cast<int>(nq);
      const int y0 = MODE == 0 ? oh * a.SH - a.PH : MODE == 1 ? oh + a.PH : a.cls_q0h + oh;
      const int x0 = MODE == 0 ? ow * a.SW - a.PW : MODE == 1 ? ow + a.PW : a.cls_q0w + ow;
      const int ch = 8 * ((lane & 7) ^ ((row >> 1) & 7));
      a_off[i] = static_cast<unsigned>(((n * GH + y0) * GW + x0) * GC + ch);
      unsigned mask = 0;
      if (ok) {
        for (int tt = 0; tt < ntaps; ++tt) {
          const int kh = tt / TKW, kw = tt - kh * TKW;
          const int iy = MODE == 0 ? y0 + kh * DHe : y0 - kh * DHe;
          const int ix = MODE == 0 ? x0 + kw * DWe : x0 - kw * DWe;
          if (iy >= 0 && iy < GH && ix >= 0 && ix < GW) mask |= 1u << tt;
        }
      }
      a_mask[i] = mask;
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int row = 8 * (wave + NW * i) + lrow;
      const int n = n0 + row;
      const int ch = 8 * ((lane & 7) ^ ((row >> 1) & 7));
      const int e = MODE == 0 ? n * a.K + ch : n * a.Cout + ch;
      b_off[i] = n < a.Ncol ? static_cast<unsigned>(e * 2) : OOB;
    }
  };

  struct Walk { int t, kh, kw, c0, k0; };
  Walk wa{0, 0, 0, 0, 0}, wb{0, 0, 0, 0, 0};
  auto advance = [&](Walk& w) {
    w.k0 += 64;
    w.c0 += 64;
    const int wrap = w.c0 == GC ? 1 : 0;
    w.c0 = wrap ? 0 : w.c0;
    w.t += wrap;
    w.kw += wrap;
    const int wrap2 = w.kw == TKW ? 1 : 0;
    w.kw = wrap2 ? 0 : w.kw;
    w.kh += wrap2;
  };
  char* const ringB = smem_raw + SA * BM * ROWB;
  auto stage_a = [&](int buf) {
    const int tap_e = (MODE == 0 ? (wa.kh * DHe * GW + wa.kw * DWe) : -(wa.kh * DHe * GW + wa.kw * DWe)) * GC + wa.c0;
    char* lds = smem_raw + buf * (BM * ROWB);
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const bool ok = (a_mask[i] >> wa.t) & 1u;
      const unsigned voff = ok ? (a_off[i] + (unsigned)tap_e) * 2u : OOB;
      dma16(a.src, bytes_a, lds + (wave + NW * i) * 1024, voff, 0);
    }
    advance(wa);
  };
  auto stage_b = [&](int buf) {
    char* ldsb = ringB + buf * (BN * ROWB);
    const int wtap = MODE == 2 ? (a.cls_kh0 + a.SH * wb.kh) * a.KW + a.cls_kw0 + a.SW * wb.kw : wb.t;
    const int sb = MODE == 0 ? wb.k0 * 2 : (wtap * a.Cin * a.Cout + wb.c0) * 2;
#pragma unroll
    for (int i = 0; i < RB; ++i) dma16(a.wgt, bytes_b, ldsb + (wave + NW * i) * 1024, b_off[i], sb);
    advance(wb);
  };
  auto prologue = [&]() {
    wa = Walk{0, 0, 0, 0, 0};
    wb = Walk{0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < SA - 1; ++s) {
      if (s <= SB - 2 && s < KT) stage_b(s);
      if (s < KT) stage_a(s);
    }
  };
  auto nb_of = [&](int j) { return (j + SB - 1 < KT ? RB : 0); };
  auto na_of = [&](int j) { return (j + SA - 1 < KT ? RA : 0); };

  int w = blockIdx.x;
  setup(w);
  prologue();
  int E = 0;            // memory instructions this wave issued after the current tile's prologue (lower bound)
  const int fr = lane & 15, fq = lane >> 4;
  const int g = fq, li = fr;
  for (;;) {
    float4v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    int ca = 0, cb = 0;
    for (int kt = 0; kt < KT; ++kt) {
      int younger = 0;
      if (kt <= SB - 2) {                    // A(kt) last, in prologue group kt (the epilogue ops came after it)
        for (int s = kt + 1; s <= SA - 2; ++s) younger += (s <= SB - 2 && s < KT ? RB : 0) + (s < KT ? RA : 0);
        younger += E;
        for (int j = 0; j < kt; ++j) younger += nb_of(j) + na_of(j);
      } else {
        const int g0 = kt - SB + 1;          // B(kt) (or, SA == SB, A(kt)) last, in loop group g0
        younger = SA > SB ? na_of(g0) : 0;
        for (int j = g0 + 1; j < kt; ++j) younger += nb_of(j) + na_of(j);
      }
      wait_vmcnt_le<(SA - 1) * PER_STAGE + EMAX>(younger);
      __builtin_amdgcn_s_barrier();
      if (kt + SB - 1 < KT) stage_b(cb == 0 ? SB - 1 : cb - 1);
      if (kt + SA - 1 < KT) stage_a(ca == 0 ? SA - 1 : ca - 1);
      const char* As = smem_raw + ca * (BM * ROWB);
      const char* Bs = ringB + cb * (BN * ROWB);
      ca = ca + 1 == SA ? 0 : ca + 1;
      cb = cb + 1 == SB ? 0 : cb + 1;
      bf16x8_t fa[2][TM], fb[2][TN];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * (TM * 16) + i * 16 + fr;
          const int pc = (h * 4 + fq) ^ ((row >> 1) & 7);
          fa[h][i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(As + row * ROWB + pc * 16));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * (TN * 16) + j * 16 + fr;
          const int pc = (h * 4 + fq) ^ ((row >> 1) & 7);
          fb[h][j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(Bs + row * ROWB + pc * 16));
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fb[h][j], fa[h][i], acc[i][j]);
      {
        constexpr int R = TM + TN, MF = TM * TN, PER = MF / R > 0 ? MF / R : 1;
        __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
#pragma unroll
        for (int i = 0; i < R; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * MF, 0);
      }
    }
    // every wave is past its last LDS read of this tile: the ring may be refilled
    __builtin_amdgcn_s_barrier();
    const int cur_mt = mt;
    const long long cur_m0 = m0;
    const int cur_n0 = n0;
    const int w_next = w + static_cast<int>(gridDim.x);
    const bool more = w_next < total;
    if (more && !heavy) {
      setup(w_next);
      prologue();
    }
    // ---- register epilogue of tile (cur_m0, cur_n0)
    int issued = 0;
    constexpr int NBS = heavy ? TN / 2 : 1;
    float bs0[NBS][8], bs1[NBS][8];
#pragma unroll
    for (int jp = 0; jp < NBS; ++jp)
#pragma unroll
      for (int k = 0; k < 8; ++k) bs0[jp][k] = bs1[jp][k] = 0.f;
    const int pcol = 16 * (fq & 1) + 8 * (fq >> 1);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const long long m = cur_m0 + wm * (TM * 16) + i * 16 + li;
      const bool rok = m < a.M;
      long long pix = m;
      if (MODE == 2) {
        const unsigned mu = rok ? static_cast<unsigned>(m) : 0u;
        const unsigned t = fdiv31(mu, a.mg_rw, a.sh_rw);
        const int jj = static_cast<int>(mu - t * static_cast<unsigned>(a.cls_Wc));
        const unsigned nb = fdiv31(t, a.mg_rh, a.sh_rh);
        const int ii = static_cast<int>(t - nb * static_cast<unsigned>(a.cls_Hc));
        pix = (static_cast<long long>(nb) * a.H + a.cls_h0 + a.SH * ii) * a.W + a.cls_w0 + a.SW * jj;
      }
#pragma unroll
      for (int jp = 0; jp < TN / 2; ++jp) {
        const int j = 2 * jp;
        const float4v v0 = acc[i][j], v1 = acc[i][j + 1];
        const uint32_t x0 = pack_bf2(v0[0], v0[1]), y0 = pack_bf2(v0[2], v0[3]);
        const uint32_t x1 = pack_bf2(v1[0], v1[1]), y1 = pack_bf2(v1[2], v1[3]);
        const auto sx = __builtin_amdgcn_permlane16_swap(x0, x1, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(y0, y1, false, false);
        uint4 o = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        const int ch = cur_n0 + wn * (TN * 16) + 16 * j + pcol;
        const bool ok = rok && ch < a.Ncol;
        const long long off = ok ? pix * a.Ncol + ch : 0;
        const unsigned voff = ok ? static_cast<unsigned>(off * 2) : OOB;
        if constexpr (heavy) {
          float c[8];
          unpack8(o, c);
          if (a.accumulate) {
            const bf16_t* src = a.acc_src ? a.acc_src : a.out;
            uint4 old = ok ? *reinterpret_cast<const uint4*>(src + off) : make_uint4(0, 0, 0, 0);
            if (a.acc_mask && ok) old = mask_bf8(old, a.acc_mask[off >> 3]);
            float ov[8];
            unpack8(old, ov);
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = __uint_as_float((uint32_t)f2bf(c[k] + ov[k]) << 16);   // as stored
            o = make_uint4(pack_bf2(c[0], c[1]), pack_bf2(c[2], c[3]), pack_bf2(c[4], c[5]), pack_bf2(c[6], c[7]));
          }
          if (bstat && ok) {
            const uint4 xq = *reinterpret_cast<const uint4*>(a.bx + off);
            const uint32_t mb = a.bmask ? a.bmask[off >> 3] : 0xffu;
            float xv[8];
            unpack8(xq, xv);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float gk = ((mb >> k) & 1u) ? c[k] : 0.f;
              bs0[jp][k] += gk;
              bs1[jp][k] += gk * xv[k];
            }
          }
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, o), rs_out, voff, 0, 0);
        ++issued;
      }
    }
    if constexpr (heavy) if (bstat) {
      // channels of (jp, lane group fq) summed over the wave's 16 pixel lanes, then over the WM waves of a
      // column block in LDS (the ring is free: heavy epilogues issue the next prologue afterwards)
#pragma unroll
      for (int jp = 0; jp < TN / 2; ++jp)
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int o2 = 1; o2 < 16; o2 <<= 1) {
            bs0[jp][k] += __shfl_xor(bs0[jp][k], o2, 64);
            bs1[jp][k] += __shfl_xor(bs1[jp][k], o2, 64);
          }
      float* rb = reinterpret_cast<float*>(smem_raw);           // [2][WM][BN]
      if (li == 0) {
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int nl = wn * (TN * 16) + 32 * jp + pcol + k;
            rb[wm * BN + nl] = bs0[jp][k];
            rb[WM * BN + wm * BN + nl] = bs1[jp][k];
          }
      }
      __syncthreads();
      for (int nl = tid; nl < BN; nl += NT) {
        const int n = cur_n0 + nl;
        if (n < a.Ncol) {
          float sv = 0.f, q = 0.f;
#pragma unroll
          for (int w2 = 0; w2 < WM; ++w2) {
            sv += rb[w2 * BN + nl];
            q += rb[WM * BN + w2 * BN + nl];
          }
          const long long slot = (long long)(cur_mt % a.bslots) * a.Ncol + n;
          atomicAdd(a.bsum + slot, sv);
          atomicAdd(a.bsq + slot, q);
        }
      }
    }
    if (STATS) {
      float ssum[TN][4], ssq[TN][4];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[j][r] = ssq[j][r] = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool mok = cur_m0 + wm * (TM * 16) + i * 16 + li < a.M;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (mok) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              ssum[j][r] += acc[i][j][r];
              ssq[j][r] += acc[i][j][r] * acc[i][j][r];
            }
          }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int o2 = 1; o2 < 16; o2 <<= 1) {
            ssum[j][r] += __shfl_xor(ssum[j][r], o2, 64);
            ssq[j][r] += __shfl_xor(ssq[j][r], o2, 64);
          }
      if (li == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nl = wn * (TN * 16) + j * 16 + 4 * g + r;
            red[wm * BN + nl] = ssum[j][r];
            red[WM * BN + wm * BN + nl] = ssq[j][r];
          }
      }
      __syncthreads();
      for (int nl = tid; nl < BN; nl += NT) {
        const int n = cur_n0 + nl;
        if (n < a.Ncol) {
          float sv = 0.f, q = 0.f;
#pragma unroll
          for (int w2 = 0; w2 < WM; ++w2) {
            sv += red[w2 * BN + nl];
            q += red[WM * BN + w2 * BN + nl];
          }
          const long long slot = (long long)(cur_mt % a.stat_slots) * a.Ncol + n;
          atomicAdd(a.stat_sum + slot, sv);
          atomicAdd(a.stat_sq + slot, q);
        }
      }
    }
    if (!more) break;
    if (heavy) {
      __syncthreads();                       // the statistics reduction is done with the ring
      setup(w_next);
      prologue();
      E = 0;
    } else {
      E = issued;                            // stores after the prologue (atomics not counted: lower bound)
    }
    w = w_next;
  }
}

// MDTF_CONV_PERSIST=1: the v2 forward / data-gradient launches run the persistent register-epilogue kernel
// (conv_fd_p) where its ring fits; =0 (default until the in-step A/B says otherwise) keeps conv_fd_v2
int conv_persist_mode() {
  static const int m = [] {
    const char* e = getenv("MDTF_CONV_PERSIST");
    return e ? atoi(e) : 0;
  }();
  return m;
}

int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      return 256;
    return v;
  }();
  return n;
}

template <int BM, int BN, int MODE, bool STATS, int STAGES, int NW>
int launch_fd_p(ConvArgs& a, hipStream_t st) {
  constexpr int NT = 64 * NW;
  constexpr int WM = NW == 4 ? 2 : (BM > BN ? 4 : 2), WN = NW / WM;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int SA = STAGES >= 10 ? STAGES / 10 : STAGES, SB = STAGES >= 10 ? STAGES % 10 : STAGES;
  const bool heavy = (MODE == 1 || MODE == 2) && (a.accumulate || a.bsum != nullptr);
  // MDTF_CONV_PERSIST=2: only the 8-wave 256 x 256 forward (plain / statistics epilogue)
  if (conv_persist_mode() == 2 && !(MODE == 0 && NW == 8 && BM == 256 && BN == 256)) return MDTF_EUNSUPPORTED;
  // (wave tiles of 7-8 row fragments with a reading epilogue, 256 x 256 / 448 x 128 dgrads: the persistent state
  // does not fit 2 waves per SIMD next to their 128 accumulator registers -- they stay on conv_fd_v2)
  if constexpr (MODE > 2 || TN % 2 != 0 || SB < 2) {
    return MDTF_EUNSUPPORTED;
  } else {
    if (heavy && TM > 4) return MDTF_EUNSUPPORTED;
    const size_t ring = ((size_t)SA * BM + (size_t)SB * BN) * 128;
    const size_t lds = ring + (STATS ? (size_t)2 * WM * BN * sizeof(float) : 0);
    if (lds > 160 * 1024) return MDTF_EUNSUPPORTED;
    // the heavy instantiation only where its registers fit (TM <= 4)
    auto kern = heavy ? conv_fd_p<BM, BN, MODE, STATS, STAGES, NW, (MODE != 0 && TM <= 4)>
                      : conv_fd_p<BM, BN, MODE, STATS, STAGES, NW, false>;
    static int occ[2] = {0, 0};
    if (occ[heavy] == 0) {
      int o = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, NT, lds) != hipSuccess || o < 1) o = 1;
      occ[heavy] = o;
    }
    const long long total = (long long)a.mtiles * a.ntiles;
    const long long cap = (long long)num_cus() * occ[heavy];
    const unsigned grid = (unsigned)(total < cap ? total : cap);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, st, a);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
}

// MDTF_CONV_TAIL=1: tile-count tail split for tails under a quarter of a wave; 2: every partial wave; 0 (default:
// neutral in the ResNet-50 step, 13090 vs 13086 img/s, profiles/ab_r6.md): off
int conv_tail_mode() {
  static const int m = [] {
    const char* e = getenv("MDTF_CONV_TAIL");
    return e ? atoi(e) : 0;
  }();
  return m;
}

extern "C" int mdtf_get_deterministic();

template <int BM, int BN, int MODE, bool STATS, int STAGES, int NW = 4>
int launch_fd_v2(ConvArgs& a, hipStream_t st);

// The 8-wave 256-row tiles hold one workgroup per CU, so a tile count just past a multiple of the CU count costs a
// whole extra round for a few tiles (ResNet-50 at batch 256: 784 = 3 x 256 + 16 tiles, 1568 = 6 x 256 + 32).  The
// rows of the full rounds run as one launch; the tail rows as a second launch on 4-wave 128 x 128 tiles (two
// workgroups per CU), which spreads the tail's work over 4x as many workgroups.  Off in deterministic mode (the
// statistics slot of a tile must stay one per M tile).  Returns 1 if it launched, 0 if not applicable.
template <int BM, int BN, int MODE, bool STATS, int STAGES, int NW>
int launch_fd_tail_split(ConvArgs& a, hipStream_t st, int* rc) {
  if constexpr (NW == 8 && BM == 256 && (MODE == 0 || MODE == 1)) {
    if (!conv_tail_mode() || a.m_base != 0 || mdtf_get_deterministic()) return 0;
    const long long mtiles = ceil_div(a.M, BM), ntiles = ceil_div(a.Ncol, BN);
    const long long cus = num_cus(), total = mtiles * ntiles;
    const long long rounds = total / cus, rem = total - rounds * cus;
    // MDTF_CONV_TAIL=1: tails under a quarter of a wave; 2: any partial last wave
    if (rounds < 1 || rem == 0 || (conv_tail_mode() == 1 && rem * 4 > cus) || (rounds * cus) % ntiles) return 0;
    const long long m1 = rounds * cus / ntiles * BM;        // rows of the full rounds
    if (m1 >= a.M) return 0;
    const long long M = a.M;
    ConvArgs tail = a;
    tail.m_base = m1;
    a.M = m1;
    *rc = launch_fd_v2<BM, BN, MODE, STATS, STAGES, NW>(a, st);
    a.M = M;
    if (*rc == 0) *rc = launch_fd_v2<128, 128, MODE, STATS, 2, 4>(tail, st);
    a.mtiles = static_cast<int>(mtiles);
    a.ntiles = static_cast<int>(ntiles);
    return 1;
  } else {
    (void)a;
    (void)st;
    (void)rc;
    return 0;
  }
}

template <int BM, int BN, int MODE, bool STATS, int STAGES, int NW>
int launch_fd_v2(ConvArgs& a, hipStream_t st) {
  constexpr int NT = 64 * NW;
  {
    int rc = 0;
    if (launch_fd_tail_split<BM, BN, MODE, STATS, STAGES, NW>(a, st, &rc)) return rc;
  }
  a.mtiles = static_cast<int>(ceil_div(a.M - a.m_base, BM));
  a.ntiles = static_cast<int>(ceil_div(a.Ncol, BN));
  const long long nblk = (long long)a.mtiles * a.ntiles;
  if (nblk > 0x7fffffff) return MDTF_EUNSUPPORTED;
  const size_t stage_bytes = STAGES >= 10 ? ((size_t)(STAGES / 10) * BM + (size_t)(STAGES % 10) * BN) * 128
                                          : STAGES * (size_t)(BM + BN) * 128;
  const size_t ctile = (size_t)BM * (BN * 2 + 16);
  size_t lds = stage_bytes > ctile ? stage_bytes : ctile;
  if (lds < (size_t)(NT + 8) * 16 * sizeof(float)) lds = (size_t)(NT + 8) * 16 * sizeof(float);   // BN-stat reduction
  if (STAGES == 1 && a.K > 64) return MDTF_EINVAL;      // single buffer: one K step only
  if (lds > 160 * 1024) return MDTF_EUNSUPPORTED;
  if (a.M >= (1LL << 31)) return MDTF_EUNSUPPORTED;
  {
    constexpr int AM = MODE == 3 ? 0 : MODE == 4 ? 1 : MODE;       // as in the kernel
    const int RH = AM == 0 ? a.OH : AM == 1 ? a.H : a.cls_Hc;
    const int RW = AM == 0 ? a.OW : AM == 1 ? a.W : a.cls_Wc;
    if (RH < 1 || RW < 1) return MDTF_EINVAL;
    magic31(static_cast<unsigned>(RW), &a.mg_rw, &a.sh_rw);
    magic31(static_cast<unsigned>(RH), &a.mg_rh, &a.sh_rh);
  }
  if (MODE <= 2 && STAGES >= 2 && conv_persist_mode() && a.K >= 64) {
    const int rc = launch_fd_p<BM, BN, MODE, STATS, STAGES, NW>(a, st);
    if (rc != MDTF_EUNSUPPORTED) return rc;
  }
  {
    // measured -0.65 % in the ResNet-50 step (13080 -> 12992 img/s, profiles/ab_r6.md) despite the conflict-free
    // reads: off unless MDTF_FD_COREMAP=1
    static const int remap = [] {
      const char* e = getenv("MDTF_FD_COREMAP");
      return (e && e[0] == '1') ? 1 : 0;
    }();
    a.co_remap = remap;
  }
  hipLaunchKernelGGL((conv_fd_v2<BM, BN, MODE, STATS, STAGES, NW>), dim3((unsigned)nblk), dim3(NT), lds, st, a);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// tile code: bm, bn and the pipeline depth (stages 2..4)
template <int MODE, bool STATS, int STAGES>
int dispatch_fd_v2s(ConvArgs& a, int bm, int bn, hipStream_t st) {
  if (bm == 128 && bn == 128) return launch_fd_v2<128, 128, MODE, STATS, STAGES>(a, st);
  if (bm == 128 && bn == 64) return launch_fd_v2<128, 64, MODE, STATS, STAGES>(a, st);
  if (bm == 256 && bn == 128) return launch_fd_v2<256, 128, MODE, STATS, STAGES>(a, st);
  if (bm == 256 && bn == 64) return launch_fd_v2<256, 64, MODE, STATS, STAGES>(a, st);
  if (bm == 64 && bn == 128) return launch_fd_v2<64, 128, MODE, STATS, STAGES>(a, st);
  if (bm == 64 && bn == 64) return launch_fd_v2<64, 64, MODE, STATS, STAGES>(a, st);
  return MDTF_EUNSUPPORTED;
}

// 8-wave tiles (bm code >= 10000): 256 x {256, 128, 64} and 128 x 256, LDS ring <= 160 KiB
template <int MODE, bool STATS>
int dispatch_fd_v2w8(ConvArgs& a, int bm, int bn, int stages, hipStream_t st) {
#define FD8(BM_, BN_, S_) \
  if (bm == BM_ && bn == BN_ && stages == S_) return launch_fd_v2<BM_, BN_, MODE, STATS, S_, 8>(a, st);
  FD8(256, 256, 1) FD8(256, 256, 2) FD8(256, 128, 1) FD8(256, 128, 2) FD8(256, 128, 3) FD8(256, 64, 2)
  FD8(256, 64, 3) FD8(256, 64, 4) FD8(128, 256, 2) FD8(128, 256, 3)
  // split rings (stages = 10 SA + SB): more A stages in flight in the same LDS
  FD8(256, 256, 32) FD8(256, 128, 32) FD8(256, 128, 42) FD8(128, 256, 32) FD8(128, 256, 42)
  // 448 = 7 x 64 rows: at batch 256 every row count is 49 * 4^k * 256, so 256-row tiles leave 196 * 4^k * (N / BN)
  // tiles = 0.77 of a 256-CU wave; 448-row tiles give 112 * 4^k * (N / 128) = 0.875 of one (4 x 2 waves of 112 x 64)
  // (not the dense act-backward mode: its 14 pre-activation vectors per thread spill)
  if constexpr (MODE != 4) {
    FD8(448, 128, 1) FD8(448, 128, 2)
  }
#undef FD8
  return MDTF_EUNSUPPORTED;
}

template <int MODE, bool STATS>
int dispatch_fd_v2(ConvArgs& a, int bm, int bn, int stages, hipStream_t st) {
  if (bm >= 10000) return dispatch_fd_v2w8<MODE, STATS>(a, bm % 10000, bn, stages, st);
  if (stages == 32) {                      // 4-wave split rings
    if (bm == 128 && bn == 128) return launch_fd_v2<128, 128, MODE, STATS, 32>(a, st);
    if (bm == 64 && bn == 128) return launch_fd_v2<64, 128, MODE, STATS, 32>(a, st);
    return MDTF_EUNSUPPORTED;
  }
  if (stages == 42) {
    if (bm == 64 && bn == 128) return launch_fd_v2<64, 128, MODE, STATS, 42>(a, st);
    return MDTF_EUNSUPPORTED;
  }
  if (stages == 1) return dispatch_fd_v2s<MODE, STATS, 1>(a, bm, bn, st);
  if (stages == 2) return dispatch_fd_v2s<MODE, STATS, 2>(a, bm, bn, st);
  if (stages == 3) return dispatch_fd_v2s<MODE, STATS, 3>(a, bm, bn, st);
  if (stages == 4) return dispatch_fd_v2s<MODE, STATS, 4>(a, bm, bn, st);
  return MDTF_EUNSUPPORTED;
}

// ============================================================================
// v2 wgrad (Cin % 64 == 0, Cout % 64 == 0): DW[r=(kh,kw,ci)][co] += sum_m X[m; r] DY[m][co]
// K = output pixels in steps of 64.  Both operands are k-strided (row = pixel),
// so the LDS images are [64 pixel rows][64 channels] half-tiles filled by
// LDS-DMA, and fragments are read with ds_read_b64_tr_b16 (CDNA4 transposed
// read, 4 pixels x 16 channels per 16-lane group).  Chunk swizzle for the tr
// reads: 16-B chunk c of row k lives at c ^ 2 f(k), f(k) = ((k>>1)&1) | ((k>>3)&1)<<1,
// which puts the 8 rows a 32-lane half reads at 8 distinct 32-B bank slots.
// Each lane walks two pixel rows (k and k + 32 of every step) incrementally; the
// split-K partial tiles accumulate into DW with fp32 atomics (16 consecutive
// co per 16-lane group).
// ============================================================================

// register budget: as many waves per SIMD as the LDS ring lets blocks be resident
template <int BM, int BN, int STAGES, int NW>
constexpr int wgrad_min_waves() {
  constexpr int blocks = (160 * 1024) / (STAGES * (BM + BN) * 128);
  constexpr int w = blocks * NW / 4;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

template <int BM, int BN, int STAGES, int NW, bool PIPE>
__global__ void __launch_bounds__(64 * NW, (wgrad_min_waves<BM, BN, STAGES, NW>()))
    conv_wgrad_v2(ConvArgs a) {
  // NW = 4 (2x2 waves) or 8 (one 256-row/col block per CU, 4x2 or 2x4 waves by aspect)
  constexpr int WM = NW == 4 ? 2 : (BM > BN ? 4 : 2), WN = NW / WM;
  constexpr int U = 8 / NW;                       // 8-row DMA blocks per wave per 64-pixel step
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int HA = BM / 64, HB = BN / 64;       // 64-column half-images per operand
  constexpr int IA = HA * U, IB = HB * U;         // DMA instructions per wave per stage
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int PER_STAGE = IA + IB;
  constexpr unsigned OOB = 0x80000000u;
  static_assert(HA >= 1 && HB >= 1, "tile too small");
  static_assert(STAGES >= 2 && (STAGES - 2) * PER_STAGE < 64, "pipeline depth");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_mn = a.mtiles * a.ntiles;
  // the finalize's workgroups last (default) or first (MDTF_BN_WG_FIN_FIRST=1: dispatched with the first round;
  // measured neutral), the GEMM's in the rest
  const int nwg = static_cast<int>(gridDim.x) - a.fin_blocks;
  const int fb = a.fin_first ? static_cast<int>(blockIdx.x) : static_cast<int>(blockIdx.x) - nwg;
  if (fb >= 0 && fb < a.fin_blocks) {
    fin_bwd_block(const_cast<float*>(a.fin_psum), const_cast<float*>(a.fin_psq), a.fin_P, a.fin_C, a.fin_M,
                  a.fin_gamma, a.fin_mean, a.fin_invstd, a.fin_ws, fb, smem_raw);
    return;
  }
  const int gb = a.fin_first ? static_cast<int>(blockIdx.x) - a.fin_blocks : static_cast<int>(blockIdx.x);
  // consecutive blocks run on different XCDs (round robin); with wg_xcd the tiles of one pixel split
  // (which read the same DY rows / X pixels) are consecutive in the remapped order, i.e. on one XCD's L2
  const int lb = a.wg_xcd ? xcd_remap(gb, nwg) : gb;
  const int tile = lb % tiles_mn;
  const int split = lb / tiles_mn;
  const int mt = tile / a.ntiles, nt = tile % a.ntiles;
  const int r0 = mt * BM, n0 = nt * BN;
  const int R = a.KH * a.KW * a.Cin;
  const long long Mpix = a.M;
  const int KT_total = static_cast<int>((Mpix + 63) / 64);
  const int kt_begin = split * a.ksplit_steps;
  const int kt_end = min(KT_total, kt_begin + a.ksplit_steps);
  if (kt_begin >= kt_end) return;

  const int bytes_x = (int)((long long)a.N * a.H * a.W * a.Cin * 2);
  const int bytes_dy = (int)((Mpix - 1) * a.ld_dy * 2 + a.Cout * 2);
  const i32x4_t rsrc_x = buffer_rsrc(a.src, bytes_x), rsrc_dy = buffer_rsrc(a.dy, bytes_dy);

  // A half h: rows r0 + 64h .. +63 lie in one tap (Cin % 64 == 0)
  int h_dy[HA], h_dx[HA], h_c[HA];
  bool h_ok[HA];
#pragma unroll
  for (int h = 0; h < HA; ++h) {
    const int r = r0 + 64 * h;
    h_ok[h] = r < R;
    const int rr = h_ok[h] ? r : 0;
    const int t = rr / a.Cin;
    h_c[h] = rr - t * a.Cin;
    const int kh = t / a.KW, kw = t - kh * a.KW;
    h_dy[h] = kh * a.DH - a.PH;
    h_dx[h] = kw * a.DW - a.PW;
  }
  // this lane's U pixel rows per step: k = 8*wave + (lane>>3) (+ 8*NW*u)
  const int krow0 = 8 * wave + (lane >> 3);
  int gch[U];
#pragma unroll
  for (int u = 0; u < U; ++u) gch[u] = ((lane & 7) ^ trswz(krow0 + 8 * NW * u)) * 8;
  int p_ow[U], p_oh[U], p_n[U];
  long long p_m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long m = (long long)kt_begin * 64 + krow0 + 8 * NW * u;
    p_m[u] = m;
    p_ow[u] = static_cast<int>(m % a.OW);
    const long long t = m / a.OW;
    p_oh[u] = static_cast<int>(t % a.OH);
    p_n[u] = static_cast<int>(t / a.OH);
  }
  const int d_ow = 64 % a.OW, d_oh = (64 / a.OW) % a.OH, d_n = 64 / (a.OW * a.OH);

  auto stage = [&](int buf) {
    char* lds = smem_raw + buf * STAGE;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool mok = p_m[u] < Mpix;
      const int iy0 = p_oh[u] * a.SH, ix0 = p_ow[u] * a.SW;
      // A halves: X[n, iy, ix, c + chunk]
#pragma unroll
      for (int h = 0; h < HA; ++h) {
        const int iy = iy0 + h_dy[h], ix = ix0 + h_dx[h];
        const bool ok = mok && h_ok[h] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const unsigned voff =
            ok ? (unsigned)((((p_n[u] * a.H + iy) * a.W + ix) * a.Cin + h_c[h] + gch[u]) * 2) : OOB;
        // instruction slot: half h, row block (wave + NW u) -> LDS rows 8*(wave+NW u) ..
        if constexpr (PIPE)
          dma16_asm(rsrc_x, lds + h * 8192 + (wave + NW * u) * 1024, voff);
        else
          dma16(a.src, bytes_x, lds + h * 8192 + (wave + NW * u) * 1024, voff, 0);
      }
      // B halves: DY[m, n0 + 64h + chunk]
      char* ldsb = lds + BM * 128;
#pragma unroll
      for (int h = 0; h < HB; ++h) {
        const int co = n0 + 64 * h;
        const unsigned voff = (mok && co < a.Cout) ? (unsigned)((p_m[u] * a.ld_dy + co + gch[u]) * 2) : OOB;
        if constexpr (PIPE)
          dma16_asm(rsrc_dy, ldsb + h * 8192 + (wave + NW * u) * 1024, voff);
        else
          dma16(a.dy, bytes_dy, ldsb + h * 8192 + (wave + NW * u) * 1024, voff, 0);
      }
      // advance this row by 64 pixels
      p_m[u] += 64;
      p_ow[u] += d_ow;
      int c1 = p_ow[u] >= a.OW;
      p_ow[u] -= c1 ? a.OW : 0;
      p_oh[u] += d_oh + c1;
      int c2 = p_oh[u] >= a.OH;
      p_oh[u] -= c2 ? a.OH : 0;
      p_n[u] += d_n + c2;
    }
  };

  float4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient: C = ones(16x32) x B-fragment puts each column's sum in every row
  constexpr bool CAN_BIAS = NW == 4;          // the 8-wave tiles have no registers to spare
  const bool do_bias = CAN_BIAS && a.dbias != nullptr && mt == 0 && wm == 0;
  float4v accb[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) accb[j] = float4v{0.f, 0.f, 0.f, 0.f};
  const bf16x8_t ones = __builtin_bit_cast(
      bf16x8_t, short8{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80});
  auto bias_mfma = [&](const bf16x8_t (&fb)[TN]) {
    if constexpr (CAN_BIAS) {
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < TN; ++j) accb[j] = mfma(ones, fb[j], accb[j]);
      }
    }
  };

  const int KT = kt_end - kt_begin;
  if constexpr (PIPE) {
    // Software-pipelined variant: the k-step is split in halves.  The second half's fragments
    // are read while the first half's MFMAs run, and the next step's first-half fragments
    // while the second half's MFMAs run, so LDS reads hide under MFMAs.  The DMA for step
    // kt + STAGES goes out right after the mid-step barrier that frees its buffer: every
    // buffer is in flight from the prologue on, and each lands one step ahead of its use.
    // The DMAs are inline asm (dma16_asm), so the compiler adds no vmcnt(0) before LDS reads;
    // the counted waits below and the barriers order them.
    bf16x8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
    auto read_half = [&](bf16x8_t (&fa)[TM], bf16x8_t (&fb)[TN], int buf, int kh2) {
      const char* As = smem_raw + buf * STAGE;
      const char* Bs = As + BM * 128;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (TM * 16) + i * 16;
        fa[i] = frag_tr(As + (col >> 6) * 8192, col & 63, 32 * kh2, lane);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (TN * 16) + j * 16;
        fb[j] = frag_tr(Bs + (col >> 6) * 8192, col & 63, 32 * kh2, lane);
      }
    };
    // wait until at most n stages (newest first) are still in flight
    auto wait_stages = [&](int n) {
      if (n <= 0)
        wait_vmcnt<0>();
      else if (n == 1)
        wait_vmcnt<PER_STAGE>();
      else if (n == 2)
        wait_vmcnt<2 * PER_STAGE>();
      else if (n == 3 || 4 * PER_STAGE > 63)
        wait_vmcnt<3 * PER_STAGE>();
      else
        wait_vmcnt<(4 * PER_STAGE > 63 ? 3 : 4) * PER_STAGE>();
    };
    // interleave this half's fragment reads with the other half's MFMAs (both in one block)
    constexpr int NRD = 2 * (TM + TN), NMF = TM * TN, NIL = NRD < NMF ? NRD : NMF;
    auto interleave = [&]() {
#pragma unroll
      for (int q = 0; q < NIL; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one LDS read
      }
      if constexpr (NRD > NIL) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NIL, 0);
      if constexpr (NMF > NIL) __builtin_amdgcn_sched_group_barrier(0x008, NMF - NIL, 0);
    };
    const int pro = KT < STAGES ? KT : STAGES;
    for (int s = 0; s < pro; ++s) stage(s);
    wait_stages(pro - 1);
    asm volatile("s_barrier" ::: "memory");
    read_half(fa0, fb0, 0, 0);
    int cur = 0;
    for (int kt = 0; kt < KT; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      read_half(fa1, fb1, cur, 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fa0[i], fb0[j], acc[i][j]);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      bias_mfma(fb0);
      const int nxt = cur + 1 == STAGES ? 0 : cur + 1;
      if (kt + 1 < KT) {
        // issued so far: steps 0 .. min(KT-1, kt-1+STAGES); wait for step kt+1
        const int newer = (KT - 2 - kt) < (STAGES - 2) ? (KT - 2 - kt) : (STAGES - 2);
        wait_stages(newer);
      }
      // this wave's second-half reads are complete, so after the barrier no wave reads `cur`
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (kt + STAGES < KT) stage(cur);
      __builtin_amdgcn_sched_barrier(0);
      // the next step's first-half fragments (a harmless stale read after the last step)
      read_half(fa0, fb0, nxt, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fa1[i], fb1[j], acc[i][j]);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      bias_mfma(fb1);
      cur = nxt;
    }
    __builtin_amdgcn_sched_barrier(0);
  } else {
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < KT) stage(s);
  int cur = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + STAGES - 2 < KT)
      wait_vmcnt<(STAGES - 2) * PER_STAGE>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    const char* As = smem_raw + cur * STAGE;
    const char* Bs = As + BM * 128;
    cur = cur + 1 == STAGES ? 0 : cur + 1;
    // all of this step's transposed reads are issued BEFORE the next stage's LDS-DMA: the
    // compiler makes an LDS read that follows an LDS-DMA wait for it (vmcnt(0)), which would
    // serialise the DMA with this step's MFMAs
    bf16x8_t fa[2][TM], fb[2][TN];
#pragma unroll
    for (int kh2 = 0; kh2 < 2; ++kh2) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (TM * 16) + i * 16;           // column within the BM tile
        fa[kh2][i] = frag_tr(As + (col >> 6) * 8192, col & 63, 32 * kh2, lane);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (TN * 16) + j * 16;
        fb[kh2][j] = frag_tr(Bs + (col >> 6) * 8192, col & 63, 32 * kh2, lane);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const int nk = kt + STAGES - 1;                      // its buffer was last read in step kt-1
      if (nk < KT) stage(nk % STAGES);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kh2 = 0; kh2 < 2; ++kh2)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma(fa[kh2][i], fb[kh2][j], acc[i][j]);
    bias_mfma(fb[0]);
    bias_mfma(fb[1]);
  }
  }
  const int g = lane >> 4, li = lane & 15;
  if (CAN_BIAS && do_bias && g == 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = n0 + wn * (TN * 16) + j * 16 + li;
      if (co < a.Cout) atomicAdd(a.dbias + co, accb[j][0]);
    }
  }
  if (a.slab && a.cnt) {
    // In-kernel split-K reduction.  Each split stores its partial tile write-through (16-B sc1 buffer stores,
    // aux 16) into the tile's slab region, drains its stores, and takes one ticket per workgroup after the
    // barrier; the workgroup whose add comes last (told by the returned value) sums every split in split order
    // with sc1 loads (deterministic whatever the arrival order) and adds the sum into DW once -- no reduction
    // launch, no agent fences (MI355X_MICROARCH.md: publish-large, Valid forms row 1; gemm_wg.hip, +2 % BERT).
    constexpr int NT = 64 * NW;
    const int nsp = nwg / tiles_mn;                          // every split is non-empty (launch_wgrad_v2)
    float* tslab = a.slab + (long long)tile * nsp * (BM * BN);
    const __amdgpu_buffer_rsrc_t srs =
        __builtin_amdgcn_make_buffer_rsrc(tslab, (short)0, nsp * (BM * BN) * 4, 0x00020000);
    const int sb = split * (TM * TN);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, acc[i][j]), srs,
                                               ((sb + i * TN + j) * NT + tid) * 16, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem_raw);
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == nsp - 1;
      if (last) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    float4v sum[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) sum[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < nsp; ++s) {              // workgroup-uniform: all TM * TN loads of a split in flight
      if (s == split) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) sum[i][j] += acc[i][j];
      } else {
        float4v p[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            p[i][j] = __builtin_bit_cast(
                float4v, __builtin_amdgcn_raw_buffer_load_b128(srs, ((s * (TM * TN) + i * TN + j) * NT + tid) * 16,
                                                               0, 16));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) sum[i][j] += p[i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = n0 + wn * (TN * 16) + j * 16 + li;
        if (co >= a.Cout) continue;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = r0 + wm * (TM * 16) + i * 16 + 4 * g + rr;
          if (r < R) a.dw[(long long)r * a.ld_dw + co] += sum[i][j][rr];
        }
      }
    return;
  }
  float* slab = a.slab ? a.slab + (long long)split * R * a.Cout : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = n0 + wn * (TN * 16) + j * 16 + li;
      if (co >= a.Cout) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = r0 + wm * (TM * 16) + i * 16 + 4 * g + rr;
        if (r >= R) continue;
        if (slab)
          if (a.slab_nt)
            __builtin_nontemporal_store(acc[i][j][rr], slab + (long long)r * a.Cout + co);
          else
            slab[(long long)r * a.Cout + co] = acc[i][j][rr];
        else
          atomicAdd(a.dw + (long long)r * a.ld_dw + co, acc[i][j][rr]);
      }
    }
}

// DW[r][c] (row stride ld) += sum_s slab[s][r][c]  (slab rows dense, C % 4 == 0); 4 splits in flight.
// (Spreading the splits of a small filter over more blocks with fp32 atomics measured 1.7 % slower in the ResNet
// step: profiles/ab_r5.md.)
// Split-parallel form for small filters with many splits (e.g. 64 x 256 over 128 splits: 16 blocks of the plain
// form, each thread 128 dependent-ish loads): G thread groups of 256 / G per block, group g sums splits g, g + G, ..
// of the block's 256 / G float4 outputs, then the G partials are added in LDS (fixed order: deterministic).
template <bool NT, int G>
__global__ void __launch_bounds__(256) wgrad_slab_reduce_g(const float* __restrict__ slab, int splits,
                                                           long long RC, int C, long long ld, float* __restrict__ dw,
                                                           int store) {
  constexpr int W = 256 / G;                                // float4 outputs per block
  __shared__ float4 part[G][W];
  const int g = threadIdx.x / W, l = threadIdx.x - g * W;
  const long long q = (long long)blockIdx.x * W + l;       // float4 index
  const long long st = RC / 4;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const float4* s4 = reinterpret_cast<const float4*>(slab);
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q < st) {
    int sp = g;
    for (; sp + 3 * G < splits; sp += 4 * G) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long i = q + (long long)(sp + u * G) * st;
        if constexpr (NT)
          v[u] = __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f4v*>(s4) + i));
        else
          v[u] = s4[i];
      }
      t.x += (v[0].x + v[1].x) + (v[2].x + v[3].x);
      t.y += (v[0].y + v[1].y) + (v[2].y + v[3].y);
      t.z += (v[0].z + v[1].z) + (v[2].z + v[3].z);
      t.w += (v[0].w + v[1].w) + (v[2].w + v[3].w);
    }
    for (; sp < splits; sp += G) {
      const float4 a = s4[q + (long long)sp * st];
      t.x += a.x;
      t.y += a.y;
      t.z += a.z;
      t.w += a.w;
    }
  }
  part[g][l] = t;
  __syncthreads();
  if (g != 0 || q >= st) return;
#pragma unroll
  for (int h = 1; h < G; ++h) {
    const float4 a = part[h][l];
    t.x += a.x;
    t.y += a.y;
    t.z += a.z;
    t.w += a.w;
  }
  const long long e = q * 4, r = e / C, c = e - r * C;
  float4* o = reinterpret_cast<float4*>(dw + r * ld + c);
  if (store) {                 // the step's first writer of the gradient slot: DW is not read
    *o = t;
    return;
  }
  float4 v = *o;
  v.x += t.x;
  v.y += t.y;
  v.z += t.z;
  v.w += t.w;
  *o = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) wgrad_slab_reduce(const float* __restrict__ slab, int splits, long long RC,
                                                         int C, long long ld, float* __restrict__ dw, int store) {
  const long long q = blockIdx.x * 256LL + threadIdx.x;     // float4 index
  if (q * 4 >= RC) return;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const float4* s4 = reinterpret_cast<const float4*>(slab);
  auto ldq = [&](long long i) -> float4 {
    if constexpr (NT) return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f4v*>(s4) + i));
    return s4[i];
  };
  const long long st = RC / 4;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  int sp = 0;
  for (; sp + 3 < splits; sp += 4) {
    const float4 a = ldq(q + sp * st), b = ldq(q + (sp + 1) * st), c = ldq(q + (sp + 2) * st), d = ldq(q + (sp + 3) * st);
    t.x += (a.x + b.x) + (c.x + d.x);
    t.y += (a.y + b.y) + (c.y + d.y);
    t.z += (a.z + b.z) + (c.z + d.z);
    t.w += (a.w + b.w) + (c.w + d.w);
  }
  for (; sp < splits; ++sp) {
    const float4 a = ldq(q + sp * st);
    t.x += a.x;
    t.y += a.y;
    t.z += a.z;
    t.w += a.w;
  }
  const long long e = q * 4, r = e / C, c = e - r * C;
  float4* o = reinterpret_cast<float4*>(dw + r * ld + c);
  if (store) {
    *o = t;
    return;
  }
  float4 v = *o;
  v.x += t.x;
  v.y += t.y;
  v.z += t.z;
  v.w += t.w;
  *o = v;
}

// Slab reduction on a side stream (mdtf_set_slab_stream): the reduction only feeds the gradient buffer, so it can
// leave the dgrad -> BN-backward chain.  The side stream waits for the weight-gradient kernel through one event
// (captured hipGraphs turn it into a fork edge); the caller joins the side stream before the gradients are read.
hipStream_t g_slab_stream = nullptr;
// Per-tile ticket buffer (zeroed ints, n of them) for in-kernel split-K reductions of the following weight-gradient
// launches (mdtf_set_wgrad_tickets); null: slab + reduction launch.
int* g_wg_cnt = nullptr;
long long g_wg_cnt_n = 0;
// The following weight-gradient launch overwrites DW instead of accumulating (mdtf_set_wgrad_store: the step's
// first writer of that gradient slot, ops.conv / train.variables claim_store): the slab reduction stores its sum;
// without one (fp32 atomics, in-kernel split reduction) DW is zeroed before the kernel.
int g_wg_store = 0;
// BN backward finalize job for the next weight-gradient launch (mdtf_set_wgrad_fin; C = 0: none)
struct FinReq {
  const float *psum, *psq, *gamma, *mean, *invstd;
  float* ws;
  int P, C;
  long long M;
};
FinReq g_wg_fin = {};
hipEvent_t slab_event() {
  static hipEvent_t ev = [] {
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    return e;
  }();
  return ev;
}

template <int BM, int BN, int STAGES, int NW = 4, bool PIPE = false>
int launch_wgrad_v2(ConvArgs& a, int splits, hipStream_t st) {
  const int R = a.KH * a.KW * a.Cin;
  a.mtiles = static_cast<int>(ceil_div(R, BM));
  a.ntiles = static_cast<int>(ceil_div(a.Cout, BN));
  const int kt_total = static_cast<int>(ceil_div(a.M, 64));
  if (splits < 1) {
    const int tiles = a.mtiles * a.ntiles;
    const int target = NW == 8 ? 512 : 1024;      // ~2 (8-wave) / ~4 (4-wave) blocks per CU
    splits = (target + tiles - 1) / tiles;
  }
  if (splits > kt_total) splits = kt_total;
  a.ksplit_steps = (kt_total + splits - 1) / splits;
  splits = (kt_total + a.ksplit_steps - 1) / a.ksplit_steps;
  const size_t lds = STAGES * (size_t)(BM + BN) * 128;
  if (lds > 160 * 1024) return MDTF_EUNSUPPORTED;
  ConvArgs b = a;
  if (a.slab && (splits < 2 || splits > a.slab_cap || (a.ld_dw % 4) || (a.Cout % 4))) b.slab = nullptr;
  // in-kernel reduction: the slab (>= splits * R * Cout floats, the caller pads to 256-multiples of R and Cout) holds
  // tiles * splits * BM * BN floats whenever BM, BN divide 256; tickets for every tile
  b.cnt = nullptr;
  if (b.slab && g_wg_cnt && g_wg_cnt_n >= (long long)a.mtiles * a.ntiles && 256 % BM == 0 && 256 % BN == 0 &&
      (long long)splits * BM * BN * a.mtiles * a.ntiles * 4 < (1ll << 31) &&
      (long long)a.mtiles * BM <= ceil_div(R, 256) * 256 && (long long)a.ntiles * BN <= ceil_div(a.Cout, 256) * 256)
    b.cnt = g_wg_cnt;
  {
    static const int nt = [] {
      const char* e = getenv("MDTF_SLAB_NT");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    b.slab_nt = nt;
  }
  const int store = g_wg_store;
  if (g_wg_fin.C > 0) {
    // finalize blocks beside the GEMM's (their reduction buffer: 2 x (threads / 32) x 32 doubles of the LDS)
    b.fin_blocks = static_cast<int>(ceil_div(g_wg_fin.C, 32));
    b.fin_psum = g_wg_fin.psum;
    b.fin_psq = g_wg_fin.psq;
    b.fin_P = g_wg_fin.P;
    b.fin_C = g_wg_fin.C;
    b.fin_M = g_wg_fin.M;
    b.fin_gamma = g_wg_fin.gamma;
    b.fin_mean = g_wg_fin.mean;
    b.fin_invstd = g_wg_fin.invstd;
    b.fin_ws = g_wg_fin.ws;
    static const int first = [] {      // measured neutral (r6w): 12973 vs 12972 img/s
      const char* e = getenv("MDTF_BN_WG_FIN_FIRST");
      return (e && e[0] == '1') ? 1 : 0;
    }();
    b.fin_first = first;
    g_wg_fin = FinReq{};
  } else {
    b.fin_blocks = 0;
    b.fin_first = 0;
  }
  if (store && !(b.slab && !b.cnt)) {     // accumulating epilogues: the slot must start at zero
    if (hipMemset2DAsync(a.dw, (size_t)a.ld_dw * 4, 0, (size_t)a.Cout * 4, (size_t)R, st) != hipSuccess)
      return MDTF_EUNSUPPORTED;
  }
  hipLaunchKernelGGL((conv_wgrad_v2<BM, BN, STAGES, NW, PIPE>), dim3(a.mtiles * a.ntiles * splits + b.fin_blocks),
                     dim3(64 * NW), lds, st, b);
  MDTF_LAUNCH_CHECK();
  if (b.slab && !b.cnt) {
    if (g_slab_stream && g_slab_stream != st) {
      hipEvent_t ev = slab_event();
      if (!ev || hipEventRecord(ev, st) != hipSuccess || hipStreamWaitEvent(g_slab_stream, ev, 0) != hipSuccess)
        return MDTF_EUNSUPPORTED;
      st = g_slab_stream;
    }
    const long long RC = (long long)R * a.Cout;
    // few outputs, many splits: spread the splits of each output over G thread groups (MDTF_SLAB_G=1: plain form)
    static const int gmax = [] {
      const char* e = getenv("MDTF_SLAB_G");
      return e ? atoi(e) : 16;
    }();
    const long long q4 = RC / 4;
    int G = 1;
    while (G < gmax && G < 16 && q4 * G < 256LL * 256 && splits >= 8 * G) G *= 4;
    if (G == 16)
      hipLaunchKernelGGL((b.slab_nt ? wgrad_slab_reduce_g<true, 16> : wgrad_slab_reduce_g<false, 16>),
                         dim3((unsigned)ceil_div(q4, 16)), dim3(256), 0, st, b.slab, splits, RC, a.Cout,
                         (long long)a.ld_dw, a.dw, store);
    else if (G == 4)
      hipLaunchKernelGGL((b.slab_nt ? wgrad_slab_reduce_g<true, 4> : wgrad_slab_reduce_g<false, 4>),
                         dim3((unsigned)ceil_div(q4, 64)), dim3(256), 0, st, b.slab, splits, RC, a.Cout,
                         (long long)a.ld_dw, a.dw, store);
    else
      hipLaunchKernelGGL((b.slab_nt ? wgrad_slab_reduce<true> : wgrad_slab_reduce<false>),
                         dim3((unsigned)ceil_div(RC / 4, 256)), dim3(256), 0, st, b.slab, splits, RC, a.Cout,
                         (long long)a.ld_dw, a.dw, store);
    MDTF_LAUNCH_CHECK();
  }
  return 0;
}

template <int BM, int BN, int MODE, bool STATS>
size_t fd_lds() {
  const size_t a = (size_t)BM * (BK + PADK);
  const size_t b = MODE == 0 ? (size_t)BK * (BN + PADN) : (size_t)BN * (BK + PADK);
  size_t bytes = 2 * (a + b) * sizeof(bf16_t);
  const size_t red = 2 * 2 * BN * sizeof(float);
  return bytes > red ? bytes : red;
}

template <int BM, int BN, int MODE, bool STATS>
int launch_fd(ConvArgs& a, hipStream_t st) {
  a.mtiles = static_cast<int>(ceil_div(a.M, BM));
  a.ntiles = static_cast<int>(ceil_div(a.Ncol, BN));
  const long long nblk = (long long)a.mtiles * a.ntiles;
  if (nblk > 0x7fffffff) return MDTF_EUNSUPPORTED;
  const size_t lds = fd_lds<BM, BN, MODE, STATS>();
  hipLaunchKernelGGL((conv_fd_kernel<BM, BN, MODE, STATS>), dim3((unsigned)nblk), dim3(NT), lds, st, a);
  MDTF_LAUNCH_CHECK();
  return 0;
}

template <int MODE, bool STATS>
int dispatch_fd(ConvArgs& a, int bm, int bn, hipStream_t st) {
  if (bm == 128 && bn == 128) return launch_fd<128, 128, MODE, STATS>(a, st);
  if (bm == 128 && bn == 64) return launch_fd<128, 64, MODE, STATS>(a, st);
  if (bm == 64 && bn == 64) return launch_fd<64, 64, MODE, STATS>(a, st);
  if (bm == 256 && bn == 64) return launch_fd<256, 64, MODE, STATS>(a, st);
  return MDTF_EUNSUPPORTED;
}

template <int BM, int BN>
int launch_wgrad(ConvArgs& a, int splits, hipStream_t st) {
  const int R = a.KH * a.KW * a.Cin;
  a.mtiles = static_cast<int>(ceil_div(R, BM));
  a.ntiles = static_cast<int>(ceil_div(a.Cout, BN));
  const int kt_total = static_cast<int>(ceil_div(a.M, BK));
  if (splits < 1) {
    const int tiles = a.mtiles * a.ntiles;
    splits = (1024 + tiles - 1) / tiles;
  }
  if (splits > kt_total) splits = kt_total;
  a.ksplit_steps = (kt_total + splits - 1) / splits;
  splits = (kt_total + a.ksplit_steps - 1) / a.ksplit_steps;
  const size_t lds = 2 * ((size_t)BK * (BM + PADN) + (size_t)BK * (BN + PADN)) * sizeof(bf16_t);
  hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN>), dim3(a.mtiles * a.ntiles * splits), dim3(NT), lds, st, a);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// v2 wgrad tile table; w8: 8-wave (512-thread) tiles
int dispatch_wgrad_v2(ConvArgs& a, int bm, int bn, int stages, int w8, int splits, hipStream_t st) {
  // MDTF_WGRAD_PIPE=0 selects the non-pipelined main loop (A/B switch)
  static const bool pipe = [] {
    const char* e = getenv("MDTF_WGRAD_PIPE");
    return !(e && e[0] == '0');
  }();
  // MDTF_WGRAD_XCD=0: blocks in launch order instead of the XCD-grouped order (A/B switch)
  static const int xcd = [] {
    const char* e = getenv("MDTF_WGRAD_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  a.wg_xcd = xcd;
#define WG2(BM_, BN_, S_, NW_) \
  if (bm == BM_ && bn == BN_ && stages == S_ && (NW_ == 8) == (w8 != 0)) \
    return pipe ? launch_wgrad_v2<BM_, BN_, S_, NW_, true>(a, splits, st) \
                : launch_wgrad_v2<BM_, BN_, S_, NW_, false>(a, splits, st);
  WG2(128, 128, 2, 4) WG2(128, 128, 3, 4) WG2(128, 64, 2, 4) WG2(128, 64, 3, 4) WG2(64, 128, 2, 4)
  WG2(64, 128, 3, 4) WG2(64, 64, 2, 4) WG2(64, 64, 3, 4) WG2(64, 64, 4, 4)
  WG2(256, 256, 2, 8) WG2(256, 128, 2, 8) WG2(256, 128, 3, 8) WG2(128, 256, 2, 8) WG2(128, 256, 3, 8)
  WG2(128, 128, 2, 8) WG2(128, 128, 3, 8) WG2(128, 128, 4, 8)
  // deeper rings (more LDS-DMA in flight per block): 4-5 stages of 128 x 128, 4-6 of 64 x 128
  WG2(128, 128, 5, 8) WG2(128, 128, 4, 4) WG2(128, 128, 5, 4) WG2(64, 128, 4, 4) WG2(64, 128, 6, 4)
  // skinny 8-wave tiles for 64-row / 64-column filters (the stage-1 1x1 convs, R or Cout = 64): a 128 x 128 tile
  // there leaves half its rows (columns) empty and reads the other operand twice; 64 x 256 / 256 x 64 read each once
  WG2(64, 256, 3, 8) WG2(64, 256, 4, 8) WG2(256, 64, 3, 8) WG2(256, 64, 4, 8)
#undef WG2
  return MDTF_EUNSUPPORTED;
}

// Strided dgrad, the stride-parity classes whose filter-tap set is empty (3 of the 4 classes of a 1x1 stride-2
// conv): DX there is 0 + the accumulate source, so these pixels are a streaming pass, not a GEMM.  One launch
// covers every such class.  Thread = one 16-B channel chunk of one DX pixel; with C8 = Cin / 8 dividing the block,
// a thread keeps one chunk for the whole grid-stride walk, so the BN-backward partials (Σ g·mask, Σ g·mask·x)
// stay in registers and are reduced once per block.  Pixels of classes with taps are skipped (their GEMM
// launch writes them).  out = acc ? (acc_src ? acc_src * acc_mask : out) : 0.
template <bool BSTAT>
__global__ void __launch_bounds__(256) dgrad_zero_classes(ConvArgs a, int C8) {
  const int tid = threadIdx.x;
  const int ppb = 256 / C8;                          // pixels per block iteration
  const int c8 = tid % C8, pl = tid / C8;
  // 32-bit pixel index math with the host's magic divisors (mg_rw: W, mg_rh: H; P < 2^31 host-checked): the
  // 64-bit p % W, (p / W) % H of every iteration were ~250 VALU instructions per 32-48 B moved
  const unsigned P = (unsigned)a.N * a.H * a.W;
  float s0[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s0[k] = s1[k] = 0.f;
  for (unsigned p = blockIdx.x * (unsigned)ppb + pl; p < P; p += gridDim.x * (unsigned)ppb) {
    const unsigned q = fdiv31(p, a.mg_rw, a.sh_rw);
    const int w = static_cast<int>(p - q * (unsigned)a.W);
    const int h = static_cast<int>(q - fdiv31(q, a.mg_rh, a.sh_rh) * (unsigned)a.H);
    const int rh = (h + a.PH) % a.SH, rw = (w + a.PW) % a.SW;
    if (rh < a.KH && rw < a.KW) continue;            // this class has taps: the GEMM launch owns it
    const long long off = (long long)p * a.Ncol + c8 * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (a.accumulate) {
      v = *reinterpret_cast<const uint4*>((a.acc_src ? a.acc_src : a.out) + off);
      if (a.acc_mask) v = mask_bf8(v, a.acc_mask[off >> 3]);
    }
    if (a.acc_src || !a.accumulate) *reinterpret_cast<uint4*>(a.out + off) = v;
    if constexpr (BSTAT) {
      const uint4 x4 = *reinterpret_cast<const uint4*>(a.bx + off);
      const uint32_t mb = a.bmask ? a.bmask[off >> 3] : 0xffu;
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, xw[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g = (k & 1) ? __uint_as_float(vw[k >> 1] & 0xffff0000u) : __uint_as_float(vw[k >> 1] << 16);
        const float xk = (k & 1) ? __uint_as_float(xw[k >> 1] & 0xffff0000u) : __uint_as_float(xw[k >> 1] << 16);
        const float gm = ((mb >> k) & 1u) ? g : 0.f;
        s0[k] += gm;
        s1[k] += gm * xk;
      }
    }
  }
  if constexpr (BSTAT) {
    // rows padded to 260 floats (4 mod 32 banks): a 32-lane half of the reads below takes channels k = 0..7 x
    // thread chunks cc = 0..3, at bank 4 k + cc -- 32 distinct.  (256: the 8 k of one cc shared a bank, 78 %
    // conflicts in pmc_resnet50_r4p; 257: bank k + cc, 11 banks for 32 lanes, 60 % in pmc_resnet50_r5f)
    __shared__ float red[2][8][260];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[0][k][tid] = s0[k];
      red[1][k][tid] = s1[k];
    }
    __syncthreads();
    const long long slot = (long long)(blockIdx.x % a.bslots) * a.Ncol;
    for (int ch = tid; ch < a.Ncol; ch += 256) {
      const int cc = ch >> 3, k = ch & 7;
      float sv = 0.f, q = 0.f;
      for (int t = cc; t < 256; t += C8) {
        sv += red[0][k][t];
        q += red[1][k][t];
      }
      atomicAdd(a.bsum + slot + ch, sv);
      atomicAdd(a.bsq + slot + ch, q);
    }
  }
}

// MDTF_ZERO_CLASS=gemm: the tap-less classes run the GEMM kernel with K = 0 as before (A/B switch)
bool zero_class_gemm() {
  static const bool g = [] {
    const char* e = getenv("MDTF_ZERO_CLASS");
    return e && e[0] == 'g';
  }();
  return g;
}

// v2 fwd / dgrad tile code -> (10000 if 8 waves) + rows, and the stage code (2 if unset).  Codes >= 100000 carry a
// two-digit stage code (split rings): 100000 (1 + w8) + 1000 stages + rows.
void decode_tile(int* bm, int* stages) {
  const int c = *bm;
  if (c >= 100000) {
    *stages = (c % 100000) / 1000;
    *bm = (c / 100000 - 1) * 10000 + c % 1000;
    return;
  }
  *stages = (c % 10000) / 1000 ? (c % 10000) / 1000 : 2;
  *bm = (c / 10000) * 10000 + c % 1000;
}

ConvArgs make_args(int N, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW, int SH, int SW, int PH,
                   int PW, int DH, int DW) {
  ConvArgs a{};
  a.N = N;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.OH = OH;
  a.OW = OW;
  a.Cout = Cout;
  a.KH = KH;
  a.KW = KW;
  a.SH = SH;
  a.SW = SW;
  a.PH = PH;
  a.PW = PW;
  a.DH = DH;
  a.DW = DW;
  return a;
}

}  // namespace

// Y = conv(X, W); optional per-M-tile BN partials (stat_sum/stat_sq [mtiles][Cout]).
// Returns the number of M tiles through *mtiles_out (for the BN finalize).
MDTF_EXPORT int mdtf_conv_fwd(const void* x, const void* w, void* y, float* stat_sum, float* stat_sq, int stat_slots,
                              int N, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW, int SH, int SW,
                              int PH, int PW, int DH, int DW, int bm, int bn, int* mtiles_out, hipStream_t st) {
  if (Cin % 8 || Cout % 8) return MDTF_EINVAL;
  ConvArgs a = make_args(N, H, W, Cin, OH, OW, Cout, KH, KW, SH, SW, PH, PW, DH, DW);
  a.src = (const bf16_t*)x;
  a.wgt = (const bf16_t*)w;
  a.out = (bf16_t*)y;
  a.stat_sum = stat_sum;
  a.stat_sq = stat_sq;
  a.stat_slots = stat_slots > 0 ? stat_slots : kStatSlots;
  a.M = (long long)N * OH * OW;
  a.Ncol = Cout;
  a.K = KH * KW * Cin;
  int rc = stat_sum ? dispatch_fd<0, true>(a, bm, bn, st) : dispatch_fd<0, false>(a, bm, bn, st);
  if (mtiles_out) *mtiles_out = a.mtiles;
  return rc;
}

// DX = dgrad(DY, W)   (DX [N,H,W,Cin], DY [N,OH,OW,Cout])
MDTF_EXPORT int mdtf_conv_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int Cin, int OH, int OW,
                                int Cout, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW, int bm, int bn,
                                hipStream_t st) {
  if (Cin % 8 || Cout % 8) return MDTF_EINVAL;
  ConvArgs a = make_args(N, H, W, Cin, OH, OW, Cout, KH, KW, SH, SW, PH, PW, DH, DW);
  a.src = (const bf16_t*)dy;
  a.wgt = (const bf16_t*)w;
  a.out = (bf16_t*)dx;
  a.M = (long long)N * H * W;
  a.Ncol = Cin;
  a.K = KH * KW * Cout;
  return dispatch_fd<1, false>(a, bm, bn, st);
}

// DW (fp32, HWIO, must be zeroed) += wgrad(X, DY)
MDTF_EXPORT int mdtf_conv_wgrad(const void* x, const void* dy, float* dw, int N, int H, int W, int Cin, int OH, int OW,
                                int Cout, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW, int bm, int bn,
                                int splits, hipStream_t st) {
  if (Cin % 8 || Cout % 8) return MDTF_EINVAL;
  ConvArgs a = make_args(N, H, W, Cin, OH, OW, Cout, KH, KW, SH, SW, PH, PW, DH, DW);
  a.src = (const bf16_t*)x;
  a.dy = (const bf16_t*)dy;
  a.dw = dw;
  a.M = (long long)N * OH * OW;
  a.Ncol = Cout;
  if (bm == 128 && bn == 128) return launch_wgrad<128, 128>(a, splits, st);
  if (bm == 64 && bn == 64) return launch_wgrad<64, 64>(a, splits, st);
  if (bm == 128 && bn == 64) return launch_wgrad<128, 64>(a, splits, st);
  if (bm == 64 && bn == 128) return launch_wgrad<64, 128>(a, splits, st);
  return MDTF_EUNSUPPORTED;
}

// v2 (C % 64 == 0): Y = conv(X, W) with the filter given transposed, Wt[co][(kh,kw,ci)]
MDTF_EXPORT int mdtf_conv_fwd_v2(const void* x, const void* wt, void* y, float* stat_sum, float* stat_sq,
                                 int stat_slots, int N, int H, int W, int Cin, int OH, int OW, int Cout, int KH, int KW,
                                 int SH, int SW, int PH, int PW, int DH, int DW, int bm, int bn, int* mtiles_out,
                                 hipStream_t st) {
  if (Cin % 64 || Cout % 8) return MDTF_EINVAL;
  if (KH * KW > 32 || (long long)N * H * W * Cin * 2 > 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  ConvArgs a = make_args(N, H, W, Cin, OH, OW, Cout, KH, KW, SH, SW, PH, PW, DH, DW);
  a.src = (const bf16_t*)x;
  a.wgt = (const bf16_t*)wt;
  a.out = (bf16_t*)y;
  a.stat_sum = stat_sum;
  a.stat_sq = stat_sq;
  a.stat_slots = stat_slots > 0 ? stat_slots : kStatSlots;
  a.M = (long long)N * OH * OW;
  a.Ncol = Cout;
  a.K = KH * KW * Cin;
  // bm = 10000 (8 waves) + stages * 1000 + tile rows, or (two-digit stages) 100000 (8 waves) + stages * 1000 + rows
  int stages;
  decode_tile(&bm, &stages);
  int rc = stat_sum ? dispatch_fd_v2<0, true>(a, bm, bn, stages, st) : dispatch_fd_v2<0, false>(a, bm, bn, stages, st);
  if (mtiles_out) *mtiles_out = a.mtiles;
  return rc;
}

// v2 (Cout % 64 == 0): DX = dgrad(DY, W), W in HWIO
MDTF_EXPORT int mdtf_conv_dgrad_v2(const void* dy, const void* w, void* dx, int N, int H, int W, int Cin, int OH,
                                   int OW, int Cout, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW,
                                   int bm, int bn, int accumulate, const void* bx, const void* bmask,
                                   float* bsum, float* bsq, int bslots, const void* acc_src, const void* acc_mask,
                                   hipStream_t st) {
  if (Cout % 64 || Cin % 8) return MDTF_EINVAL;
  if ((acc_src || acc_mask) && !accumulate) return MDTF_EINVAL;
  if ((long long)N * OH * OW * Cout * 2 > 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  if ((SH != 1 || SW != 1) && (DH != 1 || DW != 1)) return MDTF_EUNSUPPORTED;
  // <= 32 taps per K walk (per stride-parity class when strided)
  if (ceil_div(KH, SH) * ceil_div(KW, SW) > 32) return MDTF_EUNSUPPORTED;
  ConvArgs a = make_args(N, H, W, Cin, OH, OW, Cout, KH, KW, SH, SW, PH, PW, DH, DW);
  a.src = (const bf16_t*)dy;
  a.wgt = (const bf16_t*)w;
  a.out = (bf16_t*)dx;
  a.accumulate = accumulate;
  a.acc_src = (const bf16_t*)acc_src;       // null: out itself
  a.acc_mask = (const uint8_t*)acc_mask;
  a.bx = (const bf16_t*)bx;
  a.bmask = (const uint8_t*)bmask;
  a.bsum = bsum;
  a.bsq = bsq;
  a.bslots = bslots > 0 ? bslots : 1;
  a.Ncol = Cin;
  int stages;
  decode_tile(&bm, &stages);
  if (SH == 1 && SW == 1) {
    a.M = (long long)N * H * W;
    a.K = KH * KW * Cout;
    return dispatch_fd_v2<1, false>(a, bm, bn, stages, st);
  }
  // strided: one launch per stride-parity class (rh, rw) = ((h + PH) % SH, (w + PW) % SW); the classes without
  // taps go to one streaming launch (dgrad_zero_classes) when their pixels must be written or counted
  const int C8 = Cin / 8;
  const bool zero_stream = C8 <= 256 && 256 % C8 == 0 && !zero_class_gemm();
  bool zero_pending = false;
  for (int rh = 0; rh < SH; ++rh)
    for (int rw = 0; rw < SW; ++rw) {
      ConvArgs c = a;
      c.cls_h0 = ((rh - PH) % SH + SH) % SH;
      c.cls_w0 = ((rw - PW) % SW + SW) % SW;
      c.cls_Hc = c.cls_h0 < H ? (H - c.cls_h0 + SH - 1) / SH : 0;
      c.cls_Wc = c.cls_w0 < W ? (W - c.cls_w0 + SW - 1) / SW : 0;
      c.cls_kh0 = rh;
      c.cls_kw0 = rw;
      c.cls_th = rh < KH ? (KH - rh + SH - 1) / SH : 0;
      c.cls_tw = rw < KW ? (KW - rw + SW - 1) / SW : 0;
      c.cls_q0h = (c.cls_h0 + PH - rh) / SH;
      c.cls_q0w = (c.cls_w0 + PW - rw) / SW;
      c.M = (long long)N * c.cls_Hc * c.cls_Wc;
      c.K = c.cls_th * c.cls_tw * Cout;
      // no pixels / nothing to add (unless the BN statistics need every pixel)
      // (with a separate accumulate source the class's pixels must still be written)
      if (c.M == 0 || (c.K == 0 && accumulate && !bsum && !acc_src)) continue;
      if (c.K == 0 && zero_stream) {
        zero_pending = true;
        continue;
      }
      const int cs = c.K > 64 && stages == 1 ? 2 : stages;
      const int rc = dispatch_fd_v2<2, false>(c, bm, bn, cs, st);
      if (rc) return rc;
    }
  if (zero_pending) {
    if ((long long)N * H * W >= (1LL << 31)) return MDTF_EUNSUPPORTED;
    magic31(static_cast<unsigned>(W), &a.mg_rw, &a.sh_rw);
    magic31(static_cast<unsigned>(H), &a.mg_rh, &a.sh_rh);
    const long long chunks = (long long)N * H * W * C8;
    const int blocks = static_cast<int>(ceil_div(chunks, 256) < 4096 ? ceil_div(chunks, 256) : 4096);
    if (bsum)
      hipLaunchKernelGGL(dgrad_zero_classes<true>, dim3(blocks), dim3(256), 0, st, a, C8);
    else
      hipLaunchKernelGGL(dgrad_zero_classes<false>, dim3(blocks), dim3(256), 0, st, a, C8);
    MDTF_LAUNCH_CHECK();
  }
  return 0;
}

// The next v2 weight-gradient launch also runs the backward finalize of a BatchNorm (see fin_bwd_block): psum / psq
// [P][C] partial statistics (re-zeroed), gamma (or null), mean, invstd [C], M rows; ws [5][C] receives k1 | k2 | k3 |
// dgamma | dbeta.  The request is consumed by that launch.
MDTF_EXPORT int mdtf_set_wgrad_fin(const float* psum, const float* psq, int P, const float* gamma, const float* mean,
                                   const float* invstd, float* ws, long long M, int C) {
  if (C < 0 || (C > 0 && (!psum || !psq || !mean || !invstd || !ws || P <= 0 || M <= 0))) return MDTF_EINVAL;
  g_wg_fin = FinReq{psum, psq, gamma, mean, invstd, ws, P, C, M};
  return 0;
}

// The following v2 weight-gradient launches overwrite DW instead of accumulating into it (1) or accumulate (0).
MDTF_EXPORT int mdtf_set_wgrad_store(int on) {
  g_wg_store = on ? 1 : 0;
  return 0;
}

// Tickets for in-kernel split-K reductions of the following v2 weight-gradient launches (null / n = 0: off).
MDTF_EXPORT int mdtf_set_wgrad_tickets(int* cnt, long long n) {
  g_wg_cnt = cnt;
  g_wg_cnt_n = cnt ? n : 0;
  return 0;
}

// Side stream for the split-K slab reductions of the following weight-gradient launches (null: in line).
MDTF_EXPORT int mdtf_set_slab_stream(hipStream_t s) {
  g_slab_stream = s;
  return 0;
}

// v2 wgrad (Cin % 64 == 0, Cout % 64 == 0): DW (fp32, HWIO, zeroed or a grad slot) += wgrad(X, DY)
// bm encodes stages * 1000 + tile rows
MDTF_EXPORT int mdtf_conv_wgrad_v2(const void* x, const void* dy, float* dw, int N, int H, int W, int Cin, int OH,
                                   int OW, int Cout, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW,
                                   int bm, int bn, int splits, float* slab, int slab_cap, hipStream_t st) {
  if (Cin % 64 || Cout % 64) return MDTF_EINVAL;
  if ((long long)N * H * W * Cin * 2 > 0x7fffffffLL || (long long)N * OH * OW * Cout * 2 > 0x7fffffffLL)
    return MDTF_EUNSUPPORTED;
  ConvArgs a = make_args(N, H, W, Cin, OH, OW, Cout, KH, KW, SH, SW, PH, PW, DH, DW);
  a.src = (const bf16_t*)x;
  a.dy = (const bf16_t*)dy;
  a.dw = dw;
  a.ld_dy = a.ld_dw = Cout;
  a.M = (long long)N * OH * OW;
  a.Ncol = Cout;
  a.slab = slab;
  a.slab_cap = slab_cap;
  const int w8 = bm / 10000, stages = (bm % 10000) / 1000 ? (bm % 10000) / 1000 : 2;
  bm %= 1000;
  return dispatch_wgrad_v2(a, bm, bn, stages, w8, splits, st);
}

// dW[K][N] (fp32, row stride ld_dw) += X[M][K]^T DY[M][N] (DY row stride ld_dy): the dense-layer
// weight gradient on the v2 wgrad kernel (a 1x1 convolution over M "pixels").  K % 64 == 0, N % 64 == 0.
// dbias (optional, fp32 [N]): += column sums of dy (4-wave tiles only; else MDTF_EUNSUPPORTED)
MDTF_EXPORT int mdtf_gemm_wgrad(const void* x, const void* dy, float* dw, long long M, int K, int N, int ld_dy,
                                int ld_dw, int bm, int bn, int stages, int splits, float* slab, int slab_cap,
                                float* dbias, hipStream_t st) {
  if (dbias && bm >= 10000) return MDTF_EUNSUPPORTED;
  if (K % 64 || N % 64 || ld_dy % 8 || M > 0x7fffffff) return MDTF_EINVAL;
  if (M * K * 2 > 0x7fffffffLL || M * (long long)ld_dy * 2 > 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  ConvArgs a = make_args((int)M, 1, 1, K, 1, 1, N, 1, 1, 1, 1, 0, 0, 1, 1);
  a.src = (const bf16_t*)x;
  a.dy = (const bf16_t*)dy;
  a.dw = dw;
  a.ld_dy = ld_dy;
  a.ld_dw = ld_dw;
  a.M = M;
  a.Ncol = N;
  a.slab = slab;
  a.slab_cap = slab_cap;
  a.dbias = dbias;
  return dispatch_wgrad_v2(a, bm % 10000, bn, stages, bm / 10000, splits, st);
}

// Dense forward on the fd v2 kernel (MODE 3): Y[M][nseg * seg_cols] = act(X[M][K] [W_0 | .. | W_{nseg-1}] + bias),
// each W_s bf16 [K][seg_cols] (row-major, no transposed copy), bias bf16 [nseg * seg_cols] or null; with act != 0
// the pre-activation is also written to pre (null: not kept).  K % 64 == 0, seg_cols % bn == 0, nseg <= 4.
// bm encodes [10000 if 8 waves] + stages * 1000 + tile rows.
MDTF_EXPORT int mdtf_gemm_fwd(const void* x, const void* w0, const void* w1, const void* w2, const void* w3, int nseg,
                              int seg_cols, const void* bias, void* y, void* pre, int act, long long M, int K, int bm,
                              int bn, hipStream_t st) {
  if (nseg < 1 || nseg > 4 || K % 64 || bn <= 0 || seg_cols % bn || seg_cols % 64 || M <= 0 || act < 0 || act > 2)
    return MDTF_EINVAL;
  if (M > 0x7fffffff || M * K * 2 > 0x7fffffffLL || (long long)K * seg_cols * 2 > 0x7fffffffLL)
    return MDTF_EUNSUPPORTED;
  ConvArgs a = make_args((int)M, 1, 1, K, 1, 1, nseg * seg_cols, 1, 1, 1, 1, 0, 0, 1, 1);
  a.src = (const bf16_t*)x;
  const void* ws[4] = {w0, w1, w2, w3};
  for (int s = 0; s < 4; ++s) {
    if (s < nseg && !ws[s]) return MDTF_EINVAL;
    a.wseg[s] = (const bf16_t*)(s < nseg ? ws[s] : w0);
  }
  a.seg_cols = seg_cols;
  a.ld_b = seg_cols;
  a.bias = (const bf16_t*)bias;
  a.pre_out = (bf16_t*)pre;
  a.act = act;
  a.out = (bf16_t*)y;
  a.M = M;
  a.Ncol = nseg * seg_cols;
  a.K = K;
  const int w8 = bm / 10000, stages = (bm % 10000) / 1000 ? (bm % 10000) / 1000 : 2;
  bm = w8 * 10000 + bm % 1000;
  return dispatch_fd_v2<3, false>(a, bm, bn, stages, st);
}

// Dense data gradient with the producer's activation backward in the epilogue (fd v2 MODE 1 as a 1x1 "conv"):
// dx[M][K] = (dy[M][N] W[K][N]^T) * act'(pre[M][K]); act 1 relu (pre = the forward output), 2 gelu.
// N % 64 == 0, K % 8 == 0.  bm encodes [10000 if 8 waves] + stages * 1000 + tile rows.
MDTF_EXPORT int mdtf_gemm_dgrad_act(const void* dy, const void* w, void* dx, const void* pre, int act, long long M,
                                    int K, int N, int bm, int bn, hipStream_t st) {
  if (N % 64 || K % 8 || M <= 0 || !pre || act < 1 || act > 2) return MDTF_EINVAL;
  if (M > 0x7fffffff || M * N * 2 > 0x7fffffffLL || M * K * 2 > 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  ConvArgs a = make_args((int)M, 1, 1, K, 1, 1, N, 1, 1, 1, 1, 0, 0, 1, 1);
  a.src = (const bf16_t*)dy;
  a.wgt = (const bf16_t*)w;
  a.out = (bf16_t*)dx;
  a.pre_out = (bf16_t*)pre;
  a.act = act;
  a.Ncol = K;
  a.M = M;
  a.K = N;
  const int w8 = bm / 10000, stages = (bm % 10000) / 1000 ? (bm % 10000) / 1000 : 2;
  bm = w8 * 10000 + bm % 1000;
  return dispatch_fd_v2<4, false>(a, bm, bn, stages, st);
}
