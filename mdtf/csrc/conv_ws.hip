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
#include "mdtf_common.h"

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr unsigned kOOB = 0x80000000u;   // buffer offset past num_records -> the load returns zeros

struct WsArgs {
  const bf16_t* src;     // gathered operand [N][H][W][C]
  const bf16_t* wgt;     // filter (layout by wmode)
  bf16_t* out;           // [M][Ncol]
  int N, H, W, C;        // src dims; C % 32 == 0 (the reduction elements per filter tap)
  int cs;                // elements between neighbouring src pixels (C, or 4 for the packed stem input)
  int OH, OW, Ncol;      // output pixel grid, output channels (Ncol % (64*CG) == 0)
  int KH, KW, SH, SW, PH, PW, DH, DW;
  int Cw;                // wmode 1: channels of W's last axis (the conv's Cout == C); wmode 0: unused
  int wmode;
  int K;                 // KH*KW*C
  long long M;           // N*OH*OW output pixels
  int ptiles;            // ceil(M / (16*TP))
  int cblocks;           // Ncol / (64*CG)
  int pgroups;           // persistent pixel groups per channel block
  // forward BatchNorm statistics of out (fp32 accumulators): [sslots][Ncol] partial rows
  float* ssum;
  float* ssq;
  int sslots;
  // dgrad writing the complete gradient g of a BatchNorm output: sum g*mask, sum g*mask*x
  const bf16_t* bx;
  const uint8_t* bmask;
  float* bsum;
  float* bsq;
  int bslots;
  int accumulate;        // out += result (fan-out gradient)
  int direct;            // 1x1, stride 1, no padding, same grid: pixel p reads src row p
  unsigned mow, mohh;    // magic multipliers of the pixel decomposition p -> (n, oh, ow)
  int sow, sohh;         //   q = (umulhi(p, m) + p) >> s  (exact for p < 2^31)
  int dbg;               // probe only (bits): 1 = skip the output stores, 2 = skip the operand loads, 4 = skip MFMA
};

__device__ __forceinline__ float4v mfma(const bf16x8_t& a, const bf16x8_t& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// output channel (within the wave's 64) of MFMA row rr of channel subtile i: lane group g = rr>>2
// ends up holding channels 8g..8g+7 (subtiles 0,1) and 32+8g..32+8g+7 (subtiles 2,3)
__device__ __forceinline__ int chan_of(int i, int rr) { return (i >> 1) * 32 + 8 * (rr >> 2) + (i & 1) * 4 + (rr & 3); }

__device__ __forceinline__ void unpack8(const uint4& raw, float (&f)[8]) {
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pack_bf2(f[2 * i], f[2 * i + 1]);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Epilogue modes: 0 plain store, 1 + forward BN statistics, 2 accumulate (out += result),
// 3 + BN-backward statistics, 4 accumulate + BN-backward statistics.
template <int EPI>
struct Epi {
  static constexpr bool stats = EPI == 1;
  static constexpr bool acc = EPI == 2 || EPI == 4;
  static constexpr bool bstat = EPI == 3 || EPI == 4;
};

// TP: 16-pixel subtiles per wave tile; NW waves per block; CG 64-channel groups per block
// (waves w and w+CG.. share a channel group and stream different pixel tiles); D: depth of the
// B-fragment load ring in 32-deep k-steps (loads run D steps ahead, across tile boundaries).
// KSC: k-steps per tile as a compile-time constant (short reductions, D % KSC == 0), or 0: runtime
// KS with KS % D == 0.
template <int TP, int NW, int CG, int D, int KSC, int EPI>
__global__ void __launch_bounds__(64 * NW, 2) conv_ws_kernel(WsArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using E = Epi<EPI>;
  constexpr int PS = NW / CG;              // pixel streams per block
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int KS = KSC > 0 ? KSC : (a.K >> 5);   // 32-deep k-steps

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = bid % a.cblocks, pg = bid / a.cblocks;

  // ---- filter slice -> LDS, fragment order: frag f = (cg*KS + ks)*4 + i, 1 KiB each
  {
    const int nfrag = CG * KS * 4;
    for (int f = wave; f < nfrag; f += NW) {
      const int cg = f / (KS * 4), rem = f - cg * (KS * 4), ks = rem >> 2, i = rem & 3;
      const int n = (cb * CG + cg) * 64 + chan_of(i, li);
      const int k = ks * 32 + 8 * g;
      long long off;
      if (a.wmode == 0) {
        off = (long long)n * a.K + k;
      } else {
        const int tap = k / a.Cw, co = k - tap * a.Cw;
        off = ((long long)(a.KH * a.KW - 1 - tap) * a.Ncol + n) * a.Cw + co;
      }
      *reinterpret_cast<uint4*>(lds + f * 1024 + lane * 16) = *reinterpret_cast<const uint4*>(a.wgt + off);
    }
  }
  __syncthreads();

  const int cg = wave % CG, ps = wave / CG;
  const int n0 = (cb * CG + cg) * 64;                  // this wave's first output channel
  const char* wfr = lds + (size_t)cg * KS * 4 * 1024 + lane * 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.src), (short)0, (int)((long long)a.N * a.H * a.W * a.cs * 2), 0x00020000);
  const int tstride = a.pgroups * PS;
  const int ntaps = a.KH * a.KW;

  // ---- per-lane pixel state of the tile being loaded: element offset of tap (0,0) channel 0 (may
  // point outside the image) and the valid-tap bitmask (0 for pixels past M)
  int lpb[TP];
  unsigned lpm[TP];
  auto tile_setup = [&](int tile) {
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int p = tile * (16 * TP) + 16 * j + li;       // M < 2^31 (host-checked)
      unsigned m = 0;
      int base = 0;
      if (p < a.M && a.direct) {
        base = p * a.C;
        m = 1u;
      } else if (p < a.M) {
        const int q = (int)((__umulhi((unsigned)p, a.mow) + (unsigned)p) >> a.sow), ow = p - q * a.OW;
        const int n = (int)((__umulhi((unsigned)q, a.mohh) + (unsigned)q) >> a.sohh), oh = q - n * a.OH;
        const int y0 = oh * a.SH - a.PH, x0 = ow * a.SW - a.PW;
        base = ((n * a.H + y0) * a.W + x0) * a.cs;
        // separable validity: rows kh with 0 <= y0 + kh*DH < H, columns likewise
        unsigned rows = 0, cols = 0;
        for (int kh = 0; kh < a.KH; ++kh) rows |= (unsigned)((unsigned)(y0 + kh * a.DH) < (unsigned)a.H) << kh;
        for (int kw = 0; kw < a.KW; ++kw) cols |= (unsigned)((unsigned)(x0 + kw * a.DW) < (unsigned)a.W) << kw;
        for (int kh = 0; kh < a.KH; ++kh)
          if ((rows >> kh) & 1u) m |= cols << (kh * a.KW);
      }
      lpb[j] = base;
      lpm[j] = m;
    }
  };
  // B fragments of k-step ks of the tile described by (lpb, lpm)
  auto issue_step = [&](bf16x8_t (&b)[TP], int ks) {
    if ((a.dbg & 2)) {
#pragma unroll
      for (int j = 0; j < TP; ++j) b[j] = __builtin_bit_cast(bf16x8_t, make_uint4(ks, lpb[j], j, 0));
      return;
    }
    const int k = ks * 32;
    int tap = 0, toff = k + 8 * g;
    if (!a.direct) {
      tap = k / a.C;
      const int c0 = k - tap * a.C;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
      toff = (kh * a.DH * a.W + kw * a.DW) * a.cs + c0 + 8 * g;
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const unsigned vo = ((lpm[j] >> tap) & 1u) ? (unsigned)(lpb[j] + toff) * 2u : kOOB;
      b[j] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
    }
  };
  auto no_tile = [&]() {
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      lpb[j] = 0;
      lpm[j] = 0;        // every load of a step past the last tile reads zeros (never consumed)
    }
  };

  float s0[16], s1[16];                    // per-lane BN partials of its 16 channels
  if (E::stats || E::bstat) {
#pragma unroll
    for (int e = 0; e < 16; ++e) s0[e] = s1[e] = 0.f;
  }

  // ---- epilogue of compute tile t: lane holds channels n0+8g..+7 and n0+32+8g..+7 of pixels 16j+li
  // fragment layout (chunk g, pixel li) -> row layout (pixel rp = lane>>2, chunk rc = lane&3): after it
  // every 4 consecutive lanes hold 64 contiguous bytes of one output row, so each 16-B-per-lane store
  // instruction writes 16 full 64-B segments (the fragment layout scatters them over 16 rows per quad)
  const int rp = lane >> 2, rc = lane & 3;
  const int xsrc = (16 * rc + rp) * 4;
  auto xpose = [&](const uint4& v) {
    return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.x),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.y),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.z),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.w));
  };

  // ---- epilogue of compute tile t.  Accumulators: lane (g, li) holds channels n0+8g..+7 and
  // n0+32+8g..+7 of pixel 16j+li; stores / fan-out adds / BN-backward statistics run in row layout
  auto epilogue = [&](int t, float4v (&acc)[4][TP]) {
    long long off[TP];
    uint4 old0[TP], old1[TP], x0v[TP], x1v[TP];
    uint32_t mk0[TP], mk1[TP];
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const long long p = (long long)t * (16 * TP) + 16 * j + rp;
      off[j] = p < a.M ? p * a.Ncol + n0 + 8 * rc : -1;
      if (off[j] >= 0) {
        if (E::acc) {
          old0[j] = *reinterpret_cast<const uint4*>(a.out + off[j]);
          old1[j] = *reinterpret_cast<const uint4*>(a.out + off[j] + 32);
        }
        if (E::bstat) {
          x0v[j] = *reinterpret_cast<const uint4*>(a.bx + off[j]);
          x1v[j] = *reinterpret_cast<const uint4*>(a.bx + off[j] + 32);
          mk0[j] = a.bmask ? a.bmask[off[j] >> 3] : 0xffu;
          mk1[j] = a.bmask ? a.bmask[(off[j] + 32) >> 3] : 0xffu;
        }
      }
    }
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
      if (E::stats) {           // from the fp32 accumulators (pixels past M accumulated zeros)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s0[e] += v0[e];
          s1[e] += v0[e] * v0[e];
          s0[8 + e] += v1[e];
          s1[8 + e] += v1[e] * v1[e];
        }
      }
      uint4 w0 = xpose(pack8(v0)), w1 = xpose(pack8(v1));
      if (off[j] < 0) continue;
      if (E::acc) {
        float c0[8], c1[8], o0[8], o1[8];
        unpack8(w0, c0);
        unpack8(w1, c1);
        unpack8(old0[j], o0);
        unpack8(old1[j], o1);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          c0[e] += o0[e];
          c1[e] += o1[e];
        }
        w0 = pack8(c0);
        w1 = pack8(c1);
      }
      if (E::bstat) {
        // statistics of the gradient as stored (bf16), like a separate reduction would see it
        float q0[8], q1[8], xa[8], xb[8];
        unpack8(w0, q0);
        unpack8(w1, q1);
        unpack8(x0v[j], xa);
        unpack8(x1v[j], xb);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float ga = ((mk0[j] >> e) & 1u) ? q0[e] : 0.f;
          const float gb = ((mk1[j] >> e) & 1u) ? q1[e] : 0.f;
          s0[e] += ga;
          s1[e] += ga * xa[e];
          s0[8 + e] += gb;
          s1[8 + e] += gb * xb[e];
        }
      }
      if ((a.dbg & 1)) {
        if (w0.x == 0x12345678u && w1.y == 0x9abcdef0u) a.out[0] = 1;   // keep the math live
        continue;
      }
      *reinterpret_cast<uint4*>(a.out + off[j]) = w0;
      *reinterpret_cast<uint4*>(a.out + off[j] + 32) = w1;
    }
  };

  auto mma_step = [&](float4v (&acc)[4][TP], const bf16x8_t (&b)[TP], int ks) {
    if (a.dbg & 4) {         // probe: no MFMA (keep the operands live)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[0][j][0] += __builtin_bit_cast(uint4, b[j]).x;
      return;
    }
    bf16x8_t af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(wfr + (ks * 4 + i) * 1024));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = mfma(af[i], b[j], acc[i][j]);
  };
  auto zero = [&](float4v (&acc)[4][TP]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  };

  // ---- main loop.  The B fragments of D k-steps are in flight in ring slots; consuming a slot
  // refills it with the step D later (which may belong to a later tile of this wave).
  int ct = pg * PS + ps;
  if (ct < a.ptiles) {
    bf16x8_t ring[D][TP];
    float4v acc[4][TP];
    if constexpr (KSC > 0) {
      // short reduction (KS = KSC <= D): a ring holds TPC whole tiles; loads run TPC tiles ahead
      constexpr int TPC = D / KSC;
      static_assert(TPC * KSC == D, "ring depth must be a multiple of the k-steps per tile");
      int lt = ct;
#pragma unroll
      for (int u = 0; u < TPC; ++u) {
        if (lt < a.ptiles) tile_setup(lt); else no_tile();
#pragma unroll
        for (int ks = 0; ks < KSC; ++ks) issue_step(ring[u * KSC + ks], ks);
        lt += tstride;
      }
      bool live = true;
      while (live) {
#pragma unroll
        for (int u = 0; u < TPC; ++u) {
          if (live) {
            if (lt < a.ptiles) tile_setup(lt); else no_tile();
            zero(acc);
#pragma unroll
            for (int ks = 0; ks < KSC; ++ks) {
              mma_step(acc, ring[u * KSC + ks], ks);
              issue_step(ring[u * KSC + ks], ks);
            }
            lt += tstride;
            epilogue(ct, acc);
            ct += tstride;
            live = ct < a.ptiles;
          }
        }
      }
    } else {
      // long reduction (KS % D == 0): D-step chunks inside a tile; the next tile's first D steps
      // are loaded during this tile's last chunk
      const int KS = a.K >> 5, NCH = KS / D;
      tile_setup(ct);
#pragma unroll
      for (int d = 0; d < D; ++d) issue_step(ring[d], d);
      while (true) {
        zero(acc);
        const int nt = ct + tstride;
        for (int c = 0; c < NCH; ++c) {
          const bool last = c == NCH - 1;
          if (last) {
            if (nt < a.ptiles) tile_setup(nt); else no_tile();
          }
#pragma unroll
          for (int d = 0; d < D; ++d) {
            mma_step(acc, ring[d], c * D + d);
            issue_step(ring[d], last ? d : c * D + d + D);
          }
        }
        epilogue(ct, acc);
        ct = nt;
        if (ct >= a.ptiles) break;
      }
    }
  }

  if (E::stats || E::bstat) {
    // forward statistics live in fragment layout (channel chunk g = lane>>4; reduce over lane bits 0-3),
    // backward statistics in row layout (chunk rc = lane&3; reduce over lane bits 2-5); one atomic per channel
#pragma unroll
    for (int e = 0; e < 16; ++e) {
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const int m = E::stats ? (1 << o) : (4 << o);
        s0[e] += __shfl_xor(s0[e], m, 64);
        s1[e] += __shfl_xor(s1[e], m, 64);
      }
    }
    float* ps0 = E::stats ? a.ssum : a.bsum;
    float* ps1 = E::stats ? a.ssq : a.bsq;
    const int slots = E::stats ? a.sslots : a.bslots;
    const bool writer = E::stats ? li == 0 : rp == 0;
    const int grp = E::stats ? g : rc;
    if (writer) {
      const long long row = (long long)(blockIdx.x % slots) * a.Ncol;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + (e < 8 ? 8 * grp + e : 32 + 8 * grp + (e - 8));
        atomicAdd(ps0 + row + n, s0[e]);
        atomicAdd(ps1 + row + n, s1[e]);
      }
    }
  }
}

template <int TP, int NW, int CG, int D, int KSC, int EPI>
int launch_ws(WsArgs& a, int grid_cap, hipStream_t st) {
  const int KS = a.K / 32;
  if (KSC > 0 ? KS != KSC : (KS % D != 0)) return MDTF_EINVAL;
  a.ptiles = (int)ceil_div(a.M, 16LL * TP);
  a.cblocks = a.Ncol / (64 * CG);
  const size_t lds = (size_t)CG * a.K * 128;            // CG*64 channels x K bf16
  if (lds > 160 * 1024) return MDTF_EUNSUPPORTED;
  const int per_cu_lds = (int)((160 * 1024) / lds);
  const int per_cu_w = NW == 8 ? 1 : 2;                  // 2 waves per SIMD (the register budget)
  const int per_cu = per_cu_lds < per_cu_w ? per_cu_lds : per_cu_w;
  long long want = grid_cap > 0 ? grid_cap : 256LL * per_cu;
  long long pgroups = want / a.cblocks;
  const long long need = ceil_div(a.ptiles, (long long)(NW / CG));
  if (pgroups > need) pgroups = need;
  if (pgroups < 1) pgroups = 1;
  a.pgroups = (int)pgroups;
  const long long nblk = pgroups * a.cblocks;
  hipLaunchKernelGGL((conv_ws_kernel<TP, NW, CG, D, KSC, EPI>), dim3((unsigned)nblk), dim3(64 * NW), lds, st, a);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// (TP, NW, CG) x ring depth; K = 64 / 128 take the compile-time short-reduction loop
template <int EPI, int TP, int NW, int CG>
int dispatch_ws_d(WsArgs& a, int d, int grid_cap, hipStream_t st) {
  const int KS = a.K / 32;
  if (KS == 1 && d == 2) return launch_ws<TP, NW, CG, 2, 1, EPI>(a, grid_cap, st);
  if (KS == 1 && d == 4) return launch_ws<TP, NW, CG, 4, 1, EPI>(a, grid_cap, st);
  if (KS == 3 && d == 3) return launch_ws<TP, NW, CG, 3, 3, EPI>(a, grid_cap, st);
  if (KS == 2 && d == 4) return launch_ws<TP, NW, CG, 4, 2, EPI>(a, grid_cap, st);
  if (KS == 2 && d == 2) return launch_ws<TP, NW, CG, 2, 2, EPI>(a, grid_cap, st);
  if (KS == 4 && d == 4) return launch_ws<TP, NW, CG, 4, 4, EPI>(a, grid_cap, st);
  if (KS <= 4) return MDTF_EINVAL;
  if (d == 4) return launch_ws<TP, NW, CG, 4, 0, EPI>(a, grid_cap, st);
  if (d == 3) return launch_ws<TP, NW, CG, 3, 0, EPI>(a, grid_cap, st);
  if (d == 6) return launch_ws<TP, NW, CG, 6, 0, EPI>(a, grid_cap, st);
  return MDTF_EUNSUPPORTED;
}

template <int EPI>
int dispatch_ws(WsArgs& a, int tp, int nw, int cg, int d, int grid_cap, hipStream_t st) {
#define WS(TP_, NW_, CG_) \
  if (tp == TP_ && nw == NW_ && cg == CG_) return dispatch_ws_d<EPI, TP_, NW_, CG_>(a, d, grid_cap, st);
  WS(4, 8, 1) WS(4, 8, 2) WS(4, 8, 4) WS(4, 4, 1) WS(4, 4, 2)
  WS(2, 8, 1) WS(2, 8, 2) WS(2, 8, 4) WS(2, 4, 1) WS(2, 4, 2)
#undef WS
  return MDTF_EUNSUPPORTED;
}

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
                 float* bsq, int bslots, int accumulate, hipStream_t st) {
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
  const bool stats = ssum != nullptr, bstat = bsum != nullptr;
  if (stats && bstat) return MDTF_EINVAL;
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
                             hipStream_t st) {
  return conv_ws_impl(src, wgt, out, N, H, W, C, C, OH, OW, Ncol, KH, KW, SH, SW, PH, PW, DH, DW, wmode, tile,
                      grid_cap, ssum, ssq, sslots, bx, bmask, bsum, bsq, bslots, accumulate, st);
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
__global__ void __launch_bounds__(256) stem_pack4(const bf16_t* __restrict__ x, uint2* __restrict__ x4, int N, int H,
                                                  int W, int C, int pt, int pl, int H4, int W4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)N * H4 * W4;
  if (i >= total) return;
  const int xw = (int)(i % W4);
  const long long q = i / W4;
  const int yh = (int)(q % H4);
  const int n = (int)(q / H4);
  const int ih = yh - pt, iw = xw - pl;
  uint32_t v[4] = {0u, 0u, 0u, 0u};
  if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
    const bf16_t* p = x + (((long long)n * H + ih) * W + iw) * C;
    for (int c = 0; c < C; ++c) v[c] = p[c];
  }
  x4[i] = make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
}
}  // namespace

MDTF_EXPORT int mdtf_stem_pack4(const void* x, void* x4, int N, int H, int W, int C, int pt, int pl, int H4, int W4,
                                hipStream_t st) {
  if (C < 1 || C > 4) return MDTF_EINVAL;
  const long long total = (long long)N * H4 * W4;
  hipLaunchKernelGGL(stem_pack4, dim3((unsigned)ceil_div(total, 256LL)), dim3(256), 0, st, (const bf16_t*)x,
                     (uint2*)x4, N, H, W, C, pt, pl, H4, W4);
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
                      ssq, sslots, nullptr, nullptr, nullptr, nullptr, 0, 0, st);
}
