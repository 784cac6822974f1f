// Row-staged 3x3 convolution for 64 -> 64 channels at stride 1, pad 1 (ResNet stage 1's conv2: forward and
// data gradient, 56 x 56 images).
//
// Why: the weight-stationary streamed kernel (conv_ws.hip) reads every B fragment from global memory, so
// each input pixel is fetched 9 times (once per tap) through the vector-memory path; at 64 channels that
// path, not the MFMA, bounds it (~450 TF/s).  Here a 512-thread block owns 8 consecutive output rows of one
// image (one row per wave, 4 x 16 pixels, all 64 output channels):
//   * the whole filter (9 taps x 64 x 64 bf16 = 72 KiB) sits in LDS in MFMA fragment order for the block's
//     life (persistent: one block per CU walks groups of rows);
//   * the 10 input rows a group reads (with the zero halo of the padding) are staged in LDS once -- the
//     next group's rows are loaded into registers while this group's MFMAs run and written after them;
//   * both MFMA operands come from LDS with ds_read_b128: filter fragments lane-linear, activation chunks
//     XOR-swizzled (chunk c of pixel px at slot c ^ (px & 6)) so each 16-lane read group hits 16 distinct
//     16-B slots for every tap offset.
// Epilogues: plain store, forward BN statistics (sum y, sum y^2), or the BN-backward statistics of the
// gradient it completes (sum g*mask, sum g*mask*x), as the weight-stationary kernel's modes 0 / 1 / 3.
// Replaces the cuDNN conv2d the reference reaches through tf.nn.conv2d (distribute_tools.py:76,88) and its
// autodiff backward (distribute_tower.py:27) for this shape; SURVEY §2.5 K1.
#include "conv_ws_kernel.inc"

using namespace mdtf;
using namespace mdtf::ws;

namespace {
constexpr int kR3Rows = 8;          // output rows per group (one per wave)
constexpr int kR3Stage = 10;        // 16-B staging chunks per thread per group
constexpr int kR3FilterBytes = 72 * 1024;

// Σ over lanes of a 16-lane DPP row with the lane-bit-0 parity kept: lanes 14 / 15 end with the sums of the
// row's even / odd lanes (three row_shr adds, zero fill past the row start)
__device__ __forceinline__ float row_sum8_pairs(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}
__device__ __forceinline__ float row_sum16_all(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  return row_sum8_pairs(v);
}

// EPI: 0 plain, 1 forward statistics, 3 BN-backward statistics (Epi<> of conv_ws_kernel.inc; no accumulate).
// WI: image width (compile-time: the staging index math is constant divisions).  H = OH, W = OW.
// wmode 0: wgt = Wt[co][(kh, kw, ci)]; wmode 1: wgt = W HWIO used flipped (the stride-1 data gradient, src = DY).
template <int EPI, int WI>
__global__ void __launch_bounds__(512, 1) conv3_rows(const bf16_t* __restrict__ src, const bf16_t* __restrict__ wgt,
                                                      bf16_t* __restrict__ out, int H, int wmode, int rblocks,
                                                      int ngroups, int nbytes, float* __restrict__ ps0,
                                                      float* __restrict__ ps1, int slots,
                                                      const bf16_t* __restrict__ bx, const uint8_t* __restrict__ bmask) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using E = Epi<EPI>;
  constexpr int WP = WI + 2;                      // staged pixels per row (zero halo both sides)
  constexpr int pitch = WP * 128;                 // bytes per staged row (64 channels)
  constexpr int chunks_r = (kR3Rows + 2) * WP * 8;
  constexpr int TP = (WI + 15) / 16;
  static_assert(chunks_r <= kR3Stage * 512, "staged rows exceed the register batch");
  char* rows_s = lds + kR3FilterBytes;
  float* stat_s = reinterpret_cast<float*>(rows_s + chunks_r * 16);   // [2][64] block partials
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  if (threadIdx.x < 128) stat_s[threadIdx.x] = 0.f;

  // ---- filter fragments once per block: f = ks*4 + i (ks = 2*tap + channel half), lane l holds output channel
  // chan_of(i, l & 15), k = 32 ks + 8 (l >> 4)
  for (int q = threadIdx.x; q < 72 * 64; q += 512) {
    const int f = q >> 6, l = q & 63;
    const int n = chan_of(f & 3, l & 15);
    const int k = (f >> 2) * 32 + 8 * (l >> 4);
    const int off = wmode == 0 ? n * 576 + k : ((8 - (k >> 6)) * 64 + n) * 64 + (k & 63);
    reinterpret_cast<uint4*>(lds)[q] = *reinterpret_cast<const uint4*>(wgt + off);
  }

  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(src), (short)0, nbytes, 0x00020000);

  // ---- staging: chunk q of a group = (staged row r, pixel px, LDS slot pos); it holds channel chunk
  // c = pos ^ (px & 6) of input pixel (oh0 - 1 + r, px - 1), zero outside the image
  auto load_rows = [&](int grp, uint4 (&v)[kR3Stage]) {
    const int n = grp / rblocks, oh0 = (grp - n * rblocks) * kR3Rows;
#pragma unroll
    for (int u = 0; u < kR3Stage; ++u) {
      const int q = u * 512 + threadIdx.x;
      const int r = q / (WP * 8), rem = q - r * (WP * 8), px = rem >> 3, c = (rem & 7) ^ (px & 6);
      const int ih = oh0 - 1 + r, iw = px - 1;
      const bool ok = grp < ngroups && q < chunks_r && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)WI;
      const unsigned vo = ok ? (unsigned)((((n * H + ih) * WI + iw) * 64 + 8 * c) * 2) : kOOB;
      v[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
    }
  };
  auto store_rows = [&](const uint4 (&v)[kR3Stage]) {
#pragma unroll
    for (int u = 0; u < kR3Stage; ++u) {
      const int q = u * 512 + threadIdx.x;
      if (q < chunks_r) reinterpret_cast<uint4*>(rows_s)[q] = v[u];
    }
  };

  // row layout of the epilogue (as conv_ws_kernel's): pixel rp, chunk rc; conflict-free ds_bpermute sources
  const int rp = (lane & 31) >> 1, rc = (lane & 1) | ((lane >> 5) << 1);
  const int xsrc = (16 * rc + rp) * 4;
  auto xpose = [&](const uint4& v) {
    return make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.x),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.y),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.z),
                      (uint32_t)__builtin_amdgcn_ds_bpermute(xsrc, (int)v.w));
  };

  // B-fragment byte offsets within a staged row: pixel px = 16 j + li + kw (clamped for pixels past the row:
  // their results are never stored nor counted), channel chunk g of the first half; the second half is ^ 64
  int boff[TP][3];
#pragma unroll
  for (int j = 0; j < TP; ++j)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      int px = 16 * j + li + kw;
      px = px < WP - 1 ? px : WP - 1;
      boff[j][kw] = px * 128 + ((16 * g) ^ ((px & 6) << 4));
    }

  auto run_group = [&](int grp) {
    const int n = grp / rblocks, oh = (grp - n * rblocks) * kR3Rows + wave;
    if (oh >= H) return;                                   // wave-uniform
    float4v acc[4][TP];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const char* row = rows_s + (wave + kh) * pitch;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int hc = 0; hc < 2; ++hc) {
          const int ks = (kh * 3 + kw) * 2 + hc;
          bf16x8_t af[4], b[TP];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            af[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(lds + (ks * 4 + i) * 1024 + lane * 16));
#pragma unroll
          for (int j = 0; j < TP; ++j)
            b[j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(row + (boff[j][kw] ^ (hc * 64))));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < TP; ++j) acc[i][j] = mfma(af[i], b[j], acc[i][j]);
        }
    }

    // ---- epilogue: fragment layout (chunk g, pixel li) -> row layout (pixel rp, chunk rc), 2 x 16-B stores
    // per pixel; statistics per lane, row-reduced with DPP and added to the block's LDS partials
    float s0[16], s1[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) s0[e] = s1[e] = 0.f;
    const long long prow = ((long long)n * H + oh) * WI;
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
      if (E::stats && 16 * j + li < WI) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s0[e] += v0[e];
          s1[e] += v0[e] * v0[e];
          s0[8 + e] += v1[e];
          s1[8 + e] += v1[e] * v1[e];
        }
      }
      const uint4 w0 = xpose(pack8(v0)), w1 = xpose(pack8(v1));
      const int ow = 16 * j + rp;
      if (ow < WI) {
        const long long off = (prow + ow) * 64 + 8 * rc;
        if (E::bstat) {
          // statistics of the gradient as stored (bf16), like a separate reduction would see it
          const uint4 x0v = *reinterpret_cast<const uint4*>(bx + off), x1v = *reinterpret_cast<const uint4*>(bx + off + 32);
          const uint32_t mk0 = bmask ? bmask[off >> 3] : 0xffu, mk1 = bmask ? bmask[(off + 32) >> 3] : 0xffu;
          float q0[8], q1[8], xa[8], xb[8];
          unpack8(w0, q0);
          unpack8(w1, q1);
          unpack8(x0v, xa);
          unpack8(x1v, xb);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float ga = ((mk0 >> e) & 1u) ? q0[e] : 0.f;
            const float gb = ((mk1 >> e) & 1u) ? q1[e] : 0.f;
            s0[e] += ga;
            s1[e] += ga * xa[e];
            s0[8 + e] += gb;
            s1[8 + e] += gb * xb[e];
          }
        }
        bf16_t* o = out + off;
        *reinterpret_cast<uint4*>(o) = w0;
        *reinterpret_cast<uint4*>(o + 32) = w1;
      }
    }
    if (E::stats) {              // fragment layout: channel chunk g, reduce over li
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        s0[e] = row_sum16_all(s0[e]);
        s1[e] = row_sum16_all(s1[e]);
      }
      if (li == 15) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int c = e < 8 ? 8 * g + e : 32 + 8 * g + (e - 8);
          atomicAdd(stat_s + c, s0[e]);
          atomicAdd(stat_s + 64 + c, s1[e]);
        }
      }
    }
    if (E::bstat) {              // row layout: chunk rc = (lane & 1) | (lane >> 5) << 1, reduce over lane bits 1-4
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        s0[e] = row_sum8_pairs(s0[e]);
        s1[e] = row_sum8_pairs(s1[e]);
      }
      if (li >= 14) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int c = e < 8 ? 8 * rc + e : 32 + 8 * rc + (e - 8);
          atomicAdd(stat_s + c, s0[e]);
          atomicAdd(stat_s + 64 + c, s1[e]);
        }
      }
    }
  };

  uint4 pv[kR3Stage];
  load_rows(bid, pv);
  store_rows(pv);
  for (int grp = bid; grp < ngroups; grp += gridDim.x) {
    __syncthreads();                                     // this group's rows (and the filter) are in LDS
    const int nxt = grp + gridDim.x;
    load_rows(nxt, pv);                                  // in flight during this group's MFMAs
    run_group(grp);
    __syncthreads();                                     // every wave is done with this group's rows
    if (nxt < ngroups) store_rows(pv);
  }
  if (E::stats || E::bstat) {
    __syncthreads();
    if (threadIdx.x < 128) {
      float* dst = (threadIdx.x < 64 ? ps0 : ps1) + (long long)(blockIdx.x % slots) * 64 + (threadIdx.x & 63);
      atomicAdd(dst, stat_s[threadIdx.x]);
    }
  }
}

template <int EPI>
void launch_rows(const void* src, const void* wgt, void* out, int N, int H, int wmode, float* s0, float* s1,
                 int slots, const void* bx, const void* bmask, hipStream_t st) {
  constexpr int WI = 56;
  const int rblocks = (H + kR3Rows - 1) / kR3Rows;
  const int ngroups = N * rblocks;
  const size_t lds = kR3FilterBytes + (size_t)(kR3Rows + 2) * (WI + 2) * 128 + 128 * sizeof(float);
  const int nblk = ngroups < 256 ? ngroups : 256;       // one block per CU (LDS-bound), persistent
  hipLaunchKernelGGL((conv3_rows<EPI, WI>), dim3((unsigned)nblk), dim3(512), lds, st, (const bf16_t*)src,
                     (const bf16_t*)wgt, (bf16_t*)out, H, wmode, rblocks, ngroups, (int)((long long)N * H * WI * 128),
                     s0, s1, slots > 0 ? slots : 1, (const bf16_t*)bx, (const uint8_t*)bmask);
}
}  // namespace

// out[N][H][W][64] = conv3x3(src[N][H][W][64], filter), stride 1, pad 1 (W = 56).
// wmode 0: wgt = Wt[64][9*64] (transpose_filter); s0/s1 non-null: forward BN statistics ([slots][64] partials).
// wmode 1: wgt = HWIO [3][3][64][64] used flipped, src = DY, out = DX; s0/s1 non-null: BN-backward statistics
// of DX against bx (the BN input) and the optional ReLU bitmask bmask.
MDTF_EXPORT int mdtf_conv3_rows(const void* src, const void* wgt, void* out, int N, int H, int W, int wmode, float* s0,
                                float* s1, int slots, const void* bx, const void* bmask, hipStream_t st) {
  if (W != 56 || H < 1 || N < 1 || (wmode != 0 && wmode != 1) || (!s0) != (!s1)) return MDTF_EINVAL;
  if ((long long)N * H * W * 128 >= 0x80000000LL) return MDTF_EUNSUPPORTED;   // 32-bit buffer offsets
  if (wmode == 1 && s0 && !bx) return MDTF_EINVAL;
  if (!s0)
    launch_rows<0>(src, wgt, out, N, H, wmode, s0, s1, slots, bx, bmask, st);
  else if (wmode == 0)
    launch_rows<1>(src, wgt, out, N, H, wmode, s0, s1, slots, bx, bmask, st);
  else
    launch_rows<3>(src, wgt, out, N, H, wmode, s0, s1, slots, bx, bmask, st);
  MDTF_LAUNCH_CHECK();
  return 0;
}
