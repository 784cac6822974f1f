// Fused multi-head attention for any sequence length S % 64 == 0 (192, 384, 512, ...) and head dim 64 / 128
// (gfx950, bf16 MFMA).
//
// BASELINE config 4 (BERT-base; phase-2 pre-training runs seq 512) -- csrc/attention.hip keeps the
// whole-sequence-in-LDS kernels for S = 128, D = 64; these kernels tile the other dimension and
// carry the softmax online, so LDS holds one 64-key (or 32/64-query) tile pair at a time:
//   forward  (workgroup = 128 queries of one (batch, head), wave = 32 queries): loop over 64-key tiles
//     of K and V (LDS-DMA, double-buffered); S^T = K Q^T with Q fragments in registers; running max /
//     sum per query (in-lane over the tile, then 2 cross-lane shuffles), O^T rescaled and accumulated
//     with V^T P^T (P^T fed from registers as the B operand, V^T read with ds_read_b64_tr_b16 under the
//     same key permutation); attention dropout by the counter hash of attention.hip; lse per query;
//   backward: Dq = rowsum(dO * O) (small kernel), then
//     dK/dV (workgroup = 64 keys, wave = 16 keys): loop over 32-query tiles of Q and dO: S = Q K^T and
//       dP = dO V^T with K, V fragments in registers; dS = P (dP - Dq); dV^T += dO^T P, dK^T += Q^T dS
//       with the accumulators of S / dS used directly as B operands (key columns on the lanes);
//     dQ (workgroup = 64 queries, wave = 16 queries): loop over 64-key tiles: S^T, dP^T, dS^T as in the
//       forward orientation, dQ^T += K^T dS^T.
//   Every pass reads Q/K/V straight out of the fused projection [B*S, 3H] and writes [B*S, H] / dQKV.
// Reference: the attention the BERT family adds on top of the reference's dense toolkit
// (distribute_tools.py:204-206); SURVEY §2.5 K8.
#include "mdtf_common.h"

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int NT = 256;   // 4 waves

// 16-B chunk swizzles of 128-B-row images (involutions)
struct SwzA {    // read 16 rows at a time with ds_read_b128
  __device__ static int f(int r, int c) { return c ^ ((r >> 1) & 7); }
};
struct SwzV {    // read transposed, rows {4g+q} / {16+4g+q}
  __device__ static int f(int r, int c) { return c ^ (((r >> 1) & 3) << 1); }
};

__device__ __forceinline__ float4v mfma(const bf16x8_t& a, const bf16x8_t& b, const float4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t step_seed(uint32_t seed, const long long* seed_off) {
  return seed_off ? seed ^ ((uint32_t)(*seed_off) * 0x85EBCA6Bu) : seed;
}

// keep bit of attention-dropout element (bh, q, k) -- the same stream as attention.hip at S = 128
__device__ __forceinline__ bool keep_elem(uint32_t seed, int bh, int S, int q, int k, uint32_t thr) {
  const uint32_t idx = ((uint32_t)bh * S + (uint32_t)q) * S + (uint32_t)k;
  return hash_u32(idx * 0x9E3779B1u ^ seed) >= thr;
}

// DMA rows [r0, r0 + R) x 64 columns (elements col0 .. col0 + 63 of row r at t + (rowbase + r*ld)) into a
// R x 128-B image; NWV waves, one 1-KiB (8-row) piece per wave instruction
template <class SW, int R>
__device__ __forceinline__ void load_tile(const bf16_t* t, int tbytes, long long rowbase, int ld, int col0, char* img,
                                          int wave, int lane) {
#pragma unroll
  for (int jj = 0; jj < R / 32; ++jj) {
    const int j = wave + 4 * jj;                  // 8-row block
    const int r = 8 * j + (lane >> 3);
    const int c = SW::f(r, lane & 7);
    const unsigned voff = (unsigned)((rowbase + (long long)r * ld + col0 + c * 8) * 2);
    dma16(t, tbytes, img + j * 1024, voff, 0);
  }
}

template <class SW>
__device__ __forceinline__ bf16x8_t row_frag(const char* img, int r0, int c0, int lane) {
  const int r = r0 + (lane & 15);
  const int c = c0 + (lane >> 4);
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(img + r * 128 + (SW::f(r, c) << 4)));
}

__device__ __forceinline__ v4s tr4(const char* img, int r, int col) {
  const char* p = img + r * 128 + (SwzV::f(r, col >> 3) << 4) + (col & 7) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p);
}

// A operand X^T[col][k] from a [k rows][64 cols] image (SwzV), 32-deep k-step at kb, k order
// {4g..4g+3, 16+4g..16+4g+3} (the order of two stacked 16x16 accumulator tiles used as a B operand)
__device__ __forceinline__ bf16x8_t trp_frag(const char* img, int kb, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
  const v4s lo = tr4(img, kb + 4 * g + q4, col0 + 4 * p4);
  const v4s hi = tr4(img, kb + 16 + 4 * g + q4, col0 + 4 * p4);
  const short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, f);
}

// two stacked 16x16 fp32 accumulator tiles -> one bf16 B fragment (k order as trp_frag)
__device__ __forceinline__ bf16x8_t pack_acc(const float4v& a0, const float4v& a1) {
  const uint4 w = make_uint4(pack_bf2(a0[0], a0[1]), pack_bf2(a0[2], a0[3]), pack_bf2(a1[0], a1[1]),
                             pack_bf2(a1[2], a1[3]));
  return __builtin_bit_cast(bf16x8_t, w);
}

__device__ __forceinline__ bf16x8_t gfrag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}

__device__ __forceinline__ float4 mask4(const float* mask, long long off) {
  return mask ? *reinterpret_cast<const float4*>(mask + off) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// ================================================================================ forward
template <int D>
__global__ void __launch_bounds__(NT, 2) attn_fwd_flash(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                         bf16_t* __restrict__ out, float* __restrict__ lse_out, int B,
                                                         int S, int nh, float scale, float p_drop, uint32_t seed,
                                                         const long long* __restrict__ seed_off) {
  constexpr int DH = D / 64;                     // 64-column halves of a head
  constexpr int TILE = 64 * 128 * DH;            // one K or V tile image (64 keys)
  seed = step_seed(seed, seed_off);
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];   // [buf][K | V]
  const int bh = blockIdx.x, b = bh / nh, h = bh - b * nh;
  const int q0 = blockIdx.y * 128;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long rowb = (long long)b * S * ld;
  const int tbytes = (int)((long long)B * S * ld * 2);
  const int nkt = S / 64;

  auto load_kv = [&](int kb, int buf) {
    char* Ki = smem + buf * 2 * TILE;
    char* Vi = Ki + TILE;
#pragma unroll
    for (int hh = 0; hh < DH; ++hh) {
      load_tile<SwzA, 64>(qkv, tbytes, rowb + (long long)kb * 64 * ld, ld, H + h * D + 64 * hh, Ki + hh * 8192, wave,
                          lane);
      load_tile<SwzV, 64>(qkv, tbytes, rowb + (long long)kb * 64 * ld, ld, 2 * H + h * D + 64 * hh, Vi + hh * 8192,
                          wave, lane);
    }
  };
  load_kv(0, 0);
  bf16x8_t qf[2][D / 32];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds) {
      // the last block of an S % 128 == 64 sequence has 64 queries: waves past S load a valid row and store nothing
      const int q = min(q0 + 32 * wave + 16 * qt + li, S - 1);
      qf[qt][ds] = gfrag(qkv + rowb + (long long)q * ld + h * D + 32 * ds + 8 * g);
    }
  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  float m[2] = {-3.0e38f, -3.0e38f}, l[2] = {0.f, 0.f};
  float4v oacc[D / 16][2];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) oacc[dt][0] = oacc[dt][1] = float4v{0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkt; ++kb) {
    wait_vmcnt<0>();
    __syncthreads();                                   // tile kb landed; tile kb-1's buffer is free
    if (kb + 1 < nkt) load_kv(kb + 1, (kb + 1) & 1);
    const char* Ki = smem + (kb & 1) * 2 * TILE;
    const char* Vi = Ki + TILE;
    float4v sacc[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) sacc[kt][0] = sacc[kt][1] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8_t kf = row_frag<SwzA>(Ki + (ds >> 1) * 8192, kt * 16, 4 * (ds & 1), lane);
        sacc[kt][0] = mfma(kf, qf[0][ds], sacc[kt][0]);
        sacc[kt][1] = mfma(kf, qf[1][ds], sacc[kt][1]);
      }
    float mk[4][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const float4 m4 = mask4(mask, (long long)b * S + kb * 64 + kt * 16 + 4 * g);
      mk[kt][0] = m4.x;
      mk[kt][1] = m4.y;
      mk[kt][2] = m4.z;
      mk[kt][3] = m4.w;
    }
    bf16x8_t pf[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = -3.0e38f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float s = sacc[kt][qt][i] * scale + mk[kt][i];
          sacc[kt][qt][i] = s;
          mx = fmaxf(mx, s);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[qt], mx);
      const float corr = __expf(m[qt] - mn);
      m[qt] = mn;
      float sum = 0.f;
      const int q = q0 + 32 * wave + 16 * qt + li;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __expf(sacc[kt][qt][i] - mn);
          sum += e;
          sacc[kt][qt][i] = (thr && !keep_elem(seed, bh, S, q, kb * 64 + kt * 16 + 4 * g + i, thr)) ? 0.f
                                                                                                       : e * inv_keep;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l[qt] = l[qt] * corr + sum;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) oacc[dt][qt] *= corr;
      pf[qt][0] = pack_acc(sacc[0][qt], sacc[1][qt]);
      pf[qt][1] = pack_acc(sacc[2][qt], sacc[3][qt]);
    }
    // O^T[d][q] += V^T P^T
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        const bf16x8_t vf = trp_frag(Vi + (dt >> 2) * 8192, 32 * ks, (dt & 3) * 16, lane);
        oacc[dt][0] = mfma(vf, pf[0][ks], oacc[dt][0]);
        oacc[dt][1] = mfma(vf, pf[1][ks], oacc[dt][1]);
      }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 32 * wave + 16 * qt + li;
    if (q >= S) continue;
    const float inv = 1.f / l[qt];
    if (g == 0) lse_out[(long long)bh * S + q] = m[qt] + __logf(l[qt]);
    bf16_t* o = out + ((long long)b * S + q) * H + h * D;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      const float4v v = oacc[dt][qt];
      *reinterpret_cast<uint2*>(o + dt * 16 + 4 * g) =
          make_uint2(pack_bf2(v[0] * inv, v[1] * inv), pack_bf2(v[2] * inv, v[3] * inv));
    }
  }
}

// ================================================================================ backward
// Dq[bh][q] = sum_d dO[q][d] * O[q][d]; one wave per (q, head) row group of 64 elements x 8 rows
__global__ void __launch_bounds__(256) attn_bwd_pre(const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                    float* __restrict__ dq, int B, int S, int nh, int D) {
  const long long row = (long long)blockIdx.x * 32 + (threadIdx.x >> 3);   // (b*S + q) * nh + h
  const int sub = threadIdx.x & 7;
  const long long total = (long long)B * S * nh;
  float part = 0.f;
  if (row < total) {
    const long long bq = row / nh;
    const int h = (int)(row - bq * nh);
    const long long base = bq * nh * D + (long long)h * D;
    for (int d = sub * 8; d < D; d += 64) {
      float o8[8], g8[8];
      load_bf8(out + base + d, o8);
      load_bf8(dout + base + d, g8);
#pragma unroll
      for (int e = 0; e < 8; ++e) part += o8[e] * g8[e];
    }
  }
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) part += __shfl_xor(part, o, 64);
  if (row < total && sub == 0) {
    const long long bq = row / nh;
    const int h = (int)(row - bq * nh);
    const long long b = bq / S;
    const int q = (int)(bq - b * S);
    dq[(b * nh + h) * S + q] = part;
  }
}

// dK, dV for 64 keys of one (b, h); wave = 16 keys; loop over 32-query tiles
template <int D>
__global__ void __launch_bounds__(NT, 2) attn_bwd_dkv(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                       const bf16_t* __restrict__ dout, const float* __restrict__ lse,
                                                       const float* __restrict__ dqv, bf16_t* __restrict__ dqkv,
                                                       int B, int S, int nh, float scale, float p_drop, uint32_t seed,
                                                       const long long* __restrict__ seed_off) {
  constexpr int DH = D / 64;
  constexpr int IMG = 32 * 128;                  // [32 queries][64 d]
  constexpr int BUF = 4 * DH * IMG;              // Q_A, dO_A, Q_V, dO_V (each DH halves)
  seed = step_seed(seed, seed_off);
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int bh = blockIdx.x, b = bh / nh, h = bh - b * nh;
  const int k0 = blockIdx.y * 64;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long rowb = (long long)b * S * ld, orow = (long long)b * S * H;
  const int tbytes = (int)((long long)B * S * ld * 2), obytes = (int)((long long)B * S * H * 2);
  const int nqt = S / 32;

  auto load_q = [&](int qb, int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int hh = 0; hh < DH; ++hh) {
      const long long qrow = rowb + (long long)qb * 32 * ld, orw = orow + (long long)qb * 32 * H;
      load_tile<SwzA, 32>(qkv, tbytes, qrow, ld, h * D + 64 * hh, base + (0 * DH + hh) * IMG, wave, lane);
      load_tile<SwzA, 32>(dout, obytes, orw, H, h * D + 64 * hh, base + (1 * DH + hh) * IMG, wave, lane);
      load_tile<SwzV, 32>(qkv, tbytes, qrow, ld, h * D + 64 * hh, base + (2 * DH + hh) * IMG, wave, lane);
      load_tile<SwzV, 32>(dout, obytes, orw, H, h * D + 64 * hh, base + (3 * DH + hh) * IMG, wave, lane);
    }
  };
  load_q(0, 0);
  const int key = k0 + 16 * wave + li;           // this lane's key column
  bf16x8_t kf[D / 32], vf[D / 32];
#pragma unroll
  for (int ds = 0; ds < D / 32; ++ds) {
    kf[ds] = gfrag(qkv + rowb + (long long)key * ld + H + h * D + 32 * ds + 8 * g);
    vf[ds] = gfrag(qkv + rowb + (long long)key * ld + 2 * H + h * D + 32 * ds + 8 * g);
  }
  const float mkey = mask ? mask[(long long)b * S + key] : 0.f;
  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  float4v vacc[D / 16], kacc[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) vacc[dt] = kacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};

  for (int qb = 0; qb < nqt; ++qb) {
    wait_vmcnt<0>();
    __syncthreads();
    if (qb + 1 < nqt) load_q(qb + 1, (qb + 1) & 1);
    const char* base = smem + (qb & 1) * BUF;
    const char* QA = base;
    const char* OA = base + DH * IMG;
    const char* QV = base + 2 * DH * IMG;
    const char* OV = base + 3 * DH * IMG;
    // S[q][k], dP[q][k] for 32 queries x this wave's 16 keys
    float4v sacc[2], pacc[2];
    sacc[0] = sacc[1] = pacc[0] = pacc[1] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const bf16x8_t qa = row_frag<SwzA>(QA + (ds >> 1) * IMG, 16 * qt, 4 * (ds & 1), lane);
        const bf16x8_t oa = row_frag<SwzA>(OA + (ds >> 1) * IMG, 16 * qt, 4 * (ds & 1), lane);
        sacc[qt] = mfma(qa, kf[ds], sacc[qt]);
        pacc[qt] = mfma(oa, vf[ds], pacc[qt]);
      }
    // lane holds queries 16qt + 4g + i of key `key`
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = qb * 32 + 16 * qt + 4 * g + i;
        const float p = __expf(sacc[qt][i] * scale + mkey - lse[(long long)bh * S + q]);
        float dp = pacc[qt][i], pk = p;
        if (thr) {
          const bool keep = keep_elem(seed, bh, S, q, key, thr);
          pk = keep ? p * inv_keep : 0.f;
          dp = keep ? dp * inv_keep : 0.f;
        }
        sacc[qt][i] = pk;                                   // P_drop
        pacc[qt][i] = p * (dp - dqv[(long long)bh * S + q]);  // dS
      }
    const bf16x8_t pb = pack_acc(sacc[0], sacc[1]);
    const bf16x8_t sb = pack_acc(pacc[0], pacc[1]);
    // dV^T[d][k] += dO^T P_drop, dK^T[d][k] += Q^T dS  (k-dim = the 32 queries, permuted order)
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      const bf16x8_t of = trp_frag(OV + (dt >> 2) * IMG, 0, (dt & 3) * 16, lane);
      const bf16x8_t qf = trp_frag(QV + (dt >> 2) * IMG, 0, (dt & 3) * 16, lane);
      vacc[dt] = mfma(of, pb, vacc[dt]);
      kacc[dt] = mfma(qf, sb, kacc[dt]);
    }
  }
  // lane holds rows d = 16dt + 4g .. +3 of key column `key`
  bf16_t* rowp = dqkv + rowb + (long long)key * ld + h * D;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    const float4v kv = kacc[dt], vv = vacc[dt];
    *reinterpret_cast<uint2*>(rowp + H + dt * 16 + 4 * g) =
        make_uint2(pack_bf2(kv[0] * scale, kv[1] * scale), pack_bf2(kv[2] * scale, kv[3] * scale));
    *reinterpret_cast<uint2*>(rowp + 2 * H + dt * 16 + 4 * g) =
        make_uint2(pack_bf2(vv[0], vv[1]), pack_bf2(vv[2], vv[3]));
  }
}

// dQ for 64 queries of one (b, h); wave = 16 queries; loop over 64-key tiles
template <int D>
__global__ void __launch_bounds__(NT, 2) attn_bwd_dq(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                      const bf16_t* __restrict__ dout, const float* __restrict__ lse,
                                                      const float* __restrict__ dqv, bf16_t* __restrict__ dqkv, int B,
                                                      int S, int nh, float scale, float p_drop, uint32_t seed,
                                                      const long long* __restrict__ seed_off) {
  constexpr int DH = D / 64;
  constexpr int IMG = 64 * 128;                  // [64 keys][64 d]
  constexpr int BUF = 3 * DH * IMG;              // K_A, V_A, K_V
  seed = step_seed(seed, seed_off);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bh = blockIdx.x, b = bh / nh, h = bh - b * nh;
  const int q0 = blockIdx.y * 64;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long rowb = (long long)b * S * ld, orow = (long long)b * S * H;
  const int tbytes = (int)((long long)B * S * ld * 2);
  const int nkt = S / 64;

  auto load_k = [&](int kb, int buf) {
    char* base = smem + buf * BUF;
    const long long krow = rowb + (long long)kb * 64 * ld;
#pragma unroll
    for (int hh = 0; hh < DH; ++hh) {
      load_tile<SwzA, 64>(qkv, tbytes, krow, ld, H + h * D + 64 * hh, base + (0 * DH + hh) * IMG, wave, lane);
      load_tile<SwzA, 64>(qkv, tbytes, krow, ld, 2 * H + h * D + 64 * hh, base + (1 * DH + hh) * IMG, wave, lane);
      load_tile<SwzV, 64>(qkv, tbytes, krow, ld, H + h * D + 64 * hh, base + (2 * DH + hh) * IMG, wave, lane);
    }
  };
  load_k(0, 0);
  const int q = q0 + 16 * wave + li;             // this lane's query column
  bf16x8_t qf[D / 32], of[D / 32];
#pragma unroll
  for (int ds = 0; ds < D / 32; ++ds) {
    qf[ds] = gfrag(qkv + rowb + (long long)q * ld + h * D + 32 * ds + 8 * g);
    of[ds] = gfrag(dout + orow + (long long)q * H + h * D + 32 * ds + 8 * g);
  }
  const float lq = lse[(long long)bh * S + q], Dq = dqv[(long long)bh * S + q];
  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  float4v qacc[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) qacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkt; ++kb) {
    wait_vmcnt<0>();
    __syncthreads();
    if (kb + 1 < nkt) load_k(kb + 1, (kb + 1) & 1);
    const char* base = smem + (kb & 1) * BUF;
    const char* KA = base;
    const char* VA = base + DH * IMG;
    const char* KV = base + 2 * DH * IMG;
    // S^T[k][q], dP^T[k][q] for 64 keys x this wave's 16 queries
    float4v sacc[4], pacc[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) sacc[kt] = pacc[kt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8_t ka = row_frag<SwzA>(KA + (ds >> 1) * IMG, 16 * kt, 4 * (ds & 1), lane);
        const bf16x8_t va = row_frag<SwzA>(VA + (ds >> 1) * IMG, 16 * kt, 4 * (ds & 1), lane);
        sacc[kt] = mfma(ka, qf[ds], sacc[kt]);
        pacc[kt] = mfma(va, of[ds], pacc[kt]);
      }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const float4 m4 = mask4(mask, (long long)b * S + kb * 64 + kt * 16 + 4 * g);
      const float mk[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = kb * 64 + kt * 16 + 4 * g + i;
        const float p = __expf(sacc[kt][i] * scale + mk[i] - lq);
        float dp = pacc[kt][i];
        if (thr) dp = keep_elem(seed, bh, S, q, k, thr) ? dp * inv_keep : 0.f;
        sacc[kt][i] = p * (dp - Dq);                           // dS^T
      }
    }
    // dQ^T[d][q] += K^T dS^T  (k-dim = keys, 2 steps of 32, permuted order)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8_t sb = pack_acc(sacc[2 * ks], sacc[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        const bf16x8_t kt_ = trp_frag(KV + (dt >> 2) * IMG, 32 * ks, (dt & 3) * 16, lane);
        qacc[dt] = mfma(kt_, sb, qacc[dt]);
      }
    }
  }
  bf16_t* rowp = dqkv + rowb + (long long)q * ld + h * D;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    const float4v v = qacc[dt];
    *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * g) =
        make_uint2(pack_bf2(v[0] * scale, v[1] * scale), pack_bf2(v[2] * scale, v[3] * scale));
  }
}

bool shape_ok(int B, int S, int nh, int dh) {
  if (S % 64 || S < 64 || (dh != 64 && dh != 128)) return false;
  return (long long)B * S * 3 * nh * dh * 2 <= 0x7fffffffLL && (long long)B * nh * S * S < 0xffffffffLL;
}

}  // namespace

// ctx[B*S, H] = attention(qkv[B*S, 3H]) for S % 64 == 0, head dim 64 / 128; lse [B*nh, S] (fp32)
MDTF_EXPORT int mdtf_attn_fwd_flash(const void* qkv, const float* mask, void* out, float* lse, int B, int seq, int nh,
                                    int dh, float scale, float p_drop, unsigned seed, const long long* seed_off,
                                    hipStream_t st) {
  if (!shape_ok(B, seq, nh, dh)) return MDTF_EUNSUPPORTED;
  const dim3 grid(B * nh, (seq + 127) / 128);
  if (dh == 64)
    hipLaunchKernelGGL(attn_fwd_flash<64>, grid, dim3(NT), 0, st, (const bf16_t*)qkv, mask, (bf16_t*)out, lse, B, seq,
                       nh, scale, p_drop, (uint32_t)seed, seed_off);
  else
    hipLaunchKernelGGL(attn_fwd_flash<128>, grid, dim3(NT), 0, st, (const bf16_t*)qkv, mask, (bf16_t*)out, lse, B,
                       seq, nh, scale, p_drop, (uint32_t)seed, seed_off);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// dqkv[B*S, 3H] (every element written) from dout[B*S, H]; ws: fp32 [B*nh*seq] (Dq = rowsum(dO*O))
MDTF_EXPORT int mdtf_attn_bwd_flash(const void* qkv, const float* mask, const void* out, const void* dout,
                                    const float* lse, void* dqkv, float* ws, int B, int seq, int nh, int dh,
                                    float scale, float p_drop, unsigned seed, const long long* seed_off,
                                    hipStream_t st) {
  if (!shape_ok(B, seq, nh, dh)) return MDTF_EUNSUPPORTED;
  const long long rows = (long long)B * seq * nh;
  hipLaunchKernelGGL(attn_bwd_pre, dim3((unsigned)ceil_div(rows, 32LL)), dim3(256), 0, st, (const bf16_t*)out,
                     (const bf16_t*)dout, ws, B, seq, nh, dh);
  const dim3 gk(B * nh, seq / 64), gq(B * nh, seq / 64);
  if (dh == 64) {
    hipLaunchKernelGGL(attn_bwd_dkv<64>, gk, dim3(NT), 0, st, (const bf16_t*)qkv, mask, (const bf16_t*)dout, lse, ws,
                       (bf16_t*)dqkv, B, seq, nh, scale, p_drop, (uint32_t)seed, seed_off);
    hipLaunchKernelGGL(attn_bwd_dq<64>, gq, dim3(NT), 2 * 3 * 1 * 64 * 128, st, (const bf16_t*)qkv, mask,
                       (const bf16_t*)dout, lse, ws, (bf16_t*)dqkv, B, seq, nh, scale, p_drop, (uint32_t)seed,
                       seed_off);
  } else {
    hipLaunchKernelGGL(attn_bwd_dkv<128>, gk, dim3(NT), 0, st, (const bf16_t*)qkv, mask, (const bf16_t*)dout, lse,
                       ws, (bf16_t*)dqkv, B, seq, nh, scale, p_drop, (uint32_t)seed, seed_off);
    hipLaunchKernelGGL(attn_bwd_dq<128>, gq, dim3(NT), 2 * 3 * 2 * 64 * 128, st, (const bf16_t*)qkv, mask,
                       (const bf16_t*)dout, lse, ws, (bf16_t*)dqkv, B, seq, nh, scale, p_drop, (uint32_t)seed,
                       seed_off);
  }
  MDTF_LAUNCH_CHECK();
  return 0;
}
