// Fused multi-head attention for BERT-style encoders on bf16 MFMA (gfx950).
//
// BASELINE config "BERT-base data-parallel (MFMA bf16 GEMM + fused Adam)": the
// attention core softmax(Q K^T * scale + mask) V of every (batch, head) runs as
// ONE workgroup that reads Q/K/V straight out of the fused QKV projection
// output [B*S, 3H] and writes the context straight into [B*S, H] (the layout
// the output projection consumes) -- no permute copies, no [B, heads, S, S]
// score tensor in HBM.  Sequence length 128, head dim 64 (BERT-base/large).
//
// Forward (per workgroup = (b, h), 4 waves, wave w owns queries 32w..32w+31):
//   * K and V head slices ([128][64] bf16) -> LDS by LDS-DMA (buffer_load ... lds);
//     Q fragments straight to registers;
//   * S^T = K Q^T on v_mfma_f32_16x16x32_bf16 (lane owns one query column);
//   * scale + additive key mask, softmax over keys (in-lane over 32 values, then
//     2 cross-lane shuffles), attention dropout (counter-hash RNG, regenerated
//     identically in backward), logsumexp saved per query;
//   * O^T = V^T P^T with P^T fed from registers (bf16) as the B operand and V^T
//     read with ds_read_b64_tr_b16 (hardware transpose) -- the key order of the two
//     operands is permuted identically, which the k-reduction does not see.
// Backward (one workgroup per (b, h), 144 KiB LDS):
//   phase 1 (wave = 32 queries): recompute P from the saved logsumexp,
//     dP = dO V^T, D = rowsum(dO * O), dS = P (dP - D); P_drop and dS go to LDS
//     as [q][k] images;
//   phase 2 (wave = 32 keys for dK/dV, 32 queries for dQ):
//     dV = P_drop^T dO, dK = scale dS^T Q, dQ = scale dS K, all operands from LDS
//     (row reads or transposed reads), written into dQKV [B*S, 3H] directly.
// LDS images use XOR chunk swizzles chosen per access pattern so the 16-row
// ds_read_b128 and the 8-row transposed reads are (near) conflict-free.
#include "mdtf_common.h"

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int S = 128;   // sequence length (keys = queries)
constexpr int D = 64;    // head dim
constexpr int NT = 256;

// 16-B chunk swizzles (involutions): logical chunk c of row r sits at physical chunk swz(r, c)
struct SwzA {    // 128-B rows read 16 rows at a time with ds_read_b128
  __device__ static int f(int r, int c) { return c ^ ((r >> 1) & 7); }
};
struct SwzT {    // 128-B rows read transposed, rows {8g+q} / {8g+4+q}
  __device__ static int f(int r, int c) { return c ^ ((((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1); }
};
struct SwzV {    // 128-B rows read transposed, rows {4g+q} / {16+4g+q}
  __device__ static int f(int r, int c) { return c ^ (((r >> 1) & 3) << 1); }
};
struct Swz256 {  // 256-B rows ([q][k] images): transposed reads rows {8g+q}/{8g+4+q}, and row reads
  __device__ static int f(int r, int c) { return c ^ (((r & 3) | (((r >> 3) & 1) << 2)) << 1); }
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

// per-step seed: host seed of the call site mixed with the device step counter (hipGraph replay)
__device__ __forceinline__ uint32_t step_seed(uint32_t seed, const long long* seed_off) {
  return seed_off ? seed ^ ((uint32_t)(*seed_off) * 0x85EBCA6Bu) : seed;
}

// keep bit of attention-dropout element (bh, q, k)
__device__ __forceinline__ bool keep_elem(uint32_t seed, int bh, int q, int k, uint32_t thr) {
  const uint32_t idx = ((uint32_t)bh * S + (uint32_t)q) * S + (uint32_t)k;
  return hash_u32(idx * 0x9E3779B1u ^ seed) >= thr;
}

// DMA a [128 rows][64 cols] bf16 slice (row r at elements row0 + r * ld) into a 16 KiB image
template <class SW, int NWV = 4>
__device__ __forceinline__ void load_head(const bf16_t* t, int tbytes, long long row0, int ld, char* img, int wave,
                                          int lane) {
#pragma unroll
  for (int jj = 0; jj < 16 / NWV; ++jj) {
    const int j = wave + NWV * jj;                // 8-row block
    const int r = 8 * j + (lane >> 3);
    const int c = SW::f(r, lane & 7);             // logical chunk this lane's LDS slot holds
    const unsigned voff = (unsigned)((row0 + (long long)r * ld + c * 8) * 2);
    dma16(t, tbytes, img + j * 1024, voff, 0);
  }
}

// row-read fragment (16 rows x 32 k) of a 128-B-row image: lane -> row r0 + (l & 15), k chunk c0 + (l >> 4)
template <class SW>
__device__ __forceinline__ bf16x8_t row_frag(const char* img, int r0, int c0, int lane) {
  const int r = r0 + (lane & 15);
  const int c = c0 + (lane >> 4);
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(img + r * 128 + (SW::f(r, c) << 4)));
}

// same for a 256-B-row image
template <class SW>
__device__ __forceinline__ bf16x8_t row_frag256(const char* img, int r0, int c0, int lane) {
  const int r = r0 + (lane & 15);
  const int c = c0 + (lane >> 4);
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(img + r * 256 + (SW::f(r, c) << 4)));
}

// one ds_read_b64_tr_b16: rows r..r+3 of the lane's 16-lane group block, columns col0 + 4p
template <class SW, int ROWB>
__device__ __forceinline__ v4s tr4(const char* img, int r, int col) {
  const char* p = img + r * ROWB + (SW::f(r, col >> 3) << 4) + (col & 7) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p);
}

// transposed fragment: lane -> column col0 + (l & 15), k rows kb + 8g + (0..3) and kb + 8g + 4 + (0..3)
template <class SW, int ROWB>
__device__ __forceinline__ bf16x8_t tr_frag(const char* img, int kb, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  v4s lo = tr4<SW, ROWB>(img, kb + 8 * g + q, col0 + 4 * p);
  v4s hi = tr4<SW, ROWB>(img, kb + 8 * g + 4 + q, col0 + 4 * p);
  short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, f);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ bf16x8_t load_frag_global(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}

// ============================================================================ forward
// MINW: minimum waves per SIMD the register allocation must allow (2: at most 256 registers, so
// two 4-wave workgroups share a CU; 1: the allocator may use up to 512)
template <int MINW>
__global__ void __launch_bounds__(NT, MINW) attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                      bf16_t* __restrict__ out, float* __restrict__ lse_out, int B,
                                                      int nh, float scale, float p_drop, uint32_t seed,
                                                      const long long* __restrict__ seed_off) {
  seed = step_seed(seed, seed_off);
  __shared__ __attribute__((aligned(16))) char smem[2 * S * D * 2];
  char* Kimg = smem;
  char* Vimg = smem + S * D * 2;
  const int bh = blockIdx.x, b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long row0 = (long long)b * S * ld;
  const int tbytes = (int)((long long)B * S * ld * 2);

  load_head<SwzA>(qkv, tbytes, row0 + H + h * D, ld, Kimg, wave, lane);
  load_head<SwzV>(qkv, tbytes, row0 + 2 * H + h * D, ld, Vimg, wave, lane);
  bf16x8_t qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      const int q = 32 * wave + 16 * qt + li;
      qf[qt][ds] = load_frag_global(qkv + row0 + (long long)q * ld + h * D + 32 * ds + 8 * g);
    }
  float mk[8][4];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    if (mask) {
      const float4 m4 = *reinterpret_cast<const float4*>(mask + (long long)b * S + kt * 16 + 4 * g);
      mk[kt][0] = m4.x;
      mk[kt][1] = m4.y;
      mk[kt][2] = m4.z;
      mk[kt][3] = m4.w;
    } else {
      mk[kt][0] = mk[kt][1] = mk[kt][2] = mk[kt][3] = 0.f;
    }
  }
  wait_vmcnt<0>();
  __syncthreads();

  // S^T[k][q] = K Q^T
  float4v sacc[8][2];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) sacc[kt][qt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ds = 0; ds < 2; ++ds)
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      const bf16x8_t kf = row_frag<SwzA>(Kimg, kt * 16, 4 * ds, lane);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) sacc[kt][qt] = mfma(kf, qf[qt][ds], sacc[kt][qt]);
    }

  // softmax over keys for each query column (scale, mask), dropout, logsumexp
  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float m = -3.0e38f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float s = sacc[kt][qt][i] * scale + mk[kt][i];
        sacc[kt][qt][i] = s;
        m = fmaxf(m, s);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __expf(sacc[kt][qt][i] - m);
        sacc[kt][qt][i] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    const int q = 32 * wave + 16 * qt + li;
    if (g == 0) lse_out[(long long)bh * S + q] = m + __logf(sum);
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float p = sacc[kt][qt][i] * inv;
        if (thr) p = keep_elem(seed, bh, q, kt * 16 + 4 * g + i, thr) ? p * inv_keep : 0.f;
        sacc[kt][qt][i] = p;
      }
  }

  // O^T[d][q] = V^T P^T ; key order inside each 32-key step: {4g..4g+3, 16+4g..16+4g+3}
  float4v oacc[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) oacc[dt][qt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    bf16x8_t pf[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float4v a0 = sacc[2 * ks][qt], a1 = sacc[2 * ks + 1][qt];
      uint4 w = make_uint4(pack2(a0[0], a0[1]), pack2(a0[2], a0[3]), pack2(a1[0], a1[1]), pack2(a1[2], a1[3]));
      pf[qt] = __builtin_bit_cast(bf16x8_t, w);
    }
    const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      v4s lo = tr4<SwzV, 128>(Vimg, 32 * ks + 4 * g + q4, dt * 16 + 4 * p4);
      v4s hi = tr4<SwzV, 128>(Vimg, 32 * ks + 16 + 4 * g + q4, dt * 16 + 4 * p4);
      short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const bf16x8_t vf = __builtin_bit_cast(bf16x8_t, f);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) oacc[dt][qt] = mfma(vf, pf[qt], oacc[dt][qt]);
    }
  }
  // context rows [b*S + q][h*D + d]: lane holds 4 consecutive d of one query
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * wave + 16 * qt + li;
    bf16_t* o = out + ((long long)b * S + q) * H + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float4v v = oacc[dt][qt];
      *reinterpret_cast<uint2*>(o + dt * 16 + 4 * g) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}

// ============================================================================ backward
constexpr int kBwdLds = 5 * S * D * 2 + 2 * S * S * 2;   // K_A V_A K_T Q_T dO_T | P dS  = 144 KiB

// BW waves per workgroup (8: 16 queries / keys per wave; twice the waves per CU of the 4-wave
// version at the same 144 KiB of LDS, which allows one workgroup per CU)
template <int BW>
__global__ void __launch_bounds__(64 * BW) attn_bwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                      const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                      const float* __restrict__ lse, bf16_t* __restrict__ dqkv, int B,
                                                      int nh, float scale, float p_drop, uint32_t seed,
                                                      const long long* __restrict__ seed_off) {
  constexpr int QPW = S / BW, NQT = QPW / 16;     // rows per wave, 16-row tiles per wave
  static_assert(NQT >= 1 && NQT * 16 * BW == S, "waves");
  seed = step_seed(seed, seed_off);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* KA = smem;
  char* VA = KA + S * D * 2;
  char* KT = VA + S * D * 2;
  char* QT = KT + S * D * 2;
  char* OT = QT + S * D * 2;
  char* PI = OT + S * D * 2;        // P_drop [q][k]
  char* SI = PI + S * S * 2;        // dS     [q][k]
  const int bh = blockIdx.x, b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long row0 = (long long)b * S * ld;
  const long long orow0 = (long long)b * S * H;
  const int tbytes = (int)((long long)B * S * ld * 2);
  const int obytes = (int)((long long)B * S * H * 2);

  load_head<SwzA, BW>(qkv, tbytes, row0 + H + h * D, ld, KA, wave, lane);
  load_head<SwzA, BW>(qkv, tbytes, row0 + 2 * H + h * D, ld, VA, wave, lane);
  load_head<SwzT, BW>(qkv, tbytes, row0 + H + h * D, ld, KT, wave, lane);
  load_head<SwzT, BW>(qkv, tbytes, row0 + h * D, ld, QT, wave, lane);
  load_head<SwzT, BW>(dout, obytes, orow0 + h * D, H, OT, wave, lane);

  // phase-1 register operands: Q and dO fragments (B operands), D = rowsum(dO * O), lse, mask
  bf16x8_t qf[NQT][2], of[NQT][2];
  float Dq[NQT], lq[NQT];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    const int q = QPW * wave + 16 * qt + li;
    float part = 0.f;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      const int d = 32 * ds + 8 * g;
      qf[qt][ds] = load_frag_global(qkv + row0 + (long long)q * ld + h * D + d);
      of[qt][ds] = load_frag_global(dout + orow0 + (long long)q * H + h * D + d);
      float o8[8], do8[8];
      load_bf8(out + orow0 + (long long)q * H + h * D + d, o8);
      load_bf8(dout + orow0 + (long long)q * H + h * D + d, do8);
#pragma unroll
      for (int e = 0; e < 8; ++e) part += o8[e] * do8[e];
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    Dq[qt] = part;
    lq[qt] = lse[(long long)bh * S + q];
  }
  float mk[8][4];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    if (mask) {
      const float4 m4 = *reinterpret_cast<const float4*>(mask + (long long)b * S + kt * 16 + 4 * g);
      mk[kt][0] = m4.x;
      mk[kt][1] = m4.y;
      mk[kt][2] = m4.z;
      mk[kt][3] = m4.w;
    } else {
      mk[kt][0] = mk[kt][1] = mk[kt][2] = mk[kt][3] = 0.f;
    }
  }
  wait_vmcnt<0>();
  __syncthreads();

  // ---- phase 1: S^T and dP'^T = V dO^T for this wave's 32 queries
  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  {
    float4v sacc[8][NQT], pacc[8][NQT];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt) sacc[kt][qt] = pacc[kt][qt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < 2; ++ds)
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        const bf16x8_t kf = row_frag<SwzA>(KA, kt * 16, 4 * ds, lane);
        const bf16x8_t vf = row_frag<SwzA>(VA, kt * 16, 4 * ds, lane);
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) {
          sacc[kt][qt] = mfma(kf, qf[qt][ds], sacc[kt][qt]);
          pacc[kt][qt] = mfma(vf, of[qt][ds], pacc[kt][qt]);
        }
      }
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
      const int q = QPW * wave + 16 * qt + li;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        float pd[4], dsv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = kt * 16 + 4 * g + i;
          const float p = __expf(sacc[kt][qt][i] * scale + mk[kt][i] - lq[qt]);
          float dp = pacc[kt][qt][i];
          float pk = p;
          if (thr) {
            const bool keep = keep_elem(seed, bh, q, k, thr);
            pk = keep ? p * inv_keep : 0.f;
            dp = keep ? dp * inv_keep : 0.f;
          }
          pd[i] = pk;
          dsv[i] = p * (dp - Dq[qt]);
        }
        const int k0 = kt * 16 + 4 * g;
        const int off = q * 256 + (Swz256::f(q, k0 >> 3) << 4) + (k0 & 7) * 2;
        *reinterpret_cast<uint2*>(PI + off) = make_uint2(pack2(pd[0], pd[1]), pack2(pd[2], pd[3]));
        *reinterpret_cast<uint2*>(SI + off) = make_uint2(pack2(dsv[0], dsv[1]), pack2(dsv[2], dsv[3]));
      }
    }
  }
  __syncthreads();

  // ---- phase 2a: dV^T[d][k] = dO^T P_drop, dK^T[d][k] = scale Q^T dS for keys 32w .. 32w+31
  {
    float4v vacc[4][NQT], kacc[4][NQT];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int kt = 0; kt < NQT; ++kt) vacc[dt][kt] = kacc[dt][kt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {          // 32 queries per step
      bf16x8_t pf[NQT], sf[NQT];
#pragma unroll
      for (int kt = 0; kt < NQT; ++kt) {
        pf[kt] = tr_frag<Swz256, 256>(PI, 32 * ks, QPW * wave + 16 * kt, lane);
        sf[kt] = tr_frag<Swz256, 256>(SI, 32 * ks, QPW * wave + 16 * kt, lane);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8_t df = tr_frag<SwzT, 128>(OT, 32 * ks, dt * 16, lane);
        const bf16x8_t qq = tr_frag<SwzT, 128>(QT, 32 * ks, dt * 16, lane);
#pragma unroll
        for (int kt = 0; kt < NQT; ++kt) {
          vacc[dt][kt] = mfma(df, pf[kt], vacc[dt][kt]);
          kacc[dt][kt] = mfma(qq, sf[kt], kacc[dt][kt]);
        }
      }
    }
#pragma unroll
    for (int kt = 0; kt < NQT; ++kt) {
      const int k = QPW * wave + 16 * kt + li;
      bf16_t* rowp = dqkv + row0 + (long long)k * ld + h * D;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float4v kv = kacc[dt][kt], vv = vacc[dt][kt];
        *reinterpret_cast<uint2*>(rowp + H + dt * 16 + 4 * g) =
            make_uint2(pack2(kv[0] * scale, kv[1] * scale), pack2(kv[2] * scale, kv[3] * scale));
        *reinterpret_cast<uint2*>(rowp + 2 * H + dt * 16 + 4 * g) =
            make_uint2(pack2(vv[0], vv[1]), pack2(vv[2], vv[3]));
      }
    }
  }
  // ---- phase 2b: dQ^T[d][q] = scale K^T dS^T for this wave's queries
  {
    float4v qacc[4][NQT];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt) qacc[dt][qt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {          // 32 keys per step
      bf16x8_t sf[NQT];
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt) sf[qt] = row_frag256<Swz256>(SI, QPW * wave + 16 * qt, 4 * ks, lane);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8_t kf = tr_frag<SwzT, 128>(KT, 32 * ks, dt * 16, lane);
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) qacc[dt][qt] = mfma(kf, sf[qt], qacc[dt][qt]);
      }
    }
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
      const int q = QPW * wave + 16 * qt + li;
      bf16_t* rowp = dqkv + row0 + (long long)q * ld + h * D;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float4v v = qacc[dt][qt];
        *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * g) =
            make_uint2(pack2(v[0] * scale, v[1] * scale), pack2(v[2] * scale, v[3] * scale));
      }
    }
  }
}

// ============================================================================ backward v2
// One workgroup per (b, h), 8 waves; wave w owns keys 16w..16w+15 (phase A: dK, dV) and queries 16w..16w+15
// (phase B: dQ).  Every product takes its operands from registers or the four LDS images, and every
// intermediate of the softmax backward stays in registers:
//   phase A (per 32-query step): S = Q K^T and dP = dO V^T with the queries on the MFMA rows (Q / dO row
//     fragments from LDS, this wave's K / V fragments held in registers), P and dS = P (dP - D) per element,
//     then dV^T += dO^T P and dK^T += Q^T dS with P / dS packed straight from the accumulators as B operands
//     (query order {4g..4g+3, 16+4g..16+4g+3} of the step) and dO^T / Q^T read transposed under the same order;
//   phase B (per 32-key step): S^T = K Q^T and dP^T = V dO^T (this wave's Q / dO fragments in registers),
//     dS^T, then dQ^T += K^T dS^T.
// S and dP are recomputed per phase (7 products instead of 5) so no [q][k] image is written, read back or
// barrier-separated: LDS holds Q, K, V, dO (64 KiB, one SwzV layout that is conflict-free for both the
// 16-row ds_read_b128 and the ds_read_b64_tr_b16 patterns) + lse / D / mask vectors, so two workgroups share
// a CU.  (v1 above: one workgroup per CU, 144 KiB with [q][k] images of P and dS.)
constexpr int kBwd2Lds = 4 * S * D * 2 + 3 * S * 4;

__global__ void __launch_bounds__(512, 2) attn_bwd_v2(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                    const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                    const float* __restrict__ lse, bf16_t* __restrict__ dqkv, int B,
                                                    int nh, float scale, float p_drop, uint32_t seed,
                                                    const long long* __restrict__ seed_off) {
  seed = step_seed(seed, seed_off);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* QI = smem;
  char* KI = QI + S * D * 2;
  char* VI = KI + S * D * 2;
  char* OI = VI + S * D * 2;                  // dO
  float* LS = reinterpret_cast<float*>(OI + S * D * 2);
  float* DV = LS + S;                         // D = rowsum(dO * O)
  float* MK = DV + S;                         // additive key mask
  const int bh = blockIdx.x, b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long row0 = (long long)b * S * ld;
  const long long orow0 = (long long)b * S * H;
  const int tbytes = (int)((long long)B * S * ld * 2);
  const int obytes = (int)((long long)B * S * H * 2);

  load_head<SwzV, 8>(qkv, tbytes, row0 + h * D, ld, QI, wave, lane);
  load_head<SwzV, 8>(qkv, tbytes, row0 + H + h * D, ld, KI, wave, lane);
  load_head<SwzV, 8>(qkv, tbytes, row0 + 2 * H + h * D, ld, VI, wave, lane);
  load_head<SwzV, 8>(dout, obytes, orow0 + h * D, H, OI, wave, lane);

  // register operands: row 16*wave + li is this lane's query (phase B) and its key (phase A)
  const int r = 16 * wave + li;
  bf16x8_t qf[2], of[2], kf[2], vf[2];
  float part = 0.f;
#pragma unroll
  for (int ds = 0; ds < 2; ++ds) {
    const int d = 32 * ds + 8 * g;
    qf[ds] = load_frag_global(qkv + row0 + (long long)r * ld + h * D + d);
    kf[ds] = load_frag_global(qkv + row0 + (long long)r * ld + H + h * D + d);
    vf[ds] = load_frag_global(qkv + row0 + (long long)r * ld + 2 * H + h * D + d);
    of[ds] = load_frag_global(dout + orow0 + (long long)r * H + h * D + d);
    float o8[8], do8[8];
    load_bf8(out + orow0 + (long long)r * H + h * D + d, o8);
    load_bf8(dout + orow0 + (long long)r * H + h * D + d, do8);
#pragma unroll
    for (int e = 0; e < 8; ++e) part += o8[e] * do8[e];
  }
  part += __shfl_xor(part, 16, 64);
  part += __shfl_xor(part, 32, 64);
  const float lq = lse[(long long)bh * S + r];
  const float mr = mask ? mask[(long long)b * S + r] : 0.f;
  if (g == 0) {
    LS[r] = lq;
    DV[r] = part;
    MK[r] = mr;
  }
  wait_vmcnt<0>();
  __syncthreads();

  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const int q4 = li >> 2, p4 = li & 3;

  // ---- phase A: keys r (lane column) -- dV^T[d][k] = dO^T P, dK^T[d][k] = Q^T dS over all queries
  {
    float4v dvacc[4], dkacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dvacc[dt] = dkacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < 4; ++s) {                       // queries 32s .. 32s+31
      float4v sc[2], dp[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) sc[t] = dp[t] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8_t qa = row_frag<SwzV>(QI, 32 * s + 16 * t, 4 * ds, lane);
          const bf16x8_t oa = row_frag<SwzV>(OI, 32 * s + 16 * t, 4 * ds, lane);
          sc[t] = mfma(qa, kf[ds], sc[t]);
          dp[t] = mfma(oa, vf[ds], dp[t]);
        }
      float pv[8], sv[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int q0 = 32 * s + 16 * t + 4 * g;       // this lane's 4 queries of the tile
        const float4 l4 = *reinterpret_cast<const float4*>(LS + q0);
        const float4 d4 = *reinterpret_cast<const float4*>(DV + q0);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __expf(sc[t][i] * scale + mr - lv[i]);
          float dpv = dp[t][i], pk = p;
          if (thr) {
            const bool keep = keep_elem(seed, bh, q0 + i, r, thr);
            pk = keep ? p * inv_keep : 0.f;
            dpv = keep ? dpv * inv_keep : 0.f;
          }
          pv[4 * t + i] = pk;
          sv[4 * t + i] = p * (dpv - dv[i]);
        }
      }
      const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(pv[0], pv[1]), pack2(pv[2], pv[3]),
                                                                  pack2(pv[4], pv[5]), pack2(pv[6], pv[7])));
      const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]),
                                                                  pack2(sv[4], sv[5]), pack2(sv[6], sv[7])));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        v4s lo = tr4<SwzV, 128>(OI, 32 * s + 4 * g + q4, dt * 16 + 4 * p4);
        v4s hi = tr4<SwzV, 128>(OI, 32 * s + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 fo = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        dvacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fo), pf, dvacc[dt]);
        lo = tr4<SwzV, 128>(QI, 32 * s + 4 * g + q4, dt * 16 + 4 * p4);
        hi = tr4<SwzV, 128>(QI, 32 * s + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 fq = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        dkacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fq), sf, dkacc[dt]);
      }
    }
    bf16_t* rowp = dqkv + row0 + (long long)r * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float4v kv = dkacc[dt], vv = dvacc[dt];
      *reinterpret_cast<uint2*>(rowp + H + dt * 16 + 4 * g) =
          make_uint2(pack2(kv[0] * scale, kv[1] * scale), pack2(kv[2] * scale, kv[3] * scale));
      *reinterpret_cast<uint2*>(rowp + 2 * H + dt * 16 + 4 * g) = make_uint2(pack2(vv[0], vv[1]), pack2(vv[2], vv[3]));
    }
  }

  // ---- phase B: query r (lane column) -- dQ^T[d][q] = K^T dS^T over all keys
  {
    float4v qacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) qacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < 4; ++ks) {                    // keys 32ks .. 32ks+31
      float4v sc[2], dp[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) sc[t] = dp[t] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8_t ka = row_frag<SwzV>(KI, 32 * ks + 16 * t, 4 * ds, lane);
          const bf16x8_t va = row_frag<SwzV>(VI, 32 * ks + 16 * t, 4 * ds, lane);
          sc[t] = mfma(ka, qf[ds], sc[t]);
          dp[t] = mfma(va, of[ds], dp[t]);
        }
      float sv[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k0 = 32 * ks + 16 * t + 4 * g;       // this lane's 4 keys of the tile
        const float4 m4 = *reinterpret_cast<const float4*>(MK + k0);
        const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __expf(sc[t][i] * scale + mv[i] - lq);
          float dpv = dp[t][i];
          if (thr) dpv = keep_elem(seed, bh, r, k0 + i, thr) ? dpv * inv_keep : 0.f;
          sv[4 * t + i] = p * (dpv - part);
        }
      }
      const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]),
                                                                  pack2(sv[4], sv[5]), pack2(sv[6], sv[7])));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        v4s lo = tr4<SwzV, 128>(KI, 32 * ks + 4 * g + q4, dt * 16 + 4 * p4);
        v4s hi = tr4<SwzV, 128>(KI, 32 * ks + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 fk = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        qacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fk), sf, qacc[dt]);
      }
    }
    bf16_t* rowp = dqkv + row0 + (long long)r * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float4v v = qacc[dt];
      *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * g) =
          make_uint2(pack2(v[0] * scale, v[1] * scale), pack2(v[2] * scale, v[3] * scale));
    }
  }
}

// ============================================================================ backward v2, split phases (round 6)
// attn_bwd_v2's two phases as separate workgroups: block 2 bh runs phase A (dK, dV: Q and dO images in LDS, this
// wave's K / V rows in registers), block 2 bh + 1 phase B (dQ: K and V images, this wave's Q / dO rows).  Each
// phase needs only two of the four 16 KiB images, so a workgroup does half the work on half the LDS.  Why: 768
// (batch, head) items on 512 slots of the one-workgroup-per-item kernel run as 1.5 rounds of whole items; 1536
// half items on 512 slots are 3 full rounds of half items.  The per-lane D = rowsum(dO * O) of the lane's row is
// computed by both phases (phase A needs it for every query, phase B for its own).  Numerics, dropout bits and
// outputs are those of attn_bwd_v2.  Measured in the BERT-base step: -0.8 % (two workgroups per CU), -3.5 % with
// the 80-register build (three per CU, spills): the backward is bound by its operand loads, which the split
// repeats (both halves load their rows' Q / dO / O), not by the half-empty last round.  MDTF_ATTN_BWD=v2s: opt-in.
constexpr int kBwd2sLds = 2 * S * D * 2 + 3 * S * 4;

// MINB: 512-thread workgroups per CU the register allocation must allow (launch bound 2 MINB waves per SIMD; 2:
// <= 128 VGPRs; 3: <= 80, 1536 half items in 2 rounds of 768 slots)
template <int MINB>
__global__ void __launch_bounds__(512, 2 * MINB) attn_bwd_v2s(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                     const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                     const float* __restrict__ lse, bf16_t* __restrict__ dqkv, int B,
                                                     int nh, float scale, float p_drop, uint32_t seed,
                                                     const long long* __restrict__ seed_off) {
  seed = step_seed(seed, seed_off);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* I0 = smem;                            // phase A: Q    phase B: K
  char* I1 = I0 + S * D * 2;                  // phase A: dO   phase B: V
  float* LS = reinterpret_cast<float*>(I1 + S * D * 2);
  float* DV = LS + S;                         // D = rowsum(dO * O)
  float* MK = DV + S;                         // additive key mask
  const int bh = blockIdx.x >> 1, phase = blockIdx.x & 1;
  const int b = bh / nh, h = bh - b * nh;
  const int H = nh * D, ld = 3 * H;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const long long row0 = (long long)b * S * ld;
  const long long orow0 = (long long)b * S * H;
  const int tbytes = (int)((long long)B * S * ld * 2);
  const int obytes = (int)((long long)B * S * H * 2);

  if (phase == 0) {
    load_head<SwzV, 8>(qkv, tbytes, row0 + h * D, ld, I0, wave, lane);
    load_head<SwzV, 8>(dout, obytes, orow0 + h * D, H, I1, wave, lane);
  } else {
    load_head<SwzV, 8>(qkv, tbytes, row0 + H + h * D, ld, I0, wave, lane);
    load_head<SwzV, 8>(qkv, tbytes, row0 + 2 * H + h * D, ld, I1, wave, lane);
  }
  // register operands of row 16*wave + li: phase A its key (K, V rows), phase B its query (Q, dO rows)
  const int r = 16 * wave + li;
  bf16x8_t f0[2], f1[2];
  float part = 0.f;
#pragma unroll
  for (int ds = 0; ds < 2; ++ds) {
    const int d = 32 * ds + 8 * g;
    if (phase == 0) {
      f0[ds] = load_frag_global(qkv + row0 + (long long)r * ld + H + h * D + d);
      f1[ds] = load_frag_global(qkv + row0 + (long long)r * ld + 2 * H + h * D + d);
    } else {
      f0[ds] = load_frag_global(qkv + row0 + (long long)r * ld + h * D + d);
      f1[ds] = load_frag_global(dout + orow0 + (long long)r * H + h * D + d);
    }
    float o8[8], do8[8];
    load_bf8(out + orow0 + (long long)r * H + h * D + d, o8);
    load_bf8(dout + orow0 + (long long)r * H + h * D + d, do8);
#pragma unroll
    for (int e = 0; e < 8; ++e) part += o8[e] * do8[e];
  }
  part += __shfl_xor(part, 16, 64);
  part += __shfl_xor(part, 32, 64);
  const float lq = lse[(long long)bh * S + r];
  const float mr = mask ? mask[(long long)b * S + r] : 0.f;
  if (g == 0) {
    LS[r] = lq;
    DV[r] = part;
    MK[r] = mr;
  }
  wait_vmcnt<0>();
  __syncthreads();

  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const int q4 = li >> 2, p4 = li & 3;

  if (phase == 0) {
    // ---- phase A: keys r (lane column) -- dV^T[d][k] = dO^T P, dK^T[d][k] = Q^T dS over all queries
    const char* QI = I0;
    const char* OI = I1;
    float4v dvacc[4], dkacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dvacc[dt] = dkacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < 4; ++s) {                       // queries 32s .. 32s+31
      float4v sc[2], dp[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) sc[t] = dp[t] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8_t qa = row_frag<SwzV>(QI, 32 * s + 16 * t, 4 * ds, lane);
          const bf16x8_t oa = row_frag<SwzV>(OI, 32 * s + 16 * t, 4 * ds, lane);
          sc[t] = mfma(qa, f0[ds], sc[t]);
          dp[t] = mfma(oa, f1[ds], dp[t]);
        }
      float pv[8], sv[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int q0 = 32 * s + 16 * t + 4 * g;       // this lane's 4 queries of the tile
        const float4 l4 = *reinterpret_cast<const float4*>(LS + q0);
        const float4 d4 = *reinterpret_cast<const float4*>(DV + q0);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __expf(sc[t][i] * scale + mr - lv[i]);
          float dpv = dp[t][i], pk = p;
          if (thr) {
            const bool keep = keep_elem(seed, bh, q0 + i, r, thr);
            pk = keep ? p * inv_keep : 0.f;
            dpv = keep ? dpv * inv_keep : 0.f;
          }
          pv[4 * t + i] = pk;
          sv[4 * t + i] = p * (dpv - dv[i]);
        }
      }
      const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(pv[0], pv[1]), pack2(pv[2], pv[3]),
                                                                  pack2(pv[4], pv[5]), pack2(pv[6], pv[7])));
      const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]),
                                                                  pack2(sv[4], sv[5]), pack2(sv[6], sv[7])));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        v4s lo = tr4<SwzV, 128>(OI, 32 * s + 4 * g + q4, dt * 16 + 4 * p4);
        v4s hi = tr4<SwzV, 128>(OI, 32 * s + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 fo = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        dvacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fo), pf, dvacc[dt]);
        lo = tr4<SwzV, 128>(QI, 32 * s + 4 * g + q4, dt * 16 + 4 * p4);
        hi = tr4<SwzV, 128>(QI, 32 * s + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 fq = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        dkacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fq), sf, dkacc[dt]);
      }
    }
    bf16_t* rowp = dqkv + row0 + (long long)r * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float4v kv = dkacc[dt], vv = dvacc[dt];
      *reinterpret_cast<uint2*>(rowp + H + dt * 16 + 4 * g) =
          make_uint2(pack2(kv[0] * scale, kv[1] * scale), pack2(kv[2] * scale, kv[3] * scale));
      *reinterpret_cast<uint2*>(rowp + 2 * H + dt * 16 + 4 * g) = make_uint2(pack2(vv[0], vv[1]), pack2(vv[2], vv[3]));
    }
  } else {
    // ---- phase B: query r (lane column) -- dQ^T[d][q] = K^T dS^T over all keys
    const char* KI = I0;
    const char* VI = I1;
    float4v qacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) qacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < 4; ++ks) {                    // keys 32ks .. 32ks+31
      float4v sc[2], dp[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) sc[t] = dp[t] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8_t ka = row_frag<SwzV>(KI, 32 * ks + 16 * t, 4 * ds, lane);
          const bf16x8_t va = row_frag<SwzV>(VI, 32 * ks + 16 * t, 4 * ds, lane);
          sc[t] = mfma(ka, f0[ds], sc[t]);
          dp[t] = mfma(va, f1[ds], dp[t]);
        }
      float sv[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k0 = 32 * ks + 16 * t + 4 * g;       // this lane's 4 keys of the tile
        const float4 m4 = *reinterpret_cast<const float4*>(MK + k0);
        const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __expf(sc[t][i] * scale + mv[i] - lq);
          float dpv = dp[t][i];
          if (thr) dpv = keep_elem(seed, bh, r, k0 + i, thr) ? dpv * inv_keep : 0.f;
          sv[4 * t + i] = p * (dpv - part);
        }
      }
      const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]),
                                                                  pack2(sv[4], sv[5]), pack2(sv[6], sv[7])));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        v4s lo = tr4<SwzV, 128>(KI, 32 * ks + 4 * g + q4, dt * 16 + 4 * p4);
        v4s hi = tr4<SwzV, 128>(KI, 32 * ks + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 fk = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        qacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fk), sf, qacc[dt]);
      }
    }
    bf16_t* rowp = dqkv + row0 + (long long)r * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float4v v = qacc[dt];
      *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * g) =
          make_uint2(pack2(v[0] * scale, v[1] * scale), pack2(v[2] * scale, v[3] * scale));
    }
  }
}

// ============================================================================ persistent forms (round 5)
// The kernels above give each (batch, head) item its own workgroup: every workgroup pays one HBM load latency,
// computes for ~1 us, then stores, so the chip streams at about half the HBM rate (attn_fwd 20 us for 50 MB,
// attn_bwd_v2 39 us for 100 MB at BERT-base batch 64; 768 items on 512 backward slots also leave a half wave).
// The persistent forms run ONE workgroup per CU that walks items bh = blockIdx.x, + gridDim.x, ...: the operands
// of item i+1 go to the other half of a double-buffered LDS by LDS-DMA while item i computes, and item i's stores
// drain under item i+1's loads.  The DMA is inline asm (invisible to the compiler, so it adds no vmcnt(0) in
// front of the LDS reads); every wave waits for its own DMA with a counted vmcnt that leaves only the previous
// item's stores (the youngest vector-memory operations) in flight, and an s_barrier then makes every wave's DMA
// visible and frees the other buffer.  Numerics and dropout bits are those of the per-item kernels.
constexpr int kImg = S * D * 2;                 // one [128][64] bf16 head slice
constexpr int kFwdBuf = 3 * kImg + 1024;        // Q | K | V | key mask (512 B used)
constexpr int kFwdPpLds = 2 * kFwdBuf;
constexpr int kFwdPpStores = 5;                 // per wave and item: 4 context stores + 1 logsumexp store
constexpr unsigned kOOBoff = 0x80000000u;

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 8 waves, wave w = queries 16w .. 16w+15 of the item
__global__ void __launch_bounds__(512) attn_fwd_pp(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                   bf16_t* __restrict__ out, float* __restrict__ lse_out, int B,
                                                   int nh, float scale, float p_drop, uint32_t seed,
                                                   const long long* __restrict__ seed_off) {
  seed = step_seed(seed, seed_off);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int H = nh * D, ld = 3 * H;
  const int nitems = B * nh;
  const i32x4_t rq = buffer_rsrc(qkv, (int)((long long)B * S * ld * 2));
  const i32x4_t rm = buffer_rsrc(mask, mask ? B * S * 4 : 0);
  const bool has_mask = mask != nullptr;

  // this wave's share of item bh's loads: 1-KiB blocks j = wave, wave + 8 of Q, K (row-read swizzle) and V
  // (transposed-read swizzle); the key mask (512 B) by wave 0
  auto issue = [&](int bh, char* buf) {
    const int b = bh / nh, h = bh - b * nh;
    const long long row0 = (long long)b * S * ld;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wave + 8 * jj;
      const int r = 8 * j + (lane >> 3);
      const unsigned base = (unsigned)((row0 + (long long)r * ld + h * D) * 2);
      dma16_asm(rq, buf + j * 1024, base + (SwzA::f(r, lane & 7) << 4));
      dma16_asm(rq, buf + kImg + j * 1024, base + H * 2 + (SwzA::f(r, lane & 7) << 4));
      dma16_asm(rq, buf + 2 * kImg + j * 1024, base + H * 4 + (SwzV::f(r, lane & 7) << 4));
    }
    if (wave == 0 && has_mask) dma16_asm(rm, buf + 3 * kImg, lane < 32 ? (unsigned)(b * S * 4 + lane * 16) : kOOBoff);
  };

  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const int q = 16 * wave + li;                  // this lane's query (column of S^T / O^T)
  int bh = blockIdx.x;
  if (bh < nitems) issue(bh, smem);
  for (int it = 0; bh < nitems; ++it, bh += gridDim.x) {
    // this wave's DMA of item bh landed (only the previous item's stores are younger), then every wave's
    if (it == 0) wait_vmcnt<0>();
    else wait_vmcnt<kFwdPpStores>();
    pp_barrier();
    char* buf = smem + (it & 1) * kFwdBuf;
    if (bh + (int)gridDim.x < nitems) issue(bh + gridDim.x, smem + ((it + 1) & 1) * kFwdBuf);
    const char* Qimg = buf;
    const char* Kimg = buf + kImg;
    const char* Vimg = buf + 2 * kImg;
    const float* Mimg = reinterpret_cast<const float*>(buf + 3 * kImg);
    const int b = bh / nh, h = bh - b * nh;

    bf16x8_t qf[2];
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) qf[ds] = row_frag<SwzA>(Qimg, 16 * wave, 4 * ds, lane);
    // S^T[k][q] = K Q^T
    float4v sacc[8];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) sacc[kt] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < 2; ++ds)
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) sacc[kt] = mfma(row_frag<SwzA>(Kimg, kt * 16, 4 * ds, lane), qf[ds], sacc[kt]);
    // softmax over keys (scale, additive key mask), dropout, logsumexp
    float m = -3.0e38f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      const float4 m4 = has_mask ? *reinterpret_cast<const float4*>(Mimg + kt * 16 + 4 * g) : make_float4(0, 0, 0, 0);
      const float mk[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float s = sacc[kt][i] * scale + mk[i];
        sacc[kt][i] = s;
        m = fmaxf(m, s);
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __expf(sacc[kt][i] - m);
        sacc[kt][i] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float p = sacc[kt][i] * inv;
        if (thr) p = keep_elem(seed, bh, q, kt * 16 + 4 * g + i, thr) ? p * inv_keep : 0.f;
        sacc[kt][i] = p;
      }
    // O^T[d][q] = V^T P^T (key order inside each 32-key step: {4g..4g+3, 16+4g..16+4g+3})
    float4v oacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
    const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float4v a0 = sacc[2 * ks], a1 = sacc[2 * ks + 1];
      const bf16x8_t pf = __builtin_bit_cast(
          bf16x8_t, make_uint4(pack2(a0[0], a0[1]), pack2(a0[2], a0[3]), pack2(a1[0], a1[1]), pack2(a1[2], a1[3])));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        v4s lo = tr4<SwzV, 128>(Vimg, 32 * ks + 4 * g + q4, dt * 16 + 4 * p4);
        v4s hi = tr4<SwzV, 128>(Vimg, 32 * ks + 16 + 4 * g + q4, dt * 16 + 4 * p4);
        short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        oacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, f), pf, oacc[dt]);
      }
    }
    // stores (kFwdPpStores vector-memory instructions per wave): logsumexp, then 4 x 8 B of context per lane
    lse_out[(long long)bh * S + q] = m + __logf(sum);      // (every lane: lanes of one query store equal values)
    bf16_t* o = out + ((long long)b * S + q) * H + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float4v v = oacc[dt];
      *reinterpret_cast<uint2*>(o + dt * 16 + 4 * g) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
}

// Backward: 16 waves.  Waves 0-7 = phase A of attn_bwd_v2 for keys 16w .. 16w+15 (dK, dV), waves 8-15 = its
// phase B for queries 16(w-8) .. +15 (dQ), side by side instead of one after the other.  Per item: Q, K, V, dO
// images (SwzV), logsumexp and key mask by LDS-DMA into a double buffer; D = rowsum(dO * O) from O (one more
// LDS-DMA image, single-buffered: every wave reads back only the 1-KiB block its own lanes loaded, before it
// issues the next item's block) and dO, published through a small LDS vector behind a second barrier.
constexpr int kBwdBuf = 4 * kImg + 2048;        // Q | K | V | dO | lse (512 B used) | key mask (512 B used)
constexpr int kBwdPpLds = 2 * kBwdBuf + kImg + S * 4;  // + O + D
constexpr int kBwdStoresA = 8, kBwdStoresB = 4;

__global__ void __launch_bounds__(1024) attn_bwd_pp(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                    const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                    const float* __restrict__ lse, bf16_t* __restrict__ dqkv, int B,
                                                    int nh, float scale, float p_drop, uint32_t seed,
                                                    const long long* __restrict__ seed_off) {
  seed = step_seed(seed, seed_off);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Obuf = smem + 2 * kBwdBuf;
  float* DVs = reinterpret_cast<float*>(Obuf + kImg);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool phaseA = wave < 8;
  const int g = lane >> 4, li = lane & 15;
  const int H = nh * D, ld = 3 * H;
  const int nitems = B * nh;
  const i32x4_t rq = buffer_rsrc(qkv, (int)((long long)B * S * ld * 2));
  const i32x4_t ro = buffer_rsrc(dout, (int)((long long)B * S * H * 2));
  const i32x4_t rO = buffer_rsrc(out, (int)((long long)B * S * H * 2));
  const i32x4_t rl = buffer_rsrc(lse, nitems * S * 4);
  const i32x4_t rm = buffer_rsrc(mask, mask ? B * S * 4 : 0);
  const bool has_mask = mask != nullptr;

  // 64 1-KiB blocks (Q, K, V, dO; block j = 8-row block j & 15 of image j >> 4): wave w issues j = w + 16 t;
  // + block w of O (linear layout: lane l holds row 8w + l / 8, columns 8 (l & 7) .. +7)
  auto issue = [&](int bh, char* buf) {
    const int b = bh / nh, h = bh - b * nh;
    const long long row0 = (long long)b * S * ld, orow0 = (long long)b * S * H;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = wave + 16 * t;
      const int img = j >> 4, rb = j & 15;
      const int r = 8 * rb + (lane >> 3);
      const int c = SwzV::f(r, lane & 7);
      if (img < 3)
        dma16_asm(rq, buf + img * kImg + rb * 1024,
                  (unsigned)((row0 + (long long)r * ld + img * H + h * D + c * 8) * 2));
      else
        dma16_asm(ro, buf + 3 * kImg + rb * 1024, (unsigned)((orow0 + (long long)r * H + h * D + c * 8) * 2));
    }
    dma16_asm(rO, Obuf + wave * 1024,
              (unsigned)((orow0 + (long long)(8 * wave + (lane >> 3)) * H + h * D + (lane & 7) * 8) * 2));
    if (wave == 0) dma16_asm(rl, buf + 4 * kImg, lane < 32 ? (unsigned)(bh * S * 4 + lane * 16) : kOOBoff);
    if (wave == 1 && has_mask)
      dma16_asm(rm, buf + 4 * kImg + 1024, lane < 32 ? (unsigned)(b * S * 4 + lane * 16) : kOOBoff);
  };
  const int drow = 8 * wave + (lane >> 3), dc = lane & 7;

  const uint32_t thr = p_drop > 0.f ? (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f) : 0u;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const int q4 = li >> 2, p4 = li & 3;
  const int r = 16 * (wave & 7) + li;            // phase A: this lane's key; phase B: its query
  int bh = blockIdx.x;
  if (bh < nitems) issue(bh, smem);
  for (int it = 0; bh < nitems; ++it, bh += gridDim.x) {
    if (it == 0) wait_vmcnt<0>();
    else if (phaseA) wait_vmcnt<kBwdStoresA>();
    else wait_vmcnt<kBwdStoresB>();
    pp_barrier();
    const char* buf = smem + (it & 1) * kBwdBuf;
    const char* OI = buf + 3 * kImg;             // dO
    // D = rowsum(dO * O): 8 lanes per query row; O from this lane's own DMA slot (read before it is refilled)
    float part = 0.f;
    {
      const uint4 ov = *reinterpret_cast<const uint4*>(Obuf + wave * 1024 + lane * 16);
      const uint4 dv = *reinterpret_cast<const uint4*>(OI + drow * 128 + (SwzV::f(drow, dc) << 4));
      const uint32_t ow[4] = {ov.x, ov.y, ov.z, ov.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        part += __uint_as_float(ow[e] << 16) * __uint_as_float(dw[e] << 16) +
                __uint_as_float(ow[e] & 0xffff0000u) * __uint_as_float(dw[e] & 0xffff0000u);
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      part += __shfl_xor(part, 4, 64);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // the O slot has been read: it may be refilled
    const int nb = bh + gridDim.x;
    if (nb < nitems) issue(nb, smem + ((it + 1) & 1) * kBwdBuf);
    if (dc == 0) DVs[drow] = part;
    // raw barrier: a __syncthreads() fence would drain vmcnt, i.e. wait for the next item's DMA just issued
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_barrier();
    const char* QI = buf;
    const char* KI = buf + kImg;
    const char* VI = buf + 2 * kImg;
    const float* LS = reinterpret_cast<const float*>(buf + 4 * kImg);
    const float* MK = reinterpret_cast<const float*>(buf + 4 * kImg + 1024);
    const int b = bh / nh, h = bh - b * nh;
    bf16x8_t rf0[2], rf1[2];                     // A: this wave's K / V rows; B: its Q / dO rows
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      rf0[ds] = row_frag<SwzV>(phaseA ? KI : QI, 16 * (wave & 7), 4 * ds, lane);
      rf1[ds] = row_frag<SwzV>(phaseA ? VI : OI, 16 * (wave & 7), 4 * ds, lane);
    }
    bf16_t* rowp = dqkv + ((long long)b * S + r) * ld + h * D;
    if (phaseA) {
      // keys r (lane column): dV^T[d][k] = dO^T P, dK^T[d][k] = Q^T dS over all queries
      const float mr = has_mask ? MK[r] : 0.f;
      float4v dvacc[4], dkacc[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dvacc[dt] = dkacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < 4; ++s) {                     // queries 32s .. 32s+31
        float4v sc[2], dp[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) sc[t] = dp[t] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ds = 0; ds < 2; ++ds)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            sc[t] = mfma(row_frag<SwzV>(QI, 32 * s + 16 * t, 4 * ds, lane), rf0[ds], sc[t]);
            dp[t] = mfma(row_frag<SwzV>(OI, 32 * s + 16 * t, 4 * ds, lane), rf1[ds], dp[t]);
          }
        float pv[8], sv[8];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int q0 = 32 * s + 16 * t + 4 * g;       // this lane's 4 queries of the tile
          const float4 l4 = *reinterpret_cast<const float4*>(LS + q0);
          const float4 d4 = *reinterpret_cast<const float4*>(DVs + q0);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __expf(sc[t][i] * scale + mr - lv[i]);
            float dpv = dp[t][i], pk = p;
            if (thr) {
              const bool keep = keep_elem(seed, bh, q0 + i, r, thr);
              pk = keep ? p * inv_keep : 0.f;
              dpv = keep ? dpv * inv_keep : 0.f;
            }
            pv[4 * t + i] = pk;
            sv[4 * t + i] = p * (dpv - dv[i]);
          }
        }
        const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(pv[0], pv[1]), pack2(pv[2], pv[3]),
                                                                    pack2(pv[4], pv[5]), pack2(pv[6], pv[7])));
        const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]),
                                                                    pack2(sv[4], sv[5]), pack2(sv[6], sv[7])));
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          v4s lo = tr4<SwzV, 128>(OI, 32 * s + 4 * g + q4, dt * 16 + 4 * p4);
          v4s hi = tr4<SwzV, 128>(OI, 32 * s + 16 + 4 * g + q4, dt * 16 + 4 * p4);
          short8 fo = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          dvacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fo), pf, dvacc[dt]);
          lo = tr4<SwzV, 128>(QI, 32 * s + 4 * g + q4, dt * 16 + 4 * p4);
          hi = tr4<SwzV, 128>(QI, 32 * s + 16 + 4 * g + q4, dt * 16 + 4 * p4);
          short8 fq = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          dkacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fq), sf, dkacc[dt]);
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float4v kv = dkacc[dt], vv = dvacc[dt];
        *reinterpret_cast<uint2*>(rowp + H + dt * 16 + 4 * g) =
            make_uint2(pack2(kv[0] * scale, kv[1] * scale), pack2(kv[2] * scale, kv[3] * scale));
        *reinterpret_cast<uint2*>(rowp + 2 * H + dt * 16 + 4 * g) =
            make_uint2(pack2(vv[0], vv[1]), pack2(vv[2], vv[3]));
      }
    } else {
      // query r (lane column): dQ^T[d][q] = K^T dS^T over all keys
      const float lq = LS[r], part = DVs[r];
      float4v qacc[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) qacc[dt] = float4v{0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < 4; ++ks) {                  // keys 32ks .. 32ks+31
        float4v sc[2], dp[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) sc[t] = dp[t] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ds = 0; ds < 2; ++ds)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            sc[t] = mfma(row_frag<SwzV>(KI, 32 * ks + 16 * t, 4 * ds, lane), rf0[ds], sc[t]);
            dp[t] = mfma(row_frag<SwzV>(VI, 32 * ks + 16 * t, 4 * ds, lane), rf1[ds], dp[t]);
          }
        float sv[8];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int k0 = 32 * ks + 16 * t + 4 * g;       // this lane's 4 keys of the tile
          const float4 m4 = has_mask ? *reinterpret_cast<const float4*>(MK + k0) : make_float4(0, 0, 0, 0);
          const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __expf(sc[t][i] * scale + mv[i] - lq);
            float dpv = dp[t][i];
            if (thr) dpv = keep_elem(seed, bh, r, k0 + i, thr) ? dpv * inv_keep : 0.f;
            sv[4 * t + i] = p * (dpv - part);
          }
        }
        const bf16x8_t sf = __builtin_bit_cast(bf16x8_t, make_uint4(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]),
                                                                    pack2(sv[4], sv[5]), pack2(sv[6], sv[7])));
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          v4s lo = tr4<SwzV, 128>(KI, 32 * ks + 4 * g + q4, dt * 16 + 4 * p4);
          v4s hi = tr4<SwzV, 128>(KI, 32 * ks + 16 + 4 * g + q4, dt * 16 + 4 * p4);
          short8 fk = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          qacc[dt] = mfma(__builtin_bit_cast(bf16x8_t, fk), sf, qacc[dt]);
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float4v v = qacc[dt];
        *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * g) =
            make_uint2(pack2(v[0] * scale, v[1] * scale), pack2(v[2] * scale, v[3] * scale));
      }
    }
  }
}

}  // namespace

// persistent forms: 0 off, 1 on (one workgroup per CU), n >= 2 on with at most n workgroups (tests: several items per
// workgroup at small sizes); -1: from MDTF_ATTN_PP at the first call.  Default off: graph-timed at BERT-base's
// batch 64 x 12 heads they are slower than the per-item kernels (fwd 17.6 vs 16.7 us, bwd 37.1 vs 35.5 us,
// bench/attn_probe.py, profiles/ab_r5.md) -- three per-item workgroups per CU already keep as many loads in flight
// as the double buffer does.
static int g_attn_pp = -1;

// select the persistent S = 128 kernels (tests / A/B); returns the previous choice
MDTF_EXPORT int mdtf_set_attn_pp(int on) {
  const int prev = g_attn_pp;
  g_attn_pp = on;
  return prev;
}

static bool attn_pp_on() {
  if (g_attn_pp < 0) {
    const char* e = getenv("MDTF_ATTN_PP");
    g_attn_pp = (e && e[0] == '1') ? 1 : 0;
  }
  return g_attn_pp >= 1;
}

static int pp_grid(int items) {
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n;
  }();
  int g = items < cus ? items : cus;
  if (g_attn_pp >= 2 && g > g_attn_pp) g = g_attn_pp;
  return g;
}

// ctx[B*S, H] = attention(qkv[B*S, 3H]); lse [B*nh, S] (fp32) saved for backward
MDTF_EXPORT int mdtf_attn_fwd(const void* qkv, const float* mask, void* out, float* lse, int B, int seq, int nh,
                              int dh, float scale, float p_drop, unsigned seed, const long long* seed_off,
                              hipStream_t st) {
  if (seq != S || dh != D) return MDTF_EUNSUPPORTED;
  if ((long long)B * S * 3 * nh * D * 2 > 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  // MDTF_ATTN_FWD_MINW=1: no register cap (A/B switch)
  static const bool w1 = [] {
    const char* e = getenv("MDTF_ATTN_FWD_MINW");
    return e && e[0] == '1';
  }();
  if (attn_pp_on()) {
    hipLaunchKernelGGL(attn_fwd_pp, dim3(pp_grid(B * nh)), dim3(512), kFwdPpLds, st, (const bf16_t*)qkv, mask, (bf16_t*)out, lse,
                       B, nh, scale, p_drop, (uint32_t)seed, seed_off);
  } else if (w1)
    hipLaunchKernelGGL(attn_fwd_kernel<1>, dim3(B * nh), dim3(NT), 0, st, (const bf16_t*)qkv, mask, (bf16_t*)out, lse,
                       B, nh, scale, p_drop, (uint32_t)seed, seed_off);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<2>, dim3(B * nh), dim3(NT), 0, st, (const bf16_t*)qkv, mask, (bf16_t*)out, lse,
                       B, nh, scale, p_drop, (uint32_t)seed, seed_off);
  MDTF_LAUNCH_CHECK();
  return 0;
}

static int g_attn_bwd = -1;    // backward kernel version: 1 = v1, 2 = v2, 3 = v2s; -1: from MDTF_ATTN_BWD at the first call

// select the S = 128 backward kernel (tests / A/B); returns the previous choice
MDTF_EXPORT int mdtf_set_attn_bwd(int version) {
  const int prev = g_attn_bwd;
  g_attn_bwd = version;
  return prev;
}

// dqkv[B*S, 3H] (every element written) from dout[B*S, H]
MDTF_EXPORT int mdtf_attn_bwd(const void* qkv, const float* mask, const void* out, const void* dout, const float* lse,
                              void* dqkv, int B, int seq, int nh, int dh, float scale, float p_drop, unsigned seed,
                              const long long* seed_off, hipStream_t st) {
  if (seq != S || dh != D) return MDTF_EUNSUPPORTED;
  if ((long long)B * S * 3 * nh * D * 2 > 0x7fffffffLL) return MDTF_EUNSUPPORTED;
  // v2 (default; in the BERT-base step 39 vs 45 us per call, profiles/attention_bwd_v2_r3.md); MDTF_ATTN_BWD=v1:
  // the r1 kernel with [q][k] images (MDTF_ATTN_BWD_WAVES=4: its 4-wave form) -- A/B switches
  if (g_attn_bwd < 0) {     // MDTF_ATTN_BWD=v1 | v2 (default) | v2s (split phases: -0.8 % BERT-base, profiles/ab_r6.md)
    const char* e = getenv("MDTF_ATTN_BWD");
    g_attn_bwd = (e && e[0] == 'v' && e[1] == '1') ? 1 : (e && e[0] == 'v' && e[1] == '2' && e[2] == 's') ? 3 : 2;
  }
  const bool v1 = g_attn_bwd == 1;
  static const bool w4 = [] {
    const char* e = getenv("MDTF_ATTN_BWD_WAVES");
    return e && e[0] == '4';
  }();
  if (!v1 && attn_pp_on()) {
    hipLaunchKernelGGL(attn_bwd_pp, dim3(pp_grid(B * nh)), dim3(1024), kBwdPpLds, st, (const bf16_t*)qkv, mask,
                       (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv, B, nh, scale, p_drop,
                       (uint32_t)seed, seed_off);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  if (g_attn_bwd == 3 && !w4) {
    // MDTF_ATTN_BWD_OCC=3: the 80-register build (three workgroups per CU)
    static const int occ = [] {
      const char* e = getenv("MDTF_ATTN_BWD_OCC");
      return (e && e[0] == '3') ? 3 : 2;
    }();
    hipLaunchKernelGGL((occ == 3 ? attn_bwd_v2s<3> : attn_bwd_v2s<2>), dim3(2 * B * nh), dim3(512), kBwd2sLds, st,
                       (const bf16_t*)qkv, mask, (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv, B, nh,
                       scale, p_drop, (uint32_t)seed, seed_off);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  if (!v1 && !w4) {
    hipLaunchKernelGGL(attn_bwd_v2, dim3(B * nh), dim3(512), kBwd2Lds, st, (const bf16_t*)qkv, mask,
                       (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv, B, nh, scale, p_drop,
                       (uint32_t)seed, seed_off);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  if (w4) {
    hipLaunchKernelGGL(attn_bwd_kernel<4>, dim3(B * nh), dim3(256), kBwdLds, st, (const bf16_t*)qkv, mask,
                       (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv, B, nh, scale, p_drop,
                       (uint32_t)seed, seed_off);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(attn_bwd_kernel<8>, dim3(B * nh), dim3(512), kBwdLds, st, (const bf16_t*)qkv, mask,
                     (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv, B, nh, scale, p_drop,
                     (uint32_t)seed, seed_off);
  MDTF_LAUNCH_CHECK();
  return 0;
}
