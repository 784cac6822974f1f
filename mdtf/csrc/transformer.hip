// Transformer (BERT) kernels: fused residual+LayerNorm, masked scaled softmax,
// embedding gather / scatter-add.  bf16 activations, fp32 statistics.
//
// BASELINE config "BERT-base data-parallel (MFMA bf16 GEMM + fused Adam)".  The
// plain GEMMs go to hipBLASLt; everything between them runs here:
//   * ln_fwd:  s = x (+ res);  y = (s - mean) * rstd * gamma + beta   (one wave per row,
//              bf16x8 vectors, the row stays in registers: one read, two writes)
//   * ln_bwd:  dx = rstd * (g·dy - mean(g·dy) - xhat·mean(g·dy·xhat)); per-block
//              dgamma/dbeta partials accumulated in registers over the block's rows,
//              stored to a workspace, then summed by the shared partial-reduction
//              kernel (no hot atomics; ~1024 blocks keep every CU busy)
//   * softmax: y = softmax(scale·x + mask[b, key]) over the key axis, one wave per row
//   * embed:   out[t] = table[id[t]] gather; backward = fp32 atomic scatter-add
#include "mdtf_common.h"

using namespace mdtf;

namespace {

constexpr int kT = 256;
constexpr int kMaxVec = 16;   // H <= 64 lanes * 8 * 16 = 8192

// dropout keep bit of element idx (same counter-hash as csrc/attention.hip)
__device__ __forceinline__ bool drop_keep(uint32_t idx, uint32_t seed, uint32_t thr) {
  uint32_t x = idx * 0x9E3779B1u ^ seed;
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x >= thr;
}

// per-step seed: the host seed of the call site mixed with the device step counter
// (hipGraph replays re-use the captured host seed; the counter advances per replay)
__device__ __forceinline__ uint32_t step_seed(uint32_t seed, const long long* seed_off) {
  return seed_off ? seed ^ ((uint32_t)(*seed_off) * 0x85EBCA6Bu) : seed;
}

// sum over the LPR lanes that share a row (LPR = 64: the wave; 32: each half-wave holds its own row)
template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LPR lanes per row: 64 (a wave per row) or 32 (two rows per wave: H = 768 is 96 vectors = 32 lanes x 3, where a
// whole wave would leave half its lanes idle on the second vector)
template <int NV, int LPR>
__global__ void __launch_bounds__(kT) ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   bf16_t* __restrict__ y, bf16_t* __restrict__ s_out,
                                                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                   long long rows, int H, float eps, uint32_t thr, float inv_keep,
                                                   uint32_t seed, const long long* __restrict__ seed_off, int nt_s) {
  seed = step_seed(seed, seed_off);
  const int lane = threadIdx.x & (LPR - 1);
  const long long row = (long long)blockIdx.x * (kT / LPR) + (threadIdx.x / LPR);
  if (row >= rows) return;      // (LPR = 32: the row sums shuffle inside each 32-lane half only)
  const int nvec = H / 8;
  float v[NV][8];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + i * LPR);
    if (c < nvec) {
      load_bf8(x + row * H + c * 8, v[i]);
      if (thr) {      // fused dropout on the branch input (before the residual add)
#pragma unroll
        for (int k = 0; k < 8; ++k)
          v[i][k] = drop_keep((uint32_t)(row * H + c * 8 + k), seed, thr) ? v[i][k] * inv_keep : 0.f;
      }
      if (res) {
        float r[8];
        load_bf8(res + row * H + c * 8, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[i][k] += r[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += v[i][k];
    }
  }
  const float mean = row_sum<LPR>(sum) / (float)H;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + i * LPR);
    if (c < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[i][k] - mean;
        sq += d * d;
      }
    }
  }
  const float rstd = rsqrtf(row_sum<LPR>(sq) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + i * LPR);
    if (c < nvec) {
      if (s_out) {             // the residual sum is read again only by the backward: nt_s streams it out
        if (nt_s) {
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          u32x4_t w;
#pragma unroll
          for (int k = 0; k < 4; ++k) w[k] = pack_bf2(v[i][2 * k], v[i][2 * k + 1]);
          __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(s_out + row * H + c * 8));
        } else {
          store_bf8(s_out + row * H + c * 8, v[i]);
        }
      }
      const float4 g0 = *reinterpret_cast<const float4*>(gamma + c * 8);
      const float4 g1 = *reinterpret_cast<const float4*>(gamma + c * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(beta + c * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(beta + c * 8 + 4);
      const float gk[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bk[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (v[i][k] - mean) * rstd * gk[k] + bk[k];
      store_bf8(y + row * H + c * 8, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// each block (kT / LPR row slices: whole waves, or half-waves for LPR = 32) walks rows_per_block rows;
// dgamma/dbeta partials live in registers
template <int NV, int LPR>
__global__ void __launch_bounds__(kT) ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                   const float* __restrict__ gamma, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, bf16_t* __restrict__ dx,
                                                   bf16_t* __restrict__ dx_branch, float* __restrict__ ws,
                                                   long long rows, int H, int rows_per_block, int beta_first,
                                                   uint32_t thr, float inv_keep, uint32_t seed,
                                                   const long long* __restrict__ seed_off, float* __restrict__ dg_out,
                                                   float* __restrict__ db_out) {
  seed = step_seed(seed, seed_off);
  constexpr int W = kT / LPR;                 // row slices per block
  const int lane = threadIdx.x & (LPR - 1), slice = threadIdx.x / LPR;
  const int nvec = H / 8;
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[i][k] = db[i][k] = 0.f;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  // gamma in registers for the whole block
  float gm[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * LPR;
    if (c < nvec) {
      const float4 g0 = *reinterpret_cast<const float4*>(gamma + c * 8);
      const float4 g1 = *reinterpret_cast<const float4*>(gamma + c * 8 + 4);
      gm[i][0] = g0.x; gm[i][1] = g0.y; gm[i][2] = g0.z; gm[i][3] = g0.w;
      gm[i][4] = g1.x; gm[i][5] = g1.y; gm[i][6] = g1.z; gm[i][7] = g1.w;
    }
  }
  auto load_row = [&](long long row, uint4 (&gr)[NV], uint4 (&sr)[NV], float& mu, float& rs) {
    mu = mean[row];       // issued with the row's vectors, not behind the previous row's stores
    rs = rstd[row];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * LPR;
      if (c < nvec) {
        gr[i] = *reinterpret_cast<const uint4*>(dy + row * H + c * 8);
        sr[i] = *reinterpret_cast<const uint4*>(s + row * H + c * 8);
      }
    }
  };
  auto do_row = [&](long long row, const uint4 (&gr)[NV], const uint4 (&sr)[NV], const float mu, const float rs) {
    float g[NV][8], xh[NV][8];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * LPR;
      if (c < nvec) {
        const uint32_t gw[4] = {gr[i].x, gr[i].y, gr[i].z, gr[i].w};
        const uint32_t sw[4] = {sr[i].x, sr[i].y, sr[i].z, sr[i].w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          g[i][k] = __uint_as_float(k & 1 ? gw[k >> 1] & 0xffff0000u : gw[k >> 1] << 16);
          const float sv = __uint_as_float(k & 1 ? sw[k >> 1] & 0xffff0000u : sw[k >> 1] << 16);
          xh[i][k] = (sv - mu) * rs;
          dg[i][k] += g[i][k] * xh[i][k];
          db[i][k] += g[i][k];
          const float gg = g[i][k] * gm[i][k];
          a += gg;
          b += gg * xh[i][k];
        }
      }
    }
    a = row_sum<LPR>(a) / (float)H;
    b = row_sum<LPR>(b) / (float)H;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * LPR;
      if (c < nvec) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rs * (g[i][k] * gm[i][k] - a - xh[i][k] * b);
        store_bf8(dx + row * H + c * 8, o);
        if (dx_branch) {     // gradient of the dropped-out branch input
#pragma unroll
          for (int k = 0; k < 8; ++k)
            o[k] = (!thr || drop_keep((uint32_t)(row * H + c * 8 + k), seed, thr)) ? o[k] * inv_keep : 0.f;
          store_bf8(dx_branch + row * H + c * 8, o);
        }
      }
    }
  };
  // RIF rows per slice per iteration, all their loads in flight before the first is reduced
  constexpr int RIF = NV <= 2 ? 4 : (NV == 3 ? 2 : 1);
  for (long long row = r0 + slice; row < r1; row += RIF * W) {
    uint4 gr[RIF][NV], sr[RIF][NV];
    float mu[RIF], rs[RIF];
#pragma unroll
    for (int j = 0; j < RIF; ++j)
      if (row + j * W < r1) load_row(row + j * W, gr[j], sr[j], mu[j], rs[j]);
#pragma unroll
    for (int j = 0; j < RIF; ++j)
      if (row + j * W < r1) do_row(row + j * W, gr[j], sr[j], mu[j], rs[j]);
  }
  // combine the W slices through LDS; block partials -> ws[block][2][H] (plain stores, summed by a reduction pass:
  // deterministic) or, ws == null, one fp32 atomic per column per block straight into the grad slots
  constexpr int SPAN = LPR * 8;               // columns one pass over i covers
  __shared__ __attribute__((aligned(16))) float L[2][W][SPAN];
  float* wg = ws ? ws + (long long)blockIdx.x * 2 * H : nullptr;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    // a lane's 8 columns as two 16-B halves, each half-set lane-contiguous (position h * 4 LPR + 4 lane + e holds
    // column 8 lane + 4 h + e): the 16 lanes one ds_write_b128 cycle serves write 256 contiguous bytes -- all 64
    // banks once.  (Both halves at 8 lane, 8 lane + 4 put lanes l and l + 8 on the same banks: 2-way conflicts.)
    float4* l0 = reinterpret_cast<float4*>(&L[0][slice][0]);
    float4* l1 = reinterpret_cast<float4*>(&L[1][slice][0]);
    l0[lane] = make_float4(dg[i][0], dg[i][1], dg[i][2], dg[i][3]);
    l0[LPR + lane] = make_float4(dg[i][4], dg[i][5], dg[i][6], dg[i][7]);
    l1[lane] = make_float4(db[i][0], db[i][1], db[i][2], db[i][3]);
    l1[LPR + lane] = make_float4(db[i][4], db[i][5], db[i][6], db[i][7]);
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * SPAN; j += kT) {
      const int which = j / SPAN, cc = j % SPAN;       // 0: dgamma, 1: dbeta
      const int h = cc / (4 * LPR), ln = (cc / 4) % LPR, e = cc % 4;
      const int col = i * SPAN + ln * 8 + h * 4 + e;
      if (col < H) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) t += L[which][w][cc];
        if (wg) wg[(which ^ beta_first) * H + col] = t;      // partial rows follow the grad slots' order
        else unsafeAtomicAdd((which ? db_out : dg_out) + col, t);
      }
    }
    __syncthreads();
  }
}

// LayerNorm backward, lean form (MDTF_LN_BWD=2 / 3; default ln_bwd_kernel above).  ln_bwd_kernel keeps two rows'
// fp32 intermediates, gamma and the dgamma / dbeta partials in registers: 232 VGPRs at H = 768, two waves per SIMD,
// ~2 TB/s.  Here a slice reduces ONE row at a time in two passes over its raw bf16 vectors (pass 1: the row sums
// and the dgamma / dbeta partials; pass 2 recomputes g and xhat from the raw registers and stores dx), gamma is read
// from LDS, and PF = true loads the slice's next row before the current one is reduced.  Same outputs and the same
// block-partial epilogue as ln_bwd_kernel.
template <int NV, int LPR, bool PF>
__global__ void __launch_bounds__(kT, 3) ln_bwd_lean(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                 const float* __restrict__ gamma, const float* __restrict__ mean,
                                                 const float* __restrict__ rstd, bf16_t* __restrict__ dx,
                                                 bf16_t* __restrict__ dx_branch, float* __restrict__ ws,
                                                 long long rows, int H, int rows_per_block, int beta_first,
                                                 uint32_t thr, float inv_keep, uint32_t seed,
                                                 const long long* __restrict__ seed_off, float* __restrict__ dg_out,
                                                 float* __restrict__ db_out) {
  seed = step_seed(seed, seed_off);
  constexpr int W = kT / LPR;
  constexpr int SPAN = LPR * 8;
  const int lane = threadIdx.x & (LPR - 1), slice = threadIdx.x / LPR;
  const int nvec = H / 8;
  __shared__ __attribute__((aligned(16))) float Lg[NV * SPAN];
  __shared__ __attribute__((aligned(16))) float L[2][W][SPAN];
  for (int c = threadIdx.x; c < NV * SPAN; c += kT) Lg[c] = c < H ? gamma[c] : 0.f;
  __syncthreads();
  float dg[NV][8], db[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) dg[i][k] = db[i][k] = 0.f;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  auto load_row = [&](long long row, uint4 (&gr)[NV], uint4 (&sr)[NV], float& mu, float& rs) {
    mu = mean[row];
    rs = rstd[row];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * LPR;
      if (c < nvec) {
        gr[i] = *reinterpret_cast<const uint4*>(dy + row * H + c * 8);
        sr[i] = *reinterpret_cast<const uint4*>(s + row * H + c * 8);
      }
    }
  };
  auto bf = [](const uint4& v, int k) {
    const uint32_t w = k < 2 ? v.x : (k < 4 ? v.y : (k < 6 ? v.z : v.w));
    return __uint_as_float(k & 1 ? w & 0xffff0000u : w << 16);
  };
  uint4 gr[NV], sr[NV];
  float mu = 0.f, rs = 0.f;
  long long row = r0 + slice;
  if (row < r1) load_row(row, gr, sr, mu, rs);
  for (; row < r1; row += W) {
    const long long nrow = row + W;
    uint4 gn[NV], sn[NV];
    float mn = 0.f, rn = 0.f;
    if (PF && nrow < r1) load_row(nrow, gn, sn, mn, rn);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * LPR;
      if (c < nvec) {
        const float4 q0 = *reinterpret_cast<const float4*>(&Lg[c * 8]);
        const float4 q1 = *reinterpret_cast<const float4*>(&Lg[c * 8 + 4]);
        const float gmk[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = bf(gr[i], k), xh = (bf(sr[i], k) - mu) * rs;
          dg[i][k] += g * xh;
          db[i][k] += g;
          const float gg = g * gmk[k];
          a += gg;
          b += gg * xh;
        }
      }
    }
    a = row_sum<LPR>(a) / (float)H;
    b = row_sum<LPR>(b) / (float)H;
    // pass 2 re-derives g and xhat from the raw registers: an empty asm "modifies" them, so the compiler cannot keep
    // pass 1's 2 x 8 NV unpacked floats alive across the row sums (that CSE costs ~50 VGPRs)
#pragma unroll
    for (int i = 0; i < NV; ++i)
      asm volatile("" : "+v"(gr[i].x), "+v"(gr[i].y), "+v"(gr[i].z), "+v"(gr[i].w), "+v"(sr[i].x), "+v"(sr[i].y),
                   "+v"(sr[i].z), "+v"(sr[i].w));
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * LPR;
      if (c < nvec) {
        const float4 q0 = *reinterpret_cast<const float4*>(&Lg[c * 8]);
        const float4 q1 = *reinterpret_cast<const float4*>(&Lg[c * 8 + 4]);
        const float gmk[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = bf(gr[i], k), xh = (bf(sr[i], k) - mu) * rs;
          o[k] = rs * (g * gmk[k] - a - xh * b);
        }
        store_bf8(dx + row * H + c * 8, o);
        if (dx_branch) {
#pragma unroll
          for (int k = 0; k < 8; ++k)
            o[k] = (!thr || drop_keep((uint32_t)(row * H + c * 8 + k), seed, thr)) ? o[k] * inv_keep : 0.f;
          store_bf8(dx_branch + row * H + c * 8, o);
        }
      }
    }
    if (nrow < r1) {
      if (PF) {
        mu = mn;
        rs = rn;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          gr[i] = gn[i];
          sr[i] = sn[i];
        }
      } else {
        load_row(nrow, gr, sr, mu, rs);
      }
    }
  }
  float* wg = ws ? ws + (long long)blockIdx.x * 2 * H : nullptr;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float4* l0 = reinterpret_cast<float4*>(&L[0][slice][0]);
    float4* l1 = reinterpret_cast<float4*>(&L[1][slice][0]);
    l0[lane] = make_float4(dg[i][0], dg[i][1], dg[i][2], dg[i][3]);
    l0[LPR + lane] = make_float4(dg[i][4], dg[i][5], dg[i][6], dg[i][7]);
    l1[lane] = make_float4(db[i][0], db[i][1], db[i][2], db[i][3]);
    l1[LPR + lane] = make_float4(db[i][4], db[i][5], db[i][6], db[i][7]);
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * SPAN; j += kT) {
      const int which = j / SPAN, cc = j % SPAN;
      const int h = cc / (4 * LPR), ln = (cc / 4) % LPR, e = cc % 4;
      const int col = i * SPAN + ln * 8 + h * 4 + e;
      if (col < H) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) t += L[which][w][cc];
        if (wg) wg[(which ^ beta_first) * H + col] = t;
        else unsafeAtomicAdd((which ? db_out : dg_out) + col, t);
      }
    }
    __syncthreads();
  }
}

// masked, scaled softmax over the last axis; rows = B*heads*Sq, cols = Sk
// mask (optional): additive fp32 [B][Sk]; batch index of a row = row / rows_per_batch
template <int NV>
__global__ void __launch_bounds__(kT) softmax_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ mask,
                                                        bf16_t* __restrict__ y, long long rows, int cols, float scale,
                                                        long long rows_per_batch) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* mk = mask ? mask + (row / rows_per_batch) * cols : nullptr;
  const int nvec = cols / 8;
  float v[NV][8];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      load_bf8(x + row * cols + c * 8, v[i]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[i][k] = v[i][k] * scale + (mk ? mk[c * 8 + k] : 0.f);
        m = fmaxf(m, v[i][k]);
      }
    }
  }
  m = wave_max(m);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[i][k] = __expf(v[i][k] - m);
        sum += v[i][k];
      }
    }
  }
  const float inv = 1.f / wave_sum(sum);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[i][k] *= inv;
      store_bf8(y + row * cols + c * 8, v[i]);
    }
  }
}

template <int NV>
__global__ void __launch_bounds__(kT) softmax_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                        bf16_t* __restrict__ dx, long long rows, int cols, float scale) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = cols / 8;
  float g[NV][8], p[NV][8];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      load_bf8(dy + row * cols + c * 8, g[i]);
      load_bf8(y + row * cols + c * 8, p[i]);
#pragma unroll
      for (int k = 0; k < 8; ++k) dot += g[i][k] * p[i][k];
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = scale * p[i][k] * (g[i][k] - dot);
      store_bf8(dx + row * cols + c * 8, o);
    }
  }
}

__global__ void embed_fwd_kernel(const bf16_t* __restrict__ table, const long long* __restrict__ ids,
                                 bf16_t* __restrict__ out, long long n, int H, long long vocab) {
  const int nvec = H / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n * nvec;
       i += (long long)gridDim.x * blockDim.x) {
    const long long t = i / nvec;
    const int c = static_cast<int>(i % nvec);
    long long id = ids[t];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (id >= 0 && id < vocab) v = *reinterpret_cast<const uint4*>(table + id * H + c * 8);
    *reinterpret_cast<uint4*>(out + t * H + c * 8) = v;
  }
}

__global__ void embed_bwd_kernel(const bf16_t* __restrict__ dy, const long long* __restrict__ ids,
                                 float* __restrict__ dtable, long long n, int H, long long vocab) {
  const long long total = n * H;
  if (total < 0x7fffffffLL) {         // 32-bit index math: one 32-bit division per element instead of two 64-bit
    const unsigned tot = (unsigned)total, h = (unsigned)H;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x) {
      const unsigned t = i / h, c = i - t * h;
      const long long id = ids[t];
      if (id >= 0 && id < vocab) atomicAdd(dtable + id * H + c, bf2f(dy[i]));
    }
    return;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long t = i / H;
    const int c = static_cast<int>(i % H);
    long long id = ids[t];
    if (id >= 0 && id < vocab) atomicAdd(dtable + id * H + c, bf2f(dy[i]));
  }
}

// Tiny tables (token types: 2 rows) would take ~n fp32 atomics per element on one or two rows.
// Instead each block sums a run of kSmallTok tokens per (row, 8-column vector) in registers
// (thread = vector) and adds its partials once.
constexpr int kSmallVocab = 4, kSmallTok = 64;
__global__ void embed_bwd_small_kernel(const bf16_t* __restrict__ dy, const long long* __restrict__ ids,
                                       float* __restrict__ dtable, long long n, int H, int vocab) {
  const int v8 = threadIdx.x;
  if (v8 * 8 >= H) return;
  const long long t0 = (long long)blockIdx.x * kSmallTok;
  const long long t1 = t0 + kSmallTok < n ? t0 + kSmallTok : n;
  float acc[kSmallVocab][8];
#pragma unroll
  for (int r = 0; r < kSmallVocab; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[r][k] = 0.f;
  for (long long t = t0; t < t1; ++t) {
    const long long id = ids[t];
    if (id < 0 || id >= vocab) continue;
    float g[8];
    load_bf8(dy + t * H + v8 * 8, g);
#pragma unroll
    for (int r = 0; r < kSmallVocab; ++r)
      if (r == id) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[r][k] += g[k];
      }
  }
  for (int r = 0; r < vocab; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (acc[r][k] != 0.f) atomicAdd(dtable + (long long)r * H + v8 * 8 + k, acc[r][k]);
}

// Small tables, deterministic two-pass form: block b sums tokens [16 b, 16 b + 16) per (row, 8-column vector) in
// registers (four tokens' loads in flight) and writes its partial rows ws[b][vocab][H]; the shared partial-row
// reduction then adds them into the table gradient.  512 blocks at 8192 tokens instead of 128 blocks whose
// atomics all hit the same vocab x H addresses (the type embedding: 2 x 768).
constexpr int kSmallTok2 = 16;
__global__ void embed_bwd_small_part(const bf16_t* __restrict__ dy, const long long* __restrict__ ids,
                                     float* __restrict__ ws, long long n, int H, int vocab) {
  const int v8 = threadIdx.x;
  if (v8 * 8 >= H) return;
  const long long t0 = (long long)blockIdx.x * kSmallTok2;
  const long long t1 = t0 + kSmallTok2 < n ? t0 + kSmallTok2 : n;
  float acc[kSmallVocab][8];
#pragma unroll
  for (int r = 0; r < kSmallVocab; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[r][k] = 0.f;
  for (long long t = t0; t < t1; t += 4) {
    long long id[4];
    float g[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = t + u < t1;
      id[u] = ok ? ids[t + u] : -1;
      if (ok) load_bf8(dy + (t + u) * H + v8 * 8, g[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < kSmallVocab; ++r)
        if (id[u] == r) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[r][k] += g[u][k];
        }
  }
  for (int r = 0; r < vocab; ++r) {
    float* dst = ws + ((long long)blockIdx.x * vocab + r) * H + v8 * 8;
    *reinterpret_cast<float4*>(dst) = make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[r][4], acc[r][5], acc[r][6], acc[r][7]);
  }
}

inline int gcap(long long work) {
  long long b = ceil_div(work, kT);
  return static_cast<int>(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

// LayerNorm: 32 lanes per row when the row's vectors fill 32-lane slices exactly but not whole waves (H = 768:
// 96 vectors = 3 x 32), else a wave per row
#define LN_DISPATCH(H, KERNEL, GRID32, GRID64, ...)                                                        \
  do {                                                                                                     \
    const int nvec_ = (H) / 8;                                                                             \
    if (nvec_ % 64 != 0 && nvec_ % 32 == 0 && nvec_ / 32 <= 3) {                                           \
      if (nvec_ == 32) hipLaunchKernelGGL((KERNEL<1, 32>), GRID32, dim3(kT), 0, st, __VA_ARGS__);         \
      else hipLaunchKernelGGL((KERNEL<3, 32>), GRID32, dim3(kT), 0, st, __VA_ARGS__);                     \
      break;                                                                                               \
    }                                                                                                      \
    const int nv_ = static_cast<int>(ceil_div(nvec_, 64));                                                 \
    if (nv_ <= 1) hipLaunchKernelGGL((KERNEL<1, 64>), GRID64, dim3(kT), 0, st, __VA_ARGS__);               \
    else if (nv_ <= 2) hipLaunchKernelGGL((KERNEL<2, 64>), GRID64, dim3(kT), 0, st, __VA_ARGS__);          \
    else if (nv_ <= 4) hipLaunchKernelGGL((KERNEL<4, 64>), GRID64, dim3(kT), 0, st, __VA_ARGS__);          \
    else if (nv_ <= 8) hipLaunchKernelGGL((KERNEL<8, 64>), GRID64, dim3(kT), 0, st, __VA_ARGS__);          \
    else if (nv_ <= 16) hipLaunchKernelGGL((KERNEL<16, 64>), GRID64, dim3(kT), 0, st, __VA_ARGS__);        \
    else return MDTF_EUNSUPPORTED;                                                                         \
  } while (0)

// LN_DISPATCH with a third template argument X (the lean backward's prefetch switch)
#define LN_DISPATCH3(H, KERNEL, X, GRID32, GRID64, ...)                                                   \
  do {                                                                                                     \
    const int nvec_ = (H) / 8;                                                                             \
    if (nvec_ % 64 != 0 && nvec_ % 32 == 0 && nvec_ / 32 <= 3) {                                           \
      if (nvec_ == 32) hipLaunchKernelGGL((KERNEL<1, 32, X>), GRID32, dim3(kT), 0, st, __VA_ARGS__);      \
      else hipLaunchKernelGGL((KERNEL<3, 32, X>), GRID32, dim3(kT), 0, st, __VA_ARGS__);                  \
      break;                                                                                               \
    }                                                                                                      \
    const int nv_ = static_cast<int>(ceil_div(nvec_, 64));                                                 \
    if (nv_ <= 1) hipLaunchKernelGGL((KERNEL<1, 64, X>), GRID64, dim3(kT), 0, st, __VA_ARGS__);            \
    else if (nv_ <= 2) hipLaunchKernelGGL((KERNEL<2, 64, X>), GRID64, dim3(kT), 0, st, __VA_ARGS__);       \
    else if (nv_ <= 4) hipLaunchKernelGGL((KERNEL<4, 64, X>), GRID64, dim3(kT), 0, st, __VA_ARGS__);       \
    else if (nv_ <= 8) hipLaunchKernelGGL((KERNEL<8, 64, X>), GRID64, dim3(kT), 0, st, __VA_ARGS__);       \
    else if (nv_ <= 16) hipLaunchKernelGGL((KERNEL<16, 64, X>), GRID64, dim3(kT), 0, st, __VA_ARGS__);     \
    else return MDTF_EUNSUPPORTED;                                                                         \
  } while (0)

#define NV_DISPATCH(H, KERNEL, GRID, ...)                                                                  \
  do {                                                                                                     \
    const int nv_ = static_cast<int>(ceil_div((H) / 8, 64));                                               \
    if (nv_ <= 1) hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(kT), 0, st, __VA_ARGS__);                       \
    else if (nv_ <= 2) hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(kT), 0, st, __VA_ARGS__);                  \
    else if (nv_ <= 4) hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(kT), 0, st, __VA_ARGS__);                  \
    else if (nv_ <= 8) hipLaunchKernelGGL(KERNEL<8>, GRID, dim3(kT), 0, st, __VA_ARGS__);                  \
    else if (nv_ <= 16) hipLaunchKernelGGL(KERNEL<16>, GRID, dim3(kT), 0, st, __VA_ARGS__);                \
    else return MDTF_EUNSUPPORTED;                                                                         \
  } while (0)

static uint32_t drop_thr(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

// y = LN(dropout_p(x) + res); s = dropout_p(x) + res saved for backward (p = 0: no dropout)
MDTF_EXPORT int mdtf_ln_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y, void* s,
                            float* mean, float* rstd, long long rows, int H, float eps, float p_drop, unsigned seed,
                            const long long* seed_off, hipStream_t st) {
  if (H % 8) return MDTF_EINVAL;
  if (rows * H > 0xffffffffLL && p_drop > 0.f) return MDTF_EUNSUPPORTED;
  const uint32_t thr = drop_thr(p_drop);
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  // MDTF_LN_NT=1: nontemporal stores of the saved residual sum (A/B switch)
  static const int nt_s = [] {
    const char* e = getenv("MDTF_LN_NT");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  LN_DISPATCH(H, ln_fwd_kernel, dim3(ceil_div(rows, kT / 32)), dim3(ceil_div(rows, kT / 64)), (const bf16_t*)x,
              (const bf16_t*)res, gamma, beta, (bf16_t*)y, (bf16_t*)s, mean, rstd, rows, H, eps, thr, inv_keep,
              (uint32_t)seed, seed_off, nt_s);
  MDTF_LAUNCH_CHECK();
  return 0;
}

extern "C" int mdtf_reduce_partials(const float* ws, int B, int C, float* out, hipStream_t st);
extern "C" int mdtf_get_deterministic();
extern "C" int mdtf_reduce_partials_strided(const float* ws, int B, int C, long long ld, float* out, hipStream_t st);

// MDTF_LN_BWD: 1 ln_bwd_kernel (default), 2 ln_bwd_lean, 3 ln_bwd_lean with the next row prefetched.  Graph-timed at
// BERT-base's 8192 x 768 (bench/ln_probe.py, profiles/ln_probe_r6h.jsonl) the lean form's extra occupancy (138 vs
// 232 VGPRs) does not pay: 19.2 us (form 1, 16 rows per block) vs 20.4 (2) / 19.5 (3) incl. the partial reduction.
static int ln_bwd_form() {
  static const int v = [] {
    const char* e = getenv("MDTF_LN_BWD");
    const int f = e ? atoi(e) : 1;
    return (f >= 1 && f <= 3) ? f : 1;
  }();
  return v;
}

// MDTF_LN_BWD_RPB: minimum rows per LayerNorm-backward block (default 16 for ln_bwd_kernel: 512 blocks at 8192 rows;
// 8 for the lean form: 1024 blocks, one row per 32-lane slice; A/B switch)
static long long ln_bwd_rpb() {
  static const long long v = [] {
    const char* e = getenv("MDTF_LN_BWD_RPB");
    const long long r = e ? atoll(e) : 0;
    return r > 0 ? r : (ln_bwd_form() == 1 ? 16LL : 8LL);
  }();
  return v;
}

static void ln_bwd_geometry(long long rows, int* blocks, int* rpb) {
  long long b = ceil_div(rows, ln_bwd_rpb());  // >= 4 rows per wave (all in flight together) by default
  const long long cap = ln_bwd_rpb() == 16 ? 512 : 2048;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  *rpb = static_cast<int>(ceil_div(rows, b));
  *blocks = static_cast<int>(ceil_div(rows, *rpb));
}

// Side stream for the gamma / beta partial reductions of the following LayerNorm backward launches (null: in line;
// mdtf.ops.conv SLAB_SIDE): they only feed the gradient buffer, so they leave the backward chain through one event.
static hipStream_t g_ln_red_stream = nullptr;
MDTF_EXPORT int mdtf_set_ln_reduce_stream(hipStream_t s) {
  g_ln_red_stream = s;
  return 0;
}

// fp32 workspace elements mdtf_ln_bwd needs
MDTF_EXPORT long long mdtf_ln_bwd_ws(long long rows, int H) {
  int blocks, rpb;
  ln_bwd_geometry(rows, &blocks, &rpb);
  return (long long)blocks * 2 * H;
}

// dgamma/dbeta accumulate (+=) into zeroed buffers or fp32 grad slots;
// dgamma and dbeta must be ONE buffer pair [dgamma | dbeta] when contiguous is
// not guaranteed -> reduced separately.
// dx = d(loss)/d(s); dx_branch (optional) = d(loss)/d(x) through the fused dropout
MDTF_EXPORT int mdtf_ln_bwd(const void* dy, const void* s, const float* gamma, const float* mean, const float* rstd,
                            void* dx, void* dx_branch, float* dgamma, float* dbeta, float* ws, long long rows, int H,
                            float p_drop, unsigned seed, const long long* seed_off, hipStream_t st) {
  if (H % 8) return MDTF_EINVAL;
  if (rows <= 0) return 0;
  int blocks, rpb;
  ln_bwd_geometry(rows, &blocks, &rpb);
  // gamma/beta grad slots adjacent in either order -> one [blocks, 2H] reduction into the pair
  const int beta_first = (dgamma == dbeta + H) ? 1 : 0;
  const uint32_t thr = drop_thr(p_drop);
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  // block partial rows + one fixed-order reduction launch (default).  MDTF_LN_ATOMICS=1: the block partials go
  // straight into dgamma / dbeta by fp32 atomics instead (no reduction launch) -- measured slower in the BERT-base
  // step: ln_bwd 15.1 -> 25.5 us per call (512 blocks contend on 1536 addresses) vs the 4.8 us reduction it saves
  static const bool atomics_env = [] {
    const char* e = getenv("MDTF_LN_ATOMICS");
    return e && e[0] == '1';
  }();
  const bool atomics = atomics_env && !mdtf_get_deterministic();
  if (ln_bwd_form() == 1 || H > 2048)       // (the lean form spills past 4 vectors per lane)
    LN_DISPATCH(H, ln_bwd_kernel, dim3(blocks), dim3(blocks), (const bf16_t*)dy, (const bf16_t*)s, gamma, mean, rstd,
                (bf16_t*)dx, (bf16_t*)dx_branch, atomics ? nullptr : ws, rows, H, rpb, beta_first, thr, inv_keep,
                (uint32_t)seed, seed_off, dgamma, dbeta);
  else if (ln_bwd_form() == 2)
    LN_DISPATCH3(H, ln_bwd_lean, false, dim3(blocks), dim3(blocks), (const bf16_t*)dy, (const bf16_t*)s, gamma, mean,
                 rstd, (bf16_t*)dx, (bf16_t*)dx_branch, atomics ? nullptr : ws, rows, H, rpb, beta_first, thr,
                 inv_keep, (uint32_t)seed, seed_off, dgamma, dbeta);
  else
    LN_DISPATCH3(H, ln_bwd_lean, true, dim3(blocks), dim3(blocks), (const bf16_t*)dy, (const bf16_t*)s, gamma, mean,
                 rstd, (bf16_t*)dx, (bf16_t*)dx_branch, atomics ? nullptr : ws, rows, H, rpb, beta_first, thr,
                 inv_keep, (uint32_t)seed, seed_off, dgamma, dbeta);
  MDTF_LAUNCH_CHECK();
  if (atomics) return 0;
  if (g_ln_red_stream && g_ln_red_stream != st) {
    static hipEvent_t ev = [] {
      hipEvent_t e = nullptr;
      (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
      return e;
    }();
    if (!ev || hipEventRecord(ev, st) != hipSuccess || hipStreamWaitEvent(g_ln_red_stream, ev, 0) != hipSuccess)
      return MDTF_EUNSUPPORTED;
    st = g_ln_red_stream;
  }
  if (beta_first) return mdtf_reduce_partials(ws, blocks, 2 * H, dbeta, st);
  // ws rows are [dgamma(H) | dbeta(H)]: reduce as a [blocks, 2H] matrix when the
  // two outputs are adjacent, else as two strided passes
  if (dbeta == dgamma + H) return mdtf_reduce_partials(ws, blocks, 2 * H, dgamma, st);
  int rc = mdtf_reduce_partials_strided(ws, blocks, H, 2 * H, dgamma, st);
  if (rc) return rc;
  return mdtf_reduce_partials_strided(ws + H, blocks, H, 2 * H, dbeta, st);
}

MDTF_EXPORT int mdtf_softmax_fwd(const void* x, const float* mask, void* y, long long rows, int cols, float scale,
                                 long long rows_per_batch, hipStream_t st) {
  if (cols % 8) return MDTF_EINVAL;
  NV_DISPATCH(cols, softmax_fwd_kernel, dim3(ceil_div(rows, kT / 64)), (const bf16_t*)x, mask, (bf16_t*)y, rows,
              cols, scale, rows_per_batch);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_softmax_bwd(const void* dy, const void* y, void* dx, long long rows, int cols, float scale,
                                 hipStream_t st) {
  if (cols % 8) return MDTF_EINVAL;
  NV_DISPATCH(cols, softmax_bwd_kernel, dim3(ceil_div(rows, kT / 64)), (const bf16_t*)dy, (const bf16_t*)y,
              (bf16_t*)dx, rows, cols, scale);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// BERT input embedding in one pass each way: out[t] = word[ids[t]] + pos[t % S] + type[types[t]] (fp32 sum, one
// rounding).  Backward: word rows by per-element fp32 atomics over the whole grid (embed_bwd_kernel); position and
// <= 4 token-type rows by one thread per (position, 8-column vector) summing 8 batch rows in registers, then one
// atomic each.  Replaces three gathers + two adds forward and three scatter passes back.
namespace {
constexpr int kTypeRows = 4;
constexpr int kEmbBatch = 8;    // batch rows per backward block (grid.y = B / 8): the position partials add by atomics
__global__ void bert_embed_fwd_kernel(const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                      const bf16_t* __restrict__ typ, const long long* __restrict__ ids,
                                      const long long* __restrict__ types, bf16_t* __restrict__ out, long long n, int S,
                                      int H, long long vocab, int ntypes) {
  const int nvec = H / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n * nvec;
       i += (long long)gridDim.x * blockDim.x) {
    const long long t = i / nvec;
    const int c = static_cast<int>(i % nvec);
    const long long id = ids[t], ty = types[t];
    const int s = static_cast<int>(t % S);
    float a[8], b[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = 0.f;
    if (id >= 0 && id < vocab) load_bf8(word + id * H + c * 8, o);
    load_bf8(pos + (long long)s * H + c * 8, a);
    if (ty >= 0 && ty < ntypes) {
      load_bf8(typ + ty * H + c * 8, b);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) b[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] += a[k] + b[k];
    store_bf8(out + t * H + c * 8, o);
  }
}

__global__ void bert_embed_bwd_kernel(const bf16_t* __restrict__ dy, const long long* __restrict__ types,
                                      float* __restrict__ dpos, float* __restrict__ dtyp, int B, int S, int H,
                                      int ntypes) {
  const int nvec = H / 8;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)S * nvec) return;
  const int s = static_cast<int>(i / nvec), c = static_cast<int>(i % nvec);
  float ps[8], ts[kTypeRows][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ps[k] = 0.f;
#pragma unroll
    for (int r = 0; r < kTypeRows; ++r) ts[r][k] = 0.f;
  }
  const int b0 = blockIdx.y * kEmbBatch, b1 = b0 + kEmbBatch < B ? b0 + kEmbBatch : B;
  for (int b = b0; b < b1; ++b) {
    const long long t = (long long)b * S + s;
    float g[8];
    load_bf8(dy + t * H + c * 8, g);
    const long long ty = types[t];
#pragma unroll
    for (int k = 0; k < 8; ++k) ps[k] += g[k];
#pragma unroll
    for (int r = 0; r < kTypeRows; ++r)
      if (r == ty) {
#pragma unroll
        for (int k = 0; k < 8; ++k) ts[r][k] += g[k];
      }
  }
  if (dpos) {
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(dpos + (long long)s * H + c * 8 + k, ps[k]);
  }
  if (dtyp) {
    for (int r = 0; r < ntypes && r < kTypeRows; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) atomicAdd(dtyp + (long long)r * H + c * 8 + k, ts[r][k]);
  }
}
}  // namespace

MDTF_EXPORT int mdtf_bert_embed_fwd(const void* word, const void* pos, const void* typ, const long long* ids,
                                    const long long* types, void* out, long long n, int S, int H, long long vocab,
                                    int npos, int ntypes, hipStream_t st) {
  if (H % 8 || S > npos || ntypes > kTypeRows || n % S) return MDTF_EUNSUPPORTED;
  hipLaunchKernelGGL(bert_embed_fwd_kernel, dim3(gcap(n * H / 8)), dim3(kT), 0, st, (const bf16_t*)word,
                     (const bf16_t*)pos, (const bf16_t*)typ, ids, types, (bf16_t*)out, n, S, H, vocab, ntypes);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// dword/dpos/dtyp: fp32 [V][H] / [npos][H] / [ntypes][H] accumulated (zeroed buffers or gradient slots)
MDTF_EXPORT int mdtf_bert_embed_bwd(const void* dy, const long long* ids, const long long* types, float* dword,
                                    float* dpos, float* dtyp, int B, int S, int H, long long vocab, int ntypes,
                                    hipStream_t st) {
  if (H % 8 || ntypes > kTypeRows) return MDTF_EUNSUPPORTED;
  // word rows: one thread per element (fp32 atomics spread over the whole grid); position / type rows: one thread
  // per (position, 8-column vector) summing 8 batch rows in registers
  const long long n = (long long)B * S;
  if (dword)
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(gcap(n * H)), dim3(kT), 0, st, (const bf16_t*)dy, ids, dword, n, H,
                       vocab);
  const long long threads = (long long)S * (H / 8);
  hipLaunchKernelGGL(bert_embed_bwd_kernel, dim3((unsigned)ceil_div(threads, kT), (unsigned)ceil_div(B, kEmbBatch)),
                     dim3(kT), 0, st, (const bf16_t*)dy, types, dpos, dtyp, B, S, H, ntypes);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_embed_fwd(const void* table, const long long* ids, void* out, long long n, int H,
                               long long vocab, hipStream_t st) {
  if (H % 8) return MDTF_EINVAL;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(gcap(n * H / 8)), dim3(kT), 0, st, (const bf16_t*)table, ids,
                     (bf16_t*)out, n, H, vocab);
  MDTF_LAUNCH_CHECK();
  return 0;
}

extern "C" int mdtf_reduce_partials(const float* ws, int B, int C, float* out, hipStream_t st);

// fp32 workspace floats mdtf_embed_bwd_ws needs (0: the table is not small)
MDTF_EXPORT long long mdtf_embed_bwd_ws_floats(long long n, int H, long long vocab) {
  if (vocab > kSmallVocab || H % 8 || H / 8 > 1024 || n <= 0) return 0;
  return ceil_div(n, kSmallTok2) * vocab * H;
}

// dtable += scatter of dy by ids for a small table (vocab <= 4), deterministic: partial rows + one reduction
MDTF_EXPORT int mdtf_embed_bwd_ws(const void* dy, const long long* ids, float* dtable, long long n, int H,
                                  long long vocab, float* ws, hipStream_t st) {
  if (mdtf_embed_bwd_ws_floats(n, H, vocab) == 0) return MDTF_EINVAL;
  const int nb = static_cast<int>(ceil_div(n, kSmallTok2));
  const int threads = static_cast<int>(ceil_div(H / 8, 64) * 64);
  hipLaunchKernelGGL(embed_bwd_small_part, dim3((unsigned)nb), dim3(threads), 0, st, (const bf16_t*)dy, ids, ws, n,
                     H, static_cast<int>(vocab));
  MDTF_LAUNCH_CHECK();
  return mdtf_reduce_partials(ws, nb, static_cast<int>(vocab) * H, dtable, st);
}

MDTF_EXPORT int mdtf_embed_bwd(const void* dy, const long long* ids, float* dtable, long long n, int H,
                               long long vocab, hipStream_t st) {
  if (vocab <= kSmallVocab && H % 8 == 0 && H / 8 <= 1024 && n > 0) {
    const int threads = static_cast<int>(ceil_div(H / 8, 64) * 64);
    hipLaunchKernelGGL(embed_bwd_small_kernel, dim3((unsigned)ceil_div(n, kSmallTok)), dim3(threads), 0, st,
                       (const bf16_t*)dy, ids, dtable, n, H, static_cast<int>(vocab));
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(gcap(n * H)), dim3(kT), 0, st, (const bf16_t*)dy, ids, dtable, n, H,
                     vocab);
  MDTF_LAUNCH_CHECK();
  return 0;
}
