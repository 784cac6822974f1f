// Memory-bound NHWC kernels: activations, pooling, softmax-xent, layout, LRN, column sums.
//
// Reference ops (distribute_tools.py): tf.nn.relu (:78,127), bias_add (:77,206),
// max_pool / avg_pool (:160-165), lrn (:185), sparse softmax cross entropy
// (user Loss), plus the NCHW<->NHWC transform and ResNet's
// global average pool.  All bf16 traffic is 16-byte vectorised (bf16x8 per
// lane); pooling backward is a deterministic gather (no atomics).
#include "mdtf_common.h"

using namespace mdtf;

namespace {

constexpr int kT = 256;

inline int grid_cap(long long work, int cap = 4096) {
  long long b = ceil_div(work, kT);
  return static_cast<int>(b < cap ? (b > 0 ? b : 1) : cap);
}

#define GRID_STRIDE(i, n) \
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

// ---------------------------------------------------------------- activations
// act: 0 none, 1 relu, 2 gelu(tanh)
__device__ __forceinline__ float act_f(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) {
    float u = 0.7978845608f * (v + 0.044715f * v * v * v);
    return 0.5f * v * (1.f + tanhf(u));
  }
  return v;
}

__device__ __forceinline__ float act_grad(float x, float y, int act) {
  // x: pre-activation, y: post-activation
  if (act == 1) return y > 0.f ? 1.f : 0.f;
  if (act == 2) {
    float x3 = x * x * x;
    float u = 0.7978845608f * (x + 0.044715f * x3);
    float t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608f * (1.f + 3.f * 0.044715f * x * x);
  }
  return 1.f;
}

__global__ void bias_act_fwd(const bf16_t* __restrict__ x, const float* __restrict__ bias, bf16_t* __restrict__ y,
                             bf16_t* __restrict__ pre, long long n8, int C, int act) {
  GRID_STRIDE(i, n8) {
    long long off = i * 8;
    int c = static_cast<int>(off % C);
    float v[8];
    load_bf8(x + off, v);
    if (bias) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += bias[c + k];
    }
    if (pre) store_bf8(pre + off, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_f(v[k], act);
    store_bf8(y + off, v);
  }
}

// dx = dy * act'(pre, y)
__global__ void act_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ pre, const bf16_t* __restrict__ y,
                        bf16_t* __restrict__ dx, long long n8, int act) {
  GRID_STRIDE(i, n8) {
    long long off = i * 8;
    float g[8], p[8], o[8];
    load_bf8(dy + off, g);
    if (act == 1) {
      load_bf8(y + off, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = o[k] > 0.f ? g[k] : 0.f;
    } else if (act == 2) {
      load_bf8(pre + off, p);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] *= act_grad(p[k], 0.f, 2);
    }
    store_bf8(dx + off, g);
  }
}

// generic (any C, any length) scalar variants for shapes that are not bf16x8 friendly
__global__ void bias_act_fwd_scalar(const bf16_t* __restrict__ x, const float* __restrict__ bias,
                                    bf16_t* __restrict__ y, bf16_t* __restrict__ pre, long long n, int C, int act) {
  GRID_STRIDE(i, n) {
    float v = bf2f(x[i]);
    if (bias) v += bias[i % C];
    if (pre) pre[i] = f2bf(v);
    y[i] = f2bf(act_f(v, act));
  }
}

__global__ void act_bwd_scalar(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ pre,
                               const bf16_t* __restrict__ y, bf16_t* __restrict__ dx, long long n, int act) {
  GRID_STRIDE(i, n) {
    float g = bf2f(dy[i]);
    if (act == 1) g = bf2f(y[i]) > 0.f ? g : 0.f;
    if (act == 2) g *= act_grad(bf2f(pre[i]), 0.f, 2);
    dx[i] = f2bf(g);
  }
}

__global__ void colsum_scalar(const bf16_t* __restrict__ x, long long M, int C, float* __restrict__ out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (long long r = blockIdx.y; r < M; r += gridDim.y) s += bf2f(x[r * C + c]);
  atomicAdd(out + c, s);
}

// column sums of a [M, C] bf16 matrix -> fp32 [C] (bias gradients), two stages,
// atomic-free in the hot part:
//   colsum_partial: block (bx, by) sums rows [bx*rpb, (bx+1)*rpb) of a 512-column
//     slab (64 lanes x bf16x8); each wave takes every 4th row with 4 independent
//     loads in flight, the 4 waves combine through LDS, one coalesced fp32 row
//     of partials per block goes to ws[bx][C];
//   reduce_partials: out[c] += sum_b ws[b][c] (64 columns x 4 row groups per
//     block, kSlices blocks per column slab, one atomic per column per slice).
constexpr int kColsumWaves = 2048;   // target waves in flight for the partial pass
constexpr int kSlices = 8;

__global__ void __launch_bounds__(kT) colsum_partial(const bf16_t* __restrict__ x, long long M, int C, int rpb,
                                                     float* __restrict__ ws) {
  const int cv = C / 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cvec = blockIdx.y * 64 + lane;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = r0 + rpb < M ? r0 + rpb : M;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cvec < cv) {
    long long r = r0 + wave;
    for (; r + 12 < r1; r += 16) {
      float a[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_bf8(x + (r + 4 * u) * C + cvec * 8, a[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += a[u][k];
    }
    for (; r < r1; r += 4) {
      float a[8];
      load_bf8(x + r * C + cvec * 8, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += a[k];
    }
  }
  __shared__ float L[4][64 * 8];
#pragma unroll
  for (int k = 0; k < 8; ++k) L[wave][lane * 8 + k] = s[k];
  __syncthreads();
  // 256 threads write the slab's 512 partial columns, two each, coalesced
  for (int j = threadIdx.x; j < 512; j += kT) {
    const int col = blockIdx.y * 512 + j;
    if (col < C) ws[(long long)blockIdx.x * C + col] = L[0][j] + L[1][j] + L[2][j] + L[3][j];
  }
}

__global__ void __launch_bounds__(kT) reduce_partials(const float* __restrict__ ws, int B, int C, long long ld,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float t = 0.f;
  if (c < C) {
    int b = blockIdx.y * 4 + grp;
    const int step = gridDim.y * 4;
    for (; b + 3 * step < B; b += 4 * step)
      t += ws[(long long)b * ld + c] + ws[(long long)(b + step) * ld + c] + ws[(long long)(b + 2 * step) * ld + c] +
           ws[(long long)(b + 3 * step) * ld + c];
    for (; b < B; b += step) t += ws[(long long)b * ld + c];
  }
  __shared__ float L[4][64];
  L[grp][lane] = t;
  __syncthreads();
  if (grp == 0 && c < C) atomicAdd(out + c, L[0][lane] + L[1][lane] + L[2][lane] + L[3][lane]);
}

void colsum_geometry(long long M, int C, int* gx, int* rpb) {
  const int gy = static_cast<int>(ceil_div(C / 8, 64));
  long long want = kColsumWaves / 4 / gy;
  if (want < 1) want = 1;
  long long g = ceil_div(M, 16);
  if (g > want) g = want;
  if (g < 1) g = 1;
  *rpb = static_cast<int>(ceil_div(M, g));
  *gx = static_cast<int>(ceil_div(M, *rpb));
}

// ---------------------------------------------------------------- pooling
struct PoolGeo {
  int N, H, W, C, OH, OW, KH, KW, SH, SW, PT, PL;
};

// Max pooling, one 8-channel vector per thread and one contiguous chunk of vectors per block
// (index math in IDX = int when the tensor has < 2^31 vectors: 64-bit divisions per element made
// the grid-stride version run at ~2 TB/s).
template <typename IDX>
__global__ void __launch_bounds__(kT) maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                  uint8_t* __restrict__ arg, PoolGeo g, IDX total) {
  const IDX i = (IDX)blockIdx.x * kT + threadIdx.x;
  if (i >= total) return;
  const int cv = g.C / 8;
  const int c8 = static_cast<int>(i % cv);
  IDX p = i / cv;
  const int ow = static_cast<int>(p % g.OW);
  p /= g.OW;
  const int oh = static_cast<int>(p % g.OH);
  const IDX n = p / g.OH;
  float best[8];
  uint8_t bi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    best[k] = -INFINITY;
    bi[k] = 0;
  }
  for (int kh = 0; kh < g.KH; ++kh) {
    const int h = oh * g.SH - g.PT + kh;
    if (h < 0 || h >= g.H) continue;
    for (int kw = 0; kw < g.KW; ++kw) {
      const int w = ow * g.SW - g.PL + kw;
      if (w < 0 || w >= g.W) continue;
      float v[8];
      load_bf8(x + ((long long)((n * g.H + h) * g.W + w)) * g.C + c8 * 8, v);
      const uint8_t idx = static_cast<uint8_t>(kh * g.KW + kw);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (v[k] > best[k]) {
          best[k] = v[k];
          bi[k] = idx;
        }
    }
  }
  const long long o = (long long)i * 8;
  store_bf8(y + o, best);
  if (arg) {
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + o) = packed;
  }
}

// gather form: each input vector collects dy from every window whose argmax it is
template <typename IDX>
__global__ void __launch_bounds__(kT) maxpool_bwd(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                  bf16_t* __restrict__ dx, PoolGeo g, IDX total) {
  const IDX i = (IDX)blockIdx.x * kT + threadIdx.x;
  if (i >= total) return;
  const int cv = g.C / 8;
  const int c8 = static_cast<int>(i % cv);
  IDX p = i / cv;
  const int w = static_cast<int>(p % g.W);
  p /= g.W;
  const int h = static_cast<int>(p % g.H);
  const IDX n = p / g.H;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int oh0 = h + g.PT - g.KH + 1 + g.SH - 1;
  oh0 = oh0 < 0 ? 0 : oh0 / g.SH;
  int oh1 = (h + g.PT) / g.SH;
  int ow0 = w + g.PL - g.KW + 1 + g.SW - 1;
  ow0 = ow0 < 0 ? 0 : ow0 / g.SW;
  int ow1 = (w + g.PL) / g.SW;
  if (oh1 >= g.OH) oh1 = g.OH - 1;
  if (ow1 >= g.OW) ow1 = g.OW - 1;
  for (int oh = oh0; oh <= oh1; ++oh) {
    const int kh = h - (oh * g.SH - g.PT);
    if (kh < 0 || kh >= g.KH) continue;
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int kw = w - (ow * g.SW - g.PL);
      if (kw < 0 || kw >= g.KW) continue;
      const long long o = (long long)((n * g.OH + oh) * g.OW + ow) * g.C + c8 * 8;
      const uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
      const uint32_t me = static_cast<uint32_t>(kh * g.KW + kw);
      float gv[8];
      load_bf8(dy + o, gv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t id = ((k < 4 ? packed.x : packed.y) >> (8 * (k & 3))) & 0xffu;
        if (id == me) acc[k] += gv[k];
      }
    }
  }
  store_bf8(dx + (long long)i * 8, acc);
}

__device__ __forceinline__ int win_count(const PoolGeo& g, int oh, int ow) {
  int h0 = oh * g.SH - g.PT, w0 = ow * g.SW - g.PL;
  int h1 = min(h0 + g.KH, g.H), w1 = min(w0 + g.KW, g.W);
  h0 = max(h0, 0);
  w0 = max(w0, 0);
  return (h1 - h0) * (w1 - w0);
}

__global__ void avgpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, PoolGeo g) {
  const int cv = g.C / 8;
  long long total = (long long)g.N * g.OH * g.OW * cv;
  GRID_STRIDE(i, total) {
    int c8 = static_cast<int>(i % cv);
    long long p = i / cv;
    int ow = static_cast<int>(p % g.OW);
    p /= g.OW;
    int oh = static_cast<int>(p % g.OH);
    int n = static_cast<int>(p / g.OH);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int kh = 0; kh < g.KH; ++kh) {
      int h = oh * g.SH - g.PT + kh;
      if (h < 0 || h >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        int w = ow * g.SW - g.PL + kw;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        load_bf8(x + (((long long)n * g.H + h) * g.W + w) * g.C + c8 * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[k];
      }
    }
    float inv = 1.f / (float)win_count(g, oh, ow);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= inv;
    store_bf8(y + (((long long)n * g.OH + oh) * g.OW + ow) * g.C + c8 * 8, acc);
  }
}

__global__ void avgpool_bwd(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, PoolGeo g) {
  const int cv = g.C / 8;
  long long total = (long long)g.N * g.H * g.W * cv;
  GRID_STRIDE(i, total) {
    int c8 = static_cast<int>(i % cv);
    long long p = i / cv;
    int w = static_cast<int>(p % g.W);
    p /= g.W;
    int h = static_cast<int>(p % g.H);
    int n = static_cast<int>(p / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int oh0 = h + g.PT - g.KH + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + g.SH - 1) / g.SH;
    int oh1 = min((h + g.PT) / g.SH, g.OH - 1);
    int ow0 = w + g.PL - g.KW + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + g.SW - 1) / g.SW;
    int ow1 = min((w + g.PL) / g.SW, g.OW - 1);
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        float gv[8];
        load_bf8(dy + (((long long)n * g.OH + oh) * g.OW + ow) * g.C + c8 * 8, gv);
        float inv = 1.f / (float)win_count(g, oh, ow);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += gv[k] * inv;
      }
    store_bf8(dx + (((long long)n * g.H + h) * g.W + w) * g.C + c8 * 8, acc);
  }
}

// global average pool [N, HW, C] -> [N, C]; block = (n, 512-channel slab), 4 row groups
__global__ void gap_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int HW, int C) {
  const int n = blockIdx.x;
  const int lane = threadIdx.x % 64, grp = threadIdx.x / 64;
  const int cvec = blockIdx.y * 64 + lane;
  const int cv = C / 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cvec < cv)
    for (int r = grp; r < HW; r += 4) {
      float v[8];
      load_bf8(x + ((long long)n * HW + r) * C + cvec * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
  __shared__ float L[4][64 * 8];
#pragma unroll
  for (int k = 0; k < 8; ++k) L[grp][lane * 8 + k] = s[k];
  __syncthreads();
  if (grp == 0 && cvec < cv) {
    float o[8];
    float inv = 1.f / (float)HW;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      o[k] = (L[0][lane * 8 + k] + L[1][lane * 8 + k] + L[2][lane * 8 + k] + L[3][lane * 8 + k]) * inv;
    store_bf8(y + (long long)n * C + cvec * 8, o);
  }
}

__global__ void gap_bwd(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW, int C) {
  const int cv = C / 8;
  long long total = (long long)N * HW * cv;
  float inv = 1.f / (float)HW;
  GRID_STRIDE(i, total) {
    int c8 = static_cast<int>(i % cv);
    int n = static_cast<int>(i / ((long long)HW * cv));
    float g[8];
    load_bf8(dy + (long long)n * C + c8 * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] *= inv;
    store_bf8(dx + i * 8, g);
  }
}

// ---------------------------------------------------------------- softmax cross entropy
// one wave per row; logits bf16 or fp32 (is_bf16); loss[n], lse[n] fp32
template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) {
  return bf2f(p[i]);
}
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) {
  return p[i];
}

template <typename T>
__global__ void xent_fwd(const T* __restrict__ logits, const long long* __restrict__ labels, int N, int K,
                         long long ldr, float* __restrict__ loss, float* __restrict__ lse) {
  int row = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  int lane = threadIdx.x % 64;
  if (row >= N) return;
  const T* p = logits + (long long)row * ldr;
  float m = -INFINITY;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, ld(p, k));
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += __expf(ld(p, k) - m);
  s = wave_sum(s);
  if (lane == 0) {
    float l = m + __logf(s);
    long long lab = labels[row];
    float xl = (lab >= 0 && lab < K) ? ld(p, lab) : 0.f;
    lse[row] = l;
    loss[row] = l - xl;
  }
}

// one 256-thread block per row: a single online pass (running max, rescaled exp-sum) over
// 4-byte bf16 pairs (rows of an even vocabulary are 4-byte aligned), then a (max, sum)
// reduction across the block; the label's logit is read by thread 0
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
  m = mn;
}

__global__ void __launch_bounds__(256) xent_fwd_row_bf16(const bf16_t* __restrict__ logits,
                                                         const long long* __restrict__ labels, int K, long long ld,
                                                         float* __restrict__ loss, float* __restrict__ lse) {
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* p = logits + (long long)row * ld;
  const uint32_t* p2 = reinterpret_cast<const uint32_t*>(p);
  const int K2 = K >> 1;
  float m = -INFINITY, s = 0.f;
  for (int k = tid; k < K2; k += 256) {
    const uint32_t w = p2[k];
    const float a = __uint_as_float(w << 16), b = __uint_as_float(w & 0xffff0000u);
    const float mx = fmaxf(a, b);
    if (mx > m) {
      s = (m == -INFINITY ? 0.f : s * __expf(m - mx));
      m = mx;
    }
    s += __expf(a - m) + __expf(b - m);
  }
  if ((K & 1) && tid == 0) lse_merge(m, s, bf2f(p[K - 1]), 1.f);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  __shared__ float sm[4], ss[4];
  if ((tid & 63) == 0) {
    sm[tid >> 6] = m;
    ss[tid >> 6] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float M = sm[0], S = ss[0];
    for (int w = 1; w < 4; ++w) lse_merge(M, S, sm[w], ss[w]);
    const float l = M + __logf(S);
    const long long lab = labels[row];
    const float xl = (lab >= 0 && lab < K) ? bf2f(p[lab]) : 0.f;
    lse[row] = l;
    loss[row] = l - xl;
  }
}

// rows 16-B aligned with a stride that is a multiple of 8 (the padded decoder's [rows][30720] logits): 16-B loads,
// four in flight per thread, columns >= K masked out; the same online (max, sum) merge as xent_fwd_row_bf16
__global__ void __launch_bounds__(256) xent_fwd_row_v8(const bf16_t* __restrict__ logits,
                                                       const long long* __restrict__ labels, int K, long long ld,
                                                       float* __restrict__ loss, float* __restrict__ lse) {
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* p = logits + (long long)row * ld;
  const int kv = (K + 7) >> 3;
  float m = -INFINITY, s = 0.f;
  auto eat = [&](const uint4& w, int v) {
    const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
    float a[8];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      a[2 * h] = v * 8 + 2 * h < K ? __uint_as_float(wv[h] << 16) : -INFINITY;
      a[2 * h + 1] = v * 8 + 2 * h + 1 < K ? __uint_as_float(wv[h] & 0xffff0000u) : -INFINITY;
    }
    float mx = a[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mx = fmaxf(mx, a[j]);
    if (mx > m) {
      s = (m == -INFINITY ? 0.f : s * __expf(m - mx));
      m = mx;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(a[j] - m);
  };
  int v = tid;
  for (; v + 3 * 256 < kv; v += 4 * 256) {
    uint4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = *reinterpret_cast<const uint4*>(p + (v + u * 256) * 8);
#pragma unroll
    for (int u = 0; u < 4; ++u) eat(w[u], v + u * 256);
  }
  for (; v < kv; v += 256) eat(*reinterpret_cast<const uint4*>(p + v * 8), v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  __shared__ float sm[4], ss[4];
  if ((tid & 63) == 0) {
    sm[tid >> 6] = m;
    ss[tid >> 6] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float M = sm[0], S = ss[0];
    for (int w = 1; w < 4; ++w) lse_merge(M, S, sm[w], ss[w]);
    const float l = M + __logf(S);
    const long long lab = labels[row];
    const float xl = (lab >= 0 && lab < K) ? bf2f(p[lab]) : 0.f;
    lse[row] = l;
    loss[row] = l - xl;
  }
}

template <typename T>
__global__ void xent_bwd(const T* __restrict__ logits, const long long* __restrict__ labels,
                         const float* __restrict__ lse, const float* __restrict__ dloss, T* __restrict__ dlogits,
                         int N, int K, long long ldi, long long ldo) {
  long long total = (long long)N * K;
  GRID_STRIDE(i, total) {
    int row = static_cast<int>(i / K);
    int k = static_cast<int>(i % K);
    float pr = __expf(ld(logits, row * ldi + k) - lse[row]);
    float g = (pr - (labels[row] == k ? 1.f : 0.f)) * dloss[row];
    if constexpr (sizeof(T) == 2)
      dlogits[row * ldo + k] = f2bf(g);
    else
      dlogits[row * ldo + k] = g;
  }
}

// bf16 rows whose strides are multiples of 8 (the padded MLM decoder's [rows][30720] logits): one 256-thread block
// per row, 16-B vectors, no per-element division; columns K .. ldo of the output row are written as zeros (the
// decoder's split-K data gradient and weight gradient read the whole padded row)
__global__ void __launch_bounds__(256) xent_bwd_row_bf16(const bf16_t* __restrict__ logits,
                                                         const long long* __restrict__ labels,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ dloss, bf16_t* __restrict__ dlogits,
                                                         int K, long long ldi, long long ldo) {
  const int row = blockIdx.x;
  const float l = lse[row], dl = dloss[row];
  const long long lab = labels[row];
  const bf16_t* p = logits + row * ldi;
  bf16_t* q = dlogits + row * ldo;
  const int nv = static_cast<int>(ldo >> 3), kv = (K + 7) >> 3;
  for (int v = threadIdx.x; v < nv; v += 256) {
    uint4 o = {0u, 0u, 0u, 0u};
    if (v < kv) {
      const uint4 w = *reinterpret_cast<const uint4*>(p + v * 8);
      const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
      uint32_t ov[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int k0 = v * 8 + 2 * h;
        float g0 = __expf(__uint_as_float(wv[h] << 16) - l) - (lab == k0 ? 1.f : 0.f);
        float g1 = __expf(__uint_as_float(wv[h] & 0xffff0000u) - l) - (lab == k0 + 1 ? 1.f : 0.f);
        g0 = k0 < K ? g0 * dl : 0.f;
        g1 = k0 + 1 < K ? g1 * dl : 0.f;
        ov[h] = f2bf(g0) | (f2bf(g1) << 16);
      }
      o = {ov[0], ov[1], ov[2], ov[3]};
    }
    *reinterpret_cast<uint4*>(q + v * 8) = o;
  }
}

// ---------------------------------------------------------------- layout transform
// [B, R, S] -> [B, S, R] (NCHW->NHWC: R=C, S=HW; NHWC->NCHW: R=HW, S=C)
template <typename T>
__global__ void transpose_kernel(const T* __restrict__ in, T* __restrict__ out, int R, int S) {
  __shared__ T tile[64][65];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 64, s0 = blockIdx.x * 64;
  const T* src = in + (long long)b * R * S;
  T* dst = out + (long long)b * R * S;
  const int tx = threadIdx.x % 64, ty = threadIdx.x / 64;  // 64 x 4
  for (int r = ty; r < 64; r += 4)
    if (r0 + r < R && s0 + tx < S) tile[r][tx] = src[(long long)(r0 + r) * S + s0 + tx];
  __syncthreads();
  for (int s = ty; s < 64; s += 4)
    if (s0 + s < S && r0 + tx < R) dst[(long long)(s0 + s) * R + r0 + tx] = tile[tx][s];
}

// bf16 [B, R, S] -> [B, S, R] in 64x64 tiles, 16-B global accesses on both sides:
// each thread loads 2 x 8 consecutive s of one r row, the tile is stored
// transposed in LDS (pad 1 column per 64: conflict-light scalar writes), then
// each thread emits 2 x 8 consecutive r of one s row.  Requires R % 8 == S % 8 == 0.
__global__ void __launch_bounds__(256) transpose16_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                          int R, int S) {
  __shared__ uint16_t tile[64][66];   // [s][r]
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 64, s0 = blockIdx.x * 64;
  const uint16_t* src = in + (long long)b * R * S;
  uint16_t* dst = out + (long long)b * R * S;
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = t + h * 256;           // 512 chunks: 64 rows x 8 chunks
    const int rr = idx >> 3, sc = (idx & 7) * 8;
    if (r0 + rr < R && s0 + sc < S) {
      uint4 v = *reinterpret_cast<const uint4*>(src + (long long)(r0 + rr) * S + s0 + sc);
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) tile[sc + k][rr] = e[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = t + h * 256;
    const int ss = idx >> 3, rc = (idx & 7) * 8;
    if (s0 + ss < S && r0 + rc < R) {
      uint4 v;
      uint16_t* e = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = tile[ss][rc + k];
      *reinterpret_cast<uint4*>(dst + (long long)(s0 + ss) * R + r0 + rc) = v;
    }
  }
}

// ---------------------------------------------------------------- LRN (cross-channel)
__global__ void lrn_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, float* __restrict__ dsave, long long P,
                        int C, int r, float bias, float alpha, float beta) {
  long long total = P * C;
  GRID_STRIDE(i, total) {
    int c = static_cast<int>(i % C);
    long long base = i - c;
    float s = 0.f;
    for (int j = max(0, c - r); j <= min(C - 1, c + r); ++j) {
      float v = bf2f(x[base + j]);
      s += v * v;
    }
    float d = bias + alpha * s;
    dsave[i] = d;
    y[i] = f2bf(bf2f(x[i]) * __powf(d, -beta));
  }
}

__global__ void lrn_bwd(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                        const float* __restrict__ dsave, bf16_t* __restrict__ dx, long long P, int C, int r,
                        float alpha, float beta) {
  long long total = P * C;
  GRID_STRIDE(i, total) {
    int c = static_cast<int>(i % C);
    long long base = i - c;
    float xi = bf2f(x[i]);
    float acc = bf2f(dy[i]) * __powf(dsave[i], -beta);
    float t = 0.f;
    for (int j = max(0, c - r); j <= min(C - 1, c + r); ++j)
      t += bf2f(dy[base + j]) * bf2f(y[base + j]) / dsave[base + j];
    acc -= 2.f * alpha * beta * xi * t;
    dx[i] = f2bf(acc);
  }
}

// out = g * [mask bit] (+ out): materialise a ReLU-masked gradient a fan-out sink held unmaterialised
__global__ void __launch_bounds__(256) mask_mul_kernel(const uint4* __restrict__ g, const uint8_t* __restrict__ mask,
                                                      uint4* __restrict__ out, long long n8, int accumulate) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const uint4 v = g[i];
  const uint32_t m = mask[i];
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  float f[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = ((m >> (2 * k)) & 1u) ? __uint_as_float(w[k] << 16) : 0.f;
    f[2 * k + 1] = ((m >> (2 * k + 1)) & 1u) ? __uint_as_float(w[k] & 0xffff0000u) : 0.f;
  }
  if (accumulate) {
    const uint4 o = out[i];
    const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] += __uint_as_float(ow[k] << 16);
      f[2 * k + 1] += __uint_as_float(ow[k] & 0xffff0000u);
    }
  }
  store_bf8(reinterpret_cast<bf16_t*>(out + i), f);
}

// Zero the nr float ranges of a buffer in one launch (a gradient buffer whose store-written slots are skipped):
// rg = [nr][2] (start, length) in elements, ascending, disjoint; each block owns 4096 elements of the
// concatenation of the ranges; rows = {prefix of lengths} staged in LDS, one binary search per 4-element group.
constexpr int kFillMaxRanges = 1024;
__global__ void __launch_bounds__(256) fill_ranges_kernel(float* __restrict__ base, const long long* __restrict__ rg,
                                                          int nr, long long total) {
  __shared__ long long pre[kFillMaxRanges + 1];
  __shared__ long long st[kFillMaxRanges];
  // prefix sums: every thread loads starts / lengths in parallel; thread 0 scans them in LDS (nr is small)
  for (int r = threadIdx.x; r < nr; r += 256) {
    st[r] = rg[2 * r];
    pre[r + 1] = rg[2 * r + 1];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    pre[0] = 0;
    for (int r = 0; r < nr; ++r) pre[r + 1] += pre[r];
  }
  __syncthreads();
  const long long e0 = (long long)blockIdx.x * 4096;
  for (int q = threadIdx.x; q < 1024; q += 256) {
    const long long e = e0 + 4LL * q;
    if (e >= total) break;
    int lo = 0, hi = nr - 1;               // largest r with pre[r] <= e
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= e) lo = mid; else hi = mid - 1;
    }
    long long p = st[lo] + (e - pre[lo]);
    const long long left = pre[lo + 1] - e;   // elements left in this range
    if (left >= 4 && (p & 3) == 0) {
      *reinterpret_cast<float4*>(base + p) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      int r = lo;
      for (int k = 0; k < 4 && e + k < total; ++k) {
        while (e + k >= pre[r + 1]) ++r;
        base[st[r] + (e + k - pre[r])] = 0.f;
      }
    }
  }
}

}  // namespace

MDTF_EXPORT int mdtf_fill_ranges_zero(float* base, const long long* ranges, int nr, long long total, hipStream_t st) {
  if (nr <= 0 || total <= 0) return 0;
  if (nr > kFillMaxRanges) return MDTF_EUNSUPPORTED;
  hipLaunchKernelGGL(fill_ranges_kernel, dim3((unsigned)ceil_div(total, 4096)), dim3(256), 0, st, base, ranges, nr,
                     total);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// ============================================================== exports
MDTF_EXPORT int mdtf_bias_act_fwd(const void* x, const float* bias, void* y, void* pre, long long M, int C, int act,
                                  hipStream_t st) {
  if (C % 8) {
    hipLaunchKernelGGL(bias_act_fwd_scalar, dim3(grid_cap(M * C)), dim3(kT), 0, st, (const bf16_t*)x, bias,
                       (bf16_t*)y, (bf16_t*)pre, M * C, C, act);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  long long n8 = M * C / 8;
  hipLaunchKernelGGL(bias_act_fwd, dim3(grid_cap(n8)), dim3(kT), 0, st, (const bf16_t*)x, bias, (bf16_t*)y,
                     (bf16_t*)pre, n8, C, act);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_act_bwd(const void* dy, const void* pre, const void* y, void* dx, long long n, int act,
                             hipStream_t st) {
  if (n % 8) {
    hipLaunchKernelGGL(act_bwd_scalar, dim3(grid_cap(n)), dim3(kT), 0, st, (const bf16_t*)dy, (const bf16_t*)pre,
                       (const bf16_t*)y, (bf16_t*)dx, n, act);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(act_bwd, dim3(grid_cap(n / 8)), dim3(kT), 0, st, (const bf16_t*)dy, (const bf16_t*)pre,
                     (const bf16_t*)y, (bf16_t*)dx, n / 8, act);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// out must be zeroed by the caller
// out[c] += sum_b ws[b][c]   (shared by every two-stage column reduction)
int g_deterministic = 0;   // 1: fixed-order reductions (no cross-block float atomics)

// (row stride ld >= C)
MDTF_EXPORT int mdtf_reduce_partials_strided(const float* ws, int B, int C, long long ld, float* out, hipStream_t st) {
  int slices = B < kSlices * 4 ? static_cast<int>(ceil_div(B, 4)) : kSlices;
  if (slices < 1 || g_deterministic) slices = 1;
  hipLaunchKernelGGL(reduce_partials, dim3(ceil_div(C, 64), slices), dim3(kT), 0, st, ws, B, C, ld, out);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_mask_mul(const void* g, const void* mask, void* out, long long n, int accumulate,
                              hipStream_t st) {
  if (n % 8) return MDTF_EINVAL;
  const long long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(mask_mul_kernel, dim3((unsigned)ceil_div(n8, 256LL)), dim3(256), 0, st, (const uint4*)g,
                     (const uint8_t*)mask, (uint4*)out, n8, accumulate);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT void mdtf_set_deterministic(int on) { g_deterministic = on ? 1 : 0; }
MDTF_EXPORT int mdtf_get_deterministic() { return g_deterministic; }

MDTF_EXPORT int mdtf_reduce_partials(const float* ws, int B, int C, float* out, hipStream_t st) {
  return mdtf_reduce_partials_strided(ws, B, C, C, out, st);
}

// fp32 workspace (elements) mdtf_colsum needs for an [M, C] input
MDTF_EXPORT long long mdtf_colsum_ws(long long M, int C) {
  if (C % 8) return 0;
  int gx, rpb;
  colsum_geometry(M, C, &gx, &rpb);
  return (long long)gx * C;
}

// out[c] += sum_r x[r][c]; ws: mdtf_colsum_ws(M, C) floats (unused when C % 8)
MDTF_EXPORT int mdtf_colsum(const void* x, long long M, int C, float* out, float* ws, hipStream_t st) {
  if (M <= 0) return 0;
  if (C % 8) {
    long long gy = M < 256 ? M : 256;
    hipLaunchKernelGGL(colsum_scalar, dim3(ceil_div(C, kT), gy > 0 ? gy : 1), dim3(kT), 0, st, (const bf16_t*)x, M, C,
                       out);
    MDTF_LAUNCH_CHECK();
    return 0;
  }
  int gx, rpb;
  colsum_geometry(M, C, &gx, &rpb);
  const int gy = static_cast<int>(ceil_div(C / 8, 64));
  hipLaunchKernelGGL(colsum_partial, dim3(gx, gy), dim3(kT), 0, st, (const bf16_t*)x, M, C, rpb, ws);
  MDTF_LAUNCH_CHECK();
  return mdtf_reduce_partials(ws, gx, C, out, st);
}

MDTF_EXPORT int mdtf_pool_fwd(int is_max, const void* x, void* y, void* argmax, int N, int H, int W, int C, int OH,
                              int OW, int KH, int KW, int SH, int SW, int PT, int PL, hipStream_t st) {
  if (C % 8 || KH * KW > 255) return MDTF_EINVAL;
  PoolGeo g{N, H, W, C, OH, OW, KH, KW, SH, SW, PT, PL};
  long long work = (long long)N * OH * OW * (C / 8);
  if (is_max) {
    const dim3 grid((unsigned)ceil_div(work, kT));
    if (work < 0x7fffffffLL && (long long)N * H * W * C < 0x7fffffffLL)
      hipLaunchKernelGGL(maxpool_fwd<int>, grid, dim3(kT), 0, st, (const bf16_t*)x, (bf16_t*)y, (uint8_t*)argmax, g,
                         (int)work);
    else
      hipLaunchKernelGGL(maxpool_fwd<long long>, grid, dim3(kT), 0, st, (const bf16_t*)x, (bf16_t*)y,
                         (uint8_t*)argmax, g, work);
  } else
    hipLaunchKernelGGL(avgpool_fwd, dim3(grid_cap(work)), dim3(kT), 0, st, (const bf16_t*)x, (bf16_t*)y, g);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_pool_bwd(int is_max, const void* dy, const void* argmax, void* dx, int N, int H, int W, int C,
                              int OH, int OW, int KH, int KW, int SH, int SW, int PT, int PL, hipStream_t st) {
  if (C % 8) return MDTF_EINVAL;
  PoolGeo g{N, H, W, C, OH, OW, KH, KW, SH, SW, PT, PL};
  long long work = (long long)N * H * W * (C / 8);
  if (is_max) {
    const dim3 grid((unsigned)ceil_div(work, kT));
    if (work < 0x7fffffffLL && (long long)N * H * W * C < 0x7fffffffLL)
      hipLaunchKernelGGL(maxpool_bwd<int>, grid, dim3(kT), 0, st, (const bf16_t*)dy, (const uint8_t*)argmax,
                         (bf16_t*)dx, g, (int)work);
    else
      hipLaunchKernelGGL(maxpool_bwd<long long>, grid, dim3(kT), 0, st, (const bf16_t*)dy, (const uint8_t*)argmax,
                         (bf16_t*)dx, g, work);
  } else
    hipLaunchKernelGGL(avgpool_bwd, dim3(grid_cap(work)), dim3(kT), 0, st, (const bf16_t*)dy, (bf16_t*)dx, g);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return MDTF_EINVAL;
  hipLaunchKernelGGL(gap_fwd, dim3(N, ceil_div(C / 8, 64)), dim3(kT), 0, st, (const bf16_t*)x, (bf16_t*)y, HW, C);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return MDTF_EINVAL;
  hipLaunchKernelGGL(gap_bwd, dim3(grid_cap((long long)N * HW * C / 8)), dim3(kT), 0, st, (const bf16_t*)dy,
                     (bf16_t*)dx, N, HW, C);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// logits rows ld elements apart (ld >= K)
MDTF_EXPORT int mdtf_xent_fwd(const void* logits, int is_bf16, const long long* labels, int N, int K, long long ld,
                              float* loss, float* lse, hipStream_t st) {
  if (ld < K) return MDTF_EINVAL;
  dim3 grid(ceil_div(N, 4));
  if (is_bf16 && K >= 2048 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0 && (ld & 7) == 0)
    hipLaunchKernelGGL(xent_fwd_row_v8, dim3(N), dim3(256), 0, st, (const bf16_t*)logits, labels, K, ld, loss, lse);
  else if (is_bf16 && K >= 2048 && (reinterpret_cast<uintptr_t>(logits) & 3) == 0 && (K & 1) == 0 && (ld & 1) == 0)
    hipLaunchKernelGGL(xent_fwd_row_bf16, dim3(N), dim3(256), 0, st, (const bf16_t*)logits, labels, K, ld, loss, lse);
  else if (is_bf16)
    hipLaunchKernelGGL(xent_fwd<bf16_t>, grid, dim3(kT), 0, st, (const bf16_t*)logits, labels, N, K, ld, loss, lse);
  else
    hipLaunchKernelGGL(xent_fwd<float>, grid, dim3(kT), 0, st, (const float*)logits, labels, N, K, ld, loss, lse);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// dlogits rows ldo elements apart; with the vector kernel (bf16, strides multiples of 8, 16-B aligned rows) the
// columns K .. ldo are zero-filled, otherwise left untouched
MDTF_EXPORT int mdtf_xent_bwd(const void* logits, int is_bf16, const long long* labels, const float* lse,
                              const float* dloss, void* dlogits, int N, int K, long long ldi, long long ldo,
                              hipStream_t st) {
  if (ldi < K || ldo < K) return MDTF_EINVAL;
  const bool vec = is_bf16 && (ldi % 8) == 0 && (ldo % 8) == 0 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(dlogits) & 15) == 0;
  long long total = (long long)N * K;
  if (vec)
    hipLaunchKernelGGL(xent_bwd_row_bf16, dim3(N), dim3(256), 0, st, (const bf16_t*)logits, labels, lse, dloss,
                       (bf16_t*)dlogits, K, ldi, ldo);
  else if (is_bf16)
    hipLaunchKernelGGL(xent_bwd<bf16_t>, dim3(grid_cap(total)), dim3(kT), 0, st, (const bf16_t*)logits, labels, lse,
                       dloss, (bf16_t*)dlogits, N, K, ldi, ldo);
  else
    hipLaunchKernelGGL(xent_bwd<float>, dim3(grid_cap(total)), dim3(kT), 0, st, (const float*)logits, labels, lse,
                       dloss, (float*)dlogits, N, K, ldi, ldo);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// elem_bytes: 2 (bf16/fp16) or 4 (fp32)
// Many [R][S] -> [S][R] bf16 transposes in ONE launch (every conv filter -> its K-contiguous copy, once per
// step): desc[i] = {src, dst, R | S << 32, first tile, tiles along S}; block b serves the descriptor whose
// tile range holds b (linear scan over <= a few hundred scalar-loaded entries).
struct TDesc {
  const uint16_t* src;
  uint16_t* dst;
  long long rs;
  int tile0, ts;
};

// Index of the last record whose first block is <= b, records sorted by first block (f0: that int field of record
// 0, stride: record size).  Wave-parallel: each lane loads one record's field and a ballot counts the prefix, one
// global round trip per 64 records.  (A per-thread linear scan was one dependent scalar load per record: ~36-53
// round trips per block before any data moved -- copy2d_multi 40 us for 84 MB, transpose16_multi 30 us.)
__device__ __forceinline__ int find_record(const char* f0, int stride, int count, int b) {
  const int lane = threadIdx.x & 63;
  int i = 0;
  for (int base = 0; base < count; base += 64) {
    const int r = base + lane;
    const int v = r < count ? *reinterpret_cast<const int*>(f0 + (long long)r * stride) : 0x7fffffff;
    const int c = __popcll(__ballot(v <= b));
    i = base + c - 1;
    if (c < 64) break;
  }
  return i < 0 ? 0 : i;
}

__global__ void __launch_bounds__(256) transpose16_multi(const TDesc* __restrict__ desc, int count) {
  __shared__ uint16_t tile[64][66];
  const int i = find_record(reinterpret_cast<const char*>(&desc[0].tile0), (int)sizeof(TDesc), count,
                            (int)blockIdx.x);
  const TDesc d = desc[i];
  const int R = (int)(d.rs & 0xffffffff), S = (int)(d.rs >> 32);
  const int local = blockIdx.x - d.tile0;
  const int r0 = (local / d.ts) * 64, s0 = (local % d.ts) * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = t + h * 256;
    const int rr = idx >> 3, sc = (idx & 7) * 8;
    if (r0 + rr < R && s0 + sc < S) {
      uint4 v = *reinterpret_cast<const uint4*>(d.src + (long long)(r0 + rr) * S + s0 + sc);
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) tile[sc + k][rr] = e[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = t + h * 256;
    const int ss = idx >> 3, rc = (idx & 7) * 8;
    if (s0 + ss < S && r0 + rc < R) {
      uint4 v;
      uint16_t* e = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = tile[ss][rc + k];
      *reinterpret_cast<uint4*>(d.dst + (long long)(s0 + ss) * R + r0 + rc) = v;
    }
  }
}

// Batched 2-D copies (16-B vectors): dst[r][0:cols] = src[r][0:cols] for every record, each record a block range.
// The q|k|v weight concatenation of every transformer layer in one launch per step (ops.gemm _WeightCats).
struct CDesc {
  const uint4* src;
  uint4* dst;
  int rows, vcols;            // rows, 16-B vectors per row
  int src_ld, dst_ld;         // row strides in 16-B vectors
  int block0, pad;
};

__global__ void __launch_bounds__(256) copy2d_multi(const CDesc* __restrict__ desc, int count) {
  const int i = find_record(reinterpret_cast<const char*>(&desc[0].block0), (int)sizeof(CDesc), count,
                            (int)blockIdx.x);
  const CDesc d = desc[i];
  // each block: 256 threads x 4 vectors, rows walked in row-major vector order.  32-bit index math, one division
  // per vector (the host keeps rows * vcols < 2^31): the 64-bit divisions this loop had (twice per vector) were
  // ~800 VALU instructions per thread for 64 B moved, 1.9 TB/s on BERT-base's q|k|v weights
  const unsigned base = (unsigned)(blockIdx.x - d.block0) * 1024u + threadIdx.x;
  const unsigned n = (unsigned)d.rows * (unsigned)d.vcols;
  const unsigned vc = (unsigned)d.vcols;
  uint4 v[4];
  unsigned doff[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const unsigned idx = base + u * 256u;
    doff[u] = 0xffffffffu;
    if (idx < n) {
      const unsigned r = idx / vc, c = idx - r * vc;
      v[u] = d.src[(size_t)r * d.src_ld + c];
      doff[u] = r * (unsigned)d.dst_ld + c;
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (doff[u] != 0xffffffffu) d.dst[doff[u]] = v[u];
}

MDTF_EXPORT int mdtf_copy2d_multi(const void* desc, int count, int total_blocks, hipStream_t st) {
  if (count <= 0 || total_blocks <= 0) return 0;
  if ((long long)total_blocks * 1024 >= 0x7fffffffLL) return MDTF_EUNSUPPORTED;   // 32-bit vector indices
  hipLaunchKernelGGL(copy2d_multi, dim3(total_blocks), dim3(256), 0, st, (const CDesc*)desc, count);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_transpose_multi(const void* desc, int count, int total_tiles, hipStream_t st) {
  if (count <= 0 || total_tiles <= 0) return 0;
  hipLaunchKernelGGL(transpose16_multi, dim3(total_tiles), dim3(256), 0, st, (const TDesc*)desc, count);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_transpose_brs(const void* in, void* out, int B, int R, int S, int elem_bytes, hipStream_t st) {
  dim3 grid(ceil_div(S, 64), ceil_div(R, 64), B);
  if (elem_bytes == 2 && R % 8 == 0 && S % 8 == 0)
    hipLaunchKernelGGL(transpose16_kernel, grid, dim3(256), 0, st, (const uint16_t*)in, (uint16_t*)out, R, S);
  else if (elem_bytes == 2)
    hipLaunchKernelGGL(transpose_kernel<uint16_t>, grid, dim3(kT), 0, st, (const uint16_t*)in, (uint16_t*)out, R, S);
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(transpose_kernel<uint32_t>, grid, dim3(kT), 0, st, (const uint32_t*)in, (uint32_t*)out, R, S);
  else
    return MDTF_EINVAL;
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_lrn_fwd(const void* x, void* y, float* dsave, long long P, int C, int r, float bias, float alpha,
                             float beta, hipStream_t st) {
  hipLaunchKernelGGL(lrn_fwd, dim3(grid_cap(P * C)), dim3(kT), 0, st, (const bf16_t*)x, (bf16_t*)y, dsave, P, C, r,
                     bias, alpha, beta);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_lrn_bwd(const void* dy, const void* x, const void* y, const float* dsave, void* dx, long long P,
                             int C, int r, float alpha, float beta, hipStream_t st) {
  hipLaunchKernelGGL(lrn_bwd, dim3(grid_cap(P * C)), dim3(kT), 0, st, (const bf16_t*)dy, (const bf16_t*)x,
                     (const bf16_t*)y, dsave, (bf16_t*)dx, P, C, r, alpha, beta);
  MDTF_LAUNCH_CHECK();
  return 0;
}
