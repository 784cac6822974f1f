// Fused optimizer updates over flat fp32 parameter buffers (one launch per group).
//
// Each thread updates 4 consecutive parameters with 16-byte loads of master,
// grad and state, applies the data-parallel gradient scale and L2 weight decay,
// writes master/state back and — when a bf16 shadow buffer is given — the
// bf16 compute copy of the weights (no separate cast kernels before the next
// forward).  Memory-bound: 3-5 streams of fp32 at HBM rate; grid-stride with
// ~8 blocks/CU.  ``dyn`` (nullable) points at device-resident hyper-parameters
// {lr, lr_t, grad_scale} that override the scalar arguments: a hipGraph-captured
// training step bakes kernel arguments, so per-step values (LR schedule, Adam
// bias correction, backup-worker scale) are refreshed in that buffer instead.
// Reference ops: tf.train.AdamOptimizer / MomentumOptimizer
// apply on the PS (distribute_train.py:151-158), l2_loss*wd (distribute_tools.py:64).
#include "mdtf_common.h"

using namespace mdtf;

namespace {

constexpr int kThreads = 256;

inline int grid_for(long long n4) {
  long long b = ceil_div(n4, kThreads);
  return static_cast<int>(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

__device__ __forceinline__ void load_dyn(const float* dyn, float& lr, float& lr_t, float& gs) {
  if (dyn) {
    lr = dyn[0];
    lr_t = dyn[1];
    gs = dyn[2];
  }
}

__device__ __forceinline__ void store_shadow4(bf16_t* s, long long i, const float4& w) {
  uint32_t lo = static_cast<uint32_t>(f2bf(w.x)) | (static_cast<uint32_t>(f2bf(w.y)) << 16);
  uint32_t hi = static_cast<uint32_t>(f2bf(w.z)) | (static_cast<uint32_t>(f2bf(w.w)) << 16);
  *reinterpret_cast<uint2*>(s + i) = make_uint2(lo, hi);
}

__global__ void __launch_bounds__(kThreads) sgd_kernel(long long n, float* __restrict__ w, const float* __restrict__ g,
                                                      bf16_t* __restrict__ shadow, float lr, float gs, float wd,
                                                      const float* __restrict__ dyn) {
  float lr_t = lr;
  load_dyn(dyn, lr, lr_t, gs);
  long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    wv.x -= lr * (gv.x * gs + wd * wv.x);
    wv.y -= lr * (gv.y * gs + wd * wv.y);
    wv.z -= lr * (gv.z * gs + wd * wv.z);
    wv.w -= lr * (gv.w * gs + wd * wv.w);
    reinterpret_cast<float4*>(w)[i] = wv;
    if (shadow) store_shadow4(shadow, i * 4, wv);
  }
}

// optimizer state streams (master, gradient, moments: read and written once per step) with nontemporal loads /
// stores; the bf16 shadow the next forward reads stays cached.  MDTF_NT_OPT=0: cached forms.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ldf4(const float* p, long long i) {
  if constexpr (NT) return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p) + i));
  return reinterpret_cast<const float4*>(p)[i];
}
template <bool NT>
__device__ __forceinline__ void stf4(float* p, long long i, const float4& v) {
  if constexpr (NT)
    __builtin_nontemporal_store(__builtin_bit_cast(f32x4_t, v), reinterpret_cast<f32x4_t*>(p) + i);
  else
    reinterpret_cast<float4*>(p)[i] = v;
}
inline bool nt_opt() {
  static const bool on = [] {
    const char* e = getenv("MDTF_NT_OPT");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <bool NT>
__global__ void __launch_bounds__(kThreads) momentum_kernel(long long n, float* __restrict__ w,
                                                           const float* __restrict__ g, float* __restrict__ acc,
                                                           bf16_t* __restrict__ shadow, float lr, float mom, float gs,
                                                           float wd, int nesterov, const float* __restrict__ dyn) {
  float lr_t = lr;
  load_dyn(dyn, lr, lr_t, gs);
  long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 wv = ldf4<NT>(w, i);
    float4 gv = ldf4<NT>(g, i);
    float4 av = ldf4<NT>(acc, i);
    float gx = gv.x * gs + wd * wv.x, gy = gv.y * gs + wd * wv.y;
    float gz = gv.z * gs + wd * wv.z, gw = gv.w * gs + wd * wv.w;
    av.x = mom * av.x + gx;
    av.y = mom * av.y + gy;
    av.z = mom * av.z + gz;
    av.w = mom * av.w + gw;
    if (nesterov) {
      wv.x -= lr * (gx + mom * av.x);
      wv.y -= lr * (gy + mom * av.y);
      wv.z -= lr * (gz + mom * av.z);
      wv.w -= lr * (gw + mom * av.w);
    } else {
      wv.x -= lr * av.x;
      wv.y -= lr * av.y;
      wv.z -= lr * av.z;
      wv.w -= lr * av.w;
    }
    stf4<NT>(acc, i, av);
    stf4<NT>(w, i, wv);
    if (shadow) store_shadow4(shadow, i * 4, wv);
  }
}

__device__ __forceinline__ float adam1(float& w, float g, float& m, float& v, float lr, float lr_t, float b1, float b2,
                                       float eps, float gs, float wd, int decoupled) {
  g *= gs;
  if (!decoupled) g += wd * w;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  float upd = lr_t * m / (sqrtf(v) + eps);
  if (decoupled) upd += lr * wd * w;
  w -= upd;
  return w;
}

constexpr int kAdamVpt = 2;

template <bool NT, bool CHUNK = true>
__global__ void __launch_bounds__(kThreads) adam_kernel(long long n, float* __restrict__ w, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       bf16_t* __restrict__ shadow, float lr, float lr_t, float b1,
                                                       float b2, float eps, float gs, float wd, int decoupled,
                                                       const float* __restrict__ dyn) {
  load_dyn(dyn, lr, lr_t, gs);
  // one contiguous chunk of kAdamVpt * kThreads float4s per block, every load of the chunk issued before the math
  // (a grid-stride sweep keeps one float4 per stream in flight: 605 us for BERT-base's 110 M parameters)
  const long long n4 = n >> 2;
  if constexpr (!CHUNK) {          // MDTF_ADAM_CHUNK=0: the grid-stride sweep (A/B)
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
      float4 wq = ldf4<NT>(w, i), gq = ldf4<NT>(g, i), mq = ldf4<NT>(m, i), vq = ldf4<NT>(v, i);
      adam1(wq.x, gq.x, mq.x, vq.x, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
      adam1(wq.y, gq.y, mq.y, vq.y, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
      adam1(wq.z, gq.z, mq.z, vq.z, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
      adam1(wq.w, gq.w, mq.w, vq.w, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
      stf4<NT>(m, i, mq);
      stf4<NT>(v, i, vq);
      stf4<NT>(w, i, wq);
      if (shadow) store_shadow4(shadow, i * 4, wq);
    }
    return;
  }
  const long long base = (long long)blockIdx.x * (kThreads * kAdamVpt) + threadIdx.x;
  float4 wv[kAdamVpt], gv[kAdamVpt], mv[kAdamVpt], vv[kAdamVpt];
#pragma unroll
  for (int u = 0; u < kAdamVpt; ++u) {
    const long long i = base + u * kThreads;
    if (i < n4) {
      wv[u] = ldf4<NT>(w, i);
      gv[u] = ldf4<NT>(g, i);
      mv[u] = ldf4<NT>(m, i);
      vv[u] = ldf4<NT>(v, i);
    }
  }
#pragma unroll
  for (int u = 0; u < kAdamVpt; ++u) {
    const long long i = base + u * kThreads;
    if (i >= n4) break;
    adam1(wv[u].x, gv[u].x, mv[u].x, vv[u].x, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
    adam1(wv[u].y, gv[u].y, mv[u].y, vv[u].y, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
    adam1(wv[u].z, gv[u].z, mv[u].z, vv[u].z, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
    adam1(wv[u].w, gv[u].w, mv[u].w, vv[u].w, lr, lr_t, b1, b2, eps, gs, wd, decoupled);
    stf4<NT>(m, i, mv[u]);
    stf4<NT>(v, i, vv[u]);
    stf4<NT>(w, i, wv[u]);
    if (shadow) store_shadow4(shadow, i * 4, wv[u]);
  }
}


// ---- several sequential updates in one pass (async PS: every gradient that arrived since the last apply).
// Update i uses gradient g[i] (bf16 wire or fp32) and lr[i] / lr_t[i]; the result equals k launches of the
// single-update kernel in order, but master / state / shadow are read and written once.
constexpr int kMaxMulti = 8;
struct MultiGrads {
  const void* g[kMaxMulti];
  float lr[kMaxMulti];
  float lr_t[kMaxMulti];
};

__device__ __forceinline__ float4 load_g4(const void* g, long long i, bool bf) {
  if (bf) {
    const uint2 v = reinterpret_cast<const uint2*>(g)[i];
    return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                       __uint_as_float(v.y & 0xffff0000u));
  }
  return reinterpret_cast<const float4*>(g)[i];
}

// kind 0 sgd, 1 momentum (flag = nesterov), 2 adam (flag = decoupled weight decay)
__global__ void __launch_bounds__(kThreads) apply_multi_kernel(int kind, long long n, float* __restrict__ w,
                                                              float* __restrict__ s1, float* __restrict__ s2,
                                                              bf16_t* __restrict__ shadow, MultiGrads mg, int k,
                                                              int gbf16, float mom, float b1, float b2, float eps,
                                                              float gs, float wd, int flag) {
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 av = kind >= 1 ? reinterpret_cast<float4*>(s1)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 vv = kind == 2 ? reinterpret_cast<float4*>(s2)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float* wp = &wv.x;
    float* ap = &av.x;
    float* vp = &vv.x;
    for (int u = 0; u < k; ++u) {
      const float4 gv = load_g4(mg.g[u], i, gbf16 != 0);
      const float* gp = &gv.x;
      const float lr = mg.lr[u], lr_t = mg.lr_t[u];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (kind == 2) {
          adam1(wp[e], gp[e], ap[e], vp[e], lr, lr_t, b1, b2, eps, gs, wd, flag);
        } else {
          const float g = gp[e] * gs + wd * wp[e];
          if (kind == 1) {
            ap[e] = mom * ap[e] + g;
            wp[e] -= lr * (flag ? g + mom * ap[e] : ap[e]);
          } else {
            wp[e] -= lr * g;
          }
        }
      }
    }
    if (kind >= 1) reinterpret_cast<float4*>(s1)[i] = av;
    if (kind == 2) reinterpret_cast<float4*>(s2)[i] = vv;
    reinterpret_cast<float4*>(w)[i] = wv;
    if (shadow) store_shadow4(shadow, i * 4, wv);
  }
}

}  // namespace

// k <= 8 sequential updates of one flat group; grads: k device pointers (bf16 if gbf16 else fp32), lrs / lr_ts:
// k host floats each
MDTF_EXPORT int mdtf_fused_apply_multi(int kind, long long n, void* w, void* s1, void* s2, void* shadow,
                                       const void* const* grads, const float* lrs, const float* lr_ts, int k, int gbf16,
                                       float mom, float b1, float b2, float eps, float gs, float wd, int flag,
                                       hipStream_t st) {
  if (n % 4 || k < 1 || k > kMaxMulti || kind < 0 || kind > 2) return MDTF_EINVAL;
  MultiGrads mg{};
  for (int u = 0; u < k; ++u) {
    mg.g[u] = grads[u];
    mg.lr[u] = lrs[u];
    mg.lr_t[u] = lr_ts[u];
  }
  hipLaunchKernelGGL(apply_multi_kernel, dim3(grid_for(n / 4)), dim3(kThreads), 0, st, kind, n, (float*)w, (float*)s1,
                     (float*)s2, (bf16_t*)shadow, mg, k, gbf16, mom, b1, b2, eps, gs, wd, flag);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// n must be a multiple of 4 (flat groups are padded to 64 elements).
MDTF_EXPORT int mdtf_fused_sgd(long long n, void* w, const void* g, void* shadow, float lr, float gs, float wd,
                               const void* dyn, hipStream_t st) {
  if (n % 4) return MDTF_EINVAL;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n / 4)), dim3(kThreads), 0, st, n, (float*)w, (const float*)g,
                     (bf16_t*)shadow, lr, gs, wd, (const float*)dyn);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_fused_momentum(long long n, void* w, const void* g, void* acc, void* shadow, float lr, float mom,
                                    float gs, float wd, int nesterov, const void* dyn, hipStream_t st) {
  if (n % 4) return MDTF_EINVAL;
  hipLaunchKernelGGL((nt_opt() ? momentum_kernel<true> : momentum_kernel<false>), dim3(grid_for(n / 4)), dim3(kThreads), 0, st, n, (float*)w, (const float*)g,
                     (float*)acc, (bf16_t*)shadow, lr, mom, gs, wd, nesterov, (const float*)dyn);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT int mdtf_fused_adam(long long n, void* w, const void* g, void* m, void* v, void* shadow, float lr,
                                float lr_t, float b1, float b2, float eps, float gs, float wd, int decoupled,
                                const void* dyn, hipStream_t st) {
  if (n % 4) return MDTF_EINVAL;
  static const bool chunk = [] {
    const char* e = getenv("MDTF_ADAM_CHUNK");
    return !(e && e[0] == '0');
  }();
  const long long nb = ceil_div(n / 4, (long long)kThreads * kAdamVpt);
  auto k = chunk ? (nt_opt() ? adam_kernel<true, true> : adam_kernel<false, true>)
                 : (nt_opt() ? adam_kernel<true, false> : adam_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(chunk ? (unsigned)(nb > 0 ? nb : 1) : (unsigned)grid_for(n / 4)), dim3(kThreads), 0, st, n,
                     (float*)w, (const float*)g,
                     (float*)m, (float*)v, (bf16_t*)shadow, lr, lr_t, b1, b2, eps, gs, wd, decoupled,
                     (const float*)dyn);
  MDTF_LAUNCH_CHECK();
  return 0;
}

MDTF_EXPORT const char* mdtf_error_string(int rc) {
  if (rc == MDTF_EINVAL) return "invalid argument";
  if (rc == MDTF_EUNSUPPORTED) return "unsupported configuration";
  return hipGetErrorString(static_cast<hipError_t>(rc));
}

MDTF_EXPORT int mdtf_version() { return 1; }
