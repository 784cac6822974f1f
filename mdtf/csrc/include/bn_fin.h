// In-kernel BatchNorm finalize: the kernel that emits a BN's statistics partials finalizes them itself.
//
// The statistics of a training BN come from the epilogue of the conv that produces its input (forward:
// Σy, Σy²) or completes its output gradient (backward: Σg·mask, Σg·mask·x), as fp32 atomics into [slots][C]
// partial rows.  They used to be turned into coefficients by a separate one-block-per-32-channels launch
// (bn_finalize_fwd / bn_finalize_bwd in bn.hip): ~106 launches of ~5 us in a ResNet-50 step.  Here every
// workgroup of the producing kernel takes a ticket after its atomics; the last arriver sums the rows (fixed
// order), re-zeroes them for the next producer and writes the coefficients.  Same publish protocol as the
// split-K tickets of gemm_wg.hip: vmcnt drain, workgroup barrier, agent-scope release, relaxed agent-scope
// ticket; the last arriver resets the ticket and acquires.
//
// The host arms one launch with mdtf_bn_fin_arm (bn.hip) right before the conv export that launches the
// producer; the export takes the armed spec (bn_fin_take) and attaches it to its LAST stats-emitting launch.
#pragma once
#include "mdtf_common.h"

namespace mdtf {

struct BnFin {
  int* ticket;             // null: off.  0 on entry; the last arriver resets it
  int nwg;                 // arrivals to expect (workgroups of the launch; set by the launcher)
  int bwd;                 // 0: Σx, Σx² -> mean, invstd, scale, shift (+ moving averages)
                           // 1: Σg, Σg·x -> k1, k2, k3 (dx = k1 g + k2 x + k3), dγ, dβ
  int C, slots;            // channels, partial rows (set by the launcher from its own statistics arguments)
  float* p0;               // [slots][C] partial rows (re-zeroed here)
  float* p1;
  long long count;         // elements per channel
  const float* gamma;      // null: 1
  const float* beta;       // fwd, null: 0
  float* mmean;            // fwd moving averages (null: no update)
  float* mvar;
  float decay, eps;
  const float* mean;       // bwd: the forward's batch statistics
  const float* invstd;
  float* out;              // fwd [4][C]: mean, invstd, scale, shift;  bwd [5][C]: k1, k2, k3, dγ, dβ
};

// The spec armed by the last mdtf_bn_fin_arm call of this host thread (ticket null: none); clears it.
BnFin bn_fin_take();

// Every thread of every workgroup of the producing launch calls this once, after the workgroup's partial
// atomics were issued.  NT: threads per workgroup.  lds: >= 16 * NT bytes of LDS the caller no longer uses.
template <int NT>
__device__ __forceinline__ void bn_fin_arrive(const BnFin& fin_arg, char* lds) {
  // volatile copy out of the kernel arguments, made wave-uniform (SGPRs): read here, at the end of the kernel,
  // instead of being loaded with the other arguments at entry and kept live through the main loop
  static_assert(sizeof(BnFin) % 4 == 0, "BnFin copies as 4-byte words");
  BnFin f;
  {
    const volatile unsigned* s = reinterpret_cast<const volatile unsigned*>(&fin_arg);
    unsigned* d = reinterpret_cast<unsigned*>(&f);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(BnFin) / 4); ++i) d[i] = __builtin_amdgcn_readfirstlane(s[i]);
  }
  if (f.ticket == nullptr) return;
  const int tid = threadIdx.x;
  int* flag = reinterpret_cast<int*>(lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this thread's atomics are done
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int prev = __hip_atomic_fetch_add(f.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == f.nwg - 1;
    if (last) {
      __hip_atomic_store(f.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  const int last = *flag;
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();                                     // every thread has read the flag: LDS reusable
  // the rows as float4 column vectors: VT vectors per pass, G row groups (thread: one vector, every G-th row;
  // the host sizes slots x C <= 4096 floats, so a pass is <= 2 trips of 4 loads per thread)
  float4* red = reinterpret_cast<float4*>(lds);        // [NT] (8 KiB at NT = 512)
  const int C = f.C, S = f.slots, V = C / 4;
  const int VT = V < NT ? V : NT;
  const int G = NT / VT;
  const int gi = tid / VT, vl = tid - gi * VT;
  const float4* P0 = reinterpret_cast<const float4*>(f.p0);
  const float4* P1 = reinterpret_cast<const float4*>(f.p1);
  for (int v0 = 0; v0 < V; v0 += VT) {
    const int v = v0 + vl;
    const bool act = gi < G && v < V;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (act) {
      for (int r = gi; r < S; r += 2 * G) {            // 2 rows (4 loads) in flight per trip
        const bool ok = r + G < S;
        const float4 a0 = P0[r * V + v], b0 = P1[r * V + v];
        const float4 a1 = ok ? P0[(r + G) * V + v] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 b1 = ok ? P1[(r + G) * V + v] : make_float4(0.f, 0.f, 0.f, 0.f);
        a.x += a0.x + a1.x; a.y += a0.y + a1.y; a.z += a0.z + a1.z; a.w += a0.w + a1.w;
        b.x += b0.x + b1.x; b.y += b0.y + b1.y; b.z += b0.z + b1.z; b.w += b0.w + b1.w;
      }
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = gi; r < S; r += G) {                // re-zero for the next producer
        reinterpret_cast<float4*>(f.p0)[r * V + v] = z;
        reinterpret_cast<float4*>(f.p1)[r * V + v] = z;
      }
    }
    // Σ over the G row groups: one LDS pass for the sums, one for the squares / cross terms
    float4 sa = a, sb = b;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      red[tid] = h ? b : a;
      __syncthreads();
      if (gi == 0 && v < V) {
        float4 t = red[vl];
        for (int g2 = 1; g2 < G; ++g2) {
          const float4 e = red[g2 * VT + vl];
          t.x += e.x; t.y += e.y; t.z += e.z; t.w += e.w;
        }
        if (h) sb = t; else sa = t;
      }
      __syncthreads();
    }
    if (gi == 0 && v < V) {
      const float sv[4] = {sa.x, sa.y, sa.z, sa.w}, qv[4] = {sb.x, sb.y, sb.z, sb.w};
      const double invn = 1.0 / (double)f.count;
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * v + k;
        const float gm = f.gamma ? f.gamma[c] : 1.f;
        if (!f.bwd) {
          const double mean = (double)sv[k] * invn;
          double var = (double)qv[k] * invn - mean * mean;
          if (var < 0) var = 0;
          const float inv = rsqrtf((float)var + f.eps);
          const float bt = f.beta ? f.beta[c] : 0.f;
          f.out[c] = (float)mean;
          f.out[C + c] = inv;
          f.out[2 * C + c] = gm * inv;
          f.out[3 * C + c] = bt - (float)mean * gm * inv;
          if (f.mmean) {
            const float unbiased = f.count > 1 ? (float)(var * (double)f.count / (double)(f.count - 1)) : (float)var;
            f.mmean[c] = f.decay * f.mmean[c] + (1.f - f.decay) * (float)mean;
            f.mvar[c] = f.decay * f.mvar[c] + (1.f - f.decay) * unbiased;
          }
        } else {
          const float mu = f.mean[c], inv = f.invstd[c];
          const float db = sv[k];
          const float dg = (qv[k] - mu * sv[k]) * inv;
          const float a1 = gm * inv, invM = (float)invn;
          f.out[c] = a1;                                // dx = a (dz - dβ/M - x̂ dγ/M), x̂ = (x - μ) invstd
          f.out[C + c] = -a1 * inv * dg * invM;
          f.out[2 * C + c] = a1 * (-db * invM + mu * inv * dg * invM);
          f.out[3 * C + c] = dg;
          f.out[4 * C + c] = db;
        }
      }
    }
  }
}

}  // namespace mdtf
