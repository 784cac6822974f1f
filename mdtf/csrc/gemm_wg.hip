// Weight-gradient GEMM (gfx950 / CDNA4): C[M][N] (fp32) += sum_k A[k][m] B[k][n], both operands k-major.
//
// This is the autodiff weight gradient of every dense layer, dW = x^T dy with x [tokens][in] and dy
// [tokens][out] (the reference's tf.matmul in FC_layer, distribute_tools.py:204-206, differentiated by
// distribute_tower.py:27's compute_gradients), and of the stride-1 1x1 convolutions.
// The reduction runs over the tokens (BERT-base: K = 8192) while the output is small (768 x 768 .. 3072),
// so a chip-filling grid needs split-K.  The ping-pong core (gemm_pp.hip) measured why the usual ways lose
// (profiles/gemm_core_vs_hipblaslt_r3a.md): 256x256 tiles leave 27-36 tiles for 256 CUs, and fp32 atomics
// from many splits of a tile serialise.  Here:
//   * tiles of BM x 128 (BM = 128: 4 waves, two workgroups per CU; BM = 256: 8 waves, one), each wave a 64x64
//     block of 16x16x32 bf16 MFMAs (C^T = B^T A^T so a lane holds 4 consecutive output columns);
//   * both operands staged global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into [64 k][cols] images
//     read with ds_read_b64_tr_b16; the 32-B block XOR swizzle (by k row) is applied to the DMA's per-lane
//     source address, the image stays lane-linear;
//   * STAGES-deep ring, one barrier per 64-deep K-tile: wait for tile t (counted vmcnt, never 0 inside the
//     loop), barrier, issue tile t + STAGES - 1 into the slot tile t - 1 used, MFMAs on tile t;
//   * split-K without atomics on C: each split stores its partial tile into a slab with coalesced 16-B stores,
//     publishes it (vmcnt drain, workgroup barrier, agent-scope release, relaxed agent-scope ticket), and the
//     last workgroup of the tile (acquire) sums every slab in split order -- deterministic whatever the arrival
//     order -- and adds the sum into C once.  No workgroup ever waits for another, so the grid cannot deadlock;
//   * the bias gradient (column sums of B) comes from an all-ones MFMA over the B fragments the first row of
//     waves already holds (tile row 0 only);
//   * grid = tiles x splits, XCD-remapped (bijective) so the workgroups sharing an operand panel and K range
//     share an L2.
#include "mdtf_common.h"

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct WgArgs {
  const bf16_t* A;
  const bf16_t* B;
  long long lda, ldb;        // row (k) strides of the stored operands, elements
  int M, N, K;               // C is M x N, K a multiple of 64
  int tiles_m, tiles_n, splits, kt_split;
  int gm, gn;                // L2 groups: the workgroups one XCD runs cover a gm x gn block of tiles
  int bytes_a, bytes_b;      // buffer ranges (< 2 GiB)
  int nseg, seg_cols;        // C / bias-gradient column segments (each tile inside one segment)
  float* cf[4];
  long long ldc;
  float* db[4];              // column sums of B added here (null: none)
  float* slab;               // splits > 1: [tiles][splits][BM * 128] partial tiles (stream-K: [tiles][maxp][..])
  int* cnt;                  // splits > 1: per-tile arrival tickets, 0 on entry, reset by the last arriver
  // stream-K (sk_q > 0): worker w of the grid runs K-tile iterations [w sk_q, (w + 1) sk_q) of the tile-major
  // sequence (tile t owns [t KT, (t + 1) KT)), so every worker does the same work whatever tiles x splits is;
  // the pieces of a tile (at most maxp) are summed by its last arriver as the splits are
  int sk_q, kt_total, maxp;
  int wt;                    // slab publish form: 1 write-through (sc1) stores / loads, 0 plain + agent fences
  int store_mask;            // bit s: segment s's C is overwritten (first writer of an unzeroed slot), else +=
};

__device__ __forceinline__ void dma16(i32x4_t rsrc, unsigned lds_addr, unsigned voff, int soff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc), "s"(soff), "{m0}"(m0)
               : "memory");
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// 32-B block swizzle of a [64 k][cols] image whose pitch is a multiple of 256 B: the 8 k rows one 32-lane half
// of a transposed read touches ({0-3} + 8 fq and +4) land in 8 distinct 32-B bank slots.
__device__ __forceinline__ int trg(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

template <int BM, int STAGES, bool PIPE, bool SK = false>
__global__ void __launch_bounds__(2 * BM) gemm_wg_kernel(WgArgs a) {
  constexpr int BN = 128;
  constexpr int NT = 2 * BM, NW = NT / 64;          // waves: (BM / 64) rows x 2 columns of 64x64 blocks
  constexpr int PA = 2 * BM, PB = 2 * BN;           // image pitches (bytes)
  constexpr int BYTES_A = 64 * PA, BYTES_B = 64 * PB;
  constexpr int SLOT = BYTES_A + BYTES_B;
  constexpr int IA = BYTES_A / 1024 / NW, IB = BYTES_B / 1024 / NW;   // DMA instructions per wave per tile
  constexpr int RJA = NW * 1024 / PA, RJB = NW * 1024 / PB;           // k rows between a wave's instructions
  static_assert(RJA % 16 == 0 && RJB % 16 == 0 && IA >= 1 && IB >= 1, "geometry");
  constexpr int PER_TILE = IA + IB;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int ntiles = a.tiles_m * a.tiles_n;
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<unsigned long long>(
      (__attribute__((address_space(3))) char*)smem));
  const i32x4_t ra = buffer_rsrc(a.A, a.bytes_a);
  const i32x4_t rb = buffer_rsrc(a.B, a.bytes_b);

  // one piece: K-tiles [kt0, kt0 + T) of tile `tile`, piece `pidx` of the tile's `np` (np == 1: the whole tile)
  auto run_piece = [&](int tile, int kt0, int T, int pidx, int np) {
  // tile order: gm x gn blocks (row-major over the block grid, edge blocks partial), so the contiguous range of
  // logical ids one XCD gets shares few operand panels in its L2
  int tm, tn;
  {
    const int gi = tile / (a.gm * a.tiles_n);
    const int r2 = tile - gi * a.gm * a.tiles_n;
    const int hm = min(a.gm, a.tiles_m - gi * a.gm);
    const int gj = r2 / (hm * a.gn);
    const int r3 = r2 - gj * hm * a.gn;
    const int wn = min(a.gn, a.tiles_n - gj * a.gn);
    tm = gi * a.gm + r3 / wn;
    tn = gj * a.gn + r3 - (r3 / wn) * wn;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int seg = n0 / a.seg_cols;

  // per-lane DMA source offset of this wave's first instruction into an image of pitch P; the wave's later
  // instructions are RJ k rows further (a multiple of 16: same swizzle), a wave-uniform soffset
  auto src_off = [&](int P, long long ld, int c0) -> unsigned {
    const int off = wave * 1024 + lane * 16;
    const int row = off / P, cb = off - row * P;
    const int col = c0 + ((((cb >> 5) ^ trg(row))) << 4) + ((cb >> 4) & 1) * 8;
    return static_cast<unsigned>((((long long)kt0 * 64 + row) * ld + col) * 2);
  };
  const unsigned vA = src_off(PA, a.lda, m0), vB = src_off(PB, a.ldb, n0);
  const int stepA = (int)(64 * a.lda * 2), stepB = (int)(64 * a.ldb * 2);
  const int jA = (int)(RJA * a.lda * 2), jB = (int)(RJB * a.ldb * 2);

  auto issue_to = [&](int t, int sl) {
    const unsigned slot = lds0 + sl * SLOT;
#pragma unroll
    for (int j = 0; j < IA; ++j) dma16(ra, slot + (j * NW + wave) * 1024, vA, t * stepA + j * jA);
#pragma unroll
    for (int j = 0; j < IB; ++j) dma16(rb, slot + BYTES_A + (j * NW + wave) * 1024, vB, t * stepB + j * jB);
  };
  auto issue = [&](int t) { issue_to(t, t % STAGES); };

  // fragment reads: lane (fr, fq) gets X[k = 32 s + 8 fq + 0..7][col = c0 + fr] (the 16x16x32 operand map)
  const int fq = lane >> 4;
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  auto frag = [&](const char* img, int P, int c0, int s) -> bf16x8_t {
    const int row = 32 * s + 8 * fq + q4;
    const char* p1 = img + row * P + (((c0 >> 4) ^ trg(row)) << 5) + p4 * 8;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p1);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p1 + 4 * P));
    const short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, f);
  };

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  float4v accb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) accb[j] = float4v{0.f, 0.f, 0.f, 0.f};
  const bool dsum = a.db[0] != nullptr && tm == 0 && wr == 0;
  const short8 ones8 = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, ones8);

  auto load_frags = [&](const char* slotp, int s, bf16x8_t (&fa)[4], bf16x8_t (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(slotp, PA, wr * 64 + 16 * i, s);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag(slotp + BYTES_A, PB, wc * 64 + 16 * j, s);
  };
  auto mfmas = [&](const bf16x8_t (&fa)[4], const bf16x8_t (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    if (dsum) {
#pragma unroll
      for (int j = 0; j < 4; ++j) accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], ones, accb[j], 0, 0, 0);
    }
  };

#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < T) issue(p);
  if constexpr (!PIPE) {
    // unrolled by the ring depth: every slot address is a compile-time offset
    for (int t0 = 0; t0 < T; t0 += STAGES) {
#pragma unroll
      for (int u = 0; u < STAGES; ++u) {
        const int t = t0 + u;
        if (t < T) {
          // tile t landed: the tiles issued after it (up to STAGES - 2) may stay in flight
          if (t + STAGES - 2 < T) wait_vmcnt<(STAGES - 2) * PER_TILE>();
          else wait_vmcnt<0>();
          barrier();
          // every wave has finished reading tile t - 1: its slot takes tile t + STAGES - 1
          if (t + STAGES - 1 < T) issue_to(t + STAGES - 1, (u + STAGES - 1) % STAGES);
          const char* slotp = smem + u * SLOT;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8_t fa[4], fb[4];
            load_frags(slotp, s, fa, fb);
            mfmas(fa, fb);
          }
        }
      }
    }
  } else {
    // mid-tile barrier: the fragment reads of the next step always overlap MFMAs of the current one.
    //   iteration t:  read s1(t) | MFMA s0(t) | wait tile t+1, barrier, DMA tile t+S-1 into tile t-1's slot,
    //                 read s0(t+1) | MFMA s1(t)
    // Every read of tile t-1 retired before iteration t (its MFMAs ran in iteration t-1), so the DMA after the
    // barrier cannot overwrite live data; tile t+1 is read only after every wave's vmcnt wait + the barrier.
    static_assert(STAGES >= 3, "PIPE needs the tile after next in flight");
    if (STAGES - 2 < T) wait_vmcnt<(STAGES - 2) * PER_TILE>();
    else wait_vmcnt<0>();
    barrier();
    bf16x8_t a0[4], b0[4], a1[4], b1[4];
    load_frags(smem, 0, a0, b0);
    for (int t = 0; t < T; ++t) {
      const char* slotp = smem + (t % STAGES) * SLOT;
      load_frags(slotp, 1, a1, b1);
      mfmas(a0, b0);
      if (t + 1 < T) {
        if (t + STAGES - 2 < T) wait_vmcnt<(STAGES - 3) * PER_TILE>();
        else wait_vmcnt<0>();
        barrier();
        if (t + STAGES - 1 < T) issue(t + STAGES - 1);
        load_frags(smem + ((t + 1) % STAGES) * SLOT, 0, a0, b0);
      }
      mfmas(a1, b1);
    }
  }

  // ---- epilogue: lane holds C[m0 + 64 wr + 16 i + fr][n0 + 64 wc + 16 j + 4 fq + 0..3]
  const int fr = lane & 15;
  const int rbase = m0 + wr * 64 + fr;
  const int cbase = n0 + wc * 64 + 4 * fq;
  float* cf = a.cf[seg];
  const int cseg = cbase - seg * a.seg_cols;
  if (dsum && fr == 0) {             // bias gradient: one partial column sum per split (atomics on N floats)
    float* db = a.db[seg] + cseg;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) unsafeAtomicAdd(db + 16 * j + e, accb[j][e]);
  }
  if (np > 1) {
    // this tile's slabs: [maxp][BM * BN] fp32, addressed through one buffer resource (byte offsets < 2 MiB)
    float* tslab = a.slab + (long long)tile * a.maxp * (BM * BN);
    const __amdgpu_buffer_rsrc_t srs =
        __builtin_amdgcn_make_buffer_rsrc(tslab, (short)0, a.maxp * (BM * BN) * 4, 0x00020000);
    // Publish form (a.wt): write-through.  Every slab byte is stored sc1 (16-B buffer stores, aux 16), every storing
    // wave drains its stores, the workgroup barrier orders them before the one ticket add, and the last arriver
    // reads every slab with sc1 buffer loads (L1 bypassed) -- no L2 write-back (release) or L1 invalidate
    // (acquire) fence (MI355X_MICROARCH.md, publish-large: 3.0 vs 8.2 us for 64 KiB per workgroup).  a.wt = 0:
    // plain stores + agent release / acquire fences.
    const int sl0 = pidx * (BM * BN / 4);
    if (a.wt) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, acc[i][j]), srs,
                                                 (sl0 + (i * 4 + j) * NT + tid) * 16, 0, 16);
    } else {
      float4v* sl = reinterpret_cast<float4v*>(tslab) + sl0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sl[(i * 4 + j) * NT + tid] = acc[i][j];
    }
    // publish: the slab stores complete, then one ticket for the workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      if (!a.wt) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const int prev = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == np - 1;
      if (last) {
        __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!a.wt) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // the last arriver: sum the slabs in split order (deterministic), own partial from registers
    float4v sum[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < np; ++s) {           // wave-uniform branch: all 16 loads of a slab issue together
      if (s == pidx) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) sum[i][j] += acc[i][j];
      } else {
        const int so = s * (BM * BN / 4) + tid;
        float4v p[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int off = (so + (i * 4 + j) * NT) * 16;
            p[i][j] = __builtin_bit_cast(float4v, a.wt ? __builtin_amdgcn_raw_buffer_load_b128(srs, off, 0, 16)
                                                       : __builtin_amdgcn_raw_buffer_load_b128(srs, off, 0, 0));
          }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) sum[i][j] += p[i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = sum[i][j];
  }
  if ((a.store_mask >> seg) & 1) {      // the step's only write into this slot: store, nothing to read
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* crow = cf + (long long)(rbase + 16 * i) * a.ldc + cseg;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<float4*>(crow + 16 * j) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* crow = cf + (long long)(rbase + 16 * i) * a.ldc + cseg;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float4* dst = reinterpret_cast<float4*>(crow + 16 * j);
      float4 o = *dst;
      o.x += acc[i][j][0];
      o.y += acc[i][j][1];
      o.z += acc[i][j][2];
      o.w += acc[i][j][3];
      *dst = o;
    }
  }
  };

  if constexpr (!SK) {
    const int lid = xcd_remap(blockIdx.x, ntiles * a.splits);
    const int split = lid / ntiles, tile = lid - split * ntiles;
    const int kt0 = split * a.kt_split;
    run_piece(tile, kt0, min(a.kt_split, a.K / 64 - kt0), split, a.splits);
  } else {
    // stream-K: this worker's iteration range, cut at tile boundaries; pieces of one tile are consecutive workers
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int KT = a.kt_total;
    const long long total = (long long)ntiles * KT;
    long long it = (long long)w * a.sk_q;
    const long long end = min(total, it + a.sk_q);
    bool first = true;
    while (it < end) {
      const int tile = (int)(it / KT), k0 = (int)(it - (long long)tile * KT);
      const int T = (int)min((long long)KT - k0, end - it);
      const int wf = (int)(((long long)tile * KT) / a.sk_q), wl = (int)(((long long)tile * KT + KT - 1) / a.sk_q);
      if (!first) __syncthreads();           // every wave is done with the previous piece's LDS slots
      first = false;
      run_piece(tile, k0, T, w - wf, wl - wf + 1);
      it += T;
    }
  }
}

template <int BM, int STAGES, bool PIPE>
int launch_wg(const WgArgs& a, hipStream_t st) {
  constexpr int lds = STAGES * (BM + 128) * 128;
  auto k = a.sk_q > 0 ? gemm_wg_kernel<BM, STAGES, PIPE, true> : gemm_wg_kernel<BM, STAGES, PIPE, false>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_wg_kernel<BM, STAGES, PIPE, true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_wg_kernel<BM, STAGES, PIPE, false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const long long grid = a.sk_q > 0 ? ceil_div((long long)a.tiles_m * a.tiles_n * a.kt_total, (long long)a.sk_q)
                                     : (long long)a.tiles_m * a.tiles_n * a.splits;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(2 * BM), lds, st, a);
  MDTF_LAUNCH_CHECK();
  return 0;
}

bool fits(long long rows, long long ld) { return rows * ld * 2 < (1ll << 31); }

}  // namespace

// Workspace for a launch: slab floats (splits > 1) = tiles * splits * bm * 128, tickets = tiles ints.
MDTF_EXPORT long long mdtf_gemm_wg_slab_floats(int M, int N, int bm, int splits) {
  if (splits <= 1) return 0;
  return (long long)(M / bm) * (N / 128) * splits * bm * 128;
}

// The same with K known: splits < 0 is stream-K over -splits workers (tiles * maxp partial tiles).
MDTF_EXPORT long long mdtf_gemm_wg_slab_floats_k(int M, int N, int K, int bm, int splits) {
  if (splits >= 0) return mdtf_gemm_wg_slab_floats(M, N, bm, splits);
  const long long tiles = (long long)(M / bm) * (N / 128), KT = K / 64;
  const long long q = ceil_div(tiles * KT, (long long)-splits);
  return tiles * (ceil_div(KT, q) + 1) * bm * 128;
}

// C_s[M][seg_cols] (fp32, ldc) += A^T B over the segment's columns; A [K][lda], B [K][ldb] bf16 (k-major), M % bm,
// N % 128, K % 64 and seg_cols % 128 == 0.  bm: 128 or 256; stages 2..4 (negative: the pipelined loop); splits: K-split count (clamped so every
// split has at least one 64-deep tile), or -G: stream-K over G workers (every worker the same number of K-tiles).  dbias (per segment, may be null): += column sums of B.  slab / cnt:
// workspace of mdtf_gemm_wg_slab_floats() floats and tiles zeroed ints (splits > 1).  store_mask bit s: segment s's
// C is overwritten instead of accumulated into (the step's only write of a slot that was not zeroed).  Returns the splits used
// (> 0) or a negative MDTF status.
MDTF_EXPORT int mdtf_gemm_wg(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                             int nseg, int seg_cols, float* const* cseg, long long ldc, float* const* dbseg, int bm,
                             int stages, int splits, float* slab, int* cnt, int store_mask, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 128 || (bm != 128 && bm != 256) || M % bm) return MDTF_EUNSUPPORTED;
  if (lda % 8 || ldb % 8 || ldc % 4 || nseg < 1 || nseg > 4 || seg_cols % 128 || nseg * seg_cols != N)
    return MDTF_EUNSUPPORTED;
  if (!fits(K, lda) || !fits(K, ldb)) return MDTF_EUNSUPPORTED;
  WgArgs a{};
  a.A = A;
  a.B = B;
  a.lda = lda;
  a.ldb = ldb;
  a.M = M;
  a.N = N;
  a.K = K;
  a.tiles_m = M / bm;
  a.tiles_n = N / 128;
  const int KT = K / 64;
  a.kt_total = KT;
  if (splits < 0) {
    // stream-K over -splits workers
    const long long total = (long long)a.tiles_m * a.tiles_n * KT;
    const long long q = ceil_div(total, (long long)-splits);
    a.sk_q = (int)q;
    a.maxp = (int)ceil_div((long long)KT, q) + 1;
    a.splits = 1;
    a.kt_split = KT;
    if (slab == nullptr || cnt == nullptr) return MDTF_EINVAL;
  } else {
    if (splits < 1) splits = 1;
    if (splits > KT) splits = KT;
    a.kt_split = (KT + splits - 1) / splits;
    a.splits = (KT + a.kt_split - 1) / a.kt_split;
    a.maxp = a.splits;
    if (a.splits > 1 && (slab == nullptr || cnt == nullptr)) return MDTF_EINVAL;
  }
  a.bytes_a = (int)(K * lda * 2);
  a.bytes_b = (int)(K * ldb * 2);
  a.nseg = nseg;
  a.seg_cols = seg_cols;
  for (int i = 0; i < 4; ++i) {
    a.cf[i] = cseg[i < nseg ? i : 0];
    a.db[i] = dbseg ? dbseg[i < nseg ? i : 0] : nullptr;
  }
  a.ldc = ldc;
  a.slab = slab;
  a.cnt = cnt;
  a.store_mask = store_mask;
  {   // MDTF_WG_WT=0: plain slab stores + agent release / acquire fences (the round-3..5 publish form)
    static const int wt = [] {
      const char* e = getenv("MDTF_WG_WT");
      return (e && e[0] == '0') ? 0 : 1;
    }();
    a.wt = wt;
  }
  if (a.slab && (long long)a.maxp * bm * 128 * 4 >= (1ll << 31)) return MDTF_EUNSUPPORTED;
  // L2 block per XCD: ~ceil(grid / 8) tiles of one split as the gm x gn block with the fewest operand columns
  // (gm * bm + gn * 128) -- a speed choice only, any gm / gn is correct
  {
    const int tiles = a.tiles_m * a.tiles_n;
    const int per_xcd = a.sk_q > 0 ? (tiles + 7) / 8 : (tiles * a.splits + 7) / 8;
    const int want = per_xcd < tiles ? per_xcd : tiles;
    int best = 1 << 30;
    a.gm = a.tiles_m;
    a.gn = a.tiles_n;
    for (int g = 1; g <= a.tiles_m; ++g) {
      const int h = (want + g - 1) / g;
      if (h > a.tiles_n) continue;
      const int cost = g * bm + h * 128;
      if (cost < best) {
        best = cost;
        a.gm = g;
        a.gn = h;
      }
    }
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = MDTF_EINVAL;
  // stages < 0: the mid-tile-barrier pipelined loop with |stages| LDS stages
  if (bm == 128) {
    if (stages == 2) rc = launch_wg<128, 2, false>(a, st);
    else if (stages == 3) rc = launch_wg<128, 3, false>(a, st);
    else if (stages == 4) rc = launch_wg<128, 4, false>(a, st);
    else if (stages == -3) rc = launch_wg<128, 3, true>(a, st);
    else if (stages == -4) rc = launch_wg<128, 4, true>(a, st);
  } else {
    if (stages == 2) rc = launch_wg<256, 2, false>(a, st);
    else if (stages == 3) rc = launch_wg<256, 3, false>(a, st);
    else if (stages == -3) rc = launch_wg<256, 3, true>(a, st);
  }
  return rc == 0 ? a.splits : rc;
}
