// Ping-pong MFMA GEMM core (gfx950 / CDNA4): the dense matmul of every FC / transformer layer.
//
// Replaces the cuBLAS GEMM the reference reaches through tf.matmul in FC_layer
// (distribute_tools.py:204-206) and its autodiff backward (distribute_tower.py:27), SURVEY §2.5 K8.
//
//   C[M][N] (+)= Σ_k A(m, k) B(k, n)
//     A stored [M][K] (reduction-contiguous) or, ATR, [K][M];  B stored [N][K] or, BTR, [K][N].
//   dense forward   y  = x W       : A = x [M][K], B = W [K][N] (BTR)
//   data gradient   dx = dy W^T    : A = dy [M][N], B = W [K][N] read as [n=K][k=N]   (no transposes)
//   weight gradient dW = x^T dy    : A = x stored [m][k] (ATR), B = dy [m][n] (BTR), fp32 into the grad slot
//
// Structure (one 512-thread workgroup per CU, 8 waves = two groups of 4 that share the 4 SIMDs):
//   * 16x16x32 bf16 MFMA (on random data it holds a ~12-15 % higher clock than 32x32x16 at equal cycles
//     per FLOP, MI355X_MICROARCH.md 'DVFS give-back' item 7); each wave owns a RW x 64 output tile.
//   * K-tiles of 64, split into four LDS units per tile -- A rows half 0/1, B columns half 0/1 -- each
//     double-buffered (2 x (BM+BN) x 128 B: 128 KiB for 256 x 256).  Units are filled by LDS-DMA
//     (buffer_load_dwordx4 ... lds, bounds-checked zero fill), one unit per phase, so loads stream
//     continuously and never need a vmcnt(0) inside the loop.
//   * Four quadrant phases per K-tile.  Each phase is {ds_read fragments, issue one unit's DMA} ->
//     s_barrier -> {16..32 MFMAs} -> s_barrier.  Group 1 runs one barrier behind group 0, so on every
//     SIMD one wave issues MFMAs while its partner reads LDS and issues loads (ping-pong): the matrix
//     pipe never waits for a fragment read.  The DMA schedule below is derived from the barrier
//     numbering so every read of a unit follows (a) each issuing wave's vmcnt and (b) a barrier, and
//     every DMA into a slot follows the last read of the tile that used it (comments at `issue_unit`).
//   * Reduction-contiguous tiles are [rows][64 k] images read by ds_read_b128 with a 16-B chunk XOR
//     swizzle (conflict-free for the four 16-lane groups); k-major tiles are [64 k][cols] images read by
//     ds_read_b64_tr_b16 (hardware transpose) with a 32-B block XOR swizzle (conflict-free per 32-lane
//     half).  Both swizzles are applied to the DMA's per-lane SOURCE address, the LDS image stays linear.
//   * Epilogue straight from the accumulators: the MFMA is issued as C^T = B^T A^T, so each lane holds 4
//     consecutive output columns of one row (8 B bf16 / 16 B fp32 stores, 128-B rows per instruction),
//     with bias, ReLU/GELU (+ saved pre-activation), bf16 accumulate, or fp32 accumulate / split-K atomics.
//   * Tiles are XCD-remapped (bijective) so the column tiles of a row panel share an L2.
#include "mdtf_common.h"

using namespace mdtf;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr unsigned kOOB = 0x80000000u;   // buffer offset past num_records: the DMA writes zeros
constexpr int kCUs = 256;                 // MI355X compute units: one 512-thread GEMM block each

// Implicit-GEMM convolution on the same core (CONV = 1 forward, 2 stride-1 data gradient).  A is gathered: GEMM
// row m = one pixel of the row grid (fwd: output pixel, dgrad: DX pixel), K-tile t = 64 channels c0 of filter tap
// `tap` (taps in HWIO order, GC / 64 K-tiles per tap), read from the gathered tensor (fwd X, dgrad DY) at
//   fwd   (oh SH - PH + kh DH, ow SW - PW + kw DW)      dgrad (h + PH - kh DH, w + PW - kw DW)
// Each DMA lane keeps its row's element offset of tap (0, 0) and a bitmask of the taps that stay inside the image
// (computed once per tile with magic-number divisions); a K-tile adds a wave-uniform tap offset and tests one bit,
// taps outside the image get an offset past the buffer range (zero fill).  B is the filter, K-contiguous rows:
// fwd Wt[co][(tap, ci)] (the gemm layout), dgrad W[tap][ci][co] (row ci, tap stride Cin Cout).
struct ConvGeo {
  int GH, GW, GC;              // gathered tensor dims (per image)
  int RH, RW;                  // row-pixel grid per image
  unsigned mag_rw, mag_rh, mag_kw;
  int sh_rw, sh_rh, sh_kw;
  int SH, SW, PH, PW, DH, DW, KH, KW;
  int cpt_lg;                  // log2(GC / 64): K-tiles per tap
  long long wtap_bytes;        // dgrad: bytes per filter tap of B (Cin Cout 2)
  // forward epilogue: per-channel BatchNorm partials sum y, sum y^2 into row (tile_m % stat_slots)
  float* stat_sum;
  float* stat_sq;
  int stat_slots;
  // dgrad epilogue: out = result + (acc_src ? acc_src * acc_mask bit : out) when accumulating; BN-backward
  // statistics sum g m, sum g m x of the stored gradient g (m: bmask bit, x: bx) into row (tile_m % bslots)
  const bf16_t* acc_src;
  const uint8_t* acc_mask;
  const bf16_t* bx;
  const uint8_t* bmask;
  float* bsum;
  float* bsq;
  int bslots;
};

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  long long lda, ldb;        // row strides (elements) of the stored layouts
  int M, N, K;               // C is M x N; K = reduction (multiple of 64)
  int tiles_m, tiles_n;
  int kt_split;              // K-tiles per split (gridDim.y splits)
  int bytes_a, bytes_b;      // buffer ranges for the bounds checks (< 2 GiB)
  // bf16 output
  bf16_t* C;
  long long ldc;
  const bf16_t* bias;        // [N] bf16, added on the fp32 accumulators (null: none)
  bf16_t* pre;               // act != 0: the bf16 pre-activation is also stored here (null: not kept)
  int act;                   // 0 none, 1 relu, 2 gelu (tanh form)
  int accumulate;            // C = result + C
  // fp32 output
  float* Cf;
  long long ldcf;
  int atomic;                // 1: fp32 atomics (split-K); 0: Cf += result (one writer per element)
  // segmented operands (q|k|v as three matrices, no concatenated copy): nseg segments of seg_cols, segment s of
  // B at bseg[s] (row stride ldb), split along the output columns (fwd) or the reduction (dgrad); bias, Cf and
  // dbias are split the same way along the output columns.  nseg = 1: bseg[0] = B.
  int nseg, seg_cols;
  const bf16_t* bseg[4];
  const bf16_t* biasseg[4];
  float* cfseg[4];
  float* dbseg[4];           // wgrad: the column sums of B (dy: the bias gradient) are added here (null: none)
  const bf16_t* act_pre;     // dgrad: C = acc * act'(act_pre) (the producer's activation backward), null: none
  int act_bwd;
  int persistent;            // 1: grid = min(tiles, CUs) blocks loop over the tiles
  ConvGeo cv;                // CONV != 0
};

// n / d for n < 2^31 with a host-computed magic pair (umulhi + add + shift)
__device__ __forceinline__ unsigned fdiv(unsigned n, unsigned mag, int sh) { return (__umulhi(n, mag) + n) >> sh; }

void magic_u32(unsigned d, unsigned& mag, int& sh) {
  sh = 0;
  while ((1ull << sh) < d) ++sh;
  mag = static_cast<unsigned>(((1ull << 32) * ((1ull << sh) - d)) / d + 1);
}

__device__ __forceinline__ float act_fwd(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) {   // x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3)  (== 0.5 x (1 + tanh u))
    const float u2 = 1.5957691216f * (v + 0.044715f * v * v * v);
    return v * __builtin_amdgcn_rcpf(1.f + __expf(-u2));
  }
  return v;
}

// its derivative at the pre-activation x: relu [x > 0]; gelu s + 2 x s (1 - s) u'(x), s = sigmoid(2u)
__device__ __forceinline__ float act_grad(float x, int act) {
  if (act == 1) return x > 0.f ? 1.f : 0.f;
  const float s = __builtin_amdgcn_rcpf(1.f + __expf(-1.5957691216f * (x + 0.044715f * x * x * x)));
  return s + 2.f * x * s * (1.f - s) * 0.7978845608f * (1.f + 0.134145f * x * x);
}

__device__ __forceinline__ int seg_of(int col, int seg_cols, int nseg) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i) s += (i < nseg && col >= i * seg_cols) ? 1 : 0;
  return s;
}

// LDS-DMA of 16 B per lane: LDS destination = m0 (wave-uniform) + 16 * lane, source = rsrc + voff + soff.
// Issued from inline asm so the compiler neither sees an LDS write (no vmcnt(0) before our ds_reads) nor
// counts it: the kernel's own wait_vmcnt<N> + s_barrier order every read after it.  The s_nop 4 covers the VALU ->
// SGPR -> VMEM hazard the compiler does not pad before inline asm: an soffset / descriptor SGPR restored by
// v_readlane (SGPR spill) right before the DMA was read stale (the 256x192 conv tile loaded B rows 64..79 from
// rows 0..15), and M0 written by the SALU just before.
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

// bijective XCD-aware remap of a 1-D block index (cdna_hip_programming.md §5 T1)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// 32-B block swizzle of a [64 k][W cols] image (row pitch 2W bytes) for the transposed fragment reads:
// the 8 rows one 32-lane half reads ({0-3, 8-11} + 16 h, and +4) land in 8 distinct 32-B bank slots.
// pitch 256: 8 blocks per bank row; 128: two rows per bank row; 192: rows advance 6 slots, so only rows
// r and r+8 collide and one XOR bit separates them.
template <int PITCH>
__device__ __forceinline__ int trg(int row) {
  if constexpr (PITCH % 256 == 0) return (row & 3) | (((row >> 3) & 1) << 2);
  else if constexpr (PITCH == 192) return (row >> 3) & 1;
  else return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}

// One LDS unit image: W = rows (or, TR, columns) = half of the tile's side, 64 k deep.
template <int W, bool TR>
struct Unit {
  static constexpr int BYTES = W * 128;            // 64 k x W x 2 B
  static constexpr int NI = W / 8;                 // 1-KiB DMA wave-instructions that fill it
  static constexpr int PITCH = TR ? 2 * W : 128;   // image row pitch (bytes)
  // instructions issued by a wave of group G (wave w issues w, w + 8, ...: equal within a group)
  template <int G>
  static constexpr int per_wave() { return (NI - 4 * G + 7) / 8; }
};

// Tile geometry.  Eight waves = group G (M half) x 4 column strips; each wave owns (BM/2) x (BN/4).
//   BM = 256: four quadrant phases per 64-deep K-tile, 2 LDS stages, unit-level DMA schedule;
//   BM = 128: two k-substep phases per K-tile, 3 LDS stages, whole-tile DMA one tile further ahead.
template <int BM, int BN, bool ATR, bool BTR, int EPI, int CONV = 0>
__global__ void __launch_bounds__(512) gemm_pp_kernel(GemmArgs a) {
  static_assert(CONV == 0 || (!ATR && !BTR && EPI == 0), "conv: K-contiguous operands, bf16 output");
  constexpr int RW = BM / 2, CW = BN / 4;
  constexpr int FM = RW / 16, FN = CW / 16;
  constexpr int FMH = FM / 2, FNL = (FN + 1) / 2;
  constexpr int WA = BM / 2, WB = BN / 2;
  constexpr bool QUAD = BM == 256;
  constexpr int STAGES = QUAD ? 2 : 3;
  using UA = Unit<WA, ATR>;
  using UB = Unit<WB, BTR>;
  constexpr int SLOT = 2 * UA::BYTES + 2 * UB::BYTES;
  static_assert(FM >= 2 && FN >= 2 && CW % 16 == 0 && WA % 64 == 0 && WB % 8 == 0, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = wave >> 2, wc = wave & 3;
  // persistent over output tiles (a.persistent: grid = min(tiles, CUs)); the next tile's first loads are issued
  // before this tile's epilogue, so the pipeline fill overlaps the stores
  const int ntiles = a.tiles_m * a.tiles_n;
  int it = blockIdx.x;
  int tm = 0, tn = 0, m0 = 0, n0 = 0;
  auto set_tile = [&](int i) {
    const int tile = xcd_remap(i, ntiles);
    tm = tile / a.tiles_n;
    tn = tile - tm * a.tiles_n;
    m0 = tm * BM;
    n0 = tn * BN;
  };
  set_tile(it);
  const int kt0 = blockIdx.y * a.kt_split;
  const int T = min(a.kt_split, a.K / 64 - kt0);

  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<unsigned long long>(
      (__attribute__((address_space(3))) char*)smem));
  const i32x4_t ra = buffer_rsrc(a.A, a.bytes_a);

  // ---- per-lane DMA source offsets.  One VGPR per operand: instruction j of a wave and unit half u differ by a
  // wave-uniform byte delta (soffset), because the swizzles depend only on row bits that those steps preserve.
  // Rows past the operand (non-TR) fall past the buffer range by themselves and read zeros; columns past it
  // (TR) are marked out of range, and the host only takes TR operands whose extent is a multiple of the tile.
  auto src_off = [&](bool tr, int pitch, long long ld, int base, int limit, int ii) -> unsigned {
    const int off = ii * 1024 + lane * 16;          // byte offset inside the unit image
    if (!tr) {
      const int row = off >> 7, pc = (off >> 4) & 7;
      const int lc = pc ^ ((row >> 1) & 7);
      return static_cast<unsigned>(((long long)(base + row) * ld + (long long)kt0 * 64 + lc * 8) * 2);
    }
    const int row = off / pitch, cb = off - row * pitch;
    const int pb = cb >> 5, half = (cb >> 4) & 1;
    const int g = pitch % 256 == 0 ? trg<256>(row) : pitch == 192 ? trg<192>(row) : trg<128>(row);
    const int col = base + (pb ^ g) * 16 + half * 8;
    if (col >= limit) return kOOB;
    return static_cast<unsigned>((((long long)kt0 * 64 + row) * ld + col) * 2);
  };
  // a 192-B-pitch transposed image: instruction j = 1 does not start on a row boundary -> its own offsets
  constexpr bool B_J1 = BTR && UB::PITCH == 192;
  unsigned vA = 0, vB = 0, vB1 = 0;
  // CONV: per (unit half u, instruction j) the lane's row offset of tap (0, 0) (elements, channel chunk included)
  // and its in-image tap mask.  Row = u WA + (8 j + wave) 8 + lane / 8; its 16-B chunk swizzle does not depend
  // on u or j (WA and 64 j are multiples of 16 rows).
  constexpr int JA = (UA::NI + 7) / 8;
  unsigned cA[2][JA], mA[2][JA];
  auto conv_rows = [&]() {
    const ConvGeo& g = a.cv;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < JA; ++j) {
        const int row = u * WA + (8 * j + wave) * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        const int m = m0 + row;
        unsigned mask = 0, base = 0;
        if (m < a.M && (8 * j + wave) < UA::NI) {
          const unsigned t1 = fdiv(m, g.mag_rw, g.sh_rw);
          const int ow = m - static_cast<int>(t1) * g.RW;
          const unsigned n = fdiv(t1, g.mag_rh, g.sh_rh);
          const int oh = static_cast<int>(t1 - n * g.RH);
          const int y0 = CONV == 1 ? oh * g.SH - g.PH : oh + g.PH;
          const int x0 = CONV == 1 ? ow * g.SW - g.PW : ow + g.PW;
          unsigned wm = 0;
          for (int kw = 0; kw < g.KW; ++kw) {
            const int ix = CONV == 1 ? x0 + kw * g.DW : x0 - kw * g.DW;
            wm |= (ix >= 0 && ix < g.GW) ? (1u << kw) : 0u;
          }
          for (int kh = 0; kh < g.KH; ++kh) {
            const int iy = CONV == 1 ? y0 + kh * g.DH : y0 - kh * g.DH;
            if (iy >= 0 && iy < g.GH) mask |= wm << (kh * g.KW);
          }
          base = ((n * g.GH + y0) * g.GW + x0) * g.GC + lc * 8;
        }
        cA[u][j] = base;
        mA[u][j] = mask;
      }
  };
  auto set_offsets = [&]() {
    if constexpr (CONV != 0) conv_rows();
    vA = src_off(ATR, UA::PITCH, a.lda, m0, a.M, wave);
    vB = src_off(BTR, UB::PITCH, a.ldb, n0, a.N, wave);
    vB1 = B_J1 ? src_off(true, UB::PITCH, a.ldb, n0, a.N, 8 + wave) : 0u;
  };
  set_offsets();
  const int duA = ATR ? WA * 2 : (int)(WA * a.lda * 2);                   // unit half 1
  const int djA = ATR ? (int)((8192 / UA::PITCH) * a.lda * 2) : (int)(64 * a.lda * 2);   // instruction j = 1
  const int duB = BTR ? WB * 2 : (int)(WB * a.ldb * 2);
  const int djB = BTR ? (B_J1 ? 0 : (int)((8192 / UB::PITCH) * a.ldb * 2)) : (int)(64 * a.ldb * 2);
  const int stepA = ATR ? (int)(64 * a.lda * 2) : 128;     // per K-tile source advance
  const int stepB = BTR ? (int)(64 * a.ldb * 2) : 128;

  // this wave's (group-uniform) share of unit u of K-tile t, into slot t % STAGES
  auto issue_unit = [&](int u, int t) {
    const unsigned slot = lds0 + (t % STAGES) * SLOT;
    if (CONV != 0 && u < 2) {
      const ConvGeo& g = a.cv;
      const int tap = t >> g.cpt_lg;
      const int c0 = (t & ((1 << g.cpt_lg) - 1)) * 64;
      const int kh = static_cast<int>(fdiv(tap, g.mag_kw, g.sh_kw)), kw = tap - kh * g.KW;
      const int sp = (kh * g.DH * g.GW + kw * g.DW) * g.GC;
      const unsigned te = static_cast<unsigned>((CONV == 1 ? sp : -sp) + c0);
      const int cnt = G == 0 ? UA::template per_wave<0>() : UA::template per_wave<1>();
#pragma unroll
      for (int j = 0; j < JA; ++j)
        if (j < cnt) {
          const unsigned c = u == 0 ? cA[0][j] : cA[1][j];
          const unsigned m = u == 0 ? mA[0][j] : mA[1][j];
          dma16(ra, slot + u * UA::BYTES + (j * 8 + wave) * 1024, ((m >> tap) & 1u) ? (c + te) * 2u : kOOB, 0);
        }
      return;
    }
    if (u < 2) {
      const int cnt = G == 0 ? UA::template per_wave<0>() : UA::template per_wave<1>();
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (j < cnt) dma16(ra, slot + u * UA::BYTES + (j * 8 + wave) * 1024, vA, t * stepA + u * duA + j * djA);
    } else {
      const int cnt = G == 0 ? UB::template per_wave<0>() : UB::template per_wave<1>();
      // the segment this unit reads: by output column (transposed B) or by reduction index (dgrad)
      const int seg = BTR ? (n0 + (u - 2) * WB) / a.seg_cols : ((kt0 + t) * 64) / a.seg_cols;
      // segment rebasing folded into the descriptor (a negative soffset would break the range check): the
      // column / reduction index counts from the first segment's origin
      const i32x4_t rb = buffer_rsrc(a.bseg[seg] - seg * a.seg_cols, a.bytes_b + seg * a.seg_cols * 2);
      int sb = t * stepB + (u - 2) * duB;
      if constexpr (CONV == 2) {      // W[tap][ci][co]: the K-tile's tap block, then its 64 output channels
        const int tap = t >> a.cv.cpt_lg;
        sb = static_cast<int>(tap * a.cv.wtap_bytes) + (t & ((1 << a.cv.cpt_lg) - 1)) * 128 + (u - 2) * duB;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (j < cnt)
          dma16(rb, slot + 2 * UA::BYTES + (u - 2) * UB::BYTES + (j * 8 + wave) * 1024, (B_J1 && j) ? vB1 : vB,
                sb + j * djB);
    }
  };
  // per-wave DMA instruction counts of the groups (compile time)
  constexpr int CB0 = UB::template per_wave<0>(), CB1 = UB::template per_wave<1>();
  constexpr int CT0 = 2 * UA::template per_wave<0>() + 2 * CB0, CT1 = 2 * UA::template per_wave<1>() + 2 * CB1;

  // ---- fragment reads (bytes relative to a slot)
  const int fr = lane & 15, fq = lane >> 4;
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int ub = wc >> 1;                       // the B unit holding this wave's column strip
  const int b_col0 = (wc & 1) * CW;             // its first column inside that unit
  const unsigned baseA = G * UA::BYTES;
  const unsigned baseB = 2 * UA::BYTES + ub * UB::BYTES;

  auto frag = [&](bool tr, int pitch, unsigned ubase, int r0, int s, const char* slotp) -> bf16x8_t {
    if (!tr) {
      const int row = r0 + fr;
      const int ch = (4 * s + fq) ^ ((row >> 1) & 7);
      const uint4 v = *reinterpret_cast<const uint4*>(slotp + ubase + row * 128 + ch * 16);
      return __builtin_bit_cast(bf16x8_t, v);
    }
    const int row = 32 * s + 8 * fq + q4;
    const int g = pitch % 256 == 0 ? trg<256>(row) : pitch == 192 ? trg<192>(row) : trg<128>(row);
    const int blk = (r0 >> 4) ^ g;
    const char* p1 = slotp + ubase + row * pitch + blk * 32 + p4 * 8;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p1);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p1 + 4 * pitch));
    const short8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, f);
  };
  auto fragA = [&](int i, int s, const char* slotp) { return frag(ATR, UA::PITCH, baseA, 16 * i, s, slotp); };
  auto fragB = [&](int j, int s, const char* slotp) {
    return frag(BTR, UB::PITCH, baseB, b_col0 + 16 * j, s, slotp);
  };

  float4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  // wgrad bias gradient: the column sums of B by an all-ones A fragment, in the waves of the first row tile's
  // group 0 (each output column once per split)
  bool dsum = false;
  float4v accb[FN];
  const short8 ones8 = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, ones8);

  // the first loads of a tile: the whole K-tile 0, plus the K-tile-1 units the schedule expects in flight
  auto prologue_issue = [&]() {
#pragma unroll
    for (int u = 0; u < 4; ++u) issue_unit(u, 0);
    if (T > 1) {
      if constexpr (QUAD) {
        issue_unit(2, 1);
        if (G == 1) issue_unit(3, 1);
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) issue_unit(u, 1);
      }
    }
  };
  prologue_issue();
  bool first = true;
  // stores of a whole in-range bf16 tile (EPI 0, no conv): one 8-B store per (i, j), plus the pre-activation's
  // when it is kept.  A later tile's first wait leaves exactly those in flight (they are younger than its
  // prologue loads), so the previous tile's store drain overlaps this tile's first K-steps instead of stalling it.
  // (conv forward with BN statistics: + 2 atomics per column fragment)
  // (GEMM: the 16-B paired stores, FN / 2 + FN % 2 per row fragment; conv: 8-B stores)
  constexpr int NSTG = FM * (FN / 2 + FN % 2);
  constexpr int NST1 = NSTG, NST2 = 2 * NSTG, NST3 = NSTG + 2 * FN;
  int prev_st = 0;          // 0: the previous epilogue issued an unknown store count (or none after the prologue)
  while (true) {
    if (first && T > 1) {
      if constexpr (QUAD) {
        if (G == 0) wait_vmcnt<CB0>();
        else wait_vmcnt<2 * CB1>();    // its own B0(1) + B1(1) (CB0 != CB1 when a B unit is 96 wide)
      } else {
        if (G == 0) wait_vmcnt<CT0>();
        else wait_vmcnt<CT1>();
      }
    } else if (EPI == 0 && prev_st != 0) {
      // ops younger than this tile's prologue: its K-tile-1 units (T > 1) and the previous tile's stores; any count
      // up to their number is safe (vmcnt: all but the n youngest are done), so the sums are capped at 63
      constexpr int W0 = QUAD ? CB0 : CT0, W1 = QUAD ? 2 * CB1 : CT1;
#define PP_WAIT(NS_)                                                        \
  if (T > 1) {                                                              \
    if (G == 0) wait_vmcnt<(W0 + NS_ < 63 ? W0 + NS_ : 63)>();              \
    else wait_vmcnt<(W1 + NS_ < 63 ? W1 + NS_ : 63)>();                     \
  } else {                                                                  \
    wait_vmcnt<(NS_ < 63 ? NS_ : 63)>();                                    \
  }
      if (prev_st == 1) {
        PP_WAIT(NST1)
      } else if (prev_st == 2) {
        PP_WAIT(NST2)
      } else {
        PP_WAIT(NST3)
      }
#undef PP_WAIT
    } else {
      wait_vmcnt<0>();       // (a later tile: the previous epilogue's stores were issued after these loads)
    }
    barrier();
    if (G == 1) barrier();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    dsum = EPI == 1 && a.dbseg[0] != nullptr && tm == 0 && G == 0;
#pragma unroll
    for (int j = 0; j < FN; ++j) accb[j] = float4v{0.f, 0.f, 0.f, 0.f};
  if constexpr (QUAD) {
    // ---- DMA schedule (quadrant phases).  Barrier numbering: group 0 passes b(2P) / b(2P+1) around the MFMAs
    // of phase P (P = 4t + q), group 1 b(2P+1) / b(2P+2).  Reads of K-tile t: group 0 in phases 4t..4t+2, group
    // 1 one barrier later; the B units of tile t are last read before b(8t+4), A half 0 before b(8t+5), A half 1
    // before b(8t+6).  Tile t+1 reuses tile t-1's slots and is first read after b(8t+7).  Hence:
    //   group 0 issues in phase 4t+q:  q0 B1(t+1)  q1 A0(t+1)  q2 A1(t+1)  q3 B0(t+2)
    //   group 1 issues in phase 4t+q:  q0 A0(t+1)  q1 A1(t+1)  q2 B0(t+2)  q3 B1(t+2)
    // and each wave waits for everything but its B0(t+2) (vmcnt) before b(8t+7): group 0 after the MFMAs of
    // phase 4t+3, group 1 before its first barrier of that phase.
    bf16x8_t fa[FMH][2], fb[FN][2];
    for (int t = 0; t < T; ++t) {
      const char* slotp = smem + (t & 1) * SLOT;
      const bool n1 = t + 1 < T, n2 = t + 2 < T;
      // ---------------- q0: A top + B left; MFMA top x left
#pragma unroll
      for (int i = 0; i < FMH; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) fa[i][s] = fragA(i, s, slotp);
#pragma unroll
      for (int j = 0; j < FNL; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) fb[j][s] = fragB(j, s, slotp);
      if (n1) issue_unit(G == 0 ? 3 : 0, t + 1);
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FMH; ++i)
#pragma unroll
          for (int j = 0; j < FNL; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], acc[i][j], 0, 0, 0);
      if (dsum) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < FNL; ++j) accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], ones, accb[j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---------------- q1: B right; MFMA top x right
#pragma unroll
      for (int j = FNL; j < FN; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) fb[j][s] = fragB(j, s, slotp);
      if (n1) issue_unit(G == 0 ? 0 : 1, t + 1);
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FMH; ++i)
#pragma unroll
          for (int j = FNL; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], acc[i][j], 0, 0, 0);
      if (dsum) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = FNL; j < FN; ++j) accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], ones, accb[j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---------------- q2: A bottom; MFMA bottom x right
#pragma unroll
      for (int i = 0; i < FMH; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) fa[i][s] = fragA(FMH + i, s, slotp);
      if (G == 0) {
        if (n1) issue_unit(1, t + 1);
      } else {
        if (n2) issue_unit(2, t + 2);
      }
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FMH; ++i)
#pragma unroll
          for (int j = FNL; j < FN; ++j)
            acc[FMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], acc[FMH + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // ---------------- q3: no reads; MFMA bottom x left
      if (G == 1) {
        if (n2) wait_vmcnt<CB1>();
        else wait_vmcnt<0>();
        if (n2) issue_unit(3, t + 2);
      } else {
        if (n2) issue_unit(2, t + 2);
      }
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < FMH; ++i)
#pragma unroll
          for (int j = 0; j < FNL; ++j)
            acc[FMH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][s], fa[i][s], acc[FMH + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (G == 0) {
        if (n2) wait_vmcnt<CB0>();
        else wait_vmcnt<0>();
      }
      barrier();
    }
    if (G == 0) barrier();
  } else {
    // ---- DMA schedule (k-substep phases, 3 stages).  Phase P = 2t + s (s = k-substep); same barrier numbering.
    // Tile t's reads end before b(4t+4); tile t+2 (slot of tile t-1, free after b(4t)) is issued whole by
    // group 1 in phase 2t (after b(4t)) and by group 0 in phase 2t+1, and first read after b(4t+7).  Each wave
    // waits for tile t+1 (everything but its tile-(t+2) instructions) before b(4t+3): group 1 before its first
    // barrier of phase 2t+1, group 0 after that phase's MFMAs.
    bf16x8_t fa[FM], fb[FN];
    for (int t = 0; t < T; ++t) {
      const char* slotp = smem + (t % 3) * SLOT;
      const bool n2 = t + 2 < T;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = fragA(i, s, slotp);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = fragB(j, s, slotp);
        if (s == 1 - G && n2) {
#pragma unroll
          for (int u = 0; u < 4; ++u) issue_unit(u, t + 2);
        }
        if (s == 1 && G == 1) {
          if (n2) wait_vmcnt<CT1>();
          else wait_vmcnt<0>();
        }
        barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
        if (dsum) {
#pragma unroll
          for (int j = 0; j < FN; ++j) accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], ones, accb[j], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        if (s == 1 && G == 0) {
          if (n2) wait_vmcnt<CT0>();
          else wait_vmcnt<0>();
        }
        barrier();
      }
    }
    if (G == 0) barrier();
  }

  // ---- next tile's first loads (every LDS read of this tile is done: all waves passed the last barrier)
  const int em0 = m0, en0 = n0;
  const bool edsum = dsum;
  const int nxt = it + gridDim.x;
  const bool more = a.persistent && nxt < ntiles;
  // the compiler's own waits for epilogue loads would also wait for the (invisible) next-tile DMA: the bias is
  // loaded first; epilogues that read C or the pre-activation per element issue the next loads after them
  uint2 bpre[FN];
  if (EPI == 0 && a.biasseg[0]) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = min(en0 + wc * CW + 4 * fq + 16 * j, a.N - 4);
      const int sg = seg_of(col, a.seg_cols, a.nseg);
      bpre[j] = *reinterpret_cast<const uint2*>(a.biasseg[sg] + (col - sg * a.seg_cols));
    }
  }
  const bool early = !(a.act_bwd || a.accumulate || (EPI == 1 && !a.atomic) || (CONV == 2 && a.cv.bsum));
  if (more && early) {
    set_tile(nxt);
    set_offsets();
    prologue_issue();
  }
  // the next tile may leave this epilogue's stores in flight when their count is known: every (i, j) in range
  const bool whole = em0 + BM <= a.M && en0 + BN <= a.N;
  int next_st = 0;
  if (EPI == 0 && early && whole) {
    if constexpr (CONV == 0) next_st = (a.act && a.pre) ? 2 : 1;     // (early: no accumulate, no act_bwd)
    else if constexpr (CONV == 1) next_st = a.cv.stat_sum ? 3 : 1;
    else next_st = 1;
  }
  // ---- epilogue: lane holds C[row][col .. col+3] for each (i, j)
  const int rbase = em0 + G * (BM / 2) + fr;
  const int cbase = en0 + wc * CW + 4 * fq;
  if (edsum && fr == 0) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = cbase + 16 * j;
      if (col >= a.N) continue;
      const int sg = seg_of(col, a.seg_cols, a.nseg);
      float* db = a.dbseg[sg] + (col - sg * a.seg_cols);
#pragma unroll
      for (int e = 0; e < 4; ++e) unsafeAtomicAdd(db + e, accb[j][e]);
    }
  }
  if constexpr (CONV != 0) {
    // ---- convolution epilogue: bf16 store (dgrad: + accumulate source), BN statistics of the tile's columns
    const ConvGeo& g = a.cv;
    const bool st = CONV == 1 ? g.stat_sum != nullptr : g.bsum != nullptr;
    float s0[FN][4], s1[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) s0[j][e] = s1[j][e] = 0.f;
    if (!(CONV == 2 && a.accumulate)) {
      // no accumulate source: 16-B paired stores as in the GEMM epilogue (v_permlane16_swap of fragments j, j+1)
      const int sbase = en0 + wc * CW;
      const int pcol = 16 * (fq & 1) + 8 * (fq >> 1);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = rbase + 16 * i;
        const bool rok = row < a.M;
        uint2 pk[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = cbase + 16 * j;
          const float4v v = acc[i][j];
          pk[j] = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
          if (!rok || col >= a.N) continue;
          if (CONV == 1 && st) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              s0[j][e] += v[e];
              s1[j][e] += v[e] * v[e];
            }
          } else if (CONV == 2 && st) {
            const long long off = (long long)row * a.ldc + col;
            const uint2 xq = *reinterpret_cast<const uint2*>(g.bx + off);
            const unsigned nb = g.bmask ? (g.bmask[off >> 3] >> (off & 7)) & 15u : 15u;
            const float gv[4] = {__uint_as_float(pk[j].x << 16), __uint_as_float(pk[j].x & 0xffff0000u),
                                 __uint_as_float(pk[j].y << 16), __uint_as_float(pk[j].y & 0xffff0000u)};
            const float xv[4] = {__uint_as_float(xq.x << 16), __uint_as_float(xq.x & 0xffff0000u),
                                 __uint_as_float(xq.y << 16), __uint_as_float(xq.y & 0xffff0000u)};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float gm = ((nb >> e) & 1u) ? gv[e] : 0.f;
              s0[j][e] += gm;
              s1[j][e] += gm * xv[e];
            }
          }
        }
#pragma unroll
        for (int j = 0; j + 1 < FN; j += 2) {
          if (sbase + 16 * j + 32 <= a.N) {
            auto sx = __builtin_amdgcn_permlane16_swap(pk[j].x, pk[j + 1].x, false, false);
            auto sy = __builtin_amdgcn_permlane16_swap(pk[j].y, pk[j + 1].y, false, false);
            if (rok)
              *reinterpret_cast<uint4*>(a.C + (long long)row * a.ldc + sbase + 16 * j + pcol) =
                  make_uint4(sx[0], sy[0], sx[1], sy[1]);
          } else {
#pragma unroll
            for (int jj = j; jj < j + 2; ++jj)
              if (rok && cbase + 16 * jj < a.N) *reinterpret_cast<uint2*>(a.C + (long long)row * a.ldc + cbase + 16 * jj) = pk[jj];
          }
        }
        if constexpr (FN % 2 == 1) {
          if (rok && cbase + 16 * (FN - 1) < a.N)
            *reinterpret_cast<uint2*>(a.C + (long long)row * a.ldc + cbase + 16 * (FN - 1)) = pk[FN - 1];
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = rbase + 16 * i;
      if (row >= a.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = cbase + 16 * j;
        if (col >= a.N) continue;
        const long long off = (long long)row * a.ldc + col;
        float4v v = acc[i][j];
        if (CONV == 2 && a.accumulate) {
          uint2 o = *reinterpret_cast<const uint2*>((g.acc_src ? g.acc_src : a.C) + off);
          if (g.acc_mask) {
            const unsigned nb = (g.acc_mask[off >> 3] >> (off & 7)) & 15u;
            o.x &= ((nb & 1u) ? 0x0000ffffu : 0u) | ((nb & 2u) ? 0xffff0000u : 0u);
            o.y &= ((nb & 4u) ? 0x0000ffffu : 0u) | ((nb & 8u) ? 0xffff0000u : 0u);
          }
          v[0] += __uint_as_float(o.x << 16);
          v[1] += __uint_as_float(o.x & 0xffff0000u);
          v[2] += __uint_as_float(o.y << 16);
          v[3] += __uint_as_float(o.y & 0xffff0000u);
        }
        const uint2 pk = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        *reinterpret_cast<uint2*>(a.C + off) = pk;
        if (CONV == 1 && st) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s0[j][e] += v[e];
            s1[j][e] += v[e] * v[e];
          }
        } else if (CONV == 2 && st) {
          const uint2 xq = *reinterpret_cast<const uint2*>(g.bx + off);
          const unsigned nb = g.bmask ? (g.bmask[off >> 3] >> (off & 7)) & 15u : 15u;
          const float gv[4] = {__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                               __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
          const float xv[4] = {__uint_as_float(xq.x << 16), __uint_as_float(xq.x & 0xffff0000u),
                               __uint_as_float(xq.y << 16), __uint_as_float(xq.y & 0xffff0000u)};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gm = ((nb >> e) & 1u) ? gv[e] : 0.f;
            s0[j][e] += gm;
            s1[j][e] += gm * xv[e];
          }
        }
      }
    }
    }
    if (st) {
      // the 16 lanes of a 4-column group hold 16 rows each: butterfly over lane bits 0..3, then lanes fr = e
      // (e < 4) add column e of every group
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            s0[j][e] += __shfl_xor(s0[j][e], o, 64);
            s1[j][e] += __shfl_xor(s1[j][e], o, 64);
          }
      float* psum = CONV == 1 ? g.stat_sum : g.bsum;
      float* psq = CONV == 1 ? g.stat_sq : g.bsq;
      const int slots = CONV == 1 ? g.stat_slots : g.bslots;
      const long long srow = (long long)((em0 / BM) % slots) * a.N;
      if (fr < 4) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = cbase + 16 * j + fr;
          if (col >= a.N) continue;
          const float v0 = fr == 0 ? s0[j][0] : fr == 1 ? s0[j][1] : fr == 2 ? s0[j][2] : s0[j][3];
          const float v1 = fr == 0 ? s1[j][0] : fr == 1 ? s1[j][1] : fr == 2 ? s1[j][2] : s1[j][3];
          atomicAdd(psum + srow + col, v0);
          atomicAdd(psq + srow + col, v1);
        }
      }
    }
  } else if (EPI == 0 && !a.accumulate) {
    // bf16 epilogue with 16-B stores: a lane holds 4 consecutive columns of one row per (i, j); one
    // v_permlane16_swap per dword of fragments j, j+1 gives lanes of 16-lane rows 0 / 2 columns 16j + 8 (fq / 2) ..
    // +7 and lanes of rows 1 / 3 columns 16(j+1) + 8 (fq / 2) .. +7 (the partner lanes hold the same output row),
    // so the tile goes out in half the store instructions (the epilogue is store-issue bound: bench/gemm_ksweep.py)
    const int sbase = en0 + wc * CW;
    const int pcol = 16 * (fq & 1) + 8 * (fq >> 1);      // this lane's column inside a 32-column pair
    const bool keep_pre = a.act && a.pre;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = rbase + 16 * i;
      const bool rok = row < a.M;
      uint2 pk[FN], pr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float4v v = acc[i][j];
        if (a.biasseg[0]) {
          const uint2 b4 = bpre[j];
          v[0] += __uint_as_float(b4.x << 16);
          v[1] += __uint_as_float(b4.x & 0xffff0000u);
          v[2] += __uint_as_float(b4.y << 16);
          v[3] += __uint_as_float(b4.y & 0xffff0000u);
        }
        if (a.act_bwd) {           // the producer's activation backward on the data gradient
          const int col = cbase + 16 * j;
          const uint2 pq = (rok && col < a.N) ? *reinterpret_cast<const uint2*>(a.act_pre + (long long)row * a.ldc + col)
                                              : make_uint2(0u, 0u);
          v[0] *= act_grad(__uint_as_float(pq.x << 16), a.act_bwd);
          v[1] *= act_grad(__uint_as_float(pq.x & 0xffff0000u), a.act_bwd);
          v[2] *= act_grad(__uint_as_float(pq.y << 16), a.act_bwd);
          v[3] *= act_grad(__uint_as_float(pq.y & 0xffff0000u), a.act_bwd);
        }
        if (a.act) {
          pr[j] = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
          // the activation of the ROUNDED pre-activation (what the backward recomputes from)
          v[0] = act_fwd(__uint_as_float(pr[j].x << 16), a.act);
          v[1] = act_fwd(__uint_as_float(pr[j].x & 0xffff0000u), a.act);
          v[2] = act_fwd(__uint_as_float(pr[j].y << 16), a.act);
          v[3] = act_fwd(__uint_as_float(pr[j].y & 0xffff0000u), a.act);
        }
        pk[j] = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
      }
#pragma unroll
      for (int j = 0; j + 1 < FN; j += 2) {
        if (sbase + 16 * j + 32 <= a.N) {              // (wave-uniform)
          auto sx = __builtin_amdgcn_permlane16_swap(pk[j].x, pk[j + 1].x, false, false);
          auto sy = __builtin_amdgcn_permlane16_swap(pk[j].y, pk[j + 1].y, false, false);
          const long long off = (long long)row * a.ldc + sbase + 16 * j + pcol;
          if (rok) *reinterpret_cast<uint4*>(a.C + off) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
          if (keep_pre) {
            auto px = __builtin_amdgcn_permlane16_swap(pr[j].x, pr[j + 1].x, false, false);
            auto py = __builtin_amdgcn_permlane16_swap(pr[j].y, pr[j + 1].y, false, false);
            if (rok) *reinterpret_cast<uint4*>(a.pre + off) = make_uint4(px[0], py[0], px[1], py[1]);
          }
        } else {
#pragma unroll
          for (int jj = j; jj < j + 2; ++jj) {
            const int col = cbase + 16 * jj;
            if (!rok || col >= a.N) continue;
            const long long off = (long long)row * a.ldc + col;
            *reinterpret_cast<uint2*>(a.C + off) = pk[jj];
            if (keep_pre) *reinterpret_cast<uint2*>(a.pre + off) = pr[jj];
          }
        }
      }
      if constexpr (FN % 2 == 1) {
        const int col = cbase + 16 * (FN - 1);
        if (rok && col < a.N) {
          const long long off = (long long)row * a.ldc + col;
          *reinterpret_cast<uint2*>(a.C + off) = pk[FN - 1];
          if (keep_pre) *reinterpret_cast<uint2*>(a.pre + off) = pr[FN - 1];
        }
      }
    }
  } else {
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = rbase + 16 * i;
    if (row >= a.M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = cbase + 16 * j;
      if (col >= a.N) continue;     // N % 4 == 0 (host-checked): whole 4-column groups
      const int sg = seg_of(col, a.seg_cols, a.nseg);
      float4v v = acc[i][j];
      if constexpr (EPI == 0) {
        if (a.biasseg[0]) {
          const uint2 b4 = bpre[j];
          v[0] += __uint_as_float(b4.x << 16);
          v[1] += __uint_as_float(b4.x & 0xffff0000u);
          v[2] += __uint_as_float(b4.y << 16);
          v[3] += __uint_as_float(b4.y & 0xffff0000u);
        }
        bf16_t* dst = a.C + (long long)row * a.ldc + col;
        if (a.act_bwd) {           // the producer's activation backward on the data gradient
          const uint2 pq = *reinterpret_cast<const uint2*>(a.act_pre + (long long)row * a.ldc + col);
          v[0] *= act_grad(__uint_as_float(pq.x << 16), a.act_bwd);
          v[1] *= act_grad(__uint_as_float(pq.x & 0xffff0000u), a.act_bwd);
          v[2] *= act_grad(__uint_as_float(pq.y << 16), a.act_bwd);
          v[3] *= act_grad(__uint_as_float(pq.y & 0xffff0000u), a.act_bwd);
        }
        if (a.accumulate) {
          const uint2 o = *reinterpret_cast<const uint2*>(dst);
          v[0] += __uint_as_float(o.x << 16);
          v[1] += __uint_as_float(o.x & 0xffff0000u);
          v[2] += __uint_as_float(o.y << 16);
          v[3] += __uint_as_float(o.y & 0xffff0000u);
        }
        if (a.act) {
          const uint2 pr = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
          if (a.pre) *reinterpret_cast<uint2*>(a.pre + (long long)row * a.ldc + col) = pr;
          // the activation of the ROUNDED pre-activation (what the backward recomputes from)
          v[0] = act_fwd(__uint_as_float(pr.x << 16), a.act);
          v[1] = act_fwd(__uint_as_float(pr.x & 0xffff0000u), a.act);
          v[2] = act_fwd(__uint_as_float(pr.y << 16), a.act);
          v[3] = act_fwd(__uint_as_float(pr.y & 0xffff0000u), a.act);
        }
        *reinterpret_cast<uint2*>(dst) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
      } else {
        float* dst = a.cfseg[sg] + (long long)row * a.ldcf + (col - sg * a.seg_cols);
        if (a.atomic) {
#pragma unroll
          for (int e = 0; e < 4; ++e) unsafeAtomicAdd(dst + e, v[e]);
        } else {
          float4 o = *reinterpret_cast<const float4*>(dst);
          o.x += v[0];
          o.y += v[1];
          o.z += v[2];
          o.w += v[3];
          *reinterpret_cast<float4*>(dst) = o;
        }
      }
    }
  }
  }
  if (!more) break;
  if (!early) {
    set_tile(nxt);
    set_offsets();
    prologue_issue();
  }
  it = nxt;
  first = false;
  prev_st = next_st;
  }
}

template <int BM, int BN, bool ATR, bool BTR, int EPI, int CONV = 0>
int launch_pp(const GemmArgs& a0, int splits, hipStream_t st) {
  GemmArgs a = a0;
  // a transposed (k-major) operand's tile must not straddle its edge (see src_off)
  if ((ATR && a.M % BM) || (BTR && a.N % BN)) return MDTF_EUNSUPPORTED;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  const int KT = a.K / 64;
  if (splits < 1) splits = 1;
  if (splits > KT) splits = KT;
  a.kt_split = (KT + splits - 1) / splits;
  splits = (KT + a.kt_split - 1) / a.kt_split;
  if (EPI == 1) a.atomic = splits > 1 ? 1 : a.atomic;
  constexpr int lds = (BM == 256 ? 2 : 3) * (BM + BN) * 128;
  auto k = gemm_pp_kernel<BM, BN, ATR, BTR, EPI, CONV>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int ntiles = a.tiles_m * a.tiles_n;
  a.persistent = (splits == 1 && ntiles > kCUs) ? 1 : 0;
  dim3 grid(a.persistent ? kCUs : ntiles, splits);
  hipLaunchKernelGGL(k, grid, dim3(512), lds, st, a);
  MDTF_LAUNCH_CHECK();
  return 0;
}

// tile code: 0 = 256x256, 1 = 256x128, 2 = 128x256, 3 = 128x128, 4 = 256x192, 5 = 128x192
template <bool ATR, bool BTR, int EPI>
int dispatch(int tile, const GemmArgs& a, int splits, hipStream_t st) {
  switch (tile) {
    case 0: return launch_pp<256, 256, ATR, BTR, EPI>(a, splits, st);
    case 1: return launch_pp<256, 128, ATR, BTR, EPI>(a, splits, st);
    case 2: return launch_pp<128, 256, ATR, BTR, EPI>(a, splits, st);
    case 3: return launch_pp<128, 128, ATR, BTR, EPI>(a, splits, st);
    case 4: return launch_pp<256, 192, ATR, BTR, EPI>(a, splits, st);
    case 5: return launch_pp<128, 192, ATR, BTR, EPI>(a, splits, st);
  }
  return MDTF_EINVAL;
}

bool fits(long long rows, long long ld) { return rows * ld * 2 < (1ll << 31); }

}  // namespace

extern "C" int mdtf_get_deterministic();

// layout code: 0 = fwd (A [M][K], B [K][N] -> BTR), 1 = dgrad (A [M][K], B [N][K]), 2 = wgrad (A [K][M], B [K][N])
// C / Cf: exactly one non-null.  Segments (nseg 1..4, seg_cols): B = bseg[0..nseg) (fwd: along N, dgrad: along K),
// bias / Cf / dbias along N = biasseg / cfseg / dbseg.  act: forward activation (+ pre store); act_bwd: dgrad
// epilogue multiplies by act'(act_pre).  Returns 0, or MDTF_EUNSUPPORTED for shapes the kernel does not take.
MDTF_EXPORT int mdtf_gemm_pp(const bf16_t* A, long long lda, const bf16_t* const* bseg, long long ldb, int M, int N,
                             int K, int layout, int tile, int splits, int nseg, int seg_cols, bf16_t* C, long long ldc,
                             const bf16_t* const* biasseg, bf16_t* pre, int act, int accumulate, const bf16_t* act_pre,
                             int act_bwd, float* const* cfseg, long long ldcf, float* const* dbseg, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 4 || (lda % 8) || (ldb % 8)) return MDTF_EUNSUPPORTED;
  if (nseg < 1 || nseg > 4 || seg_cols <= 0) return MDTF_EINVAL;
  const bool fp32out = cfseg != nullptr && cfseg[0] != nullptr;
  if ((C != nullptr) == fp32out) return MDTF_EINVAL;     // exactly one output
  const bool atr = layout == 2, btr = layout == 0 || layout == 2;
  // segment geometry: whole segments cover the segmented dimension
  const int segdim = layout == 1 ? K : N;
  if (nseg * seg_cols != segdim || (nseg > 1 && (seg_cols % 64))) return MDTF_EUNSUPPORTED;
  // operand ranges (the buffer descriptors' 32-bit offsets): B per segment
  const long long brows = btr ? K : N;
  if (!(atr ? fits(K, lda) : fits(M, lda)) || !fits(brows, ldb)) return MDTF_EUNSUPPORTED;
  if (atr && M % 8) return MDTF_EUNSUPPORTED;     // k-major operands: whole 16-B column chunks
  if (btr && N % 8) return MDTF_EUNSUPPORTED;
  GemmArgs a{};
  a.A = A;
  a.B = bseg[0];
  a.lda = lda;
  a.ldb = ldb;
  a.M = M;
  a.N = N;
  a.K = K;
  a.bytes_a = (int)((atr ? (long long)K : (long long)M) * lda * 2);
  a.bytes_b = (int)(brows * ldb * 2);
  a.nseg = nseg;
  a.seg_cols = seg_cols;
  for (int i = 0; i < 4; ++i) {
    a.bseg[i] = i < nseg ? bseg[i] : bseg[0];
    a.biasseg[i] = biasseg ? (i < nseg ? biasseg[i] : biasseg[0]) : nullptr;
    a.cfseg[i] = fp32out ? (i < nseg ? cfseg[i] : cfseg[0]) : nullptr;
    a.dbseg[i] = dbseg ? (i < nseg ? dbseg[i] : dbseg[0]) : nullptr;
  }
  a.C = C;
  a.ldc = ldc;
  a.bias = a.biasseg[0];
  a.pre = pre;
  a.act = act;
  a.accumulate = accumulate;
  a.act_pre = act_pre;
  a.act_bwd = act_pre ? act_bwd : 0;
  a.Cf = a.cfseg[0];
  a.ldcf = ldcf;
  a.atomic = 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!fp32out) {
    if (splits > 1) return MDTF_EUNSUPPORTED;
    switch (layout) {
      case 0: return dispatch<false, true, 0>(tile, a, 1, st);
      case 1: return dispatch<false, false, 0>(tile, a, 1, st);
      case 2: return dispatch<true, true, 0>(tile, a, 1, st);
    }
    return MDTF_EINVAL;
  }
  if (mdtf_get_deterministic()) splits = 1;
  switch (layout) {
    case 0: return dispatch<false, true, 1>(tile, a, splits, st);
    case 1: return dispatch<false, false, 1>(tile, a, splits, st);
    case 2: return dispatch<true, true, 1>(tile, a, splits, st);
  }
  return MDTF_EINVAL;
}

// Convolution on the ping-pong core (CONV 1 = forward, 2 = stride-1 data gradient), NHWC bf16, fp32 accumulate.
//   fwd  : y[N,OH,OW,Cout] = conv(x[N,H,W,Cin], Wt[Cout][(kh,kw,ci)])      (+ BN partials stat_sum/sq[slots][Cout])
//   dgrad: dx[N,H,W,Cin]   = dgrad(dy[N,OH,OW,Cout], W[kh][kw][Cin][Cout]) (+ accumulate source, BN-bwd partials)
// The gathered channels (fwd Cin, dgrad Cout) must be 64 * 2^p; <= 32 taps; dgrad Cin % (tile cols) == 0.
// tile: gemm tile code (0 = 256x256, 1 = 256x128, 2 = 128x256, 3 = 128x128, 4 = 256x192, 5 = 128x192).
MDTF_EXPORT int mdtf_conv_pp(int pass, const void* src, const void* wgt, void* out, int N, int H, int W, int Cin,
                             int OH, int OW, int Cout, int KH, int KW, int SH, int SW, int PH, int PW, int DH, int DW,
                             int tile, float* stat_sum, float* stat_sq, int stat_slots, int accumulate,
                             const void* acc_src, const void* acc_mask, const void* bx, const void* bmask, float* bsum,
                             float* bsq, int bslots, void* stream) {
  if (pass != 1 && pass != 2) return MDTF_EINVAL;
  const int GC = pass == 1 ? Cin : Cout, NC = pass == 1 ? Cout : Cin;
  if (GC % 64 || NC % 8 || KH * KW > 32 || KH < 1 || KW < 1) return MDTF_EUNSUPPORTED;
  int lg = 0;
  while ((64 << lg) < GC) ++lg;
  if ((64 << lg) != GC) return MDTF_EUNSUPPORTED;
  if (pass == 2 && (SH != 1 || SW != 1)) return MDTF_EUNSUPPORTED;
  static const int tile_cols[6] = {256, 128, 256, 128, 192, 192};
  if (tile < 0 || tile > 5) return MDTF_EINVAL;
  if (pass == 2 && NC % tile_cols[tile]) return MDTF_EUNSUPPORTED;   // filter rows past Cin would alias a tap
  const long long gbytes = (long long)N * (pass == 1 ? H * W : OH * OW) * GC * 2;
  const long long M = (long long)N * (pass == 1 ? OH * OW : H * W);
  if (gbytes >= (1ll << 31) || M * NC >= (1ll << 31) || (long long)KH * KW * Cin * Cout * 2 >= (1ll << 31))
    return MDTF_EUNSUPPORTED;
  if ((acc_src || acc_mask) && !accumulate) return MDTF_EINVAL;
  GemmArgs a{};
  a.A = (const bf16_t*)src;
  a.B = (const bf16_t*)wgt;
  a.lda = GC;
  a.ldb = pass == 1 ? (long long)KH * KW * Cin : Cout;
  a.M = (int)M;
  a.N = NC;
  a.K = KH * KW * GC;
  a.bytes_a = (int)gbytes;
  a.bytes_b = (int)((long long)KH * KW * Cin * Cout * 2);
  a.nseg = 1;
  a.seg_cols = a.K;                 // non-transposed B: segments run along the reduction (one)
  for (int i = 0; i < 4; ++i) a.bseg[i] = a.B;
  a.C = (bf16_t*)out;
  a.ldc = NC;
  a.accumulate = pass == 2 ? accumulate : 0;
  ConvGeo& g = a.cv;
  g.GH = pass == 1 ? H : OH;
  g.GW = pass == 1 ? W : OW;
  g.GC = GC;
  g.RH = pass == 1 ? OH : H;
  g.RW = pass == 1 ? OW : W;
  magic_u32(g.RW, g.mag_rw, g.sh_rw);
  magic_u32(g.RH, g.mag_rh, g.sh_rh);
  magic_u32(KW, g.mag_kw, g.sh_kw);
  g.SH = SH; g.SW = SW; g.PH = PH; g.PW = PW; g.DH = DH; g.DW = DW; g.KH = KH; g.KW = KW;
  g.cpt_lg = lg;
  g.wtap_bytes = (long long)Cin * Cout * 2;
  g.stat_sum = stat_sum;
  g.stat_sq = stat_sq;
  g.stat_slots = stat_slots > 0 ? stat_slots : 1;
  g.acc_src = (const bf16_t*)acc_src;
  g.acc_mask = (const uint8_t*)acc_mask;
  g.bx = (const bf16_t*)bx;
  g.bmask = (const uint8_t*)bmask;
  g.bsum = bsum;
  g.bsq = bsq;
  g.bslots = bslots > 0 ? bslots : 1;
  hipStream_t st = static_cast<hipStream_t>(stream);
#define CPP(T_, BM_, BN_) \
  case T_: return pass == 1 ? launch_pp<BM_, BN_, false, false, 0, 1>(a, 1, st) : launch_pp<BM_, BN_, false, false, 0, 2>(a, 1, st);
  switch (tile) {
    CPP(0, 256, 256) CPP(1, 256, 128) CPP(2, 128, 256) CPP(3, 128, 128) CPP(4, 256, 192) CPP(5, 128, 192)
  }
#undef CPP
  return MDTF_EINVAL;
}
