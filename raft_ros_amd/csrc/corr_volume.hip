// All-pairs correlation on gfx950: pyramid build, radius-r lookup (fwd/bwd) and the
// pyramid backward, for the reference CorrBlock (core/corr.py:12-60).
//
// Semantics kept from the reference:
//   * level l = 2x2 / stride-2 average pool (floor) of level l-1 over the image-2 dims;
//   * lookup at coords / 2^l, window [-r, r]^2, bilinear, align_corners=True, zero padding
//     (grid_sample, core/utils/utils.py:57-71); channel order level-major, then x-offset
//     major (ch = l*(2r+1)^2 + ix*(2r+1) + iy, core/corr.py:37-43).
//
// MI355X design:
//   * the volume is linear in fmap2, so level l = alpha * f1 . pool_l(f2)^T: every level is
//     its own MFMA GEMM against the avg-pooled fmap2 (K = C), written once -- no pooling
//     pass over the O(HW^2) volume;
//   * the backward needs no dense dC / dC^T either: with dL_l the accumulated fp32 gradient
//     of level l (the lookup backward adds each iteration's window gradients into it),
//         dF1 = alpha * sum_l dL_l . pool_l(f2)             (GEMM, K = HW_l, accumulated)
//         dF2 = alpha * sum_l unpool_l(dL_l^T . f1)         (GEMM with a transposed A
//                                                           operand read straight from dL_l,
//                                                           the adjoint pool fused in the
//                                                           epilogue)
//   * every GEMM reads fp32 or bf16 operands and converts while staging to LDS; in split
//     mode an fp32 operand is x = hi + lo (two bf16) and the product takes three bf16 MFMAs
//     (hi.hi + hi.lo + lo.hi): fp32-faithful correlation for non-AMP runs (the reference
//     keeps the volume in fp32, core/raft.py:102-103) at 3x bf16 cost instead of the 16x of
//     the fp32 MFMA;
//   * lookup: one wave per query pixel and level loads the (2r+2)^2 integer neighbourhood
//     of its volume row once (one element per lane; the 16-column-blocked levels make it 1-2
//     contiguous runs), stages it in LDS and blends the (2r+1)^2 taps from there, the next
//     level's loads in flight meanwhile.  (A variant gathering all levels in one round trip
//     as 16-byte chunks at lower occupancy measured 15-20% slower.)
//   * lookup backward, deferred: the pyramid backward writes each query's level-gradient row
//     once, accumulated in LDS over all the step's lookups (one block per row, wave l <->
//     level l, replaying the lookups in order: no atomics, deterministic), as bf16 for the
//     AMP volume -- instead of T read-modify-write passes over a zeroed fp32 buffer.  The
//     per-lookup transpose kernel remains for rows too long for LDS.
#include "common.h"

#include <cstdlib>

namespace raft_amd {


// element offset of level pixel (y, x) within a volume row
__device__ __forceinline__ int lvl_off(int y, int x, int Hl, int Wl, int blk) {
  return blk ? ((((x >> 4) * Hl + y) << 4) | (x & 15)) : y * Wl + x;
}



namespace {

constexpr int GBM = 128, GBN = 128, GBK = 32;
constexpr int KP = GBK + 8;     // [m][k] LDS pitch (bf16): 80-byte rows
constexpr int TP = GBM + 32;    // [k][m] LDS pitch for a transposed A operand

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(reinterpret_cast<uintptr_t>(p) & 0xffffffffu));
}

__device__ __forceinline__ __bf16 bf_hi(float x) { return static_cast<__bf16>(x); }
__device__ __forceinline__ __bf16 bf_lo(float x) { return static_cast<__bf16>(x - static_cast<float>(static_cast<__bf16>(x))); }

// 8 consecutive elements (k or m) of an operand row -> hi / lo bf16 (lo = 0 unless split)
__device__ __forceinline__ void load8(const void* base, long off, bool f32, bool ok, bf16x8& hi, bf16x8& lo) {
  if (!ok) {
    hi = bf16x8{};
    lo = bf16x8{};
    return;
  }
  if (f32) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + off);
    const f32x4 b = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + off + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hi[i] = bf_hi(a[i]);
      lo[i] = bf_lo(a[i]);
      hi[4 + i] = bf_hi(b[i]);
      lo[4 + i] = bf_lo(b[i]);
    }
  } else {
    hi = *reinterpret_cast<const bf16x8*>(static_cast<const __bf16*>(base) + off);
    lo = bf16x8{};
  }
}

template <bool SPLIT, bool ATRANS>
__global__ __launch_bounds__(256) void corr_gemm_kernel(const CorrGemmArgs g) {
  // LDS: A (hi[, lo]) then B (hi[, lo])
  constexpr int ASZ = ATRANS ? GBK * TP : GBM * KP;
  constexpr int BSZ = GBN * KP;
  __shared__ __attribute__((aligned(16))) __bf16 smem[(SPLIT ? 2 : 1) * (ASZ + BSZ)];
  __bf16* sAh = smem;
  __bf16* sAl = smem + ASZ;                              // used when SPLIT
  __bf16* sBh = smem + (SPLIT ? 2 : 1) * ASZ;
  __bf16* sBl = sBh + BSZ;

  const int tilesM = (g.M + GBM - 1) / GBM, tilesN = (g.N + GBN - 1) / GBN;
  const int per_b = tilesM * tilesN;
  const int wg = xcd_remap(blockIdx.x, per_b * g.batch);
  const int b = wg / per_b, t = wg - b * per_b;
  const int m0 = (t / tilesN) * GBM, n0 = (t - (t / tilesN) * tilesN) * GBN;
  const void* A = static_cast<const char*>(g.A) + b * g.sA * (g.a_f32 ? 4 : 2);
  const void* B = static_cast<const char*>(g.B) + b * g.sB * (g.b_f32 ? 4 : 2);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // staging: 512 chunks of 8 elements per operand per K step -> 2 per thread
  bf16x8 rah[2], ral[2], rbh[2], rbl[2];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      if (ATRANS) {  // k row (32) x 16 chunks of 8 m
        const int kr = c >> 4, mc = (c & 15) * 8;
        const bool ok = k0 + kr < g.K && m0 + mc < g.M;
        load8(A, (long)(k0 + kr) * g.lda + m0 + mc, g.a_f32, ok, rah[i], ral[i]);
      } else {  // m row (128) x 4 chunks of 8 k
        const int mr = c >> 2, kc = (c & 3) * 8;
        const bool ok = m0 + mr < g.M && k0 + kc < g.K;
        load8(A, (long)(m0 + mr) * g.lda + k0 + kc, g.a_f32, ok, rah[i], ral[i]);
      }
      const int nr = c >> 2, kc = (c & 3) * 8;
      const bool okb = n0 + nr < g.N && k0 + kc < g.K;
      load8(B, (long)(n0 + nr) * g.ldb + k0 + kc, g.b_f32, okb, rbh[i], rbl[i]);
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int ao = ATRANS ? (c >> 4) * TP + (c & 15) * 8 : (c >> 2) * KP + (c & 3) * 8;
      *reinterpret_cast<bf16x8*>(sAh + ao) = rah[i];
      if (SPLIT) *reinterpret_cast<bf16x8*>(sAl + ao) = ral[i];
      const int bo = (c >> 2) * KP + (c & 3) * 8;
      *reinterpret_cast<bf16x8*>(sBh + bo) = rbh[i];
      if (SPLIT) *reinterpret_cast<bf16x8*>(sBl + bo) = rbl[i];
    }
  };

  const int fr = lane & 31, fk = (lane >> 5) * 8;
  const int hh = lane >> 5, gi = (lane >> 4) & 1, q = (lane & 15) >> 2, pq = lane & 3;
  auto afrag = [&](const __bf16* s, int i, int ks) __attribute__((always_inline)) {
    if (ATRANS) {
      const int col = wm * 64 + i * 32 + gi * 16 + 4 * pq;
      const int r0 = ks * 16 + hh * 8 + q;
      const s16x4 lo = tr_read(s + r0 * TP + col);
      const s16x4 hi = tr_read(s + (r0 + 4) * TP + col);
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
    return *reinterpret_cast<const bf16x8*>(s + (wm * 64 + i * 32 + fr) * KP + ks * 16 + fk);
  };

  load(0);
  for (int k0 = 0; k0 < g.K; k0 += GBK) {
    store();
    __syncthreads();
    if (k0 + GBK < g.K) load(k0 + GBK);
#pragma unroll
    for (int ks = 0; ks < GBK / 16; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = afrag(sAh, i, ks);
        if (SPLIT) al[i] = afrag(sAl, i, ks);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o = (wn * 64 + j * 32 + fr) * KP + ks * 16 + fk;
        bh[j] = *reinterpret_cast<const bf16x8*>(sBh + o);
        if (SPLIT) bl[j] = *reinterpret_cast<const bf16x8*>(sBl + o);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (SPLIT) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }

  // epilogue: C/D map of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + (lane & 31);
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        const float v = g.alpha * acc[i][j][r];
        if (g.epi == 0) {
          if (g.c_bf16)
            static_cast<__bf16*>(g.C)[b * g.sC + (long)m * g.ldc + n] = static_cast<__bf16>(v);
          else
            static_cast<float*>(g.C)[b * g.sC + (long)m * g.ldc + n] = v;
        } else {
          static_cast<float*>(g.C)[b * g.sC + (long)m * g.ldc + n] += v;
        }
      }
    }
}

// ---------------------------------------------------------------------------- volume build v2
// C[b][m][n] = bf16(alpha * sum_k A[b][m][k] * B[b][n][k]): bf16 operands (rows of K), fp32
// accumulation, bf16 output -- the dense correlation volume under AMP (K = C = 256 / 128,
// N = every pyramid level's pixels).  With K this short the kernel is bound by WRITING the
// volume (B * HW * ld bf16: 173 MB at 8 x 368x496, 2.8 GB at 1080p), so it is built around
// the stores:
//   * 128x128 tile, 4 waves as 2x2, each 64x64 = 2x2 v_mfma_f32_32x32x16_bf16 per 16-deep k;
//   * both operand tiles are DMA'd (buffer_load ... lds) into a 2-stage LDS ring in 64-deep
//     K steps; 128-B rows with the 16-B chunk index XOR-swizzled by (row >> 1) & 7 through
//     the SOURCE address (the lane-linear DMA image stays contiguous, and each 16-lane group
//     of a fragment ds_read_b128 hits 16 distinct bank slots); rows past M / N load zeros;
//   * the epilogue stages the bf16 tile in LDS and writes 16-byte row-contiguous chunks
//     (one wave instruction = 4 rows x 256 B), not 2-byte scattered stores;
//   * 64 KB of LDS per workgroup: two per CU, so one's stores overlap the other's MFMAs.
constexpr int VBM = 128, VBN = 128, VBK = 64;
constexpr int VSTAGE = (VBM + VBN) * VBK;  // bf16 elements per ring stage
constexpr int VCP = VBN + 8;               // epilogue tile pitch (bf16)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t vrsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
typedef __attribute__((address_space(3))) void vlds_void;
typedef __attribute__((address_space(3))) bf16x8 vlds_bf16x8;
__device__ __forceinline__ void vbload16(__amdgpu_buffer_rsrc_t r, const __bf16* lds_wave_base, unsigned voff,
                                         unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (vlds_void*)(reinterpret_cast<uintptr_t>(lds_wave_base) & 0xffffffffu), 16, voff, soff, 0, 0);
}
constexpr unsigned kVOOB = 0x80000000u;

__global__ __launch_bounds__(256, 2) void corr_volume_bf16_kernel(const CorrGemmArgs g) {
  __shared__ __attribute__((aligned(1024))) __bf16 smem[2 * VSTAGE];
  const int tilesM = (g.M + VBM - 1) / VBM, tilesN = (g.N + VBN - 1) / VBN;
  const int per_b = tilesM * tilesN;
  const int wg = xcd_remap(blockIdx.x, per_b * g.batch);
  const int b = wg / per_b, t = wg - b * per_b;
  // grouped tile order: runs of GM row tiles sweep the column tiles together, so the ~64
  // workgroups an XCD runs at once share a few A and B tiles in its L2 instead of re-streaming
  // all of B once per row tile.  Measured (profiles/r3_bench_corr_grouped.log, vs row-major):
  // GM = 8 while one image's B fits 8 MB (train 83.9 -> 80.0 us, Sintel 61.9 -> 56.8 us); at
  // 1080p (B = 22 MB, 2.8 GB of stores) GM = 4 (1272 -> 1194 us; GM = 8 / 16 lose there, the
  // store stream spreads over too many rows).  kernel_abi.h corr_group_rows.
  const int GM = corr_group_rows(g.N, g.K, g.cfg);
  const int grp = t / (GM * tilesN), first = grp * GM, gsz = min(tilesM - first, GM);
  const int r = t - grp * GM * tilesN;
  const int m0 = (first + r % gsz) * VBM, n0 = (r / gsz) * VBN;
  const __bf16* A = static_cast<const __bf16*>(g.A) + (long)b * g.sA;
  const __bf16* B = static_cast<const __bf16*>(g.B) + (long)b * g.sB;
  const __amdgpu_buffer_rsrc_t ra = vrsrc(A, (unsigned)((long)g.M * g.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = vrsrc(B, (unsigned)((long)g.N * g.ldb * 2));

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // DMA: wave-instruction q (of 16 per operand) fills tile rows 8q .. 8q+7; lane -> row
  // 8q + lane/8, LDS chunk slot lane%8 <- source chunk slot ^ ((row >> 1) & 7)
  const int lr = lane >> 3, lc = lane & 7;
  unsigned avoff[4], bvoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 8 + lr;
    const int src_chunk = lc ^ ((row >> 1) & 7);
    avoff[i] = m0 + row < g.M ? (unsigned)((long)(m0 + row) * g.lda * 2 + src_chunk * 16) : kVOOB;
    bvoff[i] = n0 + row < g.N ? (unsigned)((long)(n0 + row) * g.ldb * 2 + src_chunk * 16) : kVOOB;
  }
  auto issue = [&](int k0, int stage) __attribute__((always_inline)) {
    const __bf16* sA = smem + stage * VSTAGE;
    const __bf16* sB = sA + VBM * VBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) vbload16(ra, sA + (wave * 4 + i) * 512, avoff[i], (unsigned)k0 * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) vbload16(rb, sB + (wave * 4 + i) * 512, bvoff[i], (unsigned)k0 * 2);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // fragment rows of this lane and their swizzle
  const int fr = lane & 31, fh = lane >> 5;
  int arow[2], brow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    arow[i] = wm * 64 + i * 32 + fr;
    brow[i] = wn * 64 + i * 32 + fr;
  }
  const unsigned lds0 = (unsigned)(reinterpret_cast<uintptr_t>(smem) & 0xffffffffu);
  auto frag = [&](unsigned base, int row, int s) __attribute__((always_inline)) {
    const int chunk = (2 * s + fh) ^ ((row >> 1) & 7);
    return *(const vlds_bf16x8*)(uintptr_t)(base + (unsigned)(row * VBK * 2 + chunk * 16));
  };

  const int nk = (g.K + VBK - 1) / VBK;
  issue(0, 0);
  if (nk > 1) issue(VBK, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this stage landed, next in flight
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned sa = lds0 + (unsigned)((kt & 1) * VSTAGE * 2), sb = sa + VBM * VBK * 2;
#pragma unroll
    for (int s = 0; s < VBK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = frag(sa, arow[i], s);
        bfr[i] = frag(sb, brow[i], s);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading this stage
    if (kt + 2 < nk) issue((kt + 2) * VBK, kt & 1);
  }

  // ---- epilogue: bf16 tile through LDS, 16-byte row-contiguous stores
  __bf16* ct = smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        const int col = wn * 64 + j * 32 + fr;
        ct[row * VCP + col] = static_cast<__bf16>(g.alpha * acc[i][j][r]);
      }
  __syncthreads();
  __bf16* C = static_cast<__bf16*>(g.C) + (long)b * g.sC;
#pragma unroll
  for (int i = 0; i < (VBM * VBN / 8) / 256; ++i) {
    const int id = tid + 256 * i;
    const int row = id >> 4, c8 = (id & 15) * 8;
    const int m = m0 + row, n = n0 + c8;
    if (m >= g.M || n >= g.N) continue;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + row * VCP + c8);
    __bf16* dst = C + (long)m * g.ldc + n;
    if (n + 8 <= g.N) {
      *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n + e < g.N) dst[e] = v[e];
    }
  }
}

// v3 (cfg 6 / 7 / 8; automatic at 1080p-sized volumes): the v2 tile with (a) BK-deep K steps,
// BK = 32 halving the LDS ring (2 x 16 KB) so that, with the epilogue tile aliased on it, four
// workgroups share a CU (the stores of some overlap the MFMAs of the others; v2 runs two, and
// its store phase and MFMA phase barely overlap: 1.30 ms vs a 0.55 ms write floor + 0.28 ms of
// MFMA at 1080p), and (b) the MFMA operands swapped (C^T blocks: a lane holds 4 consecutive
// columns of one row), so the epilogue writes the LDS tile as 8-byte runs instead of 2-byte
// scattered stores.  Swizzle for BK-deep rows: R = 128 / BK rows share a 256-byte bank line,
// 16-byte chunk slot = chunk ^ ((row / R) & (BK / 8 - 1)).
// NT: the 16-byte output stores carry the nontemporal hint (streamed past the caches; cfg 11)
template <int BK, int OCC, bool NT = false>
__global__ __launch_bounds__(256, OCC) void corr_volume_v3_kernel(const CorrGemmArgs g) {
  constexpr int CH = BK / 8, R = 128 / BK, RPI = 512 / BK;  // chunks / row, rows / bank line, rows / DMA instr
  constexpr int STAGE = (VBM + VBN) * BK;                      // bf16 elements
  constexpr int NI = VBM / RPI / 4;                            // DMA instructions per wave per operand
  constexpr int LDS = 2 * STAGE > VBM * VCP ? 2 * STAGE : VBM * VCP;
  static_assert(NI >= 1 && (CH & (CH - 1)) == 0, "tile");
  __shared__ __attribute__((aligned(1024))) __bf16 smem[LDS];
  const int tilesM = (g.M + VBM - 1) / VBM, tilesN = (g.N + VBN - 1) / VBN;
  const int per_b = tilesM * tilesN;
  const int wg = xcd_remap(blockIdx.x, per_b * g.batch);
  const int b = wg / per_b, t = wg - b * per_b;
  const int GM = corr_group_rows(g.N, g.K, g.cfg);
  const int grp = t / (GM * tilesN), first = grp * GM, gsz = min(tilesM - first, GM);
  const int r = t - grp * GM * tilesN;
  const int m0 = (first + r % gsz) * VBM, n0 = (r / gsz) * VBN;
  const __bf16* A = static_cast<const __bf16*>(g.A) + (long)b * g.sA;
  const __bf16* B = static_cast<const __bf16*>(g.B) + (long)b * g.sB;
  const __amdgpu_buffer_rsrc_t ra = vrsrc(A, (unsigned)((long)g.M * g.lda * 2));
  const __amdgpu_buffer_rsrc_t rb = vrsrc(B, (unsigned)((long)g.N * g.ldb * 2));

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane / CH, lc = lane % CH;
  unsigned avoff[NI], bvoff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int row = (wave * NI + i) * RPI + lr;
    const int src_chunk = lc ^ ((row / R) & (CH - 1));
    avoff[i] = m0 + row < g.M ? (unsigned)((long)(m0 + row) * g.lda * 2 + src_chunk * 16) : kVOOB;
    bvoff[i] = n0 + row < g.N ? (unsigned)((long)(n0 + row) * g.ldb * 2 + src_chunk * 16) : kVOOB;
  }
  auto issue = [&](int k0, int stage) __attribute__((always_inline)) {
    const __bf16* sA = smem + stage * STAGE;
    const __bf16* sB = sA + VBM * BK;
#pragma unroll
    for (int i = 0; i < NI; ++i) vbload16(ra, sA + (wave * NI + i) * 512, avoff[i], (unsigned)k0 * 2);
#pragma unroll
    for (int i = 0; i < NI; ++i) vbload16(rb, sB + (wave * NI + i) * 512, bvoff[i], (unsigned)k0 * 2);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const int fr = lane & 31, fh = lane >> 5;
  int arow[2], brow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    arow[i] = wm * 64 + i * 32 + fr;
    brow[i] = wn * 64 + i * 32 + fr;
  }
  const unsigned lds0 = (unsigned)(reinterpret_cast<uintptr_t>(smem) & 0xffffffffu);
  auto frag = [&](unsigned base, int row, int s) __attribute__((always_inline)) {
    const int chunk = (2 * s + fh) ^ ((row / R) & (CH - 1));
    return *(const vlds_bf16x8*)(uintptr_t)(base + (unsigned)(row * BK * 2 + chunk * 16));
  };
  constexpr int G = 2 * NI;  // DMA instructions per wave per stage
  const int nk = (g.K + BK - 1) / BK;
  issue(0, 0);
  if (nk > 1) issue(BK, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned sa = lds0 + (unsigned)((kt & 1) * STAGE * 2), sb = sa + VBM * BK * 2;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = frag(sa, arow[i], s);
        bfr[i] = frag(sb, brow[i], s);
      }
      // swapped operands: block (i, j) holds C^T, lane = column m, registers = 4-runs of n
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue((kt + 2) * BK, kt & 1);
  }

  // ---- epilogue: 8-byte runs into the LDS tile (aliasing the drained ring), 16-byte stores
  __bf16* ct = smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int row = wm * 64 + i * 32 + fr;
        const int col = wn * 64 + j * 32 + 8 * q4 + 4 * fh;
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = static_cast<__bf16>(g.alpha * acc[i][j][4 * q4 + e]);
        *reinterpret_cast<bf16x4*>(ct + row * VCP + col) = v;
      }
  __syncthreads();
  __bf16* C = static_cast<__bf16*>(g.C) + (long)b * g.sC;
#pragma unroll
  for (int i = 0; i < (VBM * VBN / 8) / 256; ++i) {
    const int id = tid + 256 * i;
    const int row = id >> 4, c8 = (id & 15) * 8;
    const int m = m0 + row, n = n0 + c8;
    if (m >= g.M || n >= g.N) continue;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + row * VCP + c8);
    __bf16* dst = C + (long)m * g.ldc + n;
    if (n + 8 <= g.N) {
      if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(dst));
      else *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n + e < g.N) dst[e] = v[e];
    }
  }
}

// ---------------------------------------------------------------------------- pyramid backward
// The two GEMMs of the AMP pyramid backward, straight from the bf16 level gradients dL
// (B x HW x ld, every level's columns side by side; the reference differentiates through
// its fp32 matmul + avg_pool, core/corr.py:53-60):
//     dF1 = alpha * dL . f2cat        (M = HW,  N = C, K = ld; A rows K-contiguous)
//     G   = alpha * dL^T . f1         (M = ld,  N = C, K = HW; A read TRANSPOSED from dL)
// dL is 180 MB at config #2 and K is long (2.9-3.9k), so both are dL-streaming GEMMs: the
// kernel is built to read dL once at DMA speed and keep the MFMAs fed.
//   * 128x128 tiles, 4 waves of 64x64, 32-deep K steps in a 3-stage LDS ring filled by
//     buffer_load ... lds (two steps of DMA lead; one barrier per step), 48 KB per workgroup;
//     the two N tiles of an M tile are adjacent in the XCD-aware order, so the second reads its
//     dL tile from L2;
//   * non-transposed operands: 64-byte rows, 16-byte chunk slot = chunk ^ ((row >> 2) & 3)
//     through the SOURCE address (conflict-free ds_read_b128 fragments, as corr_volume_v3);
//   * transposed A (G): the DMA copies dL rows (fixed query pixel p, 128 level columns) as
//     [k = p][m] 256-byte LDS rows, chunk slot = chunk ^ ((row & 3) << 2); the MFMA A fragment
//     (8 consecutive k of one m per lane) is two ds_read_b64_tr_b16 -- the four rows a 16-lane
//     group touches land on four disjoint 64-byte bank groups;
//   * the K tail (K % 32) and the M / N edges are zero-filled by the DMA's range check (the
//     per-chunk offset is set past the buffer), no masking in the MFMA loop.
// Replaces hipBLASLt (torch.baddbmm) and the register-staged generic GEMM on this path.
namespace cbw {
constexpr int BM = 128, BN = 128, BK = 32, NS = 3;
constexpr int TILE = 128 * BK;             // bf16 elements of one operand tile
constexpr int STAGE = 2 * TILE;            // A + B
}  // namespace cbw

template <bool AT>
__device__ __forceinline__ void corr_bwd_tile(const CorrGemmArgs& g, __bf16* smem, int bid) {
  using namespace cbw;
  const int tilesM = (g.M + BM - 1) / BM, tilesN = (g.N + BN - 1) / BN;
  const int per_b = tilesM * tilesN;
  const int wg = xcd_remap(bid, per_b * g.batch);
  const int b = wg / per_b, t = wg - b * per_b;
  const int m0 = (t / tilesN) * BM, n0 = (t - (t / tilesN) * tilesN) * BN;
  const __bf16* A = static_cast<const __bf16*>(g.A) + (long)b * g.sA;
  const __bf16* B = static_cast<const __bf16*>(g.B) + (long)b * g.sB;
  const __amdgpu_buffer_rsrc_t ra =
      vrsrc(A, (unsigned)((AT ? (long)g.K * g.lda : (long)g.M * g.lda) * 2));
  const __amdgpu_buffer_rsrc_t rb = vrsrc(B, (unsigned)((long)g.N * g.ldb * 2));

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // DMA pieces: 8 instructions (1 KB) per operand tile and stage, 2 per wave
  //   rows-of-K layout (A non-trans, B): instr j -> rows 16j .. 16j+15, lane -> row 16j + lane/4
  //   transposed A: instr j -> k rows 4j .. 4j+3, lane -> k row 4j + lane/16, m chunk slot lane%16
  unsigned abase[2], bbase[2];
  int akc[2], bkc[2];  // k (element) offset of this lane's chunk within a K step (non-trans)
  int akr[2];          // transposed A: k row of this lane within a K step
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = wave * 2 + i;
    {
      const int row = 16 * j + (lane >> 2), slot = lane & 3;
      const int sc = slot ^ ((row >> 2) & 3);
      bkc[i] = sc * 8;
      bbase[i] = n0 + row < g.N ? (unsigned)((long)(n0 + row) * g.ldb * 2 + sc * 16) : kVOOB;
      if constexpr (!AT) {
        akc[i] = sc * 8;
        abase[i] = m0 + row < g.M ? (unsigned)((long)(m0 + row) * g.lda * 2 + sc * 16) : kVOOB;
      }
    }
    if constexpr (AT) {
      const int row = 4 * j + (lane >> 4), slot = lane & 15;
      const int sc = slot ^ ((row & 3) << 2);
      akr[i] = row;
      abase[i] = m0 + sc * 8 < g.M ? (unsigned)((long)row * g.lda * 2 + (m0 + sc * 8) * 2) : kVOOB;
      akc[i] = 0;
    }
  }
  auto issue = [&](int k0, int stage) __attribute__((always_inline)) {
    const __bf16* sA = smem + stage * STAGE;
    const __bf16* sB = sA + TILE;
    const int kv = g.K - k0;  // valid k of this step (>= 1)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (AT) {
        const unsigned vo = (akr[i] < kv && abase[i] != kVOOB) ? abase[i] : kVOOB;
        vbload16(ra, sA + (wave * 2 + i) * 512, vo, (unsigned)((long)k0 * g.lda * 2));
      } else {
        const unsigned vo = (akc[i] < kv && abase[i] != kVOOB) ? abase[i] : kVOOB;
        vbload16(ra, sA + (wave * 2 + i) * 512, vo, (unsigned)k0 * 2);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned vo = (bkc[i] < kv && bbase[i] != kVOOB) ? bbase[i] : kVOOB;
      vbload16(rb, sB + (wave * 2 + i) * 512, vo, (unsigned)k0 * 2);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const int fr = lane & 31, fh = lane >> 5;
  const unsigned lds0 = (unsigned)(reinterpret_cast<uintptr_t>(smem) & 0xffffffffu);
  // rows-of-K fragment (row r, 16-deep sub-step s): 8 consecutive k of row r
  auto frag = [&](unsigned base, int row, int s) __attribute__((always_inline)) {
    const int chunk = (2 * s + fh) ^ ((row >> 2) & 3);
    return *(const vlds_bf16x8*)(uintptr_t)(base + (unsigned)(row * BK * 2 + chunk * 16));
  };
  // transposed A fragment of 32-row block i, sub-step s from the [k][m] tile
  const int gi = (lane >> 4) & 1, q4 = (lane & 15) >> 2, pq = lane & 3;
  auto tfrag = [&](unsigned base, int i, int s) __attribute__((always_inline)) {
    const int chunk = (wm * 8 + i * 4 + gi * 2 + (pq >> 1)) ^ (q4 << 2);
    const unsigned off = (unsigned)(chunk * 16 + (pq & 1) * 8);
    const int r0 = s * 16 + fh * 8 + q4;
    const s16x4 lo = tr_read(reinterpret_cast<const __bf16*>((uintptr_t)(base + (unsigned)(r0 * 256) + off)));
    const s16x4 hi = tr_read(reinterpret_cast<const __bf16*>((uintptr_t)(base + (unsigned)((r0 + 4) * 256) + off)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  const int nk = (g.K + BK - 1) / BK;
  issue(0, 0);
  if (nk > 1) issue(BK, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // step kt landed, kt+1 in flight
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of step kt landed; step kt-1's stage is free
    if (kt + 2 < nk) issue((kt + 2) * BK, (kt + 2) % NS);
    const unsigned sa = lds0 + (unsigned)((kt % NS) * STAGE * 2), sb = sa + TILE * 2;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (AT) af[i] = tfrag(sa, i, s);
        else af[i] = frag(sa, wm * 64 + i * 32 + fr, s);
        bfr[i] = frag(sb, wn * 64 + i * 32 + fr, s);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: lane = column n (32 consecutive per half-wave), registers = rows
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + fr;
    if (n >= g.N) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        if (m >= g.M) continue;
        const float v = g.alpha * acc[i][j][r];
        if (g.c_bf16) static_cast<__bf16*>(g.C)[(long)b * g.sC + (long)m * g.ldc + n] = static_cast<__bf16>(v);
        else static_cast<float*>(g.C)[(long)b * g.sC + (long)m * g.ldc + n] = v;
      }
  }
}

__host__ __device__ inline int corr_bwd_tiles(const CorrGemmArgs& g) {
  return ((g.M + cbw::BM - 1) / cbw::BM) * ((g.N + cbw::BN - 1) / cbw::BN) * g.batch;
}

template <bool AT>
__global__ __launch_bounds__(256, 2) void corr_bwd_kernel(const CorrGemmArgs g) {
  __shared__ __attribute__((aligned(1024))) __bf16 smem[cbw::NS * cbw::STAGE];
  corr_bwd_tile<AT>(g, smem, blockIdx.x);
}

// Both GEMMs of the pyramid backward in ONE grid: workgroups [0, n1) run dF1 (the longer K,
// first), [n1, n1 + tiles(G)) run G.  Alone, each under-fills the chip (368 / 496 workgroups of
// 4 waves at config #2, each latency-bound on its DMA ring); together they keep ~3 workgroups
// per CU and share dL's lines in L2 / the Infinity Cache.  n1 is padded to a multiple of 8 so
// blockIdx - n1 keeps the XCD of blockIdx (xcd_remap works on the local index).
__global__ __launch_bounds__(256, 2) void corr_bwd_pair_kernel(const CorrGemmArgs g1, const CorrGemmArgs gt, int n1) {
  __shared__ __attribute__((aligned(1024))) __bf16 smem[cbw::NS * cbw::STAGE];
  const int bid = blockIdx.x;
  if (bid < n1) {
    if (bid < corr_bwd_tiles(g1)) corr_bwd_tile<false>(g1, smem, bid);
  } else {
    corr_bwd_tile<true>(gt, smem, bid - n1);
  }
}

__global__ __launch_bounds__(256) void pyramid_unpool_kernel(const UnpoolArgs u) {
  const long total = (long)u.B * u.H * u.W * u.C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % u.C);
    const long pix = i / u.C;
    const int x = (int)(pix % u.W);
    const long t = pix / u.W;
    const int y = (int)(t % u.H);
    const int b = (int)(t / u.H);
    const float* G = u.G + b * u.sG;
    float v = 0.f, s = 1.f;
    for (int l = 0; l < u.nseg; ++l, s *= 0.25f) {
      const int yl = y >> l, xl = x >> l;
      if (yl < u.h[l] && xl < u.w[l]) {
        const int r = u.blk ? ((((xl >> 4) * u.h[l] + yl) << 4) | (xl & 15)) : yl * u.w[l] + xl;
        v += s * G[(long)(u.off[l] + r) * u.C + c];
      }
    }
    u.out[i] = v;
  }
}

// ---------------------------------------------------------------------------- pyramid operand
// Level-l pixel (y, x) of 4 consecutive channels c..c+3 (C % 4 == 0): the 2^l x 2^l source block
// averaged in F.avg_pool2d's order (each level sums its 4 children from 0 then divides by 4),
// so the result is bitwise equal to the pooled tensors.  VEC: channel-contiguous source, one
// 16-byte (fp32) / 8-byte (bf16) load per source pixel.  The level-2/3 loops stay rolled, so a
// level-3 column does not keep 64 source vectors live.
__device__ __forceinline__ bool pyr_vec(const PyrOperandArgs& a) {
  return a.sC == 1 && ((a.sB | a.sH | a.sW) & 3) == 0 && (reinterpret_cast<uintptr_t>(a.src) & 15) == 0;
}

template <bool VEC>
__device__ __forceinline__ f32x4 pyr_src4(const PyrOperandArgs& a, int b, int c, int y, int x) {
  const long i = b * a.sB + c * a.sC + y * a.sH + x * a.sW;
  if (VEC) {
    if (a.src_bf16) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      const bf16x4 v = *reinterpret_cast<const bf16x4*>(static_cast<const __bf16*>(a.src) + i);
      return f32x4{static_cast<float>(v[0]), static_cast<float>(v[1]), static_cast<float>(v[2]),
                   static_cast<float>(v[3])};
    }
    return *reinterpret_cast<const f32x4*>(static_cast<const float*>(a.src) + i);
  }
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    v[e] = a.src_bf16 ? static_cast<float>(static_cast<const __bf16*>(a.src)[i + e * a.sC])
                      : static_cast<const float*>(a.src)[i + e * a.sC];
  return v;
}

template <bool VEC>
__device__ __forceinline__ f32x4 pyr_pool1(const PyrOperandArgs& a, int b, int c, int y, int x) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  s += pyr_src4<VEC>(a, b, c, 2 * y, 2 * x);
  s += pyr_src4<VEC>(a, b, c, 2 * y, 2 * x + 1);
  s += pyr_src4<VEC>(a, b, c, 2 * y + 1, 2 * x);
  s += pyr_src4<VEC>(a, b, c, 2 * y + 1, 2 * x + 1);
  return s / 4.f;
}

template <bool VEC>
__device__ f32x4 pyr_value4(const PyrOperandArgs& a, int l, int b, int c, int y, int x) {
  if (l == 0) return pyr_src4<VEC>(a, b, c, y, x);
  if (l == 1) return pyr_pool1<VEC>(a, b, c, y, x);
  if (l == 2) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k = 0; k < 4; ++k) s += pyr_pool1<VEC>(a, b, c, 2 * y + (k >> 1), 2 * x + (k & 1));
    return s / 4.f;
  }
  f32x4 s3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int k3 = 0; k3 < 4; ++k3) {
    f32x4 s2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k2 = 0; k2 < 4; ++k2)
      s2 += pyr_pool1<VEC>(a, b, c, 4 * y + 2 * (k3 >> 1) + (k2 >> 1), 4 * x + 2 * (k3 & 1) + (k2 & 1));
    s3 += s2 / 4.f;
  }
  return s3 / 4.f;
}

// column q of the operand -> (level, y, x); false for padding columns (32-bit: the launcher
// checks ld)
__device__ __forceinline__ bool pyr_column(const PyrOperandArgs& a, int q, int& l, int& y, int& x) {
  for (l = a.nseg - 1; l > 0 && q < a.off[l]; --l) {
  }
  if (q < a.off[l]) return false;
  const int j = q - a.off[l];
  const int Hl = a.h[l], Wl = a.w[l];
  if (a.blk) {
    const int blk = j / (16 * Hl), rem = j - blk * 16 * Hl;
    y = rem >> 4;
    x = blk * 16 + (rem & 15);
    return y < Hl && x < Wl;
  }
  if (j >= Hl * Wl) return false;
  y = j / Wl;
  x = j - y * Wl;
  return true;
}

// (B, C, ld) layout: a block computes a 64-column x 64-channel tile with channel-contiguous
// reads (4 channels per thread, one vector load per source pixel) and writes it transposed
// through LDS as 16-byte column-contiguous stores (4 channel rows x 256 B per wave store).
__global__ __launch_bounds__(256) void pyramid_operand_t_kernel(const PyrOperandArgs a) {
  __shared__ float tile[64][65];
  const int tid = threadIdx.x;
  const int ld = (int)a.ld;
  const int q0 = blockIdx.x * 64;
  const int c0 = blockIdx.y * 64, b = blockIdx.z;
  const int c4 = (tid & 15) * 4;
  const bool vec = pyr_vec(a);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int qq = (tid >> 4) + 16 * k;
    const int q = q0 + qq;
    int l, y, x;
    const bool live = q < ld && c0 + c4 < a.C && pyr_column(a, q, l, y, x);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (live) v = vec ? pyr_value4<true>(a, l, b, c0 + c4, y, x) : pyr_value4<false>(a, l, b, c0 + c4, y, x);
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[c4 + e][qq] = v[e];
  }
  __syncthreads();
  const int qs = (tid & 15) * 4;
  const bool vst = (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(a.out16 ? (void*)a.out16 : (void*)a.out) & 15) == 0;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int cl = (tid >> 4) + 16 * pass, c = c0 + cl;
    if (c >= a.C) break;
    if (a.out16) {
      __bf16* o16 = a.out16 + ((long)b * a.C + c) * ld + q0 + qs;
      if (vst && q0 + qs + 4 <= ld) {
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4*>(o16) = bf16x4{static_cast<__bf16>(tile[cl][qs]), static_cast<__bf16>(tile[cl][qs + 1]),
                                                 static_cast<__bf16>(tile[cl][qs + 2]), static_cast<__bf16>(tile[cl][qs + 3])};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (q0 + qs + j < ld) o16[j] = static_cast<__bf16>(tile[cl][qs + j]);
      }
      continue;
    }
    float* o = a.out + ((long)b * a.C + c) * ld + q0 + qs;
    if (vst && q0 + qs + 4 <= ld) {
      *reinterpret_cast<f32x4*>(o) = f32x4{tile[cl][qs], tile[cl][qs + 1], tile[cl][qs + 2], tile[cl][qs + 3]};
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (q0 + qs + j < ld) o[j] = tile[cl][qs + j];
    }
  }
}

__global__ __launch_bounds__(256) void pyramid_operand_kernel(const PyrOperandArgs a) {
  // (B, ld, C): 4 channels per thread (32-bit indices: the launcher checks B * ld * C)
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int C4 = a.C / 4, ld = (int)a.ld;
  if (i >= a.B * ld * C4) return;
  const int bq = i / C4, c = (i - bq * C4) * 4;
  const int b = bq / ld, q = bq - b * ld;
  int l, y, x;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (pyr_column(a, q, l, y, x))
    v = pyr_vec(a) ? pyr_value4<true>(a, l, b, c, y, x) : pyr_value4<false>(a, l, b, c, y, x);
  if (a.out16) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<bf16x4*>(a.out16 + (long)i * 4) =
        bf16x4{static_cast<__bf16>(v[0]), static_cast<__bf16>(v[1]), static_cast<__bf16>(v[2]), static_cast<__bf16>(v[3])};
    return;
  }
  *reinterpret_cast<f32x4*>(a.out + (long)i * 4) = v;
}

__device__ __forceinline__ float safe_floor(float v) {
  // keep far-out-of-range / non-finite coordinates from overflowing int math
  v = fminf(fmaxf(v, -1.0e6f), 1.0e6f);
  return floorf(v);
}

// ---------------------------------------------------------------------------- lookup
// this wave's LDS writes are visible to its other lanes: the LDS operations of one wave
// execute in order, so only the compiler must not move LDS accesses across this point
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave per query pixel, looping over the levels; 4 waves per block.  LDS per wave:
// the (2r+2)^2 neighbourhood (<= 14 x 14 for r <= 6) as fp32.
constexpr int NBMAX = 14 * 14;
constexpr int NBPITCHED = 10 * 25;  // >= NBMAX and the pitched r = 4 / 3 layouts (10 x 25, 8 x 23)

// Optionally also packs the step's flow operand (the pack_flow op, folded in: the wave
// already holds the query's coordinates): flow8[pix] = bf16 [u, v, 0 x 6] and
// motion[pix * smo + {0, 1}] = bf16 [u, v], with (u, v) = coords - (x, y).
struct FlowPack {
  __bf16* flow8;
  __bf16* motion;
  long smo;
  int f16;      // 16-bit storage is fp16 (fp16 AMP)
  int split_m;  // > 0: split-bf16 planes (fp32 mode): flow8 rows [hi | lo | hi] of 8, motion lo plane
                // split_m channels after its hi plane (ops/update_split.py)
};

// Output rows of the lookup: out_ch channels of OutT, or (SplitOut) split-bf16 planes [hi | lo |
// hi] of out_ch channels each -- the fp32 training / inference step's GEMM operand, written
// straight from the fp32 blend (no fp32 row round trip)
struct SplitOut {};
template <typename OutT>
struct OutRow {
  OutT* o;
  int G;
  static constexpr int kPlanes = 1;
  __device__ __forceinline__ void put(int ch, float v) const { o[ch] = from_f32<OutT>(v); }
};
template <>
struct OutRow<SplitOut> {
  __bf16* o;
  int G;
  static constexpr int kPlanes = 3;
  __device__ __forceinline__ void put(int ch, float v) const {
    const __bf16 hi = static_cast<__bf16>(v);
    o[ch] = hi;
    o[G + ch] = static_cast<__bf16>(v - static_cast<float>(hi));
    o[2 * G + ch] = hi;
  }
};

// RC > 0: the radius as a compile-time constant (RAFT's r = 4): the window index math divides by
// constants (a runtime 32-bit division is ~30 VALU per use)
// ALL: every level's neighbourhood loads issued up front (4 levels x 2 loads per lane for r = 4)
// instead of one level ahead, so a wave waits for one load round trip rather than one per level
template <typename OutT, int RC = 0, bool ALL = false>
__global__ __launch_bounds__(256) void lookup_fwd_kernel(PyrDesc pyr, const float* __restrict__ coords,
                                                         void* __restrict__ out_, int B, int H, int W, int r_arg,
                                                         int out_ch, const FlowPack fp) {
  const int r = RC > 0 ? RC : r_arg;
  // neighbourhood rows at a pitch that makes the blend's four reads (x-offset-major window
  // order: lane -> (ix, iy), address iy * np + ix) bank-conflict-free for r = 4 / 3 (an exhaustive
  // search over pitches; the natural pitch nd costs 8 extra LDS cycles per level)
  constexpr int NP = RC == 4 ? 25 : (RC == 3 ? 23 : 0);
  __shared__ float nb[4][NBPITCHED];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = H * W;
  const long pix0 = (long)blockIdx.x * 4 + wave;
  const bool live = pix0 < (long)B * HW;
  const long pix = live ? pix0 : 0;
  const int b = pix / HW, p = pix - (long)b * HW;
  const int rd = 2 * r + 1, nd = rd + 1, win = rd * rd, nn = nd * nd;
  const int np = NP > 0 ? NP : nd;
  const float cx0 = coords[(long)b * 2 * HW + p], cy0 = coords[(long)b * 2 * HW + HW + p];
  const bool finite = isfinite(cx0) && isfinite(cy0);
  if (fp.flow8 && live && lane < 8) {
    const int py = p / W;
    const float u = cx0 - (float)(p - py * W), v = cy0 - (float)py;
    const float fv = lane == 0 ? u : (lane == 1 ? v : 0.f);
    if (fp.split_m > 0) {  // split planes: hi = bf16(f), lo = bf16(f - hi)
      const __bf16 hi = static_cast<__bf16>(fv), lo = static_cast<__bf16>(fv - static_cast<float>(hi));
      fp.flow8[pix * 24 + lane] = hi;
      fp.flow8[pix * 24 + 8 + lane] = lo;
      fp.flow8[pix * 24 + 16 + lane] = hi;
      if (fp.motion && lane < 2) {
        __bf16* m = fp.motion + pix * fp.smo + lane;
        m[0] = hi;
        m[fp.split_m] = lo;
        m[2 * fp.split_m] = hi;
      }
    } else {
      const __bf16 f = st16(fv, fp.f16 != 0);
      fp.flow8[pix * 8 + lane] = f;
      if (fp.motion && lane < 2) fp.motion[pix * fp.smo + lane] = f;
    }
  }
  using Row = OutRow<OutT>;
  using Elem = decltype(Row::o);
  const Row o{static_cast<Elem>(out_) + pix * out_ch * Row::kPlanes, out_ch};
  // software pipeline over the levels: the neighbourhood loads of level l+1 are in flight
  // while level l is blended (the lookup is bound by the load round trips, not by bytes)
  float fx = 0.f, fy = 0.f, nfx = 0.f, nfy = 0.f;
  float v[4];
  auto issue_to = [&](int l, float& fxo, float& fyo, float (&v)[4]) __attribute__((always_inline)) {
    const float s = 1.0f / float(1 << l);
    const float cx = finite ? cx0 * s : 0.f, cy = finite ? cy0 * s : 0.f;
    const float fx0 = safe_floor(cx), fy0 = safe_floor(cy);
    fxo = cx - fx0;
    fyo = cy - fy0;
    const int xb = (int)fx0 - r, yb = (int)fy0 - r;
    const int Hl = pyr.H[l], Wl = pyr.W[l];
    const long rbase = pix * pyr.ld[l];
    const float* row = pyr.ptr[l] + rbase;
    const __bf16* rowb = reinterpret_cast<const __bf16*>(pyr.ptr[l]) + rbase;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = lane + 64 * k;
      const int a = e / nd, c = e - a * nd;  // neighbour (y = yb + a, x = xb + c)
      const int y = yb + a, x = xb + c;
      const bool in = e < nn && live && finite && (unsigned)y < (unsigned)Hl && (unsigned)x < (unsigned)Wl;
      const int off = in ? lvl_off(y, x, Hl, Wl, pyr.blk) : 0;
      v[k] = in ? (pyr.vbf16 ? static_cast<float>(rowb[off]) : row[off]) : 0.f;
    }
  };
  auto issue = [&](int l, float& fxo, float& fyo) __attribute__((always_inline)) { issue_to(l, fxo, fyo, v); };
  if constexpr (ALL) {
    static_assert(RC > 0 && (2 * RC + 2) * (2 * RC + 2) <= 128, "two loads per lane and level");
    float va[4][4], fxa[4], fya[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      fxa[l] = fya[l] = 0.f;
      va[l][0] = va[l][1] = va[l][2] = va[l][3] = 0.f;
      if (l < pyr.levels) issue_to(l, fxa[l], fya[l], va[l]);
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      if (l >= pyr.levels) break;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int e = lane + 64 * k;
        if (e < nn) nb[wave][(e / nd) * np + e % nd] = va[l][k];
      }
      wave_lds_sync();
      if (live)
        for (int ch = lane; ch < win; ch += 64) {
          const int ix = ch / rd, iy = ch - ix * rd;  // x-offset-major window order
          const float* n0 = nb[wave] + iy * np + ix;
          const float val = (1.f - fya[l]) * ((1.f - fxa[l]) * n0[0] + fxa[l] * n0[1]) +
                            fya[l] * ((1.f - fxa[l]) * n0[np] + fxa[l] * n0[np + 1]);
          o.put(l * win + ch, val);
        }
      wave_lds_sync();
    }
    if (live)
      for (int ch = pyr.levels * win + lane; ch < out_ch; ch += 64) o.put(ch, 0.f);
    return;
  }
  // the neighbourhood buffer is private to the wave: its LDS accesses execute in issue order,
  // so a wave-level fence (no workgroup barrier) orders the stores before the blend's reads
  // and those reads before the next level's stores; the 4 waves of a block run decoupled
  issue(0, fx, fy);
  for (int l = 0; l < pyr.levels; ++l) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = lane + 64 * k;
      if (e < nn) nb[wave][(e / nd) * np + e % nd] = v[k];
    }
    wave_lds_sync();
    if (l + 1 < pyr.levels) issue(l + 1, nfx, nfy);
    if (live)
      for (int ch = lane; ch < win; ch += 64) {
        const int ix = ch / rd, iy = ch - ix * rd;  // x-offset-major window order
        const float* n0 = nb[wave] + iy * np + ix;
        const float val =
            (1.f - fy) * ((1.f - fx) * n0[0] + fx * n0[1]) + fy * ((1.f - fx) * n0[np] + fx * n0[np + 1]);
        o.put(l * win + ch, val);
      }
    wave_lds_sync();
    fx = nfx;
    fy = nfy;
  }
  if (live)
    for (int ch = pyr.levels * win + lane; ch < out_ch; ch += 64) o.put(ch, 0.f);
}

// dpyr[l][pix][y][x] += window gradient, transposed bilinear blend; one wave per query.
template <typename GT>
__global__ __launch_bounds__(256) void lookup_bwd_kernel(PyrDesc dpyr, const float* __restrict__ coords,
                                                         const GT* __restrict__ gout, int B, int H, int W, int r,
                                                         int gstride) {
  __shared__ float gs[4][NBMAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HW = H * W;
  const long pix0 = (long)blockIdx.x * 4 + wave;
  const long pix = pix0 < (long)B * HW ? pix0 : 0;
  const int b = pix / HW, p = pix - (long)b * HW;
  const int rd = 2 * r + 1, nd = rd + 1, win = rd * rd;
  const float cx0 = coords[(long)b * 2 * HW + p], cy0 = coords[(long)b * 2 * HW + HW + p];
  // no early exit: the block synchronises per level
  const bool live = pix0 < (long)B * HW && isfinite(cx0) && isfinite(cy0);
  const GT* g = gout + pix * gstride;
  for (int l = 0; l < dpyr.levels; ++l) {
    const float s = 1.0f / float(1 << l);
    const float cx = live ? cx0 * s : 0.f, cy = live ? cy0 * s : 0.f;
    const float fx0 = safe_floor(cx), fy0 = safe_floor(cy);
    const float fx = cx - fx0, fy = cy - fy0;
    const int xb = (int)fx0 - r, yb = (int)fy0 - r;
    const int Hl = dpyr.H[l], Wl = dpyr.W[l];
    // window gradient in LDS as [iy][ix] (transposed from the x-major channel order)
    for (int ch = lane; ch < win; ch += 64) {
      const int ix = ch / rd, iy = ch - ix * rd;
      gs[wave][iy * rd + ix] = live ? to_f32(g[l * win + ch]) : 0.f;
    }
    __syncthreads();
    float* row = dpyr.ptr[l] + pix * dpyr.ld[l];
    for (int e = lane; live && e < nd * nd; e += 64) {
      const int a = e / nd, c = e - a * nd;
      const int y = yb + a, x = xb + c;
      if ((unsigned)y >= (unsigned)Hl || (unsigned)x >= (unsigned)Wl) continue;
      // neighbour (a, c) is corner (0,0) of tap (c, a), (0,1) of (c-1, a), (1,0) of (c, a-1),
      // (1,1) of (c-1, a-1)
      const float* gw = gs[wave];
      float v = 0.f;
      if (a < rd) {
        if (c < rd) v += (1.f - fx) * (1.f - fy) * gw[a * rd + c];
        if (c > 0) v += fx * (1.f - fy) * gw[a * rd + c - 1];
      }
      if (a > 0) {
        if (c < rd) v += (1.f - fx) * fy * gw[(a - 1) * rd + c];
        if (c > 0) v += fx * fy * gw[(a - 1) * rd + c - 1];
      }
      row[lvl_off(y, x, Hl, Wl, dpyr.blk)] += v;
    }
    __syncthreads();
  }
}

// One block per query row, wave l <-> level l: the wave replays the T lookups of the step
// in order, scattering each window gradient (transposed bilinear blend, one neighbour per
// lane) into the row's level-l region in LDS; the block then writes the whole row once
// (padding columns as zeros: no memset of the buffer).  Same per-element fp32 summation
// order as T sequential lookup_bwd launches into a zeroed buffer.
template <typename GT, int RC = 0>
__global__ __launch_bounds__(256) void lookup_grad_rows_kernel(const GradRowsArgs a) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long pix = blockIdx.x;
  const int HW = a.Hq * a.Wq;
  const int b = (int)(pix / HW), p = (int)(pix - (long)b * HW);
  const long ld = a.ld;
  float* row = lds;
  float* gs = lds + ld + wave * 176;  // this wave's window gradient, (2r+1)^2 <= 169
  if (a.accumulate) {
    if (a.out_f32) {
      const float* src = static_cast<const float*>(a.out) + pix * ld;
      for (long i = tid * 4; i < ld; i += 1024) *reinterpret_cast<f32x4*>(row + i) = *reinterpret_cast<const f32x4*>(src + i);
    } else {
      const __bf16* src = static_cast<const __bf16*>(a.out) + pix * ld;
      for (long i = tid; i < ld; i += 256) row[i] = static_cast<float>(src[i]);
    }
  } else {
    for (long i = tid * 4; i < ld; i += 1024) *reinterpret_cast<f32x4*>(row + i) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  const int r = RC > 0 ? RC : a.r, rd = 2 * r + 1, nd = rd + 1, win = rd * rd;
  if (wave < a.levels) {
    const int l = wave, Hl = a.H[l], Wl = a.W[l];
    float* lrow = row + a.off[l];
    const float s = 1.0f / float(1 << l);
    // lookups in chunks of kChunk: lane i fetches lookup t0+i's coordinates and gradient
    // pointer, then every window gradient of the chunk is loaded at once (one memory round
    // trip per chunk, nothing scalar in the replay loop)
    constexpr int kChunk = 16;
    for (int t0 = 0; t0 < a.T; t0 += kChunk) {
      const int nt = min(kChunk, a.T - t0);
      float cxv = 0.f, cyv = 0.f;
      unsigned long long gpv = 0;
      if (lane < nt) {
        const float* cp = a.c[t0 + lane];
        cxv = cp[(long)b * 2 * HW + p];
        cyv = cp[(long)b * 2 * HW + HW + p];
        gpv = reinterpret_cast<unsigned long long>(a.g[t0 + lane]);
      }
      float v[kChunk][3];
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        if (i >= nt) continue;
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)gpv, i);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(gpv >> 32), i);
        const GT* g = reinterpret_cast<const GT*>(((unsigned long long)hi << 32) | lo) + pix * a.gstride + l * win;
#pragma unroll
        for (int k = 0; k < 3; ++k) v[i][k] = lane + 64 * k < win ? to_f32(g[lane + 64 * k]) : 0.f;
      }
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        if (i >= nt) continue;
        const float cx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cxv), i));
        const float cy = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(cyv), i));
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (lane + 64 * k < win) gs[lane + 64 * k] = v[i][k];
        wave_lds_sync();
        if (isfinite(cx) && isfinite(cy)) {
          const float fx0 = safe_floor(cx * s), fy0 = safe_floor(cy * s);
          const float fx = cx * s - fx0, fy = cy * s - fy0;
          const int xb = (int)fx0 - r, yb = (int)fy0 - r;
          for (int e = lane; e < nd * nd; e += 64) {
            const int aa = e / nd, c = e - aa * nd;
            const int y = yb + aa, x = xb + c;
            if ((unsigned)y >= (unsigned)Hl || (unsigned)x >= (unsigned)Wl) continue;
            // neighbour (aa, c) is corner (0,0) of tap (c, aa), (0,1) of (c-1, aa), (1,0) of
            // (c, aa-1), (1,1) of (c-1, aa-1); taps in channel order ix * rd + iy
            float w = 0.f;
            if (aa < rd) {
              if (c < rd) w += (1.f - fx) * (1.f - fy) * gs[c * rd + aa];
              if (c > 0) w += fx * (1.f - fy) * gs[(c - 1) * rd + aa];
            }
            if (aa > 0) {
              if (c < rd) w += (1.f - fx) * fy * gs[c * rd + aa - 1];
              if (c > 0) w += fx * fy * gs[(c - 1) * rd + aa - 1];
            }
            lrow[lvl_off(y, x, Hl, Wl, 1)] += w;
          }
        }
        wave_lds_sync();
      }
    }
  }
  __syncthreads();
  if (a.out_f32) {
    float* dst = static_cast<float*>(a.out) + pix * ld;
    for (long i = tid * 4; i < ld; i += 1024) *reinterpret_cast<f32x4*>(dst + i) = *reinterpret_cast<const f32x4*>(row + i);
  } else {
    __bf16* dst = static_cast<__bf16*>(a.out) + pix * ld;
    for (long i = tid * 8; i < ld; i += 2048) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(row + i), w = *reinterpret_cast<const f32x4*>(row + i + 4);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = static_cast<__bf16>(u[e]);
        o[4 + e] = static_cast<__bf16>(w[e]);
      }
      *reinterpret_cast<bf16x8*>(dst + i) = o;
    }
  }
}

__global__ __launch_bounds__(256) void avgpool2x2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                         long rows, int H, int W, int Ho, int Wo) {
  const long total = rows * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = i % Wo;
    const long t = i / Wo;
    const int y = t % Ho;
    const long rr = t / Ho;
    const float* src = in + rr * H * W + (2 * y) * W + 2 * x;
    out[i] = 0.25f * (src[0] + src[1] + src[W] + src[W + 1]);
  }
}

inline int grid_for(long total) {
  long blocks = (total + 255) / 256;
  return (int)(blocks < (1L << 20) ? blocks : (1L << 20));
}

}  // namespace

static bool corr_bwd_ok(const CorrGemmArgs& g) {
  return !g.split && !g.a_f32 && !g.b_f32 && g.epi == 0 && g.lda % 8 == 0 && g.ldb % 8 == 0 &&
         (g.a_trans ? g.M % 8 == 0 : g.K % 8 == 0) &&
         (g.a_trans ? (long)g.K * g.lda : (long)g.M * g.lda) * 2 < (1L << 31) && (long)g.N * g.ldb * 2 < (1L << 31);
}

hipError_t launch_corr_gemm(const CorrGemmArgs& g, hipStream_t s) {
  if (g.M == 0 || g.N == 0 || g.batch == 0) return hipSuccess;
  // cfg 10: the pyramid-backward kernel (bf16 operands, store epilogue, 32-bit DMA offsets)
  if (g.cfg == 10) {
    if (!corr_bwd_ok(g)) return hipErrorInvalidValue;
    const long tiles = corr_bwd_tiles(g);
    if (g.a_trans) hipLaunchKernelGGL((corr_bwd_kernel<true>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((corr_bwd_kernel<false>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    return hipGetLastError();
  }
  // bf16 x bf16 -> bf16 store (the AMP volume build): the store-oriented v2 kernel, when its
  // 16-byte DMA / store granules and 32-bit buffer offsets fit
  const bool v2 = !g.split && !g.a_trans && !g.a_f32 && !g.b_f32 && g.c_bf16 && g.epi == 0 && g.K % VBK == 0 &&
                  g.lda % 8 == 0 && g.ldb % 8 == 0 && g.ldc % 8 == 0 && g.sC % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(g.C) % 16 == 0 && (long)g.M * g.lda * 2 < (1L << 31) &&
                  (long)g.N * g.ldb * 2 < (1L << 31) && g.cfg != 1;
  if (v2) {
    const long tiles = (long)((g.M + VBM - 1) / VBM) * ((g.N + VBN - 1) / VBN) * g.batch;
    // v3 BK 32 at four per CU by default (cfg 0 / 6; 7: GM = 8): train shape 81 -> 69-73 us,
    // Sintel 56.5 -> 50.1 us, 1080p unchanged (1.26 ms, store-bound; profiles/r5n_bench_corr.log).
    // cfg 8: v3 BK 64, two per CU; cfg 2-5 / 9: v2 (GM overrides / automatic)
    static const bool v3 = [] {  // RAFT_CORR_V3=0: v2 for the automatic choice (A/B runs)
      const char* e = std::getenv("RAFT_CORR_V3");
      return !(e && e[0] == '0');
    }();
    // nontemporal output stores for volumes larger than the 256 MB Infinity Cache (1080p: 2.8 GB,
    // 1286 -> 1144 us standalone, profiles/r6g_bench_corr.log; the training volume, 180 MB, is
    // read back by the lookups right away and keeps its cache lines: 68.5 vs 70.4 us with NT).
    // RAFT_CORR_NT=1 / 0 forces it on / off (A/B).
    static const int nt_env = [] {
      const char* e = std::getenv("RAFT_CORR_NT");
      return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    const bool nt = nt_env >= 0 ? nt_env == 1 : (long)g.M * g.batch * g.ldc * 2 > (256L << 20);
    if (g.cfg == 0 && v3 && nt) {
      hipLaunchKernelGGL((corr_volume_v3_kernel<32, 4, true>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    } else if ((g.cfg == 0 && v3) || g.cfg == 6 || g.cfg == 7) {
      hipLaunchKernelGGL((corr_volume_v3_kernel<32, 4>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    } else if (g.cfg == 8) {
      hipLaunchKernelGGL((corr_volume_v3_kernel<64, 2>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    } else if (g.cfg == 11) {
      hipLaunchKernelGGL((corr_volume_v3_kernel<32, 4, true>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    } else if (g.cfg == 12) {
      hipLaunchKernelGGL((corr_volume_v3_kernel<64, 2, true>), dim3((unsigned)tiles), dim3(256), 0, s, g);
    } else {
      hipLaunchKernelGGL(corr_volume_bf16_kernel, dim3((unsigned)tiles), dim3(256), 0, s, g);
    }
    return hipGetLastError();
  }
  const dim3 grid((unsigned)(((g.M + GBM - 1) / GBM) * ((g.N + GBN - 1) / GBN) * g.batch)), blk(256);
  if (g.split) {
    if (g.a_trans) hipLaunchKernelGGL((corr_gemm_kernel<true, true>), grid, blk, 0, s, g);
    else hipLaunchKernelGGL((corr_gemm_kernel<true, false>), grid, blk, 0, s, g);
  } else {
    if (g.a_trans) hipLaunchKernelGGL((corr_gemm_kernel<false, true>), grid, blk, 0, s, g);
    else hipLaunchKernelGGL((corr_gemm_kernel<false, false>), grid, blk, 0, s, g);
  }
  return hipGetLastError();
}

hipError_t launch_corr_bwd_pair(const CorrGemmArgs& g1, const CorrGemmArgs& gt, hipStream_t s) {
  if (g1.a_trans || !gt.a_trans || !corr_bwd_ok(g1) || !corr_bwd_ok(gt)) return hipErrorInvalidValue;
  const int n1 = (corr_bwd_tiles(g1) + 7) / 8 * 8;
  const long total = (long)n1 + corr_bwd_tiles(gt);
  if (corr_bwd_tiles(g1) == 0 || corr_bwd_tiles(gt) == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(corr_bwd_pair_kernel, dim3((unsigned)total), dim3(256), 0, s, g1, gt, n1);
  return hipGetLastError();
}

hipError_t launch_pyramid_unpool(const UnpoolArgs& u, hipStream_t s) {
  const long total = (long)u.B * u.H * u.W * u.C;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(pyramid_unpool_kernel, dim3(grid_for(total)), dim3(256), 0, s, u);
  return hipGetLastError();
}

hipError_t launch_pyramid_operand(const PyrOperandArgs& a, hipStream_t s) {
  if ((long)a.B * a.C * a.ld == 0) return hipSuccess;
  if ((long)a.B * a.C * a.ld >= (1L << 31) || a.C % 4 != 0) return hipErrorInvalidValue;
  if (a.nchw) {
    const dim3 grid((unsigned)((a.ld + 63) / 64), (unsigned)((a.C + 63) / 64), (unsigned)a.B);
    hipLaunchKernelGGL(pyramid_operand_t_kernel, grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  const long total = (long)a.B * a.ld * (a.C / 4);
  hipLaunchKernelGGL(pyramid_operand_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_avgpool2x2(const float* in, float* out, long rows, int H, int W, hipStream_t s) {
  const int Ho = H / 2, Wo = W / 2;
  const long total = rows * Ho * Wo;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(avgpool2x2_kernel, dim3(grid_for(total)), dim3(256), 0, s, in, out, rows, H, W, Ho, Wo);
  return hipGetLastError();
}

// RAFT_LOOKUP_ALL=0: the one-level-ahead pipeline (A/B runs)
static bool lookup_all_levels() {
  static const bool v = [] {
    const char* e = std::getenv("RAFT_LOOKUP_ALL");
    return !(e && e[0] == '0');
  }();
  return v;
}

hipError_t launch_corr_lookup_fwd(const PyrDesc& pyr, const float* coords, void* out, int out_dtype, int B, int H,
                                  int W, int r, int out_ch, hipStream_t s, void* flow8, void* motion, long smo,
                                  int split_m) {
  // out_dtype kSplitBF16 (= 3): split-bf16 rows of 3 * out_ch; the flow operand split too
  // (motion lo plane ``smo_split`` channels after its hi plane)
  const bool split = out_dtype == 3;
  const FlowPack fp{static_cast<__bf16*>(flow8), static_cast<__bf16*>(motion), smo, out_dtype == kF16 ? 1 : 0,
                    split ? split_m : 0};
  const long npix = (long)B * H * W;
  if (npix == 0) return hipSuccess;
  if (r > 6 || (split && flow8 && split_m <= 0 && motion)) return hipErrorInvalidValue;
  const dim3 g((unsigned)((npix + 3) / 4)), blk(256);
  const bool all = r == 4 && pyr.levels <= 4 && lookup_all_levels();
  if (split && all)
    hipLaunchKernelGGL((lookup_fwd_kernel<SplitOut, 4, true>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (split && r == 4)
    hipLaunchKernelGGL((lookup_fwd_kernel<SplitOut, 4>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (split && r == 3)
    hipLaunchKernelGGL((lookup_fwd_kernel<SplitOut, 3>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (split)
    hipLaunchKernelGGL((lookup_fwd_kernel<SplitOut>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kBF16 && all)
    hipLaunchKernelGGL((lookup_fwd_kernel<__bf16, 4, true>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kF32 && all)
    hipLaunchKernelGGL((lookup_fwd_kernel<float, 4, true>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kF16 && all)
    hipLaunchKernelGGL((lookup_fwd_kernel<_Float16, 4, true>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kBF16 && r == 4)
    hipLaunchKernelGGL((lookup_fwd_kernel<__bf16, 4>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kF32 && r == 4)
    hipLaunchKernelGGL((lookup_fwd_kernel<float, 4>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kF16 && r == 4)
    hipLaunchKernelGGL((lookup_fwd_kernel<_Float16, 4>), g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kBF16)
    hipLaunchKernelGGL(lookup_fwd_kernel<__bf16>, g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else if (out_dtype == kF16)
    hipLaunchKernelGGL(lookup_fwd_kernel<_Float16>, g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  else
    hipLaunchKernelGGL(lookup_fwd_kernel<float>, g, blk, 0, s, pyr, coords, out, B, H, W, r, out_ch, fp);
  return hipGetLastError();
}

hipError_t launch_lookup_grad_rows(const GradRowsArgs& a, int g_dtype, hipStream_t s) {
  const long npix = (long)a.B * a.Hq * a.Wq;
  if (npix == 0 || a.T == 0) return hipSuccess;
  if (a.r > 6 || a.T > kGradRowsMaxT || a.ld > kGradRowsMaxLd || a.ld % 16 != 0 || a.levels > 4)
    return hipErrorInvalidValue;
  const size_t shm = (size_t)(a.ld + 4 * 176) * sizeof(float);
  const dim3 g((unsigned)npix), blk(256);
  if (g_dtype == kBF16 && a.r == 4)
    hipLaunchKernelGGL((lookup_grad_rows_kernel<__bf16, 4>), g, blk, shm, s, a);
  else if (g_dtype == kF32 && a.r == 4)
    hipLaunchKernelGGL((lookup_grad_rows_kernel<float, 4>), g, blk, shm, s, a);
  else if (g_dtype == kBF16)
    hipLaunchKernelGGL(lookup_grad_rows_kernel<__bf16>, g, blk, shm, s, a);
  else if (g_dtype == kF16)
    hipLaunchKernelGGL(lookup_grad_rows_kernel<_Float16>, g, blk, shm, s, a);
  else
    hipLaunchKernelGGL(lookup_grad_rows_kernel<float>, g, blk, shm, s, a);
  return hipGetLastError();
}

hipError_t launch_corr_lookup_bwd(const PyrDesc& dpyr, const float* coords, const void* gout, int g_dtype, int B,
                                  int H, int W, int r, int gstride, hipStream_t s) {
  const long npix = (long)B * H * W;
  if (npix == 0) return hipSuccess;
  if (r > 6) return hipErrorInvalidValue;
  const dim3 g((unsigned)((npix + 3) / 4)), blk(256);
  if (g_dtype == kBF16)
    hipLaunchKernelGGL(lookup_bwd_kernel<__bf16>, g, blk, 0, s, dpyr, coords, static_cast<const __bf16*>(gout), B, H,
                       W, r, gstride);
  else if (g_dtype == kF16)
    hipLaunchKernelGGL(lookup_bwd_kernel<_Float16>, g, blk, 0, s, dpyr, coords, static_cast<const _Float16*>(gout), B,
                       H, W, r, gstride);
  else
    hipLaunchKernelGGL(lookup_bwd_kernel<float>, g, blk, 0, s, dpyr, coords, static_cast<const float*>(gout), B, H,
                       W, r, gstride);
  return hipGetLastError();
}

}  // namespace raft_amd
