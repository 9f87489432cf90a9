// Memory-efficient ("alternate") correlation on MFMA: all pyramid levels, fwd + bwd.
//
// Reference: alt_cuda_corr/correlation_kernel.cu:18-119 (fwd), :122-256 (bwd), driven by
// AlternateCorrBlock (core/corr.py:63-91): for every query pixel and level the dot products
// of fmap1[p] with the (2r+2)^2 integer neighbours of floor(coords / 2^l) in the pooled
// fmap2, bilinearly blended into (2r+1)^2 taps (x-offset-major), scaled by 1/sqrt(C).
// The reference recomputes every dot on scalar FMAs per 32-channel chunk, in 32-thread
// blocks, and cannot train (no autograd, atomics for dF2).
//
// MI355X design: one 256-thread workgroup per 8 x 4 tile of query pixels (32 queries).
// Neighbouring queries have overlapping neighbourhoods (the flow is locally smooth), so per
// level the workgroup takes the bounding box of its 32 neighbourhoods -- the WINDOW, ~18 x 14
// level pixels at level 0 for a smooth flow -- and computes the dense block of dot products
//     S[q][n] = f1[q] . f2_l[n]     (32 queries x window pixels, K = C)
// with v_mfma_f32_32x32x16_bf16 from LDS-staged tiles (fmap1 tile + window, 64 channels per
// stage).  Each query then blends its taps from S.  A window larger than 256 pixels (flow
// discontinuity inside the tile) is processed in 256-pixel chunks, so any flow is correct;
// only the cost grows.  The fused update block's (P, 328) bf16 feature layout is written
// directly (level l at channel l*(2r+1)^2), so no permute / pad follows.
// Backward per level and window chunk: G[q][n] = the window-pixel gradients of the 32 queries
// (transpose of the bilinear blend, built in LDS), then
//     dF1 (32 x C)   += G . F2win      (MFMA 16x16x32, accumulated in registers over levels)
//     dF2win (n x C)  = G^T . F1tile   (MFMA 32x32x16, transposed LDS reads)
// dF1 is written once per query (the tile owns its queries); dF2win is added to the level's
// fp32 gradient with 256-byte wave-wide atomics (windows of different tiles overlap), and the
// level gradients are folded to level 0 afterwards (pyramid_unpool).
#include "common.h"

#include <algorithm>

namespace raft_amd {


namespace {

constexpr int TX = 8, TY = 4, NQ = TX * TY;  // query tile
constexpr int WCAP = 256;                    // window pixels per chunk
constexpr int KC = 64;                       // channels per LDS stage
constexpr int FP = KC + 8;                   // [row][c] LDS pitch (bf16): 144-byte rows
constexpr int GP = WCAP + 8;                 // G [q][n] pitch (bf16)
constexpr int SP = WCAP + 4;                 // S [q][n] pitch (fp32)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ s16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(reinterpret_cast<uintptr_t>(p) & 0xffffffffu));
}

__device__ __forceinline__ float clampc(float v) { return fminf(fmaxf(v, -1.0e6f), 1.0e6f); }

// Per-tile geometry shared through LDS.
struct TileGeo {
  int pix[NQ];      // flat query pixel (or -1)
  float fx[NQ], fy[NQ];
  int x0[NQ], y0[NQ];  // neighbourhood origin (level coords, = floor(c) - r)
  int bx0, by0, bw, bh;  // window box
};

// Query geometry at level l + window box (wave 0 lanes 0..31 own one query each).
__device__ __forceinline__ void tile_level_geometry(const LocalCorrArgs& a, TileGeo& g, int l, const float* cx,
                                                    const float* cy, int tid) {
  if (tid < 64) {
    const int q = tid & 31;
    int xmin = 1 << 30, ymin = 1 << 30, xmax = -(1 << 30), ymax = -(1 << 30);
    if (tid < 32) {
      const float s = 1.0f / float(1 << l);
      const bool ok = g.pix[q] >= 0 && isfinite(cx[q]) && isfinite(cy[q]);
      const float x = ok ? clampc(cx[q] * s) : 0.f, y = ok ? clampc(cy[q] * s) : 0.f;
      const float fx0 = floorf(x), fy0 = floorf(y);
      g.fx[q] = x - fx0;
      g.fy[q] = y - fy0;
      g.x0[q] = ok ? (int)fx0 - a.r : (1 << 29);  // invalid queries: neighbourhood far outside
      g.y0[q] = ok ? (int)fy0 - a.r : (1 << 29);
      if (ok) {
        xmin = g.x0[q];
        ymin = g.y0[q];
        xmax = g.x0[q] + 2 * a.r + 1;
        ymax = g.y0[q] + 2 * a.r + 1;
      }
    }
    // clip to the level plane: out-of-plane neighbours are zeros and need no window pixels
    for (int o = 16; o > 0; o >>= 1) {
      xmin = min(xmin, __shfl_xor(xmin, o, 64));
      ymin = min(ymin, __shfl_xor(ymin, o, 64));
      xmax = max(xmax, __shfl_xor(xmax, o, 64));
      ymax = max(ymax, __shfl_xor(ymax, o, 64));
    }
    if (tid == 0) {
      xmin = max(xmin, 0);
      ymin = max(ymin, 0);
      xmax = min(xmax, a.w[l] - 1);
      ymax = min(ymax, a.h[l] - 1);
      g.bx0 = xmin;
      g.by0 = ymin;
      g.bw = xmax >= xmin ? xmax - xmin + 1 : 0;
      g.bh = ymax >= ymin ? ymax - ymin + 1 : 0;
    }
  }
}

// Staging of one 64-channel slice -- query tile rows (32 x 64; F1 = false: not needed by the
// dF1-only backward) and window chunk rows (256 x 64) -- split into offsets (per level and
// window chunk), loads (per slice, into registers) and LDS stores, so the next slice's global
// loads are in flight while the MFMAs of the current one run (loading and storing each slice
// in place exposed 16-32 round trips per tile and level); the window rows' division by the
// box width is done once per chunk.
struct StageOff {
  long f1;    // element offset of this thread's query-tile piece (-1: none)
  long w[8];  // element offsets of its 8 window pieces from the level base (-1: zeros)
};
struct StageRegs {
  bf16x8_t f1;
  bf16x8_t w[8];
};
template <bool F1>
__device__ __forceinline__ void stage_offsets(const LocalCorrArgs& a, const TileGeo& g, int l, int chunk, int tid,
                                              StageOff& o) {
  o.f1 = -1;
  if constexpr (F1) {
    const int row = tid >> 3, pc = tid & 7;
    if (g.pix[row] >= 0) o.f1 = (long)g.pix[row] * a.C + pc * 8;
  }
  const int area = g.bw * g.bh;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = tid + 256 * i;
    const int row = piece >> 3, pc = piece & 7;
    const int n = chunk * WCAP + row;
    o.w[i] = -1;
    if (n < area) {
      const int wy = n / g.bw, wx = n - (n / g.bw) * g.bw;
      o.w[i] = ((long)(g.by0 + wy) * a.w[l] + g.bx0 + wx) * a.C + pc * 8;
    }
  }
}
template <bool F1>
__device__ __forceinline__ void stage_load(const LocalCorrArgs& a, const __bf16* f2l, const StageOff& o, int c0,
                                           StageRegs& r) {
  if constexpr (F1) {
    r.f1 = bf16x8_t{};
    if (o.f1 >= 0) r.f1 = *reinterpret_cast<const bf16x8_t*>(a.f1 + o.f1 + c0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.w[i] = bf16x8_t{};
    if (o.w[i] >= 0) r.w[i] = *reinterpret_cast<const bf16x8_t*>(f2l + o.w[i] + c0);
  }
}
template <bool F1>
__device__ __forceinline__ void stage_store(const StageRegs& r, __bf16* sF1, __bf16* sW, int tid) {
  if constexpr (F1) *reinterpret_cast<bf16x8_t*>(sF1 + (tid >> 3) * FP + (tid & 7) * 8) = r.f1;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = tid + 256 * i;
    *reinterpret_cast<bf16x8_t*>(sW + (piece >> 3) * FP + (piece & 7) * 8) = r.w[i];
  }
}

// window index of level pixel (y, x) relative to the box, or -1
__device__ __forceinline__ int win_index(const TileGeo& g, int y, int x) {
  const int wy = y - g.by0, wx = x - g.bx0;
  return ((unsigned)wy < (unsigned)g.bh && (unsigned)wx < (unsigned)g.bw) ? wy * g.bw + wx : -1;
}

__device__ __forceinline__ void tile_setup(const LocalCorrArgs& a, TileGeo& g, float* cx, float* cy, int& b, int tid) {
  const int tilesX = (a.W + TX - 1) / TX, tilesY = (a.H + TY - 1) / TY;
  const int t = blockIdx.x;
  b = t / (tilesX * tilesY);
  const int rem = t - b * tilesX * tilesY;
  const int ty0 = (rem / tilesX) * TY, tx0 = (rem - (rem / tilesX) * tilesX) * TX;
  if (tid < NQ) {
    const int y = ty0 + tid / TX, x = tx0 + tid % TX;
    const bool in = y < a.H && x < a.W;
    const int p = y * a.W + x;
    g.pix[tid] = in ? b * a.H * a.W + p : -1;
    const long HW = (long)a.H * a.W;
    cx[tid] = in ? a.coords[(long)b * 2 * HW + p] : 0.f;
    cy[tid] = in ? a.coords[(long)b * 2 * HW + HW + p] : 0.f;
  }
}

// RC > 0: the radius as a compile-time constant (RAFT's r = 4), so the per-element window
// index math divides by constants instead of running 32-bit divisions
template <typename OutT, int RC = 0>
__global__ __launch_bounds__(256) void local_corr_mfma_fwd_kernel(const LocalCorrArgs a) {
  __shared__ TileGeo g;
  __shared__ float cx[NQ], cy[NQ];
  __shared__ __attribute__((aligned(16))) __bf16 sF1[NQ * FP];
  __shared__ __attribute__((aligned(16))) __bf16 sW[WCAP * FP];
  static_assert(NQ * SP * 4 <= WCAP * FP * 2, "S reuses the window tile's LDS");
  float* const S = reinterpret_cast<float*>(sW);  // written after the last MFMA read of sW
  __shared__ float taps[NQ * 100];  // (2r+1)^2 <= 100 per query (r <= 4)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int b;
  tile_setup(a, g, cx, cy, b, tid);
  __syncthreads();
  const int rd = 2 * (RC > 0 ? RC : a.r) + 1, win = rd * rd;
  for (int l = 0; l < a.levels; ++l) {
    tile_level_geometry(a, g, l, cx, cy, tid);
    for (int i = tid; i < NQ * win; i += 256) taps[i] = 0.f;
    __syncthreads();
    const int nchunks = (g.bw * g.bh + WCAP - 1) / WCAP;
    const __bf16* f2l = a.f2 + b * a.f2_bstride + (long)a.off[l] * a.C;
    for (int chunk = 0; chunk < nchunks; ++chunk) {
      // S (32 x 256) = F1tile . F2win^T: wave w owns window pixels [64w, 64w + 64) (2 N-tiles)
      f32x16 acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
      StageOff so;
      StageRegs sr;
      stage_offsets<true>(a, g, l, chunk, tid, so);
      stage_load<true>(a, f2l, so, 0, sr);
      for (int c0 = 0; c0 < a.C; c0 += KC) {
        stage_store<true>(sr, sF1, sW, tid);
        __syncthreads();
        if (c0 + KC < a.C) stage_load<true>(a, f2l, so, c0 + KC, sr);  // in flight during the MFMAs
#pragma unroll
        for (int ks = 0; ks < KC / 16; ++ks) {
          const int fr = lane & 31, fk = (lane >> 5) * 8;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(sF1 + fr * FP + ks * 16 + fk);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(sW + (wave * 64 + j * 32 + fr) * FP + ks * 16 + fk);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[j], 0, 0, 0);
          }
        }
        __syncthreads();
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int q = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          S[q * SP + wave * 64 + j * 32 + (lane & 31)] = acc[j][e];
        }
      __syncthreads();
      // blend: each (query, tap) adds the corners that fall in this chunk
      for (int i = tid; i < NQ * win; i += 256) {
        const int q = i / win, t = i - (i / win) * win;
        if (g.pix[q] < 0) continue;
        const int ix = t / rd, iy = t - (t / rd) * rd;  // x-offset-major
        const float fx = g.fx[q], fy = g.fy[q];
        const float wts[4] = {(1.f - fx) * (1.f - fy), fx * (1.f - fy), (1.f - fx) * fy, fx * fy};
        float v = 0.f;
#pragma unroll
        for (int cnr = 0; cnr < 4; ++cnr) {
          const int y = g.y0[q] + iy + (cnr >> 1), x = g.x0[q] + ix + (cnr & 1);
          if ((unsigned)y >= (unsigned)a.h[l] || (unsigned)x >= (unsigned)a.w[l]) continue;
          const int n = win_index(g, y, x) - chunk * WCAP;
          if ((unsigned)n < (unsigned)WCAP) v += wts[cnr] * S[q * SP + n];
        }
        taps[i] += v;
      }
      __syncthreads();
    }
    for (int i = tid; i < NQ * win; i += 256) {
      const int q = i / win, t = i - (i / win) * win;
      if (g.pix[q] < 0) continue;
      static_cast<OutT*>(a.out)[(long)g.pix[q] * a.ostride + l * win + t] = static_cast<OutT>(a.scale * taps[i]);
    }
    __syncthreads();
  }
  const int pad = a.out_ch - a.levels * win;
  for (int i = tid; i < NQ * pad; i += 256) {
    const int q = i / pad;
    if (g.pix[q] >= 0)
      static_cast<OutT*>(a.out)[(long)g.pix[q] * a.ostride + a.levels * win + (i - q * pad)] = static_cast<OutT>(0.f);
  }
}

// DF2 = false: dF1 only (dF2 by the gather kernels below, lc_gather_df2_kernel)
template <int RC = 0, bool DF2 = true>
__global__ __launch_bounds__(256) void local_corr_mfma_bwd_kernel(const LocalCorrArgs a) {
  __shared__ TileGeo g;
  __shared__ float cx[NQ], cy[NQ];
  __shared__ __attribute__((aligned(16))) __bf16 sF1[NQ * FP];
  __shared__ __attribute__((aligned(16))) __bf16 sW[WCAP * FP];
  __shared__ __attribute__((aligned(16))) __bf16 G[NQ * GP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int b;
  tile_setup(a, g, cx, cy, b, tid);
  __syncthreads();
  const int rd = 2 * (RC > 0 ? RC : a.r) + 1, nd = rd + 1, win = rd * rd;
  const int nkc = a.C / KC;  // <= 4 (C <= 256)
  const float fs = a.g2fix != nullptr ? *a.fix_scale : 0.f;  // fixed-point scale (deterministic mode)
  // dF1 accumulators: MFMA 16x16x32, wave w owns channels [16w, 16w + 16) of every 64-slice,
  // 2 M-tiles of 16 queries, 4 slices -> acc1[slice][mtile]
  f32x4 acc1[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int m = 0; m < 2; ++m) acc1[s][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int hh = lane >> 5, gi = (lane >> 4) & 1, qq = (lane & 15) >> 2, pq = lane & 3;

  for (int l = 0; l < a.levels; ++l) {
    tile_level_geometry(a, g, l, cx, cy, tid);
    __syncthreads();
    const int nchunks = (g.bw * g.bh + WCAP - 1) / WCAP;
    float* g2l = a.g2 + b * a.f2_bstride + (long)a.off[l] * a.C;
    for (int chunk = 0; chunk < nchunks; ++chunk) {
      // G[q][n]: window-pixel gradient of query q (transpose of the bilinear blend), bf16
      for (int i = tid; i < NQ * GP / 8; i += 256) reinterpret_cast<uint4*>(G)[i] = uint4{0, 0, 0, 0};
      __syncthreads();
      for (int i = tid; i < NQ * nd * nd; i += 256) {
        const int q = i / (nd * nd), e = i - (i / (nd * nd)) * (nd * nd);
        if (g.pix[q] < 0) continue;
        const int aa = e / nd, cc = e - (e / nd) * nd;  // neighbour (y0 + aa, x0 + cc)
        const int y = g.y0[q] + aa, x = g.x0[q] + cc;
        if ((unsigned)y >= (unsigned)a.h[l] || (unsigned)x >= (unsigned)a.w[l]) continue;
        const int n = win_index(g, y, x) - chunk * WCAP;
        if ((unsigned)n >= (unsigned)WCAP) continue;
        const float fx = g.fx[q], fy = g.fy[q];
        const long gbase = (long)g.pix[q] * a.gstride + l * win;
        auto gv = [&](int t) {
          return a.gout_bf16 ? static_cast<float>(static_cast<const __bf16*>(a.gout)[gbase + t])
                             : static_cast<const float*>(a.gout)[gbase + t];
        };
        // neighbour (aa, cc) is corner (0,0) of tap (ix=cc, iy=aa), (0,1) of (cc-1, aa),
        // (1,0) of (cc, aa-1), (1,1) of (cc-1, aa-1); tap channel = ix * rd + iy
        float v = 0.f;
        if (aa < rd) {
          if (cc < rd) v += (1.f - fx) * (1.f - fy) * gv(cc * rd + aa);
          if (cc > 0) v += fx * (1.f - fy) * gv((cc - 1) * rd + aa);
        }
        if (aa > 0) {
          if (cc < rd) v += (1.f - fx) * fy * gv(cc * rd + aa - 1);
          if (cc > 0) v += fx * fy * gv((cc - 1) * rd + aa - 1);
        }
        G[q * GP + n] = static_cast<__bf16>(v * a.scale);
      }
      __syncthreads();
      StageOff so;
      StageRegs sr;
      const __bf16* f2l = a.f2 + b * a.f2_bstride + (long)a.off[l] * a.C;
      stage_offsets<DF2>(a, g, l, chunk, tid, so);
      stage_load<DF2>(a, f2l, so, 0, sr);
      for (int s = 0; s < nkc; ++s) {
        stage_store<DF2>(sr, sF1, sW, tid);
        __syncthreads();
        if (s + 1 < nkc) stage_load<DF2>(a, f2l, so, (s + 1) * KC, sr);  // in flight during the MFMAs
        // dF1[q][c] += sum_n G[q][n] F2win[n][c]: M = 32 q (2 x 16), N = 16 channels (wave),
        // K = 256 window pixels.  A = G rows (k contiguous); B[k = n][col = c] = F2win column
        // -> transposed read of the [n][c] tile.
#pragma unroll
        for (int ks = 0; ks < WCAP / 32; ++ks) {
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(G + (m * 16 + (lane & 15)) * GP + ks * 32 +
                                                               (lane >> 4) * 8);
            // B fragment (16x16x32): lane holds B[k = 8 * (lane >> 4) + j][col = lane & 15]: two
            // transposed reads of 4 window rows x the wave's 16 channels (lane 4q + p of a 16-lane
            // group addresses row q, channels 4p .. 4p + 3), instead of 8 scalar 16-bit reads
            const int tr_row = ks * 32 + (lane >> 4) * 8 + ((lane & 15) >> 2), tr_col = wave * 16 + 4 * (lane & 3);
            const s16x4 blo = tr_read(sW + tr_row * FP + tr_col);
            const s16x4 bhi = tr_read(sW + (tr_row + 4) * FP + tr_col);
            const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
            acc1[s][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc1[s][m], 0, 0, 0);
          }
        }
        if constexpr (!DF2) {
          __syncthreads();
          continue;
        }
        // dF2win[n][c] = sum_q G[q][n] F1[q][c]: M = 256 n (wave: 64 = 2 tiles), N = 64 c
        // (2 tiles), K = 32 q.  A[row n][k = q] = G column -> transposed read of G [q][n];
        // B[k = q][col = c] = F1 column -> transposed read of F1 [q][c].
        f32x16 acc2[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc2[i][j][e] = 0.f;
#pragma unroll
        for (int ks = 0; ks < NQ / 16; ++ks) {
          const int r0 = ks * 16 + hh * 8 + qq;
          bf16x8 af[2], bfr[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int col = wave * 64 + i * 32 + gi * 16 + 4 * pq;
            const s16x4 lo = tr_read(G + r0 * GP + col);
            const s16x4 hi = tr_read(G + (r0 + 4) * GP + col);
            af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = j * 32 + gi * 16 + 4 * pq;
            const s16x4 lo = tr_read(sF1 + r0 * FP + col);
            const s16x4 hi = tr_read(sF1 + (r0 + 4) * FP + col);
            bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc2[i][j], 0, 0, 0);
        }
        // add the window tile into the level gradient (windows of neighbouring tiles overlap)
        const int area = g.bw * g.bh;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int n = chunk * WCAP + wave * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            if (n >= area) continue;
            const int wy = n / g.bw, wx = n - (n / g.bw) * g.bw;
            const long di = ((long)(g.by0 + wy) * a.w[l] + g.bx0 + wx) * a.C + s * KC + (lane & 31);
            if (a.g2fix != nullptr) {
              long long* dst = a.g2fix + (g2l - a.g2) + di;
#pragma unroll
              for (int j = 0; j < 2; ++j) fixed_atomic_add(dst + j * 32, acc2[i][j][e], fs);
            } else {
              float* dst = g2l + di;
#pragma unroll
              for (int j = 0; j < 2; ++j) atomicAdd(dst + j * 32, acc2[i][j][e]);
            }
          }
        __syncthreads();
      }
    }
  }
  // dF1: 16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + e
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s >= nkc) break;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = m * 16 + 4 * (lane >> 4) + e;
        if (g.pix[q] < 0) continue;
        a.g1[(long)g.pix[q] * a.C + s * KC + wave * 16 + (lane & 15)] = acc1[s][m][e];
      }
  }
}

// ---------------------------------------------------------------- dF2 by gathering (no atomics)
// The tile-window backward above adds every tile's window gradient into the level gradient with
// fp32 atomics: the windows of neighbouring 8 x 4 query tiles overlap ~7x at level 0, so a
// KITTI-size step (3 x 376 x 1248) issues ~0.44 GB of atomic adds per lookup, which the memory
// side retires at ~1.3 TB/s -- 3/4 of the kernel's 552 us (profiles/r5a_pmc_alt_summary.txt:
// 0.17 L2 hit, 5.6 M write requests).  Instead, per level, the queries are binned by the 8 x 8
// blocks of level pixels their (2r+2)^2 neighbourhood touches (count / scan / fill), and one
// workgroup per (block, segment of <= LC_SEG queries) computes
//     dF2[block px][c] = sum_q G[q][px] F1[q][c]     (M = 64 px, N = 256 c, K = the queries)
// with G built from the tap gradients in LDS -- each level pixel is written by its block's
// workgroup (a plain store when the block has one segment; segments of longer lists -- the
// coarse levels, where ~100 x 4^l queries touch a pixel -- are added with atomics, ~10x fewer
// bytes than the windows).  Query order inside a list follows the fill atomics, so the fp32
// sums are not bitwise reproducible: deterministic mode keeps the fixed-point window path.
constexpr int LC_B = 8;      // block side (level pixels)
constexpr int LC_Q = 32;     // queries per chunk (MFMA K)
constexpr int LC_SEG = 512;  // queries per workgroup item
constexpr int LC_FP = 256 + 8;  // F1 chunk pitch (bf16): C <= 256
constexpr int LC_GP = 64 + 8;   // G chunk pitch (bf16): 64 block pixels
constexpr int LC_SH = 16;       // counter shards per block (workgroup index % LC_SH): at level 3
                                // every wave of an image adds to the same few blocks

struct LcBin {
  int levels, B, H, W, r;
  int w[4], h[4], nbx[4], nby[4], blk0[5];  // blk0[levels] = total blocks
};

__device__ __forceinline__ bool lc_box(const LcBin& bn, const float* coords, long q, int l, int& bx0, int& bx1,
                                       int& by0, int& by1, int& x0, int& y0, float& fx, float& fy) {
  const long HW = (long)bn.H * bn.W;
  const long b = q / HW, p = q - b * HW;
  const float cx = coords[b * 2 * HW + p], cy = coords[b * 2 * HW + HW + p];
  if (!isfinite(cx) || !isfinite(cy)) return false;
  const float s = 1.0f / float(1 << l);
  const float x = clampc(cx * s), y = clampc(cy * s);
  const float fx0 = floorf(x), fy0 = floorf(y);
  fx = x - fx0;
  fy = y - fy0;
  x0 = (int)fx0 - bn.r;
  y0 = (int)fy0 - bn.r;
  const int nd = 2 * bn.r + 2;
  const int xa = max(x0, 0), xb = min(x0 + nd - 1, bn.w[l] - 1);
  const int ya = max(y0, 0), yb = min(y0 + nd - 1, bn.h[l] - 1);
  if (xa > xb || ya > yb) return false;
  bx0 = xa / LC_B;
  bx1 = xb / LC_B;
  by0 = ya / LC_B;
  by1 = yb / LC_B;
  return true;
}

// pass 1 / 3: count (fill == false) or fill the per-block query lists.  Neighbouring queries
// touch the same few blocks (at level 3 thousands of queries share one block), so one atomic
// per counter per WAVE: the lanes holding the same block key are matched by ballot and their
// leader adds the group's count (per-lane atomics on one counter serialised: 0.7 ms a pass)
template <bool FILL>
__global__ __launch_bounds__(256) void lc_bin_kernel(const LcBin bn, const float* __restrict__ coords,
                                                     int* __restrict__ cnt, const int* __restrict__ off,
                                                     int* __restrict__ list) {
  const long P = (long)bn.B * bn.H * bn.W;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool in = q < P;
  const int b = in ? (int)(q / ((long)bn.H * bn.W)) : 0;
  for (int l = 0; l < bn.levels; ++l) {
    int bx0 = 0, bx1 = -1, by0 = 0, by1 = -1, x0, y0;
    float fx, fy;
    if (!(in && lc_box(bn, coords, q, l, bx0, bx1, by0, by1, x0, y0, fx, fy))) bx1 = by1 = -1, bx0 = by0 = 0;
    // up to 3 x 3 blocks per query: slot k = (dy, dx) relative to (by0, bx0)
    for (int k = 0; k < 9; ++k) {
      const int by = by0 + k / 3, bx = bx0 + k % 3;
      int key = (by <= by1 && bx <= bx1) ? bn.blk0[l] + (b * bn.nby[l] + by) * bn.nbx[l] + bx : -1;
      for (;;) {
        const unsigned long long active = __ballot(key >= 0);
        if (active == 0) break;
        const int src = __ffsll((long long)active) - 1;
        const int lead = __shfl(key, src, 64);
        const unsigned long long m = __ballot(key == lead);
        const int first = __ffsll((long long)m) - 1;
        const int slot = lead * LC_SH + (int)(blockIdx.x & (LC_SH - 1));
        if constexpr (FILL) {
          // the leader fetches the list offset beside its cursor add: one dependent round trip
          int base = 0;
          if (lane == first) base = off[slot] + atomicAdd(cnt + slot, __popcll(m));
          base = __shfl(base, first, 64);
          if (key == lead) list[base + __popcll(m & ((1ull << lane) - 1ull))] = (int)q;
        } else {
          if (lane == first) atomicAdd(cnt + slot, __popcll(m));  // no return value needed
        }
        if (key == lead) key = -1;
      }
    }
  }
}

// pass 2 (one workgroup): off = exclusive scan of the (block, shard) counts -- a block's list is
// its shards back to back, [off[blk * LC_SH], off[(blk + 1) * LC_SH]) -- the work items (block,
// segment), and the counts reset to 0 for the fill pass's cursors.  hdr = {items, next item}
__global__ __launch_bounds__(1024) void lc_scan_kernel(int* __restrict__ cnt, int* __restrict__ off, int nb,
                                                       int* __restrict__ items, int* __restrict__ hdr) {
  __shared__ int sa[1024], sb[1024];
  __shared__ int carry[2];
  const int tid = threadIdx.x;
  if (tid == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + tid;
    int sh[LC_SH], c = 0;
#pragma unroll
    for (int k = 0; k < LC_SH; ++k) {
      sh[k] = i < nb ? cnt[i * LC_SH + k] : 0;
      c += sh[k];
    }
    const int ns = (c + LC_SEG - 1) / LC_SEG;
    sa[tid] = c;
    sb[tid] = ns;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scans
      const int va = tid >= d ? sa[tid - d] : 0, vb = tid >= d ? sb[tid - d] : 0;
      __syncthreads();
      sa[tid] += va;
      sb[tid] += vb;
      __syncthreads();
    }
    if (i < nb) {
      int o = carry[0] + sa[tid] - c;
      const int io = carry[1] + sb[tid] - ns;
#pragma unroll
      for (int k = 0; k < LC_SH; ++k) {
        off[i * LC_SH + k] = o;
        o += sh[k];
        cnt[i * LC_SH + k] = 0;
      }
      for (int sgi = 0; sgi < ns; ++sgi) items[io + sgi] = i * 1024 + sgi;
    }
    __syncthreads();
    if (tid == 1023) {
      carry[0] += sa[1023];
      carry[1] += sb[1023];
    }
    __syncthreads();
  }
  if (tid == 0) {
    off[nb * LC_SH] = carry[0];
    hdr[0] = carry[1];
    hdr[1] = 0;
  }
}

// pass 4: persistent workgroups pull (block, segment) items; dF2 rows of the block.  Every
// wave covers the block's 64 pixels and NJ 32-channel tiles (C = 128 NJ: 4 waves x NJ x 32)
template <int RC, int NJ>
__global__ __launch_bounds__(256) void lc_gather_df2_kernel(const LocalCorrArgs a, const LcBin bn,
                                                            const int* __restrict__ off,
                                                            const int* __restrict__ list,
                                                            const int* __restrict__ items, int* __restrict__ hdr) {
  __shared__ __attribute__((aligned(16))) __bf16 sF1[LC_Q * LC_FP];
  __shared__ __attribute__((aligned(16))) __bf16 G[LC_Q * LC_GP];
  __shared__ int qpix[LC_Q], qx0[LC_Q], qy0[LC_Q];
  __shared__ float qfx[LC_Q], qfy[LC_Q];
  __shared__ float sg[LC_Q * 84];  // the chunk's level-l tap gradients ((2r+1)^2 <= 81 per query)
  __shared__ int s_item;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rd = 2 * (RC > 0 ? RC : a.r) + 1, nd = rd + 1, win = rd * rd;
  const int nitems = hdr[0];
  const int hh = lane >> 5, gi = (lane >> 4) & 1, qq = (lane & 15) >> 2, pq = lane & 3;
  const int C = a.C;
  for (;;) {
    if (tid == 0) s_item = atomicAdd(hdr + 1, 1);
    __syncthreads();
    const int item = s_item;
    __syncthreads();  // s_item read by every wave before the next dequeue
    if (item >= nitems) break;
    const int blk = items[item] >> 10, seg = items[item] & 1023;
    int l = 0;
    while (l + 1 < bn.levels && blk >= bn.blk0[l + 1]) ++l;
    const int lb = blk - bn.blk0[l];
    const int b = lb / (bn.nbx[l] * bn.nby[l]);
    const int rem = lb - b * bn.nbx[l] * bn.nby[l];
    const int by = rem / bn.nbx[l], bx = rem - (rem / bn.nbx[l]) * bn.nbx[l];
    const int lb0 = off[blk * LC_SH], lb1 = off[(blk + 1) * LC_SH];
    const int lbeg = lb0 + seg * LC_SEG, lend = min(lb1, lbeg + LC_SEG);
    const bool single = lb1 - lb0 <= LC_SEG;
    f32x16 acc[2][NJ];  // [32-pixel tile][32-channel tile of the wave]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    constexpr int cw = NJ * 32;  // channels per wave
    for (int q0 = lbeg; q0 < lend; q0 += LC_Q) {
      if (tid < LC_Q) {
        const int li = q0 + tid;
        int pix = -1, x0 = 0, y0 = 0;
        float fx = 0.f, fy = 0.f;
        if (li < lend) {
          pix = list[li];
          int t0, t1, t2, t3;
          if (!lc_box(bn, a.coords, pix, l, t0, t1, t2, t3, x0, y0, fx, fy)) pix = -1;
        }
        qpix[tid] = pix;
        qx0[tid] = x0;
        qy0[tid] = y0;
        qfx[tid] = fx;
        qfy[tid] = fy;
      }
      __syncthreads();
      // the chunk's tap gradients (coalesced rows of win values) -> sg [q][t]
      for (int i = tid; i < LC_Q * win; i += 256) {
        const int qi = i / win, t = i - (i / win) * win;
        const int pix = qpix[qi];
        float v = 0.f;
        if (pix >= 0) {
          const long gi_ = (long)pix * a.gstride + l * win + t;
          v = a.gout_bf16 ? static_cast<float>(static_cast<const __bf16*>(a.gout)[gi_])
                          : static_cast<const float*>(a.gout)[gi_];
        }
        sg[qi * 84 + t] = v;
      }
      // F1 rows of the chunk -> sF1 [q][c]
      for (int i = tid; i < LC_Q * (C / 8); i += 256) {
        const int row = i / (C / 8), pc = i - (i / (C / 8)) * (C / 8);
        bf16x8_t v{};
        if (qpix[row] >= 0) v = *reinterpret_cast<const bf16x8_t*>(a.f1 + (long)qpix[row] * C + pc * 8);
        *reinterpret_cast<bf16x8_t*>(sF1 + row * LC_FP + pc * 8) = v;
      }
      __syncthreads();
      // G[q][px]: the gradient of block pixel px through query q's bilinear taps (the transpose
      // of the forward blend, as in local_corr_mfma_bwd_kernel); thread = (query, block row)
      {
        const int q = tid & 31, ry = tid >> 5;
        const int pix = qpix[q];
        const int y = by * LC_B + ry;
        const float fx = qfx[q], fy = qfy[q];
        const float* gq = sg + q * 84;
        auto gv = [&](int t) { return gq[t]; };
#pragma unroll
        for (int rx = 0; rx < LC_B; ++rx) {
          const int x = bx * LC_B + rx;
          const int aa = y - qy0[q], cc = x - qx0[q];
          float v = 0.f;
          if (pix >= 0 && y < bn.h[l] && x < bn.w[l] && (unsigned)aa < (unsigned)nd && (unsigned)cc < (unsigned)nd) {
            if (aa < rd) {
              if (cc < rd) v += (1.f - fx) * (1.f - fy) * gv(cc * rd + aa);
              if (cc > 0) v += fx * (1.f - fy) * gv((cc - 1) * rd + aa);
            }
            if (aa > 0) {
              if (cc < rd) v += (1.f - fx) * fy * gv(cc * rd + aa - 1);
              if (cc > 0) v += fx * fy * gv((cc - 1) * rd + aa - 1);
            }
          }
          G[q * LC_GP + ry * LC_B + rx] = static_cast<__bf16>(v * a.scale);
        }
      }
      __syncthreads();
      // acc[i][j] += G^T[px tile i][q] F1[q][c tile j]: A = transposed read of G [q][px],
      // B = transposed read of sF1 [q][c] (the k permutation of both reads is the same)
#pragma unroll
      for (int ks = 0; ks < LC_Q / 16; ++ks) {
        const int r0 = ks * 16 + hh * 8 + qq;
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int col = i * 32 + gi * 16 + 4 * pq;
          const s16x4 lo = tr_read(G + r0 * LC_GP + col);
          const s16x4 hi = tr_read(G + (r0 + 4) * LC_GP + col);
          af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int col = wave * cw + j * 32 + gi * 16 + 4 * pq;
          const s16x4 lo = tr_read(sF1 + r0 * LC_FP + col);
          const s16x4 hi = tr_read(sF1 + (r0 + 4) * LC_FP + col);
          const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
        }
      }
      __syncthreads();
    }
    // store / add the block's rows: C/D map row = px (e), col = channel (lane & 31)
    float* g2l = a.g2 + (long)b * a.f2_bstride + (long)a.off[l] * C;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int px = i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int y = by * LC_B + px / LC_B, x = bx * LC_B + px % LC_B;
        if (y >= bn.h[l] || x >= bn.w[l]) continue;
        float* dst = g2l + ((long)y * bn.w[l] + x) * C + wave * cw + (lane & 31);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if (single) dst[j * 32] = acc[i][j][e];
          else atomicAdd(dst + j * 32, acc[i][j][e]);
        }
      }
  }
}

__global__ __launch_bounds__(256) void fixed_to_float_kernel(const long long* __restrict__ in, float* __restrict__ out,
                                                             long n, const float* __restrict__ fix_scale) {
  const double inv = 1.0 / static_cast<double>(*fix_scale);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    out[i] += static_cast<float>(static_cast<double>(in[i]) * inv);
}

}  // namespace

hipError_t launch_fixed_to_float(const long long* in, float* out, long n, const float* fix_scale, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const long blocks = std::min<long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(fixed_to_float_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, out, n, fix_scale);
  return hipGetLastError();
}

hipError_t launch_local_corr_mfma(const LocalCorrArgs& a, bool backward, hipStream_t s) {
  // the forward loops over any number of 64-channel slices (split-bf16 inference: C = 3 x 256,
  // [hi | lo | hi] . [hi | hi | lo]); the backward keeps dF1 of <= 4 slices in registers
  if (a.r > 4 || a.C % KC != 0 || a.C > (backward ? 256 : 768) || a.levels < 1 || a.levels > 4)
    return hipErrorInvalidValue;
  const long tiles = (long)a.B * ((a.H + TY - 1) / TY) * ((a.W + TX - 1) / TX);
  if (tiles == 0) return hipSuccess;
  const bool r4 = a.r == 4;
  if (backward && r4)
    hipLaunchKernelGGL(local_corr_mfma_bwd_kernel<4>, dim3((unsigned)tiles), dim3(256), 0, s, a);
  else if (backward)
    hipLaunchKernelGGL(local_corr_mfma_bwd_kernel<0>, dim3((unsigned)tiles), dim3(256), 0, s, a);
  else if (a.out_f32 && r4)
    hipLaunchKernelGGL((local_corr_mfma_fwd_kernel<float, 4>), dim3((unsigned)tiles), dim3(256), 0, s, a);
  else if (a.out_f32)
    hipLaunchKernelGGL((local_corr_mfma_fwd_kernel<float, 0>), dim3((unsigned)tiles), dim3(256), 0, s, a);
  else if (r4)
    hipLaunchKernelGGL((local_corr_mfma_fwd_kernel<__bf16, 4>), dim3((unsigned)tiles), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((local_corr_mfma_fwd_kernel<__bf16, 0>), dim3((unsigned)tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---- gather backward: dF1 by the tile kernel (no dF2 part), dF2 by binning + gathering
namespace {
LcBin lc_bin(const LocalCorrArgs& a) {
  LcBin bn{};
  bn.levels = a.levels;
  bn.B = a.B;
  bn.H = a.H;
  bn.W = a.W;
  bn.r = a.r;
  int tot = 0;
  for (int l = 0; l < a.levels; ++l) {
    bn.w[l] = a.w[l];
    bn.h[l] = a.h[l];
    bn.nbx[l] = (a.w[l] + LC_B - 1) / LC_B;
    bn.nby[l] = (a.h[l] + LC_B - 1) / LC_B;
    bn.blk0[l] = tot;
    tot += a.B * bn.nbx[l] * bn.nby[l];
  }
  bn.blk0[a.levels] = tot;
  return bn;
}
// a neighbourhood of 2r + 2 <= 10 pixels touches at most 3 blocks of 8 per axis
constexpr int kLcMaxBlocksPerQuery = 9;
long lc_list_bound(const LocalCorrArgs& a) { return (long)a.B * a.H * a.W * a.levels * kLcMaxBlocksPerQuery; }
}  // namespace

bool local_corr_gather_ok(const LocalCorrArgs& a) { return (a.C == 128 || a.C == 256) && a.r <= 4 && a.levels <= 4; }

long local_corr_gather_scratch(const LocalCorrArgs& a) {
  const LcBin bn = lc_bin(a);
  const long nb = bn.blk0[a.levels];
  const long lists = lc_list_bound(a);
  return nb * LC_SH + (nb * LC_SH + 1) + 2 + (nb + lists / LC_SEG + 1) + lists;
}

hipError_t launch_local_corr_mfma_bwd_gather(const LocalCorrArgs& a, int* scratch, hipStream_t s) {
  if (!local_corr_gather_ok(a)) return hipErrorInvalidValue;
  const long tiles = (long)a.B * ((a.H + TY - 1) / TY) * ((a.W + TX - 1) / TX);
  if (tiles == 0) return hipSuccess;
  const LcBin bn = lc_bin(a);
  const int nb = bn.blk0[a.levels];
  const long lists = lc_list_bound(a);
  int* cnt = scratch;
  int* off = cnt + nb * LC_SH;
  int* hdr = off + nb * LC_SH + 1;
  int* items = hdr + 2;
  int* list = items + (nb + lists / LC_SEG + 1);
  const long P = (long)a.B * a.H * a.W;
  const unsigned pblocks = (unsigned)((P + 255) / 256);
  if (hipMemsetAsync(cnt, 0, (size_t)nb * LC_SH * sizeof(int), s) != hipSuccess) return hipGetLastError();
  hipLaunchKernelGGL(lc_bin_kernel<false>, dim3(pblocks), dim3(256), 0, s, bn, a.coords, cnt, off, list);
  hipLaunchKernelGGL(lc_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, off, nb, items, hdr);
  hipLaunchKernelGGL(lc_bin_kernel<true>, dim3(pblocks), dim3(256), 0, s, bn, a.coords, cnt, off, list);
  // dF1 (the tile kernel without its window-gradient atomics)
  if (a.r == 4)
    hipLaunchKernelGGL((local_corr_mfma_bwd_kernel<4, false>), dim3((unsigned)tiles), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((local_corr_mfma_bwd_kernel<0, false>), dim3((unsigned)tiles), dim3(256), 0, s, a);
  // dF2: persistent workgroups over the (block, segment) items
  const unsigned wgs = (unsigned)std::min<long>(1024, nb + lists / LC_SEG + 1);
  if (a.C == 256) {
    if (a.r == 4) hipLaunchKernelGGL((lc_gather_df2_kernel<4, 2>), dim3(wgs), dim3(256), 0, s, a, bn, off, list, items, hdr);
    else hipLaunchKernelGGL((lc_gather_df2_kernel<0, 2>), dim3(wgs), dim3(256), 0, s, a, bn, off, list, items, hdr);
  } else {
    if (a.r == 4) hipLaunchKernelGGL((lc_gather_df2_kernel<4, 1>), dim3(wgs), dim3(256), 0, s, a, bn, off, list, items, hdr);
    else hipLaunchKernelGGL((lc_gather_df2_kernel<0, 1>), dim3(wgs), dim3(256), 0, s, a, bn, off, list, items, hdr);
  }
  return hipGetLastError();
}

}  // namespace raft_amd
