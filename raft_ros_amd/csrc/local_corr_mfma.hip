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

// Stage one 64-channel slice: query tile rows (32 x 64) and window chunk rows (256 x 64).
__device__ __forceinline__ void stage_tiles(const LocalCorrArgs& a, const TileGeo& g, int b, int l, int chunk, int c0,
                                            __bf16* sF1, __bf16* sW, int tid) {
  {  // 32 rows x 8 chunks of 16 B = 256 pieces, one per thread
    const int row = tid >> 3, pc = tid & 7;
    bf16x8_t v{};
    if (g.pix[row] >= 0) v = *reinterpret_cast<const bf16x8_t*>(a.f1 + (long)g.pix[row] * a.C + c0 + pc * 8);
    *reinterpret_cast<bf16x8_t*>(sF1 + row * FP + pc * 8) = v;
  }
  const __bf16* f2l = a.f2 + b * a.f2_bstride + (long)a.off[l] * a.C;
  const int area = g.bw * g.bh;
#pragma unroll 4
  for (int i = 0; i < 8; ++i) {  // 256 rows x 8 pieces = 2048 pieces
    const int piece = tid + 256 * i;
    const int row = piece >> 3, pc = piece & 7;
    const int n = chunk * WCAP + row;
    bf16x8_t v{};
    if (n < area) {
      const int wy = n / g.bw, wx = n - (n / g.bw) * g.bw;
      const int y = g.by0 + wy, x = g.bx0 + wx;
      v = *reinterpret_cast<const bf16x8_t*>(f2l + ((long)y * a.w[l] + x) * a.C + c0 + pc * 8);
    }
    *reinterpret_cast<bf16x8_t*>(sW + row * FP + pc * 8) = v;
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
    for (int chunk = 0; chunk < nchunks; ++chunk) {
      // S (32 x 256) = F1tile . F2win^T: wave w owns window pixels [64w, 64w + 64) (2 N-tiles)
      f32x16 acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
      for (int c0 = 0; c0 < a.C; c0 += KC) {
        stage_tiles(a, g, b, l, chunk, c0, sF1, sW, tid);
        __syncthreads();
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

template <int RC = 0>
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
      for (int s = 0; s < nkc; ++s) {
        stage_tiles(a, g, b, l, chunk, s * KC, sF1, sW, tid);
        __syncthreads();
        // dF1[q][c] += sum_n G[q][n] F2win[n][c]: M = 32 q (2 x 16), N = 16 channels (wave),
        // K = 256 window pixels.  A = G rows (k contiguous); B[k = n][col = c] = F2win column
        // -> transposed read of the [n][c] tile.
#pragma unroll
        for (int ks = 0; ks < WCAP / 32; ++ks) {
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(G + (m * 16 + (lane & 15)) * GP + ks * 32 +
                                                               (lane >> 4) * 8);
            // B fragment (16x16x32): lane holds B[k = 8 * (lane >> 4) + j][col = lane & 15]
            const int col = wave * 16 + (lane & 15);
            bf16x8 bfr;
#pragma unroll
            for (int j = 0; j < 8; ++j) bfr[j] = sW[(ks * 32 + (lane >> 4) * 8 + j) * FP + col];
            acc1[s][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc1[s][m], 0, 0, 0);
          }
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

}  // namespace raft_amd
