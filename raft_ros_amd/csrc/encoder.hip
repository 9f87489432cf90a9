// Residual CNN encoders on gfx950 MFMA: strided NHWC convolutions (forward, data and
// weight gradients) and the normalisation / residual glue around them.
//
// Reference: core/extractor.py:6-267 (BasicEncoder / SmallEncoder: 7x7/s2 stem,
// ResidualBlock / BottleneckBlock stages at strides 1, 2, 2, 1x1 output conv; norms
// batch / instance / none).  The reference runs these on cuDNN with separate norm,
// ReLU and add kernels; here an encoder is one native op sequence:
//
//   conv (implicit GEMM, M = output pixels, N = out channels, K = taps x in channels)
//     epilogue: + bias, per-tile (sum, M2) statistics of the output -> no separate
//     statistics pass for the following InstanceNorm / BatchNorm;
//   stats finalize: Chan-combined per-(image, channel) [instance] or per-channel [batch]
//     mean / variance in a fixed order (deterministic), BatchNorm running statistics;
//   apply: relu(norm(a)) or the residual tail relu(relu(norm(a2)) + norm3(ad) | x);
//   backward: data gradients as the same conv kernel over dY with flipped / transposed
//     packed weights; a stride-2 conv's data gradient is split into its 4 output parity
//     classes (each a dense conv over the taps that hit it) so no zero-stuffed dY or
//     wasted MFMA; the 3x3/s2 conv and the 1x1/s2 downsample of a block share one launch
//     (their K ranges are concatenated); the epilogue adds the identity-residual gradient
//     and applies the ReLU' mask of the block input;
//   norm backward: partial sums of dy' and dy'*xhat -> coefficients -> one apply pass
//     (both tail branches at once);
//   weight gradient: dW[co][k] = sum_p dY[p][co] im2col(X)[p][k] over a pixel split
//     (fp32 slab per split, fixed-order reduce into the fp32 parameter layout).
//
// All gathers use a per-launch K-chunk decode table (8 consecutive K columns = 8
// channels of one tap of one source): every conv shape of both encoders, including the
// 3-channel stem (padded to 8) and the small encoder's 8/16/24-channel bottlenecks, runs
// through one kernel family.
#include "common.h"
#include "kernel_abi.h"

#include <algorithm>

namespace raft_amd {








namespace {

constexpr int EBK = 64, ELDK = EBK + 8;

// 8 channels of 16-bit storage: bf16, or fp16 under fp16 AMP (common.h st16 / ld16)
__device__ __forceinline__ void load8(const __bf16* p, float* v, bool f16 = false) {
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = ld16(x[i], f16);
}
__device__ __forceinline__ void store8(__bf16* p, const float* v, bool f16 = false) {
  bf16x8 x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = st16(v[i], f16);
  *reinterpret_cast<bf16x8*>(p) = x;
}
// split-bf16 planes (kernel_abi.h EncConvArgs::split), planes of S channels at p, p + S, p + 2S:
//   mode 1: hi, lo = bf16(x - hi), hi again   (x ~ hi + lo: a 16-bit mantissa)
//   mode 2: hi, mid = bf16(x - hi), lo = bf16(x - hi - mid)   (x = hi + mid + lo: the fp32 value)
// The first two planes are the same in both modes, so readers of [hi | lo] (the weight
// gradients, the gradient planes of the backward) work on either.
__device__ __forceinline__ void store8_split(__bf16* p, int S, const float* v, int mode = 1) {
  bf16x8 hi, lo, third;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    hi[i] = static_cast<__bf16>(v[i]);
    const float r = v[i] - static_cast<float>(hi[i]);
    lo[i] = static_cast<__bf16>(r);
    third[i] = mode == 2 ? static_cast<__bf16>(r - static_cast<float>(lo[i])) : hi[i];
  }
  *reinterpret_cast<bf16x8*>(p) = hi;
  *reinterpret_cast<bf16x8*>(p + S) = lo;
  *reinterpret_cast<bf16x8*>(p + 2 * S) = third;
}
__device__ __forceinline__ void load8_split(const __bf16* p, int S, float* v, int mode = 1) {
  const bf16x8 hi = *reinterpret_cast<const bf16x8*>(p), lo = *reinterpret_cast<const bf16x8*>(p + S);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(hi[i]) + static_cast<float>(lo[i]);
  if (mode == 2) {
    const bf16x8 l3 = *reinterpret_cast<const bf16x8*>(p + 2 * S);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += static_cast<float>(l3[i]);
  }
}
__device__ __forceinline__ void loadf8(const float* p, float* v) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = a[i];
    v[i + 4] = b[i];
  }
}

// Raw buffer loads: out-of-range offsets return zeros, so padding / masked lanes need no
// branch (an exec-masked branch per row costs more VALU/SALU than the load itself).
constexpr unsigned kEncOOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t enc_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t r, unsigned voff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}

__device__ __forceinline__ EncClass pick_class(const EncConvArgs& a, int wg, int& ci) {
  ci = 0;
#pragma unroll
  for (int c = 1; c < 4; ++c)
    if (c < a.ncls && wg >= a.cls[c].blk0) ci = c;
  EncClass cl = a.cls[0];
  if (ci == 1) cl = a.cls[1];
  if (ci == 2) cl = a.cls[2];
  if (ci == 3) cl = a.cls[3];
  return cl;
}

// ============================================================================ conv fwd / dgrad
// BM x BN output tile, BK = 64, 256 threads as WM x WN waves, each wave TM x TN MFMA
// 32x32x16 tiles; register-staged double-buffered LDS, one barrier per K step.
template <int BM, int BN, int WM, int WN>
struct EncCfg {
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static constexpr int ACH = BM * EBK / 8 / 256, BCH = BN * EBK / 8 / 256;
  static constexpr int STAGE = (BM + BN) * ELDK;
  static constexpr int RING_BYTES = 2 * STAGE * 2;
  static constexpr int EPI_BYTES = (BM * (BN + 4) + 2 * WM * BN) * 4;
  static constexpr int SMEM = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
  static_assert(TM * 32 * WM == BM && TN * 32 * WN == BN && WM * WN == 4, "tile shape");
  static_assert(ACH * 256 * 8 == BM * EBK && BCH * 256 * 8 == BN * EBK, "staging shape");
};

template <int BM, int BN, int WM, int WN, int NSRC, bool F16 = false>
__global__ __launch_bounds__(256) void enc_conv_kernel(const EncConvArgs a) {
  using C = EncCfg<BM, BN, WM, WN>;
  constexpr int TM = C::TM, TN = C::TN, ACH = C::ACH, BCH = C::BCH, STAGE = C::STAGE;
  __shared__ __attribute__((aligned(16))) char smem_raw[C::SMEM];
  __shared__ int s_tab[kEncTabMax];
  __shared__ int s_out[BM];  // output pixel offset of each tile row (-1: past the grid)
  __bf16* smem = reinterpret_cast<__bf16*>(smem_raw);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (a.tab_ptr)
    for (int e = tid; e < kEncTabMax; e += 256) s_tab[e] = a.tab_ptr[e];
  else
    for (int e = tid; e < kEncTab; e += 256) s_tab[e] = a.tab[e];

  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int ci;
  const EncClass cl = pick_class(a, wg, ci);
  const int local = wg - cl.blk0;
  const int tm = local / a.tilesN, tn = local - (local / a.tilesN) * a.tilesN;
  const int b = tm / cl.tiles_img, tile = tm - (tm / cl.tiles_img) * cl.tiles_img;
  const int GHW = cl.Gh * cl.Gw;
  const int q0 = tile * BM;
  const int n0 = tn * BN;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int kc = tid & 7;
  // grid coordinates of tile row r = (gy0, gx0) + r: one uniform division, then small
  // float-reciprocal divisions (exact after the +-1 fix-up) instead of an integer division per row
  const int gy0 = q0 / cl.Gw, gx0 = q0 - (q0 / cl.Gw) * cl.Gw;
  const float inv_gw = 1.f / (float)cl.Gw;
  auto row_coord = [&](int r, int& gy, int& gx) __attribute__((always_inline)) {
    const int v = gx0 + r;
    int d = (int)((float)v * inv_gw);
    d -= (d * cl.Gw > v) ? 1 : 0;
    d += ((d + 1) * cl.Gw <= v) ? 1 : 0;
    gy = gy0 + d;
    gx = v - d * cl.Gw;
  };
  for (int r = tid; r < BM; r += 256) {
    int off = -1;
    if (q0 + r < GHW) {
      int gy, gx;
      row_coord(r, gy, gx);
      off = ((b * a.Ho + gy * a.os + cl.oy0) * a.Wo + gx * a.os + cl.ox0);
    }
    s_out[r] = off;
  }

  // rows this thread stages, per source: top-left source coordinate of the grid pixel and
  // its 32-bit element offset (rows past the grid get a coordinate that fails every bounds test)
  int sy[NSRC][ACH], sx[NSRC][ACH], sbase[NSRC][ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int q = q0 + (tid >> 3) + 32 * i;
    const bool valid = q < GHW;
    int gy = 0, gx = 0;
    if (valid) row_coord((tid >> 3) + 32 * i, gy, gx);
#pragma unroll
    for (int s2 = 0; s2 < NSRC; ++s2) {
      const EncSrc& S = a.src[s2];
      sy[s2][i] = valid ? gy * S.is : -(1 << 20);
      sx[s2][i] = gx * S.is;
      sbase[s2][i] = ((b * S.H + gy * S.is) * S.W + gx * S.is) * S.stride;
    }
  }
  // weight rows: 32-bit offsets of this thread's chunk column (K offset added per step)
  int wrow[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    const int n = n0 + (tid >> 3) + 32 * i;
    wrow[i] = n < a.N ? n * cl.Kpad + kc * 8 : -1;
  }
  const __bf16* wt = a.wt + cl.wofs;
  const int nk = cl.Kpad / EBK;

  __syncthreads();  // s_tab, s_out

  // two register sets: the global loads of step t+2 are in flight while step t computes
  u32x4 ra[2][ACH], rb[2][BCH];
  __amdgpu_buffer_rsrc_t rs[NSRC];
#pragma unroll
  for (int s2 = 0; s2 < NSRC; ++s2)
    rs[s2] = enc_rsrc(a.src[s2].ptr, (unsigned)((long)a.B * a.src[s2].H * a.src[s2].W * a.src[s2].stride * 2));
  const __amdgpu_buffer_rsrc_t rw = enc_rsrc(wt, (unsigned)((long)a.N * cl.Kpad * 2));
  auto load = [&](int k0, u32x4 (&ra_)[ACH], u32x4 (&rb_)[BCH]) __attribute__((always_inline)) {
    const int ent = s_tab[cl.t0 + (k0 >> 3) + kc];
    const bool ev = ent >= 0;  // -1: zero columns (K padding)
    const int dy = (ent & 0xff) - 128, dx = ((ent >> 8) & 0xff) - 128, c = ent >> 17;
    if constexpr (NSRC == 1) {
      const EncSrc& S = a.src[0];
      const int tapoff = (dy * S.W + dx) * S.stride + c;
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        const bool ok = ev && (unsigned)(sy[0][i] + dy) < (unsigned)S.H && (unsigned)(sx[0][i] + dx) < (unsigned)S.W;
        ra_[i] = bload(rs[0], ok ? (unsigned)(sbase[0][i] + tapoff) * 2u : kEncOOB);
      }
    } else {
      // per-lane source: one load per source, the other one masked out-of-range (zeros)
      const int sidx = (ent >> 16) & 1;
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        u32x4 v = {0, 0, 0, 0};
#pragma unroll
        for (int s2 = 0; s2 < NSRC; ++s2) {
          const EncSrc& S = a.src[s2];
          const int tapoff = (dy * S.W + dx) * S.stride + c;
          const bool ok = ev && sidx == s2 && (unsigned)(sy[s2][i] + dy) < (unsigned)S.H &&
                          (unsigned)(sx[s2][i] + dx) < (unsigned)S.W;
          v |= bload(rs[s2], ok ? (unsigned)(sbase[s2][i] + tapoff) * 2u : kEncOOB);
        }
        ra_[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) rb_[i] = bload(rw, wrow[i] >= 0 ? (unsigned)(wrow[i] + k0) * 2u : kEncOOB);
  };
  auto store = [&](int buf, const u32x4 (&ra_)[ACH], const u32x4 (&rb_)[BCH]) __attribute__((always_inline)) {
    __bf16* sA = smem + buf * STAGE;
    __bf16* sB = sA + BM * ELDK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) *reinterpret_cast<u32x4*>(sA + ((tid >> 3) + 32 * i) * ELDK + kc * 8) = ra_[i];
#pragma unroll
    for (int i = 0; i < BCH; ++i) *reinterpret_cast<u32x4*>(sB + ((tid >> 3) + 32 * i) * ELDK + kc * 8) = rb_[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fk = (lane >> 5) * 8;
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const __bf16* sA = smem + buf * STAGE;
    const __bf16* sB = sA + BM * ELDK;
#pragma unroll
    for (int s = 0; s < EBK / 16; ++s) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(sA + (wm * (BM / WM) + i * 32 + fr) * ELDK + s * 16 + fk);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + (wn * (BN / WN) + j * 32 + fr) * ELDK + s * 16 + fk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mma16<F16>(af[i], bfr[j], acc[i][j]);
    }
  };
  // step t computes LDS buffer t&1; registers: set t&1 receives step t+2, set (t+1)&1 holds
  // step t+1 (stored after the compute); the loop is unrolled by 2 so the sets are static
  load(0, ra[0], rb[0]);
  if (nk > 1) load(EBK, ra[1], rb[1]);
  store(0, ra[0], rb[0]);
  __syncthreads();
  for (int t = 0; t < nk; t += 2) {
    if (t + 2 < nk) load((t + 2) * EBK, ra[0], rb[0]);
    compute(0);
    if (t + 1 < nk) store(1, ra[1], rb[1]);
    __syncthreads();
    if (t + 1 >= nk) break;
    if (t + 3 < nk) load((t + 3) * EBK, ra[1], rb[1]);
    compute(1);
    if (t + 2 < nk) store(0, ra[0], rb[0]);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  const int rows = min(BM, GHW - q0);  // valid rows of this tile
  float* stile = reinterpret_cast<float*>(smem_raw);
  float* sst1 = stile + BM * (BN + 4);
  float* sst2 = sst1 + WM * BN;
  float biasv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
    biasv[j] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
  }
  if (a.stats) {
    // per-column (sum, M2) of this tile's valid rows in one pass: sum and sum of squares,
    // M2 = sq - s^2 / n (n <= BM values per tile: fp32 cancellation is negligible; the
    // tiles are Chan-combined by the finalize kernel)
    const bool full = rows == BM;  // uniform: every tile but the last of an image
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const float v = (full || rl < rows) ? acc[i][j][r] + biasv[j] : 0.f;
          sm += v;
          sq += v * v;
        }
      sm += __shfl_xor(sm, 32, 64);
      sq += __shfl_xor(sq, 32, 64);
      if (lane < 32) {
        sst1[wm * BN + wn * (BN / WN) + j * 32 + lane] = sm;
        sst2[wm * BN + wn * (BN / WN) + j * 32 + lane] = sq;
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        sm += sst1[w * BN + tid];
        sq += sst2[w * BN + tid];
      }
      float* st = a.stats + ((long)(b * cl.tiles_img + tile) * 2) * a.N;
      st[n0 + tid] = sm;
      st[a.N + n0 + tid] = fmaxf(sq - sm * sm / (float)rows, 0.f);
    }
  }
  // stage the tile (+ bias) in LDS, then 16-byte stores of 8 channels per thread
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl_ = wn * (BN / WN) + j * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        stile[rl * (BN + 4) + cl_] = acc[i][j][r] + biasv[j];
      }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int ch = tid; ch < BM * CPR; ch += 256) {
    const int rl = ch / CPR, cc = ch - (ch / CPR) * CPR;
    const int n = n0 + cc * 8;
    if (rl >= rows || n >= a.N) continue;
    const long pix = s_out[rl];
    float v[8];
    const f32x4 lo = *reinterpret_cast<const f32x4*>(stile + rl * (BN + 4) + cc * 8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(stile + rl * (BN + 4) + cc * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = lo[e];
      v[e + 4] = hi[e];
    }
    if (a.res) {
      float r[8];
      if (a.split) load8_split(a.res + pix * a.res_stride + n, a.N, r, a.split);
      else load8(a.res + pix * a.res_stride + n, r, F16);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    if (a.mask) {
      float m[8];
      load8(a.mask + pix * a.mask_stride + n, m, F16);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = m[e] > 0.f ? v[e] : 0.f;
    }
    if (a.split)
      store8_split(a.out + pix * a.out_stride + n, a.N, v, a.split);
    else
      store8(a.out + pix * a.out_stride + n, v, F16);
  }
}

// ============================================================================ weight packing
// out[wofs + row * Kpad + k] (bf16) from fp32 parameters (any strides):
//   forward: row = out channel, column (tap, in channel)   -> W[row][local][ky][kx]
//   dgrad:   row = in channel,  column (conv, tap, out ch) -> W_w[local][row][ky][kx]
__device__ __forceinline__ void pack_row(const EncConvArgs& a, const EncClass& cl, int row, __bf16* out) {
  const int* ptab = a.ptab_ptr ? a.ptab_ptr : a.ptab;
  for (int k = threadIdx.x; k < cl.Kpad; k += 256) {
    const int ent = (k < cl.K) ? ptab[cl.t0 + (k >> 3)] : -1;
    float v = 0.f;
    if (ent >= 0) {
      const int w = ent & 15, ky = (ent >> 4) & 15, kx = (ent >> 8) & 15, loc = (ent >> 12) + (k & 7);
      const float* wp = w ? a.w[1] : a.w[0];
      const long s0 = w ? a.ws[1][0] : a.ws[0][0], s1 = w ? a.ws[1][1] : a.ws[0][1];
      const long s2 = w ? a.ws[1][2] : a.ws[0][2], s3 = w ? a.ws[1][3] : a.ws[0][3];
      const int cin = w ? a.wcin[1] : a.wcin[0];
      if (a.pack_dgrad && a.split_w) {  // split dY rows [hi | lo | hi] of Cout: [W_hi | W_hi | W_lo]
        const int pw = a.split_wd[w] > 0 ? a.split_wd[w] : a.split_w;  // this conv's Cout
        const int plane = loc / pw, co = loc - plane * pw;
        const float x = wp[co * s0 + row * s1 + ky * s2 + kx * s3];
        const float hi = static_cast<float>(static_cast<__bf16>(x));
        v = plane < 2 ? hi : x - hi;
      } else if (a.pack_dgrad) {
        v = wp[loc * s0 + row * s1 + ky * s2 + kx * s3];
      } else if (a.split_w && a.split == 2) {
        // three-plane forward: six K planes (x planes hi, mid, hi, lo, hi, mid -- the decode table
        // -- against W planes H, H, M, H, L, M): every product of relative size >= 2^-16 of
        // hi(x) hi(W), so the GEMM is fp32-exact up to ~2^-24 (fwd_tables in enc_bindings.cpp)
        const int plane = loc / a.split_w, cl = loc - plane * a.split_w;
        if (cl < cin) {
          const float x = wp[row * s0 + cl * s1 + ky * s2 + kx * s3];
          const float H = static_cast<float>(static_cast<__bf16>(x));
          const float M = static_cast<float>(static_cast<__bf16>(x - H));
          const float L = x - H - M;
          v = (plane == 2 || plane == 5) ? M : plane == 4 ? L : H;
        }
      } else if (a.split_w) {  // [W_hi | W_hi | W_lo] against the [hi | lo | hi] input planes
        const int plane = loc / a.split_w, cl = loc - plane * a.split_w;
        if (cl < cin) {
          const float x = wp[row * s0 + cl * s1 + ky * s2 + kx * s3];
          const float hi = static_cast<float>(static_cast<__bf16>(x));
          v = plane < 2 ? hi : x - hi;
        }
      } else if (loc < cin) {
        v = wp[row * s0 + loc * s1 + ky * s2 + kx * s3];
      }
    }
    out[cl.wofs + (long)row * cl.Kpad + k] = st16(v, a.f16 != 0);
  }
}

__global__ __launch_bounds__(256) void enc_pack_kernel(const EncConvArgs a, __bf16* out) {
  const int ci = blockIdx.y;
  EncClass cl = a.cls[0];
  if (ci == 1) cl = a.cls[1];
  if (ci == 2) cl = a.cls[2];
  if (ci == 3) cl = a.cls[3];
  pack_row(a, cl, blockIdx.x, out);
}

// Every conv of an encoder packed by one launch (ops/encoder.py _Prepack): ``plan`` holds
// njobs EncConvArgs (packing fields only), then each job's output offset (long) and first
// workgroup (int, njobs + 1 entries); workgroup = (job, class, row).
__global__ __launch_bounds__(256) void enc_pack_multi_kernel(const unsigned char* plan, int njobs, __bf16* out) {
  const EncConvArgs* jobs = reinterpret_cast<const EncConvArgs*>(plan);
  const long* ofs = reinterpret_cast<const long*>(plan + sizeof(EncConvArgs) * njobs);
  const int* blk0 = reinterpret_cast<const int*>(ofs + njobs);
  const int b = blockIdx.x;
  int j = 0;
  while (j + 1 < njobs && blk0[j + 1] <= b) ++j;
  const EncConvArgs& a = jobs[j];
  const int rows = a.N;
  const int local = b - blk0[j], ci = local / rows, row = local - ci * rows;
  pack_row(a, a.cls[ci], row, out + ofs[j]);
}

// ============================================================================ wgrad
// dW[co][k] = sum_p dY[p][co] * im2col(X)[p][k] over one pixel split.  Both operands are
// staged [pixel][column] (register staged, XOR-swizzled 16-byte chunks) and consumed
// with ds_read_b64_tr_b16 transposed reads (pixels = the MFMA K dimension).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(reinterpret_cast<uintptr_t>(p) & 0xffffffffu));
}
template <int COLS>
__device__ __forceinline__ int wswz(int row, int chunk) {
  return COLS == 128 ? (chunk ^ ((row & 3) << 2)) : (chunk ^ (((row >> 1) & 1) << 2));
}

template <int BM, int BN, bool F16 = false>
__global__ __launch_bounds__(256) void enc_wgrad_kernel(const EncWgradArgs a) {
  // 2x2 waves of (BM/2) x (BN/2): TM x TN MFMA 32x32x16 tiles per wave
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int ACPR = BM / 8, ARP = 256 / ACPR, AI = 64 / ARP;
  constexpr int BCPR = BN / 8, BRP = 256 / BCPR, BI = 64 / BRP;
  constexpr int STAGE = 64 * (BM + BN);
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];

  const int tiles = a.tilesM * a.tilesN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / tiles, t0 = wg - (wg / tiles) * tiles;
  const int tm = t0 / a.tilesN, tn = t0 - (t0 / a.tilesN) * a.tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const long pbeg = (long)split * a.pix_per_split;
  const long pend = min(pbeg + (long)a.pix_per_split, a.P);
  const int nsteps = pend > pbeg ? (int)((pend - pbeg + 63) / 64) : 0;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int ca = tid % ACPR;
  const bool a_ok = m0 + ca * 8 < a.N;
  const int cb = tid % BCPR;
  const int kb = n0 + cb * 8;
  const bool b_ok = kb < a.K;
  int ky = 0, kx = 0, c = 0;
  if (b_ok) {
    const int tap = kb / a.Cx;
    c = kb - tap * a.Cx;
    ky = tap / a.KW;
    kx = tap - ky * a.KW;
  }
  const int HoWo = a.Ho * a.Wo;
  const bool do_db = a.dbslab != nullptr && tn == 0;  // (HoWo: walker initialisation)
  float dbacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) dbacc[e] = 0.f;

  // pixel walkers of this thread's im2col rows (advanced by 64 pixels per step, no divisions
  // in the loop); 32-bit element offsets (host checks every tensor is < 2^31 elements)
  int wp[BI], wb[BI], wy[BI], wx[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int p = (int)pbeg + tid / BCPR + BRP * i;
    wp[i] = p;
    wb[i] = p / HoWo;
    const int rem = p - wb[i] * HoWo;
    wy[i] = rem / a.Wo;
    wx[i] = rem - wy[i] * a.Wo;
  }
  const int kyp = ky - a.pad, kxp = kx - a.pad;
  const int pe = (int)pend;
  const int aoff = m0 + ca * 8;

  u32x4 ra[AI], rb[BI];
  auto load = [&](int step) __attribute__((always_inline)) {
    const int p0 = (int)pbeg + step * 64;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int p = p0 + tid / ACPR + ARP * i;
      ra[i] = (a_ok && p < pe) ? *reinterpret_cast<const u32x4*>(a.dy + (p * a.dy_stride + aoff)) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int y = wy[i] * a.stride + kyp, x = wx[i] * a.stride + kxp;
      const bool ok = b_ok && wp[i] < pe && (unsigned)y < (unsigned)a.Hx && (unsigned)x < (unsigned)a.Wx;
      rb[i] = ok ? *reinterpret_cast<const u32x4*>(a.x + (((wb[i] * a.Hx + y) * a.Wx + x) * a.xstride + c))
                 : u32x4{0, 0, 0, 0};
      wp[i] += 64;
      wx[i] += 64;
      while (wx[i] >= a.Wo) {
        wx[i] -= a.Wo;
        if (++wy[i] >= a.Ho) {
          wy[i] = 0;
          ++wb[i];
        }
      }
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
    __bf16* sA = smem + buf * STAGE;
    __bf16* sB = sA + 64 * BM;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = tid / ACPR + ARP * i;
      *reinterpret_cast<u32x4*>(sA + row * BM + wswz<BM>(row, ca) * 8) = ra[i];
      if (do_db) {
        const bf16x8 v = __builtin_bit_cast(bf16x8, ra[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) dbacc[e] += ld16(v[e], F16);
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = tid / BCPR + BRP * i;
      *reinterpret_cast<u32x4*>(sB + row * BN + wswz<BN>(row, cb) * 8) = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int hh = lane >> 5, gi = (lane >> 4) & 1, q = (lane & 15) >> 2, pq = lane & 3;
  if (nsteps > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int t = 0; t < nsteps; ++t) {
    if (t + 1 < nsteps) load(t + 1);
    const __bf16* sA = smem + (t & 1) * STAGE;
    const __bf16* sB = sA + 64 * BM;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r0 = s * 16 + hh * 8 + q, r1 = r0 + 4;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (BM / 2) + i * 32 + gi * 16 + 4 * pq;
        const s16x4 lo = tr_read(sA + r0 * BM + wswz<BM>(r0, col >> 3) * 8 + (col & 7));
        const s16x4 hi = tr_read(sA + r1 * BM + wswz<BM>(r1, col >> 3) * 8 + (col & 7));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 32 + gi * 16 + 4 * pq;
        const s16x4 lo = tr_read(sB + r0 * BN + wswz<BN>(r0, col >> 3) * 8 + (col & 7));
        const s16x4 hi = tr_read(sB + r1 * BN + wswz<BN>(r1, col >> 3) * 8 + (col & 7));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mma16<F16>(af[i], bfr[j], acc[i][j]);
    }
    if (t + 1 < nsteps) store((t + 1) & 1);
    __syncthreads();
  }

  float* slab = a.slab + (long)split * a.Npad * a.Kpad;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        slab[(long)row * a.Kpad + col] = acc[i][j][r];
      }
  }
  if (a.dbslab != nullptr && tn == 0) {
    // fixed-order reduction of the per-thread column sums (threads sharing a chunk column)
    float* sdb = reinterpret_cast<float*>(smem);  // [ARP][BM]
#pragma unroll
    for (int e = 0; e < 8; ++e) sdb[(tid / ACPR) * BM + ca * 8 + e] = dbacc[e];
    __syncthreads();
    if (tid < BM) {
      float s = 0.f;
      for (int r = 0; r < ARP; ++r) s += sdb[r * BM + tid];
      a.dbslab[(long)split * a.Npad + m0 + tid] = s;
    }
  }
}

// Sum the split slabs in a fixed order into the fp32 parameter gradient (any strides).
// Block = 16 outputs x 16 split lanes (outputs fastest: 64-byte coalesced slab rows); each
// lane sums every 16th split with 4 independent loads in flight, the 16 lane sums are
// combined in a fixed order -- the sum is latency-bound for small weights, so the split
// dimension is spread over threads.  Outputs walk (co, tap, ci).
__global__ __launch_bounds__(256) void enc_wgrad_reduce_kernel(const float* __restrict__ slab, int nsplit, int Npad,
                                                               int Kpad, const float* __restrict__ dbslab,
                                                               float* __restrict__ dw, long s0, long s1, long s2,
                                                               long s3, int Cout, int Cin, int Cx, int KW, int taps,
                                                               float* __restrict__ db, int accumulate, int fold) {
  __shared__ float red[16][17];
  const int o = threadIdx.x & 15, sub = threadIdx.x >> 4;
  const long total = (long)Cout * taps * Cin;
  const long nout = total + (db != nullptr ? Cout : 0);  // bias gradients ride as extra outputs
  const long e = (long)blockIdx.x * 16 + o;
  float s = 0.f;
  const float* src = nullptr;
  long sstride = 0;
  int co = 0, ci = 0, tap = 0;
  if (e < total) {
    ci = (int)(e % Cin);
    const long r = e / Cin;
    tap = (int)(r % taps);
    co = (int)(r / taps);
    src = slab + (long)co * Kpad + (long)tap * Cx + ci;
    sstride = (long)Npad * Kpad;
  } else if (e < nout && dbslab != nullptr) {
    src = dbslab + (e - total);
    sstride = Npad;
  }
  if (src != nullptr) {
    int sp = sub;
    for (; sp + 48 < nsplit; sp += 64) {
      const float v0 = src[sp * sstride], v1 = src[(sp + 16) * sstride];
      const float v2 = src[(sp + 32) * sstride], v3 = src[(sp + 48) * sstride];
      s += (v0 + v1) + (v2 + v3);
    }
    for (; sp < nsplit; sp += 16) s += src[sp * sstride];
    // split-bf16 weight gradient ([X_hi | X_lo]^T dY_hi): the lo-plane columns sit ``fold``
    // channels after the hi-plane ones, the parameter gradient is their sum
    if (fold > 0 && e < total) {
      const float* s2 = src + fold;
      for (sp = sub; sp < nsplit; sp += 16) s += s2[sp * sstride];
    }
  }
  red[sub][o] = s;
  __syncthreads();
  if (sub != 0 || e >= nout) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][o];
  if (e < total) {
    const int ky = tap / KW, kx = tap - (tap / KW) * KW;
    float* d = dw + co * s0 + ci * s1 + ky * s2 + kx * s3;
    *d = accumulate ? *d + t : t;
  } else {
    // no slab: the bias feeds a re-centring norm, its gradient is exactly 0
    float* d = db + (e - total);
    *d = accumulate ? *d + t : t;
  }
}

// ============================================================================ input prep
// out[b][y][x][0..7] = (2 * img / 255 - 1, channels 3..7 zero), bf16; images NCHW-any-strides
// fp32, b < B from img0, b >= B from img1 (the feature encoder's paired batch).
__global__ __launch_bounds__(256) void enc_prep_kernel(const float* __restrict__ i0, const float* __restrict__ i1,
                                                       long sb, long sc, long sh, long sw, int B, int H, int W,
                                                       int nimg, __bf16* __restrict__ out, int split) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)nimg * H * W;
  if (p >= total) return;
  const int b = (int)(p / ((long)H * W));
  const int rem = (int)(p - (long)b * H * W);
  const int y = rem / W, x = rem - (rem / W) * W;
  const float* src = b < B ? i0 + (long)b * sb : i1 + (long)(b - B) * sb;
  const long o = (long)y * sh + (long)x * sw;
  float v[8];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = 2.f * (src[o + c * sc] / 255.f) - 1.f;
#pragma unroll
  for (int c = 3; c < 8; ++c) v[c] = 0.f;
  if (split & 1)
    store8_split(out + p * 24, 8, v, (split & 4) ? 2 : 1);
  else
    store8(out + p * 8, v, (split & 2) != 0);
}

// ============================================================================ norms
// coef layout [B][4][N]: scale, shift (y = a * scale + shift), rstd, mean (xhat = (a - mean) * rstd)
// kinds: 0 none, 1 instance, 2 batch (training statistics), 3 batch (running statistics)


__global__ __launch_bounds__(256) void enc_norm_finalize_kernel(const NormFinArgs a) {
  const int n = blockIdx.x, g = blockIdx.y;  // channel, group (image for instance norm)
  const int tid = threadIdx.x;
  __shared__ float sn[256], sm[256], s2[256];
  float mean = 0.f, var = 1.f;
  if (a.kind == 1 || a.kind == 2) {
    const int b0 = a.kind == 1 ? g : 0, b1 = a.kind == 1 ? g + 1 : a.B;
    const int E = (b1 - b0) * a.T;
    float cn = 0.f, cm = 0.f, cM2 = 0.f;
    for (int e = tid; e < E; e += 256) {
      const int b = b0 + e / a.T, t = e - (e / a.T) * a.T;
      float nb;
      if (a.tile_w > 0) {  // square tiles, row-major over the image
        const int tx_n = (a.img_w + a.tile_w - 1) / a.tile_w, ty = t / tx_n, tx = t - ty * tx_n;
        nb = (float)(min(a.tile_w, a.HW / a.img_w - ty * a.tile_w) * min(a.tile_w, a.img_w - tx * a.tile_w));
      } else {
        nb = (float)min(a.BM, a.HW - t * a.BM);
      }
      const float* st = a.stats + ((long)(b * a.T + t) * 2) * a.N;
      const float mb = st[n] / nb, M2b = st[a.N + n];
      const float nn = cn + nb, d = mb - cm;
      cm += d * nb / nn;
      cM2 += M2b + d * d * cn * nb / nn;
      cn = nn;
    }
    sn[tid] = cn;
    sm[tid] = cm;
    s2[tid] = cM2;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (tid < off) {
        const float na = sn[tid], nb = sn[tid + off];
        const float nn = na + nb;
        if (nb > 0.f) {
          const float d = sm[tid + off] - sm[tid];
          sm[tid] += d * nb / nn;
          s2[tid] += s2[tid + off] + d * d * na * nb / nn;
          sn[tid] = nn;
        }
      }
      __syncthreads();
    }
    mean = sm[0];
    var = s2[0] / sn[0];
    if (tid == 0 && a.kind == 2 && a.rmean) {
      const float cnt = sn[0];
      a.rmean[n] = (1.f - a.momentum) * a.rmean[n] + a.momentum * mean;
      a.rvar[n] = (1.f - a.momentum) * a.rvar[n] + a.momentum * var * cnt / fmaxf(cnt - 1.f, 1.f);
      if (n == 0 && a.nbt) *a.nbt += 1;
    }
  } else if (a.kind == 3) {
    mean = a.rmean[n];
    var = a.rvar[n];
  }
  if (tid != 0) return;
  float scale = 1.f, shift = 0.f, rstd = 1.f;
  if (a.kind != 0) {
    rstd = rsqrtf(var + a.eps);
    const float gm = a.gamma ? a.gamma[n] : 1.f, bt = a.beta ? a.beta[n] : 0.f;
    scale = gm * rstd;
    shift = bt - mean * scale;
  } else {
    mean = 0.f;
  }
  const int b0 = a.kind == 1 ? g : 0, b1 = a.kind == 1 ? g + 1 : a.B;
  for (int b = b0; b < b1; ++b) {
    float* c = a.coef + (long)b * 4 * a.N;
    c[n] = scale;
    c[a.N + n] = shift;
    c[2 * a.N + n] = rstd;
    c[3 * a.N + n] = mean;
  }
}

// y = relu_out( f(a) + g(r) ),  f(a) = [relu](a * scale + shift),  g(r) = r * scale_r + shift_r | r | 0
// Per-pixel elementwise passes (norm apply, norm backward apply): every thread keeps ONE
// 8-channel chunk (n = tid % G) and walks pixels with a fixed stride, so the per-image
// coefficient vectors stay in registers (reloaded only when the image changes) instead of
// ~10-20 cached 16-byte coefficient loads and a 64-bit division per chunk.
struct PixWalk {
  int n, p, stride;  // channel offset, first pixel, pixel stride (-1 p: idle thread)
};
__device__ __forceinline__ PixWalk pix_walk(int G) {
  const int ppb = 256 / G;  // pixel lanes per block (threads >= ppb * G idle)
  const int t = threadIdx.x;
  PixWalk w;
  w.n = (t % G) * 8;
  w.p = t < ppb * G ? blockIdx.x * ppb + t / G : -1;
  w.stride = gridDim.x * ppb;
  return w;
}

// SPL: split-bf16 rows (fp32 training) -- one code path per instantiation keeps the bf16 /
// fp16 kernel's registers (and so its occupancy) free of the split path's
template <bool SPL>
__global__ __launch_bounds__(256) void enc_apply_kernel(const __bf16* __restrict__ a, const float* __restrict__ ca,
                                                        int relu_a, const __bf16* __restrict__ r,
                                                        const float* __restrict__ cr, int relu_out,
                                                        __bf16* __restrict__ out, int B, int HW, int N, int split) {
  const int G = N / 8;
  const bool f16 = (split & 2) != 0;
  const int mode = (split & 4) ? 2 : 1;  // split-plane mode (store8_split)
  const int rs = SPL ? 3 * N : N;  // row stride: split rows hold three planes
  const PixWalk w = pix_walk(G);
  if (w.p < 0) return;
  const int n = w.n, P = B * HW;
  int b = -1, bend = 0;
  float s[8], t[8], s2[8], t2[8];
  for (int p = w.p; p < P; p += w.stride) {
    if (p >= bend) {  // next image: its coefficients
      b = p / HW;
      bend = (b + 1) * HW;
      loadf8(ca + (long)b * 4 * N + n, s);
      loadf8(ca + (long)b * 4 * N + N + n, t);
      if (r && cr) {
        loadf8(cr + (long)b * 4 * N + n, s2);
        loadf8(cr + (long)b * 4 * N + N + n, t2);
      }
    }
    float v[8];
    if (SPL)
      load8_split(a + (long)p * rs + n, N, v, mode);
    else
      load8(a + (long)p * N + n, v, f16);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = v[e] * s[e] + t[e];
      if (relu_a) v[e] = fmaxf(v[e], 0.f);
    }
    if (r) {
      float rv[8];
      if (SPL)
        load8_split(r + (long)p * rs + n, N, rv, mode);
      else
        load8(r + (long)p * N + n, rv, f16);
      if (cr)
#pragma unroll
        for (int e = 0; e < 8; ++e) rv[e] = rv[e] * s2[e] + t2[e];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rv[e];
    }
    if (relu_out)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    if (SPL)
      store8_split(out + (long)p * rs + n, N, v, mode);
    else
      store8(out + (long)p * N + n, v, f16);
  }
}

// Norm backward, pass 1: per (image, chunk) partial sums over pixels of
//   branch 0: dy0 = g * [a0 * scale0 + shift0 > 0 if relu0],  S1 = sum dy0, S2 = sum dy0 * xhat0
//   branch 1: dy1 = g,                                           S1, S2 with xhat1
// part [B][R][4][N] (no atomics; fixed reduction order).


// MODE: 0 bf16, 1 fp16, 2 split-bf16 rows (one code path per instantiation)
template <int MODE>
__global__ __launch_bounds__(256) void enc_norm_bwd_reduce_kernel(const NormBwdArgs a) {
  __shared__ float red[8 * (256 + 32)];
  const int r = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int N = a.N, G = N / 8, PPB = 256 / G;
  // element-e block pitch: the partials of one element occupy PPB x G words; padding the pitch
  // to (a multiple of 64 banks) + G puts the G-lane groups of different elements read by one
  // instruction on different banks (the unpadded 256-word pitch read N = 64 4-way conflicted)
  const int EP = (PPB * G + 63) / 64 * 64 + G;
  const int cg = tid % G, pr = tid / G;
  const bool active = pr < PPB;
  const int n = cg * 8;
  const int chunk = (a.HW + a.R - 1) / a.R;
  const long rs = MODE == 2 ? 3L * N : N;  // row pitch (split rows: hi / lo / hi planes of N)
  const int pb = r * chunk, pe = min(a.HW, pb + chunk);
  auto ld8 = [&](const __bf16* q, float* v) __attribute__((always_inline)) {
    if constexpr (MODE == 2) load8_split(q, N, v, a.split);
    else load8(q, v, MODE == 1);
  };
  float S[4][8];
#pragma unroll
  for (int qd = 0; qd < 4; ++qd)
#pragma unroll
    for (int e = 0; e < 8; ++e) S[qd][e] = 0.f;
  if (active) {
    // the rstd factor of S2 is applied once after the loop (fewer live registers in it)
    float sc0[8], sh0[8], mu0[8], mu1[8];
    const float* c0 = a.c0 + (long)b * 4 * N;
    loadf8(c0 + n, sc0);
    loadf8(c0 + N + n, sh0);
    loadf8(c0 + 3 * N + n, mu0);
    if (a.a1) {
      const float* c1 = a.c1 + (long)b * 4 * N;
      loadf8(c1 + 3 * N + n, mu1);
    }
    const long base = (long)b * a.HW;
    // two pixels per iteration: all of their loads are issued before the math
    for (int p = pb + pr; p < pe; p += 2 * PPB) {
      const bool two = p + PPB < pe;
      float gv[2][8], av[2][8], dv[2][8];
      ld8(a.g + (base + p) * rs + n, gv[0]);
      ld8(a.a0 + (base + p) * rs + n, av[0]);
      if (a.a1) ld8(a.a1 + (base + p) * rs + n, dv[0]);
      if (two) {
        ld8(a.g + (base + p + PPB) * rs + n, gv[1]);
        ld8(a.a0 + (base + p + PPB) * rs + n, av[1]);
        if (a.a1) ld8(a.a1 + (base + p + PPB) * rs + n, dv[1]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dy = (a.relu0 && !(av[u][e] * sc0[e] + sh0[e] > 0.f)) ? 0.f : gv[u][e];
          S[0][e] += dy;
          S[1][e] += dy * (av[u][e] - mu0[e]);
        }
        if (a.a1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            S[2][e] += gv[u][e];
            S[3][e] += gv[u][e] * (dv[u][e] - mu1[e]);
          }
        }
      }
    }
    float rs[8];
    loadf8(c0 + 2 * N + n, rs);
#pragma unroll
    for (int e = 0; e < 8; ++e) S[1][e] *= rs[e];
    if (a.a1) {
      loadf8(a.c1 + (long)b * 4 * N + 2 * N + n, rs);
#pragma unroll
      for (int e = 0; e < 8; ++e) S[3][e] *= rs[e];
    }
  }
  const int nq = a.a1 ? 4 : 2;
  for (int qd = 0; qd < nq; ++qd) {
    // layout [e][pr][cg]: consecutive lanes (consecutive cg) hit consecutive banks
    if (active)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[e * EP + pr * G + cg] = S[qd][e];
    __syncthreads();
    if (tid < N) {
      // lane -> (chunk tc, element te) with the chunk fastest, so the 64 lanes of a read read
      // consecutive words (the element-fastest order put 8 lanes 256 words apart on one bank)
      const int tc = tid % G, te = tid / G;
      float s = 0.f;
      for (int k = 0; k < PPB; ++k) s += red[te * EP + k * G + tc];
      a.part[(((long)b * a.R + r) * 4 + qd) * N + tc * 8 + te] = s;
    }
    __syncthreads();
  }
}

// pass 2: coefficients per (group, channel) and the BatchNorm parameter gradients.
// Block = (group, 16-channel chunk); 16 threads per channel split the (image, chunk)
// partials (independent loads in flight), combined in LDS in a fixed order.
__global__ __launch_bounds__(256) void enc_norm_bwd_finalize_kernel(const NormBwdArgs a) {
  __shared__ float red[4][16][17];
  const int N = a.N;
  const int nb = a.a1 ? 2 : 1;
  const int c16 = threadIdx.x & 15, sub = threadIdx.x >> 4;
  const int g = blockIdx.x, n = blockIdx.y * 16 + c16;
  const int b0 = a.kind == 1 ? g : 0, b1 = a.kind == 1 ? g + 1 : a.B;
  const int E = (b1 - b0) * a.R;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    for (int e = sub; e < E; e += 16) {
      const float* pp = a.part + ((long)(b0 * a.R + e) * 4) * N + n;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < 2 * nb) acc[q] += pp[q * N];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[q][sub][c16] = acc[q];
  __syncthreads();
  if (sub != 0 || n >= N) return;
  const float M = (float)(b1 - b0) * a.HW;
  for (int j = 0; j < nb; ++j) {
    float S1 = 0.f, S2 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      S1 += red[2 * j][k][c16];
      S2 += red[2 * j + 1][k][c16];
    }
    const float* c = (j ? a.c1 : a.c0) + (long)b0 * 4 * N;
    const float scale = c[n];
    float k1 = scale, k2 = 0.f, k3 = 0.f;
    if (a.kind == 1 || a.kind == 2) {
      k2 = -scale * S2 / M;
      k3 = -scale * S1 / M;
    }
    if (a.kind == 0) k1 = 1.f;
    for (int b = b0; b < b1; ++b) {
      float* bc = a.bcoef + ((long)b * 2 + j) * 3 * N;
      bc[n] = k1;
      bc[N + n] = k2;
      bc[2 * N + n] = k3;
    }
    if ((a.kind == 2 || a.kind == 3) && a.dgamma[j]) {
      a.dgamma[j][n] = S2;
      a.dbeta[j][n] = S1;
    }
  }
}

// pass 3: da_j = k1 * dy_j + k2 * xhat_j + k3, as k1 * dy_j + A_j * a_j + C_j with
// A = k2 * rstd, C = k3 - A * mean folded per image (five coefficient vectors per branch held
// across the pixel loop put the kernel at 173 VGPRs, two waves per SIMD, on a streaming pass)
// MODE: 0 bf16, 1 fp16, 2 split-bf16 rows; TWO: the second (downsample) branch -- one code
// path per instantiation, so the one-branch kernels do not carry the second's coefficients
template <int MODE, bool TWO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TWO || MODE == 2 ? 1 : 5)))
void enc_norm_bwd_apply_kernel(const NormBwdArgs a) {
  const int N = a.N, G = N / 8;
  const PixWalk w = pix_walk(G);
  if (w.p < 0) return;
  const int n = w.n, P = a.B * a.HW;
  const long rp = MODE == 2 ? 3L * N : N;  // row pitch (split rows: hi / lo / hi planes of N)
  auto ld8 = [&](const __bf16* q, float* v) __attribute__((always_inline)) {
    if constexpr (MODE == 2) load8_split(q, N, v, a.split);
    else load8(q, v, MODE == 1);
  };
  auto st8 = [&](__bf16* q, const float* v) __attribute__((always_inline)) {
    if constexpr (MODE == 2) store8_split(q, N, v, a.split);
    else store8(q, v, MODE == 1);
  };
  // k, A, C of branch j at j * 3 + {0, 1, 2}; loaded per image
  auto coefs = [&](int b, int j, float* k, float* A, float* Cc) __attribute__((always_inline)) {
    const float* cj = (j ? a.c1 : a.c0) + (long)b * 4 * N;
    const float* bc = a.bcoef + ((long)b * 2 + j) * 3 * N;
    float k2[8], k3[8], rs[8], mu[8];
    loadf8(bc + n, k);
    loadf8(bc + N + n, k2);
    loadf8(bc + 2 * N + n, k3);
    loadf8(cj + 2 * N + n, rs);
    loadf8(cj + 3 * N + n, mu);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      A[e] = k2[e] * rs[e];
      Cc[e] = k3[e] - A[e] * mu[e];
    }
  };
  int bend = 0;
  float k1[8], A1[8], C1[8], sc[8], sh[8];
  float q1[8], A2[8], C2[8];
  for (int p = w.p; p < P; p += w.stride) {
    if (p >= bend) {  // next image: its coefficients
      const int b = p / a.HW;
      bend = (b + 1) * a.HW;
      coefs(b, 0, k1, A1, C1);
      if (a.relu0) {
        const float* c0 = a.c0 + (long)b * 4 * N;
        loadf8(c0 + n, sc);
        loadf8(c0 + N + n, sh);
      }
      if constexpr (TWO) coefs(b, 1, q1, A2, C2);
    }
    float gv[8], av[8], o[8];
    ld8(a.g + (long)p * rp + n, gv);
    ld8(a.a0 + (long)p * rp + n, av);
    if (a.relu0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dy = (av[e] * sc[e] + sh[e] > 0.f) ? gv[e] : 0.f;
        o[e] = k1[e] * dy + A1[e] * av[e] + C1[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = k1[e] * gv[e] + A1[e] * av[e] + C1[e];
    }
    st8(a.out0 + (long)p * rp + n, o);
    if constexpr (TWO) {
      ld8(a.a1 + (long)p * rp + n, av);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = q1[e] * gv[e] + A2[e] * av[e] + C2[e];
      st8(a.out1 + (long)p * rp + n, o);
    }
  }
}

// blocks of a PixWalk launch: 256 / (N / 8) pixel lanes per block, at most 4096 blocks
int grid_pix(int B, int HW, int N) {
  const long ppb = 256 / (N / 8);
  const long g = ((long)B * HW + ppb - 1) / ppb;
  return (int)std::min<long>(std::max<long>(g, 1), 4096);
}

int grid_for(long chunks) {
  const long g = (chunks + 255) / 256;
  return (int)std::min<long>(std::max<long>(g, 1), 4096);
}

}  // namespace

// ============================================================================ launchers
// Tile configurations by output-channel count.
enum EncTile : int { kT128x128 = 0, kT128x96 = 1, kT128x64 = 2, kT128x32 = 3 };

// ============================================================================ 3x3 conv, resident weights
// The 3x3 / stride-1 convs with 64 input and 64 output channels (stage 1 of both encoders,
// at H/2 x W/2: the largest convs of a training step, forward and data gradient) on a
// persistent workgroup per CU that keeps the whole packed weight matrix [64][576] in LDS
// (73.7 KB, loaded once) and walks 16x16-pixel output tiles.  A tile's 18x18 halo block
// (64 channels, 41 KB) is DMA'd (buffer_load ... lds; out-of-image pixels load as zeros, so
// the padding needs no masking) into one of two LDS buffers while the previous tile
// computes, and all 9 taps read their A fragments from it at a row shift: each input pixel
// is fetched once per tile instead of once per tap (the register-staged kernel above
// re-gathers the im2col rows of every tap: VALU-bound at ~18 VALU per MFMA).
// 8 waves x (32 pixels x 64 channels), v_mfma_f32_32x32x16_bf16; 3 barriers per tile.
// Epilogue as enc_conv_kernel: + bias, per-tile (sum, M2) statistics, + residual,
// ReLU' mask, bf16 store (staged through the finished halo buffer).
namespace {

constexpr int C3_T = kEnc3Tile;           // output tile side
constexpr int C3_B = C3_T + 2;            // halo block side
constexpr int C3_ROWS = C3_B * C3_B;      // halo pixels (128-byte rows of 64 channels)
constexpr int C3_PIECES = (C3_ROWS * 128 + 1023) / 1024;  // 1 KB DMA pieces per halo block
constexpr int C3_HALO = C3_PIECES * 1024;  // halo buffer bytes (whole pieces)
constexpr int C3_WB = 64 * 576 * 2;        // resident weights
constexpr int C3_LDS = C3_WB + 2 * C3_HALO;
constexpr int C3_SP = 72;                  // bf16 pitch of the staged output tile
constexpr unsigned C3_OOB = 0x80000000u;
static_assert(C3_T * C3_T * C3_SP * 2 + 2 * 8 * 64 * 4 <= C3_HALO, "epilogue staging must fit a halo buffer");
static_assert(C3_LDS <= 160 * 1024, "LDS budget");

typedef __attribute__((address_space(3))) void c3_lds_void;
typedef __attribute__((address_space(3))) bf16x8 c3_lds_bf16x8;

__device__ __forceinline__ int c3swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// MFMA row m (0..31) of a wave -> its pixel (0..31) of the wave's two tile rows.  ds_read_b128
// serves a wave in four 16-lane groups, {0-3, 12-15, 20-27} and {4-11, 16-19, 28-31} (+ 32); with
// the natural map (pixel = m) a group spans px 0-3 / 12-15 of one tile row and px 4-11 of the
// next, whose halo rows collide modulo 16 (the swizzle's period) -- ~1 extra LDS cycle per A
// read.  Mapping each group onto one tile row (16 consecutive halo rows) makes it conflict-free.
__device__ __forceinline__ int c3_pix(int m) {
  if (m < 4) return m;               // group 0: px 0-3
  if (m < 12) return 16 + (m - 4);   // group 1: px 0-7 of the second row
  if (m < 16) return 4 + (m - 12);   // group 0: px 4-7
  if (m < 20) return 24 + (m - 16);  // group 1: px 8-11
  if (m < 28) return 8 + (m - 20);   // group 0: px 8-15
  return 28 + (m - 28);              // group 1: px 12-15
}

__device__ __forceinline__ void c3_dma16(__amdgpu_buffer_rsrc_t r, unsigned lds_byte, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (c3_lds_void*)(uintptr_t)lds_byte, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 c3_read16(unsigned lds_byte) { return *(const c3_lds_bf16x8*)(uintptr_t)lds_byte; }

template <bool F16 = false>
__global__ __launch_bounds__(512) void enc_conv3_kernel(const EncConvArgs a, int ntiles, int tiles_x,
                                                        int tiles_img) {
  extern __shared__ __attribute__((aligned(1024))) char c3smem[];
  const unsigned lds0 = (unsigned)(reinterpret_cast<uintptr_t>(c3smem) & 0xffffffffu);
  const unsigned ldsW = lds0, ldsH = lds0 + C3_WB;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.src[0].H, W = a.src[0].W;
  const __amdgpu_buffer_rsrc_t rx = enc_rsrc(a.src[0].ptr, (unsigned)((long)a.B * H * W * 128));
  const __amdgpu_buffer_rsrc_t rw = enc_rsrc(a.wt, (unsigned)C3_WB);
  // halo-row shift of each tap (taps in decode-table order = packed-weight order)
  int tshift[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ent = a.tab[a.cls[0].t0 + t * 8];
    tshift[t] = ((ent & 0xff) - 127) * C3_B + (((ent >> 8) & 0xff) - 127);
  }

  // weights -> LDS once: [64 rows][72 chunks], chunk index XOR-swizzled within each tap
#pragma unroll 1
  for (int q = wave; q < C3_WB / 1024; q += 8) {
    const int pos = q * 1024 + lane * 16;
    const int n = pos / 1152, pc = (pos - n * 1152) >> 4;
    const int j = (pc & ~7) | c3swz(n, pc & 7);
    c3_dma16(rw, ldsW + q * 1024, (unsigned)(n * 576 + j * 8) * 2u);
  }
  auto load_halo = [&](int tile, int buf) __attribute__((always_inline)) {
    const int b = tile / tiles_img, tr = tile - b * tiles_img;
    const int ty = tr / tiles_x;
    const int y0 = ty * C3_T - 1, x0 = (tr - ty * tiles_x) * C3_T - 1;
#pragma unroll 1
    for (int q = wave; q < C3_PIECES; q += 8) {
      const int pos = q * 1024 + lane * 16;
      const int r = pos >> 7, pc = (pos >> 4) & 7;
      const int hy = r / C3_B, hx = r - hy * C3_B;
      const int y = y0 + hy, x = x0 + hx;
      const bool ok = r < C3_ROWS && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      const unsigned voff = ok ? (unsigned)((((b * H + y) * W + x) << 6) + c3swz(r, pc) * 8) * 2u : C3_OOB;
      c3_dma16(rx, ldsH + buf * C3_HALO + q * 1024, voff);
    }
  };

  // fragment geometry: this lane's pixel (py, px) of the tile and its 64-channel half
  const int lh = lane >> 5;
  const int pm = c3_pix(lane & 31);
  const int py = 2 * wave + (pm >> 4), px = pm & 15;
  const int hb = py * C3_B + px;  // halo row of the pixel at tap (0, 0) offset (-1, -1)
  const int n0 = lane & 31;       // B columns n0 and n0 + 32
  const unsigned wrow = ldsW + n0 * 1152;
  unsigned bsw[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) bsw[s2] = (unsigned)(c3swz(n0, s2 * 2 + lh) << 4);
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias[j] = a.bias ? a.bias[n0 + 32 * j] : 0.f;

  int tile = blockIdx.x;
  if (tile < ntiles) load_halo(tile, 0);
#pragma unroll 1
  for (int it = 0; tile < ntiles; tile += gridDim.x, ++it) {
    const int cur = it & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // halo (+ weights) landed; the previous tile's epilogue is done with its buffer
    if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x, cur ^ 1);
    const unsigned hbuf = ldsH + cur * C3_HALO;

    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int row = hb + tshift[t];
      const unsigned abase = hbuf + (unsigned)row * 128u;
      const int sw = (row >> 1) & 7;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const bf16x8 fa = c3_read16(abase + (unsigned)(((s2 * 2 + lh) ^ sw) << 4));
        const bf16x8 fb0 = c3_read16(wrow + t * 128 + bsw[s2]);
        const bf16x8 fb1 = c3_read16(wrow + 32 * 1152 + t * 128 + bsw[s2]);
        acc[0] = mma16<F16>(fa, fb0, acc[0]);
        acc[1] = mma16<F16>(fa, fb1, acc[1]);
      }
    }

    // ---- epilogue
    const int b = tile / tiles_img, tr = tile - b * tiles_img;
    const int ty = tr / tiles_x;
    const int oy = ty * C3_T, ox = (tr - ty * tiles_x) * C3_T;
    const int vh = min(C3_T, H - oy), vw = min(C3_T, W - ox);  // valid rows / columns of the tile
    __syncthreads();  // every wave is done reading the halo buffer: reuse it for staging
    __bf16* stg = reinterpret_cast<__bf16*>(c3smem + C3_WB + cur * C3_HALO);
    float* sst = reinterpret_cast<float*>(c3smem + C3_WB + cur * C3_HALO + C3_T * C3_T * C3_SP * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = wave * 32 + c3_pix((r & 3) + 8 * (r >> 2) + 4 * lh);  // tile pixel of this element
        const float v = acc[j][r] + bias[j];
        const bool valid = (i >> 4) < vh && (i & 15) < vw;
        sm += valid ? v : 0.f;
        sq += valid ? v * v : 0.f;
        stg[i * C3_SP + n0 + 32 * j] = st16(v, F16);
      }
      if (a.stats) {
        sm += __shfl_xor(sm, 32, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (lane < 32) {
          sst[wave * 64 + n0 + 32 * j] = sm;
          sst[512 + wave * 64 + n0 + 32 * j] = sq;
        }
      }
    }
    __syncthreads();
    if (a.stats && tid < 64) {
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        sm += sst[w * 64 + tid];
        sq += sst[512 + w * 64 + tid];
      }
      float* st = a.stats + ((long)(b * tiles_img + tr) * 2) * 64;
      st[tid] = sm;
      st[64 + tid] = fmaxf(sq - sm * sm / (float)(vh * vw), 0.f);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = tid + 512 * k;
      const int i = idx >> 3, c8 = (idx & 7) * 8;
      const int yy = i >> 4, xx = i & 15;
      if (yy >= vh || xx >= vw) continue;
      const long pix = ((long)b * a.Ho + oy + yy) * a.Wo + ox + xx;
      const bf16x8 sv = *reinterpret_cast<const bf16x8*>(stg + i * C3_SP + c8);
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ld16(sv[e], F16);
      if (a.res) {
        float r8[8];
        load8(a.res + pix * a.res_stride + c8, r8, F16);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r8[e];
      }
      if (a.mask) {
        float m8[8];
        load8(a.mask + pix * a.mask_stride + c8, m8, F16);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = m8[e] > 0.f ? v[e] : 0.f;
      }
      store8(a.out + pix * a.out_stride + c8, v, F16);
    }
  }
}

}  // namespace

int enc_tile_bn(int N) {
  if (N % 128 == 0) return 128;
  if (N == 96) return 96;
  if (N % 64 == 0) return 64;
  if (N <= 32) return 32;
  return 64;
}
constexpr int kEncBM = 128;

hipError_t launch_enc_pack(const EncConvArgs& a, int rows, void* out, hipStream_t s) {
  hipLaunchKernelGGL(enc_pack_kernel, dim3(rows, a.ncls), dim3(256), 0, s, a, static_cast<__bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_enc_pack_multi(const void* plan, int njobs, int nblocks, void* out, hipStream_t s) {
  hipLaunchKernelGGL(enc_pack_multi_kernel, dim3(nblocks), dim3(256), 0, s, static_cast<const unsigned char*>(plan),
                     njobs, static_cast<__bf16*>(out));
  return hipGetLastError();
}

template <int NSRC, bool F16>
void launch_enc_conv_n(const EncConvArgs& a, int nblocks, hipStream_t s) {
  switch (enc_tile_bn(a.N)) {
    case 128:
      hipLaunchKernelGGL((enc_conv_kernel<128, 128, 2, 2, NSRC, F16>), dim3(nblocks), dim3(256), 0, s, a);
      break;
    case 96:
      hipLaunchKernelGGL((enc_conv_kernel<128, 96, 4, 1, NSRC, F16>), dim3(nblocks), dim3(256), 0, s, a);
      break;
    case 64:
      hipLaunchKernelGGL((enc_conv_kernel<128, 64, 2, 2, NSRC, F16>), dim3(nblocks), dim3(256), 0, s, a);
      break;
    default:
      hipLaunchKernelGGL((enc_conv_kernel<128, 32, 4, 1, NSRC, F16>), dim3(nblocks), dim3(256), 0, s, a);
      break;
  }
}

hipError_t launch_enc_conv3(const EncConvArgs& a, hipStream_t s) {
  static int num_cu = 0;
  static bool lds_set = false;
  if (!num_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || num_cu <= 0)
      num_cu = 256;
  }
  if (!lds_set) {
    (void)hipFuncSetAttribute((const void*)enc_conv3_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, C3_LDS);
    (void)hipFuncSetAttribute((const void*)enc_conv3_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, C3_LDS);
    lds_set = true;
  }
  const int tiles_x = (a.Wo + C3_T - 1) / C3_T, tiles_img = tiles_x * ((a.Ho + C3_T - 1) / C3_T);
  const int ntiles = a.B * tiles_img;
  if (ntiles == 0) return hipSuccess;
  const int grid = std::min(ntiles, num_cu);
  if (a.f16)
    hipLaunchKernelGGL(enc_conv3_kernel<true>, dim3(grid), dim3(512), C3_LDS, s, a, ntiles, tiles_x, tiles_img);
  else
    hipLaunchKernelGGL(enc_conv3_kernel<false>, dim3(grid), dim3(512), C3_LDS, s, a, ntiles, tiles_x, tiles_img);
  return hipGetLastError();
}

hipError_t launch_enc_conv(const EncConvArgs& a, int nblocks, hipStream_t s) {
  if (a.src[1].ptr != nullptr)
    a.f16 ? launch_enc_conv_n<2, true>(a, nblocks, s) : launch_enc_conv_n<2, false>(a, nblocks, s);
  else
    a.f16 ? launch_enc_conv_n<1, true>(a, nblocks, s) : launch_enc_conv_n<1, false>(a, nblocks, s);
  return hipGetLastError();
}

hipError_t launch_enc_wgrad(const EncWgradArgs& a, int BM, int BN, hipStream_t s) {
  const int nwg = a.nsplit * a.tilesM * a.tilesN;
  auto go = [&](auto f16c) {
    constexpr bool F = decltype(f16c)::value;
    if (BM == 128 && BN == 128)
      hipLaunchKernelGGL((enc_wgrad_kernel<128, 128, F>), dim3(nwg), dim3(256), 0, s, a);
    else if (BM == 128)
      hipLaunchKernelGGL((enc_wgrad_kernel<128, 64, F>), dim3(nwg), dim3(256), 0, s, a);
    else if (BN == 128)
      hipLaunchKernelGGL((enc_wgrad_kernel<64, 128, F>), dim3(nwg), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((enc_wgrad_kernel<64, 64, F>), dim3(nwg), dim3(256), 0, s, a);
  };
  if (a.f16) go(std::true_type{});
  else go(std::false_type{});
  return hipGetLastError();
}

hipError_t launch_enc_wgrad_reduce(const float* slab, int nsplit, int Npad, int Kpad, const float* dbslab, float* dw,
                                   const long* ws, int Cout, int Cin, int Cx, int KH, int KW, float* db,
                                   bool accumulate, int fold, hipStream_t s) {
  const long total = (long)Cout * KH * KW * Cin + (db != nullptr ? Cout : 0);
  const int blocks = (int)std::max<long>((total + 15) / 16, 1);
  hipLaunchKernelGGL(enc_wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, slab, nsplit, Npad, Kpad, dbslab, dw,
                     ws[0], ws[1], ws[2], ws[3], Cout, Cin, Cx, KW, KH * KW, db, accumulate ? 1 : 0, fold);
  return hipGetLastError();
}

hipError_t launch_enc_prep(const float* i0, const float* i1, const long* st, int B, int H, int W, int nimg,
                           void* out, int split, hipStream_t s) {
  const long total = (long)nimg * H * W;
  hipLaunchKernelGGL(enc_prep_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, i0, i1, st[0], st[1],
                     st[2], st[3], B, H, W, nimg, static_cast<__bf16*>(out), split);
  return hipGetLastError();
}

hipError_t launch_enc_norm_finalize(const NormFinArgs& a, hipStream_t s) {
  const int groups = a.kind == 1 ? a.B : 1;
  hipLaunchKernelGGL(enc_norm_finalize_kernel, dim3(a.N, groups), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_enc_apply(const void* a, const float* ca, bool relu_a, const void* r, const float* cr,
                            bool relu_out, void* out, int B, int HW, int N, int split, hipStream_t s) {
  if (N % 8 != 0 || N / 8 > 256 || (long)B * HW >= (1L << 31)) return hipErrorInvalidValue;
  if (split & 1)
    hipLaunchKernelGGL(enc_apply_kernel<true>, dim3(grid_pix(B, HW, N)), dim3(256), 0, s,
                       static_cast<const __bf16*>(a), ca, relu_a ? 1 : 0, static_cast<const __bf16*>(r), cr,
                       relu_out ? 1 : 0, static_cast<__bf16*>(out), B, HW, N, split);
  else
    hipLaunchKernelGGL(enc_apply_kernel<false>, dim3(grid_pix(B, HW, N)), dim3(256), 0, s,
                       static_cast<const __bf16*>(a), ca, relu_a ? 1 : 0, static_cast<const __bf16*>(r), cr,
                       relu_out ? 1 : 0, static_cast<__bf16*>(out), B, HW, N, split);
  return hipGetLastError();
}

hipError_t launch_enc_norm_bwd_stages(const NormBwdArgs& a, int stages, int b_fin, hipStream_t s) {
  if (stages & 1) {
    const dim3 g(a.R, a.B);
    if (a.split) hipLaunchKernelGGL(enc_norm_bwd_reduce_kernel<2>, g, dim3(256), 0, s, a);
    else if (a.f16) hipLaunchKernelGGL(enc_norm_bwd_reduce_kernel<1>, g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(enc_norm_bwd_reduce_kernel<0>, g, dim3(256), 0, s, a);
    RAFT_HIP_CHECK(hipGetLastError());
  }
  if (stages & 2) {
    // synchronized BatchNorm: the finalize runs over the partial sums of every rank's images
    // (a.part holds b_fin images' partials, bcoef b_fin rows); the apply below uses a.B
    NormBwdArgs f = a;
    if (b_fin > 0) f.B = b_fin;
    const int groups = f.kind == 1 ? f.B : 1;
    hipLaunchKernelGGL(enc_norm_bwd_finalize_kernel, dim3(groups, (f.N + 15) / 16), dim3(256), 0, s, f);
    RAFT_HIP_CHECK(hipGetLastError());
  }
  if (stages & 4) {
    if (a.N % 8 != 0 || a.N / 8 > 256 || (long)a.B * a.HW >= (1L << 31)) return hipErrorInvalidValue;
    const dim3 g(grid_pix(a.B, a.HW, a.N));
    const bool two = a.a1 != nullptr;
    if (a.split && two) hipLaunchKernelGGL((enc_norm_bwd_apply_kernel<2, true>), g, dim3(256), 0, s, a);
    else if (a.split) hipLaunchKernelGGL((enc_norm_bwd_apply_kernel<2, false>), g, dim3(256), 0, s, a);
    else if (a.f16 && two) hipLaunchKernelGGL((enc_norm_bwd_apply_kernel<1, true>), g, dim3(256), 0, s, a);
    else if (a.f16) hipLaunchKernelGGL((enc_norm_bwd_apply_kernel<1, false>), g, dim3(256), 0, s, a);
    else if (two) hipLaunchKernelGGL((enc_norm_bwd_apply_kernel<0, true>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((enc_norm_bwd_apply_kernel<0, false>), g, dim3(256), 0, s, a);
    RAFT_HIP_CHECK(hipGetLastError());
  }
  return hipSuccess;
}

hipError_t launch_enc_norm_bwd(const NormBwdArgs& a, hipStream_t s) { return launch_enc_norm_bwd_stages(a, 7, 0, s); }

}  // namespace raft_amd
