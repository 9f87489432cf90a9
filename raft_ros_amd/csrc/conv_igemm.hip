// Implicit-GEMM NHWC convolutions on gfx950 MFMA for the RAFT update block
// (reference core/update.py:6-136: motion encoder, SepConvGRU/ConvGRU, flow and
// mask heads), forward + both backward GEMMs, bf16 operands, fp32 accumulate.
//
// Forward / data-gradient:  Y[p][n] = epi( sum_{tap,c} X[p + d_tap][c] * W[n][tap][c] )
//   * M = pixels (B*H*W), N = output channels, K = taps * Cin.
//   * X may be the channel-concatenation of up to 3 NHWC sources (pointer +
//     pixel stride each), so torch.cat of [h, inp, motion] etc. is never
//     materialised; outputs may be written into a channel slice of a wider
//     buffer (pixel stride != N), which fuses the concatenations on the output
//     side too (e.g. motion features = [conv out (126) | flow (2)]).
//   * fused epilogues: bias + ReLU / identity; GRU z||r gates (sigmoid, r*h);
//     GRU candidate + blend ((1-z) h + z tanh(q)); gradient store with ReLU'
//     mask of the conv input and partial (channel-range) accumulation.
//   * the data-gradient of a stride-1 conv is the same kernel on dY with
//     flipped/transposed packed weights and padding K-1-P.
//   * kernels: v4 (DMA ring, 64x128 / 64x64 tiles) for 1x1 convs and as the
//     default, v5 (halo strip: one LDS strip per 64-channel chunk serves every
//     tap) for the multi-tap update-block convs, an N<=2 register kernel for
//     the flow-head output, and a generic register-staged kernel for the odd
//     shapes the DMA kernels do not take.
// Weight gradient:  dW[n][tap][c] = sum_p dY[p][n] * X[p + d_tap][c]
//   * M = out channels, N = K = taps * Cin, reduction over pixels split over
//     workgroups (one fp32 partial slab per split, summed in a fixed order by
//     csrc/weights.hip: deterministic, no atomics).  A source may be
//     "periodic" (period = pixel count of one refinement iteration): the
//     update block's context features are shared by every iteration, so the
//     weight gradient of all iterations is one reduction over iters*P pixels
//     that re-reads the same context rows (ops/update_fused.py).
//
// Tiling: 256 threads = 4 wave64s in a 2x2 arrangement, v_mfma_f32_32x32x16_bf16,
// BK = 64 per LDS stage, XCD-aware tile order.
#include "common.h"
#include <cstdlib>
#include "kernel_abi.h"

#include <algorithm>
#include <utility>

namespace raft_amd {





namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) { return 1.f - 2.f / (__expf(2.f * x) + 1.f); }

struct SrcSel {
  const __bf16* ptr;
  long stride;
  int c;
};

// Source segment holding concatenated channel c (segments are consecutive).
__device__ __forceinline__ SrcSel select_src(const ConvSrc* src, int c) {
  const int c0 = src[0].C, c1 = src[1].C;
  if (c < c0) return {src[0].ptr, src[0].stride, c};
  if (c < c0 + c1) return {src[1].ptr, src[1].stride, c - c0};
  return {src[2].ptr, src[2].stride, c - c0 - c1};
}

// Generic 16-byte im2col chunk (per-thread tap decode): 8 consecutive k of pixel (b, py, px).
__device__ __forceinline__ u32x4 im2col_chunk(const ConvSrc* src, int Cin, int K, int H, int W, int KW,
                                              int PH, int PW, bool pvalid, int b, int py, int px, int k) {
  u32x4 v = {0, 0, 0, 0};
  if (!pvalid || k >= K) return v;
  const int tap = k / Cin;
  const int c = k - tap * Cin;
  const int ky = tap / KW;
  const int kx = tap - ky * KW;
  const int y = py + ky - PH, x = px + kx - PW;
  if (y < 0 || y >= H || x < 0 || x >= W) return v;
  const SrcSel s = select_src(src, c);
  return *reinterpret_cast<const u32x4*>(s.ptr + ((long)(b * H + y) * W + x) * s.stride + s.c);
}

// Per-thread pixel coordinates of the rows it stages.
struct PixCoord {
  long p;  // flat pixel index (or -1 when out of range)
  int py, px;
};

__device__ __forceinline__ PixCoord decode_pix(long p, long P, int H, int W) {
  PixCoord c{-1, 0, 0};
  if (p < P) {
    const int HW = H * W;
    const long b = p / HW;
    const int rem = (int)(p - b * HW);
    c.p = p;
    c.py = rem / W;
    c.px = rem - c.py * W;
  }
  return c;
}

// K step of the forward / dgrad kernels; padded LDS row of the generic kernel: 144 B ->
// conflict-free ds_read_b128 groups
constexpr int FBK = 64, FLDK = FBK + 8;

// ============================================================================ DMA helpers
// Direct-to-LDS pipeline: every 16-byte chunk of the A (im2col) and B (packed weight)
// tiles is fetched with global_load_lds_dwordx4 into an S-stage LDS ring, so S-1
// K steps are in flight with no staging registers.  LDS rows are 128 B (64 bf16)
// with the chunk index XOR-swizzled by (row>>1)&7: the lane-linear DMA image stays
// contiguous (the swizzle is applied to the per-lane SOURCE address) and every
// 16-lane ds_read_b128 group of the MFMA fragment reads hits 16 distinct bank slots.
// Padding / out-of-image taps are redirected to a zero page.  Waits are counted
// (s_waitcnt vmcnt(N)) and barriers are raw s_barrier so the DMA stays in flight
// across them (cdna_hip_programming.md "Pipelining across barriers").
__device__ __attribute__((aligned(64))) uint32_t g_zero_page[64];

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, __bf16* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)(reinterpret_cast<uintptr_t>(lds_wave_base) & 0xffffffffu),
                                   16, 0, 0);
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// ============================================================================ forward v4
// Same direct-to-LDS ring as v3, but every load is a bounds-checked raw buffer load
// (buffer_load_dwordx4 ... lds): the per-lane byte offset is one v_mad_u32_u24 of a
// precomputed pixel index, padding taps / rows past P / N use an out-of-range offset
// (the hardware returns zeros), the weight tile needs no per-step VALU at all
// (its K offset rides in the scalar soffset), and the epilogue is staged through
// LDS so each thread finishes 8 consecutive output channels with 16-byte accesses.
// (rocprofv3 PMC on v2/v3: ~15 VALU instructions per MFMA from 64-bit address math
// and per-element epilogues -- the kernels were VALU-issue bound.)
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void bload16(__amdgpu_buffer_rsrc_t r, __bf16* lds_wave_base, unsigned voff,
                                        unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (lds_void*)(reinterpret_cast<uintptr_t>(lds_wave_base) & 0xffffffffu), 16, voff, soff, 0, 0);
}

struct Fwd4Src {
  __amdgpu_buffer_rsrc_t r0, r1, r2;
  unsigned st0, st1, st2;
  int sc0, sc1;
};
struct Fwd4Geo {
  int Cin, K, H, W, KW, PH, PW, ntaps;
  bool uniform;
};

// Issue one K step (64 columns) of A (im2col) and B (weights) into an LDS stage.
template <int BM, int BN, int AI, int BI>
__device__ __forceinline__ void fwd4_issue(const Fwd4Src& src, const __amdgpu_buffer_rsrc_t rw, const Fwd4Geo& g,
                                           __bf16* sA, int wave, int k0, const int (&pix)[AI],
                                           const int (&py)[AI], const int (&px)[AI], const int (&achunk)[AI],
                                           const unsigned (&bvoff)[BI]) {
  __bf16* sB = sA + BM * 64;
  if (g.uniform) {
    int tap = 0, c0 = k0;
    if (g.ntaps != 1) {
      tap = k0 / g.Cin;
      c0 = k0 - tap * g.Cin;
    }
    const int ky = tap / g.KW;
    const int dy = ky - g.PH, dx = tap - ky * g.KW - g.PW;
    const int doff = dy * g.W + dx;
    const bool kin = k0 < g.K;
    if (c0 < src.sc0) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bool ok = kin && (unsigned)(py[i] + dy) < (unsigned)g.H && (unsigned)(px[i] + dx) < (unsigned)g.W;
        const unsigned voff = ok ? (unsigned)(pix[i] + doff) * src.st0 + (unsigned)(achunk[i] * 16) : kOOB;
        bload16(src.r0, sA + (wave * AI + i) * 512, voff, (unsigned)c0 * 2);
      }
    } else if (c0 < src.sc0 + src.sc1) {
      const int cc = c0 - src.sc0;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bool ok = kin && (unsigned)(py[i] + dy) < (unsigned)g.H && (unsigned)(px[i] + dx) < (unsigned)g.W;
        const unsigned voff = ok ? (unsigned)(pix[i] + doff) * src.st1 + (unsigned)(achunk[i] * 16) : kOOB;
        bload16(src.r1, sA + (wave * AI + i) * 512, voff, (unsigned)cc * 2);
      }
    } else {
      const int cc = c0 - src.sc0 - src.sc1;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const bool ok = kin && (unsigned)(py[i] + dy) < (unsigned)g.H && (unsigned)(px[i] + dx) < (unsigned)g.W;
        const unsigned voff = ok ? (unsigned)(pix[i] + doff) * src.st2 + (unsigned)(achunk[i] * 16) : kOOB;
        bload16(src.r2, sA + (wave * AI + i) * 512, voff, (unsigned)cc * 2);
      }
    }
  } else {
    // non-uniform K steps: single source segment only (host check)
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int k = k0 + achunk[i] * 8;
      unsigned voff = kOOB;
      if (pix[i] >= 0 && k < g.K) {
        const int tap = k / g.Cin;
        const int c = k - tap * g.Cin;
        const int ky = tap / g.KW;
        const int kx = tap - ky * g.KW;
        const int y = py[i] + ky - g.PH, x = px[i] + kx - g.PW;
        if ((unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W)
          voff = (unsigned)(pix[i] + (ky - g.PH) * g.W + (kx - g.PW)) * src.st0 + (unsigned)c * 2;
      }
      bload16(src.r0, sA + (wave * AI + i) * 512, voff, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) bload16(rw, sB + (wave * BI + i) * 512, bvoff[i], (unsigned)k0 * 2);
}

// split-bf16 planes (see ConvFwdArgs::split_g): store 8 consecutive channels [n, n + nv) of one
// pixel row as hi / lo / hi planes of group width G; read hi + lo of 8 channels at plane offset S
__device__ __forceinline__ void split_store8(__bf16* row, int G, int n, int nv, const float (&v)[8]) {
  __bf16* o = row + (long)(n / G) * 3 * G + n % G;
  bf16x8 hi, lo;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    hi[q] = static_cast<__bf16>(v[q]);
    lo[q] = static_cast<__bf16>(v[q] - static_cast<float>(hi[q]));
  }
  if (nv == 8) {
    *reinterpret_cast<bf16x8*>(o) = hi;
    *reinterpret_cast<bf16x8*>(o + G) = lo;
    *reinterpret_cast<bf16x8*>(o + 2 * G) = hi;
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < nv) {
        o[q] = hi[q];
        o[G + q] = lo[q];
        o[2 * G + q] = hi[q];
      }
  }
}

__device__ __forceinline__ void load8(const __bf16* row, int S, float (&x)[8], bool f16 = false) {
  const bf16x8 hv = *reinterpret_cast<const bf16x8*>(row);
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = ld16(hv[q], f16 && S == 0);
  if (S > 0) {
    const bf16x8 lv = *reinterpret_cast<const bf16x8*>(row + S);
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] += static_cast<float>(lv[q]);
  }
}

// Shared epilogue of the forward kernels: the fp32 accumulators go through an LDS tile
// (et, BM x (BN+4) floats) so each thread finishes 8 consecutive output channels of one
// pixel with 16-byte accesses; applies alpha/bias and the fused epilogue selected by a.epi.
// Output-row -> pixel mapping of a tile: flat (TW2D == 0: rows m0 .. m0 + BM - 1 of the pixel
// order) or a 2-D tile of TW2D columns (conv_fwd6 on wide images: row r -> image pixel
// (y0 + r / TW2D, x0 + r % TW2D) of image pbase / (H W), rows outside the image are skipped)
struct Tile2D {
  long pbase;
  int y0, x0, H, W;
};
template <int TW2D>
__device__ __forceinline__ bool row_pixel(int row, int m0, int P, const Tile2D& t, long& p) {
  if constexpr (TW2D == 0) {
    p = m0 + row;
    return p < P;
  } else {
    const int y = t.y0 + row / TW2D, x = t.x0 + row % TW2D;
    p = t.pbase + (long)y * t.W + x;
    return y < t.H && x < t.W;
  }
}

template <int BM, int BN, int TM, int TN, int NW = 4, int WGN = 2, int TW2D = 0, bool F16 = false>
__device__ __forceinline__ void fwd_epilogue(const ConvFwdArgs& a, float* et, f32x16 (&acc)[TM][TN], int m0,
                                             int n0, int P, int Nn, const Tile2D& t2 = Tile2D{}) {
  constexpr int EPI_LD = BN + 4;  // fp32 epilogue tile row pitch
  constexpr int NT = NW * 64;     // threads; waves are laid out (NW/WGN) x WGN over the tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr bool f16 = F16;  // 16-bit operands / outputs are fp16 (fp16 AMP)
  const int wm = wave / WGN, wn = wave % WGN;
  constexpr int CPR = BN / 8;  // 8-channel chunks per tile row
  static_assert(NT % CPR == 0, "a thread keeps one channel chunk across rows");
  // Fast path (uniform branch) for the plain bias/act store (epi 0) and the gradient store
  // (epi 1) without split planes: straight-line rows, the bias fetched as two 16-byte loads
  // before the LDS staging so its latency hides behind it.  The generic path below (GRU gates,
  // fused GRU backward, split-bf16 planes) tests its mode per row; for epi 0 / 1 its per-lane
  // mode, masked scalar bias loads and branches cost ~5 us per launch (scripts/bench_conv6.py
  // --probe, profiles/r3_conv6_probe.log).
  const bool fast = a.epi <= 3 && a.split_g == 0;
  f32x4 fb0{0.f, 0.f, 0.f, 0.f}, fb1{0.f, 0.f, 0.f, 0.f};
  {
    const int n = n0 + (tid % CPR) * 8;
    if (fast && a.bias && n < Nn) {
      if (n + 8 <= Nn && (reinterpret_cast<uintptr_t>(a.bias) & 15) == 0) {
        fb0 = *reinterpret_cast<const f32x4*>(a.bias + n);
        fb1 = *reinterpret_cast<const f32x4*>(a.bias + n + 4);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (n + q < Nn) fb0[q] = a.bias[n + q];
          if (n + 4 + q < Nn) fb1[q] = a.bias[n + 4 + q];
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / (NW / WGN)) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wn * (BN / WGN) + j * 32 + (lane & 31);
        et[row * EPI_LD + col] = acc[i][j][r];
      }
  __syncthreads();
  if (fast) {
    const int ch = tid % CPR;
    const int n = n0 + ch * 8;
    if (n >= Nn) return;
    const bool full = n + 8 <= Nn;
    const float alpha = a.alpha;
    const bool relu = a.epi == 0 && a.act == 1;
    const bool grad = a.epi == 1;
    const bool accum = grad && n >= a.acc_c0;  // acc_c0 is a multiple of 8
    const bool f32o = a.out_f32 != 0;
    const bool vec = full && (!f32o || (a.out_stride & 3) == 0);
    if constexpr (CPR >= 8) {
      // epi 0 + the folded narrow conv (ConvFwdArgs::n2y; host: bf16 out, N % 64 == 0 or
      // N >= n2_cols): each aligned group of 8 lanes is one 64-channel slot of one row
      if (a.n2y != nullptr && a.epi == 0 && n0 < a.n2_cols) {
        const bool in2 = n < a.n2_cols;  // uniform per 8-lane group (n2_cols % 64 == 0)
        const int c8 = ch & 7;
        const long slot = n / 64;
#pragma unroll 1
        for (int row = tid / CPR; row < BM; row += NT / CPR) {
          long p;
          if (!row_pixel<TW2D>(row, m0, P, t2, p)) {
            if constexpr (TW2D == 0) break;
            else continue;
          }
          f32x4 lo = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8);
          f32x4 hi = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8 + 4);
          lo = lo * alpha + fb0;
          hi = hi * alpha + fb1;
          bf16x8 w;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            w[q] = st16(relu ? fmaxf(lo[q], 0.f) : lo[q], f16);
            w[q + 4] = st16(relu ? fmaxf(hi[q], 0.f) : hi[q], f16);
          }
          *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.out) + p * a.out_stride + n) = w;
          // the 18 weight rows are re-read per row (L1-resident, 9 KB in all): hoisting them
          // out of the row loop would hold 72 more VGPRs in every forward kernel and halve the
          // occupancy of the two-workgroups-per-CU tiles.  The empty asm makes the channel
          // offset opaque per row so the compiler cannot hoist the loads.
          int nn = in2 ? n : 0;
          asm volatile("" : "+v"(nn));
          const __bf16* wr = a.n2w + nn;
          float s[18];
#pragma unroll
          for (int j = 0; j < 18; ++j) {
            const int o = j / 9, t = j - (j / 9) * 9;
            const bf16x8 wv = *reinterpret_cast<const bf16x8*>(wr + (long)o * a.n2_kpad + t * a.n2_cols);
            float acc2 = 0.f;
#pragma unroll
            for (int q = 0; q < 8; ++q) acc2 += ld16(w[q], f16) * ld16(wv[q], f16);
            s[j] = acc2;
          }
#pragma unroll
          for (int off = 4; off > 0; off >>= 1)
#pragma unroll
            for (int j = 0; j < 18; ++j) s[j] += __shfl_xor(s[j], off, 64);
          if (in2) {
            // lanes write planes j = c8, c8 + 8, c8 + 16 (< 18) of this row (selects, not a dynamic
            // index into s, which would put s in scratch)
            float v0 = s[0], v1 = s[8], v2 = s[16];
#pragma unroll
            for (int q = 1; q < 8; ++q)
              if (c8 == q) {
                v0 = s[q];
                v1 = s[q + 8];
                if (q < 2) v2 = s[q + 16];
              }
            float* y = a.n2y + (slot * 18 + c8) * P + p;  // planar: plane j at y + j * P
            y[0] = v0;
            y[8 * (long)P] = v1;
            if (c8 < 2) y[16 * (long)P] = v2;
          }
        }
        return;
      }
    }
    if (a.epi >= 2) {
      // GRU gates (bf16, channel counts multiples of 8): epi 2 z||r: out = sigmoid, and for the r
      // half out2 = r * h; epi 3: q = tanh, out = (1 - z) h + z q, out2 = q
      const bool zr = a.epi == 2;
      const int hc = zr ? n - (Nn >> 1) : n;  // h channel of this chunk (epi 2: r half only)
      const bool has_h = !zr || hc >= 0;
#pragma unroll 4
      for (int row = tid / CPR; row < BM; row += NT / CPR) {
        long p;
        if (!row_pixel<TW2D>(row, m0, P, t2, p)) {
          if constexpr (TW2D == 0) break;
          else continue;
        }
        f32x4 lo = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8);
        f32x4 hi = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8 + 4);
        lo = lo * alpha + fb0;
        hi = hi * alpha + fb1;
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bf16x8 hv{};
        if (has_h) hv = *reinterpret_cast<const bf16x8*>(a.h + p * a.h_stride + hc);
        bf16x8 w0, w1;
        if (zr) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float sg = sigmoidf_(v[q]);
            w0[q] = st16(sg, f16);
            w1[q] = st16(ld16(w0[q], f16) * ld16(hv[q], f16), f16);
          }
          *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.out) + p * a.out_stride + n) = w0;
          if (has_h) *reinterpret_cast<bf16x8*>(a.out2 + p * a.out2_stride + hc) = w1;
        } else {
          const bf16x8 zv = *reinterpret_cast<const bf16x8*>(a.z + p * a.z_stride + n);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float qq = tanhf_(v[q]);
            const float z = ld16(zv[q], f16);
            w0[q] = st16((1.f - z) * ld16(hv[q], f16) + z * qq, f16);
            w1[q] = st16(qq, f16);
          }
          *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.out) + p * a.out_stride + n) = w0;
          *reinterpret_cast<bf16x8*>(a.out2 + p * a.out2_stride + n) = w1;
        }
      }
      return;
    }
#pragma unroll 4
    for (int row = tid / CPR; row < BM; row += NT / CPR) {
      long p;
      if (!row_pixel<TW2D>(row, m0, P, t2, p)) {
        if constexpr (TW2D == 0) break;
        else continue;
      }
      f32x4 lo = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8);
      f32x4 hi = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8 + 4);
      lo = lo * alpha + fb0;
      hi = hi * alpha + fb1;
      if (relu) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          lo[q] = fmaxf(lo[q], 0.f);
          hi[q] = fmaxf(hi[q], 0.f);
        }
      }
      if (grad && a.mask) {
        const bf16x8 m = *reinterpret_cast<const bf16x8*>(a.mask + p * a.mask_stride + n);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (!(ld16(m[q], f16) > 0.f)) lo[q] = 0.f;
          if (!(ld16(m[q + 4], f16) > 0.f)) hi[q] = 0.f;
        }
      }
      if (f32o) {
        float* o = static_cast<float*>(a.out) + p * a.out_stride + n;
        if (vec) {
          if (accum) {
            lo += *reinterpret_cast<const f32x4*>(o);
            hi += *reinterpret_cast<const f32x4*>(o + 4);
          }
          *reinterpret_cast<f32x4*>(o) = lo;
          *reinterpret_cast<f32x4*>(o + 4) = hi;
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (n + q < Nn) {
              const float x = q < 4 ? lo[q] : hi[q - 4];
              o[q] = accum ? o[q] + x : x;
            }
        }
      } else {
        __bf16* o = static_cast<__bf16*>(a.out) + p * a.out_stride + n;
        if (full) {
          if (accum) {
            const bf16x8 old = *reinterpret_cast<const bf16x8*>(o);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              lo[q] += ld16(old[q], f16);
              hi[q] += ld16(old[q + 4], f16);
            }
          }
          bf16x8 w;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            w[q] = st16(lo[q], f16);
            w[q + 4] = st16(hi[q], f16);
          }
          *reinterpret_cast<bf16x8*>(o) = w;
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (n + q < Nn) {
              const float x = q < 4 ? lo[q] : hi[q - 4];
              o[q] = st16(accum ? ld16(o[q], f16) + x : x, f16);
            }
        }
      }
    }
    return;
  }
  // generic path: every thread owns the same 8-channel chunk in all of its rows (NT % CPR
  // == 0): the bias is loaded once, before the row loop, instead of as a dependent load per row
  const int ch = tid % CPR;
  const int n = n0 + ch * 8;
  if (n >= Nn) return;
  const int nv = Nn - n < 8 ? Nn - n : 8;  // valid channels in this chunk
  float bia[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bia[q] = (a.bias && q < nv) ? a.bias[n + q] : 0.f;
  const float alpha = a.alpha;
  // this thread's 8 channels: the GRU-backward epilogues cover [0, gru_cols), epi 1 the rest
  int epi = a.epi;
  if (epi == 4 || epi == 5) epi = n < a.gru_cols ? epi : 1;
  else if (epi == 6) epi = (n < a.gru_cols || n >= a.cm_c0) ? 6 : 1;
  // one row loop per mode (the mode of a lane is fixed; in practice uniform per tile), so the
  // mode tests are resolved at compile time instead of per row
  auto rows = [&](auto mc) __attribute__((always_inline)) {
    constexpr int M = decltype(mc)::value;
#pragma unroll 2
    for (int row = tid / CPR; row < BM; row += NT / CPR) {
      long p;
      if (!row_pixel<TW2D>(row, m0, P, t2, p)) {
        if constexpr (TW2D == 0) break;
        else continue;
      }
      const f32x4 lo = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(et + row * EPI_LD + ch * 8 + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = v[q] * alpha + bia[q];
      if (M == 4 || M == 5) {
        // fused GRU backward gate math (fp32 gradient rows; gru_cols is a multiple of 8)
        float* o = static_cast<float*>(a.out) + p * a.out_stride + n;
        if (n >= a.acc_c0) {
          const f32x4 o0 = *reinterpret_cast<const f32x4*>(o), o1 = *reinterpret_cast<const f32x4*>(o + 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[q] += o0[q];
            v[q + 4] += o1[q];
          }
        }
        if (a.addsrc) {
          float av[8];
          load8(a.addsrc + p * a.addsrc_stride + n, a.split_add, av, f16);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] += av[q];
        }
        // gate operands: bf16, or split planes (hi + lo) in fp32 training
        float gv[8], hv[8];
        load8(a.g0 + p * a.g0_stride + n, a.split_g0, gv, f16);
        load8(a.h + p * a.h_stride + n, a.split_h, hv, f16);
        float* cp = a.carry + p * a.carry_stride + n;
        float d3[8];
        if (M == 4) {
          float zv[8];
          load8(a.z + p * a.z_stride + n, a.split_z, zv, f16);
          float dq[8], cr[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float zz = zv[q], qq = gv[q], hh = hv[q];
            dq[q] = v[q] * zz * (1.f - qq * qq);
            d3[q] = v[q] * (qq - hh) * zz * (1.f - zz);
            cr[q] = v[q] * (1.f - zz);
          }
          if (a.split_g2 > 0) {
            split_store8(a.out2 + p * a.out2_stride, a.split_g2, n, 8, dq);
          } else {
            bf16x8 w;
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = st16(dq[q], f16);
            *reinterpret_cast<bf16x8*>(a.out2 + p * a.out2_stride + n) = w;
          }
          *reinterpret_cast<f32x4*>(cp) = f32x4{cr[0], cr[1], cr[2], cr[3]};
          *reinterpret_cast<f32x4*>(cp + 4) = f32x4{cr[4], cr[5], cr[6], cr[7]};
        } else {
          const f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
          const float cv[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
          float ov[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float rr = gv[q], hh = hv[q];
            d3[q] = v[q] * hh * rr * (1.f - rr);
            ov[q] = cv[q] + v[q] * rr;
          }
          *reinterpret_cast<f32x4*>(o) = f32x4{ov[0], ov[1], ov[2], ov[3]};
          *reinterpret_cast<f32x4*>(o + 4) = f32x4{ov[4], ov[5], ov[6], ov[7]};
        }
        if (a.split_g3 > 0) {
          split_store8(a.out3 + p * a.out3_stride, a.split_g3, n, 8, d3);
        } else {
          bf16x8 w;
#pragma unroll
          for (int q = 0; q < 8; ++q) w[q] = st16(d3[q], f16);
          *reinterpret_cast<bf16x8*>(a.out3 + p * a.out3_stride + n) = w;
        }
      } else if (M == 6) {
        // last GRU data gradient: bf16 d net / fp32 d inp / masked bf16 d motion
        const float* o = static_cast<const float*>(a.out) + p * a.out_stride + n;
        const f32x4 o0 = *reinterpret_cast<const f32x4*>(o), o1 = *reinterpret_cast<const f32x4*>(o + 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] += o0[q];
          v[q + 4] += o1[q];
        }
        bf16x8 w;
        if (n < a.gru_cols) {
          if (a.split_g3 > 0) {
            split_store8(a.out3 + p * a.out3_stride, a.split_g3, n, 8, v);
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = st16(v[q], f16);
            *reinterpret_cast<bf16x8*>(a.out3 + p * a.out3_stride + n) = w;
          }
        } else {
          const int c = n - a.cm_c0;
          if (c < a.cm_valid) {  // chunks wholly past cm_valid are not stored (cout may be narrower)
            const bf16x8 m = *reinterpret_cast<const bf16x8*>(a.cmask + p * a.cmask_stride + c);
            float mv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) mv[q] = (c + q < a.cm_valid && ld16(m[q], f16) > 0.f) ? v[q] : 0.f;
            if (a.split_cout > 0) {
              split_store8(a.cout + p * a.cout_stride, a.split_cout, c, 8, mv);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) w[q] = st16(mv[q], f16);
              *reinterpret_cast<bf16x8*>(a.cout + p * a.cout_stride + c) = w;
            }
          }
        }
      } else if (M == 0) {
        if (a.act == 1)
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
        if (a.split_g > 0 && !a.out_f32) {
          split_store8(static_cast<__bf16*>(a.out) + p * a.out_stride, a.split_g, n, nv, v);
        } else if (a.out_f32) {
          float* o = static_cast<float*>(a.out) + p * a.out_stride + n;
          if (nv == 8 && (a.out_stride & 3) == 0) {
            *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
            *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (q < nv) o[q] = v[q];
          }
        } else {
          __bf16* o = static_cast<__bf16*>(a.out) + p * a.out_stride + n;
          if (nv == 8) {
            bf16x8 w;
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = st16(v[q], f16);
            *reinterpret_cast<bf16x8*>(o) = w;
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (q < nv) o[q] = st16(v[q], f16);
          }
        }
      } else if (M == 1) {
        if (a.mask) {
          const bf16x8 m = *reinterpret_cast<const bf16x8*>(a.mask + p * a.mask_stride + n);
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (!(ld16(m[q], f16) > 0.f)) v[q] = 0.f;
        }
        const bool accum = n >= a.acc_c0;  // acc_c0 is a multiple of 8
        if (a.split_g > 0) {  // split planes (fp32 training data gradients; never accumulated)
          split_store8(static_cast<__bf16*>(a.out) + p * a.out_stride, a.split_g, n, nv, v);
        } else if (a.out_f32) {
          float* o = static_cast<float*>(a.out) + p * a.out_stride + n;
          if (nv == 8) {
            f32x4 x0 = {v[0], v[1], v[2], v[3]}, x1 = {v[4], v[5], v[6], v[7]};
            if (accum) {
              x0 += *reinterpret_cast<const f32x4*>(o);
              x1 += *reinterpret_cast<const f32x4*>(o + 4);
            }
            *reinterpret_cast<f32x4*>(o) = x0;
            *reinterpret_cast<f32x4*>(o + 4) = x1;
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (q < nv) o[q] = accum ? o[q] + v[q] : v[q];
          }
        } else {
          __bf16* o = static_cast<__bf16*>(a.out) + p * a.out_stride + n;
          if (nv == 8) {
            bf16x8 w;
            const bf16x8 old = accum ? *reinterpret_cast<const bf16x8*>(o) : bf16x8{};
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = st16(accum ? ld16(old[q], f16) + v[q] : v[q], f16);
            *reinterpret_cast<bf16x8*>(o) = w;
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (q < nv) o[q] = st16(accum ? ld16(o[q], f16) + v[q] : v[q], f16);
          }
        }
      } else if (M == 2 && a.split_g > 0) {
        // split mode: sigmoid in fp32, r * h from the fp32-faithful h (hi + lo planes)
        const int C = Nn >> 1;
        float sg[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) sg[q] = sigmoidf_(v[q]);
        split_store8(static_cast<__bf16*>(a.out) + p * a.out_stride, a.split_g, n, 8, sg);
        if (n >= C) {
          float hv[8];
          load8(a.h + p * a.h_stride + (n - C), a.split_h, hv);
#pragma unroll
          for (int q = 0; q < 8; ++q) hv[q] *= sg[q];
          split_store8(a.out2 + p * a.out2_stride, a.split_g2, n - C, 8, hv);
        }
      } else if (M == 3 && a.split_g > 0) {
        float zv[8], hv[8], hn[8];
        load8(a.z + p * a.z_stride + n, a.split_z, zv);
        load8(a.h + p * a.h_stride + n, a.split_h, hv);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float qq = tanhf_(v[q]);
          hn[q] = (1.f - zv[q]) * hv[q] + zv[q] * qq;
          v[q] = qq;
        }
        split_store8(static_cast<__bf16*>(a.out) + p * a.out_stride, a.split_g, n, 8, hn);
        if (a.out2) split_store8(a.out2 + p * a.out2_stride, a.split_g2 > 0 ? a.split_g2 : a.split_g, n, 8, v);
      } else if (M == 2) {
        const int C = Nn >> 1;
        bf16x8 sg;
#pragma unroll
        for (int q = 0; q < 8; ++q) sg[q] = st16(sigmoidf_(v[q]), f16);
        *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.out) + p * a.out_stride + n) = sg;
        if (n >= C) {
          const bf16x8 hv = *reinterpret_cast<const bf16x8*>(a.h + p * a.h_stride + (n - C));
          bf16x8 rh;
#pragma unroll
          for (int q = 0; q < 8; ++q) rh[q] = st16(ld16(sg[q], f16) * ld16(hv[q], f16), f16);
          *reinterpret_cast<bf16x8*>(a.out2 + p * a.out2_stride + (n - C)) = rh;
        }
      } else {
        const bf16x8 zv = *reinterpret_cast<const bf16x8*>(a.z + p * a.z_stride + n);
        const bf16x8 hv = *reinterpret_cast<const bf16x8*>(a.h + p * a.h_stride + n);
        bf16x8 hn, qo;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float qq = tanhf_(v[q]);
          const float z = ld16(zv[q], f16);
          hn[q] = st16((1.f - z) * ld16(hv[q], f16) + z * qq, f16);
          qo[q] = st16(qq, f16);
        }
        *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.out) + p * a.out_stride + n) = hn;
        *reinterpret_cast<bf16x8*>(a.out2 + p * a.out2_stride + n) = qo;
      }
    }
  };
  switch (epi) {
    case 0: rows(std::integral_constant<int, 0>{}); break;
    case 1: rows(std::integral_constant<int, 1>{}); break;
    case 2: rows(std::integral_constant<int, 2>{}); break;
    case 3: rows(std::integral_constant<int, 3>{}); break;
    case 4: rows(std::integral_constant<int, 4>{}); break;
    case 5: rows(std::integral_constant<int, 5>{}); break;
    default: rows(std::integral_constant<int, 6>{}); break;
  }
}

// ============================================================================ forward / dgrad (generic)
// BM x BN output tile, BK = 64, 256 threads as 2x2 waves, each wave (BM/2)x(BN/2)
// = TM x TN MFMA 32x32x16 tiles; two LDS stages, one barrier per K step; register-staged
// im2col for any source layout (the DMA kernels below need 64-channel segments).
template <int BM, int BN, bool F16 = false>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const ConvFwdArgs a) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int ACH = BM * FBK / 8 / 256, BCH = BN * FBK / 8 / 256;
  constexpr int STAGE = (BM + BN) * FLDK;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];

  const int tilesN = (a.N + BN - 1) / BN;
  const int tilesM = (int)((a.P + BM - 1) / BM);
  const int wg = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int tm = wg / tilesN, tn = wg - (wg / tilesN) * tilesN;
  const long m0 = (long)tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int kc = tid & 7;  // fixed 16-byte column of every chunk this thread stages

  PixCoord pc[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) pc[i] = decode_pix(m0 + (tid >> 3) + 32 * i, a.P, a.H, a.W);

  // the K step never straddles a tap / source segment when every segment is a multiple
  // of FBK channels (or the conv is 1x1): tap + segment are then wave-uniform (scalar)
  bool uniform = (a.KH * a.KW == 1) || (a.Cin % FBK == 0);
  for (int i = 0; i < 3; ++i) uniform = uniform && (a.src[i].C % FBK == 0 || a.KH * a.KW == 1);
  const int nk = a.Kpad / FBK;

  u32x4 ra[ACH], rb[BCH];
  auto load = [&](int k0) __attribute__((always_inline)) {
    if (uniform) {
      int tap = k0 / a.Cin;
      int c0 = k0 - tap * a.Cin;
      if (a.KH * a.KW == 1) { tap = 0; c0 = k0; }
      const int ky = tap / a.KW, kx = tap - (tap / a.KW) * a.KW;
      const int dy = ky - a.PH, dx = kx - a.PW;
      const SrcSel s = select_src(a.src, c0);
      const long doff = (long)dy * a.W + dx;
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        const int y = pc[i].py + dy, x = pc[i].px + dx;
        const bool ok = pc[i].p >= 0 && k0 + kc * 8 < a.K && y >= 0 && y < a.H && x >= 0 && x < a.W;
        ra[i] = ok ? *reinterpret_cast<const u32x4*>(s.ptr + (pc[i].p + doff) * s.stride + s.c + kc * 8)
                   : u32x4{0, 0, 0, 0};
      }
    } else {
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        const long p = pc[i].p;
        const int b = p >= 0 ? (int)(p / ((long)a.H * a.W)) : 0;
        ra[i] = im2col_chunk(a.src, a.Cin, a.K, a.H, a.W, a.KW, a.PH, a.PW, p >= 0, b, pc[i].py, pc[i].px,
                             k0 + kc * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int n = n0 + (tid >> 3) + 32 * i;
      rb[i] = n < a.N ? *reinterpret_cast<const u32x4*>(a.wt + (long)n * a.Kpad + k0 + kc * 8)
                      : u32x4{0, 0, 0, 0};
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
    __bf16* sA = smem + buf * STAGE;
    __bf16* sB = sA + BM * FLDK;
#pragma unroll
    for (int i = 0; i < ACH; ++i)
      *reinterpret_cast<u32x4*>(sA + ((tid >> 3) + 32 * i) * FLDK + kc * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BCH; ++i)
      *reinterpret_cast<u32x4*>(sB + ((tid >> 3) + 32 * i) * FLDK + kc * 8) = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fk = (lane >> 5) * 8;
  load(0);
  store(0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) load((t + 1) * FBK);
    const __bf16* sA = smem + (t & 1) * STAGE;
    const __bf16* sB = sA + BM * FLDK;
#pragma unroll
    for (int s = 0; s < FBK / 16; ++s) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(sA + (wm * (BM / 2) + i * 32 + fr) * FLDK + s * 16 + fk);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + (wn * (BN / 2) + j * 32 + fr) * FLDK + s * 16 + fk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mma16<F16>(af[i], bfr[j], acc[i][j]);
    }
    if (t + 1 < nk) store((t + 1) & 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  // the shared LDS-staged epilogue of the DMA kernels (every store mode, GRU gates and their
  // backward, split-bf16 planes); the operand ring is free after the last K step's barrier
  static_assert(BM * (BN + 4) * 4 <= 2 * STAGE * 2, "epilogue tile must fit the operand ring");
  fwd_epilogue<BM, BN, TM, TN, 4, 2, 0, F16>(a, reinterpret_cast<float*>(smem), acc, (int)m0, n0, (int)a.P, a.N);
}

template <int BM, int BN, int S, bool F16 = false>
__global__ __launch_bounds__(256) void conv_fwd4_kernel(const ConvFwdArgs a) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int AI = BM / 32, BI = BN / 32;
  constexpr int G = AI + BI;
  constexpr int STAGE = (BM + BN) * 64;
  constexpr int EPI_LD = BN + 4;  // fp32 epilogue tile row pitch
  static_assert(S * STAGE * 2 >= BM * EPI_LD * 4, "epilogue tile must fit in the ring");
  __shared__ __attribute__((aligned(1024))) __bf16 smem[S * STAGE];

  const int Cin = a.Cin, K = a.K, Kpad = a.Kpad, H = a.H, W = a.W, KW = a.KW, PH = a.PH, PW = a.PW;
  const int ntaps = a.KH * a.KW;
  const int P = (int)a.P;
  const int Nn = a.N;
  const int sc0 = a.src[0].C, sc1 = a.src[1].C;
  const int nsrc = a.nsrc;
  // one buffer resource per source segment (+ the weights)
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.src[0].ptr, (unsigned)(a.P * a.src[0].stride * 2));
  const __amdgpu_buffer_rsrc_t r1 =
      make_rsrc(nsrc > 1 ? a.src[1].ptr : a.src[0].ptr, nsrc > 1 ? (unsigned)(a.P * a.src[1].stride * 2) : 0u);
  const __amdgpu_buffer_rsrc_t r2 =
      make_rsrc(nsrc > 2 ? a.src[2].ptr : a.src[0].ptr, nsrc > 2 ? (unsigned)(a.P * a.src[2].stride * 2) : 0u);
  const unsigned st0 = (unsigned)a.src[0].stride * 2, st1 = (unsigned)a.src[1].stride * 2,
                 st2 = (unsigned)a.src[2].stride * 2;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wt, (unsigned)((long)Nn * Kpad * 2));

  const int tilesN = (Nn + BN - 1) / BN;
  const int tilesM = (P + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int tm = wg / tilesN, tn = wg - (wg / tilesN) * tilesN;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int lrow = lane >> 3, lpc = lane & 7;

  int pix[AI], py[AI], px[AI], achunk[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wave * AI + i) * 8 + lrow;
    const int p = m0 + row;
    achunk[i] = swz(row, lpc);
    if (p < P) {
      const int HW = H * W;
      const int rem = p % HW;
      pix[i] = p;
      py[i] = rem / W;
      px[i] = rem - py[i] * W;
    } else {
      pix[i] = -1;
      py[i] = px[i] = -(1 << 20);
    }
  }
  unsigned bvoff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * 8 + lrow;
    bvoff[i] = (n0 + row < Nn) ? (unsigned)((n0 + row) * Kpad * 2 + swz(row, lpc) * 16) : kOOB;
  }
  const bool uniform = (ntaps == 1) || (Cin % 64 == 0 && sc0 % 64 == 0 && sc1 % 64 == 0);
  const int nk = Kpad / 64;

  Fwd4Src src{r0, r1, r2, st0, st1, st2, sc0, sc1};
  Fwd4Geo geo{Cin, K, H, W, KW, PH, PW, ntaps, uniform};
#define RAFT_FWD4_ISSUE(step, stage) \
  fwd4_issue<BM, BN, AI, BI>(src, rw, geo, smem + (stage) * STAGE, wave, (step) * 64, pix, py, px, achunk, bvoff)
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nk) RAFT_FWD4_ISSUE(i, i);

  for (int t = 0; t < nk; ++t) {
    const int ahead = (nk - 1 - t) < (S - 2) ? (nk - 1 - t) : (S - 2);
    if (ahead >= S - 2) wait_vmcnt<(S - 2) * G>();
    else if (ahead == 2) wait_vmcnt<2 * G>();
    else if (ahead == 1) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + S - 1 < nk) RAFT_FWD4_ISSUE(t + S - 1, (t + S - 1) % S);
    const __bf16* sA = smem + (t % S) * STAGE;
    const __bf16* sB = sA + BM * 64;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 2 * s + fh;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / 2) + i * 32 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(sA + row * 64 + swz(row, c) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / 2) + j * 32 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + row * 64 + swz(row, c) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mma16<F16>(af[i], bfr[j], acc[i][j]);
    }
  }
#undef RAFT_FWD4_ISSUE
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  fwd_epilogue<BM, BN, TM, TN, 4, 2, 0, F16>(a, reinterpret_cast<float*>(smem), acc, m0, n0, P, Nn);
}

// ============================================================================ forward v5 (halo strip)
// Implicit GEMM with operand reuse across taps.  v4 re-fetches the im2col A tile for
// every tap (9x the activation bytes for a 3x3 conv) and a BM=64 tile re-reads the
// whole weight slice for every 64 pixels; on MI355X those L2->CU fills (~70 GB/s per
// CU) bound the update-block convs, not the MFMA.  v5 stages, per 64-channel chunk,
// ONE contiguous strip of input pixels covering the tile plus its halo
//     rows [m0 - (PH*W+PW), m0 + BM + (KH-1)*W + KW-1 - (PH*W+PW))
// (flat NHWC pixel order, so a tap is a constant row shift of the strip) and then
// runs every tap of the chunk from it: only the BN x 64 weight tile is fetched per
// tap.  Pixels outside the image (row ends, image borders, batch borders) are
// zeroed at the A-fragment read by a per-lane (py, px) bounds test.
//   steps t = chunk * ntaps + tap;  3-stage weight ring, 2 strip buffers; the strip of
//   chunk c+1 is fetched with the weights two steps ahead (same counted-vmcnt DMA
//   pipeline as v4).  Dynamic LDS: 2 strips + 3 weight stages (<= 160 KB).
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;

// 16-byte LDS read at a 32-bit LDS byte address
__device__ __forceinline__ bf16x8 lds_read16(unsigned addr) { return *(const lds_bf16x8*)(uintptr_t)addr; }

// Measurement probes of this kernel (MFMA-, DMA- and read-free variants, cfg 30..32; removed
// after the measurement: profiles/r3_probe_conv5.log, profiles/r3_probe_conv6.log) led to v6.
template <int BM, int BN, int NW = 4, bool F16 = false>
__global__ __launch_bounds__(NW * 64) void conv_fwd5_kernel(const ConvFwdArgs a, int strip_rows) {
  extern __shared__ __attribute__((aligned(1024))) __bf16 dsm[];
  // NW waves in an (NW/2) x 2 layout; NW = 8 puts two waves on every SIMD of the CU (one
  // workgroup per CU when the strip ring fills the LDS), so one wave's LDS reads and waits
  // overlap the other's MFMAs
  constexpr int WGM = NW / 2;
  constexpr int TM = BM / (32 * WGM), TN = BN / 64;
  constexpr int BI = BN / (8 * NW);  // weight wave-instructions (8 rows each) per wave per step
  static_assert(TM >= 1 && BI >= 1, "tile too small for the wave count");
  constexpr int BSTAGE = BN * 64;
  const int strip_elems = strip_rows * 64;
  __bf16* const strips = dsm;
  __bf16* const bring = dsm + 2 * strip_elems;
  __bf16* const zrow = bring + 3 * BSTAGE;  // 64 zero bf16: the A row of out-of-image taps

  const int Cin = a.Cin, Kpad = a.Kpad, H = a.H, W = a.W, KW = a.KW, PH = a.PH, PW = a.PW;
  const int ntaps = a.KH * a.KW;
  const int P = (int)a.P;
  const int Nn = a.N;
  const int sc0 = a.src[0].C, sc1 = a.src[1].C;
  const int nsrc = a.nsrc;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.src[0].ptr, (unsigned)(a.P * a.src[0].stride * 2));
  const __amdgpu_buffer_rsrc_t r1 =
      make_rsrc(nsrc > 1 ? a.src[1].ptr : a.src[0].ptr, nsrc > 1 ? (unsigned)(a.P * a.src[1].stride * 2) : 0u);
  const __amdgpu_buffer_rsrc_t r2 =
      make_rsrc(nsrc > 2 ? a.src[2].ptr : a.src[0].ptr, nsrc > 2 ? (unsigned)(a.P * a.src[2].stride * 2) : 0u);
  const unsigned st0 = (unsigned)a.src[0].stride * 2, st1 = (unsigned)a.src[1].stride * 2,
                 st2 = (unsigned)a.src[2].stride * 2;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wt, (unsigned)((long)Nn * Kpad * 2));

  const int tilesN = (Nn + BN - 1) / BN;
  const int tilesM = (P + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int tm = wg / tilesN, tn = wg - (wg / tilesN) * tilesN;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int halo_lo = PH * W + PW;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int lrow = lane >> 3, lpc = lane & 7;
  const int fr = lane & 31, fh = lane >> 5;
  if (tid < 8) reinterpret_cast<u32x4*>(zrow)[tid] = u32x4{0, 0, 0, 0};

  // A-fragment rows of this lane: tile row and image coordinates
  int frow[TM], fpy[TM], fpx[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    frow[i] = wm * (BM / WGM) + i * 32 + fr;
    const int p = m0 + frow[i];
    if (p < P) {
      const int rem = p % (H * W);
      fpy[i] = rem / W;
      fpx[i] = rem - fpy[i] * W;
    } else {
      fpy[i] = fpx[i] = -(1 << 20);
    }
  }
  // B-fragment LDS byte offsets (within a stage) of this lane, per sub-step; fragment j adds
  // j*32 rows (a multiple of 16 rows leaves the swizzle unchanged -> immediate offset)
  unsigned boff[4];
  {
    const int row = wn * (BN / 2) + fr;
#pragma unroll
    for (int s = 0; s < 4; ++s) boff[s] = (unsigned)(row * 128 + swz(row, 2 * s + fh) * 16);
  }
  unsigned bvoff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * 8 + lrow;
    bvoff[i] = (n0 + row < Nn) ? (unsigned)((n0 + row) * Kpad * 2 + swz(row, lpc) * 16) : kOOB;
  }
  const int nchunks = Cin / 64;
  const int nsteps = nchunks * ntaps;
  const int strip_instr = strip_rows / 8;  // 8 rows (1 KB) per wave-instruction
  const unsigned lds_strips = (unsigned)(reinterpret_cast<uintptr_t>(strips) & 0xffffffffu);
  const unsigned lds_bring = (unsigned)(reinterpret_cast<uintptr_t>(bring) & 0xffffffffu);
  const unsigned lds_zero = (unsigned)(reinterpret_cast<uintptr_t>(zrow) & 0xffffffffu);

  // ---- DMA issue state (step `is_t`): chunk, tap, weight k offset, stage
  int is_t = 0, is_cc = 0, is_tap = 0, is_stage = 0;
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (is_tap == 0) {
      const int c0 = is_cc * 64;
      __amdgpu_buffer_rsrc_t rs = r0;
      unsigned st = st0, soff = (unsigned)c0 * 2;
      if (c0 >= sc0 + sc1) {
        rs = r2; st = st2; soff = (unsigned)(c0 - sc0 - sc1) * 2;
      } else if (c0 >= sc0) {
        rs = r1; st = st1; soff = (unsigned)(c0 - sc0) * 2;
      }
      __bf16* sbuf = strips + (is_cc & 1) * strip_elems;
      for (int q = wave; q < strip_instr; q += NW) {
        const int row = q * 8 + lrow;
        const int p = m0 - halo_lo + row;
        const unsigned voff = (p >= 0 && p < P) ? (unsigned)p * st + (unsigned)(swz(row, lpc) * 16) : kOOB;
        bload16(rs, sbuf + q * 512, voff, soff);
      }
    }
    __bf16* sB = bring + is_stage * BSTAGE;
    const unsigned k0 = (unsigned)(is_tap * Cin + is_cc * 64);
#pragma unroll
    for (int i = 0; i < BI; ++i) bload16(rw, sB + (wave * BI + i) * 512, bvoff[i], k0 * 2);
    ++is_t;
    is_stage = is_stage == 2 ? 0 : is_stage + 1;
    if (++is_tap == ntaps) {
      is_tap = 0;
      ++is_cc;
    }
  };

  // ---- fragment-read state (step `rd_t`)
  int rd_cc = 0, rd_ky = 0, rd_kx = 0, rd_stage = 0;
  auto read_frags = [&](bf16x8 (&fa)[TM][4], bf16x8 (&fb)[TN][4]) __attribute__((always_inline)) {
    const int shift = rd_ky * W + rd_kx;
    const int dy = rd_ky - PH, dx = rd_kx - PW;
    const unsigned sbase = lds_strips + (unsigned)((rd_cc & 1) * strip_elems * 2);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = frow[i] + shift;
      const bool ok = (unsigned)(fpy[i] + dy) < (unsigned)H && (unsigned)(fpx[i] + dx) < (unsigned)W;
      const unsigned base = ok ? sbase + (unsigned)row * 128u : lds_zero;
      const unsigned x = (unsigned)((((row >> 1) & 7) ^ fh) << 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        fa[i][s] = lds_read16(base + (x ^ (unsigned)(s << 5)));
    }
    const unsigned bbase = lds_bring + (unsigned)(rd_stage * BSTAGE * 2);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        fb[j][s] = lds_read16(bbase + boff[s] + (unsigned)(j * 32 * 128));
    rd_stage = rd_stage == 2 ? 0 : rd_stage + 1;
    if (++rd_kx == KW) {
      rd_kx = 0;
      if (++rd_ky == a.KH) {
        rd_ky = 0;
        ++rd_cc;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto mfma_sub = [&](bf16x8 (&fa)[TM][4], bf16x8 (&fb)[TN][4], int s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = mma16<F16>(fa[i][s], fb[j][s], acc[i][j]);
  };

  bf16x8 fa0[TM][4], fb0[TN][4], fa1[TM][4], fb1[TN][4];
  // prologue: three steps in flight, fragments of step 0 in registers
  issue_next();
  if (nsteps > 1) issue_next();
  if (nsteps > 2) issue_next();
  if (nsteps > 2) wait_vmcnt<2 * BI>();
  else wait_vmcnt<0>();
  __syncthreads();  // also publishes the zero row
  read_frags(fa0, fb0);

  // one step: MFMAs of step t from (ca, cb) with the next step's LDS reads (into na, nb)
  // in the middle, after the wait + barrier that make step t+1 (and the strip) visible
  auto step = [&](bf16x8 (&ca)[TM][4], bf16x8 (&cb)[TN][4], bf16x8 (&na)[TM][4], bf16x8 (&nb)[TN][4],
                  int t) __attribute__((always_inline)) {
    mfma_sub(ca, cb, 0);
    mfma_sub(ca, cb, 1);
    if (t + 1 < nsteps) {
      if (t + 2 < nsteps) wait_vmcnt<BI>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (is_t < nsteps) issue_next();
      read_frags(na, nb);
    }
    mfma_sub(ca, cb, 2);
    mfma_sub(ca, cb, 3);
  };
  for (int t = 0; t < nsteps; t += 2) {
    step(fa0, fb0, fa1, fb1, t);
    if (t + 1 < nsteps) step(fa1, fb1, fa0, fb0, t + 1);
  }
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  fwd_epilogue<BM, BN, TM, TN, NW, 2, 0, F16>(a, reinterpret_cast<float*>(dsm), acc, m0, n0, P, Nn);
}

// raise a kernel's dynamic-LDS limit once (it only ever grows)
inline void set_lds_limit(const void* fn, int bytes) {
  static thread_local const void* last_fn[8] = {};
  static thread_local int last_bytes[8] = {};
  for (int i = 0; i < 8; ++i)
    if (last_fn[i] == fn && last_bytes[i] >= bytes) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int i = 0; i < 8; ++i)
    if (last_fn[i] == nullptr || last_fn[i] == fn) {
      last_fn[i] = fn;
      last_bytes[i] = 160 * 1024;
      return;
    }
}

// LDS bytes of conv_fwd5<BM, BN> for a given strip (0 if it does not fit in 160 KB)
inline long fwd5_lds_bytes(int BM, int BN, int strip_rows) {
  const long ring = 2L * strip_rows * 64 * 2 + 3L * BN * 64 * 2 + 128;
  const long epi = (long)BM * (BN + 4) * 4;
  const long need = ring > epi ? ring : epi;
  return need <= 160 * 1024 ? need : 0;
}

// ============================================================================ forward v6 (lean halo strip)
// Same operand reuse as v5 (one LDS strip per 64-channel chunk serves every tap, 3-stage
// weight ring, LDS-DMA), re-built for instruction issue: a v5 K step issued ~185 instructions
// per wave (~100 of them scalar bookkeeping of the runtime tap/chunk state machine) and
// 2.5 LDS-DMA pieces around 8 MFMAs, so the waves were issue-bound (the MFMA-, DMA- and
// read-free probes of profiles/r3_probe_conv5.log each removed only part of the step).  v6:
//   * taps are template parameters: the tap loop is fully unrolled, the strip parity and the
//     weight-ring stage of every step are compile-time, so LDS addresses are per-lane
//     registers computed once (A: one base per tap and 32-row fragment with out-of-image
//     taps redirected to a zero row; B: one per sub-step) plus immediate offsets;
//   * 64x64 wave tiles (16 MFMAs per 64-deep step, 1 KB of LDS fragment reads per MFMA);
//   * fragments of step t+1 are read right after step t's barrier, behind all 16 MFMAs of
//     step t (one full step of latency cover);
//   * tile shapes with fewer DMA pieces per MAC: 256x64 (4 waves, 4x1) moves 32% fewer bytes
//     into the CU per MAC than 128x128 on a 3x3 conv (weights 8 KB + strip ~5 KB per 1 MMAC
//     step vs 16 + 3.6 KB).
// LDS (bytes): [0, RING) weight ring (NS stages of BN rows x 128 B), then two strip buffers of
// SB bytes; the last 128-B row of each strip buffer is a zero row.
constexpr int kLdsMax = 160 * 1024;

// Flat strips (TW == 0) take the whole 160 KB (their strip length depends on the image width);
// 2-D tiles size the strip buffers to their halo block, so a small tile (BM = 128) fits two
// workgroups per CU -- two waves per SIMD, and a grid quantised over 512 slots instead of 256.
// NS: weight-ring stages = K steps of DMA lead.  (A 4-stage ring on the 2-D tiles measured -1 %,
// profiles/r5y_bench_ns4*.json: the convs are not DMA-latency bound.)
template <int BM, int BN, int NW, int KH, int KW, int TW>
struct Fwd6Cfg {
  static constexpr int NT = KH * KW;
  static constexpr int NS = 3;                        // weight ring stages
  // chunks per unrolled block: U * NT % lcm(NS, 2) == 0 and U even, so the stage (step % NS),
  // register set (step & 1) and strip parity (chunk & 1) are compile-time
  static constexpr int U = (NT % 3 == 0) ? 2 : 6;
  static constexpr int RING = NS * BN * 128;
  // strip rows: a 2-D tile's halo block; a flat 1 x KW strip's BM + KW - 1 pixels (independent of
  // the image width); other flat strips take what the 160 KB leave
  static constexpr int HROWS2 = TW > 0 ? (BM / (TW > 0 ? TW : 1) + KH - 1) * (TW + KW - 1) : 0;
  static constexpr int HALO = TW > 0   ? fwd6_halo_rows(BM / (TW > 0 ? TW : 1), TW, KH, KW, NW)
                              : KH == 1 ? (BM + KW - 1 + 8 * NW - 1) / (8 * NW) * (8 * NW)
                                        : 0;
  static constexpr int SB = HALO > 0 && BM <= 128 ? (HALO + 1) * 128 : fwd6_sb(BN);  // odd strip = +SB
  static constexpr int MAX_ROWS = SB / 128 - 1;       // strip rows (the last row is the zero row)
  static constexpr int EPI = BM * (BN + 4) * 4;       // the epilogue's fp32 staging tile
  static constexpr int LDS = (RING + 2 * SB) > EPI ? (RING + 2 * SB) : EPI;
  static_assert(LDS <= kLdsMax && SB <= 65408, "LDS budget");
};

template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int N>
__device__ __forceinline__ void wait_vmcnt_le(int n) {
  // s_waitcnt needs an immediate: dispatch a runtime count (uniform) to the nearest
  // immediate <= n (waiting for more than needed is safe)
  if constexpr (N <= 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N) wait_vmcnt<N>();
    else wait_vmcnt_le<N - 1>(n);
  }
}

// TW > 0: 2-D output tiles of (BM / TW) image rows x TW columns (wide images, where the flat
// strip of BM + (KH-1) W + KW-1 rows no longer fits in LDS): the strip is the tile's halo
// block of (BM/TW + KH-1) x (TW + KW-1) pixels with pitch TW + KW-1, so a tap is still one
// constant row shift, and pixels outside the image are DMA'd as zeros (no per-tap masking).
template <int BM, int BN, int WGM, int WGN, int KH, int KW, int TW = 0, bool F16 = false>
__global__ __launch_bounds__(WGM * WGN * 64) void conv_fwd6_kernel(const ConvFwdArgs a, int strip_rows) {
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;  // wave tile
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int NT = KH * KW;
  using CF = Fwd6Cfg<BM, BN, WGM * WGN, KH, KW, TW>;
  constexpr int NS = CF::NS, SB = CF::SB, RING = CF::RING;
  constexpr int BI = BN / (8 * NW);  // weight pieces (8 rows x 128 B) per wave per step
  constexpr int BSTAGE = BN * 128;
  static_assert(BI >= 1 && TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "tile");
  static_assert((NS - 1) * BSTAGE + (TN - 1) * 4096 < 65536, "ring offsets must fit the ds_read immediate");
  extern __shared__ __attribute__((aligned(1024))) __bf16 dsm[];
  char* const lds = reinterpret_cast<char*>(dsm);
  const unsigned lds0 = (unsigned)(reinterpret_cast<uintptr_t>(dsm) & 0xffffffffu);

  const int Cin = a.Cin, Kpad = a.Kpad, H = a.H, W = a.W, PH = a.PH, PW = a.PW;
  const int P = (int)a.P;
  const int Nn = a.N;
  const int sc0 = a.src[0].C, sc1 = a.src[1].C;
  const int nsrc = a.nsrc;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.src[0].ptr, (unsigned)(a.P * a.src[0].stride * 2));
  const __amdgpu_buffer_rsrc_t r1 =
      make_rsrc(nsrc > 1 ? a.src[1].ptr : a.src[0].ptr, nsrc > 1 ? (unsigned)(a.P * a.src[1].stride * 2) : 0u);
  const __amdgpu_buffer_rsrc_t r2 =
      make_rsrc(nsrc > 2 ? a.src[2].ptr : a.src[0].ptr, nsrc > 2 ? (unsigned)(a.P * a.src[2].stride * 2) : 0u);
  const unsigned st0 = (unsigned)a.src[0].stride * 2, st1 = (unsigned)a.src[1].stride * 2,
                 st2 = (unsigned)a.src[2].stride * 2;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wt, (unsigned)((long)Nn * Kpad * 2));

  constexpr int TH = TW > 0 ? BM / TW : 1;          // 2-D tile rows
  constexpr int HWD = TW + KW - 1;                  // 2-D halo block pitch (pixels)
  constexpr int HROWS = (TH + KH - 1) * HWD;        // 2-D halo block pixels
  constexpr int SPW2 = (HROWS + 8 * NW - 1) / (8 * NW);  // its DMA pieces per wave (at most)
  // 8-row pieces of the halo block (the halo is padded to whole pieces, not to SPW2 * NW)
  constexpr int NPIECE = (HROWS + 7) / 8;
  // LDS chunk swizzle of halo row r: (r >> 1) & 7 keeps a 16-lane ds_read_b128 group on 16
  // distinct slots when its rows are consecutive, but a 3x3 tap on 16-wide tiles reads two tile
  // rows 18 halo rows apart, and the row-parity / (r >> 1) pairs then collide (2-way on every
  // group: 1.21 conflict cycles per LDS instruction, profiles/r5q_pmc_summary.txt).  Keyed on
  // the halo COLUMN instead ((r % HWD) >> 1) those groups are conflict-free (the 1x5 / 5x1
  // halo shapes keep the row key, conflict-free there).
  const bool colsw = TW >= 16 && KW == 3 && a.swz_col != 0;
  auto fsw = [&](int r) { return colsw ? (((r % HWD) >> 1) & 7) : ((r >> 1) & 7); };
  static_assert(TW == 0 || (BM % TW == 0 && TW % 8 == 0 && NPIECE * 8 <= CF::MAX_ROWS), "2-D tile");
  const int tilesN = (Nn + BN - 1) / BN;
  int tilesM;
  if constexpr (TW == 0) tilesM = (P + BM - 1) / BM;
  else tilesM = a.B * ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
  const int wg = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int tm = wg / tilesN, tn = wg - (wg / tilesN) * tilesN;
  const int m0 = TW == 0 ? tm * BM : 0;
  const int n0 = tn * BN;
  const int halo_lo = PH * W + PW;
  Tile2D t2{};
  if constexpr (TW > 0) {
    const int tx = (W + TW - 1) / TW, per_img = tx * ((H + TH - 1) / TH);
    const int b = tm / per_img, rem = tm - b * per_img;
    t2 = Tile2D{(long)b * H * W, (rem / tx) * TH, (rem - (rem / tx) * tx) * TW, H, W};
  }

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int lrow = lane >> 3, lpc = lane & 7;
  const int fr = lane & 31, fh = lane >> 5;
  // zero rows (the last row of each strip buffer)
  if (tid < 16) {
    const int b = tid >> 3, c = tid & 7;
    *reinterpret_cast<u32x4*>(lds + RING + b * SB + (SB - 128) + c * 16) = u32x4{0, 0, 0, 0};
  }

  // A: per (tap, 32-row fragment) LDS byte address of this lane's row in an even-chunk strip,
  // XOR-ready (sub-step s reads addr ^ (s << 5)); out-of-image taps point at the zero row
  unsigned abase[NT][TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int frow = wm * WM + i * 32 + fr;
    if constexpr (TW > 0) {
#pragma unroll
      for (int tap = 0; tap < NT; ++tap) {
        const int row = (frow / TW + tap / KW) * HWD + frow % TW + tap % KW;
        abase[tap][i] = lds0 + RING + (unsigned)row * 128u + (((unsigned)fsw(row) ^ fh) << 4);
      }
      continue;
    }
    const int p = m0 + frow;
    int py = -(1 << 20), px = -(1 << 20);
    if (p < P) {
      const int rem = p % (H * W);
      py = rem / W;
      px = rem - py * W;
    }
#pragma unroll
    for (int tap = 0; tap < NT; ++tap) {
      const int ky = tap / KW, kx = tap % KW;
      const int row = frow + ky * W + kx;
      const bool ok = (unsigned)(py + ky - PH) < (unsigned)H && (unsigned)(px + kx - PW) < (unsigned)W;
      abase[tap][i] = ok ? lds0 + RING + (unsigned)row * 128u + ((((row >> 1) & 7) ^ fh) << 4)
                         : lds0 + RING + (SB - 128);
    }
  }
  // B: per sub-step LDS byte offset of this lane's weight row within a stage
  unsigned bb[4];
  {
    const int row = wn * WN + fr;
#pragma unroll
    for (int s = 0; s < 4; ++s) bb[s] = lds0 + (unsigned)(row * 128) + (((((row >> 1) & 7) ^ fh) << 4) ^ (s << 5));
  }
  // weight DMA pieces of this wave: rows (wave * BI + i) * 8 + lrow of the stage
  unsigned bvoff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * 8 + lrow;
    bvoff[i] = (n0 + row < Nn) ? (unsigned)((n0 + row) * Kpad * 2 + swz(row, lpc) * 16) : kOOB;
  }
  const int nchunks = Cin / 64;
  // strip pieces of this wave (flat: strip_rows % (8 NW) == 0; 2-D: pieces wave, wave + NW, ...)
  const int spw = TW > 0 ? (NPIECE - wave + NW - 1) / NW : strip_rows / (8 * NW);
  const unsigned sswz = (unsigned)((lpc ^ (((wave & 1) << 2) | (lrow >> 1))) * 16);
  const int pstrip = m0 - halo_lo + wave * 8 + lrow;  // pixel of this lane's row in piece 0
  // 2-D: image pixel of this lane's halo row in each of its pieces (-1: outside the image)
  int spix[TW > 0 ? SPW2 : 1];
  unsigned sswq[TW > 0 ? SPW2 : 1];  // 2-D: source chunk offset of this lane's row in each piece
  if constexpr (TW > 0) {
#pragma unroll
    for (int q = 0; q < SPW2; ++q) {
      const int r = (wave + q * NW) * 8 + lrow;
      sswq[q] = (unsigned)((lpc ^ fsw(r)) * 16);
      const int y = t2.y0 - PH + r / HWD, x = t2.x0 - PW + r % HWD;
      spix[q] = (r < HROWS && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) ? (int)t2.pbase + y * W + x
                                                                                     : -1;
    }
  }

  // ---- DMA issue of a step: chunk cu (runtime), tap TU, ring stage SU, strip parity HU
  auto issue = [&](int cu, auto tuc, auto suc, auto huc) __attribute__((always_inline)) {
    constexpr int TU = decltype(tuc)::value, SU = decltype(suc)::value, HU = decltype(huc)::value;
    const unsigned k0b = (unsigned)((TU * Cin + cu * 64) * 2);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      bload16(rw, reinterpret_cast<__bf16*>(lds + SU * BSTAGE + (wave * BI + i) * 1024), bvoff[i], k0b);
    if constexpr (TU == 0) {
      const int c0 = cu * 64;
      __amdgpu_buffer_rsrc_t rs = r0;
      unsigned st = st0, soff = (unsigned)c0 * 2;
      if (c0 >= sc0 + sc1) {
        rs = r2; st = st2; soff = (unsigned)(c0 - sc0 - sc1) * 2;
      } else if (c0 >= sc0) {
        rs = r1; st = st1; soff = (unsigned)(c0 - sc0) * 2;
      }
      char* const sbuf = lds + RING + HU * SB + wave * 1024;
      if constexpr (TW > 0) {
#pragma unroll
        for (int q = 0; q < SPW2; ++q) {
          if (NPIECE == SPW2 * NW || wave + q * NW < NPIECE) {  // uniform per wave
            const unsigned voff = spix[q] >= 0 ? (unsigned)spix[q] * st + sswq[q] : kOOB;
            bload16(rs, reinterpret_cast<__bf16*>(sbuf + q * NW * 1024), voff, soff);
          }
        }
      } else {
        for (int q = 0; q < spw; ++q) {
          const int p = pstrip + q * NW * 8;
          const unsigned voff = (unsigned)p < (unsigned)P ? (unsigned)p * st + sswz : kOOB;
          bload16(rs, reinterpret_cast<__bf16*>(sbuf + q * NW * 1024), voff, soff);
        }
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  bf16x8 fa[2][TM][4], fb[2][TN][4];
  // fragments of the step with in-block index G (tap G % NT, stage G % 3, strip parity
  // (G / NT) & 1) into register set G & 1
  // sub-step s (16 k) of the fragments of the step with in-block index G
  auto read_s = [&](auto gc, auto sc) __attribute__((always_inline)) {
    constexpr int G = decltype(gc)::value, s = decltype(sc)::value;
    constexpr int T = G % NT, R = G & 1;
    constexpr unsigned AOFF = ((G / NT) & 1) ? (unsigned)SB : 0u;
    constexpr unsigned BOFF = (unsigned)((G % NS) * BSTAGE);
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[R][i][s] = lds_read16((abase[T][i] ^ (unsigned)(s << 5)) + AOFF);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[R][j][s] = lds_read16(bb[s] + BOFF + (unsigned)(j * 4096));
  };
  auto read = [&](auto gc) __attribute__((always_inline)) {
    static_for<4>([&](auto sc) __attribute__((always_inline)) { read_s(gc, sc); });
  };
  auto mfma_s = [&](auto rc, auto sc) __attribute__((always_inline)) {
    constexpr int R = decltype(rc)::value, s = decltype(sc)::value;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = mma16<F16>(fa[R][i][s], fb[R][j][s], acc[i][j]);
  };
  // issue the step with in-block index GU of the block starting at chunk cb (GU may run past
  // the block: stage and parity stay compile-time because U * NT % 6 == 0)
  auto issue_g = [&](int cb, auto guc) __attribute__((always_inline)) {
    constexpr int GU = decltype(guc)::value;
    const int cu = cb + GU / NT;
    if (cu < nchunks)
      issue(cu, std::integral_constant<int, GU % NT>{}, std::integral_constant<int, GU % NS>{},
            std::integral_constant<int, (GU / NT) & 1>{});
  };

  // prologue: steps 0 .. NS-1 in flight (NT >= 5: all in chunk 0), fragments of step 0
  static_for<NS>([&](auto gc) __attribute__((always_inline)) { issue_g(0, gc); });
  wait_vmcnt<(NS - 1) * BI>();
  __syncthreads();  // also publishes the zero rows
  read(std::integral_constant<int, 0>{});

  // one K step: in-block index G of the block starting at chunk cb
  auto step = [&](int cb, auto gc) __attribute__((always_inline)) {
    constexpr int G = decltype(gc)::value;
    const bool has1 = cb + (G + 1) / NT < nchunks;  // step t+1 exists
    const bool has2 = cb + (G + 2) / NT < nchunks;  // step t+2 exists (issued one step ago)
    // sched_barrier(0) fences keep the compiler from sinking each MFMA next to its fragment
    // read (it would otherwise trade the one-step read-ahead for registers)
    __builtin_amdgcn_sched_barrier(0);
    if (has1) {
      // step t+1 landed; steps t+2 .. t+NS-1 may stay in flight (BI pieces each, + the strip
      // of the one that opens a chunk)
      constexpr int OPEN = (G + 2) % NT == 0 ? 1 : 0;
      if (!has2) wait_vmcnt<0>();
      else if constexpr (OPEN) wait_vmcnt_le<40>(BI + spw);
      else wait_vmcnt<BI>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // step t+NS into the stage of step t (its fragments were read before this barrier)
      issue_g(cb, std::integral_constant<int, G + NS>{});
      __builtin_amdgcn_sched_barrier(0);
      // MFMA sub-step s of step t, then the sub-step-s reads of step t+1: every MFMA group
      // precedes the reads issued after it, so the compiler's lgkmcnt (at most 15 in flight)
      // never holds an MFMA behind this step's new reads
      static_for<4>([&](auto sc) __attribute__((always_inline)) {
        mfma_s(std::integral_constant<int, G & 1>{}, sc);
        __builtin_amdgcn_sched_barrier(0);
        read_s(std::integral_constant<int, G + 1>{}, sc);
        __builtin_amdgcn_sched_barrier(0);
      });
    } else {
      static_for<4>([&](auto sc) __attribute__((always_inline)) {
        mfma_s(std::integral_constant<int, G & 1>{}, sc);
      });
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int cb = 0; cb < nchunks; cb += CF::U) {
    static_for<CF::U * NT>([&](auto gc) __attribute__((always_inline)) {
      constexpr int G = decltype(gc)::value;
      if (cb + G / NT < nchunks) step(cb, gc);
    });
  }
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  fwd_epilogue<BM, BN, TM, TN, NW, WGN, TW, F16>(a, reinterpret_cast<float*>(dsm), acc, m0, n0, P, Nn, t2);
}


// ============================================================================ 1x1 GEMM (v7)
// The update block's 1x1 convs (convc1 324 -> 256, mask.2 256 -> 576 and their data gradients)
// are plain GEMMs with a short K (256-576): on v4 each 64x128 tile ran 4-9 K steps whose issue
// recomputed the im2col tap / bounds state per piece (~19 VALU per MFMA, r4_pmc_summary_final)
// and read its fragments in front of the MFMAs.  v7: a single source row per pixel, so every
// lane's DMA offsets are computed once and the K step rides in the scalar soffset; the
// fwd6 pipeline (3-stage ring, fragments of step t+1 read behind the MFMAs of step t, raw
// barriers, counted vmcnt); 128 x 64 tiles in 72 KB so two workgroups share a CU.  (A 2-stage
// ring at three workgroups per CU ran faster alone but -1.2 % in-step, profiles/r5ai_*.)
template <int BM, int BN, int WGM, int WGN, bool F16 = false>
__global__ __launch_bounds__(WGM * WGN * 64) void conv_fwd7_kernel(const ConvFwdArgs a) {
  constexpr int NS = 3;
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW);  // DMA pieces per wave per step
  constexpr int STAGE = (BM + BN) * 128;                 // bytes
  static_assert(AI >= 1 && BI >= 1 && TM >= 1 && TN >= 1, "tile");
  static_assert(NS * STAGE >= BM * (BN + 4) * 4, "epilogue tile must fit the ring");
  extern __shared__ __attribute__((aligned(1024))) __bf16 dsm[];
  char* const lds = reinterpret_cast<char*>(dsm);
  const unsigned lds0 = (unsigned)(reinterpret_cast<uintptr_t>(dsm) & 0xffffffffu);

  const int P = (int)a.P, Nn = a.N, Kpad = a.Kpad;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.src[0].ptr, (unsigned)(a.P * a.src[0].stride * 2));
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.wt, (unsigned)((long)Nn * Kpad * 2));
  const unsigned xst = (unsigned)a.src[0].stride * 2;
  const int tilesN = (Nn + BN - 1) / BN, tilesM = (P + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int tm = wg / tilesN, tn = wg - (wg / tilesN) * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int lrow = lane >> 3, lpc = lane & 7;
  const int fr = lane & 31, fh = lane >> 5;
  unsigned avoff[AI], bvoff[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wave * AI + i) * 8 + lrow;
    avoff[i] = (m0 + row < P) ? (unsigned)(m0 + row) * xst + (unsigned)(swz(row, lpc) * 16) : kOOB;
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * 8 + lrow;
    bvoff[i] = (n0 + row < Nn) ? (unsigned)((n0 + row) * Kpad * 2 + swz(row, lpc) * 16) : kOOB;
  }
  // per-lane LDS fragment addresses (XOR-ready: sub-step s reads addr ^ (s << 5))
  unsigned aaddr[TM], baddr[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wm * WM + i * 32 + fr;
    aaddr[i] = lds0 + (unsigned)row * 128u + ((((row >> 1) & 7) ^ fh) << 4);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int row = BM + wn * WN + j * 32 + fr;
    baddr[j] = lds0 + (unsigned)row * 128u + ((((row >> 1) & 7) ^ fh) << 4);
  }
  const int nk = Kpad / 64;
  auto issue = [&](int t, int st) __attribute__((always_inline)) {
    const unsigned soff = (unsigned)t * 128u;  // 64 channels = 128 bytes per step
    char* sa = lds + st * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i) bload16(rx, reinterpret_cast<__bf16*>(sa + (wave * AI + i) * 1024), avoff[i], soff);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      bload16(rw, reinterpret_cast<__bf16*>(sa + BM * 128 + (wave * BI + i) * 1024), bvoff[i], soff);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  bf16x8 fa[2][TM][4], fb[2][TN][4];
  auto read = [&](auto rc, int st) __attribute__((always_inline)) {
    constexpr int R = decltype(rc)::value;
    const unsigned off = (unsigned)(st * STAGE);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[R][i][s] = lds_read16((aaddr[i] ^ (unsigned)(s << 5)) + off);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[R][j][s] = lds_read16((baddr[j] ^ (unsigned)(s << 5)) + off);
    }
  };
  constexpr int G = AI + BI;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  if (nk > 2) issue(2, 2);
  if (nk > 2) wait_vmcnt<2 * G>();
  else if (nk > 1) wait_vmcnt<G>();
  else wait_vmcnt<0>();
  __syncthreads();
  read(std::integral_constant<int, 0>{}, 0);
  auto step = [&](int t, auto rc) __attribute__((always_inline)) {
    constexpr int R = decltype(rc)::value;
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nk) {
      if (t + 2 < nk) wait_vmcnt<G>();  // step t+1 landed, t+2 may stay in flight
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + NS < nk) issue(t + NS, t % NS);  // into the stage step t was read from
      __builtin_amdgcn_sched_barrier(0);
      const unsigned off = (unsigned)(((t + 1) % NS) * STAGE);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma16<F16>(fa[R][i][s], fb[R][j][s], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[R ^ 1][i][s] = lds_read16((aaddr[i] ^ (unsigned)(s << 5)) + off);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[R ^ 1][j][s] = lds_read16((baddr[j] ^ (unsigned)(s << 5)) + off);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma16<F16>(fa[R][i][s], fb[R][j][s], acc[i][j]);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < nk; t += 2) {
    step(t, std::integral_constant<int, 0>{});
    if (t + 1 < nk) step(t + 1, std::integral_constant<int, 1>{});
  }
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  fwd_epilogue<BM, BN, TM, TN, NW, WGN, 0, F16>(a, reinterpret_cast<float*>(dsm), acc, m0, n0, P, Nn);
}

// ============================================================================ wgrad helpers
constexpr int WBK = kWgradBK;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(reinterpret_cast<uintptr_t>(p) & 0xffffffffu));
}

}  // namespace

namespace {
// ============================================================================ wgrad v2
// dW[n][k] += sum_p dY[p][n] * im2col(X)[p][k], reduction over 64-pixel K steps.
// Both operands are DMA'd by bounds-checked buffer_load ... lds into an S-stage ring
// in their natural [pixel][column] layout and consumed with ds_read_b64_tr_b16
// transposed reads.  The lane -> (row, 16-byte chunk) map of the DMA image fixes each
// lane's column chunk for the whole reduction, so its k -> (tap, channel) decode is done
// once; pixel rows advance incrementally.  Chunks are XOR-swizzled inside 64-byte groups
// so the 4 rows one transposed read touches fall on disjoint banks.
template <int COLS>
__device__ __forceinline__ int wswz(int row, int chunk) {
  return COLS == 128 ? (chunk ^ ((row & 3) << 2)) : (chunk ^ (((row >> 1) & 1) << 2));
}

template <int BM, int BN, int S, bool F16 = false>
__global__ __launch_bounds__(256) void conv_wgrad2_kernel(const ConvWgradArgs a) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;      // chunks per row
  constexpr int ARPI = 64 / ACPR, BRPI = 64 / BCPR;  // rows per wave-instruction
  constexpr int AI = 64 / (4 * ARPI), BI = 64 / (4 * BRPI);
  constexpr int G = AI + BI;
  constexpr int STAGE = 64 * (BM + BN);
  __shared__ __attribute__((aligned(1024))) __bf16 smem[S * STAGE];

  const int tilesM = (a.N + BM - 1) / BM;
  const int tilesN = (a.K + BN - 1) / BN;
  const int tiles = tilesM * tilesN;
  int split, t0;
  wgrad_block_map(blockIdx.x, tiles, a.xcd_g, split, t0);
  const int tm = t0 / tilesN, tn = t0 - (t0 / tilesN) * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int P = (int)a.P;
  const int pbeg = (int)(split * a.pix_per_split);
  const int pend = min(pbeg + (int)a.pix_per_split, P);
  const int H = a.H, W = a.W;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // ---- A = dY rows: lane's logical chunk (fixed), byte offsets of its rows
  const int arl = lane / ACPR;  // row within the instruction's row block
  const int achunk = wswz<BM>(arl, lane % ACPR);
  const bool a_ok = m0 + achunk * 8 < a.N;
  const unsigned dyst = (unsigned)a.dy_stride * 2;
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(a.dy, (unsigned)(a.P * a.dy_stride * 2));

  // ---- B = im2col(X) rows: lane's k chunk -> tap / channel, once
  const int brl = lane / BCPR;
  const int bchunk = wswz<BN>(brl, lane % BCPR);
  const int kb = n0 + bchunk * 8;
  const bool b_ok = kb < a.K;
  int tap = 0, c = 0;
  if (b_ok) {
    tap = kb / a.Cin;
    c = kb - tap * a.Cin;
  }
  const int ky = tap / a.KW;
  const int dyy = ky - a.PH, dxx = tap - ky * a.KW - a.PW;
  // the whole k tile lies in one source segment (host check) -> uniform resource
  const int kt0 = n0 % a.Cin;
  int seg = 0, cseg = c;
  if (kt0 >= a.src[0].C) {
    seg = 1;
    if (kt0 >= a.src[0].C + a.src[1].C) seg = 2;
  }
  if (seg >= 1) cseg -= a.src[0].C;
  if (seg == 2) cseg -= a.src[1].C;
  const __bf16* xptr = seg == 0 ? a.src[0].ptr : (seg == 1 ? a.src[1].ptr : a.src[2].ptr);
  const long xstride = seg == 0 ? a.src[0].stride : (seg == 1 ? a.src[1].stride : a.src[2].stride);
  const int xper0 = seg == 0 ? a.src[0].period : (seg == 1 ? a.src[1].period : a.src[2].period);
  const int xper = xper0 > 0 ? xper0 : P;  // rows of this source (pixel p reads row p % xper)
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(xptr, (unsigned)((long)xper * xstride * 2));
  const unsigned xst = (unsigned)xstride * 2;
  const int doff = dyy * W + dxx;

  // pixel walkers for this lane's B rows: flat pixel (bounds), source row (address), image coords
  int bp[BI], bw[BI], bpy[BI], bpx[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int p = pbeg + (wave * BI + i) * BRPI + brl;
    bp[i] = p;
    bw[i] = p % xper;
    const int rem = p % (H * W);
    bpy[i] = rem / W;
    bpx[i] = rem - bpy[i] * W;
  }

  const int nsteps = pend > pbeg ? (pend - pbeg + 63) / 64 : 0;

#define RAFT_WG_ISSUE(step, stage)                                                                         \
  do {                                                                                                     \
    __bf16* sA_ = smem + (stage) * STAGE;                                                                  \
    __bf16* sB_ = sA_ + 64 * BM;                                                                           \
    const int p0_ = pbeg + (step) * 64;                                                                    \
    _Pragma("unroll") for (int i = 0; i < AI; ++i) {                                                       \
      const int p = p0_ + (wave * AI + i) * ARPI + arl;                                                    \
      const unsigned voff = (a_ok && p < pend) ? (unsigned)p * dyst + (unsigned)(achunk * 16) : kOOB;      \
      bload16(rdy, sA_ + (wave * AI + i) * 512, voff, (unsigned)m0 * 2);                                   \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < BI; ++i) {                                                       \
      const bool ok = b_ok && bp[i] < pend && (unsigned)(bpy[i] + dyy) < (unsigned)H &&                    \
                      (unsigned)(bpx[i] + dxx) < (unsigned)W;                                              \
      const unsigned voff = ok ? (unsigned)(bw[i] + doff) * xst + (unsigned)cseg * 2 : kOOB;              \
      bload16(rx, sB_ + (wave * BI + i) * 512, voff, 0);                                                   \
      bp[i] += 64;                                                                                         \
      bw[i] += 64;                                                                                         \
      while (bw[i] >= xper) bw[i] -= xper;                                                                 \
      bpx[i] += 64;                                                                                        \
      while (bpx[i] >= W) {                                                                                \
        bpx[i] -= W;                                                                                       \
        if (++bpy[i] >= H) bpy[i] = 0;                                                                     \
      }                                                                                                    \
    }                                                                                                      \
  } while (0)

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // bias gradient: dY fragments are also multiplied by a ones B-operand, so every output
  // column of accb holds the pixel sum of dY rows.  The 64-pixel steps are dealt to the
  // (column tile, wave column) pairs round-robin -- step t goes to tn == t % tilesN,
  // wn == (t / tilesN) & 1 -- so the extra MFMAs are spread over the whole grid.
  const bool do_db = a.dbslab != nullptr;
  f32x16 accb[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) accb[i][r] = 0.f;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = st16(1.0f, F16);

  // transposed-read lane geometry
  const int hh = lane >> 5, gi = (lane >> 4) & 1, q = (lane & 15) >> 2, pq = lane & 3;
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nsteps) RAFT_WG_ISSUE(i, i);

  for (int t = 0; t < nsteps; ++t) {
    const int ahead = (nsteps - 1 - t) < (S - 2) ? (nsteps - 1 - t) : (S - 2);
    if (ahead >= S - 2) wait_vmcnt<(S - 2) * G>();
    else if (ahead == 1) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + S - 1 < nsteps) RAFT_WG_ISSUE(t + S - 1, (t + S - 1) % S);
    const __bf16* sA = smem + (t % S) * STAGE;
    const __bf16* sB = sA + 64 * BM;
    const int tq = t / tilesN;
    const bool db_step = do_db && (t - tq * tilesN) == tn && (tq & 1) == wn;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (BM / 2) + i * 32 + gi * 16 + 4 * pq;  // logical column
        const int r0 = s * 16 + hh * 8 + q, r1 = r0 + 4;
        const s16x4 lo = tr_read(sA + r0 * BM + wswz<BM>(r0, col >> 3) * 8 + (col & 7));
        const s16x4 hi = tr_read(sA + r1 * BM + wswz<BM>(r1, col >> 3) * 8 + (col & 7));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 32 + gi * 16 + 4 * pq;
        const int r0 = s * 16 + hh * 8 + q, r1 = r0 + 4;
        const s16x4 lo = tr_read(sB + r0 * BN + wswz<BN>(r0, col >> 3) * 8 + (col & 7));
        const s16x4 hi = tr_read(sB + r1 * BN + wswz<BN>(r1, col >> 3) * 8 + (col & 7));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mma16<F16>(af[i], bfr[j], acc[i][j]);
      if (db_step) {
#pragma unroll
        for (int i = 0; i < TM; ++i) accb[i] = mma16<F16>(af[i], ones, accb[i]);
      }
    }
  }
#undef RAFT_WG_ISSUE
  wait_vmcnt<0>();
  if (a.dbslab) {
    // every column of accb holds the row sums: stage column 0 of both wave columns in LDS
    // (the ring is free now) and write this workgroup's BM partial bias sums (zeros if it
    // took no bias steps) -- the reduce kernel sums them in a fixed order
    float* sdb = reinterpret_cast<float*>(smem);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if ((lane & 31) == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sdb[wn * BM + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)] = accb[i][r];
    }
    __syncthreads();
    if (tid < BM) a.dbslab[((long)split * tilesN + tn) * a.Npad + m0 + tid] = sdb[tid] + sdb[BM + tid];
  }

  // partial dW tile of this split: plain stores (32 consecutive floats per 32 lanes)
  float* slab = a.slab + (long)split * a.Npad * a.Kpad;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + (lane & 31);
    if (col >= a.Kpad) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        slab[(long)row * a.Kpad + col] = acc[i][j][r];
      }
  }
}

// ============================================================================ wgrad v3 (tap-batched)
// dW[n][tap][c] = sum_p dY[p][n] X[p + d_tap][c] for every tap of a KHxKW conv at once.
// wgrad v2 re-fetches im2col(X) per tap (5-9x the activation bytes) and its 128x128 tile
// does 32 MAC per operand byte, so on MI355X it is bound by the L2->LDS fills, not the MFMA.
// v3 gives a workgroup BM output channels x one 64-channel input chunk x ALL taps
// (columns tap*64 + c), and per step a 2-D tile of TH x TW = 64 pixels:
//   * dY tile [64 px][BM] and the tile's halo block [(TH+KH-1) x (TW+KW-1) px][64 ch] are
//     DMA'd (buffer_load ... lds) into an S-stage ring; out-of-image rows load as zeros, so
//     the conv padding needs no masking at all;
//   * every tap reads its B fragments from the SAME halo block at a per-lane row shift
//     (ds_read_b64_tr_b16, rows = pixels), the A fragments (dY^T) are shared by all taps;
//   * ~110 MAC per operand byte (3.5x v2).
// Pixel tiles never cross an image; the (T*B, H, W) image stack is tiled, the tile list is
// split over workgroups (XCD-grouped like v2) and each split writes its own fp32 slab.
// Periodic sources: image i reads source image i % (period / HW).
template <int KH, int KW, int TH, int TW, int NW = 4>
struct WG3Geo {
  static constexpr int BH = TH + KH - 1, BW = TW + KW - 1;
  static constexpr int ROWS = (BH * BW + NW * 8 - 1) / (NW * 8) * (NW * 8);  // halo-block rows, whole DMA pieces
  static constexpr int TAPS = KH * KW;
};

// NW = 8 (8 waves as 4 x 2, MT = 1): the 128-channel tile of the 5-tap convs with half the
// accumulators per wave (80 + 16 instead of 160 + 32 registers), so one workgroup per CU still
// gives every SIMD two waves; NW = 4 with MT = 2 holds 274 registers per lane: one wave per
// SIMD, the DMA / transposed-read latency exposed (r5 profile: 376-381 us per dispatch).
template <int KH, int KW, int TH, int TW, int MT, int S, bool F16 = false, int NW = 4>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void conv_wgrad3_kernel(const ConvWgradArgs a) {
  using G3 = WG3Geo<KH, KW, TH, TW, NW>;
  static_assert(TH * TW == 64, "64-pixel tiles");
  static_assert(TW % 4 == 0, "4 consecutive tile pixels share a tile row (transposed-read rows)");
  static_assert(NW == 4 || NW == 8, "2 wave columns x 2 or 4 wave rows");
  constexpr int WR = NW / 2;           // wave rows
  constexpr int BM = 32 * WR * MT;     // WR wave rows x MT 32-row tiles
  constexpr int NT = G3::TAPS;         // 32-column tiles per wave: 2 wave columns x NT = TAPS x 64
  constexpr int ACPR = BM / 8;         // dY chunks per row
  constexpr int ARPI = 64 / ACPR;      // dY rows per wave-instruction
  constexpr int AI = 64 / (NW * ARPI);  // dY wave-instructions per wave per step
  constexpr int SI = G3::ROWS / (NW * 8);  // halo-block wave-instructions per wave per step
  static_assert(AI >= 1 && AI * NW * ARPI == 64, "dY tile DMA pieces");
  constexpr int G = AI + SI;
  constexpr int STAGE = 64 * BM + G3::ROWS * 64;  // bf16 elements
  __shared__ __attribute__((aligned(1024))) __bf16 smem[S * STAGE];

  const int H = a.H, W = a.W;
  const int tilesY = (H + TH - 1) / TH, tilesX = (W + TW - 1) / TW;
  const int tiles_img = tilesY * tilesX;
  const int nimg = a.B;
  const int ntiles = nimg * tiles_img;
  const int nchunk = a.Cin / 64;
  const int tilesM = (a.N + BM - 1) / BM;
  const int wtiles = tilesM * nchunk;
  int split, t0;
  wgrad_block_map(blockIdx.x, wtiles, a.xcd_g, split, t0);
  const int tm = t0 / nchunk, cc = t0 - tm * nchunk;
  const int m0 = tm * BM;
  const int tbeg = split * (int)a.pix_per_split;  // pix_per_split counts pixel TILES here
  const int tend = min(tbeg + (int)a.pix_per_split, ntiles);
  const int nsteps = tend > tbeg ? tend - tbeg : 0;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = H * W;

  // ---- dY (A operand) DMA geometry: lane -> (tile pixel row of its instruction, chunk)
  const int arl = lane / ACPR;
  const int achunk = wswz<BM>(arl, lane % ACPR);
  const bool a_ok = m0 + achunk * 8 < a.N;
  const unsigned dyst = (unsigned)a.dy_stride * 2;
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(a.dy, (unsigned)(a.P * a.dy_stride * 2));
  int aty[AI], atx[AI];  // tile-local pixel of each of this lane's dY rows
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int k = (wave * AI + i) * ARPI + arl;
    aty[i] = k / TW;
    atx[i] = k - aty[i] * TW;
  }

  // ---- X (B operand) source: the chunk's segment (64-channel chunks never straddle one)
  const int c0 = cc * 64;
  int seg = 0, cseg = c0;
  if (c0 >= a.src[0].C) {
    seg = 1;
    cseg -= a.src[0].C;
    if (cseg >= a.src[1].C) {
      seg = 2;
      cseg -= a.src[1].C;
    }
  }
  const __bf16* xptr = seg == 0 ? a.src[0].ptr : (seg == 1 ? a.src[1].ptr : a.src[2].ptr);
  const long xstride = seg == 0 ? a.src[0].stride : (seg == 1 ? a.src[1].stride : a.src[2].stride);
  const int xper = seg == 0 ? a.src[0].period : (seg == 1 ? a.src[1].period : a.src[2].period);
  const int ximgs = xper > 0 ? xper / HW : nimg;  // images held by the source
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(xptr, (unsigned)((long)ximgs * HW * xstride * 2));
  const unsigned xst = (unsigned)xstride * 2;
  const int lrow = lane >> 3;
  int bby[SI], bbx[SI], bchk[SI];  // halo-block position of each of this lane's block rows
#pragma unroll
  for (int i = 0; i < SI; ++i) {
    const int r = (wave * SI + i) * 8 + lrow;
    bby[i] = r < G3::BH * G3::BW ? r / G3::BW : (1 << 20);  // padding rows: never in the image
    bbx[i] = r - (r / G3::BW) * G3::BW;
    bchk[i] = wswz<64>(lrow, lane & 7);
  }

  auto issue = [&](int step, int stage) __attribute__((always_inline)) {
    __bf16* sA = smem + stage * STAGE;
    __bf16* sB = sA + 64 * BM;
    const int tile = tbeg + step;
    const int img = tile / tiles_img;
    const int trem = tile - img * tiles_img;
    const int ty0 = (trem / tilesX) * TH, tx0 = (trem - (trem / tilesX) * tilesX) * TW;
    const int pimg = img * HW;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int y = ty0 + aty[i], x = tx0 + atx[i];
      const bool ok = a_ok && y < H && x < W;
      const unsigned voff = ok ? (unsigned)(pimg + y * W + x) * dyst + (unsigned)(achunk * 16) : kOOB;
      bload16(rdy, sA + (wave * AI + i) * 512, voff, (unsigned)m0 * 2);
    }
    const int ximg = img % ximgs;
    const int by0 = ty0 - (KH / 2), bx0 = tx0 - (KW / 2);
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int y = by0 + bby[i], x = bx0 + bbx[i];
      const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      const unsigned voff = ok ? (unsigned)((ximg * H + y) * W + x) * xst + (unsigned)(bchk[i] * 16) : kOOB;
      bload16(rx, sB + (wave * SI + i) * 512, voff, (unsigned)cseg * 2);
    }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // bias gradient via a ones B operand; step t goes to chunk t % nchunk, wave column
  // (t / nchunk) & 1, so the extra MFMAs are spread over the grid
  const bool do_db = a.dbslab != nullptr;
  f32x16 accb[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) accb[i][r] = 0.f;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = st16(1.0f, F16);

  // transposed-read lane geometry: 16-lane group gi, row q within a 4-row block, column group pq
  const int hh = lane >> 5, gi = (lane >> 4) & 1, q = (lane & 15) >> 2, pq = lane & 3;
  // halo-block row of tile pixel k for tap (0, 0): (k / TW) * BW + k % TW; tap (ky, kx) adds ky*BW + kx
  int brow[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = s * 16 + hh * 8 + q + 4 * u;
      brow[s][u] = (k / TW) * G3::BW + (k - (k / TW) * TW);
    }

#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nsteps) issue(i, i);

  for (int t = 0; t < nsteps; ++t) {
    const int ahead = (nsteps - 1 - t) < (S - 2) ? (nsteps - 1 - t) : (S - 2);
    if (ahead >= S - 2) wait_vmcnt<(S - 2) * G>();
    else if (ahead == 1) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + S - 1 < nsteps) issue(t + S - 1, (t + S - 1) % S);
    const __bf16* sA = smem + (t % S) * STAGE;
    const __bf16* sB = sA + 64 * BM;
    const int tq = t / nchunk;
    const bool db_step = do_db && (t - tq * nchunk) == cc && (tq & 1) == wn;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 af[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int col = wm * (BM / WR) + i * 32 + gi * 16 + 4 * pq;
        const int r0 = s * 16 + hh * 8 + q, r1 = r0 + 4;
        const s16x4 lo = tr_read(sA + r0 * BM + wswz<BM>(r0, col >> 3) * 8 + (col & 7));
        const s16x4 hi = tr_read(sA + r1 * BM + wswz<BM>(r1, col >> 3) * 8 + (col & 7));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        // global 32-column tile jj = wn * NT + j  ->  tap jj / 2, channels (jj & 1) * 32 + ...
        const int jj = wn * NT + j;
        const int tap = jj >> 1;
        const int ky = tap / KW, kx = tap - (tap / KW) * KW;
        const int col = (jj & 1) * 32 + gi * 16 + 4 * pq;
        const int r0 = brow[s][0] + ky * G3::BW + kx, r1 = brow[s][1] + ky * G3::BW + kx;
        const s16x4 lo = tr_read(sB + r0 * 64 + wswz<64>(r0, col >> 3) * 8 + (col & 7));
        const s16x4 hi = tr_read(sB + r1 * 64 + wswz<64>(r1, col >> 3) * 8 + (col & 7));
        const bf16x8 bfr = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int i = 0; i < MT; ++i)
          acc[i][j] = mma16<F16>(af[i], bfr, acc[i][j]);
      }
      if (db_step) {
#pragma unroll
        for (int i = 0; i < MT; ++i) accb[i] = mma16<F16>(af[i], ones, accb[i]);
      }
    }
  }
  wait_vmcnt<0>();
  if (a.dbslab) {
    float* sdb = reinterpret_cast<float*>(smem);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if ((lane & 31) == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sdb[wn * BM + wm * (BM / WR) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)] = accb[i][r];
    }
    __syncthreads();
    if (tid < BM) a.dbslab[((long)split * nchunk + cc) * a.Npad + m0 + tid] = sdb[tid] + sdb[BM + tid];
  }
  // partial dW of this split, packed columns k = tap * Cin + c0 + c
  float* slab = a.slab + (long)split * a.Npad * a.Kpad;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int jj = wn * NT + j;
    const int col = (jj >> 1) * a.Cin + c0 + (jj & 1) * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / WR) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        slab[(long)row * a.Kpad + col] = acc[i][j][r];
      }
  }
}

// ============================================================================ flow encoder conv1 (7x7, 2 channels)
// convf1 (core/update.py BasicMotionEncoder: 7x7, the 2 flow channels -> 128 / 64, ReLU) has a
// tiny K (49 taps x 2 channels) that the generic paths pad 4x (flow8 carries the flow as 8
// channels, the DMA tiles work in 8-channel pieces: K = 392 -> 448).  Here the packed
// K' = tap * 2 + c (98 -> 7 MFMA K-blocks of 16) is gathered straight from a halo tile of
// the (u, v) pairs in LDS: one workgroup = an 8 x 16 pixel tile x all N output channels,
// lane fragments built from 4 32-bit LDS reads per K-block; the weights' (u, v) pairs come
// from the packed [N][Kpad] rows (k = tap * 8 + c).  Bias + ReLU + 16-bit store through an
// LDS tile (16-byte rows).
template <int N, bool F16>
__global__ __launch_bounds__(256) void conv_flow7_kernel(const ConvFwdArgs a) {
  constexpr int TH = 8, TW = 16, HH = TH + 6, HWD = TW + 6;
  constexpr int NBLK = N / 32;  // 32-column blocks; waves per column block = 4 / NBLK
  constexpr int MPW = NBLK;     // 32-pixel blocks per wave (4 in the tile)
  constexpr int OLD = N + 8;    // output tile pitch (16-bit elements)
  static_assert(N == 64 || N == 128, "convf1 widths");
  __shared__ uint32_t halo[HH * HWD];
  __shared__ __attribute__((aligned(16))) __bf16 otile[TH * TW * OLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const int tw = (W + TW - 1) / TW, th = (H + TH - 1) / TH;
  int bid = blockIdx.x;
  const int b = bid / (tw * th);
  bid -= b * tw * th;
  const int y0 = (bid / tw) * TH, x0 = (bid - (bid / tw) * tw) * TW;
  const long pbase = (long)b * H * W;
  const long sst = a.src[0].stride;
  for (int i = tid; i < HH * HWD; i += 256) {
    const int hy = i / HWD, hx = i - (i / HWD) * HWD;
    const int y = y0 + hy - 3, x = x0 + hx - 3;
    uint32_t v = 0u;
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
      v = *reinterpret_cast<const uint32_t*>(a.src[0].ptr + (pbase + (long)y * W + x) * sst);
    halo[i] = v;
  }
  const int nb = wave % NBLK, mb0 = (wave / NBLK) * MPW;
  const int fr = lane & 31, fh = lane >> 5;
  // B fragments: k' = kb * 16 + fh * 8 + i -> tap kb * 8 + fh * 4 + i / 2, channel i % 2
  bf16x8 bw[7];
  {
    const __bf16* wrow = a.wt + (long)(nb * 32 + fr) * a.Kpad;
#pragma unroll
    for (int kb = 0; kb < 7; ++kb) {
      u32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int tap = kb * 8 + fh * 4 + q;
        v[q] = tap < 49 ? *reinterpret_cast<const uint32_t*>(wrow + tap * 8) : 0u;
      }
      bw[kb] = __builtin_bit_cast(bf16x8, v);
    }
  }
  __syncthreads();
  f32x16 acc[MPW];
#pragma unroll
  for (int i = 0; i < MPW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
  for (int i = 0; i < MPW; ++i) {
    const int m = (mb0 + i) * 32 + fr;  // tile pixel of this lane's A row
    const int ty = m / TW, tx = m - (m / TW) * TW;
#pragma unroll
    for (int kb = 0; kb < 7; ++kb) {
      u32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int tap = kb * 8 + fh * 4 + q;
        const int ky = tap / 7, kx = tap - (tap / 7) * 7;
        v[q] = tap < 49 ? halo[(ty + ky) * HWD + tx + kx] : 0u;
      }
      acc[i] = mma16<F16>(__builtin_bit_cast(bf16x8, v), bw[kb], acc[i]);
    }
  }
  const int n = nb * 32 + fr;
  const float bias = a.bias ? a.bias[n] : 0.f;
  const bool relu = a.act == 1;
#pragma unroll
  for (int i = 0; i < MPW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = (mb0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
      float v = acc[i][r] * a.alpha + bias;
      if (relu) v = fmaxf(v, 0.f);
      otile[m * OLD + n] = st16(v, F16);
    }
  __syncthreads();
  constexpr int CPR = N / 8;
  for (int i = tid; i < TH * TW * CPR; i += 256) {
    const int m = i / CPR, c = i - (i / CPR) * CPR;
    const int y = y0 + m / TW, x = x0 + m % TW;
    if (y < H && x < W)
      *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(a.out) + (pbase + (long)y * W + x) * a.out_stride + c * 8) =
          *reinterpret_cast<const bf16x8*>(otile + m * OLD + c * 8);
  }
}

// ============================================================================ narrow input (Cin = 8)
// flow_head.conv2's data gradient (3x3, the 2 flow gradients in an 8-channel row -> 256,
// ReLU'-masked by the heads activation) has K = 72: on the GEMM tiles every 64-wide K step
// re-derives its im2col taps (53 us in-step at config #2 for 0.8 GFLOP, on the critical path
// of the step's backward).  With 8 channels per tap, an MFMA K block of 16 is exactly two taps,
// so a lane's A fragment (8 consecutive k) is ONE 16-byte source row: the 64-pixel tile's halo
// (6 x 18 rows) is staged in LDS and fragment (tap, pixel) is a single ds_read_b128; B
// fragments are 16-byte weight-row loads (k contiguous).  Operands swapped (C^T blocks) so a
// lane holds 4 consecutive output channels of one pixel: 8-byte masked stores.
// NPW: output channels per wave (4 waves per workgroup).  32 (128 channels per workgroup): twice
// the workgroups of NPW = 64 (384 -> 768 at config #2, ~1.5 -> 3 waves per SIMD), and the ReLU'
// mask of the epilogue is loaded before the MFMAs -- the kernel is latency-bound (0.2 GFLOP,
// 24 MB of traffic in ~30 us per call with NPW = 64).
template <bool F16, int NPW = 32>
__global__ __launch_bounds__(256) void conv_cin8_dgrad_kernel(const ConvFwdArgs a) {
  constexpr int TH = 4, TW = 16, HH = TH + 2, HWD = TW + 2;
  constexpr int JB = NPW / 32;  // 32-channel blocks per wave
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) bf16x8 halo[HH * HWD + 1];  // + a zero row (tap 9)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const int tw = (W + TW - 1) / TW, th = (H + TH - 1) / TH;
  const int nb_tiles = (a.N + 4 * NPW - 1) / (4 * NPW);
  int bid = blockIdx.x;
  const int ntile = bid % nb_tiles;
  bid /= nb_tiles;
  const int b = bid / (tw * th);
  bid -= b * tw * th;
  const int y0 = (bid / tw) * TH, x0 = (bid - (bid / tw) * tw) * TW;
  const long pbase = (long)b * H * W;
  const long sst = a.src[0].stride;
  for (int i = tid; i < HH * HWD + 1; i += 256) {
    const int hy = i / HWD, hx = i - (i / HWD) * HWD;
    const int y = y0 + hy - a.PH, x = x0 + hx - a.PW;
    bf16x8 v{};
    if (i < HH * HWD && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
      v = *reinterpret_cast<const bf16x8*>(a.src[0].ptr + (pbase + (long)y * W + x) * sst);
    halo[i] = v;
  }
  const int fr = lane & 31, fh = lane >> 5;
  const int n0 = ntile * 4 * NPW + wave * NPW;  // this wave's NPW output channels (JB blocks of 32)
  // B fragments (become the MFMA's A operand: rows = output channels): weight row n, k = kb * 16
  // + fh * 8 .. + 8 = tap 2 kb + fh, all 8 channels (taps >= 9 are zero)
  bf16x8 wf[JB][5];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int n = n0 + j * 32 + fr;
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) {
      const int tap = 2 * kb + fh;
      wf[j][kb] = (n < a.N && tap < 9) ? *reinterpret_cast<const bf16x8*>(a.wt + (long)n * a.Kpad + tap * 8) : bf16x8{};
    }
  }
  // the epilogue's ReLU' mask, loaded ahead of the MFMAs (lane: pixel i * 32 + fr, channels
  // n0 + j * 32 + 8 g + 4 fh .. + 4)
  bf16x4 mk[2][JB][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = i * 32 + fr;
    const int y = y0 + m / TW, x = x0 + m % TW;
    const bool in = y < H && x < W;
    const long p = pbase + (long)y * W + x;
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + j * 32 + 8 * g + 4 * fh;
        mk[i][j][g] = (a.mask && in && n < a.N) ? *reinterpret_cast<const bf16x4*>(a.mask + p * a.mask_stride + n)
                                                 : bf16x4{};
      }
  }
  __syncthreads();
  f32x16 acc[2][JB];  // [pixel block][channel block]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = i * 32 + fr;  // tile pixel
    const int ty = m / TW, tx = m - (m / TW) * TW;
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) {
      const int tap = 2 * kb + fh;
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
      const bf16x8 xa = halo[tap < 9 ? (ty + ky) * HWD + tx + kx : HH * HWD];
#pragma unroll
      for (int j = 0; j < JB; ++j) acc[i][j] = mma16<F16>(wf[j][kb], xa, acc[i][j]);
    }
  }
  // lane: pixel m = i * 32 + fr, channels n0 + j * 32 + 8 g + 4 fh .. + 4 (registers 4 g .. 4 g + 3)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = i * 32 + fr;
    const int y = y0 + m / TW, x = x0 + m % TW;
    if (y >= H || x >= W) continue;
    const long p = pbase + (long)y * W + x;
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + j * 32 + 8 * g + 4 * fh;
        if (n >= a.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * g + e] * a.alpha;
        if (a.mask) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (!(ld16(mk[i][j][g][e], F16) > 0.f)) v[e] = 0.f;
        }
        if (a.out_f32) {
          *reinterpret_cast<f32x4*>(static_cast<float*>(a.out) + p * a.out_stride + n) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          bf16x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = st16(v[e], F16);
          *reinterpret_cast<bf16x4*>(static_cast<__bf16*>(a.out) + p * a.out_stride + n) = w;
        }
      }
  }
}

// ============================================================================ narrow output (N <= 2)
// flow_head.conv2 (3x3, 256 -> 2) is a pair of 2,304-long dot products per pixel: a
// bandwidth problem, not a GEMM (a 64-wide MFMA tile would be 97% padding).  LPP lanes
// own one pixel, each lane 8 channels (one 16-byte load per tap); the weights live in
// registers; lanes combine with a butterfly.  Single source, bf16 in, epilogue 0
// (bias, optional ReLU) with fp32 or bf16 output.
template <int LPP>
__global__ __launch_bounds__(256) void conv_n2_fwd_kernel(const ConvFwdArgs a) {
  constexpr int PPW = 64 / LPP;  // pixels per wave per pass
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / LPP, cl = lane - sub * LPP;
  const int ntaps = a.KH * a.KW;
  const bool f16 = a.f16 != 0;
  const int Cin = a.Cin;
  float w[2][9][8];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      bf16x8 v{};
      if (n < a.N && t < ntaps) v = *reinterpret_cast<const bf16x8*>(a.wt + (long)n * a.Kpad + t * Cin + cl * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) w[n][t][q] = ld16(v[q], f16);
    }
  const float b0 = a.bias ? a.bias[0] : 0.f, b1 = (a.bias && a.N > 1) ? a.bias[1] : 0.f;
  const int HW = a.H * a.W;
  const long stride = a.src[0].stride;
  const long step = (long)gridDim.x * 4 * PPW;
  // 32-bit pixel arithmetic (the host guarantees P < 2^31): a 64-bit modulo per pixel was a
  // large share of this short loop body
  const int P = (int)a.P;
  for (int p = (blockIdx.x * 4 + wave) * PPW + sub; p < P + sub; p += (int)step) {
    float s0 = 0.f, s1 = 0.f;
    if (p < P) {
      const int rem = p % HW;
      const int py = rem / a.W, px = rem - py * a.W;
      // no break/continue: the tap loop must fully unroll so that w[][t][] stays in
      // registers (a data-dependent exit demotes w to scratch -- 6x slower); out-of-range
      // taps load zeros under the exec mask instead
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / a.KW, kx = t - (t / a.KW) * a.KW;
        const int y = py + ky - a.PH, x = px + kx - a.PW;
        const bool ok = t < ntaps && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W;
        bf16x8 v{};
        if (ok)
          v = *reinterpret_cast<const bf16x8*>(a.src[0].ptr + (p + (long)(ky - a.PH) * a.W + (kx - a.PW)) * stride +
                                               cl * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float xv = ld16(v[q], f16);
          s0 += xv * w[0][t][q];
          s1 += xv * w[1][t][q];
        }
      }
    }
#pragma unroll
    for (int off = LPP / 2; off > 0; off >>= 1) {
      s0 += __shfl_xor(s0, off, 64);
      s1 += __shfl_xor(s1, off, 64);
    }
    if (cl == 0 && p < a.P) {
      float v0 = s0 * a.alpha + b0, v1 = s1 * a.alpha + b1;
      if (a.act == 1) {
        v0 = fmaxf(v0, 0.f);
        v1 = fmaxf(v1, 0.f);
      }
      if (a.out_f32) {
        float* o = static_cast<float*>(a.out) + p * a.out_stride;
        o[0] = v0;
        if (a.N > 1) o[1] = v1;
      } else {
        __bf16* o = static_cast<__bf16*>(a.out) + p * a.out_stride;
        o[0] = st16(v0, f16);
        if (a.N > 1) o[1] = st16(v1, f16);
      }
    }
  }
}

}  // namespace

namespace {
template <int BM, int BN, int WGM, int WGN, int KH, int KW, int TW, bool F16>
bool launch_fwd6_t(const ConvFwdArgs& a, hipStream_t s) {
  using CF = Fwd6Cfg<BM, BN, WGM * WGN, KH, KW, TW>;
  constexpr int NW = WGM * WGN;
  int rows = 0;
  long tiles;
  if constexpr (TW == 0) {
    rows = fwd6_strip_rows(BM, NW, KH, KW, a.W, CF::MAX_ROWS);
    if (rows == 0) return false;
    tiles = (a.P + BM - 1) / BM;
  } else {
    constexpr int TH = BM / TW;
    tiles = (long)a.B * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  }
  const dim3 grid((unsigned)(tiles * ((a.N + BN - 1) / BN)));
  set_lds_limit((const void*)conv_fwd6_kernel<BM, BN, WGM, WGN, KH, KW, TW, F16>, CF::LDS);
  hipLaunchKernelGGL((conv_fwd6_kernel<BM, BN, WGM, WGN, KH, KW, TW, F16>), grid, dim3(NW * 64), CF::LDS, s, a,
                     rows);
  return true;
}
// v6 tiles (forced with cfg, chosen per shape by launch_conv_fwd): 41 = 256x64 flat strip (4x1
// waves of 64x64; 3x3 / 1x5 / 5x1), 45 = 256x128 flat strip (2x2 waves of 128x64), 59 = 256x64
// as 2-D 4 x 64 tiles (3x3, 1x5), 60 = 256x64 as 2-D 8 x 32 tiles (5x1), 61 = 256x64 as 2-D
// 16 x 16 tiles (3x3, 5x1).  (Measured and
// dropped: 128x128 4-wave flat and 2-D tiles, cfg 40 / 57 / 58; all next-step reads before the
// step's MFMAs, cfg 43 / 44 / 46: profiles/r3_bench_conv6_tiles.log, r3_bench_conv6_2d.log.)
template <bool F16>
bool launch_conv_fwd6(const ConvFwdArgs& a, int cfg, hipStream_t s) {
  const bool t33 = a.KH == 3 && a.KW == 3, t15 = a.KH == 1 && a.KW == 5, t51 = a.KH == 5 && a.KW == 1;
  switch (cfg) {
    case 41:
      if (t33) return launch_fwd6_t<256, 64, 4, 1, 3, 3, 0, F16>(a, s);
      if (t15) return launch_fwd6_t<256, 64, 4, 1, 1, 5, 0, F16>(a, s);
      return t51 && launch_fwd6_t<256, 64, 4, 1, 5, 1, 0, F16>(a, s);
    case 45:
      if (t33) return launch_fwd6_t<256, 128, 2, 2, 3, 3, 0, F16>(a, s);
      if (t15) return launch_fwd6_t<256, 128, 2, 2, 1, 5, 0, F16>(a, s);
      return false;
    case 59:
      if (t33) return launch_fwd6_t<256, 64, 4, 1, 3, 3, 64, F16>(a, s);
      return t15 && launch_fwd6_t<256, 64, 4, 1, 1, 5, 64, F16>(a, s);
    case 60:
      return t51 && launch_fwd6_t<256, 64, 4, 1, 5, 1, 32, F16>(a, s);
    case 61:  // 16 x 16 2-D tiles (less halo per output pixel than 8 x 32 / 4 x 64)
      if (t33) return launch_fwd6_t<256, 64, 4, 1, 3, 3, 16, F16>(a, s);
      return t51 && launch_fwd6_t<256, 64, 4, 1, 5, 1, 16, F16>(a, s);
    // 128 x 64 2-D tiles, two workgroups (8 waves) per CU: 62 = 4x1 waves of 32 x 64, 63 = 2x2
    // waves of 64 x 32; 3x3 as 8 x 16, 1x5 as 2 x 64, 5x1 as 16 x 8 (64: 5x1 as 8 x 16)
    case 62:
      if (t33) return launch_fwd6_t<128, 64, 4, 1, 3, 3, 16, F16>(a, s);
      if (t15) return launch_fwd6_t<128, 64, 4, 1, 1, 5, 64, F16>(a, s);
      return t51 && launch_fwd6_t<128, 64, 4, 1, 5, 1, 8, F16>(a, s);
    case 63:
      if (t33) return launch_fwd6_t<128, 64, 2, 2, 3, 3, 16, F16>(a, s);
      if (t15) return launch_fwd6_t<128, 64, 2, 2, 1, 5, 64, F16>(a, s);
      return t51 && launch_fwd6_t<128, 64, 2, 2, 5, 1, 8, F16>(a, s);
    case 64:
      return t51 && launch_fwd6_t<128, 64, 4, 1, 5, 1, 16, F16>(a, s);
    case 65:  // 1x5 as a flat 128-pixel strip (132 halo rows at any width), two workgroups per CU
      return t15 && launch_fwd6_t<128, 64, 4, 1, 1, 5, 0, F16>(a, s);
    // 64 x 64 2-D tiles, 2x2 waves of 32 x 32, <= 53.5 KB of LDS: three workgroups per CU and
    // twice the workgroups of the 128 x 64 tiles (small grids: batch 1-2 per GPU).
    // 74: 3x3 as 4 x 16, 1x5 as 1 x 64, 5x1 as 8 x 8;  75: 3x3 as 8 x 8, 1x5 as 2 x 32, 5x1 as 4 x 16
    case 74:
      if (t33) return launch_fwd6_t<64, 64, 2, 2, 3, 3, 16, F16>(a, s);
      if (t15) return launch_fwd6_t<64, 64, 2, 2, 1, 5, 64, F16>(a, s);
      return t51 && launch_fwd6_t<64, 64, 2, 2, 5, 1, 8, F16>(a, s);
    case 75:
      if (t33) return launch_fwd6_t<64, 64, 2, 2, 3, 3, 8, F16>(a, s);
      if (t15) return launch_fwd6_t<64, 64, 2, 2, 1, 5, 32, F16>(a, s);
      return t51 && launch_fwd6_t<64, 64, 2, 2, 5, 1, 16, F16>(a, s);
    default:
      return false;
  }
}
}  // namespace

// v7 for the automatic 1x1 choice (RAFT_CONV_V7=0: back to v4 for A/B runs)
static const bool kUseV7 = [] {
  const char* e = std::getenv("RAFT_CONV_V7");
  return !(e && e[0] == '0');
}();

template <bool F16>
hipError_t conv_fwd_dispatch(const ConvFwdArgs& a, hipStream_t s) {
  if (a.P == 0 || a.N == 0) return hipSuccess;
  if (a.Kpad % FBK != 0) return hipErrorInvalidValue;
  const int cfg = a.cfg;
  if ((cfg == 0 || cfg == 68) && a.KH == 7 && a.KW == 7 && a.PH == 3 && a.PW == 3 && a.nsrc == 1 && a.Cin == 8 &&
      a.src[0].C == 8 && a.Kpad >= 49 * 8 && a.epi == 0 && !a.out_f32 && a.split_g == 0 && a.n2y == nullptr &&
      (a.N == 64 || a.N == 128) && a.out_stride % 8 == 0 && (reinterpret_cast<uintptr_t>(a.out) & 15) == 0 &&
      a.src[0].stride % 2 == 0 && (reinterpret_cast<uintptr_t>(a.src[0].ptr) & 3) == 0) {
    // convf1: the flow channels are the first 2 of 8 (pack_flow zero-fills the rest)
    const long tiles = (long)a.B * ((a.H + 7) / 8) * ((a.W + 15) / 16);
    if (a.N == 128) hipLaunchKernelGGL((conv_flow7_kernel<128, F16>), dim3((unsigned)tiles), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_flow7_kernel<64, F16>), dim3((unsigned)tiles), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if ((cfg == 69 || cfg == 0) && a.KH == 3 && a.KW == 3 && a.nsrc == 1 && a.Cin == 8 &&
      a.src[0].C == 8 && a.epi == 1 && a.acc_c0 >= a.N && a.split_g == 0 && a.N % 8 == 0 && a.Kpad >= 72 &&
      a.PH == 1 && a.PW == 1 && a.src[0].stride % 8 == 0 && a.out_stride % 4 == 0 &&
      (a.mask == nullptr || a.mask_stride % 4 == 0) && a.P < (1L << 31)) {
    // narrow input (flow_head.conv2's data gradient): one-tap-pair MFMA K blocks from an LDS halo
    const long tiles = (long)a.B * ((a.H + 3) / 4) * ((a.W + 15) / 16) * ((a.N + 127) / 128);  // NPW = 32
    hipLaunchKernelGGL((conv_cin8_dgrad_kernel<F16>), dim3((unsigned)tiles), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (cfg == 0 && a.N <= 2 && a.epi == 0 && a.nsrc == 1 && a.KH * a.KW <= 9 && a.src[0].C == a.Cin &&
      a.P < (1L << 30) &&
      (a.Cin == 64 || a.Cin == 128 || a.Cin == 256 || a.Cin == 512)) {
    // narrow output (flow-head conv2): register dot products, not a GEMM
    const int lpp = a.Cin / 8;
    const int ppb = 4 * (64 / lpp);
    static const long max_blocks = [] {
      const char* e = std::getenv("RAFT_N2_BLOCKS");  // experiments (scripts/bench_convs.py fh2 row)
      return e ? std::max(64L, std::atol(e)) : 2048L;
    }();
    const long blocks = std::min<long>((a.P + ppb - 1) / ppb, max_blocks);
    if (lpp == 8) hipLaunchKernelGGL(conv_n2_fwd_kernel<8>, dim3(blocks), dim3(256), 0, s, a);
    else if (lpp == 16) hipLaunchKernelGGL(conv_n2_fwd_kernel<16>, dim3(blocks), dim3(256), 0, s, a);
    else if (lpp == 32) hipLaunchKernelGGL(conv_n2_fwd_kernel<32>, dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(conv_n2_fwd_kernel<64>, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  auto tiles = [&](int bm, int bn) { return (long)((a.P + bm - 1) / bm) * ((a.N + bn - 1) / bn); };
  // DMA kernels (v4/v5) need either 64-aligned K steps or a single source segment, and
  // 32-bit buffer offsets; everything else takes the generic register-staged kernel
  const bool uniform = (a.KH * a.KW == 1) || (a.Cin % 64 == 0 && a.src[0].C % 64 == 0 && a.src[1].C % 64 == 0);
  long maxbytes = 0;
  for (int i = 0; i < a.nsrc; ++i) maxbytes = std::max(maxbytes, a.P * a.src[i].stride * 2);
  const bool dma_ok = (uniform || a.nsrc == 1) && maxbytes < (1L << 31) && (long)a.N * a.Kpad * 2 < (1L << 31);
  if (!dma_ok || cfg == 1) {
    if (a.P >= (1L << 31)) return hipErrorInvalidValue;  // 32-bit tile rows in the shared epilogue
    hipLaunchKernelGGL((conv_fwd_kernel<64, 64, F16>), dim3(tiles(64, 64)), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  // v5 (halo strip): multi-tap convs whose 64-channel chunks never straddle a source segment.
  // Tile per shape, from scripts/bench_convs.py on MI355X (B=8, 46x62): 256x128 for wide 3x3
  // convs, 128x128 for 3x3 with ~128 outputs, 128x256 for the 384-channel 1x5 z||r conv;
  // every other shape measured faster on v4.
  bool ok5 = a.KH * a.KW > 1 && a.Cin % 64 == 0 && a.N >= 64 && a.P < (1L << 30);
  for (int i = 0; i < a.nsrc; ++i) ok5 = ok5 && a.src[i].C % 64 == 0;
  int v5 = cfg >= 20 ? cfg : 0;
  if (cfg == 41 || cfg == 45 || (cfg >= 59 && cfg <= 65) || cfg == 74 || cfg == 75) {  // v6 tiles (tests / microbenchmarks)
    // (a strip buffer pair per chunk needs >= 3 taps per chunk: no 1x1 variant)
    const bool shape6 = (a.KH == 3 && a.KW == 3) || (a.KH * a.KW == 5 && (a.KH == 1 || a.KW == 1));
    if (!ok5 || !shape6 || a.PH != a.KH / 2 || a.PW != a.KW / 2) return hipErrorInvalidValue;
    return launch_conv_fwd6<F16>(a, cfg, s) ? hipGetLastError() : hipErrorInvalidValue;
  }
  if (ok5 && cfg == 0 && a.PH == a.KH / 2 && a.PW == a.KW / 2) {
    // v6 on 128 x 64 tiles (two workgroups per CU) or 64 x 64 tiles (three per CU) for every
    // 3x3 / 1x5 / 5x1 update-block shape (the rule and its measurements: choose_fwd6 in
    // kernel_abi.h, unit-tested on the host; profiles/r5b_conv6_*.log, r6t_conv6_*.log).  Before round 5: 256 x 64 / 256 x 128 one-workgroup
    // tiles (profiles/r3_bench_conv6_*.log, r4_bench_conv6_16x16.log), now forced variants.
    static const bool small_tiles = [] {  // RAFT_FWD6_SMALL=0: 128 x 64 tiles only (A/B runs)
      const char* e = std::getenv("RAFT_FWD6_SMALL");
      return !(e && e[0] == '0');
    }();
    const int v6 = choose_fwd6(a.KH, a.KW, a.N, a.B, a.H, a.W, small_tiles);
    if (v6 && launch_conv_fwd6<F16>(a, v6, s)) return hipGetLastError();
  }
  if (ok5 && v5 == 0 && cfg == 0) {
    // 8-wave tiles (two waves per SIMD, no register spills) for every shape they win on
    // (scripts/bench_convs.py, profiles/r2_bench_convs_nw.log): 3x3 with N >= 192 -> 256x128,
    // 3x3 with 64 < N < 192 -> 128x128; 1x5/5x1: the 1x5 z||r forward (N = 256) -> 128x256,
    // the 5x1 one (4-row halo), the q forwards and the 5x1 z||r data gradient -> 128x128; the
    // 1x5 data gradients (N = 384: d[h | inp | motion]) -> 64x128 with 4 waves (2x the
    // workgroups: z||r 52.3 -> 45.7 us, q 33.3 -> 29.9 us, profiles/r2_bench_convs_v5_all.log);
    // the 5x1 q data gradient (128 input channels) stays on v4
    const int taps = a.KH * a.KW;
    if (taps == 5 && a.KH == 1 && a.N == 384) v5 = 20;
    else if (taps == 9 && a.N >= 192) v5 = 24;
    else if (taps == 9 && a.N > 64) v5 = 25;
    else if (taps == 5 && a.KH == 1 && a.Cin >= 384 && a.N == 256) v5 = 26;
    else if (taps == 5 && a.Cin >= 256) v5 = 25;
  }
  if (ok5 && v5 >= 20) {
    // 20 / 21: 64x128 / 128x128 with 4 waves per workgroup; 24..26: the 256x128 / 128x128 /
    // 128x256 tiles with 8 waves
    if (v5 == 22 || v5 == 23 || v5 > 26) return hipErrorInvalidValue;
    auto bm_of = [](int v) { return v == 20 ? 64 : v == 24 ? 256 : 128; };
    auto bn_of = [](int v) { return v == 26 ? 256 : 128; };
    auto rows_of = [&](int v) { return (bm_of(v) + (a.KH - 1) * a.W + a.KW - 1 + 7) / 8 * 8; };
    long lds = fwd5_lds_bytes(bm_of(v5), bn_of(v5), rows_of(v5));
    if (lds == 0 && v5 != 21) {
      v5 = 21;
      lds = fwd5_lds_bytes(128, 128, rows_of(v5));
    }
    const int rows = rows_of(v5);
    if (lds > 0) {
      const dim3 grid(tiles(bm_of(v5), bn_of(v5)));
      switch (v5) {
        case 20:
          set_lds_limit((const void*)conv_fwd5_kernel<64, 128, 4, F16>, (int)lds);
          hipLaunchKernelGGL((conv_fwd5_kernel<64, 128, 4, F16>), grid, dim3(256), lds, s, a, rows);
          break;
        case 24:
          set_lds_limit((const void*)conv_fwd5_kernel<256, 128, 8, F16>, (int)lds);
          hipLaunchKernelGGL((conv_fwd5_kernel<256, 128, 8, F16>), grid, dim3(512), lds, s, a, rows);
          break;
        case 25:
          set_lds_limit((const void*)conv_fwd5_kernel<128, 128, 8, F16>, (int)lds);
          hipLaunchKernelGGL((conv_fwd5_kernel<128, 128, 8, F16>), grid, dim3(512), lds, s, a, rows);
          break;
        case 26:
          set_lds_limit((const void*)conv_fwd5_kernel<128, 256, 8, F16>, (int)lds);
          hipLaunchKernelGGL((conv_fwd5_kernel<128, 256, 8, F16>), grid, dim3(512), lds, s, a, rows);
          break;
        default:
          set_lds_limit((const void*)conv_fwd5_kernel<128, 128, 4, F16>, (int)lds);
          hipLaunchKernelGGL((conv_fwd5_kernel<128, 128, 4, F16>), grid, dim3(256), lds, s, a, rows);
      }
      return hipGetLastError();
    }
  }
  // v4 (scripts/bench_convs.py on MI355X): 64x128 tiles for N > 64 (the 576-wide mask-head 1x1:
  // 34.3 -> 30.0 us, profiles/r2_bench_convs_cfg8.log), 64x64 otherwise; 128x128 tiles (one
  // workgroup per CU) measured 21-30% slower on every 1x1 shape (profiles/r3_conv_1x1_tiles.log),
  // full-width 64x256 / 128x256 tiles 0-60 % slower (profiles/r5h_conv1x1*.log)
  // v7 (lean 1x1 GEMM, 128 x 64 tiles, two workgroups per CU) for single-source 1x1 convs
  const bool v7ok = a.KH == 1 && a.KW == 1 && a.nsrc == 1 && a.src[0].C == a.Cin && a.N >= 64 &&
                    (a.src[0].stride % 8) == 0 && a.P * a.src[0].stride * 2 < (1L << 31);
  if (cfg == 67 || (cfg == 0 && v7ok && kUseV7)) {
    if (!v7ok) return hipErrorInvalidValue;
    constexpr int lds7 = 3 * (128 + 64) * 128;
    set_lds_limit((const void*)conv_fwd7_kernel<128, 64, 4, 1, F16>, lds7);
    hipLaunchKernelGGL((conv_fwd7_kernel<128, 64, 4, 1, F16>), dim3(tiles(128, 64)), dim3(256), lds7, s, a);
    return hipGetLastError();
  }
  const bool wide = cfg == 8 || (cfg != 9 && a.N > 64);
  if (wide)
    hipLaunchKernelGGL((conv_fwd4_kernel<64, 128, 3, F16>), dim3(tiles(64, 128)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv_fwd4_kernel<64, 64, 4, F16>), dim3(tiles(64, 64)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_conv_fwd(const ConvFwdArgs& a_in, hipStream_t s) {
  static const int swz_col = [] {  // RAFT_SWZ_COL=0: the row-keyed swizzle everywhere (A/B runs)
    const char* e = std::getenv("RAFT_SWZ_COL");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  ConvFwdArgs a = a_in;
  a.swz_col = swz_col;
  return a.f16 ? conv_fwd_dispatch<true>(a, s) : conv_fwd_dispatch<false>(a, s);
}

template <bool F16>
hipError_t conv_wgrad_dispatch(const ConvWgradArgs& a, const WgradPlan& pl, hipStream_t s) {
  const dim3 grid((unsigned)((long)pl.tilesM * pl.tilesN * pl.nsplit));
  if (pl.kind == 3) {
    if (a.KH == 3)
      hipLaunchKernelGGL((conv_wgrad3_kernel<3, 3, 8, 8, 1, 3, F16>), grid, dim3(256), 0, s, a);
    else if (a.KH == 5 && pl.BM == 128)
      hipLaunchKernelGGL((conv_wgrad3_kernel<5, 1, 16, 4, 2, 3, F16>), grid, dim3(256), 0, s, a);
    else if (a.KH == 5)
      hipLaunchKernelGGL((conv_wgrad3_kernel<5, 1, 16, 4, 1, 3, F16>), grid, dim3(256), 0, s, a);
    else if (pl.BM == 128)
      hipLaunchKernelGGL((conv_wgrad3_kernel<1, 5, 1, 64, 2, 3, F16>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad3_kernel<1, 5, 1, 64, 1, 3, F16>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (a.wg2_stages == 2) {  // two workgroups per CU (see ConvWgradArgs::wg2_stages)
    if (pl.BM == 128)
      hipLaunchKernelGGL((conv_wgrad2_kernel<128, 128, 2, F16>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_wgrad2_kernel<64, 128, 2, F16>), grid, dim3(256), 0, s, a);
  } else if (pl.BM == 128) {
    hipLaunchKernelGGL((conv_wgrad2_kernel<128, 128, 3, F16>), grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_wgrad2_kernel<64, 128, 3, F16>), grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_conv_wgrad(ConvWgradArgs a, const WgradPlan& pl, hipStream_t s) {
  if (a.P == 0 || a.N == 0) return hipSuccess;
  if (!wgrad_supported(a)) return hipErrorInvalidValue;
  a.pix_per_split = pl.pix_per_split;
  a.xcd_g = pl.xcd_g;
  a.Npad = pl.Npad;
  return a.f16 ? conv_wgrad_dispatch<true>(a, pl, s) : conv_wgrad_dispatch<false>(a, pl, s);
}

}  // namespace raft_amd
