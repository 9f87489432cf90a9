// All-pairs correlation pyramid: pooling, radius-r lookup (fwd/bwd) and the
// pyramid-gradient combine, for gfx950.
//
// Semantics follow the reference CorrBlock (core/corr.py:12-50):
//   * level l+1 = 2x2 / stride-2 average pool (floor) of level l over the image-2 dims;
//   * lookup at coords / 2^l, window [-r, r]^2, bilinear with align_corners=True and
//     zero padding (grid_sample semantics, core/utils/utils.py:57-71);
//   * output channel order is level-major, then x-offset-major, then y-offset
//     (ch = l*(2r+1)^2 + ix*(2r+1) + iy) -- the order CorrBlock produces because its
//     meshgrid(dy, dx) delta is added to (x, y) centroids (core/corr.py:37-43).
//
// The MI355X-first differences:
//   * every window tap shares one set of bilinear weights (the taps are integer
//     offsets of a single centroid), so the (2r+2)^2 integer neighbours are read
//     once per level and the 4-corner blend is done in registers;
//   * the backward is a *gather*: query pixel p only ever touches row p of the
//     volume, so each (pixel, level, neighbour) thread owns its output element.
//     No atomics, deterministic, and gradients of all refinement iterations are
//     accumulated in place into ONE pyramid-gradient buffer (instead of autograd
//     materialising and summing a dense gradient per iteration as
//     grid_sample's backward does);
//   * the 4-level gradient is folded back to level 0 (pool backward) and cast to
//     bf16 in one tiled pass that also writes the transposed copy needed by the
//     fmap2 gradient GEMM.
#include "common.h"

namespace raft_amd {

struct PyrDesc {
  float* ptr[4];
  int H[4];
  int W[4];
  int levels;
};

namespace {

__global__ __launch_bounds__(256) void avgpool2x2_kernel(const float* __restrict__ in,
                                                         float* __restrict__ out, long rows, int H,
                                                         int W, int Ho, int Wo) {
  const long total = rows * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int x = i % Wo;
    const long t = i / Wo;
    const int y = t % Ho;
    const long r = t / Ho;
    const float* src = in + r * H * W + (2 * y) * W + 2 * x;
    out[i] = 0.25f * (src[0] + src[1] + src[W] + src[W + 1]);
  }
}

__device__ __forceinline__ float safe_floor(float v) {
  // keep far-out-of-range / non-finite coordinates from overflowing int math
  v = fminf(fmaxf(v, -1.0e6f), 1.0e6f);
  return floorf(v);
}

template <typename OutT>
__global__ __launch_bounds__(256) void corr_lookup_fwd_kernel(PyrDesc pyr,
                                                              const float* __restrict__ coords,
                                                              OutT* __restrict__ out, int B, int H,
                                                              int W, int r, int out_ch) {
  const int rd = 2 * r + 1;
  const int win = rd * rd;
  const int Ch = pyr.levels * win;
  const int HW = H * W;
  const long total = (long)B * HW * out_ch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ch = i % out_ch;
    const long pix = i / out_ch;
    if (ch >= Ch) {  // zero padding channels (K padding of the consuming conv)
      out[i] = from_f32<OutT>(0.f);
      continue;
    }
    const int b = pix / HW;
    const int p = pix - (long)b * HW;
    const int l = ch / win;
    const int rem = ch - l * win;
    const int ix = rem / rd;
    const int iy = rem - ix * rd;
    const float scale = 1.0f / float(1 << l);
    const float cx = coords[(long)b * 2 * HW + p] * scale;
    const float cy = coords[(long)b * 2 * HW + HW + p] * scale;
    float val = 0.f;
    if (isfinite(cx) && isfinite(cy)) {
      const float fx0 = safe_floor(cx), fy0 = safe_floor(cy);
      const float fx = cx - fx0, fy = cy - fy0;
      const int x0 = (int)fx0 - r + ix, y0 = (int)fy0 - r + iy;
      const int Hl = pyr.H[l], Wl = pyr.W[l];
      const float* row = pyr.ptr[l] + pix * (long)Hl * Wl;
      const bool x0ok = x0 >= 0 && x0 < Wl, x1ok = x0 + 1 >= 0 && x0 + 1 < Wl;
      const bool y0ok = y0 >= 0 && y0 < Hl, y1ok = y0 + 1 >= 0 && y0 + 1 < Hl;
      if (y0ok) {
        if (x0ok) val += (1.f - fx) * (1.f - fy) * row[y0 * Wl + x0];
        if (x1ok) val += fx * (1.f - fy) * row[y0 * Wl + x0 + 1];
      }
      if (y1ok) {
        if (x0ok) val += (1.f - fx) * fy * row[(y0 + 1) * Wl + x0];
        if (x1ok) val += fx * fy * row[(y0 + 1) * Wl + x0 + 1];
      }
    }
    out[i] = from_f32<OutT>(val);
  }
}

// One thread per (pixel, level, neighbour a, neighbour b) of the (2r+2)^2 integer
// neighbourhood; accumulates (+=) into the pyramid-gradient buffer it owns.
template <typename GT>
__global__ __launch_bounds__(256) void corr_lookup_bwd_kernel(PyrDesc dpyr,
                                                              const float* __restrict__ coords,
                                                              const GT* __restrict__ gout, int B,
                                                              int H, int W, int r, int gstride) {
  const int rd = 2 * r + 1;
  const int nb = rd + 1;
  const int win = rd * rd;
  const int Ch = dpyr.levels * win;
  const int per_pix = dpyr.levels * nb * nb;
  const int HW = H * W;
  const long total = (long)B * HW * per_pix;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int e = i % per_pix;
    const long pix = i / per_pix;
    const int b = pix / HW;
    const int p = pix - (long)b * HW;
    const int l = e / (nb * nb);
    const int ab = e - l * nb * nb;
    const int a = ab / nb;  // y neighbour index
    const int c = ab - a * nb;  // x neighbour index
    const float scale = 1.0f / float(1 << l);
    const float cx = coords[(long)b * 2 * HW + p] * scale;
    const float cy = coords[(long)b * 2 * HW + HW + p] * scale;
    if (!(isfinite(cx) && isfinite(cy))) continue;
    const float fx0 = safe_floor(cx), fy0 = safe_floor(cy);
    const float fx = cx - fx0, fy = cy - fy0;
    const int yy = (int)fy0 - r + a, xx = (int)fx0 - r + c;
    const int Hl = dpyr.H[l], Wl = dpyr.W[l];
    if (yy < 0 || yy >= Hl || xx < 0 || xx >= Wl) continue;
    const GT* g = gout + pix * gstride + l * win;
    float v = 0.f;
    // tap (ix, iy) touches (iy + {0,1}, ix + {0,1}); this element is corner
    //   (0,0) of tap (c, a), (0,1) of tap (c-1, a), (1,0) of (c, a-1), (1,1) of (c-1, a-1)
    if (a < rd) {
      if (c < rd) v += (1.f - fx) * (1.f - fy) * to_f32(g[c * rd + a]);
      if (c > 0) v += fx * (1.f - fy) * to_f32(g[(c - 1) * rd + a]);
    }
    if (a > 0) {
      if (c < rd) v += (1.f - fx) * fy * to_f32(g[c * rd + a - 1]);
      if (c > 0) v += fx * fy * to_f32(g[(c - 1) * rd + a - 1]);
    }
    dpyr.ptr[l][pix * (long)Hl * Wl + yy * Wl + xx] += v;
  }
}

// Fold the 4-level pyramid gradient into level 0 (adjoint of the floor 2x2 pools),
// scale, cast to bf16 and emit both dC[b][p][q] and dCt[b][q][p] (row stride ldp,
// zero padding in [HW, ldp)).
constexpr int CT = 64;
__global__ __launch_bounds__(256) void pyramid_grad_combine_kernel(PyrDesc dpyr, __bf16* __restrict__ dC,
                                                                   __bf16* __restrict__ dCt, int B,
                                                                   int H, int W, int ldp,
                                                                   float alpha) {
  __shared__ float tile[CT][CT + 1];
  const int HW = H * W;
  const int tiles = (ldp + CT - 1) / CT;
  const int per_b = tiles * tiles;
  const int b = blockIdx.x / per_b;
  const int t = blockIdx.x - b * per_b;
  const int p0 = (t / tiles) * CT, q0 = (t % tiles) * CT;
  const int tid = threadIdx.x;
#pragma unroll 4
  for (int i = 0; i < CT * CT / 256; ++i) {
    const int e = tid + i * 256;
    const int rr = e / CT, cc = e % CT;
    const int p = p0 + rr, q = q0 + cc;
    float v = 0.f;
    if (p < HW && q < HW) {
      const long pix = (long)b * HW + p;
      const int y = q / W, x = q - (q / W) * W;
      v = dpyr.ptr[0][pix * HW + q];
      float s = 0.25f;
      for (int l = 1; l < dpyr.levels; ++l, s *= 0.25f) {
        const int yl = y >> l, xl = x >> l;
        if (yl < dpyr.H[l] && xl < dpyr.W[l])
          v += s * dpyr.ptr[l][pix * (long)dpyr.H[l] * dpyr.W[l] + yl * dpyr.W[l] + xl];
      }
      v *= alpha;
    }
    tile[rr][cc] = v;
    if (p < HW && q < ldp) dC[((long)b * HW + p) * ldp + q] = static_cast<__bf16>(v);
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < CT * CT / 256; ++i) {
    const int e = tid + i * 256;
    const int rr = e / CT, cc = e % CT;  // rr: q offset, cc: p offset
    const int q = q0 + rr, p = p0 + cc;
    if (q < HW && p < ldp) dCt[((long)b * HW + q) * ldp + p] = static_cast<__bf16>(tile[cc][rr]);
  }
}

inline int grid_for(long total) {
  long blocks = (total + 255) / 256;
  return (int)(blocks < (1L << 20) ? blocks : (1L << 20));
}

}  // namespace

hipError_t launch_avgpool2x2(const float* in, float* out, long rows, int H, int W, hipStream_t s) {
  const int Ho = H / 2, Wo = W / 2;
  const long total = rows * Ho * Wo;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(avgpool2x2_kernel, dim3(grid_for(total)), dim3(256), 0, s, in, out, rows, H, W,
                     Ho, Wo);
  return hipGetLastError();
}

hipError_t launch_corr_lookup_fwd(const PyrDesc& pyr, const float* coords, void* out, int out_dtype,
                                  int B, int H, int W, int r, int out_ch, hipStream_t s) {
  const long total = (long)B * H * W * out_ch;
  if (total == 0) return hipSuccess;
  const dim3 g(grid_for(total)), blk(256);
  if (out_dtype == kBF16)
    hipLaunchKernelGGL(corr_lookup_fwd_kernel<__bf16>, g, blk, 0, s, pyr, coords,
                       static_cast<__bf16*>(out), B, H, W, r, out_ch);
  else if (out_dtype == kF16)
    hipLaunchKernelGGL(corr_lookup_fwd_kernel<_Float16>, g, blk, 0, s, pyr, coords,
                       static_cast<_Float16*>(out), B, H, W, r, out_ch);
  else
    hipLaunchKernelGGL(corr_lookup_fwd_kernel<float>, g, blk, 0, s, pyr, coords,
                       static_cast<float*>(out), B, H, W, r, out_ch);
  return hipGetLastError();
}

hipError_t launch_corr_lookup_bwd(const PyrDesc& dpyr, const float* coords, const void* gout,
                                  int g_dtype, int B, int H, int W, int r, int gstride, hipStream_t s) {
  const long total = (long)B * H * W * dpyr.levels * (2 * r + 2) * (2 * r + 2);
  if (total == 0) return hipSuccess;
  const dim3 g(grid_for(total)), blk(256);
  if (g_dtype == kBF16)
    hipLaunchKernelGGL(corr_lookup_bwd_kernel<__bf16>, g, blk, 0, s, dpyr, coords,
                       static_cast<const __bf16*>(gout), B, H, W, r, gstride);
  else if (g_dtype == kF16)
    hipLaunchKernelGGL(corr_lookup_bwd_kernel<_Float16>, g, blk, 0, s, dpyr, coords,
                       static_cast<const _Float16*>(gout), B, H, W, r, gstride);
  else
    hipLaunchKernelGGL(corr_lookup_bwd_kernel<float>, g, blk, 0, s, dpyr, coords,
                       static_cast<const float*>(gout), B, H, W, r, gstride);
  return hipGetLastError();
}

hipError_t launch_pyramid_grad_combine(const PyrDesc& dpyr, void* dC, void* dCt, int B, int H,
                                       int W, int ldp, float alpha, hipStream_t s) {
  const int tiles = (ldp + CT - 1) / CT;
  hipLaunchKernelGGL(pyramid_grad_combine_kernel, dim3(B * tiles * tiles), dim3(256), 0, s, dpyr,
                     static_cast<__bf16*>(dC), static_cast<__bf16*>(dCt), B, H, W, ldp, alpha);
  return hipGetLastError();
}

}  // namespace raft_amd
