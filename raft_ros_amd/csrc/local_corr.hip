// On-the-fly local correlation (the memory-efficient "alternate" path).
//
// Reference: alt_cuda_corr/correlation_kernel.cu:18-119 (forward) and :122-256
// (backward), driven by AlternateCorrBlock (core/corr.py:63-91).  The reference
// kernel uses 32-thread blocks (half a wave64), recomputes the dot product of
// every window cell per 32-channel chunk and has no autograd wiring.
//
// This implementation is organised around one wave64 per query pixel:
//   1. the (2r+2)^2 integer neighbours of floor(coords) are the only fmap2 rows
//      touched; each lane owns neighbours {lane, lane+64} and computes the full
//      C-channel dot product with vector (16 B) loads of both rows;
//   2. the dots are parked in LDS and the (2r+1)^2 bilinear taps (one shared
//      set of weights, since taps are integer offsets of one centroid) are
//      blended from them;
//   3. the backward forms the per-neighbour gradient with the same gather rule
//      as the dense lookup, then computes dF1 with lanes across channels
//      (no atomics) and scatters dF2 with fp32 atomics (neighbourhoods of
//      different query pixels overlap, and their positions are data dependent).
// Output layout (B, H1, W1, (2r+1)^2) with x-offset-major taps, matching CorrBlock.
#include "common.h"

namespace raft_amd {
namespace {

constexpr int kMaxNb = 128;  // (2r+2)^2 <= 128  ->  r <= 4

template <typename T>
struct Vec8;
template <>
struct Vec8<__bf16> {
  static __device__ __forceinline__ void load(const __bf16* p, float* v) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(x[i]);
  }
};
template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p);
    const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[i + 4] = b[i];
    }
  }
};

template <typename T>
__device__ __forceinline__ float dot_rows(const T* a, const T* b, int C) {
  float s = 0.f;
  for (int c = 0; c < C; c += 8) {
    float va[8], vb[8];
    Vec8<T>::load(a + c, va);
    Vec8<T>::load(b + c, vb);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += va[i] * vb[i];
  }
  return s;
}

__device__ __forceinline__ float clampf(float v) { return fminf(fmaxf(v, -1.0e6f), 1.0e6f); }

template <typename T>
__global__ __launch_bounds__(256) void local_corr_fwd_kernel(const T* __restrict__ f1,
                                                             const T* __restrict__ f2,
                                                             const float* __restrict__ coords,
                                                             float* __restrict__ out, int B, int H1,
                                                             int W1, int H2, int W2, int C, int r,
                                                             float scale) {
  __shared__ float dots[4][kMaxNb];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long pix = (long)blockIdx.x * 4 + w;
  const long HW1 = (long)H1 * W1;
  const bool active = pix < (long)B * HW1;
  const int rd = 2 * r + 1, nb = rd + 1;
  float fx = 0.f, fy = 0.f;
  if (active) {
    const int b = pix / HW1;
    const long p = pix - b * HW1;
    const float cx = coords[(long)b * 2 * HW1 + p], cy = coords[(long)b * 2 * HW1 + HW1 + p];
    const bool ok = isfinite(cx) && isfinite(cy);
    const float x0f = floorf(clampf(cx)), y0f = floorf(clampf(cy));
    fx = cx - x0f;
    fy = cy - y0f;
    const T* a = f1 + pix * C;
    for (int n = lane; n < nb * nb; n += 64) {
      const int yy = (int)y0f - r + n / nb, xx = (int)x0f - r + n % nb;
      float d = 0.f;
      if (ok && yy >= 0 && yy < H2 && xx >= 0 && xx < W2)
        d = dot_rows(a, f2 + (((long)b * H2 + yy) * W2 + xx) * C, C);
      dots[w][n] = d;
    }
  }
  __syncthreads();
  if (!active) return;
  for (int t = lane; t < rd * rd; t += 64) {
    const int ix = t / rd, iy = t - ix * rd;
    const float* d = dots[w];
    const float v = (1.f - fx) * (1.f - fy) * d[iy * nb + ix] + fx * (1.f - fy) * d[iy * nb + ix + 1] +
                    (1.f - fx) * fy * d[(iy + 1) * nb + ix] + fx * fy * d[(iy + 1) * nb + ix + 1];
    out[pix * rd * rd + t] = v * scale;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void local_corr_bwd_kernel(
    const T* __restrict__ f1, const T* __restrict__ f2, const float* __restrict__ coords,
    const float* __restrict__ gout, float* __restrict__ g1, float* __restrict__ g2, long long* __restrict__ g2fix,
    const float* __restrict__ fix_scale, int B, int H1, int W1, int H2, int W2, int C, int r, float scale) {
  __shared__ float gn[4][kMaxNb];
  __shared__ int pos[4][kMaxNb];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long pix = (long)blockIdx.x * 4 + w;
  const long HW1 = (long)H1 * W1;
  const bool active = pix < (long)B * HW1;
  const int rd = 2 * r + 1, nb = rd + 1;
  int b = 0;
  if (active) {
    b = pix / HW1;
    const long p = pix - b * HW1;
    const float cx = coords[(long)b * 2 * HW1 + p], cy = coords[(long)b * 2 * HW1 + HW1 + p];
    const bool ok = isfinite(cx) && isfinite(cy);
    const float x0f = floorf(clampf(cx)), y0f = floorf(clampf(cy));
    const float fx = cx - x0f, fy = cy - y0f;
    const float* g = gout + pix * rd * rd;
    for (int n = lane; n < nb * nb; n += 64) {
      const int a = n / nb, c = n - a * nb;
      const int yy = (int)y0f - r + a, xx = (int)x0f - r + c;
      float v = 0.f;
      int q = -1;
      if (ok && yy >= 0 && yy < H2 && xx >= 0 && xx < W2) {
        q = yy * W2 + xx;
        if (a < rd) {
          if (c < rd) v += (1.f - fx) * (1.f - fy) * g[c * rd + a];
          if (c > 0) v += fx * (1.f - fy) * g[(c - 1) * rd + a];
        }
        if (a > 0) {
          if (c < rd) v += (1.f - fx) * fy * g[c * rd + a - 1];
          if (c > 0) v += fx * fy * g[(c - 1) * rd + a - 1];
        }
      }
      gn[w][n] = v * scale;
      pos[w][n] = q;
    }
  }
  __syncthreads();
  if (!active) return;
  const T* a = f1 + pix * C;
  const T* f2b = f2 + (long)b * H2 * W2 * C;
  float* g2b = g2 + (long)b * H2 * W2 * C;
  const float fs = g2fix != nullptr ? *fix_scale : 0.f;
  for (int c0 = lane; c0 < C; c0 += 64) {
    const float av = to_f32(a[c0]);
    float acc = 0.f;
    for (int n = 0; n < nb * nb; ++n) {
      const int q = pos[w][n];
      if (q < 0) continue;
      const float gv = gn[w][n];
      acc += gv * to_f32(f2b[(long)q * C + c0]);
      if (g2fix != nullptr)
        fixed_atomic_add(g2fix + (g2b - g2) + (long)q * C + c0, gv * av, fs);
      else
        atomicAdd(g2b + (long)q * C + c0, gv * av);
    }
    g1[pix * C + c0] = acc;
  }
}

}  // namespace

hipError_t launch_local_corr_fwd(const void* f1, const void* f2, int dtype, const float* coords,
                                 float* out, int B, int H1, int W1, int H2, int W2, int C, int r,
                                 float scale, hipStream_t s) {
  if ((2 * r + 2) * (2 * r + 2) > kMaxNb) return hipErrorInvalidValue;
  const long npix = (long)B * H1 * W1;
  if (npix == 0) return hipSuccess;
  const dim3 g((npix + 3) / 4), blk(256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(local_corr_fwd_kernel<__bf16>, g, blk, 0, s, static_cast<const __bf16*>(f1),
                       static_cast<const __bf16*>(f2), coords, out, B, H1, W1, H2, W2, C, r, scale);
  else if (dtype == kF32)
    hipLaunchKernelGGL(local_corr_fwd_kernel<float>, g, blk, 0, s, static_cast<const float*>(f1),
                       static_cast<const float*>(f2), coords, out, B, H1, W1, H2, W2, C, r, scale);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_local_corr_bwd(const void* f1, const void* f2, int dtype, const float* coords,
                                 const float* gout, float* g1, float* g2, long long* g2fix, const float* fix_scale,
                                 int B, int H1, int W1, int H2, int W2, int C, int r, float scale, hipStream_t s) {
  if ((2 * r + 2) * (2 * r + 2) > kMaxNb) return hipErrorInvalidValue;
  const long npix = (long)B * H1 * W1;
  if (npix == 0) return hipSuccess;
  const dim3 g((npix + 3) / 4), blk(256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(local_corr_bwd_kernel<__bf16>, g, blk, 0, s, static_cast<const __bf16*>(f1),
                       static_cast<const __bf16*>(f2), coords, gout, g1, g2, g2fix, fix_scale, B, H1, W1, H2, W2, C, r,
                       scale);
  else if (dtype == kF32)
    hipLaunchKernelGGL(local_corr_bwd_kernel<float>, g, blk, 0, s, static_cast<const float*>(f1),
                       static_cast<const float*>(f2), coords, gout, g1, g2, g2fix, fix_scale, B, H1, W1, H2, W2, C, r,
                       scale);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace raft_amd
