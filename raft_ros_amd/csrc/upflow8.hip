// Bilinear 8x flow upsampling, reference upflow8 (core/utils/utils.py:80-82):
//   out[b, c, Y, X] = 8 * bilinear(flow[b, c], Y * (H-1)/(8H-1), X * (W-1)/(8W-1))   (align_corners=True)
// RAFT-small upsamples every iterate with it (core/raft.py:131-134).
//
// Forward: one thread per output pixel, both channels.  Backward (the adjoint) is a gather,
// not a scatter: one thread per low-resolution pixel walks the ~17x17 output pixels whose
// bilinear stencil touches it and sums weight * grad -- deterministic, no atomics.  It can
// write the flow gradient NCHW fp32 or as bf16 pixel rows [du, dv, 0, ...] (the fused
// RAFT-small step's delta-gradient layout, ops/update_fused.py).
#include "common.h"

namespace raft_amd {
namespace {

__device__ __forceinline__ void src_coord(int O, int n, float scale, int& i0, int& i1, float& w) {
  const float s = O * scale;
  i0 = min((int)s, n - 1);
  i1 = min(i0 + 1, n - 1);
  w = s - (float)i0;
}

__global__ __launch_bounds__(256) void upflow8_fwd_kernel(const float* __restrict__ flow, float* __restrict__ out,
                                                          int B, int H, int W, float sy, float sx) {
  const long H8 = 8L * H, W8 = 8L * W;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * H8 * W8) return;
  const int X = (int)(idx % W8);
  const int Y = (int)((idx / W8) % H8);
  const int b = (int)(idx / (H8 * W8));
  int y0, y1, x0, x1;
  float wy, wx;
  src_coord(Y, H, sy, y0, y1, wy);
  src_coord(X, W, sx, x0, x1, wx);
  const long HW = (long)H * W;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float* f = flow + ((long)b * 2 + c) * HW;
    const float v = (1.f - wy) * ((1.f - wx) * f[y0 * W + x0] + wx * f[y0 * W + x1]) +
                    wy * ((1.f - wx) * f[y1 * W + x0] + wx * f[y1 * W + x1]);
    out[((long)b * 2 + c) * H8 * W8 + (long)Y * W8 + X] = 8.f * v;
  }
}

// weight of low-res index i in the stencil of output index O
__device__ __forceinline__ float tap_weight(int O, int i, int n, float scale) {
  int i0, i1;
  float w;
  src_coord(O, n, scale, i0, i1, w);
  return (i0 == i ? 1.f - w : 0.f) + (i1 == i ? w : 0.f);
}

__global__ __launch_bounds__(256) void upflow8_bwd_kernel(const float* __restrict__ g, float* __restrict__ dflow,
                                                          __bf16* __restrict__ rows, int rows_ld, int B, int H,
                                                          int W, float sy, float sx) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H * W) return;
  const int x = (int)(idx % W), y = (int)((idx / W) % H), b = (int)(idx / ((long)H * W));
  const int H8 = 8 * H, W8 = 8 * W;
  // output rows / columns whose stencil can reach y / x (scale ~ 1/8: a +-9 window)
  const float iy = sy > 0.f ? 1.f / sy : 0.f, ix = sx > 0.f ? 1.f / sx : 0.f;
  const int Y0 = max(0, (int)floorf((y - 1) * iy) - 1), Y1 = min(H8 - 1, (int)ceilf((y + 1) * iy) + 1);
  const int X0 = max(0, (int)floorf((x - 1) * ix) - 1), X1 = min(W8 - 1, (int)ceilf((x + 1) * ix) + 1);
  float a0 = 0.f, a1 = 0.f;
  const long oHW = (long)H8 * W8;
  const float* g0 = g + (long)b * 2 * oHW;
  for (int Y = (H == 1 ? 0 : Y0); Y <= (H == 1 ? H8 - 1 : Y1); ++Y) {
    const float wy = tap_weight(Y, y, H, sy);
    if (wy == 0.f) continue;
    float r0 = 0.f, r1 = 0.f;
    for (int X = (W == 1 ? 0 : X0); X <= (W == 1 ? W8 - 1 : X1); ++X) {
      const float wx = tap_weight(X, x, W, sx);
      r0 += wx * g0[(long)Y * W8 + X];
      r1 += wx * g0[oHW + (long)Y * W8 + X];
    }
    a0 += wy * r0;
    a1 += wy * r1;
  }
  a0 *= 8.f;
  a1 *= 8.f;
  if (rows) {
    __bf16* r = rows + idx * rows_ld;
    r[0] = static_cast<__bf16>(a0);
    r[1] = static_cast<__bf16>(a1);
    for (int c = 2; c < rows_ld; ++c) r[c] = static_cast<__bf16>(0.f);
  }
  if (dflow) {
    const long HW = (long)H * W;
    dflow[(long)b * 2 * HW + (long)y * W + x] = a0;
    dflow[(long)b * 2 * HW + HW + (long)y * W + x] = a1;
  }
}

inline float ac_scale(int n) { return n > 1 ? (float)(n - 1) / (float)(8 * n - 1) : 0.f; }

}  // namespace

hipError_t launch_upflow8_fwd(const float* flow, float* out, int B, int H, int W, hipStream_t s) {
  const long tot = (long)B * 64 * H * W;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(upflow8_fwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, flow, out, B, H, W,
                     ac_scale(H), ac_scale(W));
  return hipGetLastError();
}

hipError_t launch_upflow8_bwd(const float* g, float* dflow, void* rows, int rows_ld, int B, int H, int W,
                              hipStream_t s) {
  const long tot = (long)B * H * W;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(upflow8_bwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, g, dflow,
                     static_cast<__bf16*>(rows), rows_ld, B, H, W, ac_scale(H), ac_scale(W));
  return hipGetLastError();
}

}  // namespace raft_amd
