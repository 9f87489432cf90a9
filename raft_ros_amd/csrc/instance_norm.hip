// Channels-last (NHWC) InstanceNorm (affine=False) with optional fused ReLU, fwd + bwd.
//
// The feature encoder (reference core/extractor.py:118-192, norm_fn='instance')
// normalises every conv output per (image, channel) over H x W.  PyTorch lowers
// instance_norm to batch_norm on a (1, N*C, H, W) *contiguous* view, so a
// channels-last activation is copied to NCHW and back around every norm (forward
// and backward) -- ~70 full-resolution copies per training step.  These kernels
// work on the NHWC layout directly:
//   stats:  per (n, c) sum / sum of squares, 16-byte loads of 8 channels per
//           thread, fixed-order LDS reduction to one partial per 1024-pixel chunk,
//           then a fixed-order sum of the partials (deterministic, no atomics);
//   apply:  y = relu?((x - mean) * rstd), vectorised;
//   bwd:    dxhat = dy * [xhat > 0 if relu]; per (n, c) sums of dxhat and
//           dxhat*xhat; dx = rstd * (dxhat - mean(dxhat) - xhat * mean(dxhat*xhat)).
// ReLU'(y) is recomputed from xhat (relu(xhat) > 0 <=> xhat > 0), so only the
// input and the (mean, rstd) statistics are saved for backward.
#include "common.h"

namespace raft_amd {
namespace {

template <typename T>
struct Vec8IO;
template <>
struct Vec8IO<__bf16> {
  static __device__ __forceinline__ void load(const __bf16* p, float* v) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(x[i]);
  }
  static __device__ __forceinline__ void store(__bf16* p, const float* v) {
    bf16x8 x;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = static_cast<__bf16>(v[i]);
    *reinterpret_cast<bf16x8*>(p) = x;
  }
};
template <>
struct Vec8IO<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[i + 4] = b[i];
    }
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = v[i];
      b[i] = v[i + 4];
    }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};

constexpr int PIX_PER_BLOCK = 1024;

// Per-(image, channel) partial sums over one PIX_PER_BLOCK pixel chunk.
// mode 0: sums of x and x^2.  mode 1: sums of dxhat and dxhat*xhat (needs stats + dy).
// Every block writes its own partial (no atomics, no memset): the reduction order is
// fixed, so the statistics are bit-reproducible run to run and graph replays need no
// zero-initialised accumulator.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void in_partial_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const float* __restrict__ mr, float* __restrict__ part,
                                                         int N, int HW, int C, int relu) {
  __shared__ float r1[2048], r2[2048];  // [R][C], R * C <= 256 * 8
  const int n = blockIdx.y;
  const int G = C / 8;
  const int R = 256 / G;
  const int tid = threadIdx.x;
  const int cg = tid % G, pr = tid / G;
  float a1[8], a2[8], mean[8], rstd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a1[j] = a2[j] = 0.f;
    mean[j] = rstd[j] = 0.f;
    if (MODE == 1 && pr < R) {
      mean[j] = mr[((long)n * C + cg * 8 + j) * 2];
      rstd[j] = mr[((long)n * C + cg * 8 + j) * 2 + 1];
    }
  }
  if (pr < R) {
    const int p0 = blockIdx.x * PIX_PER_BLOCK;
    const int p1 = min(p0 + PIX_PER_BLOCK, HW);
    for (int p = p0 + pr; p < p1; p += R) {
      const long off = ((long)n * HW + p) * C + cg * 8;
      float v[8];
      Vec8IO<T>::load(x + off, v);
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a1[j] += v[j];
          a2[j] += v[j] * v[j];
        }
      } else {
        float g[8];
        Vec8IO<T>::load(dy + off, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (v[j] - mean[j]) * rstd[j];
          const float d = (relu && !(xh > 0.f)) ? 0.f : g[j];
          a1[j] += d;
          a2[j] += d * xh;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r1[pr * C + cg * 8 + j] = a1[j];
      r2[pr * C + cg * 8 + j] = a2[j];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float s1 = 0.f, s2 = 0.f;
    for (int r = 0; r < R; ++r) {
      s1 += r1[r * C + c];
      s2 += r2[r * C + c];
    }
    const long o = (((long)blockIdx.x * N + n) * C + c) * 2;
    part[o] = s1;
    part[o + 1] = s2;
  }
}

// Sum the per-chunk partials in a fixed order.  mode 0 -> (mean, rstd); mode 1 -> raw sums.
__global__ void in_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, int chunks, long NC,
                                 int HW, float eps, int mode) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= NC) return;
  float s1 = 0.f, s2 = 0.f;
  for (int k = 0; k < chunks; ++k) {
    s1 += part[(k * NC + i) * 2];
    s2 += part[(k * NC + i) * 2 + 1];
  }
  if (mode == 0) {
    const float m = s1 / HW;
    const float var = fmaxf(s2 / HW - m * m, 0.f);
    out[2 * i] = m;
    out[2 * i + 1] = rsqrtf(var + eps);
  } else {
    out[2 * i] = s1;
    out[2 * i + 1] = s2;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void in_apply_kernel(const T* __restrict__ x, const float* __restrict__ mr,
                                                       T* __restrict__ y, long total8, int HW, int C, int relu) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total8) return;
  const int G = C / 8;
  const int cg = i % G;
  const long pix = i / G;
  const int n = pix / HW;
  float v[8];
  Vec8IO<T>::load(x + i * 8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long s = ((long)n * C + cg * 8 + j) * 2;
    float o = (v[j] - mr[s]) * mr[s + 1];
    if (relu) o = fmaxf(o, 0.f);
    v[j] = o;
  }
  Vec8IO<T>::store(y + i * 8, v);
}

template <typename T>
__global__ __launch_bounds__(256) void in_bwd_apply_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                           const float* __restrict__ mr,
                                                           const float* __restrict__ gs, T* __restrict__ dx,
                                                           long total8, int HW, int C, int relu) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total8) return;
  const int G = C / 8;
  const int cg = i % G;
  const long pix = i / G;
  const int n = pix / HW;
  float v[8], g[8];
  Vec8IO<T>::load(x + i * 8, v);
  Vec8IO<T>::load(dy + i * 8, g);
  const float inv = 1.f / HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long s = ((long)n * C + cg * 8 + j) * 2;
    const float rstd = mr[s + 1];
    const float xh = (v[j] - mr[s]) * rstd;
    const float d = (relu && !(xh > 0.f)) ? 0.f : g[j];
    v[j] = rstd * (d - gs[s] * inv - xh * gs[s + 1] * inv);
  }
  Vec8IO<T>::store(dx + i * 8, v);
}

}  // namespace

int instance_norm_chunks(int HW) { return (HW + PIX_PER_BLOCK - 1) / PIX_PER_BLOCK; }

hipError_t launch_instance_norm_fwd(int dtype, const void* x, void* y, float* stats, float* part, int N, int HW,
                                    int C, int relu, float eps, hipStream_t s) {
  if (C % 8 || C > 512) return hipErrorInvalidValue;
  const int chunks = instance_norm_chunks(HW);
  const dim3 g(chunks, N);
  const long total8 = (long)N * HW * C / 8;
  const dim3 ga((total8 + 255) / 256);
  if (dtype == kBF16) {
    hipLaunchKernelGGL((in_partial_kernel<__bf16, 0>), g, dim3(256), 0, s, (const __bf16*)x, nullptr, nullptr,
                       part, N, HW, C, relu);
  } else {
    hipLaunchKernelGGL((in_partial_kernel<float, 0>), g, dim3(256), 0, s, (const float*)x, nullptr, nullptr,
                       part, N, HW, C, relu);
  }
  RAFT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(in_reduce_kernel, dim3((N * C + 255) / 256), dim3(256), 0, s, part, stats, chunks,
                     (long)N * C, HW, eps, 0);
  RAFT_HIP_CHECK(hipGetLastError());
  if (dtype == kBF16)
    hipLaunchKernelGGL(in_apply_kernel<__bf16>, ga, dim3(256), 0, s, (const __bf16*)x, stats, (__bf16*)y,
                       total8, HW, C, relu);
  else
    hipLaunchKernelGGL(in_apply_kernel<float>, ga, dim3(256), 0, s, (const float*)x, stats, (float*)y, total8,
                       HW, C, relu);
  return hipGetLastError();
}

hipError_t launch_instance_norm_bwd(int dtype, const void* x, const void* dy, const float* stats, float* gsum,
                                    float* part, void* dx, int N, int HW, int C, int relu, hipStream_t s) {
  if (C % 8 || C > 512) return hipErrorInvalidValue;
  const int chunks = instance_norm_chunks(HW);
  const dim3 g(chunks, N);
  const long total8 = (long)N * HW * C / 8;
  const dim3 ga((total8 + 255) / 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL((in_partial_kernel<__bf16, 1>), g, dim3(256), 0, s, (const __bf16*)x, (const __bf16*)dy,
                       stats, part, N, HW, C, relu);
  else
    hipLaunchKernelGGL((in_partial_kernel<float, 1>), g, dim3(256), 0, s, (const float*)x, (const float*)dy,
                       stats, part, N, HW, C, relu);
  RAFT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(in_reduce_kernel, dim3((N * C + 255) / 256), dim3(256), 0, s, part, gsum, chunks,
                     (long)N * C, HW, 0.f, 1);
  RAFT_HIP_CHECK(hipGetLastError());
  if (dtype == kBF16)
    hipLaunchKernelGGL(in_bwd_apply_kernel<__bf16>, ga, dim3(256), 0, s, (const __bf16*)x, (const __bf16*)dy,
                       stats, gsum, (__bf16*)dx, total8, HW, C, relu);
  else
    hipLaunchKernelGGL(in_bwd_apply_kernel<float>, ga, dim3(256), 0, s, (const float*)x, (const float*)dy, stats,
                       gsum, (float*)dx, total8, HW, C, relu);
  return hipGetLastError();
}

}  // namespace raft_amd
