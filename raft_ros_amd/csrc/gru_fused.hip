// Fused ConvGRU gate math (reference core/update.py:16-60):
//   gates_zr:  z = sigmoid(a), rh = sigmoid(b) * h          where [a | b] = conv_{z||r}([h, x])
//   blend:     h' = (1 - z) * h + z * tanh(q)                where q = conv_q([rh, x])
// plus both backwards.  Tensors are channels-last (NHWC): the fused z||r conv
// output has 2C channels per pixel, z in [0, C) and r in [C, 2C).
// One thread handles 8 consecutive channels of one pixel with 16-byte (bf16)
// or 2x16-byte (fp32) vector accesses; math is fp32.
#include "common.h"

namespace raft_amd {
namespace {

template <typename T>
struct V8 {
  float v[8];
  __device__ __forceinline__ void load(const T* p);
  __device__ __forceinline__ void store(T* p) const;
};
template <>
__device__ __forceinline__ void V8<__bf16>::load(const __bf16* p) {
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(x[i]);
}
template <>
__device__ __forceinline__ void V8<__bf16>::store(__bf16* p) const {
  bf16x8 x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = static_cast<__bf16>(v[i]);
  *reinterpret_cast<bf16x8*>(p) = x;
}
template <>
__device__ __forceinline__ void V8<float>::load(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = a[i];
    v[i + 4] = b[i];
  }
}
template <>
__device__ __forceinline__ void V8<float>::store(float* p) const {
  f32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = v[i];
    b[i] = v[i + 4];
  }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) {
  // tanh(x) = 1 - 2 / (exp(2x) + 1); saturates correctly for |x| large
  return 1.f - 2.f / (__expf(2.f * x) + 1.f);
}

template <typename T>
__global__ __launch_bounds__(256) void gates_zr_fwd(const T* __restrict__ zr, const T* __restrict__ h,
                                                    T* __restrict__ z, T* __restrict__ rh, long npix,
                                                    int C) {
  const int cg = C / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix * cg) return;
  const long p = i / cg;
  const int c = (i - p * cg) * 8;
  V8<T> a, b, hv, zo, ro;
  a.load(zr + p * 2 * C + c);
  b.load(zr + p * 2 * C + C + c);
  hv.load(h + p * C + c);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    zo.v[k] = sigm(a.v[k]);
    ro.v[k] = sigm(b.v[k]) * hv.v[k];
  }
  zo.store(z + p * C + c);
  ro.store(rh + p * C + c);
}

template <typename T>
__global__ __launch_bounds__(256) void gates_zr_bwd(const T* __restrict__ zr, const T* __restrict__ h,
                                                    const T* __restrict__ gz, const T* __restrict__ grh,
                                                    T* __restrict__ dzr, T* __restrict__ dh, long npix,
                                                    int C) {
  const int cg = C / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= npix * cg) return;
  const long p = i / cg;
  const int c = (i - p * cg) * 8;
  V8<T> a, b, hv, g1, g2, da, db, dhv;
  a.load(zr + p * 2 * C + c);
  b.load(zr + p * 2 * C + C + c);
  hv.load(h + p * C + c);
  g1.load(gz + p * C + c);
  g2.load(grh + p * C + c);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float zs = sigm(a.v[k]), rs = sigm(b.v[k]);
    da.v[k] = g1.v[k] * zs * (1.f - zs);
    db.v[k] = g2.v[k] * hv.v[k] * rs * (1.f - rs);
    dhv.v[k] = g2.v[k] * rs;
  }
  da.store(dzr + p * 2 * C + c);
  db.store(dzr + p * 2 * C + C + c);
  dhv.store(dh + p * C + c);
}

template <typename T>
__global__ __launch_bounds__(256) void blend_fwd(const T* __restrict__ z, const T* __restrict__ q,
                                                 const T* __restrict__ h, T* __restrict__ out, long n8) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  V8<T> zv, qv, hv, o;
  zv.load(z + i * 8);
  qv.load(q + i * 8);
  hv.load(h + i * 8);
#pragma unroll
  for (int k = 0; k < 8; ++k) o.v[k] = (1.f - zv.v[k]) * hv.v[k] + zv.v[k] * tanh_fast(qv.v[k]);
  o.store(out + i * 8);
}

template <typename T>
__global__ __launch_bounds__(256) void blend_bwd(const T* __restrict__ z, const T* __restrict__ q,
                                                 const T* __restrict__ h, const T* __restrict__ g,
                                                 T* __restrict__ dz, T* __restrict__ dq,
                                                 T* __restrict__ dh, long n8) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  V8<T> zv, qv, hv, gv, a, b, c;
  zv.load(z + i * 8);
  qv.load(q + i * 8);
  hv.load(h + i * 8);
  gv.load(g + i * 8);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float t = tanh_fast(qv.v[k]);
    a.v[k] = gv.v[k] * (t - hv.v[k]);
    b.v[k] = gv.v[k] * zv.v[k] * (1.f - t * t);
    c.v[k] = gv.v[k] * (1.f - zv.v[k]);
  }
  a.store(dz + i * 8);
  b.store(dq + i * 8);
  c.store(dh + i * 8);
}

inline dim3 g1d(long n) { return dim3((n + 255) / 256); }

}  // namespace

hipError_t launch_gru_gates_fwd(int dtype, const void* zr, const void* h, void* z, void* rh, long npix,
                                int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const long n = npix * (C / 8);
  if (!n) return hipSuccess;
  if (dtype == kBF16)
    hipLaunchKernelGGL(gates_zr_fwd<__bf16>, g1d(n), dim3(256), 0, s, (const __bf16*)zr, (const __bf16*)h,
                       (__bf16*)z, (__bf16*)rh, npix, C);
  else
    hipLaunchKernelGGL(gates_zr_fwd<float>, g1d(n), dim3(256), 0, s, (const float*)zr, (const float*)h,
                       (float*)z, (float*)rh, npix, C);
  return hipGetLastError();
}

hipError_t launch_gru_gates_bwd(int dtype, const void* zr, const void* h, const void* gz, const void* grh,
                                void* dzr, void* dh, long npix, int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const long n = npix * (C / 8);
  if (!n) return hipSuccess;
  if (dtype == kBF16)
    hipLaunchKernelGGL(gates_zr_bwd<__bf16>, g1d(n), dim3(256), 0, s, (const __bf16*)zr, (const __bf16*)h,
                       (const __bf16*)gz, (const __bf16*)grh, (__bf16*)dzr, (__bf16*)dh, npix, C);
  else
    hipLaunchKernelGGL(gates_zr_bwd<float>, g1d(n), dim3(256), 0, s, (const float*)zr, (const float*)h,
                       (const float*)gz, (const float*)grh, (float*)dzr, (float*)dh, npix, C);
  return hipGetLastError();
}

hipError_t launch_gru_blend_fwd(int dtype, const void* z, const void* q, const void* h, void* out,
                                long numel, hipStream_t s) {
  if (numel % 8) return hipErrorInvalidValue;
  const long n = numel / 8;
  if (!n) return hipSuccess;
  if (dtype == kBF16)
    hipLaunchKernelGGL(blend_fwd<__bf16>, g1d(n), dim3(256), 0, s, (const __bf16*)z, (const __bf16*)q,
                       (const __bf16*)h, (__bf16*)out, n);
  else
    hipLaunchKernelGGL(blend_fwd<float>, g1d(n), dim3(256), 0, s, (const float*)z, (const float*)q,
                       (const float*)h, (float*)out, n);
  return hipGetLastError();
}

hipError_t launch_gru_blend_bwd(int dtype, const void* z, const void* q, const void* h, const void* g,
                                void* dz, void* dq, void* dh, long numel, hipStream_t s) {
  if (numel % 8) return hipErrorInvalidValue;
  const long n = numel / 8;
  if (!n) return hipSuccess;
  if (dtype == kBF16)
    hipLaunchKernelGGL(blend_bwd<__bf16>, g1d(n), dim3(256), 0, s, (const __bf16*)z, (const __bf16*)q,
                       (const __bf16*)h, (const __bf16*)g, (__bf16*)dz, (__bf16*)dq, (__bf16*)dh, n);
  else
    hipLaunchKernelGGL(blend_bwd<float>, g1d(n), dim3(256), 0, s, (const float*)z, (const float*)q,
                       (const float*)h, (const float*)g, (float*)dz, (float*)dq, (float*)dh, n);
  return hipGetLastError();
}

}  // namespace raft_amd
