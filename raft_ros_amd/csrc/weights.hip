// Weight-side glue of the fused update block, as two HIP kernels instead of
// ~10 PyTorch ops per conv per step (ops/update_fused.py):
//
//   pack_conv_weights: fp32 module parameters -> the bf16 GEMM operands of one
//     implicit-GEMM conv (reference parameter layout: core/update.py, Conv2d
//     weight (Cout, Cin, kh, kw) in any memory format):
//       forward  wf[n][tap*Cin_pad + c]                = s * W[n][c][ky][kx]
//       dgrad    wd[c][tapflip*Cout_pad + n]           = s * W[n][c][ky][kx]
//       bias     bf[n]                                 = s * b[n]
//     Up to two parameters are stacked along N (z||r GRU gates, flow head ||
//     mask head), input channels can be re-laid into padded segments (corr
//     features 324 -> 328, flow 2 -> 8), padding is zero.
//   wgrad_reduce: the per-split fp32 partial slabs of a weight-gradient launch
//     (csrc/conv_igemm.hip) are summed in a fixed split order (deterministic)
//     and written -- scaled, un-padded, split back into the stacked
//     parameters, in the parameters' own strides -- straight into the
//     parameter gradients, or accumulated into a packed fp32 [N][Kpad] buffer.
#include "common.h"
#include "kernel_abi.h"

namespace raft_amd {


namespace {

// padded input channel -> real channel (-1 for a padding slot)
__device__ __forceinline__ int real_channel(const ConvParamDesc& d, int cp) {
  int r0 = 0, p0 = 0;
  for (int i = 0; i < d.nseg; ++i) {
    if (cp < p0 + d.seg_pad[i]) {
      const int o = cp - p0;
      return o < d.seg_real[i] ? r0 + o : -1;
    }
    r0 += d.seg_real[i];
    p0 += d.seg_pad[i];
  }
  return -1;
}

// real input channel -> padded channel
__device__ __forceinline__ int padded_channel(const ConvParamDesc& d, int c) {
  int r0 = 0, p0 = 0;
  for (int i = 0; i < d.nseg; ++i) {
    if (c < r0 + d.seg_real[i]) return p0 + (c - r0);
    r0 += d.seg_real[i];
    p0 += d.seg_pad[i];
  }
  return -1;
}

__device__ __forceinline__ float param_at(const ConvParamDesc& d, int n, int c, int ky, int kx) {
  const int which = n < d.rows[0] ? 0 : 1;
  const int nn = which == 0 ? n : n - d.rows[0];
  const float* w = d.w[which];
  return w[nn * d.ws[which][0] + c * d.ws[which][1] + ky * d.ws[which][2] + kx * d.ws[which][3]];
}

// split-bf16 plane of a scaled fp32 weight: planes 0 / 1 -> hi = bf16(v), plane 2 -> lo = bf16(v - hi)
__device__ __forceinline__ __bf16 plane_of(float v, int plane) {
  const __bf16 hi = static_cast<__bf16>(v);
  return plane < 2 ? hi : static_cast<__bf16>(v - static_cast<float>(hi));
}

// forward column c3 of a split operand (every segment tripled) -> (real channel or -1, plane)
__device__ __forceinline__ int split_channel(const ConvParamDesc& d, int c3, int& plane) {
  int r0 = 0, p0 = 0;
  for (int i = 0; i < d.nseg; ++i) {
    const int w = 3 * d.seg_pad[i];
    if (c3 < p0 + w) {
      const int loc = c3 - p0;
      plane = loc / d.seg_pad[i];
      const int o = loc - plane * d.seg_pad[i];
      return o < d.seg_real[i] ? r0 + o : -1;
    }
    r0 += d.seg_real[i];
    p0 += w;
  }
  plane = 0;
  return -1;
}

// one element i < N Kf + Cin_pad Kd + N of a split-bf16 pack (see pack_conv_weights_split)
__device__ __forceinline__ void pack_split_elem(const ConvParamDesc& d, int N, __bf16* __restrict__ wf, int Kf,
                                                __bf16* __restrict__ wd, int Kd, float* __restrict__ bias, long i) {
  const int taps = d.KH * d.KW;
  const int Cin3 = 3 * d.Cin_pad, G = d.split_dy;
  const long nf = (long)N * Kf;
  const long nd = wd ? (long)d.Cin_pad * Kd : 0;
  if (i < nf) {
    const int n = (int)(i / Kf), k = (int)(i - (long)n * Kf);
    const int tap = k / Cin3;
    __bf16 v = static_cast<__bf16>(0.f);
    if (tap < taps) {
      int plane;
      const int c = split_channel(d, k - tap * Cin3, plane);
      if (c >= 0) v = plane_of(d.scale * param_at(d, n, c, tap / d.KW, tap - (tap / d.KW) * d.KW), plane);
    }
    wf[i] = v;
  } else if (i < nf + nd) {
    const long j = i - nf;
    const int cp = (int)(j / Kd), k = (int)(j - (long)cp * Kd);
    const int tapf = k / (3 * G), n3 = k - tapf * 3 * G;
    const int plane = n3 / G, n = n3 - plane * G;
    __bf16 v = static_cast<__bf16>(0.f);
    if (tapf < taps && n < N) {
      const int c = real_channel(d, cp);
      const int kyf = tapf / d.KW, kxf = tapf - kyf * d.KW;
      if (c >= 0) v = plane_of(d.scale * param_at(d, n, c, d.KH - 1 - kyf, d.KW - 1 - kxf), plane);
    }
    wd[j] = v;
  } else {
    const int n = (int)(i - nf - nd);
    const int which = n < d.rows[0] ? 0 : 1;
    const float* b = d.b[which];
    bias[n] = b ? d.scale * b[which == 0 ? n : n - d.rows[0]] : 0.f;
  }
}

// one element i < N Kf + Cin_pad Kd + N of a bf16 / fp16 pack (see pack_conv_weights)
__device__ __forceinline__ void pack_elem(const ConvParamDesc& d, int N, __bf16* __restrict__ wf, int Kf,
                                          __bf16* __restrict__ wd, int Kd, int Cout_pad, float* __restrict__ bias,
                                          long i) {
  const int taps = d.KH * d.KW;
  const long nf = (long)N * Kf;
  const long nd = wd ? (long)d.Cin_pad * Kd : 0;
  if (i < nf) {
    const int n = (int)(i / Kf), k = (int)(i - (long)n * Kf);
    float v = 0.f;
    const int tap = k / d.Cin_pad;
    if (tap < taps) {
      const int c = real_channel(d, k - tap * d.Cin_pad);
      if (c >= 0) v = d.scale * param_at(d, n, c, tap / d.KW, tap - (tap / d.KW) * d.KW);
    }
    wf[i] = st16(v, d.f16 != 0);
  } else if (i < nf + nd) {
    const long j = i - nf;
    const int cp = (int)(j / Kd), k = (int)(j - (long)cp * Kd);
    float v = 0.f;
    const int tapf = k / Cout_pad, n = k - tapf * Cout_pad;
    if (tapf < taps && n < N) {
      const int c = real_channel(d, cp);
      const int kyf = tapf / d.KW, kxf = tapf - kyf * d.KW;
      if (c >= 0) v = d.scale * param_at(d, n, c, d.KH - 1 - kyf, d.KW - 1 - kxf);
    }
    wd[j] = st16(v, d.f16 != 0);
  } else {
    const int n = (int)(i - nf - nd);
    const int which = n < d.rows[0] ? 0 : 1;
    const float* b = d.b[which];
    bias[n] = b ? d.scale * b[which == 0 ? n : n - d.rows[0]] : 0.f;
  }
}

__global__ __launch_bounds__(256) void pack_conv_weights_split_kernel(ConvParamDesc d, int N, __bf16* __restrict__ wf,
                                                                      int Kf, __bf16* __restrict__ wd, int Kd,
                                                                      float* __restrict__ bias) {
  const long total = (long)N * Kf + (wd ? (long)d.Cin_pad * Kd : 0) + N;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256)
    pack_split_elem(d, N, wf, Kf, wd, Kd, bias, i);
}

__global__ __launch_bounds__(256) void pack_conv_weights_kernel(ConvParamDesc d, int N, __bf16* __restrict__ wf,
                                                                int Kf, __bf16* __restrict__ wd, int Kd,
                                                                int Cout_pad, float* __restrict__ bias) {
  const long total = (long)N * Kf + (wd ? (long)d.Cin_pad * Kd : 0) + N;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256)
    pack_elem(d, N, wf, Kf, wd, Kd, Cout_pad, bias, i);
}

// Every layer of a refinement step in one launch (the step's weights are packed once per
// forward; 12 single-layer launches left the GPU waiting on their host-side issue): the
// element range of job q is [begin_q, begin_{q+1}); a grid-stride loop visits the ranges in
// order, so the job index only moves forward.
__global__ __launch_bounds__(256) void pack_conv_weights_multi_kernel(const PackJobs js) {
  int q = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < js.total; i += (long)gridDim.x * 256) {
    while (q + 1 < js.n && i >= js.j[q + 1].begin) ++q;
    const PackJob& jb = js.j[q];
    const long e = i - jb.begin;
    if (jb.d.split_fw)
      pack_split_elem(jb.d, jb.N, jb.wf, jb.Kf, jb.wd, jb.Kd, jb.bias, e);
    else
      pack_elem(jb.d, jb.N, jb.wf, jb.Kf, jb.wd, jb.Kd, jb.aux, jb.bias, e);
  }
}

// Both reduce kernels: block = 64 consecutive packed columns k of one row n (lane = column),
// its 4 waves sum interleaved subsets of the splits (so a 128-split reduction keeps 32
// independent loads per lane in flight instead of 128 dependent ones), LDS combines the 4
// partial sums in a fixed order.  Blocks past the weight rows reduce the bias partials.
__device__ __forceinline__ float split_sum(const float* __restrict__ src, long sstride, int nsplit, int wave) {
  float v = 0.f;
#pragma unroll 8
  for (int sp = wave; sp < nsplit; sp += 4) v += src[sp * sstride];
  return v;
}

__device__ __forceinline__ float combine4(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  red[wave * 64 + lane] = v;
  __syncthreads();
  return ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
}

// fold layout (ConvParamDesc::fold): packed column kk of a tap -> real channel of its hi-plane
// column (-1 for padding and for lo-plane columns, which the hi lane sums), lo = plane offset
__device__ __forceinline__ int fold_channel(const ConvParamDesc& d, int kk, int& lo) {
  int r0 = 0, p0 = 0;
  for (int i = 0; i < d.nseg; ++i) {
    if (kk < p0 + d.seg_pad[i]) {
      const int o = kk - p0;
      lo = d.seg_pad[i];
      return o < d.seg_real[i] ? r0 + o : -1;
    }
    if (kk < p0 + 2 * d.seg_pad[i]) return -1;
    r0 += d.seg_real[i];
    p0 += 2 * d.seg_pad[i];
  }
  return -1;
}

// Parameter-layout output (scaled, un-padded, split into the stacked parameters).
__global__ __launch_bounds__(256) void wgrad_reduce_params_kernel(const float* __restrict__ slab, int nsplit,
                                                                  int Npad, int Kpad,
                                                                  const float* __restrict__ dbslab, int ndb,
                                                                  ConvParamDesc d, int N, int accumulate) {
  __shared__ float red[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ktap = d.fold ? 2 * d.Cin_pad : d.Cin_pad;  // packed columns per tap
  const int kch = (d.KH * d.KW * ktap + 63) / 64;
  const long blk = blockIdx.x;
  if (blk < (long)N * kch) {
    const int n = (int)(blk / kch);
    const int k = (int)(blk - (long)n * kch) * 64 + lane;
    const int tap = k / ktap;
    const bool live = tap < d.KH * d.KW;
    int lo = 0;
    const int c = !live ? -1 : (d.fold ? fold_channel(d, k - tap * ktap, lo) : real_channel(d, k - tap * ktap));
    const long ss = (long)Npad * Kpad;
    float v0 = 0.f;
    if (c >= 0) {
      v0 = split_sum(slab + (long)n * Kpad + k, ss, nsplit, wave);
      if (lo) v0 += split_sum(slab + (long)n * Kpad + k + lo, ss, nsplit, wave);
    }
    const float v = combine4(v0, red);
    if (wave != 0 || c < 0) return;
    const int which = n < d.rows[0] ? 0 : 1;
    const int nn = which == 0 ? n : n - d.rows[0];
    const int ky = tap / d.KW, kx = tap - ky * d.KW;
    float* o = d.w[which] + nn * d.ws[which][0] + c * d.ws[which][1] + ky * d.ws[which][2] + kx * d.ws[which][3];
    *o = accumulate ? *o + d.scale * v : d.scale * v;
  } else {
    const int n = (int)(blk - (long)N * kch) * 64 + lane;
    float v = 0.f;
    if (n < N && dbslab)
      for (int j = wave; j < ndb; j += 4) v += dbslab[(long)j * Npad + n];
    v = combine4(v, red);
    if (wave != 0 || n >= N) return;
    const int which = n < d.rows[0] ? 0 : 1;
    float* b = d.b[which];
    if (b) {
      float* o = b + (which == 0 ? n : n - d.rows[0]);
      *o = accumulate ? *o + d.scale * v : d.scale * v;
    }
  }
}

// Packed output: dw[n][k] (+)= sum_s slab[s][n][k] for n < N, k < Kpad; db[n] (+)= sum of partials.
__global__ __launch_bounds__(256) void wgrad_reduce_packed_kernel(const float* __restrict__ slab, int nsplit,
                                                                  int Npad, int Kpad, int K,
                                                                  const float* __restrict__ dbslab, int ndb,
                                                                  float* __restrict__ dw, long ldw,
                                                                  float* __restrict__ db, int N, int accumulate) {
  __shared__ float red[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kch = Kpad / 64;
  const long blk = blockIdx.x;
  if (blk < (long)N * kch) {
    const int n = (int)(blk / kch);
    const int k = (int)(blk - (long)n * kch) * 64 + lane;
    // slab columns past K may be unwritten
    const float v = combine4(k < K ? split_sum(slab + (long)n * Kpad + k, (long)Npad * Kpad, nsplit, wave) : 0.f,
                             red);
    if (wave != 0) return;
    float* o = dw + (long)n * ldw + k;
    *o = accumulate ? *o + v : v;
  } else {
    const int n = (int)(blk - (long)N * kch) * 64 + lane;
    float v = 0.f;
    if (n < N)
      for (int j = wave; j < ndb; j += 4) v += dbslab[(long)j * Npad + n];
    v = combine4(v, red);
    if (wave != 0 || n >= N || !db) return;
    db[n] = accumulate ? db[n] + v : v;
  }
}

inline dim3 grid_of(long total) {
  long b = (total + 255) / 256;
  return dim3((unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192));
}

}  // namespace

hipError_t launch_pack_conv_weights(const ConvParamDesc& d, int N, void* wf, int Kf, void* wd, int Kd, int Cout_pad,
                                    float* bias, hipStream_t s) {
  const long total = (long)N * Kf + (wd ? (long)d.Cin_pad * Kd : 0) + N;
  if (d.split_fw) {
    if (wd && d.split_dy <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pack_conv_weights_split_kernel, grid_of(total), dim3(256), 0, s, d, N, static_cast<__bf16*>(wf),
                       Kf, static_cast<__bf16*>(wd), Kd, bias);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pack_conv_weights_kernel, grid_of(total), dim3(256), 0, s, d, N, static_cast<__bf16*>(wf), Kf,
                     static_cast<__bf16*>(wd), Kd, Cout_pad, bias);
  return hipGetLastError();
}

hipError_t launch_pack_conv_weights_multi(const PackJobs& js, hipStream_t s) {
  if (js.n < 1 || js.n > kPackJobs) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_conv_weights_multi_kernel, grid_of(js.total), dim3(256), 0, s, js);
  return hipGetLastError();
}

hipError_t launch_wgrad_reduce_params(const float* slab, int nsplit, int Npad, int Kpad, const float* dbslab, int ndb,
                                      const ConvParamDesc& d, int N, int accumulate, hipStream_t s) {
  const long kch = (d.KH * d.KW * (d.fold ? 2 : 1) * d.Cin_pad + 63) / 64;
  // bias blocks also without partials: they write the exact zero bias gradient (convs in front of
  // InstanceNorm / training BatchNorm) in this launch instead of a separate fill
  const long blocks = (long)N * kch + ((dbslab || d.b[0] || d.b[1]) ? (N + 63) / 64 : 0);
  hipLaunchKernelGGL(wgrad_reduce_params_kernel, dim3((unsigned)blocks), dim3(256), 0, s, slab, nsplit, Npad, Kpad,
                     dbslab, ndb, d, N, accumulate);
  return hipGetLastError();
}

hipError_t launch_wgrad_reduce_packed(const float* slab, int nsplit, int Npad, int Kpad, int K, const float* dbslab,
                                      int ndb, float* dw, long ldw, float* db, int N, int accumulate, hipStream_t s) {
  const long blocks = (long)N * (Kpad / 64) + (db ? (N + 63) / 64 : 0);
  hipLaunchKernelGGL(wgrad_reduce_packed_kernel, dim3((unsigned)blocks), dim3(256), 0, s, slab, nsplit, Npad, Kpad, K,
                     dbslab, ndb, dw, ldw, db, N, accumulate);
  return hipGetLastError();
}

}  // namespace raft_amd
