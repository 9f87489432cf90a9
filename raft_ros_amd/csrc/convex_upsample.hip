// Fused convex 8x upsampling of the flow field (reference RAFT.upsample_flow,
// core/raft.py:72-83):
//   out[b, c, 8y+i, 8x+j] = sum_k softmax_k(mask[b, k*64 + i*8 + j, y, x]) * 8 * flow[b, c, y+ky-1, x+kx-1]
// with k = ky*3 + kx (F.unfold order) and zero padding outside the field.
//
// One wave64 per low-resolution pixel: lane = i*8 + j owns one of the 64
// sub-pixels, so the 9-way softmax, the gather and the pixel shuffle are a
// single pass with no intermediate tensors (the reference materialises the
// (N,1,9,8,8,H,W) softmax, the unfold and a permute copy every iteration).
// The mask may be in any memory format (strides are passed), so the
// channels-last output of the mask head is consumed without a copy.
//
// Backward: dmask is produced in the same pass; the flow gradient is reduced
// across the wave per neighbour (deterministic, no atomics) into a
// (B, 9, 2, H, W) partial buffer that a second tiny kernel gathers.
#include "common.h"

namespace raft_amd {
namespace {

template <typename MT>
__global__ __launch_bounds__(256) void convex_up_fwd_kernel(const float* __restrict__ flow,
                                                            const MT* __restrict__ mask, long msN,
                                                            long msC, long msH, long msW,
                                                            float* __restrict__ out, int B, int H,
                                                            int W) {
  const int lane = threadIdx.x & 63;
  const long pix = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pix >= (long)B * H * W) return;
  const int x = pix % W;
  const int y = (pix / W) % H;
  const int b = pix / ((long)H * W);
  const int i = lane >> 3, j = lane & 7;
  const MT* m = mask + b * msN + y * msH + x * msW;
  float logit[9];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    logit[k] = to_f32(m[(long)(k * 64 + lane) * msC]);
    mx = fmaxf(mx, logit[k]);
  }
  float den = 0.f, o0 = 0.f, o1 = 0.f;
  const long HW = (long)H * W;
  const float* f0 = flow + (long)b * 2 * HW;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float e = __expf(logit[k] - mx);
    den += e;
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      o0 += e * f0[yy * W + xx];
      o1 += e * f0[HW + yy * W + xx];
    }
  }
  const float inv = 8.f / den;
  const long W8 = 8L * W;
  const long oHW = 64L * HW;
  float* o = out + (long)b * 2 * oHW + (8L * y + i) * W8 + 8L * x + j;
  o[0] = o0 * inv;
  o[oHW] = o1 * inv;
}

template <typename MT>
__global__ __launch_bounds__(256) void convex_up_bwd_kernel(
    const float* __restrict__ flow, const MT* __restrict__ mask, long msN, long msC, long msH,
    long msW, const float* __restrict__ gout, MT* __restrict__ dmask, long dsN, long dsC, long dsH, long dsW,
    float* __restrict__ part, int B, int H, int W) {
  const int lane = threadIdx.x & 63;
  const long pix = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pix >= (long)B * H * W) return;
  const int x = pix % W;
  const int y = (pix / W) % H;
  const int b = pix / ((long)H * W);
  const int i = lane >> 3, j = lane & 7;
  const long HW = (long)H * W;
  const long moff = b * msN + y * msH + x * msW;
  float p[9];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    p[k] = to_f32(mask[moff + (long)(k * 64 + lane) * msC]);
    mx = fmaxf(mx, p[k]);
  }
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    p[k] = __expf(p[k] - mx);
    den += p[k];
  }
  const float inv = 1.f / den;
  const long W8 = 8L * W, oHW = 64L * HW;
  const float* g = gout + (long)b * 2 * oHW + (8L * y + i) * W8 + 8L * x + j;
  const float g0 = g[0], g1 = g[oHW];
  const float* f0 = flow + (long)b * 2 * HW;
  float gv[9];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    p[k] *= inv;
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    float v0 = 0.f, v1 = 0.f;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      v0 = 8.f * f0[yy * W + xx];
      v1 = 8.f * f0[HW + yy * W + xx];
    }
    gv[k] = g0 * v0 + g1 * v1;
    dot += p[k] * gv[k];
  }
#pragma unroll
  for (int k = 0; k < 9; ++k)
    dmask[b * dsN + y * dsH + x * dsW + (long)(k * 64 + lane) * dsC] = from_f32<MT>(p[k] * (gv[k] - dot));
  // d flow(neighbour k, c) = sum over the 64 sub-pixels of 8 * p_k * g_c
  float* pt = part + (long)b * 18 * HW + (long)y * W + x;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float s0 = wave_sum(8.f * p[k] * g0);
    const float s1 = wave_sum(8.f * p[k] * g1);
    if (lane == 0) {
      pt[(k * 2 + 0) * HW] = s0;
      pt[(k * 2 + 1) * HW] = s1;
    }
  }
}

// ---- row-segment kernels for a dense channels-last mask (msC == 1, msW == 576: the mask head's
// (P, 576) rows). A workgroup owns kUpSeg consecutive low-res pixels of one image row: their mask
// rows (one contiguous block) are staged in LDS with 16-byte loads and the 3 x (kUpSeg + 2) flow
// neighbourhood beside them (zero outside the field, which is F.unfold's padding). Thread t then
// owns pixel t / 16 and the 4 sub-pixels (i, j0..j0+3), i = (t / 2) % 8, j0 = 4 (t % 2): the
// output goes out as float4s, 128 contiguous bytes per pixel row, and a pixel's 16 threads sit
// in one 16-lane row of the wave for the flow-gradient reduction. All index math is 32-bit
// (the launcher checks the sizes); the per-pixel kernels above stay for any other mask layout.
constexpr int kUpSeg = 16;

template <typename MT>
struct UpSegSmem {
  MT m[kUpSeg * 576];
  float f[2][3][kUpSeg + 2];
};

template <typename MT>
__device__ __forceinline__ void up_seg_stage(UpSegSmem<MT>& sm, const float* __restrict__ flow,
                                             const MT* __restrict__ mrow, int b, int y, int x0, int npx,
                                             int H, int W) {
  constexpr int CH = 16 / sizeof(MT);
  const int t = threadIdx.x;
  const int nch = npx * 576 / CH;
  for (int c = t; c < nch; c += 256)
    reinterpret_cast<u32x4*>(sm.m)[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(mrow) + c);
  constexpr int FW = kUpSeg + 2;
  if (t < 6 * FW) {
    const int c = t / (3 * FW), r = (t / FW) % 3, q = t % FW;
    const int yy = y - 1 + r, xx = x0 - 1 + q;
    const int HW = H * W;
    sm.f[c][r][q] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? flow[(b * 2 + c) * HW + yy * W + xx] : 0.f;
  }
  __syncthreads();
}

// softmax over the 9 neighbours of the thread's 4 sub-pixels, from the staged mask row
template <typename MT>
__device__ __forceinline__ void up_seg_softmax(const MT* mp, float p[9][4]) {
  typedef MT mt4 __attribute__((ext_vector_type(4)));
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const mt4 v = *reinterpret_cast<const mt4*>(mp + k * 64);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      p[k][s] = to_f32(v[s]);
      mx[s] = fmaxf(mx[s], p[k][s]);
    }
  }
  float den[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      p[k][s] = __expf(p[k][s] - mx[s]);
      den[s] += p[k][s];
    }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float inv = 1.f / den[s];
#pragma unroll
    for (int k = 0; k < 9; ++k) p[k][s] *= inv;
  }
}

template <typename MT>
__global__ __launch_bounds__(256) void convex_up_fwd_seg_kernel(const float* __restrict__ flow,
                                                                const MT* __restrict__ mask, int msN, int msH,
                                                                float* __restrict__ out, int H, int W, int nseg) {
  __shared__ __align__(16) UpSegSmem<MT> sm;
  int tile = blockIdx.x;
  const int sx = tile % nseg;
  tile /= nseg;
  const int y = tile % H, b = tile / H;
  const int x0 = sx * kUpSeg, npx = min(kUpSeg, W - x0);
  up_seg_stage(sm, flow, mask + b * msN + y * msH + x0 * 576, b, y, x0, npx, H, W);
  const int t = threadIdx.x, px = t >> 4, i = (t >> 1) & 7, j0 = (t & 1) * 4;
  if (px >= npx) return;
  float p[9][4];
  up_seg_softmax(sm.m + px * 576 + i * 8 + j0, p);
  f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float u = 8.f * sm.f[0][k / 3][px + k % 3], v = 8.f * sm.f[1][k / 3][px + k % 3];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      o0[s] += p[k][s] * u;
      o1[s] += p[k][s] * v;
    }
  }
  const int W8 = 8 * W, oHW = 64 * H * W;
  float* o = out + b * 2 * oHW + (8 * y + i) * W8 + 8 * (x0 + px) + j0;
  *reinterpret_cast<f32x4*>(o) = o0;
  *reinterpret_cast<f32x4*>(o + oHW) = o1;
}

template <typename MT>
__global__ __launch_bounds__(256) void convex_up_bwd_seg_kernel(const float* __restrict__ flow,
                                                                const MT* __restrict__ mask, int msN, int msH,
                                                                const float* __restrict__ gout,
                                                                MT* __restrict__ dmask, int dsN, int dsH,
                                                                float* __restrict__ part, int H, int W, int nseg) {
  __shared__ __align__(16) UpSegSmem<MT> sm;
  int tile = blockIdx.x;
  const int sx = tile % nseg;
  tile /= nseg;
  const int y = tile % H, b = tile / H;
  const int x0 = sx * kUpSeg, npx = min(kUpSeg, W - x0);
  up_seg_stage(sm, flow, mask + b * msN + y * msH + x0 * 576, b, y, x0, npx, H, W);
  const int t = threadIdx.x, px = t >> 4, i = (t >> 1) & 7, j0 = (t & 1) * 4;
  const bool live = px < npx;
  const int HW = H * W;
  if (live) {
    const int W8 = 8 * W, oHW = 64 * HW;
    const float* g = gout + b * 2 * oHW + (8 * y + i) * W8 + 8 * (x0 + px) + j0;
    const f32x4 g0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g));
    const f32x4 g1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + oHW));
    MT* mp = sm.m + px * 576 + i * 8 + j0;
    float p[9][4], gv[9][4];
    up_seg_softmax(mp, p);
    float dot[4] = {0.f, 0.f, 0.f, 0.f};
    float pf[9][2];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float u = 8.f * sm.f[0][k / 3][px + k % 3], v = 8.f * sm.f[1][k / 3][px + k % 3];
      pf[k][0] = pf[k][1] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        gv[k][s] = g0[s] * u + g1[s] * v;
        dot[s] += p[k][s] * gv[k][s];
        pf[k][0] += p[k][s] * g0[s];
        pf[k][1] += p[k][s] * g1[s];
      }
    }
    // dmask over the thread's own staged mask entries (no other thread reads them)
    typedef MT mt4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      mt4 d;
#pragma unroll
      for (int s = 0; s < 4; ++s) d[s] = from_f32<MT>(p[k][s] * (gv[k][s] - dot[s]));
      *reinterpret_cast<mt4*>(mp + k * 64) = d;
    }
    // d flow(neighbour k, c) = sum over the pixel's 64 sub-pixels of 8 p_k g_c: its 16 lanes
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float v = pf[k][c];
#pragma unroll
        for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off, 16);
        pf[k][c] = v;
      }
    if ((t & 15) == 0) {
      float* pt = part + b * 18 * HW + y * W + x0 + px;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        pt[(k * 2 + 0) * HW] = 8.f * pf[k][0];
        pt[(k * 2 + 1) * HW] = 8.f * pf[k][1];
      }
    }
  }
  __syncthreads();
  constexpr int CH = 16 / sizeof(MT);
  const int nch = npx * 576 / CH;
  u32x4* drow = reinterpret_cast<u32x4*>(dmask + b * dsN + y * dsH + x0 * 576);
  for (int c = t; c < nch; c += 256) drow[c] = reinterpret_cast<const u32x4*>(sm.m)[c];
}

// dflow[b, c, y', x'] = sum_k part[b, k, c, y'-ky+1, x'-kx+1]
__global__ __launch_bounds__(256) void convex_up_gather_kernel(const float* __restrict__ part,
                                                               float* __restrict__ dflow, int B,
                                                               int H, int W) {
  const long HW = (long)H * W;
  const long total = (long)B * 2 * HW;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int x = idx % W;
  const int y = (idx / W) % H;
  const int c = (idx / HW) % 2;
  const int b = idx / (2 * HW);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y - (k / 3) + 1, xx = x - (k % 3) + 1;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) s += part[((long)b * 18 + k * 2 + c) * HW + yy * W + xx];
  }
  dflow[idx] = s;
}

// Per low-res pixel: both flow-gradient channels, written as (P, ld) bf16 rows [du, dv, 0..0]
// (the dY operand of the flow head's last conv in the fused update block) and optionally fp32.
__global__ __launch_bounds__(256) void convex_up_gather_rows_kernel(const float* __restrict__ part,
                                                                    __bf16* __restrict__ rows, int ld,
                                                                    float* __restrict__ dflow, int B, int H,
                                                                    int W, int f16) {
  const long HW = (long)H * W;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)B * HW) return;
  const int x = p % W;
  const int y = (p / W) % H;
  const int b = p / HW;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y - (k / 3) + 1, xx = x - (k % 3) + 1;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      const long o = ((long)b * 18 + k * 2) * HW + yy * W + xx;
      s0 += part[o];
      s1 += part[o + HW];
    }
  }
  __bf16* r = rows + p * ld;
  r[0] = st16(s0, f16 != 0);
  r[1] = st16(s1, f16 != 0);
  for (int c = 2; c < ld; ++c) r[c] = st16(0.f, false);
  if (dflow) {
    dflow[(long)b * 2 * HW + y * W + x] = s0;
    dflow[(long)b * 2 * HW + HW + y * W + x] = s1;
  }
}

}  // namespace

hipError_t launch_convex_up_fwd(const float* flow, const void* mask, int m_dtype, long msN, long msC,
                                long msH, long msW, float* out, int B, int H, int W, hipStream_t s) {
  const long npix = (long)B * H * W;
  if (npix == 0) return hipSuccess;
  const int esz = m_dtype == kF32 ? 4 : 2;
  if (up_seg_ok(reinterpret_cast<uintptr_t>(mask), esz, msN, msC, msH, msW, B, H, W)) {
    const int nseg = (W + kUpSeg - 1) / kUpSeg;
    const dim3 g(B * H * nseg), blk(256);
    if (m_dtype == kBF16)
      hipLaunchKernelGGL(convex_up_fwd_seg_kernel<__bf16>, g, blk, 0, s, flow, static_cast<const __bf16*>(mask),
                         (int)msN, (int)msH, out, H, W, nseg);
    else if (m_dtype == kF16)
      hipLaunchKernelGGL(convex_up_fwd_seg_kernel<_Float16>, g, blk, 0, s, flow,
                         static_cast<const _Float16*>(mask), (int)msN, (int)msH, out, H, W, nseg);
    else
      hipLaunchKernelGGL(convex_up_fwd_seg_kernel<float>, g, blk, 0, s, flow, static_cast<const float*>(mask),
                         (int)msN, (int)msH, out, H, W, nseg);
    return hipGetLastError();
  }
  const dim3 g((npix + 3) / 4), blk(256);
  if (m_dtype == kBF16)
    hipLaunchKernelGGL(convex_up_fwd_kernel<__bf16>, g, blk, 0, s, flow,
                       static_cast<const __bf16*>(mask), msN, msC, msH, msW, out, B, H, W);
  else if (m_dtype == kF16)
    hipLaunchKernelGGL(convex_up_fwd_kernel<_Float16>, g, blk, 0, s, flow,
                       static_cast<const _Float16*>(mask), msN, msC, msH, msW, out, B, H, W);
  else
    hipLaunchKernelGGL(convex_up_fwd_kernel<float>, g, blk, 0, s, flow,
                       static_cast<const float*>(mask), msN, msC, msH, msW, out, B, H, W);
  return hipGetLastError();
}

hipError_t launch_convex_up_bwd(const float* flow, const void* mask, int m_dtype, long msN, long msC,
                                long msH, long msW, const float* gout, void* dmask, long dsN, long dsC,
                                long dsH, long dsW, float* part, float* dflow, void* rows, int rows_ld, int B,
                                int H, int W, hipStream_t s) {
  const long npix = (long)B * H * W;
  if (npix == 0) return hipSuccess;
  const dim3 blk(256);
  const int esz = m_dtype == kF32 ? 4 : 2;
  if (up_seg_ok(reinterpret_cast<uintptr_t>(mask), esz, msN, msC, msH, msW, B, H, W) &&
      up_seg_ok(reinterpret_cast<uintptr_t>(dmask), esz, dsN, dsC, dsH, dsW, B, H, W)) {
    const int nseg = (W + kUpSeg - 1) / kUpSeg;
    const dim3 g(B * H * nseg);
    if (m_dtype == kBF16)
      hipLaunchKernelGGL(convex_up_bwd_seg_kernel<__bf16>, g, blk, 0, s, flow, static_cast<const __bf16*>(mask),
                         (int)msN, (int)msH, gout, static_cast<__bf16*>(dmask), (int)dsN, (int)dsH, part, H, W,
                         nseg);
    else if (m_dtype == kF16)
      hipLaunchKernelGGL(convex_up_bwd_seg_kernel<_Float16>, g, blk, 0, s, flow,
                         static_cast<const _Float16*>(mask), (int)msN, (int)msH, gout,
                         static_cast<_Float16*>(dmask), (int)dsN, (int)dsH, part, H, W, nseg);
    else
      hipLaunchKernelGGL(convex_up_bwd_seg_kernel<float>, g, blk, 0, s, flow, static_cast<const float*>(mask),
                         (int)msN, (int)msH, gout, static_cast<float*>(dmask), (int)dsN, (int)dsH, part, H, W,
                         nseg);
  } else {
  const dim3 g((npix + 3) / 4);
  if (m_dtype == kBF16)
    hipLaunchKernelGGL(convex_up_bwd_kernel<__bf16>, g, blk, 0, s, flow,
                       static_cast<const __bf16*>(mask), msN, msC, msH, msW, gout,
                       static_cast<__bf16*>(dmask), dsN, dsC, dsH, dsW, part, B, H, W);
  else if (m_dtype == kF16)
    hipLaunchKernelGGL(convex_up_bwd_kernel<_Float16>, g, blk, 0, s, flow,
                       static_cast<const _Float16*>(mask), msN, msC, msH, msW, gout,
                       static_cast<_Float16*>(dmask), dsN, dsC, dsH, dsW, part, B, H, W);
  else
    hipLaunchKernelGGL(convex_up_bwd_kernel<float>, g, blk, 0, s, flow,
                       static_cast<const float*>(mask), msN, msC, msH, msW, gout,
                       static_cast<float*>(dmask), dsN, dsC, dsH, dsW, part, B, H, W);
  }
  RAFT_HIP_CHECK(hipGetLastError());
  if (rows) {
    hipLaunchKernelGGL(convex_up_gather_rows_kernel, dim3((npix + 255) / 256), blk, 0, s, part,
                       static_cast<__bf16*>(rows), rows_ld, dflow, B, H, W, m_dtype == kF16 ? 1 : 0);
    return hipGetLastError();
  }
  const long tot = (long)B * 2 * H * W;
  hipLaunchKernelGGL(convex_up_gather_kernel, dim3((tot + 255) / 256), blk, 0, s, part, dflow, B, H,
                     W);
  return hipGetLastError();
}

}  // namespace raft_amd
