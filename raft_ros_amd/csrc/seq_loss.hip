// Fused RAFT sequence loss (forward + backward) and final-iterate flow metrics.
//
// Reference: train.py:47-72 (sequence_loss) -- per prediction i the reference
// launches ~6 elementwise/reduce kernels forward and ~5 backward (sub, abs,
// mul by the valid mask, mean, weighted add; sign, mul, ...), plus ~15 more
// for the EPE / 1-3-5 px metrics: ~150 launches and 2-3 full passes over every
// (B, 2, 8H, 8W) fp32 prediction per step.  Here:
//   * forward: ONE pass that reads gt/valid once per pixel, streams all n
//     predictions, and emits per-workgroup partials of
//     {weighted L1 sum, EPE sum, <1px, <3px, <5px, valid count} (metrics of the
//     last prediction);
//   * backward: ONE pass writing every prediction's gradient
//     g_i = dL * gamma^(n-1-i) * vmask * sign(p_i - gt) / (B*2*H*W).
// Both are HBM-bound streaming kernels (one pixel per lane, coalesced plane
// reads); partials are reduced by the host wrapper (deterministic, no atomics).
#include "common.h"

#include <algorithm>

namespace raft_amd {



namespace {

constexpr int kLossThreads = 256;

__device__ __forceinline__ float pixel_mask(const float* gt, const float* valid, long b, long pix,
                                            long HW, float max_flow, float& u, float& v) {
  u = gt[(b * 2) * HW + pix];
  v = gt[(b * 2 + 1) * HW + pix];
  const float mag = sqrtf(u * u + v * v);
  return (valid[b * HW + pix] >= 0.5f && mag < max_flow) ? 1.f : 0.f;
}

__global__ void __launch_bounds__(kLossThreads)
seq_loss_fwd_kernel(SeqPreds preds, int n, const float* __restrict__ gt,
                    const float* __restrict__ valid, float gamma, float max_flow, long B, long HW,
                    float* __restrict__ partial) {
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const long P = B * HW;
  for (long i = (long)blockIdx.x * kLossThreads + threadIdx.x; i < P;
       i += (long)gridDim.x * kLossThreads) {
    const long b = i / HW, pix = i - b * HW;
    float gu, gv;
    const float m = pixel_mask(gt, valid, b, pix, HW, max_flow, gu, gv);
    const long ou = (b * 2) * HW + pix, ov = ou + HW;
    float w = 1.f, l1 = 0.f;
    for (int k = n - 1; k >= 0; --k) {  // gamma^(n-1-k): last prediction weight 1
      const float du = preds.p[k][ou] - gu;
      const float dv = preds.p[k][ov] - gv;
      l1 += w * (fabsf(du) + fabsf(dv));
      w *= gamma;
      if (k == n - 1) {
        const float epe = sqrtf(du * du + dv * dv);
        acc[1] += m * epe;
        acc[2] += (epe < 1.f) ? m : 0.f;
        acc[3] += (epe < 3.f) ? m : 0.f;
        acc[4] += (epe < 5.f) ? m : 0.f;
      }
    }
    acc[0] += m * l1;
    acc[5] += m;
  }
  __shared__ float red[kLossThreads / kWave][6];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const float s = wave_sum(acc[j]);
    if (lane == 0) red[wid][j] = s;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    float s = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < kLossThreads / kWave; ++w2) s += red[w2][threadIdx.x];
    partial[(long)blockIdx.x * 6 + threadIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kLossThreads)
seq_loss_bwd_kernel(SeqPreds preds, SeqGrads grads, int n, const float* __restrict__ gt,
                    const float* __restrict__ valid, const float* __restrict__ dloss, float gamma,
                    float max_flow, long B, long HW) {
  const long P = B * HW;
  const float scale = dloss[0] / (float)(2 * P);
  for (long i = (long)blockIdx.x * kLossThreads + threadIdx.x; i < P;
       i += (long)gridDim.x * kLossThreads) {
    const long b = i / HW, pix = i - b * HW;
    float gu, gv;
    const float m = pixel_mask(gt, valid, b, pix, HW, max_flow, gu, gv);
    const long ou = (b * 2) * HW + pix, ov = ou + HW;
    float w = scale * m;
    for (int k = n - 1; k >= 0; --k) {
      const float du = preds.p[k][ou] - gu;
      const float dv = preds.p[k][ov] - gv;
      // d|x|/dx = sign(x), sign(0) = 0 (matches torch.abs backward)
      grads.g[k][ou] = du > 0.f ? w : (du < 0.f ? -w : 0.f);
      grads.g[k][ov] = dv > 0.f ? w : (dv < 0.f ? -w : 0.f);
      w *= gamma;
    }
  }
}

int loss_grid(long P) {
  // ~8 workgroups per CU on 256 CUs; each lane then streams a handful of pixels
  return (int)std::min<long>((P + kLossThreads - 1) / kLossThreads, 2048);
}

}  // namespace

int seq_loss_num_blocks(long P) { return loss_grid(P); }

hipError_t launch_seq_loss_fwd(const SeqPreds& preds, int n, const float* gt, const float* valid,
                               float gamma, float max_flow, long B, long HW, float* partial,
                               hipStream_t s) {
  if (n < 1 || n > kMaxPreds) return hipErrorInvalidValue;
  const int grid = loss_grid(B * HW);
  hipLaunchKernelGGL(seq_loss_fwd_kernel, dim3(grid), dim3(kLossThreads), 0, s, preds, n, gt, valid,
                     gamma, max_flow, B, HW, partial);
  return hipGetLastError();
}

hipError_t launch_seq_loss_bwd(const SeqPreds& preds, const SeqGrads& grads, int n, const float* gt,
                               const float* valid, const float* dloss, float gamma, float max_flow,
                               long B, long HW, hipStream_t s) {
  if (n < 1 || n > kMaxPreds) return hipErrorInvalidValue;
  const int grid = loss_grid(B * HW);
  hipLaunchKernelGGL(seq_loss_bwd_kernel, dim3(grid), dim3(kLossThreads), 0, s, preds, grads, n, gt,
                     valid, dloss, gamma, max_flow, B, HW);
  return hipGetLastError();
}

}  // namespace raft_amd
