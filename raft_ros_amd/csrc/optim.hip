// Gradient clipping + AdamW in two launches (the reference's optimizer step, train.py:75-86 and
// :154-157: clip_grad_norm_(model.parameters(), args.clip) followed by AdamW.step()).
//
// torch's eager version of this step is ~10 launches and ~2.6 ms of HOST time per training step
// on MI355X (clip 1.5 ms: per-step grouping of ~200 gradients by device / dtype, _foreach_norm,
// stack, norm, clamp, _foreach_mul_; fused AdamW 1.1 ms: _init_group over every parameter;
// profiles/r5o_host_lead.log).  Here:
//   1. adamw_norm_kernel: one block per 16 K-element chunk of the parameter set writes the
//      chunk's sum of squared gradients (one partial per block, no atomics);
//   2. adamw_update_kernel: every block sums ALL partials in the same fixed order (a few hundred
//      floats from L2), so the norm and the clip coefficient are bitwise identical in every
//      block and run-to-run; a non-finite norm skips the step (no update, step counter kept,
//      ``skipped`` += 1: the trainer's failure guard); otherwise clip + AdamW on its chunk.
// The step counter lives on the device in a two-slot buffer (read slot `par`, block 0 writes
// slot par ^ 1), so no block reads a value another block has already advanced.
// Gradient pointers change every step (autograd allocates them), so they travel in the kernel
// arguments (128 per launch); parameter / moment pointers and the chunk table are device tables
// built once per parameter set.
#include "common.h"

namespace raft_amd {

namespace {

constexpr int kOptChunk = 16384;  // elements per block (kernel_abi.h kAdamChunk)
static_assert(kOptChunk == kAdamChunk, "chunk size");

__device__ __forceinline__ float block_sum(float v, float* red) {
  // fixed-order block reduction: wave butterfly, then wave 0 adds the four wave sums in order
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  const float s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void adamw_norm_kernel(const AdamArgs a) {
  __shared__ float red[4];
  const int blk = a.blk0 + blockIdx.x;
  const int t = a.blocks[3 * blk], start = a.blocks[3 * blk + 1], len = a.blocks[3 * blk + 2];
  const float* g = a.g[t - a.t0];
  float s = 0.f;
  if ((reinterpret_cast<uintptr_t>(g + start) & 15) == 0 && (len & 3) == 0) {
    const f32x4* g4 = reinterpret_cast<const f32x4*>(g + start);
    for (int i = threadIdx.x; i < len / 4; i += 256) {
      const f32x4 v = g4[i];
      s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    }
  } else {
    for (int i = threadIdx.x; i < len; i += 256) s += g[start + i] * g[start + i];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) a.partial[blk] = s;
}

__global__ __launch_bounds__(256) void adamw_update_kernel(const AdamArgs a) {
  __shared__ float red[4];
  // the global norm: every block, same order
  float s = 0.f;
  for (int i = threadIdx.x; i < a.nblocks; i += 256) s += a.partial[i];
  const float norm = sqrtf(block_sum(s, red));
  const bool finite = isfinite(norm);
  const float step_old = a.steps[a.par];
  const int blk = a.blk0 + blockIdx.x;
  if (blk == 0 && threadIdx.x == 0) {
    a.steps[a.par ^ 1] = finite ? step_old + 1.f : step_old;
    if (a.norm_out) *a.norm_out = norm;
    if (!finite && a.skipped) *a.skipped += 1.f;
  }
  if (!finite) return;
  const float coef = a.max_norm > 0.f ? fminf(a.max_norm / (norm + 1e-6f), 1.f) : 1.f;
  const float step = step_old + 1.f;
  const float bc1 = 1.f - powf(a.beta1, step), bc2 = 1.f - powf(a.beta2, step);
  const float step_size = a.lr / bc1, bc2_sqrt = sqrtf(bc2);
  const float decay = 1.f - a.lr * a.wd;
  const int t = a.blocks[3 * blk], start = a.blocks[3 * blk + 1], len = a.blocks[3 * blk + 2];
  const float* g = a.g[t - a.t0] + start;
  float* p = reinterpret_cast<float*>(a.ptrs[3 * t]) + start;
  float* m = reinterpret_cast<float*>(a.ptrs[3 * t + 1]) + start;
  float* v = reinterpret_cast<float*>(a.ptrs[3 * t + 2]) + start;
  for (int i = threadIdx.x; i < len; i += 256) {
    const float gi = g[i] * coef;
    const float mi = a.beta1 * m[i] + (1.f - a.beta1) * gi;
    const float vi = a.beta2 * v[i] + (1.f - a.beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + a.eps;
    p[i] = p[i] * decay - step_size * mi / denom;
  }
}

}  // namespace

hipError_t launch_adamw(const AdamArgs& a, int nblk, bool update, hipStream_t s) {
  if (nblk <= 0) return hipSuccess;
  if (update) hipLaunchKernelGGL(adamw_update_kernel, dim3((unsigned)nblk), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(adamw_norm_kernel, dim3((unsigned)nblk), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace raft_amd
