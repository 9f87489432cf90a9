// Small fused elementwise kernels around the implicit-GEMM convs of the fused
// RAFT update block (raft_ros_amd/ops/update_fused.py).  All tensors are
// pixel-major (P, C) views with a pixel stride; one thread per (pixel, channel).
//
//   gru_bwd_a:  from dH (fp32), z, q, h of a GRU stage (core/update.py:43-58)
//               dq_pre = dH * z * (1 - q^2)        -> bf16 (dy of the q conv)
//               dz_pre = dH * (q - h) * z (1 - z)  -> bf16 (first half of the z||r dy)
//               carry  = dH * (1 - z)              -> fp32
//   gru_bwd_b:  from d(rh) (fp32, in place), r, h, carry
//               dr_pre = d(rh) * h * r (1 - r)     -> bf16 (second half of the z||r dy)
//               dh     = carry + d(rh) * r         -> fp32, written over d(rh)
//   masked_cast: out_bf16 = src_fp32 * (mask > 0)   (ReLU' + cast for the next dy)
//   pack_flow:  (B, 2, H, W) fp32 flow -> (P, 8) bf16 [u, v, 0...] and the two
//               flow channels of the motion-feature buffer (torch.cat in
//               BasicMotionEncoder.forward, core/update.py:96); with from_coords
//               the input is coords1 and flow = coords1 - coords0 is formed here
//               (coords0 = the pixel grid, core/raft.py:63-70,126)
//   apply_delta: coords1 += delta (the flow head output, core/raft.py:131) and the
//               new low-resolution flow = coords1 - coords0 for the upsampler
#include "common.h"

namespace raft_amd {
namespace {

__global__ __launch_bounds__(256) void gru_bwd_a_kernel(const float* __restrict__ dH, long sdh,
                                                        const __bf16* __restrict__ z, long sz,
                                                        const __bf16* __restrict__ q, long sq,
                                                        const __bf16* __restrict__ h, long sh,
                                                        __bf16* __restrict__ dq, long sdq,
                                                        __bf16* __restrict__ dz, long sdz,
                                                        float* __restrict__ carry, long sc, long P,
                                                        int C) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= P * C) return;
  const long p = i / C;
  const int c = i - p * C;
  const float g = dH[p * sdh + c];
  const float zv = static_cast<float>(z[p * sz + c]);
  const float qv = static_cast<float>(q[p * sq + c]);
  const float hv = static_cast<float>(h[p * sh + c]);
  dq[p * sdq + c] = static_cast<__bf16>(g * zv * (1.f - qv * qv));
  dz[p * sdz + c] = static_cast<__bf16>(g * (qv - hv) * zv * (1.f - zv));
  carry[p * sc + c] = g * (1.f - zv);
}

__global__ __launch_bounds__(256) void gru_bwd_b_kernel(float* __restrict__ drh, long sd,
                                                        const __bf16* __restrict__ r, long sr,
                                                        const __bf16* __restrict__ h, long sh,
                                                        const float* __restrict__ carry, long sc,
                                                        __bf16* __restrict__ dr, long sdr, long P,
                                                        int C) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= P * C) return;
  const long p = i / C;
  const int c = i - p * C;
  const float g = drh[p * sd + c];
  const float rv = static_cast<float>(r[p * sr + c]);
  const float hv = static_cast<float>(h[p * sh + c]);
  dr[p * sdr + c] = static_cast<__bf16>(g * hv * rv * (1.f - rv));
  drh[p * sd + c] = carry[p * sc + c] + g * rv;
}

__global__ __launch_bounds__(256) void masked_cast_kernel(const float* __restrict__ src, long ss,
                                                          const __bf16* __restrict__ mask, long sm,
                                                          __bf16* __restrict__ out, long so, long P,
                                                          int C, int Cvalid) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= P * C) return;
  const long p = i / C;
  const int c = i - p * C;
  float v = c < Cvalid ? src[p * ss + c] : 0.f;
  if (mask && !(static_cast<float>(mask[p * sm + c]) > 0.f)) v = 0.f;
  out[p * so + c] = static_cast<__bf16>(v);
}

__global__ __launch_bounds__(256) void pack_flow_kernel(const float* __restrict__ flow,
                                                        __bf16* __restrict__ flow8,
                                                        __bf16* __restrict__ motion, long smo, int B,
                                                        int HW, int W, int from_coords) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)B * HW) return;
  const int b = p / HW;
  const int s = p - (long)b * HW;
  float u = flow[(long)b * 2 * HW + s], v = flow[(long)b * 2 * HW + HW + s];
  const bool f16 = (from_coords & 2) != 0;  // bit 1: fp16 storage (fp16 AMP)
  if (from_coords & 1) {
    const int y = s / W;
    u -= (float)(s - y * W);
    v -= (float)y;
  }
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = st16(0.f, false);
  o[0] = st16(u, f16);
  o[1] = st16(v, f16);
  *reinterpret_cast<bf16x8*>(flow8 + p * 8) = o;
  if (motion) {
    motion[p * smo] = o[0];
    motion[p * smo + 1] = o[1];
  }
}

// coords_out = coords1 + delta[:, :2]; flow_out = coords_out - grid  (both (B, 2, H, W) fp32)
__global__ __launch_bounds__(256) void apply_delta_kernel(const float* __restrict__ coords1,
                                                          const float* __restrict__ delta, long sd,
                                                          float* __restrict__ coords_out,
                                                          float* __restrict__ flow_out, int B, int HW, int W) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)B * HW) return;
  const int b = p / HW;
  const int s = p - (long)b * HW;
  const int y = s / W;
  const long i0 = (long)b * 2 * HW + s, i1 = i0 + HW;
  const float cx = coords1[i0] + delta[p * sd], cy = coords1[i1] + delta[p * sd + 1];
  coords_out[i0] = cx;
  coords_out[i1] = cy;
  flow_out[i0] = cx - (float)(s - y * W);
  flow_out[i1] = cy - (float)y;
}

// The flow head's conv2 (3x3, pad 1, 2 outputs) from the per-tap partials that the heads conv
// epilogue wrote (kernel_abi.h ConvFwdArgs::n2y: planes y[s][o * 9 + t][q] over 64-channel slots s),
// fused with apply_delta: delta[o] = bias[o] + sum_s sum_t y[s][o * 9 + t][p + off_t] (taps
// outside the image are the conv's zero padding), then coords_out / flow_out as apply_delta;
// delta itself is stored when requested (tests)
__global__ __launch_bounds__(256) void n2_apply_kernel(const float* __restrict__ y, int nslot,
                                                       const float* __restrict__ bias,
                                                       const float* __restrict__ coords1,
                                                       float* __restrict__ coords_out, float* __restrict__ flow_out,
                                                       float* __restrict__ delta, long sd, int B, int H, int W) {
  // wave w sums slot w of 64 consecutive pixels (coalesced plane rows), the 4 slot partials
  // meet in LDS: four times the waves of a thread-per-pixel form, whose single wave per
  // 64 pixels left each CU ~2 waves to hide the loads' latency
  __shared__ float part[4][2][64];
  const int HW = H * W;
  const long P = (long)B * HW;
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long p = (long)blockIdx.x * 64 + lane;
  const bool in = p < P;
  const int b = in ? (int)(p / HW) : 0;
  const int s = in ? (int)(p - (long)b * HW) : 0;
  const int py = s / W, px = s - py * W;
  float d0 = 0.f, d1 = 0.f;
  if (in && sl < nslot) {
    const float* ys = y + (long)sl * 18 * P + p;
    float v[18], keep[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {  // branch-free taps: clamped offset, zero weight outside the image
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      const bool ok = (unsigned)(py + dy) < (unsigned)H && (unsigned)(px + dx) < (unsigned)W;
      const long off = ok ? (long)dy * W + dx : 0;
      keep[t] = ok ? 1.f : 0.f;
      v[t] = ys[t * P + off];
      v[9 + t] = ys[(9 + t) * P + off];
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      d0 += keep[t] * v[t];
      d1 += keep[t] * v[9 + t];
    }
  }
  part[sl][0][lane] = d0;
  part[sl][1][lane] = d1;
  __syncthreads();
  if (sl != 0 || !in) return;
  d0 = (bias ? bias[0] : 0.f) + ((part[0][0][lane] + part[1][0][lane]) + (part[2][0][lane] + part[3][0][lane]));
  d1 = (bias ? bias[1] : 0.f) + ((part[0][1][lane] + part[1][1][lane]) + (part[2][1][lane] + part[3][1][lane]));
  if (delta) {
    delta[p * sd] = d0;
    delta[p * sd + 1] = d1;
  }
  const long i0 = (long)b * 2 * HW + s, i1 = i0 + HW;
  const float cx = coords1[i0] + d0, cy = coords1[i1] + d1;
  coords_out[i0] = cx;
  coords_out[i1] = cy;
  flow_out[i0] = cx - (float)px;
  flow_out[i1] = cy - (float)py;
}

// fp32 rows -> split-bf16 planes (kernel_abi.h ConvFwdArgs::split_g): channel c of src row p
// (zero for C <= c < Cpad) goes to output channel n = c0 + c of a group-G split row of dst
__global__ __launch_bounds__(256) void split_pack_kernel(const float* __restrict__ src, long ss, int C, int Cpad,
                                                         __bf16* __restrict__ dst, long sd, int G, int c0, long P) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= P * Cpad) return;
  const long p = i / Cpad;
  const int c = (int)(i - p * Cpad);
  const float x = c < C ? src[p * ss + c] : 0.f;
  const __bf16 hi = static_cast<__bf16>(x), lo = static_cast<__bf16>(x - static_cast<float>(hi));
  const int n = c0 + c;
  __bf16* o = dst + p * sd + (long)(n / G) * 3 * G + n % G;
  o[0] = hi;
  o[G] = lo;
  o[2 * G] = hi;
}

inline dim3 grid1(long n) { return dim3((unsigned)((n + 255) / 256)); }

// host-overhead probes (scripts/launch_probe.py): empty kernels with an 8-byte and a
// ConvFwdArgs-sized argument block
__global__ void probe_small_kernel(int* p) {
  if (p != nullptr && threadIdx.x == 1024) p[0] = 1;  // never true: an empty body the compiler keeps
}
__global__ void probe_big_kernel(const ConvFwdArgs a) {
  if (a.out != nullptr && threadIdx.x == 1024) static_cast<int*>(a.out)[0] = 1;
}

}  // namespace

hipError_t launch_probe(int kind, hipStream_t s) {
  if (kind == 0) {
    hipLaunchKernelGGL(probe_small_kernel, dim3(1), dim3(64), 0, s, nullptr);
  } else {
    ConvFwdArgs a{};
    hipLaunchKernelGGL(probe_big_kernel, dim3(1), dim3(64), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_split_pack(const float* src, long ss, int C, int Cpad, void* dst, long sd, int G, int c0, long P,
                             hipStream_t s) {
  if (P * Cpad == 0) return hipSuccess;
  hipLaunchKernelGGL(split_pack_kernel, grid1(P * Cpad), dim3(256), 0, s, src, ss, C, Cpad, static_cast<__bf16*>(dst),
                     sd, G, c0, P);
  return hipGetLastError();
}

hipError_t launch_gru_bwd_a(const float* dH, long sdh, const void* z, long sz, const void* q, long sq,
                            const void* h, long sh, void* dq, long sdq, void* dz, long sdz, float* carry,
                            long sc, long P, int C, hipStream_t s) {
  if (P * C == 0) return hipSuccess;
  hipLaunchKernelGGL(gru_bwd_a_kernel, grid1(P * C), dim3(256), 0, s, dH, sdh, (const __bf16*)z, sz,
                     (const __bf16*)q, sq, (const __bf16*)h, sh, (__bf16*)dq, sdq, (__bf16*)dz, sdz, carry,
                     sc, P, C);
  return hipGetLastError();
}

hipError_t launch_gru_bwd_b(float* drh, long sd, const void* r, long sr, const void* h, long sh,
                            const float* carry, long sc, void* dr, long sdr, long P, int C,
                            hipStream_t s) {
  if (P * C == 0) return hipSuccess;
  hipLaunchKernelGGL(gru_bwd_b_kernel, grid1(P * C), dim3(256), 0, s, drh, sd, (const __bf16*)r, sr,
                     (const __bf16*)h, sh, carry, sc, (__bf16*)dr, sdr, P, C);
  return hipGetLastError();
}

hipError_t launch_masked_cast(const float* src, long ss, const void* mask, long sm, void* out, long so,
                              long P, int C, int Cvalid, hipStream_t s) {
  if (P * C == 0) return hipSuccess;
  hipLaunchKernelGGL(masked_cast_kernel, grid1(P * C), dim3(256), 0, s, src, ss, (const __bf16*)mask, sm,
                     (__bf16*)out, so, P, C, Cvalid);
  return hipGetLastError();
}

hipError_t launch_pack_flow(const float* flow, void* flow8, void* motion, long smo, int B, int HW, int W,
                            int from_coords, hipStream_t s) {
  const long P = (long)B * HW;
  if (!P) return hipSuccess;
  hipLaunchKernelGGL(pack_flow_kernel, grid1(P), dim3(256), 0, s, flow, (__bf16*)flow8, (__bf16*)motion,
                     smo, B, HW, W, from_coords);
  return hipGetLastError();
}

hipError_t launch_apply_delta(const float* coords1, const float* delta, long sd, float* coords_out,
                              float* flow_out, int B, int HW, int W, hipStream_t s) {
  const long P = (long)B * HW;
  if (!P) return hipSuccess;
  hipLaunchKernelGGL(apply_delta_kernel, grid1(P), dim3(256), 0, s, coords1, delta, sd, coords_out, flow_out, B,
                     HW, W);
  return hipGetLastError();
}

hipError_t launch_n2_apply(const float* y, int nslot, const float* bias, const float* coords1, float* coords_out,
                           float* flow_out, float* delta, long sd, int B, int H, int W, hipStream_t s) {
  const long P = (long)B * H * W;
  if (!P) return hipSuccess;
  if (nslot > 4) return hipErrorInvalidValue;
  // 64 pixels x 4 slots per workgroup: a 1080p frame is 32,400 pixels, 507 workgroups of 4 waves
  hipLaunchKernelGGL(n2_apply_kernel, dim3((unsigned)((P + 63) / 64)), dim3(256), 0, s, y, nslot, bias, coords1,
                     coords_out, flow_out, delta, sd, B, H, W);
  return hipGetLastError();
}

}  // namespace raft_amd
