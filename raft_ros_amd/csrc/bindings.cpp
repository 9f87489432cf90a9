// Torch dispatcher registration of the raft_ros_amd native ops.
//
// The reference exposes its single native extension through pybind11
// (alt_cuda_corr/correlation.cpp:51-54, forward/backward of the on-the-fly
// correlation).  Here every native op is a TORCH_LIBRARY schema with a HIP
// implementation on the CUDA(=HIP) dispatch key, launched on the current torch
// HIP stream with error checks.  Autograd wiring lives in raft_ros_amd/ops/.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/core/DeviceGuard.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <vector>

#include <hip/hip_runtime.h>

#include "kernel_abi.h"

namespace raft_amd {


enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

// launchers (defined in the .hip translation units)
hipError_t launch_corr_gemm(const CorrGemmArgs& g, hipStream_t s);
hipError_t launch_corr_bwd_pair(const CorrGemmArgs& g1, const CorrGemmArgs& gt, hipStream_t s);
hipError_t launch_fixed_to_float(const long long* in, float* out, long n, const float* fix_scale, hipStream_t s);
hipError_t launch_local_corr_mfma(const LocalCorrArgs& a, bool backward, hipStream_t s);
bool local_corr_gather_ok(const LocalCorrArgs& a);
long local_corr_gather_scratch(const LocalCorrArgs& a);
hipError_t launch_local_corr_mfma_bwd_gather(const LocalCorrArgs& a, int* scratch, hipStream_t s);
hipError_t launch_pyramid_unpool(const UnpoolArgs& u, hipStream_t s);
hipError_t launch_pyramid_operand(const PyrOperandArgs& a, hipStream_t s);
hipError_t launch_avgpool2x2(const float* in, float* out, long rows, int H, int W, hipStream_t s);
hipError_t launch_corr_lookup_fwd(const PyrDesc& pyr, const float* coords, void* out, int out_dtype,
                                  int B, int H, int W, int r, int out_ch, hipStream_t s, void* flow8 = nullptr,
                                  void* motion = nullptr, long smo = 0, int split_m = 0);
hipError_t launch_corr_lookup_bwd(const PyrDesc& dpyr, const float* coords, const void* gout,
                                  int g_dtype, int B, int H, int W, int r, int gstride, hipStream_t s);
hipError_t launch_lookup_grad_rows(const GradRowsArgs& a, int g_dtype, hipStream_t s);
hipError_t launch_gru_bwd_a(const float* dH, long sdh, const void* z, long sz, const void* q, long sq,
                            const void* h, long sh, void* dq, long sdq, void* dz, long sdz, float* carry,
                            long sc, long P, int C, hipStream_t s);
hipError_t launch_gru_bwd_b(float* drh, long sd, const void* r, long sr, const void* h, long sh,
                            const float* carry, long sc, void* dr, long sdr, long P, int C,
                            hipStream_t s);
hipError_t launch_masked_cast(const float* src, long ss, const void* mask, long sm, void* out, long so,
                              long P, int C, int Cvalid, hipStream_t s);
hipError_t launch_split_pack(const float* src, long ss, int C, int Cpad, void* dst, long sd, int G, int c0, long P,
                             hipStream_t s);
hipError_t launch_pack_flow(const float* flow, void* flow8, void* motion, long smo, int B, int HW, int W,
                            int from_coords, hipStream_t s);
hipError_t launch_apply_delta(const float* coords1, const float* delta, long sd, float* coords_out,
                              float* flow_out, int B, int HW, int W, hipStream_t s);
hipError_t launch_probe(int kind, hipStream_t s);
hipError_t launch_n2_apply(const float* y, int nslot, const float* bias, const float* coords1, float* coords_out,
                           float* flow_out, float* delta, long sd, int B, int H, int W, hipStream_t s);
hipError_t launch_convex_up_fwd(const float* flow, const void* mask, int m_dtype, long msN, long msC,
                                long msH, long msW, float* out, int B, int H, int W, hipStream_t s);
hipError_t launch_convex_up_bwd(const float* flow, const void* mask, int m_dtype, long msN, long msC,
                                long msH, long msW, const float* gout, void* dmask, long dsN, long dsC,
                                long dsH, long dsW, float* part, float* dflow, void* rows, int rows_ld, int B,
                                int H, int W, hipStream_t s);
int seq_loss_num_blocks(long P);
hipError_t launch_seq_loss_fwd(const SeqPreds& preds, int n, const float* gt, const float* valid,
                               float gamma, float max_flow, long B, long HW, float* partial,
                               hipStream_t s);
hipError_t launch_seq_loss_bwd(const SeqPreds& preds, const SeqGrads& grads, int n, const float* gt,
                               const float* valid, const float* dloss, float gamma, float max_flow,
                               long B, long HW, hipStream_t s);
hipError_t launch_local_corr_fwd(const void* f1, const void* f2, int dtype, const float* coords,
                                 float* out, int B, int H1, int W1, int H2, int W2, int C, int r,
                                 float scale, hipStream_t s);
hipError_t launch_local_corr_bwd(const void* f1, const void* f2, int dtype, const float* coords,
                                 const float* gout, float* g1, float* g2, long long* g2fix, const float* fix_scale,
                                 int B, int H1, int W1,
                                 int H2, int W2, int C, int r, float scale, hipStream_t s);

hipError_t launch_gru_gates_fwd(int dtype, const void* zr, const void* h, void* z, void* rh, long npix,
                                int C, hipStream_t s);
hipError_t launch_gru_gates_bwd(int dtype, const void* zr, const void* h, const void* gz,
                                const void* grh, void* dzr, void* dh, long npix, int C, hipStream_t s);
hipError_t launch_gru_blend_fwd(int dtype, const void* z, const void* q, const void* h, void* out,
                                long numel, hipStream_t s);
hipError_t launch_gru_blend_bwd(int dtype, const void* z, const void* q, const void* h, const void* g,
                                void* dz, void* dq, void* dh, long numel, hipStream_t s);


int instance_norm_chunks(int HW);
hipError_t launch_instance_norm_fwd(int dtype, const void* x, void* y, float* stats, float* part, int N, int HW,
                                    int C, int relu, float eps, hipStream_t s);
hipError_t launch_instance_norm_bwd(int dtype, const void* x, const void* dy, const float* stats, float* gsum,
                                    float* part, void* dx, int N, int HW, int C, int relu, hipStream_t s);

namespace {

#define HIP_OK(expr)                                                                     \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "raft_amd HIP error: ", hipGetErrorString(_e), " at ", \
                __FILE__, ":", __LINE__);                                                  \
  } while (0)

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
void pm_any(const at::Tensor& t, const char* name, long P, at::ScalarType dt);

int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return kF32;
    case at::kBFloat16: return kBF16;
    case at::kHalf: return kF16;
    default: TORCH_CHECK(false, "raft_amd: unsupported dtype ", t);
  }
  return -1;
}

void check_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "raft_amd: ", name, " must be a GPU tensor");
}

// Pyramid levels: (rows, Hl, Wl) fp32 views with unit x stride and y stride Wl; the row
// stride may exceed Hl*Wl (padded rows, as the GEMM operands need 8-element-aligned pitches).
PyrDesc make_desc(const std::vector<at::Tensor>& levels, long rows, bool allow_bf16 = false) {
  // level views: (rows, Hl, Wl) row-major images, or (rows, Wl/16, Hl, 16) 16-column blocks
  TORCH_CHECK(levels.size() >= 1 && levels.size() <= 4, "raft_amd: 1..4 pyramid levels supported");
  PyrDesc d{};
  d.levels = static_cast<int>(levels.size());
  for (size_t l = 0; l < levels.size(); ++l) {
    const auto& t = levels[l];
    check_gpu(t, "pyramid level");
    const bool bf = t.scalar_type() == at::kBFloat16;
    const bool blk = t.dim() == 4;
    TORCH_CHECK(t.scalar_type() == at::kFloat || (allow_bf16 && bf),
                "raft_amd: pyramid levels must be fp32 (bf16: forward lookups only)");
    if (blk) {
      // (strides of size-1 dims are free: torch reports such views contiguous as they are)
      TORCH_CHECK(t.size(3) == 16 && t.stride(3) == 1 && (t.size(2) == 1 || t.stride(2) == 16) &&
                      (t.size(1) == 1 || t.stride(1) == t.size(2) * 16) && t.stride(0) >= t.size(1) * t.size(2) * 16,
                  "raft_amd: blocked pyramid levels must be (rows, W/16, H, 16) views");
    } else {
      TORCH_CHECK(t.dim() == 3 && (t.size(2) == 1 || t.stride(2) == 1) && (t.size(1) == 1 || t.stride(1) == t.size(2)) &&
                      t.stride(0) >= t.size(1) * t.size(2),
                  "raft_amd: pyramid levels must be (B*H*W, Hl, Wl) row views");
    }
    TORCH_CHECK(l == 0 || ((bf ? 1 : 0) == d.vbf16 && (blk ? 1 : 0) == d.blk),
                "raft_amd: pyramid levels must share one dtype and layout");
    d.vbf16 = bf ? 1 : 0;
    d.blk = blk ? 1 : 0;
    TORCH_CHECK(t.size(0) == rows, "raft_amd: pyramid level rows mismatch");
    const long span = blk ? t.size(1) * t.size(2) * 16 : t.size(1) * t.size(2);
    TORCH_CHECK(t.storage_offset() + (rows - 1) * t.stride(0) + span <= (long)(t.storage().nbytes() / t.element_size()),
                "raft_amd: pyramid level view exceeds its storage");
    d.ptr[l] = static_cast<float*>(t.data_ptr());
    d.H[l] = static_cast<int>(blk ? t.size(2) : t.size(1));
    d.W[l] = static_cast<int>(blk ? t.size(1) * 16 : t.size(2));
    d.ld[l] = t.stride(0);
  }
  return d;
}

// ---------------------------------------------------------------- GEMM
long elem_span(const at::Tensor& t) {  // elements addressable from data_ptr()
  return (long)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
}

// C (op)= alpha * A . B^T on the correlation-path MFMA kernel (csrc/corr_volume.hip): flat
// operands with explicit pitches, fp32/bf16 inputs (split = 3-pass bf16 for fp32 accuracy),
// transposed A, epilogues store (epi 0) / accumulate (epi 1, fp32).
void corr_gemm(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, int64_t M, int64_t N, int64_t K,
               int64_t batch, int64_t lda, int64_t sA, int64_t ldb, int64_t sB, int64_t ldc, int64_t sC, double alpha,
               bool a_trans, bool split, int64_t epi, int64_t cfg) {
  check_gpu(A, "A");
  check_gpu(B, "B");
  check_gpu(C, "C");
  auto ok_t = [](const at::Tensor& t) { return t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16; };
  TORCH_CHECK(ok_t(A) && ok_t(B) && ok_t(C), "raft_amd::corr_gemm: operands must be fp32 or bf16");
  TORCH_CHECK(epi == 0 || C.scalar_type() == at::kFloat, "raft_amd::corr_gemm: accumulating epilogues write fp32");
  TORCH_CHECK(M >= 0 && N >= 0 && K > 0 && batch >= 1 && (epi == 0 || epi == 1), "raft_amd::corr_gemm: bad sizes");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && sA % 8 == 0 && sB % 8 == 0,
              "raft_amd::corr_gemm: operand pitches must be multiples of 8 elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
              "raft_amd::corr_gemm: operands must be 16-byte aligned");
  auto r8 = [](long v) { return (v + 7) / 8 * 8; };
  // every 8-element chunk the kernel may touch lies inside the storage
  const long a_need = a_trans ? (batch - 1) * sA + (K - 1) * lda + r8(M) : (batch - 1) * sA + (M - 1) * lda + r8(K);
  const long b_need = (batch - 1) * sB + (N - 1) * ldb + r8(K);
  TORCH_CHECK(a_need <= elem_span(A), "raft_amd::corr_gemm: A too small");
  TORCH_CHECK(b_need <= elem_span(B), "raft_amd::corr_gemm: B too small");
  const long c_need = (batch - 1) * sC + (M - 1) * ldc + N;
  CorrGemmArgs g{};
  TORCH_CHECK(c_need <= elem_span(C), "raft_amd::corr_gemm: C too small");
  if (M == 0 || N == 0) return;
  g.A = A.data_ptr(); g.lda = lda; g.sA = sA;
  g.B = B.data_ptr(); g.ldb = ldb; g.sB = sB;
  g.C = C.data_ptr(); g.ldc = ldc; g.sC = sC;
  g.M = (int)M; g.N = (int)N; g.K = (int)K; g.batch = (int)batch;
  g.alpha = (float)alpha;
  g.a_f32 = A.scalar_type() == at::kFloat;
  g.b_f32 = B.scalar_type() == at::kFloat;
  g.a_trans = a_trans;
  g.split = split;
  g.c_bf16 = C.scalar_type() == at::kBFloat16;
  g.epi = (int)epi;
  g.cfg = (int)cfg;
  const c10::DeviceGuard guard(A.device());
  HIP_OK(launch_corr_gemm(g, cur_stream()));
}

// The AMP pyramid backward's two GEMMs in one launch (csrc/corr_volume.hip corr_bwd_pair_kernel):
//   d1 (B, HW, C) bf16 = alpha * dL . f2t^T      dL (B, HW, ld) bf16, f2t (B, C, ld) bf16
//   G  (B, ld, C) fp32 = alpha * dL^T . f1t^T    f1t (B, C, hp >= HW) bf16
void corr_pyramid_bwd(const at::Tensor& dL, const at::Tensor& f2t, const at::Tensor& f1t, const at::Tensor& d1,
                      const at::Tensor& G, double alpha) {
  for (const auto* t : {&dL, &f2t, &f1t, &d1, &G}) check_gpu(*t, "corr_pyramid_bwd operand");
  TORCH_CHECK(dL.scalar_type() == at::kBFloat16 && f2t.scalar_type() == at::kBFloat16 &&
                  f1t.scalar_type() == at::kBFloat16 && d1.scalar_type() == at::kBFloat16 && G.scalar_type() == at::kFloat,
              "raft_amd::corr_pyramid_bwd: bf16 dL / f2t / f1t / d1, fp32 G");
  TORCH_CHECK(f2t.dim() == 3 && f1t.dim() == 3 && d1.dim() == 3 && G.dim() == 3, "raft_amd::corr_pyramid_bwd: 3-d operands");
  for (const auto* t : {&dL, &f2t, &f1t, &d1, &G}) TORCH_CHECK(t->is_contiguous(), "raft_amd::corr_pyramid_bwd: contiguous operands");
  const long B = f2t.size(0), C = f2t.size(1), ld = f2t.size(2), HW = d1.size(1), hp = f1t.size(2);
  TORCH_CHECK(f1t.size(0) == B && f1t.size(1) == C && hp >= HW && d1.size(0) == B && d1.size(2) == C &&
                  G.size(0) == B && G.size(1) == ld && G.size(2) == C && dL.numel() == B * HW * ld,
              "raft_amd::corr_pyramid_bwd: shape mismatch");
  TORCH_CHECK(ld % 8 == 0 && hp % 8 == 0, "raft_amd::corr_pyramid_bwd: ld and the f1t pitch must be multiples of 8");
  if (B == 0 || HW == 0 || C == 0) return;
  CorrGemmArgs g1{}, gt{};
  g1.A = dL.data_ptr(); g1.lda = ld; g1.sA = HW * ld;
  g1.B = f2t.data_ptr(); g1.ldb = ld; g1.sB = C * ld;
  g1.C = d1.data_ptr(); g1.ldc = C; g1.sC = HW * C;
  g1.M = (int)HW; g1.N = (int)C; g1.K = (int)ld; g1.batch = (int)B; g1.alpha = (float)alpha; g1.c_bf16 = 1; g1.cfg = 10;
  gt.A = dL.data_ptr(); gt.lda = ld; gt.sA = HW * ld; gt.a_trans = 1;
  gt.B = f1t.data_ptr(); gt.ldb = hp; gt.sB = C * hp;
  gt.C = G.data_ptr(); gt.ldc = C; gt.sC = ld * C;
  gt.M = (int)ld; gt.N = (int)C; gt.K = (int)HW; gt.batch = (int)B; gt.alpha = (float)alpha; gt.c_bf16 = 0; gt.cfg = 10;
  const c10::DeviceGuard guard(dL.device());
  HIP_OK(launch_corr_bwd_pair(g1, gt, cur_stream()));
}

at::Tensor gemm_nt(const at::Tensor& A, const at::Tensor& B, double alpha, at::ScalarType out_dtype) {
  check_gpu(A, "A");
  check_gpu(B, "B");
  TORCH_CHECK(A.dim() == 3 && B.dim() == 3, "raft_amd::gemm_nt expects (batch, rows, K)");
  TORCH_CHECK(A.stride(2) == 1 && B.stride(2) == 1, "raft_amd::gemm_nt: K must be contiguous");
  const long batch = A.size(0), M = A.size(1), K = A.size(2), N = B.size(1);
  TORCH_CHECK(B.size(0) == batch && B.size(2) == K, "raft_amd::gemm_nt: shape mismatch");
  TORCH_CHECK(K % 8 == 0, "raft_amd::gemm_nt: K must be a multiple of 8 (got ", K, ")");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "raft_amd::gemm_nt: out dtype must be fp32 or bf16");
  auto C = at::empty({batch, M, N}, A.options().dtype(out_dtype));
  if (batch == 0 || M == 0 || N == 0) return C;
  corr_gemm(A, B, C, M, N, K, batch, A.stride(1), A.stride(0), B.stride(1), B.stride(0), N, M * N, alpha, false,
            false, 0, 0);
  return C;
}

// out (B, H*W, C) = adjoint of the pyramid pools applied to the concatenated level rows of G
// (B, ld, C); segs = [off, Hl, Wl] per level (level l pools 2^l x 2^l blocks).
at::Tensor pyramid_unpool(const at::Tensor& G, int64_t H, int64_t W, at::IntArrayRef segs, bool blocked) {
  check_gpu(G, "G");
  TORCH_CHECK(G.scalar_type() == at::kFloat && G.dim() == 3 && G.is_contiguous(),
              "raft_amd::pyramid_unpool: G must be contiguous fp32 (B, rows, C)");
  TORCH_CHECK(segs.size() % 3 == 0 && segs.size() >= 3 && segs.size() <= 12, "raft_amd::pyramid_unpool: 1..4 levels");
  UnpoolArgs u{};
  u.B = (int)G.size(0); u.C = (int)G.size(2); u.H = (int)H; u.W = (int)W;
  u.nseg = (int)(segs.size() / 3);
  u.blk = blocked ? 1 : 0;
  for (int l = 0; l < u.nseg; ++l) {
    u.off[l] = (int)segs[3 * l]; u.h[l] = (int)segs[3 * l + 1]; u.w[l] = (int)segs[3 * l + 2];
    const long span = blocked ? (long)((u.w[l] + 15) / 16) * u.h[l] * 16 : (long)u.h[l] * u.w[l];
    TORCH_CHECK(u.off[l] >= 0 && u.h[l] <= (H >> l) && u.w[l] <= (W >> l) && (long)u.off[l] + span <= G.size(1),
                "raft_amd::pyramid_unpool: level ", l, " does not fit");
  }
  u.G = G.data_ptr<float>();
  u.sG = G.stride(0);
  const c10::DeviceGuard guard(G.device());
  auto out = at::empty({G.size(0), H * W, G.size(2)}, G.options());
  u.out = out.data_ptr<float>();
  HIP_OK(launch_pyramid_unpool(u, cur_stream()));
  return out;
}

// Dense-pyramid GEMM operand straight from a feature map (B, C, H, W) of any strides, bf16 or
// fp32: levels [off, h, w] (2x2 average pools, floor), fp32 (B, ld, C) or (B, C, ld) (nchw).
at::Tensor pyramid_operand(const at::Tensor& fmap, at::IntArrayRef segs, int64_t ld, bool blocked, bool nchw,
                           bool bf16_out) {
  check_gpu(fmap, "fmap");
  TORCH_CHECK(fmap.dim() == 4 && (fmap.scalar_type() == at::kFloat || fmap.scalar_type() == at::kBFloat16),
              "raft_amd::pyramid_operand: fmap must be (B, C, H, W) fp32 or bf16");
  TORCH_CHECK(segs.size() % 3 == 0 && segs.size() >= 3 && segs.size() <= 12, "raft_amd::pyramid_operand: 1..4 levels");
  PyrOperandArgs a{};
  a.B = (int)fmap.size(0); a.C = (int)fmap.size(1); a.H = (int)fmap.size(2); a.W = (int)fmap.size(3);
  TORCH_CHECK(nchw || a.C % 4 == 0, "raft_amd::pyramid_operand: channels must be a multiple of 4");
  a.nseg = (int)(segs.size() / 3);
  a.blk = blocked ? 1 : 0;
  a.nchw = nchw ? 1 : 0;
  a.ld = ld;
  for (int l = 0; l < a.nseg; ++l) {
    a.off[l] = (int)segs[3 * l]; a.h[l] = (int)segs[3 * l + 1]; a.w[l] = (int)segs[3 * l + 2];
    const long span = blocked ? (long)((a.w[l] + 15) / 16) * a.h[l] * 16 : (long)a.h[l] * a.w[l];
    TORCH_CHECK(a.off[l] >= 0 && (l == 0 || a.off[l] >= a.off[l - 1]) && a.h[l] <= (a.H >> l) &&
                    a.w[l] <= (a.W >> l) && (long)a.off[l] + span <= ld,
                "raft_amd::pyramid_operand: level ", l, " does not fit");
  }
  a.src = fmap.data_ptr();
  a.src_bf16 = fmap.scalar_type() == at::kBFloat16 ? 1 : 0;
  a.sB = fmap.stride(0); a.sC = fmap.stride(1); a.sH = fmap.stride(2); a.sW = fmap.stride(3);
  const c10::DeviceGuard guard(fmap.device());
  const auto odt = bf16_out ? at::kBFloat16 : at::kFloat;
  auto out = nchw ? at::empty({a.B, a.C, ld}, fmap.options().dtype(odt)) : at::empty({a.B, ld, a.C}, fmap.options().dtype(odt));
  if (bf16_out) a.out16 = reinterpret_cast<__bf16*>(out.data_ptr());
  else a.out = out.data_ptr<float>();
  HIP_OK(launch_pyramid_operand(a, cur_stream()));
  return out;
}

// ---------------------------------------------------------------- pyramid
at::Tensor avgpool2x2(const at::Tensor& x) {
  check_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 3, "raft_amd::avgpool2x2 expects fp32 (R,H,W)");
  auto xc = x.contiguous();
  const c10::DeviceGuard guard(x.device());
  auto out = at::empty({x.size(0), x.size(1) / 2, x.size(2) / 2}, x.options());
  HIP_OK(launch_avgpool2x2(xc.data_ptr<float>(), out.data_ptr<float>(), x.size(0), x.size(1),
                           x.size(2), cur_stream()));
  return out;
}

void check_coords(const at::Tensor& coords) {
  check_gpu(coords, "coords");
  TORCH_CHECK(coords.scalar_type() == at::kFloat && coords.is_contiguous() && coords.dim() == 4 &&
                  coords.size(1) == 2,
              "raft_amd: coords must be contiguous fp32 (B, 2, H, W)");
}

at::Tensor corr_lookup(at::TensorList pyramid, const at::Tensor& coords, int64_t radius,
                       at::ScalarType out_dtype, int64_t out_channels) {
  check_coords(coords);
  const long B = coords.size(0), H = coords.size(2), W = coords.size(3);
  std::vector<at::Tensor> lv(pyramid.begin(), pyramid.end());
  PyrDesc d = make_desc(lv, B * H * W, true);
  const long win = (2 * radius + 1) * (2 * radius + 1);
  const c10::DeviceGuard guard(coords.device());
  const long och = out_channels > 0 ? out_channels : d.levels * win;
  TORCH_CHECK(och >= d.levels * win, "raft_amd::corr_lookup: out_channels < L*(2r+1)^2");
  auto out = at::empty({B, H, W, och}, coords.options().dtype(out_dtype));
  HIP_OK(launch_corr_lookup_fwd(d, coords.data_ptr<float>(), out.data_ptr(), dtype_code(out_dtype),
                                B, H, W, static_cast<int>(radius), static_cast<int>(och), cur_stream()));
  return out;
}

void corr_lookup_backward_(at::TensorList dpyr, const at::Tensor& coords, const at::Tensor& grad,
                           int64_t radius) {
  check_coords(coords);
  const long B = coords.size(0), H = coords.size(2), W = coords.size(3);
  std::vector<at::Tensor> lv(dpyr.begin(), dpyr.end());
  PyrDesc d = make_desc(lv, B * H * W);
  const long win = (2 * radius + 1) * (2 * radius + 1);
  check_gpu(grad, "grad");
  TORCH_CHECK(grad.dim() == 4 && grad.size(0) == B && grad.size(1) == H && grad.size(2) == W &&
                  grad.size(3) >= d.levels * win,
              "raft_amd::corr_lookup_backward_: grad must be (B, H, W, >= L*(2r+1)^2)");
  auto g = grad.contiguous();
  const c10::DeviceGuard guard(coords.device());
  HIP_OK(launch_corr_lookup_bwd(d, coords.data_ptr<float>(), g.data_ptr(),
                                dtype_code(g.scalar_type()), B, H, W, static_cast<int>(radius),
                                static_cast<int>(g.size(3)), cur_stream()));
}

// Deferred lookup backward: out (B*H*W, ld) bf16 / fp32 rows of 16-column-blocked level
// gradients (segments: off, Hl, Wl per level) from the window gradients grads[t] (B, H, W,
// >= L*(2r+1)^2) of the lookups at coords[t]; accumulate: add to out instead of overwriting.
void corr_lookup_grad_rows(const at::Tensor& out, at::TensorList coords, at::TensorList grads,
                           at::IntArrayRef segments, int64_t radius, bool accumulate) {
  TORCH_CHECK(coords.size() == grads.size() && !coords.empty() && (long)coords.size() <= kGradRowsMaxT,
              "raft_amd::corr_lookup_grad_rows: 1..32 (coords, grad) pairs");
  TORCH_CHECK(segments.size() % 3 == 0 && segments.size() >= 3 && segments.size() <= 12,
              "raft_amd::corr_lookup_grad_rows: segments = (off, Hl, Wl) per level, 1..4 levels");
  TORCH_CHECK(radius >= 0 && radius <= 6, "raft_amd::corr_lookup_grad_rows: radius <= 6");
  check_coords(coords[0]);
  const long B = coords[0].size(0), H = coords[0].size(2), W = coords[0].size(3);
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.size(0) == B * H * W &&
                  (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16),
              "raft_amd::corr_lookup_grad_rows: out must be contiguous (B*H*W, ld) fp32 / bf16");
  GradRowsArgs a{};
  a.ld = out.size(1);
  TORCH_CHECK(a.ld % 16 == 0 && a.ld <= kGradRowsMaxLd, "raft_amd::corr_lookup_grad_rows: ld");
  a.levels = (int)segments.size() / 3;
  long end = 0;
  for (int l = 0; l < a.levels; ++l) {
    a.off[l] = (int)segments[3 * l];
    a.H[l] = (int)segments[3 * l + 1];
    a.W[l] = (int)((segments[3 * l + 2] + 15) / 16 * 16);
    TORCH_CHECK(a.off[l] == end, "raft_amd::corr_lookup_grad_rows: levels must tile the row");
    end += (long)a.H[l] * a.W[l];
  }
  TORCH_CHECK(end == a.ld, "raft_amd::corr_lookup_grad_rows: levels must tile the row");
  const long win = (2 * radius + 1) * (2 * radius + 1);
  const auto gt = grads[0].scalar_type();
  a.T = (int)coords.size();
  for (int t = 0; t < a.T; ++t) {
    check_coords(coords[t]);
    const auto& g = grads[t];
    check_gpu(g, "grad");
    TORCH_CHECK(coords[t].sizes() == coords[0].sizes() && g.scalar_type() == gt && g.dim() == 4 && g.size(0) == B &&
                    g.size(1) == H && g.size(2) == W && g.size(3) >= a.levels * win && g.stride(3) == 1 &&
                    g.stride(2) == g.size(3) && g.stride(1) == W * g.size(3) && g.stride(0) == H * W * g.size(3) &&
                    g.size(3) == grads[0].size(3),
                "raft_amd::corr_lookup_grad_rows: grads must be contiguous (B, H, W, >= L*(2r+1)^2), one shape");
    a.g[t] = g.data_ptr();
    a.c[t] = coords[t].data_ptr<float>();
  }
  a.gstride = (int)grads[0].size(3);
  a.out = out.data_ptr();
  a.out_f32 = out.scalar_type() == at::kFloat;
  a.accumulate = accumulate ? 1 : 0;
  a.B = (int)B;
  a.Hq = (int)H;
  a.Wq = (int)W;
  a.r = (int)radius;
  const c10::DeviceGuard guard(out.device());
  HIP_OK(launch_lookup_grad_rows(a, dtype_code(gt), cur_stream()));
}

// fp32-mode lookup (ops/update_split.py): the window features of every level as split-bf16 rows
// [hi | lo | hi] of G >= L*(2r+1)^2 channels (zero padded) in out (P, >= 3G) bf16, from the fp32
// pyramid; optionally the step's split flow operand: flow8 (P, 24) rows and the 2 flow channels
// of the motion features (motion: a view starting at the flow's hi channel, lo plane G_m after)
void corr_lookup_split_into(at::TensorList pyramid, const at::Tensor& coords, int64_t radius, const at::Tensor& out,
                            int64_t G, const c10::optional<at::Tensor>& flow8, const c10::optional<at::Tensor>& motion,
                            int64_t G_m) {
  check_coords(coords);
  const long B = coords.size(0), H = coords.size(2), W = coords.size(3);
  std::vector<at::Tensor> lv(pyramid.begin(), pyramid.end());
  PyrDesc d = make_desc(lv, B * H * W, false);
  const long win = (2 * radius + 1) * (2 * radius + 1);
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.scalar_type() == at::kBFloat16 && out.size(0) == B * H * W &&
                  out.size(1) == 3 * G && G >= d.levels * win,
              "raft_amd::corr_lookup_split_into: out must be contiguous bf16 (P, 3G), G >= L*(2r+1)^2");
  void* f8 = nullptr;
  void* mo = nullptr;
  long smo = 0;
  if (flow8) {
    TORCH_CHECK(flow8->is_contiguous() && flow8->scalar_type() == at::kBFloat16 && flow8->numel() == B * H * W * 24,
                "raft_amd::corr_lookup_split_into: flow8 must be contiguous bf16 (P, 24) split rows");
    f8 = flow8->data_ptr();
    if (motion) {
      pm_any(*motion, "motion", B * H * W, at::kBFloat16);
      TORCH_CHECK(G_m > 0 && motion->size(1) >= 2 * G_m + 2, "raft_amd::corr_lookup_split_into: motion split slice");
      mo = motion->data_ptr();
      smo = motion->stride(0);
    }
  }
  const c10::DeviceGuard guard(coords.device());
  HIP_OK(launch_corr_lookup_fwd(d, coords.data_ptr<float>(), out.data_ptr(), 3, B, H, W, static_cast<int>(radius),
                                static_cast<int>(G), cur_stream(), f8, mo, smo, static_cast<int>(G_m)));
}

// ---------------------------------------------------------------- convex upsampling
void check_up_inputs(const at::Tensor& flow, const at::Tensor& mask) {
  check_gpu(flow, "flow");
  check_gpu(mask, "mask");
  TORCH_CHECK(flow.scalar_type() == at::kFloat && flow.is_contiguous() && flow.dim() == 4 &&
                  flow.size(1) == 2,
              "raft_amd::convex_upsample: flow must be contiguous fp32 (B, 2, H, W)");
  TORCH_CHECK(mask.dim() == 4 && mask.size(0) == flow.size(0) && mask.size(1) == 576 &&
                  mask.size(2) == flow.size(2) && mask.size(3) == flow.size(3),
              "raft_amd::convex_upsample: mask must be (B, 576, H, W)");
}

at::Tensor convex_upsample(const at::Tensor& flow, const at::Tensor& mask) {
  check_up_inputs(flow, mask);
  const long B = flow.size(0), H = flow.size(2), W = flow.size(3);
  const c10::DeviceGuard guard(flow.device());
  auto out = at::empty({B, 2, 8 * H, 8 * W}, flow.options());
  HIP_OK(launch_convex_up_fwd(flow.data_ptr<float>(), mask.data_ptr(), dtype_code(mask.scalar_type()),
                              mask.stride(0), mask.stride(1), mask.stride(2), mask.stride(3),
                              out.data_ptr<float>(), B, H, W, cur_stream()));
  return out;
}

std::tuple<at::Tensor, at::Tensor> convex_upsample_backward(const at::Tensor& flow,
                                                            const at::Tensor& mask,
                                                            const at::Tensor& grad) {
  check_up_inputs(flow, mask);
  const long B = flow.size(0), H = flow.size(2), W = flow.size(3);
  TORCH_CHECK(grad.dim() == 4 && grad.size(0) == B && grad.size(1) == 2 && grad.size(2) == 8 * H &&
                  grad.size(3) == 8 * W,
              "raft_amd::convex_upsample_backward: bad grad shape");
  auto g = grad.to(at::kFloat).contiguous();
  const c10::DeviceGuard guard(flow.device());
  auto dmask = at::empty_strided(mask.sizes(), mask.strides(), mask.options());
  auto part = at::empty({B, 18, H, W}, flow.options());
  auto dflow = at::empty_like(flow);
  HIP_OK(launch_convex_up_bwd(flow.data_ptr<float>(), mask.data_ptr(), dtype_code(mask.scalar_type()),
                              mask.stride(0), mask.stride(1), mask.stride(2), mask.stride(3),
                              g.data_ptr<float>(), dmask.data_ptr(), dmask.stride(0), dmask.stride(1),
                              dmask.stride(2), dmask.stride(3), part.data_ptr<float>(), dflow.data_ptr<float>(),
                              nullptr, 0, B, H, W, cur_stream()));
  return {dflow, dmask};
}

// Fused update block: dmask into a caller buffer (any strides, mask dtype) and the low-res
// flow gradient as bf16 rows [du, dv, 0..] of a (P, ld) buffer (the flow head's dY).
void convex_upsample_backward_into(const at::Tensor& flow, const at::Tensor& mask, const at::Tensor& grad,
                                   const at::Tensor& dmask, const at::Tensor& rows) {
  check_up_inputs(flow, mask);
  const long B = flow.size(0), H = flow.size(2), W = flow.size(3);
  TORCH_CHECK(grad.dim() == 4 && grad.size(0) == B && grad.size(1) == 2 && grad.size(2) == 8 * H &&
                  grad.size(3) == 8 * W,
              "raft_amd::convex_upsample_backward_into: bad grad shape");
  TORCH_CHECK(dmask.sizes() == mask.sizes() && dmask.scalar_type() == mask.scalar_type(),
              "raft_amd::convex_upsample_backward_into: dmask must match mask");
  pm_any(rows, "rows", B * H * W, mask.scalar_type() == at::kHalf ? at::kHalf : at::kBFloat16);
  TORCH_CHECK(rows.size(1) >= 2, "raft_amd::convex_upsample_backward_into: rows need >= 2 channels");
  auto g = grad.to(at::kFloat).contiguous();
  const c10::DeviceGuard guard(flow.device());
  auto part = at::empty({B, 18, H, W}, flow.options());
  HIP_OK(launch_convex_up_bwd(flow.data_ptr<float>(), mask.data_ptr(), dtype_code(mask.scalar_type()),
                              mask.stride(0), mask.stride(1), mask.stride(2), mask.stride(3),
                              g.data_ptr<float>(), dmask.data_ptr(), dmask.stride(0), dmask.stride(1),
                              dmask.stride(2), dmask.stride(3), part.data_ptr<float>(), nullptr, rows.data_ptr(),
                              (int)rows.stride(0), B, H, W, cur_stream()));
}

// ---------------------------------------------------------------- fused sequence loss
SeqPreds check_seq_inputs(const std::vector<at::Tensor>& preds, const at::Tensor& gt,
                          const at::Tensor& valid) {
  TORCH_CHECK(!preds.empty() && preds.size() <= (size_t)kMaxPreds,
              "raft_amd::seq_loss: 1..32 predictions supported");
  check_gpu(gt, "flow_gt");
  check_gpu(valid, "valid");
  TORCH_CHECK(gt.scalar_type() == at::kFloat && gt.is_contiguous() && gt.dim() == 4 && gt.size(1) == 2,
              "raft_amd::seq_loss: flow_gt must be contiguous fp32 (B, 2, H, W)");
  TORCH_CHECK(valid.scalar_type() == at::kFloat && valid.is_contiguous() && valid.dim() == 3 &&
                  valid.size(0) == gt.size(0) && valid.size(1) == gt.size(2) &&
                  valid.size(2) == gt.size(3),
              "raft_amd::seq_loss: valid must be contiguous fp32 (B, H, W)");
  SeqPreds d{};
  for (size_t i = 0; i < preds.size(); ++i) {
    const auto& p = preds[i];
    check_gpu(p, "flow prediction");
    TORCH_CHECK(p.scalar_type() == at::kFloat && p.is_contiguous() && p.sizes() == gt.sizes(),
                "raft_amd::seq_loss: predictions must be contiguous fp32 shaped like flow_gt");
    d.p[i] = p.data_ptr<float>();
  }
  return d;
}

// -> (6,) fp32: {sum_i w_i * sum(vmask*|p_i-gt|), sum epe, #<1px, #<3px, #<5px, #valid}
at::Tensor seq_loss(const std::vector<at::Tensor>& preds, const at::Tensor& gt, const at::Tensor& valid,
                    double gamma, double max_flow) {
  SeqPreds d = check_seq_inputs(preds, gt, valid);
  const c10::DeviceGuard guard(gt.device());
  const long B = gt.size(0), HW = gt.size(2) * gt.size(3);
  auto partial = at::empty({seq_loss_num_blocks(B * HW), 6}, gt.options());
  HIP_OK(launch_seq_loss_fwd(d, (int)preds.size(), gt.data_ptr<float>(), valid.data_ptr<float>(),
                             (float)gamma, (float)max_flow, B, HW, partial.data_ptr<float>(),
                             cur_stream()));
  return partial.sum(0);
}

std::vector<at::Tensor> seq_loss_backward(const std::vector<at::Tensor>& preds, const at::Tensor& gt,
                                          const at::Tensor& valid, const at::Tensor& dloss, double gamma,
                                          double max_flow) {
  SeqPreds d = check_seq_inputs(preds, gt, valid);
  TORCH_CHECK(dloss.is_cuda() && dloss.scalar_type() == at::kFloat && dloss.numel() == 1,
              "raft_amd::seq_loss_backward: dloss must be a one-element fp32 GPU tensor");
  const c10::DeviceGuard guard(gt.device());
  const long B = gt.size(0), HW = gt.size(2) * gt.size(3);
  auto dl = dloss.contiguous();
  std::vector<at::Tensor> grads;
  SeqGrads g{};
  for (size_t i = 0; i < preds.size(); ++i) {
    grads.push_back(at::empty_like(gt));
    g.g[i] = grads.back().data_ptr<float>();
  }
  HIP_OK(launch_seq_loss_bwd(d, g, (int)preds.size(), gt.data_ptr<float>(), valid.data_ptr<float>(),
                             dl.data_ptr<float>(), (float)gamma, (float)max_flow, B, HW, cur_stream()));
  return grads;
}

// ---------------------------------------------------------------- local (alternate) correlation
void check_local(const at::Tensor& f1, const at::Tensor& f2, const at::Tensor& coords) {
  check_gpu(f1, "fmap1");
  check_gpu(f2, "fmap2");
  check_coords(coords);
  TORCH_CHECK(f1.dim() == 4 && f2.dim() == 4 && f1.is_contiguous() && f2.is_contiguous(),
              "raft_amd::local_corr: fmaps must be contiguous NHWC (B, H, W, C)");
  TORCH_CHECK(f1.scalar_type() == f2.scalar_type(), "raft_amd::local_corr: fmap dtypes differ");
  TORCH_CHECK(f1.size(0) == f2.size(0) && f1.size(3) == f2.size(3), "raft_amd::local_corr: shape mismatch");
  TORCH_CHECK(f1.size(3) % 8 == 0, "raft_amd::local_corr: C must be a multiple of 8");
  TORCH_CHECK(coords.size(0) == f1.size(0) && coords.size(2) == f1.size(1) &&
                  coords.size(3) == f1.size(2),
              "raft_amd::local_corr: coords must be (B, 2, H1, W1)");
}

at::Tensor local_corr(const at::Tensor& f1, const at::Tensor& f2, const at::Tensor& coords,
                      int64_t radius, double scale) {
  check_local(f1, f2, coords);
  const long B = f1.size(0), H1 = f1.size(1), W1 = f1.size(2), C = f1.size(3);
  const long H2 = f2.size(1), W2 = f2.size(2);
  const long rd = 2 * radius + 1;
  const c10::DeviceGuard guard(f1.device());
  auto out = at::empty({B, H1, W1, rd * rd}, f1.options().dtype(at::kFloat));
  HIP_OK(launch_local_corr_fwd(f1.data_ptr(), f2.data_ptr(), dtype_code(f1.scalar_type()),
                               coords.data_ptr<float>(), out.data_ptr<float>(), B, H1, W1, H2, W2, C,
                               static_cast<int>(radius), static_cast<float>(scale), cur_stream()));
  return out;
}

// Per-tensor scale of the deterministic fixed-point gradient accumulators (common.h
// fixed_atomic_add): the power of two that maps the largest possible accumulated value,
// nterms * max|g| * max|f1| * |scale|, to 2^62.  A device scalar, computed without a host
// sync (reductions are deterministic, so the scale is too).
at::Tensor fixed_point_scale(const at::Tensor& g, const at::Tensor& f1, double scale, double nterms) {
  auto bound = g.abs().amax().to(at::kFloat) * f1.abs().amax().to(at::kFloat) *
               static_cast<float>(std::abs(scale) * nterms);
  auto e = at::floor(62.0 - at::log2(bound.clamp_min(1e-30f))).clamp(-60.0, 120.0);
  return at::exp2(e).reshape({1}).contiguous();
}

std::tuple<at::Tensor, at::Tensor> local_corr_backward(const at::Tensor& f1, const at::Tensor& f2,
                                                       const at::Tensor& coords,
                                                       const at::Tensor& grad, int64_t radius,
                                                       double scale, bool deterministic) {
  check_local(f1, f2, coords);
  const long B = f1.size(0), H1 = f1.size(1), W1 = f1.size(2), C = f1.size(3);
  const long H2 = f2.size(1), W2 = f2.size(2);
  auto g = grad.to(at::kFloat).contiguous();
  const long rd = 2 * radius + 1;
  TORCH_CHECK(g.dim() == 4 && g.size(0) == B && g.size(1) == H1 && g.size(2) == W1 && g.size(3) == rd * rd,
              "raft_amd::local_corr_backward: bad grad shape");
  const c10::DeviceGuard guard(f1.device());
  auto g1 = at::empty({B, H1, W1, C}, f1.options().dtype(at::kFloat));
  auto g2 = at::zeros({B, H2, W2, C}, f1.options().dtype(at::kFloat));
  at::Tensor fix = deterministic ? at::zeros({B, H2, W2, C}, f1.options().dtype(at::kLong)) : at::Tensor();
  long long* fp = deterministic ? reinterpret_cast<long long*>(fix.data_ptr<int64_t>()) : nullptr;
  // the accumulator bound must hold for ANY coordinates: lookups follow the predicted flow, so a
  // converging / zooming-out flow can send every query of an image onto one f2 pixel, each
  // through up to 4 (2r+2)^2 window corners.  With the 2^62 target that still leaves >= 2^40
  // fixed-point steps below the magnitude of a typical pixel's sum.
  const double nq = (double)(H1 * W1);
  at::Tensor fs = deterministic ? fixed_point_scale(g, f1, scale, nq * 4.0 * (rd + 1) * (rd + 1)) : at::Tensor();
  HIP_OK(launch_local_corr_bwd(f1.data_ptr(), f2.data_ptr(), dtype_code(f1.scalar_type()),
                               coords.data_ptr<float>(), g.data_ptr<float>(), g1.data_ptr<float>(),
                               g2.data_ptr<float>(), fp, deterministic ? fs.data_ptr<float>() : nullptr, B, H1, W1,
                               H2, W2, C, static_cast<int>(radius), static_cast<float>(scale), cur_stream()));
  if (deterministic)
    HIP_OK(launch_fixed_to_float(fp, g2.data_ptr<float>(), g2.numel(), fs.data_ptr<float>(), cur_stream()));
  return {g1, g2};
}

// ---------------------------------------------------------------- local correlation on MFMA
// f1 (P, C) bf16 query rows; f2 (B, R, C) bf16 concatenated pooled fmap2 levels with
// segs = [off, h, w] per level; coords (B, 2, H, W).
// max_c: 256 for the backward (dF1 tile in registers); the forward also takes the 3C-channel
// split-bf16 operands ([hi | lo | hi] . [hi | hi | lo], fp32-faithful inference)
LocalCorrArgs local_mfma_args(const at::Tensor& f1, const at::Tensor& f2, const at::Tensor& coords,
                              at::IntArrayRef segs, int64_t radius, double scale, long max_c = 256) {
  check_gpu(f1, "fmap1");
  check_gpu(f2, "fmap2");
  check_coords(coords);
  TORCH_CHECK(f1.scalar_type() == at::kBFloat16 && f2.scalar_type() == at::kBFloat16 && f1.dim() == 2 &&
                  f2.dim() == 3 && f1.is_contiguous() && f2.is_contiguous(),
              "raft_amd::local_corr_mfma: fmap1 (P, C) and fmap2 (B, R, C) must be contiguous bf16");
  const long B = coords.size(0), H = coords.size(2), W = coords.size(3), C = f1.size(1);
  TORCH_CHECK(f1.size(0) == B * H * W && f2.size(0) == B && f2.size(2) == C && C % 64 == 0 && C <= max_c,
              "raft_amd::local_corr_mfma: shape mismatch (C must be a multiple of 64, <= ", max_c, ")");
  TORCH_CHECK(radius >= 1 && radius <= 4, "raft_amd::local_corr_mfma: radius 1..4");
  TORCH_CHECK(segs.size() % 3 == 0 && segs.size() >= 3 && segs.size() <= 12, "raft_amd::local_corr_mfma: 1..4 levels");
  LocalCorrArgs a{};
  a.levels = (int)(segs.size() / 3);
  for (int l = 0; l < a.levels; ++l) {
    a.off[l] = (int)segs[3 * l]; a.h[l] = (int)segs[3 * l + 1]; a.w[l] = (int)segs[3 * l + 2];
    TORCH_CHECK(a.off[l] >= 0 && a.h[l] > 0 && a.w[l] > 0 && (long)a.off[l] + (long)a.h[l] * a.w[l] <= f2.size(1),
                "raft_amd::local_corr_mfma: level ", l, " exceeds fmap2");
  }
  a.f1 = static_cast<const __bf16*>(f1.data_ptr()); a.f2 = static_cast<const __bf16*>(f2.data_ptr()); a.f2_bstride = f2.stride(0);
  a.coords = coords.data_ptr<float>();
  a.B = (int)B; a.H = (int)H; a.W = (int)W; a.C = (int)C; a.r = (int)radius;
  a.scale = (float)scale;
  return a;
}

void local_corr_mfma(const at::Tensor& f1, const at::Tensor& f2, const at::Tensor& coords, at::IntArrayRef segs,
                     int64_t radius, double scale, const at::Tensor& out) {
  LocalCorrArgs a = local_mfma_args(f1, f2, coords, segs, radius, scale, 768);
  const long win = (2 * radius + 1) * (2 * radius + 1);
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(0) == f1.size(0) && out.size(1) >= a.levels * win &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "raft_amd::local_corr_mfma: out must be a (P, >= L*(2r+1)^2) bf16/fp32 row view");
  a.out = out.data_ptr(); a.ostride = out.stride(0); a.out_f32 = out.scalar_type() == at::kFloat;
  a.out_ch = (int)out.size(1);
  const c10::DeviceGuard guard(f1.device());
  HIP_OK(launch_local_corr_mfma(a, false, cur_stream()));
}

void local_corr_mfma_backward(const at::Tensor& f1, const at::Tensor& f2, const at::Tensor& coords,
                              at::IntArrayRef segs, int64_t radius, double scale, const at::Tensor& gout,
                              const at::Tensor& g1, const at::Tensor& g2, bool deterministic) {
  LocalCorrArgs a = local_mfma_args(f1, f2, coords, segs, radius, scale);
  const long win = (2 * radius + 1) * (2 * radius + 1);
  check_gpu(gout, "gout");
  TORCH_CHECK(gout.dim() == 2 && gout.stride(1) == 1 && gout.size(0) == f1.size(0) && gout.size(1) >= a.levels * win &&
                  (gout.scalar_type() == at::kBFloat16 || gout.scalar_type() == at::kFloat),
              "raft_amd::local_corr_mfma_backward: gout must be a (P, >= L*(2r+1)^2) row view");
  TORCH_CHECK(g1.scalar_type() == at::kFloat && g1.sizes() == f1.sizes() && g1.is_contiguous(),
              "raft_amd::local_corr_mfma_backward: g1 must be contiguous fp32 like fmap1");
  TORCH_CHECK(g2.scalar_type() == at::kFloat && g2.sizes() == f2.sizes() && g2.is_contiguous(),
              "raft_amd::local_corr_mfma_backward: g2 must be contiguous fp32 like fmap2 (accumulated)");
  a.gout = gout.data_ptr(); a.gstride = gout.stride(0); a.gout_bf16 = gout.scalar_type() == at::kBFloat16;
  a.g1 = g1.data_ptr<float>(); a.g2 = g2.data_ptr<float>();
  const c10::DeviceGuard guard(f1.device());
  // deterministic: 32.32 fixed-point integer atomics (order-independent), then added into g2
  at::Tensor fix = deterministic ? at::zeros(g2.sizes(), g2.options().dtype(at::kLong)) : at::Tensor();
  a.g2fix = deterministic ? reinterpret_cast<long long*>(fix.data_ptr<int64_t>()) : nullptr;
  at::Tensor fs;
  if (deterministic) {
    // worst case over any coordinates (see local_corr_backward): every query of an image on one
    // pooled-f2 pixel, through up to 4 (2r+2)^2 window corners of each of the L levels
    fs = fixed_point_scale(gout, f1, scale,
                           (double)a.H * a.W * a.levels * 4.0 * (2 * radius + 2) * (2 * radius + 2));
    a.fix_scale = fs.data_ptr<float>();
  }
  static const bool gather_env = [] {
    const char* e = std::getenv("RAFT_LC_GATHER");  // 0: the round-4 window-atomic backward (A/B)
    return !(e && e[0] == '0');
  }();
  if (!deterministic && gather_env && local_corr_gather_ok(a)) {
    // dF2 by binning the queries per 8 x 8 level block and gathering (local_corr_mfma.hip):
    // plain stores instead of ~0.4 GB of overlapping window atomics per lookup at KITTI size
    at::Tensor scratch = at::empty({local_corr_gather_scratch(a)}, g2.options().dtype(at::kInt));
    HIP_OK(launch_local_corr_mfma_bwd_gather(a, scratch.data_ptr<int>(), cur_stream()));
    return;
  }
  HIP_OK(launch_local_corr_mfma(a, true, cur_stream()));
  if (deterministic) HIP_OK(launch_fixed_to_float(a.g2fix, a.g2, g2.numel(), a.fix_scale, cur_stream()));
}

// ---------------------------------------------------------------- fused GRU gates
void check_cl(const at::Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast),
              "raft_amd gru: ", name, " must be a channels-last contiguous 4-D tensor");
}

at::Tensor empty_cl(at::IntArrayRef sizes, const at::TensorOptions& o) {
  return at::empty(sizes, o.memory_format(at::MemoryFormat::ChannelsLast));
}

std::tuple<at::Tensor, at::Tensor> gru_gates(const at::Tensor& zr, const at::Tensor& h) {
  check_cl(zr, "zr");
  check_cl(h, "h");
  TORCH_CHECK(zr.scalar_type() == h.scalar_type(), "raft_amd gru_gates: dtype mismatch");
  const long C = h.size(1);
  TORCH_CHECK(zr.size(1) == 2 * C && zr.size(0) == h.size(0) && zr.size(2) == h.size(2) &&
                  zr.size(3) == h.size(3),
              "raft_amd gru_gates: zr must be (B, 2C, H, W) for h (B, C, H, W)");
  const c10::DeviceGuard guard(h.device());
  auto z = empty_cl(h.sizes(), h.options());
  auto rh = empty_cl(h.sizes(), h.options());
  HIP_OK(launch_gru_gates_fwd(dtype_code(h.scalar_type()), zr.data_ptr(), h.data_ptr(), z.data_ptr(),
                              rh.data_ptr(), h.size(0) * h.size(2) * h.size(3), C, cur_stream()));
  return {z, rh};
}

std::tuple<at::Tensor, at::Tensor> gru_gates_backward(const at::Tensor& zr, const at::Tensor& h,
                                                      const at::Tensor& gz, const at::Tensor& grh) {
  check_cl(zr, "zr");
  check_cl(h, "h");
  auto gzc = gz.to(h.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  auto grc = grh.to(h.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  const c10::DeviceGuard guard(h.device());
  auto dzr = empty_cl(zr.sizes(), zr.options());
  auto dh = empty_cl(h.sizes(), h.options());
  HIP_OK(launch_gru_gates_bwd(dtype_code(h.scalar_type()), zr.data_ptr(), h.data_ptr(), gzc.data_ptr(),
                              grc.data_ptr(), dzr.data_ptr(), dh.data_ptr(),
                              h.size(0) * h.size(2) * h.size(3), h.size(1), cur_stream()));
  return {dzr, dh};
}

at::Tensor gru_blend(const at::Tensor& z, const at::Tensor& q, const at::Tensor& h) {
  check_cl(z, "z");
  check_cl(q, "q");
  check_cl(h, "h");
  TORCH_CHECK(z.sizes() == q.sizes() && z.sizes() == h.sizes(), "raft_amd gru_blend: shape mismatch");
  TORCH_CHECK(z.scalar_type() == q.scalar_type() && z.scalar_type() == h.scalar_type(),
              "raft_amd gru_blend: dtype mismatch");
  const c10::DeviceGuard guard(h.device());
  auto out = empty_cl(h.sizes(), h.options());
  HIP_OK(launch_gru_blend_fwd(dtype_code(h.scalar_type()), z.data_ptr(), q.data_ptr(), h.data_ptr(),
                              out.data_ptr(), h.numel(), cur_stream()));
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> gru_blend_backward(const at::Tensor& z,
                                                                  const at::Tensor& q,
                                                                  const at::Tensor& h,
                                                                  const at::Tensor& g) {
  check_cl(z, "z");
  check_cl(q, "q");
  check_cl(h, "h");
  auto gc = g.to(h.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  const c10::DeviceGuard guard(h.device());
  auto dz = empty_cl(h.sizes(), h.options());
  auto dq = empty_cl(h.sizes(), h.options());
  auto dh = empty_cl(h.sizes(), h.options());
  HIP_OK(launch_gru_blend_bwd(dtype_code(h.scalar_type()), z.data_ptr(), q.data_ptr(), h.data_ptr(),
                              gc.data_ptr(), dz.data_ptr(), dq.data_ptr(), dh.data_ptr(), h.numel(),
                              cur_stream()));
  return {dz, dq, dh};
}

// ---------------------------------------------------------------- implicit-GEMM convs
// Pixel-major operands are 2-D (P, C) views: stride(1) == 1, stride(0) = pixel stride.
void check_pm(const at::Tensor& t, const char* name, long P) {
  check_gpu(t, name);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.size(0) == P,
              "raft_amd conv: ", name, " must be a (P, C) pixel-major view with unit channel stride");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "raft_amd conv: ", name, " needs 16-byte aligned pixel rows");
}

// Sources of a conv: (rows, C) pixel-major views.  rows == P, or (weight gradient only) a
// divisor of P: a periodic source whose row p % rows is read for pixel p.
// 16-bit operand dtype of a conv launch: bf16, or fp16 (fp16 AMP) -> ConvFwdArgs::f16
bool is_half16(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, "raft_amd conv: ", what,
              " must be bf16 or fp16");
  return t.scalar_type() == at::kHalf;
}

int fill_srcs(at::TensorList srcs, long P, ConvSrc* out, bool allow_period) {
  TORCH_CHECK(srcs.size() >= 1 && srcs.size() <= 3, "raft_amd conv: 1..3 input sources");
  int Cin = 0;
  for (int i = 0; i < 3; ++i) out[i] = ConvSrc{nullptr, 0, 0, 0};
  for (size_t i = 0; i < srcs.size(); ++i) {
    const long rows = srcs[i].size(0);
    const bool periodic = allow_period && rows != P && rows > 0 && P % rows == 0;
    check_pm(srcs[i], "src", periodic ? rows : P);
    TORCH_CHECK(srcs[i].scalar_type() == srcs[0].scalar_type() && (srcs[i].scalar_type() == at::kBFloat16 ||
                                                                   srcs[i].scalar_type() == at::kHalf),
                "raft_amd conv: sources must share one 16-bit dtype (bf16, or fp16 for fp16 AMP)");
    TORCH_CHECK(srcs[i].size(1) % 8 == 0, "raft_amd conv: source channels must be multiples of 8");
    out[i] = ConvSrc{static_cast<const __bf16*>(srcs[i].data_ptr()), srcs[i].stride(0), static_cast<int>(srcs[i].size(1)),
                     periodic ? static_cast<int>(rows) : 0};
    Cin += static_cast<int>(srcs[i].size(1));
  }
  return Cin;
}

void conv_fwd(at::TensorList srcs, const at::Tensor& wt, at::IntArrayRef geom, int64_t N, const c10::optional<at::Tensor>& bias,
              int64_t epi, int64_t act, double alpha, const at::Tensor& out, int64_t acc_c0,
              const c10::optional<at::Tensor>& mask, const c10::optional<at::Tensor>& h,
              const c10::optional<at::Tensor>& z, const c10::optional<at::Tensor>& out2, int64_t cfg,
              const c10::optional<at::Tensor>& g0, const c10::optional<at::Tensor>& carry,
              const c10::optional<at::Tensor>& out3, int64_t gru_cols, const c10::optional<at::Tensor>& addsrc,
              const c10::optional<at::Tensor>& cout, const c10::optional<at::Tensor>& cmask, int64_t cm_c0,
              int64_t cm_valid, at::IntArrayRef split, const c10::optional<at::Tensor>& n2w,
              const c10::optional<at::Tensor>& n2y) {
  TORCH_CHECK(geom.size() == 7, "raft_amd conv_fwd: geom = (B, H, W, KH, KW, PH, PW)");
  ConvFwdArgs a{};
  if (!split.empty()) {
    // split-bf16 epilogues (kernel_abi.h ConvFwdArgs::split_g): [G_out, G_out2, S_h, S_z] and, for
    // the fp32-training backward, [.., S_g0, G_out3, S_add, G_cout]
    TORCH_CHECK((split.size() == 4 || split.size() == 8) && epi >= 0 && epi <= 6,
                "raft_amd conv_fwd: split = [G_out, G_out2, S_h, S_z(, S_g0, G_out3, S_add, G_cout)]");
    for (size_t i = 0; i < split.size(); ++i)
      TORCH_CHECK(split[i] >= 0 && split[i] % 8 == 0, "raft_amd conv_fwd: split entries are multiples of 8");
    a.split_g = (int)split[0];
    a.split_g2 = (int)split[1];
    a.split_h = (int)split[2];
    a.split_z = (int)split[3];
    if (split.size() == 8) {
      a.split_g0 = (int)split[4];
      a.split_g3 = (int)split[5];
      a.split_add = (int)split[6];
      a.split_cout = (int)split[7];
    }
    TORCH_CHECK((epi != 0 && epi != 2 && epi != 3) || a.split_g > 0, "raft_amd conv_fwd: split store needs G_out");
    TORCH_CHECK(epi != 1 || acc_c0 >= N, "raft_amd conv_fwd: a split gradient store does not accumulate");
    TORCH_CHECK(epi < 4 || a.split_g == 0, "raft_amd conv_fwd: GRU backward epilogues write fp32 out");
    TORCH_CHECK(epi != 2 || (a.split_g2 > 0 && a.split_h > 0), "raft_amd conv_fwd: split z||r needs G_out2 and S_h");
    TORCH_CHECK(epi != 3 || (a.split_h > 0 && a.split_z > 0), "raft_amd conv_fwd: split blend needs S_h and S_z");
  }
  a.B = geom[0]; a.H = geom[1]; a.W = geom[2]; a.KH = geom[3]; a.KW = geom[4]; a.PH = geom[5]; a.PW = geom[6];
  a.P = (long)a.B * a.H * a.W;
  a.nsrc = static_cast<int>(srcs.size());
  a.Cin = fill_srcs(srcs, a.P, a.src, false);
  a.K = a.KH * a.KW * a.Cin;
  a.cfg = static_cast<int>(cfg);
  a.f16 = is_half16(srcs[0], "sources") ? 1 : 0;
  const at::ScalarType dt16 = srcs[0].scalar_type();
  TORCH_CHECK(!a.f16 || split.empty(), "raft_amd conv_fwd: split-bf16 planes are bf16");
  check_gpu(wt, "wt");
  TORCH_CHECK(wt.scalar_type() == dt16 && wt.dim() == 2 && wt.is_contiguous() && wt.size(0) >= N &&
                  wt.size(1) >= a.K && wt.size(1) % 64 == 0,
              "raft_amd conv_fwd: wt must be contiguous bf16 [>=N][Kpad], Kpad % 64 == 0, Kpad >= K (", a.K, ")");
  a.Kpad = static_cast<int>(wt.size(1));
  a.wt = static_cast<const __bf16*>(wt.data_ptr());
  a.N = static_cast<int>(N);
  a.epi = static_cast<int>(epi);
  a.act = static_cast<int>(act);
  a.alpha = static_cast<float>(alpha);
  a.acc_c0 = static_cast<int>(acc_c0);
  if (bias) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() >= N,
                "raft_amd conv_fwd: bias must be contiguous fp32 [N]");
    a.bias = bias->data_ptr<float>();
  }
  check_pm(out, "out", a.P);
  TORCH_CHECK(out.size(1) >= N, "raft_amd conv_fwd: out has too few channels");
  a.out = out.data_ptr();
  a.out_stride = out.stride(0);
  a.out_f32 = out.scalar_type() == at::kFloat;
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == dt16,
              "raft_amd conv_fwd: out must be fp32 or the sources' 16-bit dtype");
  // 16-bit epilogue operands share the sources' dtype
  for (const auto* t : {&mask, &h, &z, &out2, &g0, &out3, &addsrc, &cout, &cmask})
    if (t->has_value()) TORCH_CHECK((*t)->scalar_type() == dt16, "raft_amd conv_fwd: epilogue operands must be ",
                                    dt16 == at::kHalf ? "fp16" : "bf16", " like the sources");
  if (epi == 2 || epi == 3) TORCH_CHECK(!a.out_f32, "raft_amd conv_fwd: GRU epilogues write bf16");
  if (mask) {
    check_pm(*mask, "mask", a.P);
    a.mask = static_cast<const __bf16*>(mask->data_ptr());
    a.mask_stride = mask->stride(0);
  }
  if (h) {
    check_pm(*h, "h", a.P);
    a.h = static_cast<const __bf16*>(h->data_ptr());
    a.h_stride = h->stride(0);
  }
  if (z) {
    check_pm(*z, "z", a.P);
    a.z = static_cast<const __bf16*>(z->data_ptr());
    a.z_stride = z->stride(0);
  }
  if (out2) {
    check_pm(*out2, "out2", a.P);
    a.out2 = static_cast<__bf16*>(out2->data_ptr());
    a.out2_stride = out2->stride(0);
  }
  if (epi == 2) TORCH_CHECK(h && out2 && N % 2 == 0, "raft_amd conv_fwd: GRU z||r epilogue needs h, out2");
  if (epi == 3) TORCH_CHECK(h && z && (out2 || a.split_g > 0), "raft_amd conv_fwd: GRU blend epilogue needs h, z, out2");
  TORCH_CHECK(a.split_g == 0 || !a.out_f32, "raft_amd conv_fwd: a split output is bf16 (its planes)");
  if (epi >= 4) {
    // fused GRU backward: fp32 gradient rows, bf16 gate tensors, fp32 carry; every operand is
    // accessed as 8 channels (16 or 32 bytes) per pixel
    TORCH_CHECK(epi <= 6 && a.out_f32 && N % 8 == 0, "raft_amd conv_fwd: GRU backward epilogue needs fp32 out");
    TORCH_CHECK(gru_cols > 0 && gru_cols % 8 == 0 && gru_cols <= N, "raft_amd conv_fwd: gru_cols");
    auto al16 = [](const void* ptr) { return ptr == nullptr || reinterpret_cast<uintptr_t>(ptr) % 16 == 0; };
    // bf16 rows of an epilogue operand: checked, returned as a writable pointer (the input
    // operands convert to const on assignment)
    auto bf_rows = [&](const c10::optional<at::Tensor>& t, const char* what, long& stride) -> __bf16* {
      TORCH_CHECK(t.has_value(), "raft_amd conv_fwd: GRU backward epilogue needs ", what);
      check_pm(*t, what, a.P);
      TORCH_CHECK(t->scalar_type() == dt16 && t->stride(0) % 8 == 0 && al16(t->data_ptr()),
                  "raft_amd conv_fwd: ", what, " must be 16-bit (the sources' dtype) with 16-byte aligned rows");
      stride = t->stride(0);
      return static_cast<__bf16*>(t->data_ptr());
    };
    a.out3 = bf_rows(out3, "out3", a.out3_stride);
    a.gru_cols = static_cast<int>(gru_cols);
    if (epi == 4 || epi == 5) {
      a.h = bf_rows(h, "h", a.h_stride);
      a.g0 = bf_rows(g0, "g0", a.g0_stride);
      TORCH_CHECK(carry.has_value() && carry->scalar_type() == at::kFloat && carry->dim() == 2 &&
                      carry->size(0) >= a.P && carry->size(1) >= gru_cols && carry->stride(1) == 1 &&
                      carry->stride(0) % 4 == 0 && al16(carry->data_ptr()),
                  "raft_amd conv_fwd: carry must be fp32 [P, >=gru_cols] with 16-byte aligned rows");
      a.carry = carry->data_ptr<float>();
      a.carry_stride = carry->stride(0);
    }
    if (epi == 4) {
      a.z = bf_rows(z, "z", a.z_stride);
      a.out2 = bf_rows(out2, "out2", a.out2_stride);
      if (addsrc) a.addsrc = bf_rows(addsrc, "addsrc", a.addsrc_stride);
    }
    if (epi == 6) {
      TORCH_CHECK(cm_c0 >= gru_cols && cm_c0 % 8 == 0 && cm_c0 <= N && cm_valid >= 0, "raft_amd conv_fwd: cm_c0");
      a.cout = bf_rows(cout, "cout", a.cout_stride);
      a.cmask = bf_rows(cmask, "cmask", a.cmask_stride);
      const int64_t cw = std::min<int64_t>(N - cm_c0, (cm_valid + 7) / 8 * 8);  // columns stored / read
      TORCH_CHECK(cout->size(1) >= cw && cmask->size(1) >= cw, "raft_amd conv_fwd: cout / cmask width");
      a.cm_c0 = static_cast<int>(cm_c0);
      a.cm_valid = static_cast<int>(cm_valid);
    }
    TORCH_CHECK(a.out_stride % 4 == 0 && al16(a.out), "raft_amd conv_fwd: out needs 16-byte aligned rows");
  }
  if (n2y) {
    // the flow head's conv2 folded into this conv's epilogue (kernel_abi.h ConvFwdArgs::n2y):
    // 3x3 weights [>=2][Kpad] over the first n2_cols = 64 * slots output channels
    TORCH_CHECK(n2w.has_value() && epi == 0 && split.empty() && !a.out_f32 && a.N % 64 == 0,
                "raft_amd conv_fwd: n2y needs n2w, epilogue 0, a 16-bit output and N % 64 == 0");
    check_gpu(*n2w, "n2w");
    check_gpu(*n2y, "n2y");
    TORCH_CHECK(n2y->scalar_type() == at::kFloat && n2y->dim() == 3 && n2y->is_contiguous() && n2y->size(1) == 18 &&
                    n2y->size(2) == a.P,
                "raft_amd conv_fwd: n2y must be contiguous fp32 [slots][18][P]");
    const int64_t cols = n2y->size(0) * 64;
    TORCH_CHECK(cols <= a.N && n2w->scalar_type() == dt16 && n2w->dim() == 2 && n2w->is_contiguous() &&
                    n2w->size(0) >= 2 && n2w->size(1) >= 9 * cols,
                "raft_amd conv_fwd: n2w must be contiguous [>=2][>=9 * 64 * slots] in the sources' dtype");
    a.n2w = static_cast<const __bf16*>(n2w->data_ptr());
    a.n2y = n2y->data_ptr<float>();
    a.n2_kpad = static_cast<int>(n2w->size(1));
    a.n2_cols = static_cast<int>(cols);
    TORCH_CHECK(a.P * 18 * n2y->size(0) < (1L << 31), "raft_amd conv_fwd: n2y too large");
  }
  const c10::DeviceGuard guard(wt.device());
  HIP_OK(launch_conv_fwd(a, cur_stream()));
}

ConvWgradArgs wgrad_args(at::TensorList srcs, const at::Tensor& dy, at::IntArrayRef geom, int64_t N) {
  TORCH_CHECK(geom.size() == 7, "raft_amd conv_wgrad: geom = (B, H, W, KH, KW, PH, PW)");
  ConvWgradArgs a{};
  a.B = geom[0]; a.H = geom[1]; a.W = geom[2]; a.KH = geom[3]; a.KW = geom[4]; a.PH = geom[5]; a.PW = geom[6];
  a.P = (long)a.B * a.H * a.W;
  a.nsrc = static_cast<int>(srcs.size());
  a.Cin = fill_srcs(srcs, a.P, a.src, true);
  a.K = a.KH * a.KW * a.Cin;
  a.Kpad = (a.K + 63) / 64 * 64;
  check_pm(dy, "dy", a.P);
  TORCH_CHECK(dy.scalar_type() == srcs[0].scalar_type(), "raft_amd conv_wgrad: dy must share the sources' dtype");
  a.f16 = is_half16(dy, "dy") ? 1 : 0;
  TORCH_CHECK(dy.size(1) >= (N + 7) / 8 * 8, "raft_amd conv_wgrad: dy must hold N channels (rounded to 8)");
  a.dy = static_cast<const __bf16*>(dy.data_ptr());
  a.dy_stride = dy.stride(0);
  a.N = static_cast<int>(N);
  TORCH_CHECK(wgrad_supported(a), "raft_amd conv_wgrad: unsupported source layout (multi-source convs need "
              "128-channel segments; every operand must stay below 2 GiB)");
  return a;
}

// Runs the split weight-gradient GEMM into fresh partial slabs; returns (slab, dbslab, plan).
// 128-row workgroups for the 1x5 / 5x1 weight gradients: 12 % slower per launch standalone
// (scripts/bench_convs.py, profiles/r4_convs_wgrad_mt.log) but +0.4 % on the training step
// (5 of 5 interleaved A/B pairs, profiles/r4_bench_wgrad_mt_ab.log): half the workgroups, so the
// tail stream leaves more of the chip to the encoders' backward running beside it.
// (Measured and dropped: the 128-row tile on 8 waves, -1.3 % on the training step,
// profiles/r5o_bench_mt2*.json; planning the weight gradients for fewer workgroups, -0.5 /
// -1.9 %, profiles/r5ad_*.json.)
std::tuple<at::Tensor, at::Tensor, WgradPlan> run_wgrad(ConvWgradArgs& a, bool with_bias, const at::Tensor& like) {
  a.mt5 = 2;  // (64-row 5-tap workgroups: neutral to -0.5 %, profiles/r6l_mt1*.json)
  a.grid_div = 1;
  // v2 weight gradients (the 1x1 convs, convf1) on a 2-stage ring, two workgroups per CU:
  // 219 -> 136 us per call at config #2 (profiles/r6l_kernels.txt; RAFT_WGRAD2_STAGES=3: the
  // 3-stage one-per-CU ring, A/B)
  static const int wg2s = [] {
    const char* e = std::getenv("RAFT_WGRAD2_STAGES");
    return e && e[0] == '3' ? 3 : 2;
  }();
  a.wg2_stages = wg2s;
  const WgradPlan pl = plan_conv_wgrad(a);
  auto opts = like.options().dtype(at::kFloat);
  auto slab = at::empty({(long)pl.nsplit * pl.Npad * a.Kpad}, opts);
  at::Tensor dbslab;
  if (with_bias) dbslab = at::empty({(long)pl.nsplit * pl.tilesN * pl.Npad}, opts);
  a.slab = slab.data_ptr<float>();
  a.dbslab = with_bias ? dbslab.data_ptr<float>() : nullptr;
  HIP_OK(launch_conv_wgrad(a, pl, cur_stream()));
  return {slab, dbslab, pl};
}

// dw[N][Kpad] (+)= dW in the packed GEMM layout (tests, microbenchmarks); deterministic.
void conv_wgrad(at::TensorList srcs, const at::Tensor& dy, at::IntArrayRef geom, int64_t N, const at::Tensor& dw,
                const c10::optional<at::Tensor>& db, bool accumulate) {
  ConvWgradArgs a = wgrad_args(srcs, dy, geom, N);
  check_gpu(dw, "dw");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 2 && dw.stride(1) == 1 && dw.size(0) >= N &&
                  dw.size(1) >= a.Kpad,
              "raft_amd conv_wgrad: dw must be fp32 [>=N][>=Kpad] with unit column stride");
  if (db) {
    TORCH_CHECK(db->scalar_type() == at::kFloat && db->is_contiguous() && db->numel() >= N,
                "raft_amd conv_wgrad: db must be contiguous fp32 [N]");
  }
  if (a.P == 0 || N == 0) return;
  const c10::DeviceGuard guard(dy.device());
  auto [slab, dbslab, pl] = run_wgrad(a, db.has_value(), dy);
  HIP_OK(launch_wgrad_reduce_packed(slab.data_ptr<float>(), pl.nsplit, pl.Npad, a.Kpad, a.K,
                                    db ? dbslab.data_ptr<float>() : nullptr, pl.nsplit * pl.tilesN,
                                    dw.data_ptr<float>(), dw.stride(0), db ? db->data_ptr<float>() : nullptr,
                                    (int)N, accumulate ? 1 : 0, cur_stream()));
}

// Parameter descriptor: 1..2 stacked (Cout_i, Cin, KH, KW) fp32 tensors + optional biases, input
// channel segments [real0, pad0, real1, pad1, ...].
ConvParamDesc param_desc(at::TensorList w, const c10::List<c10::optional<at::Tensor>>& b, at::IntArrayRef segs,
                         double scale, const char* what) {
  TORCH_CHECK(w.size() >= 1 && w.size() <= 2, "raft_amd ", what, ": 1..2 stacked weights");
  TORCH_CHECK(b.size() == w.size(), "raft_amd ", what, ": one bias entry per weight");
  TORCH_CHECK(segs.size() % 2 == 0 && segs.size() >= 2 && segs.size() <= 6, "raft_amd ", what, ": bad segments");
  ConvParamDesc d{};
  for (size_t i = 0; i < w.size(); ++i) {
    const auto& t = w[i];
    check_gpu(t, "weight");
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 4, "raft_amd ", what, ": weights must be fp32 4-D");
    TORCH_CHECK(t.size(1) == w[0].size(1) && t.size(2) == w[0].size(2) && t.size(3) == w[0].size(3),
                "raft_amd ", what, ": stacked weights must agree in (Cin, kh, kw)");
    d.w[i] = t.data_ptr<float>();
    for (int j = 0; j < 4; ++j) d.ws[i][j] = t.stride(j);
    d.rows[i] = static_cast<int>(t.size(0));
    const auto& bi = b.get(i);
    if (bi.has_value()) {
      TORCH_CHECK(bi->scalar_type() == at::kFloat && bi->is_contiguous() && bi->numel() == t.size(0),
                  "raft_amd ", what, ": bias must be contiguous fp32 [Cout]");
      d.b[i] = bi->data_ptr<float>();
    }
  }
  d.nseg = static_cast<int>(segs.size() / 2);
  int real = 0, pad = 0;
  for (int i = 0; i < d.nseg; ++i) {
    d.seg_real[i] = static_cast<int>(segs[2 * i]);
    d.seg_pad[i] = static_cast<int>(segs[2 * i + 1]);
    TORCH_CHECK(d.seg_real[i] <= d.seg_pad[i], "raft_amd ", what, ": segment real > padded");
    real += d.seg_real[i];
    pad += d.seg_pad[i];
  }
  TORCH_CHECK(real == w[0].size(1), "raft_amd ", what, ": segments do not cover Cin");
  d.Cin = real;
  d.Cin_pad = pad;
  d.KH = static_cast<int>(w[0].size(2));
  d.KW = static_cast<int>(w[0].size(3));
  d.scale = static_cast<float>(scale);
  return d;
}

// Weight gradient of all stacked parameters of one conv, written (or accumulated) into the
// parameter gradients themselves: split GEMM -> fixed-order slab reduce (deterministic).
// fold (split-bf16 training): the sources hold every segment as [hi | lo] planes (2 x seg_pad
// channels each), and the parameter gradient is the sum of the two planes' columns.
void conv_wgrad_params(at::TensorList srcs, const at::Tensor& dy, at::IntArrayRef geom, at::TensorList wgrad,
                       const c10::List<c10::optional<at::Tensor>>& bgrad, at::IntArrayRef segs, double scale,
                       bool accumulate, bool fold) {
  ConvParamDesc d = param_desc(wgrad, bgrad, segs, scale, "conv_wgrad_params");
  d.fold = fold ? 1 : 0;
  const int N = d.rows[0] + d.rows[1];
  ConvWgradArgs a = wgrad_args(srcs, dy, geom, N);
  TORCH_CHECK(a.Cin == (fold ? 2 : 1) * d.Cin_pad && a.KH == d.KH && a.KW == d.KW,
              "raft_amd conv_wgrad_params: sources / geometry do not match the parameter layout");
  bool with_bias = false;
  for (size_t i = 0; i < bgrad.size(); ++i) with_bias = with_bias || bgrad.get(i).has_value();
  if (a.P == 0 || N == 0) return;
  const c10::DeviceGuard guard(dy.device());
  auto [slab, dbslab, pl] = run_wgrad(a, with_bias, dy);
  HIP_OK(launch_wgrad_reduce_params(slab.data_ptr<float>(), pl.nsplit, pl.Npad, a.Kpad,
                                    with_bias ? dbslab.data_ptr<float>() : nullptr, pl.nsplit * pl.tilesN, d, N,
                                    accumulate ? 1 : 0, cur_stream()));
}

// fp32 parameters -> bf16 forward operand [N][Kf], optional data-gradient operand
// [Cin_pad][Kd] (flipped taps, Cout padded to cout_pad), fp32 scaled bias [N].
std::tuple<at::Tensor, c10::optional<at::Tensor>, at::Tensor> pack_conv_weights(
    at::TensorList w, const c10::List<c10::optional<at::Tensor>>& b, at::IntArrayRef segs, double scale, int64_t Kf,
    int64_t Kd, int64_t cout_pad, bool f16) {
  ConvParamDesc d = param_desc(w, b, segs, scale, "pack_conv_weights");
  d.f16 = f16 ? 1 : 0;
  const int N = d.rows[0] + d.rows[1];
  const int taps = d.KH * d.KW;
  TORCH_CHECK(Kf >= taps * d.Cin_pad && Kf % 64 == 0, "raft_amd pack_conv_weights: Kf too small / not % 64");
  TORCH_CHECK(Kd == 0 || (cout_pad >= N && Kd >= taps * cout_pad && Kd % 64 == 0),
              "raft_amd pack_conv_weights: bad dgrad layout");
  const c10::DeviceGuard guard(w[0].device());
  auto bopt = w[0].options().dtype(f16 ? at::kHalf : at::kBFloat16);
  auto wf = at::empty({N, Kf}, bopt);
  c10::optional<at::Tensor> wd;
  if (Kd > 0) wd = at::empty({d.Cin_pad, Kd}, bopt);
  auto bias = at::empty({N}, w[0].options());
  HIP_OK(launch_pack_conv_weights(d, N, wf.data_ptr(), (int)Kf, Kd > 0 ? wd->data_ptr() : nullptr, (int)Kd,
                                  (int)cout_pad, bias.data_ptr<float>(), cur_stream()));
  return {wf, wd, bias};
}

// Split-bf16 (fp32-mode) operands: forward [N][Kf] over every segment's [hi | lo | hi] planes
// against [W_hi | W_hi | W_lo]; optional data-gradient operand [Cin_pad][Kd] over dY planes of
// width G_dy (ops/update_split.py); fp32 scaled bias [N].
std::tuple<at::Tensor, c10::optional<at::Tensor>, at::Tensor> pack_conv_weights_split(
    at::TensorList w, const c10::List<c10::optional<at::Tensor>>& b, at::IntArrayRef segs, double scale, int64_t Kf,
    int64_t Kd, int64_t G_dy) {
  ConvParamDesc d = param_desc(w, b, segs, scale, "pack_conv_weights_split");
  const int N = d.rows[0] + d.rows[1];
  const int taps = d.KH * d.KW;
  TORCH_CHECK(Kf >= taps * 3 * d.Cin_pad && Kf % 64 == 0, "raft_amd pack_conv_weights_split: Kf too small / not % 64");
  TORCH_CHECK(Kd == 0 || (G_dy >= N && G_dy % 8 == 0 && Kd >= taps * 3 * G_dy && Kd % 64 == 0),
              "raft_amd pack_conv_weights_split: bad data-gradient layout");
  d.split_fw = 1;
  d.split_dy = (int)G_dy;
  const c10::DeviceGuard guard(w[0].device());
  auto bopt = w[0].options().dtype(at::kBFloat16);
  auto wf = at::empty({N, Kf}, bopt);
  c10::optional<at::Tensor> wd;
  if (Kd > 0) wd = at::empty({d.Cin_pad, Kd}, bopt);
  auto bias = at::empty({N}, w[0].options());
  HIP_OK(launch_pack_conv_weights(d, N, wf.data_ptr(), (int)Kf, Kd > 0 ? wd->data_ptr() : nullptr, (int)Kd, 0,
                                  bias.data_ptr<float>(), cur_stream()));
  return {wf, wd, bias};
}

// Several layers' operands in ONE launch.  Per layer q: nw[q] stacked weights (and biases) from
// the flat lists, nseg[q] (real, padded) segment pairs from ``segs``, scale[q], Kf[q], Kd[q]
// (0: no data-gradient operand) and aux[q] (Cout_pad, or G_dy in split mode).  Returns
// [wf_0, wd_0, bias_0, wf_1, ...] (wd_q empty when Kd[q] == 0): views of one 16-bit buffer and
// one fp32 buffer.
std::vector<at::Tensor> pack_conv_weights_multi(at::TensorList w, const c10::List<c10::optional<at::Tensor>>& b,
                                                at::IntArrayRef nw, at::IntArrayRef segs, at::IntArrayRef nseg,
                                                at::ArrayRef<double> scale, at::IntArrayRef Kf, at::IntArrayRef Kd,
                                                at::IntArrayRef aux, bool f16, bool split) {
  const int L = (int)nw.size();
  TORCH_CHECK(L >= 1 && L <= kPackJobs && (int)nseg.size() == L && (int)scale.size() == L && (int)Kf.size() == L &&
                  (int)Kd.size() == L && (int)aux.size() == L && (int)b.size() == (int)w.size(),
              "raft_amd pack_conv_weights_multi: 1..", kPackJobs, " layers with one entry per list");
  TORCH_CHECK(!(split && f16), "raft_amd pack_conv_weights_multi: split packs are bf16");
  PackJobs js{};
  js.n = L;
  int wi = 0, si = 0;
  long total = 0, n16 = 0, n32 = 0;
  std::vector<long> off16(L), offd(L), off32(L);
  for (int q = 0; q < L; ++q) {
    TORCH_CHECK(nw[q] >= 1 && nw[q] <= 2 && wi + nw[q] <= (int)w.size(), "raft_amd pack_conv_weights_multi: nw");
    TORCH_CHECK(nseg[q] >= 1 && si + 2 * nseg[q] <= (int)segs.size(), "raft_amd pack_conv_weights_multi: segs");
    c10::List<c10::optional<at::Tensor>> bq;
    for (int k = 0; k < nw[q]; ++k) bq.push_back(b.get(wi + k));
    PackJob& jb = js.j[q];
    jb.d = param_desc(w.slice(wi, nw[q]), bq, segs.slice(si, 2 * nseg[q]), scale[q], "pack_conv_weights_multi");
    wi += (int)nw[q];
    si += 2 * (int)nseg[q];
    const int N = jb.d.rows[0] + jb.d.rows[1], taps = jb.d.KH * jb.d.KW;
    jb.N = N;
    jb.Kf = (int)Kf[q];
    jb.Kd = (int)Kd[q];
    jb.aux = (int)aux[q];
    if (split) {
      TORCH_CHECK(Kf[q] >= taps * 3 * jb.d.Cin_pad && Kf[q] % 64 == 0 &&
                      (Kd[q] == 0 || (aux[q] >= N && aux[q] % 8 == 0 && Kd[q] >= taps * 3 * aux[q] && Kd[q] % 64 == 0)),
                  "raft_amd pack_conv_weights_multi: bad split layout of layer ", q);
      jb.d.split_fw = 1;
      jb.d.split_dy = (int)aux[q];
    } else {
      TORCH_CHECK(Kf[q] >= taps * jb.d.Cin_pad && Kf[q] % 64 == 0 &&
                      (Kd[q] == 0 || (aux[q] >= N && Kd[q] >= taps * aux[q] && Kd[q] % 64 == 0)),
                  "raft_amd pack_conv_weights_multi: bad layout of layer ", q);
      jb.d.f16 = f16 ? 1 : 0;
    }
    jb.begin = total;
    total += (long)N * Kf[q] + (Kd[q] > 0 ? (long)jb.d.Cin_pad * Kd[q] : 0) + N;
    off16[q] = n16;
    auto r64 = [](long v) { return (v + 63) / 64 * 64; };  // 128-byte aligned views
    n16 += r64((long)N * Kf[q]);
    offd[q] = n16;
    n16 += Kd[q] > 0 ? r64((long)jb.d.Cin_pad * Kd[q]) : 0;
    off32[q] = n32;
    n32 += r64((long)N);
  }
  TORCH_CHECK(wi == (int)w.size() && si == (int)segs.size(), "raft_amd pack_conv_weights_multi: unused list entries");
  js.total = total;
  const c10::DeviceGuard guard(w[0].device());
  auto buf16 = at::empty({n16}, w[0].options().dtype(f16 ? at::kHalf : at::kBFloat16));
  auto buf32 = at::empty({n32}, w[0].options().dtype(at::kFloat));
  std::vector<at::Tensor> out;
  for (int q = 0; q < L; ++q) {
    PackJob& jb = js.j[q];
    at::Tensor wf = buf16.narrow(0, off16[q], (long)jb.N * jb.Kf).view({jb.N, jb.Kf});
    at::Tensor wd = jb.Kd > 0 ? buf16.narrow(0, offd[q], (long)jb.d.Cin_pad * jb.Kd).view({jb.d.Cin_pad, jb.Kd})
                              : buf16.new_empty({0});
    at::Tensor bias = buf32.narrow(0, off32[q], jb.N);
    jb.wf = reinterpret_cast<__bf16*>(wf.data_ptr());
    jb.wd = jb.Kd > 0 ? reinterpret_cast<__bf16*>(wd.data_ptr()) : nullptr;
    jb.bias = bias.data_ptr<float>();
    out.push_back(wf);
    out.push_back(wd);
    out.push_back(bias);
  }
  HIP_OK(launch_pack_conv_weights_multi(js, cur_stream()));
  return out;
}

// ---------------------------------------------------------------- update-block elementwise
void pm_any(const at::Tensor& t, const char* name, long P, at::ScalarType dt) {
  check_gpu(t, name);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.size(0) == P && t.scalar_type() == dt,
              "raft_amd: ", name, " must be a (P, C) pixel-major view of dtype ", dt);
}

void gru_bwd_a(const at::Tensor& dH, const at::Tensor& z, const at::Tensor& q, const at::Tensor& h,
               const at::Tensor& dq, const at::Tensor& dz, const at::Tensor& carry) {
  const long P = dH.size(0), C = dH.size(1);
  pm_any(dH, "dH", P, at::kFloat);
  pm_any(z, "z", P, at::kBFloat16);
  pm_any(q, "q", P, at::kBFloat16);
  pm_any(h, "h", P, at::kBFloat16);
  pm_any(dq, "dq", P, at::kBFloat16);
  pm_any(dz, "dz", P, at::kBFloat16);
  pm_any(carry, "carry", P, at::kFloat);
  TORCH_CHECK(z.size(1) >= C && q.size(1) >= C && h.size(1) >= C && dq.size(1) >= C && dz.size(1) >= C &&
                  carry.size(1) >= C, "raft_amd gru_bwd_a: channel mismatch");
  const c10::DeviceGuard guard(dH.device());
  HIP_OK(launch_gru_bwd_a(dH.data_ptr<float>(), dH.stride(0), z.data_ptr(), z.stride(0), q.data_ptr(),
                          q.stride(0), h.data_ptr(), h.stride(0), dq.data_ptr(), dq.stride(0), dz.data_ptr(),
                          dz.stride(0), carry.data_ptr<float>(), carry.stride(0), P, C, cur_stream()));
}

void gru_bwd_b(const at::Tensor& drh, const at::Tensor& r, const at::Tensor& h, const at::Tensor& carry,
               const at::Tensor& dr) {
  const long P = drh.size(0), C = drh.size(1);
  pm_any(drh, "drh", P, at::kFloat);
  pm_any(r, "r", P, at::kBFloat16);
  pm_any(h, "h", P, at::kBFloat16);
  pm_any(carry, "carry", P, at::kFloat);
  pm_any(dr, "dr", P, at::kBFloat16);
  const c10::DeviceGuard guard(drh.device());
  HIP_OK(launch_gru_bwd_b(drh.data_ptr<float>(), drh.stride(0), r.data_ptr(), r.stride(0), h.data_ptr(),
                          h.stride(0), carry.data_ptr<float>(), carry.stride(0), dr.data_ptr(), dr.stride(0), P,
                          C, cur_stream()));
}

void masked_cast(const at::Tensor& src, const c10::optional<at::Tensor>& mask, const at::Tensor& out) {
  const long P = out.size(0), C = out.size(1);
  pm_any(src, "src", P, at::kFloat);
  pm_any(out, "out", P, at::kBFloat16);
  TORCH_CHECK(src.size(1) <= C, "raft_amd masked_cast: src wider than out");
  const void* m = nullptr;
  long sm = 0;
  if (mask) {
    pm_any(*mask, "mask", P, at::kBFloat16);
    TORCH_CHECK(mask->size(1) >= C, "raft_amd masked_cast: mask too narrow");
    m = mask->data_ptr();
    sm = mask->stride(0);
  }
  const c10::DeviceGuard guard(src.device());
  HIP_OK(launch_masked_cast(src.data_ptr<float>(), src.stride(0), m, sm, out.data_ptr(), out.stride(0), P, C,
                            static_cast<int>(src.size(1)), cur_stream()));
}

void pack_flow(const at::Tensor& flow, const at::Tensor& flow8, const c10::optional<at::Tensor>& motion,
               bool from_coords) {
  check_gpu(flow, "flow");
  TORCH_CHECK(flow.scalar_type() == at::kFloat && flow.is_contiguous() && flow.dim() == 4 && flow.size(1) == 2,
              "raft_amd pack_flow: flow must be contiguous fp32 (B, 2, H, W)");
  const long B = flow.size(0), HW = flow.size(2) * flow.size(3);
  TORCH_CHECK(flow8.is_contiguous() && (flow8.scalar_type() == at::kBFloat16 || flow8.scalar_type() == at::kHalf) &&
                  flow8.numel() == B * HW * 8,
              "raft_amd pack_flow: flow8 must be contiguous bf16 / fp16 (P, 8)");
  void* mo = nullptr;
  long smo = 0;
  if (motion) {
    pm_any(*motion, "motion", B * HW, flow8.scalar_type());
    TORCH_CHECK(motion->size(1) >= 2, "raft_amd pack_flow: motion slice needs 2 channels");
    mo = motion->data_ptr();
    smo = motion->stride(0);
  }
  const c10::DeviceGuard guard(flow.device());
  HIP_OK(launch_pack_flow(flow.data_ptr<float>(), flow8.data_ptr(), mo, smo, B, HW, (int)flow.size(3),
                          (from_coords ? 1 : 0) | (flow8.scalar_type() == at::kHalf ? 2 : 0), cur_stream()));
}

// fp32 (P, C) rows -> split-bf16 planes of group width G in dst (P, *) bf16 rows, channels
// [c0, c0 + Cpad) (zero past C); see kernel_abi.h ConvFwdArgs::split_g
void split_pack(const at::Tensor& src, const at::Tensor& dst, int64_t G, int64_t c0, int64_t Cpad) {
  check_gpu(src, "src");
  check_gpu(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && src.scalar_type() == at::kFloat && src.stride(1) == 1,
              "raft_amd split_pack: src must be fp32 (P, C) rows");
  TORCH_CHECK(dst.dim() == 2 && dst.scalar_type() == at::kBFloat16 && dst.stride(1) == 1 && dst.size(0) == src.size(0),
              "raft_amd split_pack: dst must be bf16 (P, *) rows");
  const long C = src.size(1);
  TORCH_CHECK(G > 0 && c0 >= 0 && Cpad >= C, "raft_amd split_pack: G, c0, Cpad");
  const long last = c0 + Cpad - 1;  // highest output channel: its hi-again plane must fit in the row
  TORCH_CHECK((last / G) * 3 * G + 2 * G + last % G < dst.size(1) || dst.size(0) == 0,
              "raft_amd split_pack: dst rows too narrow for the split planes");
  const c10::DeviceGuard guard(src.device());
  HIP_OK(launch_split_pack(src.data_ptr<float>(), src.stride(0), (int)C, (int)Cpad, dst.data_ptr(), dst.stride(0),
                           (int)G, (int)c0, src.size(0), cur_stream()));
}

// coords_out = coords1 + delta[:, :2] (delta: (P, >=2) fp32 rows), flow_out = coords_out - grid
void apply_delta(const at::Tensor& coords1, const at::Tensor& delta, const at::Tensor& coords_out,
                 const at::Tensor& flow_out) {
  check_coords(coords1);
  check_coords(coords_out);
  check_coords(flow_out);
  TORCH_CHECK(coords_out.sizes() == coords1.sizes() && flow_out.sizes() == coords1.sizes(),
              "raft_amd apply_delta: shape mismatch");
  const long B = coords1.size(0), HW = coords1.size(2) * coords1.size(3);
  pm_any(delta, "delta", B * HW, at::kFloat);
  TORCH_CHECK(delta.size(1) >= 2, "raft_amd apply_delta: delta needs 2 channels");
  const c10::DeviceGuard guard(coords1.device());
  HIP_OK(launch_apply_delta(coords1.data_ptr<float>(), delta.data_ptr<float>(), delta.stride(0),
                            coords_out.data_ptr<float>(), flow_out.data_ptr<float>(), B, HW, (int)coords1.size(3),
                            cur_stream()));
}

// the flow head's conv2 from the heads conv's per-tap partials (conv_fwd n2y) + apply_delta;
// delta (P, >=2) fp32 rows is also written when given
void n2_apply(const at::Tensor& y, const at::Tensor& bias, const at::Tensor& coords1, const at::Tensor& coords_out,
              const at::Tensor& flow_out, const c10::optional<at::Tensor>& delta) {
  check_coords(coords1);
  check_coords(coords_out);
  check_coords(flow_out);
  TORCH_CHECK(coords_out.sizes() == coords1.sizes() && flow_out.sizes() == coords1.sizes(),
              "raft_amd n2_apply: shape mismatch");
  const long B = coords1.size(0), H = coords1.size(2), W = coords1.size(3);
  check_gpu(y, "y");
  TORCH_CHECK(y.scalar_type() == at::kFloat && y.dim() == 3 && y.is_contiguous() && y.size(0) <= 4 && y.size(1) == 18 &&
                  y.size(2) == B * H * W,
              "raft_amd n2_apply: y must be contiguous fp32 [slots <= 4][18][P]");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.is_contiguous() && bias.numel() >= 2 &&
                  bias.device() == y.device(),
              "raft_amd n2_apply: bias must be fp32 [>=2] on the device");
  float* dp = nullptr;
  long sd = 0;
  if (delta) {
    pm_any(*delta, "delta", B * H * W, at::kFloat);
    TORCH_CHECK(delta->size(1) >= 2, "raft_amd n2_apply: delta needs 2 channels");
    dp = delta->data_ptr<float>();
    sd = delta->stride(0);
  }
  const c10::DeviceGuard guard(coords1.device());
  HIP_OK(launch_n2_apply(y.data_ptr<float>(), (int)y.size(0), bias.data_ptr<float>(), coords1.data_ptr<float>(),
                         coords_out.data_ptr<float>(), flow_out.data_ptr<float>(), dp, sd, (int)B, (int)H, (int)W,
                         cur_stream()));
}

// corr_lookup into a caller buffer (B, H, W, och) with och >= L*(2r+1)^2 (zero padded)
// flow8 / motion (optional): the step's packed flow operand, written by the same launch
// (pack_flow(coords, flow8, motion, from_coords=true) folded into the lookup)
void corr_lookup_into(at::TensorList pyramid, const at::Tensor& coords, int64_t radius, const at::Tensor& out,
                      const c10::optional<at::Tensor>& flow8, const c10::optional<at::Tensor>& motion) {
  check_coords(coords);
  const long B = coords.size(0), H = coords.size(2), W = coords.size(3);
  std::vector<at::Tensor> lv(pyramid.begin(), pyramid.end());
  PyrDesc d = make_desc(lv, B * H * W, true);
  const long win = (2 * radius + 1) * (2 * radius + 1);
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 4 && out.is_contiguous() && out.size(0) == B && out.size(1) == H && out.size(2) == W &&
                  out.size(3) >= d.levels * win,
              "raft_amd::corr_lookup_into: out must be contiguous (B, H, W, >= L*(2r+1)^2)");
  void* f8 = nullptr;
  void* mo = nullptr;
  long smo = 0;
  if (flow8) {
    TORCH_CHECK(flow8->is_contiguous() && flow8->scalar_type() == out.scalar_type() &&
                    (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kHalf) &&
                    flow8->numel() == B * H * W * 8,
                "raft_amd::corr_lookup_into: flow8 must be contiguous (P, 8) in the 16-bit out dtype");
    f8 = flow8->data_ptr();
    if (motion) {
      pm_any(*motion, "motion", B * H * W, out.scalar_type());
      TORCH_CHECK(motion->size(1) >= 2, "raft_amd::corr_lookup_into: motion slice needs 2 channels");
      mo = motion->data_ptr();
      smo = motion->stride(0);
    }
  }
  const c10::DeviceGuard guard(coords.device());
  HIP_OK(launch_corr_lookup_fwd(d, coords.data_ptr<float>(), out.data_ptr(), dtype_code(out.scalar_type()), B, H, W,
                                static_cast<int>(radius), static_cast<int>(out.size(3)), cur_stream(), f8, mo, smo));
}

// ---------------------------------------------------------------- NHWC instance norm
void check_in(const at::Tensor& x, const char* name) {
  check_gpu(x, name);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) && x.size(1) % 8 == 0 &&
                  x.size(1) <= 512,
              "raft_amd instance_norm: ", name, " must be channels-last bf16/fp32 (N, C%8==0, H, W)");
}

std::tuple<at::Tensor, at::Tensor> instance_norm_fwd(const at::Tensor& x, bool relu, double eps) {
  check_in(x, "x");
  const long N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  const c10::DeviceGuard guard(x.device());
  auto y = at::empty(x.sizes(), x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stats = at::empty({N, C, 2}, x.options().dtype(at::kFloat));
  auto part = at::empty({instance_norm_chunks(HW), N, C, 2}, x.options().dtype(at::kFloat));
  HIP_OK(launch_instance_norm_fwd(dtype_code(x.scalar_type()), x.data_ptr(), y.data_ptr(), stats.data_ptr<float>(),
                                  part.data_ptr<float>(), N, HW, C, relu, static_cast<float>(eps), cur_stream()));
  return {y, stats};
}

at::Tensor instance_norm_bwd(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& stats, bool relu) {
  check_in(x, "x");
  auto g = dy.to(x.scalar_type()).contiguous(at::MemoryFormat::ChannelsLast);
  const long N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(stats.is_contiguous() && stats.numel() == N * C * 2, "raft_amd instance_norm_bwd: bad stats");
  const c10::DeviceGuard guard(x.device());
  auto dx = at::empty(x.sizes(), x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto gsum = at::empty({N, C, 2}, x.options().dtype(at::kFloat));
  auto part = at::empty({instance_norm_chunks(HW), N, C, 2}, x.options().dtype(at::kFloat));
  HIP_OK(launch_instance_norm_bwd(dtype_code(x.scalar_type()), x.data_ptr(), g.data_ptr(), stats.data_ptr<float>(),
                                  gsum.data_ptr<float>(), part.data_ptr<float>(), dx.data_ptr(), N, HW, C, relu,
                                  cur_stream()));
  return dx;
}


// ============================================================================ step executor
// One refinement iteration of the fused RAFT-base update (ops/update_fused.py _Step.forward,
// reference core/raft.py:122-139 + core/update.py:79-136) issued from C++ in one op call: the
// ~17 launches, the side-stream fork / join of the flow branch and the tail-stream mask head,
// with the arena slot views, packed weights and stream handles handed in by the caller.  The
// Python body it replaces spent ~0.35 ms of host time per iteration (op dispatch with ~27
// boxed arguments per conv, views, stream context managers) -- the training forward was
// host-bound (6.6 ms host vs 5.9 ms GPU, profiles/r5j_host_lead.log).
namespace step_exec {
enum Buf {
  B_H0, B_CORR, B_FLOW8, B_MOTION, B_C1, B_CF, B_F1, B_ZR1, B_RH1, B_Q1, B_H1, B_ZR2, B_RH2, B_Q2, B_H2,
  B_HD, B_MASK, B_N2Y, B_COORDS1, B_INP, B_COUNT
};
enum Layer { L_CONVC1, L_CONVC2, L_CONVF1, L_CONVF2, L_CONV, L_ZR1, L_Q1, L_ZR2, L_Q2, L_HEADS, L_FH2, L_MASK2, L_COUNT };
constexpr int kHid = 128, kCorrPad = 328;

// fork / join events: a ring per process, each record is waited on immediately after
hipEvent_t next_event() {
  static std::vector<hipEvent_t> ring;
  static size_t i = 0;
  if (ring.empty()) {
    ring.resize(64);
    for (auto& e : ring) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  return ring[i++ % ring.size()];
}
void order(hipStream_t after, hipStream_t before) {  // `after` waits for the work queued on `before`
  if (after == before) return;
  hipEvent_t e = next_event();
  HIP_OK(hipEventRecord(e, before));
  HIP_OK(hipStreamWaitEvent(after, e, 0));
}
}  // namespace step_exec

std::vector<at::Tensor> fused_step_fwd(at::TensorList bufs, at::TensorList wf, at::TensorList bias, at::TensorList levels,
                                       const c10::optional<at::Tensor>& corr_in, at::IntArrayRef cfg) {
  using namespace step_exec;
  TORCH_CHECK(bufs.size() == B_COUNT && wf.size() == L_COUNT && bias.size() == L_COUNT && cfg.size() == 9,
              "raft_amd fused_step_fwd: bufs / weights / cfg layout");
  const int64_t B = cfg[0], H = cfg[1], W = cfg[2], radius = cfg[3];
  const bool up = cfg[4] != 0, fold = cfg[7] != 0;
  const at::Tensor &h0 = bufs[B_H0], &corr = bufs[B_CORR], &flow8 = bufs[B_FLOW8], &motion = bufs[B_MOTION];
  const at::Tensor &c1 = bufs[B_C1], &cf = bufs[B_CF], &f1 = bufs[B_F1], &hd = bufs[B_HD], &mask = bufs[B_MASK];
  const at::Tensor &coords1 = bufs[B_COORDS1], &inp = bufs[B_INP];
  const c10::DeviceGuard guard(coords1.device());
  const auto dev = coords1.device().index();
  auto main_s = c10::hip::getCurrentHIPStream();
  const hipStream_t hm = main_s.stream();
  const hipStream_t hs = cfg[5] ? reinterpret_cast<hipStream_t>(cfg[5]) : hm;
  const hipStream_t ht = (cfg[6] && up) ? reinterpret_cast<hipStream_t>(cfg[6]) : nullptr;
  auto side_s = c10::hip::getStreamFromExternal(hs, dev);
  const c10::optional<at::Tensor> none;
  auto geom = [&](int64_t kh, int64_t kw) { return std::vector<int64_t>{B, H, W, kh, kw, kh / 2, kw / 2}; };
  // the plain conv launch (epilogue 0: bias + optional ReLU)
  auto conv = [&](std::vector<at::Tensor> srcs, const at::Tensor& w, int64_t kh, int64_t kw, int64_t N,
                  const at::Tensor& out, const at::Tensor& b, int64_t act, const c10::optional<at::Tensor>& n2w = {},
                  const c10::optional<at::Tensor>& n2y = {}) {
    conv_fwd(srcs, w, geom(kh, kw), N, b, 0, act, 1.0, out, 1 << 30, none, none, none, none, 0, none, none, none, 0,
             none, none, none, 0, 0, {}, n2w, n2y);
  };

  // correlation features (+ the step's flow operand)
  if (levels.size() > 0) {
    corr_lookup_into(levels, coords1, radius, corr.view({B, H, W, kCorrPad}), flow8, motion.narrow(1, 126, 2));
  } else {
    TORCH_CHECK(corr_in.has_value(), "raft_amd fused_step_fwd: no pyramid and no correlation rows");
    corr.copy_(corr_in->reshape({B * H * W, kCorrPad}));
    pack_flow(coords1, flow8, motion.narrow(1, 126, 2), true);
  }
  // motion encoder: the flow branch on the side stream beside the correlation branch
  order(hs, hm);
  {
    c10::hip::HIPStreamGuard sg(side_s);
    conv({flow8}, wf[L_CONVF1], 7, 7, 128, f1, bias[L_CONVF1], 1);
    conv({f1}, wf[L_CONVF2], 3, 3, 64, cf.narrow(1, 192, 64), bias[L_CONVF2], 1);
  }
  conv({corr}, wf[L_CONVC1], 1, 1, 256, c1, bias[L_CONVC1], 1);
  conv({c1}, wf[L_CONVC2], 3, 3, 192, cf.narrow(1, 0, 192), bias[L_CONVC2], 1);
  order(hm, hs);
  conv({cf}, wf[L_CONV], 3, 3, 126, motion, bias[L_CONV], 1);
  // SepConvGRU: 1x5 then 5x1; gates in the epilogues
  at::Tensor h = h0;
  const Buf zrb[2] = {B_ZR1, B_ZR2}, rhb[2] = {B_RH1, B_RH2}, qb[2] = {B_Q1, B_Q2}, hb[2] = {B_H1, B_H2};
  const Layer zrl[2] = {L_ZR1, L_ZR2}, ql[2] = {L_Q1, L_Q2};
  for (int st = 0; st < 2; ++st) {
    const int64_t kh = st == 0 ? 1 : 5, kw = st == 0 ? 5 : 1;
    const at::Tensor &zr = bufs[zrb[st]], &rh = bufs[rhb[st]], &q = bufs[qb[st]], &hn = bufs[hb[st]];
    conv_fwd({h, inp, motion}, wf[zrl[st]], geom(kh, kw), 2 * kHid, bias[zrl[st]], 2, 0, 1.0, zr, 1 << 30, none, h,
             none, rh, 0, none, none, none, 0, none, none, none, 0, 0, {}, none, none);
    conv_fwd({rh, inp, motion}, wf[ql[st]], geom(kh, kw), kHid, bias[ql[st]], 3, 0, 1.0, hn, 1 << 30, none, h,
             zr.narrow(1, 0, kHid), q, 0, none, none, none, 0, none, none, none, 0, 0, {}, none, none);
    h = hn;
  }
  // flow head (+ conv2 folded into its epilogue) and the coordinate update
  auto coords_out = at::empty_like(coords1), flow = at::empty_like(coords1);
  const at::Tensor& n2y = bufs[B_N2Y];
  const int64_t nh = (up && !ht) ? 512 : 256;
  if (fold) {
    conv({h}, wf[L_HEADS], 3, 3, nh, hd, bias[L_HEADS], 1, wf[L_FH2], n2y);
    n2_apply(n2y, bias[L_FH2], coords1, coords_out, flow, none);
  } else {
    conv({h}, wf[L_HEADS], 3, 3, nh, hd, bias[L_HEADS], 1);
    auto delta = at::empty({B * H * W, 8}, coords1.options());
    conv({hd.narrow(1, 0, 256)}, wf[L_FH2], 3, 3, 2, delta, bias[L_FH2], 0);
    apply_delta(coords1, delta, coords_out, flow);
  }
  if (!up) return {coords_out, flow};
  // mask head + convex upsampling: they feed only the loss, so on the tail stream beside the
  // next step (the caller joins it before the loss reads the flows)
  at::Tensor flow_up;
  {
    c10::optional<c10::hip::HIPStreamGuard> tg;
    if (ht) {
      order(ht, hm);
      tg.emplace(c10::hip::getStreamFromExternal(ht, dev));
      conv({h}, wf[L_HEADS].narrow(0, 256, 256), 3, 3, 256, hd.narrow(1, 256, 256), bias[L_HEADS].narrow(0, 256, 256), 1);
    }
    conv({hd.narrow(1, 256, 256)}, wf[L_MASK2], 1, 1, 576, mask, bias[L_MASK2], 0);
    flow_up = convex_upsample(flow, mask.reshape({B, H, W, 576}).permute({0, 3, 1, 2}));
  }
  if (ht) c10::hip::HIPCachingAllocator::recordStream(flow_up.storage().data_ptr(), main_s);
  return {coords_out, flow, flow_up};
}

// The backward of one refinement iteration (ops/update_fused.py _Step.backward; reference
// core/update.py:79-136 and core/raft.py:122-139 differentiated) issued from C++: the upsampler /
// head data gradients on the head stream, the GRU data gradients with the gate backward in their
// epilogues on the main stream, the motion-encoder data gradients on the tail stream.  The Python
// body it replaces cost ~0.28 ms of host time per iteration (11 boxed conv_fwd calls, ~30 arena
// views, stream context managers): at batch 1-2 per GPU the training step is host-bound.
// bufs: the per-forward arena buffers ([slots * P, C], step t at rows [t P, (t + 1) P); "h" has
// iters + 1 slots), see BwdBuf; wd: the packed data-gradient weights in _LAYERS order; g_all:
// [iters, P, 3 * 128] fp32 rows of [d h | d inp | d motion]; cfg = (B, H, W, t, head stream,
// tail stream).  Returns (d net (P, 128), d corr (P, 328)) in the arena's 16-bit dtype.
namespace step_exec {
enum BwdBuf {
  Q_HD, Q_MASK, Q_H, Q_H1, Q_ZR1, Q_ZR2, Q_Q1, Q_Q2, Q_MOTION, Q_CF, Q_C1, Q_F1, Q_DMASK, Q_DD8, Q_DHD, Q_DQ1,
  Q_DQ2, Q_DZR1, Q_DZR2, Q_DMO, Q_DCF, Q_DC1, Q_DF1, Q_COUNT
};
}  // namespace step_exec

std::vector<at::Tensor> fused_step_bwd(at::TensorList bufs, at::TensorList wd, const at::Tensor& g_all,
                                       const at::Tensor& flow, const c10::optional<at::Tensor>& g_net,
                                       const c10::optional<at::Tensor>& g_flow_up, at::IntArrayRef cfg) {
  using namespace step_exec;
  TORCH_CHECK(bufs.size() == Q_COUNT && wd.size() == L_COUNT && cfg.size() == 6,
              "raft_amd fused_step_bwd: bufs / weights / cfg layout");
  const int64_t B = cfg[0], H = cfg[1], W = cfg[2], t = cfg[3];
  const int64_t P = B * H * W;
  TORCH_CHECK(t >= 0 && g_all.dim() == 3 && t < g_all.size(0) && g_all.size(1) == P && g_all.size(2) == 3 * kHid &&
                  g_all.scalar_type() == at::kFloat && g_all.is_contiguous(),
              "raft_amd fused_step_bwd: g_all must be a contiguous fp32 [iters, P, 384] buffer");
  for (int i = 0; i < Q_COUNT; ++i)
    TORCH_CHECK(bufs[i].dim() == 2 && bufs[i].size(0) >= (t + 1 + (i == Q_H)) * P,
                "raft_amd fused_step_bwd: arena buffer ", i, " has no slot ", t);
  auto R = [&](BwdBuf b) { return bufs[b].narrow(0, t * P, P); };
  const at::Tensor hd = R(Q_HD), mask = R(Q_MASK), dmask = R(Q_DMASK), dd8 = R(Q_DD8), dhd = R(Q_DHD);
  const at::Tensor h_in = R(Q_H), h1 = R(Q_H1), zr1 = R(Q_ZR1), zr2 = R(Q_ZR2), q1 = R(Q_Q1), q2 = R(Q_Q2);
  const at::Tensor dq1 = R(Q_DQ1), dq2 = R(Q_DQ2), dzr1 = R(Q_DZR1), dzr2 = R(Q_DZR2), motion = R(Q_MOTION);
  const at::Tensor cf = R(Q_CF), c1 = R(Q_C1), f1 = R(Q_F1), dmo = R(Q_DMO), dcf = R(Q_DCF), dc1 = R(Q_DC1);
  const at::Tensor df1 = R(Q_DF1);
  const auto dt16 = hd.scalar_type();
  const c10::DeviceGuard guard(hd.device());
  const auto dev = hd.device().index();
  auto main_s = c10::hip::getCurrentHIPStream();
  const hipStream_t hm = main_s.stream();
  const hipStream_t hh = cfg[4] ? reinterpret_cast<hipStream_t>(cfg[4]) : hm;
  const hipStream_t ht = cfg[5] ? reinterpret_cast<hipStream_t>(cfg[5]) : hm;
  const c10::optional<at::Tensor> none;
  // data-gradient geometry: the transposed conv's padding
  auto gd = [&](int64_t kh, int64_t kw) {
    return std::vector<int64_t>{B, H, W, kh, kw, kh - 1 - kh / 2, kw - 1 - kw / 2};
  };
  auto dgrad = [&](const at::Tensor& dy, Layer l, int64_t kh, int64_t kw, int64_t n, const at::Tensor& out,
                   const c10::optional<at::Tensor>& relu_mask) {
    conv_fwd({dy}, wd[l], gd(kh, kw), n, none, 1, 0, 1.0, out, 1 << 30, relu_mask, none, none, none, 0, none, none,
             none, 0, none, none, none, 0, 0, {}, none, none);
  };
  auto nchw = [&](const at::Tensor& rows, int64_t C) { return rows.reshape({B, H, W, C}).permute({0, 3, 1, 2}); };

  // ---- upsampler + head data gradients (head stream; the caller ordered it after the loss
  // gradient's ready event)
  {
    c10::optional<c10::hip::HIPStreamGuard> g;
    if (hh != hm) g.emplace(c10::hip::getStreamFromExternal(hh, dev));
    if (g_flow_up.has_value()) {
      convex_upsample_backward_into(flow, nchw(mask, 576), *g_flow_up, nchw(dmask, 576), dd8);
    } else {
      dmask.zero_();
      dd8.zero_();
    }
    dgrad(dd8, L_FH2, 3, 3, 256, dhd.narrow(1, 0, 256), hd.narrow(1, 0, 256));
    dgrad(dmask, L_MASK2, 1, 1, 256, dhd.narrow(1, 256, 256), hd.narrow(1, 256, 256));
  }
  order(hm, hh);
  // ---- GRU stages in reverse: the conv producing a stage's dH finishes (dq, dz, carry) of that
  // stage in its epilogue (4 = EPI_GRU_BWD_A), the q conv's data gradient dr and d h (5 = _B),
  // the last one d net, d inp and the ReLU'-masked d motion (6 = _LAST)
  auto carry = at::empty({P, kHid}, hd.options().dtype(at::kFloat));
  c10::optional<at::Tensor> add;
  if (g_net.has_value()) add = g_net->permute({0, 2, 3, 1}).reshape({P, kHid}).to(dt16).contiguous();
  auto gate_a = [&](const at::Tensor& dy, const at::Tensor& w, std::vector<int64_t> geom, int64_t n,
                    const at::Tensor& out, int64_t acc_c0, const at::Tensor& h, const at::Tensor& zr,
                    const at::Tensor& q, const at::Tensor& dq, const at::Tensor& dzr,
                    const c10::optional<at::Tensor>& addsrc) {
    conv_fwd({dy}, w, geom, n, none, 4, 0, 1.0, out, acc_c0, none, h, zr.narrow(1, 0, kHid), dq, 0, q, carry,
             dzr.narrow(1, 0, kHid), kHid, addsrc, none, none, 0, 0, {}, none, none);
  };
  // heads data gradient = dH of stage 2 (+ the incoming d net); carry stands in for the output
  gate_a(dhd, wd[L_HEADS], gd(3, 3), kHid, carry, 1 << 30, h1, zr2, q2, dq2, dzr2, add);
  const at::Tensor G = g_all[t];
  auto d_net = at::empty({P, kHid}, hd.options());
  // stage 2 (5x1)
  conv_fwd({dq2}, wd[L_Q2], gd(5, 1), 3 * kHid, none, 5, 0, 1.0, G, 3 * kHid, none, h1, none, none, 0,
           zr2.narrow(1, kHid, kHid), carry, dzr2.narrow(1, kHid, kHid), kHid, none, none, none, 0, 0, {}, none,
           none);
  gate_a(dzr2, wd[L_ZR2], gd(5, 1), 3 * kHid, G, 0, h_in, zr1, q1, dq1, dzr1, none);
  // stage 1 (1x5)
  conv_fwd({dq1}, wd[L_Q1], gd(1, 5), 3 * kHid, none, 5, 0, 1.0, G, kHid, none, h_in, none, none, 0,
           zr1.narrow(1, kHid, kHid), carry, dzr1.narrow(1, kHid, kHid), kHid, none, none, none, 0, 0, {}, none,
           none);
  conv_fwd({dzr1}, wd[L_ZR1], gd(1, 5), 3 * kHid, none, 6, 0, 1.0, G, 0, none, none, none, none, 0, none, none,
           d_net, kHid, none, dmo, motion, 2 * kHid, 126, {}, none, none);
  // ---- motion encoder (tail stream with the dense pyramid: it feeds only the pyramid and the
  // batched weight gradients, not the d net the earlier step waits for)
  auto dcorr = at::empty({P, kCorrPad}, hd.options());
  {
    c10::optional<c10::hip::HIPStreamGuard> g;
    if (ht != hm) {
      order(ht, hm);
      g.emplace(c10::hip::getStreamFromExternal(ht, dev));
      c10::hip::HIPCachingAllocator::recordStream(dcorr.storage().data_ptr(),
                                                  c10::hip::getStreamFromExternal(ht, dev));
    }
    dgrad(dmo, L_CONV, 3, 3, 256, dcf, cf);
    dgrad(dcf.narrow(1, 192, 64), L_CONVF2, 3, 3, 128, df1, f1);
    dgrad(dcf.narrow(1, 0, 192), L_CONVC2, 3, 3, 256, dc1, c1);
    dgrad(dc1, L_CONVC1, 1, 1, kCorrPad, dcorr, none);
  }
  return {d_net, dcorr};
}

// Host cost of the runtime pieces a training step is made of (scripts/launch_probe.py): mean
// microseconds per operation over n repetitions.  kind 0 / 1: kernel launch with an 8-byte /
// ConvFwdArgs-sized (sizeof = kind 1's bytes) argument block; 2: an event record + a wait on
// another stream (the fork / join of the update step); 3: at::empty of 1 MB.
double probe_host_cost(int64_t n, int64_t kind, int64_t other_stream) {
  const hipStream_t s = cur_stream();
  const hipStream_t o = other_stream ? reinterpret_cast<hipStream_t>(other_stream) : s;
  const auto opts = at::TensorOptions().device(at::kCUDA, c10::hip::current_device()).dtype(at::kFloat);
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t i = 0; i < n; ++i) {
    if (kind <= 1) {
      HIP_OK(launch_probe(static_cast<int>(kind), s));
    } else if (kind == 2) {
      step_exec::order(o, s);
    } else {
      auto t = at::empty({1 << 18}, opts);
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / std::max<int64_t>(n, 1);
}
}  // namespace
}  // namespace raft_amd

TORCH_LIBRARY(raft_amd, m) {
  m.def("instance_norm_fwd(Tensor x, bool relu, float eps) -> (Tensor, Tensor)");
  m.def("instance_norm_bwd(Tensor x, Tensor dy, Tensor stats, bool relu) -> Tensor");
  m.def(
      "conv_fwd(Tensor[] srcs, Tensor wt, int[] geom, int N, Tensor? bias, int epi, int act, float alpha, "
      "Tensor(a!) out, int acc_c0, Tensor? mask, Tensor? h, Tensor? z, Tensor(b!)? out2, int cfg=0, "
      "Tensor? g0=None, Tensor(c!)? carry=None, Tensor(d!)? out3=None, int gru_cols=0, Tensor? addsrc=None, "
      "Tensor(e!)? cout=None, Tensor? cmask=None, int cm_c0=0, int cm_valid=0, int[] split=[], Tensor? n2w=None, "
      "Tensor(f!)? n2y=None) -> ()");
  m.def("split_pack(Tensor src, Tensor(a!) dst, int G, int c0, int Cpad) -> ()");
  m.def("conv_wgrad(Tensor[] srcs, Tensor dy, int[] geom, int N, Tensor(a!) dw, Tensor(b!)? db, "
        "bool accumulate=True) -> ()");
  m.def("conv_wgrad_params(Tensor[] srcs, Tensor dy, int[] geom, Tensor(a!)[] wgrad, Tensor?[] bgrad, int[] segs, "
        "float scale, bool accumulate, bool fold=False) -> ()");
  m.def("pack_conv_weights_split(Tensor[] w, Tensor?[] b, int[] segs, float scale, int Kf, int Kd, int G_dy) -> "
        "(Tensor, Tensor?, Tensor)");
  m.def("pack_conv_weights_multi(Tensor[] w, Tensor?[] b, int[] nw, int[] segs, int[] nseg, float[] scale, "
        "int[] Kf, int[] Kd, int[] aux, bool f16=False, bool split=False) -> Tensor[]");
  m.def("pack_conv_weights(Tensor[] w, Tensor?[] b, int[] segs, float scale, int Kf, int Kd, int cout_pad, "
        "bool f16=False) -> "
        "(Tensor, Tensor?, Tensor)");
  m.def("gru_gates(Tensor zr, Tensor h) -> (Tensor, Tensor)");
  m.def("gru_gates_backward(Tensor zr, Tensor h, Tensor gz, Tensor grh) -> (Tensor, Tensor)");
  m.def("gru_blend(Tensor z, Tensor q, Tensor h) -> Tensor");
  m.def("gru_blend_backward(Tensor z, Tensor q, Tensor h, Tensor g) -> (Tensor, Tensor, Tensor)");
  m.def("gemm_nt(Tensor A, Tensor B, float alpha, ScalarType out_dtype) -> Tensor");
  m.def("avgpool2x2(Tensor x) -> Tensor");
  m.def("corr_lookup(Tensor[] pyramid, Tensor coords, int radius, ScalarType out_dtype, int out_channels=0) -> Tensor");
  m.def(
      "gru_bwd_a(Tensor dH, Tensor z, Tensor q, Tensor h, Tensor(a!) dq, Tensor(b!) dz, Tensor(c!) carry) -> ()");
  m.def("gru_bwd_b(Tensor(a!) drh, Tensor r, Tensor h, Tensor carry, Tensor(b!) dr) -> ()");
  m.def("masked_cast(Tensor src, Tensor? mask, Tensor(a!) out) -> ()");
  m.def("pack_flow(Tensor flow, Tensor(a!) flow8, Tensor(b!)? motion, bool from_coords=False) -> ()");
  m.def("apply_delta(Tensor coords1, Tensor delta, Tensor(a!) coords_out, Tensor(b!) flow_out) -> ()");
  m.def("n2_apply(Tensor y, Tensor bias, Tensor coords1, Tensor(a!) coords_out, Tensor(b!) flow_out, "
        "Tensor(c!)? delta=None) -> ()");
  m.def("launch_probe(int n, int kind, int other_stream=0) -> float", &raft_amd::probe_host_cost);  // no tensors: catch-all
  m.def("fused_step_fwd(Tensor[] bufs, Tensor[] wf, Tensor[] bias, Tensor[] levels, Tensor? corr_in, int[] cfg) "
        "-> Tensor[]");
  m.def("fused_step_bwd(Tensor[] bufs, Tensor[] wd, Tensor g_all, Tensor flow, Tensor? g_net, Tensor? g_flow_up, "
        "int[] cfg) -> Tensor[]");
  m.def(
      "corr_lookup_into(Tensor[] pyramid, Tensor coords, int radius, Tensor(a!) out, Tensor(b!)? flow8=None, "
      "Tensor(c!)? motion=None) -> ()");
  m.def("convex_upsample_backward_into(Tensor flow, Tensor mask, Tensor grad, Tensor(a!) dmask, Tensor(b!) rows) -> ()");
  m.def("corr_lookup_backward_(Tensor(a!)[] dpyramid, Tensor coords, Tensor grad, int radius) -> ()");
  m.def("corr_lookup_grad_rows(Tensor(a!) out, Tensor[] coords, Tensor[] grads, int[] segments, int radius, "
        "bool accumulate=False) -> ()");
  m.def(
      "corr_gemm(Tensor A, Tensor B, Tensor(a!) C, int M, int N, int K, int batch, int lda, int sA, int ldb, int sB, "
      "int ldc, int sC, float alpha, bool a_trans, bool split, int epi, int cfg=0) -> ()");
  m.def("corr_pyramid_bwd(Tensor dL, Tensor f2t, Tensor f1t, Tensor(a!) d1, Tensor(b!) G, float alpha) -> ()");
  m.def("pyramid_unpool(Tensor G, int H, int W, int[] segs, bool blocked=False) -> Tensor");
  m.def("pyramid_operand(Tensor fmap, int[] segs, int ld, bool blocked, bool nchw, bool bf16_out=False) -> Tensor");
  m.def("corr_lookup_split_into(Tensor[] pyramid, Tensor coords, int radius, Tensor(a!) out, int G, Tensor(b!)? flow8, "
        "Tensor(c!)? motion, int G_m) -> ()");
  m.def("convex_upsample(Tensor flow, Tensor mask) -> Tensor");
  m.def("convex_upsample_backward(Tensor flow, Tensor mask, Tensor grad) -> (Tensor, Tensor)");
  m.def("seq_loss(Tensor[] preds, Tensor gt, Tensor valid, float gamma, float max_flow) -> Tensor");
  m.def(
      "seq_loss_backward(Tensor[] preds, Tensor gt, Tensor valid, Tensor dloss, float gamma, float "
      "max_flow) -> Tensor[]");
  m.def("local_corr(Tensor fmap1, Tensor fmap2, Tensor coords, int radius, float scale) -> Tensor");
  m.def("local_corr_mfma(Tensor f1, Tensor f2, Tensor coords, int[] segs, int radius, float scale, Tensor(a!) out) -> ()");
  m.def(
      "local_corr_mfma_backward(Tensor f1, Tensor f2, Tensor coords, int[] segs, int radius, float scale, Tensor gout, "
      "Tensor(a!) g1, Tensor(b!) g2, bool deterministic=False) -> ()");
  m.def(
      "local_corr_backward(Tensor fmap1, Tensor fmap2, Tensor coords, Tensor grad, int radius, float "
      "scale, bool deterministic=False) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(raft_amd, CUDA, m) {
  m.impl("gemm_nt", &raft_amd::gemm_nt);
  m.impl("avgpool2x2", &raft_amd::avgpool2x2);
  m.impl("corr_lookup", &raft_amd::corr_lookup);
  m.impl("corr_lookup_backward_", &raft_amd::corr_lookup_backward_);
  m.impl("corr_lookup_grad_rows", &raft_amd::corr_lookup_grad_rows);
  m.impl("corr_gemm", &raft_amd::corr_gemm);
  m.impl("corr_pyramid_bwd", &raft_amd::corr_pyramid_bwd);
  m.impl("pyramid_unpool", &raft_amd::pyramid_unpool);
  m.impl("convex_upsample", &raft_amd::convex_upsample);
  m.impl("pyramid_operand", &raft_amd::pyramid_operand);
  m.impl("convex_upsample_backward", &raft_amd::convex_upsample_backward);
  m.impl("seq_loss", &raft_amd::seq_loss);
  m.impl("seq_loss_backward", &raft_amd::seq_loss_backward);
  m.impl("local_corr", &raft_amd::local_corr);
  m.impl("local_corr_mfma", &raft_amd::local_corr_mfma);
  m.impl("local_corr_mfma_backward", &raft_amd::local_corr_mfma_backward);
  m.impl("local_corr_backward", &raft_amd::local_corr_backward);
  m.impl("conv_fwd", &raft_amd::conv_fwd);
  m.impl("instance_norm_fwd", &raft_amd::instance_norm_fwd);
  m.impl("instance_norm_bwd", &raft_amd::instance_norm_bwd);
  m.impl("gru_bwd_a", &raft_amd::gru_bwd_a);
  m.impl("gru_bwd_b", &raft_amd::gru_bwd_b);
  m.impl("masked_cast", &raft_amd::masked_cast);
  m.impl("pack_flow", &raft_amd::pack_flow);
  m.impl("split_pack", &raft_amd::split_pack);
  m.impl("apply_delta", &raft_amd::apply_delta);
  m.impl("n2_apply", &raft_amd::n2_apply);
  m.impl("fused_step_fwd", &raft_amd::fused_step_fwd);
  m.impl("fused_step_bwd", &raft_amd::fused_step_bwd);
  m.impl("corr_lookup_into", &raft_amd::corr_lookup_into);
  m.impl("convex_upsample_backward_into", &raft_amd::convex_upsample_backward_into);
  m.impl("conv_wgrad", &raft_amd::conv_wgrad);
  m.impl("conv_wgrad_params", &raft_amd::conv_wgrad_params);
  m.impl("pack_conv_weights", &raft_amd::pack_conv_weights);
  m.impl("pack_conv_weights_multi", &raft_amd::pack_conv_weights_multi);
  m.impl("pack_conv_weights_split", &raft_amd::pack_conv_weights_split);
  m.impl("corr_lookup_split_into", &raft_amd::corr_lookup_split_into);
  m.impl("gru_gates", &raft_amd::gru_gates);
  m.impl("gru_gates_backward", &raft_amd::gru_gates_backward);
  m.impl("gru_blend", &raft_amd::gru_blend);
  m.impl("gru_blend_backward", &raft_amd::gru_blend_backward);
}
