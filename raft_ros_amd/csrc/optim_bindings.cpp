// Torch binding of the two-launch clip + AdamW step (csrc/optim.hip; Python side
// raft_ros_amd/ops/optim.py ClipAdamW).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <vector>

#include <hip/hip_runtime.h>

#include "kernel_abi.h"

namespace raft_amd {

namespace {

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "raft_amd::", what, ": ", hipGetErrorString(e));
}

// params / grads: the parameter set in table order; ptrs [n][3] int64 and blocks [nb][3] int32
// device tables (ops/optim.py builds them once per parameter set); tblk: first block of every
// tensor, plus the total.
void clip_adamw_(at::TensorList params, at::TensorList grads, const at::Tensor& ptrs, const at::Tensor& blocks,
                 at::IntArrayRef tblk, const at::Tensor& partial, const at::Tensor& steps, int64_t par, double lr,
                 double beta1, double beta2, double eps, double wd, double max_norm,
                 const c10::optional<at::Tensor>& norm_out, const c10::optional<at::Tensor>& skipped) {
  const long n = (long)params.size();
  TORCH_CHECK(n > 0 && (long)grads.size() == n && (long)tblk.size() == n + 1, "raft_amd::clip_adamw_: sizes");
  TORCH_CHECK(ptrs.is_cuda() && ptrs.scalar_type() == at::kLong && ptrs.numel() == 3 * n, "raft_amd::clip_adamw_: ptrs");
  const long nb = tblk[n];
  TORCH_CHECK(blocks.is_cuda() && blocks.scalar_type() == at::kInt && blocks.numel() == 3 * nb,
              "raft_amd::clip_adamw_: blocks");
  TORCH_CHECK(partial.is_cuda() && partial.scalar_type() == at::kFloat && partial.numel() >= nb,
              "raft_amd::clip_adamw_: partial");
  TORCH_CHECK(steps.is_cuda() && steps.scalar_type() == at::kFloat && steps.numel() == 2 && (par == 0 || par == 1),
              "raft_amd::clip_adamw_: steps");
  for (const auto* o : {&norm_out, &skipped})
    TORCH_CHECK(!o->has_value() || ((*o)->is_cuda() && (*o)->scalar_type() == at::kFloat && (*o)->numel() == 1),
                "raft_amd::clip_adamw_: norm_out / skipped must be one-element fp32 device tensors");
  for (long i = 0; i < n; ++i) {
    const at::Tensor& p = params[i];
    const at::Tensor& g = grads[i];
    // the kernels walk the raw storage: the gradient must have the parameter's exact layout
    TORCH_CHECK(g.defined() && g.is_cuda() && g.scalar_type() == at::kFloat && p.scalar_type() == at::kFloat &&
                    g.sizes() == p.sizes() && g.strides() == p.strides() && p.is_non_overlapping_and_dense(),
                "raft_amd::clip_adamw_: gradient ", i, " must be a dense fp32 tensor in its parameter's layout");
    TORCH_CHECK(tblk[i + 1] - tblk[i] == (p.numel() + kAdamChunk - 1) / kAdamChunk, "raft_amd::clip_adamw_: block table");
  }
  const c10::DeviceGuard guard(params[0].device());
  hipStream_t s = c10::hip::getCurrentHIPStream().stream();
  AdamArgs a{};
  a.ptrs = reinterpret_cast<const long long*>(ptrs.data_ptr<int64_t>());
  a.blocks = blocks.data_ptr<int>();
  a.nblocks = (int)nb;
  a.partial = partial.data_ptr<float>();
  a.steps = steps.data_ptr<float>();
  a.par = (int)par;
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps; a.wd = (float)wd;
  a.max_norm = (float)max_norm;
  a.norm_out = norm_out.has_value() ? norm_out->data_ptr<float>() : nullptr;
  a.skipped = skipped.has_value() ? skipped->data_ptr<float>() : nullptr;
  for (int pass = 0; pass < 2; ++pass) {  // every partial before any update
    for (long t0 = 0; t0 < n; t0 += kAdamGrads) {
      const long t1 = std::min(n, t0 + (long)kAdamGrads);
      a.t0 = (int)t0;
      for (long t = t0; t < t1; ++t) a.g[t - t0] = grads[t].data_ptr<float>();
      a.blk0 = (int)tblk[t0];
      hip_check(launch_adamw(a, (int)(tblk[t1] - tblk[t0]), pass == 1, s), "clip_adamw_");
    }
  }
}

}  // namespace

}  // namespace raft_amd

TORCH_LIBRARY_FRAGMENT(raft_amd, m) {
  m.def("clip_adamw_(Tensor(a!)[] params, Tensor[] grads, Tensor ptrs, Tensor blocks, int[] tblk, Tensor(b!) partial, "
        "Tensor(c!) steps, int par, float lr, float beta1, float beta2, float eps, float wd, float max_norm, "
        "Tensor(d!)? norm_out=None, Tensor(e!)? skipped=None) -> ()");
}

TORCH_LIBRARY_IMPL(raft_amd, CUDA, m) { m.impl("clip_adamw_", &raft_amd::clip_adamw_); }
