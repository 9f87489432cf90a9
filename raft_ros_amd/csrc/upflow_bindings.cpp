// Torch ops for the bilinear 8x flow upsampler (csrc/upflow8.hip); autograd in ops/upsample.py.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>

namespace raft_amd {

hipError_t launch_upflow8_fwd(const float* flow, float* out, int B, int H, int W, hipStream_t s);
hipError_t launch_upflow8_bwd(const float* g, float* dflow, void* rows, int rows_ld, int B, int H, int W,
                              hipStream_t s);

namespace {
void check_flow(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 4 && t.size(1) == 2 && t.is_contiguous(),
              "raft_amd::upflow8: ", name, " must be a contiguous fp32 (B, 2, H, W) CUDA tensor");
}
hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
}  // namespace

at::Tensor upflow8(const at::Tensor& flow) {
  check_flow(flow, "flow");
  const int B = (int)flow.size(0), H = (int)flow.size(2), W = (int)flow.size(3);
  at::Tensor out = at::empty({B, 2, 8L * H, 8L * W}, flow.options());
  TORCH_CHECK(launch_upflow8_fwd(flow.data_ptr<float>(), out.data_ptr<float>(), B, H, W, stream()) == hipSuccess,
              "upflow8 launch failed");
  return out;
}

// dflow (B, 2, H, W) fp32 of d out; rows (optional, (B*H*W, C>=2) bf16): [du, dv, 0...] pixel rows
at::Tensor upflow8_backward(const at::Tensor& grad, int64_t H, int64_t W, const c10::optional<at::Tensor>& rows) {
  check_flow(grad, "grad");
  const int B = (int)grad.size(0);
  TORCH_CHECK(grad.size(2) == 8 * H && grad.size(3) == 8 * W, "upflow8_backward: grad must be (B, 2, 8H, 8W)");
  at::Tensor dflow = at::empty({B, 2, H, W}, grad.options());
  void* rp = nullptr;
  int ld = 0;
  if (rows.has_value() && rows->defined()) {
    TORCH_CHECK(rows->scalar_type() == at::kBFloat16 && rows->dim() == 2 && rows->size(0) == (long)B * H * W &&
                    rows->size(1) >= 2 && rows->stride(1) == 1 && rows->stride(0) == rows->size(1),
                "upflow8_backward: rows must be a contiguous (B*H*W, C>=2) bf16 tensor");
    rp = rows->data_ptr();
    ld = (int)rows->size(1);
  }
  TORCH_CHECK(launch_upflow8_bwd(grad.data_ptr<float>(), dflow.data_ptr<float>(), rp, ld, B, (int)H, (int)W,
                                 stream()) == hipSuccess,
              "upflow8_backward launch failed");
  return dflow;
}

}  // namespace raft_amd

TORCH_LIBRARY_FRAGMENT(raft_amd, m) {
  m.def("upflow8(Tensor flow) -> Tensor");
  m.def("upflow8_backward(Tensor grad, int H, int W, Tensor(a!)? rows) -> Tensor");
}

TORCH_LIBRARY_IMPL(raft_amd, CUDA, m) {
  m.impl("upflow8", &raft_amd::upflow8);
  m.impl("upflow8_backward", &raft_amd::upflow8_backward);
}
