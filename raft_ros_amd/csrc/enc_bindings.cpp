// Torch dispatcher ops for the native encoders (csrc/encoder.hip): host-side planning
// of the strided implicit-GEMM convolutions (K-chunk decode tables, stride-parity
// classes of the data gradient, pixel splits of the weight gradient) and the norm ops.
// Autograd wiring: raft_ros_amd/ops/encoder.py.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include <hip/hip_runtime.h>

#include "kernel_abi.h"

namespace raft_amd {


namespace {

constexpr int kBM = 128;  // conv M tile (pixels), fixed for every encoder conv
constexpr int kNormChunks = 64;
// chunking of the norm-backward reduction (experiments: RAFT_NORM_R / RAFT_NORM_PIX)
int norm_chunks_max() {
  static const int v = [] {
    const char* e = std::getenv("RAFT_NORM_R");
    return e ? std::max(1, std::atoi(e)) : kNormChunks;
  }();
  return v;
}
int norm_chunk_pixels() {
  static const int v = [] {
    const char* e = std::getenv("RAFT_NORM_PIX");
    return e ? std::max(16, std::atoi(e)) : 256;
  }();
  return v;
}

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

// activations are bf16, or fp16 under fp16 AMP (EncConvArgs::f16)
bool is16(const at::Tensor& t) { return t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf; }

void check_nhwc(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && is16(t) && t.dim() == 4 && t.is_contiguous(), name,
              ": expected a contiguous [B, H, W, C] bf16 / fp16 CUDA tensor");
  TORCH_CHECK(t.size(3) % 8 == 0, name, ": channels must be a multiple of 8");
  TORCH_CHECK(t.numel() < (1L << 31), name, ": too large");
}

void check_w(const at::Tensor& w, const char* name) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4, name, ": expected a fp32 4-D CUDA weight");
}

int round_up(long v, int m) { return (int)((v + m - 1) / m * m); }

// typed views of bf16 tensor storage for the kernel argument structs
const __bf16* cbf(const at::Tensor& t) { return static_cast<const __bf16*>(t.data_ptr()); }
__bf16* mbf(const at::Tensor& t) { return static_cast<__bf16*>(t.data_ptr()); }

int enc_tab_entry(int dy, int dx, int src, int c) {
  TORCH_CHECK(dy > -128 && dy < 128 && dx > -128 && dx < 128 && c < (1 << 14), "decode table range");
  return (dy + 128) | ((dx + 128) << 8) | (src << 16) | (c << 17);
}
int enc_ptab_entry(int w, int ky, int kx, int local) {
  TORCH_CHECK(ky < 16 && kx < 16, "kernel size");
  return w | (ky << 4) | (kx << 8) | (local << 12);
}

void set_weight(EncConvArgs& a, int j, const at::Tensor& w) {
  a.w[j] = w.data_ptr<float>();
  for (int d = 0; d < 4; ++d) a.ws[j][d] = w.stride(d);
  a.wcin[j] = (int)w.size(1);
}

// Packed-weight layout of a planned launch: per class, rows x Kpad (returns the total; sets the
// classes' weight offsets and block ranges).
long pack_layout(EncConvArgs& a, int rows, int& blocks) {
  long wtotal = 0;
  blocks = 0;
  a.tilesN = (a.N + enc_tile_bn(a.N) - 1) / enc_tile_bn(a.N);
  for (int c = 0; c < a.ncls; ++c) {
    EncClass& cl = a.cls[c];
    cl.wofs = wtotal;
    wtotal += (long)rows * cl.Kpad;
    cl.tiles_img = (cl.Gh * cl.Gw + kBM - 1) / kBM;
    cl.blk0 = blocks;
    blocks += a.B * cl.tiles_img * a.tilesN;
  }
  return wtotal;
}

// Pack + run one planned conv launch (fwd or dgrad); classes and tables already filled.
// ``prepacked``: the weights packed earlier by enc_pack_fwd / enc_pack_dgrad (same layout; the
// packing launches then run off the encoder's critical path, ops/encoder.py).
void run_conv(EncConvArgs& a, int rows, const at::TensorOptions& o,
              const c10::optional<at::Tensor>& prepacked = c10::nullopt) {
  int blocks = 0;
  const long wtotal = pack_layout(a, rows, blocks);
  at::Tensor wt;
  if (prepacked.has_value() && prepacked->defined()) {
    TORCH_CHECK(prepacked->numel() == wtotal && prepacked->is_contiguous() && is16(*prepacked),
                "enc conv: prepacked weights do not match the launch's packed layout");
    a.wt = cbf(*prepacked);
  } else {
    wt = at::empty({wtotal}, o.dtype(at::kBFloat16));
    a.wt = cbf(wt);
    check(launch_enc_pack(a, rows, wt.data_ptr(), stream()), "enc_pack");
  }
  if (blocks == 0) return;
  if (enc_conv3_eligible(a))
    check(launch_enc_conv3(a, stream()), "enc_conv3");  // 3x3 64 -> 64: resident-weight kernel
  else
    check(launch_enc_conv(a, blocks, stream()), "enc_conv");
}

// Decode / packing tables too deep for the kernel arguments (the split-bf16 layout's 3x
// channels): one device copy per distinct table, built on first use (so a HIP-graph capture
// must follow a warm-up forward, as GraphedRAFT's does).  The cache is a leaked heap object:
// its device tensors must not be freed by static destructors after the HIP runtime is gone.
const int* device_tables(const std::vector<int>& tab, const std::vector<int>& ptab, int device,
                         const at::TensorOptions& o) {
  using Key = std::pair<int, std::vector<int>>;
  static auto* cache = new std::map<Key, at::Tensor>();
  static auto* mu = new std::mutex();
  std::lock_guard<std::mutex> lock(*mu);
  std::vector<int> both(tab);
  both.insert(both.end(), ptab.begin(), ptab.end());
  Key key{device, both};
  auto it = cache->find(key);
  if (it == cache->end()) {
    at::Tensor host = at::from_blob(both.data(), {(long)both.size()}, at::TensorOptions().dtype(at::kInt)).clone();
    it = cache->emplace(std::move(key), host.to(o.dtype(at::kInt))).first;
  }
  return it->second.data_ptr<int>();
}

// Fill the decode / packing tables of a launch: inline when they fit the arguments, else the
// device copies (tables of kEncTabMax entries, -1 = zero columns)
void set_tables(EncConvArgs& a, const std::vector<int>& tab, const std::vector<int>& ptab, int used, int device,
                const at::TensorOptions& o) {
  TORCH_CHECK(used <= kEncTabMax, "conv too deep for the decode table");
  if (used <= kEncTab) {
    std::copy(tab.begin(), tab.begin() + kEncTab, a.tab);
    std::copy(ptab.begin(), ptab.begin() + kEncTab, a.ptab);
  } else {
    const int* dt = device_tables(tab, ptab, device, o);
    a.tab_ptr = dt;
    a.ptab_ptr = dt + kEncTabMax;
  }
}

void init_args(EncConvArgs& a) {
  std::memset(&a, 0, sizeof(a));
  for (int i = 0; i < kEncTab; ++i) a.tab[i] = a.ptab[i] = -1;
}

}  // namespace

namespace {
// decode / packing tables of a KHxKW conv over Cx input channels (one class); returns Kpad.
// split == 2 (three-plane fp32 forward): x rows hold [hi | mid | lo] planes of cx = Cx / 3
// channels and the GEMM runs over SIX K planes -- x planes hi, mid, hi, lo, hi, mid against the
// weight planes H, H, M, H, L, M packed by enc_pack (encoder.hip pack_row) -- i.e. every
// product hi(x) H + mid H + hi M + lo H + hi L + mid M down to ~2^-24 of x W: the fp32 conv.
int fwd_tables(EncConvArgs& a, int Cx, int KH, int KW, int pad, int device, const at::TensorOptions& o,
               int split = 0) {
  std::vector<int> tab(kEncTabMax, -1), ptab(kEncTabMax, -1);
  int e = 0;
  static const int kXPlane[6] = {0, 1, 0, 2, 0, 1};
  const int cx = Cx / 3, nk = split == 2 ? 2 * Cx : Cx;
  for (int ky = 0; ky < KH; ++ky)
    for (int kx = 0; kx < KW; ++kx)
      for (int c = 0; c < nk; c += 8) {
        TORCH_CHECK(e < kEncTabMax, "conv too deep for the decode table");
        const int src_c = split == 2 ? kXPlane[c / cx] * cx + c % cx : c;
        tab[e] = enc_tab_entry(ky - pad, kx - pad, 0, src_c);
        ptab[e] = enc_ptab_entry(0, ky, kx, c);
        ++e;
      }
  const int K = e * 8, Kpad = round_up(K, 64);
  set_tables(a, tab, ptab, Kpad / 8, device, o);
  a.cls[0] = EncClass{0, 1, 1, 0, 0, K, Kpad, 0, 0, 0};
  a.ncls = 1;
  return Kpad;
}
}  // namespace

// A packing job as bytes of its EncConvArgs, with its packed size and workgroup count
std::tuple<at::Tensor, int64_t, int64_t> job_bytes(EncConvArgs& a, int rows) {
  int blocks = 0;
  const long wtotal = pack_layout(a, rows, blocks);
  at::Tensor t = at::empty({(long)sizeof(EncConvArgs)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &a, sizeof(EncConvArgs));
  return {t, wtotal, (int64_t)rows * a.ncls};
}

// The forward weight operand of enc_conv_fwd for an input of Cx channels as a packing job of
// enc_pack_multi (the layout run_conv would pack: N rows of round_up(KH*KW*Cx, 64))
std::tuple<at::Tensor, int64_t, int64_t> enc_pack_fwd_job(const at::Tensor& w, int64_t Cx, int64_t pad, int64_t split,
                                                          bool f16) {
  check_w(w, "w");
  TORCH_CHECK(split >= 0 && split <= 2, "split mode 0 / 1 / 2");
  EncConvArgs a;
  init_args(a);
  a.f16 = f16 ? 1 : 0;
  a.B = 1;
  a.N = (int)w.size(0);
  fwd_tables(a, (int)Cx, (int)w.size(2), (int)w.size(3), (int)pad, w.get_device(), w.options(), (int)split);
  a.split = (int)split;
  a.split_w = split ? (int)Cx / 3 : 0;
  set_weight(a, 0, w);
  a.pack_dgrad = 0;
  return job_bytes(a, a.N);
}

// Pack the jobs of ``plan`` (device bytes: the jobs' EncConvArgs, their output offsets, their
// first workgroups) into ``out`` with one launch
void enc_pack_multi(const at::Tensor& plan, int64_t njobs, int64_t nblocks, at::Tensor out) {
  TORCH_CHECK(plan.is_cuda() && plan.scalar_type() == at::kByte && plan.is_contiguous() &&
                  plan.numel() >= njobs * (long)(sizeof(EncConvArgs) + sizeof(long) + sizeof(int)) + 4,
              "enc_pack_multi: plan bytes");
  TORCH_CHECK(out.is_cuda() && is16(out) && out.is_contiguous(), "enc_pack_multi: out");
  if (njobs == 0 || nblocks == 0) return;
  check(launch_enc_pack_multi(plan.data_ptr(), (int)njobs, (int)nblocks, out.data_ptr(), stream()), "enc_pack_multi");
}

// y[B,Ho,Wo,N] = conv(x[B,H,W,Cx], w[N,Cin,KH,KW]) + bias; stats [B, T, 2, N] (column sum, M2 per 128-pixel tile)
std::tuple<at::Tensor, at::Tensor> enc_conv_fwd(const at::Tensor& x, const at::Tensor& w,
                                                const c10::optional<at::Tensor>& bias, int64_t stride, int64_t pad,
                                                bool want_stats, int64_t split,
                                                const c10::optional<at::Tensor>& prepacked) {
  check_nhwc(x, "x");
  check_w(w, "w");
  TORCH_CHECK(split >= 0 && split <= 2, "split mode 0 / 1 / 2");
  const int B = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), Cx = (int)x.size(3);
  const int N = (int)w.size(0), Cin = (int)w.size(1), KH = (int)w.size(2), KW = (int)w.size(3);
  TORCH_CHECK(Cin <= (split ? Cx / 3 : Cx), "weight has more input channels than x");
  TORCH_CHECK(!split || Cx % 3 == 0, "split x must hold three planes");
  TORCH_CHECK(N % 8 == 0 && N <= 1024, "out channels");
  TORCH_CHECK(!split || x.scalar_type() == at::kBFloat16, "split planes are bf16");
  const int Ho = (H + 2 * (int)pad - KH) / (int)stride + 1, Wo = (W + 2 * (int)pad - KW) / (int)stride + 1;
  EncConvArgs a;
  init_args(a);
  a.f16 = x.scalar_type() == at::kHalf ? 1 : 0;
  a.src[0] = {cbf(x), Cx, Cx, H, W, (int)stride};
  a.B = B;
  a.N = N;
  fwd_tables(a, Cx, KH, KW, (int)pad, x.get_device(), x.options(), (int)split);
  a.cls[0].Gh = Ho;
  a.cls[0].Gw = Wo;
  at::Tensor y = at::empty({B, Ho, Wo, split ? 3 * N : N}, x.options());
  a.Ho = Ho;
  a.Wo = Wo;
  a.os = 1;
  a.out = mbf(y);
  a.out_stride = split ? 3 * N : N;
  a.split = (int)split;
  a.split_w = split ? Cx / 3 : 0;  // the fp32 weight is split while packing
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(at::kFloat).contiguous();
    a.bias = b.data_ptr<float>();
  }
  // tile statistics: [B, T, 2, N] over 128-pixel row tiles, or [B, Ty, Tx, 2, N] over the
  // square tiles of the resident-weight 3x3 kernel (enc_norm_stats reads the layout from the rank)
  at::Tensor st;
  if (want_stats) {
    const auto fo = x.options().dtype(at::kFloat);
    if (enc_conv3_eligible(a))
      st = at::empty({B, (Ho + kEnc3Tile - 1) / kEnc3Tile, (Wo + kEnc3Tile - 1) / kEnc3Tile, 2, N}, fo);
    else
      st = at::empty({B, (Ho * Wo + kBM - 1) / kBM, 2, N}, fo);
  }
  if (want_stats) a.stats = st.data_ptr<float>();
  set_weight(a, 0, w);
  a.pack_dgrad = 0;
  run_conv(a, N, x.options(), prepacked);
  return {y, st};
}

// dx[B,H,W,Cin] = sum_j conv_transpose(dys[j], ws[j]) (+ res) (* [mask > 0]);
// stride[j] / pad[j] per conv, every conv maps x[B,H,W,Cin] -> dys[j].
//
// split (fp32 training): dys are split rows [hi | lo | hi] of 3 Cout channels, the weights are
// packed [W_hi | W_hi | W_lo] along Cout, dx (and res) are split rows of 3 Cin, the ReLU' mask
// is read from the hi plane of split rows.
namespace {
// decode / packing tables of a dgrad launch: one class per output phase (py, px) of the largest
// stride S, each gathering the taps of every conv that land on that phase (C[j]: dy channels)
// split == 2: the dY rows hold [hi | mid | lo] planes (store8_split mode 2); the K plane that
// pairs with W_lo must read hi, so its decode entries point at plane 0 instead of plane 2
void dgrad_tables(EncConvArgs& a, at::TensorList ws, const std::vector<int>& C, at::IntArrayRef strides,
                  at::IntArrayRef pads, int H, int W, int S, int device, const at::TensorOptions& o,
                  int split = 0) {
  const int nconv = (int)ws.size();
  std::vector<int> tab(kEncTabMax, -1), ptab(kEncTabMax, -1);
  int e = 0, ncls = 0;
  for (int py = 0; py < S; ++py)
    for (int px = 0; px < S; ++px) {
      const int Gh = (H - py + S - 1) / S, Gw = (W - px + S - 1) / S;
      if (Gh <= 0 || Gw <= 0) continue;
      const int t0 = e;
      for (int j = 0; j < nconv; ++j) {
        const int s = (int)strides[j], p = (int)pads[j];
        const int KH = (int)ws[j].size(2), KW = (int)ws[j].size(3);
        for (int ky = 0; ky < KH; ++ky) {
          const int vy = py + p - ky;
          if (((vy % s) + s) % s) continue;
          for (int kx = 0; kx < KW; ++kx) {
            const int vx = px + p - kx;
            if (((vx % s) + s) % s) continue;
            const int co = C[j] / 3;  // split: Cout of conv j
            for (int c = 0; c < C[j]; c += 8) {
              TORCH_CHECK(e < kEncTabMax, "dgrad too deep for the decode table");
              const int src_c = (split == 2 && c >= 2 * co) ? c - 2 * co : c;
              tab[e] = enc_tab_entry(vy / s, vx / s, j, src_c);
              ptab[e] = enc_ptab_entry(j, ky, kx, c);
              ++e;
            }
          }
        }
      }
      const int K = (e - t0) * 8, Kpad = std::max(64, round_up(K, 64));
      TORCH_CHECK(t0 + Kpad / 8 <= kEncTabMax, "dgrad too deep for the decode table");
      e = t0 + Kpad / 8;  // padded entries stay -1
      a.cls[ncls++] = EncClass{t0, Gh, Gw, py, px, K, Kpad, 0, 0, 0};
    }
  a.ncls = ncls;
  set_tables(a, tab, ptab, e, device, o);
}

int largest_stride(at::IntArrayRef strides) {
  int S = 1;
  for (auto s : strides) S = std::max<int>(S, (int)s);
  for (auto s : strides) TORCH_CHECK(S % s == 0, "strides must divide the largest stride");
  return S;
}
}  // namespace

// The dgrad weight operand of enc_conv_dgrad (convs ws over an H x W input) as a packing job of
// enc_pack_multi: the weights do not change between the forward and the optimizer step
std::tuple<at::Tensor, int64_t, int64_t> enc_pack_dgrad_job(at::TensorList ws, at::IntArrayRef strides,
                                                            at::IntArrayRef pads, int64_t H, int64_t W, int64_t split,
                                                            bool f16) {
  const int nconv = (int)ws.size();
  TORCH_CHECK(nconv >= 1 && nconv <= 2 && (int)strides.size() == nconv && (int)pads.size() == nconv,
              "enc_pack_dgrad_job: 1 or 2 convs");
  const int Cin = (int)ws[0].size(1);
  EncConvArgs a;
  init_args(a);
  a.B = 1;
  a.N = Cin;
  a.f16 = f16 ? 1 : 0;
  std::vector<int> C(nconv);
  for (int j = 0; j < nconv; ++j) {
    check_w(ws[j], "w");
    TORCH_CHECK(ws[j].size(1) == Cin, "dgrad shapes");
    C[j] = (split ? 3 : 1) * (int)ws[j].size(0);
    set_weight(a, j, ws[j]);
  }
  dgrad_tables(a, ws, C, strides, pads, (int)H, (int)W, largest_stride(strides), ws[0].get_device(), ws[0].options(),
               (int)split);
  a.split = (int)split;
  a.split_w = split ? (int)ws[0].size(0) : 0;
  for (int j = 0; j < nconv; ++j) a.split_wd[j] = split ? (int)ws[j].size(0) : 0;
  a.pack_dgrad = 1;
  return job_bytes(a, Cin);
}

at::Tensor enc_conv_dgrad(at::TensorList dys, at::TensorList ws, at::IntArrayRef strides, at::IntArrayRef pads,
                          int64_t H, int64_t W, const c10::optional<at::Tensor>& res,
                          const c10::optional<at::Tensor>& mask, int64_t split,
                          const c10::optional<at::Tensor>& prepacked) {
  const int nconv = (int)dys.size();
  TORCH_CHECK(nconv >= 1 && nconv <= 2 && (int)ws.size() == nconv && (int)strides.size() == nconv &&
                  (int)pads.size() == nconv,
              "enc_conv_dgrad: 1 or 2 convs");
  const int B = (int)dys[0].size(0);
  const int Cin = (int)ws[0].size(1);
  TORCH_CHECK(Cin % 8 == 0 && Cin <= 1024, "in channels");
  const int S = largest_stride(strides);
  EncConvArgs a;
  init_args(a);
  a.B = B;
  a.N = Cin;
  a.f16 = dys[0].scalar_type() == at::kHalf ? 1 : 0;
  TORCH_CHECK(!split || !a.f16, "split planes are bf16");
  std::vector<int> Cs(nconv);
  for (int j = 0; j < nconv; ++j) {
    check_nhwc(dys[j], "dy");
    TORCH_CHECK(dys[j].scalar_type() == dys[0].scalar_type(), "dgrad: dys share one dtype");
    check_w(ws[j], "w");
    TORCH_CHECK(dys[j].size(0) == B && ws[j].size(1) == Cin && dys[j].size(3) == (split ? 3 : 1) * ws[j].size(0),
                "dgrad shapes");
    const int KH = (int)ws[j].size(2), KW = (int)ws[j].size(3);
    const int Ho = ((int)H + 2 * (int)pads[j] - KH) / (int)strides[j] + 1;
    const int Wo = ((int)W + 2 * (int)pads[j] - KW) / (int)strides[j] + 1;
    TORCH_CHECK(dys[j].size(1) == Ho && dys[j].size(2) == Wo, "dy spatial shape does not match the conv");
    const int C = (int)dys[j].size(3);
    a.src[j] = {cbf(dys[j]), C, C, Ho, Wo, S / (int)strides[j]};
    Cs[j] = C;
    set_weight(a, j, ws[j]);
  }
  dgrad_tables(a, ws, Cs, strides, pads, (int)H, (int)W, S, dys[0].get_device(), dys[0].options(), (int)split);
  const int rs = split ? 3 * Cin : Cin;  // dx / res / mask row pitch
  at::Tensor dx = at::empty({B, H, W, rs}, dys[0].options());
  a.Ho = (int)H;
  a.Wo = (int)W;
  a.os = S;
  a.out = mbf(dx);
  a.out_stride = rs;
  a.split = (int)split;
  a.split_w = split ? (int)ws[0].size(0) : 0;
  for (int j = 0; j < nconv; ++j) a.split_wd[j] = split ? (int)ws[j].size(0) : 0;
  if (res.has_value() && res->defined()) {
    check_nhwc(*res, "res");
    TORCH_CHECK(res->sizes() == dx.sizes() && res->scalar_type() == dx.scalar_type(), "res shape / dtype");
    a.res = cbf(*res);
    a.res_stride = rs;
  }
  if (mask.has_value() && mask->defined()) {
    check_nhwc(*mask, "mask");
    TORCH_CHECK(mask->sizes() == dx.sizes() && mask->scalar_type() == dx.scalar_type(), "mask shape / dtype");
    a.mask = cbf(*mask);
    a.mask_stride = rs;
  }
  a.pack_dgrad = 1;
  run_conv(a, Cin, dys[0].options(), prepacked);
  return dx;
}

// dw (fp32, any strides, [Cout, Cin, KH, KW]) (+)= wgrad; db (+)= sum_p dy
// x and dy may be channel slices of NHWC rows (a split tensor's [hi | lo] or hi planes):
// unit channel stride, pixel pitch stride(2), rows of one image contiguous in pitch.
void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && is16(t) && t.dim() == 4 && t.stride(3) == 1, name,
              ": expected [B, H, W, C] bf16 / fp16 rows with unit channel stride");
  TORCH_CHECK(t.size(3) % 8 == 0 && t.stride(2) % 8 == 0 && t.stride(2) >= t.size(3) &&
                  t.stride(1) == t.size(2) * t.stride(2) && t.stride(0) == t.size(1) * t.stride(1) &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, ": channel slice of contiguous NHWC rows (channels and pitch multiples of 8, 16-byte aligned)");
  TORCH_CHECK(t.size(0) * t.stride(0) < (1L << 31), name, ": too large");
}

// fold > 0 (split-bf16 training): x = [hi | lo] planes of ``fold`` channels each; the gradient of
// the fp32 parameter is the sum of the hi- and lo-plane columns (folded in the reduction)
void enc_conv_wgrad(const at::Tensor& x, const at::Tensor& dy, at::Tensor dw, const c10::optional<at::Tensor>& db,
                    int64_t stride, int64_t pad, bool accumulate, bool db_zero, int64_t fold) {
  check_rows(x, "x");
  check_rows(dy, "dy");
  const int xpitch = (int)x.stride(2), dypitch = (int)dy.stride(2);
  TORCH_CHECK(x.scalar_type() == dy.scalar_type(), "wgrad: x and dy share one dtype");
  const int f16 = x.scalar_type() == at::kHalf ? 1 : 0;
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat && dw.dim() == 4, "dw: fp32 4-D");
  const int B = (int)x.size(0), Hx = (int)x.size(1), Wx = (int)x.size(2), Cx = (int)x.size(3);
  const int N = (int)dw.size(0), Cin = (int)dw.size(1), KH = (int)dw.size(2), KW = (int)dw.size(3);
  const int Ho = (int)dy.size(1), Wo = (int)dy.size(2);
  TORCH_CHECK(dy.size(0) == B && dy.size(3) == N && Cin <= (fold > 0 ? fold : Cx), "wgrad shapes");
  TORCH_CHECK(fold == 0 || (fold % 8 == 0 && Cx == 2 * fold), "wgrad fold: x holds two planes of fold channels");
  TORCH_CHECK(Ho == (Hx + 2 * (int)pad - KH) / (int)stride + 1 && Wo == (Wx + 2 * (int)pad - KW) / (int)stride + 1,
              "wgrad spatial shapes");
  const bool want_db = db.has_value() && db->defined();
  if (want_db) {
    TORCH_CHECK(db->scalar_type() == at::kFloat && db->numel() == N && db->is_contiguous(), "db: fp32 [N]");
  }
  // 3x3 / stride-1 convs on 64 channels (stage 1 at H/2): the tap-batched halo-block weight
  // gradient of the update block (conv_igemm.hip conv_wgrad3_kernel: every tap from one DMA'd
  // halo block, two waves per SIMD) instead of the per-tap im2col kernel below, reduced
  // straight into the fp32 parameter layout (weights.hip).  scripts/bench_enc.py on MI355X:
  // 158 -> 122 us at 16 x 184 x 248; the 128-channel stage-3 conv is faster below (47 vs 55 us)
  if (KH == 3 && KW == 3 && stride == 1 && pad == 1 && Cin == Cx && Cin == 64 && N % 8 == 0 && fold == 0) {
    ConvWgradArgs w{};
    w.src[0] = ConvSrc{cbf(x), (long)xpitch, Cin, 0};
    w.nsrc = 1;
    w.Cin = Cin;
    w.B = B;
    w.H = Hx;
    w.W = Wx;
    w.KH = 3;
    w.KW = 3;
    w.PH = 1;
    w.PW = 1;
    w.K = 9 * Cin;
    w.Kpad = round_up(w.K, 64);
    w.dy = cbf(dy);
    w.dy_stride = dypitch;
    w.N = N;
    w.P = (long)B * Hx * Wx;
    w.f16 = f16;
    if (wgrad_supported(w)) {
      const WgradPlan pl = plan_conv_wgrad(w);
      const bool with_b = want_db && !db_zero;
      auto fo = x.options().dtype(at::kFloat);
      at::Tensor slab = at::empty({(long)pl.nsplit * pl.Npad * w.Kpad}, fo);
      at::Tensor dbslab = with_b ? at::empty({(long)pl.nsplit * pl.tilesN * pl.Npad}, fo) : at::Tensor();
      w.slab = slab.data_ptr<float>();
      w.dbslab = with_b ? dbslab.data_ptr<float>() : nullptr;
      check(launch_conv_wgrad(w, pl, stream()), "conv_wgrad (encoder)");
      ConvParamDesc d{};
      d.w[0] = dw.data_ptr<float>();
      for (int k = 0; k < 4; ++k) d.ws[0][k] = dw.stride(k);
      d.b[0] = want_db ? db->data_ptr<float>() : nullptr;  // db_zero: the reduce writes 0 (no partials)
      d.rows[0] = N;
      d.nseg = 1;
      d.seg_real[0] = d.seg_pad[0] = Cin;
      d.Cin = d.Cin_pad = Cin;
      d.KH = d.KW = 3;
      d.scale = 1.f;
      check(launch_wgrad_reduce_params(w.slab, pl.nsplit, pl.Npad, w.Kpad, w.dbslab, pl.nsplit * pl.tilesN, d, N,
                                       accumulate ? 1 : 0, stream()),
            "wgrad_reduce_params (encoder)");
      return;
    }
  }
  EncWgradArgs a{};
  a.x = cbf(x);
  a.xstride = xpitch;
  a.Cx = Cx;
  a.B = B;
  a.Hx = Hx;
  a.Wx = Wx;
  a.Ho = Ho;
  a.Wo = Wo;
  a.KH = KH;
  a.KW = KW;
  a.stride = (int)stride;
  a.pad = (int)pad;
  a.dy = cbf(dy);
  a.dy_stride = dypitch;
  a.N = N;
  a.f16 = f16;
  const int BM = (N % 128 == 0) ? 128 : 64;
  a.tilesM = (N + BM - 1) / BM;
  a.Npad = a.tilesM * BM;
  a.K = KH * KW * Cx;
  // 128 K-columns per workgroup when there are enough (twice the MFMAs per staged dY tile)
  // (small pixel counts keep 64 columns: more workgroups -- scripts/bench_enc.py on MI355X)
  const long Pn = (long)B * Ho * Wo;
  const int BN = (a.K >= 256 && Pn >= 100000) ? 128 : 64;
  a.tilesN = (a.K + BN - 1) / BN;
  a.Kpad = a.tilesN * BN;
  a.P = (long)B * Ho * Wo;
  const long tiles = (long)a.tilesM * a.tilesN;
  // ~640 workgroups (2.5 per CU): long pixel loops per workgroup, few slabs to reduce
  long pps = (a.P * tiles + 639) / 640;
  pps = std::max<long>(256, (pps + 63) / 64 * 64);
  a.pix_per_split = (int)pps;
  a.nsplit = (int)((a.P + pps - 1) / pps);
  at::Tensor slab = at::empty({(long)a.nsplit * a.Npad * a.Kpad}, x.options().dtype(at::kFloat));
  a.slab = slab.data_ptr<float>();
  at::Tensor dbslab;
  if (want_db && !db_zero) {
    dbslab = at::empty({(long)a.nsplit * a.Npad}, x.options().dtype(at::kFloat));
    a.dbslab = dbslab.data_ptr<float>();
  }
  check(launch_enc_wgrad(a, BM, BN, stream()), "enc_wgrad");
  long wsd[4];
  for (int d = 0; d < 4; ++d) wsd[d] = dw.stride(d);
  check(launch_enc_wgrad_reduce(a.slab, a.nsplit, a.Npad, a.Kpad, a.dbslab, dw.data_ptr<float>(), wsd, N, Cin, Cx, KH,
                                KW, want_db ? db->data_ptr<float>() : nullptr, accumulate, (int)fold, stream()),
        "enc_wgrad_reduce");
}

// [img0; img1] (fp32 0..255, [B,3,H,W] any strides) -> [nimg, H, W, 8] bf16 in [-1, 1]
at::Tensor enc_prep(const at::Tensor& img0, const c10::optional<at::Tensor>& img1, int64_t split, bool f16) {
  TORCH_CHECK(img0.is_cuda() && img0.scalar_type() == at::kFloat && img0.dim() == 4 && img0.size(1) == 3,
              "images: fp32 [B, 3, H, W]");
  const int B = (int)img0.size(0), H = (int)img0.size(2), W = (int)img0.size(3);
  int nimg = B;
  if (img1.has_value() && img1->defined()) {
    TORCH_CHECK(img1->sizes() == img0.sizes() && img1->strides() == img0.strides() &&
                    img1->scalar_type() == at::kFloat,
                "paired images must match");
    nimg = 2 * B;
  }
  TORCH_CHECK(!(split && f16), "enc_prep: split planes are bf16");
  at::Tensor out = at::empty({nimg, H, W, split ? 24 : 8}, img0.options().dtype(f16 ? at::kHalf : at::kBFloat16));
  long st[4] = {img0.stride(0), img0.stride(1), img0.stride(2), img0.stride(3)};
  check(launch_enc_prep(img0.data_ptr<float>(), nimg > B ? img1->data_ptr<float>() : nullptr, st, B, H, W, nimg,
                        out.data_ptr(), (split ? 1 : 0) | (f16 ? 2 : 0) | (split == 2 ? 4 : 0), stream()),
        "enc_prep");
  return out;
}

// coef [B, 4, N] = (scale, shift, rstd, mean) from conv tile statistics (kind 1 / 2) or running statistics (3)
at::Tensor enc_norm_stats(const c10::optional<at::Tensor>& stats, int64_t B, int64_t HW, int64_t N, int64_t kind,
                          const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                          const c10::optional<at::Tensor>& rmean, const c10::optional<at::Tensor>& rvar,
                          const c10::optional<at::Tensor>& nbt, double momentum, double eps, int64_t W) {
  NormFinArgs a{};
  a.B = (int)B;
  a.HW = (int)HW;
  a.N = (int)N;
  a.kind = (int)kind;
  a.BM = kBM;
  const bool has_stats = stats.has_value() && stats->defined();
  TORCH_CHECK(!(kind == 1 || kind == 2) || has_stats, "training statistics need the conv tile statistics");
  at::TensorOptions o;
  if (has_stats) {
    const int d = (int)stats->dim();
    TORCH_CHECK((d == 4 || d == 5) && stats->size(0) == B && stats->size(d - 2) == 2 && stats->size(d - 1) == N &&
                    stats->is_contiguous(),
                "stats shape");
    a.stats = stats->data_ptr<float>();
    a.T = (int)(d == 5 ? stats->size(1) * stats->size(2) : stats->size(1));
    if (d == 5) {  // square tiles of the 3x3 kernel: the tile pixel counts need the image width
      TORCH_CHECK(W > 0 && HW % W == 0 && (W + kEnc3Tile - 1) / kEnc3Tile == stats->size(2) &&
                      (HW / W + kEnc3Tile - 1) / kEnc3Tile == stats->size(1),
                  "enc_norm_stats: square-tile statistics need the image width W");
      a.tile_w = kEnc3Tile;
      a.img_w = (int)W;
    }
    o = stats->options();
  }
  auto fp = [](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "norm parameters: contiguous fp32");
    return t->data_ptr<float>();
  };
  a.gamma = fp(gamma);
  a.beta = fp(beta);
  a.rmean = fp(rmean);
  a.rvar = fp(rvar);
  if (!has_stats) {
    TORCH_CHECK(rmean.has_value() && rmean->defined(), "enc_norm_stats: pass the conv statistics or running stats");
    o = rmean->options();
  }
  if (kind == 3) TORCH_CHECK(a.rmean && a.rvar, "running statistics");
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->scalar_type() == at::kLong, "num_batches_tracked");
    a.nbt = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  }
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  at::Tensor coef = at::empty({B, 4, N}, o.dtype(at::kFloat));
  a.coef = coef.data_ptr<float>();
  check(launch_enc_norm_finalize(a, stream()), "enc_norm_finalize");
  return coef;
}

at::Tensor enc_apply(const at::Tensor& x, const at::Tensor& coef, bool relu_a, const c10::optional<at::Tensor>& r,
                     const c10::optional<at::Tensor>& coef_r, bool relu_out, int64_t split) {
  check_nhwc(x, "a");
  TORCH_CHECK(!split || x.size(3) % 24 == 0, "enc_apply: split rows hold 3 planes of a multiple of 8 channels");
  const int B = (int)x.size(0), HW = (int)(x.size(1) * x.size(2)), N = (int)x.size(3) / (split ? 3 : 1);
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == (long)B * 4 * N, "coef");
  const void* rp = nullptr;
  const float* crp = nullptr;
  if (r.has_value() && r->defined()) {
    check_nhwc(*r, "r");
    TORCH_CHECK(r->sizes() == x.sizes(), "residual shape");
    rp = r->data_ptr();
    if (coef_r.has_value() && coef_r->defined()) {
      TORCH_CHECK(coef_r->numel() == (long)B * 4 * N && coef_r->is_contiguous(), "coef_r");
      crp = coef_r->data_ptr<float>();
    }
  }
  at::Tensor out = at::empty_like(x);
  if (r.has_value() && r->defined()) TORCH_CHECK(r->scalar_type() == x.scalar_type(), "residual dtype");
  check(launch_enc_apply(x.data_ptr(), coef.data_ptr<float>(), relu_a, rp, crp, relu_out, out.data_ptr(), B, HW, N,
                         (split ? 1 : 0) | (x.scalar_type() == at::kHalf ? 2 : 0) | (split == 2 ? 4 : 0), stream()),
        "enc_apply");
  return out;
}

// returns [da0, da1 | empty, dgamma0, dbeta0, dgamma1, dbeta1] (BatchNorm kinds; empty otherwise)
//
// ``stage``: 0 = all three passes; 1 = reduce only, returns [part] ([B][R][4][N] fp32
// partial sums of this rank's images); 2 = finalize + apply from ``part`` holding the
// partials of ``b_fin`` images -- every rank's, gathered rank-major (synchronized BatchNorm:
// parallel/sync_bn.py) -- dgamma / dbeta then come out as the sums over those b_fin images.
std::vector<at::Tensor> enc_norm_bwd_impl(const at::Tensor& g, const at::Tensor& a0, const at::Tensor& c0, bool relu0,
                                          const c10::optional<at::Tensor>& a1, const c10::optional<at::Tensor>& c1,
                                          int64_t kind, int stage, const c10::optional<at::Tensor>& part_in,
                                          int64_t b_fin, int64_t split) {
  check_nhwc(g, "g");
  check_nhwc(a0, "a0");
  TORCH_CHECK(a0.sizes() == g.sizes(), "a0 shape");
  TORCH_CHECK(!split || g.size(3) % 24 == 0, "norm backward: split rows hold 3 planes of a multiple of 8 channels");
  const int B = (int)g.size(0), HW = (int)(g.size(1) * g.size(2)), N = (int)g.size(3) / (split ? 3 : 1);
  TORCH_CHECK(N <= 256, "norm backward: at most 256 channels");
  NormBwdArgs a{};
  a.g = cbf(g);
  a.a0 = cbf(a0);
  a.c0 = c0.data_ptr<float>();
  a.relu0 = relu0 ? 1 : 0;
  const bool two = a1.has_value() && a1->defined();
  if (two) {
    check_nhwc(*a1, "a1");
    TORCH_CHECK(a1->sizes() == g.sizes(), "a1 shape");
    a.a1 = cbf(*a1);
    a.c1 = c1->data_ptr<float>();
  }
  a.B = B;
  a.HW = HW;
  a.N = N;
  a.R = std::min(norm_chunks_max(), std::max(1, HW / norm_chunk_pixels()));
  a.kind = (int)kind;
  a.split = (int)split;
  a.f16 = g.scalar_type() == at::kHalf ? 1 : 0;
  TORCH_CHECK(a0.scalar_type() == g.scalar_type(), "norm backward: g and a0 share one dtype");
  auto fo = g.options().dtype(at::kFloat);
  const long bf = stage == 2 ? (long)b_fin : (long)B;
  TORCH_CHECK(stage != 2 || (kind == 2 && bf >= B && part_in.has_value() && part_in->defined() &&
                             part_in->scalar_type() == at::kFloat && part_in->is_contiguous() &&
                             part_in->numel() == bf * a.R * 4 * N),
              "enc_norm_bwd_finish: training BatchNorm and [b_fin, R, 4, N] fp32 partials");
  at::Tensor part = stage == 2 ? *part_in : at::empty({(long)B, (long)a.R, 4L, (long)N}, fo);
  a.part = part.data_ptr<float>();
  if (stage == 1) {
    check(launch_enc_norm_bwd_stages(a, 1, 0, stream()), "enc_norm_bwd_part");
    return {part};
  }
  at::Tensor bcoef = at::empty({bf * 2 * 3 * N}, fo);
  a.bcoef = bcoef.data_ptr<float>();
  at::Tensor da0 = at::empty_like(g), da1 = two ? at::empty_like(g) : at::Tensor();
  a.out0 = mbf(da0);
  a.out1 = two ? mbf(da1) : nullptr;
  std::vector<at::Tensor> out{da0, da1, at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor()};
  if (kind == 2 || kind == 3) {
    for (int j = 0; j < (two ? 2 : 1); ++j) {
      out[2 + 2 * j] = at::empty({N}, fo);
      out[3 + 2 * j] = at::empty({N}, fo);
      a.dgamma[j] = out[2 + 2 * j].data_ptr<float>();
      a.dbeta[j] = out[3 + 2 * j].data_ptr<float>();
    }
  }
  if (stage == 2)
    check(launch_enc_norm_bwd_stages(a, 6, (int)bf, stream()), "enc_norm_bwd_finish");
  else
    check(launch_enc_norm_bwd(a, stream()), "enc_norm_bwd");
  return out;
}

std::vector<at::Tensor> enc_norm_bwd(const at::Tensor& g, const at::Tensor& a0, const at::Tensor& c0, bool relu0,
                                     const c10::optional<at::Tensor>& a1, const c10::optional<at::Tensor>& c1,
                                     int64_t kind, int64_t split) {
  return enc_norm_bwd_impl(g, a0, c0, relu0, a1, c1, kind, 0, c10::nullopt, 0, split);
}

at::Tensor enc_norm_bwd_part(const at::Tensor& g, const at::Tensor& a0, const at::Tensor& c0, bool relu0,
                             const c10::optional<at::Tensor>& a1, const c10::optional<at::Tensor>& c1, int64_t kind,
                             int64_t split) {
  return enc_norm_bwd_impl(g, a0, c0, relu0, a1, c1, kind, 1, c10::nullopt, 0, split)[0];
}

std::vector<at::Tensor> enc_norm_bwd_finish(const at::Tensor& g, const at::Tensor& a0, const at::Tensor& c0,
                                            bool relu0, const c10::optional<at::Tensor>& a1,
                                            const c10::optional<at::Tensor>& c1, int64_t kind, const at::Tensor& part,
                                            int64_t b_fin, int64_t split) {
  return enc_norm_bwd_impl(g, a0, c0, relu0, a1, c1, kind, 2, part, b_fin, split);
}

}  // namespace raft_amd

TORCH_LIBRARY_FRAGMENT(raft_amd, m) {
  // split: 0 = bf16 / fp16 rows, 1 = split-bf16 [hi | lo | hi] planes, 2 = three-plane [hi | mid | lo]
  // rows with the six-plane fp32-exact forward GEMM (encoder.hip store8_split, fwd_tables)
  m.def("enc_conv_fwd(Tensor x, Tensor w, Tensor? bias, int stride, int pad, bool stats, int split=0, "
        "Tensor? prepacked=None) -> (Tensor, Tensor)");
  m.def(
      "enc_conv_dgrad(Tensor[] dys, Tensor[] ws, int[] strides, int[] pads, int H, int W, Tensor? res, Tensor? mask, "
      "int split=0, Tensor? prepacked=None) -> Tensor");
  m.def("enc_pack_fwd_job(Tensor w, int Cx, int pad, int split, bool f16) -> (Tensor, int, int)");
  m.def("enc_pack_dgrad_job(Tensor[] ws, int[] strides, int[] pads, int H, int W, int split, bool f16) -> "
        "(Tensor, int, int)");
  m.def("enc_pack_multi(Tensor plan, int njobs, int nblocks, Tensor(a!) out) -> ()");
  m.def("enc_conv_wgrad(Tensor x, Tensor dy, Tensor(a!) dw, Tensor(b!)? db, int stride, int pad, bool accumulate, "
        "bool db_zero=False, int fold=0) -> ()");
  m.def("enc_prep(Tensor img0, Tensor? img1, int split=0, bool f16=False) -> Tensor");
  m.def(
      "enc_norm_stats(Tensor? stats, int B, int HW, int N, int kind, Tensor? gamma, Tensor? beta, Tensor(a!)? rmean, "
      "Tensor(b!)? rvar, Tensor(c!)? nbt, float momentum, float eps, int W=0) -> Tensor");
  m.def("enc_apply(Tensor a, Tensor coef, bool relu_a, Tensor? r, Tensor? coef_r, bool relu_out, int split=0) "
        "-> Tensor");
  m.def("enc_norm_bwd(Tensor g, Tensor a0, Tensor c0, bool relu0, Tensor? a1, Tensor? c1, int kind, "
        "int split=0) -> Tensor[]");
  m.def("enc_norm_bwd_part(Tensor g, Tensor a0, Tensor c0, bool relu0, Tensor? a1, Tensor? c1, int kind, "
        "int split=0) -> Tensor");
  m.def(
      "enc_norm_bwd_finish(Tensor g, Tensor a0, Tensor c0, bool relu0, Tensor? a1, Tensor? c1, int kind, Tensor part, "
      "int b_fin, int split=0) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(raft_amd, CUDA, m) {
  m.impl("enc_conv_fwd", &raft_amd::enc_conv_fwd);
  m.impl("enc_conv_dgrad", &raft_amd::enc_conv_dgrad);
  m.impl("enc_conv_wgrad", &raft_amd::enc_conv_wgrad);
  m.impl("enc_pack_fwd_job", &raft_amd::enc_pack_fwd_job);
  m.impl("enc_pack_dgrad_job", &raft_amd::enc_pack_dgrad_job);
  m.impl("enc_pack_multi", &raft_amd::enc_pack_multi);
  m.impl("enc_prep", &raft_amd::enc_prep);
  m.impl("enc_norm_stats", &raft_amd::enc_norm_stats);
  m.impl("enc_apply", &raft_amd::enc_apply);
  m.impl("enc_norm_bwd", &raft_amd::enc_norm_bwd);
  m.impl("enc_norm_bwd_part", &raft_amd::enc_norm_bwd_part);
  m.impl("enc_norm_bwd_finish", &raft_amd::enc_norm_bwd_finish);
}
