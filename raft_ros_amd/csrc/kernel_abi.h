// Kernel ABI of the native extension: the argument structs shared by the HIP kernels
// (csrc/*.hip, device side) and the torch bindings (csrc/*bindings.cpp, host side), their
// launchers, and the host-only planning of the weight-gradient launches.  One definition
// for both sides, so a field added for a kernel cannot silently shift the host layout.
// Everything above the launcher section is plain C++ (the planning is unit-tested under
// AddressSanitizer / UBSan on the host: tests/native/plan_test.cpp).
#pragma once

#include <algorithm>

#if defined(__HIP__)
#define RAFT_HD __host__ __device__
#else
#define RAFT_HD
#endif

namespace raft_amd {

// ============================================================================ work mapping
// Workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8).  xcd_remap: contiguous
// tile ranges per XCD (neighbouring tiles share operand rows in that XCD's L2); a bijection
// of [0, nwg).
RAFT_HD inline int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

// Weight-gradient launches: workgroup -> (pixel split, output tile).  With xcd_g > 0
// (nsplit == 8 * xcd_g) every tile of a split runs on one XCD so the split's dY / X rows are
// fetched into that XCD's L2 once; otherwise splits are laid out consecutively.
RAFT_HD inline void wgrad_block_map(int bid, int tiles, int xcd_g, int& split, int& tile) {
  if (xcd_g > 0) {
    const int xcd = bid & 7, local = bid >> 3;
    const int si = local / tiles;
    tile = local - si * tiles;
    split = xcd * xcd_g + si;
  } else {
    split = bid / tiles;
    tile = bid - split * tiles;
  }
}

// ============================================================================ update-block convs
struct ConvSrc {
  const __bf16* ptr;
  long stride;  // elements between consecutive pixels
  int C;        // channels taken from this source (multiple of 8)
  int period;   // wgrad only: >0 -> pixel p reads row p % period (0: no wrap)
};

struct ConvFwdArgs {
  ConvSrc src[3];
  int nsrc, Cin;
  int B, H, W, KH, KW, PH, PW;
  int K, Kpad;
  const __bf16* wt;  // packed weights [N][Kpad], k = tap*Cin + c
  int N;
  long P;
  // epilogue
  int epi;      // 0: bias+act store, 1: grad store, 2: GRU z||r, 3: GRU q+blend
  int act;      // 0: none, 1: relu
  int out_f32;  // output element type (epi 0/1)
  int acc_c0;   // epi 1: accumulate (+=) into out for channels n >= acc_c0
  float alpha;
  const float* bias;
  void* out;
  long out_stride;
  const __bf16* mask;  // epi 1: multiply by (mask[p][n] > 0) (ReLU' of the conv input)
  long mask_stride;
  const __bf16* h;  // epi 2/3: hidden state
  long h_stride;
  const __bf16* z;  // epi 3: update gate
  long z_stride;
  __bf16* out2;  // epi 2: r*h, epi 3: tanh(q), epi 4: dq
  long out2_stride;
  // fused GRU backward (data-gradient launches of the update block): output channels
  // [0, gru_cols) finish the gate math in the epilogue, the rest are stored as epi 1
  //   epi 4 (after the dH-producing dgrad): g = dH; dq = g z (1 - q^2) -> out2,
  //          dz = g (q - h) z (1 - z) -> out3, carry = g (1 - z)  (out not written)
  //   epi 5 (the q dgrad, g = d(r*h)): dr = g h r (1 - r) -> out3, out = carry + g r
  //   epi 6 (the last GRU dgrad): channels [0, gru_cols) -> bf16 out3 (d net), [gru_cols,
  //          cm_c0) -> out as epi 1, [cm_c0, N) -> bf16 cout = (cmask > 0 ? g : 0), zero past
  //          cm_valid (the ReLU' of the motion features; out not written)
  const __bf16* g0;  // epi 4: q, epi 5: r
  long g0_stride;
  float* carry;
  long carry_stride;
  __bf16* out3;
  long out3_stride;
  int gru_cols;
  const __bf16* addsrc;  // epi 4: incoming bf16 gradient added to g (null: none)
  long addsrc_stride;
  __bf16* cout;
  long cout_stride;
  const __bf16* cmask;
  long cmask_stride;
  int cm_c0, cm_valid;
  int cfg;  // kernel variant: 0 = automatic, otherwise forced (tests / microbenchmarks)
  // split-bf16 ("fp32-faithful") mode of epilogues 0 / 2 / 3 (inference without AMP): a bf16
  // output value x is stored as three planes hi = bf16(x), lo = bf16(x - hi), hi again, in
  // groups of G channels: channel n of an output lives at (n / G) * 3G + plane * G + n % G.
  // A consumer conv reads a group as ONE source of 3G channels [hi | lo | hi] against packed
  // weights [W_hi | W_hi | W_lo], so its bf16 MFMAs compute x_hi W_hi + x_lo W_hi + x_hi W_lo
  // (fp32 accumulate): the fp32 product up to the dropped x_lo * W_lo term (~2^-16 relative).
  // Epilogue operands read from such tensors (h, z) add their hi and lo planes.
  int split_g;   // > 0: out is split with group width G = split_g
  int split_g2;  // > 0: out2 is split with group width split_g2
  int split_h;   // > 0: h is split; its lo plane is split_h channels after the hi plane
  int split_z;   // > 0: z is split (lo plane offset)
  // fp32 training (split-bf16 backward, ops/update_split.py): epilogue 1 stores split planes
  // (split_g, no accumulation); the GRU-backward epilogues 4 / 5 / 6 read g0 and addsrc as
  // split planes (lo plane offsets) and store out3 / cout as split planes of group widths
  // split_g3 / split_cout; mask / cmask are then hi-plane views (x > 0 <=> hi(x) > 0)
  int split_g0;    // > 0: g0 is split (lo plane offset)
  int split_g3;    // > 0: out3 is split with group width split_g3
  int split_add;   // > 0: addsrc is split (lo plane offset)
  int split_cout;  // > 0: cout is split with group width split_cout
  // fp16 AMP (the reference's --mixed_precision dtype): every 16-bit operand, epilogue operand
  // and 16-bit output is IEEE fp16 (v_mfma_f32_32x32x16_f16) instead of bf16; the pointers
  // keep their __bf16 type as 16-bit storage
  int f16;
  // Narrow follow-up conv folded into epilogue 0 (the flow head: heads conv 3x3 + ReLU ->
  // flow_head.conv2 3x3, 256 -> 2).  For the first n2_cols output channels, each 64-channel
  // slot s of a tile also writes the per-tap partial products of the NEXT conv,
  //   n2y[s][o * 9 + t][p] = sum_{c in slot s} out_bf16[p][c] * n2w[o][t * n2_cols + c],
  // and launch_n2_apply sums the 3x3 neighbourhood (out2[p][o] = bias + sum_s sum_t
  // n2y[s][o * 9 + t][p + off_t]; planar, so its loads coalesce): the 256-channel activation
  // is never re-read 9 times.
  const __bf16* n2w;  // [2][n2_kpad] packed 3x3 weights of the follow-up conv (k = tap * n2_cols + c)
  float* n2y;         // [n2_cols / 64][18][P] fp32 partials
  int n2_kpad, n2_cols;
  int swz_col;  // conv_fwd6 3x3 2-D tiles: LDS chunk swizzle keyed on the halo column (set by the launcher)
};

struct ConvWgradArgs {
  ConvSrc src[3];
  int nsrc, Cin;
  int B, H, W, KH, KW, PH, PW;
  int K, Kpad;
  const __bf16* dy;  // [P][dy_stride], N channels used
  long dy_stride;
  int N;
  long P;
  long pix_per_split;
  float* slab;    // [nsplit][Npad][Kpad] fp32: the split's partial dW (written, not accumulated)
  float* dbslab;  // [nsplit][tilesN][Npad] fp32 bias partials (may be null)
  int Npad;       // slab rows (N rounded up to the row tile)
  int xcd_g;      // >0: XCD-grouped split mapping with xcd_g splits per XCD (set by the launcher)
  int f16;        // fp16 operands (see ConvFwdArgs::f16)
  int mt5;        // wgrad v3 on 1x5 / 5x1 convs: 1 = 64-row workgroups, 2 = 128 rows on 4 waves (the default)
  int grid_div;   // > 1: plan for 1 / grid_div of the workgroups (leave CUs to the work beside it)
  int wg2_stages; // wgrad v2 (1x1 / generic) DMA ring stages: 3 (0 = 3; 98 KB at 128 x 128, one
                  // workgroup per CU) or 2 (64 KB, two per CU: the plan targets 512 workgroups)
};

// Plan of one weight-gradient launch (the caller sizes the slabs from it).
//   kind 2: wgrad v2, tilesN = column tiles, pix_per_split = pixels per split
//   kind 3: wgrad v3 (tap-batched), tilesN = 64-channel chunks, pix_per_split = pixel TILES per split
// Bias partials: nsplit * tilesN rows of Npad floats.
struct WgradPlan {
  int BM, BN, tilesM, tilesN, nsplit, Npad, xcd_g;
  long pix_per_split;
  int kind;
};

struct ConvParamDesc {
  float* w[2];     // parameter (pack: read) / gradient (reduce: written) tensors
  long ws[2][4];   // strides (Cout, Cin, kh, kw) in elements
  float* b[2];     // biases / bias gradients (may be null)
  int rows[2];     // Cout of each stacked parameter (rows[1] = 0: single)
  int nseg;
  int seg_real[3], seg_pad[3];
  int Cin, Cin_pad, KH, KW;
  float scale;
  // split-bf16 packing (fp32 mode, ops/update_split.py): split_fw = 1 -> the forward operand
  // runs over every segment's [hi | lo | hi] planes (3 x seg_pad channels each) against
  // [W_hi | W_hi | W_lo]; split_dy = G > 0 -> the data-gradient operand runs over dY planes
  // [hi | lo | hi] of width G (k = tapflip * 3G + plane * G + n) against [W_hi | W_hi | W_lo]
  int split_fw, split_dy;
  int f16;  // pack: fp16 operands instead of bf16 (fp16 AMP)
  // reduce: the weight-gradient columns hold every segment as [hi | lo] planes of seg_pad
  // channels (split-bf16 training, [X_hi | X_lo]^T dY_hi); the parameter gradient is their sum
  int fold;
};

// Several layers' packs in one launch (pack_conv_weights_multi): job q covers the element
// range [begin, begin + N Kf + Cin_pad Kd + N) of the launch; split_fw in ``d`` selects the
// split-bf16 layout (aux = unused) over the bf16 / fp16 one (aux = Cout_pad of the dgrad operand)
struct PackJob {
  ConvParamDesc d;
  __bf16* wf;
  __bf16* wd;
  float* bias;
  long begin;
  int N, Kf, Kd, aux;
};
constexpr int kPackJobs = 14;
struct PackJobs {
  PackJob j[kPackJobs];
  long total;
  int n;
};
static_assert(sizeof(PackJobs) <= 4000, "pack jobs must fit the kernel-argument segment");

// ============================================================================ encoder convs
constexpr int kEncTab = 256;  // K/8 decode-table entries per launch (all classes) held in the arguments
// deeper convs (the split-bf16 layout's 3x channels) read their tables from device memory
constexpr int kEncTabMax = 1024;  // the three-plane forward doubles K (six planes)

struct EncSrc {
  const __bf16* ptr;
  int stride;  // elements between consecutive pixels
  int C;       // channels (multiple of 8)
  int H, W;    // spatial dims
  int is;      // source step per grid step
};

struct EncClass {
  int t0;            // first decode-table entry
  int Gh, Gw;        // pixel grid per image
  int oy0, ox0;      // output coordinate = grid * os + o0
  int K, Kpad;       // GEMM depth (Kpad: multiple of 64)
  int tiles_img;     // BM-row tiles per image
  int blk0;          // first workgroup of this class
  long wofs;         // element offset of the class's packed weights [N][Kpad]
};

struct EncConvArgs {
  EncSrc src[2];
  int B;
  // decode table: (dy+128) | (dx+128) << 8 | src << 16 | c << 17, -1 = zero columns
  int tab[kEncTab];
  // packing table: w | ky << 4 | kx << 8 | local << 12, -1 = zero columns
  int ptab[kEncTab];
  EncClass cls[4];
  int ncls, N, tilesN;
  const __bf16* wt;
  int Ho, Wo, os;
  __bf16* out;
  int out_stride;
  const float* bias;
  const __bf16* res;
  int res_stride;
  const __bf16* mask;
  int mask_stride;
  float* stats;  // [B * tiles_img][2][N]: per tile column sum and M2
  // weight packing
  const float* w[2];
  long ws[2][4];
  int wcin[2];
  int pack_dgrad;
  // split-bf16 input planes (forward packing): > 0 = the plane width cx of x = [hi | lo | hi];
  // the fp32 weight is packed as [W_hi | W_hi | W_lo], each plane zero-padded from Cin to cx
  int split_w;
  // tables of more than kEncTab entries: device copies [kEncTabMax] (null: the arrays above)
  const int* tab_ptr;
  const int* ptab_ptr;
  int f16;  // 16-bit activations / packed weights are fp16 (fp16 AMP) instead of bf16
  int split_wd[2];  // split data gradient: the dY plane width (Cout) of conv 0 / 1 (0: split_w)
  // split-bf16 output (fp32-faithful inference, see ConvFwdArgs::split_g): out rows hold
  // [hi | lo | hi] planes of N channels each (out_stride = 3N).  A split data gradient (fp32
  // training) also reads res as split rows (res_stride = 3N, lo plane at +N) and the ReLU'
  // mask from the hi plane of split rows (mask_stride = 3N); its dY sources are split rows of
  // 3 Cout channels, packed against [W_hi | W_hi | W_lo] along Cout (split_w = Cout)
  int split;
};

struct EncWgradArgs {
  const __bf16* x;
  int xstride, Cx;
  int B, Hx, Wx, Ho, Wo, KH, KW, stride, pad;
  const __bf16* dy;
  int dy_stride, N;
  int K, Kpad, Npad, tilesM, tilesN;
  long P;
  int pix_per_split, nsplit;
  float* slab;    // [nsplit][Npad][Kpad]
  float* dbslab;  // [nsplit][Npad] or null
  int f16;        // fp16 operands (fp16 AMP)
};

struct NormFinArgs {
  const float* stats;  // conv epilogue tiles [B][T][2][N]
  int B, T, BM, HW, N, kind;
  int tile_w, img_w;   // tile_w > 0: T = square tile_w x tile_w tiles in row-major order of an
                       // img_w-wide image (the 3x3 resident-weight conv); else BM-pixel row tiles
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;
  float momentum, eps;
  float* coef;
};

struct NormBwdArgs {
  const __bf16* g;
  const __bf16* a0;
  const float* c0;
  int relu0;
  const __bf16* a1;  // null: one branch
  const float* c1;
  float* part;
  int B, HW, N, R, kind;
  float* bcoef;  // [B][2][3][N]: da = k1 * dy + k2 * xhat + k3
  float* dgamma[2];
  float* dbeta[2];
  __bf16* out0;
  __bf16* out1;
  int split;  // g, a0, a1, out0, out1 are split-bf16 rows of 3N (hi / lo / hi planes; fp32 training)
  int f16;    // g, a0, a1, out0, out1 are fp16 (fp16 AMP)
};

// 3x3 / stride-1 encoder convs with 64 input and 64 output channels (both encoders' stage-1
// residual convs and their data gradients) run on a resident-weight kernel over square
// output tiles (encoder.hip enc_conv3_kernel).
constexpr int kEnc3Tile = 16;

// Host check: can enc_conv3_kernel run this planned launch?  (one class, one source of
// exactly 64 channels, 64 outputs, the 9 taps of a 3x3 window at offsets in [-1, 1], output
// grid = input grid.)
inline bool enc_conv3_eligible(const EncConvArgs& a) {
  if (a.ncls != 1 || a.src[1].ptr != nullptr || a.N != 64 || a.os != 1) return false;
  const EncSrc& s = a.src[0];
  const EncClass& c = a.cls[0];
  if (s.C != 64 || s.stride != 64 || s.is != 1 || c.K != 576 || c.Kpad != 576 || c.oy0 || c.ox0) return false;
  if (c.Gh != a.Ho || c.Gw != a.Wo || s.H != a.Ho || s.W != a.Wo) return false;
  for (int t = 0; t < 9; ++t)
    for (int e = 0; e < 8; ++e) {
      const int ent = a.tab[c.t0 + t * 8 + e];
      if (ent < 0) return false;
      const int dy = (ent & 0xff) - 128, dx = ((ent >> 8) & 0xff) - 128, src = (ent >> 16) & 1, ch = ent >> 17;
      const int dy0 = (a.tab[c.t0 + t * 8] & 0xff) - 128, dx0 = ((a.tab[c.t0 + t * 8] >> 8) & 0xff) - 128;
      if (src != 0 || ch != e * 8 || dy != dy0 || dx != dx0 || dy < -1 || dy > 1 || dx < -1 || dx > 1) return false;
    }
  return true;
}

// ============================================================================ correlation
struct PyrDesc {
  float* ptr[4];
  int H[4];
  int W[4];
  long ld[4];  // row pitch (elements) of level l: row `pix` starts at ptr[l] + pix * ld[l]
  int levels;
  int vbf16;   // levels hold bf16 (the AMP volume; forward lookups only -- gradients stay fp32)
  int blk;     // levels stored in 16-column blocks [W/16][H][16] (W = blocks * 16)
};

// Deferred lookup backward (csrc/corr_volume.hip lookup_grad_rows_kernel): the window
// gradients of all T lookups of a step -> the dense level-gradient rows, each row
// accumulated in LDS and written once (bf16 or fp32), replacing T read-modify-write passes
// over an fp32 buffer and its memset.
constexpr int kGradRowsMaxT = 32;
constexpr int kGradRowsMaxLd = 15616;  // row floats in LDS (+ window staging) within 64 KB
struct GradRowsArgs {
  const void* g[kGradRowsMaxT];   // window gradients of lookup t: row pix at g[t] + pix * gstride
  const float* c[kGradRowsMaxT];  // coordinates of lookup t, (B, 2, H, W) fp32
  int T, gstride;
  void* out;  // (B*H*W, ld) rows, 16-column-blocked levels at off[l]
  long ld;
  int out_f32, accumulate;  // accumulate: add to the rows already in out
  int levels, off[4], H[4], W[4];  // W: padded to whole 16-column blocks
  int B, Hq, Wq, r;
};

// One GEMM of the correlation path: C[b][m][n] (op)= alpha * sum_k A[b][m][k] * B[b][n][k]
struct CorrGemmArgs {
  const void* A;  // fp32 or bf16; a_trans: element (m, k) at A[k * lda + m]
  long lda, sA;
  const void* B;  // fp32 or bf16, element (n, k) at B[n * ldb + k]
  long ldb, sB;
  void* C;  // fp32 (or bf16 for epi 0)
  long ldc, sC;
  int M, N, K, batch;
  float alpha;
  int a_f32, b_f32, a_trans, split, c_bf16;
  int epi;  // 0 store, 1 accumulate
  int cfg;  // 1: force the generic kernel (tests); 2-5: v2 volume kernel with a forced tile grouping
};

// Adjoint of the pyramid pools: out[b][y][x][c] = sum_l G[b][off_l + (y>>l)*w_l + (x>>l)][c] / 4^l
// over the levels whose (floor-sized) plane covers (y, x).  G holds the per-level gradients
// of all levels (rows = concatenated levels), so each output element is one thread's sum:
// deterministic, no read-modify-write races between levels.
struct UnpoolArgs {
  const float* G;
  long sG;  // batch stride of G (elements); row pitch = C
  float* out;
  int B, H, W, C, nseg;
  int off[4], h[4], w[4];
  int blk;  // level rows in 16-column block order (the dense pyramid's layout)
};

// GEMM operand of the dense pyramid: the 2x2 average-pooled levels of a feature map
// (any strides, bf16 or fp32), every level at column offset off[l] of a ld-long pixel
// axis (16-column block order when blk), zero rows/columns in the padding; written as
// fp32 (B, ld, C) rows (nchw = 0) or (B, C, ld) (nchw = 1).  Pool sums follow
// F.avg_pool2d's order, so the operand is bitwise equal to the torch op sequence.
struct PyrOperandArgs {
  const void* src;
  int src_bf16;
  long sB, sC, sH, sW;  // element strides of src viewed as (B, C, H, W)
  int B, C, H, W, nseg;
  int off[4], h[4], w[4];
  int blk, nchw;
  long ld;
  float* out;
  __bf16* out16;  // non-null: bf16 output instead (the bf16 GEMM operands, no conversion pass)
};

struct LocalCorrArgs {
  const __bf16* f1;   // (B*H*W, C) query features (NHWC rows)
  const __bf16* f2;   // (B, R, C): pooled fmap2 levels, level l rows [off[l], off[l] + h[l]*w[l])
  long f2_bstride;    // R * C
  const float* coords;  // (B, 2, H, W) level-0 pixel coordinates
  int B, H, W, C, r, levels;
  int off[4], h[4], w[4];
  float scale;
  // forward
  void* out;  // (B*H*W, ostride) features; level l taps at channel l*(2r+1)^2
  long ostride;
  int out_f32;
  int out_ch;  // channels written per row: taps, then zeros up to out_ch (K padding of convc1)
  // backward
  const void* gout;  // (B*H*W, gstride) tap gradients (same layout as out), fp32 or bf16
  long gstride;
  int gout_bf16;
  float* g1;  // (B*H*W, C) fp32
  float* g2;  // (B, R, C) fp32, accumulated (atomics)
  long long* g2fix;  // non-null: deterministic mode, fixed-point accumulator like g2
  const float* fix_scale;  // deterministic mode: device scalar, the power-of-two fixed-point scale
};

// ============================================================================ sequence loss
constexpr int kMaxPreds = 32;

struct SeqPreds {
  const float* p[kMaxPreds];
};

struct SeqGrads {
  float* g[kMaxPreds];
};

// ============================================================================ host-side planning
constexpr int kWgradBK = 64;  // pixels per K step of wgrad v2 (conv_igemm.hip WBK)

inline bool wgrad_supported(const ConvWgradArgs& a) {
  bool seg_ok = a.nsrc == 1;
  if (!seg_ok) {
    seg_ok = a.Cin % 128 == 0;
    for (int i = 0; i < a.nsrc; ++i) seg_ok = seg_ok && a.src[i].C % 128 == 0;
  }
  long maxbytes = 0;
  for (int i = 0; i < a.nsrc; ++i) {
    const long rows = a.src[i].period > 0 ? a.src[i].period : a.P;
    maxbytes = std::max(maxbytes, rows * a.src[i].stride * 2);
  }
  return seg_ok && maxbytes < (1L << 31) && a.P * a.dy_stride * 2 < (1L << 31) && a.P < (1L << 30);
}

// wgrad v3 shapes: (KH, KW) -> pixel tile (TH x TW)
inline bool wgrad3_shape(int KH, int KW) {
  return (KH == 1 && KW == 5) || (KH == 5 && KW == 1) || (KH == 3 && KW == 3);
}

// Split count: ~one round of workgroups over the 256 CUs.  When a whole number of splits per
// XCD fills >= 7/8 of its 32 CUs, every tile of a split runs on one XCD (its rows are fetched
// into that XCD's L2 once); otherwise splits are interleaved over the chip.
inline void choose_splits(long tiles, long work_units, long& splits, long& g, long target = 256) {
  g = (target / 8) / tiles;
  if (g * tiles < (target / 8) * 7 / 8) g = 0;
  splits = g > 0 ? 8 * g : std::max(1L, (target + tiles / 2) / tiles);
  if (splits > work_units) splits = work_units, g = 0;
  if (splits < 1) splits = 1;
}

inline WgradPlan plan_conv_wgrad3(const ConvWgradArgs& a) {
  WgradPlan pl{};
  pl.kind = 3;
  const bool sq = a.KH == 3;
  // 64 output channels per workgroup and ~2 workgroups per CU: the kernel is built for two
  // waves per SIMD (amdgpu_waves_per_eu(2)), which hides the DMA / transposed-read latency
  // that bound the one-wave 128-channel variant (scripts/bench_convs.py on MI355X: 3x3
  // wgrads 1.2-1.3x faster, 1x5/5x1 1.05-1.1x)
  // 1x5 / 5x1 (a.mt5 == 2): 128 output channels per workgroup -- twice the MFMAs per staged
  // dY tile and halo block for the 5-tap convs, whose 64-channel steps are short
  pl.BM = (!sq && a.mt5 >= 2) ? 128 : 64;
  pl.BN = 64 * a.KH * a.KW;
  pl.tilesM = (a.N + pl.BM - 1) / pl.BM;
  pl.tilesN = a.Cin / 64;
  pl.Npad = pl.tilesM * pl.BM;
  const int TH = sq ? 8 : (a.KH == 5 ? 16 : 1), TW = 64 / TH;
  const long ntiles = (long)a.B * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  long splits, g;
  choose_splits((long)pl.tilesM * pl.tilesN, ntiles, splits, g,
                512 / std::max(1, a.grid_div));
  long per = (ntiles + splits - 1) / splits;
  if ((ntiles + per - 1) / per != splits) g = 0;
  pl.nsplit = (int)((ntiles + per - 1) / per);
  pl.pix_per_split = per;
  pl.xcd_g = (int)g;
  return pl;
}

inline WgradPlan plan_conv_wgrad(const ConvWgradArgs& a) {
  bool v3 = wgrad3_shape(a.KH, a.KW) && a.Cin % 64 == 0;
  for (int i = 0; i < a.nsrc; ++i) v3 = v3 && a.src[i].C % 64 == 0;
  if (v3) return plan_conv_wgrad3(a);
  WgradPlan pl{};
  pl.kind = 2;
  const bool big = a.N > 64;
  pl.BM = big ? 128 : 64;
  pl.BN = 128;
  pl.tilesM = (a.N + pl.BM - 1) / pl.BM;
  pl.tilesN = (a.K + pl.BN - 1) / pl.BN;
  pl.Npad = pl.tilesM * pl.BM;
  long splits, g;
  choose_splits((long)pl.tilesM * pl.tilesN, (a.P + 255) / 256, splits, g,
                (a.wg2_stages == 2 ? 512 : 256) / std::max(1, a.grid_div));
  long per = (a.P + splits - 1) / splits;
  per = (per + kWgradBK - 1) / kWgradBK * kWgradBK;
  if ((a.P + per - 1) / per != splits) g = 0;  // rounding dropped a split: plain mapping
  pl.nsplit = (int)((a.P + per - 1) / per);
  pl.pix_per_split = per;
  pl.xcd_g = (int)g;
  return pl;
}


// ---------------------------------------------------------------------------- conv_fwd6 plan
// LDS of a conv_fwd6 workgroup (csrc/conv_igemm.hip): a 3-stage weight ring of BN rows x 128 B,
// then two strip buffers of fwd6_sb(BN) bytes whose last 128-B row is a zero row.  The odd
// strip is reached with the ds_read immediate offset, hence SB <= 65408.
constexpr int kFwd6Lds = 160 * 1024;
RAFT_HD constexpr int fwd6_sb(int BN) {
  return (((kFwd6Lds - 3 * BN * 128) / 2) & ~127) < 65408 ? (((kFwd6Lds - 3 * BN * 128) / 2) & ~127) : 65408;
}
RAFT_HD constexpr int fwd6_max_rows(int BN) { return fwd6_sb(BN) / 128 - 1; }

// flat strip (rows m0 - (PH W + PW) ... of the pixel order) of a BM-pixel tile, padded to
// whole DMA pieces of the NW waves; 0 when it does not fit
RAFT_HD inline int fwd6_strip_rows(int BM, int NW, int KH, int KW, int W, int max_rows) {
  const int need = BM + (KH - 1) * W + KW - 1;
  const int rows = (need + 8 * NW - 1) / (8 * NW) * (8 * NW);
  return rows <= max_rows ? rows : 0;
}

// 2-D tile of TH x TW output pixels: its halo block of (TH + KH - 1) x (TW + KW - 1) pixels,
// padded to whole 8-row DMA pieces (the NW waves take pieces wave, wave + NW, ...; the last
// round may leave some waves without one).  Padding to 8 rows instead of 8 * NW keeps the 64 x 64
// tiles' LDS under a third of the CU (three workgroups per CU).
RAFT_HD constexpr int fwd6_halo_rows(int TH, int TW, int KH, int KW, int NW) {
  const int rows = (TH + KH - 1) * (TW + KW - 1);
  return NW > 0 ? (rows + 7) / 8 * 8 : 0;
}

// v6 variant the forward dispatcher picks for a multi-tap stride-1 conv of N outputs over
// B x H x W pixels (0: v5 / v4).  Two tile families:
//   128 x 64 (4 waves of 32 x 64, <= 74 KB of LDS: two workgroups per CU, 512 slots):
//     62 = 2-D tiles: 3x3 as 8 x 16, 1x5 as 2 x 64, 5x1 as 16 x 8;  64 = 5x1 as 8 x 16;
//     65 = 1x5 as a flat 128-pixel strip (132 halo rows at any width: wide images);
//   64 x 64 (2x2 waves of 32 x 32, <= 53.5 KB: three workgroups per CU, 768 slots):
//     74 = 3x3 as 4 x 16, 5x1 as 8 x 8;  75 = 1x5 as 2 x 32.
// The choice is the lower modelled time of the two families (fwd6_grid_cost): whole rounds of
// workgroups over the slots cost 1 each, a partial round of fraction f costs 0.35 + 0.65 f (its
// workgroups share their CUs with fewer others), and a 64 x 64 round costs 0.83 of a 128 x 64
// round.  Fitted on scripts/bench_conv6.py over the update-block forward / data-gradient shapes
// at batch 8 x 46 x 62, 1 and 2 x 46 x 96 and 1080p (profiles/r6t_conv6_*.log): 64 x 64 wins
// 10-30 % at batch 1-2 per GPU (70-300 workgroups of 128 x 64 for 512 slots) and on the batch-8
// shapes with < 1.2 or 2.2-2.9 rounds of 128 x 64 workgroups; 4 % below automatic over the 72
// measured cases, 0.7 % above the per-case best.
RAFT_HD inline int fwd6_tiles2d(int B, int H, int W, int TH, int TW) {
  return B * ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
}
RAFT_HD inline double fwd6_grid_cost(long wgs, int slots) {
  const long full = wgs / slots;
  const double f = (double)(wgs - full * slots) / slots;
  return (double)full + (f > 0.0 ? 0.35 + 0.65 * f : 0.0);
}
RAFT_HD inline int choose_fwd6(int KH, int KW, int N, int B, int H, int W, bool small_tiles = true) {
  const long tn = (N + 63) / 64;
  int base;
  long wb, ws;  // workgroups of the 128 x 64 choice / of the 64 x 64 one
  if (KH == 3 && KW == 3) {
    base = 62;
    wb = fwd6_tiles2d(B, H, W, 8, 16) * tn;
    ws = fwd6_tiles2d(B, H, W, 4, 16) * tn;
  } else if (KH == 1 && KW == 5) {
    base = W <= 64 ? 62 : 65;
    wb = (base == 62 ? (long)fwd6_tiles2d(B, H, W, 2, 64) : ((long)B * H * W + 127) / 128) * tn;
    ws = fwd6_tiles2d(B, H, W, 2, 32) * tn;
  } else if (KH == 5 && KW == 1) {
    // 16 x 8 or 8 x 16: fewer 512-slot rounds (16 x 8: less halo per pixel, 8 x 16: fewer tiles
    // on 1080p's 135-row planes)
    const long r62 = (fwd6_tiles2d(B, H, W, 16, 8) * tn + 511) / 512;
    const long r64 = (fwd6_tiles2d(B, H, W, 8, 16) * tn + 511) / 512;
    base = r64 < r62 ? 64 : 62;
    wb = (base == 62 ? fwd6_tiles2d(B, H, W, 16, 8) : fwd6_tiles2d(B, H, W, 8, 16)) * tn;
    ws = fwd6_tiles2d(B, H, W, 8, 8) * tn;
  } else {
    return 0;
  }
  const int small = KH == 1 ? 75 : 74;
  return small_tiles && 0.83 * fwd6_grid_cost(ws, 768) < fwd6_grid_cost(wb, 512) ? small : base;
}

// ============================================================================ convex upsampling
// The row-segment kernels (csrc/convex_upsample.hip) take a dense channels-last mask: (P, 576)
// rows (channel stride 1, pixel stride 576), 16-byte aligned rows of a 2- or 4-byte type, and
// every offset they form (B * H * W * 128 output floats, B * sN mask elements) within 32 bits.
inline bool up_seg_ok(unsigned long addr, int esz, long sN, long sC, long sH, long sW, int B, int H, int W) {
  const long align = 16 / esz;
  return sC == 1 && sW == 576 && sH % align == 0 && sN % align == 0 && (addr & 15) == 0 &&
         (long)B * sN < (1L << 31) && (long)B * H * W * 128 < (1L << 31) && (long)sH * H <= sN;
}

// ============================================================================ correlation build
// Row tiles per group of the v2 volume build's tile order (cfg 2-5 force 1 / 2 / 4 / 16):
// 8 while one image's B operand (N x K bf16) fits 8 MB, 4 beyond (the 1080p store stream).
// Clip + AdamW optimizer step (optim.hip): parameter chunks of kAdamChunk elements, one block
// each; gradients of up to kAdamGrads tensors per launch travel in the kernel arguments.
constexpr int kAdamChunk = 16384;
constexpr int kAdamGrads = 128;
struct AdamArgs {
  const float* g[kAdamGrads];  // gradients of tensors [t0, t0 + kAdamGrads)
  int t0;
  const long long* ptrs;       // [ntensor][3]: parameter, exp_avg, exp_avg_sq (fp32, grad layout)
  const int* blocks;           // [nblocks][3]: tensor, first element, length
  int blk0, nblocks;           // first block of this launch; blocks of the whole parameter set
  float* partial;              // [nblocks] sums of squared gradients
  float* steps;                // [2] step counter slots: read [par], block 0 writes [par ^ 1]
  int par;
  float lr, beta1, beta2, eps, wd, max_norm;  // max_norm <= 0: no clipping
  float* norm_out;             // the total gradient norm (may be null)
  float* skipped;              // += 1 when the norm is not finite (may be null)
};

RAFT_HD inline int corr_group_rows(long N, long K, int cfg) {
  if (cfg >= 2 && cfg <= 5) return cfg == 2 ? 1 : cfg == 3 ? 2 : cfg == 4 ? 4 : 16;
  if (cfg == 7) return 8;
  return N * K * 2 <= (8L << 20) ? 8 : 4;
}

}  // namespace raft_amd

#ifndef RAFT_ABI_NO_HIP
#include <hip/hip_runtime_api.h>

namespace raft_amd {
// optim.hip
hipError_t launch_adamw(const AdamArgs& a, int nblk, bool update, hipStream_t s);
// conv_igemm.hip
hipError_t launch_conv_fwd(const ConvFwdArgs& a, hipStream_t s);
hipError_t launch_conv_wgrad(ConvWgradArgs a, const WgradPlan& pl, hipStream_t s);
// weights.hip
hipError_t launch_pack_conv_weights(const ConvParamDesc& d, int N, void* wf, int Kf, void* wd, int Kd, int Cout_pad,
                                    float* bias, hipStream_t s);
hipError_t launch_pack_conv_weights_multi(const PackJobs& js, hipStream_t s);
hipError_t launch_wgrad_reduce_params(const float* slab, int nsplit, int Npad, int Kpad, const float* dbslab, int ndb,
                                      const ConvParamDesc& d, int N, int accumulate, hipStream_t s);
hipError_t launch_wgrad_reduce_packed(const float* slab, int nsplit, int Npad, int Kpad, int K, const float* dbslab,
                                      int ndb, float* dw, long ldw, float* db, int N, int accumulate, hipStream_t s);
// encoder.hip
int enc_tile_bn(int N);
hipError_t launch_enc_pack(const EncConvArgs& a, int rows, void* out, hipStream_t s);
hipError_t launch_enc_pack_multi(const void* plan, int njobs, int nblocks, void* out, hipStream_t s);
hipError_t launch_enc_conv(const EncConvArgs& a, int nblocks, hipStream_t s);
hipError_t launch_enc_conv3(const EncConvArgs& a, hipStream_t s);
hipError_t launch_enc_wgrad(const EncWgradArgs& a, int BM, int BN, hipStream_t s);
hipError_t launch_enc_wgrad_reduce(const float* slab, int nsplit, int Npad, int Kpad, const float* dbslab, float* dw,
                                   const long* ws, int Cout, int Cin, int Cx, int KH, int KW, float* db,
                                   bool accumulate, int fold, hipStream_t s);
hipError_t launch_enc_prep(const float* i0, const float* i1, const long* st, int B, int H, int W, int nimg,
                           void* out, int split, hipStream_t s);
hipError_t launch_enc_norm_finalize(const NormFinArgs& a, hipStream_t s);
hipError_t launch_enc_apply(const void* a, const float* ca, bool relu_a, const void* r, const float* cr,
                            bool relu_out, void* out, int B, int HW, int N, int split, hipStream_t s);
hipError_t launch_enc_norm_bwd(const NormBwdArgs& a, hipStream_t s);
// stages: bit 0 reduce (partials of a.B images), bit 1 finalize (over b_fin > 0 images'
// partials when given: synchronized BatchNorm), bit 2 apply
hipError_t launch_enc_norm_bwd_stages(const NormBwdArgs& a, int stages, int b_fin, hipStream_t s);
}  // namespace raft_amd
#endif
