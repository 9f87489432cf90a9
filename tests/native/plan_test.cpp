// Host-side unit test of the kernel work planning in csrc/kernel_abi.h, built and run under
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_plan_cpu.py (no GPU):
//   * xcd_remap is a bijection of [0, nwg) for every grid size;
//   * every weight-gradient plan (v2 pixel splits, v3 tap-batched tile splits, with and
//     without the XCD-grouped mapping) covers each (split, output tile) pair exactly once,
//     has no empty split, pads N to whole row tiles and keeps the pixel ranges in bounds;
//   * the slab sizes the bindings allocate from a plan stay addressable;
//   * the conv_fwd6 variant choice (measured winners at the benchmark shapes; every chosen
//     strip / halo block fits the kernel's LDS at any width);
//   * the convex-upsampling kernel choice and the correlation build's tile grouping.
#define RAFT_ABI_NO_HIP
#include "kernel_abi.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace raft_amd;

static int failures = 0;
#define EXPECT(cond, ...)                                  \
  do {                                                     \
    if (!(cond)) {                                         \
      ++failures;                                          \
      if (failures < 20) {                                 \
        std::fprintf(stderr, "FAIL %s:%d: %s | ", __FILE__, __LINE__, #cond); \
        std::fprintf(stderr, __VA_ARGS__);                 \
        std::fprintf(stderr, "\n");                        \
      }                                                    \
    }                                                      \
  } while (0)

static void test_xcd_remap() {
  for (int nwg = 1; nwg <= 4099; nwg += (nwg < 64 ? 1 : 37)) {
    std::vector<int> seen(nwg, 0);
    for (int b = 0; b < nwg; ++b) {
      const int w = xcd_remap(b, nwg);
      EXPECT(w >= 0 && w < nwg, "nwg=%d b=%d -> %d", nwg, b, w);
      if (w >= 0 && w < nwg) ++seen[w];
    }
    for (int w = 0; w < nwg; ++w) EXPECT(seen[w] == 1, "nwg=%d tile %d seen %d times", nwg, w, seen[w]);
  }
}

static ConvWgradArgs make_args(int B, int H, int W, int KH, int KW, int Cin, int N, int nsrc) {
  ConvWgradArgs a{};
  a.B = B;
  a.H = H;
  a.W = W;
  a.KH = KH;
  a.KW = KW;
  a.PH = KH / 2;
  a.PW = KW / 2;
  a.nsrc = nsrc;
  a.Cin = Cin;
  const int per = Cin / nsrc;
  for (int i = 0; i < nsrc; ++i) {
    a.src[i].C = per;
    a.src[i].stride = per;
    a.src[i].period = 0;
  }
  a.K = KH * KW * Cin;
  a.Kpad = (a.K + 63) / 64 * 64;
  a.N = N;
  a.dy_stride = (N + 7) / 8 * 8;
  a.P = (long)B * H * W;
  return a;
}

static void check_plan(const ConvWgradArgs& a) {
  const WgradPlan pl = plan_conv_wgrad(a);
  EXPECT(pl.kind == 2 || pl.kind == 3, "kind %d", pl.kind);
  EXPECT(pl.nsplit >= 1 && pl.tilesM >= 1 && pl.tilesN >= 1, "nsplit %d tiles %dx%d", pl.nsplit, pl.tilesM,
         pl.tilesN);
  EXPECT(pl.Npad == pl.tilesM * pl.BM && pl.Npad >= a.N && pl.Npad - a.N < pl.BM, "Npad %d N %d BM %d", pl.Npad,
         a.N, pl.BM);
  // work units split over the grid: pixels (v2) or 64-pixel tiles (v3)
  long units;
  if (pl.kind == 3) {
    const int TH = a.KH == 3 ? 8 : (a.KH == 5 ? 16 : 1), TW = 64 / TH;
    units = (long)a.B * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
    EXPECT(pl.tilesN == a.Cin / 64, "v3 chunks %d for Cin %d", pl.tilesN, a.Cin);
  } else {
    units = a.P;
    EXPECT(pl.pix_per_split % kWgradBK == 0, "v2 split %ld not a multiple of the K step", pl.pix_per_split);
    EXPECT(pl.tilesN * pl.BN >= a.K, "v2 column tiles %d x %d < K %d", pl.tilesN, pl.BN, a.K);
  }
  EXPECT(pl.pix_per_split >= 1, "pix_per_split %ld", pl.pix_per_split);
  EXPECT((long)(pl.nsplit - 1) * pl.pix_per_split < units, "empty split: %d x %ld vs %ld", pl.nsplit,
         pl.pix_per_split, units);
  EXPECT((long)pl.nsplit * pl.pix_per_split >= units, "uncovered work: %d x %ld < %ld", pl.nsplit, pl.pix_per_split,
         units);
  if (pl.xcd_g > 0) EXPECT(pl.nsplit == 8 * pl.xcd_g, "xcd_g %d with nsplit %d", pl.xcd_g, pl.nsplit);
  // the launch grid and its workgroup -> (split, tile) map
  const int tiles = pl.tilesM * pl.tilesN;
  const long grid = (long)tiles * pl.nsplit;
  std::vector<int> seen(grid, 0);
  for (long b = 0; b < grid; ++b) {
    int split, tile;
    wgrad_block_map((int)b, tiles, pl.xcd_g, split, tile);
    EXPECT(split >= 0 && split < pl.nsplit && tile >= 0 && tile < tiles, "bid %ld -> split %d tile %d", b, split,
           tile);
    if (split >= 0 && split < pl.nsplit && tile >= 0 && tile < tiles) ++seen[(long)split * tiles + tile];
  }
  for (long i = 0; i < grid; ++i) EXPECT(seen[i] == 1, "(split, tile) %ld visited %d times", i, seen[i]);
  // slabs the bindings allocate: [nsplit][Npad][Kpad] fp32 (+ bias partials)
  const double slab_bytes = 4.0 * pl.nsplit * (double)pl.Npad * a.Kpad;
  EXPECT(slab_bytes < 16e9, "slab %.1f GB", slab_bytes / 1e9);
}

static void test_wgrad_plans() {
  const int shapes[][2] = {{1, 1}, {3, 3}, {1, 5}, {5, 1}, {7, 7}};
  const int couts[] = {2, 8, 64, 96, 126, 128, 192, 256, 384, 512, 576};
  const int cins[] = {64, 128, 256, 384};
  const int dims[][3] = {{8, 46, 62}, {96, 46, 62}, {1, 16, 16}, {2, 55, 156}, {6, 135, 240}};
  int n = 0;
  for (auto& s : shapes)
    for (int N : couts)
      for (int Cin : cins)
        for (auto& d : dims)
          for (int nsrc = 1; nsrc <= 3; ++nsrc) {
            if (Cin % nsrc || (Cin / nsrc) % (nsrc > 1 ? 128 : 8)) continue;
            ConvWgradArgs a = make_args(d[0], d[1], d[2], s[0], s[1], Cin, N, nsrc);
            if (!wgrad_supported(a)) continue;
            for (int mt5 = 1; mt5 <= 2; ++mt5) {  // 64- / 128-row workgroups of the 1x5 / 5x1 v3 kernel
              a.mt5 = mt5;
              check_plan(a);
              if (s[0] * s[1] == 5 && plan_conv_wgrad(a).kind == 3)
                EXPECT(plan_conv_wgrad(a).BM == (mt5 >= 2 ? 128 : 64), "1x5 / 5x1 v3 rows %d for mt5 %d",
                       plan_conv_wgrad(a).BM, mt5);
              ++n;
            }
          }
  EXPECT(n > 300, "only %d plans checked", n);
  std::printf("checked %d weight-gradient plans\n", n);
}

// conv_fwd6 selection: the measured choices at the benchmark shapes, and every chosen variant's
// strip / halo block fits the LDS the kernel allocates, at any image width
static void test_fwd6_plan() {
  // config #2 (8 x 46 x 62), measured per shape (profiles/r6t_conv6_b8.log): 64 x 64 tiles where
  // the 128 x 64 grid leaves a partial round (conv 384, convc2 576 workgroups for 512 slots) ...
  EXPECT(choose_fwd6(3, 3, 126, 8, 46, 62) == 74, "conv");
  EXPECT(choose_fwd6(3, 3, 192, 8, 46, 62) == 74, "convc2");
  EXPECT(choose_fwd6(3, 3, 64, 8, 46, 62) == 74, "convf2");
  EXPECT(choose_fwd6(1, 5, 128, 8, 46, 62) == 75, "q 1x5");
  EXPECT(choose_fwd6(5, 1, 384, 8, 46, 62) == 74, "5x1 data gradient");
  // ... and 128 x 64 on whole rounds (heads: 1536 = 3 x 512)
  EXPECT(choose_fwd6(3, 3, 512, 8, 46, 62) == 62, "heads");
  // (N = 256: 768 vs 1536 workgroups model and measure as a tie, 21.9 vs 22.3 us)
  // batch 1 at 368 x 768 (46 x 96, the per-rank work of train_standard.sh on 8 GPUs): 64 x 64
  for (int N : {64, 126, 192, 256, 384, 512}) {
    EXPECT(choose_fwd6(3, 3, N, 1, 46, 96) == 74, "b1 3x3 N=%d", N);
    EXPECT(choose_fwd6(1, 5, N, 1, 46, 96) == 75, "b1 1x5 N=%d", N);
  }
  // batch 2: the N = 384 data gradients stay on 128 x 64 (864 / 1104 small workgroups > 768)
  EXPECT(choose_fwd6(5, 1, 384, 2, 46, 96) == 62, "b2 5x1 data gradient");
  EXPECT(choose_fwd6(1, 5, 384, 2, 46, 96) == 65, "b2 1x5 data gradient");
  EXPECT(choose_fwd6(3, 3, 512, 2, 46, 96) == 74, "b2 heads");
  // 1080p (1 x 135 x 240): flat 1x5 strips; the 5x1 z||r on 8 x 16 (1020 vs 1080 workgroups)
  EXPECT(choose_fwd6(1, 5, 256, 1, 135, 240) == 65, "1080p 1x5");
  EXPECT(choose_fwd6(5, 1, 256, 1, 135, 240) == 64, "1080p 5x1 z||r");
  EXPECT(choose_fwd6(5, 1, 128, 1, 135, 240) == 64, "1080p 5x1 q");
  EXPECT(choose_fwd6(3, 3, 126, 1, 135, 240) == 62, "1080p conv");
  EXPECT(choose_fwd6(7, 7, 128, 1, 135, 240) == 0, "7x7 -> v4");
  // every choice fits: 2-D halo blocks / the flat 1x5 strip within the LDS of two (128 x 64) or
  // three (64 x 64) workgroups per CU
  const int taps[3][2] = {{3, 3}, {1, 5}, {5, 1}};
  for (int B : {1, 2, 8})
    for (int W = 1; W <= 400; W += (B == 2 ? 1 : 7))
      for (int H = 1; H <= 140; H += 13)
        for (const auto& t : taps)
          for (int N = 64; N <= 576; N += 64) {
            const int kh = t[0], kw = t[1];
            const int c = choose_fwd6(kh, kw, N, B, H, W);
            EXPECT(c == 62 || c == 64 || c == 65 || c == 74 || c == 75, "cfg %d", c);
            if (c == 64) EXPECT(kh == 5, "64 is a 5x1 tile");
            if (c == 65) EXPECT(kh == 1 && W > 64, "65: wide 1x5");
            if (c == 74) EXPECT(kw == 3 || kh == 5, "74: 3x3 / 5x1");
            if (c == 75) EXPECT(kh == 1, "75: 1x5");
            if (c >= 74) {
              const int halo = kh == 3 ? fwd6_halo_rows(4, 16, 3, 3, 4)
                               : kh == 5 ? fwd6_halo_rows(8, 8, 5, 1, 4) : fwd6_halo_rows(2, 32, 1, 5, 4);
              EXPECT(3 * 64 * 128 + 2 * (halo + 1) * 128 <= kFwd6Lds / 3, "three workgroups per CU: halo %d", halo);
              continue;
            }
            const int halo = c == 65 ? (128 + 4 + 31) / 32 * 32
                             : c == 64 ? fwd6_halo_rows(8, 16, kh, kw, 4)
                             : kh == 3 ? fwd6_halo_rows(8, 16, 3, 3, 4)
                             : kh == 1 ? fwd6_halo_rows(2, 64, 1, 5, 4) : fwd6_halo_rows(16, 8, 5, 1, 4);
            EXPECT(3 * 64 * 128 + 2 * (halo + 1) * 128 <= kFwd6Lds / 2, "two workgroups per CU: halo %d", halo);
          }
  EXPECT(2 * fwd6_sb(128) + 3 * 128 * 128 <= kFwd6Lds && fwd6_sb(64) <= 65408, "LDS layout");
}

// convex upsampling: channels-last masks (the mask head's rows) take the row-segment kernels,
// NCHW / misaligned / oversized ones the per-pixel kernels
static void test_upsample_and_corr_selection() {
  const int B = 8, H = 46, W = 62;
  const long HW = (long)H * W;
  EXPECT(up_seg_ok(0x1000, 2, HW * 576, 1, W * 576L, 576, B, H, W), "channels-last bf16");
  EXPECT(up_seg_ok(0x1000, 4, HW * 576, 1, W * 576L, 576, B, H, W), "channels-last fp32");
  EXPECT(!up_seg_ok(0x1000, 2, 576 * HW, HW, W, 1, B, H, W), "NCHW");
  EXPECT(!up_seg_ok(0x1008, 2, HW * 576, 1, W * 576L, 576, B, H, W), "misaligned");
  EXPECT(!up_seg_ok(0x1000, 2, HW * 576 + 4, 1, W * 576L, 576, B, H, W), "unaligned image stride");
  EXPECT(!up_seg_ok(0x1000, 2, 4000L * 4000 * 576, 1, 4000L * 576, 576, 2, 4000, 4000), "32-bit offsets");
  // correlation build tile groups: 8 at config #2 / Sintel, 4 at 1080p, forced by cfg 2-5
  EXPECT(corr_group_rows(3936, 256, 0) == 8 && corr_group_rows(9280, 256, 0) == 8, "small B");
  EXPECT(corr_group_rows(43600, 256, 0) == 4, "1080p");
  EXPECT(corr_group_rows(43600, 256, 2) == 1 && corr_group_rows(10, 256, 5) == 16, "forced");
}

int main() {
  test_xcd_remap();
  test_upsample_and_corr_selection();
  test_wgrad_plans();
  test_fwd6_plan();
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
