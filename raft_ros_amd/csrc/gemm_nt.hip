// Batched "NT" bf16 GEMM on gfx950 MFMA:  C[b][m][n] = alpha * sum_k A[b][m][k] * B[b][n][k]
//
// Both operands are K-contiguous rows, which is the natural layout of every
// GEMM in the RAFT correlation path (reference core/corr.py:53-60 builds the
// all-pairs volume as fmap1^T . fmap2 / sqrt(C)):
//   forward   corr[p][q]  = f1_nhwc[p][:] . f2_nhwc[q][:]            (K = C)
//   backward  dF1[p][c]   = dC[p][:]   . f2_nchw[c][:]               (K = HW, padded)
//             dF2[q][c]   = dCt[q][:]  . f1_nchw[c][:]               (K = HW, padded)
//
// Tiling: 256-thread workgroup (4 waves), 128x128 output tile, each wave a
// 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_bf16 accumulators (64 AGPRs).
// K advances 64 per LDS stage; the next stage's global loads are issued into
// registers before the current stage's MFMAs (register double buffering).
// LDS rows are padded by 16 B, which makes the 16-lane ds_read_b128 groups
// conflict-free (row stride 36 dwords -> 16 distinct 4-bank slots).
// Workgroup ids are remapped XCD-aware so neighbouring tiles share an L2.
//
// Requirements (checked on the host): K % 64 == 0, lda/ldb % 8 == 0, 16-byte
// aligned base pointers.  Rows >= M / >= N are zero-filled, not read.
#include "common.h"

namespace raft_amd {

namespace {
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int LDS_ROW = BK + 8;  // bf16 elements per padded LDS row
constexpr int NTHREADS = 256;
constexpr int CHUNKS = BM * BK / 8 / NTHREADS;  // 16-byte chunks per thread per operand (=4)

template <typename OutT>
__global__ __launch_bounds__(NTHREADS) void gemm_nt_bf16_kernel(
    const __bf16* __restrict__ A, long lda, long strideA,
    const __bf16* __restrict__ B, long ldb, long strideB,
    OutT* __restrict__ C, long ldc, long strideC,
    int M, int N, int K, float alpha, int tilesM, int tilesN, int batch) {
  __shared__ __attribute__((aligned(16))) __bf16 sA[BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) __bf16 sB[BN * LDS_ROW];

  const int per_batch = tilesM * tilesN;
  const int nwg = per_batch * batch;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int b = wg / per_batch;
  const int t = wg - b * per_batch;
  const int tm = t / tilesN, tn = t - (t / tilesN) * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;

  A += b * strideA;
  B += b * strideB;
  C += b * strideC;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  u32x4 ra[CHUNKS], rb[CHUNKS];

  auto load_stage = [&](int k0) {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i) {
      const int c = tid + i * NTHREADS;
      const int row = c >> 3, col = (c & 7) * 8;
      const int gm = m0 + row, gn = n0 + row;
      ra[i] = gm < M ? *reinterpret_cast<const u32x4*>(A + (long)gm * lda + k0 + col) : u32x4{0, 0, 0, 0};
      rb[i] = gn < N ? *reinterpret_cast<const u32x4*>(B + (long)gn * ldb + k0 + col) : u32x4{0, 0, 0, 0};
    }
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i) {
      const int c = tid + i * NTHREADS;
      const int row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<u32x4*>(sA + row * LDS_ROW + col) = ra[i];
      *reinterpret_cast<u32x4*>(sB + row * LDS_ROW + col) = rb[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int frag_row = lane & 31;
  const int frag_k = (lane >> 5) * 8;

  load_stage(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    store_stage();
    __syncthreads();
    if (k0 + BK < K) load_stage(k0 + BK);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(sA + (wm * 64 + i * 32 + frag_row) * LDS_ROW + s * 16 + frag_k);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(sB + (wn * 64 + j * 32 + frag_row) * LDS_ROW + s * 16 + frag_k);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) C[(long)row * ldc + col] = from_f32<OutT>(alpha * acc[i][j][r]);
      }
    }
}
}  // namespace

hipError_t launch_gemm_nt_bf16(const void* A, long lda, long strideA, const void* B, long ldb,
                               long strideB, void* C, int out_dtype, long ldc, long strideC, int M,
                               int N, int K, float alpha, int batch, hipStream_t stream) {
  const int tilesM = cdiv(M, BM), tilesN = cdiv(N, BN);
  const dim3 grid(tilesM * tilesN * batch), block(NTHREADS);
  const __bf16* a = static_cast<const __bf16*>(A);
  const __bf16* b = static_cast<const __bf16*>(B);
  if (out_dtype == kF32) {
    hipLaunchKernelGGL(gemm_nt_bf16_kernel<float>, grid, block, 0, stream, a, lda, strideA, b, ldb,
                       strideB, static_cast<float*>(C), ldc, strideC, M, N, K, alpha, tilesM, tilesN,
                       batch);
  } else {
    hipLaunchKernelGGL(gemm_nt_bf16_kernel<__bf16>, grid, block, 0, stream, a, lda, strideA, b, ldb,
                       strideB, static_cast<__bf16*>(C), ldc, strideC, M, N, K, alpha, tilesM, tilesN,
                       batch);
  }
  return hipGetLastError();
}

}  // namespace raft_amd
