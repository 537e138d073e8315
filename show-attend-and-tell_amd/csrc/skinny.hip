// Register-direct skinny GEMM for the decoder's per-step products (gfx950 / MI355X).
//
//   C_s[m, n] = sum_{k in split s} A[m, k] W[n, k]  (+ bias[n] in split 0),  M <= 128 rows (the batch),
//   A, W bf16 row-major (k contiguous), C fp32; split s writes its own slab C + s * split_stride
//   (the decoder's partial-output split-K contract, SatGemm::partial_splits), or plain C when unsplit.
//
// Why: the per-step GEMMs of the recurrent loop -- [U; f_beta; W_hh] h (N 4608, K 512), the context half of the LSTM
// input GEMM (N 2048, K 2048) and the BPTT's dL/d(gated context) / dL/dh products at M = B = 128 (decoder.py:96-115)
// -- move 5-10 MB each and sit in a dependent chain, so their time is latency, not bandwidth.  The LDS-DMA
// tile kernel (convgemm.hip) runs a 3-stage ring with a barrier per 64-deep k-tile and holds 74 KB of
// LDS, which also keeps it off every CU where a concurrent encoder workgroup lives.  Here:
//   * a workgroup owns 32 output columns x all rows; its NW waves split the workgroup's K range
//     (<= 128 per wave: 4 k-steps of 32);
//   * every operand fragment of the wave -- A rows (MB 16-row blocks) and W rows (2 16-column blocks),
//     16 B per lane per k-step -- is requested at kernel entry straight into VGPRs, so the launch pays
//     one memory latency; no LDS ring, no per-k-tile barrier;
//   * v_mfma_f32_16x16x32_bf16 with W as the A operand computes C^T, so a lane ends with 4 consecutive
//     columns of one row;
//   * the NW partial tiles meet in one 18 KB LDS tile in wave order (fixed summation order: results
//     do not depend on scheduling), then the workgroup stores 16-B row pieces.
// Measured and not kept (profiles/r5_s10, r5_s16): an XCD-aware workgroup order (the column blocks of one split on
// one XCD: fewer fabric reads of A, the h GEMM 7.5 -> 9.1 us), 64-column workgroups of eight waves (half the
// workgroups and ~60 % of the bytes moved: 7.6 -> 11.9 us per product, step 6.40 -> 6.47-6.50 ms).
#include "sat_common.h"
#include "sat_internal.h"

namespace {

constexpr int SK_COLS = 32;            // output columns per workgroup
constexpr int SK_RLD = SK_COLS + 4;    // LDS tile row stride (floats)
constexpr int SK_KW = 128;             // max k per wave

struct SkArgs {
  int M, N, K, kc, kw;                 // kc: k per split (multiple of 32); kw: k per wave (<= 128)
  const bf16* A; long lda;
  const bf16* W; long ldw;
  float* C; long ldc; long split_stride;
  const float* bias;
  int gate_E;                          // > 0: gate-interleaved columns (local column c of block x = W row / output
                                       // column (c >> 3) * gate_E + 8 x + (c & 7)); 0: block x owns 32 x .. 32 x + 31
  SatStamps st;
};

__device__ __forceinline__ int col_of(const SkArgs& a, int c) {
  return a.gate_E > 0 ? (c >> 3) * a.gate_E + (int)blockIdx.x * 8 + (c & 7) : (int)blockIdx.x * SK_COLS + c;
}

// The GEMM of one (column block, split): every fragment load at entry, the MFMAs, and the waves' partial tiles
// folded into red[MB * 16][SK_RLD] in wave order (ends behind a barrier).
template <int MB, int NW>
__device__ __forceinline__ void skinny_tile(const SkArgs& a, float* red) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int s = blockIdx.y;
  const int kbeg = s * a.kc + w * a.kw;
  int kend = kbeg + a.kw;
  kend = min(kend, min((s + 1) * a.kc, a.K));
  const int nks = kend > kbeg ? (kend - kbeg) >> 5 : 0;   // wave-uniform, <= 4

  // every fragment load of the wave up front (rows past M re-read row M-1 and are never stored)
  const bf16* wr[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) wr[j] = a.W + (long)col_of(a, j * 16 + fr) * a.ldw;
  bf16x8 af[4][MB], bw[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if (ks < nks) {
      const int k = kbeg + ks * 32 + 8 * fh;
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int row = min(i * 16 + fr, a.M - 1);
        af[ks][i] = *(const bf16x8*)(a.A + (long)row * a.lda + k);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) bw[ks][j] = *(const bf16x8*)(wr[j] + k);
    }
  }
  f32x4 acc[MB][2];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if (ks < nks) {
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
    }
  }
  // lane holds C[i*16 + fr][j*16 + 4fh .. +3]: the waves' partial tiles meet in LDS in wave order
  for (int r = 0; r < NW; ++r) {
    if (w == r) {
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float4* p = (float4*)(red + (i * 16 + fr) * SK_RLD + j * 16 + 4 * fh);
          float4 v = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
          if (r > 0) {
            const float4 o = *p;
            v.x = o.x + v.x; v.y = o.y + v.y; v.z = o.z + v.z; v.w = o.w + v.w;
          }
          *p = v;
        }
    }
    __syncthreads();
  }
}

template <int MB, int NW>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(SkArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  __shared__ __attribute__((aligned(16))) float red[MB * 16 * SK_RLD];
  skinny_tile<MB, NW>(a, red);
  // store: 8 float4 pieces per row, bias in split 0
  const int s = blockIdx.y;
  float* const Cs = a.C + (long)s * a.split_stride;
  const float* const bias = s == 0 ? a.bias : nullptr;
  constexpr int PIECES = MB * 16 * (SK_COLS / 4);
  // write-through (sat_common.h): the slabs go to memory while the kernel runs, so its end-of-kernel L2 writeback --
  // on the decoder's per-step critical path -- has little left to flush
  const __amdgpu_buffer_rsrc_t rC = sat_out_rsrc(Cs, 0x7fffffffL);
  for (int q = threadIdx.x; q < PIECES; q += NW * 64) {
    const int row = q >> 3, c4 = (q & 7) * 4;
    if (row >= a.M) continue;
    float4 v = *(const float4*)(red + row * SK_RLD + c4);
    const int n = col_of(a, c4);
    if (bias) {
      const float4 b = *(const float4*)(bias + n);
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    sat_st16(rC, (unsigned)(((long)row * a.ldc + n) * 4), *(const uint4*)&v);
  }
  sat_stamp_end(a.st, t0);
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Shape / split eligibility of the skinny kernel for g (no pointer checks); fills a (pointers included) and nw.
bool skinny_shape(const SatGemm& g, int mode, SkArgs* a, int* nw) {
  if (mode == 1) return false;
  // mode 0: only products the decoder split for this kernel (partial splits of 256 - 1024 deep K ranges in
  // whole 256-deep slabs: the context GEMM 9.2 vs 10.9 us per step; the backward's products through the
  // transposed weight copies); the [U; f_beta; W_hh] h GEMM (one split) stays on the tile kernel (8.2 vs 8.6
  // us: with K = 512 every workgroup reads all of A); mode 2: every eligible problem (tests)
  if (mode == 0 && !(g.partial_splits > 1 && g.K % g.partial_splits == 0 && (g.K / g.partial_splits) % 256 == 0 &&
                     g.K / g.partial_splits <= 1024))
    return false;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_F32 || g.batch != 1 || g.conv.C > 0) return false;
  if (g.transA || g.transB || g.aux || g.add1 || g.act != SAT_ACT_NONE || g.beta != 0.f || g.alpha != 1.f) return false;
  if (g.M < 1 || g.M > 128 || g.N % SK_COLS || g.K % 32 || g.K <= 0) return false;
  if (g.lda % 8 || g.ldb % 8 || g.ldc % 4) return false;
  const int S = g.partial_splits > 1 ? g.partial_splits : 1;
  if (S > 1 && g.split_stride % 4) return false;
  // the fast path's split geometry: split s covers [s kc, (s+1) kc), kc a multiple of 64
  const int kc = sat_cdiv(sat_cdiv(g.K, S), 64) * 64;
  if (kc > 8 * SK_KW) return false;
  *nw = kc > 4 * SK_KW ? 8 : 4;
  SkArgs x{};
  x.M = g.M; x.N = g.N; x.K = g.K; x.kc = kc;
  x.kw = sat_cdiv(sat_cdiv(kc, *nw), 32) * 32;
  if (x.kw > SK_KW) return false;
  x.A = (const bf16*)g.A; x.lda = g.lda;
  x.W = (const bf16*)g.B; x.ldw = g.ldb;
  x.C = (float*)g.C; x.ldc = g.ldc; x.split_stride = S > 1 ? g.split_stride : 0;
  x.bias = g.bias;
  *a = x;
  return true;
}

bool skinny_ptrs(const SatGemm& g) {
  // + the slab stores' buffer resource takes 32-bit offsets (sat_out_rsrc's 2 GiB cap)
  return al16(g.A) && al16(g.B) && al16(g.C) && (!g.bias || al16(g.bias)) &&
         4L * ((long)(g.M - 1) * g.ldc + g.N) < (1L << 31);
}

template <int MB>
void launch_mb(int nw, dim3 grid, hipStream_t st, const SkArgs& a) {
  if (nw == 8) hipLaunchKernelGGL((skinny_gemm_kernel<MB, 8>), grid, dim3(512), 0, st, a);
  else hipLaunchKernelGGL((skinny_gemm_kernel<MB, 4>), grid, dim3(256), 0, st, a);
}

}  // namespace

int sat_skinny_try(const SatGemm& g, hipStream_t st, int* err) {
  *err = 0;
  SkArgs a;
  int nw;
  if (!skinny_shape(g, sat_policy().skinny, &a, &nw) || !skinny_ptrs(g)) return 0;
  a.st = sat_launch_stamps();
  const dim3 grid(g.N / SK_COLS, g.partial_splits > 1 ? g.partial_splits : 1);
  if (g.M <= 32) launch_mb<2>(nw, grid, st, a);
  else if (g.M <= 64) launch_mb<4>(nw, grid, st, a);
  else launch_mb<8>(nw, grid, st, a);
  *err = (int)hipGetLastError();
  return 1;
}

// splits the decoder asks for when the skinny kernel runs its per-step GEMMs: 256-deep K per split
// (less A per workgroup: every workgroup reads all M rows of its K range), 0 = not eligible
int sat_skinny_splits(int M, int N, int K) {
  if (sat_policy().skinny == 1 || M > 128 || N % SK_COLS || K % 256 || K < 1024) return 0;
  return K / 256;
}

