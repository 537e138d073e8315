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
#include <utility>

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
  // dual launch (sat_skinny_dual_try): column blocks x >= nb1 run a second product with the same M, K and split
  // geometry (A2 . W2^T -> C2 slabs), so two per-step products that read different operands share one launch
  int nb1;
  const bf16* A2; long lda2;
  const bf16* W2; long ldw2;
  float* C2; long ldc2; long split_stride2;
  SatStamps st;
};

// The GEMM of one tile: rows row0 .. row0 + MB*16 - 1 of A (rows past M re-read row M-1 and are never stored) x
// output columns col0 .. col0 + 31 (W rows past n_lim - 1 re-read row n_lim - 1), over the k range [kbeg, kend) of
// this workgroup, which its NW waves split in kw-deep pieces (<= 4 k-steps of 32 each).  Every fragment load of a
// wave is requested at entry; the waves' partial tiles are folded into red[MB * 16][SK_RLD] in wave order (ends
// behind a barrier).
template <int MB, int NW>
__device__ __forceinline__ void skinny_tile(const bf16* __restrict__ A, long lda, int M, int row0,
                                            const bf16* __restrict__ W, long ldw, int n_lim, int col0, int kbeg,
                                            int kend, int kw, float* red) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int k0 = kbeg + w * kw;
  const int k1 = min(k0 + kw, kend);
  const int nks = k1 > k0 ? (k1 - k0) >> 5 : 0;   // wave-uniform, <= 4

  const bf16* wr[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) wr[j] = W + (long)min(col0 + j * 16 + fr, n_lim - 1) * ldw;
  bf16x8 af[4][MB], bw[4][2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    if (ks < nks) {
      const int k = k0 + ks * 32 + 8 * fh;
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int row = min(row0 + i * 16 + fr, M - 1);
        af[ks][i] = *(const bf16x8*)(A + (long)row * lda + k);
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
  const int s = blockIdx.y;
  const bool second = (int)blockIdx.x >= a.nb1;   // workgroup-uniform
  const int bx = second ? (int)blockIdx.x - a.nb1 : (int)blockIdx.x;
  const bf16* A = second ? a.A2 : a.A;
  const bf16* W = second ? a.W2 : a.W;
  const long lda = second ? a.lda2 : a.lda, ldw = second ? a.ldw2 : a.ldw;
  skinny_tile<MB, NW>(A, lda, a.M, 0, W, ldw, 0x7fffffff, bx * SK_COLS, s * a.kc, min((s + 1) * a.kc, a.K), a.kw,
                      red);
  // store: 8 float4 pieces per row, bias in split 0 (first product only)
  float* const Cs = second ? a.C2 + (long)s * a.split_stride2 : a.C + (long)s * a.split_stride;
  const long ldc = second ? a.ldc2 : a.ldc;
  const float* const bias = s == 0 && !second ? a.bias : nullptr;
  constexpr int PIECES = MB * 16 * (SK_COLS / 4);
  // write-through (sat_common.h): the slabs go to memory while the kernel runs, so its end-of-kernel L2 writeback --
  // on the decoder's per-step critical path -- has little left to flush
  const __amdgpu_buffer_rsrc_t rC = sat_out_rsrc(Cs, 0x7fffffffL);
  for (int q = threadIdx.x; q < PIECES; q += NW * 64) {
    const int row = q >> 3, c4 = (q & 7) * 4;
    if (row >= a.M) continue;
    float4 v = *(const float4*)(red + row * SK_RLD + c4);
    const int n = bx * SK_COLS + c4;
    if (bias) {
      const float4 b = *(const float4*)(bias + n);
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    sat_st16(rC, (unsigned)(((long)row * ldc + n) * 4), *(const uint4*)&v);
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
  // (and, for narrow products, N <= 1024, 128-multiple-deep ones from 256 on: dL/dh at K = 4608 over 12, r6_s78;
  // the wide h GEMM keeps 256-multiples -- cfg5's, K = 768 over 2, was 7.25 vs 9.58 us as a 384-deep skinny product)
  if (mode == 0) {
    const int kd = g.partial_splits > 1 && g.K % g.partial_splits == 0 ? g.K / g.partial_splits : 0;
    if (!(kd > 0 && kd <= 1024 && (kd % 256 == 0 || (kd % 128 == 0 && kd >= 256 && g.N <= 1024)))) return false;
  }
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
  x.nb1 = g.N / SK_COLS;
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

// ---- the greedy decoder step's output head (no teacher forcing: decoder.py:117-133 per step) ----
// Waves for a K = E product at <= 4 k-steps of 32 per wave.
inline int head_waves(int E) { return E <= 512 ? 4 : 8; }
inline int head_kw(int E) { return sat_cdiv(sat_cdiv(E, head_waves(E)), 32) * 32; }

// advanced deep output's middle (decoder.py:149-156) for 32 rows x 32 columns: the f_h tile over all of K = E, then
// fh = relu(. + b_h), fz = relu(sum of the f_z slabs + b_z), comb = fh + fz + emb (ado_combine_rows_kernel's order)
template <int NW>
__global__ __launch_bounds__(NW * 64) void head_mid_kernel(HeadMidArgs a, int kw) {
  __shared__ __attribute__((aligned(16))) float red[2 * 16 * SK_RLD];
  const int bx = blockIdx.x, row0 = blockIdx.y * 32;
  // the epilogue's operands of this thread's piece (32 rows x 8 pieces = 256: one per thread of the first four waves),
  // requested before the tile's fragment loads so their latency hides under the MFMAs
  const int q = threadIdx.x, rl = q >> 3, c4 = (q & 7) * 4, row = row0 + rl, n = bx * SK_COLS + c4;
  const bool mine = q < 32 * 8 && row < a.B;
  float4 bh = make_float4(0.f, 0.f, 0.f, 0.f), bz = bh, zp = bh;
  uint2 eu = make_uint2(0u, 0u);
  if (mine) {
    bh = *(const float4*)(a.fh_b + n);
    bz = *(const float4*)(a.fz_b + n);
    zp = sum_parts4(a.fzp, (long)row * a.fzp_ld + n, a.fz_splits, a.fz_split_stride);
    eu = *(const uint2*)(a.emb + (long)row * a.emb_ld + n);
  }
  skinny_tile<2, NW>(a.hd, a.hd_ld, a.B, row0, a.fh_w, a.E, a.E, bx * SK_COLS, 0, a.E, kw, red);
  if (mine) {
    const float4 acc = *(const float4*)(red + rl * SK_RLD + c4);
    const bf16* ev = (const bf16*)&eu;
    const float h4[4] = {acc.x + bh.x, acc.y + bh.y, acc.z + bh.z, acc.w + bh.w};
    const float z4[4] = {zp.x + bz.x, zp.y + bz.y, zp.z + bz.z, zp.w + bz.w};
    float fh[4], fz[4];
    uint2 cu;
    bf16* cv = (bf16*)&cu;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      fh[k] = h4[k] > 0.f ? h4[k] : 0.f;
      fz[k] = z4[k] > 0.f ? z4[k] : 0.f;
      cv[k] = (bf16)(fh[k] + fz[k] + (float)ev[k]);
    }
    *(float4*)(a.fh + (long)row * a.f_ld + n) = make_float4(fh[0], fh[1], fh[2], fh[3]);
    *(float4*)(a.fz + (long)row * a.f_ld + n) = make_float4(fz[0], fz[1], fz[2], fz[3]);
    *(uint2*)(a.comb + (long)row * a.comb_ld + n) = cu;
  }
}

// vocabulary head of the step for all rows x 32 columns (K = E unsplit): act(x W^T + b) rounded to bf16 into preds,
// and every row's argmax over the block's rounded logits into the partials
template <int MB, int NW>
__global__ __launch_bounds__(NW * 64) void head_out_kernel(HeadOutArgs a, int kw, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  __shared__ __attribute__((aligned(16))) float red[MB * 16 * SK_RLD];
  const int bx = blockIdx.x;
  // this thread's four bias columns (the same in every pass of the epilogue: NW * 64 is a multiple of 8), requested
  // before the tile's fragment loads
  float bias4[4];
  {
    const int n = bx * SK_COLS + (threadIdx.x & 7) * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) bias4[k] = n + k < a.V ? a.bias[n + k] : 0.f;
  }
  skinny_tile<MB, NW>(a.x, a.x_ld, a.B, 0, a.w, a.E, a.V, bx * SK_COLS, 0, a.E, kw, red);
  constexpr int PIECES = MB * 16 * (SK_COLS / 4);   // a multiple of 64: whole waves take part in the shuffles
  const bool vec = (a.V & 3) == 0 && (((uintptr_t)a.preds | (uintptr_t)(a.preds_ld * 2)) & 7) == 0;
  for (int q = threadIdx.x; q < PIECES; q += NW * 64) {
    const int row = q >> 3, c4 = (q & 7) * 4, n = bx * SK_COLS + c4;
    const float4 v4 = *(const float4*)(red + row * SK_RLD + c4);
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    float best = -INFINITY;
    int bi = 0x7fffffff;
    uint2 pu;
    bf16* pv = (bf16*)&pu;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = n + k;
      float x = v[k] + bias4[k];
      if (a.relu) x = x > 0.f ? x : 0.f;
      pv[k] = (bf16)x;
      if (row < a.B && col < a.V) {
        const float xr = (float)pv[k];
        if (sat_argmax_better(xr, col, best, bi)) { best = xr; bi = col; }
      }
    }
    if (row < a.B) {
      bf16* dst = a.preds + (long)row * a.preds_ld + n;
      if (vec && n + 3 < a.V) {
        *(uint2*)dst = pu;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (n + k < a.V) dst[k] = pv[k];
      }
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {   // the 8 lanes of a row (consecutive q)
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (sat_argmax_better(ov, oi, best, bi)) { best = ov; bi = oi; }
    }
    if ((q & 7) == 0 && row < a.B) {
      a.pval[(long)bx * a.B + row] = best;
      a.pidx[(long)bx * a.B + row] = bi;
    }
  }
  sat_stamp_end(st, t0);
}

// The vocabulary head at E = 512 with the step's input rows staged once in LDS: 64 columns per workgroup (157 at
// V = 10000: one round on 256 CUs, where the skinny form above needs 313 workgroups), each of the four waves owning 16
// columns over all of K -- its 16 weight fragments register-direct, the A fragments read from LDS -- so no wave-order
// K fold.  The rows (MB x 16 x 512 bf16, 128 KiB at B = 128) land by LDS-DMA in four K quarters, quarter-major
// ([q][row][256 B], 16-B chunk c of a row at chunk c ^ (row & 15): one 1 KiB instruction = 4 rows of a quarter, the
// fragment reads of 16 rows x 4 k-chunks conflict-free), each quarter waited for right before its k-steps, so the
// MFMAs of the first quarters run while the later ones land.  Argmax partials per 64 columns (the waves' per-row
// winners meet in LDS).
constexpr int HO_K = 512, HO_COLS = 64, HO_BLK = 64, HO_Q = 4, HO_QB = HO_K * 2 / HO_Q;   // 256-B quarter rows
typedef __attribute__((address_space(3))) void sk_lds_void;
// every wave's LDS-DMAs older than its N youngest vector-memory operations have landed, then a barrier
template <int N>
__device__ __forceinline__ void ho_vm_barrier() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)\n\ts_barrier" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}
template <typename F, int... Ts>
__device__ __forceinline__ void sk_static_for_impl(F&& f, std::integer_sequence<int, Ts...>) {
  (f(std::integral_constant<int, Ts>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sk_static_for(F&& f) {
  sk_static_for_impl(f, std::make_integer_sequence<int, N>{});
}
template <int MB>
__global__ __launch_bounds__(256) void head_out_lds_kernel(HeadOutArgs a, SatStamps st) {
  static_assert(MB % 2 == 0, "DMA instructions cover 4 rows: MB * 16 / 4 per quarter, a multiple of the 4 waves");
  constexpr int MR = MB * 16, INSTR = MR / 4 / 4;   // DMA instructions per wave per quarter
  const SatStampT0 t0 = sat_stamp_begin(st);
  // one LDS array per K quarter: distinct objects get distinct alias scopes, so the compiler's wait before a read of
  // quarter q covers only quarter q's DMAs (with one array it waits for every pending LDS-DMA)
  __shared__ __attribute__((aligned(16))) char sA0[MR * HO_QB];
  __shared__ __attribute__((aligned(16))) char sA1[MR * HO_QB];
  __shared__ __attribute__((aligned(16))) char sA2[MR * HO_QB];
  __shared__ __attribute__((aligned(16))) char sA3[MR * HO_QB];
  auto quarter = [&](int q) -> char* { return q == 0 ? sA0 : q == 1 ? sA1 : q == 2 ? sA2 : sA3; };
  __shared__ float s_bv[4][MR];
  __shared__ int s_bi[4][MR];
  const int lane = threadIdx.x & 63, fr = lane & 15, fh = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * HO_COLS + w * 16;   // this wave's 16 columns
  // the wave's weight fragments (all 16 k-steps of 32) and bias, requested first
  const bf16* wr = a.w + (long)min(n0 + fr, a.V - 1) * HO_K + 8 * fh;
  bf16x8 bw[HO_K / 32];
#pragma unroll
  for (int ks = 0; ks < HO_K / 32; ++ks) bw[ks] = *(const bf16x8*)(wr + ks * 32);
  // (branch-free: a predicated load splits the block, and the compiler's wait-count pass then waits for every load
  // before the first MFMA instead of the quarter the asm waits name)
  float bias4[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias4[r] = a.bias[min(n0 + 4 * fh + r, a.V - 1)];
  // the rows by LDS-DMA, quarter by quarter: instruction j of wave w covers rows 4 (w + 4 j) .. + 3; lane l fills slot
  // l % 16 of row 4 (w + 4 j) + l / 16 with chunk (l % 16) ^ (row & 15) of the quarter
  // (buffer_load ... lds through a resource over the rows, as convblock.hip stages its planes: the wait for quarter q
  // is the asm's counted vmcnt, with no compiler-inserted vmcnt(0) in front of the first LDS read)
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)(2L * ((long)(a.B - 1) * a.x_ld + HO_K)), 0x00020000);
#pragma unroll
  for (int q = 0; q < HO_Q; ++q)
#pragma unroll
    for (int j = 0; j < INSTR; ++j) {
      const int r0 = 4 * (w + 4 * j), row = r0 + (lane >> 4);
      const int off = (int)(2L * ((long)min(row, a.B - 1) * a.x_ld + q * (HO_K / HO_Q) + 8 * ((lane & 15) ^ (row & 15))));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (sk_lds_void*)(quarter(q) + r0 * HO_QB), 16, off, 0, 0, 0);
    }
  f32x4 acc[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][MB];
  auto frag = [&](int ks, bf16x8 (&dst)[MB]) {
    const int q = ks / 4, c = 4 * (ks % 4) + fh;
#pragma unroll
    for (int i = 0; i < MB; ++i) dst[i] = *(const bf16x8*)(quarter(q) + (i * 16 + fr) * HO_QB + 16 * (c ^ fr));
  };
  // quarter q is waited for (the DMAs of the later quarters, INSTR each, may stay in flight) right before its k-steps;
  // within a quarter the next k-step's A fragments are read before this one's MFMAs
  sk_static_for<HO_K / 32>([&](auto KS) {
    constexpr int ks = decltype(KS)::value;
    if constexpr (ks == 0) {
      ho_vm_barrier<(HO_Q - 1) * INSTR>();
      frag(0, af[0]);
    }
    if constexpr (ks + 1 < HO_K / 32 && (ks + 1) % 4 != 0) frag(ks + 1, af[(ks + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);   // the next k-step's reads stay ahead of this k-step's MFMAs
#pragma unroll
    for (int i = 0; i < MB; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ks], af[ks & 1][i], acc[i], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ks + 1 < HO_K / 32 && (ks + 1) % 4 == 0) {
      ho_vm_barrier<(HO_Q - 1 - (ks + 1) / 4) * INSTR>();
      frag(ks + 1, af[(ks + 1) & 1]);
    }
  });
  // lane holds columns n0 + 4 fh .. + 3 of row i * 16 + fr
  const bool vec = (a.V & 3) == 0 && (((uintptr_t)a.preds | (uintptr_t)(a.preds_ld * 2)) & 7) == 0;
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int row = i * 16 + fr, n = n0 + 4 * fh;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    uint2 pu;
    bf16* pv = (bf16*)&pu;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = acc[i][r] + bias4[r];
      if (a.relu) x = x > 0.f ? x : 0.f;
      pv[r] = (bf16)x;
      if (row < a.B && n + r < a.V) {
        const float xr = (float)pv[r];
        if (sat_argmax_better(xr, n + r, best, bi)) { best = xr; bi = n + r; }
      }
    }
    if (row < a.B) {
      bf16* dst = a.preds + (long)row * a.preds_ld + n;
      if (vec && n + 3 < a.V) {
        *(uint2*)dst = pu;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < a.V) dst[r] = pv[r];
      }
    }
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {   // the 4 lanes (fh) of a row
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (sat_argmax_better(ov, oi, best, bi)) { best = ov; bi = oi; }
    }
    if (fh == 0) { s_bv[w][row] = best; s_bi[w][row] = bi; }
  }
  __syncthreads();
  if ((int)threadIdx.x < min(MR, a.B)) {   // the four waves' winners of a row, in wave order
    const int row = threadIdx.x;
    float best = s_bv[0][row];
    int bi = s_bi[0][row];
#pragma unroll
    for (int v = 1; v < 4; ++v)
      if (sat_argmax_better(s_bv[v][row], s_bi[v][row], best, bi)) { best = s_bv[v][row]; bi = s_bi[v][row]; }
    a.pval[(long)blockIdx.x * a.B + row] = best;
    a.pidx[(long)blockIdx.x * a.B + row] = bi;
  }
  sat_stamp_end(st, t0);
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

// Two products with the same M, K and partial-split geometry, no bias on the second, in one launch (the greedy step's
// context GEMM and the ado head's f_z pre-activation, decoder.py:109-115,151-155: both read the attention output of
// the step).  Returns 1 when it launched, 0 when either is not a skinny problem of that shape (the caller then
// launches them one by one).
int sat_skinny_dual_try(const SatGemm& g1, const SatGemm& g2, hipStream_t st, int* err) {
  *err = 0;
  SkArgs a, b;
  int nw1, nw2;
  const int mode = sat_policy().skinny;
  if (!skinny_shape(g1, mode, &a, &nw1) || !skinny_ptrs(g1) || !skinny_shape(g2, mode, &b, &nw2) || !skinny_ptrs(g2))
    return 0;
  if (g1.M != g2.M || g1.K != g2.K || a.kc != b.kc || a.kw != b.kw || nw1 != nw2 || g2.bias) return 0;
  const int S1 = g1.partial_splits > 1 ? g1.partial_splits : 1, S2 = g2.partial_splits > 1 ? g2.partial_splits : 1;
  if (S1 != S2) return 0;
  a.A2 = b.A; a.lda2 = b.lda; a.W2 = b.W; a.ldw2 = b.ldw; a.C2 = b.C; a.ldc2 = b.ldc; a.split_stride2 = b.split_stride;
  a.st = sat_launch_stamps();
  const dim3 grid(g1.N / SK_COLS + g2.N / SK_COLS, S1);
  if (g1.M <= 32) launch_mb<2>(nw1, grid, st, a);
  else if (g1.M <= 64) launch_mb<4>(nw1, grid, st, a);
  else launch_mb<8>(nw1, grid, st, a);
  *err = (int)hipGetLastError();
  return 1;
}

// splits the decoder asks for when the skinny kernel runs its per-step GEMMs: 256-deep K per split
// (less A per workgroup: every workgroup reads all M rows of its K range), 0 = not eligible
int sat_skinny_splits(int M, int N, int K) {
  if (sat_policy().skinny == 1 || M > 128 || N % SK_COLS || K % 256 || K < 1024) return 0;
  return K / 256;
}


int sat_greedy_supported(int B, int E) { return B >= 1 && B <= 128 && E % 64 == 0 && E >= 64 && E <= 1024; }

int sat_greedy_head_mid(const HeadMidArgs& a, hipStream_t s) {
  if (!sat_greedy_supported(a.B, a.E)) return (int)hipErrorInvalidValue;
  const dim3 grid(a.E / SK_COLS, sat_cdiv(a.B, 32));
  if (head_waves(a.E) == 4) hipLaunchKernelGGL(head_mid_kernel<4>, grid, dim3(256), 0, s, a, head_kw(a.E));
  else hipLaunchKernelGGL(head_mid_kernel<8>, grid, dim3(512), 0, s, a, head_kw(a.E));
  return (int)hipGetLastError();
}

// the vocabulary head's form for (B, V, E): the LDS-staged one at E = 512 (partials per 16 columns), else the skinny
// tile (per 32)
static bool head_out_lds(int B, int E) { return E == HO_K && B <= 128; }
int sat_greedy_head_blocks(int B, int V, int E) { return sat_cdiv(V, head_out_lds(B, E) ? HO_BLK : SK_COLS); }

int sat_greedy_head_out(const HeadOutArgs& a, hipStream_t s) {
  if (!sat_greedy_supported(a.B, a.E) || a.V < 1) return (int)hipErrorInvalidValue;
  const SatStamps st = sat_launch_stamps();
  if (head_out_lds(a.B, a.E)) {
    if (((uintptr_t)a.x & 15) || (a.x_ld & 7) || ((uintptr_t)a.w & 15)) return (int)hipErrorInvalidValue;
    const dim3 grid(sat_cdiv(a.V, HO_COLS));
    if (a.B <= 32) hipLaunchKernelGGL(head_out_lds_kernel<2>, grid, dim3(256), 0, s, a, st);
    else if (a.B <= 64) hipLaunchKernelGGL(head_out_lds_kernel<4>, grid, dim3(256), 0, s, a, st);
    else hipLaunchKernelGGL(head_out_lds_kernel<8>, grid, dim3(256), 0, s, a, st);
    return (int)hipGetLastError();
  }
  const dim3 grid(sat_cdiv(a.V, SK_COLS));
  const int nw = head_waves(a.E), kw = head_kw(a.E);
#define SAT_HEAD_OUT(MB)                                                                                            \
  do {                                                                                                            \
    if (nw == 4) hipLaunchKernelGGL((head_out_kernel<MB, 4>), grid, dim3(256), 0, s, a, kw, st);                   \
    else hipLaunchKernelGGL((head_out_kernel<MB, 8>), grid, dim3(512), 0, s, a, kw, st);                           \
  } while (0)
  if (a.B <= 32) SAT_HEAD_OUT(2);
  else if (a.B <= 64) SAT_HEAD_OUT(4);
  else SAT_HEAD_OUT(8);
#undef SAT_HEAD_OUT
  return (int)hipGetLastError();
}
