// The LSTM cell folded into the GEMM that feeds it, with no split-K and so no cross-workgroup hand-off
// (decoder.py:107-115: gates = [emb, gated ctx] . W_ih^T + b_ih + h . W_hh^T + b_hh; c' = f c + i g; h' = o tanh c').
//
//   lstm_gemm_fwd_kernel: the context half of the gate GEMM of step t, gated_ctx[B, D] . W_ih[:, E:]^T, for a block
//     of 16 MB rows x 8 units (all four gates: gate-interleaved W rows q E + u), the full K = D in ONE workgroup
//     (8 waves split K, their partial tiles summed in LDS in a fixed order), then the cell forward of those 8 units
//     x 16 MB rows in the epilogue: gates = (x part + h slabs) + context sum, c, h (fp32 and the bf16 next input).
//   lstm_gemm_bwd_kernel: the recurrent dL/dh GEMM of BPTT step t, [dU h | d f_beta h | d gates] . [U; f_beta;
//     W_hh] through the transposed copy hcat^T (rows = units), for a block of 16 rows x 16 units with the full
//     K = E + D + 4E, then step t-1's cell backward for those cells in the epilogue (d gates fp32 + bf16, dc).
//
// Why: the split-K skinny GEMM (skinny.hip) spreads K over 4 / 9 workgroups per column block, so the cell had to run
// in a kernel of its own (or in the last-arriving split: measured slower, DESIGN.md 4.6 -- the write-through
// publish + ticket + slab reads cost more than the launch boundary).  Here a workgroup owns whole rows of its
// output columns: the cell needs nothing from another workgroup.  The price is more operand traffic per workgroup
// (forward: 32 rows x 32 columns x K 2048 = 256 KB, every row block re-reads its W_ih slice -- from the same XCD's
// L2: the row blocks of one column block are dispatched to one XCD), bought back by one launch and one boundary
// less per time step and no fp32 partial slabs (4 MB written and read per step at B = 128).
// v_mfma_f32_16x16x32_bf16 computes C^T = W . A^T (W rows as the A operand), so a lane holds 4 consecutive output
// columns of one row; every fragment of a wave (16 B per lane per k-step) is requested at entry.
#include "sat_common.h"
#include "sat_internal.h"

namespace {


struct LstmGemmFwdArgs {
  int B, E, K;                 // K = D
  const bf16* A; long lda;     // gated context of step t [B][K]
  const bf16* W; long ldw;     // W_ih[:, E:] as [4E][ldw] rows, k-contiguous
  LstmFwdArgs l;               // x part, h slabs, c_prev and the outputs (cpart unused)
};

struct LstmGemmBwdArgs {
  int B, E, K;                 // K = E + D + 4E
  const bf16* A; long lda;     // [dU h | d f_beta h | d gates] of step t [B][K]
  const bf16* W; long ldw;     // hcat^T [E][ldw]: unit u's row, k-contiguous
  LstmBwdArgs l;               // step t-1's cell backward (dh_rec unused: the GEMM result)
};

// Per wave (NW waves, wave w): K slice [w KS 32, (w + 1) KS 32) in batches of KB k-steps (every fragment of a batch
// requested before its first MFMA); MB row blocks of 16 starting at row0, NJ column blocks of 16 whose W row for lane
// fr of block j is wrow[j]; the wave's partial tile goes to red[w] ([MB 16][NJ 16 + 4] floats).
template <int NW, int MB, int NJ, int KS, int KB>
__device__ __forceinline__ void full_k_tile(const bf16* A, long lda, int row0, int M, const bf16* const (&wrow)[NJ],
                                            float* red) {
  static_assert(KS % KB == 0, "whole batches");
  constexpr int LD = NJ * 16 + 4;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int kbeg = w * KS * 32 + 8 * fh;
  const bf16* ar[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) ar[i] = A + (long)min(row0 + i * 16 + fr, M - 1) * lda;   // rows past M: never stored
  f32x4 acc[MB][NJ];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < KS; b += KB) {
    bf16x8 af[KB][MB], bw[KB][NJ];
#pragma unroll
    for (int ks = 0; ks < KB; ++ks) {
#pragma unroll
      for (int i = 0; i < MB; ++i) af[ks][i] = *(const bf16x8*)(ar[i] + kbeg + (b + ks) * 32);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bw[ks][j] = *(const bf16x8*)(wrow[j] + kbeg + (b + ks) * 32);
    }
    // the batch's loads all go out before its first MFMA: one memory round trip per batch (left to itself the
    // scheduler interleaves them with the MFMAs to save registers, and the wave waits once per k-step)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KB; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  float* r = red + w * (MB * 16 * LD);
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      *(float4*)(r + (i * 16 + fr) * LD + j * 16 + 4 * fh) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
  __syncthreads();
}

// the NW waves' partials of one output element, in a fixed order
template <int NW, int MB, int NJ>
__device__ __forceinline__ float wave_partials_sum(const float* red, int row, int col) {
  constexpr int LD = NJ * 16 + 4, TS = MB * 16 * LD;
  const float* p = red + row * LD + col;
  if constexpr (NW == 4) return (p[0] + p[TS]) + (p[2 * TS] + p[3 * TS]);
  else return ((p[0] + p[TS]) + (p[2 * TS] + p[3 * TS])) + ((p[4 * TS] + p[5 * TS]) + (p[6 * TS] + p[7 * TS]));
}

template <int NW, int MB, int KS, int KB>
__global__ __launch_bounds__(NW * 64) void lstm_gemm_fwd_kernel(LstmGemmFwdArgs a) {
  static_assert(NW * 64 >= MB * 16 * 8, "one thread per cell");
  const SatStampT0 t0 = sat_stamp_begin(a.l.st);
  __shared__ __attribute__((aligned(16))) float red[NW * MB * 16 * (2 * 16 + 4)];
  const int E = a.E, u0 = blockIdx.x * 8, row0 = blockIdx.y * 16 * MB;
  const int fr = threadIdx.x & 15;
  const LstmFwdArgs& l = a.l;
  // the cell operands of this thread's (row, unit) -- requested first, they stay in flight under the GEMM
  const int r = threadIdx.x >> 3, k = threadIdx.x & 7, b = row0 + r, j = u0 + k;
  const bool cell = threadIdx.x < MB * 16 * 8 && b < a.B;
  float xq[4] = {0.f, 0.f, 0.f, 0.f}, hq[4] = {0.f, 0.f, 0.f, 0.f}, cp = 0.f;
  if (cell) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // sum_parts over <= 2 h slabs: p0 (+ p1)
      const long o = (long)b * l.hpart_ld + q * E + j;
      xq[q] = l.xpart[(long)b * l.xpart_ld + q * E + j];
      hq[q] = l.h_splits > 1 ? l.hpart[o] + l.hpart[o + l.h_split_stride] : l.hpart[o];
    }
    cp = l.c_prev[(long)b * l.c_prev_ld + j];
  }
  // local column c = j 16 + fr: gate q = c >> 3, unit u0 + (c & 7)
  const bf16* wrow[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int c = jj * 16 + fr;
    wrow[jj] = a.W + (long)((c >> 3) * E + u0 + (c & 7)) * a.ldw;
  }
  full_k_tile<NW, MB, 2, KS, KB>(a.A, a.lda, row0, a.B, wrow, red);
  if (cell) {
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) g[q] = (xq[q] + hq[q]) + wave_partials_sum<NW, MB, 2>(red, r, q * 8 + k);   // lstm_fwd_gp's grouping
    float c, h;
    lstm_cell_fwd(g[0], g[1], g[2], g[3], cp, c, h);
#pragma unroll
    for (int q = 0; q < 4; ++q) l.gates[(long)b * l.gates_ld + q * E + j] = g[q];
    l.c_out[(long)b * l.c_out_ld + j] = c;
    if (l.c_next_in) l.c_next_in[(long)b * l.c_next_in_ld + j] = c;
    l.h_out[(long)b * l.h_out_ld + j] = h;
    if (l.h_out_t) ((bf16*)l.h_out_t)[(long)b * l.h_out_t_ld + j] = (bf16)h;
    if (l.h_next_in_t) ((bf16*)l.h_next_in_t)[(long)b * l.h_next_in_t_ld + j] = (bf16)h;
  }
  sat_stamp_end(a.l.st, t0);
}

template <int NW, int KS, int KB>
__global__ __launch_bounds__(NW * 64) void lstm_gemm_bwd_kernel(LstmGemmBwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.l.st);
  __shared__ __attribute__((aligned(16))) float red[NW * 16 * (16 + 4)];
  const int E = a.E, u0 = blockIdx.x * 16, row0 = blockIdx.y * 16;
  const int fr = threadIdx.x & 15;
  const LstmBwdArgs& l = a.l;
  // the cell operands of this thread's (row, unit), requested before the GEMM's fragments
  const int r = threadIdx.x >> 4, k = threadIdx.x & 15, b = row0 + r, j = u0 + k;
  const bool cell = threadIdx.x < 256 && b < a.B;   // 16 x 16 cells
  const long i = (long)b * E + j;
  float gq[4] = {0.f, 0.f, 0.f, 0.f}, cp = 0.f, cn = 0.f, dcin = 0.f, hh = 0.f;
  if (cell) {
#pragma unroll
    for (int q = 0; q < 4; ++q) gq[q] = l.gates[(long)b * l.gates_ld + q * E + j];
    cp = l.c_prev[(long)b * l.c_prev_ld + j];
    cn = l.c_new[(long)b * l.c_new_ld + j];
    if (!l.dc_zero) dcin = l.dc[i];
    if (l.dh_head) {
      hh = l.dh_head[(long)b * l.dh_head_ld + j];
      if (l.mask) hh = l.mask[(long)b * l.mask_ld + j] ? hh * 2.f : 0.f;
    }
  }
  const bf16* wrow[1] = {a.W + (long)(u0 + fr) * a.ldw};
  full_k_tile<NW, 1, 1, KS, KB>(a.A, a.lda, row0, a.B, wrow, red);
  if (cell) {
    const float dh = wave_partials_sum<NW, 1, 1>(red, r, k) + hh;
    float d4[4], dco;
    lstm_cell_bwd(gq[0], gq[1], gq[2], gq[3], cp, cn, dcin, dh, d4, dco);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      l.d_gates[(long)b * l.d_gates_ld + q * E + j] = d4[q];
      if (l.d_gates_t) ((bf16*)l.d_gates_t)[(long)b * l.d_gates_t_ld + q * E + j] = (bf16)d4[q];
    }
    l.dc[i] = dco;
  }
  sat_stamp_end(a.l.st, t0);
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Forms (SatPolicy::fused_lstm, opt-in: beside the encoder both lose to the separate launches): 2 eight
// waves, every fragment of a wave requested at once (alone the fastest); 3 four waves in two batches per wave
// (half the wave slots).  Compile-time k-steps per wave: K / (NW x 32).
template <int NW>
inline int ks_of(int K) { return K % (NW * 32) ? 0 : K / (NW * 32); }

template <int MB>
bool launch_fwd(int form, int K, dim3 grid, hipStream_t s, const LstmGemmFwdArgs& a) {
  if (form == 3) {
    switch (ks_of<4>(K)) {
      case 4: hipLaunchKernelGGL((lstm_gemm_fwd_kernel<4, MB, 4, 2>), grid, dim3(256), 0, s, a); return true;
      case 16: hipLaunchKernelGGL((lstm_gemm_fwd_kernel<4, MB, 16, 8>), grid, dim3(256), 0, s, a); return true;
      default: return false;
    }
  }
  switch (ks_of<8>(K)) {
    case 2: hipLaunchKernelGGL((lstm_gemm_fwd_kernel<8, MB, 2, 2>), grid, dim3(512), 0, s, a); return true;
    case 8: hipLaunchKernelGGL((lstm_gemm_fwd_kernel<8, MB, 8, 8>), grid, dim3(512), 0, s, a); return true;
    default: return false;
  }
}
bool launch_bwd(int form, int K, dim3 grid, hipStream_t s, const LstmGemmBwdArgs& a) {
  if (form == 3) {
    switch (ks_of<4>(K)) {
      case 24: hipLaunchKernelGGL((lstm_gemm_bwd_kernel<4, 24, 12>), grid, dim3(256), 0, s, a); return true;
      case 34: hipLaunchKernelGGL((lstm_gemm_bwd_kernel<4, 34, 17>), grid, dim3(256), 0, s, a); return true;
      case 36: hipLaunchKernelGGL((lstm_gemm_bwd_kernel<4, 36, 18>), grid, dim3(256), 0, s, a); return true;
      default: return false;
    }
  }
  switch (ks_of<8>(K)) {
    case 12: hipLaunchKernelGGL((lstm_gemm_bwd_kernel<8, 12, 12>), grid, dim3(512), 0, s, a); return true;
    case 17: hipLaunchKernelGGL((lstm_gemm_bwd_kernel<8, 17, 17>), grid, dim3(512), 0, s, a); return true;
    case 18: hipLaunchKernelGGL((lstm_gemm_bwd_kernel<8, 18, 18>), grid, dim3(512), 0, s, a); return true;
    default: return false;
  }
}
inline int form() { return sat_policy().fused_lstm == 3 ? 3 : 2; }
inline bool fwd_ks_ok(int K) {
  const int ks = form() == 3 ? ks_of<4>(K) : ks_of<8>(K);
  return form() == 3 ? (ks == 4 || ks == 16) : (ks == 2 || ks == 8);
}
inline bool bwd_ks_ok(int K) {
  const int ks = form() == 3 ? ks_of<4>(K) : ks_of<8>(K);
  return form() == 3 ? (ks == 24 || ks == 34 || ks == 36) : (ks == 12 || ks == 17 || ks == 18);
}

}  // namespace

int sat_lstm_gemm_fwd_ok(int B, int E, int K) {
  const int f = sat_policy().fused_lstm;   // 2, 3: both directions; 4: backward only; 5: forward only
  return (f == 2 || f == 3 || f == 5) && B >= 1 && B <= 1024 && E % 8 == 0 && fwd_ks_ok(K);
}
int sat_lstm_gemm_bwd_ok(int B, int E, int K) {
  const int f = sat_policy().fused_lstm;
  return (f == 2 || f == 3 || f == 4) && B >= 1 && B <= 1024 && E % 16 == 0 && bwd_ks_ok(K);
}

int sat_lstm_gemm_fwd_try(const void* A, long lda, const void* W, long ldw, int K, const LstmFwdArgs& l, hipStream_t s,
                          int* err) {
  *err = 0;
  if (l.dtype != SAT_BF16 || !sat_lstm_gemm_fwd_ok(l.B, l.E, K) || lda % 8 || ldw % 8 || !al16(A) || !al16(W) ||
      l.h_splits > 2)
    return 0;
  LstmGemmFwdArgs a{};
  a.B = l.B; a.E = l.E; a.K = K;
  a.A = (const bf16*)A; a.lda = lda; a.W = (const bf16*)W; a.ldw = ldw;
  a.l = l;
  a.l.st = sat_launch_stamps();
  // 32-row blocks (256 workgroups at B = 128); 16-row blocks below that keep the workgroup count up (and always for
  // the four-wave form: one thread per cell)
  const int f = form();
  const bool mb2 = l.B > 64 && f != 3;
  const dim3 grid(l.E / 8, sat_cdiv(l.B, mb2 ? 32 : 16));
  const bool ok = mb2 ? launch_fwd<2>(f, K, grid, s, a) : launch_fwd<1>(f, K, grid, s, a);
  if (!ok) return 0;
  *err = (int)hipGetLastError();
  return 1;
}

int sat_lstm_gemm_bwd_try(const void* A, long lda, const void* W, long ldw, int K, const LstmBwdArgs& l, hipStream_t s,
                          int* err) {
  *err = 0;
  if (l.dtype != SAT_BF16 || !sat_lstm_gemm_bwd_ok(l.B, l.E, K) || lda % 8 || ldw % 8 || !al16(A) || !al16(W)) return 0;
  LstmGemmBwdArgs a{};
  a.B = l.B; a.E = l.E; a.K = K;
  a.A = (const bf16*)A; a.lda = lda; a.W = (const bf16*)W; a.ldw = ldw;
  a.l = l;
  a.l.st = sat_launch_stamps();
  const dim3 grid(l.E / 16, sat_cdiv(l.B, 16));
  if (!launch_bwd(form(), K, grid, s, a)) return 0;
  *err = (int)hipGetLastError();
  return 1;
}
