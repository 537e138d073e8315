// 256-row pipelined bf16 GEMM with fp32 output and k-major operands, for gfx950 (MI355X): the decoder's batched
// weight gradients and head input gradients (decoder.py:117-125,149-158 backward, train.py:150).
//
//   C[M,N] (+)= A(m,k) . B(n,k)  (+ bias[n], act)      bf16 in, fp32 accumulate, fp32 out
//   A(m,k) = AT ? A[k lda + m] : A[m lda + k];   B(n,k) = BT ? B[k ldb + n] : B[n ldb + k]
//
// The weight gradients dW = dY^T X read both operands k-major (the activations and their gradients are stored
// row per (step, batch row), K = B (T-1) rows), the input gradients dX = dY W read W k-major.  The 128x128 tile
// kernel (convgemm.hip) ran these at ~0.4 PF: two workgroups per CU, a two-stage ring drained with vmcnt(0) every
// k-tile.  This kernel takes convpipe.hip's pipeline (cdna_hip_programming.md sec. 5) to k-major operands:
//   * block tile 256 x 128 x 64, 8 waves (4 M x 2 N), 64 x 64 per wave, ONE workgroup per CU;
//   * 3-stage LDS ring (3 x 48 KiB) filled by buffer_load ... lds (16 B per lane; offsets past an operand's end
//     land zeros: K tails and M / N edges cost no branches), one counted vmcnt wait + raw s_barrier per k-tile,
//     tile t+2 in flight while t+1 lands and t is consumed;
//   * k-major tiles as 64 k-rows of 256 B (128 elements; A as two such halves), 16-B chunk c of k-row r at slot
//     c ^ swz(r): the fragments come out of ds_read_b64_tr_b16 pairs conflict-free (the layout fast_gemm_kernel
//     uses); m/n-major tiles as convpipe's 128-B rows;
//   * fragments of a tile's second 32-deep half requested before its first half's MFMAs, the next tile's first
//     half right after the barrier;
//   * split-K over blockIdx.y when the tiles alone leave CUs idle (the split count minimises rounds x k-tiles),
//     fp32 atomics into C; otherwise the tile goes through LDS to 16-B row stores (bias, act fused);
//   * XCD-aware tile order: the N-tiles of one 256-row panel share an L2.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

typedef __attribute__((address_space(3))) void gp_lds_void;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 gp_lds_bf16x4;

constexpr int GBM = 256, GBN = 128, GBK = 64;
constexpr int G_STAGE_A = GBM * GBK * 2, G_STAGE_B = GBN * GBK * 2, G_STAGE = G_STAGE_A + G_STAGE_B;
constexpr int G_NSTG = 3, G_LDS = G_NSTG * G_STAGE;   // 147456 B
constexpr int G_EPI_LD = GBN + 4;
static_assert(GBM * G_EPI_LD * 4 <= G_LDS, "epilogue tile must fit in the ring");
constexpr int G_AI = G_STAGE_A / 1024 / 8, G_BI = G_STAGE_B / 1024 / 8;   // 1 KiB DMAs per wave per stage
constexpr int G_INSTR = G_AI + G_BI;
constexpr unsigned G_OOB = 0x80000000u;

struct GArgs {
  int M, N, K;
  const bf16* A; long lda;
  const bf16* B; long ldb;
  float* C; long ldc;
  const float* bias;      // plain epilogue only
  int act;                // plain epilogue only
  int atomic;             // fp32 atomics into C (split-K, or beta = 1)
  int kchunk;             // K range of split blockIdx.y: [y kchunk, min(K, (y + 1) kchunk)), a multiple of GBK
  int a_mlim;             // k-major A: 8-element chunks are read while m + 8 <= a_mlim (SatGemm::a_tail)
  int tiles_n;
  unsigned a_bytes, b_bytes;
  SatStamps st;
};

// k-major tile of 256-B rows: chunk slot of k-row r
__device__ __forceinline__ int swz256(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// MFMA 16x16x32 operand fragment (8 consecutive k of column x = xt + lane & 15) from a k-major tile: two
// transposing reads of 4 k-rows x 16 columns
__device__ __forceinline__ bf16x8 frag_kmajor(const char* tile, int kbase, int xt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = (xt >> 3) + (p >> 1);
  const int r0 = kbase + 8 * g + q, r1 = r0 + 4;
  const char* a0 = tile + r0 * 256 + 16 * (ch ^ swz256(r0)) + 8 * (p & 1);
  const char* a1 = tile + r1 * 256 + 16 * (ch ^ swz256(r1)) + 8 * (p & 1);
  const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((gp_lds_bf16x4*)(uintptr_t)(const void*)a0);
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((gp_lds_bf16x4*)(uintptr_t)(const void*)a1);
  bf16x8 r;
  r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
  r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
  return r;
}

template <int N>
__device__ __forceinline__ void gp_wait_barrier() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

__device__ __forceinline__ void gpdma(__amdgpu_buffer_rsrc_t r, char* dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (gp_lds_void*)dst, 16, (int)voff, 0, 0, 0);
}

template <bool AT, bool BT>
__device__ __forceinline__ void gemm_pipe_body(const GArgs& a) {
  static_assert(G_INSTR == 6, "the counted wait below assumes 6 DMAs per wave per stage");
  constexpr int MI = 4, NJ = 4;
  __shared__ __attribute__((aligned(16))) char smem[G_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  int tile = blockIdx.x;
  {   // XCD-aware order (cdna_hip_programming.md T1, bijective form)
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = tile % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
  }
  const int m0 = (tile / a.tiles_n) * GBM, n0 = (tile % a.tiles_n) * GBN;
  const int M = a.M, N = a.N;
  const int kbeg = blockIdx.y * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.b_bytes, 0x00020000);
  // per-lane DMA pieces: k-major (4 k-rows of 256 B per 1 KiB instruction: lane -> k-row lane >> 4, slot lane & 15)
  // or row-major (8 rows of 128 B: lane -> row lane >> 3, slot lane & 7); fixed part of the element offset + the
  // k-row / k-chunk the lane adds per tile
  int a_off[G_AI], a_k[G_AI];
  bool a_ok[G_AI];
#pragma unroll
  for (int j = 0; j < G_AI; ++j) {
    if constexpr (AT) {
      const int q = (w * G_AI + j) * 4 + (lane >> 4);       // 0..127: half q >> 6, k-row q & 63
      const int kr = q & 63, ch = (lane & 15) ^ swz256(kr);
      const int m = m0 + (q >> 6) * 128 + 8 * ch;
      a_ok[j] = m + 8 <= a.a_mlim;
      a_off[j] = m;
      a_k[j] = kr;
    } else {
      const int r = (w * G_AI + j) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((r >> 1) & 7);
      a_ok[j] = m0 + r < M;
      a_off[j] = (int)((long)(m0 + r) * a.lda);
      a_k[j] = 8 * ch;
    }
  }
  int b_off[G_BI], b_k[G_BI];
  bool b_ok[G_BI];
#pragma unroll
  for (int j = 0; j < G_BI; ++j) {
    if constexpr (BT) {
      const int kr = (w * G_BI + j) * 4 + (lane >> 4), ch = (lane & 15) ^ swz256(kr);
      const int n = n0 + 8 * ch;
      b_ok[j] = n + 8 <= N;
      b_off[j] = n;
      b_k[j] = kr;
    } else {
      const int r = (w * G_BI + j) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((r >> 1) & 7);
      b_ok[j] = n0 + r < N;
      b_off[j] = (int)((long)(n0 + r) * a.ldb);
      b_k[j] = 8 * ch;
    }
  }
  auto stage = [&](int buf, int k0) {
    char* sa = smem + buf * G_STAGE;
    char* sb = sa + G_STAGE_A;
#pragma unroll
    for (int j = 0; j < G_AI; ++j) {
      const int k = k0 + a_k[j];
      const bool ok = a_ok[j] && k < kend;
      const unsigned off = AT ? 2u * (unsigned)((long)k * a.lda + a_off[j]) : 2u * (unsigned)(a_off[j] + k);
      gpdma(rA, sa + (w * G_AI + j) * 1024, ok ? off : G_OOB);
    }
#pragma unroll
    for (int j = 0; j < G_BI; ++j) {
      const int k = k0 + b_k[j];
      const bool ok = b_ok[j] && k < kend;
      const unsigned off = BT ? 2u * (unsigned)((long)k * a.ldb + b_off[j]) : 2u * (unsigned)(b_off[j] + k);
      gpdma(rB, sb + (w * G_BI + j) * 1024, ok ? off : G_OOB);
    }
  };

  // fragments of 32-deep half h of the tile in buf
  const int fr = lane & 15, fh = lane >> 4, sw = (fr >> 1) & 7;
  auto frags = [&](int buf, int h, bf16x8 (&fa)[MI], bf16x8 (&fb)[NJ]) {
    const char* sa = smem + buf * G_STAGE;
    const char* sb = sa + G_STAGE_A;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if constexpr (AT) fa[i] = frag_kmajor(sa + (wm >> 1) * (64 * 256), h * 32, (wm & 1) * 64 + i * 16, lane);
      else fa[i] = *(const bf16x8*)(sa + (wm * 64 + i * 16 + fr) * 128 + 16 * ((h * 4 + fh) ^ sw));
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (BT) fb[j] = frag_kmajor(sb, h * 32, wn * 64 + j * 16, lane);
      else fb[j] = *(const bf16x8*)(sb + (wn * 64 + j * 16 + fr) * 128 + 16 * ((h * 4 + fh) ^ sw));
    }
  };
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](const bf16x8 (&fa)[MI], const bf16x8 (&fb)[NJ]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };

  bf16x8 xa[MI], xb[NJ], ya[MI], yb[NJ];
  if (nk > 0) {
    stage(0, kbeg);
    if (nk > 1) {
      stage(1, kbeg + GBK);
      gp_wait_barrier<G_INSTR>();
    } else {
      gp_wait_barrier<0>();
    }
    frags(0, 0, xa, xb);
    int cur = 0;
    for (int t = 0; t < nk; ++t) {
      frags(cur, 1, ya, yb);   // second half of tile t (retired before this tile's barrier)
      __builtin_amdgcn_sched_barrier(0);
      // tile t+2 into the stage tile t-1 used: every wave's reads of it retired before tile t-1's barrier
      const bool dma = t + 2 < nk;
      if (dma) stage(cur == 0 ? 2 : cur - 1, kbeg + (t + 2) * GBK);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mfma(xa, xb);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < nk) {
        // this wave's DMAs of tile t+1 have landed (t+2's stay in flight); after the barrier every wave's have
        if (dma) gp_wait_barrier<G_INSTR>();
        else gp_wait_barrier<0>();
        cur = cur == 2 ? 0 : cur + 1;
        frags(cur, 0, xa, xb);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mfma(ya, yb);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (a.atomic) {   // split-K / accumulate: fp32 atomics straight from the accumulators (bias / act host-excluded)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn * 64 + j * 16 + fr;
        if (col >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + i * 16 + fh * 4 + r;
          if (row < M) atomicAdd(a.C + (long)row * a.ldc + col, acc[i][j][r]);
        }
      }
    return;
  }
  gp_wait_barrier<0>();   // ring free for the epilogue
  float* ep = (float*)smem;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int cl = wn * 64 + j * 16 + fr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(wm * 64 + i * 16 + fh * 4 + r) * G_EPI_LD + cl] = acc[i][j][r];
  }
  __syncthreads();
  // 16 chunks of 8 columns x 32 rows per pass
  const int cc = tid & 15, r0 = tid >> 4;
  const int col = n0 + cc * 8;
  if (col >= N) return;   // N % 8 == 0 (host-checked): a chunk is all in or all out
  float b8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) b8[e] = a.bias ? a.bias[col + e] : 0.f;
#pragma unroll
  for (int it = 0; it < GBM / 32; ++it) {
    const int rl = r0 + it * 32, row = m0 + rl;
    if (row >= M) break;
    const float4 x0 = *(const float4*)(ep + rl * G_EPI_LD + cc * 8);
    const float4 x1 = *(const float4*)(ep + rl * G_EPI_LD + cc * 8 + 4);
    float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e] + b8[e], a.act);
    float* p = a.C + (long)row * a.ldc + col;
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <bool AT, bool BT>
__global__ __launch_bounds__(512) void gemm_pipe_kernel(GArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  gemm_pipe_body<AT, BT>(a);
  sat_stamp_end(a.st, t0);
}

inline bool gal16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// split count for `tiles` output tiles of nk k-tiles on 256 CUs (one workgroup each), at least 4 k-tiles per split:
// SatPolicy::gemm_split_wgs > 0 aims at that many workgroups; else the s in [1, 16] minimising rounds x (k-tiles per
// split + epilogue), the atomic epilogue priced at 3 k-tiles and the plain one at 1 (ties: fewer splits)
int pick_splits(long tiles, int nk) {
  const int smax = nk / 4 < 16 ? (nk / 4 > 1 ? nk / 4 : 1) : 16;
  const int wgs = sat_policy().gemm_split_wgs;
  if (wgs > 0) {
    const int s = sat_cdiv(wgs, tiles);
    return s < 1 ? 1 : (s > smax ? smax : s);
  }
  int best = 1;
  long best_cost = sat_cdiv(tiles, 256) * (long)(nk + 1);
  for (int s = 2; s <= smax; ++s) {
    const long cost = sat_cdiv(tiles * s, 256) * (long)(sat_cdiv(nk, s) + 3);
    if (cost < best_cost) { best = s; best_cost = cost; }
  }
  return best;
}

}  // namespace

int sat_gemm_pipe_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  // 0 auto = off: measured slower than the tile kernel on the decoder's shapes, 2 every eligible
  const int mode = sat_policy().gemm_pipe;
  if (mode != 2) return 0;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_F32 || g.batch != 1 || g.aux || g.add1 || g.conv.C > 0) return 0;
  if (g.alpha != 1.f || (g.beta != 0.f && g.beta != 1.f) || g.partial_splits > 1) return 0;
  const bool at = g.transA != 0, bt = g.transB != 0;
  // 16-B pieces: the contiguous dimension of each operand in whole 8-element chunks
  if (g.K % 8 || g.lda % 8 || g.ldb % 8 || g.ldc % 4 || (at && g.M % 8 && !g.a_tail) || g.N % 8) return 0;
  if (!gal16(g.A) || !gal16(g.B) || !gal16(g.C) || (g.bias && !gal16(g.bias))) return 0;
  const double flops = 2.0 * g.M * g.N * g.K;
  if (mode == 0 && (!(at || bt) || flops < 4e9)) return 0;   // NN problems: convpipe / fast_gemm
  const long a_bytes = at ? 2L * ((long)(g.K - 1) * g.lda + (g.a_tail ? sat_cdiv(g.M, 8) * 8 : g.M))
                          : 2L * ((long)(g.M - 1) * g.lda + g.K);
  const long b_bytes = bt ? 2L * ((long)(g.K - 1) * g.ldb + g.N) : 2L * ((long)(g.N - 1) * g.ldb + g.K);
  if (a_bytes >= (1L << 31) || b_bytes >= (1L << 31)) return 0;
  const long tiles = (long)sat_cdiv(g.M, GBM) * sat_cdiv(g.N, GBN);
  const int nk = sat_cdiv(g.K, GBK);
  const bool plain_ok = g.beta == 0.f;
  int splits = (g.bias || g.act != SAT_ACT_NONE) ? 1 : pick_splits(tiles, nk);
  if ((g.bias || g.act != SAT_ACT_NONE) && !plain_ok) return 0;
  GArgs a{};
  a.M = g.M; a.N = g.N; a.K = g.K;
  a.A = (const bf16*)g.A; a.lda = g.lda; a.B = (const bf16*)g.B; a.ldb = g.ldb;
  a.C = (float*)g.C; a.ldc = g.ldc;
  a.bias = g.bias; a.act = g.act;
  a.a_mlim = at && g.a_tail ? sat_cdiv(g.M, 8) * 8 : g.M;
  a.kchunk = sat_cdiv(nk, splits) * GBK;
  splits = sat_cdiv(g.K, a.kchunk);
  a.atomic = splits > 1 || !plain_ok;
  if (a.atomic && g.beta == 0.f && !g.c_zeroed) SAT_CHECK((hipError_t)sat_zero_rows((float*)g.C, g.ldc, g.M, g.N, s));
  a.tiles_n = sat_cdiv(g.N, GBN);
  a.a_bytes = (unsigned)a_bytes; a.b_bytes = (unsigned)b_bytes;
  a.st = sat_launch_stamps();
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  if (at && bt) hipLaunchKernelGGL((gemm_pipe_kernel<true, true>), grid, dim3(512), 0, s, a);
  else if (at) hipLaunchKernelGGL((gemm_pipe_kernel<true, false>), grid, dim3(512), 0, s, a);
  else if (bt) hipLaunchKernelGGL((gemm_pipe_kernel<false, true>), grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((gemm_pipe_kernel<false, false>), grid, dim3(512), 0, s, a);
  *err = (int)hipGetLastError();
  return 1;
}

// whether sat_gemm_pipe_try would run g as fp32 atomics that need C zeroed first (decoder.hip's prezero)
int sat_gemm_pipe_atomic(const SatGemm& g) {
  const int mode = sat_policy().gemm_pipe;
  if (mode != 2 || g.dtype != SAT_BF16 || g.c_dtype != SAT_F32 || g.beta != 0.f || g.bias || g.act != SAT_ACT_NONE ||
      g.add1 || g.partial_splits > 1 || g.conv.C > 0)
    return 0;
  if (mode == 0 && (!(g.transA || g.transB) || 2.0 * g.M * g.N * g.K < 4e9)) return 0;
  const long tiles = (long)sat_cdiv(g.M, GBM) * sat_cdiv(g.N, GBN);
  const int nk = sat_cdiv(g.K, GBK);
  const int kchunk = sat_cdiv(nk, pick_splits(tiles, nk)) * GBK;
  return sat_cdiv(g.K, kchunk) > 1;
}
