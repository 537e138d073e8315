// 256-row pipelined bf16 implicit-GEMM convolution / NT GEMM for gfx950 (MI355X).
//
//   C[M,N] = act(A[M,K] . B[N,K]^T + bias[N] (+ res[M,N]))     bf16 in, fp32 accumulate, bf16 out
//   A: row-major bf16 [M][lda] (AM = 0) or the implicit im2col of an NHWC bf16 image whose
//      channel count is a multiple of 64 (AM = 1: a 64-deep k-tile lies inside one filter tap);
//   B: conv weights [Cout][KH][KW][Cin] / Linear weights [out][in], row-major bf16.
//
// Why a second conv kernel (convgemm.hip's fast_gemm_kernel stays for short-K / residual shapes):
// the 128x128, two-workgroups-per-CU loop drains every LDS-DMA with vmcnt(0) before each k-tile
// and waits lgkmcnt(0) between small read/MFMA groups, so a CU spends most of a k-tile waiting
// (27 % of its MFMA rate; profiles/r1_s8_conv_ablation.txt).  This kernel is built around the
// cdna_hip_programming.md sec. 5 pipelining rules instead:
//   * block tile 256 x 128 x 64, 8 waves (4 M x 2 N), a 64 x 64 output tile per wave (16
//     accumulators), ONE workgroup per CU;
//   * a 3-stage LDS ring (3 x 48 KiB) filled by global_load_lds_dwordx4: while k-tile t is
//     consumed, tile t+1 is landing and tile t+2 is issued, and the only vmcnt wait in the loop
//     is a counted vmcnt(6) (this wave's 6 DMAs of tile t+2 stay in flight across the barrier);
//   * one raw s_barrier per k-tile, in the middle of the tile: the fragments of the tile's second
//     32-deep half are requested before its first half's 16 MFMAs, and the first-half fragments
//     of tile t+1 are requested right after the barrier, before the second half's MFMAs, so LDS
//     latency hides behind MFMAs and no wave waits on its own fragment reads;
//   * WAR on the ring: stage (t+2)%3 was last read by tile t-1's fragment reads, every one of
//     which retired (lgkmcnt(0)) before tile t-1's barrier;
//   * im2col: per lane a precomputed element offset of its pixel and a bit mask of the filter
//     taps that stay inside the image (bit kh*KW+kw), per k-tile one block-uniform delta; taps
//     in the padding read a 16-byte zero line so every lane always issues its DMA;
//   * LDS image lane-linear (DMA), bank swizzle on the SOURCE: slot s of row r holds k-chunk
//     s ^ ((r >> 1) & 7) -> conflict-free ds_read_b128 fragment reads;
//   * XCD-aware tile order (bijective remap): the N-tiles of one 256-row A panel share an L2;
//   * epilogue: fp32 (acc + bias) staged in LDS, then 16-byte row segments with the residual
//     added in fp32, activation, one rounding to bf16 -- the same arithmetic order as
//     fast_gemm_kernel, so both kernels give bit-identical outputs.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

typedef __attribute__((address_space(3))) void p_lds_void;
typedef __attribute__((address_space(1))) const void p_gbl_void;

constexpr int PBM = 256, PBN = 128, PBK = 64, PROW = PBK * 2;   // 128-byte LDS rows
constexpr int P_STAGE_A = PBM * PROW, P_STAGE_B = PBN * PROW, P_STAGE = P_STAGE_A + P_STAGE_B;
constexpr int P_NSTG = 3;
constexpr int P_EPI_LD = PBN + 4;                                  // fp32 epilogue row pitch
constexpr int P_LDS = P_NSTG * P_STAGE;                            // 147456 B
static_assert(PBM * P_EPI_LD * 4 <= P_LDS, "epilogue tile must fit in the ring");

struct PArgs {
  int M, N, K;
  const bf16* A; long lda;
  const bf16* B; long ldb;
  bf16* C; long ldc;
  const float* bias;
  const bf16* res; long ldr;
  int H, W, Cin, KW, stride, pad, OH, OW;   // AM = 1 geometry
  const bf16* zero16;
  int tiles_n;
  int xcd_remap;
  unsigned a_bytes, b_bytes;   // buffer-resource extents (offsets beyond them read zeros)
  int var;                     // experiment: bit 0 DMA after the first MFMA half, bit 1 split DMA, bit 2 no setprio
  SatStamps st;                      // in-kernel launch timestamps (SatPolicy::stamps)
};

// s_waitcnt vmcnt(N) + raw s_barrier (never __syncthreads: its fence would drain the DMA ring)
template <int N>
__device__ __forceinline__ void p_wait_barrier() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

__device__ __forceinline__ void pdma(const void* src, char* dst) {
  __builtin_amdgcn_global_load_lds((p_gbl_void*)src, (p_lds_void*)dst, 16, 0, 0);
}
// LDS-DMA through a raw buffer resource: out-of-range offsets (0x80000000) land zeros in LDS, so
// padding taps / rows past M or N need one v_cndmask on a 32-bit offset instead of 64-bit
// address arithmetic and a zero line.
__device__ __forceinline__ void pbdma(__amdgpu_buffer_rsrc_t r, char* dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (p_lds_void*)dst, 16, (int)voff, (int)soff, 0, 0);
}
constexpr unsigned P_OOB = 0x80000000u;
__device__ __forceinline__ const void* psel(bool ok, const void* p, const void* z) {
  const uintptr_t x = (uintptr_t)p, y = (uintptr_t)z;
  return (const void*)(ok ? x : y);
}

// NW = 8: waves 4 (M) x 2 (N), 64 x 64 per wave;  NW = 4: waves 2 x 2, 128 x 64 per wave.
// ABL (diagnostics only, tools/pipe_ab.py): bit 0 = no MFMA, bit 1 = no in-loop DMA,
// bit 2 = no in-loop fragment reads.
template <int NW, int AM, int ACT, bool RES, int ABL, bool BUF>
__device__ __forceinline__ void conv_pipe_kernel_body(const PArgs& a) {
  constexpr int WGM = NW == 8 ? 4 : 2;
  constexpr int WTM = PBM / WGM, MI = WTM / 16, NJ = 4;
  constexpr int P_AI = PBM / (8 * NW), P_BI = PBN / (8 * NW);   // 1 KiB DMAs per wave per stage
  constexpr int P_INSTR = P_AI + P_BI;
  __shared__ __attribute__((aligned(16))) char smem[P_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  int tile = blockIdx.x;
  if (a.xcd_remap) {   // cdna_hip_programming.md T1, bijective form
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = tile % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
  }
  const int m0 = (tile / a.tiles_n) * PBM, n0 = (tile % a.tiles_n) * PBN;
  const int M = a.M, N = a.N;

  // ---- per-lane DMA bookkeeping: lane -> (row lane>>3 of an 8-row piece, 16-B slot lane&7) ----
  const int lrow = lane >> 3, slot = lane & 7;
  int a_off[P_AI];
  unsigned a_ok[P_AI];
#pragma unroll
  for (int j = 0; j < P_AI; ++j) {
    const int r = (w * P_AI + j) * 8 + lrow;
    const int chunk = slot ^ ((r >> 1) & 7);
    const int row = m0 + r;
    a_off[j] = 0;
    a_ok[j] = 0u;
    if (row < M) {
      if constexpr (AM == 0) {
        a_off[j] = (int)((long)row * a.lda) + 8 * chunk;
        a_ok[j] = 1u;
      } else {
        const int ohw = a.OH * a.OW;
        const int n = row / ohw, rem = row - n * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
        a_off[j] = ((n * a.H + ih0) * a.W + iw0) * a.Cin + 8 * chunk;
        const int KH = a.K / (a.KW * a.Cin);
        unsigned m = 0u;
        for (int kh = 0; kh < KH; ++kh)
          for (int kw = 0; kw < a.KW; ++kw)
            if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
              m |= 1u << (kh * a.KW + kw);
        a_ok[j] = m;
      }
    }
  }
  int b_off[P_BI];
  bool b_ok[P_BI];
#pragma unroll
  for (int j = 0; j < P_BI; ++j) {
    const int r = (w * P_BI + j) * 8 + lrow;
    const int chunk = slot ^ ((r >> 1) & 7);
    b_ok[j] = n0 + r < N;
    b_off[j] = b_ok[j] ? (int)((long)(n0 + r) * a.ldb) + 8 * chunk : 0;
  }

  // block-uniform k state of the next tile to issue: k0, filter tap, element delta of the tap
  int s_k0 = 0, s_tap = 0, s_ci0 = 0, s_kw = 0, s_delta = 0;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.b_bytes, 0x00020000);
  unsigned b_voff[P_BI];
#pragma unroll
  for (int j = 0; j < P_BI; ++j) b_voff[j] = b_ok[j] ? 2u * (unsigned)b_off[j] : P_OOB;
  // part 0: the A operand, part 1: the B operand, part 2: both
  auto stage_part = [&](int buf, int part) {
    char* sa = smem + buf * P_STAGE;
    char* sb = sa + P_STAGE_A;
    if (part != 1) {
#pragma unroll
      for (int j = 0; j < P_AI; ++j) {
        if constexpr (BUF) {
          const bool ok = (a_ok[j] >> s_tap) & 1u;
          pbdma(rA, sa + (w * P_AI + j) * 1024, ok ? 2u * (unsigned)(a_off[j] + s_delta) : P_OOB, 0u);
        } else {
          const bool ok = (a_ok[j] >> s_tap) & 1u;
          pdma(psel(ok, a.A + (a_off[j] + s_delta), a.zero16), sa + (w * P_AI + j) * 1024);
        }
      }
    }
    if (part != 0) {
#pragma unroll
      for (int j = 0; j < P_BI; ++j) {
        if constexpr (BUF) pbdma(rB, sb + (w * P_BI + j) * 1024, b_voff[j], 2u * (unsigned)s_k0);
        else pdma(psel(b_ok[j], a.B + (b_off[j] + s_k0), a.zero16), sb + (w * P_BI + j) * 1024);
      }
    }
  };
  auto advance = [&]() {
    s_k0 += PBK;
    if constexpr (AM == 0) {
      s_delta = s_k0;
    } else {
      s_ci0 += PBK;
      if (s_ci0 == a.Cin) {   // next filter tap
        s_ci0 = 0;
        ++s_tap;
        if (++s_kw == a.KW) s_kw = 0;
        const int kh = s_tap / a.KW;   // uniform scalar
        s_delta = (kh * a.W + s_kw) * a.Cin;
      } else {
        s_delta += PBK;
      }
    }
  };
  auto stage = [&](int buf) { stage_part(buf, 2); advance(); };

  // ---- fragments: lane l reads row (l & 15) of a 16-row block, k-chunk (ks*4 + l>>4) ----
  const int fr = lane & 15, fh = lane >> 4, sw = (fr >> 1) & 7;
  const int a_rd = (wm * WTM + fr) * PROW, b_rd = P_STAGE_A + (wn * 64 + fr) * PROW;
  const int co0 = 16 * ((0 * 4 + fh) ^ sw), co1 = 16 * ((1 * 4 + fh) ^ sw);

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[MI], xb[NJ], ya[MI], yb[NJ];
  auto frags = [&](int buf, int co, bf16x8 (&fa)[MI], bf16x8 (&fb)[NJ]) {
    const char* base = smem + buf * P_STAGE;
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *(const bf16x8*)(base + a_rd + i * 16 * PROW + co);
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb[j] = *(const bf16x8*)(base + b_rd + j * 16 * PROW + co);
  };
  auto mfma = [&](const bf16x8 (&fa)[MI], const bf16x8 (&fb)[NJ]) {
    if constexpr (ABL & 1) {
#pragma unroll
      for (int i = 0; i < MI; ++i) asm volatile("" :: "v"(fa[i]));
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" :: "v"(fb[j]));
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = a.K / PBK;
  stage(0);
  if (nk > 1) {
    stage(1);
    p_wait_barrier<P_INSTR>();
  } else {
    p_wait_barrier<0>();
  }
  frags(0, co0, xa, xb);
  int cur = 0;
  const bool dma_late = a.var & 1, dma_split = a.var & 2, prio = !(a.var & 4);
  for (int t = 0; t < nk; ++t) {
    if constexpr (!(ABL & 4)) frags(cur, co1, ya, yb);   // second half of tile t (retired before this tile's barrier)
    else if (t == 0) frags(cur, co1, ya, yb);
    __builtin_amdgcn_sched_barrier(0);
    const bool dma = !(ABL & 2) && t + 2 < nk;
    const int nb = cur == 0 ? 2 : cur - 1;   // tile t+2 goes into the stage tile t-1 used
    if (dma && !dma_late) {
      if (dma_split) stage_part(nb, 0);
      else stage(nb);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (prio) __builtin_amdgcn_s_setprio(1);
    mfma(xa, xb);
    if (prio) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (dma) {
      if (dma_late && !dma_split) stage(nb);
      else if (dma_split) { stage_part(nb, dma_late ? 2 : 1); advance(); }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nk) {
      // this wave's DMAs of tile t+1 have landed (t+2's stay in flight); after the barrier every
      // wave's have, and every wave's fragment reads of tile t have retired
      if (dma) p_wait_barrier<P_INSTR>();
      else p_wait_barrier<0>();
      cur = cur == 2 ? 0 : cur + 1;
      if constexpr (!(ABL & 4)) frags(cur, co0, xa, xb);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (prio) __builtin_amdgcn_s_setprio(1);
    mfma(ya, yb);
    if (prio) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  p_wait_barrier<0>();   // ring free for the epilogue

  // ---- epilogue: fp32 (acc + bias) tile in LDS, then 16-B row segments ----
  float* ep = (float*)smem;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int cl = wn * 64 + j * 16 + fr;
    const float bcol = (a.bias && n0 + cl < N) ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(wm * WTM + i * 16 + fh * 4 + r) * P_EPI_LD + cl] = acc[i][j][r] + bcol;
  }
  __syncthreads();
  constexpr int RPP = NW * 64 / 16, PASSES = PBM / RPP;   // 16 chunks of 8 columns x RPP rows per pass
  const int cc = tid & 15, r0 = tid >> 4;
  const int col = n0 + cc * 8;
  const __amdgpu_buffer_rsrc_t rC = sat_out_rsrc(a.C, 2L * M * a.ldc);
  if (col < N) {
    uint4 rv[PASSES];
    if constexpr (RES) {
#pragma unroll
      for (int it = 0; it < PASSES; ++it) {
        const int row = m0 + r0 + it * RPP;
        rv[it] = row < M ? *(const uint4*)(a.res + (long)row * a.ldr + col) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < PASSES; ++it) {
      const int rl = r0 + it * RPP, row = m0 + rl;
      if (row >= M) continue;
      const float4 x0 = *(const float4*)(ep + rl * P_EPI_LD + cc * 8);
      const float4 x1 = *(const float4*)(ep + rl * P_EPI_LD + cc * 8 + 4);
      float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      if constexpr (RES) {
        const bf16* h = (const bf16*)&rv[it];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)h[e];
      }
      uint4 u;
      bf16* o = (bf16*)&u;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)apply_act(v[e], ACT);
      sat_st16(rC, (unsigned)(((long)row * a.ldc + col) * 2), u);
    }
  }
}

template <int NW, int AM, int ACT, bool RES, int ABL, bool BUF>
__global__ __launch_bounds__(NW * 64) void conv_pipe_kernel(PArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  conv_pipe_kernel_body<NW, AM, ACT, RES, ABL, BUF>(a);
  sat_stamp_end(a.st, t0);
}

__device__ __attribute__((aligned(16))) bf16 g_pipe_zero16[64];

// DMA placement (PArgs::var): A before / B after the first MFMA half (measured best of the variants)
constexpr int kPipeVar = 2;

template <int NW, int AM, bool RES>
void launch_act(int act, dim3 grid, hipStream_t s, const PArgs& a) {
  if (act == SAT_ACT_RELU) hipLaunchKernelGGL((conv_pipe_kernel<NW, AM, SAT_ACT_RELU, RES, 0, true>), grid, dim3(NW * 64), 0, s, a);
  else hipLaunchKernelGGL((conv_pipe_kernel<NW, AM, SAT_ACT_NONE, RES, 0, true>), grid, dim3(NW * 64), 0, s, a);
}
template <int NW>
void launch_nw(bool conv, bool res, int act, dim3 grid, hipStream_t s, const PArgs& a) {
  if (conv) {
    if (res) launch_act<NW, 1, true>(act, grid, s, a);
    else launch_act<NW, 1, false>(act, grid, s, a);
  } else {
    if (res) launch_act<NW, 0, true>(act, grid, s, a);
    else launch_act<NW, 0, false>(act, grid, s, a);
  }
}

inline bool pal16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// Returns 1 if the problem was launched by the pipelined kernel (error code in *err), 0 otherwise.
int sat_conv_pipe_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  // 0 auto, 1 off, 2 every eligible problem
  const int mode = sat_policy().conv_pipe;
  if (mode == 1) return 0;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_BF16 || g.batch != 1 || g.aux || g.transA || g.transB) return 0;
  if (g.beta != 0.f || g.alpha != 1.f || g.partial_splits > 1) return 0;
  if (g.act != SAT_ACT_NONE && g.act != SAT_ACT_RELU) return 0;
  if (g.K % PBK || g.K < PBK || g.N % 8 || g.ldb % 8 || g.ldc % 8) return 0;
  if (!pal16(g.A) || !pal16(g.B) || !pal16(g.C) || (g.bias && ((uintptr_t)g.bias & 3))) return 0;
  if (g.add1 && (g.add1_dtype != SAT_BF16 || g.ld_add1 % 8 || !pal16(g.add1))) return 0;
  const bool conv = g.conv.C > 0;
  if (conv) {
    if (g.conv.C % PBK || g.conv.KH * g.conv.KW > 32) return 0;
    if ((long)g.conv.N * g.conv.H * g.conv.W * g.conv.C >= (1L << 31)) return 0;
  } else if (g.lda % 8 || (long)g.M * g.lda >= (1L << 31)) {
    return 0;
  }
  if ((long)g.N * g.ldb >= (1L << 31)) return 0;
  const long tiles = (long)sat_cdiv(g.M, PBM) * sat_cdiv(g.N, PBN);
  if (mode != 2) {
    // long-K problems that fill most of the chip with 256 x 128 tiles (tools/pipe_ab.py: ResNet152
    // L3 c1/c2, L2 c2, L4, every VGG19 conv from 128 channels on: 1.05-1.26x); short-K problems,
    // N < 128 and the residual 1x1 convs stay on fast_gemm_kernel (two workgroups per CU)
    if (tiles < 150 || g.N < 128 || g.add1) return 0;
    if (!(g.K >= 1024 || (g.K >= 512 && g.N >= 512))) return 0;
  }
  static bf16* zero = nullptr;
  if (!zero) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_pipe_zero16)) != hipSuccess) return 0;
    zero = (bf16*)p;
  }
  PArgs a{};
  a.M = g.M; a.N = g.N; a.K = g.K;
  a.A = (const bf16*)g.A; a.lda = g.lda;
  a.B = (const bf16*)g.B; a.ldb = g.ldb;
  a.C = (bf16*)g.C; a.ldc = g.ldc;
  a.bias = g.bias;
  a.res = (const bf16*)g.add1; a.ldr = g.ld_add1;
  if (conv) {
    a.H = g.conv.H; a.W = g.conv.W; a.Cin = g.conv.C; a.KW = g.conv.KW;
    a.stride = g.conv.stride; a.pad = g.conv.pad; a.OH = g.conv.OH; a.OW = g.conv.OW;
  }
  a.zero16 = zero;
  a.tiles_n = sat_cdiv(g.N, PBN);
  a.xcd_remap = 1;
  a.var = kPipeVar;
  a.st = sat_launch_stamps();
  {
    const long a_bytes = conv ? 2L * g.conv.N * g.conv.H * g.conv.W * g.conv.C : 2L * ((long)(g.M - 1) * g.lda + g.K);
    const long b_bytes = 2L * ((long)(g.N - 1) * g.ldb + g.K);
    // every buffer offset is 32-bit (sat_out_rsrc caps the C resource at 2 GiB): C below that too
    const long c_bytes = 2L * ((long)(g.M - 1) * g.ldc + g.N);
    if (a_bytes >= (1L << 31) || b_bytes >= (1L << 31) || c_bytes >= (1L << 31)) return 0;
    a.a_bytes = (unsigned)a_bytes;
    a.b_bytes = (unsigned)b_bytes;
  }
  const dim3 grid((unsigned)tiles);
  launch_nw<8>(conv, g.add1 != nullptr, g.act, grid, s, a);
  *err = (int)hipGetLastError();
  return 1;
}
