// Pipelined bf16 GEMM with fp32 output and deterministic split-K, for gfx950 (MI355X): the decoder's batched weight
// gradients dW = dY^T X and input gradients dX = dY W -- the autograd backward of the reference's nn.Linear /
// nn.LSTMCell weights (decoder.py:115,118-125,149-158, attention.py:15-16) that train.py:163's loss.backward() runs.
//
//   C[M,N] = A(m,k) . B(n,k) (+ add1[M,N]) (+ C when beta = 1)      bf16 in, fp32 accumulate, fp32 out
//   A(m,k) = AT ? A[k lda + m] : A[m lda + k];   B(n,k) = BT ? B[k ldb + n] : B[n ldb + k]
//
// These products have a long K (B (T-1) = 3,328 rows, or the vocabulary) and few output tiles (32-316), so most of
// them need split-K to fill 256 CUs.  Split-K by fp32 atomics into C (the tile kernel's form) is bound by the memory
// side's ~1.3 TB/s of added bytes (MI355X_MICROARCH.md, Global float atomics): 20-30 MB of atomics per product, as
// long as the GEMM itself.  Here:
//   * BM x 128 x 64 block tiles, BM = 256 (4 M x 2 N waves of 64 x 64) or 128 (2 x 4 waves of 64 x 32), one 8-wave
//     workgroup per CU; what bounds a tile is the bytes each CU's load path delivers (~45-50 GB/s per CU measured:
//     DESIGN.md 4.3), so the taller tile moves 25 % fewer bytes per FLOP and the planner below picks per shape;
//   * 3-stage LDS ring filled by buffer_load ... lds (16 B per lane; offsets past an operand's end read zeros, so K
//     tails and M / N edges need no branches), one counted vmcnt + raw s_barrier per k-tile with tile t+2 in
//     flight while t is consumed; k-major operands staged as 64 k-rows of 256 B and read by ds_read_b64_tr_b16
//     (cdna_hip_programming.md T10), m/n-major ones as 128-B rows read by ds_read_b128, both conflict-free;
//   * split-K without atomics: split s stores its fp32 partial tile, in the accumulator layout (1 KiB per wave
//     instruction), with write-through (sc1) stores into slab s of the caller's workspace, drains them, and takes
//     an agent-scope ticket; the workgroup that draws the last ticket adds the partials in split order 0, 1, ...,
//     S-1 (its own from registers, the others by sc1 loads) and writes C.  The sum does not depend on which split
//     finished last: bit-identical run to run.  Hand-off: the payload write-through (sc1) and drained by every storing
//     wave, a barrier, an agent-scope release + relaxed ticket add by one lane; the last adder takes an agent-scope
//     acquire before its sc1 loads (cdna_hip_programming.md Guideline 16: a release / acquire pair under the memory
//     model, besides the sc1 form MI355X_MICROARCH.md measures valid on its own);
//   * XCD-aware order: the n-tiles of one (split, m-tile) panel share an XCD's L2.
#include "sat_common.h"
#include "sat_internal.h"

// The partial-tile hand-off without agent-scope fences: every partial is stored `sc1` (write-through, 16 B), every
// storing wave waits vmcnt(0) before the workgroup barrier, one lane per workgroup then adds to the tile's ticket
// (agent atomic), the workgroup whose add returned splits - 1 is the reader, and every load of the partials is a 16-B
// `sc1` buffer load issued after that add returned (the other waves after the barrier the adding wave joins): the
// first row of MI355X_MICROARCH.md's table of hand-offs measured valid with `sc1` loads in place of the acquire, whose
// condition (2) makes the release redundant too (one workgroup per CU, hipMalloc'd workspace).  The fences cost a
// `buffer_wbl2` / `buffer_inv` per tile: bench line 6.111-6.136 -> 6.069-6.088 ms with both hand-offs fence-free
// (profiles/r6_s65, with the attention backward's); 1 = the fenced forms (A/B builds).
#ifndef SAT_SPLIT_RELEASE
#define SAT_SPLIT_RELEASE 0
#endif
#ifndef SAT_SPLIT_ACQUIRE
#define SAT_SPLIT_ACQUIRE 0
#endif
#ifndef SAT_SPLIT_DEBUG     // diagnostics builds: 1 = record every ticket draw (tools/debug_split_tickets.py)
#define SAT_SPLIT_DEBUG 0
#endif
#if SAT_SPLIT_DEBUG
__device__ unsigned g_sdbg[1 << 20];
__device__ unsigned g_sdbg_n;
__device__ unsigned g_sdbg_cs[64 * 256];   // per (launch % 64, tile): XOR of the final tile's bits
static unsigned g_sdbg_launch = 0;
#endif

namespace {

typedef __attribute__((address_space(3))) void sg_lds_void;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 sg_lds_bf16x4;

constexpr int SBN = 128, SBK = 64, SNSTG = 3;
constexpr unsigned SG_OOB = 0x80000000u;
constexpr int kMaxSplits = 8;
constexpr int kSplitCUs = 256;   // one workgroup per CU: a split grid stays within one round

template <int BM>
struct SGeom {
  static constexpr int WGN = BM == 256 ? 2 : 4;   // waves along N
  static constexpr int WGM = 8 / WGN;
  static constexpr int WTM = BM / WGM, WTN = SBN / WGN;
  static constexpr int MI = WTM / 16, NJ = WTN / 16;
  static constexpr int STAGE_A = BM * SBK * 2, STAGE_B = SBN * SBK * 2, STAGE = STAGE_A + STAGE_B;
  static constexpr int AI = STAGE_A / 1024 / 8, BI = STAGE_B / 1024 / 8, INSTR = AI + BI;   // 1 KiB DMAs per wave
  static constexpr int EPI_LD = SBN + 4;
  static constexpr int EPI_BYTES = BM * EPI_LD * 4;
  static constexpr int LDS = SNSTG * STAGE;
  static_assert(WTM == 64 && MI == 4, "wave tiles are 64 rows high");
  static_assert(EPI_BYTES + 16 <= LDS, "epilogue tile + ticket word must fit in the ring");
};

struct SArgs {
  int M, N, K;
  const bf16* A; long lda;
  const bf16* B; long ldb;
  float* C; long ldc;
  int beta1;              // C += product (beta = 1)
  const float* add1; long ld_add1;   // fp32 addend (nullable)
  int splits, kchunk;     // split s: K range [s kchunk, min(K, (s + 1) kchunk)), kchunk a multiple of SBK
  int a_mlim;             // k-major A: 8-element chunks are read while m + 8 <= a_mlim (SatGemm::a_tail)
  int tiles_m, tiles_n;
  unsigned a_bytes, b_bytes, c_bytes, slab_bytes;
  float* slab;            // splits > 1: [tile][split][BM x SBN] partials in the accumulator layout
  unsigned* tickets;      // splits > 1: one arrival counter per tile, zero at launch
  SatStamps st;
  unsigned dbg_launch;    // SAT_SPLIT_DEBUG builds: launch number
};

// k-major tile of 256-B rows: chunk slot of k-row r (conflict-free for ds_read_b64_tr_b16)
__device__ __forceinline__ int sg_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// MFMA 16x16x32 operand fragment (8 consecutive k of column xt + lane & 15) from a k-major tile: two transposing
// reads of 4 k-rows x 16 columns
__device__ __forceinline__ bf16x8 sg_frag_kmajor(const char* tile, int kbase, int xt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = (xt >> 3) + (p >> 1);
  const int r0 = kbase + 8 * g + q, r1 = r0 + 4;
  const char* a0 = tile + r0 * 256 + 16 * (ch ^ sg_swz(r0)) + 8 * (p & 1);
  const char* a1 = tile + r1 * 256 + 16 * (ch ^ sg_swz(r1)) + 8 * (p & 1);
  const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((sg_lds_bf16x4*)(uintptr_t)(const void*)a0);
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((sg_lds_bf16x4*)(uintptr_t)(const void*)a1);
  bf16x8 r;
  r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
  r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
  return r;
}

// this wave's vector-memory ops down to the N youngest, then a raw barrier (no __syncthreads: its fence would drain
// every LDS-DMA in flight)
template <int N>
__device__ __forceinline__ void sg_wait_barrier() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

__device__ __forceinline__ void sgdma(__amdgpu_buffer_rsrc_t r, char* dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (sg_lds_void*)dst, 16, (int)voff, 0, 0, 0);
}

__device__ __forceinline__ uint4 f4u(f32x4 v) {
  return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
}

template <int BM, bool AT, bool BT>
__device__ __forceinline__ void split_gemm_body(const SArgs& a) {
  using G = SGeom<BM>;
  constexpr int MI = G::MI, NJ = G::NJ, AI = G::AI, BI = G::BI;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / G::WGN, wn = w % G::WGN;

  int lin = blockIdx.x;
  {   // XCD-aware order (cdna_hip_programming.md T1, bijective form): each XCD takes a contiguous run of
      // (split, m-tile, n-tile) indices, so the workgroups on one XCD share their A panel
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = lin % 8;
    lin = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lin / 8;
  }
  const int nt = lin % a.tiles_n;
  const int rest = lin / a.tiles_n;
  const int mt = rest % a.tiles_m, split = rest / a.tiles_m;
  const int m0 = mt * BM, n0 = nt * SBN;
  const int M = a.M, N = a.N;
  const int kbeg = split * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + SBK - 1) / SBK : 0;

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, (short)0, (int)a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, (int)a.b_bytes, 0x00020000);
  // per-lane DMA pieces, fixed across k-tiles: k-major (4 k-rows of 256 B per 1 KiB instruction: lane -> k-row
  // lane >> 4, slot lane & 15) or m/n-major (8 rows of 128 B: lane -> row lane >> 3, slot lane & 7); the element
  // offset without k, and the k-row / k-chunk the lane adds per tile
  int a_off[AI], a_k[AI];
  bool a_ok[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    if constexpr (AT) {
      const int q = (w * AI + j) * 4 + (lane >> 4);   // half q >> 6 (128 m each), k-row q & 63
      const int kr = q & 63, ch = (lane & 15) ^ sg_swz(kr);
      const int m = m0 + (q >> 6) * 128 + 8 * ch;
      a_ok[j] = m + 8 <= a.a_mlim;
      a_off[j] = m;
      a_k[j] = kr;
    } else {
      const int r = (w * AI + j) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((r >> 1) & 7);
      a_ok[j] = m0 + r < M;
      a_off[j] = (int)((long)(m0 + r) * a.lda);
      a_k[j] = 8 * ch;
    }
  }
  int b_off[BI], b_k[BI];
  bool b_ok[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    if constexpr (BT) {
      const int kr = (w * BI + j) * 4 + (lane >> 4), ch = (lane & 15) ^ sg_swz(kr);
      const int n = n0 + 8 * ch;
      b_ok[j] = n + 8 <= N;
      b_off[j] = n;
      b_k[j] = kr;
    } else {
      const int r = (w * BI + j) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((r >> 1) & 7);
      b_ok[j] = n0 + r < N;
      b_off[j] = (int)((long)(n0 + r) * a.ldb);
      b_k[j] = 8 * ch;
    }
  }
  auto stage = [&](int buf, int k0) {
    char* sa = smem + buf * G::STAGE;
    char* sb = sa + G::STAGE_A;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int k = k0 + a_k[j];
      const bool ok = a_ok[j] && k < kend;
      const unsigned off = AT ? 2u * (unsigned)((long)k * a.lda + a_off[j]) : 2u * (unsigned)(a_off[j] + k);
      sgdma(rA, sa + (w * AI + j) * 1024, ok ? off : SG_OOB);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int k = k0 + b_k[j];
      const bool ok = b_ok[j] && k < kend;
      const unsigned off = BT ? 2u * (unsigned)((long)k * a.ldb + b_off[j]) : 2u * (unsigned)(b_off[j] + k);
      sgdma(rB, sb + (w * BI + j) * 1024, ok ? off : SG_OOB);
    }
  };

  // fragments of 32-deep half h of the tile in buf
  const int fr = lane & 15, fh = lane >> 4, sw = (fr >> 1) & 7;
  const int am = wm * G::WTM;   // the wave's first row in the tile
  auto frags = [&](int buf, int h, bf16x8 (&fa)[MI], bf16x8 (&fb)[NJ]) {
    const char* sa = smem + buf * G::STAGE;
    const char* sb = sa + G::STAGE_A;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if constexpr (AT) fa[i] = sg_frag_kmajor(sa + (am >> 7) * (64 * 256), h * 32, (am & 127) + i * 16, lane);
      else fa[i] = *(const bf16x8*)(sa + (am + i * 16 + fr) * 128 + 16 * ((h * 4 + fh) ^ sw));
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (BT) fb[j] = sg_frag_kmajor(sb, h * 32, wn * G::WTN + j * 16, lane);
      else fb[j] = *(const bf16x8*)(sb + (wn * G::WTN + j * 16 + fr) * 128 + 16 * ((h * 4 + fh) ^ sw));
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
      stage(1, kbeg + SBK);
      sg_wait_barrier<G::INSTR>();
    } else {
      sg_wait_barrier<0>();
    }
    frags(0, 0, xa, xb);
    int cur = 0;
    for (int t = 0; t < nk; ++t) {
      frags(cur, 1, ya, yb);   // second half of tile t (its reads retire before this tile's barrier)
      __builtin_amdgcn_sched_barrier(0);
      // tile t+2 into the stage tile t-1 used: every wave's reads of it retired before tile t-1's barrier
      const bool dma = t + 2 < nk;
      if (dma) stage(cur == 0 ? 2 : cur - 1, kbeg + (t + 2) * SBK);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mfma(xa, xb);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < nk) {
        // this wave's DMAs of tile t+1 have landed (t+2's stay in flight); after the barrier every wave's have
        if (dma) sg_wait_barrier<G::INSTR>();
        else sg_wait_barrier<0>();
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

  if (a.splits > 1) {
    // ---- publish this split's partial tile; the last arriver of the tile sums all of them in split order ----
    const long tile = (long)mt * a.tiles_n + nt;
    const __amdgpu_buffer_rsrc_t rS = sat_out_rsrc(a.slab, a.slab_bytes);
    constexpr unsigned PART = (unsigned)BM * SBN * 4;   // bytes of one partial tile
    const unsigned tbase = (unsigned)(tile * a.splits) * PART;
    auto slot = [&](int i, int j) { return (unsigned)((((w * MI + i) * NJ + j) * 64 + lane) * 16); };
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) sat_st16<16>(rS, tbase + (unsigned)split * PART + slot(i, j), f4u(acc[i][j]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its write-through stores are done
    __syncthreads();
    volatile unsigned* flag = (volatile unsigned*)(smem + G::EPI_BYTES);
    if (tid == 0) {
      if constexpr (SAT_SPLIT_RELEASE) {   // agent-scope release before the ticket (second wait: Guideline 16 Pitfall 12)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const unsigned prev = __hip_atomic_fetch_add(a.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if SAT_SPLIT_DEBUG
      {
        const unsigned i = atomicAdd(&g_sdbg_n, 1u);
        if (i < (1u << 18)) {
          g_sdbg[4 * i] = a.dbg_launch; g_sdbg[4 * i + 1] = (unsigned)tile; g_sdbg[4 * i + 2] = (unsigned)split;
          g_sdbg[4 * i + 3] = prev;
        }
      }
#endif
      if constexpr (SAT_SPLIT_ACQUIRE) {
        if (prev == (unsigned)(a.splits - 1)) {
          // the last arriver: agent-scope acquire before it reads the other partial tiles
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      *flag = prev;
    }
    __syncthreads();
    if (*flag != (unsigned)(a.splits - 1)) return;   // workgroup-uniform
    f32x4 tot[MI][NJ], part[MI][NJ];
    for (int s = 0; s < a.splits; ++s) {   // split order: the same sums whichever split arrives last
      if (s == split) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) part[i][j] = acc[i][j];
      } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const sat_u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rS, (int)(tbase + (unsigned)s * PART + slot(i, j)), 0, 16);
            part[i][j] = f32x4{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3])};
          }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) tot[i][j] = s == 0 ? part[i][j] : tot[i][j] + part[i][j];
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = tot[i][j];
  }

#if SAT_SPLIT_DEBUG
  {
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) x ^= __float_as_uint(acc[i][j][r]) * (unsigned)(1 + ((i * NJ + j) * 4 + r));
    atomicXor(&g_sdbg_cs[(a.dbg_launch % 64) * 256 + ((long)mt * a.tiles_n + nt) % 256], x);
  }
#endif
  // ---- C: the fp32 tile through LDS, 16-B row pieces (beta = 1 adds C) ----
  sg_wait_barrier<0>();   // every wave done with the ring
  float* ep = (float*)smem;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int cl = wn * G::WTN + j * 16 + fr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(am + i * 16 + fh * 4 + r) * G::EPI_LD + cl] = acc[i][j][r];
  }
  __syncthreads();
  const int cc = tid & 15, r0 = tid >> 4;   // 16 chunks of 8 columns x 32 rows per pass
  const int col = n0 + cc * 8;
  if (col >= N) return;   // N % 8 == 0 (host-checked): a chunk is all in or all out
  const __amdgpu_buffer_rsrc_t rC = sat_out_rsrc(a.C, a.c_bytes);
#pragma unroll
  for (int it = 0; it < BM / 32; ++it) {
    const int rl = r0 + it * 32, row = m0 + rl;
    if (row >= M) break;
    float4 x0 = *(const float4*)(ep + rl * G::EPI_LD + cc * 8);
    float4 x1 = *(const float4*)(ep + rl * G::EPI_LD + cc * 8 + 4);
    const unsigned off = (unsigned)(((long)row * a.ldc + col) * 4);
    if (a.add1) {
      const float* p = a.add1 + (long)row * a.ld_add1 + col;
      x0 = f4add(x0, *(const float4*)p);
      x1 = f4add(x1, *(const float4*)(p + 4));
    }
    if (a.beta1) {
      const float* p = a.C + (long)row * a.ldc + col;
      x0 = f4add(x0, *(const float4*)p);
      x1 = f4add(x1, *(const float4*)(p + 4));
    }
    sat_st16<0>(rC, off, make_uint4(__float_as_uint(x0.x), __float_as_uint(x0.y), __float_as_uint(x0.z), __float_as_uint(x0.w)));
    sat_st16<0>(rC, off + 16, make_uint4(__float_as_uint(x1.x), __float_as_uint(x1.y), __float_as_uint(x1.z), __float_as_uint(x1.w)));
  }
}

template <int BM, bool AT, bool BT>
__global__ __launch_bounds__(512) void split_gemm_kernel(SArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  split_gemm_body<BM, AT, BT>(a);
  sat_stamp_end(a.st, t0);
}

inline bool sal16(const void* p) { return ((uintptr_t)p & 15) == 0; }

struct SPlan {
  int bm = 0, splits = 1, kchunk = 0, tiles_m = 0, tiles_n = 0;
  double us = 0;
};

// Cost model (microseconds), one 8-wave workgroup per CU: a k-tile per workgroup takes what the CU's load path
// needs for its bytes (128 x 128: 32 KiB, 256 x 128: 48 KiB at ~45 GB/s per CU), the C epilogue ~1 us, and the
// last arriver of a split tile reads S-1 partial tiles at ~70 GB/s (MI355X_MICROARCH.md handoff-payload).
constexpr double kKtileUs[2] = {0.73, 1.10};   // BM = 128, 256
constexpr double kEpiUs = 1.0;
constexpr double kPartUs[2] = {0.94, 1.87};
// SatPolicy::split_gemm: 0 auto, 2 128-row tiles, 3 256-row tiles; SatPolicy::split_k > 0 forces the split count
SPlan plan_split(const SatGemm& g, bool have_ws) {
  const SatPolicy& pol = sat_policy();
  const int nk = sat_cdiv(g.K, SBK);
  SPlan best;
  best.us = 1e30;
  for (int b = 0; b < 2; ++b) {
    const int bm = b ? 256 : 128;
    if ((pol.split_gemm == 2 && bm != 128) || (pol.split_gemm == 3 && bm != 256)) continue;
    const int tm = sat_cdiv(g.M, bm), tn = sat_cdiv(g.N, SBN);
    const long tiles = (long)tm * tn;
    for (int s = 1; s <= kMaxSplits; ++s) {
      if (pol.split_k > 0 && s != pol.split_k) continue;
      if (s > 1 && (!have_ws || tiles * s > kSplitCUs || nk < 2 * s)) continue;
      const int kch = sat_cdiv(nk, s);
      const int splits = sat_cdiv(nk, kch);   // no empty split
      if (splits != s) continue;
      const double us = sat_cdiv(tiles * s, kSplitCUs) * (kch * kKtileUs[b] + kEpiUs) + (s - 1) * kPartUs[b];
      if (us < best.us - 1e-9) {
        best.bm = bm; best.splits = s; best.kchunk = kch * SBK; best.tiles_m = tm; best.tiles_n = tn; best.us = us;
      }
    }
  }
  return best;
}

// the problems this kernel takes: bf16 operands, fp32 C, C = A B (+ add1) (+ C), a k-major operand or an NN product
// the tile kernel would split with atomics, 16-B pieces
bool split_eligible(const SatGemm& g) {
  const int mode = sat_policy().split_gemm;
  if (mode == 1) return false;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_F32 || g.batch != 1 || g.aux || g.bias || g.conv.C > 0 ||
      g.act != SAT_ACT_NONE || g.partial_splits > 1 || g.alpha != 1.f || (g.beta != 0.f && g.beta != 1.f))
    return false;
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return false;
  // both operands k-contiguous (NN): only the products the tile kernel would split with fp32 atomics (few 128 x 128
  // tiles, K >= 1024) -- here they keep a fixed summation order (the decoder's gradients are bit-reproducible)
  if (!(g.transA || g.transB) && !((long)sat_cdiv(g.M, 128) * sat_cdiv(g.N, 128) < 160 && g.K >= 1024)) return false;
  const bool at = g.transA != 0, bt = g.transB != 0;
  if (g.lda % 8 || g.ldb % 8 || g.ldc % 4 || g.N % 8) return false;
  // a K tail (K % 8 != 0) only where the straddling 8-element chunks read zeros: an m-major A zero-padded to the next
  // multiple of 8 (SatGemm::a_tail) against a k-major B, whose rows past K the loader skips
  if (at ? (g.M % 8 && !g.a_tail) : (g.K % 8 && !(g.a_tail && bt))) return false;
  if (!bt && g.K % 8) return false;
  if (!sal16(g.A) || !sal16(g.B) || !sal16(g.C)) return false;
  if (g.add1 && (g.add1_dtype != SAT_F32 || !sal16(g.add1) || g.ld_add1 % 4)) return false;
  // buffer offsets are 32-bit: every operand and C below 2 GiB
  const long a_bytes = at ? 2L * ((long)(g.K - 1) * g.lda + (g.a_tail ? sat_cdiv(g.M, 8) * 8 : g.M))
                          : 2L * ((long)(g.M - 1) * g.lda + sat_cdiv(g.K, 8) * 8);
  const long b_bytes = bt ? 2L * ((long)(g.K - 1) * g.ldb + g.N) : 2L * ((long)(g.N - 1) * g.ldb + g.K);
  const long c_bytes = 4L * ((long)(g.M - 1) * g.ldc + g.N);
  if (a_bytes >= (1L << 31) || b_bytes >= (1L << 31) || c_bytes >= (1L << 31)) return false;
  // auto: the long-K products (the weight gradients and the vocabulary / embedding input gradients)
  if (mode == 0 && g.K < 512) return false;
  return true;
}

}  // namespace

size_t sat_split_gemm_ws_bytes() {
  static_assert(kSatSplitTickets >= kSplitCUs, "a split launch has at most kSplitCUs tiles");
  return (size_t)kSplitCUs * 256 * SBN * 4 + kSatSplitTickets * 4;   // partial tiles + tickets
}

// Without a workspace the kernel can only run unsplit: it takes such a call only where the planner would not split
// it anyway.  A long-K product with few tiles (the NN shapes the tile kernel splits with atomics over ~300
// workgroups, or a k-major weight gradient) falls through to sat_fast_gemm_try instead of running on a handful of
// workgroups.
static bool split_takes(const SatGemm& g) {
  if (!split_eligible(g)) return false;
  if (g.split_ws && g.split_tickets) return true;
  return plan_split(g, true).splits <= 1;
}

int sat_split_gemm_takes(const SatGemm& g) { return split_takes(g) ? 1 : 0; }

int sat_split_gemm_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  if (!split_takes(g)) return 0;
  const bool have_ws = g.split_ws && g.split_tickets;
  const SPlan p = plan_split(g, have_ws);
  if (p.bm == 0) return 0;
  const bool at = g.transA != 0, bt = g.transB != 0;
  SArgs a{};
  a.M = g.M; a.N = g.N; a.K = g.K;
  a.A = (const bf16*)g.A; a.lda = g.lda; a.B = (const bf16*)g.B; a.ldb = g.ldb;
  a.C = (float*)g.C; a.ldc = g.ldc;
  a.beta1 = g.beta != 0.f;
  a.add1 = (const float*)g.add1; a.ld_add1 = g.ld_add1;
  a.splits = p.splits; a.kchunk = p.kchunk;
  a.a_mlim = at && g.a_tail ? sat_cdiv(g.M, 8) * 8 : g.M;
  a.tiles_m = p.tiles_m; a.tiles_n = p.tiles_n;
  a.a_bytes = (unsigned)(at ? 2L * ((long)(g.K - 1) * g.lda + a.a_mlim)
                            : 2L * ((long)(g.M - 1) * g.lda + sat_cdiv(g.K, 8) * 8));
  a.b_bytes = (unsigned)(bt ? 2L * ((long)(g.K - 1) * g.ldb + g.N) : 2L * ((long)(g.N - 1) * g.ldb + g.K));
  a.c_bytes = (unsigned)(4L * ((long)(g.M - 1) * g.ldc + g.N));
  if (p.splits > 1) {
    const long slab = (long)p.tiles_m * p.tiles_n * p.splits * p.bm * SBN * 4;
    SAT_REQUIRE(slab <= g.split_ws_bytes && (long)p.tiles_m * p.tiles_n <= kSplitCUs);
    a.slab = g.split_ws; a.slab_bytes = (unsigned)slab;
    a.tickets = g.split_tickets;
    if (!g.tickets_zeroed)
      SAT_CHECK((hipError_t)sat_zero_rows((float*)g.split_tickets, (long)p.tiles_m * p.tiles_n, 1,
                                          (long)p.tiles_m * p.tiles_n, s));
  }
  a.st = sat_launch_stamps();
#if SAT_SPLIT_DEBUG
  a.dbg_launch = ++g_sdbg_launch;
#endif
  const dim3 grid((unsigned)((long)p.tiles_m * p.tiles_n * p.splits));
  if (p.bm == 256) {
    if (at && bt) hipLaunchKernelGGL((split_gemm_kernel<256, true, true>), grid, dim3(512), 0, s, a);
    else if (at) hipLaunchKernelGGL((split_gemm_kernel<256, true, false>), grid, dim3(512), 0, s, a);
    else if (bt) hipLaunchKernelGGL((split_gemm_kernel<256, false, true>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((split_gemm_kernel<256, false, false>), grid, dim3(512), 0, s, a);
  } else {
    if (at && bt) hipLaunchKernelGGL((split_gemm_kernel<128, true, true>), grid, dim3(512), 0, s, a);
    else if (at) hipLaunchKernelGGL((split_gemm_kernel<128, true, false>), grid, dim3(512), 0, s, a);
    else if (bt) hipLaunchKernelGGL((split_gemm_kernel<128, false, true>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((split_gemm_kernel<128, false, false>), grid, dim3(512), 0, s, a);
  }
  *err = (int)hipGetLastError();
  return 1;
}

#if SAT_SPLIT_DEBUG
// diagnostics builds: copy the ticket-draw records {launch, tile, split, prev} (n4 = 4 x records) and reset them
extern "C" int sat_split_debug_read(unsigned* out, int n4, unsigned* count) {
  SAT_CHECK(hipDeviceSynchronize());
  SAT_CHECK(hipMemcpyFromSymbol(count, HIP_SYMBOL(g_sdbg_n), sizeof(unsigned)));
  const unsigned m = *count * 4 < (unsigned)n4 ? *count * 4 : (unsigned)n4;
  if (m) SAT_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdbg), m * sizeof(unsigned)));
  const unsigned z = 0;
  SAT_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sdbg_n), &z, sizeof(unsigned)));
  return 0;
}
extern "C" int sat_split_debug_checksums(unsigned* out) {   // 64 x 256 words, then zeroed
  SAT_CHECK(hipDeviceSynchronize());
  SAT_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdbg_cs), 64 * 256 * sizeof(unsigned)));
  static unsigned zeros[64 * 256] = {};
  SAT_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sdbg_cs), zeros, sizeof(zeros)));
  return 0;
}
#endif
