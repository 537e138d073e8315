// Register-direct skinny GEMM for the decoder's per-step products (gfx950 / MI355X), and the same GEMM with the
// LSTM cell folded into its split-K reduction.
//
//   C_s[m, n] = sum_{k in split s} A[m, k] W[n, k]  (+ bias[n] in split 0),  M <= 128 rows (the batch),
//   A, W bf16 row-major (k contiguous), C fp32; split s writes its own slab C + s * split_stride
//   (the decoder's partial-output split-K contract, SatGemm::partial_splits), or plain C when unsplit.
//
// Why: the per-step GEMMs of the recurrent loop -- the context half of the LSTM input GEMM (N 2048, K 2048) and
// the BPTT's dL/d(gated context) / dL/dh products at M = B = 128 (decoder.py:96-115) -- move 5-10 MB each and
// sit in a dependent chain, so their time is latency, not bandwidth.  The LDS-DMA tile kernel (convgemm.hip) runs
// a 3-stage ring with a barrier per 64-deep k-tile and holds 74 KB of LDS, which also keeps it off every CU where
// a concurrent encoder workgroup lives.  Here:
//   * a workgroup owns 32 output columns x all rows; its NW waves split the workgroup's K range
//     (<= 128 per wave: 4 k-steps of 32);
//   * every operand fragment of the wave -- A rows (MB 16-row blocks) and W rows (2 16-column blocks),
//     16 B per lane per k-step -- is requested at kernel entry straight into VGPRs, so the launch pays
//     one memory latency; no LDS ring, no per-k-tile barrier;
//   * v_mfma_f32_16x16x32_bf16 with W as the A operand computes C^T, so a lane ends with 4 consecutive
//     columns of one row;
//   * the NW partial tiles meet in one 18 KB LDS tile in wave order (fixed summation order: results
//     do not depend on scheduling), then the workgroup stores 16-B row pieces.
//
// Fused forms (decoder.py:107-115 LSTMCell after the gate GEMM; its backward):
//   * skinny_lstm_fwd_kernel: the context GEMM gated_ctx . W_ih[:, E:]^T with gate-interleaved columns -- block x
//     owns units 8x .. 8x+7 of all four gates (W rows q E + 8x + i), so one block row holds whole LSTM cells;
//   * skinny_lstm_bwd_kernel: the recurrent dL/dh GEMM of step t (block x: units 32x .. 32x+31), whose sums are the
//     dL/dh of step t-1's cell.
// Each split's partial tile goes to its slab with write-through (sc1) 16-B stores; every wave drains (vmcnt 0),
// the workgroup meets at a barrier, one lane adds to the block's arrival ticket (agent scope), and the workgroup
// whose add returns S-1 -- the last to arrive -- reads every slab with sc1 loads and runs the LSTM cell
// forward / backward for its units in the summation order of lstm_fwd_gp_kernel / lstm_bwd_gp_kernel (bit-identical
// to the separate launches), then re-zeroes the ticket for the next step.  That is the counter form of
// MI355X_MICROARCH.md's hand-off table (row 1: sc1 stores drained before one lane's agent-scope add, the
// last adder's workgroup loading after a barrier, every load of the slabs sc1; cdna_hip_programming.md §6
// Guideline 16).  It removes one launch (and its ~2-5 us boundary) per time step in each direction.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

constexpr int SK_COLS = 32;            // output columns per workgroup
constexpr int SK_RLD = SK_COLS + 4;    // LDS tile row stride (floats)
constexpr int SK_KW = 128;             // max k per wave

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;               // buffer instruction cache-policy bits: sc1 (write-through / L1 bypass)

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
  for (int q = threadIdx.x; q < PIECES; q += NW * 64) {
    const int row = q >> 3, c4 = (q & 7) * 4;
    if (row >= a.M) continue;
    float4 v = *(const float4*)(red + row * SK_RLD + c4);
    const int n = col_of(a, c4);
    if (bias) {
      const float4 b = *(const float4*)(bias + n);
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    *(float4*)(Cs + (long)row * a.ldc + n) = v;
  }
  sat_stamp_end(a.st, t0);
}

// ---- fused forms: publish the split's tile, count arrivals, the last arriver runs the cell ----
__device__ __forceinline__ float4 ld4_sc1(__amdgpu_buffer_rsrc_t r, long elem) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 4), 0, kSc1);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
// sum_parts4's summation order (sat_internal.h) over N values already in registers: (a0 + a1) + (a2 + a3) with
// a1..a3 taking the slabs 1, 2, 3, 4, 5, 6, ... round robin (compile-time N: every load of a reducer is issued
// before the first add, one memory round trip per item instead of one per slab)
template <int N>
__device__ __forceinline__ float4 sum_slabs(const float4 (&p)[N]) {
  if constexpr (N == 1) {
    return p[0];
  } else {
    float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1, a3 = a1;
    int sp = 1;
#pragma unroll
    for (; sp + 2 < N; sp += 3) { a1 = f4add(a1, p[sp]); a2 = f4add(a2, p[sp + 1]); a3 = f4add(a3, p[sp + 2]); }
#pragma unroll
    for (; sp < N; ++sp) a1 = f4add(a1, p[sp]);
    return f4add(f4add(p[0], a1), f4add(a2, a3));
  }
}

// Write this split's tile to its slab (write-through), drain, count the arrival; true in the last arriver.
template <int MB, int NW>
__device__ __forceinline__ bool publish_and_count(const SkArgs& a, const float* red, __amdgpu_buffer_rsrc_t rc,
                                                  unsigned* ticket, int* s_last) {
  const int s = blockIdx.y, S = gridDim.y;
  constexpr int PIECES = MB * 16 * (SK_COLS / 4);
  for (int q = threadIdx.x; q < PIECES; q += NW * 64) {
    const int row = q >> 3, c4 = (q & 7) * 4;
    if (row >= a.M) continue;
    const float4 v = *(const float4*)(red + row * SK_RLD + c4);
    const long off = (long)s * a.split_stride + (long)row * a.ldc + col_of(a, c4);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                                                 __float_as_uint(v.w)}, rc, (int)(off * 4), 0, kSc1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its write-through stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = prev == (unsigned)(S - 1);
  }
  __syncthreads();
  return *s_last != 0;   // workgroup-uniform
}

struct SkLstmFwdArgs {
  SkArgs g;            // context GEMM, gate-interleaved (g.gate_E = E); g.C = the partial slabs ([B][4E] each)
  unsigned* ticket;    // [E / 8] arrivals per unit block (zero before the launch; the last arriver re-zeroes)
  LstmFwdArgs l;       // the cell step; its cpart / c_splits are g's slabs
};

template <typename T, int MB, int NW, int SC, int HS>
__global__ __launch_bounds__(NW * 64) void skinny_lstm_fwd_kernel(SkLstmFwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.g.st);
  __shared__ __attribute__((aligned(16))) float red[MB * 16 * SK_RLD];
  __shared__ int s_last;
  skinny_tile<MB, NW>(a.g, red);
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.g.C, (short)0, (int)((long)SC * a.g.split_stride * 4), 0x00020000);
  if (publish_and_count<MB, NW>(a.g, red, rc, a.ticket, &s_last)) {
    // the cells of units u0 .. u0+7, every row: a thread per (row, 4 units), every operand requested up front
    const LstmFwdArgs& l = a.l;
    const int E = a.g.gate_E, u0 = blockIdx.x * 8;
    for (int it = threadIdx.x; it < a.g.M * 2; it += NW * 64) {
      const int b = it >> 1, j = u0 + (it & 1) * 4;
      float4 xq[4], hq[4][HS], cq[4][SC];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xq[q] = *(const float4*)(l.xpart + (long)b * l.xpart_ld + q * E + j);
#pragma unroll
        for (int k = 0; k < HS; ++k) hq[q][k] = *(const float4*)(l.hpart + k * l.h_split_stride + (long)b * l.hpart_ld + q * E + j);
#pragma unroll
        for (int k = 0; k < SC; ++k) cq[q][k] = ld4_sc1(rc, k * a.g.split_stride + (long)b * a.g.ldc + q * E + j);
      }
      const float4 cp = *(const float4*)(l.c_prev + (long)b * l.c_prev_ld + j);
      float4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)   // lstm_fwd_gp_kernel's order: (xpart + sum of h slabs) + sum of c slabs
        v[q] = f4add(f4add(xq[q], sum_slabs<HS>(hq[q])), sum_slabs<SC>(cq[q]));
      const float gi[4] = {v[0].x, v[0].y, v[0].z, v[0].w}, gf[4] = {v[1].x, v[1].y, v[1].z, v[1].w},
                  gg[4] = {v[2].x, v[2].y, v[2].z, v[2].w}, go[4] = {v[3].x, v[3].y, v[3].z, v[3].w},
                  cpv[4] = {cp.x, cp.y, cp.z, cp.w};
      float cn[4], hn[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) lstm_cell_fwd(gi[k], gf[k], gg[k], go[k], cpv[k], cn[k], hn[k]);
#pragma unroll
      for (int q = 0; q < 4; ++q) *(float4*)(l.gates + (long)b * l.gates_ld + q * E + j) = v[q];
      const float4 c4 = make_float4(cn[0], cn[1], cn[2], cn[3]), h4 = make_float4(hn[0], hn[1], hn[2], hn[3]);
      *(float4*)(l.c_out + (long)b * l.c_out_ld + j) = c4;
      if (l.c_next_in) *(float4*)(l.c_next_in + (long)b * l.c_next_in_ld + j) = c4;
      *(float4*)(l.h_out + (long)b * l.h_out_ld + j) = h4;
      T ht[4] = {(T)hn[0], (T)hn[1], (T)hn[2], (T)hn[3]};
      if (l.h_out_t) {
        T* p = (T*)l.h_out_t + (long)b * l.h_out_t_ld + j;
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = ht[k];
      }
      if (l.h_next_in_t) {
        T* p = (T*)l.h_next_in_t + (long)b * l.h_next_in_t_ld + j;
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = ht[k];
      }
    }
    if (threadIdx.x == 0) __hip_atomic_store(a.ticket + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  sat_stamp_end(a.g.st, t0);
}

struct SkLstmBwdArgs {
  SkArgs g;            // recurrent dL/dh GEMM of step t (plain columns = units); g.C = the partial slabs ([B][E] each)
  unsigned* ticket;    // [E / 32]
  LstmBwdArgs l;       // step t-1's cell backward; its dh_rec / dh_splits are g's slabs
};

template <typename T, int MB, int NW, int SC>
__global__ __launch_bounds__(NW * 64) void skinny_lstm_bwd_kernel(SkLstmBwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.g.st);
  __shared__ __attribute__((aligned(16))) float red[MB * 16 * SK_RLD];
  __shared__ int s_last;
  skinny_tile<MB, NW>(a.g, red);
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.g.C, (short)0, (int)((long)SC * a.g.split_stride * 4), 0x00020000);
  if (publish_and_count<MB, NW>(a.g, red, rc, a.ticket, &s_last)) {
    const LstmBwdArgs& l = a.l;
    const int E = l.E, u0 = blockIdx.x * SK_COLS;
    for (int it = threadIdx.x; it < a.g.M * 8; it += NW * 64) {
      const int b = it >> 3, j = u0 + (it & 7) * 4;
      // every operand of the item requested up front
      float4 sl[SC];
#pragma unroll
      for (int sp = 0; sp < SC; ++sp) sl[sp] = ld4_sc1(rc, (long)sp * a.g.split_stride + (long)b * a.g.ldc + j);
      float4 g4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) g4[q] = *(const float4*)(l.gates + (long)b * l.gates_ld + q * E + j);
      const float4 cp = *(const float4*)(l.c_prev + (long)b * l.c_prev_ld + j);
      const float4 cn = *(const float4*)(l.c_new + (long)b * l.c_new_ld + j);
      const long di = (long)b * E + j;
      const float4 dci = l.dc_zero ? make_float4(0.f, 0.f, 0.f, 0.f) : *(const float4*)(l.dc + di);
      float hh[4] = {0.f, 0.f, 0.f, 0.f};
      if (l.dh_head) {
        const float4 h4 = *(const float4*)(l.dh_head + (long)b * l.dh_head_ld + j);
        hh[0] = h4.x; hh[1] = h4.y; hh[2] = h4.z; hh[3] = h4.w;
        if (l.mask) {
          const uchar4 m = *(const uchar4*)(l.mask + (long)b * l.mask_ld + j);
          hh[0] = m.x ? hh[0] * 2.f : 0.f; hh[1] = m.y ? hh[1] * 2.f : 0.f;
          hh[2] = m.z ? hh[2] * 2.f : 0.f; hh[3] = m.w ? hh[3] * 2.f : 0.f;
        }
      }
      // lstm_bwd_gp_kernel's order: p_q = sum of slabs q, q+4, ... (q = 0..3), dh = ((p0 + p1) + (p2 + p3)) + head
      float4 p[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        p[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int sp = q; sp < SC; sp += 4) p[q] = f4add(p[q], sl[sp]);
      }
      const float4 dh4 = f4add(f4add(p[0], p[1]), f4add(p[2], p[3]));
      const float dhs[4] = {dh4.x + hh[0], dh4.y + hh[1], dh4.z + hh[2], dh4.w + hh[3]};
      const float gi[4] = {g4[0].x, g4[0].y, g4[0].z, g4[0].w}, gf[4] = {g4[1].x, g4[1].y, g4[1].z, g4[1].w},
                  gg[4] = {g4[2].x, g4[2].y, g4[2].z, g4[2].w}, go[4] = {g4[3].x, g4[3].y, g4[3].z, g4[3].w};
      const float cpv[4] = {cp.x, cp.y, cp.z, cp.w}, cnv[4] = {cn.x, cn.y, cn.z, cn.w},
                  dcv[4] = {dci.x, dci.y, dci.z, dci.w};
      float dq[4][4], dco[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float d[4];
        lstm_cell_bwd(gi[k], gf[k], gg[k], go[k], cpv[k], cnv[k], dcv[k], dhs[k], d, dco[k]);
#pragma unroll
        for (int q = 0; q < 4; ++q) dq[q][k] = d[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        *(float4*)(l.d_gates + (long)b * l.d_gates_ld + q * E + j) = make_float4(dq[q][0], dq[q][1], dq[q][2], dq[q][3]);
        if (l.d_gates_t) {
          T* o = (T*)l.d_gates_t + (long)b * l.d_gates_t_ld + q * E + j;
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = (T)dq[q][k];
        }
      }
      *(float4*)(l.dc + di) = make_float4(dco[0], dco[1], dco[2], dco[3]);
    }
    if (threadIdx.x == 0) __hip_atomic_store(a.ticket + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  sat_stamp_end(a.g.st, t0);
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
  return al16(g.A) && al16(g.B) && al16(g.C) && (!g.bias || al16(g.bias));
}

template <int MB>
void launch_mb(int nw, dim3 grid, hipStream_t st, const SkArgs& a) {
  if (nw == 8) hipLaunchKernelGGL((skinny_gemm_kernel<MB, 8>), grid, dim3(512), 0, st, a);
  else hipLaunchKernelGGL((skinny_gemm_kernel<MB, 4>), grid, dim3(256), 0, st, a);
}

// the fused kernels' compile-time slab counts: context slabs x h slabs (forward), dh slabs (backward); other
// counts run the separate launches (the *_ok predicates say no)
constexpr bool fwd_counts_ok(int sc, int hs) { return (sc == 2 || sc == 4) && (hs == 1 || hs == 2); }
constexpr bool bwd_count_ok(int sc) { return sc == 6 || sc == 9; }

template <int MB, int NW, int SC, int HS>
void launch_fwd4(dim3 grid, hipStream_t st, const SkLstmFwdArgs& a) {
  hipLaunchKernelGGL((skinny_lstm_fwd_kernel<bf16, MB, NW, SC, HS>), grid, dim3(NW * 64), 0, st, a);
}
template <int MB, int NW>
void launch_fwd(int sc, int hs, dim3 grid, hipStream_t st, const SkLstmFwdArgs& a) {
  if (sc == 2) hs == 1 ? launch_fwd4<MB, NW, 2, 1>(grid, st, a) : launch_fwd4<MB, NW, 2, 2>(grid, st, a);
  else hs == 1 ? launch_fwd4<MB, NW, 4, 1>(grid, st, a) : launch_fwd4<MB, NW, 4, 2>(grid, st, a);
}
template <int MB, int NW>
void launch_bwd(int sc, dim3 grid, hipStream_t st, const SkLstmBwdArgs& a) {
  if (sc == 6) hipLaunchKernelGGL((skinny_lstm_bwd_kernel<bf16, MB, NW, 6>), grid, dim3(NW * 64), 0, st, a);
  else hipLaunchKernelGGL((skinny_lstm_bwd_kernel<bf16, MB, NW, 9>), grid, dim3(NW * 64), 0, st, a);
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

int sat_skinny_lstm_fwd_ok(const SatGemm& g, int E, int h_splits) {
  SkArgs a;
  int nw;
  const int S = g.partial_splits > 1 ? g.partial_splits : 1;
  return sat_policy().fused_lstm == 2 && E % 8 == 0 && g.N == 4 * E && !g.bias && fwd_counts_ok(S, h_splits) &&
         skinny_shape(g, sat_policy().skinny, &a, &nw);
}

int sat_skinny_lstm_bwd_ok(const SatGemm& g, int E) {
  SkArgs a;
  int nw;
  const int S = g.partial_splits > 1 ? g.partial_splits : 1;
  return sat_policy().fused_lstm == 2 && E % SK_COLS == 0 && g.N == E && !g.bias && bwd_count_ok(S) &&
         skinny_shape(g, sat_policy().skinny, &a, &nw);
}

int sat_skinny_lstm_fwd_try(const SatGemm& g, int E, unsigned* ticket, const LstmFwdArgs& l, hipStream_t st, int* err) {
  *err = 0;
  SkLstmFwdArgs a{};
  int nw;
  const int hs = l.h_splits > 1 ? l.h_splits : 1;
  if (!sat_skinny_lstm_fwd_ok(g, E, hs) || !skinny_shape(g, sat_policy().skinny, &a.g, &nw) || !skinny_ptrs(g) ||
      !ticket)
    return 0;
  if (l.dtype != SAT_BF16 || (l.xpart_ld | l.hpart_ld | l.c_prev_ld | l.gates_ld | l.c_out_ld | l.h_out_ld) % 4 ||
      (hs > 1 && l.h_split_stride % 4) || !al16(l.xpart) || !al16(l.hpart) || !al16(l.c_prev) ||
      !al16(l.gates) || !al16(l.c_out) || !al16(l.h_out) || (l.c_next_in && (!al16(l.c_next_in) || l.c_next_in_ld % 4)))
    return 0;
  a.g.gate_E = E;
  a.g.split_stride = g.partial_splits > 1 ? g.split_stride : 0;
  a.g.st = sat_launch_stamps();
  a.ticket = ticket;
  a.l = l;
  const int S = g.partial_splits > 1 ? g.partial_splits : 1;
  const dim3 grid(E / 8, S);
  if (g.M <= 32) nw == 8 ? launch_fwd<2, 8>(S, hs, grid, st, a) : launch_fwd<2, 4>(S, hs, grid, st, a);
  else if (g.M <= 64) nw == 8 ? launch_fwd<4, 8>(S, hs, grid, st, a) : launch_fwd<4, 4>(S, hs, grid, st, a);
  else nw == 8 ? launch_fwd<8, 8>(S, hs, grid, st, a) : launch_fwd<8, 4>(S, hs, grid, st, a);
  *err = (int)hipGetLastError();
  return 1;
}

int sat_skinny_lstm_bwd_try(const SatGemm& g, unsigned* ticket, const LstmBwdArgs& l, hipStream_t st, int* err) {
  *err = 0;
  SkLstmBwdArgs a{};
  int nw;
  if (!sat_skinny_lstm_bwd_ok(g, l.E) || !skinny_shape(g, sat_policy().skinny, &a.g, &nw) || !skinny_ptrs(g) ||
      !ticket)
    return 0;
  if (l.dtype != SAT_BF16 || (l.gates_ld | l.c_prev_ld | l.c_new_ld | l.d_gates_ld | l.dh_head_ld) % 4 ||
      !al16(l.gates) || !al16(l.c_prev) || !al16(l.c_new) || !al16(l.dc) || !al16(l.d_gates) ||
      (l.dh_head && !al16(l.dh_head)) || (l.mask && (((uintptr_t)l.mask & 3) || l.mask_ld % 4)))
    return 0;
  // eight waves: the cell backward of a 32-unit block is 8 M items, two per thread (the K split per wave halves)
  a.g.kw = sat_cdiv(sat_cdiv(a.g.kc, 8), 32) * 32;
  a.g.split_stride = g.partial_splits > 1 ? g.split_stride : 0;
  a.g.st = sat_launch_stamps();
  a.ticket = ticket;
  a.l = l;
  const int S = g.partial_splits > 1 ? g.partial_splits : 1;
  const dim3 grid(g.N / SK_COLS, S);
  if (g.M <= 32) launch_bwd<2, 8>(S, grid, st, a);
  else if (g.M <= 64) launch_bwd<4, 8>(S, grid, st, a);
  else launch_bwd<8, 8>(S, grid, st, a);
  *err = (int)hipGetLastError();
  return 1;
}
