// Fast bf16 NT GEMM / implicit-GEMM convolution for gfx950 (MI355X).
//
//   C[M,N] = act(A[M,K] . B[N,K]^T + bias[N] + add1[M,N])
//   A: row-major bf16 matrix (lda) or the implicit im2col of an NHWC bf16 image;
//   B: row-major [N][K] bf16 (conv weights [Cout][KH][KW][Cin], Linear weights [out][in]).
//
// Design (cdna_hip_programming.md sec. 5, "glds vs register staging"):
//   * 512 threads = 8 waves, 2 (M) x 4 (N); block tile 128 x BN (BN = 128 or 64), BK = 64; two
//     workgroups per CU (three for 128x64); 4-wave and 256-row tiles exist for experiments;
//   * operands move HBM -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR round
//     trip), one 1 KiB wave-instruction = 8 LDS rows of 128 B, two-stage ring;
//   * the LDS image is lane-linear, so the bank swizzle is applied to the SOURCE address:
//     LDS slot s of row r holds k-chunk s ^ ((r >> 1) & 7); the fragment reads
//     (ds_read_b128, lane l -> row l&15, chunk 4ks + l>>4) are then conflict-free;
//   * out-of-range rows / k-chunks / conv padding read a 16-byte zero line in HBM instead
//     of being predicated, so every lane always issues its DMA;
//   * im2col: when Cin % 64 == 0 a whole k-tile lies in one filter tap, so (kh, kw, ci0)
//     are block-uniform scalars and each lane only adds its pixel's row offset;
//   * v_mfma_f32_16x16x32_bf16, fp32 accumulation;
//   * epilogue, bf16 output and N % BN == 0 (RL, the default for the conv trunk): the bf16
//     residual tile is LDS-DMA'd into the ring stage the last k-tile leaves free, added in the
//     MFMA accumulator layout via ds_read_b64_tr_b16 with bias and activation, rounded once to
//     bf16 into the other stage, and stored as 16-byte row segments; otherwise the fp32 tile is
//     staged in LDS and the same fusions run on 16-byte row segments.
// Measured limits (profiles/r1_s8_conv_ablation.txt): a 128x128 k-tile takes ~1.27 us per
// workgroup at two per CU, which is both the L2 -> LDS DMA rate of that configuration
// (tools/dma_probe.hip, ~54 GB/s per CU) and its LDS-read + MFMA time.  Variants that did not
// beat it on the ResNet152 shapes: fragment reads hoisted or fully prefetched, persistent tiles
// with a register epilogue, non-temporal epilogue traffic, 16-wave and 4-wave (incl. interleaved)
// tiles, 3- and 4-stage rings, half the waves issuing the DMA, residual rows requested before
// the main loop, start offsets, round-filling M-tiles, a halo-tiled 3x3 kernel, and stream-K
// (2 x CUs workgroups, last-arriver fixups from sc1-published fp32 partials: 30 -> 46 us and
// 53 -> 68 us on the 392-tile L3 shapes).
#include "sat_common.h"

#ifndef SAT_SLAB_WT   // diagnostics builds: 0 = the per-step partial slabs with write-back stores
#define SAT_SLAB_WT 1
#endif
#include "sat_internal.h"

namespace {

constexpr int BK = 64, ROWB = BK * 2;   // 128-byte LDS rows

struct FArgs {
  int M, N, K;
  int a_mlim;              // k-major A: chunks of 8 m's are loaded while m + 8 <= a_mlim (SatGemm::a_tail)
  const bf16* A; long lda;
  const bf16* B; long ldb;
  void* C; long ldc; int c_bf16;
  const float* bias;
  const void* add1; long ld_add1; int add1_bf16;
  int act;
  // implicit im2col (amode 1: Cin % 64 == 0, amode 2: Cin % 8 == 0)
  int amode, H, W, Cin, KW, stride, pad, OH, OW;
  const bf16* zero16;
  int splitk, kchunk;      // atomic split-K (fp32 C, act NONE): blockIdx.z = split
  int xcd_remap;
  int partial; long split_stride;   // partial-output split-K: split s stores plain into C + s*split_stride
  int res_lds;             // fast_gemm_kernel<..., RL = true> epilogue (host-checked shape)
  SatStamps st;                      // in-kernel launch timestamps (SatPolicy::stamps)
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// k-major ("transposed") operand tile: 64 k-rows x 128 elements = 256-B rows, 16-B chunk ch of
// row r stored at slot ch ^ swz(r) (cdna_hip_programming.md T10, image (b)): conflict-free for
// ds_read_b64_tr_b16 fragment reads.
__device__ __forceinline__ int swz256(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// bf16 LDS epilogue images (fast_gemm_kernel RL): residual tile for ds_read_b64_tr_b16 and the
// finished output tile, rows of BN*2 bytes; both conflict-free for their access patterns
template <int BN> __device__ __forceinline__ int res_swz(int r) {
  if constexpr (BN == 128) return swz256(r);
  else return ((r >> 1) & 3) << 1;   // 128-B rows: rows r and r+2 share banks
}
__device__ __forceinline__ int out_swz(int r) { return ((r >> 2) & 3) << 1; }

// MFMA 16x16x32 operand fragment (8 consecutive k of one row x) from a k-major tile:
// two transposing reads of 4 k-rows x 16 columns each.
__device__ __forceinline__ bf16x8 frag_tr(const char* tile, int kbase, int xt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = (xt >> 3) + (p >> 1);
  const int r0 = kbase + 8 * g + q, r1 = r0 + 4;
  const char* a0 = tile + r0 * 256 + 16 * (ch ^ swz256(r0)) + 8 * (p & 1);
  const char* a1 = tile + r1 * 256 + 16 * (ch ^ swz256(r1)) + 8 * (p & 1);
  const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(uintptr_t)(const void*)a0);
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(uintptr_t)(const void*)a1);
  bf16x8 r;
  r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
  r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
  return r;
}
typedef __attribute__((address_space(1))) const void gbl_void;

__device__ __forceinline__ void dma16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_dst, 16, 0, 0);
}
// select the DMA source without control flow (v_cndmask on the address, one DMA per lane)
__device__ __forceinline__ const void* sel(bool ok, const void* p, const void* z) {
  const uintptr_t a = (uintptr_t)p, b = (uintptr_t)z;
  return (const void*)(ok ? a : b);
}

// AT: A stored [K][M] (m-contiguous); BT: B stored [K][N] (n-contiguous).  Transposed operands
// need a 128-wide tile (256-B k-rows) and M, N multiples of 8.
// Wait until at most N of this wave's vector-memory ops are outstanding, then barrier.  Raw
// s_barrier (not __syncthreads, whose fence would drain every in-flight LDS-DMA stage).
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 18) asm volatile("s_waitcnt vmcnt(18)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)\n\ts_barrier" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}

// Tile configurations: BM x BN block tile, WGM x WGN waves (wave tile BM/WGM x BN/WGN).
// RL: bf16 residual + bf16 output epilogue through LDS (128x128 / 128x64 tiles, NS = 2, N % BN == 0): the
// residual tile is DMA'd into the free ring stage during the last k-tile, added in the MFMA
// accumulator layout (ds_read_b64_tr_b16), and the finished bf16 tile is staged for 16-B row stores.
template <int BM, int BN, int WGM, int WGN, bool AT, bool BT, int NS, bool RL = false>
__device__ __forceinline__ void fast_gemm_kernel_body(const FArgs& a) {
  constexpr int NW = WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MI = WTM / 16, NJ = WTN / 16;
  constexpr int STAGE_A = BM * ROWB, STAGE_B = BN * ROWB, STAGE = STAGE_A + STAGE_B;
  constexpr int A_INSTR = AT ? 16 / NW : BM / (8 * NW);   // 1 KiB DMA instructions per wave per stage
  constexpr int B_INSTR = BT ? 16 / NW : BN / (8 * NW);
  static_assert(A_INSTR >= 1 && B_INSTR >= 1 && MI >= 1 && NJ >= 1, "tile/wave mismatch");
  static_assert(!(AT || BT) || (BM == 128 && BN == 128), "k-major operands need 128-wide tiles");
  constexpr int INSTR = A_INSTR + B_INSTR;
  constexpr int EPI_LD = BN + 4;
  constexpr int EPI_BYTES = BM * EPI_LD * 4;
  constexpr int LDS_BYTES = (NS * STAGE > EPI_BYTES) ? NS * STAGE : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  // XCD-aware tile order (cdna_hip_programming.md T1, bijective form): dispatch round-robins
  // consecutive workgroups over the 8 XCDs; give each XCD a contiguous run of row-major tiles so
  // the blocks sharing an A row-panel share one L2.
  int tile = blockIdx.y * gridDim.x + blockIdx.x;
  if (a.xcd_remap) {
    const int nwg = gridDim.x * gridDim.y, q = nwg / 8, r = nwg % 8, x = tile % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
  }
  const int m0 = (tile / gridDim.x) * BM, n0 = (tile % gridDim.x) * BN;
  const int M = a.M, N = a.N;
  const int split = blockIdx.z;
  const int kbeg = split * a.kchunk;
  const int K = min(a.K, kbeg + a.kchunk);

  // ---- per-lane DMA row bookkeeping (rows are fixed across k-tiles) ----
  const int lrow = lane >> 3, slot = lane & 7;
  long a_base[A_INSTR];   // plain: element offset of the row; conv: pixel index (n*H*W) or -1
  int a_ih[A_INSTR], a_iw[A_INSTR], a_chunk[A_INSTR];
#pragma unroll
  for (int j = 0; j < A_INSTR; ++j) {
    const int r = (w * A_INSTR + j) * 8 + lrow;
    a_chunk[j] = slot ^ ((r >> 1) & 7);
    const int row = m0 + r;
    if (a.amode == 0) {
      a_base[j] = row < M ? (long)row * a.lda : -1;
      a_ih[j] = a_iw[j] = 0;
    } else if (row < M) {
      const int ohw = a.OH * a.OW;
      const int n = row / ohw, rem = row - n * ohw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      a_base[j] = (long)n * a.H * a.W;
      a_ih[j] = oh * a.stride - a.pad;
      a_iw[j] = ow * a.stride - a.pad;
    } else {
      a_base[j] = -1; a_ih[j] = a_iw[j] = 0;
    }
  }
  long b_base[B_INSTR];
  int b_chunk[B_INSTR];
#pragma unroll
  for (int j = 0; j < B_INSTR; ++j) {
    const int r = (w * B_INSTR + j) * 8 + lrow;
    b_chunk[j] = slot ^ ((r >> 1) & 7);
    b_base[j] = (n0 + r < N) ? (long)(n0 + r) * a.ldb : -1;
  }

  // k-major operands: lane -> (k-row within the 4-row DMA piece, chunk slot)
  const int trow = lane >> 4, tslot = lane & 15;

  auto stage = [&](int buf, int k0) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + STAGE_A;
    if constexpr (AT) {
#pragma unroll
      for (int j = 0; j < A_INSTR; ++j) {
        const int r = (w * A_INSTR + j) * 4 + trow;       // k-row of the tile
        const int ch = tslot ^ swz256(r);
        const int k = k0 + r, m = m0 + 8 * ch;
        const bool ok = k < K && m + 8 <= a.a_mlim;
        dma16(sel(ok, a.A + (long)k * a.lda + m, a.zero16), sa + (w * A_INSTR + j) * 1024);
      }
    } else if (a.amode == 1) {   // block-uniform filter tap
      const int tap = k0 / a.Cin, ci0 = k0 - tap * a.Cin;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
      for (int j = 0; j < A_INSTR; ++j) {
        const int ih = a_ih[j] + kh, iw = a_iw[j] + kw;
        const bool ok = a_base[j] >= 0 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const void* src = sel(ok, a.A + ((a_base[j] + (long)ih * a.W + iw) * a.Cin + ci0 + 8 * a_chunk[j]), a.zero16);
        dma16(src, sa + (w * A_INSTR + j) * 1024);
      }
    } else if (a.amode == 2) {  // per-lane tap (small Cin, e.g. the padded 3->8 stem)
#pragma unroll
      for (int j = 0; j < A_INSTR; ++j) {
        const int k = k0 + 8 * a_chunk[j];
        bool ok = a_base[j] >= 0 && k < K;
        long off = 0;
        if (ok) {
          const int tap = k / a.Cin, ci = k - tap * a.Cin;
          const int kh = tap / a.KW, kw = tap - kh * a.KW;
          const int ih = a_ih[j] + kh, iw = a_iw[j] + kw;
          ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          off = (a_base[j] + (long)ih * a.W + iw) * a.Cin + ci;
        }
        dma16(sel(ok, a.A + off, a.zero16), sa + (w * A_INSTR + j) * 1024);
      }
    } else {
#pragma unroll
      for (int j = 0; j < A_INSTR; ++j) {
        const int k = k0 + 8 * a_chunk[j];
        const bool ok = a_base[j] >= 0 && k < K;
        dma16(sel(ok, a.A + a_base[j] + k, a.zero16), sa + (w * A_INSTR + j) * 1024);
      }
    }
    if constexpr (BT) {
#pragma unroll
      for (int j = 0; j < B_INSTR; ++j) {
        const int r = (w * B_INSTR + j) * 4 + trow;
        const int ch = tslot ^ swz256(r);
        const int k = k0 + r, n = n0 + 8 * ch;
        const bool ok = k < K && n + 8 <= N;
        dma16(sel(ok, a.B + (long)k * a.ldb + n, a.zero16), sb + (w * B_INSTR + j) * 1024);
      }
    } else {
#pragma unroll
      for (int j = 0; j < B_INSTR; ++j) {
        const int k = k0 + 8 * b_chunk[j];
        const bool ok = b_base[j] >= 0 && k < K;
        dma16(sel(ok, a.B + b_base[j] + k, a.zero16), sb + (w * B_INSTR + j) * 1024);
      }
    }
  };

  // RL: the 128 x BN bf16 residual tile into ring stage buf (rows of BN*2 bytes, 1 KiB per
  // instruction), 16-B chunk ch of row r at slot ch ^ res_swz<BN>(r)
  auto stage_res = [&](int buf) {
    if constexpr (RL) {
      static_assert(BM == 128 && (BN == 128 || BN == 64) && NS == 2, "RL epilogue geometry");
      constexpr int CPR = BN / 8, RPI = 64 / CPR, NINS = BM / RPI;
      if (!a.add1) return;
#pragma unroll
      for (int j = 0; j < NINS / NW; ++j) {
        const int ins = w * (NINS / NW) + j, r = ins * RPI + lane / CPR;
        const int ch = (lane % CPR) ^ res_swz<BN>(r);
        const bool ok = m0 + r < M;
        dma16(sel(ok, (const bf16*)a.add1 + (long)(m0 + r) * a.ld_add1 + n0 + 8 * ch, a.zero16),
              smem + buf * STAGE + ins * 1024);
      }
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fh = lane >> 4;
  auto compute = [&](int buf) {
    const char* sa = smem + buf * STAGE;
    const char* sb = sa + STAGE_A;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (AT) {
          af[i] = frag_tr(sa, ks * 32, wm * WTM + i * 16, lane);
        } else {
          const int r = wm * WTM + i * 16 + fr;
          af[i] = *(const bf16x8*)(sa + r * ROWB + 16 * ((ks * 4 + fh) ^ ((r >> 1) & 7)));
        }
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (BT) {
          bfr[j] = frag_tr(sb, ks * 32, wn * WTN + j * 16, lane);
        } else {
          const int r = wn * WTN + j * 16 + fr;
          bfr[j] = *(const bf16x8*)(sb + r * ROWB + 16 * ((ks * 4 + fh) ^ ((r >> 1) & 7)));
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // NS-stage LDS-DMA ring: NS-1 k-tiles in flight while one is consumed.
  const int nk = K > kbeg ? (K - kbeg + BK - 1) / BK : 0;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) stage(p, kbeg + p * BK);
  for (int kt = 0; kt < nk; ++kt) {
    const int after = min(NS - 2, nk - 1 - kt);   // stages issued after tile kt (uniform)
    if constexpr (NS >= 4) {
      if (after >= 2) wait_vm_barrier<2 * INSTR>();
      else if (after == 1) wait_vm_barrier<INSTR>();
      else wait_vm_barrier<0>();
    } else if constexpr (NS == 3) {
      if (after == 1) wait_vm_barrier<INSTR>();
      else wait_vm_barrier<0>();
    } else {
      wait_vm_barrier<0>();
    }
    if (kt + NS - 1 < nk) stage((kt + NS - 1) % NS, kbeg + (kt + NS - 1) * BK);
    else if (RL && kt == nk - 1) stage_res((kt + 1) % NS);
    compute(kt % NS);
  }
  if constexpr (RL) {
    wait_vm_barrier<0>();   // residual landed, every wave done with the ring
    constexpr int ROWB2 = BN * 2, CPR = BN / 8;
    const char* rs = smem + (nk % NS) * STAGE;          // residual tile
    char* os = smem + ((nk + NS - 1) % NS) * STAGE;     // finished bf16 tile
    const int q = fr >> 2, p = fr & 3;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cl = wn * WTN + j * 16;                 // block column base (tile-local)
      const float bcol = a.bias ? a.bias[n0 + cl + fr] : 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int rb = wm * WTM + i * 16 + 4 * fh;      // this lane group's 4 rows
        const int rq = rb + q, ch = (cl >> 3) + (p >> 1);
        bf16x4 r4 = bf16x4{};
        if (a.add1)
          r4 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(uintptr_t)(const void*)(rs + rq * ROWB2 + 16 * (ch ^ res_swz<BN>(rq)) + 8 * (p & 1)));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = apply_act(acc[i][j][r] + bcol + (float)r4[r], a.act);
          const int row = rb + r, col = cl + fr;
          *(bf16*)(os + row * ROWB2 + 16 * ((col >> 3) ^ out_swz(row)) + 2 * (col & 7)) = (bf16)v;
        }
      }
    }
    __syncthreads();
    const int cc = tid % CPR;
    constexpr int RPP = NW * 64 / CPR;
    const __amdgpu_buffer_rsrc_t rC = sat_out_rsrc(a.C, 2L * M * a.ldc);
#pragma unroll
    for (int it = 0; it < BM / RPP; ++it) {
      const int rl = tid / CPR + it * RPP;
      const int row = m0 + rl;
      const uint4 u = *(const uint4*)(os + rl * ROWB2 + 16 * (cc ^ out_swz(rl)));
      if (row < M) sat_st16(rC, (unsigned)(((long)row * a.ldc + n0 + cc * 8) * 2), u);
    }
  } else {
  __syncthreads();   // every wave done reading the ring before the epilogue reuses the LDS

  if (a.splitk > 1 && !a.partial) {   // atomic split-K: fp32 C, bias in split 0, act NONE (host-checked)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn * WTN + j * 16 + fr;
        if (col >= N) continue;
        const float bcol = (split == 0 && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * WTM + i * 16 + fh * 4 + r;
          if (row < M) atomicAdd((float*)a.C + (long)row * a.ldc + col, acc[i][j][r] + bcol);
        }
      }
    return;
  }
  // ---- epilogue: stage the block's 128 x BN fp32 tile in LDS, then every thread writes
  //      16-byte pieces of full BN-wide row segments (bias, residual, activation, bf16 fused) ----
  float* ep = (float*)smem;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ep[(wm * WTM + i * 16 + fh * 4 + r) * EPI_LD + wn * WTN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  constexpr int CPR = BN / 8;                  // 8-column chunks per tile row
  constexpr int RPP = NW * 64 / CPR;           // rows per pass
  constexpr int ITER = BM / RPP;
  const int tid2 = threadIdx.x;
  const int cc = tid2 % CPR, r0 = tid2 / CPR;
  const int col = n0 + cc * 8;
  const bool vec_ok = (a.ldc % 8 == 0) && (!a.add1 || a.ld_add1 % 8 == 0) && col + 8 <= N;
  void* const Cb = a.partial ? (void*)((float*)a.C + split * a.split_stride) : a.C;
  const float* const bias = (a.partial && split > 0) ? nullptr : a.bias;
  float bias8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias8[e] = (bias && col + e < N) ? bias[col + e] : 0.f;
  if (vec_ok) {
    const __amdgpu_buffer_rsrc_t rCb = sat_out_rsrc(Cb, (a.c_bf16 ? 2L : 4L) * M * a.ldc);
    // all residual loads of this thread go out before the first store
    uint4 res[ITER];
    if (a.add1 && a.add1_bf16) {
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        const int row = m0 + r0 + it * RPP;
        res[it] = row < M ? *(const uint4*)((const bf16*)a.add1 + (long)row * a.ld_add1 + col) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int rl = r0 + it * RPP;
      const int row = m0 + rl;
      if (row >= M) continue;
      float v[8];
      const float4 x0 = *(const float4*)(ep + rl * EPI_LD + cc * 8);
      const float4 x1 = *(const float4*)(ep + rl * EPI_LD + cc * 8 + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias8[e];
      if (a.add1) {
        if (a.add1_bf16) {
          const bf16* h = (const bf16*)&res[it];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)h[e];
        } else {
          const float* p = (const float*)a.add1 + (long)row * a.ld_add1 + col;
          const float4 p0 = *(const float4*)p, p1 = *(const float4*)(p + 4);
          v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w; v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], a.act);
      if (a.c_bf16) {
        uint4 u;
        bf16* h = (bf16*)&u;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
        sat_st16(rCb, (unsigned)(((long)row * a.ldc + col) * 2), u);
      } else {
        // fp32 outputs: the per-step partial slabs (read once by the next launch, on the per-step chain) write
        // through; the batched outputs (x gates, f_h / f_z: re-read by later kernels) stay write-back --
        // write-through for those measured slower (6.45 vs 6.40 ms per step, profiles/r4_s25)
        const unsigned off = (unsigned)(((long)row * a.ldc + col) * 4);
        const uint4 u0 = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
        const uint4 u1 = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7]));
        if (a.partial && SAT_SLAB_WT) {
          sat_st16(rCb, off, u0);
          sat_st16(rCb, off + 16, u1);
        } else {
          sat_st16<0>(rCb, off, u0);
          sat_st16<0>(rCb, off + 16, u1);
        }
      }
    }
  } else if (col < N) {
    for (int it = 0; it < ITER; ++it) {
      const int rl = r0 + it * RPP;
      const int row = m0 + rl;
      if (row >= M) continue;
      for (int e = 0; e < 8 && col + e < N; ++e) {
        float x = ep[rl * EPI_LD + cc * 8 + e] + bias8[e];
        if (a.add1) x += ld_as_f32(a.add1, (long)row * a.ld_add1 + col + e, a.add1_bf16 ? SAT_BF16 : SAT_F32);
        x = apply_act(x, a.act);
        st_from_f32(Cb, (long)row * a.ldc + col + e, a.c_bf16 ? SAT_BF16 : SAT_F32, x);
      }
    }
  }
  }   // !RL
}

template <int BM, int BN, int WGM, int WGN, bool AT, bool BT, int NS, bool RL = false>
__global__ __launch_bounds__(WGM * WGN * 64) void fast_gemm_kernel(FArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  fast_gemm_kernel_body<BM, BN, WGM, WGN, AT, BT, NS, RL>(a);
  sat_stamp_end(a.st, t0);
}

__device__ __attribute__((aligned(16))) bf16 g_zero16[64];

// tile configurations (ids of SatPolicy::gemm_tile)
enum { T_AUTO = 0, T128x128W8 = 1, T128x64W8 = 2, T128x128W4 = 3, T128x256W8 = 4, T256x128W8 = 5 };
inline int tile_bm(int t) { return t == T256x128W8 ? 256 : 128; }
inline int tile_bn(int t) { return t == T128x64W8 ? 64 : t == T128x256W8 ? 256 : 128; }

template <int BM, int BN, int WGM, int WGN, bool AT, bool BT>
void launch_ns(int ns, dim3 grid, hipStream_t s, const FArgs& a) {
  if constexpr (BM == 128 && (BN == 128 || BN == 64) && WGM == 2 && WGN == 4 && !AT && !BT) {
    if (ns == 2 && a.res_lds) {
      hipLaunchKernelGGL((fast_gemm_kernel<128, BN, 2, 4, false, false, 2, true>), grid, dim3(512), 0, s, a);
      return;
    }
  }
  if (ns == 3) hipLaunchKernelGGL((fast_gemm_kernel<BM, BN, WGM, WGN, AT, BT, 3>), grid, dim3(WGM * WGN * 64), 0, s, a);
  else hipLaunchKernelGGL((fast_gemm_kernel<BM, BN, WGM, WGN, AT, BT, 2>), grid, dim3(WGM * WGN * 64), 0, s, a);
}

template <bool AT, bool BT>
void launch_tile(int t, int ns, dim3 grid, hipStream_t s, const FArgs& a) {
  if constexpr (AT || BT) {
    if (t == T128x128W4) launch_ns<128, 128, 2, 2, AT, BT>(ns, grid, s, a);
    else launch_ns<128, 128, 2, 4, AT, BT>(ns, grid, s, a);
  } else {
    switch (t) {
      case T128x64W8: launch_ns<128, 64, 2, 4, false, false>(ns, grid, s, a); break;
      case T128x128W4: launch_ns<128, 128, 2, 2, false, false>(ns, grid, s, a); break;
      case T128x256W8: launch_ns<128, 256, 2, 4, false, false>(2, grid, s, a); break;
      case T256x128W8: launch_ns<256, 128, 4, 2, false, false>(2, grid, s, a); break;
      default: launch_ns<128, 128, 2, 4, false, false>(ns, grid, s, a); break;
    }
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// workgroups the atomic split-K of an fp32-output product aims for (the k-major products split on gemmsplit.hip)
constexpr int kSplitWgs = 320;

}  // namespace

// Returns 1 if the problem was handled by the fast path, 0 if the caller should use the generic kernel.
// the atomic split-K decision of sat_fast_gemm_try for a plain bf16 product with fp32 output (the decoder's
// weight gradients), so a caller can zero several such targets in one launch and set SatGemm::c_zeroed
int sat_gemm_splits_atomically(const SatGemm& g) {
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_F32 || g.act != SAT_ACT_NONE || g.add1 || g.beta != 0.f ||
      g.conv.C > 0 || g.partial_splits > 1 || g.K < 1024)
    return 0;
  const bool tr = g.transA || g.transB;
  const int tcfg = (!tr && g.N <= 64) ? T128x64W8 : T128x128W8;
  const long tiles = (long)sat_cdiv(g.M, tile_bm(tcfg)) * sat_cdiv(g.N, tile_bn(tcfg));
  return tiles < kSplitWgs / 2 ? 1 : 0;
}

int sat_fast_gemm_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  if (g.dtype != SAT_BF16 || g.batch != 1 || g.aux) return 0;
  const SatPolicy& pol = sat_policy();
  const int force_tile = pol.gemm_tile >= T128x128W8 && pol.gemm_tile <= T256x128W8 ? pol.gemm_tile : 0;
  const int force_stages = pol.gemm_stages == 2 || pol.gemm_stages == 3 ? pol.gemm_stages : 0;
  const int res_lds = pol.gemm_epilogue == 1 ? 1 : (pol.gemm_epilogue == 2 ? 0 : 2);
  if (!al16(g.B) || !al16(g.A)) return 0;
  // the epilogues store through a buffer resource (32-bit offsets, sat_out_rsrc's 2 GiB cap): larger outputs take the
  // generic kernel's plain stores
  if ((long)(g.c_dtype == SAT_BF16 ? 2 : 4) * ((long)(g.M - 1) * g.ldc + g.N) >= (1L << 31)) return 0;
  const bool conv = g.conv.C > 0;
  const bool at = g.transA != 0, bt = g.transB != 0;
  if (conv && at) return 0;
  if (at && ((g.M % 8 && !g.a_tail) || g.lda % 8)) return 0;
  if (bt && (g.N % 8 || g.ldb % 8)) return 0;
  // a K tail needs B guarded per k row (k-major B) and A readable to the next 8
  if (!at && ((g.K % 8 && !(g.a_tail && bt && !conv)) || (!conv && g.lda % 8))) return 0;
  if (!bt && (g.K % 8 || g.ldb % 8)) return 0;
  if (g.bias && !al16(g.bias)) return 0;
  if (g.add1 && !al16(g.add1)) return 0;
  const bool partial = g.partial_splits > 1;
  if (partial && (g.c_dtype != SAT_F32 || g.act != SAT_ACT_NONE || g.add1 || g.beta != 0.f || conv)) return 0;
  // skinny partial-split problems (per-step decoder GEMMs): narrow N tiles for more blocks
  // narrow N tiles: skinny N, partial-split problems, and single-k-tile convs (ResNet152 L1 1x1
  // convs with K = 64: three 128x64 workgroups per CU move their epilogue bytes faster, 111 -> 103 us)
  int tcfg = ((g.N <= 64 || partial || (conv && g.K <= BK)) && !at && !bt) ? T128x64W8 : T128x128W8;
  if (force_tile && !partial) tcfg = force_tile;
  if ((at || bt) && tcfg != T128x128W4) tcfg = T128x128W8;
  const int bm = tile_bm(tcfg);
  int bn = tile_bn(tcfg);
  const long tiles = (long)sat_cdiv(g.M, bm) * sat_cdiv(g.N, bn);
  // atomic split-K for weight-gradient-like problems (long K, few tiles, fp32 output)
  int splitk = 1;
  const bool can_split = g.c_dtype == SAT_F32 && g.act == SAT_ACT_NONE && !g.add1 && (g.beta == 0.f || g.beta == 1.f) && !conv;
  if (g.beta != 0.f && !(can_split && g.beta == 1.f)) return 0;
  // workgroups the atomic split-K aims for (split when tiles < half of it)
  const int split_wgs = kSplitWgs;
  if (partial) {
    splitk = 1;
  } else if (tiles < split_wgs / 2) {
    if (can_split && g.K >= 1024) {
      splitk = (int)((split_wgs + tiles - 1) / tiles);
      const int by_k = g.K / 256;
      if (splitk > by_k) splitk = by_k;
      if (splitk > 16) splitk = 16;
      if (splitk < 2) splitk = 1;
    }
    // no split: still the LDS-DMA kernel (the register-staged one is slower per tile); narrow
    // N tiles double the block count of non-transposed problems
    if (splitk == 1 && !at && !bt && !force_tile && tcfg == T128x128W8) {
      tcfg = T128x64W8;
      bn = tile_bn(tcfg);
    }
  } else if (g.beta != 0.f) {
    splitk = 1;   // beta == 1 accumulate through the atomic epilogue with a single split
  }
  static bf16* zero = nullptr;
  if (!zero) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_zero16)) != hipSuccess) return 0;
    zero = (bf16*)p;
  }
  FArgs a{};
  a.M = g.M; a.N = g.N; a.K = g.K;
  a.a_mlim = at && g.a_tail ? sat_cdiv(g.M, 8) * 8 : g.M;
  a.A = (const bf16*)g.A; a.lda = g.lda; a.B = (const bf16*)g.B; a.ldb = g.ldb;
  a.C = g.C; a.ldc = g.ldc; a.c_bf16 = g.c_dtype == SAT_BF16;
  a.bias = g.bias;
  a.add1 = g.add1; a.ld_add1 = g.ld_add1; a.add1_bf16 = g.add1_dtype == SAT_BF16;
  a.act = g.act;
  a.zero16 = zero;
  const bool atomic = splitk > 1 || g.beta != 0.f;
  a.splitk = atomic ? (splitk > 1 ? splitk : 2) : 1;   // the atomic epilogue is selected by splitk > 1
  a.kchunk = g.K;
  if (atomic) {
    const int chunks = splitk > 1 ? splitk : 1;
    a.kchunk = sat_cdiv(sat_cdiv(g.K, chunks), BK) * BK;
    a.splitk = chunks > 1 ? sat_cdiv(g.K, a.kchunk) : 1;
    if (a.splitk == 1) {   // beta == 1, single split: still accumulate atomically
      a.splitk = 2; a.kchunk = sat_cdiv(g.K, BK) * BK;   // split 1 has an empty K range and adds 0
    }
    if (g.beta == 0.f && !g.c_zeroed) {
      SAT_CHECK((hipError_t)sat_zero_rows((float*)g.C, g.ldc, g.M, g.N, s));
    }
  }
  a.partial = partial ? 1 : 0;
  a.split_stride = g.split_stride;
  if (partial) {   // every split writes its slab (an empty K range writes zeros): grid z = splits
    a.splitk = g.partial_splits;
    a.kchunk = sat_cdiv(sat_cdiv(g.K, g.partial_splits), BK) * BK;
  }
  if (conv) {
    if (g.conv.C % 8) return 0;
    a.amode = (g.conv.C % BK == 0) ? 1 : 2;
    a.H = g.conv.H; a.W = g.conv.W; a.Cin = g.conv.C; a.KW = g.conv.KW;
    a.stride = g.conv.stride; a.pad = g.conv.pad; a.OH = g.conv.OH; a.OW = g.conv.OW;
  }
  a.xcd_remap = pol.gemm_linear_order ? 0 : 1;
  a.st = sat_launch_stamps();
  a.res_lds = res_lds && (tcfg == T128x128W8 || tcfg == T128x64W8) && !at && !bt && a.splitk == 1 && !partial &&
              a.c_bf16 && (!g.add1 || (a.add1_bf16 && g.ld_add1 % 8 == 0)) && g.N % bn == 0 && g.ldc % 8 == 0 &&
              al16(g.C) &&
              (g.add1 || res_lds > 1) &&
              (force_stages == 0 || force_stages == 2);
  dim3 grid(sat_cdiv(g.N, bn), sat_cdiv(g.M, bm), a.splitk);
  // skinny partial-split GEMMs run 2-4 k-tiles per block: a 3-deep ring puts the first two in
  // flight at once (their block counts leave LDS occupancy irrelevant)
  const int ns = force_stages ? force_stages : (partial ? 3 : 2);
  if (at && bt) launch_tile<true, true>(tcfg, ns, grid, s, a);
  else if (at) launch_tile<true, false>(tcfg, ns, grid, s, a);
  else if (bt) launch_tile<false, true>(tcfg, ns, grid, s, a);
  else launch_tile<false, false>(tcfg, ns, grid, s, a);
  *err = (int)hipGetLastError();
  return 1;
}
