// 3x3 / stride 1 / pad 1 convolution with an input halo staged once per channel chunk (gfx950).
//
//   C[M,N] = act(conv3x3(X) + bias (+ res)),  X NHWC bf16 with C % 64 == 0, W <= 56,
//   weights [Cout][3][3][Cin] bf16, fp32 accumulation, bf16 output.
//
// The implicit-GEMM kernels (convpipe.hip, convgemm.hip) stage a 256 x 64 (or 128 x 64) A tile per
// k-tile: for a 3x3 conv that is the same input rows nine times, shifted by one pixel per tap, so
// 2/3 of every k-tile's LDS-DMA bytes are A (32 of 48 KiB) and the per-CU DMA rate bounds the loop
// (profiles/r2_s1_pipe_ablation.txt: no-MFMA 30.2 us vs MFMA-only 29.1 us vs both 41.5 us on L3 c2).
// Here the k-loop is channel-chunk-major, tap-minor: per 64-channel chunk the workgroup DMAs the
// input rows its 256 output pixels need under all nine taps ONCE -- flattened pixel range
// [m0 - W - 1, m0 + 256 + W + 1), HR <= 384 rows of 128 B, double-buffered across chunks -- and
// per tap only the 128 x 64 weight tile (16 KiB, 3-stage ring as in convpipe.hip).  A fragments of
// tap (dh, dw) are the halo rows shifted by dh * W + dw; taps that fall into the padding (image
// border, or a flattened neighbour that wraps to another row / image) are zeroed in registers
// from a per-lane 9-bit validity mask.  A-side DMA bytes per chunk drop from 9 x 32 KiB to HR x 128 B.
//   * tile 256 x 128, 8 waves (4 M x 2 N), 64 x 64 per wave, v_mfma_f32_16x16x32_bf16, one workgroup
//     per CU; same mid-tile barrier / fragment double-buffering / counted-vmcnt structure as
//     convpipe.hip (the count now includes the halo DMAs issued after the awaited weight tile);
//   * halo image: 16-B chunk c of LDS row r at slot c ^ (r & 7) -- conflict-free ds_read_b128 for
//     every row shift (checked for all 16 shifts); weights: c ^ ((r >> 1) & 7) as in convpipe.hip;
//   * epilogue identical to convpipe.hip (fp32 tile in LDS, 16-B row segments, residual in fp32,
//     one rounding): the k-order differs (chunk-major), so results match the other kernels to fp32
//     summation order, not bit for bit.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

typedef __attribute__((address_space(3))) void h_lds_void;

constexpr int HBM_ = 256, HBN = 128, HROW = 128;              // 64 channels x 2 B per LDS row
constexpr int H_HRMAX = 384;                                  // halo rows (W <= 56)
constexpr int H_HALO = H_HRMAX * HROW;                        // 48 KiB per halo buffer
constexpr int H_BST = HBN * HROW;                             // 16 KiB weight stage
constexpr int H_EPI_LD = HBN + 4;
constexpr int H_LDS = 2 * H_HALO + 3 * H_BST;                 // 144 KiB
static_assert(HBM_ * H_EPI_LD * 4 <= H_LDS, "epilogue tile must fit");
constexpr unsigned H_OOB = 0x80000000u;

struct HArgs {
  int M, N, Cin, H, W;         // M = NB * H * W output pixels (= input pixels)
  const bf16* X; const bf16* Wt; bf16* C;
  const float* bias;
  const bf16* res;
  int tiles_n, xcd_remap;
  int hr;                      // halo rows per chunk (multiple of 64)
  unsigned x_bytes, w_bytes;
};

template <int N>
__device__ __forceinline__ void h_wait_barrier_n() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else static_assert(N < 0, "unsupported vmcnt");
}
// runtime-uniform count -> literal
__device__ __forceinline__ void h_wait_barrier(int n) {
  switch (n) {
    case 2: h_wait_barrier_n<2>(); break;
    case 4: h_wait_barrier_n<4>(); break;
    case 5: h_wait_barrier_n<5>(); break;
    case 6: h_wait_barrier_n<6>(); break;
    case 7: h_wait_barrier_n<7>(); break;
    case 8: h_wait_barrier_n<8>(); break;
    default: h_wait_barrier_n<0>(); break;
  }
}

template <int ACT, bool RES>
__global__ __launch_bounds__(512) void conv3x3_halo_kernel(HArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[H_LDS];
  char* const halo0 = smem;
  char* const bring = smem + 2 * H_HALO;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  int tile = blockIdx.x;
  if (a.xcd_remap) {   // cdna_hip_programming.md T1, bijective form
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = tile % 8;
    tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
  }
  const int m0 = (tile / a.tiles_n) * HBM_, n0 = (tile % a.tiles_n) * HBN;
  const int M = a.M, N = a.N, W = a.W, Cin = a.Cin, K = 9 * Cin;
  const int nch = Cin / 64, nk = 9 * nch;
  const int hr = a.hr, hd = hr / 64;      // halo DMAs per lane per chunk

  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)a.X, (short)0, (int)a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)a.Wt, (short)0, (int)a.w_bytes, 0x00020000);

  // halo of chunk cc into buffer hb: row r = input pixel q = m0 - W - 1 + r, 64 channels of chunk cc
  const int q0 = m0 - W - 1;
  auto stage_halo = [&](int cc, int hb) {
    char* dst = halo0 + hb * H_HALO;
    for (int d = 0; d < hd; ++d) {   // hd is workgroup-uniform
      const int ins = d * 8 + w;      // 1 KiB = 8 rows per instruction
      const int r = ins * 8 + (lane >> 3), pc = lane & 7, c = pc ^ (r & 7);
      const int q = q0 + r;
      const unsigned off = (q >= 0 && q < M) ? (unsigned)((((long)q * Cin) + cc * 64 + 8 * c) * 2) : H_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (h_lds_void*)(dst + ins * 1024), 16, (int)off, 0, 0, 0);
    }
  };
  // weight tile of k-tile t = (chunk t / 9, tap t % 9) into ring stage s: rows n0 + r, 64 k at tap*Cin + cc*64
  const int b_row0 = w * 16 + (lane >> 3);       // two 8-row pieces per wave: rows w*16 + {0..7, 8..15}
  auto stage_b = [&](int t, int s) {
    const int cc = t / 9, tap = t - cc * 9;
    const int kb = tap * Cin + cc * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = b_row0 + j * 8, pc = lane & 7, c = pc ^ ((r >> 1) & 7);
      const unsigned off = n0 + r < N ? (unsigned)((((long)(n0 + r) * K) + kb + 8 * c) * 2) : H_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (h_lds_void*)(bring + s * H_BST + (w * 2 + j) * 1024), 16,
                                               (int)off, 0, 0, 0);
    }
  };

  // ---- fragments ----
  const int fr = lane & 15, fh = lane >> 4;
  // per-lane tap-validity masks of this lane's 4 output rows (wm*64 + i*16 + fr)
  unsigned vmask[4];
  int hbase[4];   // halo row of the lane's output row under tap (0, 0)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ro = wm * 64 + i * 16 + fr, m = m0 + ro;
    unsigned mk = 0u;
    if (m < M) {
      const int hw = a.H * W, rem = m % hw, h = rem / W, x = rem - h * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dh = t / 3 - 1, dw = t % 3 - 1;
        if ((unsigned)(h + dh) < (unsigned)a.H && (unsigned)(x + dw) < (unsigned)W) mk |= 1u << t;
      }
    }
    vmask[i] = mk;
    hbase[i] = ro + W + 1;
  }
  const int b_rd = (wn * 64 + fr) * HROW;
  const int bsw = (fr >> 1) & 7;   // weight rows wn*64 + j*16 + fr: (r >> 1) & 7 depends on fr only

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[4], xb[4], ya[4], yb[4];
  // fragments of k-tile t (chunk cc in halo buffer hb, weight stage s), 32-deep half ks
  auto frags = [&](int t, int hb, int s, int ks, bf16x8 (&fa)[4], bf16x8 (&fb)[4]) {
    const int tap = t % 9, dh = tap / 3 - 1, dw = tap % 3 - 1;
    const int shift = dh * W + dw;
    const char* hbp = halo0 + hb * H_HALO;
    const int c = ks * 4 + fh;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = hbase[i] + shift;
      bf16x8 v = *(const bf16x8*)(hbp + r * HROW + 16 * (c ^ (r & 7)));
      if (!((vmask[i] >> tap) & 1u)) v = bf16x8{};
      fa[i] = v;
    }
    const char* bp = bring + s * H_BST + b_rd + 16 * (c ^ bsw);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(bp + j * 16 * HROW);
  };
  auto mfma = [&](const bf16x8 (&fa)[4], const bf16x8 (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };

  // prologue: halo of chunk 0, weights of k-tiles 0 and 1 -> wait for halo 0 + weights 0
  stage_halo(0, 0);
  stage_b(0, 0);
  if (nk > 1) {
    stage_b(1, 1);
    h_wait_barrier_n<2>();
  } else {
    h_wait_barrier_n<0>();
  }
  frags(0, 0, 0, 0, xa, xb);
  int s = 0;
  for (int t = 0; t < nk; ++t) {
    const int cc = t / 9, tap = t - cc * 9, hb = cc & 1;
    frags(t, hb, s, 1, ya, yb);
    __builtin_amdgcn_sched_barrier(0);
    // DMAs issued this tile, in order: weights of t+2, then (first tap of a chunk) the next chunk's halo
    int younger = 0;   // DMAs this wave issues after the weight tile t+1 (awaited at this tile's barrier)
    if (t + 2 < nk) {
      stage_b(t + 2, s == 0 ? 2 : s - 1);
      younger += 2;
    }
    if (tap == 0 && cc + 1 < nch) {
      stage_halo(cc + 1, hb ^ 1);
      younger += hd;
    }
    // the halo of chunk cc+1 was issued at tap 0 of chunk cc, i.e. after the weights of k-tile
    // 9cc + 1: while k-tile 9cc + 2's weights (issued at tap 0 too, before it) are awaited (tap 1)
    // it is younger as well
    if (tap == 1 && cc + 1 < nch) younger += hd;
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma(xa, xb);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nk) {
      h_wait_barrier(younger);
      s = s == 2 ? 0 : s + 1;
      frags(t + 1, ((t + 1) / 9) & 1, s, 0, xa, xb);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma(ya, yb);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  h_wait_barrier_n<0>();   // LDS free for the epilogue

  // ---- epilogue (as convpipe.hip): fp32 (acc + bias) tile in LDS, then 16-B row segments ----
  float* ep = (float*)smem;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wn * 64 + j * 16 + fr;
    const float bcol = (a.bias && n0 + cl < N) ? a.bias[n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(wm * 64 + i * 16 + fh * 4 + r) * H_EPI_LD + cl] = acc[i][j][r] + bcol;
  }
  __syncthreads();
  const int cc8 = tid & 15, r0 = tid >> 4;
  const int col = n0 + cc8 * 8;
  if (col < N) {
    uint4 rv[8];
    if constexpr (RES) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = m0 + r0 + it * 32;
        rv[it] = row < M ? *(const uint4*)(a.res + (long)row * N + col) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int rl = r0 + it * 32, row = m0 + rl;
      if (row >= M) continue;
      const float4 x0 = *(const float4*)(ep + rl * H_EPI_LD + cc8 * 8);
      const float4 x1 = *(const float4*)(ep + rl * H_EPI_LD + cc8 * 8 + 4);
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
      *(uint4*)(a.C + (long)row * N + col) = u;
    }
  }
}

int g_halo_mode = 0;   // 0 off (default: slower than convpipe.hip on every ResNet152 shape, profiles/r2_s9_halo_ab.txt), 1 auto, 2 every eligible problem

inline bool hal16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

// Returns 1 if the 3x3 conv was launched by the halo kernel (error code in *err), 0 otherwise.
int sat_conv_halo_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  if (g_halo_mode == 0) return 0;
  const SatConvGeom& cv = g.conv;
  if (cv.C <= 0 || cv.KH != 3 || cv.KW != 3 || cv.stride != 1 || cv.pad != 1 || cv.OH != cv.H || cv.OW != cv.W)
    return 0;
  if (cv.C % 64 || cv.W > 56) return 0;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_BF16 || g.batch != 1 || g.aux || g.transB) return 0;
  if (g.beta != 0.f || g.alpha != 1.f || g.partial_splits > 1) return 0;
  if (g.act != SAT_ACT_NONE && g.act != SAT_ACT_RELU) return 0;
  if (g.N % 8 || g.ldc != g.N || g.ldb != g.K) return 0;
  if (g.add1 && (g.add1_dtype != SAT_BF16 || g.ld_add1 != g.N || !hal16(g.add1))) return 0;
  if (!hal16(g.A) || !hal16(g.B) || !hal16(g.C)) return 0;
  const long x_bytes = 2L * cv.N * cv.H * cv.W * cv.C, w_bytes = 2L * g.N * g.K;
  if (x_bytes >= (1L << 31) || w_bytes >= (1L << 31)) return 0;
  const int hr = sat_cdiv(HBM_ + 2 * cv.W + 2, 64) * 64;
  if (hr > H_HRMAX) return 0;
  const long tiles = (long)sat_cdiv(g.M, HBM_) * sat_cdiv(g.N, HBN);
  if (g_halo_mode == 1 && (tiles < 150 || g.N < 128)) return 0;
  HArgs a{};
  a.M = g.M; a.N = g.N; a.Cin = cv.C; a.H = cv.H; a.W = cv.W;
  a.X = (const bf16*)g.A; a.Wt = (const bf16*)g.B; a.C = (bf16*)g.C;
  a.bias = g.bias; a.res = (const bf16*)g.add1;
  a.tiles_n = sat_cdiv(g.N, HBN);
  a.xcd_remap = 1;
  a.hr = hr;
  a.x_bytes = (unsigned)x_bytes; a.w_bytes = (unsigned)w_bytes;
  const dim3 grid((unsigned)tiles);
  if (g.add1) {
    if (g.act == SAT_ACT_RELU) hipLaunchKernelGGL((conv3x3_halo_kernel<SAT_ACT_RELU, true>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv3x3_halo_kernel<SAT_ACT_NONE, true>), grid, dim3(512), 0, s, a);
  } else {
    if (g.act == SAT_ACT_RELU) hipLaunchKernelGGL((conv3x3_halo_kernel<SAT_ACT_RELU, false>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv3x3_halo_kernel<SAT_ACT_NONE, false>), grid, dim3(512), 0, s, a);
  }
  *err = (int)hipGetLastError();
  return 1;
}

extern "C" int sat_conv_halo_set_mode(int mode) {
  if (mode < 0 || mode > 2) return SAT_ERR_INVALID;
  g_halo_mode = mode;
  return 0;
}
