// Weight-stationary 3x3 convolution for 64 -> 64 channels (gfx950 / MI355X).
//
//   y = act(conv3x3(x, w, stride 1, pad 1) + bias),  x / y NHWC bf16 with C = Cout = 64, fp32 accumulation
//
// Shapes: ResNet152 layer1's c2 (56 x 56, 3 launches per forward) and VGG19's conv1_2 (224 x 224, the
// largest launch of that trunk: 473 GFLOP per 128 images) -- encoder.py:13-17,23-27 through
// torchvision.  On the 128 x 64 implicit-GEMM tile kernel these ran at ~0.2 of the MFMA peak: each
// tile re-fetched its 128 output pixels' input rows once per filter tap (9 x 16 KB of A plus 8 KB of
// weights per 64-deep k-tile) through the CU's ~50 GB/s LDS-DMA intake.  Here:
//   * one persistent 8-wave workgroup per CU (two waves per SIMD: one wave's fragment reads hide
//     behind the other's MFMAs -- with one wave per SIMD the loop ran at a fifth of the MFMA rate,
//     waiting on every ds_read); wave w owns output channels 16 (w % 4) .. +15 of half the item's
//     pixels and keeps the weight fragments of its channels for all K = 9 x 64 in VGPRs for the whole
//     kernel (18 x 16 B per lane), so the only bytes streamed per item are activations;
//   * an item is 224 output pixels (4 image rows of 56, or 2 x 112 of a 224-wide image); its input
//     halo ((rows + 2) x (cols + 2) pixels of 128 B, zero outside the image through out-of-range
//     buffer offsets) lands in LDS ONCE by LDS-DMA and every tap reads it shifted: 45-58 KB per item
//     instead of 9 x 56 KB;
//   * ring of NSTG stages (3 at width 56, 2 at width 224), counted vmcnt across one barrier per item
//     (the previous items' stores stay in flight), as in convstream.hip;
//   * LDS image swizzled on the source: 16-B chunk c of pixel row r at slot c ^ (r & 7), so the 16
//     pixels an MFMA fragment reads under any tap shift hit distinct bank groups;
//   * C^T = W . X^T on v_mfma_f32_16x16x32_bf16: a lane ends with 4 consecutive channels of one pixel;
//     bias, activation and one bf16 rounding, 8-B stores.
// Summation order: k ascending (tap-major, channel within tap) like the tile kernel's k-loop, so the
// fp32 sums differ from it only by the MFMA's internal 32-deep grouping (same instruction, same k
// grouping): results are bit-identical to the tile kernel (tests/test_gpu_parity.py).
#include "sat_common.h"
#include "sat_internal.h"

namespace {

typedef __attribute__((address_space(3))) void w_lds_void;
typedef unsigned __attribute__((ext_vector_type(2))) w_u32x2;

constexpr int WS_NW = 8;                 // waves per workgroup: 4 channel groups x 2 pixel halves
constexpr int WS_NOUT = 64;              // output channels (4 groups of 16)
constexpr int WS_MB = 7;                 // 16-pixel m-blocks per wave (112 of the item's 224 pixels)
constexpr unsigned WS_OOB = 0x80000000u;

struct WArgs {
  const bf16* x; const bf16* w; const float* bias; bf16* y;
  int N, H, W;                           // images, height, width (= output height, width)
  int items, items_per_img, tiles_x;     // items = N * (H / TR) * tiles_x
  unsigned x_bytes, y_bytes;
  SatStamps st;                      // in-kernel launch timestamps (SatPolicy::stamps)
};

template <int N>
__device__ __forceinline__ void w_wait_barrier_n() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// KK x KK window with PADT rows / columns of top-left padding over C input channels (3 / 64 / 1: the
// 3x3 convs; 4 / 16 / 2: ResNet152's stem as a 4x4 conv over the 2x2 space-to-depth input);
// TR x TW output pixels per item (TR * TW = 224); HP halo pixels, DMA rounds of 8 KB (16 B per lane)
template <int KK, int C, int PADT, int TR, int TW, int NSTG, int ACT>
__device__ __forceinline__ void conv_ws_kernel_body(const WArgs& a) {
  static_assert(TR * TW == 2 * WS_MB * 16, "224 pixels per item");
  static_assert(NSTG == 2 || NSTG == 3, "ring depth");
  static_assert(C == 64 || C == 16, "8 or 2 16-B chunks per pixel");
  constexpr int K = KK * KK * C, KSN = K / 32;             // k-steps of 32
  constexpr int CPX = C / 8;                               // 16-B chunks per halo pixel
  constexpr int HW_ = TW + KK - 1, HP = (TR + KK - 1) * HW_;
  constexpr int ROWB = C * 2;                              // bytes per halo pixel
  constexpr int NDMA = (HP * ROWB + WS_NW * 1024 - 1) / (WS_NW * 1024);   // DMA instructions per lane per item
  constexpr int STG = NDMA * WS_NW * 1024;                 // LDS bytes per stage
  static_assert(NSTG * STG <= 160 * 1024, "ring fits in LDS");
  constexpr int ST = WS_MB;                                // 8-B stores per lane per item
  __shared__ __attribute__((aligned(16))) char smem[NSTG * STG];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = w & 3, ph = w >> 2;                      // channel group, pixel half
  const int fr = lane & 15, fh = lane >> 4;

  // weight fragments of this wave's 16 channels for all of K (k = tap * C + ci), loaded once
  bf16x8 bq[KSN];
#pragma unroll
  for (int ks = 0; ks < KSN; ++ks) bq[ks] = *(const bf16x8*)(a.w + (long)(16 * cg + fr) * K + ks * 32 + 8 * fh);
  float bias4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias4[j] = a.bias ? a.bias[16 * cg + 4 * fh + j] : 0.f;
  // consume the weights and biases here: otherwise the compiler's vmcnt tracking still sees them
  // pending inside the item loop and inserts waits that also drain the next items' halo DMAs
#pragma unroll
  for (int ks = 0; ks < KSN; ++ks) asm volatile("" ::"v"(bq[ks]));
#pragma unroll
  for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bias4[j]));

  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, (int)a.y_bytes, 0x00020000);

  auto item_origin = [&](int it, int& n, int& y0, int& x0) {
    n = it / a.items_per_img;
    const int r = it - n * a.items_per_img;
    const int ty = r / a.tiles_x;
    y0 = ty * TR;
    x0 = (r - ty * a.tiles_x) * TW;
  };
  // halo of item `it` into stage `buf`: LDS byte b = (d * NW + w) * 1024 + lane * 16 holds chunk
  // pc = (b % ROWB) / 16 of halo pixel hp = b / ROWB, i.e. logical chunk c = pc ^ (hp & 7) (C = 64;
  // two chunks per pixel at C = 16 need no swizzle)
  auto stage = [&](int it, int buf) {
    int n, y0, x0;
    item_origin(it, n, y0, x0);
    char* st = smem + buf * STG;
#pragma unroll
    for (int d = 0; d < NDMA; ++d) {
      const int byte = (d * WS_NW + w) * 1024 + lane * 16;
      const int hp = byte / ROWB, pc = (byte % ROWB) >> 4, c = CPX == 8 ? pc ^ (hp & 7) : pc;
      const int hy = hp / HW_, hx = hp - hy * HW_;
      const int yy = y0 + hy - PADT, xx = x0 + hx - PADT;
      const bool ok = hp < HP && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      const unsigned off = ok ? (unsigned)(((((long)n * a.H + yy) * a.W + xx) * C + 8 * c) * 2) : WS_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (w_lds_void*)(st + (d * WS_NW + w) * 1024), 16, (int)off, 0, 0, 0);
    }
  };
  // the halo pixel of output pixel i*16 + fr under tap (kh, kw) = hp0[i] + kh * HW_ + kw
  int hp0[WS_MB];
#pragma unroll
  for (int i = 0; i < WS_MB; ++i) {
    const int p = (ph * WS_MB + i) * 16 + fr, py = p / TW, px = p - py * TW;
    hp0[i] = py * HW_ + px;
  }

  int it = blockIdx.x;
  if (it >= a.items) return;   // workgroup-uniform
  const int step = gridDim.x;
  stage(it, 0);
  if (NSTG == 3 && it + step < a.items) stage(it + step, 1);
  int buf = 0;
  for (int k = 0;; ++k) {
    // this item's DMAs have landed once only younger ops remain: (3 stages) the next item's DMAs and
    // the stores of the previous one or two items, (2 stages) the previous item's stores -- they
    // stay in flight across the barrier
    if constexpr (NSTG == 3) {
      const int younger = (it + step < a.items ? NDMA : 0) + (k >= 1 ? ST : 0) + (k >= 2 ? ST : 0);
      switch (younger) {
        case NDMA + 2 * ST: w_wait_barrier_n<NDMA + 2 * ST>(); break;
        case NDMA + ST: w_wait_barrier_n<NDMA + ST>(); break;
        case NDMA: w_wait_barrier_n<NDMA>(); break;
        case 2 * ST: w_wait_barrier_n<2 * ST>(); break;
        case ST: w_wait_barrier_n<ST>(); break;
        default: w_wait_barrier_n<0>(); break;
      }
      if (it + 2 * step < a.items) stage(it + 2 * step, buf == 0 ? 2 : buf - 1);
    } else {
      if (k >= 1) w_wait_barrier_n<ST>();
      else w_wait_barrier_n<0>();
      if (it + step < a.items) stage(it + step, buf ^ 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* base = smem + buf * STG;
    // opaque per item: keeps the 126 per-(m-block, tap) LDS addresses from being hoisted out of the
    // item loop into registers (they are a few VALU ops each, recomputed next to their reads)
#pragma unroll
    for (int i = 0; i < WS_MB; ++i) asm volatile("" : "+v"(hp0[i]));
    f32x4 acc[WS_MB];
#pragma unroll
    for (int i = 0; i < WS_MB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto afrag = [&](int i, int ks) {   // k = ks * 32 + 8 fh: tap k / C, chunk (k % C) / 8
      const int k = ks * 32 + 8 * fh, tap = k / C, c = (k % C) >> 3;
      const int hp = hp0[i] + (tap / KK) * HW_ + tap % KK;
      return *(const bf16x8*)(base + hp * ROWB + 16 * (CPX == 8 ? c ^ (hp & 7) : c));
    };
    bf16x8 af[2][WS_MB];
#pragma unroll
    for (int i = 0; i < WS_MB; ++i) af[0][i] = afrag(i, 0);
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      if (ks + 1 < KSN) {
#pragma unroll
        for (int i = 0; i < WS_MB; ++i) af[(ks + 1) & 1][i] = afrag(i, ks + 1);
      }
#pragma unroll
      for (int i = 0; i < WS_MB; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks], af[ks & 1][i], acc[i], 0, 0, 0);
    }
    // epilogue: lane holds channels 16 cg + 4fh .. +3 of output pixel (ph * 7 + i) * 16 + fr
    int n, y0, x0;
    item_origin(it, n, y0, x0);
    auto out_at = [&](int i, unsigned& off) {   // bias + act of m-block i, rounded once; its byte offset
      const int p = (ph * WS_MB + i) * 16 + fr, py = p / TW, px = p - py * TW;
      w_u32x2 o;
      bf16* ob = (bf16*)&o;
#pragma unroll
      for (int j = 0; j < 4; ++j) ob[j] = (bf16)apply_act(acc[i][j] + bias4[j], ACT);
      off = (unsigned)(((((long)n * a.H + y0 + py) * a.W + x0 + px) * WS_NOUT + 16 * cg + 4 * fh) * 2);
      return o;
    };
    // m-block pairs through 16-B stores (sat_common.h, sat_st_pair16), an odd last one with 8 B; plain write-back
    // here: write-through stores of the stem / layer1 outputs measured slower (6.28-6.31 vs 6.38-6.40 ms per step,
    // profiles/r4_s19)
#pragma unroll
    for (int i = 0; i + 1 < WS_MB; i += 2) {
      unsigned offA, offB;
      const w_u32x2 oa = out_at(i, offA), ob2 = out_at(i + 1, offB);
      sat_st_pair16<0>(rY, offA, offB, oa, ob2, true, true);
    }
    if constexpr (WS_MB % 2) {
      unsigned off;
      const w_u32x2 o = out_at(WS_MB - 1, off);
      __builtin_amdgcn_raw_buffer_store_b64(o, rY, (int)off, 0, 0);
    }
    it += step;
    if (it >= a.items) break;
    buf = NSTG == 3 ? (buf == 2 ? 0 : buf + 1) : buf ^ 1;
  }
}

template <int KK, int C, int PADT, int TR, int TW, int NSTG, int ACT>
__global__ __launch_bounds__(WS_NW * 64) void conv_ws_kernel(WArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  conv_ws_kernel_body<KK, C, PADT, TR, TW, NSTG, ACT>(a);
  sat_stamp_end(a.st, t0);
}

int g_ws_cus = 0;    // CU count (queried once)

inline bool wal16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int KK, int C, int PADT, int TR, int TW, int NSTG>
void launch_ws(int act, dim3 grid, hipStream_t s, const WArgs& a) {
  if (act == SAT_ACT_RELU)
    hipLaunchKernelGGL((conv_ws_kernel<KK, C, PADT, TR, TW, NSTG, SAT_ACT_RELU>), grid, dim3(WS_NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((conv_ws_kernel<KK, C, PADT, TR, TW, NSTG, SAT_ACT_NONE>), grid, dim3(WS_NW * 64), 0, s, a);
}

}  // namespace

// Returns 1 if the conv was launched by the weight-stationary kernel (3x3 / pad 1 over 64 channels at
// width 56 or 224; the 4x4 / top-left-pad-2 stem over the 16-channel space-to-depth input at width
// 112), 0 otherwise.
int sat_conv3x3_ws_try(const SatGemm& g, hipStream_t s, int* err) {
  *err = 0;
  if (sat_policy().conv3x3_ws == 1) return 0;
  const SatConvGeom& cv = g.conv;
  const bool c3 = cv.C == 64 && cv.KH == 3 && cv.KW == 3 && cv.pad == 1 && (cv.W == 56 || cv.W == 224);
  const bool stem = cv.C == 16 && cv.KH == 4 && cv.KW == 4 && cv.pad == 2 && cv.W == 112;
  if (!(c3 || stem) || g.N != WS_NOUT || cv.stride != 1 || cv.OH != cv.H || cv.OW != cv.W) return 0;
  if (g.dtype != SAT_BF16 || g.c_dtype != SAT_BF16 || g.batch != 1 || g.aux || g.transB || g.add1) return 0;
  if (g.beta != 0.f || g.alpha != 1.f || g.partial_splits > 1) return 0;
  if (g.act != SAT_ACT_NONE && g.act != SAT_ACT_RELU) return 0;
  if (g.ldb != cv.KH * cv.KW * cv.C || g.ldc != WS_NOUT) return 0;
  if (!wal16(g.A) || !wal16(g.B) || !wal16(g.C) || (g.bias && !wal16(g.bias))) return 0;
  const int TR = cv.W == 56 ? 4 : 2, TW = cv.W == 56 ? 56 : 112;
  if (cv.H % TR) return 0;
  const long xb = 2L * cv.N * cv.H * cv.W * cv.C, yb = 2L * cv.N * cv.H * cv.W * WS_NOUT;
  if (xb >= (1L << 31) || yb >= (1L << 31)) return 0;
  if (g_ws_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return 0;
    g_ws_cus = n;
  }
  WArgs a{};
  a.x = (const bf16*)g.A; a.w = (const bf16*)g.B; a.bias = g.bias; a.y = (bf16*)g.C;
  a.N = cv.N; a.H = cv.H; a.W = cv.W;
  a.tiles_x = cv.W / TW;
  a.items_per_img = (cv.H / TR) * a.tiles_x;
  a.items = cv.N * a.items_per_img;
  a.x_bytes = (unsigned)xb; a.y_bytes = (unsigned)yb;
  a.st = sat_launch_stamps();
  // the stem variant (72 KB of LDS, 108 VGPRs) fits two workgroups per CU
  const int slots = g_ws_cus * (stem ? 2 : 1);
  const int grid = a.items < slots ? a.items : slots;
  if (stem) launch_ws<4, 16, 2, 2, 112, 3>(g.act, dim3(grid), s, a);
  else if (cv.W == 56) launch_ws<3, 64, 1, 4, 56, 3>(g.act, dim3(grid), s, a);
  else launch_ws<3, 64, 1, 2, 112, 2>(g.act, dim3(grid), s, a);
  *err = (int)hipGetLastError();
  return 1;
}
