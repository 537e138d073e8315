// Fused ResNet bottleneck block (identity residual, stride 1) for gfx950 / MI355X.
//
//   y = relu(c3(relu(c2(relu(c1(x))))) + x)        c1 1x1 Cin->Cmid, c2 3x3/pad 1 Cmid->Cmid,
//                                                  c3 1x1 Cmid->Cin, eval-BN folded into each conv
// (torchvision Bottleneck.forward as the reference's encoder runs it, encoder.py:13-17,33-36.)
//
// Why: ResNet152's layer3 has 35 such blocks at 14 x 14 x 1024 (mid 256).  As three conv launches
// each (convpipe.hip / convstream.hip) a block took ~90 us in the trunk graph: two intermediate
// activations went through HBM, every launch paid its own prologue / epilogue / launch gap, and the
// 196 tiles of 256 x 128 left 60 of 256 CUs idle.  Here one launch runs the whole block:
//   * one workgroup per half image (RO = 7 output rows = 98 pixels): 256 workgroups for B = 128;
//     c1 is computed for the 8 image rows c2 needs (its one-row halo), c1 and c2 outputs never
//     leave LDS (X1: c1 rows + a zero row, X2: c2 rows, both bf16 in 64-channel planes of 128-B
//     rows, 16-B chunk c of row r at slot c ^ (r & 7): conflict-free ds_read_b128 for every 3x3
//     row shift, as in convhalo.hip);
//   * 8 waves, each owning 32 output channels of the current 256-wide phase (n-blocks 2w, 2w+1) and
//     all 7 16-row m-blocks; MFMA v_mfma_f32_16x16x32_bf16 computes C^T = W . X^T, so a lane holds
//     4 consecutive channels of one pixel: epilogues write 8-byte pieces (X1 / X2 / global) without
//     a transpose;
//   * weights never touch LDS: they are pre-permuted once (sat_mfma_frag_layout) so that every
//     16-B-per-lane fragment load of a wave is 1 KiB contiguous, and each wave streams its own
//     n-blocks straight into VGPRs two k-tiles ahead (three register buffers); the compiler's own
//     vmcnt tracking orders them;
//   * c1's input rows are the only LDS-DMA stream (3-stage ring aliasing X2, counted vmcnt + one raw
//     barrier per k-tile); c2 reads its A operand from X1 with a per-lane row shift per filter tap
//     (taps in the image padding read the zero row), c3 from X2: neither needs a barrier per k-tile;
//   * the whole 68-k-tile schedule (c1 16, c2 36, c3 4 x 4) is unrolled at compile time, so register
//     buffers are static and the weight prefetch runs across phase boundaries.
// Arithmetic: each conv sums its K in the same order as the unfused kernels (k-tiles ascending, c2
// tap-major), adds the folded bias in fp32, applies ReLU and rounds to bf16 once; c3 adds the residual
// in fp32 before the ReLU -- bit-identical to the three-launch path (tests/test_gpu_parity.py).
#include "sat_common.h"
#include "sat_internal.h"

#include <utility>

#ifndef SAT_C2_ABL
#define SAT_C2_ABL 0
#endif

namespace {

typedef __attribute__((address_space(3))) void k_lds_void;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr unsigned K_OOB = 0x80000000u;

// compile-time loop: f(std::integral_constant<int, T>) for T = 0 .. N-1 (register arrays indexed by
// T stay static, every wait count is a literal)
template <typename F, int... Ts>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Ts...>) {
  (f(std::integral_constant<int, Ts>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

struct KArgs {
  const bf16* x;      // [N][IH][IW][CIN]
  const bf16* w1;     // fragment layout of [CMID][CIN]
  const bf16* w2;     // fragment layout of [CMID][9][CMID]
  const bf16* w3;     // fragment layout of [CIN][CMID]
  const float* b1; const float* b2; const float* b3;
  bf16* y;            // [N][IH][IW][CIN]
  unsigned x_bytes;
  SatStamps st;                      // in-kernel launch timestamps (SatPolicy::stamps)
};

template <int N>
__device__ __forceinline__ void k_wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
__device__ __forceinline__ void k_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// vmem instructions one wave issues after its input DMAs A(T) (na instructions) and before the wait
// of c1 k-tile T: the issue order is A0 B0 A1 B1 B2 .. B(PF-1) (B = nb weight loads), then per k-tile
// it, after its wait: A(it+2) (it+2 < KT1), B(it+PF) (it+PF < NT, when weights stream)
constexpr int younger_than_a(int T, int KT1, int NT, int PF, bool stream, int nb = 4, int na = 2) {
  int n = 0;
  bool after = false;
  auto ev_a = [&](int idx) {
    if (after) n += na;
    if (idx == T) after = true;
  };
  auto ev_b = [&]() {
    if (after) n += nb;
  };
  ev_a(0); ev_b(); ev_a(1); ev_b();
  for (int e = 2; e < PF; ++e) ev_b();
  for (int it = 0; it < T; ++it) {
    if (it + 2 < KT1) ev_a(it + 2);
    if (stream && it + PF < NT) ev_b();
  }
  return n;
}

// the same count for a ring whose input DMAs run `da` k-tiles ahead: prologue A0 B0 A1 B1 .. (A(e) for e < da, B(e)
// for e < PF, interleaved), then per k-tile after its wait A(it + da) (< KT1), B(it + PF) (< NT, when weights stream)
constexpr int younger_than_a_da(int T, int KT1, int NT, int PF, int da, int nb, int na) {
  int n = 0;
  bool after = false;
  auto ev_a = [&](int idx) {
    if (after) n += na;
    if (idx == T) after = true;
  };
  auto ev_b = [&]() {
    if (after) n += nb;
  };
  for (int e = 0; e < (da > PF ? da : PF); ++e) {
    if (e < da) ev_a(e);
    if (e < PF) ev_b();
  }
  for (int it = 0; it < T; ++it) {
    if (it + da < KT1) ev_a(it + da);
    if (it + PF < NT) ev_b();
  }
  return n;
}

// IW: image width = height, RO: output image rows per workgroup (IW % RO == 0, IW / RO == 2),
// CIN: block input/output channels, CMID: bottleneck width (256: one 256-wide phase per conv);
// PF: weight prefetch distance in k-tiles; ABL (diagnostics, tools/block_ab.py): bit 0 no MFMA,
// bit 1 no weight streaming (the prologue's fragments reused), bit 2 no A fragment reads; bit 3
// non-temporal input / residual loads, bit 4 non-temporal output stores (both measured slower:
// 65.6 -> 77.9 / 101.8 us, profiles/r2_s25_block_nt.txt); bit 5 per-workgroup rotation of the waves'
// n-blocks, bit 6 k-major fragment layout; bit 7 the co-residency variant (one LDS activation image,
// <= 168 VGPRs: bottleneck_kernel_share)
// bias + ReLU of one C^T accumulator (4 consecutive channels of one pixel), rounded once to bf16
__device__ __forceinline__ u32x2 relu_bf16x4(const f32x4& a, const float4& b) {
  u32x2 o;
  bf16* ob = (bf16*)&o;
  ob[0] = (bf16)fmaxf(a[0] + b.x, 0.f);
  ob[1] = (bf16)fmaxf(a[1] + b.y, 0.f);
  ob[2] = (bf16)fmaxf(a[2] + b.z, 0.f);
  ob[3] = (bf16)fmaxf(a[3] + b.w, 0.f);
  return o;
}
#ifndef SAT_C2_PF   // the half-image 3x3 kernel's weight prefetch distance in k-tiles: 3 since its input staging
#define SAT_C2_PF 3   // moved to LDS-DMA (227 VGPRs); step 6.294-6.317 -> 6.273 ms, 4: 6.287-6.293 (profiles/r5_s38, r5_s39)
#endif
#ifndef SAT_SL2_PF   // diagnostics builds: the two-slice 3x3 kernel's weight prefetch distance in k-tiles
#define SAT_SL2_PF 2
#endif
#ifndef SAT_C1_DA   // diagnostics builds: the half-image 1x1 kernel's input DMAs this many k-tiles ahead
#define SAT_C1_DA 2
#endif
#ifndef SAT_C1_PF   // diagnostics builds: the half-image 1x1 kernel's weight prefetch distance in k-tiles
#define SAT_C1_PF 2
#endif
// Weight-stream rotation (XCD-aware): the workgroups that share an XCD's L2 (blockIdx.x % 8 under round-robin
// placement) start their waves on different channel groups, so at any moment they fetch different weight lines
// instead of all hammering the same L2 channel: layer3 c2 29.2 -> 26.8 us per launch (profiles/r5_s60).
// SAT_C2_ROT (layer3 c2): 1 rotate by blockIdx.x / 8, 2 by blockIdx.x, 0 off; SAT_WROT: the band and 1x1 forms.
#ifndef SAT_C2_ROT
#define SAT_C2_ROT 1
#endif
#ifndef SAT_WROT
#define SAT_WROT 1
#endif
#ifndef SAT_PAIR_STORES   // diagnostics builds: 0 = the 8-B stores of each lane's own accumulators
#define SAT_PAIR_STORES 1
#endif

template <int IW, int RO, int CIN, int CMID, int PF, int ABL>
__device__ __forceinline__ void bottleneck_body(const KArgs& a) {
  const __amdgpu_buffer_rsrc_t rY = sat_out_rsrc(a.y, 0x7fffffffL);   // output stores (sat_common.h policy)
  static_assert(IW / RO == 2 && IW % RO == 0, "two workgroups per image");
  static_assert(CMID == 256 && CIN % 256 == 0 && CIN % 64 == 0, "256-wide phases");
  constexpr int IH = IW;
  constexpr int PO = RO * IW;                    // output pixels per workgroup (98)
  constexpr int R1 = RO + 1;                     // c1 image rows (one halo row)
  constexpr int P1 = R1 * IW;                    // c1 pixels (112)
  constexpr int MB1 = (P1 + 15) / 16, MB2 = (PO + 15) / 16;
  static_assert(MB1 == 7 && MB2 == 7, "7 m-blocks per phase");
  constexpr int MB = 7;
  constexpr int ROWB = 128;                      // 64 channels per LDS row
  constexpr int X1ROWS = P1 + 1;                 // + zero row
  constexpr int X1PL = X1ROWS * ROWB;            // X1 plane bytes
  constexpr int X2PL = MB2 * 16 * ROWB;          // X2 plane bytes
  constexpr int NPL = CMID / 64;
  // SHARE (ABL bit 7, the co-residency variant): one activation image -- c2's output overwrites c1's
  // after a barrier, and c1's input ring lives there too before c1's epilogue: 57 KB of LDS instead
  // of 113 KB, so decoder workgroups can share the CU
  constexpr bool SHARE = (ABL & 128) != 0;
  constexpr int X1 = 0, X2 = SHARE ? 0 : NPL * X1PL;   // LDS regions
  constexpr int X2P = SHARE ? X1PL : X2PL;             // X2 plane stride
  constexpr int RING = SHARE ? 0 : X2;                 // c1 input ring
  constexpr int STG = 128 * ROWB;                // 128 rows x 64 channels per stage
  static_assert(3 * STG <= NPL * (SHARE ? X1PL : X2PL), "ring fits");
  // SHARE keeps the three folded biases in LDS (read at each epilogue) instead of 16 VGPRs
  constexpr int SB = NPL * X1PL, NBIAS = 2 * CMID + CIN;
  constexpr int LDS = SHARE ? SB + NBIAS * 4 : X2 + NPL * X2PL;
  constexpr int KT1 = CIN / 64, KT2 = 9 * CMID / 64, NCK = CIN / 256, KT3C = CMID / 64;
  constexpr int NT = KT1 + KT2 + NCK * KT3C;
  constexpr int KS1 = CIN / 32, KS2 = 9 * CMID / 32, KS3 = CMID / 32;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  // the wave's 32 output channels of each phase: n-blocks 2wn, 2wn+1 (wn rotated per workgroup in the
  // bit-5 experiment so the workgroups of one XCD do not request the same weight lines together)
  const int wn = (ABL & 32) ? __builtin_amdgcn_readfirstlane((w + (blockIdx.x >> 3)) & 7) : w;
  const int img = blockIdx.x >> 1, half = blockIdx.x & 1;
  const int y0 = half * RO;                      // first output image row
  const int ws = half ? IH - R1 : 0;             // first c1 image row
  const long pix_img = (long)img * IH * IW;

  // ---- zero row of every X1 plane (taps in the padding read it; SHARE: written after the ring's use) ----
  auto zero_row = [&]() {
    if (tid < NPL * 8) *(uint4*)(smem + X1 + (tid >> 3) * X1PL + P1 * ROWB + (tid & 7) * 16) = make_uint4(0, 0, 0, 0);
  };
  if constexpr (!SHARE) zero_row();

  // ---- c1 input ring: k-tile t = channels 64t.., 128 rows (rows >= P1 read zeros) ----
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);
  unsigned dsrc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int d = w * 2 + u, r = d * 8 + (lane >> 3), c = (lane & 7) ^ (lane >> 3);
    dsrc[u] = r < P1 ? (unsigned)(((pix_img + (long)ws * IW + r) * CIN + 8 * c) * 2) : K_OOB;
  }
  auto dma_a = [&](int t) {
    char* st = smem + RING + (t % 3) * STG;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (k_lds_void*)(st + (w * 2 + u) * 1024), 16,
                                               dsrc[u] == K_OOB ? (int)K_OOB : (int)(dsrc[u] + t * 128), 0, 0,
                                               (ABL & 8) ? 2 : 0);
  };

  // ---- weight fragments: tile T of the 68-tile schedule, this wave's n-blocks, both 32-k halves ----
  bf16x8 bq[PF + 1][2][2];
  auto load_b = [&](int T, bf16x8 (&dst)[2][2]) {
    const bf16* base;
    int nb0, ks0, KS, NBW;
    if (T < KT1) { base = a.w1; nb0 = 0; ks0 = 2 * T; KS = KS1; NBW = CMID / 16; }
    else if (T < KT1 + KT2) { base = a.w2; nb0 = 0; ks0 = 2 * (T - KT1); KS = KS2; NBW = CMID / 16; }
    else { const int t = T - KT1 - KT2; base = a.w3; nb0 = (t / KT3C) * 16; ks0 = 2 * (t % KT3C); KS = KS3; NBW = CIN / 16; }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        dst[ks][j] = (ABL & 64)   // k-major fragment layout: block (nb, ks) at ks * NB + nb
                         ? *(const bf16x8*)(base + ((long)((ks0 + ks) * NBW + nb0 + wn * 2 + j) * 64 + lane) * 8)
                         : *(const bf16x8*)(base + ((long)((nb0 + wn * 2 + j) * KS + ks0 + ks) * 64 + lane) * 8);
  };

  // ---- A fragment offsets: row i*16 + fr of a 128-B-row image = i * 2048 (immediate) + per-lane part ----
  int offu[2];   // unshifted rows (c1 ring, X2)
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) offu[ks] = fr * ROWB + 16 * ((ks * 4 + fh) ^ (fr & 7));
  // c2: output pixel p = i*16 + fr reads X1 row p + (y0 - ws) * IW + dh * IW + dw under tap (dh, dw),
  // or the zero row P1 where the tap falls into the image padding (or p >= PO)
  int offs[MB][2];
  auto tap_offsets = [&](int tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int p = i * 16 + fr, py = p / IW, pxx = p - py * IW;
      const bool ok = p < PO && (unsigned)(y0 + py + dh) < (unsigned)IH && (unsigned)(pxx + dw) < (unsigned)IW;
      const int q = ok ? p + (y0 - ws + dh) * IW + dw : P1;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) offs[i][ks] = q * ROWB + 16 * ((ks * 4 + fh) ^ (q & 7));
    }
  };

  f32x4 acc[MB][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // fragments + MFMAs of one 64-deep k-tile; A row block i at base + i * 16 * ROWB + offu (unshifted)
  // or base + offs[i] (c2's shifted rows)
  auto mma = [&](const bf16x8 (&af)[2][MB], const bf16x8 (&b)[2][2]) {
    if constexpr (ABL & 1) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < MB; ++i) asm volatile("" ::"v"(af[ks][i]));
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(b[ks][j]));
      }
      return;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // SHARE: one 32-deep half's fragments at a time (28 instead of 56 VGPRs)
  auto mma_half = [&](int ks, const bf16x8 (&af)[MB], const bf16x8 (&b)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto tile_u = [&](const char* base, const bf16x8 (&b)[2][2]) {
    if constexpr (SHARE) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[MB];
#pragma unroll
        for (int i = 0; i < MB; ++i) af[i] = *(const bf16x8*)(base + i * 16 * ROWB + offu[ks]);
        mma_half(ks, af, b);
      }
      return;
    }
    bf16x8 af[2][MB];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i)
        af[ks][i] = (ABL & 4) ? b[ks][i & 1] : *(const bf16x8*)(base + i * 16 * ROWB + offu[ks]);
    mma(af, b);
  };
  auto tile_s = [&](const char* base, const bf16x8 (&b)[2][2]) {
    if constexpr (SHARE) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[MB];
#pragma unroll
        for (int i = 0; i < MB; ++i) af[i] = *(const bf16x8*)(base + offs[i][ks]);
        mma_half(ks, af, b);
      }
      return;
    }
    bf16x8 af[2][MB];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i) af[ks][i] = (ABL & 4) ? b[ks][i & 1] : *(const bf16x8*)(base + offs[i][ks]);
    mma(af, b);
  };
  // epilogue into an LDS plane image: lane holds channels w*32 + j*16 + 4fh .. +3 of pixel i*16 + fr
  // bias values of the lane's channels, loaded well before their epilogue (a load issued at the
  // epilogue would be younger than the weight prefetches and drain them)
  auto load_bias = [&](const float* bias, int ch0, float4 (&bv)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) bv[j] = *(const float4*)(bias + ch0 + wn * 32 + j * 16 + 4 * fh);
  };
  auto lds_bias = [&](int ch0, float4 (&bv)[2]) {   // SHARE: bias values from the LDS copy
#pragma unroll
    for (int j = 0; j < 2; ++j) bv[j] = *(const float4*)(smem + SB + 4 * (ch0 + wn * 32 + j * 16 + 4 * fh));
  };
  auto store_planes = [&](int region, int plane_bytes, const float4 (&bias)[2]) {
    const int plane = wn >> 1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float4 bv = bias[j];
      const int c = (wn & 1) * 4 + j * 2 + (fh >> 1);
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int r = i * 16 + fr;
        u32x2 o;
        bf16* ob = (bf16*)&o;
        ob[0] = (bf16)fmaxf(acc[i][j][0] + bv.x, 0.f);
        ob[1] = (bf16)fmaxf(acc[i][j][1] + bv.y, 0.f);
        ob[2] = (bf16)fmaxf(acc[i][j][2] + bv.z, 0.f);
        ob[3] = (bf16)fmaxf(acc[i][j][3] + bv.w, 0.f);
        *(u32x2*)(smem + region + plane * plane_bytes + r * ROWB + 16 * (c ^ (r & 7)) + 8 * (fh & 1)) = o;
      }
    }
  };

  // ---- prologue ----
  float4 bias_a[2], bias_b[2];
  if constexpr (SHARE) {   // visible after c1's first barrier
    float* sb = (float*)(smem + SB);
    for (int k = tid; k < NBIAS; k += 512) sb[k] = k < CMID ? a.b1[k] : (k < 2 * CMID ? a.b2[k - CMID] : a.b3[k - 2 * CMID]);
  } else {
    load_bias(a.b1, 0, bias_a);
  }
  dma_a(0);
  load_b(0, bq[0]);
  dma_a(1);
  load_b(1, bq[1]);
  static_for<PF - 2>([&](auto e) { load_b(2 + decltype(e)::value, bq[2 + decltype(e)::value]); });
  zero_acc();
  u32x2 resv[MB][2];

  static_for<NT>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value;
    if constexpr (T < KT1) {
      // this wave's DMAs of input tile T have landed; younger: B(T), [A(T+1)], B(T+1)
      k_wait_barrier<younger_than_a(T, KT1, NT, PF, !(ABL & 2))>();
      if constexpr (T + 2 < KT1) dma_a(T + 2);
    }
    if constexpr (T + PF < NT && !(ABL & 2)) load_b(T + PF, bq[(T + PF) % (PF + 1)]);
    constexpr int BQ = (ABL & 2) ? 0 : T % (PF + 1);
    if constexpr (T < KT1) {
      tile_u(smem + RING + (T % 3) * STG, bq[BQ]);
      if constexpr (T == KT1 - 1) {   // c1 epilogue -> X1 (the ring is read for the last time above)
        if constexpr (SHARE) k_lds_barrier();   // every wave's last ring reads retired before X1 overwrites it
        if constexpr (SHARE) lds_bias(0, bias_a);
        store_planes(X1, X1PL, bias_a);
        if constexpr (SHARE) zero_row();
        zero_acc();
        k_lds_barrier();
      }
    } else if constexpr (T < KT1 + KT2) {
      constexpr int t = T - KT1, tap = t / (CMID / 64), pl = t % (CMID / 64);
      if constexpr (t == 0 && !SHARE) load_bias(a.b2, 0, bias_b);
      if constexpr (pl == 0) tap_offsets(tap);
      tile_s(smem + X1 + pl * X1PL, bq[BQ]);
      if constexpr (t == KT2 - 1) {   // c2 epilogue -> X2
        if constexpr (SHARE) k_lds_barrier();   // every wave's c2 reads of X1 retired before X2 overwrites it
        if constexpr (SHARE) lds_bias(CMID, bias_b);
        store_planes(X2, X2P, bias_b);
        zero_acc();
        k_lds_barrier();
      }
    } else {
      constexpr int t = T - KT1 - KT2, ck = t / KT3C, kt = t % KT3C;
      if constexpr (kt == (SHARE ? KT3C - 1 : 0)) {   // residual rows + bias of this chunk, for its epilogue
        if constexpr (!SHARE) load_bias(a.b3, ck * 256, bias_a);
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {   // rows past PO load a valid row (never stored): no branch
            const int p = min(i * 16 + fr, PO - 1), ch = ck * 256 + wn * 32 + j * 16 + 4 * fh;
            const u32x2* rp = (const u32x2*)(a.x + (pix_img + (long)y0 * IW + p) * CIN + ch);
            if constexpr (ABL & 8) resv[i][j] = __builtin_nontemporal_load(rp);
            else resv[i][j] = *rp;
          }
      }
      tile_u(smem + X2 + kt * X2P, bq[BQ]);
      if constexpr (kt == KT3C - 1) {   // c3 epilogue: bias, fp32 residual add, ReLU, one rounding, 8-B stores
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ch = ck * 256 + wn * 32 + j * 16 + 4 * fh;
          if constexpr (SHARE) {
            if (j == 0) lds_bias(2 * CMID + ck * 256, bias_a);
          }
          const float4 bv = bias_a[j];
#pragma unroll
          for (int i = 0; i < MB; ++i) {
            const int p = i * 16 + fr;
            const bf16* rh = (const bf16*)&resv[i][j];
            float v[4] = {acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w};
            u32x2 o;
            bf16* ob = (bf16*)&o;
#pragma unroll
            for (int e = 0; e < 4; ++e) ob[e] = (bf16)fmaxf(v[e] + (float)rh[e], 0.f);
            u32x2* yp = (u32x2*)(a.y + (pix_img + (long)y0 * IW + p) * CIN + ch);
            if constexpr (ABL & 16) {
              if (p < PO) __builtin_nontemporal_store(o, yp);
            } else {
              if (p < PO) sat_st8(rY, (unsigned)((char*)yp - (char*)a.y), o);
            }
          }
        }
        zero_acc();
      }
    }
  });
}

template <int PF, int ABL>
__global__ __launch_bounds__(512) void bottleneck_kernel(KArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  bottleneck_body<14, 7, 1024, 256, PF, ABL>(a);
  sat_stamp_end(a.st, t0);
}

// The fused block for ResNet152's layer2 identity bottlenecks (28 x 28, 512 -> 128 -> 128 -> 512): one
// workgroup per band of RO = 7 output rows (four per image, 512 for B = 128), 8 waves.  Three launches
// move each block's two 12.8 MB intermediates through HBM and stream ~98 us at B = 128; here they stay
// in LDS:
//   * c1 (1x1, 512 -> 128) runs over the band's 9 slot rows (image rows y0 - 1 .. y0 + 7; slots outside
//     the image read zeros through the DMA's out-of-range path and are never read back), its input
//     through a 3-stage LDS-DMA ring of 256-row x 64-channel slabs (4 DMAs per wave per k-tile), its
//     bf16 output to X1 (two 64-channel planes of 253 rows: 252 slot pixels + the zero row);
//   * c2 (3x3, 128 -> 128) reads X1 with the band kernel's per-lane tap shifts (taps in the padding read
//     the zero row) and writes X2 (208 rows, aliasing the dead ring);
//   * c3 (1x1, 128 -> 512) in four 128-channel chunks reads X2, adds bias + the residual (the block's own
//     input rows) in fp32, applies ReLU, rounds once and stores.
// Every wave owns one 16-channel n-block per phase (per chunk in c3) and every m-block; weights stream
// register-direct from the fragment layout two k-tiles ahead across phase boundaries (544 KB per
// workgroup for 196 outputs).  LDS: 64,768 B (X1) + 98,304 B (ring / X2) = 163,072 of 163,840.
// Each conv sums K in the unfused kernels' order: bit-identical to the three launches.
template <int IW, int RO, int CIN, int CMID, int PF>
__device__ __forceinline__ void block_band_body(const KArgs& a) {
  const __amdgpu_buffer_rsrc_t rY = sat_out_rsrc(a.y, 0x7fffffffL);   // output stores (sat_common.h policy)
  constexpr int IH = IW, NPART = IH / RO, PO = RO * IW;
  constexpr int SLOTS = RO + 2, P1 = SLOTS * IW;           // c1 pixels (slot rows) = 252
  constexpr int MB1 = (P1 + 15) / 16, MB2 = (PO + 15) / 16;   // 16, 13
  constexpr int ROWB = 128, NPL = CMID / 64;
  constexpr int X1PL = (P1 + 1) * ROWB, X2PL = MB2 * 16 * ROWB;
  constexpr int STG = MB1 * 16 * ROWB, NA = MB1 * 16 / 64;   // ring stage bytes; DMAs per wave per k-tile
  constexpr int X1 = 0, RING = NPL * X1PL, X2 = RING;
  constexpr int LDS = RING + 3 * STG;
  static_assert(IH % RO == 0 && CMID == 128 && CIN % 128 == 0 && MB1 * 16 == 8 * 8 * NA, "band shapes");
  static_assert(NPL * X2PL <= 3 * STG && LDS <= 163840, "LDS budget");
  constexpr int KT1 = CIN / 64, KT2 = 9 * CMID / 64, NCK = CIN / 128, KT3C = CMID / 64;
  constexpr int NT = KT1 + KT2 + NCK * KT3C;
  constexpr int KS1 = CIN / 32, KS2 = 9 * CMID / 32, KS3 = CMID / 32;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int img = blockIdx.x / NPART, part = blockIdx.x % NPART;
  const int y0 = part * RO;
  const int s_lo = y0 == 0 ? 1 : 0, s_hi = y0 + RO == IH ? RO : RO + 1;   // slots inside the image
  const long pix_img = (long)img * IH * IW;

  // ---- c1 input ring: k-tile t = channels 64t .. 64t+63 of LDS row r = slot pixel r (slot r / IW) ----
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);
  unsigned dsrc[NA];
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int d = w * NA + u, r = d * 8 + (lane >> 3), c = (lane & 7) ^ (lane >> 3), s = r / IW;
    const bool ok = r < P1 && s >= s_lo && s <= s_hi;
    dsrc[u] = ok ? (unsigned)(((pix_img + (long)(y0 - 1) * IW + r) * CIN + 8 * c) * 2) : K_OOB;
  }
  auto dma_a = [&](int t) {
    char* st = smem + RING + (t % 3) * STG;
#pragma unroll
    for (int u = 0; u < NA; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (k_lds_void*)(st + (w * NA + u) * 1024), 16,
                                               dsrc[u] == K_OOB ? (int)K_OOB : (int)(dsrc[u] + t * 128), 0, 0, 0);
  };

  // ---- weight fragments of k-tile T: this wave's n-block of the phase (c3: of chunk ck), both 32-k halves ----
  bf16x8 bq[PF + 1][2];
  auto load_b = [&](int T, bf16x8 (&dst)[2]) {
    const bf16* base;
    int nb, ks0, KS;
    if (T < KT1) { base = a.w1; nb = w; ks0 = 2 * T; KS = KS1; }
    else if (T < KT1 + KT2) { base = a.w2; nb = w; ks0 = 2 * (T - KT1); KS = KS2; }
    else { const int t = T - KT1 - KT2; base = a.w3; nb = (t / KT3C) * 8 + w; ks0 = 2 * (t % KT3C); KS = KS3; }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) dst[ks] = *(const bf16x8*)(base + ((long)(nb * KS + ks0 + ks) * 64 + lane) * 8);
  };

  int offu[2];   // unshifted rows (ring, X2): row i*16 + fr at i * 16 * ROWB + offu
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) offu[ks] = fr * ROWB + 16 * ((ks * 4 + fh) ^ (fr & 7));
  int offs[MB2][2];   // c2: output pixel p = i*16 + fr under tap (dh, dw) reads X1 slot row py + 1 + dh
  auto tap_offsets = [&](int tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < MB2; ++i) {
      const int p = i * 16 + fr, py = p / IW, pxx = p - py * IW;
      const bool ok = p < PO && (unsigned)(y0 + py + dh) < (unsigned)IH && (unsigned)(pxx + dw) < (unsigned)IW;
      const int q = ok ? (py + 1 + dh) * IW + pxx + dw : P1;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) offs[i][ks] = q * ROWB + 16 * ((ks * 4 + fh) ^ (q & 7));
    }
  };

  f32x4 acc[MB1];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < MB1; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // one 64-deep k-tile over MB m-blocks, one 32-deep half at a time (MB fragments live at once)
  auto tile_u = [&](auto MBc, const char* base, const bf16x8 (&b)[2]) {
    constexpr int MB = decltype(MBc)::value;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MB];
#pragma unroll
      for (int i = 0; i < MB; ++i) af[i] = *(const bf16x8*)(base + i * 16 * ROWB + offu[ks]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MB; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks], af[i], acc[i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  auto tile_s = [&](const char* base, const bf16x8 (&b)[2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MB2];
#pragma unroll
      for (int i = 0; i < MB2; ++i) af[i] = *(const bf16x8*)(base + offs[i][ks]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MB2; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks], af[i], acc[i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  // epilogue into an LDS plane image: the lane holds channels 16w + 4fh .. +3 of row i*16 + fr
  auto store_planes = [&](auto MBc, int region, int plane_bytes, int rows, const float4& bv) {
    constexpr int MB = decltype(MBc)::value;
    const int plane = w >> 2, c = (w & 3) * 2 + (fh >> 1);
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int r = i * 16 + fr;
      u32x2 o;
      bf16* ob = (bf16*)&o;
      ob[0] = (bf16)fmaxf(acc[i][0] + bv.x, 0.f);
      ob[1] = (bf16)fmaxf(acc[i][1] + bv.y, 0.f);
      ob[2] = (bf16)fmaxf(acc[i][2] + bv.z, 0.f);
      ob[3] = (bf16)fmaxf(acc[i][3] + bv.w, 0.f);
      if (r < rows) *(u32x2*)(smem + region + plane * plane_bytes + r * ROWB + 16 * (c ^ (r & 7)) + 8 * (fh & 1)) = o;
    }
  };

  // ---- prologue: biases (older than every DMA), A0 B0 A1 B1 .. B(PF-1) ----
  const float4 bias1 = *(const float4*)(a.b1 + w * 16 + 4 * fh);
  const float4 bias2 = *(const float4*)(a.b2 + w * 16 + 4 * fh);
  float4 bias3;
  if (tid < 8) *(uint4*)(smem + X1 + (tid >> 2) * X1PL + P1 * ROWB + (tid & 3) * 32) = make_uint4(0, 0, 0, 0);
  if (tid < 8) *(uint4*)(smem + X1 + (tid >> 2) * X1PL + P1 * ROWB + (tid & 3) * 32 + 16) = make_uint4(0, 0, 0, 0);
  dma_a(0);
  load_b(0, bq[0]);
  dma_a(1);
  load_b(1, bq[1]);
  static_for<PF - 2>([&](auto e) { load_b(2 + decltype(e)::value, bq[2 + decltype(e)::value]); });
  zero_acc();
  u32x2 resv[MB2];

  static_for<NT>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (T < KT1) {
      // this wave's DMAs of tile T have landed (every wave's after the barrier, which also retires every
      // wave's reads of stage (T + 2) % 3 before it is refilled)
      k_wait_barrier<younger_than_a(T, KT1, NT, PF, true, 2, NA)>();
      if constexpr (T + 2 < KT1) dma_a(T + 2);
    }
    if constexpr (T + PF < NT) load_b(T + PF, bq[(T + PF) % (PF + 1)]);
    const bf16x8 (&b)[2] = bq[T % (PF + 1)];
    if constexpr (T < KT1) {
      tile_u(std::integral_constant<int, MB1>{}, smem + RING + (T % 3) * STG, b);
      if constexpr (T == KT1 - 1) {   // c1 epilogue -> X1 (slot pixels 0 .. P1 - 1)
        store_planes(std::integral_constant<int, MB1>{}, X1, X1PL, P1, bias1);
        zero_acc();
        k_lds_barrier();
      }
    } else if constexpr (T < KT1 + KT2) {
      constexpr int t = T - KT1, pl = t % NPL;
      if constexpr (pl == 0) tap_offsets(t / NPL);
      tile_s(smem + X1 + pl * X1PL, b);
      if constexpr (t == KT2 - 1) {   // c2 epilogue -> X2 (the ring is dead: every wave passed c1's barrier)
        store_planes(std::integral_constant<int, MB2>{}, X2, X2PL, MB2 * 16, bias2);
        zero_acc();
        k_lds_barrier();
      }
    } else {
      constexpr int t = T - KT1 - KT2, ck = t / KT3C, kt = t % KT3C;
      const int ch = ck * 128 + w * 16 + 4 * fh;
      if constexpr (kt == 0) {   // residual rows + bias of this chunk, for its epilogue
        bias3 = *(const float4*)(a.b3 + ch);
#pragma unroll
        for (int i = 0; i < MB2; ++i) {   // rows past PO load a valid row (never stored): no branch
          const int p = min(i * 16 + fr, PO - 1);
          resv[i] = *(const u32x2*)(a.x + (pix_img + (long)y0 * IW + p) * CIN + ch);
        }
      }
      tile_u(std::integral_constant<int, MB2>{}, smem + X2 + kt * X2PL, b);
      if constexpr (kt == KT3C - 1) {   // c3 epilogue: bias, fp32 residual add, ReLU, one rounding
#pragma unroll
        for (int i = 0; i < MB2; ++i) {
          const int p = i * 16 + fr;
          const bf16* rh = (const bf16*)&resv[i];
          const float v[4] = {acc[i][0] + bias3.x, acc[i][1] + bias3.y, acc[i][2] + bias3.z, acc[i][3] + bias3.w};
          u32x2 o;
          bf16* ob = (bf16*)&o;
#pragma unroll
          for (int e = 0; e < 4; ++e) ob[e] = (bf16)fmaxf(v[e] + (float)rh[e], 0.f);
          if (p < PO) sat_st8(rY, (unsigned)(((pix_img + (long)y0 * IW + p) * CIN + ch) * 2), o);
        }
        zero_acc();
      }
    }
  });
}

__global__ __launch_bounds__(512) void block_band_kernel(KArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  block_band_body<28, 7, 512, 128, 2>(a);
  sat_stamp_end(a.st, t0);
}

// The bottleneck's c2 phase as a conv of its own (the layer3 blocks the trunk leaves unfused, so the
// decoder running beside the encoder finds CUs between launches): y = relu(conv3x3(x) + b) for
// x, y [N][IW][IW][C].  The 256 x 128 tile kernel (convpipe.hip) runs this shape as 196 tiles on 256
// CUs and streams a 256-row im2col A tile plus a 128-column weight tile per k-tile (48 KB); here one
// workgroup per half image (256 workgroups for B = 128) loads its 8 input rows ONCE into the
// conflict-free X1 plane image (57 KB: two workgroups fit one CU's LDS) and streams only weights,
// register-direct from the fragment layout (32 KB per k-tile for 112 x 256 outputs).  Same k order
// (tap-major, 64-deep k-tiles ascending), bias, ReLU and one rounding as the tile kernel: bit-identical.
template <int IW, int RO, int C, int PF>
__device__ __forceinline__ void conv3x3_frag_body(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                  const float* __restrict__ bias, bf16* __restrict__ y) {
  const __amdgpu_buffer_rsrc_t rY = sat_out_rsrc(y, 0x7fffffffL);   // output stores (sat_common.h policy)
  static_assert(IW / RO == 2 && IW % RO == 0 && C == 256, "two workgroups per image, 256 channels");
  constexpr int IH = IW, PO = RO * IW, R1 = RO + 1, P1 = R1 * IW;
  constexpr int MB = (P1 + 15) / 16;
  static_assert(MB * 16 == P1, "whole m-blocks of input rows");
  constexpr int ROWB = 128, X1PL = (P1 + 1) * ROWB, NPL = C / 64;
  constexpr int NT = 9 * C / 64, KS = 9 * C / 32;
  __shared__ __attribute__((aligned(16))) char smem[NPL * X1PL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  // SAT_C2_ROT (diagnostics): the workgroups sharing an XCD (blockIdx.x % 8) rotate which 32-channel group each wave
  // owns, so at any moment they stream different weight lines
  const int wc = SAT_C2_ROT ? __builtin_amdgcn_readfirstlane((w + (int)(blockIdx.x >> (SAT_C2_ROT == 1 ? 3 : 0))) & 7) : w;
  const int img = blockIdx.x >> 1, half = blockIdx.x & 1;
  const int y0 = half * RO, ws = half ? IH - R1 : 0;
  const long pix_img = (long)img * IH * IW;

  // The input rows ws .. ws + R1 - 1 (one contiguous block) go HBM -> LDS by buffer_load ... lds, plane by plane: the
  // k-loop is tap-major with the 64-channel plane innermost, so k-tile p needs planes 0 .. p only.  Each wave DMAs
  // 1-KB pieces (8 pixel rows of one plane; lane l fetches the chunk that lands in swizzled slot l % 8) in the order
  // plane 0, [bias, the first PF weight tiles], planes 1 .. NPL-1, and waits for plane p right before k-tile p with a
  // vmcnt that counts only the later planes' DMAs (the compiler's weight loads may sit anywhere: counting none of
  // them can only wait longer), so planes 1 .. NPL-1 arrive under the MFMAs of the k-tiles before them.
  constexpr int NPC = P1 / 8, PPW = (NPC + 7) / 8;   // 1-KB pieces per plane, per wave
  static_assert(P1 % 8 == 0 && PPW == 2, "whole pieces, two per wave");
  const __amdgpu_buffer_rsrc_t rX =
      __builtin_amdgcn_make_buffer_rsrc((void*)(x + (pix_img + (long)ws * IW) * C), (short)0, P1 * C * 2, 0x00020000);
  unsigned dsrc[PPW];
  int dpc[PPW];
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const int d = w + 8 * u < NPC ? w + 8 * u : w;   // waves without a second piece repeat their first (same bytes)
    dpc[u] = d;
    dsrc[u] = (unsigned)(((d * 8 + (lane >> 3)) * C + 8 * ((lane & 7) ^ (lane >> 3))) * 2);
  }
  auto dma_plane = [&](int pl) {
#pragma unroll
    for (int u = 0; u < PPW; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (k_lds_void*)(smem + pl * X1PL + dpc[u] * 1024), 16,
                                               (int)(dsrc[u] + pl * 128), 0, 0, 0);
  };
  dma_plane(0);
  float4 bv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bv[j] = *(const float4*)(bias + wc * 32 + j * 16 + 4 * fh);

  bf16x8 bq[PF + 1][2][2];
  auto load_b = [&](int T, bf16x8 (&dst)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        dst[ks][j] = *(const bf16x8*)(wf + ((long)((wc * 2 + j) * KS + 2 * T + ks) * 64 + lane) * 8);
  };
  static_for<PF>([&](auto e) { load_b(decltype(e)::value, bq[decltype(e)::value]); });
#pragma unroll
  for (int pl = 1; pl < NPL; ++pl) dma_plane(pl);
  if (tid < NPL * 8) *(uint4*)(smem + (tid >> 3) * X1PL + P1 * ROWB + (tid & 7) * 16) = make_uint4(0, 0, 0, 0);

  int offs[MB][2];
  auto tap_offsets = [&](int tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int p = i * 16 + fr, py = p / IW, pxx = p - py * IW;
      const bool ok = p < PO && (unsigned)(y0 + py + dh) < (unsigned)IH && (unsigned)(pxx + dw) < (unsigned)IW;
      const int q = ok ? p + (y0 - ws + dh) * IW + dw : P1;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) offs[i][ks] = q * ROWB + 16 * ((ks * 4 + fh) ^ (q & 7));
    }
  };
  f32x4 acc[MB][2];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // SAT_C2_ABL (diagnostics builds only, tools/c2_ablation.py; product builds: 0): bit 0 no weight streaming (the
  // prologue's fragments reused), bit 1 no MFMA, bit 2 no A fragment reads from LDS (the first read reused)
  constexpr int ABL = SAT_C2_ABL;
  bf16x8 af0[2][MB];
  static_for<NT>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value, pl = T % NPL;
    if constexpr (T < NPL) k_wait_barrier<PPW * (NPL - 1 - T)>();   // plane T (and the zero rows) in LDS
    if constexpr (T + PF < NT && !(ABL & 1)) load_b(T + PF, bq[(T + PF) % (PF + 1)]);
    if constexpr (pl == 0) tap_offsets(T / NPL);
    const bf16x8 (&b)[2][2] = bq[(ABL & 1) ? T % PF : T % (PF + 1)];
    bf16x8 af[2][MB];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        if constexpr ((ABL & 4) && T > 0) af[ks][i] = af0[ks][i];
        else af[ks][i] = *(const bf16x8*)(smem + pl * X1PL + offs[i][ks]);
        if constexpr ((ABL & 4) && T == 0) af0[ks][i] = af[ks][i];
      }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (ABL & 2) asm volatile("" ::"v"(b[ks][j]), "v"(af[ks][i]));
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  });

  // epilogue: the lane holds channels w*32 + j*16 + 4fh .. +3 of output pixel i*16 + fr
  if constexpr (SAT_PAIR_STORES) {
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const unsigned o0 = (unsigned)(((pix_img + (long)y0 * IW + i * 16 + fr) * C + wc * 32 + 4 * fh) * 2);
      sat_st_pair16(rY, o0, o0 + 32, relu_bf16x4(acc[i][0], bv[0]), relu_bf16x4(acc[i][1], bv[1]), i * 16 + fr < PO,
                i * 16 + fr < PO);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < MB; ++i)
        if (i * 16 + fr < PO)
          sat_st8(rY, (unsigned)(((pix_img + (long)y0 * IW + i * 16 + fr) * C + wc * 32 + j * 16 + 4 * fh) * 2),
                  relu_bf16x4(acc[i][j], bv[j]));
  }
}

// The same idea for a band of RO output rows of a larger image (ResNet152 layer2's c2: 28 x 28, 128 ->
// 128, RO = 7: four workgroups per image, 512 for B = 128): the band's input rows plus a one-row halo on
// each side that lies inside the image are staged once in LDS (slot s holds image row y0 - 1 + s; taps
// outside the image read the zero row), the C x 9C weight streams register-direct, each of the 8 waves
// owns NJ = C / (128 NSL) n-blocks of 16 channels and every m-block of the band.  NSL > 1 splits the
// output channels over NSL workgroups per band (ResNet152 layer3's c2 as one 14-row band = one image per
// workgroup, two 128-channel slices: each workgroup streams half the weights -- 0.59 MB -- for 196 output
// pixels, where the half-image kernel streams all 1.18 MB for 98).  Same k order, bias, ReLU and rounding
// as the tile kernel: bit-identical.
template <int IW, int RO, int C, int NSL, int WM, int PF, int NWV = 8>
__device__ __forceinline__ void conv3x3_band_body(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                  const float* __restrict__ bias, bf16* __restrict__ y, int nbands) {
  const __amdgpu_buffer_rsrc_t rY = sat_out_rsrc(y, 0x7fffffffL);   // output stores (sat_common.h policy)
  constexpr int IH = IW, NPART = IH / RO, PO = RO * IW, MBT = (PO + 15) / 16;
  constexpr int MB = (MBT + WM - 1) / WM, WN = NWV / WM;   // m-blocks per wave; NWV waves = WM m-groups x WN
  constexpr int SLOTS = RO + 2, ZR = SLOTS * IW;        // LDS pixel rows + the zero row
  constexpr int ROWB = 128, NPL = C / 64, NJ = C / (16 * WN * NSL), CS = C / NSL;
  constexpr int NT = 9 * C / 64, KS = 9 * C / 32;
  // LDS-DMA pieces of 1 KB = 8 pixel rows of one plane, the zero row included (its lanes read out of bounds: zeros)
  constexpr int NPC = ZR / 8 + 1, PPW = (NPC + NWV - 1) / NWV, XPL = NPC * 1024;
  static_assert(C % (16 * WN * NSL) == 0 && NJ >= 1 && NWV % WM == 0 && IH % RO == 0, "whole bands, 16-channel n-blocks per wave");
  static_assert(PPW * (NPL - 1) < 64, "plane waits fit vmcnt");
  __shared__ __attribute__((aligned(16))) char smem[NPL * XPL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  const int wm = w % WM;                           // this wave's m-group and (rotated, SAT_WROT) n-group
  // (not the four-wave layer2 form: at 254 VGPRs the rotation tips it into scratch)
  constexpr bool ROT = SAT_WROT && !(NWV == 4 && NSL == 1);
  const int wn = ROT ? __builtin_amdgcn_readfirstlane((w / WM + (int)(blockIdx.x >> 3)) % WN) : w / WM;
  // slice-major over groups of 8 consecutive workgroups (one per XCD under round-robin placement), so the
  // NSL slices of one band land on one XCD and share its input rows in L2
  const int slice = NSL == 1 ? 0 : (int)((blockIdx.x >> 3) % NSL);
  const int band = NSL == 1 ? (int)blockIdx.x : (int)((blockIdx.x / (8 * NSL)) * 8 + (blockIdx.x & 7));
  if (band >= nbands) return;   // the grid rounds the bands up to whole groups of 8 (NSL > 1)
  const int img = band / NPART, part = band % NPART;
  const int y0 = part * RO;
  const int cb = slice * CS;                       // first output channel of this workgroup
  const long pix_img = (long)img * IH * IW;
  const unsigned lane_b = (unsigned)lane * 16;

  // Slot s holds image row y0 - 1 + s: the slots are consecutive image rows, so pixel row r of a plane is image pixel
  // (y0 - 1) IW + r.  They go HBM -> LDS by buffer_load ... lds, plane by plane (lane l of a piece fetches the chunk
  // that lands in swizzled slot l % 8); rows above or below the image and the zero row read out of bounds (zeros).
  // Order: plane 0, [bias, the first PF weight tiles], planes 1 .. NPL-1; k-tile p (tap-major, plane innermost) waits
  // for plane p with a vmcnt counting only the later planes' DMAs (the compiler's weight loads may sit anywhere:
  // counting none of them can only wait longer), so the later planes arrive under the first k-tiles' MFMAs.
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)(x + pix_img * C), (short)0,
                                                                       IH * IW * C * 2, 0x00020000);
  unsigned dsrc[PPW];
  int dpc[PPW];
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const int d = w + NWV * u < NPC ? w + NWV * u : w;   // waves without another piece repeat their first (same bytes)
    const int r = d * 8 + (lane >> 3), g = (y0 - 1) * IW + r;
    dpc[u] = d;
    dsrc[u] = r < ZR && g >= 0 ? (unsigned)((g * C + 8 * ((lane & 7) ^ (lane >> 3))) * 2) : K_OOB;
  }
  auto dma_plane = [&](int pl) {
#pragma unroll
    for (int u = 0; u < PPW; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (k_lds_void*)(smem + pl * XPL + dpc[u] * 1024), 16,
                                               dsrc[u] == K_OOB ? (int)K_OOB : (int)(dsrc[u] + pl * 128), 0, 0, 0);
  };
  dma_plane(0);
  float4 bv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bv[j] = *(const float4*)(bias + cb + (wn * NJ + j) * 16 + 4 * fh);
  bf16x8 bq[PF + 1][2][NJ];
  auto load_b = [&](int T, bf16x8 (&dst)[2][NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        dst[ks][j] = *(const bf16x8*)((const char*)wf + (size_t)((cb / 16 + wn * NJ + j) * KS + 2 * T + ks) * 1024 +
                                      lane_b);
  };
  static_for<PF>([&](auto e) { load_b(decltype(e)::value, bq[decltype(e)::value]); });
#pragma unroll
  for (int pl = 1; pl < NPL; ++pl) dma_plane(pl);

  int offs[MB][2];
  auto tap_offsets = [&](int tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int p = (wm * MB + i) * 16 + fr, py = p / IW, pxx = p - py * IW;
      const bool ok = p < PO && (unsigned)(y0 + py + dh) < (unsigned)IH && (unsigned)(pxx + dw) < (unsigned)IW;
      const int q = ok ? (py + 1 + dh) * IW + pxx + dw : ZR;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) offs[i][ks] = q * ROWB + 16 * ((ks * 4 + fh) ^ (q & 7));
    }
  };
  f32x4 acc[MB][NJ];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  static_for<NT>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value, pl = T % NPL;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (T < NPL) k_wait_barrier<PPW * (NPL - 1 - T)>();   // plane T in LDS
    if constexpr (T + PF < NT) load_b(T + PF, bq[(T + PF) % (PF + 1)]);
    if constexpr (pl == 0) tap_offsets(T / NPL);
    const bf16x8 (&b)[2][NJ] = bq[T % (PF + 1)];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MB];
#pragma unroll
      for (int i = 0; i < MB; ++i) af[i] = *(const bf16x8*)(smem + pl * XPL + offs[i][ks]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  });

  char* y_s = (char*)(y + (pix_img + (long)y0 * IW + wm * MB * 16) * C + cb + wn * NJ * 16);
  const unsigned row_b = (unsigned)(fr * C + 4 * fh) * 2;
  if constexpr (NJ % 2 == 0 && SAT_PAIR_STORES) {
#pragma unroll
    for (int j = 0; j < NJ; j += 2)
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const unsigned o0 = (unsigned)(y_s - (char*)y + (size_t)(i * 16 * C + j * 16) * 2 + row_b);
        sat_st_pair16(rY, o0, o0 + 32, relu_bf16x4(acc[i][j], bv[j]), relu_bf16x4(acc[i][j + 1], bv[j + 1]),
                  (wm * MB + i) * 16 + fr < PO, (wm * MB + i) * 16 + fr < PO);
      }
  } else {   // odd NJ: m-block pairs (pixels i 16 + fr and (i + 1) 16 + fr), the odd last m-block with 8-B stores
    constexpr int MP = SAT_PAIR_STORES ? MB / 2 * 2 : 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < MP; i += 2) {
        const unsigned oA = (unsigned)(y_s - (char*)y + (size_t)(i * 16 * C + j * 16) * 2 + row_b);
        sat_st_pair16(rY, oA, oA + 32 * C, relu_bf16x4(acc[i][j], bv[j]), relu_bf16x4(acc[i + 1][j], bv[j]),
                  (wm * MB + i) * 16 + fr < PO, (wm * MB + i + 1) * 16 + fr < PO);
      }
#pragma unroll
      for (int i = MP; i < MB; ++i)
        if ((wm * MB + i) * 16 + fr < PO)
          sat_st8(rY, (unsigned)(y_s - (char*)y + (size_t)(i * 16 * C + j * 16) * 2 + row_b), relu_bf16x4(acc[i][j], bv[j]));
    }
  }
}

// ResNet152 layer2's c2 (28 x 28, 128 -> 128) as 7-row bands on four waves of 32 channels (NJ = 2): every A
// fragment read from LDS feeds two MFMAs (the eight-wave form of 16 channels per wave read one per MFMA: LDS-read
// bound with MFMA and the weight stream), two workgroups per CU (65 KB of LDS, 256 threads, <= 256 VGPRs with the
// weight prefetch one k-tile ahead): 36.0 -> 28.2 us back to back, 37.4 -> 27.3 us in-step (profiles/r5_s14)
template <int PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv3x3_band4w_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                             const float* __restrict__ bias, bf16* __restrict__ y,
                                                             int nbands, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_band_body<28, 7, 128, 1, 1, PF, 4>(x, wf, bias, y, nbands);
  sat_stamp_end(st, t0);
}

// VGG19 block 2's 112 x 112, 128 -> 128 conv as 2-row bands (one-row halo each side: 115 KB of LDS), every
// workgroup streaming the whole 295 KB weight once for 224 output pixels, where the tile kernel fetches a 256-row
// im2col A tile per 128 x 128 tile: 647-657 -> 542-548 us per launch (profiles/r3_s44).  Measured and removed: block
// 1's 224 x 224, 64 -> 64 convs in the same form (two m-groups of waves): 858-860 vs 523 us.
__global__ __launch_bounds__(512) void conv3x3_band112_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                              const float* __restrict__ bias, bf16* __restrict__ y,
                                                              int nbands, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_band_body<112, 2, 128, 1, 1, 2>(x, wf, bias, y, nbands);
  sat_stamp_end(st, t0);
}

// VGG19 block 3's 56 x 56, 256 -> 256 convs (three launches) as 2-row bands: the layer3 c2 half-image geometry
// (112 output pixels x 256 channels per workgroup, 8 waves of 7 m-blocks x 2 n-blocks, 115 KB of LDS), 28
// workgroups per image
__global__ __launch_bounds__(512) void conv3x3_band56_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                             const float* __restrict__ bias, bf16* __restrict__ y,
                                                             int nbands, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_band_body<56, 2, 256, 1, 1, 2>(x, wf, bias, y, nbands);
  sat_stamp_end(st, t0);
}

// VGG19's block-5 convs (14 x 14, 512 -> 512, four launches): half images (one-row halo each side) x four
// 128-channel slices, eight waves of 16 channels (130 KB of LDS, one workgroup per CU)
__global__ __launch_bounds__(512) void conv3x3_half512_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                              const float* __restrict__ bias, bf16* __restrict__ y,
                                                              int nbands, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_band_body<14, 7, 512, 4, 1, 2>(x, wf, bias, y, nbands);
  sat_stamp_end(st, t0);
}

// The same idea for images small enough to stage whole (ResNet152 layer4's stride-1 c2: 7 x 7, 512 -> 512): a
// workgroup takes G consecutive images (G * 49 pixels, their rows contiguous in memory and in LDS, plus the zero
// row) and one of NSL output-channel slices; taps outside an image read the zero row.  The tile kernel runs this
// shape as 98 tiles of 256 x 128 on 256 CUs (each fetching a 2.4 MB im2col A tile and a 1.2 MB weight panel);
// here G = 2, NSL = 4 gives 256 workgroups that each stage 100 KB of input once and stream a 1.18 MB weight
// slice for 98 x 128 outputs.  G = 1 at B <= 64 per GPU.  Same k order, bias, ReLU and rounding: bit-identical.
template <int IW, int C, int G, int NSL, int PF>
__device__ __forceinline__ void conv3x3_img_body(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                 const float* __restrict__ bias, bf16* __restrict__ y, int nimg) {
  const __amdgpu_buffer_rsrc_t rY = sat_out_rsrc(y, 0x7fffffffL);   // output stores (sat_common.h policy)
  constexpr int IH = IW, PI = IH * IW, P = G * PI, MB = (P + 15) / 16, ZR = P;
  constexpr int ROWB = 128, XPL = (P + 1) * ROWB, NPL = C / 64, NJ = C / (16 * 8 * NSL), CS = C / NSL;
  constexpr int NT = 9 * C / 64, KS = 9 * C / 32, CPP = C / 8;
  constexpr int PER_T = (P * CPP + 511) / 512;
  static_assert(NJ >= 1 && C % (128 * NSL) == 0 && NPL * XPL <= 163840, "16-channel n-blocks per wave, LDS");
  __shared__ __attribute__((aligned(16))) char smem[NPL * XPL];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  // slice-major over groups of 8 consecutive workgroups (one per XCD under round-robin placement): the NSL
  // slices of one image group land on one XCD and share its input rows in L2
  // (measured and removed: each XCD owning one slice -- XCD x streams slice x % 4 only -- cuts the per-XCD weight
  // refetch, 2.9x -> ~2.3x of the algorithmic bytes, but runs 34.3-35.4 vs 33.5 us: not HBM-bound, profiles/r3_s39)
  const int slice = NSL == 1 ? 0 : (int)((blockIdx.x >> 3) % NSL);
  const int grp = NSL == 1 ? (int)blockIdx.x : (int)((blockIdx.x / (8 * NSL)) * 8 + (blockIdx.x & 7));
  const int ngrp = (nimg + G - 1) / G;
  if (grp >= ngrp) return;   // the grid rounds the groups up to whole groups of 8
  const int img0 = grp * G, nv = min(G, nimg - img0) * PI;   // valid pixels of this group
  const int cb = slice * CS;
  const unsigned lane_b = (unsigned)lane * 16;
  // XCD-aware weight rotation (SAT_WROT, as the band forms): the workgroups of one slice sharing an XCD start their
  // waves on different channel groups
  const int wr = SAT_WROT ? __builtin_amdgcn_readfirstlane((w + (int)((blockIdx.x >> 3) / NSL)) & 7) : w;

  uint4 xin[PER_T];
  const uint4* xs = (const uint4*)(x + (long)img0 * PI * C);
#pragma unroll
  for (int u = 0; u < PER_T; ++u) xin[u] = xs[min(u * 512 + tid, nv * CPP - 1)];
  float4 bv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bv[j] = *(const float4*)(bias + cb + (wr * NJ + j) * 16 + 4 * fh);
  bf16x8 bq[PF + 1][2][NJ];
  auto load_b = [&](int T, bf16x8 (&dst)[2][NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        dst[ks][j] = *(const bf16x8*)((const char*)wf + (size_t)((cb / 16 + wr * NJ + j) * KS + 2 * T + ks) * 1024 + lane_b);
  };
  static_for<PF>([&](auto e) { load_b(decltype(e)::value, bq[decltype(e)::value]); });
#pragma unroll
  for (int u = 0; u < PER_T; ++u) {
    const int q = u * 512 + tid, r = q / CPP, c = q % CPP;
    if (q < P * CPP) *(uint4*)(smem + (c >> 3) * XPL + r * ROWB + 16 * ((c & 7) ^ (r & 7))) = xin[u];
  }
  if (tid < NPL * 8) *(uint4*)(smem + (tid >> 3) * XPL + ZR * ROWB + (tid & 7) * 16) = make_uint4(0, 0, 0, 0);
  k_lds_barrier();

  int offs[MB][2];
  auto tap_offsets = [&](int tap) {
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int p = i * 16 + fr, g = p / PI, qq = p - g * PI, py = qq / IW, pxx = qq - py * IW;
      const bool ok = p < P && (unsigned)(py + dh) < (unsigned)IH && (unsigned)(pxx + dw) < (unsigned)IW;
      const int q = ok ? p + dh * IW + dw : ZR;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) offs[i][ks] = q * ROWB + 16 * ((ks * 4 + fh) ^ (q & 7));
    }
  };
  f32x4 acc[MB][NJ];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  static_for<NT>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value, pl = T % NPL;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (T + PF < NT) load_b(T + PF, bq[(T + PF) % (PF + 1)]);
    if constexpr (pl == 0) tap_offsets(T / NPL);
    const bf16x8 (&b)[2][NJ] = bq[T % (PF + 1)];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MB];
#pragma unroll
      for (int i = 0; i < MB; ++i) af[i] = *(const bf16x8*)(smem + pl * XPL + offs[i][ks]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  });

  char* y_s = (char*)(y + (long)img0 * PI * C + cb + wr * NJ * 16);
  const unsigned row_b = (unsigned)(fr * C + 4 * fh) * 2;
  if constexpr (NJ % 2 == 0 && SAT_PAIR_STORES) {
#pragma unroll
    for (int j = 0; j < NJ; j += 2)
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const unsigned o0 = (unsigned)(y_s - (char*)y + (size_t)(i * 16 * C + j * 16) * 2 + row_b);
        sat_st_pair16(rY, o0, o0 + 32, relu_bf16x4(acc[i][j], bv[j]), relu_bf16x4(acc[i][j + 1], bv[j + 1]),
                  i * 16 + fr < nv, i * 16 + fr < nv);
      }
  } else {   // odd NJ: m-block pairs, the odd last m-block with 8-B stores
    constexpr int MP = SAT_PAIR_STORES ? MB / 2 * 2 : 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < MP; i += 2) {
        const unsigned oA = (unsigned)(y_s - (char*)y + (size_t)(i * 16 * C + j * 16) * 2 + row_b);
        sat_st_pair16(rY, oA, oA + 32 * C, relu_bf16x4(acc[i][j], bv[j]), relu_bf16x4(acc[i + 1][j], bv[j]),
                  i * 16 + fr < nv, (i + 1) * 16 + fr < nv);
      }
#pragma unroll
      for (int i = MP; i < MB; ++i)
        if (i * 16 + fr < nv)
          sat_st8(rY, (unsigned)(y_s - (char*)y + (size_t)(i * 16 * C + j * 16) * 2 + row_b), relu_bf16x4(acc[i][j], bv[j]));
    }
  }
}

template <int G>
__global__ __launch_bounds__(512) void conv3x3_img_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                          const float* __restrict__ bias, bf16* __restrict__ y,
                                                          int nimg, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_img_body<7, 512, G, 4, 2>(x, wf, bias, y, nimg);
  sat_stamp_end(st, t0);
}

// ResNet152 layer3's c2 when half images alone would leave CUs idle (B <= 64 per GPU: 2B workgroups): each half image
// as two 128-channel slices (4B workgroups), each streaming half the weights, with four waves that own 32 channels
// each and every m-block (each A fragment feeds two MFMAs; two workgroups fit a CU): 18.5 vs 19.4 us and 4.37 vs
// 4.42-4.44 ms per B = 64 step against eight waves of 16 channels (profiles/r3_s24); weights 3 or 4 k-tiles ahead:
// 18.6-18.9 vs 18.6 us (r3_s29).  At B = 128 the half-image kernel on four waves of 64 channels (one wave per SIMD,
// VGPRs left to decoder waves): 32.4 vs 29.1 us, step 6.66 vs 6.50 ms (r3_s32).  At B = 64 four 64-channel slices
// per half image (two workgroups per CU): 19.5-20.0 vs 18.3-18.5 us, step 4.23-4.25 vs 4.04-4.13 ms (r3_s40).  Measured and removed: the
// same four-wave form over whole images (31.5 vs 29.3 us at B = 128), and (profiles/r3_s13, r3_s14, r3_s16) two
// m-groups of waves, weights 3 / 4 k-tiles ahead, whole images as four 64-channel slices -- all within noise.
__global__ __launch_bounds__(256) void conv3x3_slice2_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                             const float* __restrict__ bias, bf16* __restrict__ y,
                                                             int nbands, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_band_body<14, 7, 256, 2, 1, SAT_SL2_PF, 4>(x, wf, bias, y, nbands);
  sat_stamp_end(st, t0);
}



// The bottleneck's c1 phase as a conv of its own (the unfused layer3 blocks): y = relu(x . W^T + b) for
// x [N][IW][IW][CI], y [N][IW][IW][CM] (1x1, CI = 1024 -> CM = 256).  One workgroup per half image: its
// 98 input pixels stream through a 3-stage LDS-DMA ring of 64-channel slabs (the fused kernel's c1 ring,
// counted vmcnt + one barrier per k-tile), the weights register-direct two k-tiles ahead.  The tile
// kernel (convpipe.hip) runs this shape as 196 tiles of 256 x 128 that each fetch 768 KB; here 256
// workgroups each fetch 712 KB.  Same k order, bias, ReLU and rounding: bit-identical.
template <int IW, int RO, int CI, int CM, int PF, int NSL = 1, int DA = 2>   // DA: input DMAs DA k-tiles ahead (ring of DA + 1)
__device__ __forceinline__ void conv1x1_frag_body(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                  const float* __restrict__ bias, bf16* __restrict__ y,
                                                  unsigned x_bytes, int nhalves) {
  const __amdgpu_buffer_rsrc_t rY = sat_out_rsrc(y, 0x7fffffffL);   // output stores (sat_common.h policy)
  static_assert(IW / RO == 2 && IW % RO == 0 && CM == 256 && CI % 64 == 0, "two workgroups per image");
  constexpr int IH = IW, PO = RO * IW, MB = (PO + 15) / 16;
  constexpr int ROWB = 128, STG = 128 * ROWB;   // ring stage: 128 rows x 64 channels
  static_assert(MB * 16 <= 128, "one stage holds the half image's rows");
  constexpr int NT = CI / 64, KS = CI / 32;
  constexpr int NJ = 2 / NSL;                   // 16-channel n-blocks per wave (NSL channel slices per half image)
  static_assert(NSL == 1 || NSL == 2, "one or two channel slices");
  __shared__ __attribute__((aligned(16))) char smem[(DA + 1) * STG];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fh = lane >> 4;
  // NSL > 1: slice-major over groups of 8 consecutive workgroups (one per XCD under round-robin placement),
  // so both slices of a half image read its input from one XCD's L2
  const int slice = NSL == 1 ? 0 : (int)((blockIdx.x >> 3) % NSL);
  const int hb = NSL == 1 ? (int)blockIdx.x : (int)((blockIdx.x / (8 * NSL)) * 8 + (blockIdx.x & 7));
  if (hb >= nhalves) return;
  const int wr = SAT_WROT ? __builtin_amdgcn_readfirstlane((w + (int)(blockIdx.x >> 3)) & 7) : w;   // rotated group
  const int nb0 = slice * (CM / 16 / NSL) + wr * NJ;   // this wave's first 16-channel n-block
  const long pix0 = (long)(hb >> 1) * IH * IW + (long)(hb & 1) * PO;

  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)x_bytes, 0x00020000);
  unsigned dsrc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int d = w * 2 + u, r = d * 8 + (lane >> 3), c = (lane & 7) ^ (lane >> 3);
    dsrc[u] = r < PO ? (unsigned)(((pix0 + r) * CI + 8 * c) * 2) : K_OOB;
  }
  auto dma_a = [&](int t) {
    char* st = smem + (t % (DA + 1)) * STG;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (k_lds_void*)(st + (w * 2 + u) * 1024), 16,
                                               dsrc[u] == K_OOB ? (int)K_OOB : (int)(dsrc[u] + t * 128), 0, 0, 0);
  };
  bf16x8 bq[PF + 1][2][NJ];
  auto load_b = [&](int T, bf16x8 (&dst)[2][NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        dst[ks][j] = *(const bf16x8*)(wf + ((long)((nb0 + j) * KS + 2 * T + ks) * 64 + lane) * 8);
  };
  float4 bv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bv[j] = *(const float4*)(bias + (nb0 + j) * 16 + 4 * fh);
  int offu[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) offu[ks] = fr * ROWB + 16 * ((ks * 4 + fh) ^ (fr & 7));
  f32x4 acc[MB][NJ];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // issue order A0 B0 A1 B1 .. (A(e) for e < DA, B(e) for e < PF, interleaved), then per k-tile after its wait
  // A(T+DA), B(T+PF): the order younger_than_a_da() counts (bias loads are older than A0 and retire first)
  static_for<(DA > PF ? DA : PF)>([&](auto e) {
    constexpr int E = decltype(e)::value;
    if constexpr (E < DA) dma_a(E);
    if constexpr (E < PF) load_b(E, bq[E]);
  });

  static_for<NT>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value;
    // this wave's DMAs of tile T have landed, every wave's too after the barrier; the barrier also
    // retires every wave's reads of stage (T + 2) % 3 (tile T - 1) before it is refilled
    k_wait_barrier<younger_than_a_da(T, NT, NT, PF, DA, 2 * NJ, 2)>();
    if constexpr (T + DA < NT) dma_a(T + DA);
    if constexpr (T + PF < NT) load_b(T + PF, bq[(T + PF) % (PF + 1)]);
    const bf16x8 (&b)[2][NJ] = bq[T % (PF + 1)];
    const char* st = smem + (T % (DA + 1)) * STG;
    bf16x8 af[2][MB];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i) af[ks][i] = *(const bf16x8*)(st + i * 16 * ROWB + offu[ks]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  });

  if constexpr (NJ % 2 == 0 && SAT_PAIR_STORES) {
#pragma unroll
    for (int j = 0; j < NJ; j += 2)
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const unsigned o0 = (unsigned)(((pix0 + i * 16 + fr) * CM + (nb0 + j) * 16 + 4 * fh) * 2);
        sat_st_pair16(rY, o0, o0 + 32, relu_bf16x4(acc[i][j], bv[j]), relu_bf16x4(acc[i][j + 1], bv[j + 1]),
                  i * 16 + fr < PO, i * 16 + fr < PO);
      }
  } else {   // odd NJ: m-block pairs, the odd last m-block with 8-B stores
    constexpr int MP = SAT_PAIR_STORES ? MB / 2 * 2 : 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < MP; i += 2) {
        const unsigned oA = (unsigned)(((pix0 + i * 16 + fr) * CM + (nb0 + j) * 16 + 4 * fh) * 2);
        sat_st_pair16(rY, oA, oA + 32 * CM, relu_bf16x4(acc[i][j], bv[j]), relu_bf16x4(acc[i + 1][j], bv[j]),
                  i * 16 + fr < PO, (i + 1) * 16 + fr < PO);
      }
#pragma unroll
      for (int i = MP; i < MB; ++i)
        if (i * 16 + fr < PO)
          sat_st8(rY, (unsigned)(((pix0 + i * 16 + fr) * CM + (nb0 + j) * 16 + 4 * fh) * 2), relu_bf16x4(acc[i][j], bv[j]));
    }
  }
}

__global__ __launch_bounds__(512) void conv1x1_frag_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                           const float* __restrict__ bias, bf16* __restrict__ y,
                                                           unsigned x_bytes, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv1x1_frag_body<14, 7, 1024, 256, SAT_C1_PF, 1, SAT_C1_DA>(x, wf, bias, y, x_bytes, (int)gridDim.x);
  sat_stamp_end(st, t0);
}

// the same with each half image as two 128-channel slices (B <= 80 per GPU, as conv3x3_slice2_kernel)
__global__ __launch_bounds__(512) void conv1x1_frag2_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                            const float* __restrict__ bias, bf16* __restrict__ y,
                                                            unsigned x_bytes, int nhalves, SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv1x1_frag_body<14, 7, 1024, 256, 2, 2>(x, wf, bias, y, x_bytes, nhalves);
  sat_stamp_end(st, t0);
}


template <int PF>
__global__ __launch_bounds__(512) void conv3x3_frag_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wf,
                                                           const float* __restrict__ bias, bf16* __restrict__ y,
                                                           SatStamps st) {
  const SatStampT0 t0 = sat_stamp_begin(st);
  conv3x3_frag_body<14, 7, 256, PF>(x, wf, bias, y);
  sat_stamp_end(st, t0);
}

// [N][K] bf16 -> [N/16][K/32][64 lanes][8]: lane l = (fh << 4) | fr holds row 16 nb + fr, k 32 ks + 8 fh ..
__global__ void frag_layout_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst, int N, int K) {
  const long n8 = (long)N * K / 8;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long e = v * 8;                      // destination element
    const int lane = (int)((e / 8) % 64);
    const long blk = e / 512;                  // (nb, ks)
    const int KS = K / 32;
    const int NB = N / 16;
    const int nb = (int)(blk / KS), ks = (int)(blk % KS);
    const int row = nb * 16 + (lane & 15), k = ks * 32 + (lane >> 4) * 8;
    *(uint4*)(dst + e) = *(const uint4*)(src + (long)row * K + k);
  }
}

// Layer3 c1 / c2 launch form for a batch of N images: 1 = one workgroup per half image (2N workgroups), 2 = two
// 128-channel slices per half image (4N).  SatPolicy::conv_slices forces
// one; automatic: slices when the half images fill less than half the chip's 256 CUs (B < 64 per GPU).
int sat_frag_slices(int N) {
  const int f = sat_policy().conv_slices;
  if (f == 1 || f == 2) return f;
  // auto: slices only below 64 images (128 half images); at B = 64 the whole-half-image kernels measured faster
  // since the write-through stores (3.97-3.98 vs 4.01-4.04 ms per step, profiles/r4_s42 / r4_s43)
  return 2 * N < 128 ? 2 : 1;
}

}  // namespace

extern "C" int sat_mfma_frag_layout(int N, int K, const void* src, void* dst, void* stream) {
  SAT_REQUIRE(src && dst && N > 0 && K > 0 && N % 16 == 0 && K % 32 == 0);
  SAT_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0);
  const long n8 = (long)N * K / 8;
  const int g = (int)((n8 + 255) / 256 < 4096 ? (n8 + 255) / 256 : 4096);
  hipLaunchKernelGGL(frag_layout_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, (const bf16*)src, (bf16*)dst, N, K);
  return (int)hipGetLastError();
}

extern "C" int sat_bottleneck_fused_supported(int H, int W, int Cin, int Cmid, int dtype) {
  return dtype == SAT_BF16 && ((H == 14 && W == 14 && Cin == 1024 && Cmid == 256) ||
                               (H == 28 && W == 28 && Cin == 512 && Cmid == 128));
}

extern "C" int sat_bottleneck_fused(int N, int H, int W, int Cin, int Cmid, int dtype, const void* x, const void* w1f,
                                    const float* b1, const void* w2f, const float* b2, const void* w3f,
                                    const float* b3, void* y, const SatPolicy* policy, void* stream) {
  SAT_REQUIRE(N > 0 && x && w1f && w2f && w3f && b1 && b2 && b3 && y && x != y);
  SAT_REQUIRE(sat_bottleneck_fused_supported(H, W, Cin, Cmid, dtype));
  {   // 32-bit buffer offsets (the input resource, sat_out_rsrc's 2 GiB cap on the output): image chunks below 2 GiB
    const long img = 2L * H * W * Cin;
    const int cap = (int)(((1L << 31) - 1) / img);
    if (N > cap) {
      for (int n0 = 0; n0 < N; n0 += cap) {
        const int rc = sat_bottleneck_fused(N - n0 < cap ? N - n0 : cap, H, W, Cin, Cmid, dtype,
                                            (const char*)x + n0 * img, w1f, b1, w2f, b2, w3f, b3, (char*)y + n0 * img,
                                            policy, stream);
        if (rc) return rc;
      }
      return 0;
    }
  }
  SatPolicyScope scope(policy);
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  SAT_REQUIRE(al(x, 16) && al(y, 16) && al(w1f, 16) && al(w2f, 16) && al(w3f, 16) && al(b1, 16) && al(b2, 16) &&
              al(b3, 16));
  const long x_bytes = 2L * N * H * W * Cin;
  SAT_REQUIRE(x_bytes < (1L << 31));
  KArgs a{};
  a.x = (const bf16*)x; a.y = (bf16*)y;
  a.w1 = (const bf16*)w1f; a.w2 = (const bf16*)w2f; a.w3 = (const bf16*)w3f;
  a.b1 = b1; a.b2 = b2; a.b3 = b3;
  a.x_bytes = (unsigned)x_bytes;
  a.st = sat_launch_stamps();
  if (H == 28)   // layer2: 7-row bands, four workgroups per image
    hipLaunchKernelGGL(block_band_kernel, dim3(4 * N), dim3(512), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL((bottleneck_kernel<2, 0>), dim3(2 * N), dim3(512), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int sat_conv3x3_frag_supported(int H, int W, int C, int dtype) {
  return dtype == SAT_BF16 && ((H == 14 && W == 14 && (C == 256 || C == 512)) || (H == 28 && W == 28 && C == 128) ||
                               (H == 7 && W == 7 && C == 512) || (H == 112 && W == 112 && C == 128) ||
                               (H == 56 && W == 56 && C == 256));
}

extern "C" int sat_conv3x3_frag(int N, int H, int W, int C, int dtype, const void* x, const void* wf, const float* b,
                                void* y, const SatPolicy* policy, void* stream) {
  SAT_REQUIRE(N > 0 && x && wf && b && y && x != y);
  SAT_REQUIRE(sat_conv3x3_frag_supported(H, W, C, dtype));
  {   // image chunks whose input and output stay below 2 GiB (32-bit buffer offsets, sat_out_rsrc's cap)
    const long img = 2L * H * W * C;
    const int cap = (int)(((1L << 31) - 1) / img);
    if (N > cap) {
      for (int n0 = 0; n0 < N; n0 += cap) {
        const int rc = sat_conv3x3_frag(N - n0 < cap ? N - n0 : cap, H, W, C, dtype, (const char*)x + n0 * img, wf, b,
                                        (char*)y + n0 * img, policy, stream);
        if (rc) return rc;
      }
      return 0;
    }
  }
  SatPolicyScope scope(policy);
  const SatStamps st = sat_launch_stamps();
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  SAT_REQUIRE(al(x, 16) && al(y, 16) && al(wf, 16) && al(b, 16));
  const hipStream_t s = (hipStream_t)stream;
  const bf16 *xp = (const bf16*)x, *wp = (const bf16*)wf;
  bf16* yp = (bf16*)y;
  if (H == 7) {   // layer4 c2: whole images, two per workgroup (one at B <= 64), four 128-channel slices
    const int G = (sat_policy().conv_slices == 1 || (sat_policy().conv_slices != 2 && N > 64)) ? 2 : 1;
    const int groups = sat_cdiv(sat_cdiv(N, G), 8) * 8 * 4;
    if (G == 2)
      hipLaunchKernelGGL(conv3x3_img_kernel<2>, dim3(groups), dim3(512), 0, s, xp, wp, b, yp, N, st);
    else
      hipLaunchKernelGGL(conv3x3_img_kernel<1>, dim3(groups), dim3(512), 0, s, xp, wp, b, yp, N, st);
    return (int)hipGetLastError();
  }
  if (H == 112) {   // VGG19 block 2: 2-row bands
    hipLaunchKernelGGL(conv3x3_band112_kernel, dim3(56 * N), dim3(512), 0, s, xp, wp, b, yp, 56 * N, st);
    return (int)hipGetLastError();
  }
  if (H == 56) {   // VGG19 block 3: 2-row bands
    hipLaunchKernelGGL(conv3x3_band56_kernel, dim3(28 * N), dim3(512), 0, s, xp, wp, b, yp, 28 * N, st);
    return (int)hipGetLastError();
  }
  if (H == 14 && C == 512) {   // VGG19 block 5: half images x four 128-channel slices
    hipLaunchKernelGGL(conv3x3_half512_kernel, dim3(sat_cdiv(2 * N, 8) * 8 * 4), dim3(512), 0, s, xp, wp, b, yp, 2 * N, st);
    return (int)hipGetLastError();
  }
  if (H == 28) {   // layer2 c2: 7-row bands, four workgroups per image
    hipLaunchKernelGGL(conv3x3_band4w_kernel<1>, dim3(4 * N), dim3(256), 0, s, xp, wp, b, yp, 4 * N, st);
    return (int)hipGetLastError();
  }
  // layer3 c2: half images (two workgroups per image), or two channel slices per half image when the half
  // images alone would leave CUs idle (SatPolicy::conv_slices)
#ifdef SAT_C2_FORCE_SLICES   // diagnostics builds: layer3 c2 in the given form whatever the batch
  const int mode = SAT_C2_FORCE_SLICES;
#else
  const int mode = sat_frag_slices(N);
#endif
  const int groups = sat_cdiv(2 * N, 8) * 8 * 2;   // whole groups of 8 half images x 2 slices
  if (mode == 1)
    hipLaunchKernelGGL(conv3x3_frag_kernel<SAT_C2_PF>, dim3(2 * N), dim3(512), 0, s, xp, wp, b, yp, st);
  else
    hipLaunchKernelGGL(conv3x3_slice2_kernel, dim3(groups), dim3(256), 0, s, xp, wp, b, yp, 2 * N, st);
  return (int)hipGetLastError();
}

extern "C" int sat_conv1x1_frag_supported(int H, int W, int Cin, int Cout, int dtype) {
  return dtype == SAT_BF16 && H == 14 && W == 14 && Cin == 1024 && Cout == 256;
}

extern "C" int sat_conv1x1_frag(int N, int H, int W, int Cin, int Cout, int dtype, const void* x, const void* wf,
                                const float* b, void* y, const SatPolicy* policy, void* stream) {
  SAT_REQUIRE(N > 0 && x && wf && b && y && x != y);
  SAT_REQUIRE(sat_conv1x1_frag_supported(H, W, Cin, Cout, dtype));
  {   // image chunks whose input and output stay below 2 GiB (32-bit buffer offsets, sat_out_rsrc's cap)
    const long img = 2L * H * W * (Cin > Cout ? Cin : Cout);
    const int cap = (int)(((1L << 31) - 1) / img);
    if (N > cap) {
      for (int n0 = 0; n0 < N; n0 += cap) {
        const int rc = sat_conv1x1_frag(N - n0 < cap ? N - n0 : cap, H, W, Cin, Cout, dtype,
                                        (const char*)x + 2L * n0 * H * W * Cin, wf, b, (char*)y + 2L * n0 * H * W * Cout,
                                        policy, stream);
        if (rc) return rc;
      }
      return 0;
    }
  }
  SatPolicyScope scope(policy);
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  SAT_REQUIRE(al(x, 16) && al(y, 16) && al(wf, 16) && al(b, 16));
  const long x_bytes = 2L * N * H * W * Cin;
  SAT_REQUIRE(x_bytes < (1L << 31));
  if (sat_frag_slices(N) == 1)
    hipLaunchKernelGGL(conv1x1_frag_kernel, dim3(2 * N), dim3(512), 0, (hipStream_t)stream, (const bf16*)x,
                       (const bf16*)wf, b, (bf16*)y, (unsigned)x_bytes, sat_launch_stamps());
  else
    hipLaunchKernelGGL(conv1x1_frag2_kernel, dim3(sat_cdiv(2 * N, 8) * 8 * 2), dim3(512), 0, (hipStream_t)stream,
                       (const bf16*)x, (const bf16*)wf, b, (bf16*)y, (unsigned)x_bytes, 2 * N, sat_launch_stamps());
  return (int)hipGetLastError();
}
