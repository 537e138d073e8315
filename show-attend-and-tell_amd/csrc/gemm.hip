// MFMA GEMM and implicit-GEMM convolution for gfx950.
//
// One kernel template serves every matrix product of the hot path:
//   * nn.Linear forward / input-grad / weight-grad of the decoder
//     (attention.py:15-16, decoder.py:99,115,125,143-158 and their backward),
//   * the VGG19 / ResNet152 convolutions (encoder.py:33-40) as implicit GEMM
//     over NHWC activations (A loader does the im2col on the fly; no buffer).
//
// Tiles: 256 threads = 4 waves in a 2x2 layout, each wave owns a (BM/2)x(BN/2)
// block of 16x16 MFMA tiles.  bf16 operands use v_mfma_f32_16x16x32_bf16
// (BK=32), fp32 operands use the exact-fp32 v_mfma_f32_16x16x4_f32 (BK=16).
// Global -> registers (16-B loads) -> LDS (double buffered, padded rows) ->
// fragments; the epilogue fuses bias, an addend matrix (residual / precomputed
// gate terms), beta*C accumulation, activation and an optional second output.
#include "sat_common.h"
#include "sat_internal.h"

#include <type_traits>

namespace {

template <typename T> struct Cfg;
template <> struct Cfg<float> { static constexpr int BK = 16, VEC = 4, PAD = 4; };
template <> struct Cfg<bf16> { static constexpr int BK = 32, VEC = 8, PAD = 8; };

struct KArgs {
  int M, N, K;
  const void* A; long lda;
  const void* B; long ldb;
  void* C; long ldc; int c_dtype;
  float alpha, beta;
  const float* bias;
  const void* add1; long ld_add1; int add1_dtype;
  int act;
  void* aux; long ld_aux; int aux_dtype;
  long sA, sB, sC, s_add1, s_aux;
  SatConvGeom cv;
  int vecA, vecB;
  int splitk, kchunk;   // split-K: blockIdx.z = batch*splitk + split; K range [split*kchunk, +kchunk)
  int partial; long split_stride;   // partial-output split-K (plain stores into per-split slabs)
};

union Vec16 {
  uint4 u;
  float f[4];
  bf16 h[8];
};

// AMODE 0: A[m*lda+k]   AMODE 1: A[k*lda+m]   AMODE 2: implicit im2col of NHWC input
template <typename T, int BM, int BN, int AMODE, bool TB>
__global__ __launch_bounds__(256) void gemm_kernel(KArgs a) {
  constexpr int BK = Cfg<T>::BK, VEC = Cfg<T>::VEC, LDK = BK + Cfg<T>::PAD;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NJ = WN / 16;
  constexpr int NA = BM * BK / VEC / 256, NB = BN * BK / VEC / 256;
  static_assert(NA >= 1 && NB >= 1, "tile too small for 256 threads");
  __shared__ __attribute__((aligned(16))) T As[2][BM][LDK];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN][LDK];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const long z = blockIdx.z / a.splitk;
  const int split = blockIdx.z - (int)z * a.splitk;
  const T* Ag = (const T*)a.A + z * a.sA;
  const T* Bg = (const T*)a.B + z * a.sB;
  const int M = a.M, N = a.N;
  const int kbeg = split * a.kchunk;
  const int K = min(a.K, kbeg + a.kchunk);   // loaders treat K as the (exclusive) end of this split

  Vec16 ra[NA], rb[NB];
  int cv_pix[NA], cv_ih[NA], cv_iw[NA];
  if constexpr (AMODE == 2) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int v = tid + i * 256;
      int row = m0 + v / (BK / VEC);
      if (row < M) {
        int ohw = a.cv.OH * a.cv.OW;
        int n = row / ohw, rem = row - n * ohw;
        int oh = rem / a.cv.OW, ow = rem - oh * a.cv.OW;
        cv_pix[i] = n * a.cv.H * a.cv.W;
        cv_ih[i] = oh * a.cv.stride - a.cv.pad;
        cv_iw[i] = ow * a.cv.stride - a.cv.pad;
      } else {
        cv_pix[i] = -1; cv_ih[i] = 0; cv_iw[i] = 0;
      }
    }
  }

  auto load_a = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int v = tid + i * 256;
      if constexpr (AMODE == 1) {
        int kr = v / (BM / VEC), mc = (v % (BM / VEC)) * VEC;
        int k = k0 + kr, m = m0 + mc;
        if (k < K && m + VEC <= M && a.vecA) {
          ra[i].u = *(const uint4*)(Ag + (long)k * a.lda + m);
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            ((T*)&ra[i])[j] = (k < K && m + j < M) ? Ag[(long)k * a.lda + m + j] : (T)0.0f;
        }
      } else {
        int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
        int row = m0 + r, k = k0 + kc;
        if constexpr (AMODE == 0) {
          if (row < M && k + VEC <= K && a.vecA) {
            ra[i].u = *(const uint4*)(Ag + (long)row * a.lda + k);
          } else {
#pragma unroll
            for (int j = 0; j < VEC; ++j)
              ((T*)&ra[i])[j] = (row < M && k + j < K) ? Ag[(long)row * a.lda + k + j] : (T)0.0f;
          }
        } else {
          // implicit im2col: k -> (kh, kw, ci); C % VEC == 0 so a vector stays in one tap
          bool ok = cv_pix[i] >= 0 && k < K;
          long off = 0;
          if (ok) {
            int tap = k / a.cv.C, ci = k - tap * a.cv.C;
            int kh = tap / a.cv.KW, kw = tap - kh * a.cv.KW;
            int ih = cv_ih[i] + kh, iw = cv_iw[i] + kw;
            ok = (unsigned)ih < (unsigned)a.cv.H && (unsigned)iw < (unsigned)a.cv.W;
            off = ((long)cv_pix[i] + (long)ih * a.cv.W + iw) * a.cv.C + ci;
          }
          if (ok) ra[i].u = *(const uint4*)(Ag + off);
          else ra[i].u = make_uint4(0, 0, 0, 0);
        }
      }
    }
  };

  auto load_b = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int v = tid + i * 256;
      if constexpr (TB) {
        int kr = v / (BN / VEC), nc = (v % (BN / VEC)) * VEC;
        int k = k0 + kr, n = n0 + nc;
        if (k < K && n + VEC <= N && a.vecB) {
          rb[i].u = *(const uint4*)(Bg + (long)k * a.ldb + n);
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            ((T*)&rb[i])[j] = (k < K && n + j < N) ? Bg[(long)k * a.ldb + n + j] : (T)0.0f;
        }
      } else {
        int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
        int n = n0 + r, k = k0 + kc;
        if (n < N && k + VEC <= K && a.vecB) {
          rb[i].u = *(const uint4*)(Bg + (long)n * a.ldb + k);
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            ((T*)&rb[i])[j] = (n < N && k + j < K) ? Bg[(long)n * a.ldb + k + j] : (T)0.0f;
        }
      }
    }
  };

  auto store_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int v = tid + i * 256;
      if constexpr (AMODE == 1) {
        int kr = v / (BM / VEC), mc = (v % (BM / VEC)) * VEC;
#pragma unroll
        for (int j = 0; j < VEC; ++j) As[buf][mc + j][kr] = ((T*)&ra[i])[j];
      } else {
        int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
        *(uint4*)&As[buf][r][kc] = ra[i].u;
      }
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int v = tid + i * 256;
      if constexpr (TB) {
        int kr = v / (BN / VEC), nc = (v % (BN / VEC)) * VEC;
#pragma unroll
        for (int j = 0; j < VEC; ++j) Bs[buf][nc + j][kr] = ((T*)&rb[i])[j];
      } else {
        int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
        *(uint4*)&Bs[buf][r][kc] = rb[i].u;
      }
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    if constexpr (std::is_same<T, bf16>::value) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 af[MI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i)
          af[i] = *(const bf16x8*)&As[buf][wm * WM + i * 16 + (lane & 15)][ks * 32 + 8 * (lane >> 4)];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          bfr[j] = *(const bf16x8*)&Bs[buf][wn * WN + j * 16 + (lane & 15)][ks * 32 + 8 * (lane >> 4)];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        float af[MI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = As[buf][wm * WM + i * 16 + (lane & 15)][ks * 4 + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = Bs[buf][wn * WN + j * 16 + (lane & 15)][ks * 4 + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  const int nk = K > kbeg ? (K - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_a(kbeg); load_b(kbeg);
    store_a(0); store_b(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) { load_a(kbeg + (kt + 1) * BK); load_b(kbeg + (kt + 1) * BK); }
      compute(cur);
      if (more) { store_a(cur ^ 1); store_b(cur ^ 1); }
      __syncthreads();
    }
  }

  // ---- epilogue ----
  const void* add1 = a.add1 ? (const char*)a.add1 + z * a.s_add1 * (a.add1_dtype == SAT_BF16 ? 2 : 4) : nullptr;
  if (a.splitk > 1 && a.partial) {
    float* Cg = (float*)a.C + (long)split * a.split_stride;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn * WN + j * 16 + (lane & 15);
        if (col >= N) continue;
        const float bcol = (split == 0 && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          if (row >= M) continue;
          float v = a.alpha * acc[i][j][r] + bcol;
          if (split == 0 && add1) v += ld_as_f32(add1, (long)row * a.ld_add1 + col, a.add1_dtype);
          Cg[(long)row * a.ldc + col] = v;
        }
      }
    return;
  }
  if (a.splitk > 1) {
    // split-K: fp32 atomic accumulation into C (pre-zeroed by the host when beta == 0);
    // split 0 also contributes bias + add1.  Host guarantees act == NONE, fp32 C, no aux.
    float* Cg = (float*)a.C + z * a.sC;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn * WN + j * 16 + (lane & 15);
        if (col >= N) continue;
        const float bcol = (split == 0 && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          if (row >= M) continue;
          float v = a.alpha * acc[i][j][r] + bcol;
          if (split == 0 && add1) v += ld_as_f32(add1, (long)row * a.ld_add1 + col, a.add1_dtype);
          atomicAdd(Cg + (long)row * a.ldc + col, v);
        }
      }
    return;
  }
  auto epi = [&](auto* Cg, auto* auxg) {
    using CT = typename std::remove_pointer<decltype(Cg)>::type;
    using XT = typename std::remove_pointer<decltype(auxg)>::type;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn * WN + j * 16 + (lane & 15);
        if (col >= N) continue;
        const float bcol = a.bias ? a.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          if (row >= M) continue;
          float v = a.alpha * acc[i][j][r] + bcol;
          if (add1) v += ld_as_f32(add1, (long)row * a.ld_add1 + col, a.add1_dtype);
          const long ci = (long)row * a.ldc + col;
          if (a.beta != 0.f) v += a.beta * (float)Cg[ci];
          v = apply_act(v, a.act);
          Cg[ci] = (CT)v;
          if (auxg) auxg[(long)row * a.ld_aux + col] = (XT)v;
        }
      }
    }
  };
  char* Cb = (char*)a.C + z * a.sC * (a.c_dtype == SAT_BF16 ? 2 : 4);
  char* Xb = a.aux ? (char*)a.aux + z * a.s_aux * (a.aux_dtype == SAT_BF16 ? 2 : 4) : nullptr;
  if (a.c_dtype == SAT_BF16) {
    if (a.aux_dtype == SAT_BF16) epi((bf16*)Cb, (bf16*)Xb);
    else epi((bf16*)Cb, (float*)Xb);
  } else {
    if (a.aux_dtype == SAT_BF16) epi((float*)Cb, (bf16*)Xb);
    else epi((float*)Cb, (float*)Xb);
  }
}

template <typename T, int BM, int BN, int AMODE, bool TB>
int launch_cfg(const KArgs& k, int batch, hipStream_t s) {
  dim3 grid(sat_cdiv(k.N, BN), sat_cdiv(k.M, BM), batch * k.splitk);
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, AMODE, TB>), grid, dim3(256), 0, s, k);
  return (int)hipGetLastError();
}

template <typename T, int AMODE, bool TB>
int launch_tiles(const KArgs& k, int batch, hipStream_t s) {
  long t128 = (long)sat_cdiv(k.M, 128) * sat_cdiv(k.N, 128) * batch * k.splitk;
  long t64x128 = (long)sat_cdiv(k.M, 64) * sat_cdiv(k.N, 128) * batch * k.splitk;
  if (k.splitk == 1 && t128 >= 240) return launch_cfg<T, 128, 128, AMODE, TB>(k, batch, s);
  if (k.splitk == 1 && t64x128 >= 240) return launch_cfg<T, 64, 128, AMODE, TB>(k, batch, s);
  return launch_cfg<T, 64, 64, AMODE, TB>(k, batch, s);
}

template <typename T>
int launch_t(const KArgs& k, int amode, int tb, int batch, hipStream_t s) {
  if (amode == 2) return launch_tiles<T, 2, false>(k, batch, s);
  if (amode == 1) return tb ? launch_tiles<T, 1, true>(k, batch, s) : launch_tiles<T, 1, false>(k, batch, s);
  return tb ? launch_tiles<T, 0, true>(k, batch, s) : launch_tiles<T, 0, false>(k, batch, s);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

int sat_gemm_launch(const SatGemm& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return 0;
  SAT_REQUIRE(g.K >= 0 && g.A && g.B && g.C);
  SAT_REQUIRE(g.dtype == SAT_F32 || g.dtype == SAT_BF16);
  {
    int err = 0;
    if (sat_skinny_try(g, s, &err)) return err;
    if (sat_conv3x3_ws_try(g, s, &err)) return err;
    if (sat_conv_stream_try(g, s, &err)) return err;
    if (sat_conv_pipe_try(g, s, &err)) return err;
    if (sat_split_gemm_try(g, s, &err)) return err;
    if (sat_fast_gemm_try(g, s, &err)) return err;
  }
  const int vec = g.dtype == SAT_BF16 ? 8 : 4;
  KArgs k{};
  k.M = g.M; k.N = g.N; k.K = g.K;
  k.A = g.A; k.lda = g.lda; k.B = g.B; k.ldb = g.ldb;
  k.C = g.C; k.ldc = g.ldc; k.c_dtype = g.c_dtype;
  k.alpha = g.alpha; k.beta = g.beta; k.bias = g.bias;
  k.add1 = g.add1; k.ld_add1 = g.ld_add1; k.add1_dtype = g.add1_dtype;
  k.act = g.act; k.aux = g.aux; k.ld_aux = g.ld_aux; k.aux_dtype = g.aux_dtype;
  k.sA = g.sA; k.sB = g.sB; k.sC = g.sC; k.s_add1 = g.s_add1; k.s_aux = g.s_aux;
  k.cv = g.conv;
  int amode = g.conv.C > 0 ? 2 : (g.transA ? 1 : 0);
  if (amode == 2) {
    SAT_REQUIRE(g.conv.C % vec == 0 && aligned16(g.A));
    SAT_REQUIRE(g.K == g.conv.KH * g.conv.KW * g.conv.C);
    SAT_REQUIRE(g.M == g.conv.N * g.conv.OH * g.conv.OW);
    k.vecA = 1;
  } else {
    k.vecA = aligned16(g.A) && (g.lda % vec == 0) && (g.batch == 1 || g.sA % vec == 0);
  }
  k.vecB = aligned16(g.B) && (g.ldb % vec == 0) && (g.batch == 1 || g.sB % vec == 0);
  // split-K for skinny problems that cannot fill 256 CUs with 64x64 tiles
  k.splitk = 1;
  k.kchunk = g.K > 0 ? g.K : 1;
  k.partial = 0; k.split_stride = 0;
  const int bk = g.dtype == SAT_BF16 ? 32 : 16;
  if (g.partial_splits > 1) {
    SAT_REQUIRE(g.act == SAT_ACT_NONE && g.c_dtype == SAT_F32 && g.aux == nullptr && g.beta == 0.f &&
                g.batch == 1 && amode != 2);
    k.partial = 1; k.split_stride = g.split_stride;
    k.splitk = g.partial_splits;
    k.kchunk = sat_cdiv(sat_cdiv(g.K > 0 ? g.K : 1, g.partial_splits), bk) * bk;
    if (g.dtype == SAT_BF16) return launch_t<bf16>(k, amode, g.transB, g.batch, s);
    return launch_t<float>(k, amode, g.transB, g.batch, s);
  }
  const long tiles64 = (long)sat_cdiv(g.M, 64) * sat_cdiv(g.N, 64) * g.batch;
  const bool can_split = g.act == SAT_ACT_NONE && g.c_dtype == SAT_F32 && g.aux == nullptr &&
                         (g.beta == 0.f || g.beta == 1.f) && amode != 2 && g.batch == 1;
  // (bf16 only: the fp32 parity path stays deterministic)
  if (can_split && g.dtype == SAT_BF16 && tiles64 < 200 && g.K >= 8 * bk) {
    int sk = (int)((400 + tiles64 - 1) / tiles64);
    sk = sk > 16 ? 16 : sk;
    const int max_by_k = g.K / (4 * bk);
    if (sk > max_by_k) sk = max_by_k;
    if (sk > 1) {
      int chunk = sat_cdiv(g.K, sk);
      chunk = sat_cdiv(chunk, bk) * bk;
      k.kchunk = chunk;
      k.splitk = sat_cdiv(g.K, chunk);
      if (g.beta == 0.f) {
        SAT_CHECK((hipError_t)sat_zero_rows((float*)g.C, g.ldc, g.M, g.N, s));
      }
    }
  }
  if (g.dtype == SAT_BF16) return launch_t<bf16>(k, amode, g.transB, g.batch, s);
  return launch_t<float>(k, amode, g.transB, g.batch, s);
}

namespace {
thread_local const SatPolicy* t_policy = nullptr;
const SatPolicy k_default_policy{};
}  // namespace

const SatPolicy& sat_policy() { return t_policy ? *t_policy : k_default_policy; }

namespace {
thread_local SatStamps t_stamps{};
thread_local bool t_stamps_set = false;
}  // namespace
SatStamps sat_launch_stamps() {
  if (t_stamps_set) return t_stamps;
  return SatStamps{sat_policy().stamps, sat_policy().stamp_capacity};
}
SatStampScope::SatStampScope(uint64_t* p, int cap) : prev(t_stamps), prev_set(t_stamps_set) {
  t_stamps = SatStamps{p, cap};
  t_stamps_set = true;
}
SatStampScope::~SatStampScope() {
  t_stamps = prev;
  t_stamps_set = prev_set;
}
SatPolicyScope::SatPolicyScope(const SatPolicy* p) : prev(t_policy) { t_policy = p; }
SatPolicyScope::~SatPolicyScope() { t_policy = prev; }

extern "C" size_t sat_gemm_workspace_bytes(void) { return sat_split_gemm_ws_bytes(); }

extern "C" int sat_gemm(const SatGemmArgs* a, void* stream) {
  SAT_REQUIRE(a != nullptr);
  SatPolicyScope scope(a->policy);
  SatGemm g;
  if (a->workspace && a->workspace_bytes >= (int64_t)sat_split_gemm_ws_bytes()) {
    // [partial tiles | tickets]: the tickets are zeroed by the split launch itself (tickets_zeroed = 0)
    g.split_ws = (float*)a->workspace;
    g.split_ws_bytes = (long)(sat_split_gemm_ws_bytes() - kSatSplitTickets * 4);
    g.split_tickets = (unsigned*)((char*)a->workspace + g.split_ws_bytes);
  }
  g.M = a->M; g.N = a->N; g.K = a->K; g.dtype = a->dtype;
  g.A = a->A; g.lda = a->lda; g.transA = a->transA;
  g.B = a->B; g.ldb = a->ldb; g.transB = a->transB;
  g.C = a->C; g.ldc = a->ldc; g.c_dtype = a->c_dtype;
  g.alpha = a->alpha; g.beta = a->beta; g.bias = a->bias;
  g.add1 = a->add1; g.ld_add1 = a->ld_add1; g.add1_dtype = a->add1_dtype;
  g.act = a->act; g.aux = a->aux; g.ld_aux = a->ld_aux; g.aux_dtype = a->aux_dtype;
  return sat_gemm_launch(g, (hipStream_t)stream);
}

extern "C" int sat_conv2d_nhwc(const SatConvGeom* cg, int Cout, int dtype, const void* x, const void* w,
                               const float* bias, const void* residual, int relu, void* y, const SatPolicy* policy,
                               void* stream) {
  SAT_REQUIRE(cg != nullptr && x && w && y && Cout > 0);
  SatPolicyScope scope(policy);
  SatGemm g;
  g.conv = *cg;
  g.M = cg->N * cg->OH * cg->OW;
  g.N = Cout;
  g.K = cg->KH * cg->KW * cg->C;
  g.dtype = dtype;
  g.A = x; g.lda = 0;
  g.B = w; g.ldb = g.K; g.transB = 0;
  g.C = y; g.ldc = Cout; g.c_dtype = dtype;
  g.bias = bias;
  g.add1 = residual; g.ld_add1 = Cout; g.add1_dtype = dtype;
  g.act = relu ? SAT_ACT_RELU : SAT_ACT_NONE;
  return sat_gemm_launch(g, (hipStream_t)stream);
}
