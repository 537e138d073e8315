// Shared definitions for the Show-Attend-and-Tell MI355X (gfx950) kernels.
// Internal header: the public C-ABI lives in include/sat_hip.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/sat_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16;

#define SAT_CHECK(x)                                   \
  do {                                                 \
    hipError_t e__ = (x);                              \
    if (e__ != hipSuccess) return (int)e__;            \
  } while (0)
#define SAT_LAUNCH_CHECK() SAT_CHECK(hipGetLastError())
#define SAT_REQUIRE(cond)                              \
  do {                                                 \
    if (!(cond)) return SAT_ERR_INVALID;               \
  } while (0)

static inline int sat_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---- per-call kernel selection (SatPolicy, include/sat_hip.h) ----------------
// Every C-ABI entry point that dispatches among kernels installs its caller's policy for the duration
// of the call (SatPolicyScope); the dispatchers below it read sat_policy().  The state is per host
// thread and restored when the call returns, so it never outlives the call that set it.
const SatPolicy& sat_policy();
struct SatPolicyScope {
  const SatPolicy* prev;
  explicit SatPolicyScope(const SatPolicy* p);
  ~SatPolicyScope();
  SatPolicyScope(const SatPolicyScope&) = delete;
  SatPolicyScope& operator=(const SatPolicyScope&) = delete;
};

// ---- in-kernel launch timestamps (SatPolicy::stamps) ---------------------------
// A launch's stamp slot: p[0] = enable word (written by the host side between replays: a captured graph
// keeps its slots, so its stamps can be switched on for a diagnostic phase and off for the timed one),
// p[1] unused, then {start, end} of workgroup w at p[2 + 2 w], p[3 + 2 w] for w < cap.  Disabled, a
// launch costs one scalar load of the enable word per workgroup.
struct SatStamps {
  uint64_t* p = nullptr;
  int cap = 0;
};
struct SatStampT0 {
  uint64_t t0;
  bool on;
};
__device__ __forceinline__ SatStampT0 sat_stamp_begin(const SatStamps& st) {
  if (!st.p || st.p[0] == 0) return SatStampT0{0, false};   // uniform
  return SatStampT0{__builtin_amdgcn_s_memrealtime(), true};
}
// every wave of the workgroup has finished its work (barrier), then one lane records {start, end}
__device__ __forceinline__ void sat_stamp_end(const SatStamps& st, SatStampT0 t) {
  if (!t.on) return;   // uniform
  __syncthreads();
  const int w = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if (threadIdx.x == 0 && w < st.cap) {
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    *(ulonglong2*)(st.p + 2 + 2 * (long)w) = make_ulonglong2(t.t0, t1);
  }
}

// the stamp slots of the next launch: the innermost SatStampScope's (the decoder gives every per-step launch
// its own slot and none to the rest: p = nullptr), else the call's SatPolicy
SatStamps sat_launch_stamps();
struct SatStampScope {
  SatStamps prev;
  bool prev_set;
  SatStampScope(uint64_t* p, int cap);
  ~SatStampScope();
  SatStampScope(const SatStampScope&) = delete;
  SatStampScope& operator=(const SatStampScope&) = delete;
};
// ---- scalar load/store helpers for the two storage dtypes -------------------
__device__ __forceinline__ float ld_as_f32(const void* p, long i, int dt) {
  return dt == SAT_BF16 ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void st_from_f32(void* p, long i, int dt, float v) {
  if (dt == SAT_BF16) ((bf16*)p)[i] = (bf16)v;
  else ((float*)p)[i] = v;
}
template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

__device__ __forceinline__ float sat_sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case SAT_ACT_RELU: return v > 0.f ? v : 0.f;
    case SAT_ACT_TANH: return tanhf(v);
    case SAT_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}

// ---- output stores with a cache policy ------------------------------------------------
// The big activation writers store through a buffer resource over their output tensor so the cache policy can be
// chosen: SAT_OUT_CPOL 16 = sc1, write-through -- the line leaves the XCD's L2 clean (MI355X_MICROARCH.md, "stores of
// each flavour"), so the end-of-kernel L2 writeback of every kernel running beside it (the decoder's per-step
// chain beside the encoder) has fewer dirty lines to flush (measured: 6.51-6.57 -> 6.46-6.47 ms per step,
// profiles/r4_s13).  0 = plain write-back stores (diagnostics builds).
#ifndef SAT_OUT_CPOL
#define SAT_OUT_CPOL 16
#endif
#ifndef SAT_OUT8_CPOL   // the 8-B stores of the staged-input conv kernels (sc1 dwordx2: a fabric write per lane)
#define SAT_OUT8_CPOL 0
#endif
typedef unsigned sat_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned sat_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sat_out_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}
// loads through a buffer resource: an offset past the resource's bytes reads zeros, so a guarded load needs no
// exec-masked branch (whose register copies can make the compiler wait for a load right after issuing it)
constexpr unsigned kSatOOB = 0x80000000u;   // an offset no resource covers (num_records < 2^31)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sat_in_rsrc(const void* base, long bytes) { return sat_out_rsrc(base, bytes); }
__device__ __forceinline__ uint4 sat_ld16(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  const sat_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 sat_ld16f(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  const uint4 u = sat_ld16(r, byte_off);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
__device__ __forceinline__ float sat_ld4f(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __uint_as_float((unsigned)__builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 0));
}
template <int CPOL = SAT_OUT_CPOL>
__device__ __forceinline__ void sat_st16(__amdgpu_buffer_rsrc_t r, unsigned byte_off, uint4 u) {
  __builtin_amdgcn_raw_buffer_store_b128(sat_u32x4{u.x, u.y, u.z, u.w}, r, (int)byte_off, 0, CPOL);
}
__device__ __forceinline__ void sat_st8(__amdgpu_buffer_rsrc_t r, unsigned byte_off, sat_u32x2 u) {
  __builtin_amdgcn_raw_buffer_store_b64(u, r, (int)byte_off, 0, SAT_OUT8_CPOL);
}

// 16-B stores from two C^T accumulators A, B of each lane that cover the same 4 channels group (n-blocks j, j + 1 of
// one pixel, or m-blocks i, i + 1 of one n-block): lanes fh and fh ^ 1 swap halves, so the even lane holds channels
// 4 fh .. 4 fh + 7 of A (its own A at offA) and the odd one 4 (fh - 1) .. 4 fh + 3 of B (its own B at offB): whole
// 16-B write-through stores (sat_common.h) instead of 8-B ones.  Every lane runs the exchange.
template <int CPOL = SAT_OUT_CPOL>
__device__ __forceinline__ void sat_st_pair16(__amdgpu_buffer_rsrc_t r, unsigned offA, unsigned offB, sat_u32x2 a, sat_u32x2 b,
                                          bool okA, bool okB) {
  const bool odd = (threadIdx.x >> 4) & 1;
  const sat_u32x2 send = odd ? a : b;
  const unsigned gx = (unsigned)__shfl_xor((int)send.x, 16, 64), gy = (unsigned)__shfl_xor((int)send.y, 16, 64);
  const uint4 u = odd ? make_uint4(gx, gy, b.x, b.y) : make_uint4(a.x, a.y, gx, gy);
  if (odd ? okB : okA) sat_st16<CPOL>(r, odd ? offB - 8 : offA, u);
}

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- internal GEMM descriptor (host side) -----------------------------------
// C[m,n] = act(alpha * sum_k A(m,k) B(n,k) + bias[n] + add1[m,n] + beta*C[m,n])
//   A(m,k): transA ? A[k*lda + m] : A[m*lda + k]   (conv: implicit im2col of NHWC input)
//   B(n,k): transB ? B[k*ldb + n] : B[n*ldb + k]
struct SatGemm {
  int M = 0, N = 0, K = 0;
  int dtype = SAT_F32;  // operand dtype of A and B
  const void* A = nullptr; long lda = 0; int transA = 0;
  const void* B = nullptr; long ldb = 0; int transB = 0;
  void* C = nullptr; long ldc = 0; int c_dtype = SAT_F32;
  float alpha = 1.f, beta = 0.f;
  const float* bias = nullptr;
  const void* add1 = nullptr; long ld_add1 = 0; int add1_dtype = SAT_F32;
  int act = SAT_ACT_NONE;
  void* aux = nullptr; long ld_aux = 0; int aux_dtype = SAT_BF16;
  int batch = 1; long sA = 0, sB = 0, sC = 0, s_add1 = 0, s_aux = 0;
  SatConvGeom conv{};  // conv.C > 0 selects the implicit-im2col A loader
  // partial-output split-K: split s writes its fp32 partial product to C + s*split_stride
  // (bias/add1 in split 0 only, act must be NONE); the consumer sums the slabs.
  int partial_splits = 0; long split_stride = 0;
  // A's contiguous dimension (M when transA, else K) is readable -- zero-padded -- up to the next
  // multiple of 8, so the 16-B DMA paths may take M % 8 / K % 8 != 0 (the decoder's padded d logits)
  int a_tail = 0;
  // beta = 0 and the caller has already zeroed C: an atomic split-K launch skips its own zeroing pass
  int c_zeroed = 0;
  // deterministic split-K of the fp32-output k-major products (gemmsplit.hip): partial tiles and one arrival
  // ticket per output tile; tickets_zeroed: the caller zeroed the tickets (else the launch does)
  float* split_ws = nullptr; long split_ws_bytes = 0;
  unsigned* split_tickets = nullptr;
  int tickets_zeroed = 0;
};

int sat_gemm_launch(const SatGemm& g, hipStream_t s);
// bf16 NT fast path (convgemm.hip); returns 1 when it launched (error code in *err).
int sat_fast_gemm_try(const SatGemm& g, hipStream_t s, int* err);
// pipelined bf16 GEMM with fp32 output, a k-major operand and deterministic split-K (gemmsplit.hip: the decoder's
// batched weight / input gradients); returns 1 when it launched.  sat_split_gemm_takes: it would take g;
// sat_split_gemm_ws_bytes: the workspace (partial tiles + tickets) its largest split needs.
int sat_split_gemm_try(const SatGemm& g, hipStream_t s, int* err);
int sat_split_gemm_takes(const SatGemm& g);
size_t sat_split_gemm_ws_bytes();
constexpr size_t kSatSplitTickets = 256;   // tickets one split launch may use
// 256x128 pipelined bf16 conv / NT GEMM (convpipe.hip); returns 1 when it launched.
int sat_conv_pipe_try(const SatGemm& g, hipStream_t s, int* err);
// weight-stationary streaming kernel for K <= 512 1x1 convs (convstream.hip); returns 1 when it launched.
int sat_conv_stream_try(const SatGemm& g, hipStream_t s, int* err);
// register-direct skinny GEMM (M <= 128, NT, fp32 / partial-slab output: the decoder's per-step
// products, skinny.hip); returns 1 when it launched.
int sat_skinny_try(const SatGemm& g, hipStream_t s, int* err);
int sat_skinny_splits(int M, int N, int K);
// weight-stationary 3x3 / stride-1 conv, 64 -> 64 channels, W 56 or 224 (conv3x3ws.hip); returns 1 when it launched.
int sat_conv3x3_ws_try(const SatGemm& g, hipStream_t s, int* err);   // partial splits the skinny kernel prefers (0 = not eligible)
