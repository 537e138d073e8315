// nn.LSTMCell pointwise part (decoder.py:115) forward/backward, plus the small
// elementwise pieces of the decoder: dropout (decoder.py:121-125), the advanced
// deep-output combine/split (decoder.py:149-158), tanh-init backward
// (decoder.py:137-147).  The gate GEMMs themselves run on MFMA (gemm.hip); the
// partial gate sums meet here so no [B,4E] sum is materialised.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

inline int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

// the dropout keep bit of element (b, t, e) drawn from the seed (dropout_kernel and the fused forms share it)
__device__ __forceinline__ uint8_t dropout_keep(uint64_t seed, int b, int t, int e) {
  return (uint8_t)(mix32(seed * 0x9E3779B97F4A7C15ULL + (((uint64_t)b << 40) ^ ((uint64_t)t << 20) ^ (uint64_t)e)) & 1u);
}

// Gate-parallel forward: a 256-thread block covers 64 units; thread (q, u) sums gate q of unit u
// over its split-K slabs (4x the loads in flight of a unit-per-thread kernel: 9.5 -> 5.7 us per
// step at B=128, E=512, 4 + 8 slabs), the cell update reads the four gates back from LDS.
// GREEDY: the fused greedy step's extras (dropout of h into hd_t, the token fold), compiled out of the teacher-forced
// instance (with them in, its span went 3.5-3.7 -> 4.2 us per step, profiles/r6_s5 vs r6_s2)
// HS, CS: the h and context products' split counts when compile-time (CS = 0 with HS > 0: no context part); HS = 0:
// any counts, looped sums
template <typename T, bool GREEDY, int HS, int CS>
__device__ __forceinline__ void lstm_fwd_gp_kernel_body(LstmFwdArgs a) {
  __shared__ float sg[4][64];
  __shared__ float am_v[4];
  __shared__ int am_i[4];
  const int E = a.E;
  const int q = threadIdx.x >> 6, u = threadIdx.x & 63;
  const long units = (long)a.B * E;
  for (long base = (long)blockIdx.x * 64; base < units; base += (long)gridDim.x * 64) {
    const long i = base + u;
    const bool ok = i < units;
    const int b = ok ? (int)(i / E) : 0, j = ok ? (int)(i - (long)b * E) : 0;
    // every load this thread needs is requested here (HS / CS > 0: the products' split counts, compile-time, so
    // the slab loads are unconditional and branch-free; buffer loads, a guarded-off one reads zeros): the gate's x
    // part, its split-K slabs of the h and context products (summed after they arrive, in sum_parts's order), and
    // c_prev for the cell update after the barrier -- one memory round trip where the looped slab sums and the
    // post-barrier c_prev load took several.  HS = 0: the looped sums (any split count).
    const bool xt_mode = GREEDY && a.am_val;
    const __amdgpu_buffer_rsrc_t rX = sat_in_rsrc(a.xpart, ((long)(a.B - 1) * a.xpart_ld + 4L * E) * 4);
    const __amdgpu_buffer_rsrc_t rH =
        sat_in_rsrc(a.hpart, ((long)(HS > 1 ? HS - 1 : 0) * a.h_split_stride + (long)(a.B - 1) * a.hpart_ld + 4L * E) * 4);
    const __amdgpu_buffer_rsrc_t rC =
        sat_in_rsrc(a.cpart, ((long)(CS > 1 ? CS - 1 : 0) * a.c_split_stride + (long)(a.B - 1) * a.cpart_ld + 4L * E) * 4);
    const __amdgpu_buffer_rsrc_t rP = sat_in_rsrc(a.c_prev, ((long)(a.B - 1) * a.c_prev_ld + E) * 4);
    const long gi = (long)q * E + j;   // the gate's column
    float xv = sat_ld4f(rX, ok && !xt_mode ? (unsigned)(((long)b * a.xpart_ld + gi) * 4) : kSatOOB);
    float hp[HS > 0 ? HS : 1], cpv[CS > 0 ? CS : 1];
#pragma unroll
    for (int p = 0; p < HS; ++p)
      hp[p] = sat_ld4f(rH, ok ? (unsigned)(((long)b * a.hpart_ld + gi + p * a.h_split_stride) * 4) : kSatOOB);
#pragma unroll
    for (int p = 0; p < CS; ++p)
      cpv[p] = sat_ld4f(rC, ok ? (unsigned)(((long)b * a.cpart_ld + gi + p * a.c_split_stride) * 4) : kSatOOB);
    const float cprev = sat_ld4f(rP, ok && q == 0 ? (unsigned)(((long)b * a.c_prev_ld + j) * 4) : kSatOOB);
    int id = 0;
    if (GREEDY && a.am_val) {   // the token fold: the block's 64 units share one row (E % 64 == 0)
      const int br = (int)(base / E);
      float best = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = threadIdx.x; c < a.am_ncb; c += blockDim.x) {
        const float x = a.am_val[(long)c * a.B + br];
        const int xi = a.am_idx[(long)c * a.B + br];
        if (sat_argmax_better(x, xi, best, bi)) { best = x; bi = xi; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (sat_argmax_better(ov, oi, best, bi)) { best = ov; bi = oi; }
      }
      if (u == 0) { am_v[q] = best; am_i[q] = bi; }
      __syncthreads();
      best = am_v[0]; bi = am_i[0];
#pragma unroll
      for (int w = 1; w < 4; ++w)
        if (sat_argmax_better(am_v[w], am_i[w], best, bi)) { best = am_v[w]; bi = am_i[w]; }
      id = (bi < 0 || bi >= a.am_V) ? 0 : bi;
      if (ok) xv = a.xt[(long)id * 4 * E + q * E + j];
    }
    if (ok) {
      float v = xv + (HS > 0 ? sum_loaded_parts(hp, HS)
                             : sum_parts(a.hpart, (long)b * a.hpart_ld + q * E + j, a.h_splits, a.h_split_stride));
      if (CS > 0) v += sum_loaded_parts(cpv, CS);
      else if (HS == 0 && a.cpart) v += sum_parts(a.cpart, (long)b * a.cpart_ld + q * E + j, a.c_splits, a.c_split_stride);
      sg[q][u] = v;
      a.gates[(long)b * a.gates_ld + q * E + j] = v;
    }
    __syncthreads();
    if (q == 0 && ok) {
      float c, h;
      lstm_cell_fwd(sg[0][u], sg[1][u], sg[2][u], sg[3][u], cprev, c, h);
      a.c_out[(long)b * a.c_out_ld + j] = c;
      if (a.c_next_in) a.c_next_in[(long)b * a.c_next_in_ld + j] = c;
      a.h_out[(long)b * a.h_out_ld + j] = h;
      if (a.h_out_t) ((T*)a.h_out_t)[(long)b * a.h_out_t_ld + j] = (T)h;
      if (a.h_next_in_t) ((T*)a.h_next_in_t)[(long)b * a.h_next_in_t_ld + j] = (T)h;
      if (GREEDY && a.hd_t) {   // dropout(h) for the greedy step's head: dropout_kernel's arithmetic
        float y = h;
        if (a.drop_training) {
          uint8_t keep;
          if (a.drop_has_mask) {
            keep = a.mask_in[(long)b * a.mask_ld + j];
          } else {
            const uint64_t seed = a.seed_ptr ? a.seed ^ (*a.seed_ptr * 0xD1B54A32D192ED03ULL) : a.seed;
            keep = dropout_keep(seed, b, a.drop_t, j);
          }
          if (a.mask_out) a.mask_out[(long)b * a.mask_ld + j] = keep;
          y = keep ? h * 2.f : 0.f;
        }
        ((T*)a.hd_t)[(long)b * a.hd_ld + j] = (T)y;
      }
      if (GREEDY && a.am_val) {   // the fed token's embedding row (the head's combine, the backward) and the token itself
        ((T*)a.emb_t)[(long)b * a.emb_t_ld + j] = (T)a.emb[(long)id * E + j];
        if (j == 0) a.tok_out[(long)b * a.tok_ld] = id;
      }
    }
    __syncthreads();
  }
}

template <typename T, bool GREEDY, int HS, int CS>
__global__ __launch_bounds__(256) void lstm_fwd_gp_kernel(LstmFwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  lstm_fwd_gp_kernel_body<T, GREEDY, HS, CS>(a);
  sat_stamp_end(a.st, t0);
}

// Gate-parallel backward (layout as lstm_fwd_gp_kernel): thread (q, u) loads gate q and the
// slabs s = q, q+4, ... of the recurrent dh; the four partial sums meet in LDS in a fixed order.
template <typename T>
__device__ __forceinline__ void lstm_bwd_gp_kernel_body(LstmBwdArgs a) {
  __shared__ float sg[4][64], sdh[4][64];
  const int E = a.E;
  const int q = threadIdx.x >> 6, u = threadIdx.x & 63;
  const long units = (long)a.B * E;
  for (long base = (long)blockIdx.x * 64; base < units; base += (long)gridDim.x * 64) {
    const long i = base + u;
    const bool ok = i < units;
    const int b = ok ? (int)(i / E) : 0, j = ok ? (int)(i - (long)b * E) : 0;
    // every load requested up front, branch-free (buffer loads; zeros past the resource): the gate, this thread's
    // recurrent-dh slabs s = q, q + 4, .. (summed in that order after they arrive), c_prev, c_new, dc, the head's dh
    // and its dropout mask
    constexpr int kQ = 4;   // slabs per thread requested up front (dh_splits <= 16; more: the looped sum)
    const int ds = a.dh_rec ? a.dh_splits : 0;
    const bool d_up = ds <= 4 * kQ;
    const __amdgpu_buffer_rsrc_t rG = sat_in_rsrc(a.gates, ((long)(a.B - 1) * a.gates_ld + 4L * E) * 4);
    const __amdgpu_buffer_rsrc_t rD =
        sat_in_rsrc(a.dh_rec, ((long)(ds > 0 ? ds - 1 : 0) * a.dh_split_stride + (long)(a.B - 1) * a.dh_rec_ld + E) * 4);
    const __amdgpu_buffer_rsrc_t rCp = sat_in_rsrc(a.c_prev, ((long)(a.B - 1) * a.c_prev_ld + E) * 4);
    const __amdgpu_buffer_rsrc_t rCn = sat_in_rsrc(a.c_new, ((long)(a.B - 1) * a.c_new_ld + E) * 4);
    const __amdgpu_buffer_rsrc_t rDc = sat_in_rsrc(a.dc, units * 4);
    const __amdgpu_buffer_rsrc_t rHh = sat_in_rsrc(a.dh_head, ((long)(a.B - 1) * a.dh_head_ld + E) * 4);
    const float gv = sat_ld4f(rG, ok ? (unsigned)(((long)b * a.gates_ld + q * E + j) * 4) : kSatOOB);
    float dp[kQ];
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
      const int sp = q + 4 * k;
      dp[k] = sat_ld4f(rD, ok && d_up && sp < ds ? (unsigned)(((long)b * a.dh_rec_ld + j + sp * a.dh_split_stride) * 4)
                                                 : kSatOOB);
    }
    float cp = sat_ld4f(rCp, ok ? (unsigned)(((long)b * a.c_prev_ld + j) * 4) : kSatOOB);
    float cn = sat_ld4f(rCn, ok ? (unsigned)(((long)b * a.c_new_ld + j) * 4) : kSatOOB);
    float dcin = sat_ld4f(rDc, ok && !a.dc_zero ? (unsigned)(i * 4) : kSatOOB);
    float hh = sat_ld4f(rHh, ok && a.dh_head ? (unsigned)(((long)b * a.dh_head_ld + j) * 4) : kSatOOB);
    const __amdgpu_buffer_rsrc_t rM = sat_in_rsrc(a.mask, (long)(a.B - 1) * a.mask_ld + E);
    const bool mk = __builtin_amdgcn_raw_buffer_load_b8(
                        rM, ok && a.dh_head && a.mask ? (int)((long)b * a.mask_ld + j) : (int)kSatOOB, 0, 0) != 0;
    if (ok) {
      sg[q][u] = gv;
      float p = 0.f;
      if (d_up) {
#pragma unroll
        for (int k = 0; k < kQ; ++k)
          if (q + 4 * k < ds) p += dp[k];
      } else {
        for (int sp = q; sp < ds; sp += 4) p += a.dh_rec[(long)b * a.dh_rec_ld + j + sp * a.dh_split_stride];
      }
      sdh[q][u] = p;
      if (a.dh_head && a.mask) hh = mk ? hh * 2.f : 0.f;
    }
    __syncthreads();
    if (ok) {
      const float dh = ((sdh[0][u] + sdh[1][u]) + (sdh[2][u] + sdh[3][u])) + hh;
      float d4[4], dco;
      lstm_cell_bwd(sg[0][u], sg[1][u], sg[2][u], sg[3][u], cp, cn, dcin, dh, d4, dco);
      const float dq = d4[q];
      a.d_gates[(long)b * a.d_gates_ld + q * E + j] = dq;
      if (a.d_gates_t) ((T*)a.d_gates_t)[(long)b * a.d_gates_t_ld + q * E + j] = (T)dq;
      if (q == 0) a.dc[i] = dco;
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(256) void lstm_bwd_gp_kernel(LstmBwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  lstm_bwd_gp_kernel_body<T>(a);
  sat_stamp_end(a.st, t0);
}

// d(tanh pre) for init_h / init_c: dpre[b, 0:E] = dh (1-h^2), dpre[b, E:2E] = dc (1-c^2)
template <typename T>
__global__ void tanh_pair_bwd_kernel(const float* dh, int dh_splits, long dh_split_stride, const float* dc,
                                     const float* hc0, int B, int E, float* dpre, T* dpre_t) {
  const long n = (long)B * 2 * E;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / (2 * E)), j = (int)(i - (long)b * 2 * E);
    const float y = hc0[i];
    const float d = j < E ? sum_parts(dh, (long)b * E + j, dh_splits, dh_split_stride) : dc[(long)b * E + (j - E)];
    const float v = d * (1.f - y * y);
    dpre[i] = v;
    if (dpre_t) dpre_t[i] = (T)v;
  }
}


// hd[b,t,e] = h[b,t,e] * keep * 2 (train) | h (eval); keep drawn from (seed, b, t, e) or given.
// Rows r = b*T1 + t of this call live at r*ld in h / mask / out (per-step calls pass T1 = 1 and
// the full-sequence row stride as ld; t_offset is then the step index).
template <typename T>
__global__ void dropout_kernel(const float* h, long h_ld, int B, int T1, int E, int training, int has_mask,
                               const uint8_t* mask_in, uint8_t* mask_out, long mask_ld, uint64_t seed,
                               const uint64_t* seed_ptr, int t_offset, T* out, long out_ld) {
  const long n = (long)B * T1 * E;
  if (seed_ptr) seed ^= *seed_ptr * 0xD1B54A32D192ED03ULL;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int e = (int)(i % E);
    const long r = i / E;
    const int b = (int)(r / T1), t = (int)(r - (long)b * T1) + t_offset;
    const float x = h[r * h_ld + e];
    float y = x;
    if (training) {
      uint8_t keep;
      if (has_mask) keep = mask_in[r * mask_ld + e];
      else keep = dropout_keep(seed, b, t, e);
      if (mask_out) mask_out[r * mask_ld + e] = keep;
      y = keep ? x * 2.f : 0.f;
    }
    out[r * out_ld + e] = (T)y;
  }
}

template <typename T>
__global__ void relu_mask_kernel(const T* d, const T* ref, long n, T* out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)ref[i] > 0.f ? d[i] : (T)0.0f;
}

// rows of cols elements (ld cols) -> rows of ld_out elements, zero past cols; optional ReLU mask
// from ref (same layout as d).  bf16 pairs when cols is even (4-B aligned rows).
template <bool MASK>
__global__ void pad_rows_bf16x2_kernel(const bf16* d, const bf16* ref, int rows, int cols, int ld_out, bf16* out) {
  const int c = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (c >= ld_out) return;
  for (long r = blockIdx.y; r < rows; r += gridDim.y) {
  unsigned v = 0u;   // two bf16: low half = column c
  if (c < cols) {
    v = *(const unsigned*)(d + r * cols + c);
    if constexpr (MASK) {
      const unsigned m = *(const unsigned*)(ref + r * cols + c);
      if (!(__uint_as_float(m << 16) > 0.f)) v &= 0xffff0000u;
      if (!(__uint_as_float(m & 0xffff0000u) > 0.f)) v &= 0x0000ffffu;
    }
  }
  *(unsigned*)(out + r * ld_out + c) = v;
  }
}
template <typename T>
__global__ void pad_rows_kernel(const T* d, const T* ref, int rows, int cols, int ld_out, T* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ld_out) return;
  for (long r = blockIdx.y; r < rows; r += gridDim.y) {
  T v = (T)0.0f;
  if (c < cols) {
    v = d[r * cols + c];
    if (ref && !((float)ref[r * cols + c] > 0.f)) v = (T)0.0f;
  }
  out[r * ld_out + c] = v;
  }
}

template <typename T>
__global__ void ado_split_kernel(const float* dcomb, const float* fh, const float* fz, long n, T* dfh, T* dfz) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = dcomb[i];
    dfh[i] = (T)(fh[i] > 0.f ? d : 0.f);
    dfz[i] = (T)(fz[i] > 0.f ? d : 0.f);
  }
}

// comb = fh + fz + emb   (fz already relu'd by its GEMM epilogue)
template <typename T>
__global__ void ado_combine_kernel(const float* fh, const float* fz, const T* emb, long n, T* comb) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    comb[i] = (T)(fh[i] + fz[i] + (float)emb[i]);
}

__global__ void bump_seed_kernel(uint64_t* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *p += 1;
}
}  // namespace
int sat_bump_seed(uint64_t* p, hipStream_t s) {
  hipLaunchKernelGGL(bump_seed_kernel, dim3(1), dim3(64), 0, s, p);
  return (int)hipGetLastError();
}
namespace {
__global__ void fill_kernel(float* p, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}

// Zero a [rows, cols] fp32 block with row stride ld.  Used instead of hipMemset(2D)Async: a
// memset node inside a replayed hipGraph left every fourth dword of large buffers unwritten on
// this stack when two graphs share the buffer (bench.py's two decoder graphs), so every
// beta = 0 atomic accumulation target is cleared by a kernel node instead.
__global__ void zero_rows_kernel(float* p, long ld, long rows, long cols) {
  const long stride = (long)gridDim.x * blockDim.x;
  if (ld == cols && ((uintptr_t)p & 15) == 0) {
    const long n = rows * cols, n4 = n >> 2;
    float4* p4 = reinterpret_cast<float4*>(p);
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long i = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0.f;
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows * cols; i += stride) p[(i / cols) * ld + i % cols] = 0.f;
}

template <typename T>
__global__ void broadcast_rows_kernel(const T* src, int B, int D, int T1, T* dst) {
  const long n = (long)B * T1 * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int b = (int)(i / ((long)T1 * D));
    dst[i] = src[(long)b * D + d];
  }
}

__global__ void row_sum_acc_kernel(const float* X, int R, int N, float* out) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += X[(long)r * N + n];
  out[n] += s;
}

}  // namespace

#define DISPATCH_T(dtype, KERNEL, grid, ...)                                                   \
  do {                                                                                       \
    if ((dtype) == SAT_BF16) hipLaunchKernelGGL(KERNEL<bf16>, grid, dim3(256), 0, s, __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<float>, grid, dim3(256), 0, s, __VA_ARGS__);               \
  } while (0)

// blocks of 64 units (256 threads) for B x E units: one per 64 units, capped at 4096 (the kernels stride over the
// rest)
inline long lstm_blocks(int B, int E) {
  const long blocks = ((long)B * E + 63) / 64;
  return blocks > 4096 ? 4096 : blocks;
}
template <typename T, bool GREEDY, int HS>
bool lstm_fwd_cs(int cs, dim3 grid, hipStream_t s, const LstmFwdArgs& a) {
  switch (cs) {   // the decoder's context-product split counts (0: no context part)
    case 0: hipLaunchKernelGGL((lstm_fwd_gp_kernel<T, GREEDY, HS, 0>), grid, dim3(256), 0, s, a); return true;
    case 1: hipLaunchKernelGGL((lstm_fwd_gp_kernel<T, GREEDY, HS, 1>), grid, dim3(256), 0, s, a); return true;
    case 2: hipLaunchKernelGGL((lstm_fwd_gp_kernel<T, GREEDY, HS, 2>), grid, dim3(256), 0, s, a); return true;
    case 4: hipLaunchKernelGGL((lstm_fwd_gp_kernel<T, GREEDY, HS, 4>), grid, dim3(256), 0, s, a); return true;
    case 8: hipLaunchKernelGGL((lstm_fwd_gp_kernel<T, GREEDY, HS, 8>), grid, dim3(256), 0, s, a); return true;
    default: return false;
  }
}
template <typename T, bool GREEDY>
void lstm_fwd_launch_t(dim3 grid, hipStream_t s, const LstmFwdArgs& a) {
  const int hs = a.h_splits < 1 ? 1 : a.h_splits, cs = a.cpart ? (a.c_splits < 1 ? 1 : a.c_splits) : 0;
  // the buffer resources of the compile-time forms address < 2 GiB
  const bool fits = ((long)(hs - 1) * a.h_split_stride + (long)a.B * a.hpart_ld) * 4 < 0x7fffffffL &&
                    (!a.cpart || ((long)(cs - 1) * a.c_split_stride + (long)a.B * a.cpart_ld) * 4 < 0x7fffffffL) &&
                    (a.xt || ((long)a.B * a.xpart_ld) * 4 < 0x7fffffffL);
  if (sizeof(T) == 2 && fits) {
    if (hs == 1 && lstm_fwd_cs<T, GREEDY, 1>(cs, grid, s, a)) return;
    if (hs == 2 && lstm_fwd_cs<T, GREEDY, 2>(cs, grid, s, a)) return;
  }
  hipLaunchKernelGGL((lstm_fwd_gp_kernel<T, GREEDY, 0, 0>), grid, dim3(256), 0, s, a);
}
int sat_lstm_fwd_launch(const LstmFwdArgs& args, hipStream_t s) {
  LstmFwdArgs a = args;
  a.st = sat_launch_stamps();
  const dim3 grid((unsigned)lstm_blocks(a.B, a.E));
  const bool greedy = a.hd_t || a.am_val;
  if (a.dtype == SAT_BF16) {
    if (greedy) lstm_fwd_launch_t<bf16, true>(grid, s, a);
    else lstm_fwd_launch_t<bf16, false>(grid, s, a);
  } else {
    if (greedy) lstm_fwd_launch_t<float, true>(grid, s, a);
    else lstm_fwd_launch_t<float, false>(grid, s, a);
  }
  return (int)hipGetLastError();
}
int sat_lstm_bwd_launch(const LstmBwdArgs& args, hipStream_t s) {
  LstmBwdArgs a = args;
  a.st = sat_launch_stamps();
  const long blocks = lstm_blocks(a.B, a.E);
  DISPATCH_T(a.dtype, lstm_bwd_gp_kernel, dim3((int)blocks), a);
  return (int)hipGetLastError();
}
int sat_tanh_pair_bwd(const float* d_h, int dh_splits, long dh_split_stride, const float* d_c, const float* hc0,
                      int B, int E, float* dpre_f32, void* dpre_t, int dtype, hipStream_t s) {
  dim3 g(grid_for((long)B * 2 * E));
  if (dtype == SAT_BF16) hipLaunchKernelGGL(tanh_pair_bwd_kernel<bf16>, g, dim3(256), 0, s, d_h, dh_splits, dh_split_stride, d_c, hc0, B, E, dpre_f32, (bf16*)dpre_t);
  else hipLaunchKernelGGL(tanh_pair_bwd_kernel<float>, g, dim3(256), 0, s, d_h, dh_splits, dh_split_stride, d_c, hc0, B, E, dpre_f32, (float*)dpre_t);
  return (int)hipGetLastError();
}
int sat_dropout_apply(const float* h, long h_ld, int B, int T1, int E, int training, int has_mask,
                      const uint8_t* mask_in, uint8_t* mask_out, long mask_ld, uint64_t seed,
                      const uint64_t* seed_ptr, int t_offset, void* out_t, long out_ld, int dtype, hipStream_t s) {
  dim3 g(grid_for((long)B * T1 * E));
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16>, g, dim3(256), 0, s, h, h_ld, B, T1, E, training, has_mask, mask_in, mask_out, mask_ld, seed, seed_ptr, t_offset, (bf16*)out_t, out_ld);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, g, dim3(256), 0, s, h, h_ld, B, T1, E, training, has_mask, mask_in, mask_out, mask_ld, seed, seed_ptr, t_offset, (float*)out_t, out_ld);
  return (int)hipGetLastError();
}
int sat_relu_mask_mul(const void* d, const void* ref, long n, int dtype, void* out_t, hipStream_t s) {
  dim3 g(grid_for(n));
  if (dtype == SAT_BF16) hipLaunchKernelGGL(relu_mask_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)d, (const bf16*)ref, n, (bf16*)out_t);
  else hipLaunchKernelGGL(relu_mask_kernel<float>, g, dim3(256), 0, s, (const float*)d, (const float*)ref, n, (float*)out_t);
  return (int)hipGetLastError();
}
int sat_pad_rows(const void* d, const void* ref, int rows, int cols, int ld_out, int dtype, void* out,
                 hipStream_t s) {
  if (rows <= 0 || ld_out < cols) return (int)hipErrorInvalidValue;
  const int gy = rows < 32768 ? rows : 32768;
  if (dtype == SAT_BF16 && cols % 2 == 0 && ld_out % 2 == 0) {
    const dim3 g(sat_cdiv(ld_out / 2, 256), gy);
    if (ref) hipLaunchKernelGGL(pad_rows_bf16x2_kernel<true>, g, dim3(256), 0, s, (const bf16*)d, (const bf16*)ref, rows, cols, ld_out, (bf16*)out);
    else hipLaunchKernelGGL(pad_rows_bf16x2_kernel<false>, g, dim3(256), 0, s, (const bf16*)d, nullptr, rows, cols, ld_out, (bf16*)out);
  } else {
    const dim3 g(sat_cdiv(ld_out, 256), gy);
    if (dtype == SAT_BF16) hipLaunchKernelGGL(pad_rows_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)d, (const bf16*)ref, rows, cols, ld_out, (bf16*)out);
    else hipLaunchKernelGGL(pad_rows_kernel<float>, g, dim3(256), 0, s, (const float*)d, (const float*)ref, rows, cols, ld_out, (float*)out);
  }
  return (int)hipGetLastError();
}
int sat_ado_bwd_split(const float* d_comb, const float* fh, const float* fz, long n, int dtype, void* d_fh_t,
                      void* d_fz_t, hipStream_t s) {
  dim3 g(grid_for(n));
  if (dtype == SAT_BF16) hipLaunchKernelGGL(ado_split_kernel<bf16>, g, dim3(256), 0, s, d_comb, fh, fz, n, (bf16*)d_fh_t, (bf16*)d_fz_t);
  else hipLaunchKernelGGL(ado_split_kernel<float>, g, dim3(256), 0, s, d_comb, fh, fz, n, (float*)d_fh_t, (float*)d_fz_t);
  return (int)hipGetLastError();
}
int sat_ado_combine(const float* fh, const float* fz, const void* emb, long n, int dtype, void* comb_t,
                    hipStream_t s) {
  dim3 g(grid_for(n));
  if (dtype == SAT_BF16) hipLaunchKernelGGL(ado_combine_kernel<bf16>, g, dim3(256), 0, s, fh, fz, (const bf16*)emb, n, (bf16*)comb_t);
  else hipLaunchKernelGGL(ado_combine_kernel<float>, g, dim3(256), 0, s, fh, fz, (const float*)emb, n, (float*)comb_t);
  return (int)hipGetLastError();
}
int sat_fill_const(float* p, long n, float v, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, n, v);
  return (int)hipGetLastError();
}
int sat_zero_rows(float* p, long ld, long rows, long cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return 0;
  const long n = rows * cols;
  const long work = (ld == cols && ((uintptr_t)p & 15) == 0) ? (n + 3) / 4 : n;
  hipLaunchKernelGGL(zero_rows_kernel, dim3(grid_for(work)), dim3(256), 0, s, p, ld, rows, cols);
  return (int)hipGetLastError();
}
int sat_broadcast_rows(const void* src, int B, int D, int T1, int dtype, void* dst, hipStream_t s) {
  dim3 g(grid_for((long)B * T1 * D));
  if (dtype == SAT_BF16) hipLaunchKernelGGL(broadcast_rows_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)src, B, D, T1, (bf16*)dst);
  else hipLaunchKernelGGL(broadcast_rows_kernel<float>, g, dim3(256), 0, s, (const float*)src, B, D, T1, (float*)dst);
  return (int)hipGetLastError();
}
int sat_row_sum_accumulate(const float* X, int R, int N, float* out, hipStream_t s) {
  hipLaunchKernelGGL(row_sum_acc_kernel, dim3(sat_cdiv(N, 256)), dim3(256), 0, s, X, R, N, out);
  return (int)hipGetLastError();
}
