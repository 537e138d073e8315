// Fused soft-attention step (attention.py:14-21) with the decoder's gating
// scalar (decoder.py:97-100), and its backward.
//
// Forward, one launch per decoder step, grid (B, NS): every workgroup scores
// all L annotation slots of its row (e_l = v . tanh(Ws[b,l,:] + U h_b) + b_v,
// wave per slot, lanes over E, shuffle reduction), runs the softmax over L in
// one wave, then accumulates context[b, d] = sum_l alpha_l a[b,l,d] for its
// D-slice of 64*2 16-B vectors (lanes over d, waves over l, LDS fold) and applies
// the gate sigma(f_beta h + b).  The loop-invariant Ws = a W^T + b is hoisted out of
// the time loop (one GEMM per batch) instead of being recomputed every step as
// the reference does (attention.py:16 called from decoder.py:98).
//
// Backward, two launches per step: (1) grid (B, NS): dL/dcontext, the gate
// gradient and per-slice partial dL/dalpha; (2) grid B: softmax backward,
// recomputed tanh, dL/d(U h), running sums of dL/dv, dL/dv.bias, and the step's
// dL/d(score) rows de[b,t,:] (B*L floats).  dL/dWs is NOT accumulated per step (that
// read-modify-write of a B*L*E fp32 buffer was 8 of the step's 10 bytes per element):
// one launch after the time loop (attn_dws_kernel) forms sum_t de_t v (1 - tanh^2)
// reading Ws once; weight gradients are formed once after the loop.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

constexpr int kMaxL = 1024;

template <typename T> struct V16;
template <> struct V16<float> { static constexpr int N = 4; };
template <> struct V16<bf16> { static constexpr int N = 8; };

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* o) {
  if constexpr (sizeof(T) == 4) {
    float4 v = *(const float4*)p;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    uint2 v = *(const uint2*)p;
    const bf16* h = (const bf16*)&v;
    o[0] = (float)h[0]; o[1] = (float)h[1]; o[2] = (float)h[2]; o[3] = (float)h[3];
  }
}

__device__ __forceinline__ float f4get(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

// tanh: exact libm in the fp32 parity path; exp-based (v_exp_f32 + v_rcp_f32, ~1e-6 abs) in bf16 mode.
template <typename T>
__device__ __forceinline__ float tanh_t(float x) {
  if constexpr (sizeof(T) == 4) {
    return tanhf(x);
  } else {
    const float e = __expf(2.f * x);
    return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);   // v_rcp_f32 (1 ulp); __frcp_rn expands to a full division
  }
}

template <typename T>
__device__ __forceinline__ void loadv(const T* p, float* o) {  // 16 bytes
  uint4 v = *(const uint4*)p;
  const T* h = (const T*)&v;
#pragma unroll
  for (int j = 0; j < V16<T>::N; ++j) o[j] = (float)h[j];
}

// Loops over the L annotation slots keep UNR slots' loads in flight per wave (the scores, the
// context and the backward reductions are otherwise one L2 round trip per slot).
constexpr int UNR = 4;

// Workgroup barrier that orders LDS only: outstanding global loads stay in flight across it
// (__syncthreads may also drain vmcnt).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <typename T>
__device__ __forceinline__ uint4 ld16(const T* p, bool ok) {
  return ok ? *(const uint4*)p : make_uint4(0u, 0u, 0u, 0u);
}


// Backward kernels: 8 waves per (row, D-slice) workgroup; each wave accumulates FU slots per
// batch, the annotation rows of the first batch requested before anything else.
constexpr int ANW = 8, FU = 8;

// Forward: 16 waves per (row, D-slice) workgroup and two 16-byte context vectors per lane, so a
// row's scores are computed by cdiv(D, 64*VN*2) workgroups (2 at D = 2048 in bf16) instead of 4:
// the score pass (v . tanh, VALU / transcendental-bound) is half as redundant and one workgroup
// per CU still streams its 100 KB annotation slice.  Slots past L skip their score work (the
// wave-uniform test), and everything the epilogue needs from HBM (gate pre-activation slabs) is
// requested at kernel entry with the first annotation rows, so a step is one dependent memory
// round trip plus the score / softmax / context phases.
constexpr int FNW = 16, FFU = 4;   // the default shape: 16 waves x 4 slots per batch of loads

// FDV: 16-byte context vectors per lane (2: a workgroup owns 1024 bf16 / 512 fp32 columns)
// NW waves, FU slots per wave per batch of loads (16 x 4: every slot of L = 49 in one batch).
template <typename T, int CH, int FDV, int NW = FNW, int FU = FFU, bool PIPE = false>   // CH = e-chunks of 64 x 16 B per lane over E
__device__ __forceinline__ void attn_fwd_kernel_body(AttnFwdArgs a) {
  constexpr int VN = V16<T>::N;            // elements per 16-byte vector
  constexpr int COLS = 64 * VN * FDV;      // context columns of one workgroup
  constexpr int NT = NW * 64, CPT = (COLS + NT - 1) / NT;   // output columns per thread
  static_assert(NW % 8 == 0, "waves fold through 8 LDS rows");
  __shared__ float s_alpha[kMaxL];
  // the waves' context partials fold through 8 LDS rows in NW / 8 rounds (36 KB of LDS instead of 68 at 16
  // waves: the kernel then fits beside a 98-122 KB encoder workgroup on the same CU)
  __shared__ float s_red[8][COLS];
  const int b = blockIdx.x, s = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = a.L, D = a.D, E = a.E;
  const int c0 = s * COLS;
  // Every load of the step is requested here, branch-free (buffer loads: a guarded-off load reads past the resource
  // and returns zeros -- exec-masked branches made the compiler wait for a row right after requesting it), in order
  // of first use (vmcnt retires loads in order): the U h + b slabs and v, the first batch of score rows, the context
  // rows, the gate pre-activation slabs -- the context rows and the gate slabs stay in flight while the scores and the
  // softmax are computed.
  constexpr int kHP = 2;   // U h / gate slabs requested up front (the decoder's h GEMM: 1-2; more: the looped sum)
  const int hp = a.hg_splits < 1 ? 1 : a.hg_splits;
  const bool hp_up = hp <= kHP;
  const float* uh = a.uh + (long)b * a.uh_ld;
  const __amdgpu_buffer_rsrc_t rU = sat_in_rsrc(uh, ((long)(hp - 1) * a.hg_split_stride + E) * 4);
  const __amdgpu_buffer_rsrc_t rV = sat_in_rsrc(a.v_w, (long)E * 4);
  const __amdgpu_buffer_rsrc_t rW = sat_in_rsrc((const T*)a.Ws + (long)b * L * E, (long)L * E * sizeof(T));
  const __amdgpu_buffer_rsrc_t rA = sat_in_rsrc((const T*)a.a + (long)b * L * D, (long)L * D * sizeof(T));
  constexpr int Q4 = VN / 4;   // float4 groups per 16-B vector of T
  float4 up[CH][Q4][kHP], vp[CH][Q4];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int q = 0; q < Q4; ++q) {
      const int e = c * 64 * VN + lane * VN + 4 * q;
#pragma unroll
      for (int p = 0; p < kHP; ++p)
        up[c][q][p] = sat_ld16f(rU, hp_up && p < hp && e < E ? (unsigned)((p * a.hg_split_stride + e) * 4) : kSatOOB);
      vp[c][q] = sat_ld16f(rV, e < E ? (unsigned)(e * 4) : kSatOOB);
    }
  float4 uf[CH][Q4];   // more slabs than requested up front: the looped sum, before the rows are requested
  if (!hp_up) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int q = 0; q < Q4; ++q) {
        const int e = c * 64 * VN + lane * VN + 4 * q;
        uf[c][q] = e < E ? sum_parts4(uh, e, a.hg_splits, a.hg_split_stride) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  }
  auto ws_off = [&](int l, int e) { return l < L && e < E ? (unsigned)(((long)l * E + e) * sizeof(T)) : kSatOOB; };
  auto a_off = [&](int l, int d) { return l < L && d < D ? (unsigned)(((long)l * D + d) * sizeof(T)) : kSatOOB; };
  uint4 xv[FU][CH];
#pragma unroll
  for (int u = 0; u < FU; ++u)
#pragma unroll
    for (int c = 0; c < CH; ++c) xv[u][c] = sat_ld16(rW, ws_off(w + NW * u, c * 64 * VN + lane * VN));
  // context rows of the first batch
  uint4 xa[FU][FDV];
#pragma unroll
  for (int u = 0; u < FU; ++u)
#pragma unroll
    for (int v = 0; v < FDV; ++v) xa[u][v] = sat_ld16(rA, a_off(w + NW * u, c0 + v * 64 * VN + lane * VN));
  // the epilogue's threads own 4 consecutive columns each (col4 = 4 tid: 16-B write-through stores)
  static_assert(COLS <= 4 * NT && COLS % 4 == 0, "four columns per epilogue thread");
  const int col4 = 4 * tid;
  const bool ep = col4 < COLS && c0 + col4 < D;   // D % 4 == 0 (host-checked): a quad is all in or all out
  float4 gp[kHP];
  const __amdgpu_buffer_rsrc_t rG = sat_in_rsrc(a.gate_pre ? a.gate_pre + (long)b * a.gate_ld : a.uh,
                                                ((long)(hp - 1) * a.hg_split_stride + D) * 4);
#pragma unroll
  for (int p = 0; p < kHP; ++p)
    gp[p] = sat_ld16f(rG, a.gate_pre && ep && hp_up && p < hp ? (unsigned)((p * a.hg_split_stride + c0 + col4) * 4)
                                                             : kSatOOB);

  // ---- scores: lane owns VN consecutive e per chunk; (U h + b) and v live in registers ----
  float u_r[CH][VN], v_r[CH][VN];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int e = c * 64 * VN + lane * VN;
#pragma unroll
    for (int q = 0; q < Q4; ++q) {
      const float4 u4 = hp_up ? sum_loaded_parts4(up[c][q], hp) : uf[c][q];
      const float4 v4 = vp[c][q];
      u_r[c][4 * q] = u4.x; u_r[c][4 * q + 1] = u4.y; u_r[c][4 * q + 2] = u4.z; u_r[c][4 * q + 3] = u4.w;
      v_r[c][4 * q] = v4.x; v_r[c][4 * q + 1] = v4.y; v_r[c][4 * q + 2] = v4.z; v_r[c][4 * q + 3] = v4.w;
    }
  }
  float4 gpre4 = make_float4(0.f, 0.f, 0.f, 0.f);   // summed in the epilogue (its slabs arrive last)

  const float bv = a.v_b[0];
  // (the per-slot and per-column accumulations are explicit FMAs: the compiler's own contraction choice can differ
  // between instantiations, and the PIPE / one-batch forms must agree bit for bit)
  // slots in batches of NW x FU (one batch at L = 49).  PIPE (more slots than one batch of NW x 4, e.g. L = 196):
  // batches of NW x 2 slots, the next batch's rows requested before the current batch's arithmetic (two register
  // buffers: the same registers as one batch of NW x 4), so the batches' memory round trips overlap
  constexpr int STEP = NW * FU;
  auto load_ws = [&](int l0, uint4 (&dst)[FU][CH]) {
#pragma unroll
    for (int u = 0; u < FU; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) dst[u][c] = sat_ld16(rW, ws_off(l0 + NW * u, c * 64 * VN + lane * VN));
  };
  auto scores = [&](int l0, const uint4 (&src)[FU][CH]) {
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int l = l0 + NW * u;
      if (l >= L) break;   // wave-uniform
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const T* h = (const T*)&src[u][c];
#pragma unroll
        for (int j = 0; j < VN; ++j) acc = fmaf(v_r[c][j], tanh_t<T>((float)h[j] + u_r[c][j]), acc);   // v = 0 past E
      }
      acc = wave_sum(acc);
      if (lane == 0) s_alpha[l] = acc + bv;
    }
  };
  if constexpr (PIPE) {
    for (int l0 = w; l0 < L; l0 += 2 * STEP) {
      uint4 xn[FU][CH];
      load_ws(l0 + STEP, xn);   // unconditional: rows past L read zeros (a guarded load let the compiler
                                 // hoist the rows' unpacking next to it, waiting on them at once)
      scores(l0, xv);
      load_ws(l0 + 2 * STEP, xv);
      if (l0 + STEP < L) scores(l0 + STEP, xn);
    }
  } else {
    for (int l0 = w; l0 < L; l0 += STEP) {
      if (l0 != w) load_ws(l0, xv);
      scores(l0, xv);
    }
  }
  if (s == 0 && w == 1 && a.uh_save) {   // U h + b of this row (the registers every wave holds)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int e = c * 64 * VN + lane * VN;
      if (e < E) {
#pragma unroll
        for (int j = 0; j < VN; ++j) a.uh_save[(long)b * a.uh_save_ld + e + j] = u_r[c][j];
      }
    }
  }
  __syncthreads();
  // ---- softmax over L (one wave) ----
  if (w == 0) {
    float m = -INFINITY;
    for (int l = lane; l < L; l += 64) m = fmaxf(m, s_alpha[l]);
    m = wave_max(m);
    float sum = 0.f;
    for (int l = lane; l < L; l += 64) {
      float e = expf(s_alpha[l] - m);
      s_alpha[l] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    float inv = 1.0f / sum;
    for (int l = lane; l < L; l += 64) {
      float al = s_alpha[l] * inv;
      s_alpha[l] = al;
      if (s == 0 && a.alpha) a.alpha[(long)b * a.alpha_ld + l] = al;
    }
  }
  __syncthreads();
  // ---- context for this D-slice: lanes over d (16-byte loads), waves over l ----
  float part[FDV][VN];
#pragma unroll
  for (int v = 0; v < FDV; ++v)
#pragma unroll
    for (int j = 0; j < VN; ++j) part[v][j] = 0.f;
  auto load_a = [&](int l0, uint4 (&dst)[FU][FDV]) {
#pragma unroll
    for (int u = 0; u < FU; ++u)
#pragma unroll
      for (int v = 0; v < FDV; ++v) dst[u][v] = sat_ld16(rA, a_off(l0 + NW * u, c0 + v * 64 * VN + lane * VN));
  };
  auto context = [&](int l0, const uint4 (&src)[FU][FDV]) {
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int l = l0 + NW * u;
      if (l < L) {
        const float al = s_alpha[l];
#pragma unroll
        for (int v = 0; v < FDV; ++v) {
          const T* h = (const T*)&src[u][v];
#pragma unroll
          for (int j = 0; j < VN; ++j) part[v][j] = fmaf(al, (float)h[j], part[v][j]);
        }
      }
    }
  };
  if constexpr (PIPE) {   // the same two-buffer overlap as the scores
    for (int l0 = w; l0 < L; l0 += 2 * STEP) {
      uint4 an[FU][FDV];
      load_a(l0 + STEP, an);
      context(l0, xa);
      load_a(l0 + 2 * STEP, xa);
      if (l0 + STEP < L) context(l0 + STEP, an);
    }
  } else {
    for (int l0 = w; l0 < L; l0 += STEP) {
      if (l0 != w) load_a(l0, xa);
      context(l0, xa);
    }
  }
  // fixed summation order over the wave partials: c = sum over q = 0, 2, .., 6 of (p_q + p_(q+1)) per round of
  // 8 waves, waves 0-7 first, then waves 8-15 through the same 8 rows
  float4 cacc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int half = 0; half < NW / 8; ++half) {
    if ((w >> 3) == half) {
#pragma unroll
      for (int v = 0; v < FDV; ++v)
#pragma unroll
        for (int j = 0; j < VN; ++j) s_red[w & 7][v * 64 * VN + lane * VN + j] = part[v][j];
    }
    __syncthreads();
    if (ep) {
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        const float4 x = *(const float4*)&s_red[q][col4], y = *(const float4*)&s_red[q + 1][col4];
        cacc.x += x.x + y.x; cacc.y += x.y + y.y; cacc.z += x.z + y.z; cacc.w += x.w + y.w;
      }
    }
    if (half + 1 < NW / 8) __syncthreads();
  }
  if (a.gate_pre && ep)
    gpre4 = hp_up ? sum_loaded_parts4(gp, hp)
                  : sum_parts4(a.gate_pre + (long)b * a.gate_ld, c0 + col4, a.hg_splits, a.hg_split_stride);
  if (ep) {
    const int dout = c0 + col4;
    // fp32 outputs through 16-B write-through stores (sat_common.h): this step's end-of-kernel L2 writeback, on the
    // per-step critical path, has less to flush; the bf16 copies (8 B per thread) stay write-back
    // (a resource per batch row: its offsets stay far below the 2 GiB cap whatever B and the row stride)
    sat_st16(sat_out_rsrc(a.ctx + (long)b * a.ctx_ld, 4L * a.D), (unsigned)(dout * 4), *(const uint4*)&cacc);
    const float c[4] = {cacc.x, cacc.y, cacc.z, cacc.w};
    if (a.ctx_t) {
      T* ct = (T*)a.ctx_t + (long)b * a.ctx_t_ld + dout;
#pragma unroll
      for (int k = 0; k < 4; ++k) ct[k] = (T)c[k];
    }
    if (a.gate_pre) {
      const float gp[4] = {gpre4.x, gpre4.y, gpre4.z, gpre4.w};
      float g[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = 1.0f / (1.0f + expf(-gp[k]));
      if (a.gate)
        sat_st16(sat_out_rsrc(a.gate + (long)b * a.gate_out_ld, 4L * a.D), (unsigned)(dout * 4),
                 make_uint4(__float_as_uint(g[0]), __float_as_uint(g[1]), __float_as_uint(g[2]), __float_as_uint(g[3])));
      if (a.gated) {
        T* gd = (T*)a.gated + (long)b * a.gated_ld + dout;
#pragma unroll
        for (int k = 0; k < 4; ++k) gd[k] = (T)(g[k] * c[k]);
      }
    }
  }
}

template <typename T, int CH, int FDV, int NW = FNW, int FU = FFU, bool PIPE = false>
__global__ __launch_bounds__(NW * 64) void attn_fwd_kernel(AttnFwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  attn_fwd_kernel_body<T, CH, FDV, NW, FU, PIPE>(a);
  sat_stamp_end(a.st, t0);
}

// grid (B, NS): dL/dcontext for the workgroup's D-slice is formed ONCE (thread per column: the
// gated-context slabs, gate, context, head term; the gate gradient written on the way) into LDS,
// then every wave dots it with its slots' annotation rows (requested at kernel entry).
template <typename T>
__device__ __forceinline__ void attn_bwd1_kernel_body(AttnBwdArgs a) {
  constexpr int VD = V16<T>::N;
  constexpr int COLS = 64 * VD;
  __shared__ float s_dctx[COLS];
  const int b = blockIdx.x, s = blockIdx.y, NS = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = a.L, D = a.D;
  const int d0 = s * COLS + lane * VD;
  const T* ab = (const T*)a.a + (long)b * L * D + d0;
  // issue order = order of first use (vmcnt retires in order): this thread's column operands,
  // then the annotation rows of the first batch, which stay in flight through the LDS exchange
  static_assert(COLS <= ANW * 64, "at most one column per thread");
  const int dcol = s * COLS + tid;
  const bool col_ok = tid < COLS && dcol < D;
  float dg = 0.f, g = 0.f, cx = 0.f, dx = 0.f;
  if (col_ok) {
    dg = sum_parts(a.d_gated, (long)b * a.d_gated_ld + dcol, a.dg_splits, a.dg_split_stride);
    g = a.gate[(long)b * a.gate_ld + dcol];
    cx = a.ctx[(long)b * a.ctx_ld + dcol];
    if (a.d_ctx_ext) dx = a.d_ctx_ext[(long)b * a.d_ctx_ext_ld + dcol];
  }
  uint4 xa[FU];
#pragma unroll
  for (int u = 0; u < FU; ++u) xa[u] = ld16(ab + (long)(w + ANW * u) * D, w + ANW * u < L && d0 < D);
  if (tid < COLS) {
    float dctx = 0.f;
    if (col_ok) {
      dctx = dg * g + dx;
      const float dgp = dg * cx * g * (1.f - g);
      a.d_gpre[(long)b * a.d_gpre_ld + dcol] = dgp;
      if (a.d_gpre_t) ((T*)a.d_gpre_t)[(long)b * a.d_gpre_ld + dcol] = (T)dgp;
    }
    s_dctx[tid] = dctx;
  }
  lds_barrier();   // the annotation rows stay in flight
  float dctx[VD];
#pragma unroll
  for (int j = 0; j < VD; ++j) dctx[j] = s_dctx[lane * VD + j];
  for (int l0 = w; l0 < L; l0 += ANW * FU) {
    if (l0 != w) {
#pragma unroll
      for (int u = 0; u < FU; ++u) xa[u] = ld16(ab + (long)(l0 + ANW * u) * D, l0 + ANW * u < L && d0 < D);
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int l = l0 + ANW * u;
      if (l >= L) break;   // wave-uniform
      const T* h = (const T*)&xa[u];
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < VD; ++j) p += dctx[j] * (float)h[j];
      p = wave_sum(p);
      if (lane == 0) a.part[((long)b * NS + s) * L + l] = p;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(ANW * 64) void attn_bwd1_kernel(AttnBwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  attn_bwd1_kernel_body<T>(a);
  sat_stamp_end(a.st, t0);
}

// grid (B, E / 256): a workgroup of 8 waves per (row, 256-wide e-slice); lane owns 4 consecutive
// e, waves take BFU slots each per batch, so a row's 49 slots are two batches of loads in flight.
// The softmax backward (a few hundred flops per row) is recomputed by each slice.
constexpr int BNW = 8, BFU = 4, BEV = 4, BSLICE = 64 * BEV;

template <typename T>
__device__ __forceinline__ void load_e4(const T* p, bool ok, float* o) {
  if (!ok) { o[0] = o[1] = o[2] = o[3] = 0.f; return; }
  load4<T>(p, o);
}

template <typename T>
__device__ __forceinline__ void attn_bwd2_kernel_body(AttnBwdArgs a, int NS) {
  __shared__ float s_de[kMaxL];
  __shared__ float s_red[BNW][BSLICE];
  __shared__ float s_tmp[BNW];
  const int b = blockIdx.x, eslice = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = a.L, E = a.E;
  const int e = eslice * BSLICE + lane * BEV;
  const bool eok = e < E;
  const float* alpha = a.alpha + (long)b * a.alpha_ld;
  const float* uh = a.uh + (long)b * a.uh_ld;
  const T* Ws = (const T*)a.Ws + (long)b * L * E;
  // loop invariants and the first batch of slots: requested before the softmax backward
  float uu[BEV], vw[BEV];
  load_e4<float>(uh + e, eok, uu);
  load_e4<float>(a.v_w + e, eok, vw);
  float xw[BFU][BEV];
#pragma unroll
  for (int u = 0; u < BFU; ++u) {
    const int l = w + BNW * u;
    load_e4<T>(Ws + (long)l * E + e, l < L && eok, xw[u]);
  }
  // dL/dalpha and sum_l alpha*dalpha
  float loc = 0.f;
  for (int l = tid; l < L; l += BNW * 64) {
    float da = 0.f;
    for (int s = 0; s < NS; ++s) da += a.part[((long)b * NS + s) * L + l];
    if (a.d_alpha_ext) da += a.d_alpha_ext[(long)b * a.d_alpha_ext_ld + l];
    s_de[l] = da;
    loc += alpha[l] * da;
  }
  loc = wave_sum(loc);
  if (lane == 0) s_tmp[w] = loc;
  __syncthreads();
  float sad = 0.f;
#pragma unroll
  for (int i = 0; i < BNW; i += 2) sad += s_tmp[i] + s_tmp[i + 1];
  __syncthreads();
  for (int l = tid; l < L; l += BNW * 64) {
    const float de = alpha[l] * (s_de[l] - sad);
    s_de[l] = de;
    if (eslice == 0) a.de_out[(long)b * a.de_ld + l] = de;
  }
  __syncthreads();
  // recompute tanh, accumulate
  float duh[BEV], dv[BEV];
#pragma unroll
  for (int j = 0; j < BEV; ++j) duh[j] = dv[j] = 0.f;
  float dbv = 0.f;
  for (int l0 = w; l0 < L; l0 += BNW * BFU) {
    if (l0 != w) {
#pragma unroll
      for (int u = 0; u < BFU; ++u) {
        const int l = l0 + BNW * u;
        load_e4<T>(Ws + (long)l * E + e, l < L && eok, xw[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < BFU; ++u) {
      const int l = l0 + BNW * u;
      if (l >= L) break;   // wave-uniform
      const float de = s_de[l];
      dbv += de;
      if (!eok) continue;
#pragma unroll
      for (int j = 0; j < BEV; ++j) {
        const float t = tanh_t<T>(xw[u][j] + uu[j]);
        const float datt = de * vw[j] * (1.f - t * t);
        duh[j] += datt;
        dv[j] += de * t;
      }
    }
  }
  // fold the waves (fixed order): dU_h, then dv
#pragma unroll
  for (int j = 0; j < BEV; ++j) s_red[w][lane * BEV + j] = duh[j];
  __syncthreads();
  const int eo = eslice * BSLICE + tid;
  if (tid < BSLICE && eo < E) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < BNW; i += 2) v += s_red[i][tid] + s_red[i + 1][tid];
    a.d_uh[(long)b * a.d_uh_ld + eo] = v;
    if (a.d_uh_t) ((T*)a.d_uh_t)[(long)b * a.d_uh_ld + eo] = (T)v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < BEV; ++j) s_red[w][lane * BEV + j] = dv[j];
  if (lane == 0) s_tmp[w] = dbv;   // every lane added the same de per slot: lane 0 holds the wave's sum
  __syncthreads();
  if (tid < BSLICE && eo < E) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < BNW; i += 2) v += s_red[i][tid] + s_red[i + 1][tid];
    a.dv_acc[(long)b * E + eo] += v;
  }
  if (tid == 0 && eslice == 0) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < BNW; i += 2) v += s_tmp[i] + s_tmp[i + 1];
    a.dbv_acc[b] += v;
  }
}

template <typename T>
__global__ __launch_bounds__(BNW * 64) void attn_bwd2_kernel(AttnBwdArgs a, int NS) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  attn_bwd2_kernel_body<T>(a, NS);
  sat_stamp_end(a.st, t0);
}

// The attention backward of one step split over L: grid (B, NL), workgroup (b, c) owns the slots
// l in [c LC, (c + 1) LC) of batch row b (LC = ceil(L / NL)), so a row's annotation rows a[b, l, :] and
// Ws[b, l, :] are streamed by NL workgroups (at B = 128: 256 workgroups fill the chip, where one per row
// left half of it idle).  The softmax backward needs sum_k alpha_k dL/dalpha_k over ALL slots; it is
//   sum_k alpha_k (a_k . dctx + dalpha_ext_k) = ctx . dctx + sum_k alpha_k dalpha_ext_k
// (ctx = sum_k alpha_k a_k is the saved pre-gate context), so no workgroup needs another's dL/dalpha.
// Phases: A thread per column d: dL/dcontext (+ gate gradient, chunk 0 writes it) and ctx . dctx;
// B wave per slot: dL/dalpha_l; C de_l = alpha_l (dL/dalpha_l - sum); D tanh backward of the chunk's
// slots: partial dL/d(U h), dL/dv, dL/dv.bias.  With NL > 1 the partials meet in the last-arriving
// workgroup of the row (agent-scope ticket; payload stored and loaded sc1, so no cache fence is needed:
// MI355X_MICROARCH.md, visibility, first row of the sc1 table), summed in chunk order (deterministic).
// The split backward's chunk hand-off without agent-scope fences: the partials are stored `sc1` (agent relaxed
// atomic stores, 4 B), every storing wave waits vmcnt(0) before the barrier, lane 0 adds to the row's ticket, the
// workgroup whose add returned NL - 1 reads the partials with `sc1` loads (agent relaxed atomic loads) after that add
// returned / after the barrier: the first row of MI355X_MICROARCH.md's table of hand-offs measured valid without the
// acquire, and with an `sc1` payload without the release (one workgroup per CU, hipMalloc'd workspace).  cfg5
// (L = 196, two chunks per row) attention backward span 21.7 -> 19.8 us (profiles/r6_s64); 1 = the fenced form.
#ifndef SAT_ATTN_FENCES
#define SAT_ATTN_FENCES 0
#endif
// Diagnostics builds only (tools/build_variant.sh, -DSAT_ATTN_MARK=k): the attention backward's stamp records the time
// every wave of the workgroup has reached phase boundary k instead of the kernel's end (bench.py's per-step spans then
// measure start -> boundary k).  The product build defines no marker.
#ifdef SAT_ATTN_MARK
#define SAT_MARK(k)                                                                                                  \
  if ((k) == SAT_ATTN_MARK && a.st.p && a.st.p[0]) {                                                                 \
    __syncthreads();                                                                                                 \
    const int w_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                                   \
    if (threadIdx.x == 0 && w_ < a.st.cap) a.st.p[2 + 2 * (long)w_ + 1] = __builtin_amdgcn_s_memrealtime();          \
  }
#else
#define SAT_MARK(k)
#endif
template <typename T, int DCH, int ECH, int FBW, int FBU, bool PIPE>
__device__ __forceinline__ void attn_bwd_split_kernel_body(AttnBwdArgs a) {
  constexpr int VN = V16<T>::N;
  constexpr int EC = 64 * VN * ECH;
  __shared__ float s_dctx[64 * VN * DCH];
  __shared__ float s_al[kMaxL], s_dax[kMaxL];
  __shared__ float s_red[FBW][EC];
  __shared__ float s_tmp[FBW];
  __shared__ int s_last;
  const int b = blockIdx.x, c = blockIdx.y, NL = gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = a.L, D = a.D, E = a.E;
  const int LC = (L + NL - 1) / NL, l_beg = c * LC, l_end = min(L, l_beg + LC);
  // ---- requests in order of first use, branch-free (buffer loads: a guarded-off load reads past its resource and
  // returns zeros -- the exec-masked loads and the looped slab sums before made the compiler wait for each column's
  // slabs before requesting the next, several round trips ahead of the annotation rows) ----
  constexpr int CPT = (64 * VN * DCH + FBW * 64 - 1) / (FBW * 64);
  constexpr int kDP = 8;   // d(gated context) slabs requested up front (the transposed skinny GEMM's: 4-6; more: looped)
  const int dp = a.dg_splits < 1 ? 1 : a.dg_splits;
  const bool dp_up = dp <= kDP;
  const __amdgpu_buffer_rsrc_t rDG =
      sat_in_rsrc(a.d_gated + (long)b * a.d_gated_ld, ((long)(dp - 1) * a.dg_split_stride + D) * 4);
  const __amdgpu_buffer_rsrc_t rGt = sat_in_rsrc(a.gate + (long)b * a.gate_ld, (long)D * 4);
  const __amdgpu_buffer_rsrc_t rCx = sat_in_rsrc(a.ctx + (long)b * a.ctx_ld, (long)D * 4);
  const __amdgpu_buffer_rsrc_t rDx =
      sat_in_rsrc(a.d_ctx_ext ? a.d_ctx_ext + (long)b * a.d_ctx_ext_ld : a.ctx, (long)D * 4);
  float dgp[CPT][kDP], dcol[CPT][4];   // d(gated) slabs; dg, g, cx, dx of this thread's columns
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int d = k * FBW * 64 + tid;
    const bool ok = d < D;
#pragma unroll
    for (int p = 0; p < kDP; ++p)
      dgp[k][p] = sat_ld4f(rDG, ok && dp_up && p < dp ? (unsigned)((p * a.dg_split_stride + d) * 4) : kSatOOB);
    dcol[k][1] = sat_ld4f(rGt, ok ? (unsigned)(d * 4) : kSatOOB);
    dcol[k][2] = sat_ld4f(rCx, ok ? (unsigned)(d * 4) : kSatOOB);
    dcol[k][3] = sat_ld4f(rDx, ok && a.d_ctx_ext ? (unsigned)(d * 4) : kSatOOB);
  }
  if (!dp_up) {   // more slabs than requested up front: the looped sum, before the rows are requested
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int d = k * FBW * 64 + tid;
      dcol[k][0] = d < D ? sum_parts(a.d_gated, (long)b * a.d_gated_ld + d, a.dg_splits, a.dg_split_stride) : 0.f;
    }
  }
  // alpha (and dL/dalpha from outside) of every slot: staged in LDS by phase A, read per slot by the walk
  constexpr int LPT = kMaxL / (FBW * 64);
  const __amdgpu_buffer_rsrc_t rAl = sat_in_rsrc(a.alpha + (long)b * a.alpha_ld, (long)L * 4);
  const __amdgpu_buffer_rsrc_t rDa =
      sat_in_rsrc(a.d_alpha_ext ? a.d_alpha_ext + (long)b * a.d_alpha_ext_ld : a.alpha, (long)L * 4);
  float al_r[LPT], dax_r[LPT];
#pragma unroll
  for (int k = 0; k < LPT; ++k) {
    const int l = k * FBW * 64 + tid;
    al_r[k] = sat_ld4f(rAl, l < L ? (unsigned)(l * 4) : kSatOOB);
    dax_r[k] = sat_ld4f(rDa, l < L && a.d_alpha_ext ? (unsigned)(l * 4) : kSatOOB);
  }
  const __amdgpu_buffer_rsrc_t rA = sat_in_rsrc((const T*)a.a + (long)b * L * D, (long)L * D * sizeof(T));
  const __amdgpu_buffer_rsrc_t rW = sat_in_rsrc((const T*)a.Ws + (long)b * L * E, (long)L * E * sizeof(T));
  auto a_off = [&](int l, int q) {
    const int d = q * 64 * VN + lane * VN;
    return l < l_end && d < D ? (unsigned)(((long)l * D + d) * sizeof(T)) : kSatOOB;
  };
  auto w_off = [&](int l, int q) {
    const int e = q * 64 * VN + lane * VN;
    return l < l_end && e < E ? (unsigned)(((long)l * E + e) * sizeof(T)) : kSatOOB;
  };
  uint4 xa[FBU][DCH];
#pragma unroll
  for (int u = 0; u < FBU; ++u)
#pragma unroll
    for (int q = 0; q < DCH; ++q) xa[u][q] = sat_ld16(rA, a_off(l_beg + w + FBW * u, q));
  const __amdgpu_buffer_rsrc_t rU = sat_in_rsrc(a.uh + (long)b * a.uh_ld, (long)E * 4);
  const __amdgpu_buffer_rsrc_t rV = sat_in_rsrc(a.v_w, (long)E * 4);
  float4 uu4[ECH][VN / 4], vw4[ECH][VN / 4];
#pragma unroll
  for (int q = 0; q < ECH; ++q)
#pragma unroll
    for (int j = 0; j < VN / 4; ++j) {
      const int e = q * 64 * VN + lane * VN + 4 * j;
      uu4[q][j] = sat_ld16f(rU, e < E ? (unsigned)(e * 4) : kSatOOB);
      vw4[q][j] = sat_ld16f(rV, e < E ? (unsigned)(e * 4) : kSatOOB);
    }
  uint4 xw[FBU][ECH];
#pragma unroll
  for (int u = 0; u < FBU; ++u)
#pragma unroll
    for (int q = 0; q < ECH; ++q) xw[u][q] = sat_ld16(rW, w_off(l_beg + w + FBW * u, q));
  if (dp_up) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) dcol[k][0] = sum_loaded_parts(dgp[k], dp);
  }
  SAT_MARK(1)
  // ---- A: dL/dcontext, the gate gradient (chunk 0), ctx . dctx + sum_k alpha_k dalpha_ext_k ----
  float loc = 0.f;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int d = k * FBW * 64 + tid;
    if (d < 64 * VN * DCH) {
      float dctx = 0.f;
      if (d < D) {
        const float dg = dcol[k][0], g = dcol[k][1], cx = dcol[k][2], dx = dcol[k][3];
        dctx = dg * g + dx;
        loc += cx * dctx;
        if (c == 0) {
          const float dgp = dg * cx * g * (1.f - g);
          a.d_gpre[(long)b * a.d_gpre_ld + d] = dgp;
          if (a.d_gpre_t) ((T*)a.d_gpre_t)[(long)b * a.d_gpre_ld + d] = (T)dgp;
        }
      }
      s_dctx[d] = dctx;
    }
  }
#pragma unroll
  for (int k = 0; k < LPT; ++k) {
    const int l = k * FBW * 64 + tid;
    if (l < L) {
      if (a.d_alpha_ext) loc += al_r[k] * dax_r[k];
      s_al[l] = al_r[k];
      s_dax[l] = dax_r[k];
    }
  }
  loc = wave_sum(loc);
  if (lane == 0) s_tmp[w] = loc;
  lds_barrier();   // the annotation / Ws rows stay in flight
  SAT_MARK(2)
  float sad = 0.f;
#pragma unroll
  for (int i = 0; i < FBW; i += 2) sad += s_tmp[i] + s_tmp[i + 1];
  float dctx[DCH][VN];
#pragma unroll
  for (int q = 0; q < DCH; ++q)
#pragma unroll
    for (int j = 0; j < VN; ++j) dctx[q][j] = s_dctx[q * 64 * VN + lane * VN + j];
  // ---- B-D in one walk over the chunk's slots: per slot dL/dalpha_l (a_l . dctx), de_l = alpha_l (dL/dalpha_l -
  // sum), and at once its tanh backward over E (partial dL/d(U h), dL/dv, dL/dv.bias) -- the wave that scored a
  // slot owns it through the tanh, so a slot's annotation and Ws rows are requested together and the walk is one
  // pass of dependent batches instead of two.  PIPE (a chunk deeper than one batch of loads, e.g. L = 196): the
  // next batch's rows are requested before the current batch's arithmetic (two register buffers of half a batch)
  float duh[ECH][VN], dv[ECH][VN];
#pragma unroll
  for (int q = 0; q < ECH; ++q)
#pragma unroll
    for (int j = 0; j < VN; ++j) duh[q][j] = dv[q][j] = 0.f;
  float dbv = 0.f;   // the same in every lane (de is wave-uniform)
  constexpr int BST = FBW * FBU;
  auto load_rows = [&](int l0, uint4 (&da)[FBU][DCH], uint4 (&dw)[FBU][ECH]) {
#pragma unroll
    for (int u = 0; u < FBU; ++u)
#pragma unroll
      for (int q = 0; q < DCH; ++q) da[u][q] = sat_ld16(rA, a_off(l0 + FBW * u, q));
#pragma unroll
    for (int u = 0; u < FBU; ++u)
#pragma unroll
      for (int q = 0; q < ECH; ++q) dw[u][q] = sat_ld16(rW, w_off(l0 + FBW * u, q));
  };
  auto slots = [&](int l0, const uint4 (&sa)[FBU][DCH], const uint4 (&sw)[FBU][ECH]) {
#pragma unroll
    for (int u = 0; u < FBU; ++u) {
      const int l = l0 + FBW * u;
      if (l >= l_end) break;   // wave-uniform
      float p = 0.f;
#pragma unroll
      for (int q = 0; q < DCH; ++q) {
        const T* h = (const T*)&sa[u][q];
#pragma unroll
        for (int j = 0; j < VN; ++j) p = fmaf(dctx[q][j], (float)h[j], p);
      }
      p = wave_sum(p);
      const float de = s_al[l] * ((p + s_dax[l]) - sad);
      if (lane == 0) a.de_out[(long)b * a.de_ld + l] = de;
      dbv += de;
#pragma unroll
      for (int q = 0; q < ECH; ++q) {
        const T* h = (const T*)&sw[u][q];
#pragma unroll
        for (int j = 0; j < VN; ++j) {
          const float t = tanh_t<T>((float)h[j] + f4get(uu4[q][j / 4], j % 4));
          duh[q][j] = fmaf(de * f4get(vw4[q][j / 4], j % 4), fmaf(-t, t, 1.f), duh[q][j]);
          dv[q][j] = fmaf(de, t, dv[q][j]);
        }
      }
    }
  };
  if constexpr (PIPE) {
    for (int l0 = l_beg + w; l0 < l_end; l0 += 2 * BST) {
      uint4 an[FBU][DCH], wn[FBU][ECH];
      load_rows(l0 + BST, an, wn);   // unconditional: rows past the chunk read zeros (a guarded load let the
                                      // compiler hoist the rows' unpacking next to it, waiting on them at once)
      slots(l0, xa, xw);
      load_rows(l0 + 2 * BST, xa, xw);
      if (l0 + BST < l_end) slots(l0 + BST, an, wn);
    }
  } else {
    for (int l0 = l_beg + w; l0 < l_end; l0 += BST) {
      if (l0 != l_beg + w) load_rows(l0, xa, xw);
      slots(l0, xa, xw);
    }
  }
  SAT_MARK(3)
  // fold the waves in a fixed order: dL/d(U h) into registers of threads e < E, then dL/dv
#pragma unroll
  for (int q = 0; q < ECH; ++q)
#pragma unroll
    for (int j = 0; j < VN; ++j) s_red[w][q * 64 * VN + lane * VN + j] = duh[q][j];
  __syncthreads();
  constexpr int EPT = (EC + FBW * 64 - 1) / (FBW * 64);   // folded columns per thread
  float fu[EPT], fv[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = k * FBW * 64 + tid;
    float v = 0.f;
    if (e < EC && e < E) {
#pragma unroll
      for (int i = 0; i < FBW; i += 2) v += s_red[i][e] + s_red[i + 1][e];
    }
    fu[k] = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < ECH; ++q)
#pragma unroll
    for (int j = 0; j < VN; ++j) s_red[w][q * 64 * VN + lane * VN + j] = dv[q][j];
  if (lane == 0) s_tmp[w] = dbv;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = k * FBW * 64 + tid;
    float v = 0.f;
    if (e < EC && e < E) {
#pragma unroll
      for (int i = 0; i < FBW; i += 2) v += s_red[i][e] + s_red[i + 1][e];
    }
    fv[k] = v;
  }
  float fb = 0.f;
#pragma unroll
  for (int i = 0; i < FBW; i += 2) fb += s_tmp[i] + s_tmp[i + 1];
  SAT_MARK(4)
  if (NL == 1) {   // the whole row here: write directly
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = k * FBW * 64 + tid;
      if (e < EC && e < E) {
        a.d_uh[(long)b * a.d_uh_ld + e] = fu[k];
        if (a.d_uh_t) ((T*)a.d_uh_t)[(long)b * a.d_uh_ld + e] = (T)fu[k];
        a.dv_acc[(long)b * E + e] += fv[k];
      }
    }
    if (tid == 0) a.dbv_acc[b] += fb;
    return;
  }
  // ---- E: partials of the chunk -> the row's last-arriving workgroup ----
  unsigned* pp = (unsigned*)a.part + (long)(b * NL + c) * (2 * E + 1);
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = k * FBW * 64 + tid;
    if (e < EC && e < E) {
      __hip_atomic_store(pp + e, __float_as_uint(fu[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pp + E + e, __float_as_uint(fv[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid == 0) __hip_atomic_store(pp + 2 * E, __float_as_uint(fb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its sc1 stores are done
  __syncthreads();
  if (tid == 0) {
    // (SAT_ATTN_FENCES: an agent-scope release before the ticket; the second wait keeps the compiler from dropping
    // the fence's own, cdna_hip_programming.md Guideline 16 Pitfall 12)
#if SAT_ATTN_FENCES
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    const unsigned prev = __hip_atomic_fetch_add(a.ticket + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = prev == (unsigned)(NL - 1);
#if SAT_ATTN_FENCES
    if (last) {   // agent-scope acquire on the reading CU besides the sc1 loads below (cdna_hip_programming.md §6
                  // Guideline 16): one fence per row's last arriver, only on the NL > 1 path (small batches)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#endif
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;   // workgroup-uniform
  const unsigned* rp = (const unsigned*)a.part + (long)b * NL * (2 * E + 1);
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = k * FBW * 64 + tid;
    if (e < EC && e < E) {
      float su = 0.f, sv = 0.f;
      for (int q = 0; q < NL; ++q) {   // chunk order: the same sums whichever workgroup arrives last
        su += __uint_as_float(__hip_atomic_load(rp + (long)q * (2 * E + 1) + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        sv += __uint_as_float(__hip_atomic_load(rp + (long)q * (2 * E + 1) + E + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      a.d_uh[(long)b * a.d_uh_ld + e] = su;
      if (a.d_uh_t) ((T*)a.d_uh_t)[(long)b * a.d_uh_ld + e] = (T)su;
      a.dv_acc[(long)b * E + e] += sv;
    }
  }
  if (tid == 0) {
    float sb = 0.f;
    for (int q = 0; q < NL; ++q)
      sb += __uint_as_float(__hip_atomic_load(rp + (long)q * (2 * E + 1) + 2 * E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    a.dbv_acc[b] += sb;
    __hip_atomic_store(a.ticket + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // ready for the next step
  }
}
template <typename T, int DCH, int ECH, int FBW, int FBU, bool PIPE = false>
__global__ __launch_bounds__(FBW * 64) void attn_bwd_split_kernel(AttnBwdArgs a) {
  const SatStampT0 t0 = sat_stamp_begin(a.st);
  attn_bwd_split_kernel_body<T, DCH, ECH, FBW, FBU, PIPE>(a);
#ifdef SAT_ATTN_MARK
  if (t0.on) {   // the marker wrote the record's end; the start is written here
    const int w_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (threadIdx.x == 0 && w_ < a.st.cap) a.st.p[2 + 2 * (long)w_] = t0.t0;
  }
#else
  sat_stamp_end(a.st, t0);
#endif
}

// After the time loop: dWs[b,l,e] = sum over t = T1-1 .. 0 of de[b,t,l] v[e] (1 - tanh^2(Ws[b,l,e] +
// uh[b,t,e])) -- the per-element expression and summation order of the per-step accumulation it
// replaces, so the fp32 path is bit-identical to it.  A wave owns DWS_LG rows l of one batch row b
// and a 256-wide e-chunk (lane: 4 consecutive e): each uh[b,t,e..e+3] load feeds DWS_LG x 4 tanh and
// the next step's uh is requested before the current step's arithmetic; the wave's de[b,:,l0..]
// block is staged in LDS once (a scalar load per step would wait on the scalar cache every step).
// Ws is read once.  VALU-bound: B*L*E*(T-1) tanh.  Any caption length: the de block is staged in
// chunks of DWS_TMAX steps (newest chunk first, so the summation order stays T1-1 .. 0).
constexpr int DWS_LG = 4, DWS_WAVES = 4, DWS_TMAX = 128;   // caption steps per LDS chunk
template <typename T>
__global__ __launch_bounds__(DWS_WAVES * 64) void attn_dws_kernel(const T* Ws, const float* uh_all,
                                                                 const float* de_all, const float* v_w, int B, int L,
                                                                 int E, int T1, int n_ech, int n_lg, float* out_f32,
                                                                 T* out_t) {
  __shared__ float s_de[DWS_WAVES][DWS_TMAX * DWS_LG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wid = blockIdx.x * DWS_WAVES + wv;
  const bool wok = wid < B * n_ech * n_lg;
  const int lg = wid % n_lg, ec = (wid / n_lg) % n_ech, b = wok ? wid / (n_lg * n_ech) : 0;
  const int l0 = lg * DWS_LG, e = ec * 256 + lane * 4;
  const bool eok = e < E;
  float xw[DWS_LG][4], acc[DWS_LG][4], vw[4];
  load_e4<float>(v_w + e, wok && eok, vw);
#pragma unroll
  for (int r = 0; r < DWS_LG; ++r) {
    load_e4<T>(Ws + ((long)b * L + l0 + r) * E + e, wok && eok && l0 + r < L, xw[r]);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[r][j] = 0.f;
  }
  const float* uh = uh_all + (long)b * T1 * E + e;
  float un[4];
  load_e4<float>(uh + (long)(T1 - 1) * E, wok && eok, un);
  // every wave takes part in every chunk's staging barriers (the chunk count depends on T1 only)
  for (int c0 = (T1 - 1) / DWS_TMAX * DWS_TMAX; c0 >= 0; c0 -= DWS_TMAX) {
    const int c1 = min(T1, c0 + DWS_TMAX);
    __syncthreads();   // the previous chunk's reads are done
    // stage de[b, t, l0 + r] (t in [c0, c1)) -> s_de[wv][(t - c0) * DWS_LG + r]
    for (int i = lane; i < (c1 - c0) * DWS_LG; i += 64) {
      const int t = c0 + i / DWS_LG, r = i % DWS_LG;
      s_de[wv][i] = (wok && l0 + r < L) ? de_all[((long)b * T1 + t) * L + l0 + r] : 0.f;
    }
    __syncthreads();
    if (!wok) continue;   // wave-uniform
    for (int t = c1 - 1; t >= c0; --t) {
      float uu[4] = {un[0], un[1], un[2], un[3]};
      if (t > 0) load_e4<float>(uh + (long)(t - 1) * E, eok, un);
      const float4 d4 = *(const float4*)&s_de[wv][(t - c0) * DWS_LG];
      const float d[DWS_LG] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int r = 0; r < DWS_LG; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float th = tanh_t<T>(xw[r][j] + uu[j]);
          acc[r][j] += d[r] * vw[j] * (1.f - th * th);
        }
    }
  }
  if (!wok || !eok) return;
#pragma unroll
  for (int r = 0; r < DWS_LG; ++r) {
    if (l0 + r >= L) break;
    const long o = ((long)b * L + l0 + r) * E + e;
    *(float4*)(out_f32 + o) = make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
    if (out_t) {
      if constexpr (sizeof(T) == 2) {
        uint2 u;
        bf16* h = (bf16*)&u;
#pragma unroll
        for (int j = 0; j < 4; ++j) h[j] = (bf16)acc[r][j];
        *(uint2*)(out_t + o) = u;
      } else {
        *(float4*)(out_t + o) = make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
      }
    }
  }
}

// e-chunks per lane: 1, 2 or 4 (E <= 1024)
inline int e_chunks(int E, int VN) {
  const int c = sat_cdiv(E, 64 * VN);
  return c <= 1 ? 1 : (c <= 2 ? 2 : 4);
}

template <typename T, int FDV, int NW = FNW, int FU = FFU, bool PIPE = false>
void launch_fwd(int ch, dim3 grid, hipStream_t s, const AttnFwdArgs& a) {
  if (ch == 1) hipLaunchKernelGGL((attn_fwd_kernel<T, 1, FDV, NW, FU, PIPE>), grid, dim3(NW * 64), 0, s, a);
  else if (ch == 2) hipLaunchKernelGGL((attn_fwd_kernel<T, 2, FDV, NW, FU, PIPE>), grid, dim3(NW * 64), 0, s, a);
  else hipLaunchKernelGGL((attn_fwd_kernel<T, 4, FDV, NW, FU, PIPE>), grid, dim3(NW * 64), 0, s, a);
}

}  // namespace

int sat_attention_fwd_launch(const AttnFwdArgs& args, hipStream_t s) {
  AttnFwdArgs a = args;
  a.st = sat_launch_stamps();
  const int VD = a.dtype == SAT_BF16 ? 8 : 4;
  SAT_REQUIRE(a.L <= kMaxL && a.E % VD == 0 && a.E <= 1024);
  SAT_REQUIRE((a.uh_ld % 4) == 0 && (a.hg_splits <= 1 || a.hg_split_stride % 4 == 0));
  SAT_REQUIRE(a.D % VD == 0);
  // the kernel's buffer resources (one batch row each) address < 2 GiB
  const long elt = a.dtype == SAT_BF16 ? 2 : 4, hp = a.hg_splits < 1 ? 1 : a.hg_splits;
  SAT_REQUIRE((long)a.L * a.D * elt < 0x7fffffffL && (long)a.L * a.E * elt < 0x7fffffffL);
  SAT_REQUIRE(hp > 2 || ((hp - 1) * a.hg_split_stride + (a.D > a.E ? a.D : a.E)) * 4 < 0x7fffffffL);
  // one workgroup of 16 waves per (row, 1024 bf16 columns).  Measured and removed (profiles/r3_s14, r3_s19): 512-column
  // slices (twice the workgroups; bit-identical) -- no faster at B = 64, 15.2 vs 10.3 us per step at B = 128; 8 waves
  // x 8 slots per workgroup (half the resident waves) -- 6.61-6.66 vs 6.57-6.58 ms per overlapped step
  const int NS = sat_cdiv(a.D, 64 * VD * 2);
  dim3 grid(a.B, NS);
  // more slots than one batch of 16 x 4 (L = 196): batches of 16 x 2, double-buffered (bit-identical; cfg5 step
  // 10.75 -> 10.55 ms with the backward's likewise, profiles/r5_s19).  Measured and removed (profiles/r5_s21): the
  // row split over L into chunks whose last arriver combines the softmax (flash-decoding): 30.3 -> 26.9 us alone
  // with two chunks per row but the cfg5 step 10.53 -> 10.83 ms (twice the workgroups beside the trunk), four
  // chunks 37.8 us
  const bool pipe = a.L > FNW * FFU && sat_policy().attn_pipe != 1;
  if (a.dtype == SAT_BF16) {
    if (pipe) launch_fwd<bf16, 2, FNW, 2, true>(e_chunks(a.E, 8), grid, s, a);
    else launch_fwd<bf16, 2>(e_chunks(a.E, 8), grid, s, a);
  } else {
    if (pipe) launch_fwd<float, 2, FNW, 2, true>(e_chunks(a.E, 4), grid, s, a);
    else launch_fwd<float, 2>(e_chunks(a.E, 4), grid, s, a);
  }
  return (int)hipGetLastError();
}

namespace {

template <typename T, int DCH, int ECH>
void launch_bwd_split_e(int nl, hipStream_t s, const AttnBwdArgs& a) {
  // FBU slots per wave per batch of loads.  Measured and not kept (profiles/r4_s4): one batch of 8 x 7 slots for the
  // L = 49 row at one workgroup per row (231 VGPRs instead of 171): 17.8 -> 18.7 us per step, step 6.56 -> 6.61 ms
  constexpr int FBU = DCH >= 8 ? 2 : 4;
  // chunks deeper than one batch of 8 x FBU slots (L = 196): batches of half the size, double-buffered
  if (sat_cdiv(a.L, nl) > 8 * FBU && sat_policy().attn_pipe != 1)
    hipLaunchKernelGGL((attn_bwd_split_kernel<T, DCH, ECH, 8, FBU / 2, true>), dim3(a.B, nl), dim3(8 * 64), 0, s, a);
  else
    hipLaunchKernelGGL((attn_bwd_split_kernel<T, DCH, ECH, 8, FBU>), dim3(a.B, nl), dim3(8 * 64), 0, s, a);
}
template <typename T, int DCH>
bool launch_bwd_split_d(int ech, int nl, hipStream_t s, const AttnBwdArgs& a) {
  switch (ech) {
    case 1: launch_bwd_split_e<T, DCH, 1>(nl, s, a); return true;
    case 2: launch_bwd_split_e<T, DCH, 2>(nl, s, a); return true;
    default: break;
  }
  if constexpr (sizeof(T) == 4) {
    if (ech == 3) { launch_bwd_split_e<T, DCH, 3>(nl, s, a); return true; }
    if (ech == 4) { launch_bwd_split_e<T, DCH, 4>(nl, s, a); return true; }
  }
  return false;
}
template <typename T>
bool launch_bwd_split(const AttnBwdArgs& a, hipStream_t s) {
  constexpr int VN = V16<T>::N;
  const int dch = sat_cdiv(a.D, 64 * VN), ech = sat_cdiv(a.E, 64 * VN);
  const int nl = sat_attention_bwd_chunks(a.B, a.L, a.wg_target);
  if (nl > 1 && (!a.part || !a.ticket)) return false;
  switch (dch) {
    case 1: return launch_bwd_split_d<T, 1>(ech, nl, s, a);
    case 2: return launch_bwd_split_d<T, 2>(ech, nl, s, a);
    case 3: case 4: return launch_bwd_split_d<T, 4>(ech, nl, s, a);
    case 5: case 6: case 7: case 8: return launch_bwd_split_d<T, 8>(ech, nl, s, a);
    default: return false;
  }
}

}  // namespace

int sat_attention_bwd_launch(const AttnBwdArgs& args, hipStream_t s) {
  AttnBwdArgs a = args;
  a.st = sat_launch_stamps();
  const int VD = a.dtype == SAT_BF16 ? 8 : 4;
  SAT_REQUIRE(a.L <= kMaxL && a.E % VD == 0 && a.E <= 1024);
  SAT_REQUIRE(a.D % VD == 0);
  // the split kernel's buffer resources (one batch row each) address < 2 GiB
  const long dp = a.dg_splits < 1 ? 1 : a.dg_splits;
  const long elt = a.dtype == SAT_BF16 ? 2 : 4;
  SAT_REQUIRE((long)a.L * a.D * elt < 0x7fffffffL && (long)a.L * a.E * elt < 0x7fffffffL);
  SAT_REQUIRE(dp > 8 || ((dp - 1) * a.dg_split_stride + a.D) * 4 < 0x7fffffffL);
  if (sat_policy().attn_bwd != 1 && (a.uh_ld % 4) == 0 && (a.E % 4) == 0) {
    const bool ok = a.dtype == SAT_BF16 ? launch_bwd_split<bf16>(a, s) : launch_bwd_split<float>(a, s);
    if (ok) return (int)hipGetLastError();
  }
  const int NS = sat_cdiv(a.D, 64 * VD);
  if (a.dtype == SAT_BF16) {
    hipLaunchKernelGGL(attn_bwd1_kernel<bf16>, dim3(a.B, NS), dim3(ANW * 64), 0, s, a);
    hipLaunchKernelGGL(attn_bwd2_kernel<bf16>, dim3(a.B, sat_cdiv(a.E, BSLICE)), dim3(BNW * 64), 0, s, a, NS);
  } else {
    hipLaunchKernelGGL(attn_bwd1_kernel<float>, dim3(a.B, NS), dim3(ANW * 64), 0, s, a);
    hipLaunchKernelGGL(attn_bwd2_kernel<float>, dim3(a.B, sat_cdiv(a.E, BSLICE)), dim3(BNW * 64), 0, s, a, NS);
  }
  return (int)hipGetLastError();
}

int sat_attention_dws_launch(const void* Ws, const float* uh_all, const float* de_all, const float* v_w, int B,
                             int L, int E, int T1, int dtype, float* out_f32, void* out_t, hipStream_t s) {
  SAT_REQUIRE(E % 4 == 0 && E <= 1024 && L > 0 && B > 0 && T1 > 0);
  static_assert(DWS_LG == 4, "s_de rows are read as one float4 per step");
  const int n_ech = sat_cdiv(E, 256), n_lg = sat_cdiv(L, DWS_LG);
  const dim3 grid(sat_cdiv((long)B * n_ech * n_lg, DWS_WAVES));
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(attn_dws_kernel<bf16>, grid, dim3(DWS_WAVES * 64), 0, s, (const bf16*)Ws, uh_all, de_all, v_w, B, L, E, T1,
                       n_ech, n_lg, out_f32, (bf16*)out_t);
  else
    hipLaunchKernelGGL(attn_dws_kernel<float>, grid, dim3(DWS_WAVES * 64), 0, s, (const float*)Ws, uh_all, de_all, v_w, B, L, E,
                       T1, n_ech, n_lg, out_f32, (float*)out_t);
  return (int)hipGetLastError();
}

int sat_attention_bwd_chunks(int B, int L, int wg_target) {
  const int f = sat_policy().attn_bwd_chunks;   // forced (A/B), clamped to the slots
  if (f > 0) return f < L ? (f < 16 ? f : 16) : (L < 16 ? L : 16);
  // alone: ~256 workgroups at least 4 slots deep (B = 128 -> 2 chunks, B = 64 -> 4, small test batches more);
  // beside the encoder (the decoder's split target: 64 with ResNet152 features, 128 with VGG19's): ~target
  // workgroups but at most 128 slots each -- one workgroup per row at L = 49 (fewer resident waves for the conv
  // kernels sharing the CUs: 6.69 -> 6.59 ms per overlapped step), two at L = 196 (10.90 vs 11.3 ms with one:
  // profiles/r3_s17/)
  int nl = sat_cdiv(wg_target > 0 ? wg_target : 256, B);
  if (wg_target > 0) {
    const int by_depth = sat_cdiv(L, 128);
    if (nl < by_depth) nl = by_depth;
  }
  const int by_l = sat_cdiv(L, 4);
  if (nl > by_l) nl = by_l;
  if (nl > 16) nl = 16;
  return nl < 1 ? 1 : nl;
}

size_t sat_attention_part_floats(int B, int L, int D, int E, int dtype, int wg_target) {
  const int VD = dtype == SAT_BF16 ? 8 : 4;
  const size_t two_launch = (size_t)B * sat_cdiv(D, 64 * VD) * L;
  const size_t split = (size_t)B * sat_attention_bwd_chunks(B, L, wg_target) * (2 * E + 1);
  return two_launch > split ? two_launch : split;
}

// Standalone Attention.forward (attention.py:14-21): two GEMMs + the fused kernel.
extern "C" int sat_attention_forward(int B, int L, int D, int E, int dtype, const void* img_features,
                                     const float* hidden, const float* U_w, const float* U_b, const float* W_w,
                                     const void* W_w_lp, const float* W_b, const float* v_w, const float* v_b,
                                     float* ws_scratch, float* context, float* alpha, void* stream) {
  SAT_REQUIRE(img_features && hidden && U_w && W_w && v_w && v_b && ws_scratch && context && alpha);
  SAT_REQUIRE(dtype == SAT_F32 || W_w_lp != nullptr);
  hipStream_t s = (hipStream_t)stream;
  // scratch layout: Ws [B*L*E] (dtype) followed by uh [B*E] fp32
  float* uh = ws_scratch + (size_t)B * L * E;
  SatGemm g;  // U_h = h U^T + b  (fp32 exact)
  g.M = B; g.N = E; g.K = E; g.dtype = SAT_F32;
  g.A = hidden; g.lda = E; g.B = U_w; g.ldb = E;
  g.C = uh; g.ldc = E; g.c_dtype = SAT_F32; g.bias = U_b;
  SAT_CHECK((hipError_t)sat_gemm_launch(g, s));
  SatGemm w;  // Ws = a W^T + b
  w.M = B * L; w.N = E; w.K = D; w.dtype = dtype;
  w.A = img_features; w.lda = D; w.B = dtype == SAT_BF16 ? W_w_lp : (const void*)W_w; w.ldb = D;
  w.C = ws_scratch; w.ldc = E; w.c_dtype = dtype; w.bias = W_b;
  SAT_CHECK((hipError_t)sat_gemm_launch(w, s));
  AttnFwdArgs a{};
  a.B = B; a.L = L; a.D = D; a.E = E; a.dtype = dtype;
  a.Ws = ws_scratch; a.uh = uh; a.uh_ld = E; a.v_w = v_w; a.v_b = v_b; a.a = img_features;
  a.alpha = alpha; a.alpha_ld = L; a.ctx = context; a.ctx_ld = D;
  return sat_attention_fwd_launch(a, s);
}
