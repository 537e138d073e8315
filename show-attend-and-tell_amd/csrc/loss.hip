// Fused caption loss and in-loop metrics (train.py:135-162, utils.py:44-80,101-107).
//
//   loss = CE(preds[:, :T-2] time-major, captions[:, 1:T-1])      (pads included,
//          last decoder step never scored: pack_padded_sequence with lengths T-2)
//        + alpha_c * mean_{b,l} (1 - sum_t alpha[b,t,l])^2
//
// Forward, grid = one workgroup per (b,t) row: max / sum-exp over V, the row's
// CE term, and the rank of the target logit (top-1 / top-5 correctness of
// sequence_accuracy, pad-masked, over all T-1 steps) in the same pass.  A
// single-workgroup pass folds rows in a fixed order (deterministic), forms the
// attention regulariser and its gradient, and counts caption tokens.
// Backward recomputes softmax from preds + the saved log-sum-exp:
// dL/dlogit = g * (softmax - onehot) / (B*(T-2)) for scored rows.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

constexpr int kStat = 5;  // lse, loss_row, top1, top5, nonpad

__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = -INFINITY;
  for (int i = 0; i < nw; ++i) s = fmaxf(s, red[i]);
  return s;
}

// one pass over the row: online (max, sum-exp) per thread, then a block-level merge; rows with
// V % (16 / sizeof(T)) == 0 are read as 16-byte vectors.
__device__ __forceinline__ void online_add(float& m, float& se, float x) {
  if (x > m) { se = se * expf(m - x) + 1.f; m = x; }
  else se += expf(x - m);
}

// row r's statistics: log-sum-exp, CE term (the last step is never scored), top-1 / top-5 hits (C = number of
// logits ranked above the target), non-pad flag
__device__ __forceinline__ void write_row_stats(float* stats, int r, int T1, int t, float lse, float xt, float C,
                                                bool nonpad) {
  float* st = stats + (long)r * kStat;
  st[0] = lse;
  st[1] = (t < T1 - 1) ? lse - xt : 0.f;
  st[2] = (nonpad && C < 1.f) ? 1.f : 0.f;
  st[3] = (nonpad && C < 5.f) ? 1.f : 0.f;
  st[4] = nonpad ? 1.f : 0.f;
}

// PAIRS: the bf16 pair path for even V % 8 != 0 (its own instantiation: its 64-register row would lower the
// occupancy of the others)
template <typename TT, bool PAIRS = false>
__global__ __launch_bounds__(256) void loss_rows_kernel(const TT* __restrict__ preds, const int64_t* __restrict__ caps,
                                                        int B, int T, int V, int pad_id, float* __restrict__ stats) {
  __shared__ float red_m[4], red_s[4], red_c[4];
  const int r = blockIdx.x;
  const int T1 = T - 1;
  const int b = r / T1, t = r - b * T1;
  const TT* x = preds + (long)r * V;
  const int tgt = (int)caps[(long)b * T + t + 1];
  const float xt = (tgt >= 0 && tgt < V) ? (float)x[tgt] : 0.f;
  float m = -INFINITY, se = 0.f, cnt = 0.f;
  constexpr int VEC = 16 / sizeof(TT);
  constexpr int RV = 12;   // register-resident row: up to RV 16-byte vectors per thread (V <= 24576 bf16 / 12288 fp32)
  if (V % VEC == 0 && V / VEC <= RV * 256) {
    // the whole row in registers (every load requested up front), then two passes over registers: the
    // thread max, the block max, then one v_exp per element against it (the online form paid a branch and
    // up to two exps per element: VALU-bound at V = 10000, 36 us per 3328 rows)
    const int NV = V / VEC;
    uint4 u[RV];
#pragma unroll
    for (int k = 0; k < RV; ++k) {
      const int c = threadIdx.x + k * 256;
      u[k] = c < NV ? *(const uint4*)(x + (long)c * VEC) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < RV; ++k) {
      const int c = threadIdx.x + k * 256;
      if (c < NV) {
        const TT* h = (const TT*)&u[k];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float xv = (float)h[j];
          m = fmaxf(m, xv);
          cnt += (xv > xt || (xv == xt && c * VEC + j < tgt)) ? 1.f : 0.f;
        }
      }
    }
    const float M = block_max(m, red_m);
#pragma unroll
    for (int k = 0; k < RV; ++k) {
      const int c = threadIdx.x + k * 256;
      if (c < NV) {
        const TT* h = (const TT*)&u[k];
#pragma unroll
        for (int j = 0; j < VEC; ++j) se += __expf((float)h[j] - M);
      }
    }
    // the block's sums in a fixed order (wave shuffle tree, then the 4 waves in order)
    se = wave_sum(se);
    cnt = wave_sum(cnt);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red_s[w] = se; red_c[w] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
      const float S = (red_s[0] + red_s[1]) + (red_s[2] + red_s[3]);
      const float C = (red_c[0] + red_c[1]) + (red_c[2] + red_c[3]);
      write_row_stats(stats, r, T1, t, M + logf(S), xt, C, tgt != pad_id);
    }
    return;
  }
  if constexpr (PAIRS) {
    {
      // bf16 rows of an even length that is not a multiple of 8 (BERT's V = 30522): 4-byte aligned, so the row goes
      // into registers as bf16 pairs (up to 64 per thread, all requested up front), then the same two register
      // passes as the 16-byte path -- the element loop below paid a 2-byte load and a branchy online update per logit
      // (240 us per 3968 x 30522 logits, profiles/r6_s13)
      constexpr int RD = 64;
      const int ND = V / 2;
      const unsigned* xd = (const unsigned*)x;
      unsigned u[RD];
#pragma unroll
      for (int k = 0; k < RD; ++k) {
        const int c = threadIdx.x + k * 256;
        u[k] = c < ND ? xd[c] : 0u;
      }
#pragma unroll
      for (int k = 0; k < RD; ++k) {
        const int c = threadIdx.x + k * 256;
        if (c < ND) {
          const TT* h = (const TT*)&u[k];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float xv = (float)h[j];
            m = fmaxf(m, xv);
            cnt += (xv > xt || (xv == xt && c * 2 + j < tgt)) ? 1.f : 0.f;
          }
        }
      }
      const float M = block_max(m, red_m);
#pragma unroll
      for (int k = 0; k < RD; ++k) {
        const int c = threadIdx.x + k * 256;
        if (c < ND) {
          const TT* h = (const TT*)&u[k];
          se += __expf((float)h[0] - M);
          se += __expf((float)h[1] - M);
        }
      }
      se = wave_sum(se);
      cnt = wave_sum(cnt);
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      if (lane == 0) { red_s[w] = se; red_c[w] = cnt; }
      __syncthreads();
      if (threadIdx.x == 0) {
        const float S = (red_s[0] + red_s[1]) + (red_s[2] + red_s[3]);
        const float C = (red_c[0] + red_c[1]) + (red_c[2] + red_c[3]);
        write_row_stats(stats, r, T1, t, M + logf(S), xt, C, tgt != pad_id);
      }
      return;
    }
  }
  if (V % VEC == 0) {
    // LU vectors per thread in flight (the per-thread order c = tid, tid + 256, .. is unchanged)
    constexpr int LU = 4;
    const int NV = V / VEC;
    for (int c0 = threadIdx.x; c0 < NV; c0 += LU * 256) {
      uint4 u[LU];
#pragma unroll
      for (int k = 0; k < LU; ++k) {
        const int c = c0 + k * 256;
        u[k] = c < NV ? *(const uint4*)(x + (long)c * VEC) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int k = 0; k < LU; ++k) {
        const int c = c0 + k * 256;
        if (c >= NV) break;
        const TT* h = (const TT*)&u[k];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float xv = (float)h[j];
          const int v = c * VEC + j;
          online_add(m, se, xv);
          cnt += (xv > xt || (xv == xt && v < tgt)) ? 1.f : 0.f;
        }
      }
    }
  } else {
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
      const float xv = (float)x[v];
      online_add(m, se, xv);
      cnt += (xv > xt || (xv == xt && v < tgt)) ? 1.f : 0.f;
    }
  }
  // merge (m, se) pairs: across the wave, then the 4 waves in a fixed order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(se, o, 64);
    const float nm = fmaxf(m, om);
    se = (nm == -INFINITY) ? 0.f : se * expf(m - nm) + os * expf(om - nm);
    m = nm;
    cnt += __shfl_xor(cnt, o, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { red_m[w] = m; red_s[w] = se; red_c[w] = cnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red_m[0], S = red_s[0], C = red_c[0];
    for (int i = 1; i < 4; ++i) {
      const float nm = fmaxf(M, red_m[i]);
      S = S * expf(M - nm) + red_s[i] * expf(red_m[i] - nm);
      M = nm;
      C += red_c[i];
    }
    write_row_stats(stats, r, T1, t, M + logf(S), xt, C, tgt != pad_id);
  }
}

// attention regulariser, one thread per (b, l): the sum over steps, its gradient, and a block
// partial of sum (1 - s)^2 (folded in a fixed order by loss_reduce_kernel).
__global__ __launch_bounds__(256) void loss_reg_kernel(const float* __restrict__ alphas, int B, int T1, int L,
                                                       float alpha_c, float* __restrict__ dreg,
                                                       float* __restrict__ part) {
  __shared__ float red[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const float inv_bl = 1.0f / (float)(B * L);
  float reg = 0.f;
  if (i < B * L) {
    const int b = i / L, l = i - b * L;
    float ssum = 0.f;
    for (int t = 0; t < T1; ++t) ssum += alphas[((long)b * T1 + t) * L + l];
    const float d = 1.f - ssum;
    reg = d * d;
    dreg[i] = alpha_c * 2.f * (ssum - 1.f) * inv_bl;
  }
  reg = block_sum(reg, red);
  if (threadIdx.x == 0) part[blockIdx.x] = reg;
}

__global__ __launch_bounds__(1024) void loss_reduce_kernel(const float* __restrict__ stats, const float* __restrict__ part,
                                                           int nparts, const int64_t* __restrict__ caps, int B, int T,
                                                           int L, float alpha_c, int s0, int s1, int s2,
                                                           float* __restrict__ out, float* __restrict__ loss_out) {
  __shared__ float red[16];
  const int T1 = T - 1, R = B * T1;
  float ce = 0.f, c1 = 0.f, c5 = 0.f, np = 0.f;
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const float* st = stats + (long)r * kStat;
    ce += st[1]; c1 += st[2]; c5 += st[3]; np += st[4];
  }
  ce = block_sum(ce, red);
  c1 = block_sum(c1, red);
  c5 = block_sum(c5, red);
  np = block_sum(np, red);
  float reg = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) reg += part[i];
  reg = block_sum(reg, red);
  float cl = 0.f;
  for (int i = threadIdx.x; i < B * T; i += blockDim.x) {
    const int64_t tok = caps[i];
    cl += (tok != s0 && tok != s1 && tok != s2) ? 1.f : 0.f;
  }
  cl = block_sum(cl, red);
  if (threadIdx.x == 0) {
    const float cem = ce / (float)(B * (T1 - 1));
    const float regm = alpha_c * (reg * (1.0f / (float)(B * L)));
    out[0] = cem + regm;
    if (loss_out) loss_out[0] = cem + regm;
    out[1] = cem;
    out[2] = regm;
    out[3] = c1; out[4] = c5; out[5] = np; out[6] = cl;
  }
}

// dL/dlogit = g * (softmax - onehot) / (B*(T-2)) for scored rows, 0 for the unscored last step.
// MASK: the logits are a ReLU's output (decoder.py:117-125 advanced deep output), and the
// gradient leaves through that ReLU: zero where the logit is not positive (fused here so the
// decoder skips its own mask pass over the [B*(T-1), V] gradient).  16-byte vectors when
// V % (16 / sizeof(T)) == 0.
template <typename TT, bool MASK>
__global__ __launch_bounds__(256) void loss_bwd_kernel(const TT* __restrict__ preds, const int64_t* __restrict__ caps,
                                                       int B, int T, int V, int L, const float* __restrict__ stats,
                                                       const float* __restrict__ dreg, const float* __restrict__ grad_out,
                                                       TT* __restrict__ dpreds, long ldo, float* __restrict__ dalphas) {
  const int r = blockIdx.x;
  const int T1 = T - 1;
  const int b = r / T1, t = r - b * T1;
  const float g = grad_out ? grad_out[0] : 1.f;
  const TT* x = preds + (long)r * V;
  TT* dx = dpreds + (long)r * ldo;
  const bool scored = t < T1 - 1;
  const int tgt = scored ? (int)caps[(long)b * T + t + 1] : -1;
  const float lse = scored ? stats[(long)r * kStat] : 0.f;
  const float scale = scored ? g / (float)(B * (T1 - 1)) : 0.f;
  auto grad = [&](float xv, int v) {
    float p = scored ? expf(xv - lse) : 0.f;
    if (v == tgt) p -= 1.f;
    float d = p * scale;
    if (MASK && !(xv > 0.f)) d = 0.f;
    return d;
  };
  constexpr int VEC = 16 / sizeof(TT);
  if (V % VEC == 0 && ldo % VEC == 0) {
    const __amdgpu_buffer_rsrc_t rdx = sat_out_rsrc(dx, (long)sizeof(TT) * V);   // this row: offsets < 2 GiB
    constexpr int LU = 4;   // vectors per thread in flight
    const int NV = V / VEC;
    for (int c0 = threadIdx.x; c0 < NV; c0 += LU * 256) {
      uint4 u[LU];
#pragma unroll
      for (int k = 0; k < LU; ++k) {
        const int c = c0 + k * 256;
        u[k] = c < NV ? *(const uint4*)(x + (long)c * VEC) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int k = 0; k < LU; ++k) {
        const int c = c0 + k * 256;
        if (c >= NV) break;
        const TT* h = (const TT*)&u[k];
        uint4 o;
        TT* q = (TT*)&o;
#pragma unroll
        for (int j = 0; j < VEC; ++j) q[j] = (TT)grad((float)h[j], c * VEC + j);
        sat_st16(rdx, (unsigned)((long)c * VEC * sizeof(TT)), o);   // write-through (sat_common.h)
      }
    }
  } else if (sizeof(TT) == 2 && V % 2 == 0 && ldo % 2 == 0) {
    // even bf16 rows (4-byte aligned): pairs, LU in flight per thread
    constexpr int LU = 8;
    const int ND = V / 2;
    const unsigned* xd = (const unsigned*)x;
    unsigned* dd = (unsigned*)dx;
    for (int c0 = threadIdx.x; c0 < ND; c0 += LU * 256) {
      unsigned u[LU];
#pragma unroll
      for (int k = 0; k < LU; ++k) {
        const int c = c0 + k * 256;
        u[k] = c < ND ? xd[c] : 0u;
      }
#pragma unroll
      for (int k = 0; k < LU; ++k) {
        const int c = c0 + k * 256;
        if (c >= ND) break;
        const TT* h = (const TT*)&u[k];
        unsigned o;
        TT* q = (TT*)&o;
        q[0] = (TT)grad((float)h[0], 2 * c);
        q[1] = (TT)grad((float)h[1], 2 * c + 1);
        dd[c] = o;
      }
    }
  } else {
    for (int v = threadIdx.x; v < V; v += blockDim.x) dx[v] = (TT)grad((float)x[v], v);
  }
  // a padded destination (sat_caption_loss_backward_ld): zero columns V..ldo-1
  for (long v = V + threadIdx.x; v < ldo; v += blockDim.x) dx[v] = (TT)0.f;
  for (int l = threadIdx.x; l < L; l += blockDim.x) dalphas[(long)r * L + l] = g * dreg[(long)b * L + l];
}

}  // namespace

extern "C" size_t sat_caption_loss_workspace_bytes(int B, int T, int L) {
  return ((size_t)B * (T - 1) * kStat + (size_t)B * L + sat_cdiv((long)B * L, 256) + 64) * sizeof(float);
}

namespace {
int loss_forward(int B, int T, int V, int L, int dtype, const void* preds, const float* alphas, const int64_t* captions,
                 float alpha_c, int pad_id, int skip0, int skip1, int skip2, void* workspace, float* out,
                 float* loss_out, void* stream) {
  SAT_REQUIRE(preds && alphas && captions && workspace && out && B > 0 && T >= 3 && V > 0 && L > 0);
  hipStream_t s = (hipStream_t)stream;
  const int R = B * (T - 1);
  float* stats = (float*)workspace;
  float* dreg = stats + (size_t)R * kStat;
  if (dtype == SAT_BF16 && V % 8 != 0 && V % 2 == 0 && V / 2 <= 64 * 256)
    hipLaunchKernelGGL((loss_rows_kernel<bf16, true>), dim3(R), dim3(256), 0, s, (const bf16*)preds, captions, B, T, V,
                       pad_id, stats);
  else if (dtype == SAT_BF16)
    hipLaunchKernelGGL(loss_rows_kernel<bf16>, dim3(R), dim3(256), 0, s, (const bf16*)preds, captions, B, T, V, pad_id, stats);
  else
    hipLaunchKernelGGL(loss_rows_kernel<float>, dim3(R), dim3(256), 0, s, (const float*)preds, captions, B, T, V, pad_id, stats);
  SAT_LAUNCH_CHECK();
  float* part = dreg + (size_t)B * L;
  const int nparts = sat_cdiv((long)B * L, 256);
  hipLaunchKernelGGL(loss_reg_kernel, dim3(nparts), dim3(256), 0, s, alphas, B, T - 1, L, alpha_c, dreg, part);
  SAT_LAUNCH_CHECK();
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(1024), 0, s, stats, (const float*)part, nparts, captions, B, T,
                     L, alpha_c, skip0, skip1, skip2, out, loss_out);
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int sat_caption_loss_forward(int B, int T, int V, int L, int dtype, const void* preds, const float* alphas,
                                        const int64_t* captions, float alpha_c, int pad_id, int skip0, int skip1,
                                        int skip2, void* workspace, float* out, void* stream) {
  return loss_forward(B, T, V, L, dtype, preds, alphas, captions, alpha_c, pad_id, skip0, skip1, skip2, workspace, out,
                      nullptr, stream);
}

extern "C" int sat_caption_loss_forward_loss_out(int B, int T, int V, int L, int dtype, const void* preds,
                                                 const float* alphas, const int64_t* captions, float alpha_c,
                                                 int pad_id, int skip0, int skip1, int skip2, void* workspace,
                                                 float* out, float* loss_out, void* stream) {
  SAT_REQUIRE(loss_out);
  return loss_forward(B, T, V, L, dtype, preds, alphas, captions, alpha_c, pad_id, skip0, skip1, skip2, workspace, out,
                      loss_out, stream);
}

namespace {
int loss_backward(int B, int T, int V, int L, int dtype, const void* preds, const int64_t* captions, void* workspace,
                  const float* grad_out, void* d_preds, long ldo, float* d_alphas, bool relu_mask, hipStream_t s) {
  SAT_REQUIRE(preds && captions && workspace && d_preds && d_alphas && B > 0 && T >= 3 && ldo >= V);
  const int R = B * (T - 1);
  const float* stats = (const float*)workspace;
  const float* dreg = stats + (size_t)R * kStat;
  if (dtype == SAT_BF16) {
    if (relu_mask)
      hipLaunchKernelGGL((loss_bwd_kernel<bf16, true>), dim3(R), dim3(256), 0, s, (const bf16*)preds, captions, B, T,
                         V, L, stats, dreg, grad_out, (bf16*)d_preds, ldo, d_alphas);
    else
      hipLaunchKernelGGL((loss_bwd_kernel<bf16, false>), dim3(R), dim3(256), 0, s, (const bf16*)preds, captions, B,
                         T, V, L, stats, dreg, grad_out, (bf16*)d_preds, ldo, d_alphas);
  } else {
    if (relu_mask)
      hipLaunchKernelGGL((loss_bwd_kernel<float, true>), dim3(R), dim3(256), 0, s, (const float*)preds, captions, B,
                         T, V, L, stats, dreg, grad_out, (float*)d_preds, ldo, d_alphas);
    else
      hipLaunchKernelGGL((loss_bwd_kernel<float, false>), dim3(R), dim3(256), 0, s, (const float*)preds, captions,
                         B, T, V, L, stats, dreg, grad_out, (float*)d_preds, ldo, d_alphas);
  }
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int sat_caption_loss_backward(int B, int T, int V, int L, int dtype, const void* preds,
                                         const int64_t* captions, float alpha_c, void* workspace,
                                         const float* grad_out, void* d_preds, float* d_alphas, void* stream) {
  (void)alpha_c;
  return loss_backward(B, T, V, L, dtype, preds, captions, workspace, grad_out, d_preds, V, d_alphas, false,
                       (hipStream_t)stream);
}

extern "C" int sat_caption_loss_backward_relu(int B, int T, int V, int L, int dtype, const void* preds,
                                              const int64_t* captions, float alpha_c, void* workspace,
                                              const float* grad_out, void* d_preds, float* d_alphas, void* stream) {
  (void)alpha_c;
  return loss_backward(B, T, V, L, dtype, preds, captions, workspace, grad_out, d_preds, V, d_alphas, true,
                       (hipStream_t)stream);
}

extern "C" int sat_caption_loss_backward_ld(int B, int T, int V, int L, int dtype, const void* preds,
                                            const int64_t* captions, float alpha_c, void* workspace,
                                            const float* grad_out, void* d_preds, int64_t ld_dpreds,
                                            float* d_alphas, int relu_mask, void* stream) {
  (void)alpha_c;
  return loss_backward(B, T, V, L, dtype, preds, captions, workspace, grad_out, d_preds, (long)ld_dpreds, d_alphas,
                       relu_mask != 0, (hipStream_t)stream);
}
