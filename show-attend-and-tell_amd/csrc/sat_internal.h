// Internal host-side launchers shared between the kernel translation units.
#pragma once
#include "sat_common.h"

int sat_mean_rows(const void* a, int B, int L, int D, int dtype, float* out_f32, void* out_t, hipStream_t s);
// cols_readable: X's rows may be read up to N rounded up to the vector width (zero-padded or harmless columns that
// are summed and dropped), so an N that is not a multiple of it still takes the vector kernel
int sat_colsum(const void* X, int dtype, long ld, int R, int N, float* out, int accumulate, float* out2,
               float* scratch, hipStream_t s, int cols_readable = 0);
size_t sat_colsum_scratch_floats(int R, int N);
// several column sums in one partial + one final launch (<= 8 segments, same arithmetic as sat_colsum); the
// scratch holds sum_i 64 * N_i floats
struct SatColsumSeg {
  const void* X; int dtype; long ld; int R, N; float* out; int accumulate; float* out2;
  int cols_readable;   // as sat_colsum's
};
int sat_colsum_multi(const SatColsumSeg* segs, int n, float* scratch, hipStream_t s);
// zero n (<= 8) fp32 ranges in one launch (graph-safe memset)
int sat_zero_multi(float* const* ptrs, const long* counts, int n, hipStream_t s);
// zero up to 12 fp32 row blocks (rows x cols at row stride ld) in one launch
struct SatZeroSeg {
  float* p;
  long rows, cols, ld;
};
int sat_zero_segs(const SatZeroSeg* seg, int n, hipStream_t s);
// 1 when sat_gemm_launch would run this problem as an atomic split-K (fp32 C accumulated by atomics: with
// beta = 0 it zeroes C first unless SatGemm::c_zeroed says the caller already did)
int sat_gemm_splits_atomically(const SatGemm& g);
int sat_embed_gather(const float* W, const int32_t* tok, int B, int T1, long tok_stride_b, int E, int dtype,
                     void* out, long out_ld, hipStream_t s);
int sat_embed_scatter_add(const float* dX, const int32_t* tok, int R, int E, float* G, hipStream_t s);
// teacher forcing: tok[b, t] = captions[b, t] (t < T-1) and their embedding rows, one launch
int sat_embed_gather_captions(const float* W, const int64_t* caps, int B, int T, int E, int dtype, void* out,
                              long out_ld, int32_t* tok, hipStream_t s);
int sat_argmax_rows(const void* X, int dtype, long ld, int B, int V, int32_t* out, long out_stride,
                    const float* emb, int E, void* emb_out, long emb_ld, hipStream_t s);
// torch.argmax order (decoder.py:132): NaN is the largest value (first NaN wins), otherwise the larger value, then
// the smaller index; (x, xi) replaces (y, yi) when it comes first in that order -- a total order, so any reduction
// tree gives the same winner
__device__ __forceinline__ bool sat_argmax_better(float x, int xi, float y, int yi) {
  const bool xn = x != x, yn = y != y;
  if (xn || yn) return xn && (!yn || xi < yi);
  return x > y || (x == y && xi < yi);
}

// ---- deterministic dense embedding gradient (nn.Embedding backward = index_add over the fed tokens, decoder.py:87,
// 133): G[tok[r], :] += dX[r, :] as per-token sums in row order (one sort launch + a segment-sum launch + a fix-up
// launch for tokens whose rows span several pieces), no fp32 atomics.  R <= sat_embed_sorted_max_rows(), V < 2^18.
int sat_embed_sorted_max_rows();
size_t sat_embed_sorted_ws_bytes(int R, int E);
// accumulate = 0: the caller zeroed G on this stream (each touched row is then stored, not read back)
int sat_embed_scatter_add_sorted(const float* dX, const int32_t* tok, int R, int E, float* G, int accumulate, void* ws,
                                 hipStream_t s);

// ---- the greedy decoder step's output head (no teacher forcing, bf16; skinny.hip) ----
// sat_skinny_dual_try: two skinny products of one shape in one launch (returns 1 when launched)
int sat_skinny_dual_try(const SatGemm& g1, const SatGemm& g2, hipStream_t s, int* err);
// advanced deep output, middle part (decoder.py:149-156): fh = relu(hd f_h^T + b_h), fz = relu(sum of fz_splits
// f_z pre-activation slabs + b_z), comb = fh + fz + emb; fh / fz saved fp32 (the backward's ReLU masks)
struct HeadMidArgs {
  int B, E;
  const bf16* hd; long hd_ld;                  // dropout(h) rows of the step
  const bf16* fh_w; const float* fh_b;        // [E][E], [E]
  const float* fzp; long fzp_ld; int fz_splits; long fz_split_stride; const float* fz_b;
  const bf16* emb; long emb_ld;               // embedding rows fed at the step
  float* fh; float* fz; long f_ld;            // out fp32
  bf16* comb; long comb_ld;                   // out: f_out's input
};
int sat_greedy_head_mid(const HeadMidArgs& a, hipStream_t s);
// vocabulary head of one step (decoder.py:125 / 157): preds = act(x W^T + b) in bf16, plus per column block the
// argmax of every row over the rounded logits (pval / pidx [sat_greedy_head_blocks][B])
struct HeadOutArgs {
  int B, V, E, relu;
  const bf16* x; long x_ld;
  const bf16* w; const float* bias;           // [V][E], [V]
  bf16* preds; long preds_ld;
  float* pval; int32_t* pidx;
};
int sat_greedy_head_out(const HeadOutArgs& a, hipStream_t s);
// the number of argmax partials per row sat_greedy_head_out writes for these shapes (<= ceil(V / 16))
int sat_greedy_head_blocks(int B, int V, int E);
// the fused greedy step's shapes: B <= 128 rows, E a multiple of 64 (the LSTM kernel's token fold) up to 1024
int sat_greedy_supported(int B, int E);
int sat_cast_launch(const void* x, int xd, void* y, int yd, long n, hipStream_t s);

// ---- attention (attention.py:14-21 + decoder.py:97-100 gate) ----
struct AttnFwdArgs {
  int B, L, D, E, dtype;
  const void* Ws;            // [B,L,E]  dtype
  const float* uh; long uh_ld;        // U h + b_U, row b at uh + b*uh_ld
  const float* v_w; const float* v_b; // [E], [1]
  const void* a;             // [B,L,D] dtype
  const float* gate_pre; long gate_ld;  // f_beta h + b (nullable: plain attention)
  float* alpha; long alpha_ld;          // [B, *, L]
  float* ctx; long ctx_ld;              // fp32 context
  void* ctx_t; long ctx_t_ld;           // dtype context copy (nullable)
  float* gate; long gate_out_ld;        // sigmoid gate (nullable)
  void* gated; long gated_ld;           // dtype gate*context (nullable)
  float* uh_save; long uh_save_ld;      // copy of U h + b (nullable)
  int hg_splits; long hg_split_stride;  // uh / gate_pre are sums of hg_splits partial slabs (0|1 = plain)
  SatStamps st;                         // in-kernel launch timestamps (set by the launcher)
};
int sat_attention_fwd_launch(const AttnFwdArgs& a, hipStream_t s);

struct AttnBwdArgs {
  int B, L, D, E, dtype;
  const void* Ws; const void* a;
  const float* uh; long uh_ld;          // saved U h + b of this step
  const float* v_w;
  const float* alpha; long alpha_ld;    // this step's alpha rows
  const float* d_alpha_ext; long d_alpha_ext_ld;  // loss gradient wrt alphas (this step), nullable
  const float* d_gated; long d_gated_ld;          // dL/d(gate*context)  [B,D]
  const float* gate; long gate_ld;
  const float* ctx; long ctx_ld;
  const float* d_ctx_ext; long d_ctx_ext_ld;      // extra dL/dcontext (ado head), nullable
  float* d_uh; long d_uh_ld;            // out fp32 dL/d(U h)  (== dL/dU_b rows)
  void* d_uh_t;                         // out dtype copy (same ld), nullable
  float* d_gpre; long d_gpre_ld;        // out fp32 dL/d(f_beta h + b)
  void* d_gpre_t;                       // out dtype copy, nullable
  float* de_out; long de_ld;            // out: this step's dL/d(score) rows, row b at de_out + b*de_ld
  float* dv_acc;                        // [B,E]  += dL/dv (per row b)
  float* dbv_acc;                       // [B]    += dL/dv.bias
  float* part;                          // scratch: [B, NS, L] (two-launch form) | [B, NL, 2E+1] (split form)
  unsigned* ticket;                     // [B] arrival counters of the split form (zero between launches)
  int dg_splits; long dg_split_stride;  // d_gated = sum of dg_splits partial slabs (0|1 = plain)
  int wg_target;                        // workgroups the split form aims for (0 = 256; the decoder's split target)
  SatStamps st;                         // in-kernel launch timestamps (set by the launcher)
};
int sat_attention_bwd_launch(const AttnBwdArgs& a, hipStream_t s);
// dL/dWs[b,l,:] = sum_t de[b,t,l] v (1 - tanh^2(Ws[b,l,:] + uh[b,t,:])), summed t = T1-1 .. 0 (the
// BPTT order), after the time loop: fp32 rows (out_f32) and a dtype copy (out_t).
int sat_attention_dws_launch(const void* Ws, const float* uh_all, const float* de_all, const float* v_w, int B,
                             int L, int E, int T1, int dtype, float* out_f32, void* out_t, hipStream_t s);

// ---- LSTMCell pointwise (decoder.py:115, nn.LSTMCell gate order i,f,g,o) ----
struct LstmFwdArgs {
  int B, E, dtype;
  const float* hpart; long hpart_ld;    // h W_hh^T + b_hh     [B,4E]
  const float* xpart; long xpart_ld;    // emb W_ih_e^T + b_ih [B,4E]
  const float* cpart; long cpart_ld;    // ctx W_ih_c^T        [B,4E] (ld 0 = broadcast row)
  const float* c_prev; long c_prev_ld;
  float* gates; long gates_ld;          // pre-activation save
  float* c_out; long c_out_ld;
  float* c_next_in; long c_next_in_ld;  // nullable: copy of c_out as next step's input
  float* h_out; long h_out_ld;          // fp32
  void* h_out_t; long h_out_t_ld;       // dtype copy (nullable)
  void* h_next_in_t; long h_next_in_t_ld;  // dtype copy as next step's input (nullable)
  int h_splits; long h_split_stride;    // hpart = sum of h_splits slabs
  int c_splits; long c_split_stride;    // cpart = sum of c_splits slabs
  // nullable: dropout(h) (decoder.py:121-125) in dtype -- the greedy step's head input -- with the arithmetic of
  // sat_dropout_apply (keep from mask_in, or drawn from (seed ^ *seed_ptr, b, drop_t, e); keep-mask to mask_out)
  void* hd_t; long hd_ld;
  int drop_training, drop_has_mask, drop_t;
  const uint8_t* mask_in; uint8_t* mask_out; long mask_ld;
  uint64_t seed; const uint64_t* seed_ptr;
  // nullable: the greedy step's token fold -- the token fed at this step is the argmax of the previous step's vocabulary
  // head, reduced here from its per-block partials (am_val / am_idx [am_ncb][B], sat_greedy_head_out); the embedding
  // half of the gate pre-activation is then read from the token table xt [V][4E] (xpart unused), and the row's
  // embedding (emb_t, dtype) and the token (tok_out[b * tok_ld]) are written for the head and the backward.  E % 64 == 0
  const float* am_val; const int32_t* am_idx; int am_ncb, am_V;
  const float* xt; const float* emb; void* emb_t; long emb_t_ld;
  int32_t* tok_out; long tok_ld;
  SatStamps st;                         // in-kernel launch timestamps (set by the launcher)
};
int sat_lstm_fwd_launch(const LstmFwdArgs& a, hipStream_t s);

struct LstmBwdArgs {
  int B, E, dtype;
  const float* gates; long gates_ld;
  const float* c_prev; long c_prev_ld;
  const float* c_new; long c_new_ld;
  const float* dh_rec; long dh_rec_ld;  // nullable (last step)
  const float* dh_head; long dh_head_ld;  // nullable
  const uint8_t* mask; long mask_ld;    // dropout keep-mask for dh_head (nullable = no dropout)
  float* dc;                            // [B,E] in: dc from step t+1 (or zeros), out: dc_prev
  int dc_zero;                          // treat incoming dc as zero
  float* d_gates; long d_gates_ld;      // out fp32
  void* d_gates_t; long d_gates_t_ld;   // out dtype copy (nullable)
  int dh_splits; long dh_split_stride;  // dh_rec = sum of dh_splits slabs
  SatStamps st;                         // in-kernel launch timestamps (set by the launcher)
};
int sat_lstm_bwd_launch(const LstmBwdArgs& a, hipStream_t s);

// ---- misc decoder elementwise ----
int sat_tanh_pair_bwd(const float* d_h, int dh_splits, long dh_split_stride, const float* d_c, const float* hc0,
                      int B, int E, float* dpre_f32, void* dpre_t, int dtype, hipStream_t s);
int sat_dropout_apply(const float* h, long h_ld, int B, int T1, int E, int training, int has_mask,
                      const uint8_t* mask_in, uint8_t* mask_out, long mask_ld, uint64_t seed,
                      const uint64_t* seed_ptr, int t_offset, void* out_t, long out_ld, int dtype, hipStream_t s);
int sat_bump_seed(uint64_t* p, hipStream_t s);
int sat_relu_mask_mul(const void* d, const void* ref, long n, int dtype, void* out_t, hipStream_t s);
// [rows][cols] -> [rows][ld_out] zero-padded past cols, ReLU-masked by ref when ref != null
int sat_pad_rows(const void* d, const void* ref, int rows, int cols, int ld_out, int dtype, void* out,
                 hipStream_t s);
int sat_ado_bwd_split(const float* d_comb, const float* fh, const float* fz, long n, int dtype, void* d_fh_t,
                      void* d_fz_t, hipStream_t s);
int sat_ado_combine(const float* fh, const float* fz, const void* emb, long n, int dtype,
                    void* comb_t, hipStream_t s);
int sat_fill_const(float* p, long n, float v, hipStream_t s);
int sat_zero_rows(float* p, long ld, long rows, long cols, hipStream_t s);   // graph-safe memset
int sat_broadcast_rows(const void* src, int B, int D, int T1, int dtype, void* dst, hipStream_t s);
int sat_row_sum_accumulate(const float* X, int R, int N, float* out, hipStream_t s);
size_t sat_attention_part_floats(int B, int L, int D, int E, int dtype, int wg_target);
// chunks of L one batch row's attention backward is split over (sat_attention_bwd_launch), aiming for wg_target
// workgroups (0 = 256)
int sat_attention_bwd_chunks(int B, int L, int wg_target);

// sum of `n` partial slabs (n <= 1: plain read).  Three independent accumulators keep several
// slab loads in flight (a single running sum serialises one L2 round trip per slab).
__device__ __forceinline__ float sum_parts(const float* p, long idx, int n, long stride) {
  float a0 = p[idx];
  if (n <= 1) return a0;
  float a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 1;
  for (; s + 2 < n; s += 3) {
    const float x1 = p[idx + s * stride], x2 = p[idx + (s + 1) * stride], x3 = p[idx + (s + 2) * stride];
    a1 += x1; a2 += x2; a3 += x3;
  }
  for (; s < n; ++s) a1 += p[idx + s * stride];
  return (a0 + a1) + (a2 + a3);
}

// 16-byte form of sum_parts (same summation order per element)
__device__ __forceinline__ float4 f4add(float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); }
__device__ __forceinline__ float4 sum_parts4(const float* p, long idx, int n, long stride) {
  float4 a0 = *(const float4*)(p + idx);
  if (n <= 1) return a0;
  float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1, a3 = a1;
  int sp = 1;
  for (; sp + 2 < n; sp += 3) {
    const float4 x = *(const float4*)(p + idx + sp * stride), y = *(const float4*)(p + idx + (sp + 1) * stride),
                 z = *(const float4*)(p + idx + (sp + 2) * stride);
    a1 = f4add(a1, x); a2 = f4add(a2, y); a3 = f4add(a3, z);
  }
  for (; sp < n; ++sp) a1 = f4add(a1, *(const float4*)(p + idx + sp * stride));
  return f4add(f4add(a0, a1), f4add(a2, a3));
}

// sum_parts4 over slabs already loaded (x[q] = slab q, zeros past n; n <= NP): the same additions in the same order,
// so a kernel can request its slabs with the rest of its loads and sum them later
template <int NP>
__device__ __forceinline__ float4 sum_loaded_parts4(const float4 (&x)[NP], int n) {
  if (n <= 1) return x[0];
  const int full = 3 * ((n - 1) / 3);   // slabs 1 .. full: three accumulators in turn; the rest: the first
  float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1, a3 = a1;
#pragma unroll
  for (int q = 1; q < NP; ++q) {
    if (q >= n) break;
    if (q <= full && (q - 1) % 3 == 1) a2 = f4add(a2, x[q]);
    else if (q <= full && (q - 1) % 3 == 2) a3 = f4add(a3, x[q]);
    else a1 = f4add(a1, x[q]);
  }
  return f4add(f4add(x[0], a1), f4add(a2, a3));
}

// the scalar form (sum_parts's order)
template <int NP>
__device__ __forceinline__ float sum_loaded_parts(const float (&x)[NP], int n) {
  if (n <= 1) return x[0];
  const int full = 3 * ((n - 1) / 3);
  float a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
  for (int q = 1; q < NP; ++q) {
    if (q >= n) break;
    if (q <= full && (q - 1) % 3 == 1) a2 += x[q];
    else if (q <= full && (q - 1) % 3 == 2) a3 += x[q];
    else a1 += x[q];
  }
  return (x[0] + a1) + (a2 + a3);
}

// ---- LSTM cell arithmetic (nn.LSTMCell, gate order i, f, g, o; decoder.py:115) of the pointwise kernels
// (lstm.hip) ----
__device__ __forceinline__ void lstm_cell_fwd(float gi, float gf, float gg, float go, float c_prev, float& c, float& h) {
  const float ig = 1.f / (1.f + expf(-gi));
  const float fg = 1.f / (1.f + expf(-gf));
  const float g = tanhf(gg);
  const float og = 1.f / (1.f + expf(-go));
  c = fg * c_prev + ig * g;
  h = og * tanhf(c);
}
// dh: dL/dh of this cell (recurrent + head), dc_in: dL/dc from the next step; dq[4]: dL/d(gate pre-activations),
// dc_out: dL/dc_prev
__device__ __forceinline__ void lstm_cell_bwd(float gi, float gf, float gg, float go, float c_prev, float c_new,
                                              float dc_in, float dh, float* dq, float& dc_out) {
  const float ig = 1.f / (1.f + expf(-gi));
  const float fg = 1.f / (1.f + expf(-gf));
  const float g = tanhf(gg);
  const float og = 1.f / (1.f + expf(-go));
  const float tc = tanhf(c_new);
  const float dc = dc_in + dh * og * (1.f - tc * tc);
  dq[0] = dc * g * ig * (1.f - ig);
  dq[1] = dc * c_prev * fg * (1.f - fg);
  dq[2] = dc * ig * (1.f - g * g);
  dq[3] = dh * tc * og * (1.f - og);
  dc_out = dc * fg;
}
