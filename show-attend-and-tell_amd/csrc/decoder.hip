// Decoder forward / backward orchestration (decoder.py:69-158 and the autograd
// BPTT the reference gets from loss.backward(), train.py:163).
//
// The time loop runs here, in C++, so one C-ABI call launches the whole
// sequence (no per-step Python round trips).  Work that does not depend on the
// recurrence is hoisted out of the loop and batched over all B*(T-1) rows:
//   * Ws = a W^T + b (attention.py:16) once per batch,
//   * the embedding half of the LSTM input GEMM under teacher forcing,
//   * the whole output head (dropout, f_h/f_z/f_out or deep_output) under
//     teacher forcing, and in backward every weight gradient (one GEMM per
//     weight with K = B*(T-1) instead of T-1 small accumulations).
// Per step the forward runs: [h GEMM: U, f_beta, W_hh fused as one N=E+D+4E
// product] -> fused attention + gate -> context GEMM -> LSTM pointwise (+ the
// per-step head and greedy argmax when teacher forcing is off).  The backward
// step mirrors it: LSTM pointwise -> context-grad GEMM -> attention backward ->
// one dh GEMM against the same fused [U; f_beta; W_hh] weight.
//
// Layout: every per-step tensor is batch-major [B, T-1, X]; step t is the
// strided slice at offset t*X with row stride (T-1)*X, so the batched head /
// weight-gradient GEMMs read the same buffers as plain [B*(T-1), X] matrices.
#include "sat_common.h"
#include "sat_internal.h"

namespace {

struct WS {
  // forward (saved for backward)
  float *mean_f, *hc0, *hc0pre, *xg, *gctx_const, *hg, *gctx, *uh_all, *gates_all, *c_in, *c_out, *h_out, *ctx_all,
      *gate_all, *fh, *fz;
  void *mean_t, *Ws, *emb_t, *h_in_t, *ctx_t, *gated_t, *hd_t, *comb_t;
  int32_t* tok;
  uint8_t* dmask;
  // backward
  void *dpre_t, *dfh_t, *dfz_t, *dhg_t, *dWs_t, *dpre0_t;
  float *dcomb, *dhd, *dctx_head, *dhg, *dgated, *dh_rec, *dc, *dWs_acc, *dv_acc, *dbv_acc, *part, *demb, *dpre0,
      *colsum, *de_all;
  unsigned* ticket;
  // deterministic split-K of the batched weight / input gradients (gemmsplit.hip): partial tiles, and
  // kTicketBlocks x kSatSplitTickets arrival tickets (each product of a backward phase has its own block, all zeroed
  // by the phase's one zeroing launch)
  float* gsplit;
  unsigned* gtickets;
  // the fused greedy step (greedy_fused): token table xt [V][4E] = emb W_ih[:, :E]^T + b_ih, the ado head's f_z
  // pre-activation slabs, the vocabulary head's per-block argmax partials
  float* xt;
  float* fzp;
  float* am_val;
  int32_t* am_idx;
  // the sorted (deterministic) dense embedding gradient
  void* emb_ws;
};
constexpr int kTicketBlocks = 16;   // phase 1: blocks 0-7, phase 2: 8-15

// split counts of the per-step skinny GEMMs (M = B rows).  bf16: the LDS-DMA kernel (128 x 64
// tiles, 128 x 128 for k-major weights) with partial-output split-K -- aim for ~0.75 waves of
// blocks over the 256 CUs with splits that divide K into whole 64-deep k-tiles (fewer, longer
// splits write and re-read fewer fp32 slabs: tools/bench_decoder_splits.py, B=128 bench shape
// -1.3 % decoder time against ~1.5 waves); fp32 (parity) mode keeps a single split.
struct Splits { int h, c, g, dh, i; };
// Workgroups the split-K of one per-step GEMM aims for: 192 when the decoder has the chip to
// itself; 64 when it shares it with the next batch's encoder (bench.py / train.py overlap): fewer,
// longer workgroups cost the concurrent conv trunk less (overlapped step 8.23 -> 8.07 ms; alone the
// decoder prefers 192: 10.24 vs 10.48 ms sequential).  SatDecoderDims::split_target, 0 = 192.
constexpr int kSplitTargetDefault = 192;

// A single split on a bf16 per-step product with K >= 1024 sends it to the tile kernel's atomic split-K, whose fp32
// atomics add in arrival order: run-to-run rounding differences in the recurrent chain (dh, d gates, dc), which the
// bf16 copies of the next products amplify into whole-ulp flips at small batch.  Where no whole-k-tile divisor of K
// fits, the product splits raggedly instead: S slabs of cdiv(kt, S) k-tiles, the last one shorter (the partial-output
// kernels write an empty k range as zeros), at most 8 slabs.
constexpr int kChainAtomicK = 1024;
inline int ragged_splits(int K, long want) {
  const int kt = sat_cdiv(K, 64);
  const int cap = want < 2 ? 2 : (want > 8 ? 8 : (int)want);
  const int kc = sat_cdiv(kt, cap);
  return sat_cdiv(kt, kc);
}
inline int pick_splits(int M, int N, int K, int dtype, bool kmajor_w, int target) {
  if (dtype != SAT_BF16) return 1;
  const long tiles = (long)sat_cdiv(M, 128) * sat_cdiv(N, kmajor_w ? 128 : 64);
  long want = (target + tiles - 1) / tiles;
  if (want > 32) want = 32;
  const int kt = K / 64;
  int best = 1;
  if (K % 64 == 0)
    for (int s = 1; s <= kt && s <= want; ++s)
      if (kt % s == 0) best = s;
  if (best == 1 && K >= kChainAtomicK) best = ragged_splits(K, want);
  return best;
}
// a policy override that divides K into whole k-tiles; 1 on a K >= 1024 product keeps the automatic count (see above)
inline int forced(int f, int K, int auto_s) {
  if (f == 1 && K >= kChainAtomicK) return auto_s;
  return (f > 0 && K % 64 == 0 && (K / 64) % f == 0) ? f : auto_s;
}
// tr: the backward's dL/d(gated context) and dL/dh products read the transposed weight copies
// (SatDecoderLayout::wih_ctx_t / hcat_t, k-contiguous) and run on the skinny kernel with its own K split
inline Splits splits_for(const SatDecoderDims& d, bool tr) {
  const int E = d.E, D = d.D, HG = 5 * E + D;
  const bool bf = d.dtype == SAT_BF16;
  const int tg = d.split_target > 0 ? d.split_target : kSplitTargetDefault;
  const int KH = d.attention ? HG : 4 * E;
  Splits s;
  s.h = pick_splits(d.B, KH, E, d.dtype, false, tg);
  s.c = pick_splits(d.B, 4 * E, D, d.dtype, false, tg);
  s.g = pick_splits(d.B, D, 4 * E, d.dtype, !tr, tg);
  s.dh = pick_splits(d.B, E, KH, d.dtype, !tr, tg);
  s.i = pick_splits(d.B, 2 * E, D, d.dtype, false, tg);
  if (bf) {   // per-step products the skinny kernel runs (csrc/skinny.hip): its own K split
    int k;
    if ((k = sat_skinny_splits(d.B, KH, E))) s.h = k;
    // the context GEMM in 512-deep splits (fewer slabs for the LSTM forward to sum: decoder fwd + bwd 3.05 ->
    // 3.00 ms at B = 128 against 256-deep, profiles/r3_s13/splits128.log)
    if ((k = sat_skinny_splits(d.B, 4 * E, D))) s.c = D % 512 == 0 ? k / 2 : k;
    if ((k = sat_skinny_splits(d.B, 2 * E, D))) s.i = k;
    // the backward's products through the transposed copies: 512-deep splits (fewer slabs for the attention /
    // LSTM backward kernels that sum them: B = 128 decoder fwd + bwd 3.15 -> 3.04 ms, B = 64 2.47 -> 2.36 ms
    // against 256-deep, profiles/r3_s11_decoder_splits.txt)
    if (tr && (k = sat_skinny_splits(d.B, D, 4 * E)) && (4 * E) % 512 == 0) s.g = k / 2;
    if (tr && (k = sat_skinny_splits(d.B, E, KH)) && KH % 512 == 0) s.dh = k / 2;
    // dL/dh has only E / 32 column blocks (16 at E = 512): 512-deep splits left 112 of 256 CUs idle at K = 4608
    // (ResNet152 features, 144 workgroups).  There the most 128-multiple-deep splits that keep the launch within one
    // workgroup per CU (and the LSTM backward's up-front slab loads, <= 16): 12 (192 workgroups), span 7.33 -> 6.40 us
    // at B = 128, 4.71 -> 4.04 at B = 64 (profiles/r6_s77, r6_s78).  At K = 3072 (VGG19, 6 -> 12 splits) it measured
    // slower (10.85 -> 10.97 us, the cfg5 chain +2.7 us), so only K >= 4096 takes it.
    if (tr && s.dh > 1 && KH % 128 == 0 && KH >= 4096) {
      const int cols = E / 32, kt = KH / 128;
      for (int c = 16; c > s.dh; --c)
        if (kt % c == 0 && c * cols <= 256 && KH / c <= 1024) { s.dh = c; break; }
    }
  }
  if (bf) {   // per-call overrides (SatPolicy::decoder_splits, 0 = automatic)
    const int* f = sat_policy().decoder_splits;
    s.h = forced(f[0], E, s.h);
    s.c = forced(f[1], D, s.c);
    s.g = forced(f[2], 4 * E, s.g);
    s.dh = forced(f[3], KH, s.dh);
  }
  return s;
}
// whether a call may use the transposed weight copies (bf16, both offsets given, the skinny kernel not excluded)
inline bool use_transposed(const SatDecoderDims& d, const SatDecoderLayout& lay) {
  return d.dtype == SAT_BF16 && lay.wih_ctx_t >= 0 && lay.hcat_t >= 0 && sat_policy().skinny != 1;
}
// the fused greedy step (SatPolicy::greedy_step): bf16, no teacher forcing, the head kernels' shapes
inline bool greedy_fused(const SatDecoderDims& d) {
  return d.dtype == SAT_BF16 && !d.tf && sat_policy().greedy_step != 1 && sat_greedy_supported(d.B, d.E);
}
// the dense embedding gradient as sorted per-token sums (SatPolicy::embed_grad)
inline bool embed_sorted(const SatDecoderDims& d) {
  return !d.bert && sat_policy().embed_grad != 1 && (long)d.B * (d.T - 1) <= sat_embed_sorted_max_rows() &&
         d.V < (1 << 18) && d.E % 4 == 0;
}

struct Carver {
  char* base;
  size_t off = 0;
  template <typename P>
  void take(P*& p, size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    p = base ? (P*)(base + off) : nullptr;
    off += bytes;
  }
};

// row stride of the workspace copy of d logits: bf16 vocabularies that are not a multiple of 8
// (BERT's 30522) are padded with zero columns so the two vocab GEMMs of the head backward stay on
// the 16-B LDS-DMA kernel (SatGemm::a_tail) instead of the register-staged fallback (~4 ms / step)
inline int head_ld(const SatDecoderDims& d) { return d.dtype == SAT_BF16 && d.V % 8 ? (d.V + 7) / 8 * 8 : d.V; }

size_t carve(const SatDecoderDims& d, char* base, WS* w) {
  const size_t B = d.B, L = d.L, D = d.D, E = d.E, V = d.V, T1 = d.T - 1, R = B * T1;
  const size_t HG = 5 * E + D;
  const size_t ts = d.dtype == SAT_BF16 ? 2 : 4, f = 4;
  Splits sp = splits_for(d, false);
  {   // split-K slabs sized for either form of the backward's products (the layout decides per call)
    const Splits st = splits_for(d, true);
    sp.g = sp.g > st.g ? sp.g : st.g;
    sp.dh = sp.dh > st.dh ? sp.dh : st.dh;
  }
  Carver c{base};
  c.take(w->mean_f, B * D * f);  c.take(w->mean_t, B * D * ts);
  c.take(w->hc0, B * 2 * E * f);
  c.take(w->hc0pre, sp.i * B * 2 * E * f);
  c.take(w->Ws, B * L * E * ts);
  c.take(w->tok, R * 4);
  c.take(w->emb_t, R * E * ts);
  c.take(w->xg, R * 4 * E * f);
  c.take(w->gctx_const, B * 4 * E * f);
  c.take(w->hg, sp.h * B * HG * f);
  c.take(w->gctx, sp.c * B * 4 * E * f);
  c.take(w->uh_all, R * E * f);
  c.take(w->gates_all, R * 4 * E * f);
  c.take(w->c_in, R * E * f);   c.take(w->c_out, R * E * f);
  c.take(w->h_in_t, R * E * ts); c.take(w->h_out, R * E * f);
  c.take(w->ctx_all, R * D * f); c.take(w->ctx_t, R * D * ts);
  c.take(w->gate_all, R * D * f); c.take(w->gated_t, R * D * ts);
  c.take(w->dmask, R * E);
  c.take(w->hd_t, R * E * ts);
  c.take(w->fh, R * E * f); c.take(w->fz, R * E * f); c.take(w->comb_t, R * E * ts);
  // backward
  c.take(w->dpre_t, R * head_ld(d) * ts);
  c.take(w->dcomb, R * E * f);
  c.take(w->dfh_t, R * E * ts); c.take(w->dfz_t, R * E * ts);
  c.take(w->dhd, R * E * f);
  c.take(w->dctx_head, R * D * f);
  c.take(w->dhg, R * HG * f); c.take(w->dhg_t, R * HG * ts);
  c.take(w->dgated, sp.g * B * D * f);
  c.take(w->dh_rec, sp.dh * B * E * f); c.take(w->dc, B * E * f);
  c.take(w->dWs_acc, B * L * E * f); c.take(w->dWs_t, B * L * E * ts);
  c.take(w->dv_acc, B * E * f); c.take(w->dbv_acc, B * f);
  c.take(w->de_all, R * L * f);
  c.take(w->part, sat_attention_part_floats(d.B, d.L, d.D, d.E, d.dtype, d.split_target) * f);
  c.take(w->ticket, B * 4);
  if (d.dtype == SAT_BF16) {
    c.take(w->gsplit, sat_split_gemm_ws_bytes() - kSatSplitTickets * 4);
    c.take(w->gtickets, (size_t)kTicketBlocks * kSatSplitTickets * 4);
  } else {
    w->gsplit = nullptr;
    w->gtickets = nullptr;
  }
  c.take(w->demb, R * E * f);
  c.take(w->dpre0, B * 2 * E * f); c.take(w->dpre0_t, B * 2 * E * ts);
  if (greedy_fused(d)) {
    c.take(w->xt, V * 4 * E * f);
    c.take(w->fzp, sp.c * B * E * f);
    c.take(w->am_val, (size_t)sat_greedy_head_blocks(d.B, d.V, d.E) * B * f);
    c.take(w->am_idx, (size_t)sat_greedy_head_blocks(d.B, d.V, d.E) * B * 4);
  } else {
    w->xt = w->fzp = w->am_val = nullptr;
    w->am_idx = nullptr;
  }
  if (embed_sorted(d)) c.take(w->emb_ws, sat_embed_sorted_ws_bytes((int)R, (int)E));
  else w->emb_ws = nullptr;
  // column-sum scratch: the largest single sum, or all the bias sums of one backward phase in one launch pair
  // (phase 1: f_out / f_h / f_z biases; phase 2: attention W / v, init, [U; f_beta; W_hh] and gate biases)
  size_t maxN = V > HG ? V : HG;
  if (D > maxN) maxN = D;
  const size_t ph1 = V + 2 * E, ph2 = 9 * E + D + 1;
  if (ph1 > maxN) maxN = ph1;
  if (ph2 > maxN) maxN = ph2;
  c.take(w->colsum, sat_colsum_scratch_floats((int)R, (int)maxN) * f);
  return c.off + 256;
}

__global__ void start_tokens_kernel(int32_t* tok, int B, int T1, int start) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) tok[(long)b * T1] = start;
}

template <typename T>
__global__ void ado_combine_rows_kernel(const float* fh, const float* fz, const T* emb, int rows, int E, long ld,
                                        T* comb) {
  const long n = (long)rows * E;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / E;
    const int e = (int)(i - r * E);
    const long o = r * ld + e;
    comb[o] = (T)(fh[o] + fz[o] + (float)emb[o]);
  }
}

int combine_rows(const float* fh, const float* fz, const void* emb, int rows, int E, long ld, int dtype, void* comb,
                 hipStream_t s) {
  long n = (long)rows * E;
  int g = (int)((n + 255) / 256);
  if (g > 4096) g = 4096;
  if (dtype == SAT_BF16)
    hipLaunchKernelGGL(ado_combine_rows_kernel<bf16>, dim3(g), dim3(256), 0, s, fh, fz, (const bf16*)emb, rows, E, ld, (bf16*)comb);
  else
    hipLaunchKernelGGL(ado_combine_rows_kernel<float>, dim3(g), dim3(256), 0, s, fh, fz, (const float*)emb, rows, E, ld, (float*)comb);
  return (int)hipGetLastError();
}

// tanh of the [init_h | init_c] pre-activations (sum of `splits` slabs): hc0 (fp32, kept for the
// backward), h into step 0's GEMM-input slot (dtype), c into step 0's cell slot (fp32).
template <typename T>
__global__ void init_state_kernel(const float* pre, int splits, long stride, int B, int E, float* hc0, T* h_t,
                                  long h_ld, float* c_in, long c_ld) {
  const long n = (long)B * 2 * E;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / (2 * E)), j = (int)(i - (long)b * 2 * E);
    const float v = tanhf(sum_parts(pre, i, splits, stride));
    hc0[i] = v;
    if (j < E) h_t[(long)b * h_ld + j] = (T)v;
    else c_in[(long)b * c_ld + j - E] = v;
  }
}

struct Ctx {
  SatDecoderDims d;
  SatDecoderLayout lay;
  const float* P;
  const void* LP;
  int ts;
  long T1, R, HG;
  bool tr;   // use_transposed(d, lay)
  const void* W(int64_t off) const {
    return d.dtype == SAT_BF16 ? (const void*)((const bf16*)LP + off) : (const void*)(P + off);
  }
  const float* F(int64_t off) const { return P + off; }
  void* at(void* p, long elems) const { return (char*)p + elems * ts; }
  const void* at(const void* p, long elems) const { return (const char*)p + elems * ts; }
};

// y[rows, N] (+)= x[rows, K] . W[N, K]^T  (+bias) (act) -- all strided rows
int linear(const Ctx& c, int rows, int N, int K, const void* x, long ldx, const void* w, long ldw, const float* bias,
           void* y, long ldy, int y_dtype, int act, hipStream_t s, const void* add1 = nullptr, long ld_add1 = 0,
           int add1_dtype = SAT_F32, void* aux = nullptr, long ld_aux = 0, int aux_dtype = SAT_F32,
           int splits = 0, long split_stride = 0) {
  SatGemm g;
  g.partial_splits = splits; g.split_stride = split_stride;
  g.M = rows; g.N = N; g.K = K; g.dtype = c.d.dtype;
  g.A = x; g.lda = ldx; g.B = w; g.ldb = ldw;
  g.C = y; g.ldc = ldy; g.c_dtype = y_dtype; g.bias = bias; g.act = act;
  g.add1 = add1; g.ld_add1 = ld_add1; g.add1_dtype = add1_dtype;
  g.aux = aux; g.ld_aux = ld_aux; g.aux_dtype = aux_dtype;
  return sat_gemm_launch(g, s);
}

// Output head over `rows` rows starting at step t0 (batched: rows = R, t0 = 0, ld factor 1;
// per step: rows = B, row stride T1).  decoder.py:117-125,149-158
int head_forward(const Ctx& c, const WS& w, int rows, int t, bool per_step, void* preds, const uint8_t* mask_in,
                 hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int E = d.E, D = d.D, V = d.V;
  const long rs = per_step ? c.T1 : 1;  // row stride multiplier
  const long oE = per_step ? (long)t * E : 0, oD = per_step ? (long)t * D : 0, oV = per_step ? (long)t * V : 0;
  // dropout(h)
  if (per_step)
    SAT_CHECK((hipError_t)sat_dropout_apply(w.h_out + oE, c.T1 * E, d.B, 1, E, d.training, d.has_dropout_mask,
                                            mask_in ? mask_in + oE : nullptr, w.dmask + oE, c.T1 * E, d.seed,
                                            d.seed_ptr, t,
                                            c.at(w.hd_t, oE), c.T1 * E, d.dtype, s));
  else
    SAT_CHECK((hipError_t)sat_dropout_apply(w.h_out, E, d.B, (int)c.T1, E, d.training, d.has_dropout_mask, mask_in,
                                            w.dmask, E, d.seed, d.seed_ptr, 0, w.hd_t, E, d.dtype, s));
  if (d.ado) {
    SAT_CHECK((hipError_t)linear(c, rows, E, E, c.at(w.hd_t, oE), rs * E, c.W(c.lay.fh_w), E, c.F(c.lay.fh_b),
                                 w.fh + oE, rs * E, SAT_F32, SAT_ACT_RELU, s));
    SAT_CHECK((hipError_t)linear(c, rows, E, D, c.at(w.ctx_t, oD), rs * D, c.W(c.lay.fz_w), D, c.F(c.lay.fz_b),
                                 w.fz + oE, rs * E, SAT_F32, SAT_ACT_RELU, s));
    SAT_CHECK((hipError_t)combine_rows(w.fh + oE, w.fz + oE, c.at(w.emb_t, oE), rows, E, rs * E, d.dtype,
                                       c.at(w.comb_t, oE), s));
    SAT_CHECK((hipError_t)linear(c, rows, V, E, c.at(w.comb_t, oE), rs * E, c.W(c.lay.fout_w), E,
                                 c.F(c.lay.fout_b), c.at(preds, oV), rs * V, d.dtype, SAT_ACT_RELU, s));
  } else {
    SAT_CHECK((hipError_t)linear(c, rows, V, E, c.at(w.hd_t, oE), rs * E, c.W(c.lay.do_w), E, c.F(c.lay.do_b),
                                 c.at(preds, oV), rs * V, d.dtype, SAT_ACT_NONE, s));
  }
  return 0;
}

// ---- per-step kernels (shared by the time loops and sat_decoder_step_bench) ----
struct StepIO {
  const void* feats;          // img_features [B,L,D] (dtype)
  float* alphas;              // [B,T-1,L]
  const float* d_alphas;      // [B,T-1,L] (backward)
};

// h GEMM: [U h + b_U | f_beta h + b | W_hh h + b_hh] (one N = E+D+4E product; W_hh only without attention)
int fwd_hgemm(const Ctx& c, const WS& w, const Splits& sp, int t, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, D = d.D, E = d.E;
  const long T1 = c.T1, HG = c.HG;
  const void* h_t = c.at(w.h_in_t, (long)t * E);
  if (d.attention)
    return linear(c, B, (int)HG, E, h_t, T1 * E, c.W(c.lay.hcat_w), E, c.F(c.lay.hcat_b), w.hg, HG, SAT_F32,
                  SAT_ACT_NONE, s, nullptr, 0, SAT_F32, nullptr, 0, SAT_F32, sp.h, (long)B * HG);
  return linear(c, B, 4 * E, E, h_t, T1 * E, c.W(c.lay.hcat_w + (long)(E + D) * E), E, c.F(c.lay.hcat_b + E + D),
                w.hg + E + D, HG, SAT_F32, SAT_ACT_NONE, s, nullptr, 0, SAT_F32, nullptr, 0, SAT_F32, sp.h,
                (long)B * HG);
}

int fwd_attn(const Ctx& c, const WS& w, const Splits& sp, const StepIO& io, int t, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, L = d.L, D = d.D, E = d.E;
  const long T1 = c.T1, HG = c.HG;
  AttnFwdArgs a{};
  a.B = B; a.L = L; a.D = D; a.E = E; a.dtype = d.dtype;
  a.Ws = w.Ws; a.uh = w.hg; a.uh_ld = HG; a.v_w = c.F(c.lay.v_w); a.v_b = c.F(c.lay.v_b); a.a = io.feats;
  a.gate_pre = w.hg + E; a.gate_ld = HG;
  a.hg_splits = sp.h; a.hg_split_stride = (long)B * HG;
  a.alpha = io.alphas + (long)t * L; a.alpha_ld = T1 * L;
  a.ctx = w.ctx_all + (long)t * D; a.ctx_ld = T1 * D;
  a.ctx_t = c.at(w.ctx_t, (long)t * D); a.ctx_t_ld = T1 * D;
  a.gate = w.gate_all + (long)t * D; a.gate_out_ld = T1 * D;
  a.gated = c.at(w.gated_t, (long)t * D); a.gated_ld = T1 * D;
  a.uh_save = w.uh_all + (long)t * E; a.uh_save_ld = T1 * E;
  return sat_attention_fwd_launch(a, s);
}

// context half of the LSTM input GEMM: gated context . W_ih[:, E:]^T
int fwd_cgemm(const Ctx& c, const WS& w, const Splits& sp, int t, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, D = d.D, E = d.E;
  return linear(c, B, 4 * E, D, c.at(w.gated_t, (long)t * D), c.T1 * D, c.W(c.lay.wih + E), E + D, nullptr, w.gctx,
                4 * E, SAT_F32, SAT_ACT_NONE, s, nullptr, 0, SAT_F32, nullptr, 0, SAT_F32, sp.c, (long)B * 4 * E);
}

LstmFwdArgs lstm_fwd_args(const Ctx& c, const WS& w, const Splits& sp, int t) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, D = d.D, E = d.E;
  const long T1 = c.T1, HG = c.HG;
  const bool att = d.attention != 0;
  LstmFwdArgs l{};
  l.B = B; l.E = E; l.dtype = d.dtype;
  l.hpart = w.hg + E + D; l.hpart_ld = HG;
  l.xpart = w.xg + (long)t * 4 * E; l.xpart_ld = T1 * 4 * E;
  l.cpart = att ? w.gctx : w.gctx_const; l.cpart_ld = 4 * E;
  l.h_splits = sp.h; l.h_split_stride = (long)B * HG;
  l.c_splits = att ? sp.c : 1; l.c_split_stride = (long)B * 4 * E;
  l.c_prev = w.c_in + (long)t * E; l.c_prev_ld = T1 * E;
  l.gates = w.gates_all + (long)t * 4 * E; l.gates_ld = T1 * 4 * E;
  l.c_out = w.c_out + (long)t * E; l.c_out_ld = T1 * E;
  l.c_next_in = t + 1 < T1 ? w.c_in + (long)(t + 1) * E : nullptr; l.c_next_in_ld = T1 * E;
  l.h_out = w.h_out + (long)t * E; l.h_out_ld = T1 * E;
  l.h_next_in_t = t + 1 < T1 ? c.at(w.h_in_t, (long)(t + 1) * E) : nullptr; l.h_next_in_t_ld = T1 * E;
  return l;
}

int fwd_lstm(const Ctx& c, const WS& w, const Splits& sp, int t, hipStream_t s) {
  return sat_lstm_fwd_launch(lstm_fwd_args(c, w, sp, t), s);
}

LstmBwdArgs lstm_bwd_args(const Ctx& c, const WS& w, const Splits& sp, int t) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, D = d.D, E = d.E;
  const long T1 = c.T1, HG = c.HG;
  LstmBwdArgs l{};
  l.B = B; l.E = E; l.dtype = d.dtype;
  l.gates = w.gates_all + (long)t * 4 * E; l.gates_ld = T1 * 4 * E;
  l.c_prev = w.c_in + (long)t * E; l.c_prev_ld = T1 * E;
  l.c_new = w.c_out + (long)t * E; l.c_new_ld = T1 * E;
  l.dh_rec = t == T1 - 1 ? nullptr : w.dh_rec; l.dh_rec_ld = E;
  l.dh_splits = sp.dh; l.dh_split_stride = (long)B * E;
  l.dh_head = w.dhd + (long)t * E; l.dh_head_ld = T1 * E;
  l.mask = d.training ? w.dmask + (long)t * E : nullptr; l.mask_ld = T1 * E;
  l.dc = w.dc; l.dc_zero = t == T1 - 1;
  l.d_gates = w.dhg + (long)t * HG + E + D; l.d_gates_ld = T1 * HG;
  l.d_gates_t = c.at(w.dhg_t, (long)t * HG + E + D); l.d_gates_t_ld = T1 * HG;
  return l;
}

int bwd_lstm(const Ctx& c, const WS& w, const Splits& sp, int t, hipStream_t s) {
  return sat_lstm_bwd_launch(lstm_bwd_args(c, w, sp, t), s);
}

// the workspace a batched backward product may split K over (gemmsplit.hip): ticket block `blk`
struct SplitWS {
  float* slab;
  unsigned* tickets;
  int blk;
};
inline void use_split(SatGemm& g, const SplitWS* sw) {
  if (!sw || !sw->slab) return;
  g.split_ws = sw->slab;
  g.split_ws_bytes = (long)(sat_split_gemm_ws_bytes() - kSatSplitTickets * 4);
  g.split_tickets = sw->tickets + (long)sw->blk * kSatSplitTickets;
  g.tickets_zeroed = 1;
}

// input gradient: Y[M,N] = X[M,K] W[K,N]   (W stored [K][N] row-major = torch weight [out,in])
int dgrad_launch(const Ctx& c, int M, int N, int K, const void* X, long ldx, const void* Wt, long ldw, float* out,
                 long ldo, hipStream_t s, const float* add1 = nullptr, long ld_add1 = 0, int splits = 0,
                 long split_stride = 0, int a_tail = 0, const SplitWS* sw = nullptr) {
  SatGemm g;
  use_split(g, sw);
  g.a_tail = a_tail;
  g.partial_splits = splits; g.split_stride = split_stride;
  g.M = M; g.N = N; g.K = K; g.dtype = c.d.dtype;
  g.A = X; g.lda = ldx; g.B = Wt; g.ldb = ldw; g.transB = 1;
  g.C = out; g.ldc = ldo; g.c_dtype = SAT_F32;
  g.add1 = add1; g.ld_add1 = ld_add1; g.add1_dtype = SAT_F32;
  return sat_gemm_launch(g, s);
}

// dL/d(gated context) = d gates . W_ih[:, E:]
int bwd_ggemm(const Ctx& c, const WS& w, const Splits& sp, int t, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, D = d.D, E = d.E;
  if (c.tr)   // d gates . (W_ih[:, E:]^T)^T with the transposed copy [D][4E]: k-contiguous, the skinny kernel
    return linear(c, B, D, 4 * E, c.at(w.dhg_t, (long)t * c.HG + E + D), c.T1 * c.HG, c.W(c.lay.wih_ctx_t), 4 * E,
                  nullptr, w.dgated, D, SAT_F32, SAT_ACT_NONE, s, nullptr, 0, SAT_F32, nullptr, 0, SAT_F32, sp.g,
                  (long)B * D);
  return dgrad_launch(c, B, D, 4 * E, c.at(w.dhg_t, (long)t * c.HG + E + D), c.T1 * c.HG, c.W(c.lay.wih + E), E + D,
                      w.dgated, D, s, nullptr, 0, sp.g, (long)B * D);
}

int bwd_attn(const Ctx& c, const WS& w, const Splits& sp, const StepIO& io, int t, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, L = d.L, D = d.D, E = d.E;
  const long T1 = c.T1, HG = c.HG;
  AttnBwdArgs a{};
  a.B = B; a.L = L; a.D = D; a.E = E; a.dtype = d.dtype;
  a.Ws = w.Ws; a.a = io.feats;
  a.uh = w.uh_all + (long)t * E; a.uh_ld = T1 * E;
  a.v_w = c.F(c.lay.v_w);
  a.alpha = io.alphas + (long)t * L; a.alpha_ld = T1 * L;
  a.d_alpha_ext = io.d_alphas + (long)t * L; a.d_alpha_ext_ld = T1 * L;
  a.d_gated = w.dgated; a.d_gated_ld = D;
  a.gate = w.gate_all + (long)t * D; a.gate_ld = T1 * D;
  a.ctx = w.ctx_all + (long)t * D; a.ctx_ld = T1 * D;
  a.d_ctx_ext = d.ado ? w.dctx_head + (long)t * D : nullptr; a.d_ctx_ext_ld = T1 * D;
  a.d_uh = w.dhg + (long)t * HG; a.d_uh_ld = T1 * HG; a.d_uh_t = c.at(w.dhg_t, (long)t * HG);
  a.d_gpre = w.dhg + (long)t * HG + E; a.d_gpre_ld = T1 * HG; a.d_gpre_t = c.at(w.dhg_t, (long)t * HG + E);
  a.de_out = w.de_all + (long)t * L; a.de_ld = T1 * L; a.dv_acc = w.dv_acc; a.dbv_acc = w.dbv_acc; a.part = w.part;
  a.ticket = w.ticket;
  a.dg_splits = sp.g; a.dg_split_stride = (long)B * D;
  a.wg_target = d.split_target;   // beside the encoder: fewer workgroups (sat_attention_bwd_chunks)
  return sat_attention_bwd_launch(a, s);
}

// recurrent dL/dh = [dU_h | d(f_beta h) | d gates] . [U ; f_beta ; W_hh]   (W_hh only without attention)
int bwd_dhgemm(const Ctx& c, const WS& w, const Splits& sp, int t, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int B = d.B, D = d.D, E = d.E;
  const long T1 = c.T1, HG = c.HG;
  if (c.tr) {   // against the transposed copy hcat^T [E][HG] (k-contiguous: the skinny kernel)
    const long k0 = d.attention ? 0 : E + D;
    return linear(c, B, E, (int)(HG - k0), c.at(w.dhg_t, (long)t * HG + k0), T1 * HG, c.W(c.lay.hcat_t + k0), HG,
                  nullptr, w.dh_rec, E, SAT_F32, SAT_ACT_NONE, s, nullptr, 0, SAT_F32, nullptr, 0, SAT_F32, sp.dh,
                  (long)B * E);
  }
  if (d.attention)
    return dgrad_launch(c, B, E, (int)HG, c.at(w.dhg_t, (long)t * HG), T1 * HG, c.W(c.lay.hcat_w), E, w.dh_rec, E, s,
                        nullptr, 0, sp.dh, (long)B * E);
  return dgrad_launch(c, B, E, 4 * E, c.at(w.dhg_t, (long)t * HG + E + D), T1 * HG,
                      c.W(c.lay.hcat_w + (long)(E + D) * E), E, w.dh_rec, E, s, nullptr, 0, sp.dh, (long)B * E);
}

// In-kernel timestamps of the per-step kernels (SatPolicy::stamps, bench.py's in-step figures): the
// policy's buffer holds kStampGroups x (T-1) slots (a 16-B header + stamp_capacity records), group g (the
// sat_decoder_step_bench order: h GEMM, attention fwd, context GEMM, LSTM fwd, LSTM bwd, d(gated
// context) GEMM, attention bwd, dh GEMM) at step t in slot g * (T-1) + t; every other launch of the
// decoder records nothing.
constexpr int kStampGroups = 8;
inline uint64_t* step_slot(const SatDecoderDims& d, int g, int t) {
  const SatPolicy* p = d.policy;
  if (!p || !p->stamps || p->stamp_capacity <= 0) return nullptr;
  return p->stamps + ((long)g * (d.T - 1) + t) * 2L * (p->stamp_capacity + 1);   // slot: header + records
}
inline int stamp_cap(const SatDecoderDims& d) { return d.policy ? d.policy->stamp_capacity : 0; }

// One per-step kernel group's in-kernel timestamp slot (SatPolicy::stamps) for the launches in its scope.
struct StepTimer {
  SatStampScope stamps;
  StepTimer(const SatDecoderDims& d, int g, int t) : stamps(step_slot(d, g, t), stamp_cap(d)) {}
};

// The fused greedy step (bf16, no teacher forcing; decoder.py:96-133 with tf off).  Per time step:
//   h GEMM -> attention -> context GEMM (+ the ado head's f_z slabs in the same launch) -> LSTM cell (+ dropout of h)
//   -> [ado: f_h + ReLUs + combine, one launch] -> vocabulary head (+ per-block argmax partials)
// and the argmax itself folded into the next step's LSTM kernel (which reads the fed token's row of the token table and
// writes its embedding row), against the per-op form's per-step embedding-half GEMM, dropout, f_z / f_h GEMMs, combine, vocabulary GEMM and
// full-row argmax.  The embedding half of the gate GEMM depends only on the fed token, so it is one GEMM over the
// vocabulary per forward (xt = emb W_ih[:, :E]^T + b_ih, once per weight version) and a row gather per step.
int greedy_loop(const Ctx& c, const WS& w, const Splits& sp, const StepIO& io, void* preds, const uint8_t* mask_in,
                int32_t* tokens, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const SatDecoderLayout& lay = c.lay;
  const int B = d.B, D = d.D, E = d.E, V = d.V, T1 = d.T - 1;
  const bool att = d.attention != 0;
  SAT_CHECK((hipError_t)linear(c, V, 4 * E, E, c.W(lay.embedding), E, c.W(lay.wih), E + D, c.F(lay.bih), w.xt, 4 * E,
                               SAT_F32, SAT_ACT_NONE, s));
  // step 0's gate input: the start token's table row (the start rows' embeddings are already gathered)
  SAT_CHECK((hipError_t)sat_embed_gather(w.xt, w.tok, B, 1, T1, 4 * E, SAT_F32, w.xg, (long)T1 * 4 * E, s));
  for (int t = 0; t < T1; ++t) {
    const long oE = (long)t * E, oD = (long)t * D;
    {
      StepTimer st(d, 0, t);
      SAT_CHECK((hipError_t)fwd_hgemm(c, w, sp, t, s));
    }
    if (att) {
      {
        StepTimer st(d, 1, t);
        SAT_CHECK((hipError_t)fwd_attn(c, w, sp, io, t, s));
      }
      StepTimer st(d, 2, t);
      SatGemm g1;
      g1.partial_splits = sp.c; g1.split_stride = (long)B * 4 * E;
      g1.M = B; g1.N = 4 * E; g1.K = D; g1.dtype = d.dtype;
      g1.A = c.at(w.gated_t, oD); g1.lda = c.T1 * D; g1.B = c.W(lay.wih + E); g1.ldb = E + D;
      g1.C = w.gctx; g1.ldc = 4 * E; g1.c_dtype = SAT_F32;
      SatGemm g2 = g1;   // f_z(context) pre-activation (ungated context, decoder.py:155), same K split
      g2.N = E; g2.A = c.at(w.ctx_t, oD); g2.B = c.W(lay.fz_w); g2.ldb = D;
      g2.C = w.fzp; g2.ldc = E; g2.split_stride = (long)B * E;
      int err = 0;
      if (!(d.ado && sat_skinny_dual_try(g1, g2, s, &err))) {
        SAT_CHECK((hipError_t)sat_gemm_launch(g1, s));
        if (d.ado) SAT_CHECK((hipError_t)sat_gemm_launch(g2, s));
      }
      SAT_CHECK((hipError_t)err);
    } else if (d.ado) {   // uniform attention: f_z of the (constant) mean context, one slab
      SAT_CHECK((hipError_t)linear(c, B, E, D, c.at(w.ctx_t, oD), c.T1 * D, c.W(lay.fz_w), D, nullptr, w.fzp, E,
                                   SAT_F32, SAT_ACT_NONE, s));
    }
    {
      StepTimer st(d, 3, t);
      LstmFwdArgs l = lstm_fwd_args(c, w, sp, t);
      l.hd_t = c.at(w.hd_t, oE); l.hd_ld = c.T1 * E;
      l.drop_training = d.training; l.drop_has_mask = d.has_dropout_mask; l.drop_t = t;
      l.mask_in = mask_in ? mask_in + oE : nullptr; l.mask_out = w.dmask + oE; l.mask_ld = c.T1 * E;
      l.seed = d.seed; l.seed_ptr = d.seed_ptr;
      if (t > 0) {   // the token fed at t: the argmax of step t - 1's head partials, folded into this launch
        l.am_val = w.am_val; l.am_idx = w.am_idx; l.am_ncb = sat_greedy_head_blocks(B, V, E); l.am_V = V;
        l.xt = w.xt; l.emb = c.F(lay.embedding); l.emb_t = c.at(w.emb_t, oE); l.emb_t_ld = c.T1 * E;
        l.tok_out = w.tok + t; l.tok_ld = T1;
      }
      SAT_CHECK((hipError_t)sat_lstm_fwd_launch(l, s));
    }
    HeadOutArgs ho{};
    ho.B = B; ho.V = V; ho.E = E;
    if (d.ado) {
      HeadMidArgs hm{};
      hm.B = B; hm.E = E;
      hm.hd = (const bf16*)c.at(w.hd_t, oE); hm.hd_ld = c.T1 * E;
      hm.fh_w = (const bf16*)c.W(lay.fh_w); hm.fh_b = c.F(lay.fh_b);
      hm.fzp = w.fzp; hm.fzp_ld = E; hm.fz_splits = att ? sp.c : 1; hm.fz_split_stride = (long)B * E;
      hm.fz_b = c.F(lay.fz_b);
      hm.emb = (const bf16*)c.at(w.emb_t, oE); hm.emb_ld = c.T1 * E;
      hm.fh = w.fh + oE; hm.fz = w.fz + oE; hm.f_ld = c.T1 * E;
      hm.comb = (bf16*)c.at(w.comb_t, oE); hm.comb_ld = c.T1 * E;
      SAT_CHECK((hipError_t)sat_greedy_head_mid(hm, s));
      ho.relu = 1;
      ho.x = hm.comb; ho.x_ld = hm.comb_ld;
      ho.w = (const bf16*)c.W(lay.fout_w); ho.bias = c.F(lay.fout_b);
    } else {
      ho.relu = 0;
      ho.x = (const bf16*)c.at(w.hd_t, oE); ho.x_ld = c.T1 * E;
      ho.w = (const bf16*)c.W(lay.do_w); ho.bias = c.F(lay.do_b);
    }
    ho.preds = (bf16*)c.at(preds, (long)t * V); ho.preds_ld = c.T1 * V;
    ho.pval = w.am_val; ho.pidx = w.am_idx;
    SAT_CHECK((hipError_t)sat_greedy_head_out(ho, s));
  }
  if (d.training && d.seed_ptr) SAT_CHECK((hipError_t)sat_bump_seed(d.seed_ptr, s));
  if (tokens) SAT_CHECK(hipMemcpyAsync(tokens, w.tok, c.R * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  return 0;
}

int check_dims(const SatDecoderDims* d) {
  if (!d) return SAT_ERR_INVALID;
  if (d->B <= 0 || d->L <= 0 || d->D <= 0 || d->E <= 0 || d->V <= 0 || d->T < 3) return SAT_ERR_INVALID;
  if (d->dtype != SAT_F32 && d->dtype != SAT_BF16) return SAT_ERR_INVALID;
  if (d->E % 8 != 0 || d->D % 8 != 0 || d->E > 1024 || d->L > 1024) return SAT_ERR_INVALID;
  if (d->split_target < 0 || d->split_target > 4096) return SAT_ERR_INVALID;
  if (d->policy) {
    for (int i = 0; i < 4; ++i)
      if (d->policy->decoder_splits[i] < 0 || d->policy->decoder_splits[i] > 64) return SAT_ERR_INVALID;
  }
  return 0;
}

}  // namespace

namespace {
// dst[c * ld_dst + r] = src[r * ld_src + c] for a rows x cols bf16 block (rows, cols, ld_src, ld_dst multiples of 8,
// 16-B aligned rows): 64 x 64 tiles through LDS (16-B loads along the source rows, 16-B stores along the
// destination rows)
// two blocks per launch (the refresh's W_ih context columns and [U; f_beta; W_hh]): workgroup i < nx0 * ny0 takes
// tile (i % nx0, i / nx0) of block 0, the rest tiles of block 1
struct TransposePair {
  const bf16* src[2]; long ld_src[2]; int rows[2], cols[2]; bf16* dst[2]; long ld_dst[2]; int nx[2], ntiles0;
};
__global__ __launch_bounds__(256) void transpose_bf16_kernel(TransposePair a) {
  const int k = (int)blockIdx.x < a.ntiles0 ? 0 : 1;
  const int i = (int)blockIdx.x - (k ? a.ntiles0 : 0);
  const bf16* __restrict__ src = a.src[k];
  bf16* __restrict__ dst = a.dst[k];
  const long ld_src = a.ld_src[k], ld_dst = a.ld_dst[k];
  const int rows = a.rows[k], cols = a.cols[k];
  __shared__ bf16 tile[64][64 + 8];
  const int r0 = (i / a.nx[k]) * 64, c0 = (i % a.nx[k]) * 64;
  const int tr = threadIdx.x >> 3, tc = (threadIdx.x & 7) * 8;   // 32 rows x 8 chunks of 8 per pass
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = r0 + tr + 32 * p;
    if (r < rows && c0 + tc < cols) {
      const uint4 v = *(const uint4*)(src + (long)r * ld_src + c0 + tc);
      const bf16* e = (const bf16*)&v;
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[tr + 32 * p][tc + j] = e[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = c0 + tr + 32 * p;   // destination row = source column
    if (c < cols && r0 + tc < rows) {
      uint4 v;
      bf16* e = (bf16*)&v;
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = tile[tc + j][tr + 32 * p];
      *(uint4*)(dst + (long)c * ld_dst + r0 + tc) = v;
    }
  }
}
}  // namespace

extern "C" int sat_decoder_refresh_transposed(const SatDecoderDims* d, const SatDecoderLayout* lay, void* params_lp,
                                              void* stream) {
  SAT_CHECK((hipError_t)check_dims(d));
  SAT_REQUIRE(lay && params_lp);
  if (d->dtype != SAT_BF16 || lay->wih_ctx_t < 0 || lay->hcat_t < 0) return 0;
  const int E = d->E, D = d->D, HG = 5 * E + D;
  SAT_REQUIRE(lay->wih_ctx_t % 8 == 0 && lay->hcat_t % 8 == 0 && lay->wih % 8 == 0 && lay->hcat_w % 8 == 0);
  bf16* lp = (bf16*)params_lp;
  hipStream_t s = (hipStream_t)stream;
  // one launch: W_ih [4E][E + D]'s context columns E.. as [D][4E], and hcat [HG][E] as [E][HG]
  TransposePair a{};
  a.src[0] = lp + lay->wih + E; a.ld_src[0] = E + D; a.rows[0] = 4 * E; a.cols[0] = D;
  a.dst[0] = lp + lay->wih_ctx_t; a.ld_dst[0] = 4L * E;
  a.src[1] = lp + lay->hcat_w; a.ld_src[1] = E; a.rows[1] = (int)HG; a.cols[1] = E;
  a.dst[1] = lp + lay->hcat_t; a.ld_dst[1] = HG;
  for (int k = 0; k < 2; ++k) a.nx[k] = sat_cdiv(a.cols[k], 64);
  a.ntiles0 = a.nx[0] * sat_cdiv(a.rows[0], 64);
  const int ntiles = a.ntiles0 + a.nx[1] * sat_cdiv(a.rows[1], 64);
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(ntiles), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" size_t sat_decoder_workspace_bytes(const SatDecoderDims* d) {
  if (check_dims(d)) return 0;
  SatPolicyScope scope(d->policy);
  WS w;
  return carve(*d, nullptr, &w);
}

extern "C" int sat_decoder_instance(const SatDecoderDims* dp, const SatDecoderLayout* lay, int* out, int n) {
  SAT_CHECK((hipError_t)check_dims(dp));
  SAT_REQUIRE(out && n > 0);
  SatPolicyScope scope(dp->policy);
  const SatDecoderDims& d = *dp;
  const bool tr = lay && use_transposed(d, *lay);
  const Splits sp = splits_for(d, tr);
  const int VD = d.dtype == SAT_BF16 ? 8 : 4;
  const bool split_bwd = d.attention && sat_policy().attn_bwd != 1 && d.E % 4 == 0 && sat_cdiv(d.D, 64 * VD) <= 8 &&
                         sat_cdiv(d.E, 64 * VD) <= (d.dtype == SAT_BF16 ? 2 : 4);
  const int v[SAT_DECODER_INSTANCE_FIELDS] = {
      sp.h, sp.c, sp.g, sp.dh, split_bwd ? sat_attention_bwd_chunks(d.B, d.L, d.split_target) : 0, tr ? 1 : 0,
      d.attention ? 4 : 2, d.attention ? 4 : 2};
  for (int i = 0; i < n && i < SAT_DECODER_INSTANCE_FIELDS; ++i) out[i] = v[i];
  return 0;
}

extern "C" int sat_decoder_forward(const SatDecoderDims* dp, const SatDecoderLayout* lay, const float* params,
                                   const void* params_lp, const void* img_features, const int64_t* captions,
                                   const uint8_t* dropout_mask, void* workspace, size_t workspace_bytes, void* preds,
                                   float* alphas, int32_t* tokens, void* stream) {
  SAT_CHECK((hipError_t)check_dims(dp));
  SAT_REQUIRE(lay && params && img_features && captions && workspace && preds && alphas);
  SAT_REQUIRE(dp->dtype == SAT_F32 || params_lp);
  SAT_REQUIRE(!(dp->training && dp->has_dropout_mask) || dropout_mask);
  SatPolicyScope scope(dp->policy);
  SatStampScope no_stamps(nullptr, 0);   // only the per-step groups below record timestamps
  const SatDecoderDims& d = *dp;
  WS w;
  SAT_REQUIRE(carve(d, nullptr, &w) <= workspace_bytes);
  carve(d, (char*)workspace, &w);
  hipStream_t s = (hipStream_t)stream;
  Ctx c{d, *lay, params, params_lp, d.dtype == SAT_BF16 ? 2 : 4, d.T - 1, (long)d.B * (d.T - 1), 5L * d.E + d.D,
        use_transposed(d, *lay)};
  const int B = d.B, L = d.L, D = d.D, E = d.E, T1 = d.T - 1;
  const long HG = c.HG;
  const bool att = d.attention != 0;
  const Splits sp = splits_for(d, c.tr);
  const StepIO io{img_features, alphas, nullptr};

  // fed tokens + embeddings
  if (d.tf) {
    SAT_CHECK((hipError_t)sat_embed_gather_captions(c.F(lay->embedding), captions, B, d.T, E, d.dtype, w.emb_t, E,
                                                    w.tok, s));
  } else {
    hipLaunchKernelGGL(start_tokens_kernel, dim3(sat_cdiv(B, 256)), dim3(256), 0, s, w.tok, B, T1, d.start_token);
    SAT_LAUNCH_CHECK();
    SAT_CHECK((hipError_t)sat_embed_gather(c.F(lay->embedding), w.tok, B, 1, T1, E, d.dtype, w.emb_t, (long)T1 * E, s));
  }
  // init_lstm_state (decoder.py:137-147)
  SAT_CHECK((hipError_t)sat_mean_rows(img_features, B, L, D, d.dtype, w.mean_f, w.mean_t, s));
  // [init_h; init_c] as one N = 2E product (split-K slabs), tanh + scatter in one pass
  SAT_CHECK((hipError_t)linear(c, B, 2 * E, D, w.mean_t, D, c.W(lay->init_w), D, c.F(lay->init_b), w.hc0pre, 2 * E,
                               SAT_F32, SAT_ACT_NONE, s, nullptr, 0, SAT_F32, nullptr, 0, SAT_F32, sp.i,
                               (long)B * 2 * E));
  {
    const long n = (long)B * 2 * E;
    const int g = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
    if (d.dtype == SAT_BF16)
      hipLaunchKernelGGL(init_state_kernel<bf16>, dim3(g), dim3(256), 0, s, (const float*)w.hc0pre, sp.i,
                         (long)B * 2 * E, B, E, w.hc0, (bf16*)w.h_in_t, (long)T1 * E, w.c_in, (long)T1 * E);
    else
      hipLaunchKernelGGL(init_state_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)w.hc0pre, sp.i,
                         (long)B * 2 * E, B, E, w.hc0, (float*)w.h_in_t, (long)T1 * E, w.c_in, (long)T1 * E);
    SAT_LAUNCH_CHECK();
  }
  if (att) {  // hoisted Ws = a W^T + b
    SAT_CHECK((hipError_t)linear(c, B * L, E, D, img_features, D, c.W(lay->attW_w), D, c.F(lay->attW_b), w.Ws, E,
                                 d.dtype, SAT_ACT_NONE, s));
  } else {    // uniform attention: context = mean_L a, alpha = 1/L (decoder.py:101-105)
    SAT_CHECK((hipError_t)linear(c, B, 4 * E, D, w.mean_t, D, c.W(lay->wih + E), E + D, nullptr, w.gctx_const, 4 * E,
                                 SAT_F32, SAT_ACT_NONE, s));
    SAT_CHECK((hipError_t)sat_broadcast_rows(w.mean_t, B, D, T1, d.dtype, w.gated_t, s));
    SAT_CHECK((hipError_t)sat_broadcast_rows(w.mean_t, B, D, T1, d.dtype, w.ctx_t, s));
    SAT_CHECK((hipError_t)sat_broadcast_rows(w.mean_f, B, D, T1, SAT_F32, w.ctx_all, s));
    SAT_CHECK((hipError_t)sat_fill_const(alphas, (long)B * T1 * L, 1.0f / (float)L, s));
  }
  if (d.tf)  // embedding half of the LSTM input GEMM for all steps at once (+ b_ih)
    SAT_CHECK((hipError_t)linear(c, (int)c.R, 4 * E, E, w.emb_t, E, c.W(lay->wih), E + D, c.F(lay->bih), w.xg, 4 * E,
                                 SAT_F32, SAT_ACT_NONE, s));

  if (greedy_fused(d)) return greedy_loop(c, w, sp, io, preds, dropout_mask, tokens, s);

  for (int t = 0; t < T1; ++t) {
    if (!d.tf)
      SAT_CHECK((hipError_t)linear(c, B, 4 * E, E, c.at(w.emb_t, (long)t * E), (long)T1 * E, c.W(lay->wih), E + D,
                                   c.F(lay->bih), w.xg + (long)t * 4 * E, (long)T1 * 4 * E, SAT_F32, SAT_ACT_NONE, s));
    {
      StepTimer st(d, 0, t);
      SAT_CHECK((hipError_t)fwd_hgemm(c, w, sp, t, s));
    }
    if (att) {
      {
        StepTimer st(d, 1, t);
        SAT_CHECK((hipError_t)fwd_attn(c, w, sp, io, t, s));
      }
      StepTimer st(d, 2, t);
      SAT_CHECK((hipError_t)fwd_cgemm(c, w, sp, t, s));
    }
    {
      StepTimer st(d, 3, t);
      SAT_CHECK((hipError_t)fwd_lstm(c, w, sp, t, s));
    }
    if (!d.tf) {
      SAT_CHECK((hipError_t)head_forward(c, w, B, t, true, preds, dropout_mask, s));
      if (t + 1 < T1)   // greedy feedback: argmax -> next token + its embedding (decoder.py:131-133)
        SAT_CHECK((hipError_t)sat_argmax_rows(c.at(preds, (long)t * d.V), d.dtype, (long)T1 * d.V, B, d.V,
                                              w.tok + t + 1, T1, c.F(lay->embedding), E,
                                              c.at(w.emb_t, (long)(t + 1) * E), (long)T1 * E, s));
    }
  }
  if (d.tf) SAT_CHECK((hipError_t)head_forward(c, w, (int)c.R, 0, false, preds, dropout_mask, s));
  if (d.training && d.seed_ptr) SAT_CHECK((hipError_t)sat_bump_seed(d.seed_ptr, s));
  if (tokens) SAT_CHECK(hipMemcpyAsync(tokens, w.tok, c.R * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  return 0;
}

extern "C" int sat_decoder_backward(const SatDecoderDims* dp, const SatDecoderLayout* lay, const float* params,
                                    const void* params_lp, const void* img_features, void* workspace,
                                    size_t workspace_bytes, const void* preds, const float* alphas,
                                    const void* d_preds, const float* d_alphas, float* grads, int accumulate,
                                    int phase, void* stream) {
  SAT_CHECK((hipError_t)check_dims(dp));
  SAT_REQUIRE(lay && params && img_features && workspace && preds && alphas && d_preds && d_alphas && grads);
  // bit 4: d_preds already ReLU-masked (sat_caption_loss_backward_relu); bit 8: d_preds rows at the head's padded
  // stride with zero pad columns (sat_caption_loss_backward_ld), so no copy into padded rows
  SAT_REQUIRE((phase & 3) != 0 && phase >= 1 && phase <= 15);
  SAT_REQUIRE(dp->dtype == SAT_F32 || params_lp);
  SatPolicyScope scope(dp->policy);
  SatStampScope no_stamps(nullptr, 0);   // only the per-step groups of the BPTT loop record timestamps
  const SatDecoderDims& d = *dp;
  WS w;
  SAT_REQUIRE(carve(d, nullptr, &w) <= workspace_bytes);
  carve(d, (char*)workspace, &w);
  hipStream_t s = (hipStream_t)stream;
  Ctx c{d, *lay, params, params_lp, d.dtype == SAT_BF16 ? 2 : 4, d.T - 1, (long)d.B * (d.T - 1), 5L * d.E + d.D,
        use_transposed(d, *lay)};
  const int B = d.B, L = d.L, D = d.D, E = d.E, V = d.V, T1 = d.T - 1;
  const int R = (int)c.R;
  const int VP = head_ld(d);
  const long HG = c.HG;
  const bool att = d.attention != 0;
  const float beta = accumulate ? 1.f : 0.f;
  const Splits sp = splits_for(d, c.tr);
  auto G = [&](int64_t off) { return grads + off; };
  // weight gradient: G[M,N] (+)= X[K,M]^T Y[K,N]   (X m-contig, Y n-contig)
  auto wg = [&](int M, int N, int K, const void* X, long ldx, const void* Y, long ldy, float* out, long ldo,
                int a_tail = 0) {
    SatGemm g;
    g.a_tail = a_tail;
    g.M = M; g.N = N; g.K = K; g.dtype = d.dtype;
    g.A = X; g.lda = ldx; g.transA = 1;
    g.B = Y; g.ldb = ldy; g.transB = 1;
    g.C = out; g.ldc = ldo; g.c_dtype = SAT_F32; g.beta = beta;
    return g;
  };
  // the split-K workspace with ticket block blk (phase 1: 0-7, phase 2: 8-15; each zeroed by its phase's one
  // zeroing launch below)
  const SplitWS sws[kTicketBlocks] = {
      {w.gsplit, w.gtickets, 0}, {w.gsplit, w.gtickets, 1}, {w.gsplit, w.gtickets, 2}, {w.gsplit, w.gtickets, 3},
      {w.gsplit, w.gtickets, 4}, {w.gsplit, w.gtickets, 5}, {w.gsplit, w.gtickets, 6}, {w.gsplit, w.gtickets, 7},
      {w.gsplit, w.gtickets, 8}, {w.gsplit, w.gtickets, 9}, {w.gsplit, w.gtickets, 10}, {w.gsplit, w.gtickets, 11},
      {w.gsplit, w.gtickets, 12}, {w.gsplit, w.gtickets, 13}, {w.gsplit, w.gtickets, 14}, {w.gsplit, w.gtickets, 15}};
  const SatZeroSeg tickets_ph1{(float*)w.gtickets, 1, 8L * kSatSplitTickets, 8L * kSatSplitTickets};
  const SatZeroSeg tickets_ph2{(float*)w.gtickets + 8L * kSatSplitTickets, 1, 8L * kSatSplitTickets,
                               8L * kSatSplitTickets};
  auto wgs = [&](int blk, int M, int N, int K, const void* X, long ldx, const void* Y, long ldy, float* out, long ldo,
                 int a_tail = 0) {
    SatGemm g = wg(M, N, K, X, ldx, Y, ldy, out, ldo, a_tail);
    use_split(g, &sws[blk]);
    return g;
  };
  // the targets of this phase's weight-gradient products that run as atomic split-K on the tile kernel (beta = 0):
  // marked zeroed and appended to one zeroing launch instead of a zeroing pass per product (the split-K kernel
  // writes C itself and needs none)
  auto prezero = [&](SatGemm* const* gs, int n, SatZeroSeg* seg, int& nseg) {
    for (int i = 0; i < n; ++i)
      if (!accumulate && !sat_split_gemm_takes(*gs[i]) && sat_gemm_splits_atomically(*gs[i])) {
        seg[nseg++] = SatZeroSeg{(float*)gs[i]->C, gs[i]->M, gs[i]->N, gs[i]->ldc};
        gs[i]->c_zeroed = 1;
      }
  };
  auto dgrad = [&](int blk, int M, int N, int K, const void* X, long ldx, const void* Wt, long ldw, float* out,
                   long ldo, const float* add1 = nullptr, long ld_add1 = 0) {
    return dgrad_launch(c, M, N, K, X, ldx, Wt, ldw, out, ldo, s, add1, ld_add1, 0, 0, 0, &sws[blk]);
  };
  auto colsum = [&](const void* X, int dt, long ld, int rows, int N, float* out, float* out2 = nullptr,
                    int cols_readable = 0) {
    return sat_colsum(X, dt, ld, rows, N, out, accumulate, out2, w.colsum, s, cols_readable);
  };

  if (phase & 1) {  // ---------------- output head (decoder.py:117-125,149-158) ----------------
    if (d.ado) {
      // d logits through the ReLU of the advanced deep output; phase bit 4: the caller's d_preds is
      // already masked (sat_caption_loss_backward_relu fused it)
      const void* dpre = d_preds;
      long ldp = V;
      if (phase & 8) {
        SAT_REQUIRE(phase & 4);   // the padded layout comes from the loss, which masks
        ldp = VP;
      } else if (VP != V) {
        SAT_CHECK((hipError_t)sat_pad_rows(d_preds, (phase & 4) ? nullptr : preds, R, V, VP, d.dtype, w.dpre_t, s));
        dpre = w.dpre_t; ldp = VP;
      } else if (!(phase & 4)) {
        SAT_CHECK((hipError_t)sat_relu_mask_mul(d_preds, preds, (long)R * V, d.dtype, w.dpre_t, s));
        dpre = w.dpre_t;
      }
      SatGemm gfo = wgs(0, V, E, R, dpre, ldp, w.comb_t, E, G(lay->fout_w), E, VP != V);
      SatGemm gfh = wgs(2, E, E, R, w.dfh_t, E, w.hd_t, E, G(lay->fh_w), E);
      SatGemm gfz = wgs(3, E, D, R, w.dfz_t, E, w.ctx_t, D, G(lay->fz_w), D);
      {
        SatGemm* gs[3] = {&gfo, &gfh, &gfz};
        SatZeroSeg seg[4];
        int nseg = 0;
        if (w.gtickets) seg[nseg++] = tickets_ph1;
        prezero(gs, 3, seg, nseg);
        SAT_CHECK((hipError_t)sat_zero_segs(seg, nseg, s));
      }
      SAT_CHECK((hipError_t)sat_gemm_launch(gfo, s));
      SAT_CHECK((hipError_t)dgrad_launch(c, R, E, V, dpre, ldp, c.W(lay->fout_w), E, w.dcomb, E, s, nullptr, 0, 0, 0,
                                         VP != V, &sws[1]));
      SAT_CHECK((hipError_t)sat_ado_bwd_split(w.dcomb, w.fh, w.fz, (long)R * E, d.dtype, w.dfh_t, w.dfz_t, s));
      SAT_CHECK((hipError_t)sat_gemm_launch(gfh, s));
      SAT_CHECK((hipError_t)sat_gemm_launch(gfz, s));
      // the three bias gradients (column sums of d logits, d f_h, d f_z) in one launch pair
      const SatColsumSeg cs[3] = {{dpre, d.dtype, ldp, R, V, G(lay->fout_b), accumulate, nullptr, ldp != V},
                                  {w.dfh_t, d.dtype, E, R, E, G(lay->fh_b), accumulate, nullptr},
                                  {w.dfz_t, d.dtype, E, R, E, G(lay->fz_b), accumulate, nullptr}};
      SAT_CHECK((hipError_t)sat_colsum_multi(cs, 3, w.colsum, s));
      SAT_CHECK((hipError_t)dgrad(4, R, E, E, w.dfh_t, E, c.W(lay->fh_w), E, w.dhd, E));
      if (att) SAT_CHECK((hipError_t)dgrad(5, R, D, E, w.dfz_t, E, c.W(lay->fz_w), D, w.dctx_head, D));
    } else {
      const void* dpre = d_preds;
      long ldp = (phase & 8) ? VP : V;
      if (VP != V && !(phase & 8)) {
        SAT_CHECK((hipError_t)sat_pad_rows(d_preds, nullptr, R, V, VP, d.dtype, w.dpre_t, s));
        dpre = w.dpre_t; ldp = VP;
      }
      SatGemm gdo = wgs(0, V, E, R, dpre, ldp, w.hd_t, E, G(lay->do_w), E, VP != V);
      {
        SatGemm* gs[1] = {&gdo};
        SatZeroSeg seg[2];
        int nseg = 0;
        if (w.gtickets) seg[nseg++] = tickets_ph1;
        prezero(gs, 1, seg, nseg);
        SAT_CHECK((hipError_t)sat_zero_segs(seg, nseg, s));
      }
      SAT_CHECK((hipError_t)sat_gemm_launch(gdo, s));
      // the bias gradient from the padded copy when there is one: 16-B aligned rows take the vector column sum (the
      // unpadded BERT rows took the scalar one: 206 us per step, profiles/r6_s13)
      SAT_CHECK((hipError_t)colsum(dpre, d.dtype, ldp, R, V, G(lay->do_b), nullptr, ldp != V));
      SAT_CHECK((hipError_t)dgrad_launch(c, R, E, V, dpre, ldp, c.W(lay->do_w), E, w.dhd, E, s, nullptr, 0, 0, 0,
                                         VP != V, &sws[1]));
    }
  }
  if (!(phase & 2)) return 0;

  // ---------------- recurrent BPTT (reverse time loop) ----------------
  // this phase's weight-gradient products (launched after the loop)
  const void* dg_t = c.at(w.dhg_t, E + D);   // d gates rows (ld HG)
  SatGemm g_attw = wgs(8, E, D, B * L, w.dWs_t, E, img_features, D, G(lay->attW_w), D);
  SatGemm g_init = wgs(9, 2 * E, D, B, w.dpre0_t, 2 * E, w.mean_t, D, G(lay->init_w), D);
  SatGemm g_hcat = att ? wgs(10, (int)HG, E, R, w.dhg_t, HG, w.h_in_t, E, G(lay->hcat_w), E)
                       : wgs(10, 4 * E, E, R, dg_t, HG, w.h_in_t, E, G(lay->hcat_w + (long)(E + D) * E), E);
  SatGemm g_wihx = wgs(11, 4 * E, E, R, dg_t, HG, w.emb_t, E, G(lay->wih), E + D);
  SatGemm g_wihc = wgs(12, 4 * E, D, R, dg_t, HG, w.gated_t, D, G(lay->wih + E), E + D);
  {   // one launch zeroes the BPTT accumulators, the split attention backward's tickets, (beta = 0) the dense
      // embedding gradient the scatter-add after the loop accumulates into, and the atomic split-K targets
    SatZeroSeg seg[12];
    int nz = 0;
    if (att) {
      seg[nz++] = SatZeroSeg{w.dv_acc, 1, (long)B * E, (long)B * E};
      seg[nz++] = SatZeroSeg{w.dbv_acc, 1, B, B};
      seg[nz++] = SatZeroSeg{(float*)w.ticket, 1, B, B};
    }
    if (!d.bert && !accumulate) seg[nz++] = SatZeroSeg{G(lay->embedding), 1, (long)V * E, (long)V * E};
    if (w.gtickets) seg[nz++] = tickets_ph2;
    SatGemm* gs[5] = {&g_hcat, &g_wihx, &g_wihc, &g_init, &g_attw};
    prezero(gs, att ? 5 : 4, seg, nz);
    SAT_CHECK((hipError_t)sat_zero_segs(seg, nz, s));
  }
  const StepIO io{img_features, const_cast<float*>(alphas), d_alphas};
  for (int t = T1 - 1; t >= 0; --t) {
    {
      StepTimer st(d, 4, t);
      SAT_CHECK((hipError_t)bwd_lstm(c, w, sp, t, s));
    }
    if (att) {
      {
        StepTimer st(d, 5, t);
        SAT_CHECK((hipError_t)bwd_ggemm(c, w, sp, t, s));
      }
      StepTimer st(d, 6, t);
      SAT_CHECK((hipError_t)bwd_attn(c, w, sp, io, t, s));
    }
    StepTimer st(d, 7, t);
    SAT_CHECK((hipError_t)bwd_dhgemm(c, w, sp, t, s));
  }

  // ---------------- weight gradients, batched over all B*(T-1) rows ----------------
  if (att) {
    SAT_CHECK((hipError_t)sat_attention_dws_launch(w.Ws, w.uh_all, w.de_all, c.F(lay->v_w), B, L, E, T1, d.dtype,
                                                   w.dWs_acc, w.dWs_t, s));
    SAT_CHECK((hipError_t)sat_gemm_launch(g_attw, s));
  }
  // init_h / init_c (decoder.py:137-147): dh0 = dh_rec, dc0 = dc after the t = 0 step
  SAT_CHECK((hipError_t)sat_tanh_pair_bwd(w.dh_rec, sp.dh, (long)B * E, w.dc, w.hc0, B, E, w.dpre0, w.dpre0_t,
                                          d.dtype, s));
  SAT_CHECK((hipError_t)sat_gemm_launch(g_init, s));
  {   // every bias gradient of this phase (column sums) in one launch pair; b_hh and b_ih receive the same
      // gradient (the sum of d gates)
    SatColsumSeg cs[6];
    int n = 0;
    if (att) {
      cs[n++] = {w.dWs_acc, SAT_F32, E, B * L, E, G(lay->attW_b), accumulate, nullptr};
      cs[n++] = {w.dv_acc, SAT_F32, E, B, E, G(lay->v_w), accumulate, nullptr};
      cs[n++] = {w.dbv_acc, SAT_F32, 1, B, 1, G(lay->v_b), accumulate, nullptr};
      cs[n++] = {w.dhg, SAT_F32, HG, R, E + D, G(lay->hcat_b), accumulate, nullptr};
    }
    cs[n++] = {w.dpre0, SAT_F32, 2 * E, B, 2 * E, G(lay->init_b), accumulate, nullptr};
    cs[n++] = {w.dhg + E + D, SAT_F32, HG, R, 4 * E, G(lay->hcat_b + E + D), accumulate, G(lay->bih)};
    SAT_CHECK((hipError_t)sat_colsum_multi(cs, n, w.colsum, s));
  }

  SAT_CHECK((hipError_t)sat_gemm_launch(g_hcat, s));
  SAT_CHECK((hipError_t)sat_gemm_launch(g_wihx, s));
  SAT_CHECK((hipError_t)sat_gemm_launch(g_wihc, s));
  if (!d.bert) {  // dense embedding gradient (zeroed before the loop), scatter-added by fed token (decoder.py:87,133)
    SAT_CHECK((hipError_t)dgrad(13, R, E, 4 * E, dg_t, HG, c.W(lay->wih), E + D, w.demb, E, d.ado ? w.dcomb : nullptr,
                                E));
    if (w.emb_ws)
      SAT_CHECK((hipError_t)sat_embed_scatter_add_sorted(w.demb, w.tok, R, E, G(lay->embedding), accumulate, w.emb_ws,
                                                         s));
    else
      SAT_CHECK((hipError_t)sat_embed_scatter_add(w.demb, w.tok, R, E, G(lay->embedding), s));
  }
  return 0;
}

// Diagnostics (bench.py roofline of the per-step decoder kernels): after a forward + backward on the
// same arguments have filled the workspace, re-issue each per-step kernel group of step t = (T-1)/2
// `reps` times back to back between two HIP events on `stream`, and return the average microseconds
// per launch group in us_out[0..7]: h GEMM, attention forward, context GEMM, LSTM forward, LSTM
// backward, d(gated context) GEMM, attention backward (2 kernels), dh GEMM.  The re-issued backward
// groups overwrite the workspace's running dc / dv sums: call it only after the gradients are read.
extern "C" int sat_decoder_step_bench(const SatDecoderDims* dp, const SatDecoderLayout* lay, const float* params,
                                      const void* params_lp, const void* img_features, void* workspace,
                                      size_t workspace_bytes, float* alphas, const float* d_alphas, int reps,
                                      float* us_out, void* stream) {
  SAT_CHECK((hipError_t)check_dims(dp));
  SAT_REQUIRE(lay && params && img_features && workspace && alphas && d_alphas && us_out && reps > 0);
  SAT_REQUIRE(dp->dtype == SAT_F32 || params_lp);
  SatPolicyScope scope(dp->policy);
  SatStampScope no_stamps(nullptr, 0);
  const SatDecoderDims& d = *dp;
  WS w;
  SAT_REQUIRE(carve(d, nullptr, &w) <= workspace_bytes);
  carve(d, (char*)workspace, &w);
  hipStream_t s = (hipStream_t)stream;
  Ctx c{d, *lay, params, params_lp, d.dtype == SAT_BF16 ? 2 : 4, d.T - 1, (long)d.B * (d.T - 1), 5L * d.E + d.D,
        use_transposed(d, *lay)};
  const Splits sp = splits_for(d, c.tr);
  const StepIO io{img_features, alphas, d_alphas};
  const int t = (d.T - 1) / 2;
  hipEvent_t e0, e1;
  SAT_CHECK(hipEventCreate(&e0));
  SAT_CHECK(hipEventCreate(&e1));
  int rc = 0;
  for (int k = 0; k < 8 && rc == 0; ++k) {
    us_out[k] = 0.f;
    if (!d.attention && (k == 1 || k == 2 || k == 5 || k == 6)) continue;
    for (int r = -1; r < reps && rc == 0; ++r) {   // r = -1: warm-up launch
      if (r == 0) rc = (int)hipEventRecord(e0, s);
      switch (k) {
        case 0: rc = fwd_hgemm(c, w, sp, t, s); break;
        case 1: rc = fwd_attn(c, w, sp, io, t, s); break;
        case 2: rc = fwd_cgemm(c, w, sp, t, s); break;
        case 3: rc = fwd_lstm(c, w, sp, t, s); break;
        case 4: rc = bwd_lstm(c, w, sp, t, s); break;
        case 5: rc = bwd_ggemm(c, w, sp, t, s); break;
        case 6: rc = bwd_attn(c, w, sp, io, t, s); break;
        default: rc = bwd_dhgemm(c, w, sp, t, s); break;
      }
    }
    if (rc == 0) rc = (int)hipEventRecord(e1, s);
    if (rc == 0) rc = (int)hipEventSynchronize(e1);
    float ms = 0.f;
    if (rc == 0) rc = (int)hipEventElapsedTime(&ms, e0, e1);
    us_out[k] = ms * 1000.f / reps;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}
