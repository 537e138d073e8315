// Beam-search captioning (decoder.py:160-269, Decoder.caption) on the HIP decoder step.
//
// The reference runs one LSTM step for the k live beams per iteration, adds each beam's running
// score to its raw logits, takes the top-k of the flattened [k, V] scores, appends the words,
// retires beams that emitted an end token and compacts the survivors' (h, c, features) by their
// parent index.  Here every tensor step runs on the GPU (one fused kernel sequence per
// iteration, all rows of the live beam batched into each launch) and the host keeps only the
// per-beam word/alpha histories the reference keeps in Python lists: one small D2H of the k
// winners (+ their alpha rows) and one H2D of the compaction indices per iteration.
//
// Device state is sized for the initial beam width; each iteration ping-pongs the gathered
// per-beam feature / W·a rows so the compaction never reads what it writes.
#include <math.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "sat_common.h"
#include "sat_internal.h"

namespace {

struct BeamWS {
  void *feat[2], *Ws[2], *h_t, *h_new, *emb_t, *ctx_t, *gated_t, *comb_t, *mean_t;
  float *c, *c_new, *h_f32, *xg, *hg, *gctx, *gates, *ctx, *gate, *alpha, *fh, *fz, *logits, *top_val, *mean_f,
      *hc0;
  int32_t *upl, *top_idx;  // upl = [gather idx k | tokens k | scores k (float bits)]
};

size_t beam_carve(const SatDecoderDims& d, int R, char* base, BeamWS* w) {
  const size_t L = d.L, D = d.D, E = d.E, V = d.V, HG = 5 * E + D;
  const size_t ts = d.dtype == SAT_BF16 ? 2 : 4, f = 4;
  size_t off = 0;
  auto take = [&](auto*& p, size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    p = base ? (std::remove_reference_t<decltype(p)>)(base + off) : nullptr;
    off += bytes;
  };
  for (int i = 0; i < 2; ++i) { take(w->feat[i], R * L * D * ts); take(w->Ws[i], R * L * E * ts); }
  take(w->h_t, R * E * ts); take(w->h_new, R * E * ts); take(w->emb_t, R * E * ts);
  take(w->ctx_t, R * D * ts); take(w->gated_t, R * D * ts); take(w->comb_t, R * E * ts);
  take(w->mean_t, R * D * ts);
  take(w->c, R * E * f); take(w->c_new, R * E * f); take(w->h_f32, R * E * f);
  take(w->xg, R * 4 * E * f); take(w->hg, R * HG * f); take(w->gctx, R * 4 * E * f); take(w->gates, R * 4 * E * f);
  take(w->ctx, R * D * f); take(w->gate, R * D * f); take(w->alpha, R * L * f);
  take(w->fh, R * E * f); take(w->fz, R * E * f); take(w->logits, R * V * f);
  take(w->top_val, R * f); take(w->mean_f, R * D * f); take(w->hc0, R * 2 * E * f);
  take(w->upl, 3 * R * 4); take(w->top_idx, R * 4);
  return off + 256;
}

// ---- top-k of (logits[r, v] + score[r]) over r < rows, v < V --------------------------------
// torch.topk(largest=True, sorted=True) over the flattened scores (decoder.py:204-209).  K <= 64
// passes of one block-wide arg-max each; pass j takes the best element strictly after pass j-1's
// winner in (value desc, index asc) order, so no element is marked or copied.  Ties are broken
// by the lower flat index (torch leaves the order of equal values unspecified).
constexpr int TOPK_THREADS = 1024;

__device__ __forceinline__ bool tk_better(float v, int i, float bv, int bi) {
  return v > bv || (v == bv && i < bi);
}

__global__ void __launch_bounds__(TOPK_THREADS) beam_topk_kernel(const float* __restrict__ logits, long ld,
                                                                 const float* __restrict__ score, int rows, int V,
                                                                 int K, float* top_val, int32_t* top_idx) {
  __shared__ float sv[TOPK_THREADS / 64];
  __shared__ int si[TOPK_THREADS / 64];
  __shared__ float pv_s;
  __shared__ int pi_s;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long n = (long)rows * V;
  float pv = INFINITY;
  int pi = -1;
  for (int j = 0; j < K; ++j) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (long i = threadIdx.x; i < n; i += TOPK_THREADS) {
      const int r = (int)(i / V), c = (int)(i - (long)r * V);
      const float v = logits[(long)r * ld + c] + (score ? score[r] : 0.f);
      const bool after = v < pv || (v == pv && (int)i > pi);
      if (after && tk_better(v, (int)i, bv, bi)) { bv = v; bi = (int)i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (tk_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { sv[wid] = bv; si[wid] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float b = sv[0];
      int ib = si[0];
      for (int w = 1; w < TOPK_THREADS / 64; ++w)
        if (tk_better(sv[w], si[w], b, ib)) { b = sv[w]; ib = si[w]; }
      top_val[j] = b;
      top_idx[j] = ib;
      pv_s = b;
      pi_s = ib;
    }
    __syncthreads();
    pv = pv_s;
    pi = pi_s;
  }
}

// ---- compaction: dst_q[i] = src_q[idx[i]] for up to 6 row tensors (16-byte rows) -----------
struct GatherSet {
  const void* src[6];
  void* dst[6];
  long row_bytes[6];
  int n;
};

__global__ void beam_gather_kernel(GatherSet g, const int32_t* __restrict__ idx) {
  const int q = blockIdx.y;
  if (q >= g.n) return;
  const long rb = g.row_bytes[q] >> 4;
  const uint4* s = (const uint4*)g.src[q] + (long)idx[blockIdx.x] * rb;
  uint4* d = (uint4*)g.dst[q] + (long)blockIdx.x * rb;
  for (long i = threadIdx.x; i < rb; i += blockDim.x) d[i] = s[i];
}

struct BeamCtx {
  SatDecoderDims d;
  SatDecoderLayout lay;
  const float* P;
  const void* LP;
  const void* W(int64_t off) const {
    return d.dtype == SAT_BF16 ? (const void*)((const bf16*)LP + off) : (const void*)(P + off);
  }
  const float* F(int64_t off) const { return off < 0 ? nullptr : P + off; }
};

int lin(const BeamCtx& c, int rows, int N, int K, const void* x, long ldx, const void* w, long ldw, const float* bias,
        void* y, long ldy, int act, hipStream_t s, void* aux = nullptr, long ld_aux = 0, int aux_dtype = SAT_F32,
        int y_dtype = SAT_F32) {
  SatGemm g;
  g.M = rows; g.N = N; g.K = K; g.dtype = c.d.dtype;
  g.A = x; g.lda = ldx; g.B = w; g.ldb = ldw;
  g.C = y; g.ldc = ldy; g.c_dtype = y_dtype; g.bias = bias; g.act = act;
  g.aux = aux; g.ld_aux = ld_aux; g.aux_dtype = aux_dtype;
  return sat_gemm_launch(g, s);
}

__global__ void ado_sum_kernel(const float* fh, const float* fz, const void* emb, long n, int dt, void* out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    st_from_f32(out, i, dt, fh[i] + fz[i] + ld_as_f32(emb, i, dt));
}

// One decoder step for k live beams: decoder.py:183-204 (no dropout in caption()).  Leaves the
// raw logits in w.logits [k, V] fp32, alpha rows in w.alpha, the new state in h_new / c_new.
// `feat` / `Ws` are the current (compacted) per-beam rows; tokens are upl[R .. R+k).
int beam_step(const BeamCtx& c, const BeamWS& w, int R, int k, const void* feat, const void* Ws, hipStream_t s) {
  const SatDecoderDims& d = c.d;
  const int L = d.L, D = d.D, E = d.E, V = d.V, HG = 5 * E + D;
  const SatDecoderLayout& lay = c.lay;
  // embedding of the fed words (decoder.py:183) and its half of the LSTM input GEMM (+ b_ih)
  SAT_CHECK((hipError_t)sat_embed_gather(c.F(lay.embedding), w.upl + R, k, 1, 1, E, d.dtype, w.emb_t, E, s));
  SAT_CHECK((hipError_t)lin(c, k, 4 * E, E, w.emb_t, E, c.W(lay.wih), E + D, c.F(lay.bih), w.xg, 4 * E,
                            SAT_ACT_NONE, s));
  if (d.attention) {
    // [U h + b | f_beta h + b | W_hh h + b_hh] (attention.py:15, decoder.py:187, LSTMCell)
    SAT_CHECK((hipError_t)lin(c, k, HG, E, w.h_t, E, c.W(lay.hcat_w), E, c.F(lay.hcat_b), w.hg, HG, SAT_ACT_NONE, s));
    AttnFwdArgs a{};
    a.B = k; a.L = L; a.D = D; a.E = E; a.dtype = d.dtype;
    a.Ws = Ws; a.uh = w.hg; a.uh_ld = HG; a.v_w = c.F(lay.v_w); a.v_b = c.F(lay.v_b); a.a = feat;
    a.gate_pre = w.hg + E; a.gate_ld = HG;
    a.hg_splits = 1; a.hg_split_stride = 0;
    a.alpha = w.alpha; a.alpha_ld = L;
    a.ctx = w.ctx; a.ctx_ld = D;
    a.ctx_t = w.ctx_t; a.ctx_t_ld = D;
    a.gate = w.gate; a.gate_out_ld = D;
    a.gated = w.gated_t; a.gated_ld = D;
    SAT_CHECK((hipError_t)sat_attention_fwd_launch(a, s));
    SAT_CHECK((hipError_t)lin(c, k, 4 * E, D, w.gated_t, D, c.W(lay.wih + E), E + D, nullptr, w.gctx, 4 * E,
                              SAT_ACT_NONE, s));
  } else {  // uniform attention over the (gathered) rows: decoder.py:190-194
    SAT_CHECK((hipError_t)sat_mean_rows(feat, k, L, D, d.dtype, w.ctx, w.ctx_t, s));
    SAT_CHECK((hipError_t)sat_fill_const(w.alpha, (long)k * L, 1.0f / (float)L, s));
    SAT_CHECK((hipError_t)lin(c, k, 4 * E, D, w.ctx_t, D, c.W(lay.wih + E), E + D, nullptr, w.gctx, 4 * E,
                              SAT_ACT_NONE, s));
    SAT_CHECK((hipError_t)lin(c, k, 4 * E, E, w.h_t, E, c.W(lay.hcat_w + (long)(E + D) * E), E,
                              c.F(lay.hcat_b + E + D), w.hg + E + D, HG, SAT_ACT_NONE, s));
  }
  LstmFwdArgs l{};
  l.B = k; l.E = E; l.dtype = d.dtype;
  l.hpart = w.hg + E + D; l.hpart_ld = HG;
  l.xpart = w.xg; l.xpart_ld = 4 * E;
  l.cpart = w.gctx; l.cpart_ld = 4 * E;
  l.h_splits = 1; l.c_splits = 1;
  l.c_prev = w.c; l.c_prev_ld = E;
  l.gates = w.gates; l.gates_ld = 4 * E;
  l.c_out = w.c_new; l.c_out_ld = E;
  l.h_out = w.h_f32; l.h_out_ld = E;
  l.h_next_in_t = w.h_new; l.h_next_in_t_ld = E;
  SAT_CHECK((hipError_t)sat_lstm_fwd_launch(l, s));
  if (d.ado) {  // decoder.py:199-201,149-158 (context is the ungated one)
    SAT_CHECK((hipError_t)lin(c, k, E, E, w.h_new, E, c.W(lay.fh_w), E, c.F(lay.fh_b), w.fh, E, SAT_ACT_RELU, s));
    SAT_CHECK((hipError_t)lin(c, k, E, D, w.ctx_t, D, c.W(lay.fz_w), D, c.F(lay.fz_b), w.fz, E, SAT_ACT_RELU, s));
    const long n = (long)k * E;
    hipLaunchKernelGGL(ado_sum_kernel, dim3(sat_cdiv(n, 256)), dim3(256), 0, s, w.fh, w.fz, (const void*)w.emb_t, n,
                       d.dtype, w.comb_t);
    SAT_LAUNCH_CHECK();
    SAT_CHECK((hipError_t)lin(c, k, V, E, w.comb_t, E, c.W(lay.fout_w), E, c.F(lay.fout_b), w.logits, V,
                              SAT_ACT_RELU, s));
  } else {      // decoder.py:203
    SAT_CHECK((hipError_t)lin(c, k, V, E, w.h_new, E, c.W(lay.do_w), E, c.F(lay.do_b), w.logits, V, SAT_ACT_NONE, s));
  }
  return 0;
}

int gather_rows(const GatherSet& g, const int32_t* idx, int k, hipStream_t s) {
  for (int q = 0; q < g.n; ++q)
    if ((g.row_bytes[q] & 15) || (((uintptr_t)g.src[q] | (uintptr_t)g.dst[q]) & 15)) return SAT_ERR_INVALID;
  hipLaunchKernelGGL(beam_gather_kernel, dim3(k, g.n), dim3(256), 0, s, g, idx);
  return (int)hipGetLastError();
}

int check_beam(const SatDecoderDims* d, int beam) {
  if (!d) return SAT_ERR_INVALID;
  if (d->L <= 0 || d->D <= 0 || d->E <= 0 || d->V <= 0 || beam <= 0 || beam > 64) return SAT_ERR_INVALID;
  if (d->dtype != SAT_F32 && d->dtype != SAT_BF16) return SAT_ERR_INVALID;
  if (d->E % 8 != 0 || d->D % 8 != 0 || d->E > 1024 || d->L > 1024) return SAT_ERR_INVALID;
  if ((long)beam * d->V >= 0x7fffffffL) return SAT_ERR_INVALID;
  return 0;
}

}  // namespace

extern "C" size_t sat_decoder_beam_workspace_bytes(const SatDecoderDims* d, int beam_size) {
  if (check_beam(d, beam_size)) return 0;
  BeamWS w;
  return beam_carve(*d, beam_size, nullptr, &w);
}

extern "C" int sat_decoder_beam_search(const SatDecoderDims* dp, const SatDecoderLayout* lay, const float* params,
                                       const void* params_lp, const void* img_features, int beam_size, int max_step,
                                       void* workspace, size_t workspace_bytes, int32_t* out_ids, int* out_len,
                                       float* out_alphas, int* out_alpha_rows, float* out_score, void* stream) {
  SAT_CHECK((hipError_t)check_beam(dp, beam_size));
  SAT_REQUIRE(lay && params && img_features && workspace && out_ids && out_len && out_alphas && out_alpha_rows &&
              out_score && max_step >= 0);
  SAT_REQUIRE(dp->dtype == SAT_F32 || params_lp);
  SAT_REQUIRE(beam_size <= max_step + 2);  // out_alphas holds (max_step + 2) * L floats
  SatPolicyScope scope(dp->policy);
  SatStampScope no_stamps(nullptr, 0);
  const SatDecoderDims& d = *dp;
  const int R = beam_size, L = d.L, D = d.D, E = d.E, V = d.V;
  const size_t ts = d.dtype == SAT_BF16 ? 2 : 4;
  BeamWS w;
  SAT_REQUIRE(beam_carve(d, R, nullptr, &w) <= workspace_bytes);
  beam_carve(d, R, (char*)workspace, &w);
  hipStream_t s = (hipStream_t)stream;
  BeamCtx c{d, *lay, params, params_lp};

  // ---- initial state for the beam_size rows (decoder.py:167-180) ----
  const int start = d.start_token;   // 0 = <start>; [CLS] under BERT (decoder.py:166-169)
  std::vector<int32_t> upl(3 * R);
  for (int i = 0; i < R; ++i) { upl[i] = i; upl[R + i] = start; float z = 0.f; memcpy(&upl[2 * R + i], &z, 4); }
  SAT_CHECK(hipMemcpyAsync(w.upl, upl.data(), 3 * R * 4, hipMemcpyHostToDevice, s));
  SAT_CHECK(hipMemcpyAsync(w.feat[0], img_features, (size_t)R * L * D * ts, hipMemcpyDeviceToDevice, s));
  SAT_CHECK((hipError_t)sat_mean_rows(w.feat[0], R, L, D, d.dtype, w.mean_f, w.mean_t, s));
  SAT_CHECK((hipError_t)lin(c, R, E, D, w.mean_t, D, c.W(lay->init_w), D, c.F(lay->init_b), w.hc0, 2 * E,
                            SAT_ACT_TANH, s, w.h_t, E, d.dtype));
  SAT_CHECK((hipError_t)lin(c, R, E, D, w.mean_t, D, c.W(lay->init_w + (long)E * D), D, c.F(lay->init_b + E),
                            w.hc0 + E, 2 * E, SAT_ACT_TANH, s, w.c, E, SAT_F32));
  if (d.attention)  // hoisted W·a + b per beam row (attention.py:16), stored in the operand dtype
    SAT_CHECK((hipError_t)lin(c, R * L, E, D, w.feat[0], D, c.W(lay->attW_w), D, c.F(lay->attW_b), w.Ws[0], E,
                              SAT_ACT_NONE, s, nullptr, 0, SAT_F32, d.dtype));

  // host-side histories (the reference's Python lists, decoder.py:171-177)
  struct Hyp { std::vector<int32_t> words; std::vector<float> alphas; };
  std::vector<Hyp> beams(R);
  for (auto& b : beams) { b.words.assign(1, start); b.alphas.assign(L, 1.0f); }
  std::vector<Hyp> done;
  std::vector<float> done_score;
  std::vector<float> tv(R), al((size_t)R * L);
  std::vector<int32_t> ti(R);
  int k = R, cur = 0, last_rows = 0;
  const long feat_row = (long)L * D * ts, ws_row = (long)L * E * ts;
  for (int step = 1;; ++step) {
    SAT_CHECK((hipError_t)beam_step(c, w, R, k, w.feat[cur], w.Ws[cur], s));
    // step 1: every beam row is the same hypothesis -> top-k over row 0 only (decoder.py:206-207)
    hipLaunchKernelGGL(beam_topk_kernel, dim3(1), dim3(TOPK_THREADS), 0, s, (const float*)w.logits, (long)V,
                       step == 1 ? (const float*)nullptr : (const float*)(w.upl + 2 * R), step == 1 ? 1 : k, V, k,
                       w.top_val, w.top_idx);
    SAT_LAUNCH_CHECK();
    SAT_CHECK(hipMemcpyAsync(tv.data(), w.top_val, k * 4, hipMemcpyDeviceToHost, s));
    SAT_CHECK(hipMemcpyAsync(ti.data(), w.top_idx, k * 4, hipMemcpyDeviceToHost, s));
    SAT_CHECK(hipMemcpyAsync(al.data(), w.alpha, (size_t)k * L * 4, hipMemcpyDeviceToHost, s));
    SAT_CHECK(hipStreamSynchronize(s));
    last_rows = k;
    // extend, retire completed (decoder.py:210-241)
    std::vector<Hyp> next(k);
    std::vector<int> prev(k), word(k), keep;
    for (int j = 0; j < k; ++j) {
      prev[j] = ti[j] / V;
      word[j] = ti[j] - prev[j] * V;
      next[j].words = beams[prev[j]].words;
      next[j].words.push_back(word[j]);
      next[j].alphas = beams[prev[j]].alphas;
      next[j].alphas.insert(next[j].alphas.end(), al.begin() + (size_t)prev[j] * L, al.begin() + (size_t)(prev[j] + 1) * L);
      // BERT quick-fix of the reference: ids 1 / 0 end a BERT beam, 1 / 102 a vocabulary beam
      const bool end = d.bert ? (word[j] == 1 || word[j] == 0) : (word[j] == 1 || word[j] == 102);
      if (!end) keep.push_back(j);
    }
    for (int j = 0; j < k; ++j) {
      bool kept = false;
      for (int q : keep) kept |= (q == j);
      if (!kept) { done.push_back(next[j]); done_score.push_back(tv[j]); }
    }
    const int nk = (int)keep.size();
    if (nk == 0) break;
    // compact the survivors (decoder.py:243-250)
    std::vector<Hyp> nb(nk);
    for (int q = 0; q < nk; ++q) {
      nb[q] = std::move(next[keep[q]]);
      upl[q] = prev[keep[q]];
      upl[R + q] = word[keep[q]];
      memcpy(&upl[2 * R + q], &tv[keep[q]], 4);
    }
    beams.swap(nb);
    SAT_CHECK(hipMemcpyAsync(w.upl, upl.data(), 3 * R * 4, hipMemcpyHostToDevice, s));
    GatherSet g{};
    g.n = 0;
    auto add = [&](const void* src, void* dst, long rb) { g.src[g.n] = src; g.dst[g.n] = dst; g.row_bytes[g.n] = rb; ++g.n; };
    add(w.h_new, w.h_t, (long)E * ts);
    add(w.c_new, w.c, (long)E * 4);
    add(w.feat[cur], w.feat[cur ^ 1], feat_row);
    if (d.attention) add(w.Ws[cur], w.Ws[cur ^ 1], ws_row);
    SAT_CHECK((hipError_t)gather_rows(g, w.upl, nk, s));
    cur ^= 1;
    k = nk;
    if (step > max_step) break;
  }
  // the pageable H2D above may still be reading `upl` -> drain before the vector goes away
  SAT_CHECK(hipStreamSynchronize(s));
  if (done.empty()) {  // decoder.py:256-258: returns [0] and the last step's alpha rows
    out_ids[0] = 0;
    *out_len = 1;
    memcpy(out_alphas, al.data(), (size_t)last_rows * L * 4);
    *out_alpha_rows = last_rows;
    *out_score = -INFINITY;
    return 0;
  }
  size_t best = 0;   // first maximum (list.index(max(...)), decoder.py:265)
  for (size_t i = 1; i < done.size(); ++i)
    if (done_score[i] > done_score[best]) best = i;
  const Hyp& h = done[best];
  memcpy(out_ids, h.words.data(), h.words.size() * 4);
  *out_len = (int)h.words.size();
  memcpy(out_alphas, h.alphas.data(), h.alphas.size() * 4);
  *out_alpha_rows = (int)h.words.size();
  *out_score = done_score[best];
  return 0;
}
