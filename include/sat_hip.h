/*
 * sat_hip.h — C ABI of the MI355X-native Show-Attend-and-Tell training path.
 *
 * The reference (yvokeller/Show-Attend-and-Tell) has no FFI: its hot path is the
 * PyTorch nn.Module API (encoder.py, attention.py, decoder.py) called from the
 * inner loop of train.py.  This header is the boundary *below* that API: every
 * entry point replaces a PyTorch op sequence of the reference, cited as
 * file:line.  The Python package (show-attend-and-tell_amd/, imported as
 * ``sat_amd``) keeps the reference module API and binds these symbols with
 * ctypes; a maintainer-side binding is shown in INTEGRATION.md.
 *
 * Conventions
 *   - All tensor arguments are DEVICE pointers allocated by the caller (PyTorch's
 *     caching allocator owns every buffer, including workspaces).
 *   - ``stream`` is a hipStream_t (pass torch.cuda.current_stream().cuda_stream);
 *     every call is asynchronous on it and performs no host synchronisation, so
 *     calls are legal inside hipGraph stream capture.
 *   - Return value: 0 on success, SAT_ERR_INVALID for a rejected shape/argument,
 *     otherwise the hipError_t of the failing HIP call.  The Python layer raises
 *     RuntimeError on non-zero, as the reference raises Python exceptions.
 *   - dtype: SAT_F32 = exact fp32 path (parity mode, fp32-input MFMA);
 *            SAT_BF16 = bf16 operands, fp32 accumulation (performance mode).
 *   - Layouts are row-major; image tensors are NHWC (channels last), which makes
 *     the encoder's permute(0,2,3,1).view(B,-1,C) (encoder.py:37-39) free.
 */
#ifndef SAT_HIP_H_
#define SAT_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SAT_ABI_VERSION 9

enum { SAT_F32 = 0, SAT_BF16 = 1 };
enum { SAT_ACT_NONE = 0, SAT_ACT_RELU = 1, SAT_ACT_TANH = 2, SAT_ACT_SIGMOID = 3 };
enum { SAT_OK = 0, SAT_ERR_INVALID = 9001 };

/* Implicit-GEMM convolution geometry (NHWC input, [Cout][KH][KW][C] weights). */
typedef struct {
  int N, H, W, C, KH, KW, stride, pad, OH, OW;
} SatConvGeom;

/* Per-call kernel selection.  Every field 0 = the library's choice (what the product runs); the
 * other values force or exclude one kernel for a single call -- the tests that compare two kernels bit
 * for bit, and A/B measurements.  Passed by pointer (nullable = all defaults) to every entry point that
 * dispatches among kernels: SatGemmArgs.policy, sat_conv2d_nhwc, SatDecoderDims.policy.  There is no
 * process-global tuning state: two callers in one process never see each other's policy. */
typedef struct {
  int conv_pipe;        /* pipelined 256x128 conv / GEMM kernel: 0 auto (long-K, chip-filling problems), 1 off,
                         * 2 every eligible problem */
  int conv_stream;      /* weight-stationary 1x1 kernel (K <= 512): 0 auto, 1 off, 2 every eligible */
  int conv3x3_ws;       /* 64 -> 64 3x3 weight-stationary halo kernel: 0 on, 1 off */
  int conv_slices;      /* layer3 c1 / c2 half-image kernels (sat_conv1x1_frag, sat_conv3x3_frag at 14x14): 0 auto
                         * (two 128-channel slices per half image when B < 64), 1 one workgroup per half image, 2 the
                         * slices; sat_conv3x3_frag at 7x7: 0 auto (two images per workgroup when B > 64), 1 two
                         * images, 2 one image per workgroup */
  int skinny;           /* register-direct skinny GEMM (M <= 128): 0 the decoder's split products, 1 off,
                         * 2 every eligible problem */
  int gemm_stages;      /* LDS ring depth of the bf16 tile kernel: 0 auto, 2, 3 */
  int gemm_tile;        /* tile kernel configuration: 0 auto, 1 = 128x128 / 8 waves, 2 = 128x64 / 8, 3 = 128x128 / 4,
                         * 4 = 128x256 / 8, 5 = 256x128 / 8 (k-major operands use 1 or 3) */
  int gemm_linear_order;/* 1 = plain tile order instead of the XCD-aware one (tile kernel) */
  int gemm_epilogue;    /* bf16-output epilogue of 128-row tiles: 0 bf16 LDS epilogue for every eligible launch,
                         * 1 for residual launches only, 2 fp32 tile staged in LDS */
  int split_gemm;       /* bf16 products with fp32 output and a k-major operand (the decoder's batched weight / input
                         * gradients; gemmsplit.hip: deterministic split-K, no atomics): 0 auto, 1 off (the tile
                         * kernel), 2 128-row tiles only, 3 256-row tiles only */
  int split_k;          /* split_gemm: 0 the planner's split count, n > 0 exactly n splits when the shape allows */
  int attn_bwd;         /* attention backward per decoder step: 0 auto, 1 the two-launch form */
  int attn_bwd_chunks;  /* split attention backward: slot chunks per batch row (0 auto: ~256 workgroups) */
  int attn_pipe;        /* attention forward / split backward over more slots than one batch of loads (L = 196):
                         * 0 auto (slot batches double-buffered), 1 one batch at a time */
  int decoder_splits[4];/* split-K counts of the per-step bf16 decoder GEMMs -- h: [U; f_beta; W_hh] h, c: context
                         * part of the gate GEMM, g: dL/d(gated context), dh: recurrent dL/dh; 0 = automatic; a count
                         * that does not divide K into whole 64-deep k-tiles, or 1 on a K >= 1024 product (it would
                         * take the tile kernel's fp32-atomic split-K), keeps the automatic count */
  int greedy_step;      /* bf16 forward without teacher forcing (decoder.py:118-133 per step): 0 the fused greedy step
                         * (token table for the embedding half of the gate GEMM, dropout in the LSTM kernel, f_z beside
                         * the context GEMM, f_h + combine in one launch, the vocabulary head with in-launch argmax
                         * partials), 1 the per-op form (a GEMM / elementwise launch per reference op) */
  int embed_grad;       /* dense embedding gradient (decoder.py:87,133 nn.Embedding backward): 0 per-token sums in row
                         * order (sorted segments: bit-reproducible), 1 fp32 atomics */
  /* diagnostics (bench.py's in-step kernel timing): a device buffer; when non-null and stamps[0] != 0 (the
   * enable word, read by the kernels at every launch -- so a captured hipGraph can be replayed with stamps
   * on or off), every workgroup w < stamp_capacity of the call's launch writes {first-wave start, last-wave
   * end} of the device's 100 MHz real-time counter to stamps[2 + 2 w], stamps[3 + 2 w]; the launch's span
   * = max(end) - min(start).  The decoder calls lay out kStampGroups x (T-1) such slots of
   * 2 (stamp_capacity + 1) words, one per per-step kernel group and step (decoder.hip). */
  uint64_t* stamps;
  int stamp_capacity;
} SatPolicy;

/* Generic GEMM:  C[m,n] = act(alpha*sum_k A(m,k)B(n,k) + bias[n] + add1[m,n] + beta*C[m,n]),
 * A(m,k) = transA ? A[k*lda+m] : A[m*lda+k];  B(n,k) = transB ? B[k*ldb+n] : B[n*ldb+k].
 * Optional aux output receives the same (post-activation) value in aux_dtype.
 * Replaces torch.nn.Linear forward/backward (e.g. attention.py:15-16,
 * decoder.py:99,125,143-146,151-158).
 * workspace (nullable, device, workspace_bytes >= sat_gemm_workspace_bytes()): lets a product with fp32 output and
 * a k-major operand split K over workgroups with a deterministic in-launch reduction (partial tiles + arrival
 * tickets, zeroed by the call itself); without it such a product runs unsplit.  One workspace serves calls that
 * are ordered on one stream. */
typedef struct {
  int M, N, K, dtype;
  const void* A; int64_t lda; int transA;
  const void* B; int64_t ldb; int transB;
  void* C; int64_t ldc; int c_dtype;
  float alpha, beta;
  const float* bias;
  const void* add1; int64_t ld_add1; int add1_dtype;
  int act;
  void* aux; int64_t ld_aux; int aux_dtype;
  const SatPolicy* policy;    /* nullable: library defaults */
  void* workspace; int64_t workspace_bytes;
} SatGemmArgs;

/* Decoder problem description (decoder.py:9-67 constructor flags + shapes). */
typedef struct {
  int B, L, D, E, V, T;       /* T = caption length; the decoder runs T-1 steps (decoder.py:77) */
  int tf, ado, attention, bert, training;
  int dtype;
  int start_token;            /* 0 = <start> (decoder.py:82); 101 = [CLS] (decoder.py:80) */
  int has_dropout_mask;       /* training: 1 = use the caller's keep-mask, 0 = draw from seed */
  uint64_t seed;
  /* optional device counter: when set, masks are drawn from (seed ^ *seed_ptr) and the forward
   * increments *seed_ptr on the stream, so a hipGraph replay draws fresh masks every step. */
  uint64_t* seed_ptr;
  /* workgroups the per-step split-K GEMMs aim for (0 = the library default, 192): per call, so two
   * decoders in one process can differ and a captured graph keeps the value its workspace was sized with */
  int split_target;
  const SatPolicy* policy;    /* nullable: library defaults (must be the same for a forward and its backward) */
} SatDecoderDims;

/* Element offsets of every decoder parameter inside one flat fp32 buffer.  Keys
 * map to the reference state_dict.  Groups the kernels read as
 * one matrix are adjacent:
 *   init_w = [init_h.weight ; init_c.weight] [2E,D],  init_b = [init_h.bias ; init_c.bias]
 *   hcat_w = [attention.U.weight ; f_beta.weight ; lstm.weight_hh] [E+D+4E, E]
 *   hcat_b = [attention.U.bias ; f_beta.bias ; lstm.bias_hh]. */
typedef struct {
  int64_t embedding, init_w, init_b, hcat_w, hcat_b, attW_w, attW_b, v_w, v_b, wih, bih;
  int64_t fh_w, fh_b, fz_w, fz_b, fout_w, fout_b, do_w, do_b;
  int64_t total;
  /* bf16 mode, optional (-1 = absent): element offsets in params_lp of transposed copies
   *   wih_ctx_t = W_ih[:, E:]^T [D, 4E] and hcat_t = hcat_w^T [E, E+D+4E]
   * (sat_decoder_refresh_transposed writes them from the shadow's own rows after every weight update); the
   * BPTT's dL/d(gated context) and dL/dh products then read k-contiguous weights (the skinny kernel) */
  int64_t wih_ctx_t, hcat_t;
} SatDecoderLayout;

int sat_abi_version(void);
const char* sat_error_string(int code);

/* --- generic building blocks -------------------------------------------- */
int sat_gemm(const SatGemmArgs* args, void* stream);
size_t sat_gemm_workspace_bytes(void);
/* elementwise cast between SAT_F32 and SAT_BF16 storage (n elements). */
int sat_cast(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, void* stream);

/* mean over L: a [B,L,D] -> out_f32 [B,D] (nullable) and out_t [B,D] in dtype (nullable);
 * img_features.mean(dim=1) of decoder.py:139 / the uniform-attention context of decoder.py:104. */
int sat_mean_rows_abi(const void* a, int B, int L, int D, int dtype, float* out_f32, void* out_t, void* stream);

/* --- encoder (encoder.py:33-40 with the torchvision trunks) ------------- */
/* NCHW fp32 image batch -> NHWC (dtype) with channels zero-padded to Cp. */
int sat_nchw_to_nhwc(int N, int C, int H, int W, int Cp, int dtype, const float* x, void* y, void* stream);
/* NCHW fp32 (C <= 4, H and W even) -> space-to-depth NHWC [N, H/2, W/2, 16] (dtype): channel
 * (sy*2 + sx)*C + c holds x[n, c, 2*by + sy, 2*bx + sx], channels 4C..15 zero.  Feeds the ResNet152
 * stem as a 4x4 / stride-1 / top-left-pad-2 conv (encoder.py:13-17 conv1, re-laid out). */
int sat_nchw_to_s2d(int N, int C, int H, int W, int dtype, const float* x, void* y, void* stream);
/* y = act(conv(x, w) + bias [+ residual]); x NHWC [N,H,W,C], y NHWC [N,OH,OW,Cout]; pad is the
 * top/left padding, OH/OW are taken as given (bottom/right padding = whatever they imply);
 * covers Conv2d+ReLU (VGG19) and Conv2d+BatchNorm(eval, folded)+[residual]+ReLU (ResNet152). */
int sat_conv2d_nhwc(const SatConvGeom* g, int Cout, int dtype, const void* x, const void* w,
                    const float* bias, const void* residual, int relu, void* y, const SatPolicy* policy,
                    void* stream);
/* Weight re-layout for register-direct MFMA fragment loads (once per weight version):
 * src [N][K] bf16 row-major -> dst [N/16][K/32][64][8], lane l = 16*(k8 % 4) + (n % 16) of block
 * (n / 16, k / 32) holding src[n][32*(k/32) + 8*(l >> 4) .. +8].  N % 16 == 0, K % 32 == 0. */
int sat_mfma_frag_layout(int N, int K, const void* src, void* dst, void* stream);
/* 1 if sat_bottleneck_fused runs this geometry (today: bf16, 14x14, Cin 1024, Cmid 256 -- the 35
 * identity blocks of ResNet152 layer3), else 0. */
int sat_bottleneck_fused_supported(int H, int W, int Cin, int Cmid, int dtype);
/* One torchvision Bottleneck with identity residual and stride 1, eval-BN folded (encoder.py:13-17,
 * 33-36 through torchvision): y = relu(c3(relu(c2(relu(c1(x))))) + x) in ONE launch; c1/c2 outputs
 * stay on chip.  x, y NHWC [N,H,W,Cin] (x != y); w1f/w2f/w3f: sat_mfma_frag_layout of the folded
 * [Cmid][Cin], [Cmid][3*3*Cmid] (tap-major) and [Cin][Cmid] weights; b1/b2/b3 folded fp32 biases.
 * Bit-identical to the three sat_conv2d_nhwc launches it replaces. */
int sat_bottleneck_fused(int N, int H, int W, int Cin, int Cmid, int dtype, const void* x, const void* w1f,
                         const float* b1, const void* w2f, const float* b2, const void* w3f, const float* b3,
                         void* y, const SatPolicy* policy, void* stream);
/* 1 if sat_conv3x3_frag runs this geometry (bf16: 14x14 C 256, 28x28 C 128, 7x7 C 512 -- the c2 of ResNet152's
 * layer3 / layer2 / layer4 identity blocks -- and VGG19's 14x14 C 512 block-5 and 112x112 C 128 block-2 convs), else 0. */
int sat_conv3x3_frag_supported(int H, int W, int C, int dtype);
/* 3x3 / stride 1 / pad 1 conv C -> C + folded bias + ReLU (a bottleneck's c2, encoder.py:13-17 through
 * torchvision), one workgroup per half image (14x14), 7-row band (28x28) or one / two whole images x a
 * 128-channel slice (7x7) with its input rows staged once in LDS and the weights streamed register-direct.  x, y NHWC [N,H,W,C] (x != y); wf: sat_mfma_frag_layout of the folded
 * [C][3*3*C] (tap-major) weight; b: fp32 bias.  Bit-identical to sat_conv2d_nhwc on the same operands. */
int sat_conv3x3_frag(int N, int H, int W, int C, int dtype, const void* x, const void* wf, const float* b, void* y,
                     const SatPolicy* policy, void* stream);
/* 1 if sat_conv1x1_frag runs this geometry (today: bf16, 14x14, Cin 1024, Cout 256 -- the c1 of ResNet152's
 * layer3 identity blocks), else 0. */
int sat_conv1x1_frag_supported(int H, int W, int Cin, int Cout, int dtype);
/* 1x1 conv Cin -> Cout + folded bias + ReLU (a bottleneck's c1, encoder.py:13-17 through torchvision), one
 * workgroup per half image: input slabs by LDS-DMA, weights register-direct.  x NHWC [N,H,W,Cin], y
 * [N,H,W,Cout] (x != y); wf: sat_mfma_frag_layout of the folded [Cout][Cin] weight.  Bit-identical to
 * sat_conv2d_nhwc. */
int sat_conv1x1_frag(int N, int H, int W, int Cin, int Cout, int dtype, const void* x, const void* wf,
                     const float* b, void* y, const SatPolicy* policy, void* stream);
/* MaxPool2d (floor mode, -inf padding) on NHWC. */
int sat_maxpool2d_nhwc(int N, int H, int W, int C, int k, int stride, int pad, int dtype,
                       const void* x, void* y, int OH, int OW, void* stream);

/* --- attention (attention.py:14-21), standalone module forward ----------- */
/* Ws: workspace [B,L,E] fp32. Weights fp32 (U_w [E,E], W_w [E,D], v_w [E]); W_w_lp (bf16 copy)
 * required when dtype == SAT_BF16. context [B,D] fp32, alpha [B,L] fp32. */
int sat_attention_forward(int B, int L, int D, int E, int dtype, const void* img_features,
                          const float* hidden, const float* U_w, const float* U_b,
                          const float* W_w, const void* W_w_lp, const float* W_b,
                          const float* v_w, const float* v_b, float* ws_scratch,
                          float* context, float* alpha, void* stream);


/* --- decoder (decoder.py:69-158) ----------------------------------------- */
/* diagnostics (bench.py): after sat_decoder_forward + sat_decoder_backward filled `workspace`, re-issue
 * each per-step kernel group of step (T-1)/2 `reps` times back to back between HIP events on `stream`;
 * us_out[8] = average us per launch: h GEMM, attention fwd, context GEMM, LSTM fwd, LSTM bwd, d(gated
 * context) GEMM, attention bwd, dh GEMM (0 for groups the configuration does not run).  Overwrites the
 * workspace's running BPTT sums (call after the gradients are consumed). */
int sat_decoder_step_bench(const SatDecoderDims* dims, const SatDecoderLayout* layout, const float* params,
                           const void* params_lp, const void* img_features, void* workspace, size_t workspace_bytes,
                           float* alphas, const float* d_alphas, int reps, float* us_out, void* stream);
size_t sat_decoder_workspace_bytes(const SatDecoderDims* d);
/* The per-step kernel instance a sat_decoder_forward / _backward with these dims (and policy) runs, for tests
 * and bench reports: out[i] for i < n, in this order (SAT_DECODER_INSTANCE_FIELDS values):
 *   0 h-GEMM split-K slabs, 1 context-GEMM slabs, 2 d(gated context) slabs, 3 dh slabs,
 *   4 attention-backward slot chunks per batch row (1 = one workgroup per row, no last-arriver combine;
 *     0 = the two-launch form or no attention), 5 backward products on the transposed weight copies,
 *   6 launches per forward time step, 7 launches per BPTT time step (teacher forcing). */
enum { SAT_DECODER_INSTANCE_FIELDS = 8 };
int sat_decoder_instance(const SatDecoderDims* d, const SatDecoderLayout* lay, int* out, int n);
/* bf16 mode: rewrite the transposed weight copies layout->wih_ctx_t / hcat_t inside params_lp from the shadow's
 * own W_ih / hcat rows (after the shadow changed: the fused Adam step, a cast); a no-op when either is -1. */
int sat_decoder_refresh_transposed(const SatDecoderDims* d, const SatDecoderLayout* lay, void* params_lp,
                                   void* stream);
/* preds [B,T-1,V] (dtype), alphas [B,T-1,L] fp32, tokens [B,T-1] int32 = token fed at each step. */
int sat_decoder_forward(const SatDecoderDims* d, const SatDecoderLayout* lay, const float* params,
                        const void* params_lp, const void* img_features, const int64_t* captions,
                        const uint8_t* dropout_mask, void* workspace, size_t workspace_bytes,
                        void* preds, float* alphas, int32_t* tokens, void* stream);
/* phase 1 = output-head gradients only (f_out/f_h/f_z/deep_output), 2 = the rest
 * (needs phase 1 first), 3 = both.  accumulate=0 overwrites the active grads. */
int sat_decoder_backward(const SatDecoderDims* d, const SatDecoderLayout* lay, const float* params,
                         const void* params_lp, const void* img_features, void* workspace,
                         size_t workspace_bytes, const void* preds, const float* alphas,
                         const void* d_preds, const float* d_alphas, float* grads, int accumulate,
                         int phase, void* stream);   /* phase 1 | 2 | 3, + 4: d_preds already ReLU-masked (ado),
                                                     + 8: d_preds rows zero-padded to the bf16 head's
                                                     stride (sat_caption_loss_backward_ld; ado needs 4) */

/* --- beam-search captioning (decoder.py:160-269, Decoder.caption; generate_caption.py:86-88) ---
 * img_features: DEVICE [beam_size, L, D] (the reference expands one image to beam rows).
 * Uses d->L, D, E, V, ado, attention, bert, dtype, start_token; d->B, T, tf, training are ignored
 * (caption() applies no dropout).  Runs up to max_step + 1 decoder steps (the reference: 50),
 * synchronising `stream` once per step to retire/compact beams, so it is NOT capturable.
 * Results are written to HOST memory:
 *   out_ids    [max_step + 2]        best completed sentence incl. the start token
 *   out_alphas [(max_step + 2) * L]  its alpha rows (first row = ones, as in decoder.py:173)
 *   out_score                        its summed raw logits; -inf when no beam completed, in which
 *                                    case out_ids = [0] and out_alphas holds the last step's
 *                                    *out_alpha_rows alpha rows (decoder.py:256-258).
 * Requires 1 <= beam_size <= min(64, max_step + 2). */
size_t sat_decoder_beam_workspace_bytes(const SatDecoderDims* d, int beam_size);
int sat_decoder_beam_search(const SatDecoderDims* d, const SatDecoderLayout* lay, const float* params,
                            const void* params_lp, const void* img_features, int beam_size, int max_step,
                            void* workspace, size_t workspace_bytes, int32_t* out_ids, int* out_len,
                            float* out_alphas, int* out_alpha_rows, float* out_score, void* stream);

/* --- loss + metrics (train.py:135-162, utils.py:44-80,101-107) ----------- */
size_t sat_caption_loss_workspace_bytes(int B, int T, int L);
/* out[0]=loss, [1]=CE, [2]=att-reg, [3]=#top1-correct, [4]=#top5-correct, [5]=#non-pad targets,
 * [6]=caption length (tokens not in skip_ids). */
int sat_caption_loss_forward(int B, int T, int V, int L, int dtype, const void* preds,
                             const float* alphas, const int64_t* captions, float alpha_c,
                             int pad_id, int skip0, int skip1, int skip2, void* workspace,
                             float* out, void* stream);
/* the same, the loss (out[0]) also written to loss_out (its own 4-byte buffer: the autograd wrapper hands it out
 * as a tensor a caller may scale in place, without a device copy of out[0]) */
int sat_caption_loss_forward_loss_out(int B, int T, int V, int L, int dtype, const void* preds,
                                      const float* alphas, const int64_t* captions, float alpha_c,
                                      int pad_id, int skip0, int skip1, int skip2, void* workspace,
                                      float* out, float* loss_out, void* stream);
int sat_caption_loss_backward(int B, int T, int V, int L, int dtype, const void* preds,
                              const int64_t* captions, float alpha_c, void* workspace,
                              const float* grad_out, void* d_preds, float* d_alphas, void* stream);
/* the same with the logits a ReLU's output (decoder.py:117-125 advanced deep output): the gradient
 * leaves through that ReLU (zero where preds <= 0), so the decoder backward can skip its mask pass
 * (sat_decoder_backward phase bit 4). */
int sat_caption_loss_backward_relu(int B, int T, int V, int L, int dtype, const void* preds,
                              const int64_t* captions, float alpha_c, void* workspace,
                              const float* grad_out, void* d_preds, float* d_alphas, void* stream);
/* either of the two with d_preds rows ld_dpreds >= V elements apart and columns V..ld_dpreds-1
 * written as zeros (relu_mask != 0: the _relu form).  The bf16 decoder head pads odd vocabularies
 * to a multiple of 8 (16-B rows, e.g. BERT's 30522 -> 30528); a gradient handed over in that
 * layout skips the decoder's copy into padded rows (sat_decoder_backward phase bit 8). */
int sat_caption_loss_backward_ld(int B, int T, int V, int L, int dtype, const void* preds,
                                 const int64_t* captions, float alpha_c, void* workspace,
                                 const float* grad_out, void* d_preds, int64_t ld_dpreds,
                                 float* d_alphas, int relu_mask, void* stream);

/* --- streaming image input (train.py:27-32 transform, dataset.py:9-12 decode on the host) ------
 * Decoded uint8 RGB images of any size, packed HWC (image b at pixels + offsets[b], sizes[b] =
 * {H, W}; offsets / sizes are device arrays) -> Resize((OH, OW)) with Pillow's 8-bit BILINEAR
 * resampler (bit-identical bytes) -> ToTensor -> Normalize(mean, std) (host float[3] each) -> the
 * encoder's input layout.  max_h / max_w bound the sizes (downscale <= sat_images_max_downscale()). */
enum { SAT_IMG_NCHW = 0, SAT_IMG_NHWC = 1, SAT_IMG_S2D16 = 2 };
size_t sat_images_workspace_bytes(int B, int OH, int OW);
int sat_images_max_downscale(void);
int sat_images_to_input(const uint8_t* pixels, const int64_t* offsets, const int32_t* sizes, int B, int max_h,
                        int max_w, int OH, int OW, const float* mean, const float* std, int layout, int c_pad,
                        int dtype, void* out, void* workspace, size_t workspace_bytes, void* stream);

/* --- optimiser (torch.optim.Adam single-tensor step, train.py:71,164) ---- */
int sat_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  void* param_lp, int64_t n, float beta1, float beta2, float eps,
                  float step_size, float bias_correction2_sqrt, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SAT_HIP_H_ */
