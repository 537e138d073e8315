"""Decoder module (reference: decoder.py:9-269) on the HIP time loop.

Keeps the reference constructor ``Decoder(vocabulary_size, encoder_dim, tf, ado,
bert, attention)``, its attributes (``use_tf``, ``use_advanced_deep_output``,
``use_bert``, ``use_attention``, ``vocabulary_size``, ``embedding_size``,
``encoder_dim``), its submodules and therefore its exact state_dict keys
(SURVEY.md 8b), and ``forward(img_features, captions) -> (preds, alphas)``.

MI355X-specific internals:
  * all parameters are views into ONE flat fp32 buffer laid out so the kernels
    can read fused weights ([U; f_beta; W_hh], [init_h; init_c]) as single
    matrices and DDP can all-reduce the output-head gradients as one bucket
    before the recurrent BPTT even starts;  gradients live in a matching flat
    buffer (``p.grad`` are views), a bf16 shadow of the weights feeds the MFMA
    GEMMs in bf16 mode and is refreshed by the fused Adam kernel;
  * forward/backward are single C-ABI calls (sat_decoder_forward/_backward)
    that run the whole T-1 step loop on the GPU stream.
The dtype of ``img_features`` selects the mode: float32 = exact parity path
(fp32 MFMA), bfloat16 = performance path (bf16 operands, fp32 accumulation,
bf16 ``preds``).
"""
import ctypes
import weakref

import torch
import torch.nn as nn

from . import _lib as L
from .attention import Attention


class BertTokenizerStub:
    """Ids the reference decoder reads from BertTokenizer (decoder.py:80,229,247-250)."""
    cls_token_id = 101
    sep_token_id = 102
    pad_token_id = 0
    unk_token_id = 100

    _SPECIAL = {101: "[CLS]", 102: "[SEP]", 0: "[PAD]", 100: "[UNK]"}

    def convert_ids_to_tokens(self, ids):
        return [self._SPECIAL.get(int(i), f"tok{int(i)}") for i in ids]

    def convert_tokens_to_string(self, tokens):
        return " ".join(tokens)


def _bert_tokenizer():
    """bert-base-uncased special ids.  A tokenizer object resolved from whatever HF cache a
    machine happens to hold is NOT trusted (one GPU host returned cls_token_id=2); pass
    ``tokenizer=`` explicitly to use a real BertTokenizer."""
    return BertTokenizerStub()


class Decoder(nn.Module):
    BERT_VOCAB, BERT_HIDDEN = 30522, 768

    def __init__(self, vocabulary_size, encoder_dim, tf=False, ado=False, bert=False, attention=False,
                 bert_embedding_weight=None, tokenizer=None):
        super().__init__()
        self.use_tf = tf
        self.use_advanced_deep_output = ado
        self.use_bert = bert
        self.use_attention = attention
        self.encoder_dim = encoder_dim
        if bert:  # frozen BERT word-embedding table (decoder.py:21-36)
            self.tokenizer = tokenizer if tokenizer is not None else _bert_tokenizer()
            V = bert_embedding_weight.shape[0] if bert_embedding_weight is not None else self.BERT_VOCAB
            self.vocabulary_size = V
            self.embedding_size = self.BERT_HIDDEN
            self.embedding = nn.Embedding(V, self.BERT_HIDDEN, padding_idx=0)
            if bert_embedding_weight is not None:
                with torch.no_grad():
                    self.embedding.weight.copy_(bert_embedding_weight)
            for p in self.embedding.parameters():
                p.requires_grad = False
        else:
            self.vocabulary_size = vocabulary_size
            self.embedding_size = 512
            self.embedding = nn.Embedding(self.vocabulary_size, self.embedding_size)
        E, D, V = self.embedding_size, encoder_dim, self.vocabulary_size
        self.init_h = nn.Linear(D, E)
        self.init_c = nn.Linear(D, E)
        self.tanh = nn.Tanh()
        self.f_beta = nn.Linear(E, D)
        self.sigmoid = nn.Sigmoid()
        self.attention = Attention(D, E)
        self.lstm = nn.LSTMCell(E + D, E)
        if ado:
            self.f_h = nn.Linear(E, E)
            self.f_z = nn.Linear(D, E)
            self.f_out = nn.Linear(E, V)
            self.relu = nn.ReLU()
            self.dropout = nn.Dropout()
        self.deep_output = nn.Linear(E, V)
        self.dropout = nn.Dropout()
        # --- HIP-side state ---
        self._flat = None
        self._grad_flat = None
        self._flat_lp = None
        self._lp_versions = None
        self._offsets = {}
        self._grad_hooks = []          # callables(phase, decoder): DDP bucket all-reduce
        self.dropout_mask = None       # test hook: uint8 keep-mask [B, T-1, E] used in training mode
        self._seed_host = None
        self._seed_dev = None
        self._defer_phase2 = False     # see defer_recurrent_backward()
        # per-call kernel selection (sat_amd.Policy / SatPolicy; None = the library's defaults): A/B only
        self.policy = None
        # workgroups the per-step split-K GEMMs aim for (SatDecoderDims.split_target; 0 = library
        # default): 64 when the decoder shares the chip with the next batch's encoder (bench / train.py)
        self.split_target = 0
        # bf16: the BPTT's dL/d(gated context) and dL/dh products read transposed weight copies kept behind the
        # shadow (SatDecoderLayout.wih_ctx_t / hcat_t); False = the k-major originals (A/B)
        self.transposed_weights = True
        self._pending_bwd = None
        self.last_tokens = None        # int32 [B, T-1]: token fed at each step of the last forward
        self.record_tokens = True      # False: last_tokens stays None (training loops: no copy launch per step)

    # ------------------------------------------------------------------ layout
    def _groups(self):
        g = []
        if self.use_advanced_deep_output:
            g += [["f_out.weight"], ["f_out.bias"], ["f_h.weight"], ["f_h.bias"], ["f_z.weight"], ["f_z.bias"]]
        g += [["deep_output.weight"], ["deep_output.bias"],
              ["init_h.weight", "init_c.weight"], ["init_h.bias", "init_c.bias"],
              ["attention.U.weight", "f_beta.weight", "lstm.weight_hh"],
              ["attention.U.bias", "f_beta.bias", "lstm.bias_hh"],
              ["attention.W.weight"], ["attention.W.bias"], ["attention.v.weight"], ["attention.v.bias"],
              ["lstm.weight_ih"], ["lstm.bias_ih"], ["embedding.weight"]]
        return g

    def active_param_names(self):
        """Parameters whose .grad the reference's backward produces."""
        names = []
        for n, p in self.named_parameters():
            if not p.requires_grad:
                continue
            if self.use_advanced_deep_output and n.startswith("deep_output."):
                continue
            if not self.use_attention and (n.startswith("attention.") or n.startswith("f_beta.")):
                continue
            names.append(n)
        return names

    def _layout(self):
        o = self._offsets
        lay = L.SatDecoderLayout()
        get = lambda n: o.get(n, -1)  # noqa: E731
        lay.embedding = get("embedding.weight")
        lay.init_w, lay.init_b = get("init_h.weight"), get("init_h.bias")
        lay.hcat_w, lay.hcat_b = get("attention.U.weight"), get("attention.U.bias")
        lay.attW_w, lay.attW_b = get("attention.W.weight"), get("attention.W.bias")
        lay.v_w, lay.v_b = get("attention.v.weight"), get("attention.v.bias")
        lay.wih, lay.bih = get("lstm.weight_ih"), get("lstm.bias_ih")
        lay.fh_w, lay.fh_b = get("f_h.weight"), get("f_h.bias")
        lay.fz_w, lay.fz_b = get("f_z.weight"), get("f_z.bias")
        lay.fout_w, lay.fout_b = get("f_out.weight"), get("f_out.bias")
        lay.do_w, lay.do_b = get("deep_output.weight"), get("deep_output.bias")
        lay.total = self._flat.numel()
        # transposed copies of W_ih[:, E:] and [U; f_beta; W_hh] behind the bf16 shadow (sat_decoder_refresh_transposed)
        lay.wih_ctx_t, lay.hcat_t = self._lp_t_offsets() if self._flat_lp is not None and self.transposed_weights \
            else (-1, -1)
        return lay

    def _lp_t_offsets(self):
        """Element offsets of the transposed weight copies at the tail of the bf16 shadow:
        W_ih[:, E:]^T [D, 4E], then [U; f_beta; W_hh]^T [E, E+D+4E] (the flat size is a multiple of 64)."""
        E, D = self.embedding_size, self.encoder_dim
        base = self._flat.numel()
        return base, base + D * 4 * E

    def _lp_numel(self):
        E, D = self.embedding_size, self.encoder_dim
        return self._flat.numel() + D * 4 * E + E * (5 * E + D)

    def refresh_transposed(self):
        """Rewrite the transposed weight copies from the bf16 shadow (after the shadow changed: a cast, the
        fused Adam step); the BPTT's dL/d(gated context) and dL/dh products read them."""
        if self._flat_lp is None or not self.transposed_weights:
            return
        d = L.SatDecoderDims()
        d.B, d.L, d.D, d.E, d.V, d.T = 1, 1, self.encoder_dim, self.embedding_size, self.vocabulary_size, 3
        d.dtype = L.SAT_BF16
        lay = self._layout()
        L.check(L.lib().sat_decoder_refresh_transposed(ctypes.byref(d), ctypes.byref(lay), L.ptr(self._flat_lp),
                                                        L.stream_of(self._flat_lp)), "sat_decoder_refresh_transposed")

    def _flat_ok(self, device):
        if self._flat is None or self._flat.device != device:
            return False
        base = self._flat.data_ptr()
        for n, p in self.named_parameters():
            if p.data_ptr() != base + 4 * self._offsets[n] or p.dtype != torch.float32:
                return False
        return True

    def _build_flat(self, device):
        params = dict(self.named_parameters())
        off, offsets = 0, {}
        for group in self._groups():
            off = (off + 63) // 64 * 64
            for n in group:
                offsets[n] = off
                off += params[n].numel()
        total = (off + 63) // 64 * 64
        flat = torch.zeros(total, device=device, dtype=torch.float32)
        with torch.no_grad():
            for n, p in params.items():
                view = flat[offsets[n]:offsets[n] + p.numel()].view(p.shape)
                view.copy_(p.data)
                p.data = view
                p._sat_owner = weakref.ref(self)
                p._sat_offset = offsets[n]
        self._flat, self._offsets = flat, offsets
        self._grad_flat = torch.zeros(total, device=device, dtype=torch.float32)
        self._flat_lp = None
        self._lp_versions = None

    def _ensure_flat(self, device):
        if not self._flat_ok(device):
            self._build_flat(device)

    def _ensure_lp(self):
        versions = tuple(p._version for p in self.parameters())
        if self._flat_lp is None:
            self._flat_lp = torch.empty(self._lp_numel(), device=self._flat.device, dtype=torch.bfloat16)
            self._lp_versions = None
        if versions != self._lp_versions:
            from .ops import cast_
            cast_(self._flat, self._flat_lp[:self._flat.numel()])
            self.refresh_transposed()
            self._lp_versions = versions

    def flat_lp_for_optimizer(self):
        """bf16 weight shadow kept in sync by the fused Adam step (None in fp32-only use)."""
        return self._flat_lp

    def _attach_grads(self):
        """Make p.grad views of the flat gradient buffer; return True if they already were."""
        attached = True
        gbase = self._grad_flat
        params = dict(self.named_parameters())
        for n in self.active_param_names():
            p = params[n]
            off = self._offsets[n]
            if p.grad is None or p.grad.data_ptr() != gbase.data_ptr() + 4 * off:
                attached = False
                p.grad = gbase[off:off + p.numel()].view(p.shape)
        return attached

    def grad_bucket(self, phase):
        """Flat gradient range produced by backward phase 1 (output head) or 2 (the rest)."""
        o, params = self._offsets, dict(self.named_parameters())

        def end(n):
            return o[n] + params[n].numel()
        if phase == 1:
            if self.use_advanced_deep_output:
                return self._grad_flat[o["f_out.weight"]:end("f_z.bias")]
            return self._grad_flat[o["deep_output.weight"]:end("deep_output.bias")]
        stop = o["embedding.weight"] if self.use_bert else self._grad_flat.numel()
        return self._grad_flat[o["init_h.weight"]:stop]

    def defer_recurrent_backward(self, on=True):
        """Split the backward in two: autograd's backward then runs only phase 1 (the output head,
        whose gradient bucket is final before BPTT starts) and finish_backward() runs phase 2 (the
        recurrent BPTT + the remaining weight gradients).  Data parallelism launches the head
        bucket's all-reduce in between, so it overlaps BPTT -- also across two captured hipGraphs
        (bench.py), where no Python hook can run between the phases."""
        self._defer_phase2 = bool(on)

    def finish_backward(self):
        """Phase 2 of a backward whose recurrent part was deferred (no-op if none is pending)."""
        if self._pending_bwd is None:
            return
        dims, lay, lp, feats, ws, ws_bytes, preds, alphas, d_preds, d_alphas, accumulate, masked, _pol = \
            self._pending_bwd
        lib = L.lib()
        L.check(lib.sat_decoder_backward(ctypes.byref(dims), ctypes.byref(lay), L.ptr(self._flat), L.ptr(lp),
                                         L.ptr(feats), L.ptr(ws), ws_bytes, L.ptr(preds), L.ptr(alphas),
                                         L.ptr(d_preds), L.ptr(d_alphas), L.ptr(self._grad_flat), int(accumulate),
                                         2 | masked, L.stream_of(preds)),
                "sat_decoder_backward")
        self._pending_bwd = None
        for hook in self._grad_hooks:
            hook(2, self)

    # ----------------------------------------------------------------- forward
    def _dims(self, feats, captions):
        B, Lf, D = feats.shape
        if D != self.encoder_dim:
            raise ValueError(f"img_features last dim {D} != encoder_dim {self.encoder_dim}")
        T = captions.shape[1]   # max_timespan = T - 1 (decoder.py:77)
        d = L.SatDecoderDims()
        d.B, d.L, d.D, d.E, d.V, d.T = B, Lf, D, self.embedding_size, self.vocabulary_size, T
        d.tf, d.ado, d.attention, d.bert = int(self.use_tf), int(self.use_advanced_deep_output), \
            int(self.use_attention), int(self.use_bert)
        d.training = int(self.training)
        d.dtype = L.dtype_code(feats.dtype)
        d.start_token = self.tokenizer.cls_token_id if self.use_bert else 0
        d.has_dropout_mask = int(self.training and self.dropout_mask is not None)
        d.split_target = int(self.split_target)
        # the forward's own copy of the policy: carve() sizes and places the workspace regions from it, so a later
        # (deferred) backward must see exactly the forward's fields even if self.policy is edited in between
        if self.policy is not None:
            d._policy = L.SatPolicy.from_buffer_copy(self.policy)
            d.policy = ctypes.pointer(d._policy)
        # dropout masks: host seed drawn once per module from torch's RNG (train.py:37-43 seeding)
        # XOR a device step counter the forward itself advances -> graph replays draw fresh masks
        if self.training:
            if self._seed_host is None:
                self._seed_host = _rank_seed(int(torch.randint(0, 2 ** 62, (1,)).item()))
            if self._seed_dev is None or self._seed_dev.device != feats.device:
                self._seed_dev = torch.zeros(1, dtype=torch.int64, device=feats.device)
            d.seed = self._seed_host
            d.seed_ptr = self._seed_dev.data_ptr()
        return d

    def forward(self, img_features, captions):
        L.require_device(img_features, captions)
        self._ensure_flat(img_features.device)
        if img_features.dtype == torch.bfloat16:
            self._ensure_lp()
        params = [p for n, p in self.named_parameters()]
        preds, alphas = _DecoderFn.apply(img_features.contiguous(), captions.contiguous().long(), self, *params)
        if self.use_advanced_deep_output:
            # the logits are a ReLU's output: sat_amd.caption_loss folds the ReLU's mask into its
            # backward and tags the gradient, so the decoder's backward skips its own mask pass
            preds._sat_relu_logits = True
        return preds, alphas

    def caption(self, img_features, beam_size, max_step=50):
        """Beam search (decoder.py:160-269) as one C-ABI call (sat_decoder_beam_search).

        ``img_features`` [beam_size, L, D] (one image expanded, generate_caption.py:87).  Returns
        ``(sentence, alpha)``: word ids including the start token and the alpha rows (a list of
        lists, first row all ones) of the best completed beam; like the reference it prints a
        notice and returns ``[0]`` and the last step's alpha rows when no beam completed."""
        import numpy as np
        L.require_device(img_features)
        feats = img_features.contiguous()
        if feats.dim() != 3 or feats.shape[0] != beam_size:
            raise ValueError(f"img_features must be [beam_size={beam_size}, L, D], got {tuple(feats.shape)}")
        self._ensure_flat(feats.device)
        if feats.dtype == torch.bfloat16:
            self._ensure_lp()
        dims = self._dims(feats, torch.empty(1, 3, dtype=torch.long))
        dims.training = 0
        lay = self._layout()
        lib = L.lib()
        ws_bytes = lib.sat_decoder_beam_workspace_bytes(ctypes.byref(dims), int(beam_size))
        if ws_bytes == 0:
            raise RuntimeError("sat_amd.Decoder.caption: unsupported shape / beam size (1..64)")
        ws = torch.empty(ws_bytes, device=feats.device, dtype=torch.uint8)
        cap = max_step + 2
        ids = np.zeros(cap, dtype=np.int32)
        alphas = np.zeros(cap * dims.L, dtype=np.float32)
        n_ids, n_rows, score = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_float(0)
        lp = self._flat_lp if dims.dtype == L.SAT_BF16 else None
        L.check(lib.sat_decoder_beam_search(ctypes.byref(dims), ctypes.byref(lay), L.ptr(self._flat), L.ptr(lp),
                                            L.ptr(feats), int(beam_size), int(max_step), L.ptr(ws), ws_bytes,
                                            ids.ctypes.data, ctypes.byref(n_ids), alphas.ctypes.data,
                                            ctypes.byref(n_rows), ctypes.byref(score), L.stream_of(feats)),
                "sat_decoder_beam_search")
        self.last_caption_score = score.value
        alpha = alphas[:n_rows.value * dims.L].reshape(n_rows.value, dims.L)
        if score.value == float("-inf"):
            print("No completed sentences found")
            return [0], torch.from_numpy(alpha.copy())
        return ids[:n_ids.value].tolist(), alpha.tolist()

    def get_init_lstm_state(self, img_features):
        """decoder.py:137-147 on HIP GEMMs (inference helper)."""
        from .ops import linear
        self._ensure_flat(img_features.device)
        avg = _mean_rows(img_features)
        lp = None
        if avg.dtype == torch.bfloat16:
            self._ensure_lp()
            E, D = self.embedding_size, self.encoder_dim
            o = self._offsets
            lp = (self._flat_lp[o["init_h.weight"]:o["init_h.weight"] + E * D].view(E, D),
                  self._flat_lp[o["init_c.weight"]:o["init_c.weight"] + E * D].view(E, D))
        h = linear(avg, self.init_h.weight.detach(), self.init_h.bias.detach(), act=L.ACT_TANH,
                   weight_lp=lp[0] if lp else None)
        c = linear(avg, self.init_c.weight.detach(), self.init_c.bias.detach(), act=L.ACT_TANH,
                   weight_lp=lp[1] if lp else None)
        return h, c


def _rank_seed(seed):
    """Mix the data-parallel rank into the dropout seed.  Every rank seeds torch identically (identical
    decoder init, train.py:46), so without this rank r's sample i would draw rank 0's sample-i mask;
    the reference draws an independent Bernoulli mask per sample (decoder.py:67,121-125)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        seed = (seed + dist.get_rank() * 0x9E3779B97F4A7C15) % (1 << 64)
    return seed


def _mean_rows(feats):
    """img_features.mean(dim=1) (decoder.py:139) on the HIP path; returns (f32, feats.dtype) copies."""
    B, Lf, D = feats.shape
    feats = feats.contiguous()
    out = torch.empty(B, D, device=feats.device, dtype=torch.float32)
    out_t = torch.empty(B, D, device=feats.device, dtype=feats.dtype)
    L.check(L.lib().sat_mean_rows_abi(L.ptr(feats), B, Lf, D, L.dtype_code(feats.dtype), L.ptr(out), L.ptr(out_t),
                                  L.stream_of(out)), "sat_mean_rows")
    return out_t


class _DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feats, captions, dec, *params):
        lib = L.lib()
        dims = dec._dims(feats, captions)
        lay = dec._layout()
        ws_bytes = lib.sat_decoder_workspace_bytes(ctypes.byref(dims))
        if ws_bytes == 0:
            raise RuntimeError("sat_amd.Decoder: unsupported shape (E, D must be multiples of 8; L, E <= 1024; T >= 3)")
        dev = feats.device
        ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
        B, T1 = dims.B, dims.T - 1
        preds = torch.empty(B, T1, dims.V, device=dev, dtype=feats.dtype)
        alphas = torch.empty(B, T1, dims.L, device=dev, dtype=torch.float32)
        tokens = torch.empty(B, T1, device=dev, dtype=torch.int32) if dec.record_tokens else None
        mask = None
        if dims.has_dropout_mask:
            mask = dec.dropout_mask.to(device=dev, dtype=torch.uint8).contiguous()
            if tuple(mask.shape) != (B, T1, dims.E):
                raise ValueError(f"dropout_mask must be [B, T-1, E] = {(B, T1, dims.E)}")
        lp = dec._flat_lp if dims.dtype == L.SAT_BF16 else None
        L.check(lib.sat_decoder_forward(ctypes.byref(dims), ctypes.byref(lay), L.ptr(dec._flat), L.ptr(lp),
                                        L.ptr(feats), L.ptr(captions), L.ptr(mask), L.ptr(ws), ws_bytes,
                                        L.ptr(preds), L.ptr(alphas), L.ptr(tokens), L.stream_of(preds)),
                "sat_decoder_forward")
        dec.last_tokens = tokens
        ctx.dec, ctx.dims, ctx.lay, ctx.ws, ctx.ws_bytes, ctx.lp = dec, dims, lay, ws, ws_bytes, lp
        ctx.save_for_backward(feats, preds, alphas)
        return preds, alphas

    @staticmethod
    def backward(ctx, d_preds, d_alphas):
        feats, preds, alphas = ctx.saved_tensors
        dec = ctx.dec
        if d_preds is None:
            d_preds = torch.zeros_like(preds)
        if d_alphas is None:
            d_alphas = torch.zeros_like(alphas)
        masked = 4 if getattr(d_preds, "_sat_relu_masked", False) else 0   # phase bit: d_preds already ReLU-masked
        # phase bit 8: caption_loss wrote d_preds into rows zero-padded to the bf16 head's stride (its [..., :V]
        # view), the layout the head's backward GEMMs read: no copy into padded rows
        ld = getattr(d_preds, "_sat_padded_ld", 0)
        V = preds.shape[-1]
        if (ld and d_preds.dtype == torch.bfloat16 and ld == (V + 7) // 8 * 8 and d_preds.shape == preds.shape
                and d_preds.stride() == (preds.shape[1] * ld, ld, 1) and (masked or not dec.use_advanced_deep_output)):
            masked |= 8
        else:
            d_preds = d_preds.contiguous()
        d_alphas = d_alphas.contiguous().float()
        if d_preds.dtype != preds.dtype:
            raise TypeError("sat_amd.Decoder.backward: grad dtype must match preds")
        accumulate = dec._attach_grads()
        lib = L.lib()
        if dec._defer_phase2:
            phases = (1,)
        elif dec._grad_hooks:   # a hook (DDP bucket all-reduce) runs between the phases
            phases = (1, 2)
        else:
            phases = (3,)
        for phase in phases:
            L.check(lib.sat_decoder_backward(ctypes.byref(ctx.dims), ctypes.byref(ctx.lay), L.ptr(dec._flat),
                                             L.ptr(ctx.lp), L.ptr(feats), L.ptr(ctx.ws), ctx.ws_bytes, L.ptr(preds),
                                             L.ptr(alphas), L.ptr(d_preds), L.ptr(d_alphas),
                                             L.ptr(dec._grad_flat), int(accumulate), phase | masked,
                                             L.stream_of(preds)),
                    "sat_decoder_backward")
            for hook in dec._grad_hooks:
                hook(phase, dec)
        if dec._defer_phase2:   # phase 2 runs in dec.finish_backward()
            dec._pending_bwd = (ctx.dims, ctx.lay, ctx.lp, feats, ctx.ws, ctx.ws_bytes, preds, alphas, d_preds,
                                d_alphas, accumulate, masked, dec.policy)
        ctx.ws = None
        n_params = len(ctx.needs_input_grad) - 3
        return (None, None, None) + (None,) * n_params
