"""Adam on the HIP path (reference optimiser: train.py:71-72,100,164).

``Adam(params, lr, betas, eps)`` is a torch.optim.Optimizer (so
``torch.optim.lr_scheduler.StepLR`` drives it exactly as in the reference) whose
step runs ``sat_adam_step``: torch's single-tensor Adam arithmetic
(``exp_avg.lerp_``, ``exp_avg_sq.mul_().addcmul_()``, ``addcdiv_`` with the
bias corrections), fused, one launch per contiguous range of a decoder's flat
parameter buffer, also refreshing the decoder's bf16 weight shadow.  Params
whose grad is None are skipped and keep no state, as in torch.
"""
import math

import torch

from . import ops


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        if weight_decay != 0:
            raise ValueError("sat_amd.optim.Adam: weight_decay is not used by the reference (train.py:71)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self._flat_state = {}   # id(owner flat) -> (exp_avg flat, exp_avg_sq flat)

    def _owner(self, p):
        ref = getattr(p, "_sat_owner", None)
        owner = ref() if ref is not None else None
        if owner is None or owner._flat is None:
            return None
        if p.data_ptr() != owner._flat.data_ptr() + 4 * p._sat_offset:
            return None
        return owner

    def _state_for(self, p, owner):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0)
            if owner is not None:
                key = id(owner._flat)
                if key not in self._flat_state:
                    self._flat_state[key] = (torch.zeros_like(owner._flat), torch.zeros_like(owner._flat))
                m, v = self._flat_state[key]
                o = p._sat_offset
                st["exp_avg"] = m[o:o + p.numel()].view(p.shape)
                st["exp_avg_sq"] = v[o:o + p.numel()].view(p.shape)
            else:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps = group["lr"], group["betas"], group["eps"]
            items = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or not p.is_contiguous():
                    raise TypeError("sat_amd.optim.Adam: fp32 contiguous parameters only")
                owner = self._owner(p)
                st = self._state_for(p, owner)
                st["step"] += 1
                items.append((p, owner, st))
            # merge runs of params that are adjacent in one flat buffer (same step count); a run also spans the
            # alignment padding between two parameter groups (< 64 floats holding no parameter: zero value,
            # gradient and moments, which the update leaves at zero), so one launch covers a whole flat buffer
            runs = []
            for p, owner, st in sorted(items, key=lambda it: (id(it[1]), it[0].data_ptr())):
                step = int(st["step"].item())
                gap = (p.data_ptr() - runs[-1]["end_ptr"]) // 4 if runs else -1
                padding_only = (runs and owner is not None and runs[-1]["owner"] is owner and 0 < gap < 64
                                and not any(runs[-1]["end_off"] <= o < p._sat_offset for o in owner._offsets.values()))
                contiguous_with_prev = (runs and owner is not None and runs[-1]["owner"] is owner
                                        and runs[-1]["step"] == step
                                        and (gap == 0 or padding_only)
                                        and runs[-1]["gend"] + 4 * gap == p.grad.data_ptr()
                                        and runs[-1]["mend"] + 4 * gap == st["exp_avg"].data_ptr())
                if contiguous_with_prev:
                    r = runs[-1]
                    r["n"] += gap + p.numel()
                else:
                    runs.append(dict(owner=owner, step=step, p=p, st=st, n=p.numel()))
                    r = runs[-1]
                r["end_ptr"] = p.data_ptr() + 4 * p.numel()
                r["end_off"] = (p._sat_offset + p.numel()) if owner is not None else 0
                r["gend"] = p.grad.data_ptr() + 4 * p.numel()
                r["mend"] = st["exp_avg"].data_ptr() + 4 * p.numel()
            for r in runs:
                p, st, n, owner = r["p"], r["st"], r["n"], r["owner"]
                bc1 = 1 - b1 ** r["step"]
                bc2 = 1 - b2 ** r["step"]
                off = p._sat_offset if owner is not None else 0
                lp = None
                if owner is not None and owner._flat_lp is not None:
                    lp = owner._flat_lp[off:off + n]
                    owner._lp_versions = None if lp is None else owner._lp_versions
                if owner is not None:
                    pv = owner._flat[off:off + n]
                    gv = owner._grad_flat[off:off + n]
                    m, v = self._flat_state[id(owner._flat)]
                    mv, vv = m[off:off + n], v[off:off + n]
                else:
                    pv, gv, mv, vv = p.view(-1), p.grad.view(-1), st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1)
                ops.adam_step_(pv, gv, mv, vv, lp, b1, b2, eps, lr / bc1, math.sqrt(bc2))
            refreshed = set()
            for p, owner, st in items:
                if owner is not None and owner._flat_lp is not None:
                    owner._lp_versions = tuple(q._version for q in owner.parameters())
                    if id(owner) not in refreshed:   # the transposed copies follow the updated shadow
                        refreshed.add(id(owner))
                        owner.refresh_transposed()
        return loss
