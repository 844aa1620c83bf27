"""Adam with the update of torch.optim.Adam and one HIP launch per step (dgs_adam_step).

Drop-in for the reference's `torch.optim.Adam(l, lr=0.0, eps=1e-15)` (scene/gaussian_model.py:136,
scene/deform_model.py:332): same param_groups, same per-parameter state ("step", "exp_avg",
"exp_avg_sq"), so the densification code that edits optimizer state (gaussian_model.py:189-251,
upstream scene/gaussian_model.py:165-228) works unchanged. Parameters on the GPU are updated by the
multi-tensor HIP kernel; a CPU-only optimizer (host-side tests of densification) is plain torch Adam.
`step_all(opt_a, opt_b, ...)` updates several optimizers in the same single launch.
"""
import math

import torch

from . import _lib


class Adam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, foreach=False)
        ps = [p for g in self.param_groups for p in g["params"]]
        self._hip = bool(ps) and all(p.is_cuda for p in ps)
        if self._hip and any(g["weight_decay"] != 0.0 for g in self.param_groups):
            raise ValueError("dgs Adam: weight_decay is not supported on the HIP path (the reference's "
                             "Gaussian and deformation optimizers use none)")

    def _collect(self, out):
        """Append (betas, eps, AdamTensor) for every parameter with a gradient; advances 'step'.

        Per-parameter "step" state stays a CPU tensor (torch.optim.Adam's layout), but parameters
        that always step together share ONE step tensor (created for the optimizer's first step), so
        a step costs one tensor update per optimizer instead of one per parameter (each CPU tensor op
        is several microseconds of host time). A parameter without a gradient while its step tensor
        is shared with stepping ones gets its own copy first, so the counts stay exactly torch's."""
        keep = []
        stepping, idle = [], []
        for group in self.param_groups:
            for p in group["params"]:
                (stepping if p.grad is not None else idle).append((group, p))
        if not stepping:
            return keep
        fresh = None
        for group, p in stepping:
            st = self.state[p]
            if len(st) == 0:
                if fresh is None:
                    fresh = torch.tensor(0.0)
                st["step"] = fresh
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        moving = {id(self.state[p]["step"]) for _, p in stepping}
        for _, p in idle:
            st = self.state.get(p)
            if st and id(st["step"]) in moving:
                st["step"] = st["step"].clone()
        counts = {}
        for _, p in stepping:
            t = self.state[p]["step"]
            if id(t) not in counts:
                v = float(t) + 1.0
                t.fill_(v)
                counts[id(t)] = v
        for group, p in stepping:
            b1, b2 = group["betas"]
            lr, eps = float(group["lr"]), float(group["eps"])
            st = self.state[p]
            t = counts[id(st["step"])]
            m, v = st["exp_avg"], st["exp_avg_sq"]
            g = p.grad
            if g.is_sparse:
                raise RuntimeError("dgs Adam does not support sparse gradients")
            if not (p.is_contiguous() and m.is_contiguous() and v.is_contiguous()):
                raise RuntimeError("dgs Adam: parameters and state must be contiguous")
            if not g.is_contiguous():
                g = g.contiguous()
                keep.append(g)
            d = _lib.AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                lr / (1.0 - b1 ** t), math.sqrt(1.0 - b2 ** t))
            out.append(((float(b1), float(b2), eps), d))
        return keep

    @torch.no_grad()
    def step(self, closure=None):
        if not self._hip:
            return super().step(closure)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        step_all(self)
        return loss


@torch.no_grad()
def step_all(*optimizers):
    """One dgs_adam_step launch per distinct (betas, eps) over all HIP optimizers given."""
    lib = _lib.load()
    entries, keep = [], []
    for opt in optimizers:
        if not getattr(opt, "_hip", False):
            opt.step()
            continue
        keep += opt._collect(entries)
    if not entries:
        return
    by_cfg = {}
    for cfg, d in entries:
        by_cfg.setdefault(cfg, []).append(d)
    stream = _lib.stream_ptr()
    for (b1, b2, eps), ds in by_cfg.items():
        arr = (_lib.AdamTensor * len(ds))(*ds)
        _lib.check(lib.dgs_adam_step(len(ds), arr, b1, b2, eps, stream), "adam_step")
    del keep
