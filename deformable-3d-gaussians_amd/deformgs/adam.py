"""Adam with the update of torch.optim.Adam and one HIP launch per step (dgs_adam_step).

Drop-in for the reference's `torch.optim.Adam(l, lr=0.0, eps=1e-15)` (scene/gaussian_model.py:136,
scene/deform_model.py:332): same param_groups, same per-parameter state ("step", "exp_avg",
"exp_avg_sq"), so the densification code that edits optimizer state (gaussian_model.py:189-251,
upstream scene/gaussian_model.py:165-228) works unchanged. Parameters on the GPU are updated by the
multi-tensor HIP kernel; a CPU-only optimizer (host-side tests of densification) is plain torch Adam.
`step_all(opt_a, opt_b, ...)` updates several optimizers in the same single launch.
"""
import math
import weakref

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


# step_all's launch tables for a fixed set of (parameter, gradient) buffers: a training step with the
# native step (deformgs/native_step.py) keeps the same gradient buffers every iteration, so after the
# first step only the step counts and the per-tensor bias corrections change (~40 us of host time
# instead of ~200 us of per-parameter Python). The cache lives on the first optimizer of the set
# (`_dgs_fast`) and refers to the others weakly, so it never keeps parameters or Adam moments alive
# after training; `clear_fast_cache` drops it explicitly.


def _fast_get(hip, key):
    fast = getattr(hip[0], "_dgs_fast", None)
    if fast is None or fast["key"] != key or any(r() is not o for r, o in zip(fast["refs"], hip)):
        return None
    return fast


def clear_fast_cache(*optimizers):
    for o in optimizers:
        if hasattr(o, "_dgs_fast"):
            o._dgs_fast = None


def _signature(optimizers):
    sig = []
    for opt in optimizers:
        for group in opt.param_groups:
            for p in group["params"]:
                g, st = p.grad, opt.state.get(p)
                m = st.get("exp_avg") if st else None
                v = st.get("exp_avg_sq") if st else None
                sig.append((p.data_ptr(), p.numel(), None if g is None else g.data_ptr(),
                            None if m is None else m.data_ptr(), None if v is None else v.data_ptr()))
    return tuple(sig)


@torch.no_grad()
def step_all(*optimizers):
    """One dgs_adam_step launch per distinct (betas, eps) over all HIP optimizers given."""
    lib = _lib.load()
    hip = [opt for opt in optimizers if getattr(opt, "_hip", False)]
    for opt in optimizers:
        if not getattr(opt, "_hip", False):
            opt.step()
    if not hip:
        return
    key = tuple(id(o) for o in hip)
    sig = _signature(hip)
    fast = _fast_get(hip, key)
    stream = _lib.stream_ptr()
    if fast is not None and fast["sig"] == sig and all(float(t) == c for t, c in fast["steps"]):
        counts = {}
        for t, c in fast["steps"]:
            t.fill_(c + 1.0)
            counts[id(t)] = c + 1.0
        fast["steps"] = [(t, counts[id(t)]) for t, _ in fast["steps"]]
        for arr, ents in fast["tables"]:
            for i, (group, st) in enumerate(ents):
                b1, b2 = group["betas"]
                t = counts[id(st)]
                arr[i].step_size = float(group["lr"]) / (1.0 - b1 ** t)
                arr[i].bc2_sqrt = math.sqrt(1.0 - b2 ** t)
        for (b1, b2, eps), arr in fast["launch"]:
            _lib.check(lib.dgs_adam_step(len(arr), arr, b1, b2, eps, stream), "adam_step")
        return
    entries, keep = [], []
    for opt in hip:
        keep += opt._collect(entries)
    if not entries:
        return
    by_cfg = {}
    for cfg, d in entries:
        by_cfg.setdefault(cfg, []).append(d)
    launch = []
    for (b1, b2, eps), ds in by_cfg.items():
        arr = (_lib.AdamTensor * len(ds))(*ds)
        launch.append(((b1, b2, eps), arr))
        _lib.check(lib.dgs_adam_step(len(ds), arr, b1, b2, eps, stream), "adam_step")
    clear_fast_cache(*hip)
    if not keep and all(p.grad is not None for o in hip for g in o.param_groups for p in g["params"]):
        # cacheable: every parameter stepped with its own contiguous gradient; the tables follow the
        # entry order of _collect (group by group, parameter by parameter)
        ents, steps = [], {}
        for o in hip:
            for group in o.param_groups:
                for p in group["params"]:
                    st = o.state[p]["step"]
                    ents.append((group, st))
                    steps[id(st)] = st
        cfg_of = [cfg for cfg, _ in entries]
        tables, k = [], 0
        pos = {cfg: [] for cfg in by_cfg}
        for i, cfg in enumerate(cfg_of):
            pos[cfg].append(ents[i])
        for (cfg, arr) in launch:
            tables.append((arr, pos[cfg]))
        hip[0]._dgs_fast = {"key": key, "sig": _signature(hip), "steps": [(t, float(t)) for t in steps.values()],
                            "tables": tables, "launch": launch, "refs": [weakref.ref(o) for o in hip]}
    del keep
