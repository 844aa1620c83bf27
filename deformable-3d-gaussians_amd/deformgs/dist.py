"""Frame-parallel data parallelism: one process per GPU, each renders its own
camera/timestep, then ONE averaged all-reduce of all gradients (Gaussian params + MLP params,
~25.7 MB fp32 at 100k) over RCCL/xGMI ("nccl" backend = RCCL on ROCm); densification statistics are
summed/maxed across ranks before densify, and densify randomness comes from a rank-identical
generator so replicas never diverge. The reference is single-GPU (utils/general_utils.py:188).
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """torchrun-style env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*). Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of N ranks on fewer GPUs (tests / a one-GPU box): DGS_DEVICE pins every rank's device,
    # DGS_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU)
    local = int(os.environ.get("DGS_DEVICE", local))
    backend = backend or os.environ.get("DGS_DIST_BACKEND") or None
    from .train_step import reset_agreement
    reset_agreement()  # a new group re-agrees on the native-vs-autograd path (train_step)
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            if os.environ.get("DGS_OVERLAP_RESERVE", "0") == "1":
                reserve_cus_for_collectives()
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


# CUs the network's persistent MLP kernels leave to the gradient all-reduce, and the RCCL channel cap
# that keeps the collective's workgroups within them (one workgroup per channel). The MLP kernels take
# a CU's whole register file, so a collective workgroup and an MLP workgroup never share a CU: on one
# MI355X, a stand-in collective (24 MB read-modify-write sweeps) enqueued where the Gaussian-gradient
# all-reduce goes cost the step +0.15-0.35 ms with no CUs reserved (k_dws's static plan waited for the
# CUs it held) and +0.01-0.03 ms with 16 or 32 reserved for 16 or 32 stand-in workgroups, while the
# reserve itself cost the step 0-2.5 % (tools/overlap_probe.py --sweep --wide,
# profiles/r5c_overlap_sweep.jsonl; the collective queued after the network backward instead: +0.08-0.2
# ms). RCCL itself cannot run on a one-GPU box, so its real workgroup count and its bandwidth under the
# channel cap are unmeasured: the reserve is OPT-IN (DGS_OVERLAP_RESERVE=1) until an 8-GPU run measures
# it, so the default data-parallel step uses every CU and RCCL's own channel count.
OVERLAP_CUS = 32


def reserve_cus_for_collectives():
    """Before an RCCL process group is created (several ranks): cap RCCL's channels at OVERLAP_CUS
    (unless NCCL_MAX_NCHANNELS is set) and make the MLP kernels leave that many CUs free (unless
    DGS_MLP_RESERVE_CUS is set)."""
    os.environ.setdefault("NCCL_MAX_NCHANNELS", str(OVERLAP_CUS))
    if "DGS_MLP_RESERVE_CUS" not in os.environ:
        from . import _lib
        _lib.load().dgs_mlp_set_reserved_cus(min(64, int(os.environ["NCCL_MAX_NCHANNELS"])))


class GradAllReduce:
    """Averages .grad of a fixed parameter list across ranks with bucketed flat all-reduces.

    Buckets are sized for xGMI point-to-point links: few, large messages (default 32 MB, i.e. the
    whole 100k-Gaussian step in one call). Parameters whose .grad is None contribute zeros so every
    rank issues identical collectives.
    """

    def __init__(self, params_fn, bucket_bytes=32 << 20, group=None):
        self.params_fn = params_fn
        self.bucket_bytes = bucket_bytes
        self.group = group

    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def __call__(self):
        W = self.world()
        if W == 1:
            return
        params = [p for p in self.params_fn() if p.requires_grad]
        buckets, cur, size = [], [], 0
        for p in params:
            nb = p.numel() * 4
            if cur and size + nb > self.bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            buckets.append(cur)
        for b in buckets:
            flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in b])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            flat.div_(W)
            off = 0
            for p in b:
                n = p.numel()
                g = flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n


def _avg_op(group):
    """RCCL averages in the collective itself; gloo has no AVG (SUM, then a division)."""
    return dist.ReduceOp.AVG if dist.get_backend(group) == "nccl" else dist.ReduceOp.SUM


class OverlappedGradAllReduce:
    """The step's gradient all-reduce split in two and overlapped with the backward.

    `early_fn()` lists the parameters whose gradients are final well before the backward ends (the
    Gaussian tensors: their gradients come out of the rasterizer / render-input backward, ahead of
    the deformation MLP's backward and dW, about 1 ms of MFMA work at 100k). A post-accumulate-grad
    hook on each of them notices when the last one has been accumulated and starts ONE async
    all-reduce of their flattened gradients (23.6 MB at 100k) right then, on the collective stream,
    while the compute stream runs the MLP backward. `__call__()` (after loss.backward()) reduces the
    late parameters (the MLP: 2.1 MB), waits for the early collective and hands every parameter a
    .grad that is a view into the reduced flat buffers (no copy back). Collectives are issued in the
    same order on every rank (early, then late): a rank on which some early gradient stayed None (its
    hook never completes the group) reduces the early group in `__call__` before the late one, with
    zeros for the missing gradients, so every rank still issues early then late at the same sizes.
    """

    def __init__(self, early_fn, late_fn, group=None):
        self.early_fn, self.late_fn, self.group = early_fn, late_fn, group
        self._early = []
        self._ready = 0
        self._pending = None
        self._armed = False

    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def arm(self):
        """Call before loss.backward() each step."""
        if self.world() == 1:
            return
        self._early = [p for p in self.early_fn() if p.requires_grad]
        for p in self._early:
            if getattr(p, "_dgs_overlap_hook", None) is not self:  # once per (parameter, reducer)
                p.register_post_accumulate_grad_hook(self._hook)
                p._dgs_overlap_hook = self
        self._members = {id(p) for p in self._early}  # (the list keeps them alive for the step)
        self._ready, self._pending, self._armed = 0, None, True

    def _hook(self, p):
        if not self._armed or self._pending is not None or id(p) not in self._members:
            return
        self._ready += 1
        if self._ready == len(self._early):
            flat = torch.cat([q.grad.reshape(-1) for q in self._early])
            self._pending = (flat, dist.all_reduce(flat, op=_avg_op(self.group), group=self.group, async_op=True))

    def _reduce(self, params, flat=None, work=None):
        if flat is None:
            flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params])
            dist.all_reduce(flat, op=_avg_op(self.group), group=self.group)
        else:
            work.wait()
        if _avg_op(self.group) == dist.ReduceOp.SUM:
            flat.div_(self.world())
        off = 0
        for p in params:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p)
            off += n

    def discard(self):
        """Drop this step's reduction (the step is being redone). Every rank must have issued exactly
        one early collective for the discarded backward before the redo issues its own: the early
        collective this rank started is waited for and ignored; a rank whose hook never fired (some
        early gradient stayed None) issues the same throwaway early reduction __call__ would, so it
        pairs with the ranks whose hook did fire. Call arm() again before the redone backward."""
        if self.world() > 1 and self._armed:
            if self._pending is not None:
                self._pending[1].wait()
            else:
                self._reduce(self._early)
        self._pending, self._armed = None, False

    def __call__(self):
        """Call after loss.backward(): late group, then the early group's (overlapped) result."""
        if self.world() == 1:
            return
        self._armed = False
        early = self._early
        pending = self._pending
        late = [p for p in self.late_fn() if p.requires_grad]
        # a late group without any gradient (the network in the warm-up iterations, the same on every
        # rank) is not reduced: its parameters keep .grad None, so Adam skips them as on one rank
        if all(p.grad is None for p in late):
            late = []
        if pending is None:  # the hook did not fire on this rank: reduce the early group here
            self._reduce(early)
            if late:
                self._reduce(late)
        else:
            if late:
                self._reduce(late)
            self._reduce(early, *pending)
        self._pending = None


class OverflowAgreement:
    """Rank agreement on redoing a step whose deferred pair count overflowed its speculative capacity
    (deformgs/train_step.py deferred_count): a 1-int MAX all-reduce over a gloo (host) group, so it
    neither waits behind the gradient collectives on the RCCL stream nor touches the GPU. Every rank
    calls it once per deferred step, after its own count is resolved; all redo or none does, so the
    gradient collectives of the redone step still line up."""

    def __init__(self, group=None):
        self.group = group
        self._gloo = None

    def __call__(self, local_overflow):
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return bool(local_overflow)
        if self._gloo is None:
            if os.environ.get("DGS_AGREE_BACKEND", "gloo") != "gloo":
                self._gloo = False  # the device flag on the main group (the same env on every rank)
            else:
                # a host group of its own, also when the main group is gloo: the flag then never
                # interleaves with the gradient collectives (a rank whose early collective started
                # and one whose did not still agree). new_group is collective: a rank that cannot
                # create it fails here (no silent fallback to the main group, which would leave the
                # ranks' 1-int all-reduces on different groups and deadlock the first deferred step)
                try:
                    self._gloo = dist.new_group(backend="gloo")
                except Exception as e:
                    raise RuntimeError("OverflowAgreement: could not create the gloo host group on this rank; "
                                       "set DGS_AGREE_BACKEND=default on every rank to agree over the main "
                                       "group instead") from e
        if self._gloo is False:  # a device flag on the main group (queues behind its collectives)
            dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
            flag = torch.tensor([1 if local_overflow else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            return bool(flag.item())
        flag = torch.tensor([1 if local_overflow else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self._gloo)
        return bool(flag.item())


def sync_densification_stats(gaussians, group=None):
    """SUM xyz_gradient_accum / denom, MAX max_radii2D across ranks (before densify_and_prune)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.all_reduce(gaussians.xyz_gradient_accum, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(gaussians.denom, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(gaussians.max_radii2D, op=dist.ReduceOp.MAX, group=group)


def rank_identical_generator(device, seed=1234):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g
