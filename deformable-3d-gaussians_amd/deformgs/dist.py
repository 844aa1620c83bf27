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
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


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
