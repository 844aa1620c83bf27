"""Row selection of many (N, ...) tensors by one boolean mask in one HIP launch (dgs_select_rows):
the stream compaction of densification (prune / clone / split). CPU tensors (host-side tests) use
torch indexing; CUDA tensors always go through the HIP kernel (no torch fallback)."""
import torch

from . import _lib


def select_rows(mask, tensors):
    """[t[mask] for t in tensors] for float32 tensors whose first dimension is len(mask)."""
    n = mask.shape[0]
    if not mask.is_cuda:
        return [t[mask] for t in tensors]
    m = mask.contiguous().to(torch.uint8)
    k = int(m.sum().item())  # one host sync for every output size (torch syncs once per tensor)
    outs, jobs, keep = [], [], []
    for t in tensors:
        if t.shape[0] != n or t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError("select_rows: float32 CUDA tensors with len(mask) rows expected")
        src = t.contiguous()
        keep.append(src)
        out = torch.empty((k,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        outs.append(out)
        width = src[0].numel() if n else 1
        if k and width:
            jobs.append(_lib.RowJob(src.data_ptr(), out.data_ptr(), width))
    if jobs:
        lib = _lib.load()
        arr = (_lib.RowJob * len(jobs))(*jobs)
        _lib.check(lib.dgs_select_rows(n, m.data_ptr(), len(jobs), arr, torch.cuda.current_stream(m.device).cuda_stream),
                   "dgs_select_rows")
    return outs
