"""One RCCL rank on the one GPU of the box (tests/test_gpu_dist_step.py::test_rccl_group_runs_the_data_parallel_step);
not collected by pytest.

RCCL refuses two ranks on one device, so the 2-rank tests carry their collectives over gloo; this worker
runs the "nccl" backend (= RCCL) itself with a group of ONE rank, so every RCCL-only branch of the
data-parallel step executes on the hardware: init_process_group("nccl", device_id=...), the opt-in CU
reserve (reserve_cus_for_collectives, argv[2] == "reserve"), ReduceOp.AVG in the collective (_avg_op),
the device-side 1-int MIN of agreed_native_path, and the async all-reduces on RCCL's own stream — in
NativeStep.step_data_parallel (waited as stream dependencies under the network backward) and in the
autograd path's OverlappedGradAllReduce (post-accumulate-grad hooks). The reducers shortcut a 1-rank
group, so the step is driven through a reducer that reports two ranks; with AVG done by RCCL over the
real group (one rank) the reduced gradients must equal an un-reduced step's.

argv: out_dir [reserve]. Writes out_dir/rccl.pt.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "deformable-3d-gaussians_amd"), HERE]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_dir = sys.argv[1]
    reserve = len(sys.argv) > 2 and sys.argv[2] == "reserve"
    from dist_step_worker import build, params_of
    from deformgs import _lib
    from deformgs.arguments import PipelineParams
    from deformgs.dist import OverflowAgreement, OverlappedGradAllReduce, _avg_op, reserve_cus_for_collectives
    from deformgs.train_step import optimizer_step, reset_agreement, train_step

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if reserve:
        reserve_cus_for_collectives()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend(), "avg": _avg_op(None) == dist.ReduceOp.AVG,
           "nchannels": os.environ.get("NCCL_MAX_NCHANNELS")}

    # the collectives themselves: AVG / SUM / MAX over one rank leave the values bitwise unchanged
    gen = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(1 << 20, generator=gen).to(dev)
    ops_ok = {}
    for name, op in (("avg", dist.ReduceOp.AVG), ("sum", dist.ReduceOp.SUM), ("max", dist.ReduceOp.MAX)):
        y = x.clone()
        dist.all_reduce(y, op=op)
        ops_ok[name] = bool(torch.equal(x, y))
    y = x.clone()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        work = dist.all_reduce(y, op=dist.ReduceOp.AVG, async_op=True)
    work.wait()
    ops_ok["async"] = bool(torch.equal(x, y))
    res["ops"] = ops_ok

    class TwoRankView(OverlappedGradAllReduce):
        """Takes the multi-rank branches on a 1-rank group (the division is RCCL's AVG over 1)."""

        def world(self):
            return 2

    # count what the step issues (the module functions are looked up at call time)
    from deformgs import native_step
    calls = {"allreduce_async": 0, "allreduce_sync": 0, "dp_steps": 0}
    _ar = dist.all_reduce

    def counted_all_reduce(*a, **k):
        calls["allreduce_async" if k.get("async_op") else "allreduce_sync"] += 1
        return _ar(*a, **k)

    dist.all_reduce = counted_all_reduce
    _dp = native_step.NativeStep.step_data_parallel

    def counted_dp(self, *a, **k):
        calls["dp_steps"] += 1
        return _dp(self, *a, **k)

    native_step.NativeStep.step_data_parallel = counted_dp
    bg = torch.zeros(3, device=dev)
    out = {}
    for path in ("native", "autograd"):
        os.environ["DGS_NATIVE_STEP"] = "1" if path == "native" else "0"
        for reduced in (False, True):
            reset_agreement()
            for k in calls:
                calls[k] = 0
            gs, deform, cams, gts = build(dev)
            ar = TwoRankView(lambda: params_of(gs, deform)[:6], lambda: list(deform.deform.parameters())) \
                if reduced else None
            # learn the pair capacity (synchronous count), then the deferred step that is checked
            train_step(gs, deform, cams[0], gts[0], PipelineParams(), bg, False, deferred_count=False, allreduce=ar)
            gs.optimizer.zero_grad(set_to_none=True)
            deform.optimizer.zero_grad(set_to_none=True)
            loss, _, redone = train_step(gs, deform, cams[0], gts[0], PipelineParams(), bg, False, deferred_count=True,
                                         allreduce=ar, agreement=OverflowAgreement() if reduced else None)
            grads = [p.grad.detach().clone().cpu() for p in params_of(gs, deform)]
            optimizer_step(gs, deform, 3000)
            torch.cuda.synchronize()
            out[(path, reduced)] = {"grads": grads, "loss": float(loss), "redone": bool(redone),
                                    "native": getattr(gs, "_dgs_native", None) is not None, "calls": dict(calls)}
    res["steps"] = {f"{p}-{'rccl' if r else 'local'}": v for (p, r), v in out.items()}
    res["reserved_cus"] = int(_lib.load().dgs_mlp_reserved_cus())
    torch.save(res, os.path.join(out_dir, "rccl.pt"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
