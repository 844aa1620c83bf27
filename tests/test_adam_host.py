"""CPU: the dgs Adam keeps torch.optim.Adam's state layout (densification edits it) and, for host
tensors, is torch's own update."""
import torch

from deformgs.adam import Adam, step_all


def test_cpu_optimizer_is_torch_adam():
    p = torch.nn.Parameter(torch.randn(10, 3))
    q = torch.nn.Parameter(p.detach().clone())
    o = Adam([{"params": [p], "lr": 0.01, "name": "xyz"}], lr=0.0, eps=1e-15)
    r = torch.optim.Adam([{"params": [q], "lr": 0.01, "name": "xyz"}], lr=0.0, eps=1e-15)
    assert not o._hip
    for _ in range(3):
        g = torch.randn(10, 3)
        p.grad, q.grad = g.clone(), g.clone()
        step_all(o)
        r.step()
    torch.testing.assert_close(p.detach(), q.detach())
    st = o.state[p]
    assert set(st) >= {"step", "exp_avg", "exp_avg_sq"}
    assert o.param_groups[0]["name"] == "xyz"


def test_weight_decay_rejected_only_on_gpu_params():
    p = torch.nn.Parameter(torch.randn(3))
    Adam([p], lr=0.1, weight_decay=0.1)  # host params: torch semantics, allowed
