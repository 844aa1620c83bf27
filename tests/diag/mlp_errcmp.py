import sys, numpy as np, torch
sys.path[:0] = ["tests", "tests/golden", "deformable-3d-gaussians_amd", "."]
from oracle import mlp_ref
from test_gpu_mlp import _net, VARIANTS
for name, N, mode in [("nonblender", 4099, "uniform"), ("blender", 20000, "uniform"), ("nonblender", 20000, "random")]:
    bl, d6, fork = VARIANTS[name]
    rng = np.random.default_rng(N)
    x = rng.uniform(-1.3, 1.3, (N, 3)).astype(np.float32)
    t = np.full((N, 1), 0.37, np.float32) if mode == "uniform" else rng.uniform(0, 1, (N, 1)).astype(np.float32)
    g = None
    for exact in (False, True):
        net, w = _net(name, 77, exact)
        out, c = mlp_ref.forward(w, x, t, bl, d6)
        if g is None:
            g = {k: rng.standard_normal(out[k].shape) for k in ("d_xyz", "d_rot", "d_scale")}
            gr = mlp_ref.backward(w, c, out, g, bl, d6)
        res = net(torch.from_numpy(x).cuda(), torch.from_numpy(t).cuda())
        fe = max(np.abs(v.detach().cpu().numpy() - out[k]).max() / np.abs(out[k]).max() for k, v in zip(("d_xyz", "d_rot", "d_scale"), res))
        sum((v * torch.from_numpy(g[k]).float().cuda()).sum() for k, v in zip(("d_xyz", "d_rot", "d_scale"), res)).backward()
        worst = sorted(((np.abs(p.grad.cpu().numpy() - gr[k]).max() / np.abs(gr[k]).max(), k) for k, p in net.named_parameters()), reverse=True)[:4]
        print(name, N, mode, "exact" if exact else "split", "fwd rel %.2e" % fe, " ".join("%s %.2e" % (k, e) for e, k in worst), flush=True)
