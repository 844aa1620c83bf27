"""Dense float64 torch-autograd restatement of the rasterizer (test helper; checks oracle/raster_ref.c).

No tiling loops and no hand-written backward: every pixel evaluates every Gaussian whose tile
rectangle covers the pixel's tile, in (depth, index) order. Discrete decisions (culling, tile
coverage, the power>0 / alpha<1/255 skips and the T<1e-4 stop) are taken from the forward values
and held constant; alpha = min(0.99, o*G) is differentiated as o*G, like the CUDA kernel and the
C oracle. Autograd then gives the gradients the hand-written backward must reproduce.
"""
import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def sh_eval(deg, sh, d):
    """sh: (N, M, 3), d: (N, 3) unit -> (N, 3); utils/sh_utils.py:57-100 basis."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
                 + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
                     + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                     + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                     + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r


def quat_R(q):
    r, x, y, z = q.unbind(-1)
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)


def dense_render(H, W, tanfovx, tanfovy, bg, scale_modifier, viewmatrix, projmatrix, sh_degree, campos,
                 means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                 cov3D_precomp=None):
    dt = means3D.dtype
    V = viewmatrix.to(dt)
    Pm = projmatrix.to(dt)
    N = means3D.shape[0]
    ones = torch.ones(N, 1, dtype=dt)
    ph = torch.cat([means3D, ones], 1)
    pv = ph @ V
    tv = pv[:, :3]
    hom = ph @ Pm
    pw = 1.0 / (hom[:, 3:4] + 1e-7)
    proj = hom[:, :3] * pw
    if cov3D_precomp is None:
        Rm = quat_R(rotations)
        L = Rm * (scale_modifier * scales)[:, None, :]
        Sig = L @ L.transpose(1, 2)
    else:
        c = cov3D_precomp
        Sig = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]], -1).reshape(-1, 3, 3)
    fx = W / (2 * tanfovx)
    fy = H / (2 * tanfovy)
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    tz = tv[:, 2]
    # clamped t: the gradient is zeroed where clamped (CUDA/oracle behaviour), dependency on tz kept
    txtz = tv[:, 0] / tz
    tytz = tv[:, 1] / tz
    mx = ((txtz >= -limx) & (txtz <= limx)).to(dt)
    my = ((tytz >= -limy) & (tytz <= limy)).to(dt)
    tx = mx * tv[:, 0] + (1 - mx) * (txtz.clamp(-limx, limx) * tz).detach()
    ty = my * tv[:, 1] + (1 - my) * (tytz.clamp(-limy, limy) * tz).detach()
    Jm = torch.zeros(N, 2, 3, dtype=dt)
    Jm[:, 0, 0] = fx / tz
    Jm[:, 0, 2] = -(fx * tx) / (tz * tz)
    Jm[:, 1, 1] = fy / tz
    Jm[:, 1, 2] = -(fy * ty) / (tz * tz)
    Wm = V[:3, :3].T
    Tm = Jm @ Wm
    C2 = Tm @ Sig @ Tm.transpose(1, 2)
    a = C2[:, 0, 0] + 0.3
    b = C2[:, 0, 1]
    c = C2[:, 1, 1] + 0.3
    det = a * c - b * b
    conA, conB, conC = c / det, -b / det, a / det
    with torch.no_grad():
        mid = 0.5 * (a + c)
        l1 = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        l2 = mid - torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        rad = torch.ceil(3 * torch.sqrt(torch.maximum(l1, l2)))
    # means2D is a dummy added in NDC units: its .grad is dL/d(ndc), as the CUDA op reports it
    px = ((proj[:, 0] + means2D[:, 0] + 1) * W - 1) * 0.5
    py = ((proj[:, 1] + means2D[:, 1] + 1) * H - 1) * 0.5
    gx, gy = (W + 15) // 16, (H + 15) // 16
    with torch.no_grad():
        rminx = torch.clamp(torch.trunc((px - rad) / 16), 0, gx)
        rminy = torch.clamp(torch.trunc((py - rad) / 16), 0, gy)
        rmaxx = torch.clamp(torch.trunc((px + rad + 15) / 16), 0, gx)
        rmaxy = torch.clamp(torch.trunc((py + rad + 15) / 16), 0, gy)
        vis = (tz > 0.2) & (det != 0) & ((rmaxx - rminx) * (rmaxy - rminy) > 0)
    if colors_precomp is None:
        dvec = means3D - campos.to(dt)[None]
        dn = dvec / dvec.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_eval(sh_degree, shs, dn) + 0.5, 0.0)
    else:
        rgb = colors_precomp
    depth = tz
    # order by (depth as float32, index)
    tzf = tz.detach().float()
    order = sorted([i for i in range(N) if bool(vis[i])], key=lambda i: (float(tzf[i]), i))
    order = torch.tensor(order, dtype=torch.long)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij")
    pxf = xx.reshape(-1, 1)
    pyf = yy.reshape(-1, 1)
    tile_x = (xx.reshape(-1) // 16).long()
    tile_y = (yy.reshape(-1) // 16).long()
    if len(order) == 0:
        img = bg.to(dt)[:, None, None].expand(3, H, W)
        return img, torch.zeros(1, H, W, dtype=dt), rad.int() * vis
    o = order
    dx = px[o][None] - pxf
    dy = py[o][None] - pyf
    power = -0.5 * (conA[o][None] * dx * dx + conC[o][None] * dy * dy) - conB[o][None] * dx * dy
    G = torch.exp(power)
    opac = opacities.reshape(-1)[o][None]
    aoG = opac * G
    alpha = aoG - torch.clamp(aoG - 0.99, min=0).detach()
    with torch.no_grad():
        cover = ((tile_x[:, None] >= rminx[o][None]) & (tile_x[:, None] < rmaxx[o][None])
                 & (tile_y[:, None] >= rminy[o][None]) & (tile_y[:, None] < rmaxy[o][None]))
        use = cover & (power <= 0) & (alpha >= 1.0 / 255.0)
        # termination: walk in order
        a_np = torch.where(use, alpha, torch.zeros_like(alpha))
        keep = torch.zeros_like(use)
        Tcur = torch.ones(a_np.shape[0], dtype=dt)
        alive = torch.ones(a_np.shape[0], dtype=torch.bool)
        for k in range(a_np.shape[1]):
            u = use[:, k] & alive
            testT = Tcur * (1 - a_np[:, k])
            stop = u & (testT < 1e-4)
            alive = alive & ~stop
            u = u & ~stop
            keep[:, k] = u
            Tcur = torch.where(u, testT, Tcur)
    am = torch.where(keep, alpha, torch.zeros_like(alpha))
    Tbefore = torch.cumprod(torch.cat([torch.ones(am.shape[0], 1, dtype=dt), 1 - am], 1), 1)
    Tfinal = Tbefore[:, -1]
    Tb = Tbefore[:, :-1]
    wgt = am * Tb
    col = wgt @ rgb[o] + Tfinal[:, None] * bg.to(dt)[None]
    dep = wgt @ depth[o]
    img = col.T.reshape(3, H, W)
    return img, dep.reshape(1, H, W), (rad * vis).int()
