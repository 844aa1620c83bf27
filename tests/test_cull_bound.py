"""The blend kernels' tile culling (raster.hip `tile_reach`) is conservative: a Gaussian it drops from
a tile's staged batch has alpha < 1/255 at every pixel centre of the tile, i.e. every pixel would
have skipped it anyway (images and gradients unchanged). Checked on the CPU with a float32 numpy
restatement of the bound against brute-force alphas, on the oracle's own preprocess geometry."""
import math

import numpy as np

from deformgs.synthetic import synth_camera, synth_gaussians
from oracle.raster import OracleRaster, make_settings


def tile_reach(gx, gy, cx, cy, cz, o, x0, y0):
    """float32 restatement of raster.hip tile_reach (bound widened by 1 % + 1e-3)."""
    f = np.float32
    if not (o >= f(1.0 / 255.0)):
        return False
    thr = f(2.0) * np.log(f(255.0) * o) * f(1.01) + f(1e-3)
    dxl, dxh = gx - (x0 + f(15)), gx - x0
    dyl, dyh = gy - (y0 + f(15)), gy - y0
    if dxl <= 0 and dxh >= 0 and dyl <= 0 and dyh >= 0:
        return True

    def Q(dx, dy):
        return cx * dx * dx + f(2) * cy * dx * dy + cz * dy * dy
    q = min(Q(dxl, min(max(-cy * dxl / cz, dyl), dyh)), Q(dxh, min(max(-cy * dxh / cz, dyl), dyh)),
            Q(min(max(-cy * dyl / cx, dxl), dxh), dyl), Q(min(max(-cy * dyh / cx, dxl), dxh), dyh))
    return q <= thr


def test_tile_cull_is_conservative():
    import torch
    N, W, H = 1500, 128, 96
    g = synth_gaussians(N, seed=3, device="cpu")
    cam = synth_camera(W, H, index=1, device="cpu")
    shs = torch.cat([g["features_dc"], g["features_rest"]], 1)
    # wide and narrow footprints, low and high opacities
    sc = torch.exp(g["scaling"] + torch.linspace(-0.5, 1.5, N).unsqueeze(1))
    s = make_settings(H, W, math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), [0, 0, 0], 1.0,
                      cam.world_view_transform.numpy(), cam.full_proj_transform.numpy(), 3, cam.camera_center.numpy())
    o = OracleRaster(s, g["xyz"].numpy(), shs=shs.numpy(), opacities=torch.sigmoid(g["opacity"]).numpy(),
                     scales=sc.numpy(), rotations=torch.nn.functional.normalize(g["rotation"]).numpy())
    geo = o.geometry()
    xy, co = geo["xy"].astype(np.float32), geo["conic_opacity"].astype(np.float32)
    radii = o.radii
    gxn, gyn = (W + 15) // 16, (H + 15) // 16
    px = np.arange(16, dtype=np.float32)
    culled = kept = 0
    for i in np.nonzero(radii > 0)[0]:
        r = int(radii[i])
        x0 = min(gxn, max(0, int((xy[i, 0] - r) / 16))); x1 = min(gxn, max(0, int((xy[i, 0] + r + 15) / 16)))
        y0 = min(gyn, max(0, int((xy[i, 1] - r) / 16))); y1 = min(gyn, max(0, int((xy[i, 1] + r + 15) / 16)))
        cx, cy, cz, op = co[i]
        for ty in range(y0, y1):
            for tx in range(x0, x1):
                tx0, ty0 = np.float32(16 * tx), np.float32(16 * ty)
                if tile_reach(xy[i, 0], xy[i, 1], cx, cy, cz, op, tx0, ty0):
                    kept += 1
                    continue
                culled += 1
                dx = xy[i, 0] - (tx0 + px)[None, :]
                dy = xy[i, 1] - (ty0 + px)[:, None]
                power = np.float32(-0.5) * (cx * dx * dx + cz * dy * dy) - cy * dx * dy
                alpha = np.minimum(np.float32(0.99), op * np.exp(power))
                # every pixel of the tile skips it: power > 0 or alpha < 1/255 (the blend's two skips)
                assert np.all((alpha < np.float32(1.0 / 255.0)) | (power > 0)), (i, tx, ty)
    assert culled > 100 and kept > culled, (culled, kept)
