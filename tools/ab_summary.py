#!/usr/bin/env python3
"""Condense tools/ab_libs.sh / tools/env_ab.sh output: variant, iters/s and the named kernel classes.
usage: ab_summary.py <file> [class,class,...]"""
import re
import sys

keys = (sys.argv[2] if len(sys.argv) > 2 else "blend_fwd,blend_bwd,tile_sort,adam").split(",")
for line in open(sys.argv[1]):
    m = re.match(r"(\w+) ([\d.]+) (?:([\d.]+) )?\{(.*)\}", line.strip())
    if not m:
        print(line.rstrip()[:150])
        continue
    d = dict(re.findall(r"'(\w+)': ([\d.]+)", m.group(4)))
    mlp = sum(float(d.get(k, 0)) for k in ("mlp_fwd", "mlp_bwd", "mlp_dw"))
    print(m.group(1), m.group(2), " ".join(f"{k} {d.get(k)}" for k in keys), "mlp", round(mlp, 4))
