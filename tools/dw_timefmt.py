#!/usr/bin/env python3
"""Prints the split-arithmetic line of a tools/mlp_time.py log (last JSON line), rounded."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["split"]
print({k: round(v, 3) for k, v in d.items()})
