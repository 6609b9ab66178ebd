#!/usr/bin/env python3
"""Counters of the timed path-kernel dispatch from rocprofv3 --pmc pass directories (one JSON line).

usage: python tools/pmc_dispatch.py LABEL PASS_DIR [PASS_DIR ...]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import dispatch_counters, timed_path_dispatch  # noqa: E402

vals, kernel = {}, None
for p in sys.argv[2:]:
    p = Path(p)
    if not p.is_dir():
        continue
    c = dispatch_counters(p)
    k = timed_path_dispatch(c)
    if k is not None:
        kernel = k[1]
        vals.update(c[k])
if "WRITE_SIZE" in vals:
    vals["write_bytes"] = vals["WRITE_SIZE"] * 1024.0
if "FETCH_SIZE" in vals:
    vals["fetch_bytes_x2"] = vals["FETCH_SIZE"] * 2048.0
print(json.dumps({"label": sys.argv[1], "kernel": kernel, **vals}))
