#!/usr/bin/env python3
"""All PMC counters of the timed path-kernel dispatch, merged over tools/pmc.sh passes.

usage: python tools/pmc_dump.py gpurun_out/pmc [kernel-substring]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import dispatch_counters, timed_path_dispatch  # noqa: E402


def main():
    root = Path(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else None
    vals = {}
    for p in sorted(x for x in root.iterdir() if x.is_dir()):
        c = dispatch_counters(p)
        if sub:
            ks = sorted(k for k in c if sub in k[1])
            k = ks[-1] if ks else None
        else:
            k = timed_path_dispatch(c)
        if k is not None:
            vals.update(c[k])
    print(json.dumps(vals, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
