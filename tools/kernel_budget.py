"""Print the resource remarks of the hot kernels next to tests/test_kernel_budget.py's budget."""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import tests.test_kernel_budget as t  # noqa: E402

k = t.parse_remarks(t.REMARKS.read_text())
names = list(k)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout.splitlines()
res = {d.removeprefix("void "): k[n] for n, d in zip(names, dem)}
for pre, b in sorted(t.BUDGET.items()):
    for d, r in res.items():
        if d.startswith(pre + "("):
            got = (r["VGPRs"], r["ScratchSize [bytes/lane]"], r["Occupancy [waves/SIMD]"], r["VGPRs Spill"])
            bad = got[0] > b[0] or got[1] > b[1] or got[2] < b[2] or got[3] > b[3]
            print(f"{'OVER' if bad else 'ok  '} {pre:48s} vgpr/scratch/waves/spill {got} budget {b}")
