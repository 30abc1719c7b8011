"""Compare two statistics dumps of tools/ab_zipf.py (AB_DUMP): NUM/MIN/MAX/MED must be
bit-identical, AVG/STD identical or within the FAST bars (2.5e-7 / 1e-6 relative)."""
import sys

import torch

a, b, name = torch.load(sys.argv[1]), torch.load(sys.argv[2]), sys.argv[3]
bad = [f for f in ("num", "min", "max", "med") if not torch.equal(a[f].view(torch.int32), b[f].view(torch.int32))]
for f, tol in (("avg", 2.5e-7), ("std", 1e-6)):
    x, y = a[f].double(), b[f].double()
    if not torch.all((x == y) | ((x - y).abs() <= tol * x.abs()) | (x.isnan() & y.isnan())):
        bad.append(f)
print(f"compare {name}: {'identical' if not bad else 'DIFFER in ' + ','.join(bad)}")
