"""Device f64 pow (ROCm device library, via torch.pow) against glibc pow and the correctly
rounded value (Decimal, 60 digits) on p = n / total inputs, for the temperatures k_act sees."""
import math
from decimal import Decimal, getcontext

import numpy as np
import torch

getcontext().prec = 60


def cr(x, e):
    return float((Decimal(x).ln() * Decimal(e)).exp())


rng = np.random.default_rng(0)
n = rng.integers(1, 800, 20000)
x = n / (n + rng.integers(0, 2200, 20000))
for T in (0.7, 0.3, 1.5, 0.25, 3.0, 0.9):
    e = 1.0 / T
    dev = torch.pow(torch.from_numpy(x).cuda(), e).cpu().numpy()
    lm = np.array([math.pow(v, e) for v in x])
    c = np.array([cr(v, e) for v in x])
    ulp = np.abs(dev.view(np.int64) - c.view(np.int64))
    print(f"T={T}: dev!=libm {np.mean(dev != lm):.5f}  dev!=cr {np.mean(dev != c):.5f} "
          f"(max {ulp.max()} ulp)  libm!=cr {np.mean(lm != c):.5f}", flush=True)
