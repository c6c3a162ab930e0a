"""Test helper: the product leaf evaluator (rvz.LeafEvaluator, h2) or one of the A/B /
cross-check alternatives of tools/alt (AltEvaluator: exact f32 MFMA "resnet", 3-part bf16
"split", PyTorch "miopen"), by name."""
import numpy as np
import torch

import rvz
from alt_eval import AltEvaluator


def make_evaluator(net, kernel="h2", **kw):
    if kernel in ("h2", "auto"):
        kw.pop("fused_epilogue", None)
        return rvz.LeafEvaluator(net, kernel=kernel, **kw)
    return AltEvaluator(net, kernel=kernel, **kw)


class TableEvaluator:
    """A deterministic leaf evaluator with exact fp32 arithmetic on both sides (GPU torch here,
    NumPy in the restatement): priors ((5 i + own discs) mod 8 + 1) / 16, pass 1/32, value
    (own - opponent discs) / 64 — dyadic rationals, so the GPU and CPU searches see identical
    NN outputs and any difference is the caller's (arena, self-play)."""
    outputs_probs = True

    def __call__(self, x):
        own = x[:, 0].reshape(x.shape[0], -1).sum(1)
        opp = x[:, 1].reshape(x.shape[0], -1).sum(1)
        i = torch.arange(64, device=x.device, dtype=torch.float32)
        p = torch.empty(x.shape[0], 65, device=x.device)
        p[:, :64] = (torch.remainder(5 * i[None, :] + own[:, None], 8) + 1) / 16
        p[:, 64] = 1 / 32
        return p.contiguous(), ((own - opp) / 64).float().contiguous()

    @staticmethod
    def numpy(x):
        own = x[:, 0].reshape(len(x), -1).sum(1).astype(np.float32)
        opp = x[:, 1].reshape(len(x), -1).sum(1).astype(np.float32)
        i = np.arange(64, dtype=np.float32)
        p = np.empty((len(x), 65), np.float32)
        p[:, :64] = (np.remainder(5 * i[None, :] + own[:, None], 8) + 1) / 16
        p[:, 64] = 1 / 32
        return p, ((own - opp) / 64).astype(np.float32)
