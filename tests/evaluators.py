"""Test helper: the product leaf evaluator (rvz.LeafEvaluator, h2) or one of the A/B /
cross-check alternatives of tools/alt (AltEvaluator: exact f32 MFMA "resnet", 3-part bf16
"split", PyTorch "miopen"), by name."""
import rvz
from alt_eval import AltEvaluator


def make_evaluator(net, kernel="h2", **kw):
    if kernel in ("h2", "auto"):
        kw.pop("fused_epilogue", None)
        return rvz.LeafEvaluator(net, kernel=kernel, **kw)
    return AltEvaluator(net, kernel=kernel, **kw)
