"""The leaf-evaluator network against the reference's (tests/golden/net_tiny.npz, CPU fp32):
state_dict compatibility (same keys/shapes, TorchScript duplicates tolerated) and outputs."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "net_tiny.npz")


def _load():
    with np.load(GOLDEN) as z:
        d = {k: z[k] for k in z.files}
    sd = {k[3:]: torch.from_numpy(v) for k, v in d.items() if k.startswith("sd/")}
    return d, sd


def test_state_dict_compatible_and_outputs_match():
    import rvz
    d, sd = _load()
    net = rvz.AlphaZeroNetwork(board_size=8, num_res_blocks=1, num_filters=16)
    assert set(net.state_dict()) == set(sd)
    dup = dict(sd)
    dup.update({"_script_module." + k: v for k, v in sd.items()})   # reference checkpoints
    rvz.load_reference_state_dict(net, dup)
    net.eval()
    with torch.no_grad():
        logits, value = net.predict(torch.from_numpy(d["x"]))
    np.testing.assert_allclose(logits.numpy(), d["logits"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(value.numpy(), d["value"], rtol=1e-5, atol=1e-6)


def test_leaf_evaluator_folded_bn_cpu():
    import rvz
    d, sd = _load()
    net = rvz.AlphaZeroNetwork(8, 1, 16)
    net.load_state_dict(sd)
    ev = rvz.LeafEvaluator(net, dtype=torch.float32, device="cpu")
    logits, value = ev(torch.from_numpy(d["x"]))
    np.testing.assert_allclose(logits.numpy(), d["logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(value.numpy(), d["value"], rtol=1e-4, atol=1e-5)
    assert ev.flops_per_row() > 0
