"""Device arithmetic facts the kernels rely on."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_device_f64_sqrt_correctly_rounded_then_f32():
    """k_step takes (float)sqrt((double)N) on the device for the UCB's math.sqrt(parent N)."""
    n = np.arange(0, 4_000_001, dtype=np.float64)
    dev = torch.sqrt(torch.from_numpy(n).cuda()).cpu().numpy()
    assert np.array_equal(dev, np.sqrt(n))
    assert np.array_equal(dev.astype(np.float32), np.sqrt(n).astype(np.float32))


def test_device_f32_division_correctly_rounded():
    """q = W / N and u / (1 + N) in float32 (hipcc -fhip-fp32-correctly-rounded-divide-sqrt)."""
    rng = np.random.default_rng(0)
    a = rng.standard_normal(1 << 20).astype(np.float32)
    b = rng.integers(1, 5000, 1 << 20).astype(np.float32)
    dev = (torch.from_numpy(a).cuda() / torch.from_numpy(b).cuda()).cpu().numpy()
    assert np.array_equal(dev, a / b)
