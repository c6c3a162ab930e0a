"""Decoding of the h2 trunk's device wall-clock stamps (bench.py's in-situ kernel durations).

The trunk launched through rvz_resnet_trunk_h2_ex with a stamp ring writes, per launch row and
workgroup w, stamps[row, w] = (start, end | evaluated_boards << 56) in s_memrealtime ticks
(100 MHz); the heads launch advances the ring's device counter (include/rvz.h).
"""
from __future__ import annotations

from typing import Optional

import torch

TICKS_PER_MS = 1e5          # s_memrealtime: 100 MHz
_END_MASK = (1 << 52) - 1      # bits 52-55: XCD id, 56-63: evaluated boards


def trunk_spans(stamps: torch.Tensor, launches: int) -> Optional[dict]:
    """Mean span (first workgroup start to last workgroup end, ms) and mean evaluated boards of
    the stamped launches. stamps: int64 [ring, grid, 2]; launches: the ring counter after the
    measured region (rows wrap modulo ring, so at most `ring` launches are kept). None if empty."""
    n = min(int(launches), stamps.shape[0])
    if n <= 0:
        return None
    st = stamps[:n]
    end = st[:, :, 1] & _END_MASK
    span = (end.max(dim=1).values - st[:, :, 0].min(dim=1).values).double() / TICKS_PER_MS
    rows = (st[:, :, 1] >> 56).sum(dim=1).double()
    return {"ms": float(span.mean().item()), "rows": float(rows.mean().item()),
            "launches": int(launches)}
