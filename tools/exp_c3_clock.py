#!/usr/bin/env python3
"""C3's 10x128 evaluator two ways, for rocprofv3 --pmc passes (clock, MFMA busy, L1 / L2 / HBM):

    python tools/exp_c3_clock.py fused [plies] [launches] [c3|c2]   # k_play in bench's form
    python tools/exp_c3_clock.py iso [seconds] [boards]     # the trunk alone, back to back

fused: 32,768 games x 800 sims, 10x128, memo + deferred last batch + table, groups of 16, the
bench's blocked stagger first, then `launches` launches of `plies` plies (default 2 x 20).
iso: `k_resnet_h2` over `boards` random 0/1 leaf rows (default 32,768), launched back to back for
at least `seconds` (default 5): a sustained run, so its clock is the one the chip holds under
this load (MI355X_MICROARCH.md, DVFS give-back item 6), not a cold-start burst.
VERDICT r04 item 1 asks whether the 0.561 (in situ) vs 0.757 (isolated) trunk rate gap is the
clock (power) or the fusion; pmc_clock.py turns a GRBM_GUI_ACTIVE pass into GHz per kernel.
Prints one JSON line (launch times from HIP events on the launch stream)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "alphazero-reversi_amd")):
    sys.path.insert(0, p)
import rvz  # noqa: E402
from rvz import _lib  # noqa: E402


def fused(plies=20, launches=2, games=32768, blocks=10, filters=128, group=-16, board=8,
          sims=800):
    import bench
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(board, blocks, filters).to(dev).eval()
    eng = rvz.Engine(games, sims, 64, 1.0, board_size=board, device=dev, compact_leaves=True,
                     memo=True)
    eng.table(1 << 20, 14)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net, device=dev), temperature=1.0,
                             fused_softmax=True, autoreset=True, seed_base=42,
                             skip_last_eval=True, fused=True)
    run.play_group = group
    run.start()
    L = board * board - 4
    bud = bench.stagger_budget(run.seeds - 42, L, games, "blocked")
    eng.play(run.evaluator, L - 1, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
             reset=True, skip_last_eval=True, games_per_workgroup=group, budget=bud)
    torch.cuda.synchronize()
    timer, stream = _lib.Timer(2 * launches), _lib.stream_handle(dev)
    r0 = int(eng.play_rows.item())
    s0 = int(run.steps.item())
    for _ in range(launches):
        timer.record(stream)
        run._body(plies)
        timer.record(stream)
    torch.cuda.synchronize()
    eng.check()
    ms = [timer.elapsed(2 * i, 2 * i + 1) for i in range(launches)]
    rows = int(eng.play_rows.item()) - r0
    steps = int(run.steps.item()) - s0
    fpr = run.evaluator.mfma_flops_per_row()
    t = sum(ms) * 1e-3
    return {"mode": "fused", "plies": plies, "launches": launches, "ms": [round(m, 2) for m in ms],
            "rows": rows, "board_steps_per_s": round(steps / t, 1),
            "rows_per_ply": round(rows / max(1, steps), 3),
            "executed_tflops": round(fpr * rows / t / 1e12, 1),
            "frac": round(fpr * rows / t / 1e12 / 2500, 4)}


def iso(seconds=5.0, boards=32768, blocks=10, filters=128):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, blocks, filters).to(dev).eval()
    ev = rvz.LeafEvaluator(net, device=dev)
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.rand(boards, 3, 8, 8, device=dev, generator=g) > 0.6).float()
    ev.trunk_only(x)
    torch.cuda.synchronize()
    stream = _lib.stream_handle(dev)
    n, chunk = 0, 20
    timer = _lib.Timer(2 * 4096)
    marks = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        a = timer.record(stream)
        for _ in range(chunk):
            ev.trunk_only(x)
        marks.append((a, timer.record(stream)))
        n += chunk
        torch.cuda.synchronize()
    ms = [timer.elapsed(a, b) / chunk for a, b in marks]
    fpr = ev.mfma_flops_per_row()
    tail = ms[len(ms) // 2:]          # the second half: the clock the chip holds
    avg = sum(tail) / len(tail)
    return {"mode": "iso", "boards": boards, "launches": n, "wall_s": round(time.perf_counter() - t0, 2),
            "ms_first_chunk": round(ms[0], 3), "ms_second_half": round(avg, 3),
            "executed_tflops": round(fpr * boards / (avg * 1e-3) / 1e12, 1),
            "frac": round(fpr * boards / (avg * 1e-3) / 1e12 / 2500, 4)}


CONFIGS = {"c3": dict(games=32768, blocks=10, filters=128, group=-16),
           "c2": dict(games=4096, blocks=6, filters=64, group=-6),
           "c5": dict(games=16384, blocks=6, filters=64, group=-24, board=6, sims=400)}

if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "fused":
        cfg = CONFIGS[sys.argv[4] if len(sys.argv) > 4 else "c3"]
        out = fused(*(int(a) for a in sys.argv[2:4]), **cfg)
        out["config"] = sys.argv[4] if len(sys.argv) > 4 else "c3"
        out["lib"] = os.environ.get("RVZ_LIB", "in-tree")
    else:
        a = sys.argv[2:]
        out = iso(float(a[0]) if a else 5.0, int(a[1]) if len(a) > 1 else 32768)
    print(json.dumps(out), flush=True)
