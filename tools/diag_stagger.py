"""Diagnostic: the bench's stagger launch followed by whole-game launches at C2 size, checking
the device error word and committed plies after every launch."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("DIAG_PKG", os.path.join(ROOT, "alphazero-reversi_amd")))
import torch  # noqa: E402
import rvz  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    stag = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    gpw = int(sys.argv[3]) if len(sys.argv) > 3 else -6
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
    eng = rvz.Engine(G, 800, 64, memo=True, compact_leaves=True)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                             skip_last_eval=True, fused=True)
    run.play_group = gpw
    run.start()
    if stag:
        bud = ((run.seeds - 42) % 60).to(torch.int32).contiguous()
        t0 = time.time()
        eng.play(run.evaluator, 59, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
                 reset=True, skip_last_eval=True, games_per_workgroup=gpw, budget=bud)
        torch.cuda.synchronize()
        print("stagger", time.time() - t0, int(run._plies.sum()), int(bud.sum()), flush=True)
        eng.check()
    mode = sys.argv[4] if len(sys.argv) > 4 else "eager"
    if mode == "graph":
        run._body(60)
        torch.cuda.synchronize()
        if os.environ.get("DIAG_CHECK", "1") == "1":
            eng.check()
        print("eager warm ok", eng._play_scratch[:2].view(torch.int32).tolist(), flush=True)
        run.capture(plies=60)
        print("captured", eng._play_scratch[:2].view(torch.int32).tolist(), flush=True)
    for i in range(4):
        p0 = int(run._plies.sum())
        t0 = time.time()
        if mode == "graph":
            run.ply()
        else:
            run._body(60) if i % 2 == 0 else run._body(20)
        torch.cuda.synchronize()
        dt = time.time() - t0
        err = None
        try:
            eng.check()
        except rvz.RvzError as e:
            err = str(e)[:60]
        print(f"launch {i}: {dt:.3f}s plies {int(run._plies.sum()) - p0} err {err} q "
              f"{eng._play_scratch[:2].view(torch.int32).tolist()}", flush=True)


main()
