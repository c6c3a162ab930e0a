"""k_play12 (the team-specialised fused launch, RVZ_PLAY_TEAMS=1) against k_play built with the
same trunk knobs: every ply's move of every game, the final boards / statuses / counters / seeds /
p, and the launch times. Run with RVZ_LIB pointing at a library whose default trunk knobs are
H2Diet and k_play12 built in (tools/ab_lib_build.sh diet "-DRVZ_PLAY12_BUILD=1 -DRVZ_H2_SKIP_LDS=1
-DRVZ_H2_APD=0 -DRVZ_H2_PD=1"; add -DRVZ_PLAY_TIMING and TIMING=1 for the team phase split).
GAMES (4096), SIMS (800), PLIES (20), TABLE (1), GROUP (-6)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

G = int(os.environ.get("GAMES", 4096))
S = int(os.environ.get("SIMS", 800))
PLIES = int(os.environ.get("PLIES", 20))
TABLE = int(os.environ.get("TABLE", 1))
GROUP = int(os.environ.get("GROUP", -6))


def play(teams, reps=2):
    os.environ["RVZ_PLAY_TEAMS"] = str(teams)
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
    eng = rvz.Engine(G, S, 64, memo=True)
    if TABLE:
        eng.table(1 << 20, 14)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                             skip_last_eval=True, fused=True)
    run.start()
    hs, times = [], []
    for _ in range(reps):
        hist = torch.full((PLIES, G), -9, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        t0 = time.time()
        eng.play(run.evaluator, PLIES, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
                 reset=True, skip_last_eval=True, hist=hist, games_per_workgroup=GROUP)
        torch.cuda.synchronize()
        times.append(time.time() - t0)
        eng.check()
        hs.append(hist)
    st = [t.clone() for t in eng.get_state()]
    return (torch.cat(hs), st, run._plies.clone(), run._done.clone(), run.seeds.clone(),
            eng.p_buf.clone(), times, int(eng.play_rows.item()))


TIMING = int(os.environ.get("TIMING", 0))


def timing_summary(buf, n_wg=256):
    import numpy as np
    t = buf.ravel()[:16384 * 12].reshape(16384, 12)[:n_wg].astype(np.float64)
    tot = t[:, 11].sum()
    out = {"total_kcycles_per_wg": round(t[:, 11].mean() / 1e3, 1)}
    for i, name in ((0, "t0_wait"), (1, "t0_pass"), (2, "t1_wait"), (3, "t1_pass"),
                    (6, "s_search"), (7, "s_heads"), (8, "s_idle")):
        out[name + "_frac"] = round(t[:, i].sum() / tot, 4)
    out["t_barrier_frac"] = round(t[:, 10].sum() / 2 / tot, 4)   # per trunk team
    out["passes"] = int(t[:, 4].sum())
    out["single_row_passes"] = int(t[:, 5].sum())
    out["rows"] = int(t[:, 9].sum())
    out["pass_kcycles"] = round((t[:, 1].sum() + t[:, 3].sum()) / max(1, t[:, 4].sum()) / 1e3, 1)
    return out


if TIMING:
    import ctypes as C
    import numpy as np
    lib = rvz.load()
    lib.rvz_play_timing_read.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros((16384, 18), dtype=np.uint64)
    lib.rvz_play_timing_read(buf.ctypes.data, 16384)   # zero
    os.environ["RVZ_PLAY_TEAMS"] = "1"
    b = play(1, reps=1)
    lib.rvz_play_timing_read(buf.ctypes.data, 16384)
    print(json.dumps({"timing_k_play12": timing_summary(buf), "s": b[6]}))
    sys.exit(0)
a = play(0)
b = play(1)
out = {"games": G, "sims": S, "plies": PLIES, "table": TABLE,
       "k_play_s": [round(t, 4) for t in a[6]], "k_play12_s": [round(t, 4) for t in b[6]],
       "rows": [a[7], b[7]]}
same = torch.equal(a[0], b[0])
out["moves_equal"] = same
if not same:
    d = (a[0] != b[0])
    out["first_diff_ply"] = int(d.any(1).nonzero()[0].item())
    out["games_differing"] = int(d.any(0).sum().item())
out["state_equal"] = all(torch.equal(x, y) for x, y in zip(a[1], b[1]))
out["counters_equal"] = (torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]) and
                         torch.equal(a[4], b[4]) and torch.equal(a[5], b[5]))
print(json.dumps(out))
