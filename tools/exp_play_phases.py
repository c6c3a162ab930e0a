"""Phase split of the fused self-play kernel (k_play) from an instrumented build
(tools/ab_lib_build.sh ptime -DRVZ_PLAY_TIMING; RVZ_LIB=tools/_ab/librvz_ptime.so): per workgroup
the shader clocks of the search phase (to its barrier), the trunk passes and the FC heads, the
loop cycles, passes and rows; summarised over the workgroups of PLIES plies of the C2 workload.
GAMES (4096), SIMS (800), PLIES (20), NET (6x64), WARM (3)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

G = int(os.environ.get("GAMES", 4096))
S = int(os.environ.get("SIMS", 800))
PLIES = int(os.environ.get("PLIES", 20))
WARM = int(os.environ.get("WARM", 3))
blocks, filters = (int(x) for x in os.environ.get("NET", "6x64").split("x"))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
eng = rvz.Engine(G, S, 64, memo=True)
if int(os.environ.get("TABLE", 1)):        # bench.py's default --evals table
    eng.table(1 << 20, 14)
run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                         skip_last_eval=True, fused=True)
run.play_group = int(os.environ.get("GROUP", -6))
run.start()
if int(os.environ.get("STAGGER", 1)):      # bench.py's phase stagger (--stagger-order blocked:
    # game g of G at ply floor(60 g / G); STAGGER=2: interleaved, g mod 60)
    gi = run.seeds - 42
    bud = (gi * 60 // G if int(os.environ.get("STAGGER", 1)) == 1 else gi % 60)
    bud = bud.to(torch.int32).contiguous()
    eng.play(run.evaluator, 59, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
             reset=True, skip_last_eval=True, games_per_workgroup=run.play_group, budget=bud)
lib = rvz.load()
lib.rvz_play_timing_read.argtypes = [C.c_void_p, C.c_int]
n_wg = 16384
buf = np.zeros((n_wg, 18), dtype=np.uint64)   # [n][12] phases, then [n][6] pass / heads parts
for _ in range(WARM):
    run.ply()
torch.cuda.synchronize()
lib.rvz_play_timing_read(buf.ctypes.data, n_wg)
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
t0.record()
eng.play(run.evaluator, PLIES, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
         reset=True, skip_last_eval=True, games_per_workgroup=run.play_group)
t1.record()
torch.cuda.synchronize()
ms = t0.elapsed_time(t1)
lib.rvz_play_timing_read(buf.ctypes.data, n_wg)
flat = buf.reshape(-1)
pt = flat[n_wg * 12:n_wg * 18].reshape(n_wg, 6).astype(np.float64)
buf = flat[:n_wg * 12].reshape(n_wg, 12)
used = buf[:, 3] > 0
b = buf[used].astype(np.float64)
end_us = (b[:, 10] - b[:, 10].max()) / 100.0   # s_memrealtime ticks (100 MHz) before the last end
pt = pt[used]
tot = b[:, 3]
out = {"workgroups": int(used.sum()), "launch_ms": round(ms, 3), "plies": PLIES,
       "clock_GHz_est": round(float(np.median(tot)) / (ms * 1e6), 3),
       "search_frac": round(float((b[:, 0] / tot).mean()), 4),
       "trunk_frac": round(float((b[:, 1] / tot).mean()), 4),
       "heads_frac": round(float((b[:, 2] / tot).mean()), 4),
       "cycles_per_ply": round(float(b[:, 4].mean()) / PLIES, 2),
       "passes_per_cycle": round(float(b[:, 5].sum() / b[:, 4].sum()), 3),
       "rows_per_pass": round(float(b[:, 6].sum() / b[:, 5].sum()), 4),
       "trunk_kcycles_per_pass": round(float(b[:, 1].sum() / b[:, 5].sum()) / 1e3, 2),
       "search_kcycles_per_cycle": round(float(b[:, 0].sum() / b[:, 4].sum()) / 1e3, 2),
       "heads_kcycles_per_cycle": round(float(b[:, 2].sum() / b[:, 4].sum()) / 1e3, 2),
       "pass_stem_kcycles": round(float(pt[:, 0].sum() / pt[:, 3].sum()) / 1e3, 2),
       "pass_tower_kcycles": round(float((pt[:, 1] - pt[:, 0]).sum() / pt[:, 3].sum()) / 1e3, 2),
       "pass_headconv_kcycles": round(float(pt[:, 2].sum() / pt[:, 3].sum()) / 1e3, 2),
       "heads_weights_wait_kcycles_per_cycle": round(float(pt[:, 4].sum() / b[:, 4].sum()) / 1e3, 2),
       "heads_compute_kcycles_per_cycle": round(float(pt[:, 5].sum() / b[:, 4].sum()) / 1e3, 2),
       "queue_wait_frac": round(float((b[:, 8] / tot).mean()), 4),
       "tasks_per_wg_min_med_max": [int(b[:, 9].min()), int(np.median(b[:, 9])), int(b[:, 9].max())],
       "wg_end_us_before_last_median_max": [round(float(-np.median(end_us)), 1),
                                             round(float(-end_us.min()), 1)],
       "wg_total_kcycles_min_med_max": [round(float(x) / 1e3, 1)
                                        for x in (tot.min(), np.median(tot), tot.max())]}
print(json.dumps(out))
