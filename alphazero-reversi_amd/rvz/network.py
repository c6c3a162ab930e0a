"""The policy/value ResNet at the leaf-evaluation boundary.

``AlphaZeroNetwork`` is state_dict-compatible with the reference's
src/model/network.py:30-117 (same module names and shapes, same forward graph), so reference
checkpoints load into it; ``load_reference_state_dict`` drops the duplicated
``_script_module.*`` keys that the reference's TorchScript compile registers
(pipeline.py:410-418). It is the model protocol of the reference (``predict(x) -> (logits[B,65],
value[B])``, network.py:136-158) and stays plain PyTorch-ROCm: the leaf evaluator is the
boundary callee, not part of the rvz hot path.

``LeafEvaluator`` is the inference form used by the self-play driver: eval-mode BatchNorm folded
into the preceding convolution, the whole forward in the rvz h2 kernels (fp32-class on the f16
matrix cores), fixed-shape calls so the whole ply can be captured in one HIP graph.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Residual(nn.Module):
    """conv-bn-relu-conv-bn + skip, relu (network.py:14-28)."""

    def __init__(self, width: int):
        super().__init__()
        self.conv1 = nn.Conv2d(width, width, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + x)


class AlphaZeroNetwork(nn.Module):
    """3 -> F stem, N residual blocks, 2-plane policy head (S*S+1 logits), 1-plane value head."""

    def __init__(self, board_size: int = 8, num_res_blocks: int = 5, num_filters: int = 128):
        super().__init__()
        self.board_size = board_size
        self.num_filters = num_filters
        cells = board_size * board_size
        self.conv = nn.Conv2d(3, num_filters, 3, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(num_filters)
        self.res_blocks = nn.ModuleList(_Residual(num_filters) for _ in range(num_res_blocks))
        self.policy_conv = nn.Conv2d(num_filters, 2, 1, bias=False)
        self.policy_bn = nn.BatchNorm2d(2)
        self.policy_fc = nn.Linear(2 * cells, cells + 1)
        self.value_conv = nn.Conv2d(num_filters, 1, 1, bias=False)
        self.value_bn = nn.BatchNorm2d(1)
        self.value_fc1 = nn.Linear(cells, 256)
        self.value_fc2 = nn.Linear(256, 1)
        self.reset_parameters()

    def reset_parameters(self):
        """Kaiming-normal fan-out for conv/linear weights, BN affine = (1, 0) (network.py:71-78)."""
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def trunk(self, x):
        x = F.relu(self.bn(self.conv(x)))
        for blk in self.res_blocks:
            x = blk(x)
        return x

    def forward(self, x) -> Tuple[torch.Tensor, torch.Tensor]:
        h = self.trunk(x)
        n = h.shape[0]
        pol = F.relu(self.policy_bn(self.policy_conv(h))).reshape(n, -1)
        val = F.relu(self.value_bn(self.value_conv(h))).reshape(n, -1)
        val = torch.tanh(self.value_fc2(F.relu(self.value_fc1(val))))
        return self.policy_fc(pol), val.squeeze(1)

    def predict(self, board_state, valid_moves=None):
        """network.py:136-158: adds the batch dim for a single [3,S,S] state."""
        if board_state.dim() == 3:
            board_state = board_state.unsqueeze(0)
        return self.forward(board_state)


def load_reference_state_dict(net: nn.Module, sd: Dict[str, torch.Tensor]) -> None:
    """Load a reference checkpoint; tolerates the TorchScript `_script_module.` duplicates."""
    plain = {k: v for k, v in sd.items() if not k.startswith("_script_module.")}
    if not plain:  # only the scripted copy was saved
        plain = {k[len("_script_module."):]: v for k, v in sd.items()}
    net.load_state_dict(plain)


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d):
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    w = conv.weight * scale.reshape(-1, 1, 1, 1)
    b = bn.bias - bn.running_mean * scale
    return w.detach(), b.detach()


def pack_resnet_params(net: AlphaZeroNetwork) -> torch.Tensor:
    """BN-folded fp32 parameters in the layout of csrc/rvz_resnet.hip (rvz_resnet_fwd_f32)."""
    F = net.num_filters
    parts = []

    def put(t):                                            # every segment 16-byte aligned
        t = t.detach().float().reshape(-1)
        parts.append(t)
        if t.numel() % 4:
            parts.append(torch.zeros(4 - t.numel() % 4, device=t.device))

    w, b = _fold(net.conv, net.bn)                         # [F,3,3,3] -> [F][tap*3 + ch]
    put(w.permute(0, 2, 3, 1).reshape(F, 27))
    put(b)
    ws, bs = [], []
    for blk in net.res_blocks:
        for conv, bn in ((blk.conv1, blk.bn1), (blk.conv2, blk.bn2)):
            w, b = _fold(conv, bn)                         # [n][k][3][3] -> [tap][n][k]
            ws.append(w.permute(2, 3, 0, 1).reshape(9, F, F))
            bs.append(b)
    put(torch.stack(ws) if ws else torch.zeros(0, device=w.device))
    put(torch.stack(bs) if bs else torch.zeros(0, device=w.device))
    w, b = _fold(net.policy_conv, net.policy_bn)
    put(w.reshape(2, F))
    put(b)
    put(net.policy_fc.weight)
    put(net.policy_fc.bias)
    w, b = _fold(net.value_conv, net.value_bn)
    put(w.reshape(F))
    put(b)
    put(net.value_fc1.weight)
    put(net.value_fc1.bias)
    put(net.value_fc2.weight.reshape(-1))
    put(net.value_fc2.bias)
    return torch.cat(parts).contiguous()


# trunk widths with an h2 instantiation (k_resnet_h2 and the fused k_play alike)
H2_WIDTHS = {8: (64, 128, 256), 6: (64, 128)}


def h2_covers(net: nn.Module, dtype=torch.float32, device=None) -> bool:
    """True when the h2 kernels evaluate `net`: fp32, an 8x8 AlphaZeroNetwork of 64, 128 or 256
    filters or a 6x6 one of 64 or 128 (the reference's configs: C2/C5 6x64, C3/C4 10x128,
    ModelConfig's 5x128; 256 = network.py's wider towers), on a HIP device."""
    dev = torch.device(device) if device is not None else next(net.parameters()).device
    return (dev.type == "cuda" and dtype == torch.float32 and
            getattr(net, "num_filters", None) in H2_WIDTHS.get(getattr(net, "board_size", None),
                                                               ()) and
            hasattr(net, "res_blocks"))


class ModuleEvaluator:
    """The leaf evaluator of a net the h2 kernels do not cover (another filter count, or any
    module with the reference's forward): the module itself on the GPU through PyTorch-ROCm —
    the north star's "leaf evaluation calls the existing ResNet via PyTorch-ROCm" — in fp32,
    eval mode, logits and value as the expand wants them. Pull-style only (Engine.play runs the
    h2 kernels inside its launch). MIOpen picks its convolution algorithm per tensor shape, so a
    row's outputs would depend on how many rows share the call; the module therefore always runs
    on chunks of exactly `chunk` rows (the last one zero-padded): one shape, one algorithm, and
    every row's outputs a function of that row alone, as the engine's memo and the oracle
    comparisons assume (tests/test_gpu_dropin.py)."""
    kernel = "module"
    accepts_live_count = False

    def __init__(self, net: nn.Module, device=None, chunk: int = 64):
        dev = torch.device(device) if device is not None else next(net.parameters()).device
        if dev.type != "cuda":
            from . import _lib
            raise _lib.RvzError("ModuleEvaluator runs the net on a HIP device (no CPU fallback)")
        self.net, self.device, self.chunk = net.eval().to(dev), dev, int(chunk)
        self.board_size = int(getattr(net, "board_size", 8))

    def __call__(self, x: torch.Tensor):
        n, c = x.shape[0], self.chunk
        xp = x.float()
        if n % c:
            xp = torch.cat([xp, xp.new_zeros((c - n % c,) + tuple(x.shape[1:]))])
        outs = []
        with torch.no_grad():
            for i in range(0, xp.shape[0], c):
                lg, v = self.net(xp[i:i + c])
                outs.append((lg.float(), v.float().reshape(-1)))
        logits = torch.cat([o[0] for o in outs])[:n].contiguous()
        value = torch.cat([o[1] for o in outs])[:n].contiguous()
        return logits, value

    def overflowed(self) -> bool:
        return False

    def bind_engine(self, engine):
        """Called by an Engine the first time it searches with this evaluator (Engine._bind)."""
        import weakref
        self.__dict__.setdefault("_engines", weakref.WeakSet()).add(engine)

    def refresh(self):
        """The module's weights changed (a training step): the evaluator reads the live module,
        so only the engines' memo links to the old net's outputs are dropped (as
        LeafEvaluator.refresh does)."""
        self.net.eval()
        for eng in list(getattr(self, "_engines", ())):
            if getattr(eng, "memo_on", False) or getattr(eng, "table_slots", 0):
                eng.memo_reset()


def leaf_evaluator(net: nn.Module, dtype=torch.float32, device=None):
    """The default leaf evaluator of SelfPlay / ELOPlayer: LeafEvaluator (the h2 kernels) when
    they cover the net (h2_covers), else ModuleEvaluator, with a warning naming the shape."""
    if h2_covers(net, dtype, device):
        return LeafEvaluator(net, dtype=dtype, device=device)
    import warnings
    warnings.warn(f"rvz: the h2 kernels cover 64 / 128 (and on 8x8 256) filters in fp32; this net "
                  f"({getattr(net, 'num_filters', '?')} filters, {dtype}) is evaluated by its "
                  "PyTorch module on the GPU (ModuleEvaluator, pull-style)", stacklevel=2)
    if dtype != torch.float32:
        from . import _lib
        raise _lib.RvzError("leaf evaluation is fp32 (the reference's precision)")
    return ModuleEvaluator(net, device=device)


class LeafEvaluator:
    """The leaf evaluator of the self-play path: the reference's forward (network.py:30-117,
    eval-mode BN folded) as the rvz h2 kernels — one trunk launch (k_resnet_h2: fp32 as a two-part
    f16 split, three partial products on the f16 MFMA) and one FC-heads launch (k_heads_mfma) per
    leaf batch. Returns (logits f32 [n, S*S+1], value f32 [n]); the rvz expand kernel reads them
    directly (it fuses the softmax). fp32 only (the reference's precision), 8x8 or 6x6 boards,
    64 or 128 filters, or 256 on 8x8, on the GPU: anything else raises (no CPU or PyTorch fallback). The A/B
    alternatives (exact f32 MFMA, 3-part bf16 split, MIOpen) live in tools/alt (AltEvaluator).
    """

    def __init__(self, net: AlphaZeroNetwork, dtype=torch.float32, device=None,
                 kernel: str = "h2"):
        from . import _lib
        net = net.eval()
        self.net = net
        dev = torch.device(device) if device is not None else next(net.parameters()).device
        self.dtype, self.device = dtype, dev
        self.n_blocks, self.filters = len(net.res_blocks), net.num_filters
        self.board_size = net.board_size
        if kernel not in ("auto", "h2"):
            raise ValueError(f"unknown kernel {kernel!r}: the product evaluator is 'h2' "
                             "(A/B alternatives: tools/alt/alt_eval.py AltEvaluator)")
        if not h2_covers(net, dtype, dev):
            raise _lib.RvzError(
                "LeafEvaluator needs fp32, an 8x8 or 6x6 net of 64 or 128 filters (or 8x8 of "
                "256) and a HIP "
                f"device (got {net.board_size}x{net.board_size}, {net.num_filters} filters, "
                f"{dtype}, {dev}; no CPU fallback). For another shape hand the caller any "
                "callable leaf_x -> (logits, value), e.g. rvz.ModuleEvaluator(model) "
                "(SelfPlay / ELOPlayer pick it by themselves: rvz.network.leaf_evaluator; "
                "INTEGRATION.md)")
        self.kernel = "h2"
        # bench.py: (int64 [ring, grid, 2] stamp ring, int32 [1] device launch counter) to time
        # every h2 trunk launch from device wall-clock stamps, or None
        self.trunk_stamps = None
        self.trunk_events = None       # bench.py (eager): (rvz Timer, [(start, end) indices])
        self._outs = {}
        lib = _lib.load()
        with torch.no_grad():
            self.params = pack_resnet_params(net).to(dev).contiguous()
        want = lib.rvz_resnet_params_size(self.board_size, self.filters, self.n_blocks)
        if want != self.params.numel():
            raise _lib.RvzError(f"packed params {self.params.numel()} != layout {want}")
        n = lib.rvz_resnet_h2_size(self.filters, self.n_blocks)
        self.wsplit = torch.empty(n, dtype=torch.int16, device=dev)
        self._h2_weights()

    def _h2_weights(self):
        from . import _lib
        _lib.check(_lib.load().rvz_resnet_h2_weights(
            self.params.data_ptr(), self.filters, self.n_blocks, self.wsplit.data_ptr(),
            _lib.stream_handle(self.device)), None, "rvz_resnet_h2_weights")

    def bind_engine(self, engine):
        """Called by an Engine the first time it searches or plays with this evaluator: refresh()
        then drops that engine's NN-output memo (its carried outputs belong to the old net)."""
        import weakref
        eng = self.__dict__.setdefault("_engines", weakref.WeakSet())
        eng.add(engine)

    @torch.no_grad()
    def refresh(self):
        """Re-read the module's (trained) weights and BN statistics into this evaluator's device
        buffers, in place: the addresses a captured HIP graph holds stay valid, so the next
        replay evaluates the new net (the self-play / training loop, rvz.pipeline). Every engine
        that used this evaluator forgets its memo (Engine.memo_reset, stream-ordered after the
        new weights): a memo link would otherwise hand the old net's priors and value to the
        next search."""
        self.params.copy_(pack_resnet_params(self.net).to(self.device))
        self._h2_weights()
        for eng in list(getattr(self, "_engines", ())):
            if getattr(eng, "memo_on", False) or getattr(eng, "table_slots", 0):
                eng.memo_reset()                  # also a new generation of the play() table

    def _forward_resnet(self, x: torch.Tensor, n_live=None):
        from . import _lib
        n = x.shape[0]
        x = x.float().contiguous()
        outs = self._outs.get(n)
        if outs is None:   # fixed per batch size: stable addresses under HIP-graph capture
            outs = (torch.empty(n, self.board_size ** 2 + 1, device=self.device),
                    torch.empty(n, device=self.device),
                    torch.zeros(_lib.load().rvz_resnet_work_size(n), device=self.device))
            self._outs[n] = outs
        logits, value, work = outs
        live = int(n_live or 0)     # device address of the live row count, or 0 (all rows)
        if self.trunk_events is not None or self.trunk_stamps is not None:
            # instrumented forms (bench.py): the two launches of rvz_resnet_fwd_h2_ex with either
            # an event pair (rvz_timer, no system fence) around the trunk launch (eager), or the
            # trunk storing its workgroups' start / end wall clock in slot k of trunk_stamps
            lib, st = _lib.load(), _lib.stream_handle(x.device)
            stamps, ctr, ring, a = None, None, 0, None
            if self.trunk_events is not None:
                tm, pairs = self.trunk_events
                a = tm.record(st)
            else:
                buf, cnt = self.trunk_stamps       # int64 [ring, grid, 2], int32 [1] counter
                if buf.shape[1] != lib.rvz_resnet_h2_grid(self.board_size, self.filters, n):
                    raise _lib.RvzError("trunk stamp buffer does not match the batch")
                stamps, ctr, ring = buf.data_ptr(), cnt.data_ptr(), buf.shape[0]
            _lib.check(lib.rvz_resnet_trunk_h2_ex(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.wsplit.data_ptr(),
                self.filters, self.n_blocks, work.data_ptr(), live or None, stamps, ctr, ring,
                st), None, "rvz_resnet_trunk_h2_ex")
            if a is not None:
                pairs.append((a, tm.record(st)))
            _lib.check(lib.rvz_resnet_heads_fc_ex(
                self.board_size, work.data_ptr(), n, self.params.data_ptr(), self.filters,
                self.n_blocks, logits.data_ptr(), value.data_ptr(), live or None, ctr, st), None,
                "rvz_resnet_heads_fc_ex")
        else:
            _lib.check(_lib.load().rvz_resnet_fwd_h2_ex(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.wsplit.data_ptr(),
                self.filters, self.n_blocks, work.data_ptr(), logits.data_ptr(),
                value.data_ptr(), live or None, _lib.stream_handle(x.device)), None,
                "rvz_resnet_fwd_h2_ex")
        return logits, value

    def trunk_only(self, x: torch.Tensor):
        """The first launch alone (rvz_resnet_trunk_h2: stem, residual tower, 1x1 head convs ->
        the workspace); bench.py times the dominant kernel with it."""
        from . import _lib
        if x.shape[0] not in self._outs:
            self(x)                                # allocates the per-batch buffers
        work = self._outs[x.shape[0]][2]
        _lib.check(_lib.load().rvz_resnet_trunk_h2(
            self.board_size, x.data_ptr(), x.shape[0], self.params.data_ptr(),
            self.wsplit.data_ptr(), self.filters, self.n_blocks, work.data_ptr(),
            _lib.stream_handle(x.device)), None, "rvz_resnet_trunk_h2")

    trunk_kernel_name = "k_resnet_h2"

    def ovf_word(self) -> torch.Tensor:
        """The sticky f16-overflow word the fused self-play launch (Engine.play) sets."""
        w = getattr(self, "_ovf", None)
        if w is None:
            w = self._ovf = torch.zeros(4, device=self.device)
        return w

    def overflowed(self) -> bool:
        """True if a call's activations stayed past the f16 range limit (65520) even after the
        ranged re-run of the boards that reached it (a bound error; no finite net measured sets
        it) — the outputs of that call are then not valid (synchronises)."""
        fused = getattr(self, "_ovf", None)
        return (any(bool(w[-4].item() != 0) for _, _, w in self._outs.values()) or
                (fused is not None and bool(fused[0].item() != 0)))

    def mfma_flops_per_row(self) -> int:
        """FLOPs the trunk kernel executes on the f16 matrix cores per board: three partial
        products per fp32 product, stem K padded 27 -> 32. Pixel rows per board: 64 on 8x8; a 6x6
        board is packed (4 boards in 160 rows at 64 filters, 1 in 48 at 128). 8x8 at 64 filters
        (two row-interleaved boards per workgroup, RVZ_H2_ILV): the 3 edge taps of the 2 edge
        rows are skipped, 11/12 of each conv's products are executed."""
        f = self.filters
        rows = 64 if self.board_size == 8 else (40 if f == 64 else 48)
        conv = 2 * self.n_blocks * 9 * f
        if self.board_size == 8 and f == 64:
            conv = conv * 11 // 12
        return 3 * 2 * rows * f * (32 + conv)

    def useful_flops_per_row(self) -> int:
        """Algorithmic FLOPs (2 x multiply-adds) of what the trunk kernel computes for one board:
        the 3 -> F stem, the 2N residual 3x3 convs and the 1x1 head convs (F -> 2 + 1), SURVEY
        §8(d)'s per-evaluation figure (56.8 MFLOP at 6x64 on 8x8). mfma_flops_per_row / this is
        the executed/useful ratio (3 f16 products per fp32 product, stem K padding, skipped
        edge taps)."""
        cells, f = self.board_size ** 2, self.filters
        return 2 * cells * (f * 27 + self.n_blocks * 2 * f * f * 9 + f * 3)

    # __call__ honours n_live: rows past the live count of a compacted leaf batch are skipped
    accepts_live_count = True

    def __call__(self, x: torch.Tensor, n_live=None):
        """n_live: device address (int) of the per-stripe live counts (rvz_search_live_count):
        only those rows need outputs (mcts.py:544-623 evaluates the U live leaves)."""
        return self._forward_resnet(x, n_live)

    def flops_per_row(self) -> int:
        """Multiply-adds x2 of one leaf evaluation (convs + FCs)."""
        cells = self.board_size ** 2
        f = self.filters
        macs = cells * f * 3 * 9 + self.n_blocks * 2 * cells * f * f * 9
        macs += cells * f * 3 + 2 * cells * (cells + 1) + cells * 256 + 256
        return 2 * macs
