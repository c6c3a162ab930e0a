"""The policy/value ResNet at the leaf-evaluation boundary.

``AlphaZeroNetwork`` is state_dict-compatible with the reference's
src/model/network.py:30-117 (same module names and shapes, same forward graph), so reference
checkpoints load into it; ``load_reference_state_dict`` drops the duplicated
``_script_module.*`` keys that the reference's TorchScript compile registers
(pipeline.py:410-418). It is the model protocol of the reference (``predict(x) -> (logits[B,65],
value[B])``, network.py:136-158) and stays plain PyTorch-ROCm: the leaf evaluator is the
boundary callee, not part of the rvz hot path.

``LeafEvaluator`` is the inference form used by the self-play driver: eval-mode BatchNorm folded
into the preceding convolution, NHWC (channels_last) activations for MIOpen, fp32 (the reference's
precision) or bf16, and fixed-shape calls so the whole ply can be captured in one HIP graph.
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


class LeafEvaluator:
    """Inference-only evaluator over a fixed leaf batch: (logits f32 [n,S*S+1], value f32 [n]).

    BN is folded (eval mode), activations are channels_last, compute dtype is ``dtype``
    (torch.float32 = the reference's precision, or torch.bfloat16); outputs are float32 so the
    rvz expand kernel reads them directly (it fuses the softmax).
    """

    def __init__(self, net: AlphaZeroNetwork, dtype=torch.float32, device=None,
                 fused_epilogue: bool = None, kernel: str = "auto"):
        net = net.eval()
        self.net = net
        dev = torch.device(device) if device is not None else next(net.parameters()).device
        self.dtype, self.device = dtype, dev
        # kernel: the whole forward in one rvz kernel (fp32, 8x8 or 6x6, 64/128 filters) —
        #   "h2" = fp32 as a two-part f16 split, 3 products, on the f16 MFMA (rvz_resnet_fwd_h2),
        #   "split" = fp32 as a three-part bf16 split, 6 products, on the bf16 MFMA
        #             (rvz_resnet_fwd_split),
        #   "resnet" = the f32-input MFMA (rvz_resnet_fwd_f32, 8x8 only);
        # "miopen" = PyTorch convs (+ the fused epilogue); "auto" = h2 where it applies
        self.n_blocks, self.filters = len(net.res_blocks), net.num_filters
        self.board_size = net.board_size
        split_ok = (dev.type == "cuda" and dtype == torch.float32 and net.board_size in (6, 8)
                    and net.num_filters in (64, 128))
        if kernel not in ("auto", "h2", "split", "resnet", "miopen"):
            raise ValueError(f"unknown kernel {kernel!r}")
        if kernel in ("h2", "split") and not split_ok:
            raise ValueError(f"the {kernel} resnet kernel needs fp32, 8x8 or 6x6, 64 or 128 "
                             "filters, a GPU")
        if kernel == "resnet" and not (split_ok and net.board_size == 8):
            raise ValueError("the f32 resnet kernel needs fp32, 8x8, 64 or 128 filters, a GPU")
        if kernel == "auto":
            kernel = "h2" if split_ok else "miopen"
        self.kernel = kernel
        self.use_resnet = kernel in ("h2", "split", "resnet")
        # bench.py: (int64 [ring, grid, 2] stamp ring, int32 [1] device launch counter) to time
        # every h2 trunk launch from device wall-clock stamps, or None
        self.trunk_stamps = None
        self.trunk_events = None       # bench.py (eager): (rvz Timer, [(start, end) indices])
        self._outs = {}
        if self.use_resnet:
            from . import _lib
            lib = _lib.load()
            with torch.no_grad():
                self.params = pack_resnet_params(net).to(dev).contiguous()
            want = lib.rvz_resnet_params_size(self.board_size, self.filters, self.n_blocks)
            if want != self.params.numel():
                raise _lib.RvzError(f"packed params {self.params.numel()} != layout {want}")
            self.wsplit = None
            if kernel == "h2":
                n = lib.rvz_resnet_h2_size(self.filters, self.n_blocks)
                self.wsplit = torch.empty(n, dtype=torch.int16, device=dev)
                _lib.check(lib.rvz_resnet_h2_weights(
                    self.params.data_ptr(), self.filters, self.n_blocks, self.wsplit.data_ptr(),
                    _lib.stream_handle(dev)), None, "rvz_resnet_h2_weights")
            if kernel == "split":
                n = lib.rvz_resnet_split_size(self.filters, self.n_blocks)
                self.wsplit = torch.empty(max(n, 8), dtype=torch.int16, device=dev)
                _lib.check(lib.rvz_resnet_split_weights(
                    self.params.data_ptr(), self.filters, self.n_blocks, self.wsplit.data_ptr(),
                    _lib.stream_handle(dev)), None, "rvz_resnet_split_weights")
        # on the GPU the conv bias, ReLU and skip add run in one rvz kernel pass (rvz_nn_bias_act)
        self.fused = dev.type == "cuda" if fused_epilogue is None else bool(fused_epilogue)
        self.board_size = net.board_size
        cl = torch.channels_last

        def conv_param(conv, bn):
            w, b = _fold(conv, bn)
            return (w.to(dev, dtype).contiguous(memory_format=cl), b.to(dev, dtype))

        with torch.no_grad():
            self.stem = conv_param(net.conv, net.bn)
            self.blocks = [(conv_param(b.conv1, b.bn1), conv_param(b.conv2, b.bn2))
                           for b in net.res_blocks]
            self.pconv = conv_param(net.policy_conv, net.policy_bn)
            self.vconv = conv_param(net.value_conv, net.value_bn)
            # NCHW flatten order of the heads: permute the FC input columns once instead of
            # converting the activation back to NCHW
            cells = self.board_size ** 2

            def fc_nhwc(fc, planes):
                w = fc.weight.detach().reshape(fc.out_features, planes, cells)
                w = w.permute(0, 2, 1).reshape(fc.out_features, planes * cells)
                return w.to(dev, dtype).contiguous(), fc.bias.detach().to(dev, dtype)

            self.pfc = fc_nhwc(net.policy_fc, 2)
            self.vfc1 = fc_nhwc(net.value_fc1, 1)
            self.vfc2 = (net.value_fc2.weight.detach().to(dev, dtype),
                         net.value_fc2.bias.detach().to(dev, dtype))
            # f32 biases of the trunk convs for the fused epilogue (stem, then conv1/conv2 pairs)
            trunk = [_fold(net.conv, net.bn)[1]]
            for b in net.res_blocks:
                trunk += [_fold(b.conv1, b.bn1)[1], _fold(b.conv2, b.bn2)[1]]
            self._b32 = [t.to(dev, torch.float32).contiguous() for t in trunk]

    @torch.no_grad()
    def refresh(self):
        """Re-read the module's (trained) weights and BN statistics into this evaluator's device
        buffers, in place: the addresses a captured HIP graph holds stay valid, so the next
        replay evaluates the new net (the self-play / training loop, rvz.pipeline)."""
        net = self.net
        if self.use_resnet:
            from . import _lib
            self.params.copy_(pack_resnet_params(net).to(self.device))
            if self.kernel == "h2":
                _lib.check(_lib.load().rvz_resnet_h2_weights(
                    self.params.data_ptr(), self.filters, self.n_blocks, self.wsplit.data_ptr(),
                    _lib.stream_handle(self.device)), None, "rvz_resnet_h2_weights")
            elif self.kernel == "split":
                _lib.check(_lib.load().rvz_resnet_split_weights(
                    self.params.data_ptr(), self.filters, self.n_blocks, self.wsplit.data_ptr(),
                    _lib.stream_handle(self.device)), None, "rvz_resnet_split_weights")
        cl, dt = torch.channels_last, self.dtype

        def put(dst, conv, bn):
            w, b = _fold(conv, bn)
            dst[0].copy_(w.to(self.device, dt).contiguous(memory_format=cl))
            dst[1].copy_(b.to(self.device, dt))

        put(self.stem, net.conv, net.bn)
        for (d1, d2), blk in zip(self.blocks, net.res_blocks):
            put(d1, blk.conv1, blk.bn1)
            put(d2, blk.conv2, blk.bn2)
        put(self.pconv, net.policy_conv, net.policy_bn)
        put(self.vconv, net.value_conv, net.value_bn)
        cells = self.board_size ** 2
        for dst, fc, planes in ((self.pfc, net.policy_fc, 2), (self.vfc1, net.value_fc1, 1)):
            w = fc.weight.reshape(fc.out_features, planes, cells).permute(0, 2, 1)
            dst[0].copy_(w.reshape(fc.out_features, planes * cells).to(self.device, dt))
            dst[1].copy_(fc.bias.to(self.device, dt))
        self.vfc2[0].copy_(net.value_fc2.weight.to(self.device, dt))
        self.vfc2[1].copy_(net.value_fc2.bias.to(self.device, dt))
        trunk = [_fold(net.conv, net.bn)[1]]
        for b in net.res_blocks:
            trunk += [_fold(b.conv1, b.bn1)[1], _fold(b.conv2, b.bn2)[1]]
        for dst, t in zip(self._b32, trunk):
            dst.copy_(t.to(self.device, torch.float32))

    def _bias_act(self, y: torch.Tensor, bias: torch.Tensor, res, relu: bool):
        from . import _lib
        cl = torch.channels_last
        for t in (y, res):
            if t is not None and not t.is_contiguous(memory_format=cl):
                raise _lib.RvzError("fused epilogue needs channels_last activations")
        n_pix = y.shape[0] * y.shape[2] * y.shape[3]
        fn = (_lib.load().rvz_nn_bias_act_f32 if y.dtype == torch.float32
              else _lib.load().rvz_nn_bias_act_bf16)
        _lib.check(fn(y.data_ptr(), bias.data_ptr(), None if res is None else res.data_ptr(),
                      n_pix, y.shape[1], int(relu), _lib.stream_handle(y.device)),
                   None, "rvz_nn_bias_act")
        return y

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
        if self.kernel == "h2" and (self.trunk_events is not None or self.trunk_stamps is not None):
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
        elif self.kernel == "h2":
            _lib.check(_lib.load().rvz_resnet_fwd_h2_ex(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.wsplit.data_ptr(),
                self.filters, self.n_blocks, work.data_ptr(), logits.data_ptr(),
                value.data_ptr(), live or None, _lib.stream_handle(x.device)), None,
                "rvz_resnet_fwd_h2_ex")
        elif self.wsplit is not None:
            _lib.check(_lib.load().rvz_resnet_fwd_split(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.wsplit.data_ptr(),
                self.filters, self.n_blocks, work.data_ptr(), logits.data_ptr(),
                value.data_ptr(), _lib.stream_handle(x.device)), None, "rvz_resnet_fwd_split")
        else:
            _lib.check(_lib.load().rvz_resnet_fwd_f32(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.filters,
                self.n_blocks, logits.data_ptr(), value.data_ptr(),
                _lib.stream_handle(x.device)), None, "rvz_resnet_fwd_f32")
        return logits, value

    def trunk_only(self, x: torch.Tensor):
        """The h2 / split path's first launch alone (rvz_resnet_trunk_h2 / _split: stem,
        residual tower, 1x1 head convs -> the workspace); bench.py times the dominant kernel
        with it."""
        from . import _lib
        if self.wsplit is None:
            raise _lib.RvzError("trunk_only needs kernel='h2' or 'split'")
        if x.shape[0] not in self._outs:
            self(x)                                # allocates the per-batch buffers
        work = self._outs[x.shape[0]][2]
        fn = (_lib.load().rvz_resnet_trunk_h2 if self.kernel == "h2"
              else _lib.load().rvz_resnet_trunk_split)
        _lib.check(fn(self.board_size, x.data_ptr(), x.shape[0], self.params.data_ptr(),
                      self.wsplit.data_ptr(), self.filters, self.n_blocks, work.data_ptr(),
                      _lib.stream_handle(x.device)), None, "rvz_resnet_trunk")

    @property
    def trunk_kernel_name(self) -> str:
        return {"h2": "k_resnet_h2", "split": "k_resnet_split"}.get(self.kernel, "")

    def overflowed(self) -> bool:
        """h2 only: True if any activation of any call so far reached the f16 range limit
        (65520) — the outputs of that call are then not valid (synchronises)."""
        return any(bool(w[-4].item() != 0) for _, _, w in self._outs.values()) \
            if self.kernel == "h2" else False

    def mfma_flops_per_row(self) -> int:
        """FLOPs the trunk kernel executes on the 16-bit matrix cores per board, stem K padded
        27 -> 32: three partial products per fp32 product for h2 (f16 MFMA), six for split
        (bf16 MFMA). Pixel rows per board: 64 on 8x8; a 6x6 board is packed by h2 (4 boards in
        160 rows at 64 filters, 1 in 48 at 128) and embedded in the 8x8 grid by split."""
        f = self.filters
        if self.board_size == 8 or self.kernel != "h2":
            rows = 64
        else:
            rows = 40 if f == 64 else 48
        terms = 3 if self.kernel == "h2" else 6
        return terms * 2 * rows * f * (32 + 2 * self.n_blocks * 9 * f)

    @property
    def accepts_live_count(self) -> bool:
        """True when __call__ honours n_live (the h2 kernel): rows past the live count of a
        compacted leaf batch are skipped."""
        return self.kernel == "h2"

    def __call__(self, x: torch.Tensor, n_live=None):
        """n_live: device address (int) of an int32 count U (rvz_search_live_count): only rows
        [0, U) need outputs. Honoured by the h2 kernel; the other forms evaluate every row."""
        if self.use_resnet:
            return self._forward_resnet(x, n_live)
        if self.fused:
            return self._forward_fused(x)
        cl = torch.channels_last
        h = x.to(self.dtype).contiguous(memory_format=cl)
        w, b = self.stem
        h = F.relu(F.conv2d(h, w, b, padding=1))
        for (w1, b1), (w2, b2) in self.blocks:
            y = F.relu(F.conv2d(h, w1, b1, padding=1))
            h = F.relu(F.conv2d(y, w2, b2, padding=1) + h)
        n = h.shape[0]
        p = F.relu(F.conv2d(h, *self.pconv))          # [n,2,S,S] channels_last == NHWC memory
        p = p.permute(0, 2, 3, 1).reshape(n, -1)
        logits = F.linear(p, *self.pfc)
        v = F.relu(F.conv2d(h, *self.vconv)).reshape(n, -1)
        v = torch.tanh(F.linear(F.relu(F.linear(v, *self.vfc1)), *self.vfc2)).squeeze(1)
        return logits.float(), v.float()

    def _forward_fused(self, x: torch.Tensor):
        cl = torch.channels_last
        h = x.to(self.dtype).contiguous(memory_format=cl)
        w, b = self.stem
        h = self._bias_act(F.conv2d(h, w, padding=1), self._b32[0], None, True)
        for i, ((w1, _), (w2, _)) in enumerate(self.blocks):
            y = self._bias_act(F.conv2d(h, w1, padding=1), self._b32[1 + 2 * i], None, True)
            h = self._bias_act(F.conv2d(y, w2, padding=1), self._b32[2 + 2 * i], h, True)
        n = h.shape[0]
        p = F.relu(F.conv2d(h, *self.pconv))
        p = p.permute(0, 2, 3, 1).reshape(n, -1)
        logits = F.linear(p, *self.pfc)
        v = F.relu(F.conv2d(h, *self.vconv)).reshape(n, -1)
        v = torch.tanh(F.linear(F.relu(F.linear(v, *self.vfc1)), *self.vfc2)).squeeze(1)
        return logits.float(), v.float()

    def flops_per_row(self) -> int:
        """Multiply-adds x2 of one leaf evaluation (convs + FCs)."""
        cells = self.board_size ** 2
        f = self.stem[0].shape[0]
        macs = cells * f * 3 * 9 + len(self.blocks) * 2 * cells * f * f * 9
        macs += cells * f * 3 + 2 * cells * (cells + 1) + cells * 256 + 256
        return 2 * macs
