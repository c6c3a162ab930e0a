"""A/B and cross-check leaf evaluators (NOT the product path; the product is rvz.LeafEvaluator,
the h2 kernels of librvz.so).

``AltEvaluator(net, kernel=...)`` computes the same (logits [n, S*S+1], value [n]) as
``rvz.LeafEvaluator`` with one of the alternatives built into ``tools/alt/librvz_alt.so``:

* ``"resnet"``: the whole forward on the f32-input MFMA (rvz_resnet_fwd_f32; exact k-ordered fp32
  FMA chains, 8x8 only) — the exact-fp32 reference the tests hold h2 against;
* ``"split"``: fp32 as a 3-part bf16 split, six partial products (rvz_resnet_fwd_split), the
  previous default (h2 halves its MFMAs);
* ``"miopen"``: PyTorch-ROCm convs (MIOpen) in fp32 or bf16, with the conv bias / skip / ReLU
  fused into one pass per layer (rvz_nn_bias_act) when ``fused_epilogue``.

Same call protocol as rvz.LeafEvaluator (``ev(x) -> (logits, value)``, ``refresh()``); the
``n_live`` argument of a compacted batch is ignored (every row is evaluated), so
``accepts_live_count`` is False.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import torch
import torch.nn.functional as F

from rvz import _lib
from rvz.network import AlphaZeroNetwork, _fold, pack_resnet_params

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librvz_alt.so")
_P = C.c_void_p
SIGNATURES = {
    "rvz_nn_bias_act_f32": (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32, _P]),
    "rvz_nn_bias_act_bf16": (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32, _P]),
    "rvz_resnet_fwd_f32": (C.c_int, [C.c_int32, _P, C.c_int32, _P, C.c_int32, C.c_int32, _P, _P,
                                     _P]),
    "rvz_resnet_split_size": (C.c_int64, [C.c_int32, C.c_int32]),
    "rvz_resnet_split_weights": (C.c_int, [_P, C.c_int32, C.c_int32, _P, _P]),
    "rvz_resnet_trunk_split": (C.c_int, [C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, C.c_int32,
                                         _P, _P]),
    "rvz_resnet_fwd_split": (C.c_int, [C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, C.c_int32, _P,
                                       _P, _P, _P]),
    "rvz_alt_heads_valu": (C.c_int, [C.c_int32, _P, C.c_int32, _P, C.c_int32, C.c_int32, _P, _P,
                                     _P]),
    "rvz_alt_sqrt_count": (C.c_int, [C.c_int32, _P, _P]),
    "rvz_alt_pow": (C.c_int, [C.c_int32, _P, _P, _P, C.c_int32, _P]),
    "rvz_alt_pow_host": (C.c_int, [C.c_int32, _P, _P, _P]),
}
_alt = None


def build() -> None:
    subprocess.run(["make", "-C", HERE], check=True,
                   env=dict(os.environ, PYTORCH_ROCM_ARCH="gfx950"))


def load() -> C.CDLL:
    """librvz_alt.so (built by `make -C tools/alt`, or __graft_entry__.build())."""
    global _alt
    if _alt is None:
        if not os.path.exists(LIB_PATH):
            raise _lib.RvzError(f"{LIB_PATH} not built: make -C tools/alt")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _alt = lib
    return _alt


class AltEvaluator:
    def __init__(self, net: AlphaZeroNetwork, kernel: str = "resnet", dtype=torch.float32,
                 device=None, fused_epilogue: bool = True):
        if kernel not in ("resnet", "split", "miopen"):
            raise ValueError(f"unknown alternative {kernel!r}")
        net = net.eval()
        self.net, self.kernel = net, kernel
        dev = torch.device(device) if device is not None else next(net.parameters()).device
        self.dtype, self.device = dtype, dev
        self.n_blocks, self.filters = len(net.res_blocks), net.num_filters
        self.board_size = net.board_size
        self.fused = bool(fused_epilogue) and dev.type == "cuda"
        self._outs = {}
        if kernel in ("resnet", "split"):
            if not (dev.type == "cuda" and dtype == torch.float32 and net.num_filters in (64, 128)
                    and net.board_size in ((8,) if kernel == "resnet" else (6, 8))):
                raise ValueError(f"the {kernel} kernel needs fp32, 64 or 128 filters, a GPU and "
                                 f"board {'8' if kernel == 'resnet' else '8 or 6'}")
            self.params = pack_resnet_params(net).to(dev).contiguous()
            self.wsplit = None
            if kernel == "split":
                n = load().rvz_resnet_split_size(self.filters, self.n_blocks)
                self.wsplit = torch.empty(max(n, 8), dtype=torch.int16, device=dev)
        else:
            self._torch_params()
        self.refresh()

    accepts_live_count = False

    @torch.no_grad()
    def _torch_params(self):
        dev, dt, cl = self.device, self.dtype, torch.channels_last
        net, cells = self.net, self.board_size ** 2

        def conv_param(conv, bn):
            w, b = _fold(conv, bn)
            return (w.to(dev, dt).contiguous(memory_format=cl), b.to(dev, dt))

        def fc_nhwc(fc, planes):      # NCHW flatten order of the heads, permuted once
            w = fc.weight.detach().reshape(fc.out_features, planes, cells)
            w = w.permute(0, 2, 1).reshape(fc.out_features, planes * cells)
            return w.to(dev, dt).contiguous(), fc.bias.detach().to(dev, dt)

        self.stem = conv_param(net.conv, net.bn)
        self.blocks = [(conv_param(b.conv1, b.bn1), conv_param(b.conv2, b.bn2))
                       for b in net.res_blocks]
        self.pconv = conv_param(net.policy_conv, net.policy_bn)
        self.vconv = conv_param(net.value_conv, net.value_bn)
        self.pfc = fc_nhwc(net.policy_fc, 2)
        self.vfc1 = fc_nhwc(net.value_fc1, 1)
        self.vfc2 = (net.value_fc2.weight.detach().to(dev, dt),
                     net.value_fc2.bias.detach().to(dev, dt))
        trunk = [_fold(net.conv, net.bn)[1]]
        for b in net.res_blocks:
            trunk += [_fold(b.conv1, b.bn1)[1], _fold(b.conv2, b.bn2)[1]]
        self._b32 = [t.to(dev, torch.float32).contiguous() for t in trunk]

    @torch.no_grad()
    def refresh(self):
        if self.kernel == "miopen":
            self._torch_params()
            return
        self.params.copy_(pack_resnet_params(self.net).to(self.device))
        if self.kernel == "split":
            _lib.check(load().rvz_resnet_split_weights(
                self.params.data_ptr(), self.filters, self.n_blocks, self.wsplit.data_ptr(),
                _lib.stream_handle(self.device)), None, "rvz_resnet_split_weights")

    def _bias_act(self, y, bias, res, relu: bool):
        n_pix = y.shape[0] * y.shape[2] * y.shape[3]
        fn = load().rvz_nn_bias_act_f32 if y.dtype == torch.float32 else load().rvz_nn_bias_act_bf16
        _lib.check(fn(y.data_ptr(), bias.data_ptr(), None if res is None else res.data_ptr(),
                      n_pix, y.shape[1], int(relu), _lib.stream_handle(y.device)),
                   None, "rvz_nn_bias_act")
        return y

    def trunk_only(self, x: torch.Tensor):
        """split only: its trunk launch alone (bench.py / tools time the dominant kernel)."""
        if self.kernel != "split":
            raise _lib.RvzError("trunk_only: split only")
        work = self._buffers(x.shape[0])[2]
        _lib.check(load().rvz_resnet_trunk_split(
            self.board_size, x.data_ptr(), x.shape[0], self.params.data_ptr(),
            self.wsplit.data_ptr(), self.filters, self.n_blocks, work.data_ptr(),
            _lib.stream_handle(x.device)), None, "rvz_resnet_trunk_split")

    @property
    def trunk_kernel_name(self) -> str:
        return "k_resnet_split" if self.kernel == "split" else ""

    def mfma_flops_per_row(self) -> int:
        """split: six bf16 partial products per fp32 product, 6x6 boards in the 8x8 grid."""
        f = self.filters
        return 6 * 2 * 64 * f * (32 + 2 * self.n_blocks * 9 * f)

    def flops_per_row(self) -> int:
        cells, f = self.board_size ** 2, self.filters
        macs = cells * f * 3 * 9 + self.n_blocks * 2 * cells * f * f * 9
        macs += cells * f * 3 + 2 * cells * (cells + 1) + cells * 256 + 256
        return 2 * macs

    def overflowed(self) -> bool:
        return False

    def _buffers(self, n):
        outs = self._outs.get(n)
        if outs is None:      # fixed per batch size: stable addresses under HIP-graph capture
            outs = (torch.empty(n, self.board_size ** 2 + 1, device=self.device),
                    torch.empty(n, device=self.device),
                    torch.zeros(_lib.load().rvz_resnet_work_size(n), device=self.device))
            self._outs[n] = outs
        return outs

    @torch.no_grad()
    def __call__(self, x: torch.Tensor, n_live=None):
        if self.kernel == "miopen":
            return self._forward_torch(x)
        n = x.shape[0]
        x = x.float().contiguous()
        logits, value, work = self._buffers(n)
        st = _lib.stream_handle(x.device)
        if self.kernel == "split":
            _lib.check(load().rvz_resnet_fwd_split(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.wsplit.data_ptr(),
                self.filters, self.n_blocks, work.data_ptr(), logits.data_ptr(),
                value.data_ptr(), st), None, "rvz_resnet_fwd_split")
        else:
            _lib.check(load().rvz_resnet_fwd_f32(
                self.board_size, x.data_ptr(), n, self.params.data_ptr(), self.filters,
                self.n_blocks, logits.data_ptr(), value.data_ptr(), st), None,
                "rvz_resnet_fwd_f32")
        return logits, value

    def _forward_torch(self, x: torch.Tensor):
        cl = torch.channels_last
        h = x.to(self.dtype).contiguous(memory_format=cl)
        w, b = self.stem
        if self.fused:
            h = self._bias_act(F.conv2d(h, w, padding=1), self._b32[0], None, True)
            for i, ((w1, _), (w2, _)) in enumerate(self.blocks):
                y = self._bias_act(F.conv2d(h, w1, padding=1), self._b32[1 + 2 * i], None, True)
                h = self._bias_act(F.conv2d(y, w2, padding=1), self._b32[2 + 2 * i], h, True)
        else:
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
