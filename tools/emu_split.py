"""CPU emulation of split-operand fp32 convolution schemes for the trunk kernel (design tool).

For each 3x3 conv of the BN-folded net, the operands are split into low-precision parts and only
some partial products are accumulated (in fp32, as the MFMA does). Reports the max logit / value
error against an fp64 evaluation, next to plain fp32's, for:
  bf16x3_6 : 3 bf16 parts each, 6 products (the current k_resnet_split)
  f16x2_3  : 2 f16 parts each (weights scaled per out-channel by 2^s), 3 products x0w0+x0w1+x1w0
  f16x2_4  : same + x1w1
Usage: python tools/emu_split.py [blocks filters n seed act_scale_log2]
"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, "alphazero-reversi_amd")
import rvz  # noqa: E402
from rvz.network import _fold  # noqa: E402


def parts(x, dt, n):
    out, r = [], x
    for _ in range(n):
        p = r.to(dt).to(torch.float64)
        out.append(p)
        r = r - p
    return out


def conv_scheme(x, w, scheme, act_log2):
    """x [n,c,8,8] fp64 holding fp32 values, w [o,c,3,3] fp64 holding fp32 values."""
    if scheme == "exact64":
        return F.conv2d(x, w, padding=1)
    if scheme == "wino32":
        return winograd(x, w, False)
    if scheme == "wino_h2":
        return winograd(x, w, True)
    if scheme == "fp32":
        return F.conv2d(x.float(), w.float(), padding=1).double()
    if scheme == "bf16x3_6":
        xs, ws = parts(x, torch.bfloat16, 3), parts(w, torch.bfloat16, 3)
        hi_t, lo_t = [(0, 0)], [(0, 1), (1, 0), (1, 1), (0, 2), (2, 0)]
        sx = 1.0
        sw = torch.ones(w.shape[0], dtype=torch.float64)
    else:
        # per-out-channel power-of-two weight scale: max |w| -> [2^14, 2^15)
        m = w.abs().amax(dim=(1, 2, 3)).clamp_min(1e-30)
        sw = torch.exp2(14 - torch.floor(torch.log2(m)))
        sx = 2.0 ** act_log2
        xs = parts(x * sx, torch.float16, 2)
        ws = parts(w * sw.view(-1, 1, 1, 1), torch.float16, 2)
        hi_t = [(0, 0)]
        lo_t = [(0, 1), (1, 0)] + ([(1, 1)] if scheme == "f16x2_4" else [])
        if scheme == "f16x2_1acc":   # one fp32 accumulator for all three products
            xa = torch.cat([xs[0], xs[0], xs[1]], 1).float()
            wa = torch.cat([ws[0], ws[1], ws[0]], 1).float()
            y = F.conv2d(xa, wa, padding=1).double()
            return y / (sx * sw.view(1, -1, 1, 1))
    conv = lambda a, b: F.conv2d(a.float(), b.float(), padding=1)  # fp32 accumulation  # noqa
    hi = sum(conv(xs[i], ws[j]) for i, j in hi_t)
    lo = torch.zeros_like(hi)
    for i, j in lo_t:
        lo = lo + conv(xs[i], ws[j])
    y = (hi + lo).double()
    return y / (sx * sw.view(1, -1, 1, 1))


BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def winograd(x, w, f16split, acc32=True):
    """F(2x2, 3x3) Winograd conv (pad 1) on 8x8 boards: input / output transforms in fp32, weights
    transformed in fp64 then rounded to fp32, the 16 per-position GEMMs with the operands split
    into two f16 parts (3 products, weights scaled per out-channel) or in fp32."""
    n, c = x.shape[:2]
    o = w.shape[0]
    xp = F.pad(x.float(), (1, 1, 1, 1))                       # [n,c,10,10] fp32
    # tiles: output (ty,tx) in 4x4, input patch padded rows 2ty..2ty+3
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)                    # [n,c,4,4,4,4] (ty,tx,i,j)
    bt = BT.float()
    v = torch.einsum("ai,nctxij,bj->nctxab", bt, d, bt)       # fp32 transforms
    u = torch.einsum("ai,ocij,bj->ocab", G, w.double(), G).float()   # [o,c,4,4]
    if f16split:
        m = u.double().abs().amax(dim=(1, 2, 3)).clamp_min(1e-30)
        sw = torch.exp2(14 - torch.floor(torch.log2(m)))
        us = parts(u.double() * sw.view(-1, 1, 1, 1), torch.float16, 2)
        vs = parts(v.double(), torch.float16, 2)
        prod = lambda a, b: torch.einsum("ocab,nctxab->notxab", a.float(), b.float())  # noqa
        mm = (prod(us[0], vs[0]) + prod(us[1], vs[0]) + prod(us[0], vs[1])).double()
        mm = mm / sw.view(1, -1, 1, 1, 1, 1)
        mm = mm.float()
    else:
        mm = torch.einsum("ocab,nctxab->notxab", u, v)         # fp32
    at = AT.float()
    y = torch.einsum("pa,notxab,qb->notxpq", at, mm, at)      # [n,o,4,4,2,2] fp32
    return y.permute(0, 1, 2, 4, 3, 5).reshape(n, o, 8, 8).double()


def forward(net, x, scheme, act_log2=0):
    """BN-folded forward with every trunk 3x3 conv through `scheme`; heads in fp64 (the error
    under study is the trunk's)."""
    x = x.double()
    r32 = (lambda t: t) if scheme == "exact64" else (lambda t: t.float().double())
    w, b = _fold(net.conv, net.bn)
    h = F.relu(conv_scheme(x, w.double(), scheme.replace("_lds", ""), act_log2)
               + b.double().view(1, -1, 1, 1))
    h = r32(h)
    for blk in net.res_blocks:
        w1, b1 = _fold(blk.conv1, blk.bn1)
        w2, b2 = _fold(blk.conv2, blk.bn2)
        y = F.relu(conv_scheme(h, w1.double(), scheme.replace("_lds", ""), act_log2)
                   + b1.double().view(1, -1, 1, 1))
        y = r32(y)
        skip = h
        if scheme.endswith("_lds"):   # skip input re-read as its two f16 parts (22 bits)
            p0 = h.to(torch.float16).double()
            skip = p0 + (h - p0).to(torch.float16).double()
        h = F.relu(conv_scheme(y, w2.double(), scheme.replace("_lds", ""), act_log2)
                   + b2.double().view(1, -1, 1, 1) + skip)
        h = r32(h)
    n = h.shape[0]
    wp, bp = _fold(net.policy_conv, net.policy_bn)
    p = F.relu(F.conv2d(h, wp.double(), bp.double())).reshape(n, -1)
    logits = F.linear(p, net.policy_fc.weight.double(), net.policy_fc.bias.double())
    wv, bv = _fold(net.value_conv, net.value_bn)
    v = F.relu(F.conv2d(h, wv.double(), bv.double())).reshape(n, -1)
    v = F.relu(F.linear(v, net.value_fc1.weight.double(), net.value_fc1.bias.double()))
    v = torch.tanh(F.linear(v, net.value_fc2.weight.double(), net.value_fc2.bias.double()))
    return logits, v.squeeze(1), h


def main():
    a = [int(v) for v in sys.argv[1:]]
    blocks, filters, n, seed, act = (a + [6, 64, 256, 5, 0][len(a):])
    torch.manual_seed(seed)
    net = rvz.AlphaZeroNetwork(8, blocks, filters).eval()
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.1, 0.1)
        x = (torch.rand(n, 3, 8, 8) > 0.6).float()
        l64, v64, h64 = forward(net, x, "exact64")
        scale = l64.abs().max().item()
        print(f"net {blocks}x{filters}, n={n}: logit scale {scale:.3g}, trunk max {h64.max():.3g}")
        for s in ("fp32", "f16x2_1acc", "wino32", "wino_h2"):
            l, v, h = forward(net, x, s, act)
            print(f"{s:9s} max|dl|/scale {((l - l64).abs().max() / scale).item():.3e}  "
                  f"max|dv| {(v - v64).abs().max().item():.3e}  "
                  f"max|dh|/hmax {((h - h64).abs().max() / h64.max()).item():.3e}")


if __name__ == "__main__":
    main()
