"""Functional CPU restatement of the FCE-YOLOv11 inference forward.  TEST INFRASTRUCTURE ONLY.

Every function cites the reference code it restates.  Weights come as a plain
state_dict (reference key names, e.g. ``model.5.proj_q_h.weight``); BN is folded
exactly like ``utils/torch_utils.py:237-267`` with eps = 1e-3 (Q4,
``utils/torch_utils.py:470``).  Computation runs in the dtype of the inputs
(fp32 to mirror the reference CPU path, fp64 for a ground truth).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

BN_EPS = 1e-3  # utils/torch_utils.py:470 (initialize_weights)


# ----------------------------------------------------------------------------- weights
def fuse_state_dict(sd: dict, eps: float = BN_EPS) -> dict:
    """Fold every ``X.bn.*`` into ``X.conv.weight`` / ``X.conv.bias`` (torch_utils.py:237-267).

    w' = diag(g / sqrt(eps + var)) @ w ;  b' = diag(...) @ b_conv + (beta - g*mean / sqrt(var + eps)).
    """
    out = {}
    bn_prefixes = {k[: -len(".bn.weight")] for k in sd if k.endswith(".bn.weight")}
    for k, v in sd.items():
        if any(k.startswith(p + ".bn.") for p in bn_prefixes):
            continue
        out[k] = v
    for p in bn_prefixes:
        w = sd[p + ".conv.weight"]
        g, beta = sd[p + ".bn.weight"], sd[p + ".bn.bias"]
        mean, var = sd[p + ".bn.running_mean"], sd[p + ".bn.running_var"]
        s = g.div(torch.sqrt(eps + var))
        out[p + ".conv.weight"] = (w.view(w.shape[0], -1) * s[:, None]).view(w.shape)
        b_conv = sd.get(p + ".conv.bias", torch.zeros_like(g))
        out[p + ".conv.bias"] = s * b_conv + (beta - g.mul(mean).div(torch.sqrt(var + eps)))
    return out


def cast_sd(sd: dict, dtype) -> dict:
    return {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}


# ----------------------------------------------------------------------------- primitives
def conv(sd, p, x, s=1, g=1, act=True):
    """Fused ``Conv.forward_fuse`` (conv.py:80-89): act(conv(x) + b), autopad k//2 (conv.py:30-36)."""
    w = sd[p + ".conv.weight"]
    k = w.shape[-1]
    y = F.conv2d(x, w, sd.get(p + ".conv.bias"), s, k // 2, 1, g)
    return F.silu(y) if act else y


def dwconv(sd, p, x, act=True):
    """DWConv (conv.py:185-200): groups = gcd(c1, c2) = c for c1 == c2."""
    return conv(sd, p, x, 1, x.shape[1], act)


def conv2d(sd, p, x):
    """Plain nn.Conv2d 1x1 with bias."""
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"))


def bottleneck(sd, p, x, shortcut=True):
    """block.py:452-476."""
    y = conv(sd, p + ".cv2", conv(sd, p + ".cv1", x))
    return x + y if shortcut and x.shape[1] == y.shape[1] else y


def c3k(sd, p, x, n=2):
    """C3k -> C3.forward (block.py:338-340, 1087-1108)."""
    a = conv(sd, p + ".cv1", x)
    for i in range(n):
        a = bottleneck(sd, f"{p}.m.{i}", a)
    return conv(sd, p + ".cv3", torch.cat((a, conv(sd, p + ".cv2", x)), 1))


def c3k2(sd, p, x, args):
    """C3k2 -> C2f.forward (block.py:303-307, 1064-1084); args = [c1, c2, n, c3k, e, ...]."""
    n = args[2]
    use_c3k = args[3] if len(args) > 3 else False
    y = list(conv(sd, p + ".cv1", x).chunk(2, 1))
    for i in range(n):
        q = f"{p}.m.{i}"
        y.append(c3k(sd, q, y[-1]) if use_c3k else bottleneck(sd, q, y[-1]))
    return conv(sd, p + ".cv2", torch.cat(y, 1))


def sppf(sd, p, x, k=5):
    """block.py:208-232 (Q13: MaxPool2d pads with -inf)."""
    y = [conv(sd, p + ".cv1", x)]
    for _ in range(3):
        y.append(F.max_pool2d(y[-1], k, 1, k // 2))
    return conv(sd, p + ".cv2", torch.cat(y, 1))


def attention(sd, p, x, num_heads):
    """block.py:1247-1304."""
    B, C, H, W = x.shape
    N = H * W
    head_dim = C // num_heads
    key_dim = int(head_dim * 0.5)
    scale = key_dim**-0.5
    qkv = conv(sd, p + ".qkv", x, act=False)
    q, k, v = qkv.view(B, num_heads, key_dim * 2 + head_dim, N).split([key_dim, key_dim, head_dim], dim=2)
    attn = (q.transpose(-2, -1) @ k) * scale
    attn = attn.softmax(dim=-1)
    y = (v @ attn.transpose(-2, -1)).view(B, C, H, W) + conv(sd, p + ".pe", v.reshape(B, C, H, W), g=C, act=False)
    return conv(sd, p + ".proj", y, act=False)


def c2psa(sd, p, x, args):
    """block.py:1412-1464 with PSABlock (:1307-1354); heads = c // 64."""
    c1, n = args[0], args[2]
    c = int(c1 * 0.5)
    a, b = conv(sd, p + ".cv1", x).split((c, c), dim=1)
    for i in range(n):
        q = f"{p}.m.{i}"
        b = b + attention(sd, q + ".attn", b, c // 64)
        b = b + conv(sd, q + ".ffn.1", conv(sd, q + ".ffn.0", b), act=False)
    return conv(sd, p + ".cv2", torch.cat((a, b), 1))


# ----------------------------------------------------------------------------- FCE operators
def bifpn_concat(sd, p, xs, args):
    """fce_block.py:13-63: realign (Conv 1x1 + SiLU or Identity), w = relu(w)/(sum+1e-4), sum_i w_i x_i."""
    c1, c2 = args
    proc = [conv(sd, f"{p}.realign_convs.{i}", x) if ci != c2 else x for i, (x, ci) in enumerate(zip(xs, c1))]
    w = torch.relu(sd[p + ".w"].to(proc[0].dtype))
    weight = w / (torch.sum(w, dim=0) + 1e-4)
    out = weight[0] * proc[0]
    for i in range(1, len(proc)):
        out = out + weight[i] * proc[i]
    return out


def coordatt(sd, p, x, args):
    """fce_block.py:65-116."""
    inp, oup, _ = args
    n, c, h, w = x.shape
    x_h = x.mean(3, keepdim=True)
    x_w = x.mean(2, keepdim=True).permute(0, 1, 3, 2)
    y = conv(sd, p + ".cv1", torch.cat([x_h, x_w], dim=2))
    y_h, y_w = torch.split(y, [h, w], dim=2)
    a_h = conv2d(sd, p + ".cv_h", y_h).sigmoid()
    a_w = conv2d(sd, p + ".cv_w", y_w.permute(0, 1, 3, 2)).sigmoid()
    ident = conv2d(sd, p + ".identity", x) if inp != oup else x
    return ident * a_h * a_w


def coordcrossatt(sd, p, x, args):
    """fce_block.py:119-180 (Q3: requires oup == inp, no identity branch)."""
    inp, oup, reduction, heads = args
    mip = max(8, inp // reduction)
    scale = (mip // heads) ** -0.5
    n, c, h, w = x.shape
    x_h = x.mean(3, keepdim=True)
    x_w = x.mean(2, keepdim=True).permute(0, 1, 3, 2)
    y = conv2d(sd, p + ".cv1", torch.cat([x_h, x_w], dim=2))
    y_h, y_w = torch.split(y, [h, w], dim=2)
    q = conv2d(sd, p + ".q_conv", y_h).view(n, heads, -1, h).permute(0, 1, 3, 2)
    k = conv2d(sd, p + ".k_conv", y_w).view(n, heads, -1, w)
    v = conv2d(sd, p + ".v_conv", y_w).view(n, heads, -1, w).permute(0, 1, 3, 2)
    attn = ((q @ k) * scale).softmax(dim=-1)
    z = (attn @ v).permute(0, 1, 3, 2).contiguous().view(n, mip, h, 1)
    return x * conv2d(sd, p + ".proj", z).sigmoid()


def bicoordcrossatt(sd, p, x, args):
    """fce_block.py:183-284 (Q2: dim_head = max(8, inp//r)//heads)."""
    inp, oup, reduction, heads = args
    dh = max(8, inp // reduction) // heads
    mid = dh * heads
    scale = dh**-0.5
    n, c, h, w = x.shape
    x_h = x.mean(3, keepdim=True)  # AdaptiveAvgPool2d((None,1)) -> [N,C,H,1]
    x_w = x.mean(2, keepdim=True)  # [N,C,1,W]
    q_h = conv2d(sd, p + ".proj_q_h", x_h).view(n, heads, dh, h).permute(0, 1, 3, 2)
    k_h = conv2d(sd, p + ".proj_k_h", x_w).view(n, heads, dh, w)
    v_h = conv2d(sd, p + ".proj_v_h", x_w).view(n, heads, dh, w).permute(0, 1, 3, 2)
    y_h = (((q_h @ k_h) * scale).softmax(-1) @ v_h).permute(0, 1, 3, 2).reshape(n, mid, h, 1)
    gate_h = conv2d(sd, p + ".out_h", y_h)
    q_w = conv2d(sd, p + ".proj_q_w", x_w).view(n, heads, dh, w).permute(0, 1, 3, 2)
    k_w = conv2d(sd, p + ".proj_k_w", x_h).view(n, heads, dh, h)
    v_w = conv2d(sd, p + ".proj_v_w", x_h).view(n, heads, dh, h).permute(0, 1, 3, 2)
    y_w = (((q_w @ k_w) * scale).softmax(-1) @ v_w).permute(0, 1, 3, 2).reshape(n, mid, 1, w)
    gate_w = conv2d(sd, p + ".out_w", y_w)
    ident = conv2d(sd, p + ".identity", x) if inp != oup else x
    return ident * torch.sigmoid(gate_h + gate_w)


# ----------------------------------------------------------------------------- Detect
def make_anchors(shapes, strides, dtype, offset=0.5):
    """utils/tal.py:352-364."""
    pts, st = [], []
    for (h, w), s in zip(shapes, strides):
        sx = torch.arange(w, dtype=dtype) + offset
        sy = torch.arange(h, dtype=dtype) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2))
        st.append(torch.full((h * w, 1), s, dtype=dtype))
    return torch.cat(pts), torch.cat(st)


def detect_head_maps(sd, p, xs, nc):
    """Detect.forward (head.py:114-124), legacy=False cls branch (head.py:96-107, Q5)."""
    out = []
    for i, x in enumerate(xs):
        b = conv(sd, f"{p}.cv2.{i}.1", conv(sd, f"{p}.cv2.{i}.0", x))
        b = conv2d(sd, f"{p}.cv2.{i}.2", b)
        c = conv(sd, f"{p}.cv3.{i}.0.1", dwconv(sd, f"{p}.cv3.{i}.0.0", x))
        c = conv(sd, f"{p}.cv3.{i}.1.1", dwconv(sd, f"{p}.cv3.{i}.1.0", c))
        c = conv2d(sd, f"{p}.cv3.{i}.2", c)
        out.append(torch.cat((b, c), 1))
    return out


def detect_decode(maps, strides, nc, reg_max=16):
    """Detect._inference (head.py:149-167) + DFL (block.py:58-80) + dist2bbox (tal.py:367-376)."""
    B = maps[0].shape[0]
    no = nc + reg_max * 4
    x_cat = torch.cat([m.view(B, no, -1) for m in maps], 2)
    anchors, st = make_anchors([m.shape[2:] for m in maps], strides, x_cat.dtype)
    anchors, st = anchors.transpose(0, 1), st.transpose(0, 1)
    box, cls = x_cat.split((reg_max * 4, nc), 1)
    a = box.shape[-1]
    proj = torch.arange(reg_max, dtype=box.dtype).view(1, reg_max, 1, 1)
    dist = F.conv2d(box.view(B, 4, reg_max, a).transpose(2, 1).softmax(1), proj).view(B, 4, a)
    lt, rb = dist.chunk(2, 1)
    anc = anchors.unsqueeze(0)
    x1y1, x2y2 = anc - lt, anc + rb
    dbox = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1) * st
    return torch.cat((dbox, cls.sigmoid()), 1)


def strides_for(layers):
    """DetectionModel stride probe (tasks.py:396-411): 256 / feature-map size of each Detect input."""
    # The Detect inputs of YOLO11 are the P3/P4/P5 levels.
    return [8.0, 16.0, 32.0]


# ----------------------------------------------------------------------------- graph executor
def forward(layers, save, sd, x, return_maps=False, trace=None):
    """BaseModel._predict_once (tasks.py:160-188) over the fused state_dict ``sd``.

    ``sd`` must already be fused (``fuse_state_dict``) and in the compute dtype.
    Returns (B, 4+nc, A) decoded predictions (and the raw Detect maps when asked).
    """
    y = []
    for L in layers:
        i, f, t, args = L["i"], L["f"], L["type"], L["args"]
        if f != -1:
            x = y[f] if isinstance(f, int) else [x if j == -1 else y[j] for j in f]
        p = f"model.{i}"
        if t == "Conv":
            k = args[2] if len(args) > 2 else 1
            s = args[3] if len(args) > 3 else 1
            x = conv(sd, p, x, s)
        elif t == "C3k2":
            x = c3k2(sd, p, x, args)
        elif t == "SPPF":
            x = sppf(sd, p, x, args[2] if len(args) > 2 else 5)
        elif t == "C2PSA":
            x = c2psa(sd, p, x, args)
        elif t == "Upsample":
            x = F.interpolate(x, scale_factor=args[1], mode=args[2])
        elif t == "Concat":
            x = torch.cat(x, args[0] if args else 1)
        elif t == "BiFPN_Concat":
            x = bifpn_concat(sd, p, x, args)
        elif t == "BiCoordCrossAtt":
            x = bicoordcrossatt(sd, p, x, args)
        elif t == "CoordAtt":
            x = coordatt(sd, p, x, args)
        elif t == "CoordCrossAtt":
            x = coordcrossatt(sd, p, x, args)
        elif t == "Detect":
            nc = args[0]
            maps = detect_head_maps(sd, p, x, nc)
            out = detect_decode(maps, strides_for(layers), nc)
            if trace is not None:
                trace.append((i, t, [float(m.abs().max()) for m in maps]))
            return (out, maps) if return_maps else out
        else:
            raise NotImplementedError(t)
        if trace is not None:
            trace.append((i, t, float(x.abs().max())))
        y.append(x if i in save else None)
    return x
