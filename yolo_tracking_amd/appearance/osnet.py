"""OSNet feature extractor for the MI355X ReID producer ("OSNet forward").

Reference: boxmot/appearance/backbones/osnet.py (OSNet, OSBlock, LightConv3x3, ChannelGate,
osnet_x1_0 / x0_75 / x0_5 / x0_25; Zhou et al., ICCV 2019), built by
reid_multibackend.py:74-80 and run in eval mode (:238-241), where the network returns the 512-d
fc feature.  This is an inference graph, not a module tree: every BatchNorm is folded into the
convolution / linear layer before it (eval mode: y = gamma (x - mean) / sqrt(var + eps) + beta),
activations stay channels-last (NHWC, MIOpen's fast path on gfx950), and the four branches of
every omni-scale block run batched: their first LightConv 1x1s as one convolution over the
concatenated output channels, the deeper 1x1s as one grouped convolution per depth (groups =
branches still running), every depthwise 3x3 as one grouped convolution, and the shared channel
gate over all four branches at once.  Parameters are taken from a checkpoint in the reference's
key layout (torchreid's names: conv1.conv.weight, conv2.0.conv2b.1.bn.running_var, ...), so the
reference's .pt weight files load unchanged; parity with the reference network is pinned by
tests/golden/osnet_x0_25.npz (the reference module with random weights, eval mode).
"""
import math
import re

import numpy as np

WIDTHS = {"osnet_x1_0": (64, 256, 384, 512), "osnet_x0_75": (48, 192, 288, 384),
          "osnet_x0_5": (32, 128, 192, 256), "osnet_x0_25": (16, 64, 96, 128)}
FEATURE_DIM = 512
BN_EPS = 1e-5
CHUNK = 1024   # crops per forward pass: bounds the activations (the block's tensors stay in cache)


def model_name(weights):
    """The OSNet variant a weight file name names (reid_model_factory.get_model_name)."""
    s = str(weights)
    for name in sorted(WIDTHS, key=len, reverse=True):
        if name in s:
            return name
    return None


def random_state_dict(name="osnet_x0_25", seed=0):
    """A state_dict in the reference's key layout with freshly initialised weights (kaiming
    normal fan-out for convolutions, N(0, 0.01) for the fc, identity BatchNorms): what the
    reference's constructor gives without pretrained weights."""
    rng = np.random.default_rng(seed)
    sd = {}

    def conv(key, cout, cin, k, bias=False):
        std = math.sqrt(2.0 / (cout * k * k))
        sd[key + ".weight"] = rng.normal(0, std, (cout, cin, k, k)).astype(np.float32)
        if bias:
            sd[key + ".bias"] = np.zeros(cout, np.float32)

    def bn(key, c):
        sd[key + ".weight"] = np.ones(c, np.float32)
        sd[key + ".bias"] = np.zeros(c, np.float32)
        sd[key + ".running_mean"] = np.zeros(c, np.float32)
        sd[key + ".running_var"] = np.ones(c, np.float32)

    def light(key, c):
        conv(key + ".conv1", c, c, 1)
        std = math.sqrt(2.0 / (c * 9))
        sd[key + ".conv2.weight"] = rng.normal(0, std, (c, 1, 3, 3)).astype(np.float32)
        bn(key + ".bn", c)

    def block(key, cin, cout):
        mid = cout // 4
        conv(key + ".conv1.conv", mid, cin, 1)
        bn(key + ".conv1.bn", mid)
        light(key + ".conv2a", mid)
        for br, depth in (("conv2b", 2), ("conv2c", 3), ("conv2d", 4)):
            for d in range(depth):
                light(f"{key}.{br}.{d}", mid)
        conv(key + ".gate.fc1", mid // 16, mid, 1, bias=True)
        conv(key + ".gate.fc2", mid, mid // 16, 1, bias=True)
        conv(key + ".conv3.conv", cout, mid, 1)
        bn(key + ".conv3.bn", cout)
        if cin != cout:
            conv(key + ".downsample.conv", cout, cin, 1)
            bn(key + ".downsample.bn", cout)

    c = WIDTHS[name]
    conv("conv1.conv", c[0], 3, 7)
    bn("conv1.bn", c[0])
    for stage, (cin, cout, reduce) in enumerate(((c[0], c[1], True), (c[1], c[2], True),
                                                 (c[2], c[3], False))):
        key = f"conv{stage + 2}"
        block(key + ".0", cin, cout)
        block(key + ".1", cout, cout)
        if reduce:
            conv(key + ".2.0.conv", cout, cout, 1)
            bn(key + ".2.0.bn", cout)
    conv("conv5.conv", c[3], c[3], 1)
    bn("conv5.bn", c[3])
    sd["fc.0.weight"] = rng.normal(0, 0.01, (FEATURE_DIM, c[3])).astype(np.float32)
    sd["fc.0.bias"] = np.zeros(FEATURE_DIM, np.float32)
    bn("fc.1", FEATURE_DIM)
    return sd


def load_checkpoint(path):
    """torch.load(path, weights_only=True) of a reference weight file: a state_dict, or a dict
    holding one under 'state_dict'; 'module.' prefixes dropped (reid_model_factory
    load_pretrained_weights)."""
    import torch
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(ck, dict) and "state_dict" in ck:
        ck = ck["state_dict"]
    return {re.sub(r"^module\.", "", k): v for k, v in ck.items()}


class OSNetReID:
    """Eval-mode OSNet feature extractor: crops (N, 3, H, W) -> (N, 512) in the crops' dtype
    (float32 or float16), on the crops' device.

    On a GPU every layer runs in csrc/osnet.hip (NCHW): the stem (7x7 conv), the pools, every
    1x1 convolution and the fc as MFMA GEMMs with bias / residual / ReLU epilogues, the depthwise
    3x3s, the channel gates and the gated branch sums; PyTorch only allocates the activations.
    `hip=False` runs the same folded graph on PyTorch's kernels (MIOpen), for comparison, and is
    what a CPU device gets."""

    def __init__(self, name="osnet_x0_25", state_dict=None, device="cuda:0", half=False,
                 chunk=CHUNK, channels_last=None, hip=True):
        import torch
        if name not in WIDTHS:
            raise KeyError(f"unknown OSNet variant {name!r}")
        self.torch = torch
        self.chunk = int(chunk)
        self.name = name
        self.widths = WIDTHS[name]
        self.device = torch.device(device)
        self.hip = bool(hip) and self.device.type == "cuda"
        if channels_last is None:
            channels_last = not self.hip
        if self.hip and channels_last:
            raise ValueError("the HIP block kernels take NCHW planes (channels_last=False)")
        self.fmt = torch.channels_last if channels_last else torch.contiguous_format
        self.dtype = torch.float16 if half else torch.float32
        sd = random_state_dict(name) if state_dict is None else state_dict
        self._build({k: torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v)
                     .to(torch.float64) for k, v in sd.items()})

    # ---- parameter folding (float64 on the host, then cast once)
    def _t(self, x):
        return x.to(self.device, self.dtype).contiguous(memory_format=self.fmt) \
            if x.dim() == 4 else x.to(self.device, self.dtype).contiguous()

    @staticmethod
    def _fold(w, sd, bn):
        scale = sd[bn + ".weight"] / (sd[bn + ".running_var"] + BN_EPS).sqrt()
        shape = (-1,) + (1,) * (w.dim() - 1)
        return w * scale.reshape(shape), sd[bn + ".bias"] - sd[bn + ".running_mean"] * scale

    def _f32(self, x, shape=None):
        """float32 on the device; with `shape` = (G, cout_g, K) a 1x1 weight in the k-major
        [G][K][cout_g] layout yta_osnet_pointwise reads (lanes along the output channels)."""
        x = x.to(self.device, self.torch.float32)
        if shape is None:
            return x.contiguous()
        return x.reshape(shape).transpose(1, 2).contiguous()

    def _build(self, sd):
        P = {}
        w, b = self._fold(sd["conv1.conv.weight"], sd, "conv1.bn")
        P["stem"] = (self._t(w), self._t(b))
        H = {"stem": (self._f32(w), self._f32(b))}      # the HIP kernels' float32 operands
        self.blocks = []
        for stage in (2, 3, 4):
            for i in (0, 1):
                self.blocks.append(self._block(sd, f"conv{stage}.{i}"))
            red = f"conv{stage}.2.0"
            if red + ".conv.weight" in sd:
                w, b = self._fold(sd[red + ".conv.weight"], sd, red + ".bn")
                self.blocks.append(("reduce", self._t(w), self._t(b),
                                    self._f32(w, (1, w.shape[0], w.shape[1])), self._f32(b)))
        w, b = self._fold(sd["conv5.conv.weight"], sd, "conv5.bn")
        P["conv5"] = (self._t(w), self._t(b))
        H["conv5"] = (self._f32(w, (1, w.shape[0], w.shape[1])), self._f32(b))
        w, b = self._fold(sd["fc.0.weight"], sd, "fc.1")
        b = b + sd["fc.0.bias"] * (sd["fc.1.weight"] / (sd["fc.1.running_var"] + BN_EPS).sqrt())
        P["fc"] = (self._t(w), self._t(b))
        H["fc"] = (self._f32(w, (1,) + tuple(w.shape)), self._f32(b))
        self.P = P
        self.H = H

    def _block(self, sd, key):
        torch = self.torch
        w1, b1 = self._fold(sd[key + ".conv1.conv.weight"], sd, key + ".conv1.bn")
        mid = w1.shape[0]
        branches = [[key + ".conv2a"]] + [[f"{key}.{br}.{d}" for d in range(depth)]
                                          for br, depth in (("conv2b", 2), ("conv2c", 3),
                                                            ("conv2d", 4))]
        layers = []   # depth d: the branches still running, 1x1 weights stacked, dw folded
        pw32 = []     # the same 1x1 weights as the HIP GEMM's float32 [groups][cout_g][k]
        for d in range(4):
            live = [br[d] for br in branches if len(br) > d]
            pw = torch.cat([sd[k + ".conv1.weight"] for k in live], 0)
            pw32.append(self._f32(pw, (1 if d == 0 else len(live), -1, mid)))
            dws, dbs = zip(*[self._fold(sd[k + ".conv2.weight"], sd, k + ".bn") for k in live])
            dw, db = torch.cat(dws, 0), torch.cat(dbs, 0)
            layers.append((len(live), self._t(pw), self._t(dw), self._t(db),
                           dw.reshape(-1).to(self.device, torch.float32).contiguous(),
                           db.to(self.device, torch.float32).contiguous()))
        g = (self._t(sd[key + ".gate.fc1.weight"].reshape(-1, mid)),
             self._t(sd[key + ".gate.fc1.bias"]),
             self._t(sd[key + ".gate.fc2.weight"].reshape(mid, -1)),
             self._t(sd[key + ".gate.fc2.bias"]))
        w3, b3 = self._fold(sd[key + ".conv3.conv.weight"], sd, key + ".conv3.bn")
        ds = None
        cout, cin = w3.shape[0], w1.shape[1]
        w3k, b3k = w3.reshape(cout, mid), b3
        if key + ".downsample.conv.weight" in sd:
            wd, bd = self._fold(sd[key + ".downsample.conv.weight"], sd, key + ".downsample.bn")
            ds = (self._t(wd), self._t(bd))
            # conv3(x2) + downsample(x): one GEMM over the concatenated inputs [x2; x]
            w3k, b3k = torch.cat([w3k, wd.reshape(cout, cin)], 1), b3 + bd
        hip = {"conv1": (self._f32(w1, (1, mid, cin)), self._f32(b1)),
               "layers": pw32,
               "conv3": (self._f32(w3k, (1,) + tuple(w3k.shape)), self._f32(b3k)),
               "cin": cin, "cout": cout, "hid": g[0].shape[0]}
        return ("os", mid, (self._t(w1), self._t(b1)), layers, g, (self._t(w3), self._t(b3)), ds,
                hip)

    # ---- forward
    def _os_block(self, x, blk):
        F = self.torch.nn.functional
        torch = self.torch
        _, mid, (w1, b1), layers, (g1w, g1b, g2w, g2b), (w3, b3), ds, _ = blk
        x1 = F.relu(F.conv2d(x, w1, b1))
        outs = []                       # branch outputs, finished at depths 1, 2, 3, 4
        y = None
        for d, (nlive, pw, dw, db, _, _) in enumerate(layers):
            inp = x1 if d == 0 else y[:, mid:]          # branches that go one layer deeper
            if d == 0:
                y = F.conv2d(inp, pw)                   # all four branches' first 1x1 at once
            else:
                y = F.conv2d(inp, pw, groups=nlive)     # one 1x1 per running branch
            y = F.relu(F.conv2d(y, dw, db, padding=1, groups=dw.shape[0]))
            outs.append(y[:, :mid])                     # the branch ending at this depth
        br = torch.stack(outs, 1)                       # (N, 4, mid, H, W)
        pooled = br.float().mean(dim=(3, 4)).to(br.dtype)          # (N, 4, mid)
        gate = torch.sigmoid(F.linear(F.relu(F.linear(pooled, g1w, g1b)), g2w, g2b))
        x2 = (br * gate[..., None, None]).sum(1)
        x2 = x2.contiguous(memory_format=self.fmt)
        x3 = F.conv2d(x2, w3, b3)
        idt = F.conv2d(x, ds[0], ds[1]) if ds is not None else x
        return F.relu(x3 + idt)

    # ---- the HIP forward (csrc/osnet.hip): every layer a kernel of ours
    def _pw(self, x1, w, bias=None, *, k1, G=1, cout_g, P, N, relu, x2=None, k2=0, res=None,
            out=None, x1s=None, x2s=None, ys=None):
        """1x1 convolution / linear layer through yta_osnet_pointwise.  x1s / x2s / ys: (sample,
        channel, pixel) element strides, default NCHW-contiguous."""
        from .. import _lib
        torch = self.torch
        if out is None:
            out = torch.empty((N, G * cout_g, P), dtype=self.dtype, device=self.device)
        a = _lib.PwArgs()
        a.x1 = x1.data_ptr()
        a.x1n, a.x1c, a.x1p = x1s or (G * k1 * P, P, 1)
        if x2 is not None:
            a.x2 = x2.data_ptr()
            a.x2n, a.x2c, a.x2p = x2s or (k2 * P, P, 1)
        a.w = w.data_ptr()
        a.bias = bias.data_ptr() if bias is not None else None
        if res is not None:
            a.res = res.data_ptr()
            a.rn, a.rc, a.rp = (G * cout_g * P, P, 1)
        a.y = out.data_ptr()
        a.yn, a.yc, a.yp = ys or (G * cout_g * P, P, 1)
        a.k1, a.k2, a.G, a.cout_g, a.P, a.N, a.relu = k1, k2, G, cout_g, P, N, int(relu)
        _lib.check(_lib.load_library().yta_osnet_pointwise(self._ctypes.byref(a), self._half,
                                                           self._stream()))
        return out

    def _stream(self):
        return self._ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _os_block_hip(self, x, blk):
        """One OSBlock: conv1 (GEMM + bias + ReLU); per depth the branches' 1x1s (one GEMM, grouped
        by branch after depth 0) and the depthwise 3x3 + bias + ReLU, which routes the branch
        ending at that depth into the (N, 4, mid, H, W) stack with its plane sums; the channel gate
        on those sums; the gated branch sum; conv3 and the downsample 1x1 as one GEMM over [x2; x]
        (or + x) with ReLU."""
        ctypes = self._ctypes
        from .. import _lib
        torch = self.torch
        lib = _lib.load_library()
        _, mid, _, layers, (g1w, g1b, g2w, g2b), _, ds, hp = blk
        n, cin, h, w = x.shape
        hw = h * w
        es = 2 if self._half else 4
        st = self._stream()
        w1, b1 = hp["conv1"]
        z = self._pw(x, w1, b1, k1=cin, cout_g=mid, P=hw, N=n, relu=True)
        stack = torch.empty((n, 4, mid, h, w), dtype=self.dtype, device=self.device)
        psum = torch.empty((n, 4, mid), dtype=torch.float32, device=self.device)
        for d, (nlive, _, _, _, dwf, dbf) in enumerate(layers):
            wd = hp["layers"][d]
            y = (self._pw(z, wd, k1=mid, cout_g=4 * mid, P=hw, N=n, relu=False) if d == 0 else
                 self._pw(z, wd, k1=mid, G=nlive, cout_g=mid, P=hw, N=n, relu=False))
            rest = (torch.empty((n, (nlive - 1) * mid, h, w), dtype=self.dtype, device=self.device)
                    if nlive > 1 else None)
            _lib.check(lib.yta_osnet_dw3x3(
                ctypes.c_void_p(y.data_ptr()), nlive * mid * hw, hw,
                ctypes.c_void_p(dwf.data_ptr()), ctypes.c_void_p(dbf.data_ptr()), n, nlive * mid,
                h, w, self._half, ctypes.c_void_p(stack.data_ptr() + d * mid * hw * es),
                4 * mid * hw, mid, ctypes.c_void_p(rest.data_ptr()) if rest is not None else None,
                (nlive - 1) * mid * hw, ctypes.c_void_p(psum.data_ptr() + d * mid * 4), 4 * mid,
                st))
            z = rest
        gate = torch.empty((n, 4, mid), dtype=self.dtype, device=self.device)
        _lib.check(lib.yta_osnet_gate(ctypes.c_void_p(psum.data_ptr()), n, mid, hp["hid"], hw,
                                      ctypes.c_void_p(g1w.data_ptr()), ctypes.c_void_p(g1b.data_ptr()),
                                      ctypes.c_void_p(g2w.data_ptr()), ctypes.c_void_p(g2b.data_ptr()),
                                      self._half, ctypes.c_void_p(gate.data_ptr()), st))
        x2 = torch.empty((n, mid, h, w), dtype=self.dtype, device=self.device)
        _lib.check(lib.yta_osnet_gate_sum(ctypes.c_void_p(stack.data_ptr()),
                                          ctypes.c_void_p(gate.data_ptr()), n, mid, hw, self._half,
                                          ctypes.c_void_p(x2.data_ptr()), st))
        w3, b3 = hp["conv3"]
        cout = hp["cout"]
        if ds is not None:
            out = self._pw(x2, w3, b3, k1=mid, cout_g=cout, P=hw, N=n, relu=True, x2=x, k2=cin)
        else:
            out = self._pw(x2, w3, b3, k1=mid, cout_g=cout, P=hw, N=n, relu=True, res=x)
        return out.view(n, cout, h, w)

    def _pool(self, x, kind):
        from .. import _lib
        torch = self.torch
        n, c, h, w = x.shape
        if kind == 0:
            out = torch.empty((n, c, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=self.dtype,
                              device=self.device)
        elif kind == 1:
            out = torch.empty((n, c, h // 2, w // 2), dtype=self.dtype, device=self.device)
        else:
            out = torch.empty((n, c), dtype=self.dtype, device=self.device)
        _lib.check(_lib.load_library().yta_osnet_pool(
            self._ctypes.c_void_p(x.data_ptr()), n, c, h, w, kind, self._half,
            self._ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def _forward_hip(self, crops):
        import ctypes
        from .. import _lib
        torch = self.torch
        self._ctypes = ctypes
        self._half = int(self.dtype == torch.float16)
        x = crops.to(self.device, self.dtype).contiguous()
        n, _, H, W = x.shape
        ws, bs = self.H["stem"]
        c0 = ws.shape[0]
        stem = torch.empty((n, c0, (H - 1) // 2 + 1, (W - 1) // 2 + 1), dtype=self.dtype,
                           device=self.device)
        _lib.check(_lib.load_library().yta_osnet_stem(
            ctypes.c_void_p(x.data_ptr()), n, H, W, ctypes.c_void_p(ws.data_ptr()),
            ctypes.c_void_p(bs.data_ptr()), c0, self._half, ctypes.c_void_p(stem.data_ptr()),
            self._stream()))
        x = self._pool(stem, 0)
        for blk in self.blocks:
            if blk[0] == "reduce":
                _, _, _, wr, br = blk
                c, h, w = x.shape[1], x.shape[2], x.shape[3]
                y = self._pw(x, wr, br, k1=c, cout_g=wr.shape[2], P=h * w, N=n, relu=True)
                x = self._pool(y.view(n, wr.shape[2], h, w), 1)
            else:
                x = self._os_block_hip(x, blk)
        w5, b5 = self.H["conv5"]
        c, h, w = x.shape[1], x.shape[2], x.shape[3]
        y = self._pw(x, w5, b5, k1=c, cout_g=w5.shape[2], P=h * w, N=n, relu=True)
        v = self._pool(y.view(n, w5.shape[2], h, w), 2)                 # (n, C) means
        wf, bf = self.H["fc"]
        feat = torch.empty((n, wf.shape[2]), dtype=self.dtype, device=self.device)
        # the fc as a GEMM over the crops: one "sample", the crops on the pixel axis
        self._pw(v, wf, bf, k1=c, cout_g=wf.shape[2], P=n, N=1, relu=True, x1s=(0, 1, c),
                 ys=(0, 1, wf.shape[2]), out=feat)
        return feat

    def __call__(self, crops):
        torch = self.torch
        with torch.no_grad():
            n = crops.shape[0]
            if n <= self.chunk:
                return self._forward(crops)
            return torch.cat([self._forward(crops[i:i + self.chunk])
                              for i in range(0, n, self.chunk)])

    def _forward(self, crops):
        if self.hip:
            return self._forward_hip(crops)
        torch = self.torch
        F = torch.nn.functional
        x = crops.to(self.device, self.dtype).contiguous(memory_format=self.fmt)
        w, b = self.P["stem"]
        x = F.relu(F.conv2d(x, w, b, stride=2, padding=3))
        x = F.max_pool2d(x, 3, stride=2, padding=1)
        for blk in self.blocks:
            if blk[0] == "reduce":
                x = F.avg_pool2d(F.relu(F.conv2d(x, blk[1], blk[2])), 2, stride=2)
            else:
                x = self._os_block(x, blk)
        w, b = self.P["conv5"]
        x = F.relu(F.conv2d(x, w, b))
        v = x.float().mean(dim=(2, 3)).to(self.dtype)
        w, b = self.P["fc"]
        return F.relu(F.linear(v, w, b))
