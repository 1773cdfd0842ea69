"""Make tests/golden/osnet_x0_25.npz (container-only): the reference's OSNet x0.25
(boxmot/appearance/backbones/osnet.py, loaded from its file; it imports only torch) built with
random weights and randomised BatchNorm statistics (seeded), in eval mode, run on seeded inputs.
Stores the state_dict (reference key names, float32) and the features; the inputs are regenerated
from the seed at test time (np.random.default_rng(INPUT_SEED)).  The reference cannot download
pretrained weights here (no network), so parity is pinned on these random-weight vectors."""
import importlib.util
import os

import numpy as np
import torch

REF = "/root/reference/boxmot/appearance/backbones/osnet.py"
INPUT_SEED = 20261016
N_IN = 4


def main():
    spec = importlib.util.spec_from_file_location("ref_osnet", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(7)
    net = mod.osnet_x0_25(num_classes=751, pretrained=False)
    g = torch.Generator().manual_seed(8)
    with torch.no_grad():
        for m in net.modules():   # non-trivial BN statistics so folding is exercised
            if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm1d)):
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) * 0.5 + 0.75)
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) * 0.5 + 0.75)
                m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
            if isinstance(m, torch.nn.Conv2d) and m.bias is not None:
                m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
    net.eval()
    x = np.random.default_rng(INPUT_SEED).standard_normal((N_IN, 3, 256, 128)).astype(np.float32)
    with torch.no_grad():
        y = net(torch.from_numpy(x)).numpy()
    out = {"sd__" + k: v.detach().numpy() for k, v in net.state_dict().items()
           if v.dtype.is_floating_point and not k.startswith("classifier.")}
    out["features"] = y.astype(np.float32)
    out["input_seed"] = np.array(INPUT_SEED)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                     "osnet_x0_25.npz"), **out)
    print("features", y.shape, "params", sum(v.size for k, v in out.items() if k.startswith("sd__")))


if __name__ == "__main__":
    main()
