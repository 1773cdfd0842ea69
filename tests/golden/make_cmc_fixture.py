"""Make tests/golden/cmc_mot17.npz (container-only): the MOT17-mini frames of a few sequences
(assets/MOT17-mini/train/*/img1/*.jpg, the reference's own test data), decoded with PIL and
reduced by the restated SparseOptFlow preprocess (gray + 0.1 resize, oracle/cmc_sof.py) to the
small gray frames the estimator works on.  Inputs only: the expected outputs are computed from
the oracle at test time."""
import os
import sys

import numpy as np
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import cmc_sof as cs  # noqa: E402

ROOT = "/root/reference/assets/MOT17-mini/train"


def main():
    out = {}
    for seq in ("MOT17-04-FRCNN", "MOT17-05-FRCNN", "MOT17-13-FRCNN"):
        d = os.path.join(ROOT, seq, "img1")
        small = []
        for f in sorted(os.listdir(d)):
            rgb = np.asarray(Image.open(os.path.join(d, f)).convert("RGB"))
            small.append(cs.preprocess(np.ascontiguousarray(rgb[..., ::-1]), 0.1))
        key = seq.rsplit("-", 1)[0].replace("-", "_")
        out[f"{key}__small"] = np.stack(small)
        print(key, out[f"{key}__small"].shape)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "cmc_mot17.npz"),
                        **out)


if __name__ == "__main__":
    main()
