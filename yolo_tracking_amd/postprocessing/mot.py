"""MOT-challenge result rows (examples/utils.py:8-28, write_mot_results)."""
from pathlib import Path

import numpy as np


def write_mot_results(txt_path, results, frame_idx):
    """Append one frame of tracker output to a MOT text file: frame_idx + 1, id, left, top, width,
    height, conf, cls, -1, every value written with '%d' (examples/utils.py:8-28).

    `results` is either the (K, 8) array tracker.update() returns ([x1, y1, x2, y2, id, conf,
    cls, det_ind]) or an ultralytics-style Results object with boxes.{xyxy, id, conf, cls}."""
    if hasattr(results, "boxes"):
        b = results.boxes
        xyxy = np.asarray(b.xyxy, dtype=np.float64).reshape(-1, 4)
        ids = np.asarray(b.id, dtype=np.float64).reshape(-1)
        conf = np.asarray(b.conf, dtype=np.float64).reshape(-1)
        cls = np.asarray(b.cls, dtype=np.float64).reshape(-1)
    else:
        r = np.asarray(results, dtype=np.float64).reshape(-1, 8)
        xyxy, ids, conf, cls = r[:, :4], r[:, 4], r[:, 5], r[:, 6]
    n = len(ids)
    ltwh = np.concatenate([xyxy[:, :2], xyxy[:, 2:4] - xyxy[:, :2]], axis=1)   # ops.xyxy2ltwh
    mot = np.concatenate([np.full((n, 1), frame_idx + 1, dtype=np.float64), ids[:, None], ltwh,
                          conf[:, None], cls[:, None], np.full((n, 1), -1.0)], axis=1)
    txt_path = Path(txt_path)
    txt_path.parent.mkdir(parents=True, exist_ok=True)
    txt_path.touch(exist_ok=True)
    with open(str(txt_path), 'ab+') as f:
        np.savetxt(f, mot, fmt='%d')
