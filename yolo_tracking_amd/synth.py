"""Seeded synthetic detection streams (SURVEY.md §8(d) generator spec).

One `SyntheticStream` = one video stream: N objects on a C x C canvas (C = 64*sqrt(N) px) moving
with constant velocity plus jitter, wrap-around at the canvas edge, 2 % per-frame turnover (respawn
at a random position -> births, losses, re-identifications), single class.  Each frame yields
`dets` (M, 6) float64 `[x1, y1, x2, y2, conf, cls]` in a shuffled order (so `det_ind` is
exercised) and optionally (M, D) float32 embeddings that drift slowly per object.

The reference has no such generator (it benchmarks nothing); this is the build's own workload
definition, shared by `bench.py` and the parity tests.
"""
import numpy as np


class SyntheticStream:
    def __init__(self, n_objects, seed, low_conf_frac=0.1, emb_dim=0, turnover=0.02,
                 speed_sigma=1.5, jitter_sigma=0.5, shuffle=True, canvas=None, drop_frac=0.0, n_classes=1):
        self.n = int(n_objects)
        self.rng = np.random.default_rng(seed)
        self.canvas = float(canvas) if canvas else 64.0 * np.sqrt(max(self.n, 1))
        self.low_conf_frac = float(low_conf_frac)
        self.emb_dim = int(emb_dim)
        self.turnover = float(turnover)
        self.speed_sigma = float(speed_sigma)
        self.jitter_sigma = float(jitter_sigma)
        self.shuffle = shuffle
        self.drop_frac = float(drop_frac)   # missed detections per frame (drawn last, so 0 keeps
                                            # every other draw of the stream unchanged)
        self.n_classes = int(n_classes)     # object k has class k % n_classes (no draw)
        r = self.rng
        self.wh = r.uniform(16.0, 64.0, size=(self.n, 2))
        self.ctr = r.uniform(0.0, self.canvas, size=(self.n, 2))
        self.vel = r.normal(0.0, self.speed_sigma, size=(self.n, 2))
        self.emb = (r.standard_normal((self.n, self.emb_dim)).astype(np.float32)
                    if self.emb_dim else None)
        self.frame = 0

    @property
    def img_shape(self):
        c = int(np.ceil(self.canvas))
        return (c, c, 3)

    def _respawn(self, idx):
        r = self.rng
        k = len(idx)
        self.wh[idx] = r.uniform(16.0, 64.0, size=(k, 2))
        self.ctr[idx] = r.uniform(0.0, self.canvas, size=(k, 2))
        self.vel[idx] = r.normal(0.0, self.speed_sigma, size=(k, 2))
        if self.emb is not None:
            self.emb[idx] = r.standard_normal((k, self.emb_dim)).astype(np.float32)

    def next_frame(self):
        """Advance one frame; returns (dets float64 (M,6), embs float32 (M,D) or None)."""
        r = self.rng
        if self.frame > 0:
            self.ctr = np.mod(self.ctr + self.vel, self.canvas)
            turn = np.nonzero(r.random(self.n) < self.turnover)[0]
            if len(turn):
                self._respawn(turn)
            if self.emb is not None:
                self.emb += r.normal(0.0, 0.05, size=self.emb.shape).astype(np.float32)
        self.frame += 1
        half = self.wh / 2.0
        box = np.concatenate([self.ctr - half, self.ctr + half], axis=1)
        box = box + r.normal(0.0, self.jitter_sigma, size=box.shape)
        low = r.random(self.n) < self.low_conf_frac
        conf = np.where(low, r.uniform(0.11, 0.49, size=self.n), r.uniform(0.51, 0.99, size=self.n))
        dets = np.empty((self.n, 6), dtype=np.float64)
        dets[:, :4] = box
        dets[:, 4] = conf
        dets[:, 5] = (np.arange(self.n) % self.n_classes).astype(np.float64)
        order = r.permutation(self.n) if self.shuffle else np.arange(self.n)
        if self.drop_frac > 0:
            order = order[r.random(self.n) >= self.drop_frac]
        dets = dets[order]
        embs = self.emb[order].copy() if self.emb is not None else None
        return dets, embs


def make_frames(n_objects, n_frames, seed, **kw):
    """Materialise a stream: list of (dets, embs)."""
    s = SyntheticStream(n_objects, seed, **kw)
    return [s.next_frame() for _ in range(n_frames)]
