"""ORACLE — test infrastructure only.  CPU restatement of HybridSORT.update()
(boxmot/trackers/hybridsort/hybridsort.py:329-570) with its Kalman filter
(boxmot/motion/kalman_filters/hybridsort_kf.py: predict :339-380, freeze :383-387, unfreeze
:390-436, update :439-528) and its association (boxmot/trackers/hybridsort/association.py:
300-335 linear_assignment / cost_vel, :338-383 corner directions, :44-54 score differences,
:495-581 associate_4_points_with_score_with_reid, :667-684 embedding_distance).

The reference's live configuration (hybridsort.py:346-360, hard-wired): TCM_first_step with weight
0, EG_weight_high_score 1.3, long-term ReID with weight 0 (its correction uses the short-term
embedding cost), correction threshold 0.4, use_byte False (hybridsort.yaml), ECC off.

Reference behaviour kept on purpose:
  * dets0 = [x1, y1, x2, y2, conf, cls, conf]: the tracker's det_ind is the detection's score, and
    dets0 rows are indexed with positions in the *filtered* detection list (:464, :534-536, :549)
  * convert_bbox_to_z makes a 5-vector (x, y, s, score, r) (the score is never 0 for kept rows)
  * unfreeze unpacks the stored (x, y, s, c, r) as (x, y, s, r, c): w = sqrt(s c), h = sqrt(s / c),
    and replays (x, y, w h, w / h, interpolated r)
  * corner velocities sum the directions from every stored observation within delta_t (no
    break, :244-258); the 4 corner angle costs are summed
  * the first-round LAP has no cost limit and no fast path; a matched pair is dropped only when
    emb > 0.4 and iou - |kalman score - det score| < iou_threshold
  * ids from a counter reset at construction (count = 0, :361), reported as id + 1 (:563)
  * embeddings are float32 (update_features: feat /= |feat| in place, EMA with alpha 0.8, then
    smooth /= |smooth|); a birth's row is normalised twice (feat is smooth_feat)
The long-term feature bank (deque of 30) only enters the cost multiplied by
longterm_reid_weight = 0 and is not kept (the product adds exactly +0.0 to every finite cost).
"""
import numpy as np
from scipy.spatial.distance import cdist

from . import geometry
from .lap import linear_assignment_padded

ASSO = {"iou": geometry.iou_batch, "giou": geometry.giou_batch, "diou": geometry.diou_batch,
        "ciou": geometry.ciou_batch}

_F9 = np.eye(9, dtype=np.int64)
for _i in range(4):
    _F9[_i, 5 + _i] = 1                     # hybridsort.py:134-142 (an int array, as the reference)
_H9 = np.eye(5, 9, dtype=np.int64)          # :143-147


def bbox_to_z(b):
    """hybridsort.py:33-49 (x, y, s, score, r) — callers only pass rows with a non-zero score."""
    w = b[2] - b[0]
    h = b[3] - b[1]
    x = b[0] + w / 2.0
    y = b[1] + h / 2.0
    s = w * h
    r = w / float(h + 1e-6)
    score = b[4]
    assert score, "a zero score makes a 4-vector the 5-d filter rejects"
    return np.array([x, y, s, score, r]).reshape((5, 1))


def x_to_bbox(x):
    """hybridsort.py:52-63 with the score column."""
    w = np.sqrt(x[2] * x[4])
    h = x[2] / w
    return np.array([x[0] - w / 2.0, x[1] - h / 2.0, x[0] + w / 2.0, x[1] + h / 2.0,
                     x[3]]).reshape((1, 5))


def _dir(p1, p2):
    """speed_direction_{lt,rt,lb,rb} (hybridsort.py:74-103) on chosen corner coordinates."""
    cx1, cy1 = p1
    cx2, cy2 = p2
    speed = np.array([cy2 - cy1, cx2 - cx1])
    norm = np.sqrt((cy2 - cy1) ** 2 + (cx2 - cx1) ** 2) + 1e-6
    return speed / norm


CORNERS = ((0, 1), (0, 3), (2, 1), (2, 3))   # lt, rt, lb, rb: (x column, y column)


class KF9:
    """The HybridSORT filter: x (9,1), P (9,9); Q, R, P0 as hybridsort.py:149-154."""

    def __init__(self, z):
        self.x = np.zeros((9, 1))
        self.x[:5] = z
        self.P = np.eye(9)
        self.P[5:, 5:] *= 1000.0
        self.P *= 10.0
        self.Q = np.eye(9)
        self.Q[-1, -1] *= 0.01
        self.Q[-2, -2] *= 0.01
        self.Q[5:, 5:] *= 0.01
        self.R = np.eye(5)
        self.R[2:, 2:] *= 10.0
        self.history = []          # history_obs: z or None per update call
        self.saved = None          # attr_saved: (x, P, history, attr_saved) at the freeze
        self.observed = False

    def predict(self):
        """hybridsort_kf.py:339-380 (alpha_sq = 1, no control input)."""
        self.x = np.dot(_F9, self.x)
        self.P = 1.0 * np.dot(np.dot(_F9, self.P), _F9.T) + self.Q

    def _correct(self, z):
        """hybridsort_kf.py:492-528: y, S, inv(S), K, x, Joseph-form P."""
        y = z - np.dot(_H9, self.x)
        PHT = np.dot(self.P, _H9.T)
        S = np.dot(_H9, PHT) + self.R
        K = np.dot(PHT, np.linalg.inv(S))
        self.x = self.x + np.dot(K, y)
        I_KH = np.eye(9) - np.dot(K, _H9)
        self.P = np.dot(np.dot(I_KH, self.P), I_KH.T) + np.dot(np.dot(K, self.R), K.T)

    def update(self, z):
        """hybridsort_kf.py:439-490 incl. freeze (:383-387) and unfreeze (:390-436)."""
        self.history.append(z)
        if z is None:
            if self.observed:
                self.saved = (self.x.copy(), self.P.copy(), list(self.history), self.saved)
            self.observed = False
            return
        if not self.observed:
            self._unfreeze()
        self.observed = True
        self._correct(z)

    def _unfreeze(self):
        if self.saved is None:
            return
        new_history = list(self.history)
        x, P, hist, older = self.saved
        self.x, self.P, self.saved, self.observed = x.copy(), P.copy(), older, True
        self.history = hist[:-1]
        idx = [k for k, d in enumerate(new_history) if d is not None]
        i1, i2 = idx[-2], idx[-1]
        x1, y1, s1, r1, c1 = new_history[i1]          # (x, y, s, c, r) read as (x, y, s, r, c)
        w1, h1 = np.sqrt(s1 * r1), np.sqrt(s1 / r1)
        x2, y2, s2, r2, c2 = new_history[i2]
        w2, h2 = np.sqrt(s2 * r2), np.sqrt(s2 / r2)
        gap = i2 - i1
        dx, dy, dw, dh = (x2 - x1) / gap, (y2 - y1) / gap, (w2 - w1) / gap, (h2 - h1) / gap
        dc = (c2 - c1) / gap
        for i in range(gap):
            x = x1 + (i + 1) * dx
            y = y1 + (i + 1) * dy
            w = w1 + (i + 1) * dw
            h = h1 + (i + 1) * dh
            c = c1 + (i + 1) * dc
            self.update(np.array([x, y, w * h, w / float(h), c]).reshape((5, 1)))
            if i != gap - 1:
                self.predict()


def _normalise(v):
    """`v /= np.linalg.norm(v)` on a float32 row (returns the same object, as in place)."""
    v /= np.linalg.norm(v)
    return v


class Tracker9:
    """KalmanBoxTracker (hybridsort.py:106-326), adapfs off."""

    def __init__(self, bbox, cls, det_ind, feat, tid, delta_t):
        self.kf = KF9(bbox_to_z(bbox))
        self.tsu = 0
        self.id = tid
        self.hits = self.hit_streak = self.age = 0
        self.conf, self.cls, self.det_ind = bbox[4], cls, det_ind
        self.last_obs = np.array([-1, -1, -1, -1, -1])
        self.obs = {}
        self.vel = None            # 4 corner directions (lt, rt, lb, rb), each (2,)
        self.delta_t = delta_t
        self.confidence_pre = None
        self.confidence = bbox[4]
        self.smooth_feat = None
        self.update_features(feat)

    def update_features(self, feat):
        """:197-214 (adapfs False, alpha 0.8); feat is the caller's float32 row, modified in
        place as the reference does."""
        feat = _normalise(feat)
        if self.smooth_feat is None:
            self.smooth_feat = feat
        else:
            self.smooth_feat = 0.8 * self.smooth_feat + (1 - 0.8) * feat
        self.smooth_feat /= np.linalg.norm(self.smooth_feat)

    def update(self, bbox, cls, det_ind, feat, update_feature=True):
        """:230-294."""
        if bbox is None:
            self.kf.update(None)
            self.confidence_pre = None
            return
        self.conf, self.cls, self.det_ind = bbox[-1], cls, det_ind
        if self.last_obs.sum() >= 0:
            acc = None
            for i in range(self.delta_t):
                if self.age - i - 1 in self.obs:
                    prev = self.obs[self.age - i - 1]
                    d = [_dir((prev[cx], prev[cy]), (bbox[cx], bbox[cy])) for cx, cy in CORNERS]
                    if acc is None:
                        acc = d
                    else:
                        acc = [a + b for a, b in zip(acc, d)]
            if acc is None:
                prev = self.last_obs
                acc = [_dir((prev[cx], prev[cy]), (bbox[cx], bbox[cy])) for cx, cy in CORNERS]
            self.vel = acc
        self.last_obs = bbox
        self.obs[self.age] = bbox
        self.tsu = 0
        self.hits += 1
        self.hit_streak += 1
        self.kf.update(bbox_to_z(bbox))
        if update_feature:
            self.update_features(feat)
        self.confidence_pre = self.confidence
        self.confidence = bbox[4]

    def predict(self, track_thresh=0.6):
        """:296-320 -> (box+score (1,5), kalman score, simple score)."""
        if (self.kf.x[7] + self.kf.x[2]) <= 0:
            self.kf.x[7] *= 0.0
        self.kf.predict()
        self.age += 1
        if self.tsu > 0:
            self.hit_streak = 0
        self.tsu += 1
        b = x_to_bbox(self.kf.x)
        ks = np.clip(self.kf.x[3], track_thresh, 1.0)
        if not self.confidence_pre:
            ss = np.clip(self.confidence, 0.1, track_thresh)
        else:
            ss = np.clip(self.confidence - (self.confidence_pre - self.confidence), 0.1,
                         track_thresh)
        return b, ks, ss

    def k_previous_obs(self):
        """hybridsort.py:22-30."""
        if not self.obs:
            return [-1, -1, -1, -1, -1]
        for i in range(self.delta_t):
            if self.age - (self.delta_t - i) in self.obs:
                return self.obs[self.age - (self.delta_t - i)]
        return self.obs[max(self.obs.keys())]


def embedding_distance(tf, df):
    """association.py:667-684."""
    c = np.zeros((len(tf), len(df)), dtype=np.float64)
    if c.size == 0:
        return c
    return np.maximum(0.0, cdist(tf, df, "cosine"))


def cost_vel(Y, X, vel, dets, prev_obs, vdc_weight, n_trk):
    """association.py:314-335."""
    iy = np.repeat(vel[:, 0][:, np.newaxis], Y.shape[1], axis=1)
    ix = np.repeat(vel[:, 1][:, np.newaxis], X.shape[1], axis=1)
    cos = np.clip(ix * X + iy * Y, a_min=-1, a_max=1)
    ang = (np.pi / 2.0 - np.abs(np.arccos(cos))) / np.pi
    valid = np.ones(prev_obs.shape[0])
    valid[np.where(prev_obs[:, 4] < 0)] = 0
    scores = np.repeat(dets[:, -1][:, np.newaxis], n_trk, axis=1)
    valid = np.repeat(valid[:, np.newaxis], X.shape[1], axis=1)
    return (((valid * ang) * vdc_weight).T) * scores


def corner_dirs(dets, prev_obs, cx, cy):
    """speed_direction_batch_{lt,rt,lb,rb} (association.py:338-383): (dy, dx), tracks x dets."""
    t = prev_obs[..., np.newaxis]
    dx = dets[:, cx] - t[:, cx]
    dy = dets[:, cy] - t[:, cy]
    norm = np.sqrt(dx ** 2 + dy ** 2) + 1e-6
    return dy / norm, dx / norm


def associate_reid(dets, trks, func, thr, vels, prev_obs, inertia, emb_cost, w_emb=1.3,
                   corr_thresh=0.4):
    """associate_4_points_with_score_with_reid (association.py:495-581) as HybridSORT calls it
    (TCM weight 0, weights (1.0, 1.3), long-term weight 0, correction on)."""
    if len(trks) == 0:
        return np.empty((0, 2), dtype=int), np.arange(len(dets)), np.empty((0, 5), dtype=int)
    costs = []
    for k, (cx, cy) in enumerate(CORNERS):
        Y, X = corner_dirs(dets, prev_obs, cx, cy)
        costs.append(cost_vel(Y, X, vels[k], dets, prev_obs, inertia, trks.shape[0]))
    iou = func(dets, trks)
    score_dif = np.abs(trks[np.newaxis, :, 4] - dets[:, np.newaxis, 4])
    angle = costs[0] + costs[1] + costs[2] + costs[3]
    angle -= score_dif * 0
    if min(iou.shape) > 0:
        matched = linear_assignment_padded(1.0 * (-(iou + angle)) + w_emb * emb_cost + 0.0)
        if matched.size == 0:
            matched = np.empty(shape=(0, 2))
    else:
        matched = np.empty(shape=(0, 2))
    u_det = [d for d in range(len(dets)) if d not in matched[:, 0]]
    u_trk = [t for t in range(len(trks)) if t not in matched[:, 1]]
    thre = iou - score_dif
    matches = []
    for m in matched:
        if emb_cost[m[0], m[1]] > corr_thresh and thre[m[0], m[1]] < thr:
            u_det.append(m[0])
            u_trk.append(m[1])
        else:
            matches.append(m.reshape(1, 2))
    matches = np.concatenate(matches, axis=0) if matches else np.empty((0, 2), dtype=int)
    return matches, np.array(u_det), np.array(u_trk)


class HybridSortOracle:
    """HybridSORT.update without the PerClassDecorator (see per_class_update)."""

    def __init__(self, det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
                 asso_func="giou", inertia=0.2):
        self.max_age, self.min_hits, self.thr = max_age, min_hits, iou_threshold
        self.trackers = []
        self.frame_count = 0
        self.det_thresh, self.delta_t, self.inertia = det_thresh, delta_t, inertia
        self.func = ASSO[asso_func]
        self.count = 0                                           # :361

    def update(self, dets, feats):
        """dets (M, 6) [x1, y1, x2, y2, conf, cls]; feats: get_features' (M, D) float32 rows
        for every detection (reid_multibackend.py:310 global norm already applied)."""
        self.frame_count += 1
        scores = dets[:, 4]
        dets_embs = np.array(feats, dtype=np.float32)
        if dets_embs.ndim != 2:
            dets_embs = dets_embs.reshape(len(dets), -1)
        dets0 = np.concatenate((dets, np.expand_dims(scores, axis=-1)), axis=1)
        dets5 = np.concatenate((dets[:, :4], np.expand_dims(scores, axis=-1)), axis=1)
        remain = scores > self.det_thresh
        dets5 = dets5[remain]
        feat_keep = dets_embs[remain]
        trks = np.zeros((len(self.trackers), 8))
        to_del = []
        for k in range(len(trks)):
            pos, ks, ss = self.trackers[k].predict()
            trks[k, :6] = [pos[0][0], pos[0][1], pos[0][2], pos[0][3], ks[0], ss]
            if np.any(np.isnan(pos)):
                to_del.append(k)
        assert np.isfinite(np.delete(trks, to_del, axis=0)).all(), \
            "an infinite predicted box without NaN misaligns trks and trackers in the reference"
        trks = np.ma.compress_rows(np.ma.masked_invalid(trks))
        for k in reversed(to_del):
            self.trackers.pop(k)
        vels = [np.array([t.vel[c] if t.vel is not None else np.array((0, 0))
                          for t in self.trackers]) for c in range(4)]
        last_boxes = np.array([t.last_obs for t in self.trackers])
        k_obs = np.array([t.k_previous_obs() for t in self.trackers])
        tf = np.asarray([t.smooth_feat for t in self.trackers], dtype=np.float64)
        emb = embedding_distance(tf, feat_keep).T
        if len(self.trackers):
            vels = [v.reshape(len(self.trackers), 2) for v in vels]
        matched, u_det, u_trk = associate_reid(dets5, trks, self.func, self.thr, vels, k_obs,
                                               self.inertia, emb)
        for m in matched:
            self.trackers[m[1]].update(dets5[m[0], :], dets0[m[0], 5], dets0[m[0], 6],
                                       feat_keep[m[0], :])
        if u_det.shape[0] > 0 and u_trk.shape[0] > 0:
            iou_left = np.array(self.func(dets5[u_det], last_boxes[u_trk]))
            if iou_left.max() > self.thr:
                rd, rt = [], []
                for m in linear_assignment_padded(-iou_left):
                    di, ti = u_det[m[0]], u_trk[m[1]]
                    if iou_left[m[0], m[1]] < self.thr:
                        continue
                    self.trackers[ti].update(dets5[di, :], dets0[di, 5], dets0[di, 6],
                                             feat_keep[di, :], update_feature=False)
                    rd.append(di)
                    rt.append(ti)
                u_det = np.setdiff1d(u_det, np.array(rd))
                u_trk = np.setdiff1d(u_trk, np.array(rt))
        for k in u_trk:
            self.trackers[k].update(None, None, None, None)
        for i in u_det:
            self.trackers.append(Tracker9(dets5[i, :], dets0[i, 5], dets0[i, 6], feat_keep[i, :],
                                          self.count, self.delta_t))
            self.count += 1
        ret = []
        i = len(self.trackers)
        for t in reversed(self.trackers):
            d = x_to_bbox(t.kf.x)[0][:4] if t.last_obs.sum() < 0 else t.last_obs[:4]
            if t.tsu < 1 and (t.hit_streak >= self.min_hits or self.frame_count <= self.min_hits):
                ret.append(np.concatenate((d, [t.id + 1], [t.conf], [t.cls], [t.det_ind]))
                           .reshape(1, -1))
            i -= 1
            if t.tsu > self.max_age:
                self.trackers.pop(i)
        if ret:
            return np.concatenate(ret)
        return np.empty((0, 7))


def get_features_norm(raw):
    """The reference ReID's last step (reid_multibackend.py:310): the (n, D) rows divided by their
    global Frobenius norm."""
    raw = np.asarray(raw, dtype=np.float32)
    if raw.size == 0:
        return raw.reshape(0, raw.shape[-1] if raw.ndim == 2 else 0)
    return raw / np.linalg.norm(raw)


def per_class_update(tracker, dets, raw, get_features=get_features_norm):
    """PerClassDecorator (boxmot/utils/__init__.py:22-61) around HybridSortOracle.update: one call
    per class of the union of active and detected classes, in the iteration order of that Python
    set, each with the get_features output of its own rows; every call predicts all trackers."""
    raw = np.asarray(raw, dtype=np.float32)
    if raw.ndim != 2:
        raw = raw.reshape(len(dets), -1)
    if dets.size == 0:
        return tracker.update(dets, get_features(raw))
    dets_dict = {c: np.array([d for d in dets if d[5] == c]) for c in set(d[5] for d in dets)}
    rows = {c: [k for k, d in enumerate(dets) if d[5] == c] for c in dets_dict}
    relevant = set([t.cls for t in tracker.trackers]).union(set(dets_dict.keys()))
    mc = np.empty(shape=(0, 8))
    for c in relevant:
        d = np.array(dets_dict.get(int(c), np.empty((0, 6))))
        f = get_features(raw[rows.get(int(c), [])])
        out = tracker.update(d, f)
        if out.size != 0:
            mc = np.append(mc, out, axis=0)
    return mc
