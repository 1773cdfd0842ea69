"""ORACLE — test infrastructure only.  CPU restatement of DeepOCSort.update()
(boxmot/trackers/deepocsort/deep_ocsort.py:357-520) with its Kalman filter
(boxmot/motion/kalman_filters/deepocsort_kf.py: predict :340-379, freeze :381-385,
apply_affine_correction :387-431, unfreeze :433-478, update :480-580) and the embedding-aware
association (boxmot/utils/association.py:79-201).

Only the "new KF" path is live in the reference (new_kf_off=False; the other branch names an
undefined OCSortKalmanFilterAdapter, deep_ocsort.py:141): state (x, y, w, h, x', y', w', h'),
Q = diag((w/20)^2, (h/20)^2, (w/20)^2, (h/20)^2, (w/160)^2, ...) from the current w, h at every
predict, R = diag((w/20)^2, (h/20)^2, ...) from the predicted w, h at every update, P0 = Q(w, h)
with the position block x4 and the velocity block x100.

Reference behaviour kept on purpose:
  * the observation-centric replay (unfreeze) reads the stored (x, y, w, h) measurement as
    (x, y, s, r) (w1 = sqrt(s1 r1), h1 = sqrt(s1 / r1)) and runs with the filter's default R = I
    and Q = I (its recursive update / predict pass neither)
  * camera-motion correction (CMC) corrects last_observation in place when its sum is > 0, then
    every stored observation whose age is within delta_t of the current one; last_observation is
    the same array as the newest stored observation, which is then corrected twice
  * embeddings: the tracker's embedding stays float32 until its first update_emb, which promotes
    it to float64 (alpha is a NumPy float64, NumPy 2 promotion rules); the stage-1 cost is
    dets_embs @ trk_embs.T in the dtype of that stack
  * ids start at 1 (KalmanBoxTracker.count = 1, :347) and are reported as is (:513)
"""
import numpy as np

from .lap import linear_assignment_padded
from .ocsort import ASSO, _asso, speed_direction

_F8 = np.eye(8, dtype=np.int64)
for _i in range(4):
    _F8[_i, 4 + _i] = 1                     # deep_ocsort.py:119-130
_H8 = np.eye(4, 8, dtype=np.int64)          # :131-138


def bbox_to_z_new(b):
    """deep_ocsort.py:42-47."""
    w = b[2] - b[0]
    h = b[3] - b[1]
    return np.array([b[0] + w / 2.0, b[1] + h / 2.0, w, h]).reshape((4, 1))


def x_to_bbox_new(x):
    """deep_ocsort.py:50-52."""
    x, y, w, h = x.reshape(-1)[:4]
    return np.array([x - w / 2, y - h / 2, x + w / 2, y + h / 2]).reshape(1, 4)


def process_noise(w, h, p=1 / 20, v=1 / 160):
    """deep_ocsort.py:76-80."""
    return np.diag(((p * w) ** 2, (p * h) ** 2, (p * w) ** 2, (p * h) ** 2,
                    (v * w) ** 2, (v * h) ** 2, (v * w) ** 2, (v * h) ** 2))


def measurement_noise(w, h, m=1 / 20):
    """deep_ocsort.py:83-87."""
    wv = (m * w) ** 2
    hv = (m * h) ** 2
    return np.diag((wv, hv, wv, hv))


class KF8:
    def __init__(self, z):
        self.x = np.zeros((8, 1))
        self.x[:4] = z
        _, _, w, h = z.reshape(-1)
        self.P = process_noise(w, h)
        self.P[:4, :4] *= 4
        self.P[4:, 4:] *= 100
        self.history = []
        self.saved = None                   # (x, P, last_measurement, attr_saved at freeze)
        self.observed = False
        self.last_measurement = None

    def predict(self, Q=None):
        self.x = np.dot(_F8, self.x)
        self.P = 1.0 * np.dot(np.dot(_F8, self.P), _F8.T) + (np.eye(8) if Q is None else Q)

    def _correct(self, z, R):
        y = z - np.dot(_H8, self.x)
        PHT = np.dot(self.P, _H8.T)
        S = np.dot(_H8, PHT) + R
        K = np.dot(PHT, np.linalg.inv(S))
        self.x = self.x + np.dot(K, y)
        I_KH = np.eye(8) - np.dot(K, _H8)
        self.P = np.dot(np.dot(I_KH, self.P), I_KH.T) + np.dot(np.dot(K, R), K.T)

    def update(self, z, R=None):
        self.history.append(z)
        if z is None:
            if self.observed:
                self.last_measurement = self.history[-2]
                self.saved = dict(x=self.x.copy(), P=self.P.copy(),
                                  last_measurement=self.last_measurement.copy(),
                                  history=list(self.history), attr_saved=self.saved)
            self.observed = False
            return
        if not self.observed:
            self._unfreeze()
        self.observed = True
        self._correct(z, np.eye(4) if R is None else R)

    def _unfreeze(self):
        if self.saved is None:
            return
        new_history = list(self.history)
        sv = self.saved
        self.x, self.P = sv["x"].copy(), sv["P"].copy()
        self.last_measurement = sv["last_measurement"]
        self.saved, self.observed = sv["attr_saved"], True
        self.history = sv["history"][:-1]
        idx = [k for k, d in enumerate(new_history) if d is not None]
        i1, i2 = idx[-2], idx[-1]
        x1, y1, s1, r1 = self.last_measurement
        w1, h1 = np.sqrt(s1 * r1), np.sqrt(s1 / r1)
        x2, y2, s2, r2 = new_history[i2]
        w2, h2 = np.sqrt(s2 * r2), np.sqrt(s2 / r2)
        gap = i2 - i1
        dx, dy, dw, dh = (x2 - x1) / gap, (y2 - y1) / gap, (w2 - w1) / gap, (h2 - h1) / gap
        for i in range(gap):
            x = x1 + (i + 1) * dx
            y = y1 + (i + 1) * dy
            w = w1 + (i + 1) * dw
            h = h1 + (i + 1) * dh
            self.update(np.array([x, y, w * h, w / float(h)]).reshape((4, 1)))
            if i != gap - 1:
                self.predict()

    def affine(self, m, t):
        """deepocsort_kf.py:387-407 (new KF)."""
        big = np.kron(np.eye(4, dtype=float), m)
        self.x = big @ self.x
        self.x[:2] += t
        self.P = big @ self.P @ big.T
        if not self.observed and self.saved is not None:
            sv = self.saved
            sv["x"] = big @ sv["x"]
            sv["x"][:2] += t
            sv["P"] = big @ sv["P"] @ big.T
            sv["last_measurement"][:2] = m @ sv["last_measurement"][:2] + t
            sv["last_measurement"][2:] = m @ sv["last_measurement"][2:]


class Tracker8:
    """KalmanBoxTracker, new-KF branch (deep_ocsort.py:90-330)."""

    def __init__(self, det, tid, delta_t, emb):
        self.conf, self.cls, self.det_ind = det[4], det[5], det[6]
        self.kf = KF8(bbox_to_z_new(det[0:5]))
        self.tsu = 0
        self.id = tid
        self.hits = self.hit_streak = self.age = 0
        self.last_obs = np.array([-1, -1, -1, -1, -1])
        self.obs = {}
        self.velocity = None
        self.delta_t = delta_t
        self.emb = emb
        self.frozen = False

    def update(self, det):
        """:198-241."""
        if det is None:
            self.kf.update(None)
            self.frozen = True
            return
        bbox = det[0:5]
        self.conf, self.cls, self.det_ind = det[4], det[5], det[6]
        self.frozen = False
        if self.last_obs.sum() >= 0:
            prev = None
            for dt in range(self.delta_t, 0, -1):
                if self.age - dt in self.obs:
                    prev = self.obs[self.age - dt]
                    break
            if prev is None:
                prev = self.last_obs
            self.velocity = speed_direction(prev, bbox)
        self.last_obs = bbox
        self.obs[self.age] = bbox
        self.tsu = 0
        self.hits += 1
        self.hit_streak += 1
        R = measurement_noise(self.kf.x[2, 0], self.kf.x[3, 0])
        self.kf.update(bbox_to_z_new(bbox), R=R)

    def update_emb(self, emb, alpha):
        """:243-245."""
        self.emb = alpha * self.emb + (1 - alpha) * emb
        self.emb /= np.linalg.norm(self.emb)

    def affine(self, affine):
        """:250-267."""
        m = affine[:, :2]
        t = affine[:, 2].reshape(2, 1)
        if self.last_obs.sum() > 0:
            ps = self.last_obs[:4].reshape(2, 2).T
            ps = m @ ps + t
            self.last_obs[:4] = ps.T.reshape(-1)
        for dt in range(self.delta_t, -1, -1):
            if self.age - dt in self.obs:
                ps = self.obs[self.age - dt][:4].reshape(2, 2).T
                ps = m @ ps + t
                self.obs[self.age - dt][:4] = ps.T.reshape(-1)
        self.kf.affine(m, t)

    def predict(self):
        """:269-293."""
        if self.kf.x[2] + self.kf.x[6] <= 0:
            self.kf.x[6] = 0
        if self.kf.x[3] + self.kf.x[7] <= 0:
            self.kf.x[7] = 0
        if self.frozen:
            self.kf.x[6] = self.kf.x[7] = 0
        Q = process_noise(self.kf.x[2, 0], self.kf.x[3, 0])
        self.kf.predict(Q=Q)
        self.age += 1
        if self.tsu > 0:
            self.hit_streak = 0
        self.tsu += 1
        return x_to_bbox_new(self.kf.x)

    def k_previous_obs(self):
        if not self.obs:
            return [-1, -1, -1, -1, -1]
        for i in range(self.delta_t):
            if self.age - (self.delta_t - i) in self.obs:
                return self.obs[self.age - (self.delta_t - i)]
        return self.obs[max(self.obs.keys())]


def aw_max_metric(emb_cost, w_emb, bottom=0.5):
    """association.py:79-108."""
    w = np.full_like(emb_cost, w_emb)
    for r in range(emb_cost.shape[0]):
        inds = np.argsort(-emb_cost[r])
        if len(inds) < 2:
            continue
        if emb_cost[r, inds[0]] == 0:
            rw = 0
        else:
            rw = 1 - max((emb_cost[r, inds[1]] / emb_cost[r, inds[0]]) - bottom, 0) / (1 - bottom)
        w[r] *= rw
    for c in range(emb_cost.shape[1]):
        inds = np.argsort(-emb_cost[:, c])
        if len(inds) < 2:
            continue
        if emb_cost[inds[0], c] == 0:
            cw = 0
        else:
            cw = 1 - max((emb_cost[inds[1], c] / emb_cost[inds[0], c]) - bottom, 0) / (1 - bottom)
        w[:, c] *= cw
    return w * emb_cost


def associate_emb(dets, trks, func, thr, velocities, prev_obs, inertia, w, h, emb_cost, w_emb,
                  aw_off, aw_param):
    """association.py:111-201 with the embedding term."""
    if len(trks) == 0:
        return np.empty((0, 2), dtype=int), np.arange(len(dets)), np.empty((0, 5), dtype=int)
    t = prev_obs[..., np.newaxis]
    dx = (dets[:, 0] + dets[:, 2]) / 2.0 - (t[:, 0] + t[:, 2]) / 2.0
    dy = (dets[:, 1] + dets[:, 3]) / 2.0 - (t[:, 1] + t[:, 3]) / 2.0
    norm = np.sqrt(dx ** 2 + dy ** 2) + 1e-6
    X, Y = dx / norm, dy / norm
    iy = np.repeat(velocities[:, 0][:, np.newaxis], Y.shape[1], axis=1)
    ix = np.repeat(velocities[:, 1][:, np.newaxis], X.shape[1], axis=1)
    cos = np.clip(ix * X + iy * Y, a_min=-1, a_max=1)
    ang = (np.pi / 2.0 - np.abs(np.arccos(cos))) / np.pi
    valid = np.ones(prev_obs.shape[0])
    valid[np.where(prev_obs[:, 4] < 0)] = 0
    iou = _asso(func, dets, trks, w, h)
    scores = np.repeat(dets[:, -1][:, np.newaxis], trks.shape[0], axis=1)
    valid = np.repeat(valid[:, np.newaxis], X.shape[1], axis=1)
    angle_cost = ((valid * ang) * inertia).T * scores
    if min(iou.shape):
        a = (iou > thr).astype(np.int32)
        if a.sum(1).max() == 1 and a.sum(0).max() == 1:
            matched = np.stack(np.where(a), axis=1)
        else:
            if emb_cost is None:
                emb_cost = 0
            else:
                emb_cost[iou <= 0] = 0
                if not aw_off:
                    emb_cost = aw_max_metric(emb_cost, w_emb, bottom=aw_param)
                else:
                    emb_cost *= w_emb
            matched = linear_assignment_padded(-(iou + angle_cost + emb_cost))
            if matched.size == 0:
                matched = np.empty(shape=(0, 2))
    else:
        matched = np.empty(shape=(0, 2))
    u_det = [d for d in range(len(dets)) if d not in matched[:, 0]]
    u_trk = [k for k in range(len(trks)) if k not in matched[:, 1]]
    matches = []
    for m in matched:
        if iou[m[0], m[1]] < thr:
            u_det.append(m[0])
            u_trk.append(m[1])
        else:
            matches.append(m.reshape(1, 2))
    matches = np.concatenate(matches, axis=0) if matches else np.empty((0, 2), dtype=int)
    return matches, np.array(u_det), np.array(u_trk)


class DeepOCSortOracle:
    def __init__(self, det_thresh=0.3, max_age=30, min_hits=3, iou_threshold=0.3, delta_t=3,
                 asso_func="iou", inertia=0.2, w_association_emb=0.5, alpha_fixed_emb=0.95,
                 aw_param=0.5, embedding_off=False, cmc_off=False, aw_off=False):
        self.max_age, self.min_hits, self.thr = max_age, min_hits, iou_threshold
        self.trackers = []
        self.frame_count = 0
        self.det_thresh, self.delta_t, self.inertia = det_thresh, delta_t, inertia
        self.func = ASSO[asso_func]
        self.w_emb, self.af, self.aw_param = w_association_emb, alpha_fixed_emb, aw_param
        self.embedding_off, self.cmc_off, self.aw_off = embedding_off, cmc_off, aw_off
        self.count = 1                                           # :347

    def update(self, dets, img_shape, feats=None, warp=None):
        """dets (M, 6); feats: get_features' rows for the detections with conf > det_thresh;
        warp: the CMC 2x3 affine (identity when None)."""
        self.frame_count += 1
        h, w = img_shape[:2]
        scores = dets[:, 4]
        dets = np.hstack([dets, np.arange(len(dets)).reshape(-1, 1)])
        dets = dets[scores > self.det_thresh]
        if self.embedding_off or dets.shape[0] == 0:
            dets_embs = np.ones((dets.shape[0], 1))
        else:
            dets_embs = np.asarray(feats)
        if not self.cmc_off:
            transform = np.eye(2, 3) if warp is None else np.asarray(warp, np.float64)
            for trk in self.trackers:
                trk.affine(transform)
        trust = (dets[:, 4] - self.det_thresh) / (1 - self.det_thresh)
        dets_alpha = self.af + (1 - self.af) * (1 - trust)
        trks = np.zeros((len(self.trackers), 5))
        trk_embs, to_del = [], []
        for k in range(len(trks)):
            pos = self.trackers[k].predict()[0]
            trks[k] = [pos[0], pos[1], pos[2], pos[3], 0]
            if np.any(np.isnan(pos)):
                to_del.append(k)
            else:
                trk_embs.append(self.trackers[k].emb)
        trks = np.ma.compress_rows(np.ma.masked_invalid(trks))
        trk_embs = np.vstack(trk_embs) if trk_embs else np.array(trk_embs)
        for k in reversed(to_del):
            self.trackers.pop(k)
        vel = np.array([t.velocity if t.velocity is not None else np.array((0, 0))
                        for t in self.trackers])
        last_boxes = np.array([t.last_obs for t in self.trackers])
        k_obs = np.array([t.k_previous_obs() for t in self.trackers])
        if self.embedding_off or dets.shape[0] == 0 or trk_embs.shape[0] == 0:
            emb_cost = None
        else:
            emb_cost = dets_embs @ trk_embs.T
        matched, u_det, u_trk = associate_emb(dets[:, 0:5], trks, self.func, self.thr, vel, k_obs,
                                              self.inertia, w, h, emb_cost, self.w_emb,
                                              self.aw_off, self.aw_param)
        for m in matched:
            self.trackers[m[1]].update(dets[m[0], :])
            self.trackers[m[1]].update_emb(dets_embs[m[0]], dets_alpha[m[0]])
        if u_det.shape[0] > 0 and u_trk.shape[0] > 0:
            iou_left = np.array(self.func(dets[u_det], last_boxes[u_trk]))
            if iou_left.max() > self.thr:
                rd, rt = [], []
                for m in linear_assignment_padded(-iou_left):
                    di, ti = u_det[m[0]], u_trk[m[1]]
                    if iou_left[m[0], m[1]] < self.thr:
                        continue
                    self.trackers[ti].update(dets[di, :])
                    self.trackers[ti].update_emb(dets_embs[di], dets_alpha[di])
                    rd.append(di)
                    rt.append(ti)
                u_det = np.setdiff1d(u_det, np.array(rd))
                u_trk = np.setdiff1d(u_trk, np.array(rt))
        for k in u_trk:
            self.trackers[k].update(None)
        for i in u_det:
            self.trackers.append(Tracker8(dets[i], self.count, self.delta_t, dets_embs[i]))
            self.count += 1
        ret = []
        i = len(self.trackers)
        for t in reversed(self.trackers):
            d = x_to_bbox_new(t.kf.x)[0] if t.last_obs.sum() < 0 else t.last_obs[:4]
            if t.tsu < 1 and (t.hit_streak >= self.min_hits or self.frame_count <= self.min_hits):
                ret.append(np.concatenate((d, [t.id], [t.conf], [t.cls], [t.det_ind])).reshape(1, -1))
            i -= 1
            if t.tsu > self.max_age:
                self.trackers.pop(i)
        if ret:
            return np.concatenate(ret)
        return np.array([])
