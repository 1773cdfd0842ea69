"""ORACLE — test infrastructure only.  CPU restatement of OCSort.update()
(boxmot/trackers/ocsort/ocsort.py:188-379) with its association (boxmot/utils/association.py:8-28,
:111-201) and the live paths of its filterpy-derived Kalman filter
(boxmot/motion/kalman_filters/ocsort_kf.py:339-526: predict, update with Joseph form, freeze /
unfreeze "observation-centric re-update").

The Kalman arithmetic uses NumPy products on the full 7x7 matrices, exactly the operations the
reference performs, so states are bit-identical on the same host; the HIP engine restates them on
the block structure those matrices keep (see yolo_tracking_amd/csrc/kf_ocsort.hpp).

Per-tracker bookkeeping (ocsort.py:65-186):
  * observations: the reference keeps a dict age -> box; only ages cur_age-delta_t .. cur_age-1
    and the newest entry are ever read (k_previous_obs :14-22, update :138-150), which is what
    this restatement keeps as well (the full dict, for clarity).
  * ORU: on the first miss after an observation the filter state is frozen; on re-acquisition the
    frozen state is restored and a linear virtual trajectory between the last observation kept in
    the filter's history and the new one is replayed with update/predict pairs (:390-434).
"""
import numpy as np

from . import geometry
from .lap import linear_assignment_padded

ASSO = {"iou": geometry.iou_batch, "giou": geometry.giou_batch, "diou": geometry.diou_batch,
        "ciou": geometry.ciou_batch, "centroid": geometry.centroid_batch}

_F = np.eye(7, dtype=np.int64)
_F[0, 4] = _F[1, 5] = _F[2, 6] = 1          # ocsort.py:80-91 (an int array, as the reference)
_H = np.eye(4, 7, dtype=np.int64)           # ocsort.py:92-99


def bbox_to_z(b):
    """ocsort.py:25-37 (note the +1e-6 in the aspect ratio)."""
    w = b[2] - b[0]
    h = b[3] - b[1]
    return np.array([b[0] + w / 2.0, b[1] + h / 2.0, w * h, w / float(h + 1e-6)]).reshape((4, 1))


def x_to_bbox(x):
    """ocsort.py:40-54."""
    w = np.sqrt(x[2] * x[3])
    h = x[2] / w
    return np.array([x[0] - w / 2.0, x[1] - h / 2.0, x[0] + w / 2.0, x[1] + h / 2.0]).reshape((1, 4))


def speed_direction(b1, b2):
    """ocsort.py:57-62."""
    cx1, cy1 = (b1[0] + b1[2]) / 2.0, (b1[1] + b1[3]) / 2.0
    cx2, cy2 = (b2[0] + b2[2]) / 2.0, (b2[1] + b2[3]) / 2.0
    v = np.array([cy2 - cy1, cx2 - cx1])
    return v / (np.sqrt((cy2 - cy1) ** 2 + (cx2 - cx1) ** 2) + 1e-6)


class KF7:
    """The OCSORT filter: x (7,1), P (7,7); Q, R, P0 as ocsort.py:101-106."""

    def __init__(self, z):
        self.x = np.zeros((7, 1))
        self.x[:4] = z
        self.P = np.eye(7)
        self.P[4:, 4:] *= 1000.0
        self.P *= 10.0
        self.Q = np.eye(7)
        self.Q[-1, -1] *= 0.01
        self.Q[4:, 4:] *= 0.01
        self.R = np.eye(4)
        self.R[2:, 2:] *= 10.0
        self.history = []          # history_obs: z or None per update call
        self.saved = None          # attr_saved: (x, P, history) at the freeze
        self.observed = False

    def predict(self):
        """ocsort_kf.py:339-380 (alpha_sq = 1, no control input)."""
        self.x = np.dot(_F, self.x)
        self.P = 1.0 * np.dot(np.dot(_F, self.P), _F.T) + self.Q

    def _correct(self, z):
        """ocsort_kf.py:478-526: y, S, inv(S), K, x, Joseph-form P."""
        y = z - np.dot(_H, self.x)
        PHT = np.dot(self.P, _H.T)
        S = np.dot(_H, PHT) + self.R
        K = np.dot(PHT, np.linalg.inv(S))
        self.x = self.x + np.dot(K, y)
        I_KH = np.eye(7) - np.dot(K, _H)
        self.P = np.dot(np.dot(I_KH, self.P), I_KH.T) + np.dot(np.dot(K, self.R), K.T)

    def update(self, z):
        """ocsort_kf.py:437-476 incl. freeze (:383-387) and unfreeze (:390-434)."""
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
        # restoring the frozen __dict__ restores its attr_saved (the previous freeze) and
        # observed = True (the freeze ran before `observed` was cleared)
        self.x, self.P, self.saved, self.observed = x.copy(), P.copy(), older, True
        self.history = hist[:-1]
        idx = [k for k, d in enumerate(new_history) if d is not None]
        i1, i2 = idx[-2], idx[-1]
        x1, y1, s1, r1 = new_history[i1]
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


class Tracker:
    """KalmanBoxTracker (ocsort.py:65-186)."""

    def __init__(self, det, tid, delta_t):
        self.kf = KF7(bbox_to_z(det[:4]))
        self.det_ind = det[6]
        self.tsu = 0
        self.id = tid
        self.hits = self.hit_streak = self.age = 0
        self.conf, self.cls = det[4], det[5]
        self.last_obs = np.array([-1, -1, -1, -1, -1])
        self.obs = {}
        self.velocity = None
        self.delta_t = delta_t

    def update(self, det):
        """ocsort.py:130-166; det is a (7,) row or None."""
        if det is None:
            self.det_ind = None
            self.kf.update(None)
            return
        bbox = det[:5]
        self.det_ind = det[6]
        self.conf, self.cls = bbox[-1], det[5]
        if self.last_obs.sum() >= 0:
            prev = None
            for i in range(self.delta_t):
                if self.age - (self.delta_t - i) in self.obs:
                    prev = self.obs[self.age - (self.delta_t - i)]
                    break
            if prev is None:
                prev = self.last_obs
            self.velocity = speed_direction(prev, bbox)
        self.last_obs = bbox
        self.obs[self.age] = bbox
        self.tsu = 0
        self.hits += 1
        self.hit_streak += 1
        self.kf.update(bbox_to_z(bbox))

    def predict(self):
        """ocsort.py:168-181."""
        if (self.kf.x[6] + self.kf.x[2]) <= 0:
            self.kf.x[6] *= 0.0
        self.kf.predict()
        self.age += 1
        if self.tsu > 0:
            self.hit_streak = 0
        self.tsu += 1
        return x_to_bbox(self.kf.x)

    def k_previous_obs(self):
        """ocsort.py:14-22."""
        if not self.obs:
            return [-1, -1, -1, -1, -1]
        for i in range(self.delta_t):
            if self.age - (self.delta_t - i) in self.obs:
                return self.obs[self.age - (self.delta_t - i)]
        return self.obs[max(self.obs.keys())]


def _asso(func, a, b, w, h):
    """iou.run_asso_func (iou.py:191-212)."""
    if func is geometry.centroid_batch:
        return func(a, b, w, h)
    return func(a, b)


def associate(dets, trks, func, thr, velocities, prev_obs, inertia, w, h):
    """association.py:111-201 (no embedding term)."""
    if len(trks) == 0:
        return np.empty((0, 2), dtype=int), np.arange(len(dets)), np.empty((0, 5), dtype=int)
    # speed_direction_batch (:8-17): track k-obs -> det direction, (num_track, num_det)
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
            matched = linear_assignment_padded(-(iou + angle_cost + 0))
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


class OCSortOracle:
    def __init__(self, per_class=False, det_thresh=0.2, max_age=30, min_hits=3,
                 asso_threshold=0.3, delta_t=3, asso_func="iou", inertia=0.2, use_byte=False):
        self.max_age, self.min_hits, self.thr = max_age, min_hits, asso_threshold
        self.trackers = []
        self.frame_count = 0
        self.det_thresh, self.delta_t, self.inertia = det_thresh, delta_t, inertia
        self.func = ASSO[asso_func]
        self.use_byte = use_byte
        self.count = 0                                          # KalmanBoxTracker.count (:216)

    def update(self, dets, img_shape):
        """dets (M, 6); img_shape: img.shape (only h, w are read, :239)."""
        self.frame_count += 1
        h, w = img_shape[0:2]
        dets = np.hstack([dets, np.arange(len(dets)).reshape(-1, 1)])
        conf = dets[:, 4]
        dets_second = dets[np.logical_and(conf > 0.1, conf < self.det_thresh)]
        dets = dets[conf > self.det_thresh]
        # predict (:250-264): trackers whose predicted box has a NaN are dropped
        trks = np.zeros((len(self.trackers), 5))
        to_del = []
        for k in range(len(trks)):
            pos = self.trackers[k].predict()[0]
            trks[k] = [pos[0], pos[1], pos[2], pos[3], 0]
            if np.any(np.isnan(pos)):
                to_del.append(k)
        trks = np.ma.compress_rows(np.ma.masked_invalid(trks))
        for k in reversed(to_del):
            self.trackers.pop(k)
        vel = np.array([t.velocity if t.velocity is not None else np.array((0, 0))
                        for t in self.trackers])
        last_boxes = np.array([t.last_obs for t in self.trackers])
        k_obs = np.array([t.k_previous_obs() for t in self.trackers])
        # first round (:279-284)
        matched, u_det, u_trk = associate(dets[:, 0:5], trks, self.func, self.thr, vel, k_obs,
                                          self.inertia, w, h)
        for m in matched:
            self.trackers[m[1]].update(dets[m[0]])
        # BYTE round (:289-313)
        if self.use_byte and len(dets_second) > 0 and u_trk.shape[0] > 0:
            iou_left = np.array(self.func(dets_second, trks[u_trk]))
            if iou_left.max() > self.thr:
                taken = []
                for m in linear_assignment_padded(-iou_left):
                    if iou_left[m[0], m[1]] < self.thr:
                        continue
                    self.trackers[u_trk[m[1]]].update(dets_second[m[0]])
                    taken.append(u_trk[m[1]])
                u_trk = np.setdiff1d(u_trk, np.array(taken))
        # OCR round (:315-342): unmatched dets x the unmatched trackers' last observations
        if u_det.shape[0] > 0 and u_trk.shape[0] > 0:
            iou_left = np.array(_asso(self.func, dets[u_det], last_boxes[u_trk], w, h))
            if iou_left.max() > self.thr:
                rd, rt = [], []
                for m in linear_assignment_padded(-iou_left):
                    di, ti = u_det[m[0]], u_trk[m[1]]
                    if iou_left[m[0], m[1]] < self.thr:
                        continue
                    self.trackers[ti].update(dets[di])
                    rd.append(di)
                    rt.append(ti)
                u_det = np.setdiff1d(u_det, np.array(rd))
                u_trk = np.setdiff1d(u_trk, np.array(rt))
        for k in u_trk:
            self.trackers[k].update(None)
        # births (:347-349) in the order of the unmatched list
        for i in u_det:
            self.trackers.append(Tracker(dets[i], self.count, self.delta_t))
            self.count += 1
        # outputs in reversed tracker order, dead trackers removed (:350-379)
        ret = []
        i = len(self.trackers)
        for t in reversed(self.trackers):
            d = x_to_bbox(t.kf.x)[0] if t.last_obs.sum() < 0 else t.last_obs[:4]
            if t.tsu < 1 and (t.hit_streak >= self.min_hits or self.frame_count <= self.min_hits):
                ret.append(np.concatenate((d, [t.id + 1], [t.conf], [t.cls], [t.det_ind]))
                           .reshape(1, -1))
            i -= 1
            if t.tsu > self.max_age:
                self.trackers.pop(i)
        if ret:
            return np.concatenate(ret)
        return np.array([])
