"""ORACLE — test infrastructure only.  CPU restatement of BoTSORT.update()
(boxmot/trackers/botsort/bot_sort.py:185-425, basetrack.py).

Same list algebra as ByteTrack (oracle/bytetrack.py) with BoT-SORT's differences:
  * confidence split  high: conf > track_high_thresh, second: track_low_thresh < conf < high
    (:263-269); only high detections carry appearance features (:271-281)
  * Kalman filter in (xc, yc, w, h) (oracle/kalman_xywh.py); multi_predict zeroes BOTH vw and vh
    of non-tracked tracks (:69-93); camera-motion compensation of pool and unconfirmed tracks with
    the frame's 2x3 warp (:303-305, multi_gmc :95-111)
  * stage 1: iou distance, mask = iou > proximity_thresh, optionally fuse_score (fuse_first),
    emb = max(0, cosine cdist(smooth feats, det feats)) / 2, emb > appearance_thresh -> 1, masked
    -> 1, cost = min(iou, emb), lapjv cost_limit = match_thresh (:307-322)
  * stage 3 (unconfirmed): the same with fuse_score always applied after the mask (:355-370)
  * births need score >= new_track_thresh (:377-383)
  * feature bookkeeping exactly as the reference, including its in-place normalisations: a
    detection's features are normalised twice at construction (update_features: feat /= norm,
    then smooth_feat /= norm on the same array) and once more, in place, when a track takes the
    detection (:40-48)
  * class histogram vote update_cls (:50-67)
  * ids from a counter reset when the tracker is constructed (BaseTrack.clear_count, :205)
Embedding values follow float32 NumPy arithmetic (np.linalg.norm on float32 rows), as the
reference.
"""
import numpy as np
from scipy.spatial.distance import cdist

from . import geometry, kalman_xywh as kf
from .lap import linear_assignment_limited

NEW, TRACKED, LOST, LONGLOST, REMOVED = 0, 1, 2, 3, 4


def xyxy2xywh(d):
    """ops.xyxy2xywh (ops.py:7-21)."""
    return np.array([(d[0] + d[2]) / 2, (d[1] + d[3]) / 2, d[2] - d[0], d[3] - d[1]])


def xywh2xyxy(b):
    """ops.xywh2xyxy (ops.py:24-40)."""
    return np.array([b[0] - b[2] / 2, b[1] - b[3] / 2, b[0] + b[2] / 2, b[1] + b[3] / 2])


class Track:
    def __init__(self, det, feat=None):
        self.xywh = xyxy2xywh(det[0:4])
        self.score, self.cls, self.det_ind = det[4], det[5], det[6]
        self.mean = self.cov = None
        self.activated = False
        self.cls_hist = []
        self.update_cls(self.cls, self.score)
        self.tracklet_len = 0
        self.smooth_feat = self.curr_feat = None
        if feat is not None:
            self.update_features(feat)
        self.alpha = 0.9
        self.track_id = 0
        self.state = NEW
        self.frame_id = self.start_frame = 0

    def update_features(self, feat):
        """:40-48 (in place on the caller's array, like the reference)."""
        feat /= np.linalg.norm(feat)
        self.curr_feat = feat
        if self.smooth_feat is None:
            self.smooth_feat = feat
        else:
            self.smooth_feat = 0.9 * self.smooth_feat + (1 - 0.9) * feat
        self.smooth_feat /= np.linalg.norm(self.smooth_feat)

    def update_cls(self, cls, score):
        """:50-67."""
        if len(self.cls_hist) > 0:
            max_freq = 0
            found = False
            for c in self.cls_hist:
                if cls == c[0]:
                    c[1] += score
                    found = True
                if c[1] > max_freq:
                    max_freq = c[1]
                    self.cls = c[0]
            if not found:
                self.cls_hist.append([cls, score])
                self.cls = cls
        else:
            self.cls_hist.append([cls, score])
            self.cls = cls

    def box(self):
        """STrack.xyxy (:173-182)."""
        return xywh2xyxy(self.xywh.copy() if self.mean is None else self.mean[:4].copy())

    def take(self, det, frame_id, reactivate):
        """STrack.re_activate (:125-143) / update (:145-170)."""
        if not reactivate:
            self.frame_id = frame_id
            self.tracklet_len += 1
        self.mean, self.cov = kf.update(self.mean, self.cov, det.xywh)
        if det.curr_feat is not None:
            self.update_features(det.curr_feat)
        if reactivate:
            self.tracklet_len = 0
        self.state = TRACKED
        self.activated = True
        self.frame_id = frame_id
        self.score, self.cls, self.det_ind = det.score, det.cls, det.det_ind
        self.update_cls(det.cls, det.score)


def _iou(ta, tb):
    return geometry.iou_distance([t.box() for t in ta], [t.box() for t in tb])


def _emb(tracks, dets):
    """matching.embedding_distance (:145-167) / 2."""
    if not len(tracks) or not len(dets):
        return np.zeros((len(tracks), len(dets)))
    df = np.asarray([t.curr_feat for t in dets], dtype=np.float32)
    tf = np.asarray([t.smooth_feat for t in tracks], dtype=np.float32)
    return np.maximum(0.0, cdist(tf, df, "cosine")) / 2.0


def _union(a, b):
    seen = {t.track_id for t in a}
    out = list(a)
    for t in b:
        if t.track_id not in seen:
            seen.add(t.track_id)
            out.append(t)
    return out


def _minus(a, b):
    keyed = {}
    for t in a:
        keyed[t.track_id] = t
    for t in b:
        keyed.pop(t.track_id, None)
    return list(keyed.values())


def _dedup(ta, tb):
    d = _iou(ta, tb)
    drop_a, drop_b = set(), set()
    for p, q in zip(*np.where(d < 0.15)):
        if ta[p].frame_id - ta[p].start_frame > tb[q].frame_id - tb[q].start_frame:
            drop_b.add(q)
        else:
            drop_a.add(p)
    return ([t for i, t in enumerate(ta) if i not in drop_a],
            [t for i, t in enumerate(tb) if i not in drop_b])


class BoTSORTOracle:
    def __init__(self, track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
                 track_buffer=30, match_thresh=0.8, proximity_thresh=0.5, appearance_thresh=0.25,
                 frame_rate=30, fuse_first_associate=False, with_reid=True):
        self.tracked, self.lost, self.removed = [], [], []
        self.frame_id = 0
        self.high, self.low, self.new_thresh = track_high_thresh, track_low_thresh, new_track_thresh
        self.match_thresh = match_thresh
        self.max_time_lost = int(frame_rate / 30.0 * track_buffer)
        self.prox, self.app = proximity_thresh, appearance_thresh
        self.fuse_first, self.with_reid = fuse_first_associate, with_reid
        self.next_id = 0

    def _new_id(self):
        self.next_id += 1
        return self.next_id

    def _cost(self, tracks, dets, fuse):
        iou = _iou(tracks, dets)
        mask = iou > self.prox
        if fuse:
            iou = geometry.fuse_score(iou, [d.score for d in dets])
        if not self.with_reid:
            return iou
        emb = _emb(tracks, dets)
        emb[emb > self.app] = 1.0
        emb[mask] = 1.0
        return np.minimum(iou, emb)

    def update(self, dets, feats=None, warp=None):
        """dets (M, 6); feats: what the ReID model's get_features returns for the high detections
        (n_high, D) float32; warp: the CMC 2x3 affine (identity when None)."""
        dets = np.asarray(dets)
        assert dets.ndim == 2 and dets.shape[1] == 6
        self.frame_id += 1
        fid = self.frame_id
        dets = np.hstack([dets, np.arange(len(dets)).reshape(-1, 1)])
        conf = dets[:, 4]
        dets_second = dets[np.logical_and(conf > self.low, conf < self.high)]
        dets_first = dets[conf > self.high]
        if self.with_reid:
            feats = np.asarray(feats, dtype=np.float32)
            high = [Track(d, f) for d, f in zip(dets_first, feats)]
        else:
            high = [Track(d) for d in dets_first]
        unconfirmed = [t for t in self.tracked if not t.activated]
        active = [t for t in self.tracked if t.activated]
        pool = _union(active, self.lost)
        if pool:                                    # STrack.multi_predict (:80-93)
            m = np.asarray([t.mean.copy() for t in pool])
            c = np.asarray([t.cov for t in pool])
            for i, t in enumerate(pool):
                if t.state != TRACKED:
                    m[i][6] = 0
                    m[i][7] = 0
            m, c = kf.multi_predict(m, c)
            for i, t in enumerate(pool):
                t.mean, t.cov = m[i], c[i]
        w = np.eye(2, 3) if warp is None else np.asarray(warp, np.float64)
        for t in pool + unconfirmed:                # multi_gmc (:95-111)
            t.mean, t.cov = kf.gmc(t.mean, t.cov, w)

        activated, refind, lost_now, removed_now = [], [], [], []

        def take(t, det):
            was_tracked = t.state == TRACKED
            t.take(det, fid, reactivate=not was_tracked)
            (activated if was_tracked else refind).append(t)

        # stage 1: pool x high detections (:307-331)
        dists = self._cost(pool, high, self.fuse_first)
        matches, u_track, u_det = linear_assignment_limited(dists, self.match_thresh)
        for it, idet in matches:
            take(pool[it], high[idet])
        # stage 2: still-tracked leftovers x low detections, plain IoU, 0.5 (:333-352)
        second = [Track(d) for d in dets_second]
        r_tracked = [pool[i] for i in u_track if pool[i].state == TRACKED]
        matches, u_left, _ = linear_assignment_limited(_iou(r_tracked, second), 0.5)
        for it, idet in matches:
            take(r_tracked[it], second[idet])
        for it in u_left:
            t = r_tracked[it]
            if t.state != LOST:
                t.state = LOST
                lost_now.append(t)
        # stage 3: unconfirmed x remaining high detections, fused + emb, 0.7 (:354-375)
        rest = [high[i] for i in u_det]
        dists = self._cost(unconfirmed, rest, True)
        matches, u_unc, u_det = linear_assignment_limited(dists, 0.7)
        for it, idet in matches:
            unconfirmed[it].take(rest[idet], fid, reactivate=False)
            activated.append(unconfirmed[it])
        for it in u_unc:
            unconfirmed[it].state = REMOVED
            removed_now.append(unconfirmed[it])
        # births (:377-383)
        for inew in u_det:
            t = rest[inew]
            if t.score < self.new_thresh:
                continue
            t.track_id = self._new_id()
            t.mean, t.cov = kf.initiate(t.xywh)
            t.tracklet_len = 0
            t.state = TRACKED
            t.activated = fid == 1
            t.frame_id = t.start_frame = fid
            activated.append(t)
        # expiry (:385-389)
        for t in self.lost:
            if fid - t.frame_id > self.max_time_lost:
                t.state = REMOVED
                removed_now.append(t)
        # merge (:391-406)
        self.tracked = [t for t in self.tracked if t.state == TRACKED]
        self.tracked = _union(self.tracked, activated)
        self.tracked = _union(self.tracked, refind)
        self.lost = _minus(self.lost, self.tracked)
        self.lost.extend(lost_now)
        self.lost = _minus(self.lost, self.removed)
        self.removed.extend(removed_now)
        self.tracked, self.lost = _dedup(self.tracked, self.lost)
        rows = [np.r_[t.box(), t.track_id, t.score, t.cls, t.det_ind]
                for t in self.tracked if t.activated]
        return np.asarray(rows)
