"""ORACLE — test infrastructure only.  CPU restatement of BYTETracker.update()
(boxmot/trackers/bytetrack/byte_tracker.py:114-325, basetrack.py:8-55).

It keeps the reference's per-frame structure and every ordering rule, because list order decides
both new-track IDs and output row order:
  * confidence split  high: conf > track_thresh, second: 0.1 < conf < track_thresh (:149-158)
  * unconfirmed tracks (not activated) are NOT Kalman-predicted; pool = activated ++ lost (:169-180)
  * three association stages with lapx cost_limit thresholds match_thresh / 0.5 / 0.7 (:181-240)
  * births in ascending unmatched-detection order, activated only on frame 1 (:58-59, :242-248)
  * removed-list quirk: a lost track timed out in this frame is dropped from lost_stracks only at the
    end of the NEXT frame, and a track whose id ever entered removed_stracks is dropped from
    lost_stracks as soon as it is lost again (:250-265)
  * duplicate removal between tracked and lost at IoU distance < 0.15, younger one dropped (:312-325)
Track IDs come from a counter that lives on the tracker object (the reference's counter is
process-global, basetrack.py:16; goldens reset it per sequence).
"""
import numpy as np

from . import geometry, kalman_xyah as kf
from .lap import linear_assignment_limited

NEW, TRACKED, LOST, REMOVED = 0, 1, 2, 3


def det_to_xywh(d):
    """ops.xyxy2xywh (ops.py:7-21)."""
    return np.array([(d[0] + d[2]) / 2, (d[1] + d[3]) / 2, d[2] - d[0], d[3] - d[1]])


def xywh_to_xyah(b):
    """ops.xywh2tlwh then ops.tlwh2xyah (ops.py:43-58, :87-97)."""
    t = b[0] - b[2] / 2.0
    l_ = b[1] - b[3] / 2.0
    return np.array([t + b[2] / 2, l_ + b[3] / 2, b[2] / b[3], b[3]])


def xywh_to_xyxy(b):
    """ops.xywh2xyxy (ops.py:24-40)."""
    return np.array([b[0] - b[2] / 2, b[1] - b[3] / 2, b[0] + b[2] / 2, b[1] + b[3] / 2])


class Track:
    __slots__ = ("xywh", "xyah", "score", "cls", "det_ind", "mean", "cov", "track_id", "state",
                 "activated", "frame_id", "start_frame", "tracklet_len")

    def __init__(self, det):
        self.xywh = det_to_xywh(det)
        self.xyah = xywh_to_xyah(self.xywh)
        self.score, self.cls, self.det_ind = det[4], det[5], det[6]
        self.mean = self.cov = None
        self.track_id = 0
        self.state = NEW
        self.activated = False
        self.frame_id = 0
        self.start_frame = 0
        self.tracklet_len = 0

    def box(self):
        """STrack.xyxy (byte_tracker.py:100-111)."""
        if self.mean is None:
            return xywh_to_xyxy(self.xywh)
        b = self.mean[:4].copy()
        b[2] *= b[3]
        return xywh_to_xyxy(b)

    def take(self, det, frame_id, reactivate):
        """STrack.update (:78-98) / re_activate(new_id=False) (:64-76)."""
        self.mean, self.cov = kf.update(self.mean, self.cov, det.xyah)
        self.tracklet_len = 0 if reactivate else self.tracklet_len + 1
        self.state = TRACKED
        self.activated = True
        self.frame_id = frame_id
        self.score, self.cls, self.det_ind = det.score, det.cls, det.det_ind


def _dist(tracks_a, tracks_b):
    return geometry.iou_distance([t.box() for t in tracks_a], [t.box() for t in tracks_b])


def _fused(tracks, dets):
    d = _dist(tracks, dets)
    return geometry.fuse_score(d, [x.score for x in dets])


def _union(a, b):
    """joint_stracks (:287-298)."""
    seen = {t.track_id for t in a}
    out = list(a)
    for t in b:
        if t.track_id not in seen:
            seen.add(t.track_id)
            out.append(t)
    return out


def _minus(a, b):
    """sub_stracks (:301-309): keep a's insertion order, drop ids present in b."""
    keyed = {}
    for t in a:
        keyed[t.track_id] = t
    for t in b:
        keyed.pop(t.track_id, None)
    return list(keyed.values())


def _dedup(ta, tb):
    """remove_duplicate_stracks (:312-325)."""
    d = _dist(ta, tb)
    drop_a, drop_b = set(), set()
    for p, q in zip(*np.where(d < 0.15)):
        if ta[p].frame_id - ta[p].start_frame > tb[q].frame_id - tb[q].start_frame:
            drop_b.add(q)
        else:
            drop_a.add(p)
    return ([t for i, t in enumerate(ta) if i not in drop_a],
            [t for i, t in enumerate(tb) if i not in drop_b])


class ByteTrackOracle:
    def __init__(self, track_thresh=0.45, match_thresh=0.8, track_buffer=25, frame_rate=30):
        self.tracked, self.lost, self.removed = [], [], []
        self.frame_id = 0
        self.track_thresh = track_thresh
        self.match_thresh = match_thresh
        self.det_thresh = track_thresh
        self.max_time_lost = int(frame_rate / 30.0 * track_buffer)
        self.next_id = 0

    def _new_id(self):
        self.next_id += 1
        return self.next_id

    def update(self, dets, _img=None):
        dets = np.asarray(dets)
        assert dets.ndim == 2 and dets.shape[1] == 6
        dets = np.hstack([dets, np.arange(len(dets)).reshape(-1, 1)])
        self.frame_id += 1
        fid = self.frame_id
        conf = dets[:, 4]
        high = [Track(d) for d in dets[conf > self.track_thresh]]
        second = [Track(d) for d in dets[np.logical_and(conf > 0.1, conf < self.track_thresh)]]

        unconfirmed = [t for t in self.tracked if not t.activated]
        active = [t for t in self.tracked if t.activated]
        pool = _union(active, self.lost)
        if pool:                                    # STrack.multi_predict (:35-48)
            m = np.stack([t.mean for t in pool]).copy()
            c = np.stack([t.cov for t in pool])
            for i, t in enumerate(pool):
                if t.state != TRACKED:
                    m[i, 7] = 0
            m, c = kf.multi_predict(m, c)
            for i, t in enumerate(pool):
                t.mean, t.cov = m[i], c[i]

        activated, refound, lost_now, removed_now = [], [], [], []

        # stage 1: pool x high, fused IoU, cost_limit = match_thresh
        matches, u_track, u_det = linear_assignment_limited(_fused(pool, high), self.match_thresh)
        for r, k in matches:
            t = pool[r]
            if t.state == TRACKED:
                t.take(high[k], fid, reactivate=False)
                activated.append(t)
            else:
                t.take(high[k], fid, reactivate=True)
                refound.append(t)

        # stage 2: still-tracked leftovers x low-confidence dets, plain IoU, 0.5
        leftovers = [pool[i] for i in u_track if pool[i].state == TRACKED]
        matches, u_left, _ = linear_assignment_limited(_dist(leftovers, second), 0.5)
        for r, k in matches:
            t = leftovers[r]
            reac = t.state != TRACKED
            t.take(second[k], fid, reactivate=reac)
            (refound if reac else activated).append(t)
        for i in u_left:
            t = leftovers[i]
            if t.state != LOST:
                t.state = LOST
                lost_now.append(t)

        # stage 3: unconfirmed x unmatched high dets, fused IoU, 0.7
        rest = [high[i] for i in u_det]
        matches, u_unc, u_rest = linear_assignment_limited(_fused(unconfirmed, rest), 0.7)
        for r, k in matches:
            unconfirmed[r].take(rest[k], fid, reactivate=False)
            activated.append(unconfirmed[r])
        for i in u_unc:
            unconfirmed[i].state = REMOVED
            removed_now.append(unconfirmed[i])

        # births
        for i in u_rest:
            t = rest[i]
            if t.score < self.det_thresh:
                continue
            t.track_id = self._new_id()
            t.mean, t.cov = kf.initiate(t.xyah)
            t.tracklet_len = 0
            t.state = TRACKED
            if fid == 1:
                t.activated = True
            t.frame_id = fid
            t.start_frame = fid
            activated.append(t)

        # lost-track expiry (end_frame == frame_id)
        for t in self.lost:
            if fid - t.frame_id > self.max_time_lost:
                t.state = REMOVED
                removed_now.append(t)

        tracked = [t for t in self.tracked if t.state == TRACKED]
        tracked = _union(tracked, activated)
        tracked = _union(tracked, refound)
        lost = _minus(self.lost, tracked)
        lost.extend(lost_now)
        lost = _minus(lost, self.removed)
        self.removed.extend(removed_now)
        self.tracked, self.lost = _dedup(tracked, lost)

        rows = [list(t.box()) + [t.track_id, t.score, t.cls, t.det_ind]
                for t in self.tracked if t.activated]
        return np.asarray(rows)

    # ---- introspection for parity tests
    def state_snapshot(self):
        recs = [(0, t) for t in self.tracked] + [(1, t) for t in self.lost]
        return recs
