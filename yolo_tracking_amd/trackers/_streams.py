"""Stream-subset helpers shared by the engine classes (SURVEY.md §8(b) update(ctx, n_streams,
stream_ids, ...)): a subset call lists the streams to update; every other stream of the engine is
left exactly as it was (the C ABI's *_update_streams)."""
import numpy as np

from .. import _lib


class StreamSubset:
    def _subset(self, streams, n_items):
        """Validated stream ids as an ascending int32 array + the order that sorts the caller's
        per-stream lists (results are handed back in the caller's order)."""
        ids = np.asarray(streams, dtype=np.int64).reshape(-1)
        if len(ids) != n_items or len(ids) == 0:
            raise ValueError("one entry per listed stream")
        order = np.argsort(ids, kind="stable")
        ids = ids[order]
        if ids[0] < 0 or ids[-1] >= self.n_streams or np.any(np.diff(ids) == 0):
            raise ValueError(f"stream ids must be distinct and in 0..{self.n_streams - 1}")
        return np.ascontiguousarray(ids, dtype=np.int32), order

    @staticmethod
    def _reorder(v, order):
        return None if v is None else [v[k] for k in order]

    @staticmethod
    def _subset_check(rc, order, nid, nid_user):
        """Hand the listed streams' ID counters back to the caller's next_id (any sequence, in the
        caller's order) BEFORE raising on rc: the C layer advances them even when it reports an
        error after the launch (include/yolo_tracking_amd.h, host-buffer update rules)."""
        if nid_user is not None and nid is not None:
            for k, pos in enumerate(order):
                nid_user[pos] = int(nid[k])
        _lib.check(rc)

    def _subset_result(self, o, order):
        res = [None] * len(order)
        for k, pos in enumerate(order):
            res[pos] = self._out[o[k]:o[k + 1]].copy()
        return res
