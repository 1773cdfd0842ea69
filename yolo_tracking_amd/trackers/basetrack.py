"""Track-state constants and the process-global ID counter.

Mirrors boxmot/trackers/bytetrack/basetrack.py:8-55: `TrackState` values and `BaseTrack._count`,
which every ByteTrack tracker in the process shares (never reset by the reference).  The device
engine allocates IDs itself; the Python tracker passes this counter in and reads it back each
frame so that several trackers in one process interleave IDs exactly like the reference.
"""


class TrackState:
    New = 0
    Tracked = 1
    Lost = 2
    Removed = 3


class BaseTrack:
    _count = 0

    @staticmethod
    def next_id():
        BaseTrack._count += 1
        return BaseTrack._count

    @staticmethod
    def clear_count():
        BaseTrack._count = 0
