"""CPU: the host logic of stream-subset updates (yolo_tracking_amd/trackers/_streams.py): ids are
validated and sorted for the C ABI (which takes ascending ids), and the results go back in the
caller's order with the ID counters written to the caller's positions."""
import numpy as np
import pytest

from yolo_tracking_amd.trackers._streams import StreamSubset


class _Eng(StreamSubset):
    n_streams = 5


def test_subset_sorts_and_validates():
    e = _Eng()
    ids, order = e._subset([3, 0, 4], 3)
    assert ids.dtype == np.int32 and list(ids) == [0, 3, 4] and list(order) == [1, 0, 2]
    assert e._reorder(["a", "b", "c"], order) == ["b", "a", "c"]
    assert e._reorder(None, order) is None
    for bad, n in (([1, 1], 2), ([5], 1), ([-1], 1), ([0, 1], 3), ([], 0)):
        with pytest.raises(ValueError):
            e._subset(bad, n)


def test_subset_result_back_in_caller_order():
    e = _Eng()
    ids, order = e._subset([4, 1], 2)          # sorted: [1, 4], order [1, 0]
    e._out = np.arange(5 * 8, dtype=np.float64).reshape(5, 8)
    o = np.array([0, 2, 5], np.int32)           # stream 1: rows 0-1, stream 4: rows 2-4
    nid_user = np.zeros(2, np.int64)
    e._subset_check(0, order, np.array([11, 44], np.int64), nid_user)
    res = e._subset_result(o, order)
    assert res[0].shape == (3, 8) and res[1].shape == (2, 8)   # caller's [4, 1]
    assert np.array_equal(res[1], e._out[0:2]) and np.array_equal(res[0], e._out[2:5])
    assert list(nid_user) == [44, 11]


def test_subset_counters_written_back_before_an_error():
    """The C layer advances the listed streams' counters even when it then reports an error:
    they reach the caller's next_id (a list too) before the exception."""
    from yolo_tracking_amd import _lib
    e = _Eng()
    _, order = e._subset([4, 1], 2)
    nid_user = [0, 0]
    with pytest.raises(_lib.YTAError):
        e._subset_check(_lib.YTA_ERR_INVALID, order, np.array([11, 44], np.int64), nid_user)
    assert nid_user == [44, 11]
