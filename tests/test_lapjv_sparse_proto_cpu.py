"""CPU: the sparse-sweep restatement of lapjv's phase 3 (tools/lapjv_sparse_proto.c, the next step
for the GIoU-surge replay) gives oracle/lapjv.c's exact assignment on
surge-shaped (exact zeros, a few negative entries per column) and denser matrices."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import lapjv_sparse_check as chk  # noqa: E402


@pytest.mark.parametrize("na,nb,per_col,pos_frac", [(200, 100, 4, 0.0), (100, 200, 3, 0.0),
                                                    (600, 300, 4, 0.0), (300, 300, 6, 0.0),
                                                    (500, 250, 4, 0.01), (400, 200, 2, 0.2)])
@pytest.mark.parametrize("seed", range(3))
def test_sparse_sweeps_replay_lapjv(na, nb, per_col, pos_frac, seed):
    proto, orc = chk.load()
    rng = np.random.default_rng(seed * 1000 + na + nb)
    ok, st, _, _ = chk.run(proto, orc, chk.surge(rng, na, nb, per_col, pos_frac))
    assert ok
    assert st[0] > 0   # some sweeps did take the sparse path
