"""CPU: the oracle reproduces the reference's full-size goldens (tests/golden/full_configs.npz)
where it finishes in seconds: ByteTrack 1024 x 1024 over 45 frames (past Lost-track expiry) and
BoT-SORT 1024 x 1024 with 512-d embeddings.  The 2048 / 4096 cases are checked against the
oracle by make_goldens_full.py itself (lock-step, perturbed LAP) and on the GPU by
tests/test_gpu_full_configs.py."""
import numpy as np

import full_configs as fc
from oracle.botsort import BoTSORTOracle
from oracle.bytetrack import ByteTrackOracle
from test_oracle_golden import reid_features


def test_oracle_bytetrack_1024_45_frames():
    g = fc.load()
    name = "bt_n1024_f45"
    t = ByteTrackOracle(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)
    for f, d in enumerate(fc.bytetrack_frames(g, name)):
        fc.check_frame_close(g, name, f, t.update(d))
    recs = t.state_snapshot()
    assert np.array_equal([tr.track_id for _, tr in recs], g[f"{name}__st_id"])
    np.testing.assert_allclose(np.array([tr.mean for _, tr in recs]), g[f"{name}__st_mean"],
                               rtol=1e-9, atol=1e-8)


def test_oracle_botsort_1024_d512():
    g = fc.load()
    name = "bs_n1024_d512"
    frames, params, D = fc.botsort_frames(g, name)
    t = BoTSORTOracle(**params)
    for f, (dets, embs) in enumerate(frames):
        fc.check_frame_close(g, name, f, t.update(
            dets, reid_features(dets, embs, params["track_high_thresh"])))


def test_oracle_botsort_1024_d512_65_frames():
    """The long C3 golden (tests/golden/full_deep.npz): Lost tracks re-found and expired after
    max_time_lost = 60 (bot_sort.py:339-346, :386-390), every frame's ids and det_ind exact."""
    g = fc.load_deep()
    name = "bs_n1024_d512_f65"
    frames, params, D = fc.botsort_frames(g, name)
    t = BoTSORTOracle(**params)
    for f, (dets, embs) in enumerate(frames):
        fc.check_frame_close(g, name, f, t.update(
            dets, reid_features(dets, embs, params["track_high_thresh"])))
