"""ORACLE — test infrastructure only.

CPU restatement of the reference (BoxMOT 10.0.51) `tracker.update()` hot path, used exclusively
as the *checker* by `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py`.
Nothing in `yolo_tracking_amd/` imports this package; the product path runs on the HIP library and
fails loudly when that library is missing.

Parity pinning: the restatement is checked against golden vectors generated from the reference
itself (imported read-only in the build container, see `tests/golden/make_goldens.py`) and against
the reference's own known-answer test (`tests/test_python.py:165-185`).  The reference's LAP
dependency `lapx` is absent from the image; `oracle/lapjv.c` restates its published algorithm, and
its tie-breaking is therefore "parity unpinned" (goldens are checked tie-free).
"""
