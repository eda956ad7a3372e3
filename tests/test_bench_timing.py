"""bench.py's launch-duration bookkeeping on the CPU: the timed launches' dispatch-to-completion
times derived from their in-kernel stamps (bench.queued_durations), as rocprofv3 reports a
launch queued on an in-order stream."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_queued_durations_follow_each_stream():
    # three streams, launches i on stream i % 3; every launch runs 10 ticks of its own, the
    # first three start together at 100 and the later ones wait for CU room
    sp = np.array([[100, 110], [100, 112], [101, 115],
                   [110, 121], [113, 125], [118, 130]])
    d = bench.queued_durations(sp, 3)
    # a stream's first launch from the first start of all; later ones from their stream's
    # previous end (dispatch), so a launch's wait for room counts, as in rocprofv3's trace
    assert d.tolist() == [10, 12, 15, 11, 13, 15]
    assert (d >= sp[:, 1] - sp[:, 0]).all()   # never shorter than the in-kernel span


def test_queued_durations_one_stream_is_back_to_back():
    sp = np.array([[0, 5], [6, 11], [12, 20]])
    assert bench.queued_durations(sp, 1).tolist() == [5, 6, 9]


def test_shader_clock_from_span_records():
    # [start, end, shader cycles summed over workgroups, real-time ticks summed over them]:
    # 21,000 cycles over 1,000 ticks (10 us at 100 MHz) = 2,100 MHz
    sp = np.array([[0, 10, 10_000, 500], [5, 15, 11_000, 500]])
    assert abs(bench.shader_clock_mhz(sp) - 2100.0) < 1e-9
    assert bench.shader_clock_mhz(np.zeros((2, 4), np.int64)) is None
