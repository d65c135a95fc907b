"""The committed K5 pose trace (tests/golden/k5_trace.npz, written by
tests/golden/make_k5_trace.py) is the pinned oracle's answer for the bench's
stream: its input is the stream navslam.synth generates (SHA-256), and its
first frames regenerate bit for bit from OracleSlam here, so the GPU tests
and the K5 bench line that read it compare against the oracle itself."""
import hashlib
import os

import numpy as np
import pytest

HERE = os.path.dirname(__file__)
TRACE = os.path.join(HERE, "golden", "k5_trace.npz")


@pytest.fixture(scope="module")
def trace():
    with np.load(TRACE) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def stream(trace):
    from navslam.synth import l9_stream
    R, C, F, seed = (int(trace[k]) for k in ("R", "C", "F", "seed"))
    return l9_stream(R, C, F, seed=seed)


def test_trace_covers_the_configured_stream(trace):
    n = len(trace["pose"])
    assert n >= 1000  # BASELINE.json configs[4]: a 10k-frame stream (the generator's default)
    assert trace["pose"].shape == (n, 6) and np.isfinite(trace["pose"]).all()
    for k in ("error", "iters", "corr"):
        assert trace[k].shape == (n,)
    assert (trace["corr"] > 0).all() and (trace["iters"] > 0).all()
    assert (int(trace["R"]), int(trace["C"]), int(trace["F"]), int(trace["seed"])) == (128, 2048, 8, 11)


def test_trace_input_is_the_bench_stream(trace, stream):
    dig = hashlib.sha256(np.ascontiguousarray(stream, np.float64).tobytes()).hexdigest()
    assert dig == str(trace["frames_sha256"])


def test_trace_prefix_regenerates_bit_exact(trace, stream, orc):
    from pyoracle import OracleSlam
    from navslam.synth import l9_stream_index
    F = int(trace["F"])
    s = OracleSlam(orc, stream.shape[1], stream.shape[2])
    zero = np.zeros(6)
    s.init(zero, stream[0])
    last = zero
    for i in range(1, 4):
        f = stream[l9_stream_index(i, F)]
        meas, it, nc = s.localization(f, last, last)
        s.mapping(meas, f)
        np.testing.assert_array_equal(meas, trace["pose"][i - 1])
        assert s.error == trace["error"][i - 1]
        assert (it, nc) == (trace["iters"][i - 1], trace["corr"][i - 1])
        last = meas
