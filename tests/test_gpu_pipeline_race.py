"""Regression: a graph capture concurrent with another thread's wait on an event of the
capturing stream -- the pipelined batch's hazard (pipeline.cpp: the helper thread's
waits on ev[3]/ev[5] while phase B captures).  Before the capture lock (csrc/ctx.h
capture_mutex, guarded_stream_wait) that wait failed with
hipErrorStreamCaptureIsolation or hung.

test_forced_capture_race forces the interleaving once (fccf_debug_capture_race): the
capturing thread releases the waiter from inside the capture and then holds it for
200 ms, so the guarded wait must block until the capture ends and then succeed.
test_capture_stress_rounds keeps the end-to-end batch loop (tools/capture_stress.py)
in a child process so a regression ends at its time limit instead of hanging pytest."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_forced_capture_race(ctx):
    r = ctx.capture_race(hold_ms=200, guard=True)
    assert r["wait_error"] == 0, r
    assert r["after_capture"], r               # the wait could not slip into the capture
    assert r["wait_ms"] >= 0.9 * r["hold_ms"] and r["hold_ms"] >= 190, r


def test_capture_stress_rounds():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "capture_stress.py"), "8"],
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "round 7 ok" in r.stdout
