"""Regression: pipelined batches whose graph captures overlap cross-thread event waits.
Before the capture lock (csrc/ctx.h capture_mutex) this hung or failed with
hipErrorStreamCaptureIsolation within the first rounds.  Runs tools/capture_stress.py
in a child process, so a regression ends at the time limit instead of hanging pytest."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capture_stress_rounds():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "capture_stress.py"), "8"],
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "round 7 ok" in r.stdout
