"""Negative control for tests/test_gpu_pipeline_race.py (run by hand, in its own
process, under a time limit): the same forced interleaving with the capture lock
bypassed.  Prints the hook's result; a non-zero wait_error (or a hang, which the
caller's time limit ends) shows that the lock is what the regression test exercises."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd  # noqa: E402

c = fccf_amd.Ctx(0)
print("guarded  ", c.capture_race(200, True), flush=True)
try:
    print("unguarded", c.capture_race(200, False), flush=True)
except Exception as e:  # the capture itself may be invalidated by the foreign wait
    print("unguarded raised:", e, flush=True)
