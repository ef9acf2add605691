"""Pin of the acos convention of FCCF.cpp:369-377 (`float theta=acos(cos_theta)*180/M_PI;`).

FCCF.cpp has no `using namespace std`, so the unqualified `acos(float)` binds to the
float overload only if some PCL/VTK/FLANN header pulled libstdc++'s <math.h> wrapper
into the global namespace; otherwise it is C's double `acos`.  And the float overload's
last bit depends on the reference build's glibc acosf.  The oracle (and the HIP
product's exact cosine cut points, fccf_math.h) follow the correctly rounded float
overload; this test runs the oracle under all three candidates (oracle/fccf_oracle.cpp
theta_of_cos) and asserts that no thresholded decision flips at c2-c5:

  grow/merge    normal-angle gates of plane growth (FCCF.cpp:381, :605-628 of the oracle)
  rough         the roughness class of each plane (mean angle vs rough_threshold_gl)
  base          the included-angle window of base pairs (FCCF.cpp:443)
  pair          |angle1 - angle2| < included_angle_same_threshold between bases
  third         the third-plane normal gate (FCCF.cpp:957)
  cluster       the rotation-cluster gate (FCCF.cpp:1109)
  verify        the quick-verify normal gate (FCCF.cpp:722)

and that every discrete output of the registration (growth allocation, candidates,
fine/quick/final verification, the chosen transform) is identical across conventions.
Only stored angle values differ (base angles; roughness sums under the double form).
The per-site counts are recorded in DESIGN.md §3.
"""
import numpy as np
import pytest

import oracle_py as O

DISCRETE = ("galloc1", "galloc2", "cand0", "cand1", "cand2", "fine0", "fine1", "fine2",
            "qv0", "fv0", "high", "counts", "T")


def _run(src, tar, leaf, mode):
    prev = O.set_acos_mode(mode)
    try:
        O.acos_audit(reset=True)
        r = O.Run(src, tar, leaf)
        audit = O.acos_audit(reset=True)
    finally:
        O.set_acos_mode(prev)
    out = {}
    for k in DISCRETE:
        v = r.get(k, np.uint8)
        out[k] = None if v is None else v.tobytes()
    for k in ("bases1", "bases2"):
        b = r.get(k, np.int32).reshape(-1, 4)
        out[k] = b[:, [0, 1, 3]].tobytes()  # (i1, i2, roughness type); column 2 is the angle
    return out, audit


def test_modes_differ_on_single_angles():
    """The three conventions are really different functions (else the pin is vacuous)."""
    rng = np.random.default_rng(0)
    seen = set()
    for _ in range(2000):
        a, b = rng.normal(size=3).astype(np.float32), rng.normal(size=3).astype(np.float32)
        vals = []
        for m in (O.ACOS_CR_FLOAT, O.ACOS_LIBM_FLOAT, O.ACOS_DOUBLE):
            prev = O.set_acos_mode(m)
            vals.append(np.float32(O.normal_angle(a, b)).view(np.uint32))
            O.set_acos_mode(prev)
        seen.add((vals[0] != vals[1], vals[0] != vals[2]))
    assert (False, True) in seen or (True, True) in seen  # double form differs somewhere
    assert O.set_acos_mode(O.ACOS_CR_FLOAT) == O.ACOS_CR_FLOAT  # default restored


@pytest.mark.parametrize("cname", ["c2", "c3", "c4", "c5"])
def test_no_decision_flips_between_acos_conventions(fccf, cname):
    c = fccf.CONFIGS[cname]
    src, tar, _ = fccf.synth_pair(c["n"], c["room"])
    base, audit = _run(src, tar, c["leaf"], O.ACOS_CR_FLOAT)
    print(cname, {k: v for k, v in audit.items()})
    flips = {k: v[2] for k, v in audit.items() if v[2]}
    assert not flips, flips
    assert audit["grow"][0] > 0 and audit["pair"][0] > 0  # the sites were exercised
    assert sum(v[1] for v in audit.values()) > 0  # ... with differing angle bits
    for mode in (O.ACOS_LIBM_FLOAT, O.ACOS_DOUBLE):
        other, _ = _run(src, tar, c["leaf"], mode)
        diff = [k for k in base if base[k] != other[k]]
        assert not diff, (mode, diff)
