"""Shared helpers for the parity tests (oracle side is test infrastructure)."""
import numpy as np

import dtsffi as D
import orc


def oracle_frame(src, sw, sh, sfmt, w, h, fmt, method, param=(D.PARAM_DEFAULT, D.PARAM_DEFAULT)):
    return orc.scale_frame(src, sw, sh, sfmt, w, h, fmt, method, param)


def planes_equal(a, b):
    """Plane lists equal: same plane count (None where a format has no plane) and
    every plane bit-exact."""
    a, b = list(a), list(b)
    if len(a) != len(b):
        return False
    for pa, pb in zip(a, b):
        if (pa is None) != (pb is None):
            return False
        if pa is None and pb is None:
            continue
        if not np.array_equal(np.asarray(pa), np.asarray(pb)):
            return False
    return True


def first_diff(a, b):
    a, b = list(a), list(b)
    if len(a) != len(b):
        return f"plane count {len(a)} vs {len(b)}"
    for i, (pa, pb) in enumerate(zip(a, b)):
        if (pa is None) != (pb is None):
            return f"plane {i} present in one frame only"
        if pa is None:
            continue
        d = np.argwhere(np.asarray(pa) != np.asarray(pb))
        if len(d):
            y, x = d[0]
            return f"plane {i} first diff at (y={y}, x={x}): got {pa[y, x]} want {pb[y, x]}; {len(d)} diffs"
    return "equal"


def random_frame(w, h, fmt, rng):
    planes = D.alloc_frame(w, h, fmt)
    for p in planes:
        if p is not None:
            p[...] = rng.integers(0, 256, p.shape, dtype=np.uint8)
    return planes
