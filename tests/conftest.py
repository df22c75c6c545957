import os
import sys
import time
import weakref

import pytest

try:        # load torch's HIP runtime first so libdts binds to the same one (see bench.py)
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-transcoding-server_amd")
for p in (os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

# Graphs a test made: closed at the end of that test (not whenever __del__ runs), so their
# teardown -- slot events, the D2H stream, hipFree / hipHostFree -- happens inside the test
# that owns them and before the device check below
_LIVE_GRAPHS = []


def _track_graphs():
    import dtsffi
    if getattr(dtsffi.Graph, "_tracked", False):
        return
    init = dtsffi.Graph.__init__

    def tracked_init(self, *a, **k):
        init(self, *a, **k)
        _LIVE_GRAPHS.append(weakref.ref(self))
    dtsffi.Graph.__init__ = tracked_init
    dtsffi.Graph._tracked = True


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")


@pytest.fixture(scope="session")
def ctx():
    import dtsffi
    if dtsffi.device_count() < 1:
        pytest.fail("gpu test without a HIP device: the HIP path must run, there is no fallback")
    c = dtsffi.Context(0)
    yield c
    c.close()


# How long a GPU test's teardown waits, after its last synchronise, before checking the
# device again: a page fault of a kernel whose waves completed reaches the runtime
# asynchronously (GPUTEST_r05: reported at the NEXT test's first HIP call), so the check
# gives it time to arrive and charges it to the test that launched the work
GPU_SETTLE_S = float(os.environ.get("DTS_TEST_SETTLE_S", "0.02"))


@pytest.fixture(autouse=True)
def gpu_device_check(request):
    """Per GPU test: close the test's graphs, synchronise the device, let any asynchronous
    fault report arrive, and synchronise again -- a HIP error surfaces in the teardown of the
    test that caused it, not in whichever test touches HIP next."""
    if request.node.get_closest_marker("gpu") is None or torch is None:
        yield
        return
    _track_graphs()
    del _LIVE_GRAPHS[:]
    yield
    for r in _LIVE_GRAPHS:
        g = r()
        if g is not None:
            g.close()
    del _LIVE_GRAPHS[:]
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        time.sleep(GPU_SETTLE_S)
        torch.cuda.synchronize()
