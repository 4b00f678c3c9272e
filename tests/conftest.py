import ctypes
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle as O
    return O


_hip = None


def _device_fault():
    """hipDeviceSynchronize's error name if the device holds a sticky fault
    (an illegal address of any kernel or copy so far), else None.  Uses the
    HIP runtime torch already loaded (one runtime per process)."""
    global _hip
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_available():
        return None
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipGetErrorName.restype = ctypes.c_char_p
    rc = _hip.hipDeviceSynchronize()
    return None if rc == 0 else _hip.hipGetErrorName(rc).decode()


@pytest.fixture(autouse=True)
def _gpu_fault_check(request):
    """Every `gpu` test starts on a healthy device and leaves one behind: a
    fault raised by a test's last kernels, copies or teardown fails THAT test
    (VERDICT r5 item 1), not the next test's first copy."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    err = _device_fault()
    if err:
        pytest.fail(f"device already faulted before this test: {err}", pytrace=False)
    yield
    import gc

    gc.collect()  # (queues and buffers the test dropped are destroyed now)
    err = _device_fault()
    if err:
        pytest.fail(f"device fault left by this test: {err}", pytrace=False)
