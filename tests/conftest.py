import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")


def _make(target_dir, *args):
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, target_dir)] + list(args))


@pytest.fixture(scope="session")
def oracle():
    """ctypes handle on our CPU restatement (test infrastructure only)."""
    import ctypes
    path = os.path.join(REPO, "oracle", "liboracle_ed25519.so")
    if not os.path.exists(path):
        _make("oracle")
    lib = ctypes.CDLL(path)
    lib.fdo_verify.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    lib.fdo_verify_batch_single_msg.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    lib.fdo_sha512.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    lib.fdo_scalar_reduce.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.fdo_verify_descs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    return lib


@pytest.fixture(scope="session")
def gpu():
    """Verify context on cuda:0.  Fails loudly (no fallback) if the HIP library or device is missing."""
    import firedancer_amd as fa
    g = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 16)
    yield g
    g.close()
