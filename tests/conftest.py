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


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Which HIP runtime the library ran on in this process (torch's bundled one when
    torch was imported first, /opt/rocm's otherwise; fd_ed25519_gpu_runtime), also
    written to gpurun_out/tests_runtime.json for the round's records."""
    try:
        import json
        import firedancer_amd.ed25519 as e
        if e._LIB is None:
            return
        info = {"runtime": e.runtime_info(), "build": e.build_id(), "torch_loaded": "torch" in sys.modules,
                "markexpr": config.getoption("markexpr", "")}
    except Exception:      # noqa: BLE001 -- a summary line must never fail the run
        return
    terminalreporter.write_line("fd_ed25519_gpu runtime: %s (torch loaded: %s)" % (info["runtime"], info["torch_loaded"]))
    try:
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", "tests_runtime.json"), "w") as f:
            json.dump(info, f)
    except OSError:
        pass
