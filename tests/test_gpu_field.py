"""GPU: the device field and group operations (inline-asm products, limb-pair
adds, the complement-form square, the negated-E/G doubling, v_xad_u32
negation) held limb for limb against the host build of the same headers
(tests/csrc/field_host_check.cpp t_op), on inputs at the documented limb bounds
(firedancer_amd/csrc/fd_f25519_dev.h R / M / F classes) and random ones.  The
host build is itself pinned to big-int arithmetic at those bounds by
tests/test_field_bounds.py, so equality here carries that pin to the device
code through fd_ed25519_gpu_test_field."""
import ctypes
import os
import subprocess
import zlib

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R_E, R_O = 2**26 + 2**11, 2**25 + 2**16
M_E, M_O = 3 * 2**26 + 2**13, 3 * 2**25 + 2**18
F_E, F_O = 5 * 2**26 + 3 * 2**11, 5 * 2**25 + 3 * 2**16
N = 4096


@pytest.fixture(scope="module")
def host():
    out = os.path.join(REPO, "tests", "_build")
    os.makedirs(out, exist_ok=True)
    so = os.path.join(out, "field_host_check.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(REPO, "tests", "csrc", "field_host_check.cpp")])
    lib = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    lib.t_op.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_uint64]
    return lib


@pytest.fixture(scope="module")
def gpu():
    import firedancer_amd as fa
    g = fa.Ed25519Gpu(device_mask=1, max_batch=4096)
    yield g
    g.close()


def limbs(rng, n, be, bo, maxfrac=0.25):
    """n x 10 limbs below (be, bo); a quarter of the rows at the maxima."""
    hi = np.array([be if i % 2 == 0 else bo for i in range(10)], dtype=np.uint64)
    x = (rng.random((n, 10)) * (hi + 1)).astype(np.uint64)
    k = int(n * maxfrac)
    x[:k] = hi
    x[k:k + 16] = 0
    return x.astype(np.uint32)


def rec(*parts):
    """[n, 40] records from up to four [n, 10] limb blocks (rest zero)."""
    n = parts[0].shape[0]
    out = np.zeros((n, 40), dtype=np.uint32)
    for k, p in enumerate(parts):
        out[:, 10 * k:10 * k + 10] = p
    return out


def host_op(host, op, a, b):
    out = np.zeros_like(a)
    vp = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    host.t_op(op, vp(a), vp(b), vp(out), len(a))
    return out


def sub4p(x):
    c = np.array([4 * (2**26 - 19)] + [4 * (2**26 - 1) if i % 2 == 0 else 4 * (2**25 - 1) for i in range(1, 10)], dtype=np.uint64)
    return (c - x.astype(np.uint64)).astype(np.uint32)


CASES = {
    "mul_MxM": (0, lambda r: (rec(limbs(r, N, M_E, M_O)), rec(limbs(r, N, M_E, M_O)))),
    "mul_FxM": (0, lambda r: (rec(limbs(r, N, F_E, F_O)), rec(limbs(r, N, M_E, M_O)))),
    "sq": (1, lambda r: (rec(limbs(r, N, M_E, M_O)), rec(limbs(r, N, 0, 0)))),
    "sq_neg": (2, lambda r: (rec(limbs(r, N, M_E, M_O)), rec(limbs(r, N, 0, 0)))),
    "sq_seed": (3, lambda r: (rec(limbs(r, N, M_E, M_O)), rec(sub4p(limbs(r, N, 2 * R_E, 2 * R_O))))),
    "add": (4, lambda r: (rec(limbs(r, N, F_E, F_O)), rec(limbs(r, N, M_E, M_O)))),
    "sub": (5, lambda r: (rec(limbs(r, N, R_E, R_O)), rec(limbs(r, N, R_E, R_O)))),
    "lshl1_add": (6, lambda r: (rec(limbs(r, N, R_E, R_O)), rec(limbs(r, N, M_E, M_O)))),
    "cneg": (7, lambda r: (rec(limbs(r, N, R_E, R_O)), rec((r.random((N, 10)) < 0.5).astype(np.uint32)))),
    "dbl": (8, lambda r: (rec(*[limbs(r, N, R_E, R_O) for _ in range(4)]), rec(limbs(r, N, 0, 0)))),
    "add_cached": (9, lambda r: (rec(*[limbs(r, N, R_E, R_O) for _ in range(4)]),
                                 rec(limbs(r, N, M_E, M_O), limbs(r, N, M_E, M_O), limbs(r, N, R_E, R_O),
                                     limbs(r, N, M_E, M_O)))),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_device_field_ops_match_host(host, gpu, case):
    op, make = CASES[case]
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    a, b = make(rng)
    dev = gpu.test_field(op, a, b)
    ref = host_op(host, op, a, b)
    bad = np.nonzero((dev != ref).any(axis=1))[0]
    assert len(bad) == 0, (case, len(bad), a[bad[0]].tolist(), dev[bad[0]].tolist(), ref[bad[0]].tolist())
