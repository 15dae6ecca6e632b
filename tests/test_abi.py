"""CPU: the C-ABI library loads and exports every function include/fd_ed25519_gpu.h
declares; the host-only helpers behave like the reference (no GPU needed)."""
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "fd_ed25519_gpu.h")


@pytest.fixture(scope="module")
def lib():
    import firedancer_amd as fa
    if not os.path.exists(fa.lib_path()):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "firedancer_amd")])
    return fa.load_lib()


def declared_functions(path=HDR, prefix="fd_"):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(%s\w+)\s*\(" % prefix, src)))


def exported(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path]).decode()
    return set(l.split()[-1] for l in out.splitlines() if " T " in l)


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ["fd_ed25519_gpu_new", "fd_ed25519_gpu_delete", "fd_ed25519_verify_batch_gpu",
              "fd_ed25519_gpu_submit", "fd_ed25519_gpu_poll", "fd_ed25519_verify_batch_gpu_dev",
              "fd_ed25519_gpu_verify", "fd_ed25519_gpu_verify_batch_single_msg", "fd_ed25519_gpu_txn_reduce",
              "fd_ed25519_gpu_strerror"]:
        assert f in fns


def test_library_exports_every_declared_symbol(lib):
    import firedancer_amd as fa
    missing = [f for f in declared_functions() if f not in exported(fa.lib_path())]
    assert not missing, missing
    for f in declared_functions():
        getattr(lib, f)


def test_offload_headers_and_libraries():
    """include/fd_verify_offload.h: the client/link functions live in the
    HIP-free libfd_verify_offload.so (a sandboxed tile links only that), the
    server loop in libfd_ed25519_gpu.so; the server executable is built."""
    import firedancer_amd as fa
    fa.load_offload_lib()
    decl = declared_functions(os.path.join(REPO, "include", "fd_verify_offload.h"))
    link = exported(fa.offload.offload_lib_path())
    gpu = exported(fa.lib_path())
    assert [f for f in decl if f != "fd_verify_offload_serve" and f not in link] == []
    assert "fd_verify_offload_serve" in gpu
    needed = subprocess.check_output(["readelf", "-d", fa.offload.offload_lib_path()]).decode()
    assert "amdhip64" not in needed
    assert os.access(fa.server_path(), os.X_OK)


def test_strerror_matches_reference_strings(lib):
    import firedancer_amd as fa
    # fd_ed25519_strerror (src/ballet/ed25519/fd_ed25519_user.c:311-321)
    assert fa.strerror(0) == "success"
    assert fa.strerror(-1) == "bad signature"
    assert fa.strerror(-2) == "bad public key"
    assert fa.strerror(-3) == "bad message"
    assert fa.strerror(12345) == "unknown"


def _desc(groups):
    import firedancer_amd as fa
    d = np.zeros(sum(groups), fa.DESC_DTYPE)
    i = 0
    for t, g in enumerate(groups):
        d["txn_idx"][i:i + g] = t
        i += g
    return d


def test_txn_reduce_precedence(lib):
    """Two-phase precedence of fd_ed25519_verify_batch_single_msg (fd_ed25519_user.c:262-307)."""
    import firedancer_amd as fa
    cases = [
        ([0, 0, 0], 0),
        ([-3, -1], -1),          # phase-1 error at j=1 beats phase-2 error at j=0
        ([0, 0, -2, -3], -2),
        ([-3, 0, -3], -3),
        ([-2, -1], -2),          # first phase-1 error wins
        ([-1, -2], -1),
        ([0], 0), ([-3], -3),
    ]
    codes = np.array([c for cs, _ in cases for c in cs], np.int8)
    d = _desc([len(cs) for cs, _ in cases])
    got = fa.txn_reduce(codes, d)
    assert list(got) == [e for _, e in cases]
    # a run longer than 16 is rejected like batch_sz > 16 (fd_ed25519_user.c:238-240)
    assert list(fa.txn_reduce(np.zeros(17, np.int8), _desc([17]))) == [-1]


def test_txn_reduce_against_golden_precedence(lib):
    """Per-sig codes -> per-txn codes reproduce the reference batch codes for every
    golden multi-sig record whose per-sig codes the oracle can give."""
    import ctypes
    import firedancer_amd as fa
    from golden_io import read_txns
    orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle_ed25519.so")) if os.path.exists(
        os.path.join(REPO, "oracle", "liboracle_ed25519.so")) else None
    if orc is None:
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
        orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle_ed25519.so"))
    orc.fdo_verify.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    txns = [t for t in read_txns() if 1 <= t["n"] <= 16]
    codes, groups = [], []
    for t in txns:
        groups.append(t["n"])
        for j in range(t["n"]):
            codes.append(orc.fdo_verify(t["msg"], len(t["msg"]), t["sigs"][j], t["pubs"][j], 0))
    got = fa.txn_reduce(np.array(codes, np.int8), _desc(groups))
    assert list(got) == [t["code"] for t in txns]


def test_pack_batch_layout():
    import firedancer_amd as fa
    recs = [(b"abc", bytes(range(64)), bytes(range(32))), (b"", bytes(64), bytes(32))]
    arena, desc, sz = fa.pack_batch(recs)
    assert sz == 96 * 2 + 3
    assert bytes(arena[desc[0]["sig_off"]:desc[0]["sig_off"] + 64]) == bytes(range(64))
    assert bytes(arena[desc[0]["msg_off"]:desc[0]["msg_off"] + 3]) == b"abc"
    assert desc[1]["msg_sz"] == 0
    assert len(arena) >= sz + 8     # kernel may read up to align_up(sz,4)+8


def test_shard_ranges_cover_exactly():
    from firedancer_amd.shard import shard_range
    for n in [0, 1, 7, 65536, 1 << 20, 1000003]:
        for parts in [1, 2, 3, 4, 8]:
            rs = [shard_range(n, i, parts) for i in range(parts)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(parts - 1))


def test_txn_reduce_long_run_is_err_sig_not_an_error():
    """fd_ed25519_gpu_txn_reduce (host function, no GPU): a run of 17
    descriptors of one txn is reported as FD_ED25519_ERR_SIG for that txn,
    like the reference's batch_sz > 16 (fd_ed25519_user.c:238-240), and the
    call returns the run count, not an error (include/fd_ed25519_gpu.h)."""
    import numpy as np
    import firedancer_amd as fa
    desc = np.zeros(17 + 3 + 16, fa.DESC_DTYPE)
    desc["txn_idx"][:17] = 5
    desc["txn_idx"][17:20] = 6
    desc["txn_idx"][20:] = 7
    codes = np.zeros(len(desc), np.int8)
    codes[18] = fa.FD_ED25519_ERR_MSG
    codes[19] = fa.FD_ED25519_ERR_PUBKEY
    codes[35] = fa.FD_ED25519_ERR_MSG
    out = fa.txn_reduce(codes, desc)
    assert list(out) == [fa.FD_ED25519_ERR_SIG, fa.FD_ED25519_ERR_PUBKEY, fa.FD_ED25519_ERR_MSG]
    lib = fa.load_lib()
    small = np.zeros(1, np.int8)
    import ctypes
    t = lib.fd_ed25519_gpu_txn_reduce(codes.ctypes.data_as(ctypes.c_void_p), desc.ctypes.data_as(ctypes.c_void_p),
                                      len(desc), small.ctypes.data_as(ctypes.c_void_p), 1)
    assert t == 3 and small[0] == fa.FD_ED25519_ERR_SIG      # runs past out_cap are counted, not written


def test_queue_depth_mirror_matches_header():
    """firedancer_amd.QUEUE_DEPTH mirrors FD_ED25519_GPU_QUEUE_DEPTH: the pipelined
    kernel's three phases plus two queued launches."""
    import re
    import firedancer_amd as fa
    h = open(os.path.join(REPO, "include", "fd_ed25519_gpu.h")).read()
    m = re.search(r"#define FD_ED25519_GPU_QUEUE_DEPTH (\d+)", h)
    assert m and int(m.group(1)) == fa.QUEUE_DEPTH == 5
    m = re.search(r"#define FD_ED25519_GPU_STAGE_DEPTH (\d+)", h)
    assert m and int(m.group(1)) == fa.STAGE_DEPTH > fa.QUEUE_DEPTH
