"""ctypes mirror of include/fd_verify_offload.h: the shared-memory link between
a sandboxed verify tile (client: publish frags, read results -- only
libfd_verify_offload.so, no HIP) and the GPU offload process (server:
fd_verify_offload_serve in libfd_ed25519_gpu.so, or the executable
firedancer_amd/fd_verify_offload_server).  SURVEY.md §8(f) next-1."""
import ctypes
import os
import threading

import numpy as np

from .ed25519 import GpuError, _HERE, load_lib, strerror

ERR_FULL, ERR_ARG, ERR_SEQ = -1, -2, -3
_OLIB = None


def offload_lib_path():
    """The in-tree link library; FD_VERIFY_OFFLOAD_LIB may name a test build
    of the same source (tests/csrc/Makefile asan: ASan + UBSan)."""
    return os.environ.get("FD_VERIFY_OFFLOAD_LIB") or os.path.join(_HERE, "libfd_verify_offload.so")


def server_path():
    return os.path.join(_HERE, "fd_verify_offload_server")


def load_offload_lib():
    """The client library (no HIP dependency)."""
    global _OLIB
    if _OLIB is not None:
        return _OLIB
    path = offload_lib_path()
    if not os.path.exists(path):
        raise GpuError("libfd_verify_offload.so not built (make -C firedancer_amd)")
    lib = ctypes.CDLL(path)
    vp, u64, i64, i32, cp = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p
    for fn, res, args in [
        ("fd_verify_offload_create", vp, [cp, u64, u64]), ("fd_verify_offload_join", vp, [cp]),
        ("fd_verify_offload_leave", None, [vp]), ("fd_verify_offload_unlink", i32, [cp]),
        ("fd_verify_offload_depth", u64, [vp]), ("fd_verify_offload_dcache_sz", u64, [vp]),
        ("fd_verify_offload_publish", i64, [vp, vp, ctypes.c_uint32]),
        ("fd_verify_offload_result", i32, [vp, u64, vp, vp]),
        ("fd_verify_offload_publish_burst", u64, [vp, vp, vp, u64]),
        ("fd_verify_offload_results", u64, [vp, u64, u64, vp, vp]),
        ("fd_verify_offload_prod_seq", u64, [vp]), ("fd_verify_offload_done_seq", u64, [vp]),
        ("fd_verify_offload_halt", None, [vp]), ("fd_verify_offload_halted", i32, [vp]),
        ("fd_verify_offload_cons_seq", u64, [vp]), ("fd_verify_offload_avail", u64, [vp, vp]),
        ("fd_verify_offload_frag_laddr", vp, [vp, u64]), ("fd_verify_offload_result_laddr", vp, [vp, u64]),
        ("fd_verify_offload_sig_laddr", vp, [vp, u64]), ("fd_verify_offload_dcache", vp, [vp]),
        ("fd_verify_offload_take", None, [vp, u64]), ("fd_verify_offload_complete", None, [vp, u64]),
    ]:
        f = getattr(lib, fn)
        f.restype = res
        f.argtypes = args
    _OLIB = lib
    return lib


class OffloadLink:
    """One end of the link: OffloadLink.create(...) (server side) or
    OffloadLink.join(name) (client side)."""

    def __init__(self, handle, name, owner):
        self.lib = load_offload_lib()
        self.h = handle
        self.name = name
        self.owner = owner

    @classmethod
    def create(cls, name, depth=1 << 16, dcache_sz=64 << 20):
        lib = load_offload_lib()
        h = lib.fd_verify_offload_create(name.encode(), depth, dcache_sz)
        if not h:
            raise GpuError("fd_verify_offload_create(%s) failed" % name)
        return cls(h, name, True)

    @classmethod
    def join(cls, name):
        lib = load_offload_lib()
        h = lib.fd_verify_offload_join(name.encode())
        if not h:
            raise GpuError("fd_verify_offload_join(%s) failed" % name)
        return cls(h, name, False)

    def close(self):
        if self.h:
            self.lib.fd_verify_offload_leave(self.h)
            self.h = None
            if self.owner:
                self.lib.fd_verify_offload_unlink(self.name.encode())

    @property
    def depth(self):
        return int(self.lib.fd_verify_offload_depth(self.h))

    @property
    def dcache_sz(self):
        return int(self.lib.fd_verify_offload_dcache_sz(self.h))

    # client
    def publish(self, frag):
        """frag: bytes -> seq, or ERR_FULL / ERR_ARG."""
        buf = ctypes.create_string_buffer(bytes(frag), len(frag))
        return int(self.lib.fd_verify_offload_publish(self.h, buf, len(frag)))

    def result(self, seq):
        """-> (status, result, sig): status 1 ready, 0 not yet, ERR_SEQ."""
        r = ctypes.c_int8(0)
        s = ctypes.c_uint64(0)
        st = self.lib.fd_verify_offload_result(self.h, seq, ctypes.byref(r), ctypes.byref(s))
        return int(st), int(r.value), int(s.value)

    def publish_burst(self, arena, frags):
        """Publish frags (FRAG_DTYPE rows into arena) in order until one does
        not fit -> number published."""
        arena = np.ascontiguousarray(arena, np.uint8)
        frags = np.ascontiguousarray(frags)
        return int(self.lib.fd_verify_offload_publish_burst(self.h, arena.ctypes.data, frags.ctypes.data, len(frags)))

    def results(self, seq, res, sig):
        """Copy ready results of seqs [seq, seq + len(res)) -> count copied."""
        return int(self.lib.fd_verify_offload_results(self.h, seq, len(res), res.ctypes.data, sig.ctypes.data))

    def prod_seq(self):
        return int(self.lib.fd_verify_offload_prod_seq(self.h))

    def done_seq(self):
        return int(self.lib.fd_verify_offload_done_seq(self.h))

    def halt(self):
        self.lib.fd_verify_offload_halt(self.h)

    # server primitives
    def avail(self):
        first = ctypes.c_uint64(0)
        n = self.lib.fd_verify_offload_avail(self.h, ctypes.byref(first))
        return int(first.value), int(n)

    def frags(self, seq, n):
        p = self.lib.fd_verify_offload_frag_laddr(self.h, seq)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(n, 2))

    def results_view(self, seq, n):
        p = self.lib.fd_verify_offload_result_laddr(self.h, seq)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int8)), shape=(n,))

    def sigs_view(self, seq, n):
        p = self.lib.fd_verify_offload_sig_laddr(self.h, seq)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint64)), shape=(n,))

    def dcache_view(self):
        p = self.lib.fd_verify_offload_dcache(self.h)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(self.dcache_sz,))

    def take(self, n):
        self.lib.fd_verify_offload_take(self.h, n)

    def complete(self, done_seq):
        self.lib.fd_verify_offload_complete(self.h, done_seq)


class ServeThread:
    """fd_verify_offload_serve on a Python thread (ctypes drops the GIL for
    the call): the in-process form of the offload server, for tests."""

    def __init__(self, link, gpu, tcache, max_batch=65536, threads=4):
        lib = load_lib()
        lib.fd_verify_offload_serve.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        self.stats = (ctypes.c_uint64 * 7)()
        self.rc = None

        def run():
            self.rc = lib.fd_verify_offload_serve(link.h, gpu.ctx, tcache.tc, max_batch, threads, self.stats)
        self.t = threading.Thread(target=run, daemon=True)
        self.t.start()

    def join(self, timeout=None):
        self.t.join(timeout)
        if self.t.is_alive():
            raise GpuError("offload server did not stop")
        if self.rc:
            raise GpuError("fd_verify_offload_serve: %s (%d)" % (strerror(self.rc), self.rc))
        return list(self.stats)
