"""ctypes mirror of the verify-stage part of include/fd_ed25519_gpu.h
(SURVEY.md §8(f) next-1 / next-2): the verify tile's per-frag logic,
src/app/fdctl/run/tiles/fd_verify.c:76-124 (after_frag) and fd_txn_verify,
src/app/fdctl/run/tiles/fd_verify.h:43-88, over batches of tango frags.

  TCache        fd_tcache semantics (src/tango/tcache/fd_tcache.h), host side
  frags_to_descs  frag layout -> signature descriptors (host only, no GPU)
  VerifyStage   Ed25519Gpu + TCache: verify_frags(arena, frags) -> per-frag
                FD_TXN_VERIFY_* results and the tile's opt_sig (the dedup tag)
"""
import numpy as np

from .ed25519 import DESC_DTYPE, Ed25519Gpu, GpuError, _ptr, load_lib, strerror

FD_TXN_VERIFY_SUCCESS = 0
FD_TXN_VERIFY_FAILED = -1
FD_TXN_VERIFY_DEDUP = -2
FD_TXN_VERIFY_BAD_FRAG = -64

VERIFY_TCACHE_DEPTH = 16    # src/app/fdctl/run/tiles/fd_verify.h:6
VERIFY_TCACHE_MAP_CNT = 64  # src/app/fdctl/run/tiles/fd_verify.h:7

# fd_ed25519_gpu_frag_t (8 bytes): frag i = arena[off, off+sz)
FRAG_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4")])


class TCache:
    """fd_tcache with the tile's parameters by default (depth 16, map_cnt 64)."""

    def __init__(self, depth=VERIFY_TCACHE_DEPTH, map_cnt=VERIFY_TCACHE_MAP_CNT):
        self.lib = load_lib()
        self.tc = self.lib.fd_ed25519_gpu_tcache_new(depth, map_cnt)
        if not self.tc:
            raise ValueError("bad tcache depth / map_cnt (%d, %d)" % (depth, map_cnt))

    def close(self):
        if self.tc:
            self.lib.fd_ed25519_gpu_tcache_delete(self.tc)
            self.tc = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def depth(self):
        return int(self.lib.fd_ed25519_gpu_tcache_depth(self.tc))

    @property
    def map_cnt(self):
        return int(self.lib.fd_ed25519_gpu_tcache_map_cnt(self.tc))

    def reset(self):
        self.lib.fd_ed25519_gpu_tcache_reset(self.tc)

    def query(self, tag):
        """FD_TCACHE_QUERY: True if tag is present."""
        return bool(self.lib.fd_ed25519_gpu_tcache_query(self.tc, int(tag)))

    def insert(self, tag):
        """FD_TCACHE_INSERT: returns the dup flag."""
        return bool(self.lib.fd_ed25519_gpu_tcache_insert(self.tc, int(tag)))


def frags_to_descs(arena, arena_sz, frags):
    """-> (desc DESC_DTYPE[n], frag_status int8[m], frag_tag uint64[m])."""
    lib = load_lib()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    frags = np.ascontiguousarray(frags, dtype=FRAG_DTYPE)
    m = len(frags)
    desc = np.zeros(max(16 * m, 1), DESC_DTYPE)
    st = np.zeros(max(m, 1), np.int8)
    tag = np.zeros(max(m, 1), np.uint64)
    n = lib.fd_ed25519_gpu_frags_to_descs(_ptr(arena), arena_sz, _ptr(frags), m, _ptr(desc), len(desc), _ptr(st),
                                          _ptr(tag))
    if n < 0:
        raise GpuError("fd_ed25519_gpu_frags_to_descs: %s (%d)" % (strerror(n), n))
    return desc[:n].copy(), st[:m].copy(), tag[:m].copy()


class VerifyStage:
    """One verify tile's worth of state: a GPU verify context and its tcache."""

    def __init__(self, gpu=None, tcache=None, **gpu_kw):
        self.gpu = gpu if gpu is not None else Ed25519Gpu(**gpu_kw)
        self.tcache = tcache if tcache is not None else TCache()

    def verify_frags(self, arena, arena_sz, frags):
        """-> (result int8[m] FD_TXN_VERIFY_*, sig uint64[m])."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        frags = np.ascontiguousarray(frags, dtype=FRAG_DTYPE)
        m = len(frags)
        res = np.zeros(max(m, 1), np.int8)
        sig = np.zeros(max(m, 1), np.uint64)
        r = self.gpu.lib.fd_ed25519_gpu_verify_frags(self.gpu.ctx, self.tcache.tc, _ptr(arena), arena_sz,
                                                     _ptr(frags), m, _ptr(res), _ptr(sig))
        if r:
            raise GpuError("fd_ed25519_gpu_verify_frags: %s (%d)" % (strerror(r), r))
        return res[:m].copy(), sig[:m].copy()

    def close(self):
        self.gpu.close()
        self.tcache.close()


class AsyncStage:
    """fd_ed25519_gpu_stage_*: up to STAGE_DEPTH batches outstanding (QUEUE_DEPTH on the
    GPU), completed in order by the stage's poller and replayer threads;
    frags parsed on the GPU by default (device_parse=False: on the host)."""

    def __init__(self, gpu, tcache, max_frags, threads=4, device_parse=True):
        import ctypes as C
        lib = load_lib()
        vp = C.c_void_p
        lib.fd_ed25519_gpu_stage_new.restype = vp
        lib.fd_ed25519_gpu_stage_new.argtypes = [vp, vp, C.c_uint64, C.c_int]
        lib.fd_ed25519_gpu_stage_submit.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp]
        lib.fd_ed25519_gpu_stage_poll.argtypes = [vp, C.c_int]
        lib.fd_ed25519_gpu_stage_pending.argtypes = [vp]
        lib.fd_ed25519_gpu_stage_delete.argtypes = [vp]
        lib.fd_ed25519_gpu_stage_set_device_parse.argtypes = [vp, C.c_int]
        lib.fd_ed25519_gpu_stage_warm.argtypes = [vp, vp, C.c_uint64]
        lib.fd_ed25519_gpu_stage_stats.argtypes = [vp, vp]
        lib.fd_ed25519_gpu_stage_stats_reset.argtypes = [vp]
        self.lib, self.gpu, self.tcache = lib, gpu, tcache
        self.st = lib.fd_ed25519_gpu_stage_new(gpu.ctx, tcache.tc, max_frags, threads)
        if not self.st:
            raise GpuError("fd_ed25519_gpu_stage_new failed")
        lib.fd_ed25519_gpu_stage_set_device_parse(self.st, 1 if device_parse else 0)
        self._keep = []

    def submit(self, arena, arena_sz, frags, result, sig):
        """Enqueue a batch (arrays must stay alive until its poll returns 0).
        Raises GpuError with ERR_BUSY when STAGE_DEPTH batches are outstanding
        (poll the oldest first), like Ed25519Gpu.submit: a dropped batch must
        never pass silently."""
        r = self.lib.fd_ed25519_gpu_stage_submit(self.st, _ptr(arena), arena_sz, _ptr(frags), len(frags),
                                                 _ptr(result), _ptr(sig))
        if r:
            raise GpuError("fd_ed25519_gpu_stage_submit: %s (%d)" % (strerror(r), r))
        self._keep.append((arena, frags, result, sig))
        return True

    def poll(self, block=True):
        r = self.lib.fd_ed25519_gpu_stage_poll(self.st, 1 if block else 0)
        if r == 1:
            return False
        # any other return retired the oldest batch (a failed batch too: the
        # stage goes on with the next one), so its buffers go with it
        if self._keep:
            self._keep.pop(0)
        if r:
            raise GpuError("fd_ed25519_gpu_stage_poll: %s (%d)" % (strerror(r), r))
        return True

    def pending(self):
        return int(self.lib.fd_ed25519_gpu_stage_pending(self.st))

    _STATS = ("submit_ns", "parse_ns", "register_ns", "launch_ns", "poll_ns",
              "gpu_poll_ns", "gpu_wait_ns", "replay_ns", "batches", "frags")

    def stats(self, reset=False):
        """fd_ed25519_gpu_stage_stats: where the stage's host time went (ns) --
        the caller's submit / poll, the poller's GPU polls and
        back-off waits and tcache replays."""
        import ctypes as C
        buf = (C.c_uint64 * len(self._STATS))()
        r = self.lib.fd_ed25519_gpu_stage_stats(self.st, buf)
        if r:
            raise GpuError("fd_ed25519_gpu_stage_stats: %s (%d)" % (strerror(r), r))
        if reset:
            self.lib.fd_ed25519_gpu_stage_stats_reset(self.st)
        return dict(zip(self._STATS, list(buf)))

    def warm(self, arena=None):
        """fd_ed25519_gpu_stage_warm: pay first-use costs (first DMA from a registered
        frag area, first launches) before live traffic."""
        r = self.lib.fd_ed25519_gpu_stage_warm(self.st, None if arena is None else _ptr(arena),
                                               0 if arena is None else arena.nbytes)
        if r:
            raise GpuError("fd_ed25519_gpu_stage_warm: %s (%d)" % (strerror(r), r))

    def close(self):
        if self.st:
            self.lib.fd_ed25519_gpu_stage_delete(self.st)
            self.st = None
