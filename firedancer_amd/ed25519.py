"""ctypes mirror of include/fd_ed25519_gpu.h (see package docstring)."""
import collections
import ctypes
import os

import numpy as np

# FD_ED25519_GPU_QUEUE_DEPTH (include/fd_ed25519_gpu.h): batches in flight for submit / poll
QUEUE_DEPTH = 5
# FD_ED25519_GPU_STAGE_DEPTH: batches outstanding in the verify stage
STAGE_DEPTH = 8

FD_ED25519_SUCCESS = 0
FD_ED25519_ERR_SIG = -1
FD_ED25519_ERR_PUBKEY = -2
FD_ED25519_ERR_MSG = -3
CODE_BAD_DESC = -128

GPU_OK = 0
GPU_PENDING = 1

CODES_AVX512 = 0
CODES_REF = 1

# fd_sha512_gpu_msg_t (8 bytes)
SHA_MSG_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4")])

# fd_ed25519_gpu_precompile_t (16 bytes): data span + the txn's instruction spans [lo, lo+cnt)
PRECOMPILE_DTYPE = np.dtype([("data_off", "<u4"), ("data_sz", "<u4"), ("txn_instr_lo", "<u4"),
                             ("txn_instr_cnt", "<u4")])
SPAN_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4")])

# fd_ed25519_desc_t (16 bytes, include/fd_ed25519_gpu.h)
DESC_DTYPE = np.dtype([("sig_off", "<u4"), ("pub_off", "<u4"), ("msg_off", "<u4"),
                       ("msg_sz", "<u2"), ("txn_idx", "<u2")])
assert DESC_DTYPE.itemsize == 16

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class GpuError(RuntimeError):
    pass


def lib_path():
    """The in-tree library; FD_ED25519_GPU_LIB may name a diagnostic build
    of the same source (tools/Makefile: phase-stamp variant)."""
    return os.environ.get("FD_ED25519_GPU_LIB") or os.path.join(_HERE, "libfd_ed25519_gpu.so")


def load_lib():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    # share torch's HIP runtime if torch is used in this process (same SONAME, one runtime);
    # FD_ED25519_GPU_NO_TORCH=1: the HIP runtime the library links (/opt/rocm), torch not loaded
    if os.environ.get("FD_ED25519_GPU_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    if not os.path.exists(path):
        raise GpuError("libfd_ed25519_gpu.so not built (run `make -C firedancer_amd` or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    lib.fd_ed25519_gpu_new.restype = vp
    lib.fd_ed25519_gpu_new.argtypes = [u64, u64]
    lib.fd_ed25519_gpu_new_devs.restype = vp
    lib.fd_ed25519_gpu_new_devs.argtypes = [vp, i32, u64]
    lib.fd_ed25519_gpu_delete.argtypes = [vp]
    lib.fd_ed25519_gpu_device_cnt.argtypes = [vp]
    lib.fd_ed25519_gpu_set_codes.argtypes = [vp, i32]
    lib.fd_ed25519_verify_batch_gpu.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.fd_ed25519_gpu_submit.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.fd_ed25519_gpu_poll.argtypes = [vp]
    lib.fd_ed25519_gpu_poll_block.argtypes = [vp]
    lib.fd_ed25519_gpu_pending.argtypes = [vp]
    lib.fd_ed25519_gpu_pipe_status.argtypes = [vp, i32]
    lib.fd_ed25519_gpu_host_stats.argtypes = [vp, vp, i32]
    lib.fd_ed25519_gpu_test_ctab_stats.argtypes = [i32, vp, vp]
    lib.fd_ed25519_gpu_launch_stats.argtypes = [vp, vp, vp]
    lib.fd_ed25519_gpu_build_id.restype = ctypes.c_char_p
    lib.fd_ed25519_gpu_build_id.argtypes = []
    lib.fd_ed25519_gpu_runtime.restype = ctypes.c_char_p
    lib.fd_ed25519_gpu_runtime.argtypes = []
    lib.fd_ed25519_gpu_host_is_registered.argtypes = [vp, u64]
    lib.fd_ed25519_verify_batch_gpu_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_pipe_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_pipe_flush_dev.argtypes = [vp, i32, vp]
    lib.fd_ed25519_gpu_verify.argtypes = [vp, ctypes.c_char_p, u64, ctypes.c_char_p, ctypes.c_char_p,
                                          ctypes.POINTER(ctypes.c_int)]
    lib.fd_ed25519_gpu_verify_batch_single_msg.argtypes = [vp, ctypes.c_char_p, u64, ctypes.c_char_p,
                                                           ctypes.c_char_p, u64, ctypes.POINTER(ctypes.c_int)]
    lib.fd_ed25519_gpu_txn_reduce.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_txn_reduce.argtypes = [vp, vp, u64, vp, u64]
    lib.fd_ed25519_gpu_test_lattice.argtypes = [vp, vp, u64, vp]
    lib.fd_ed25519_gpu_test_field.argtypes = [vp, ctypes.c_int, vp, vp, u64, vp]
    lib.fd_sha512_batch_gpu.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.fd_sha512_batch_gpu_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_sha256_batch_gpu.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.fd_sha256_batch_gpu_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_tcache_new.restype = vp
    lib.fd_ed25519_gpu_tcache_new.argtypes = [u64, u64]
    lib.fd_ed25519_gpu_tcache_delete.argtypes = [vp]
    lib.fd_ed25519_gpu_tcache_reset.argtypes = [vp]
    lib.fd_ed25519_gpu_tcache_depth.restype = u64
    lib.fd_ed25519_gpu_tcache_depth.argtypes = [vp]
    lib.fd_ed25519_gpu_tcache_map_cnt.restype = u64
    lib.fd_ed25519_gpu_tcache_map_cnt.argtypes = [vp]
    lib.fd_ed25519_gpu_tcache_query.argtypes = [vp, u64]
    lib.fd_ed25519_gpu_tcache_insert.argtypes = [vp, u64]
    lib.fd_ed25519_gpu_frags_to_descs.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_frags_to_descs.argtypes = [vp, u64, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_verify_frags.argtypes = [vp, vp, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_precompile_verify.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp]
    lib.fd_ed25519_gpu_gossip_walk.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_gossip_walk.argtypes = [vp, u64, u64, u64, vp, u64, vp, vp, u64, vp]
    lib.fd_ed25519_gpu_gossip_verify.argtypes = [vp, vp, u64, u64, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_gossip_walk_crds.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_gossip_walk_crds.argtypes = [vp, u64, u64, u64, vp, u64, vp, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_gossip_verify_crds.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_gossip_verify_crds.argtypes = [vp, vp, u64, u64, u64, vp, u64, vp, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_shred_walk.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_shred_walk.argtypes = [vp, u64, u64, u64, vp, vp, u64, vp, u64, vp]
    lib.fd_ed25519_gpu_shred_verify.argtypes = [vp, vp, u64, u64, u64, vp, vp, u64, vp]
    lib.fd_ed25519_gpu_sha256.argtypes = [vp, u64, vp]
    lib.fd_ed25519_gpu_host_register.argtypes = [vp, vp, u64]
    lib.fd_ed25519_gpu_host_unregister.argtypes = [vp, vp]
    lib.fd_ed25519_gpu_keycache_reserve.argtypes = [vp, u64]
    lib.fd_ed25519_gpu_keycache_add.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_keycache_add.argtypes = [vp, ctypes.c_char_p, u64]
    lib.fd_ed25519_gpu_keycache_cnt.restype = u64
    lib.fd_ed25519_gpu_keycache_cnt.argtypes = [vp]
    lib.fd_ed25519_gpu_keycache_clear.argtypes = [vp]
    lib.fd_ed25519_gpu_strerror.restype = ctypes.c_char_p
    lib.fd_ed25519_gpu_strerror.argtypes = [i32]
    _LIB = lib
    return lib


def build_id():
    """{"code": sha-256 prefix of the embedded code object, "git": describe of the built tree}"""
    s = load_lib().fd_ed25519_gpu_build_id().decode()
    return dict(kv.split("=", 1) for kv in s.split())


def runtime_info():
    """{"hip": path of the libamdhip64 the library's HIP calls resolve to, "version": hipRuntimeGetVersion}:
    torch's bundled runtime when torch was imported first, /opt/rocm's otherwise (FD_ED25519_GPU_NO_TORCH=1)."""
    s = load_lib().fd_ed25519_gpu_runtime().decode()
    return dict(kv.split("=", 1) for kv in s.split())


def host_is_registered(buf):
    """fd_ed25519_gpu_host_is_registered: is the array page-locked (registered / hipHostMalloc'd)?"""
    return load_lib().fd_ed25519_gpu_host_is_registered(_ptr(buf), buf.nbytes) == 1


def ctab_stats(dev=0):
    """(live comb tables on HIP device dev, slots using it, tables built by this process)."""
    refs, builds = ctypes.c_uint64(0), ctypes.c_uint64(0)
    live = load_lib().fd_ed25519_gpu_test_ctab_stats(dev, ctypes.byref(refs), ctypes.byref(builds))
    return live, refs.value, builds.value


def strerror(code):
    return load_lib().fd_ed25519_gpu_strerror(int(code)).decode()


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def pack_batch(records):
    """records: iterable of (msg, sig, pub[, txn_idx]) bytes -> (arena uint8 array, desc array).

    Layout: sig | pub | msg per record, packed back to back with no alignment
    (the kernel reads unaligned fields), like payload bytes in a dcache chunk."""
    recs = list(records)
    n = len(recs)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    total = sum(96 + len(r[0]) for r in recs)
    arena = np.zeros(total + 16, dtype=np.uint8)
    off = 0
    for i, r in enumerate(recs):
        msg, sig, pub = r[0], r[1], r[2]
        txn = r[3] if len(r) > 3 else i & 0xffff
        arena[off:off + 64] = np.frombuffer(sig, np.uint8)
        arena[off + 64:off + 96] = np.frombuffer(pub, np.uint8)
        if msg:
            arena[off + 96:off + 96 + len(msg)] = np.frombuffer(msg, np.uint8)
        desc[i] = (off, off + 64, off + 96, len(msg), txn)
        off += 96 + len(msg)
    return arena, desc, total


GOSSIP_CORRUPT, GOSSIP_UNSIGNED, GOSSIP_NOT_MINE, GOSSIP_CRDS, GOSSIP_NO_VALUES = -110, -111, -112, -113, -114


def _gossip_desc_cap(pkts):
    """every signed value holds a 64-byte signature: a packet has at most sz / 64 + 1"""
    return int(np.sum(pkts["sz"] // 64)) + len(pkts) + 1


def gossip_walk(arena, arena_sz, aux_off, aux_cap, pkts, self_pubkey=None):
    """fd_ed25519_gpu_gossip_walk (host, no GPU): -> (desc, pkt_desc)."""
    lib = load_lib()
    pkts = np.ascontiguousarray(pkts, dtype=SPAN_DTYPE)
    n = len(pkts)
    desc = np.zeros(max(n, 1), DESC_DTYPE)
    pd = np.zeros(max(n, 1), np.int64)
    me = None if self_pubkey is None else ctypes.c_char_p(bytes(self_pubkey))
    nd = lib.fd_ed25519_gpu_gossip_walk(_ptr(arena), arena_sz, aux_off, aux_cap, _ptr(pkts), n, me,
                                        _ptr(desc), n, _ptr(pd))
    if nd < 0:
        raise GpuError("fd_ed25519_gpu_gossip_walk: %s (%d)" % (strerror(int(nd)), nd))
    return desc[:nd], pd[:n]


def gossip_walk_crds(arena, arena_sz, aux_off, aux_cap, pkts, self_pubkey=None):
    """fd_ed25519_gpu_gossip_walk_crds (host, no GPU): CRDS values walked too
    -> (desc, pkt_desc, pkt_cnt)."""
    lib = load_lib()
    pkts = np.ascontiguousarray(pkts, dtype=SPAN_DTYPE)
    n = len(pkts)
    cap = _gossip_desc_cap(pkts)
    desc = np.zeros(cap, DESC_DTYPE)
    pd = np.zeros(max(n, 1), np.int64)
    pc = np.zeros(max(n, 1), np.uint32)
    me = None if self_pubkey is None else ctypes.c_char_p(bytes(self_pubkey))
    nd = lib.fd_ed25519_gpu_gossip_walk_crds(_ptr(arena), arena_sz, aux_off, aux_cap, _ptr(pkts), n, me,
                                             _ptr(desc), cap, _ptr(pd), _ptr(pc))
    if nd < 0:
        raise GpuError("fd_ed25519_gpu_gossip_walk_crds: %s (%d)" % (strerror(int(nd)), nd))
    return desc[:nd], pd[:n], pc[:n]


SHRED_PARSE, SHRED_ZERO_SIG, SHRED_COUNTS, SHRED_INDEX, SHRED_DEPTH, SHRED_PROOF = -120, -121, -122, -123, -124, -125


def shred_walk(arena, arena_sz, aux_off, aux_cap, shreds, key_off):
    """fd_ed25519_gpu_shred_walk (host, no GPU): -> (desc, shred_desc)."""
    lib = load_lib()
    shreds = np.ascontiguousarray(shreds, dtype=SPAN_DTYPE)
    key_off = np.ascontiguousarray(key_off, dtype=np.uint32)
    n = len(shreds)
    desc = np.zeros(max(n, 1), DESC_DTYPE)
    sd = np.zeros(max(n, 1), np.int64)
    nd = lib.fd_ed25519_gpu_shred_walk(_ptr(arena), arena_sz, aux_off, aux_cap, _ptr(shreds), _ptr(key_off), n,
                                       _ptr(desc), n, _ptr(sd))
    if nd < 0:
        raise GpuError("fd_ed25519_gpu_shred_walk: %s (%d)" % (strerror(int(nd)), nd))
    return desc[:nd], sd[:n]


def sha256(msg):
    lib = load_lib()
    out = ctypes.create_string_buffer(32)
    lib.fd_ed25519_gpu_sha256(ctypes.c_char_p(bytes(msg)), len(msg), out)
    return out.raw


def txn_reduce(codes, desc):
    """Per-txn codes with the fd_ed25519_verify_batch_single_msg precedence (host function, no GPU)."""
    lib = load_lib()
    codes = np.ascontiguousarray(codes, dtype=np.int8)
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    out = np.zeros(max(len(desc), 1), dtype=np.int8)
    t = lib.fd_ed25519_gpu_txn_reduce(_ptr(codes), _ptr(desc), len(desc), _ptr(out), len(out))
    return out[:t].copy()


class Ed25519Gpu:
    """One verify context (fd_ed25519_gpu_t) over the GPUs in device_mask, or
    over an explicit list of shard slots (devices=[0, 0] = two slots on GPU 0:
    fd_ed25519_gpu_new_devs)."""

    def __init__(self, device_mask=0, max_batch=1 << 18, codes=CODES_AVX512, devices=None):
        self.lib = load_lib()
        self._keep = collections.deque()     # (arena, out) of the batches in flight
        if devices is not None:
            ids = (ctypes.c_int * len(devices))(*devices)
            self.ctx = self.lib.fd_ed25519_gpu_new_devs(ids, len(devices), max_batch)
        else:
            self.ctx = self.lib.fd_ed25519_gpu_new(device_mask, max_batch)
        if not self.ctx:
            raise GpuError("fd_ed25519_gpu_new failed (no HIP device?)")
        self.set_codes(codes)

    def close(self):
        if self.ctx:
            self.lib.fd_ed25519_gpu_delete(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_cnt(self):
        return self.lib.fd_ed25519_gpu_device_cnt(self.ctx)

    def set_codes(self, flavour):
        r = self.lib.fd_ed25519_gpu_set_codes(self.ctx, flavour)
        if r:
            raise GpuError(strerror(r))

    def verify_batch(self, arena, arena_sz, desc):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        out = np.zeros(len(desc), dtype=np.int8)
        r = self.lib.fd_ed25519_verify_batch_gpu(self.ctx, _ptr(arena), arena_sz, _ptr(desc), len(desc), _ptr(out))
        if r:
            raise GpuError("fd_ed25519_verify_batch_gpu: %s (%d)" % (strerror(r), r))
        return out

    def submit(self, arena, arena_sz, desc, out):
        """fd_ed25519_gpu_submit: up to QUEUE_DEPTH batches in flight (the
        pipelined kernel's three phases + two queued launches); raises GpuError
        with ERR_BUSY on one more."""
        r = self.lib.fd_ed25519_gpu_submit(self.ctx, _ptr(arena), arena_sz, _ptr(desc), len(desc), _ptr(out))
        if r:
            raise GpuError("fd_ed25519_gpu_submit: %s (%d)" % (strerror(r), r))
        self._keep.append((arena, out))

    def poll(self, block=False):
        """Completes the oldest submitted batch: True when its out is final."""
        f = self.lib.fd_ed25519_gpu_poll_block if block else self.lib.fd_ed25519_gpu_poll
        r = f(self.ctx)
        if r < 0:
            if self._keep:
                self._keep.popleft()
            raise GpuError("fd_ed25519_gpu_poll: %s (%d)" % (strerror(r), r))
        if r == GPU_OK and self._keep:
            self._keep.popleft()
        return r == GPU_OK

    _HOST_STATS = ("scan_ns", "stage_ns", "h2d_ns", "launch_ns", "out_ns", "h2d_bytes", "late_recs")

    def host_stats(self, reset=False):
        """fd_ed25519_gpu_host_stats: host time of the submit paths (ns) and the
        bytes copied to HBM."""
        import ctypes as C
        buf = (C.c_uint64 * len(self._HOST_STATS))()
        r = self.lib.fd_ed25519_gpu_host_stats(self.ctx, buf, 1 if reset else 0)
        if r:
            raise GpuError("fd_ed25519_gpu_host_stats: %s (%d)" % (strerror(r), r))
        return dict(zip(self._HOST_STATS, list(buf)))

    def launch_stats(self):
        """(pipelined launches, one-shot launches) of this context so far."""
        p, o = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self.lib.fd_ed25519_gpu_launch_stats(self.ctx, ctypes.byref(p), ctypes.byref(o))
        return p.value, o.value

    def pending(self):
        return self.lib.fd_ed25519_gpu_pending(self.ctx)

    def pipe_status(self, dev_idx=0):
        return self.lib.fd_ed25519_gpu_pipe_status(self.ctx, dev_idx)

    def host_register(self, buf):
        """Page-lock a host array (e.g. a frag area) for every device of the context
        (fd_ed25519_gpu_host_register): its per-batch copies to HBM become direct DMA."""
        r = self.lib.fd_ed25519_gpu_host_register(self.ctx, _ptr(buf), buf.nbytes)
        if r:
            raise GpuError("fd_ed25519_gpu_host_register: %s (%d)" % (strerror(r), r))

    def host_unregister(self, buf):
        r = self.lib.fd_ed25519_gpu_host_unregister(self.ctx, _ptr(buf))
        if r:
            raise GpuError("fd_ed25519_gpu_host_unregister: %s (%d)" % (strerror(r), r))

    def verify_batch_dev(self, d_arena, arena_sz, d_desc, desc_cnt, d_out, stream=0, dev_idx=0):
        """Device pointers (ints), enqueue only."""
        r = self.lib.fd_ed25519_verify_batch_gpu_dev(self.ctx, dev_idx, d_arena, arena_sz, d_desc, desc_cnt,
                                                     d_out, stream)
        if r:
            raise GpuError("fd_ed25519_verify_batch_gpu_dev: %s (%d)" % (strerror(r), r))

    def pipe_dev(self, d_arena, arena_sz, d_desc, desc_cnt, d_out, stream=0, dev_idx=0):
        """Pipelined device-pointer entry (fd_ed25519_gpu_pipe_dev): enqueues this
        batch's first phase beside the previous batch's second phase; the previous
        batch's codes land in ITS d_out when this launch completes."""
        r = self.lib.fd_ed25519_gpu_pipe_dev(self.ctx, dev_idx, d_arena, arena_sz, d_desc, desc_cnt, d_out, stream)
        if r:
            raise GpuError("fd_ed25519_gpu_pipe_dev: %s (%d)" % (strerror(r), r))

    def pipe_flush_dev(self, stream=0, dev_idx=0):
        r = self.lib.fd_ed25519_gpu_pipe_flush_dev(self.ctx, dev_idx, stream)
        if r:
            raise GpuError("fd_ed25519_gpu_pipe_flush_dev: %s (%d)" % (strerror(r), r))

    def verify(self, msg, sig, pub):
        """Mirror of fd_ed25519_verify: returns the FD_ED25519_* code."""
        out = ctypes.c_int(0)
        r = self.lib.fd_ed25519_gpu_verify(self.ctx, msg, len(msg), sig, pub, ctypes.byref(out))
        if r:
            raise GpuError(strerror(r))
        return out.value

    def verify_batch_single_msg(self, msg, sigs, pubs, n):
        """Mirror of fd_ed25519_verify_batch_single_msg (sigs/pubs concatenated bytes)."""
        out = ctypes.c_int(0)
        r = self.lib.fd_ed25519_gpu_verify_batch_single_msg(self.ctx, msg, len(msg), sigs or b"\0" * 64,
                                                            pubs or b"\0" * 32, n, ctypes.byref(out))
        if r:
            raise GpuError(strerror(r))
        return out.value

    def test_lattice(self, k_words):
        """Test hook: device lattice reduction of k (uint32 array [n, 8]) ->
        uint32 array [n, 18] = |u| (8 words), v (8 words), sign of u, iterations."""
        k_words = np.ascontiguousarray(k_words, dtype=np.uint32)
        out = np.zeros((len(k_words), 18), dtype=np.uint32)
        r = self.lib.fd_ed25519_gpu_test_lattice(self.ctx, _ptr(k_words), len(k_words), _ptr(out))
        if r:
            raise GpuError("fd_ed25519_gpu_test_lattice: %s (%d)" % (strerror(r), r))
        return out

    def test_field(self, op, a, b):
        """Test hook: one device field / group operation (fd_ed25519_gpu_test_field)
        on uint32 arrays a, b of shape [n, 40] -> uint32 array [n, 40]."""
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        assert a.shape == b.shape and a.ndim == 2 and a.shape[1] == 40, (a.shape, b.shape)
        out = np.zeros_like(a)
        r = self.lib.fd_ed25519_gpu_test_field(self.ctx, op, _ptr(a), _ptr(b), len(a), _ptr(out))
        if r:
            raise GpuError("fd_ed25519_gpu_test_field: %s (%d)" % (strerror(r), r))
        return out

    def keycache_reserve(self, capacity):
        """Size the hot-key cache (512 KB of HBM per key per device); clears it."""
        r = self.lib.fd_ed25519_gpu_keycache_reserve(self.ctx, capacity)
        if r:
            raise GpuError("fd_ed25519_gpu_keycache_reserve: %s (%d)" % (strerror(r), r))

    def keycache_add(self, pubkeys):
        """Cache public keys (iterable of 32-byte strings) -> number newly added."""
        blob = b"".join(bytes(k) for k in pubkeys)
        r = self.lib.fd_ed25519_gpu_keycache_add(self.ctx, blob, len(blob) // 32)
        if r < 0:
            raise GpuError("fd_ed25519_gpu_keycache_add: %s (%d)" % (strerror(r), r))
        return int(r)

    def keycache_cnt(self):
        return int(self.lib.fd_ed25519_gpu_keycache_cnt(self.ctx))

    def keycache_clear(self):
        r = self.lib.fd_ed25519_gpu_keycache_clear(self.ctx)
        if r:
            raise GpuError("fd_ed25519_gpu_keycache_clear: %s (%d)" % (strerror(r), r))

    def precompile_verify(self, arena, arena_sz, instrs, spans):
        """Batched fd_ed25519_program_execute: instrs PRECOMPILE_DTYPE, spans
        SPAN_DTYPE (the transactions' instruction data) -> int32 results
        (0 / -100 / -101 / -102, FD_EXECUTOR_SIGN_ERR_*)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        instrs = np.ascontiguousarray(instrs, dtype=PRECOMPILE_DTYPE)
        spans = np.ascontiguousarray(spans, dtype=SPAN_DTYPE)
        out = np.zeros(max(len(instrs), 1), np.int32)
        r = self.lib.fd_ed25519_gpu_precompile_verify(self.ctx, _ptr(arena), arena_sz, _ptr(instrs), len(instrs),
                                                      _ptr(spans), len(spans), _ptr(out))
        if r:
            raise GpuError("fd_ed25519_gpu_precompile_verify: %s (%d)" % (strerror(r), r))
        return out[:len(instrs)]

    def gossip_verify(self, arena, arena_sz, aux_off, aux_cap, pkts, self_pubkey=None):
        """Gossip packets (SPAN_DTYPE spans of arena, a writable uint8 array
        with room for the rebuilt prune messages at [aux_off, aux_off +
        aux_cap)) -> int32 per packet: the verify code of its signature or
        a GOSSIP_* walk status (include/fd_ed25519_gpu.h)."""
        pkts = np.ascontiguousarray(pkts, dtype=SPAN_DTYPE)
        out = np.zeros(max(len(pkts), 1), np.int32)
        me = None if self_pubkey is None else ctypes.c_char_p(bytes(self_pubkey))
        r = self.lib.fd_ed25519_gpu_gossip_verify(self.ctx, _ptr(arena), arena_sz, aux_off, aux_cap, _ptr(pkts),
                                                  len(pkts), me, _ptr(out))
        if r:
            raise GpuError("fd_ed25519_gpu_gossip_verify: %s (%d)" % (strerror(r), r))
        return out[:len(pkts)]

    def gossip_verify_crds(self, arena, arena_sz, aux_off, aux_cap, pkts, self_pubkey=None):
        """gossip_verify with the CRDS values of pull responses / pushes too
        -> (int8 code per descriptor, pkt_desc, pkt_cnt): packet j's values
        are codes[pkt_desc[j]:pkt_desc[j] + pkt_cnt[j]] in value order (the
        others this node's own), or pkt_desc[j] is a GOSSIP_* status."""
        pkts = np.ascontiguousarray(pkts, dtype=SPAN_DTYPE)
        n = len(pkts)
        cap = _gossip_desc_cap(pkts)
        code = np.zeros(cap, np.int8)
        pd = np.zeros(max(n, 1), np.int64)
        pc = np.zeros(max(n, 1), np.uint32)
        me = None if self_pubkey is None else ctypes.c_char_p(bytes(self_pubkey))
        r = self.lib.fd_ed25519_gpu_gossip_verify_crds(self.ctx, _ptr(arena), arena_sz, aux_off, aux_cap, _ptr(pkts),
                                                       n, me, _ptr(code), cap, _ptr(pd), _ptr(pc))
        if r < 0:
            raise GpuError("fd_ed25519_gpu_gossip_verify_crds: %s (%d)" % (strerror(int(r)), r))
        return code[:r], pd[:n], pc[:n]

    def shred_verify(self, arena, arena_sz, aux_off, aux_cap, shreds, key_off):
        """Shreds (SPAN_DTYPE spans of arena) with their leaders' keys at
        arena[key_off[j]:+32] -> int32 per shred: the verify code of the
        FEC resolver's root check or a SHRED_* status (include/fd_ed25519_gpu.h)."""
        shreds = np.ascontiguousarray(shreds, dtype=SPAN_DTYPE)
        key_off = np.ascontiguousarray(key_off, dtype=np.uint32)
        out = np.zeros(max(len(shreds), 1), np.int32)
        r = self.lib.fd_ed25519_gpu_shred_verify(self.ctx, _ptr(arena), arena_sz, aux_off, aux_cap, _ptr(shreds),
                                                 _ptr(key_off), len(shreds), _ptr(out))
        if r:
            raise GpuError("fd_ed25519_gpu_shred_verify: %s (%d)" % (strerror(r), r))
        return out[:len(shreds)]

    def sha256_batch(self, msgs):
        """Batched SHA-256 of a list of byte strings (mirror of fd_sha256_batch_add per message)."""
        return self._sha_batch(msgs, self.lib.fd_sha256_batch_gpu, 32, "fd_sha256_batch_gpu")

    def sha512_batch(self, msgs):
        """Batched SHA-512 of a list of byte strings (mirror of fd_sha512_batch_add per message)."""
        return self._sha_batch(msgs, self.lib.fd_sha512_batch_gpu, 64, "fd_sha512_batch_gpu")

    def _sha_batch(self, msgs, fn, dlen, name):
        msgs = list(msgs)
        total = sum(len(m) for m in msgs)
        arena = np.zeros(total + 16, np.uint8)
        desc = np.zeros(len(msgs), SHA_MSG_DTYPE)
        off = 0
        for i, m in enumerate(msgs):
            if m:
                arena[off:off + len(m)] = np.frombuffer(m, np.uint8)
            desc[i] = (off, len(m))
            off += len(m)
        out = np.zeros(dlen * max(len(msgs), 1), np.uint8)
        r = fn(self.ctx, _ptr(arena), total, _ptr(desc), len(msgs), _ptr(out))
        if r:
            raise GpuError("%s: %s (%d)" % (name, strerror(r), r))
        return [out[dlen * i:dlen * i + dlen].tobytes() for i in range(len(msgs))]

    def sha512_batch_dev(self, d_arena, arena_sz, d_msg, msg_cnt, d_out, stream=0, dev_idx=0):
        r = self.lib.fd_sha512_batch_gpu_dev(self.ctx, dev_idx, d_arena, arena_sz, d_msg, msg_cnt, d_out, stream)
        if r:
            raise GpuError("fd_sha512_batch_gpu_dev: %s (%d)" % (strerror(r), r))
