"""Batched Ed25519 precompile instructions:
fd_ed25519_gpu_precompile_verify against the REFERENCE
fd_ed25519_program_execute (src/flamenco/runtime/program/fd_ed25519_program.c,
compiled into oracle/_ref and run on a minimal execution context by
oracle/ref_program.c: fdref_ed25519_program_real).  The reference has no test
of its own for this program; the cases follow its branches: data_sz < 2,
truncated offsets records, out-of-range offsets and instruction indices (own
data 0xFFFF and other instructions), bad signatures before / after an offsets
error, zero signatures, empty messages.  On CPU: the line-by-line
restatement (fdref_ed25519_program) and our host walk
(fd_ed25519_gpu_precompile_walk + the reference verify per descriptor) both
equal the reference program."""
import ctypes
import os
import struct
import sys

import numpy as np
import pytest

import firedancer_amd as fa

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import synth  # noqa: E402

REF_SO = os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so")


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built")
    lib = ctypes.CDLL(REF_SO)
    for fn in (lib.fdref_ed25519_program, lib.fdref_ed25519_program_real):
        fn.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong]
    lib.fdref_verify_descs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                       ctypes.c_ulong, ctypes.c_ulong]
    return lib


def ref_program(ref, data, txn_instrs, real=True):
    """The reference program's result (real=True: fd_ed25519_program.c itself;
    False: the restatement in oracle/ref_harness.c)."""
    n = len(txn_instrs)
    bufs = [ctypes.create_string_buffer(bytes(d), max(len(d), 1)) for d in txn_instrs]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
    szs = (ctypes.c_ulong * max(n, 1))(*[len(d) for d in txn_instrs])
    fn = ref.fdref_ed25519_program_real if real else ref.fdref_ed25519_program
    r = fn(bytes(data), len(data), ptrs, szs, n)
    assert r != -1000
    return r


def pack_cases(cases):
    """-> (arena, PRECOMPILE_DTYPE instrs, SPAN_DTYPE spans) for a list of (data, txn)."""
    arena = bytearray()
    spans, instrs = [], []
    for data, txn in cases:
        lo = len(spans)
        for d in txn:
            spans.append((len(arena), len(d)))
            arena += d
        instrs.append((spans[lo][0], spans[lo][1], lo, len(txn)))
    arena = np.frombuffer(bytes(arena) + b"\0" * 16, np.uint8).copy()
    ins = np.array(instrs, dtype=[(n, "<u4") for n in ("data_off", "data_sz", "txn_instr_lo", "txn_instr_cnt")])
    sp = np.array(spans, dtype=[("off", "<u4"), ("sz", "<u4")])
    return arena, ins.view(fa.PRECOMPILE_DTYPE), sp.view(fa.SPAN_DTYPE)


@pytest.fixture(scope="module")
def cases():
    rng = np.random.default_rng(31)
    keys = synth.keypairs([rng.bytes(32) for _ in range(16)], threads=4)
    return [make_case(rng, keys) for _ in range(600)]


def make_case(rng, keys):
    """One transaction: 1-3 other instructions with random data, a precompile
    instruction with 0-6 signature records whose sig / pubkey / message live
    in its own data (index 0xFFFF) or in another instruction; then maybe one
    corruption.  Returns (precompile data, txn instruction datas)."""
    n_other = int(rng.integers(1, 4))
    others = [bytearray(rng.bytes(int(rng.integers(0, 300)))) for _ in range(n_other)]
    n_sig = int(rng.choice([0, 1, 1, 2, 3, 6]))
    recs, payload = [], bytearray()
    hdr_sz = 2 + 14 * n_sig
    for i in range(n_sig):
        seed, pub = keys[int(rng.integers(0, len(keys)))]
        msg = rng.bytes(int(rng.choice([0, 32, 100, 200])))
        sig, = synth.sign_many([(seed, pub, msg)], threads=1)
        fields = []
        for blob in (sig, pub, msg):
            if rng.random() < 0.3:                         # put it into another instruction
                k = int(rng.integers(0, n_other))
                fields.append((len(others[k]), k + 1))     # txn index: 0 is the precompile itself
                others[k] += blob
            else:
                fields.append((hdr_sz + len(payload), 0xFFFF))
                payload += blob
        recs.append((fields, len(msg)))
    data = bytearray([n_sig, 0])
    for (s_, p_, m_), msz in recs:
        data += struct.pack("<7H", s_[0], s_[1], p_[0], p_[1], m_[0], msz, m_[1])
    data += payload
    kind = rng.random()
    if kind < 0.12 and n_sig:                               # flip a signature / message / key byte
        j = int(rng.integers(hdr_sz, len(data))) if len(data) > hdr_sz else None
        if j is not None:
            data[j] ^= 1 << int(rng.integers(0, 8))
    elif kind < 0.20 and n_sig:                             # offsets past the data
        i = int(rng.integers(0, n_sig))
        struct.pack_into("<H", data, 2 + 14 * i + 2 * int(rng.choice([0, 2, 4])), 0xFFF0)
    elif kind < 0.26 and n_sig:                             # instruction index out of range
        i = int(rng.integers(0, n_sig))
        struct.pack_into("<H", data, 2 + 14 * i + 2 * int(rng.choice([1, 3, 6])), n_other + 1 + int(rng.integers(0, 5)))
    elif kind < 0.32 and n_sig:                             # truncated records
        data = data[:2 + 14 * int(rng.integers(0, n_sig)) + int(rng.integers(0, 14))]
    elif kind < 0.36:                                       # data_sz < 2
        data = data[:int(rng.integers(0, 2))]
    elif kind < 0.40 and n_sig:                             # claims more records than present
        data[0] = n_sig + int(rng.integers(1, 5))
    elif kind < 0.46 and n_sig:                             # huge message size
        struct.pack_into("<H", data, 2 + 14 * int(rng.integers(0, n_sig)) + 10, 60000)
    return bytes(data), [bytes(data)] + [bytes(o) for o in others]


def test_restatement_equals_reference_program(ref, cases):
    """The restatement used in r01 and the reference source agree on every case."""
    for data, txn in cases:
        assert ref_program(ref, data, txn, real=False) == ref_program(ref, data, txn, real=True)


def test_host_walk_vs_reference_program(ref, cases):
    """fd_ed25519_gpu_precompile_walk (host, no GPU) + the reference
    fd_ed25519_verify on its descriptors + the first-failure fold ==
    the reference program, instruction by instruction."""
    exp = [ref_program(ref, d, t) for d, t in cases]
    arena, ins, sp = pack_cases(cases)
    n = len(ins)
    lib = fa.load_lib()
    vp = ctypes.c_void_p
    lib.fd_ed25519_gpu_precompile_walk.restype = ctypes.c_int64
    lib.fd_ed25519_gpu_precompile_walk.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint64, vp, ctypes.c_uint64,
                                                   vp, ctypes.c_uint64, vp, vp]
    desc = np.zeros(255 * n, fa.DESC_DTYPE)
    first = np.zeros(n + 1, np.uint64)
    tail = np.zeros(n, np.int32)
    nd = lib.fd_ed25519_gpu_precompile_walk(arena.ctypes.data, len(arena) - 16, ins.ctypes.data, n, sp.ctypes.data,
                                            len(sp), desc.ctypes.data, len(desc), first.ctypes.data, tail.ctypes.data)
    assert nd >= 0
    codes = np.zeros(max(nd, 1), np.int8)
    if nd:
        ref.fdref_verify_descs(arena.ctypes.data, desc.ctypes.data, nd, codes.ctypes.data, 4, 1)
    got = []
    for j in range(n):
        r = int(tail[j])
        if np.any(codes[first[j]:first[j + 1]] != 0):
            r = -102
        got.append(r)
    bad = [(i, got[i], exp[i]) for i in range(n) if got[i] != exp[i]]
    assert not bad, bad[:10]
    # a descriptor array too small is an argument error, never an overrun
    assert lib.fd_ed25519_gpu_precompile_walk(arena.ctypes.data, len(arena) - 16, ins.ctypes.data, n,
                                              sp.ctypes.data, len(sp), desc.ctypes.data, max(nd - 1, 0),
                                              first.ctypes.data, tail.ctypes.data) in ((-103,) if nd else (0,))


@pytest.mark.gpu
def test_precompile_batch_vs_reference(gpu, ref, cases):
    exp = [ref_program(ref, d, t) for d, t in cases]
    arena, ins, sp = pack_cases(cases)
    out = gpu.precompile_verify(arena, len(arena) - 16, ins, sp)
    bad = [(i, int(out[i]), exp[i]) for i in range(len(cases)) if int(out[i]) != exp[i]]
    assert not bad, bad[:10]
    hist = {k: exp.count(k) for k in set(exp)}
    assert all(hist.get(k, 0) >= 20 for k in (0, -100, -101, -102)), hist
