"""Shred leader signatures as a descriptor source (SURVEY.md §8(f) next-4;
the FEC resolver's check of the shred that opens a set,
src/disco/shred/fd_fec_resolver.c:309-405).

Fixture tests/golden/shreds.bin (make_golden.py gen_shreds): the 480 shreds
of the reference's demo capture (src/disco/shred/fixtures/demo-shreds.pcap,
leader key demo-shreds.key) and 48 corrupted variants (protected / proof /
signature bytes, S >= l, zero signature, truncation, proof-length and type
nibbles, indices below the set or past the proof, data / code counts 0 or
68, bad data sizes, extra bytes, another leader), each with the result of
the REFERENCE check (oracle/ref_shred.c: the reference fd_shred_parse,
bmtree, SHA-256 and fd_ed25519_verify).  Bar: the host walk gives the same
status where the reference rejects before verifying and the same 32-byte
root where it verifies; the GPU codes equal the reference codes."""
import numpy as np
import pytest

import firedancer_amd as fa
from golden_io import read_shreds

RECS = read_shreds()
STATUS = {-101: fa.SHRED_PARSE, -102: fa.SHRED_ZERO_SIG, -103: fa.SHRED_COUNTS, -104: fa.SHRED_INDEX,
          -105: fa.SHRED_DEPTH, -106: fa.SHRED_PROOF}


def _arena():
    blob, spans, keys = bytearray(), [], []
    for r in RECS:
        keys.append(len(blob)); blob += r["leader"]
        blob += b"\x5a" * (len(blob) % 3)                  # unaligned shred starts
        spans.append((len(blob), len(r["shred"]))); blob += r["shred"]
    aux_off = len(blob)
    arena = np.zeros(aux_off + 32 * len(RECS), np.uint8)
    arena[:aux_off] = np.frombuffer(bytes(blob), np.uint8)
    return arena, np.array(spans, fa.SPAN_DTYPE), np.array(keys, np.uint32), aux_off, 32 * len(RECS)


def test_fixture_covers_the_checks():
    res = [r["result"] for r in RECS]
    assert sum(1 for r in RECS if r["tag"] < 1000 and r["result"] == 0) == 480
    for s in (-101, -102, -103, -104, -105):
        assert s in res, s
    assert {0, -1, -3} <= set(res)                         # verified: success, ERR_SIG, ERR_MSG


def test_walk_matches_reference():
    arena, spans, keys, aux_off, aux_cap = _arena()
    desc, sd = fa.shred_walk(arena, len(arena), aux_off, aux_cap, spans, keys)
    a = arena.tobytes()
    for j, r in enumerate(RECS):
        if r["result"] <= -100:
            assert sd[j] == STATUS[r["result"]], (r["tag"], sd[j], r["result"])
            continue
        assert sd[j] >= 0, (r["tag"], sd[j])
        d = desc[sd[j]]
        assert d["msg_sz"] == 32 and a[d["msg_off"]:d["msg_off"] + 32] == r["root"], r["tag"]
        assert a[d["sig_off"]:d["sig_off"] + 64] == r["shred"][:64]
        assert a[d["pub_off"]:d["pub_off"] + 32] == r["leader"]


def test_walk_codes_with_oracle(oracle):
    arena, spans, keys, aux_off, aux_cap = _arena()
    desc, sd = fa.shred_walk(arena, len(arena), aux_off, aux_cap, spans, keys)
    codes = np.zeros(max(len(desc), 1), np.int8)
    oracle.fdo_verify_descs(arena.ctypes.data, desc.ctypes.data, len(desc), codes.ctypes.data, 0)
    for j, r in enumerate(RECS):
        if sd[j] >= 0:
            assert codes[sd[j]] == r["result"], r["tag"]


def test_walk_refuses_bad_spans():
    arena, spans, keys, aux_off, aux_cap = _arena()
    with pytest.raises(fa.GpuError):                      # aux over a shred
        fa.shred_walk(arena, len(arena), 40, 64, spans, keys)
    with pytest.raises(fa.GpuError):                      # aux too small for the roots
        fa.shred_walk(arena, len(arena), aux_off, 64, spans, keys)
    bad = keys.copy(); bad[0] = len(arena) - 8
    with pytest.raises(fa.GpuError):                      # a key past the arena
        fa.shred_walk(arena, len(arena), aux_off, aux_cap, spans, bad)


@pytest.mark.gpu
def test_shred_verify_gpu(gpu):
    arena, spans, keys, aux_off, aux_cap = _arena()
    out = gpu.shred_verify(arena, len(arena), aux_off, aux_cap, spans, keys)
    exp = np.array([STATUS.get(r["result"], r["result"]) for r in RECS], np.int32)
    assert np.array_equal(out, exp), [(RECS[j]["tag"], out[j], exp[j]) for j in np.nonzero(out != exp)[0][:10]]


@pytest.mark.gpu
def test_shred_roots_on_gpu_equal_reference_roots(gpu):
    """The default shred_verify hashes the Merkle roots on the GPU
    (fd_shred_root_kernel) and copies them into aux: the same 32 bytes the
    reference bmtree gives; the host-hash path (FD_ED25519_GPU_SHRED_HOST_HASH=1)
    gives the same codes and roots."""
    import os
    arena, spans, keys, aux_off, aux_cap = _arena()
    desc, sd = fa.shred_walk(arena.copy(), len(arena), aux_off, aux_cap, spans, keys)   # descriptor order
    a1 = arena.copy()
    out = gpu.shred_verify(a1, len(a1), aux_off, aux_cap, spans, keys)
    b = a1.tobytes()
    nver = 0
    for j, r in enumerate(RECS):
        if r["result"] > -100:
            d = desc[sd[j]]
            assert b[d["msg_off"]:d["msg_off"] + 32] == r["root"], r["tag"]
            nver += 1
    assert nver >= 480
    a2 = arena.copy()
    os.environ["FD_ED25519_GPU_SHRED_HOST_HASH"] = "1"
    try:
        out2 = gpu.shred_verify(a2, len(a2), aux_off, aux_cap, spans, keys)
    finally:
        del os.environ["FD_ED25519_GPU_SHRED_HOST_HASH"]
    assert np.array_equal(out, out2)
    assert np.array_equal(a1, a2)


@pytest.mark.gpu
def test_shred_roots_many(gpu, oracle):
    """The capture's shreds tiled 64 times (30K shreds, different arena
    offsets): every root equals the host walk's, every code the fixture's."""
    reps = 64
    blob, spans, keys, want = bytearray(), [], [], []
    for t in range(reps):
        for r in RECS:
            keys.append(len(blob)); blob += r["leader"]
            blob += b"\x33" * ((t + len(blob)) % 5)
            spans.append((len(blob), len(r["shred"]))); blob += r["shred"]
            want.append(STATUS.get(r["result"], r["result"]))
    aux_off = len(blob)
    n = len(spans)
    arena = np.zeros(aux_off + 32 * n, np.uint8)
    arena[:aux_off] = np.frombuffer(bytes(blob), np.uint8)
    spans = np.array(spans, fa.SPAN_DTYPE); keys = np.array(keys, np.uint32)
    host = arena.copy()
    fa.shred_walk(host, len(host), aux_off, 32 * n, spans, keys)
    out = gpu.shred_verify(arena, len(arena), aux_off, 32 * n, spans, keys)
    assert np.array_equal(out, np.array(want, np.int32))
    assert np.array_equal(arena, host)
