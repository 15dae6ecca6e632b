"""The gossip signatures as a descriptor source (SURVEY.md §8(f) next-4;
fd_gossip.c ping :477, pong :756, CRDS values :894, prune :1026).

Fixture tests/golden/gossip.bin (make_golden.py gen_gossip): the reference's
own gossip packets (src/flamenco/types/fixtures/gossip_*.bin: pull request,
pull responses with contact-info v1/v2, node-instance, snapshot-hash and
version values, a vote push), ping / pong / prune packets signed by the
reference signer with malformed variants, and pull responses / pushes over
all twelve CRDS variants whose values are signed over the reference
ENCODER's bytes (tests/crds_gen.py: option tags 2..255, padded varints,
varint-u16 fields -- encodings the encoder does not write back), each with
the triples the REFERENCE gossip code forms (its decoder, its encoder, its
self filter, fd_ed25519_verify; oracle/ref_gossip.c).  Bar: the walks form
byte-identical triples (fd_ed25519_gpu_gossip_walk for ping / pong / prune,
fd_ed25519_gpu_gossip_walk_crds for every kind, CRDS values included) and
the same statuses where the reference verifies nothing; a differential fuzz
against the compiled reference codec (oracle/_ref) on random and mutated
packets; the GPU codes equal the reference codes for every triple."""
import struct

import numpy as np
import pytest

import firedancer_amd as fa
from golden_io import read_gossip

ME, PKTS = read_gossip()


def _arena():
    """every packet in one arena (4-byte misaligned starts), aux region after them"""
    blob, spans = bytearray(), []
    for p in PKTS:
        blob += b"\xee" * (len(blob) % 4 == 0)            # odd alignment for half the packets
        spans.append((len(blob), len(p["pkt"])))
        blob += p["pkt"]
    aux_off = len(blob)
    aux_cap = sum(len(p["pkt"]) for p in PKTS)
    arena = np.zeros(aux_off + aux_cap + 16, np.uint8)
    arena[:aux_off] = np.frombuffer(bytes(blob), np.uint8)
    return arena, np.array(spans, fa.SPAN_DTYPE), aux_off, aux_cap


def _kind(p):
    return struct.unpack_from("<I", p["pkt"])[0] if len(p["pkt"]) >= 4 else None


def test_fixture_covers_the_callers():
    kinds = {}
    for p in PKTS:
        for t in p["triples"] or []:
            kinds.setdefault(t["kind"], []).append(t["code"])
    assert set(kinds) == {1, 2, 3, 4, 5}                  # pull resp, push, prune, ping, pong
    assert sum(1 for p in PKTS if 100 <= p["tag"] < 200) == 7   # the reference's 7 gossip packet fixtures
    signed = [p for p in PKTS if p["tag"] >= 200]          # every CRDS variant, signed over the reference encoding
    assert {struct.unpack_from("<I", p["pkt"], 44 + 64)[0] for p in signed} == set(range(12))
    assert all(p["triples"] and p["triples"][0]["code"] == 0 for p in signed)
    assert any(c != 0 for c in kinds[1] + kinds[2])       # a CRDS value the reference rejects
    assert any(p["triples"] is None for p in PKTS)        # packets that do not decode
    assert any(p["triples"] == [] and _kind(p) == 3 for p in PKTS)   # a prune for another node


def test_walk_matches_reference_triples():
    arena, spans, aux_off, aux_cap = _arena()
    desc, pd = fa.gossip_walk(arena, len(arena), aux_off, aux_cap, spans, ME)
    a = arena.tobytes()
    for j, p in enumerate(PKTS):
        k, tr = _kind(p), p["triples"]
        if k in (3, 4, 5) and tr:
            assert pd[j] >= 0, (p["tag"], pd[j])
            d = desc[pd[j]]
            t = tr[0]
            assert len(tr) == 1
            assert a[d["msg_off"]:d["msg_off"] + d["msg_sz"]] == t["msg"], p["tag"]
            assert a[d["sig_off"]:d["sig_off"] + 64] == t["sig"], p["tag"]
            assert a[d["pub_off"]:d["pub_off"] + 32] == t["key"], p["tag"]
            assert d["txn_idx"] == j
        elif tr is None:
            exp = fa.GOSSIP_CRDS if k in (1, 2) else fa.GOSSIP_CORRUPT
            assert pd[j] == exp, (p["tag"], pd[j])
        elif k == 0:
            assert tr == [] and pd[j] == fa.GOSSIP_UNSIGNED
        elif k == 3:
            assert tr == [] and pd[j] == fa.GOSSIP_NOT_MINE
        else:
            assert k in (1, 2) and pd[j] == fa.GOSSIP_CRDS, (p["tag"], pd[j])
    # no self filter: the prune for another node is walked too
    _, pd2 = fa.gossip_walk(arena, len(arena), aux_off, aux_cap, spans, None)
    assert all(pd2[j] >= 0 for j, p in enumerate(PKTS) if _kind(p) == 3 and p["triples"] == [])


def test_walk_codes_with_oracle(oracle):
    """our CPU restatement on the walked descriptors == the reference codes"""
    arena, spans, aux_off, aux_cap = _arena()
    desc, pd = fa.gossip_walk(arena, len(arena), aux_off, aux_cap, spans, ME)
    codes = np.zeros(max(len(desc), 1), np.int8)
    oracle.fdo_verify_descs(arena.ctypes.data, desc.ctypes.data, len(desc), codes.ctypes.data, 0)
    for j, p in enumerate(PKTS):
        if pd[j] >= 0:
            assert codes[pd[j]] == p["triples"][0]["code"], p["tag"]


def test_walk_refuses_bad_spans():
    arena, spans, aux_off, aux_cap = _arena()
    with pytest.raises(fa.GpuError):                      # aux overlapping a packet
        fa.gossip_walk(arena, len(arena), 0, 64, spans, ME)
    bad = spans.copy(); bad[3]["sz"] = len(arena)
    with pytest.raises(fa.GpuError):                      # a packet past the arena
        fa.gossip_walk(arena, len(arena), aux_off, aux_cap, bad, ME)
    with pytest.raises(fa.GpuError):                      # aux too small for the prunes
        fa.gossip_walk(arena, len(arena), aux_off, 10, spans, ME)


def _crds_batch():
    recs = [(t["msg"], t["sig"], t["key"]) for p in PKTS for t in p["triples"] or [] if t["kind"] in (1, 2)]
    exp = [t["code"] for p in PKTS for t in p["triples"] or [] if t["kind"] in (1, 2)]
    return recs, np.array(exp, np.int8)


@pytest.mark.gpu
def test_gossip_verify_gpu(gpu):
    arena, spans, aux_off, aux_cap = _arena()
    out = gpu.gossip_verify(arena, len(arena), aux_off, aux_cap, spans, ME)
    for j, p in enumerate(PKTS):
        k, tr = _kind(p), p["triples"]
        if k in (3, 4, 5) and tr:
            assert out[j] == tr[0]["code"], (p["tag"], out[j], tr[0]["code"])
        else:
            assert out[j] < -100, (p["tag"], out[j])


@pytest.mark.gpu
def test_crds_values_gpu(gpu):
    """CRDS values: the re-encoded bytes + signature + key as descriptors"""
    recs, exp = _crds_batch()
    arena, desc, sz = fa.pack_batch(recs)
    codes = gpu.verify_batch(arena, sz, desc)
    assert np.array_equal(codes, exp)


def _arena2():
    """_arena with aux sized for the CRDS re-encodings (2 x the packets' bytes)"""
    arena, spans, aux_off, aux_cap = _arena()
    big = np.zeros(aux_off + 2 * aux_cap + 16, np.uint8)
    big[:aux_off] = arena[:aux_off]
    return big, spans, aux_off, 2 * aux_cap


def _check_crds_walk(arena, spans, desc, pd, pc, pkts, triples_of):
    a = arena.tobytes()
    for j, p in enumerate(pkts):
        k, tr = _kind(p), triples_of(j)
        if tr is None:
            assert pd[j] == fa.GOSSIP_CORRUPT and pc[j] == 0, (j, pd[j])
        elif k == 0:
            assert tr == [] and pd[j] == fa.GOSSIP_UNSIGNED
        elif tr == []:
            assert pd[j] == (fa.GOSSIP_NOT_MINE if k == 3 else fa.GOSSIP_NO_VALUES), (j, pd[j])
        else:
            assert pd[j] >= 0 and pc[j] == len(tr), (j, pd[j], pc[j], len(tr))
            for i, t in enumerate(tr):
                d = desc[pd[j] + i]
                assert a[d["msg_off"]:d["msg_off"] + d["msg_sz"]] == t["msg"], (j, i)
                assert a[d["sig_off"]:d["sig_off"] + 64] == t["sig"], (j, i)
                assert a[d["pub_off"]:d["pub_off"] + 32] == t["key"], (j, i)
                assert d["txn_idx"] == j


def test_walk_crds_matches_reference_triples():
    """every packet, CRDS values included: the walk's triples are the
    reference's (decoder + fd_crds_data_encode + self filter), byte for byte"""
    arena, spans, aux_off, aux_cap = _arena2()
    desc, pd, pc = fa.gossip_walk_crds(arena, len(arena), aux_off, aux_cap, spans, ME)
    _check_crds_walk(arena, spans, desc, pd, pc, PKTS, lambda j: PKTS[j]["triples"])
    assert sum(len(p["triples"] or []) for p in PKTS) == len(desc)
    assert any(pd[j] >= 0 and _kind(p) in (1, 2) for j, p in enumerate(PKTS))


def test_walk_crds_codes_with_oracle(oracle):
    """our CPU restatement on the walked CRDS descriptors == the reference codes"""
    arena, spans, aux_off, aux_cap = _arena2()
    desc, pd, pc = fa.gossip_walk_crds(arena, len(arena), aux_off, aux_cap, spans, ME)
    codes = np.zeros(max(len(desc), 1), np.int8)
    oracle.fdo_verify_descs(arena.ctypes.data, desc.ctypes.data, len(desc), codes.ctypes.data, 0)
    for j, p in enumerate(PKTS):
        for i, t in enumerate(p["triples"] or []):
            assert codes[pd[j] + i] == t["code"], (p["tag"], i)


def test_walk_crds_aux_and_desc_bounds():
    arena, spans, aux_off, aux_cap = _arena2()
    with pytest.raises(fa.GpuError):                      # aux too small for the re-encodings
        fa.gossip_walk_crds(arena, len(arena), aux_off, 64, spans, ME)
    lib = fa.load_lib()
    desc = np.zeros(2, fa.DESC_DTYPE)
    pd = np.zeros(len(spans), np.int64)
    pc = np.zeros(len(spans), np.uint32)
    r = lib.fd_ed25519_gpu_gossip_walk_crds(arena.ctypes.data, len(arena), aux_off, aux_cap, spans.ctypes.data,
                                            len(spans), bytes(ME), desc.ctypes.data, 2, pd.ctypes.data, pc.ctypes.data)
    assert r < 0                                          # more descriptors than desc_cap


@pytest.mark.gpu
def test_gossip_verify_crds_gpu(gpu):
    """the walked CRDS values verified on the GPU: codes == the reference's"""
    arena, spans, aux_off, aux_cap = _arena2()
    code, pd, pc = gpu.gossip_verify_crds(arena, len(arena), aux_off, aux_cap, spans, ME)
    n = 0
    for j, p in enumerate(PKTS):
        for i, t in enumerate(p["triples"] or []):
            assert code[pd[j] + i] == t["code"], (p["tag"], i)
            n += 1
    assert n == len(code)


def _ref_lib():
    import ctypes
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                        "libfdref_avx512.so")
    if not os.path.exists(path):
        pytest.skip("oracle/_ref not built (needs /root/reference: make -C oracle ref)")
    lib = ctypes.CDLL(path)
    lib.fdref_gossip_triples.restype = ctypes.c_long
    lib.fdref_gossip_triples.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p,
                                         ctypes.c_ulong]
    return lib


def _ref_triples(lib, pkt, me):
    """the reference decoder + encoder + self filter on one packet (oracle/ref_gossip.c)"""
    import ctypes
    buf = ctypes.create_string_buffer(1 << 20)
    n = lib.fdref_gossip_triples(pkt, len(pkt), me, buf, len(buf))
    assert n != -2
    if n < 0:
        return None
    out, b, at = [], buf.raw, 0
    for _ in range(n):
        kind, sz = struct.unpack_from("<II", b, at); at += 8
        msg = b[at:at + sz]; at += sz
        sig = b[at:at + 64]; key = b[at + 64:at + 96]; at += 96 + 4
        out.append({"kind": kind, "msg": msg, "sig": sig, "key": key})
    return out


def _walk_one_by_one_batch(pkts, me):
    blob, spans = bytearray(), []
    for p in pkts:
        blob += b"\x00" * (len(blob) % 3)                 # assorted alignments
        spans.append((len(blob), len(p)))
        blob += p
    aux_off = len(blob)
    aux_cap = 2 * len(blob) + 64
    arena = np.zeros(aux_off + aux_cap + 16, np.uint8)
    arena[:aux_off] = np.frombuffer(bytes(blob), np.uint8)
    spans = np.array(spans, fa.SPAN_DTYPE)
    desc, pd, pc = fa.gossip_walk_crds(arena, len(arena), aux_off, aux_cap, spans, me)
    return arena, spans, desc, pd, pc


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_walk_crds_differential_vs_reference_codec(seed):
    """Random pull responses / pushes over all twelve CRDS variants (the
    decoder-accepted encodings the encoder does not write back: option tags
    2..255, padded varints, varint-u16 fields, v0 / legacy vote txns) and
    mutations of them: the walk's triples == the reference decoder + encoder
    + self filter (oracle/_ref, compiled from the reference's sources)."""
    import crds_gen
    lib = _ref_lib()
    rng = np.random.default_rng(1000 + seed)
    pkts = []
    for i in range(600):
        p = crds_gen.random_packet(rng, ME)
        pkts.append(p if i % 3 == 0 else crds_gen.mutate(rng, p))
    for p in PKTS:                                        # the reference's own fixtures, mutated
        if _kind(p) in (1, 2):
            pkts.append(crds_gen.mutate(rng, p["pkt"]))
    refs = [_ref_triples(lib, p, ME) for p in pkts]
    arena, spans, desc, pd, pc = _walk_one_by_one_batch(pkts, ME)
    objs = [{"pkt": p} for p in pkts]
    _check_crds_walk(arena, spans, desc, pd, pc, objs, lambda j: refs[j])
    ok = sum(1 for r in refs if r)
    assert ok > 150 and sum(1 for r in refs if r is None) > 100    # both sides of the decoder exercised


def test_walk_crds_every_variant_decodes():
    """each variant alone, unmutated: decodes, and the re-encoding differs
    from the received bytes exactly where the reference's codec is not an
    inverse (so the walk must not hand the received bytes over)"""
    import crds_gen
    lib = _ref_lib()
    rng = np.random.default_rng(77)
    changed = set()
    for disc in range(12):
        for _ in range(20):
            p = crds_gen.packet(rng, 2, ME, rng.bytes(32), [(disc, None)])
            tr = _ref_triples(lib, p, ME)
            assert tr is not None and len(tr) == 1, disc
            if tr[0]["msg"] != p[44 + 64:]:
                changed.add(disc)
            arena, spans, desc, pd, pc = _walk_one_by_one_batch([p], ME)
            _check_crds_walk(arena, spans, desc, pd, pc, [{"pkt": p}], lambda j: [tr[0]])
    assert {5, 6, 7, 11} <= changed                       # option tags, varints, varint-u16 fields
