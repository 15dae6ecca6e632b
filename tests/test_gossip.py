"""The gossip signatures as a descriptor source (SURVEY.md §8(f) next-4;
fd_gossip.c ping :477, pong :756, CRDS values :894, prune :1026).

Fixture tests/golden/gossip.bin (make_golden.py gen_gossip): the reference's
own gossip packets (src/flamenco/types/fixtures/gossip_*.bin: pull request,
pull responses with contact-info v1/v2, node-instance, snapshot-hash and
version values, a vote push) and ping / pong / prune packets signed by the
reference signer with malformed variants, each with the triples the
REFERENCE gossip code forms (its decoder, its encoder, fd_ed25519_verify;
oracle/ref_gossip.c).  Bar: the host walk forms byte-identical triples for
the kinds it walks (ping / pong / prune) and the same statuses where the
reference verifies nothing; the GPU codes equal the reference codes for every
triple, CRDS ones included (re-encoded bytes handed over as descriptors)."""
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
    assert sum(1 for p in PKTS if p["tag"] >= 100) == 7   # the reference's 7 gossip packet fixtures
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
