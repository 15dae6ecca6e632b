"""Verify stage: tcache, frag -> descriptor
extraction and the whole per-frag verify over batches of tango frags.

Oracles:
  * the reference verify-tile test's transactions and assertions
    (src/app/fdctl/run/tiles/test_verify.c:4-109 data, :144-264 FD_TESTs),
    committed as tests/golden/verify_txns.json (make_verify_fixtures.py);
  * the reference tile restated over the REFERENCE tcache and batch verify
    (oracle/_ref fdref_verify_frags_seq / fdref_tcache_seq, ref_harness.c);
  * the reference fd_txn_parse for the synthetic transactions' fd_txn_t.
CPU tests need no GPU; the @gpu ones go through fd_ed25519_gpu_verify_frags.
"""
import ctypes
import json
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
S, F, D, BAD = fa.FD_TXN_VERIFY_SUCCESS, fa.FD_TXN_VERIFY_FAILED, fa.FD_TXN_VERIFY_DEDUP, fa.FD_TXN_VERIFY_BAD_FRAG


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference in the dev container)")
    lib = ctypes.CDLL(REF_SO)
    vp, ul = ctypes.c_void_p, ctypes.c_ulong
    lib.fdref_verify_frags_seq.argtypes = [vp, vp, ul, ul, ul, vp, vp]
    lib.fdref_tcache_seq.argtypes = [ul, ul, vp, ul, vp, vp, vp, vp]
    lib.fdref_txn_parse.restype = ul
    lib.fdref_txn_parse.argtypes = [ctypes.c_char_p, ul, ctypes.c_char_p]
    lib.fdref_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.fdref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ul, ctypes.c_char_p, ctypes.c_char_p]
    return lib


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def ref_seq(ref, arena, frags, depth=16, map_cnt=64):
    fr = np.ascontiguousarray(np.stack([frags["off"], frags["sz"]], 1).astype(np.uint32))
    res = np.zeros(max(len(frags), 1), np.int8)
    tag = np.zeros(max(len(frags), 1), np.uint64)
    assert ref.fdref_verify_frags_seq(_vp(arena), _vp(fr), len(frags), depth, map_cnt, _vp(res), _vp(tag)) == 0
    return res[:len(frags)], tag[:len(frags)]


def ref_seq_stream(ref, arena, batches, depth=16, map_cnt=64):
    """The reference tile over batches fed in arrival order through one tcache
    (their concatenation).  Frags lying past the arena (the tests' BAD_FRAG
    runs: off = len(arena) + 64) would make the reference read outside it; the
    tile rejects them before any tcache step (fd_verify.c:94-115), so they are
    BAD_FRAG with tag 0 and the reference runs over the rest."""
    allf = np.concatenate(batches)
    inside = (allf["off"].astype(np.int64) + allf["sz"]) <= len(arena)
    res = np.full(len(allf), BAD, np.int8)
    tag = np.zeros(len(allf), np.uint64)
    r, t = ref_seq(ref, arena, allf[inside], depth, map_cnt)
    res[inside], tag[inside] = r, t
    out, k = [], 0
    for b in batches:
        out.append((res[k:k + len(b)], tag[k:k + len(b)]))
        k += len(b)
    return out


def assert_vs_ref(got_res, got_tag, exp, what):
    for k, ((gr, gt), (er, et)) in enumerate(zip(zip(got_res, got_tag), exp)):
        bad = np.nonzero((gr != er) | (gt != et))[0]
        assert len(bad) == 0, (what, k, [(int(j), int(gr[j]), int(er[j])) for j in bad[:10]])


def fixture_txns():
    d = json.load(open(os.path.join(REPO, "tests", "golden", "verify_txns.json")))["txns"]
    return {k: (bytes.fromhex(v["payload"]), bytes.fromhex(v["txn_t"])) for k, v in d.items()}


# ---- synthetic workload generator (tools/synth.py) pinned -----------------

def test_synth_signer_rfc8032_vector():
    """RFC 8032 7.1 TEST 1 (empty message)."""
    seed = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    (_, pub), = synth.keypairs([seed])
    assert pub.hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    sig, = synth.sign_many([(seed, pub, b"")])
    assert sig.hex() == ("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e06522490155"
                         "5fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")


def test_synth_signer_matches_reference(ref):
    rng = np.random.default_rng(7)
    seeds = [rng.bytes(32) for _ in range(64)]
    kps = synth.keypairs(seeds, threads=4)
    items = [(s, p, rng.bytes(int(rng.integers(0, 300)))) for s, p in kps]
    sigs = synth.sign_many(items, threads=4)
    for (s, p, m), sig in zip(items, sigs):
        pub = ctypes.create_string_buffer(32)
        ref.fdref_public_from_private(pub, s)
        assert pub.raw == p
        rs = ctypes.create_string_buffer(64)
        ref.fdref_sign(rs, m, len(m), p, s)
        assert rs.raw == sig


@pytest.mark.parametrize("version", [synth.FD_TXN_VLEGACY, synth.FD_TXN_V0])
def test_synth_txn_t_matches_reference_parser(ref, version):
    rng = np.random.default_rng(11)
    txns = synth.build_txns(rng, 10, list(range(1, 11)), threads=4, version=version, data_sz=16)
    for payload, txn_t in txns:
        buf = ctypes.create_string_buffer(852)
        sz = ref.fdref_txn_parse(payload, len(payload), buf)
        assert sz == len(txn_t)
        assert buf.raw[:sz] == txn_t


# ---- tcache ------------------------------------------------------------------

@pytest.mark.parametrize("depth,map_cnt", [(16, 64), (5, 8), (1, 4), (16, 0), (100, 0), (30, 32)])
def test_tcache_matches_reference(ref, depth, map_cnt):
    """Random query / insert sequences over a small tag pool whose low bits
    collide (long probe runs, wrap-around, backward-shift deletions, tag 0):
    every found / dup flag equals the reference tcache's."""
    rng = np.random.default_rng(depth * 1000 + map_cnt)
    pool = [int(x) for x in rng.integers(0, 1 << 62, size=3 * depth + 8, dtype=np.int64)]
    pool = [(t & ~0x7) | (i & 0x3) for i, t in enumerate(pool)] + [0, 8, 16, 24]
    n = 4000
    kinds = rng.integers(0, 4, size=n) != 0        # 3/4 inserts
    tags = [pool[int(i)] for i in rng.integers(0, len(pool), size=n)]
    ops = np.zeros((n, 2), np.uint64)
    ops[:, 0] = kinds
    ops[:, 1] = np.array(tags, np.uint64)
    out = np.zeros(n, np.int32)
    mapo = np.zeros(4096, np.uint64); ring = np.zeros(depth, np.uint64); oldest = np.zeros(1, np.uint64)
    tmap = ref.fdref_tcache_seq(depth, map_cnt, _vp(ops), n, _vp(out), _vp(mapo), _vp(ring), _vp(oldest))
    assert tmap > 0
    tc = fa.TCache(depth, map_cnt)
    assert tc.map_cnt == tmap and tc.depth == depth
    mine = [int(tc.insert(t)) if k else int(tc.query(t)) for k, t in zip(kinds, tags)]
    assert mine == [int(x) for x in out]
    # final membership of every tag ever seen equals the reference map's
    ref_set = set(int(x) for x in mapo[:tmap] if x)
    for t in set(pool):
        assert tc.query(t) == (t in ref_set or t == 0), t


@pytest.mark.parametrize("depth,map_cnt", [(16, 64), (5, 8), (1, 4), (16, 0), (30, 32), (32, 64), (100, 0)])
def test_tcache_steps_ring_form_vs_reference(ref, depth, map_cnt):
    """The stage's tcache steps in the register-ring form (depth <= 32: the
    ring in AVX2 registers, the map rebuilt after each batch) against the
    map form and the REFERENCE tcache: per-frag results, opt_sig, and the
    final map slot for slot after every batch (colliding tags, tag 0, all
    result kinds, batches in sequence)."""
    import ctypes as C
    lib = fa.load_lib()
    vp = C.c_void_p
    lib.fd_ed25519_gpu_test_tcache_steps.argtypes = [vp, vp, vp, vp, C.c_uint64, C.c_int, vp]
    rng = np.random.default_rng(depth * 7 + map_cnt)
    pool = [int(x) for x in rng.integers(1, 1 << 62, size=3 * depth + 8, dtype=np.int64)]
    pool = [(t & ~0x7) | (i & 0x3) for i, t in enumerate(pool)] + [0, 8, 16, 24]
    codes = np.array([0, 0, 0, 0, -4, -1, -2, BAD], np.int8)        # SUCCESS x4, ERR_MSG/SIG/PUBKEY, BAD_FRAG
    tcs = [fa.TCache(depth, map_cnt), fa.TCache(depth, map_cnt)]
    mc = tcs[0].map_cnt
    ops = []
    for batch in range(4):
        n = int(rng.integers(1, 600))
        tags = np.array([pool[int(i)] for i in rng.integers(0, len(pool), size=n)], np.uint64)
        res0 = codes[rng.integers(0, len(codes), size=n)]
        outs = []
        for ring, tc in zip((1, 0), tcs):
            res = res0.copy(); sig = np.zeros(n, np.uint64); mp = np.zeros(mc, np.uint64)
            lib.fd_ed25519_gpu_test_tcache_steps(tc.tc, _vp(res), _vp(tags), _vp(sig), n, ring, _vp(mp))
            outs.append((res, sig, mp))
        assert all(np.array_equal(a, b) for a, b in zip(outs[0], outs[1]))
        res, sig, mp = outs[0]
        assert np.array_equal(sig, np.where(res == S, tags, 0).astype(np.uint64))
        # the same steps as reference tcache ops over the whole history: a
        # query per frag with a result, an insert after each that succeeds
        start = len(ops)
        for j in range(n):
            if res0[j] == BAD:
                continue
            ops.append((0, int(tags[j])))
            if res[j] == S:
                ops.append((1, int(tags[j])))
        o = np.array(ops, np.uint64).reshape(-1, 2)
        out = np.zeros(len(o), np.int32)
        mapo = np.zeros(4096, np.uint64); ringo = np.zeros(depth, np.uint64); oldest = np.zeros(1, np.uint64)
        assert ref.fdref_tcache_seq(depth, map_cnt, _vp(o), len(o), _vp(out), _vp(mapo), _vp(ringo), _vp(oldest)) == mc
        assert np.array_equal(mapo[:mc], mp), batch
        k = start
        for j in range(n):
            if res0[j] == BAD:
                assert res[j] == BAD
                continue
            found = int(out[k]); k += 1
            if found:
                assert res[j] == D
            elif res0[j] == 0:
                assert res[j] == S and int(out[k]) == 0
                k += 1
            else:
                assert res[j] == F


def test_tcache_params():
    with pytest.raises(ValueError):
        fa.TCache(0, 64)
    with pytest.raises(ValueError):
        fa.TCache(16, 48)      # not a power of two
    with pytest.raises(ValueError):
        fa.TCache(16, 16)      # < depth + 2
    assert fa.TCache(16, 0).map_cnt == 64    # fd_tcache_map_cnt_default: 2^(msb(17)+2)
    tc = fa.TCache(2, 4)
    assert tc.query(0) and not tc.insert(7) and tc.insert(7)
    assert not tc.insert(9) and not tc.insert(11)          # evicts 7
    assert not tc.query(7) and tc.query(9) and tc.query(11)
    tc.reset()
    assert not tc.query(9)


# ---- frag -> descriptors (host only) ------------------------------------

def _mk_frags(txns):
    return synth.pack_frags(txns)


def test_frags_to_descs_fixture_txns():
    fx = fixture_txns()
    names = ["valid_txn_1sig", "valid_txn_2sigs", "invalid_txn_2sigs"]
    arena, frags = _mk_frags([fx[k] for k in names])
    desc, st, tag = fa.frags_to_descs(arena, len(arena), frags)
    assert list(st) == [0, 0, 0]
    assert len(desc) == 1 + 2 + 2
    k = 0
    for i, name in enumerate(names):
        payload, txn_t = fx[name]
        n, soff, moff = txn_t[1], struct.unpack_from("<H", txn_t, 2)[0], struct.unpack_from("<H", txn_t, 4)[0]
        aoff = struct.unpack_from("<H", txn_t, 10)[0]
        base = int(frags["off"][i])
        assert int(tag[i]) == struct.unpack_from("<Q", payload, soff)[0]
        for j in range(n):
            d = desc[k]
            assert (int(d["sig_off"]), int(d["pub_off"]), int(d["msg_off"]), int(d["msg_sz"]), int(d["txn_idx"])) == \
                (base + soff + 64 * j, base + aoff + 32 * j, base + moff, len(payload) - moff, i)
            k += 1


def _corrupt_frags(arena, frags, kind, i):
    """Edit frag i in place into one of the tile's sanity-check failures."""
    off, sz = int(frags["off"][i]), int(frags["sz"][i])
    psz = struct.unpack_from("<H", arena, off + sz - 2)[0]
    t = off + psz + (psz & 1)
    if kind == "short":
        frags["sz"][i] = 1
    elif kind == "mtu":
        struct.pack_into("<H", arena, off + sz - 2, 2087)
    elif kind == "rbh":
        struct.pack_into("<H", arena, t + 12, psz)
    elif kind == "nosig":
        arena[t + 1] = 0
    elif kind == "manysig":
        arena[t + 1] = 17
    elif kind == "outside":
        frags["off"][i] = len(arena) - 4
        frags["sz"][i] = 8
    elif kind == "overclaim":
        # 16 signatures claimed by a frag too small to hold them (96 B each:
        # impossible for fd_txn_parse output) -> BAD_FRAG in both parses
        assert sz < 16 * 96
        arena[t + 1] = 16
    elif kind == "claim_at_bound":
        arena[t + 1] = sz // 96          # exactly what sz allows: parsed, verified (and failing)
    elif kind == "claim_past_bound":
        arena[t + 1] = sz // 96 + 1      # one more than sz allows: BAD_FRAG


BAD_KINDS = ["short", "mtu", "rbh", "nosig", "manysig", "outside", "overclaim", None]


def _fields_outside_stream():
    """Frags whose fd_txn_t points a field past the frag's own bytes (ADVICE
    r04: the device parse sees only the page runs the batch's frags occupy,
    gaps over 16 pages dropped): frag 1's signatures ~58 KB past it, inside
    a 20-page hole before frag 3 (so the device span's bytes there belong to
    another run); frag 2's signer keys past its end; frag 4's payload_sz
    past the frag.  Valid frags 0, 3 and 5 around them.  Expected: BAD_FRAG
    for 1, 2 and 4 in both parses."""
    fx = fixture_txns()
    txns = [fx["valid_txn_1sig"], fx["valid_txn_2sigs"], fx["valid_txn_1sig"]]
    a0, f0 = _mk_frags(txns)
    a1, f1 = _mk_frags([fx["valid_txn_2sigs"], fx["valid_txn_1sig"], fx["valid_txn_1sig"]])
    hole = 20 * 4096
    arena = np.zeros(len(a0) + hole + len(a1), np.uint8)
    arena[:len(a0)] = a0
    arena[len(a0) + hole:] = a1
    frags = np.zeros(6, f0.dtype)
    frags[:3] = f0
    frags["off"][3:] = f1["off"] + len(a0) + hole
    frags["sz"][3:] = f1["sz"]
    def txn_at(i):
        off, sz = int(frags["off"][i]), int(frags["sz"][i])
        psz = struct.unpack_from("<H", arena, off + sz - 2)[0]
        return off, sz, off + psz + (psz & 1)
    off, sz, t = txn_at(1)
    struct.pack_into("<H", arena, t + 2, 58000)                  # signature_off ~14 pages past frag 1
    arena[off + 58000:off + 58000 + 8] = 0x5a                    # (host bytes there: a nonzero tag)
    off, sz, t = txn_at(2)
    struct.pack_into("<H", arena, t + 10, sz - 16)               # acct_addr_off: the keys run past the frag
    off, sz, t = txn_at(4)
    struct.pack_into("<H", arena, off + sz - 2, sz + 8)          # payload_sz past the frag
    return arena, frags


def test_frags_fields_outside_frag_bad():
    """Host parse: every field it reads must lie inside the frag."""
    arena, frags = _fields_outside_stream()
    desc, st, tag = fa.frags_to_descs(arena, len(arena), frags)
    assert list(st) == [0, BAD, BAD, 0, BAD, 0], list(st)


def test_frags_to_descs_bad_frags():
    fx = fixture_txns()
    arena, frags = _mk_frags([fx["valid_txn_1sig"]] * len(BAD_KINDS))
    for i, k in enumerate(BAD_KINDS):
        _corrupt_frags(arena, frags, k, i)
    desc, st, tag = fa.frags_to_descs(arena, len(arena), frags)
    assert list(st) == [BAD, BAD, BAD, F, F, BAD, BAD, 0]
    assert len(desc) == 1 and int(desc[0]["txn_idx"]) == 7
    assert int(tag[3]) == int(tag[7]) != 0


def test_frags_reference_sanity_checks_agree(ref):
    """Our per-frag BAD / FAILED classification equals the restated tile's
    (reference tcache + reference verify) on the corrupted frags."""
    fx = fixture_txns()
    kinds = ["short", "mtu", "rbh", "nosig", "manysig", None]
    arena, frags = _mk_frags([fx["valid_txn_1sig"]] * len(kinds))
    for i, k in enumerate(kinds):
        _corrupt_frags(arena, frags, k, i)
    res, _ = ref_seq(ref, arena, frags)
    _, st, _ = fa.frags_to_descs(arena, len(arena), frags)
    assert list(res[:5]) == list(st[:5]) == [BAD, BAD, BAD, F, F]
    assert res[5] == S


# ---- the whole stage on the GPU -------------------------------------------

TILE_SCENARIOS = [
    # test_verify.c:144-186 test_verify_success
    ([["valid_txn_2sigs"] * 3 + ["valid_txn_1sig"] * 3], [[S, D, D, S, D, D]]),
    # :190-216 test_verify_invalid_sigs_success
    ([["invalid_txn_2sigs"] * 2], [[F, F]]),
    # :219-264 test_verify_invalid_dedup_success (tcache reset between the halves)
    ([["invalid_txn_same_1sig", "valid_txn_1sig"], ["valid_txn_1sig", "invalid_txn_same_1sig"]], [[F, S], [S, D]]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", range(len(TILE_SCENARIOS)))
@pytest.mark.parametrize("one_by_one", [False, True])
def test_verify_frags_reference_tile_tests(gpu, scenario, one_by_one):
    fx = fixture_txns()
    tc = fa.TCache()
    stage = fa.VerifyStage(gpu=gpu, tcache=tc)
    halves, expect = TILE_SCENARIOS[scenario]
    for names, exp in zip(halves, expect):
        tc.reset()
        arena, frags = _mk_frags([fx[k] for k in names])
        if one_by_one:
            got = []
            for i in range(len(frags)):
                r, _ = stage.verify_frags(arena, len(arena), frags[i:i + 1])
                got.append(int(r[0]))
        else:
            r, sig = stage.verify_frags(arena, len(arena), frags)
            got = [int(x) for x in r]
            for i, name in enumerate(names):
                pl = fx[name][0]
                assert int(sig[i]) == (struct.unpack_from("<Q", pl, 1)[0] if got[i] == S else 0)
        assert got == exp, (names, got, exp)


def _random_frag_stream(rng, n_unique, n_total):
    """n_unique synthetic txns (1..8 signers; a fifth with a corrupted
    signature or message, some 'frontrun' copies reusing a valid txn's first
    signature), then a stream of n_total frags drawn with repeats at short
    and long distances (so duplicates hit, miss after eviction, and
    invalid-first / valid-first orders both occur), plus sanity failures."""
    cnts = [int(c) for c in rng.choice([1, 1, 1, 2, 2, 3, 4, 8], size=n_unique)]
    txns = synth.build_txns(rng, n_unique, cnts, threads=16)
    txns = [(bytearray(p), t) for p, t in txns]
    extra = []
    for i in range(n_unique):
        r = rng.random()
        p, t = txns[i]
        if r < 0.10:
            j = 1 + 64 * int(rng.integers(0, cnts[i])) + int(rng.integers(0, 64))
            p[j] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.20:
            mo = struct.unpack_from("<H", t, 4)[0]
            j = mo + int(rng.integers(0, len(p) - mo))
            p[j] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.28:
            q = bytearray(p)   # frontrun: same first signature, different message
            q[-1] ^= 0x5a
            extra.append((bytes(q), t))
    pool = [(bytes(p), t) for p, t in txns] + extra
    order = []
    for k in range(n_total):
        r = rng.random()
        if order and r < 0.25:
            order.append(order[-int(rng.integers(1, min(len(order), 4) + 1))])      # near repeat
        elif order and r < 0.35:
            order.append(order[-int(rng.integers(1, len(order) + 1))])              # far repeat
        else:
            order.append(int(rng.integers(0, len(pool))))
    arena, frags = synth.pack_frags([pool[i] for i in order])
    kinds = ["short", "mtu", "rbh", "nosig", "manysig"]
    for i in rng.choice(n_total, size=n_total // 50, replace=False):
        _corrupt_frags(arena, frags, kinds[int(rng.integers(0, len(kinds)))], int(i))
    return arena, frags


@pytest.mark.gpu
def test_verify_frags_random_stream_vs_reference_tile(gpu, ref):
    """6000 frags in arrival order, fed in batches of 1, 7, 64, 500 and the
    rest with the tcache carried across calls: results and opt_sig equal the
    sequential reference tile's (reference tcache + reference verify)."""
    rng = np.random.default_rng(2024)
    arena, frags = _random_frag_stream(rng, 2500, 6000)
    exp_res, exp_tag = ref_seq(ref, arena, frags)
    stage = fa.VerifyStage(gpu=gpu, tcache=fa.TCache())
    got_res, got_tag, i = [], [], 0
    for b in [1, 7, 64, 500, len(frags)]:
        r, s = stage.verify_frags(arena, len(arena), frags[i:i + b])
        got_res.append(r); got_tag.append(s)
        i += len(r)
        if i >= len(frags):
            break
    got_res = np.concatenate(got_res); got_tag = np.concatenate(got_tag)
    bad = np.nonzero((got_res != exp_res) | (got_tag != exp_tag))[0]
    assert len(bad) == 0, [(int(j), int(got_res[j]), int(exp_res[j])) for j in bad[:10]]
    hist = {int(k): int(v) for k, v in zip(*np.unique(exp_res, return_counts=True))}
    assert hist.get(S, 0) > 1000 and hist.get(D, 0) > 300 and hist.get(F, 0) > 300 and hist.get(BAD, 0) > 30, hist


@pytest.mark.gpu
@pytest.mark.parametrize("devparse", [1, 0])
def test_stage_async_queue_depth_vs_reference_tile(gpu, ref, devparse):
    """The asynchronous stage (fd_ed25519_gpu_stage_*): batches of varying
    size submitted with up to STAGE_DEPTH outstanding (QUEUE_DEPTH of them on
    the GPU: the pipelined kernel's three phases + two queued launches; the
    rest launched by the completion worker), completed in order; results
    equal the sequential reference tile's -- with the frags parsed on the GPU
    (default) and on the host."""
    import ctypes as C
    rng = np.random.default_rng(77)
    arena, frags = _random_frag_stream(rng, 1500, 4000)
    exp_res, exp_tag = ref_seq(ref, arena, frags)
    lib = fa.load_lib()
    vp = C.c_void_p
    lib.fd_ed25519_gpu_stage_new.restype = vp
    lib.fd_ed25519_gpu_stage_new.argtypes = [vp, vp, C.c_uint64, C.c_int]
    lib.fd_ed25519_gpu_stage_submit.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp]
    lib.fd_ed25519_gpu_stage_poll.argtypes = [vp, C.c_int]
    lib.fd_ed25519_gpu_stage_pending.argtypes = [vp]
    lib.fd_ed25519_gpu_stage_delete.argtypes = [vp]
    tc = fa.TCache()
    st = lib.fd_ed25519_gpu_stage_new(gpu.ctx, tc.tc, 4096, 4)
    assert st
    lib.fd_ed25519_gpu_stage_set_device_parse.argtypes = [vp, C.c_int]
    assert lib.fd_ed25519_gpu_stage_set_device_parse(st, devparse) == 0
    # throw-away warm-up batches over this arena: must leave the tcache and results alone
    lib.fd_ed25519_gpu_stage_warm.argtypes = [vp, vp, C.c_uint64]
    assert lib.fd_ed25519_gpu_stage_warm(st, _vp(arena), len(arena)) == 0
    res = np.zeros(len(frags), np.int8)
    sig = np.zeros(len(frags), np.uint64)
    fr = np.ascontiguousarray(frags)
    bounds, i = [], 0
    for b in [1, 300, 2, 4096, 17, 1000]:
        if i >= len(frags):
            break
        b = min(b, len(frags) - i)
        bounds.append((i, b))
        i += b
    if i < len(frags):
        bounds.append((i, len(frags) - i))
    pend = 0
    for lo, b in bounds:
        while True:
            r = lib.fd_ed25519_gpu_stage_submit(st, _vp(arena), len(arena), fr[lo:].ctypes.data, b,
                                                res[lo:].ctypes.data, sig[lo:].ctypes.data)
            if r != -104:       # FD_ED25519_GPU_ERR_BUSY: complete the oldest first
                break
            assert lib.fd_ed25519_gpu_stage_poll(st, 1) == 0
        assert r == 0, r
        assert lib.fd_ed25519_gpu_stage_pending(st) <= fa.STAGE_DEPTH
    while lib.fd_ed25519_gpu_stage_pending(st):
        assert lib.fd_ed25519_gpu_stage_poll(st, 1) == 0
    lib.fd_ed25519_gpu_stage_delete(st)
    bad = np.nonzero((res != exp_res) | (sig != exp_tag))[0]
    assert len(bad) == 0, [(int(j), int(res[j]), int(exp_res[j])) for j in bad[:10]]


@pytest.mark.gpu
def test_offload_link_served_on_gpu_vs_reference_tile(gpu, ref):
    """The offload process's loop (fd_verify_offload_serve, here on a thread)
    behind the shared-memory link: a client publishes 4000 frags one by one
    (retrying on a full ring / frag area), reads the results by seq; they
    equal the sequential reference tile's."""
    rng = np.random.default_rng(78)
    arena, frags = _random_frag_stream(rng, 1500, 4000)
    exp_res, exp_tag = ref_seq(ref, arena, frags)
    name = "/fdvo_gpu_%d" % os.getpid()
    srv = fa.OffloadLink.create(name, depth=1024, dcache_sz=1 << 20)
    cli = fa.OffloadLink.join(name)
    th = fa.ServeThread(srv, gpu, fa.TCache(), max_batch=512, threads=2)
    got_r = np.zeros(len(frags), np.int8)
    got_s = np.zeros(len(frags), np.uint64)
    nxt = 0
    import time
    t0 = time.time()
    for i in range(len(frags)):
        f = arena[int(frags["off"][i]):int(frags["off"][i]) + int(frags["sz"][i])].tobytes()
        while True:
            # a result slot is reused when seq + depth is published: read first
            s = cli.publish(f) if i - nxt < 1024 else fa.offload.ERR_FULL
            if s != fa.offload.ERR_FULL:
                break
            st_, r, g = cli.result(nxt)
            if st_ == 1:
                got_r[nxt], got_s[nxt] = r, g
                nxt += 1
            assert time.time() - t0 < 90, "offload server stalled"
        assert s == i
        while nxt <= i:              # drain whatever is ready
            st_, r, g = cli.result(nxt)
            if st_ != 1:
                break
            got_r[nxt], got_s[nxt] = r, g
            nxt += 1
    while nxt < len(frags):
        st_, r, g = cli.result(nxt)
        assert st_ in (0, 1)
        if st_ == 1:
            got_r[nxt], got_s[nxt] = r, g
            nxt += 1
        assert time.time() - t0 < 90, "offload server stalled"
    cli.halt()
    stats = th.join(30)
    cli.close()
    srv.close()
    assert stats[1] == len(frags)
    bad = np.nonzero((got_r != exp_res) | (got_s != exp_tag))[0]
    assert len(bad) == 0, [(int(j), int(got_r[j]), int(exp_res[j])) for j in bad[:10]]


@pytest.mark.gpu
def test_offload_server_process_vs_reference_tile(ref):
    """The offload server as the sandboxed tile would run it: the C binary
    firedancer_amd/fd_verify_offload_server in a process of its own (no torch:
    the HIP runtime it links, /opt/rocm's), this process only a client of the
    shared-memory link (libfd_verify_offload.so, no HIP).  20,000 frags of a
    random stream (near and far repeats, corrupted signatures and messages,
    sanity failures) published in bursts; every result and opt_sig equals the
    sequential reference tile's, the server exits 0 with its stats, and its
    stderr has no failure line -- in particular no double hipHostUnregister of
    the frag area main() page-locks and the serve loop no longer re-registers
    (gpurun_out/offload_server_r05g.err)."""
    import subprocess
    import time
    rng = np.random.default_rng(5150)
    arena, frags = _random_frag_stream(rng, 3000, 20000)
    exp_res, exp_tag = ref_seq(ref, arena, frags)
    name = "/fdvo_srv_%d" % os.getpid()
    err_path = os.path.join(REPO, "gpurun_out", "offload_server_test.err")
    os.makedirs(os.path.dirname(err_path), exist_ok=True)
    env = dict(os.environ)
    env.pop("FD_ED25519_GPU_STAGE_AUTOREG", None)
    with open(err_path, "w") as ef:
        p = subprocess.Popen([fa.server_path(), "--name", name, "--batch", "4096", "--threads", "4",
                              "--dcache-mb", "64", "--depth", "8192"],
                             stdout=subprocess.PIPE, stderr=ef, env=env, text=True)
    try:
        line = p.stdout.readline()                        # {"ready": true} once the GPU is up and warm
        assert "ready" in line, (line, open(err_path).read())
        cli = fa.OffloadLink.join(name)
        n = len(frags)
        depth = cli.depth
        res = np.zeros(n, np.int8)
        sig = np.zeros(n, np.uint64)
        fr = np.ascontiguousarray(frags)
        pub = nxt = 0
        t0 = time.time()
        while nxt < n:
            if pub < n:      # a result slot is reused when seq + depth is published: stay within depth of nxt
                pub += cli.publish_burst(arena, fr[pub:min(n, nxt + depth)])
            if nxt < pub:
                nxt += cli.results(nxt, res[nxt:pub], sig[nxt:pub])
            assert time.time() - t0 < 90, ("offload server stalled", nxt, pub)
        cli.halt()
        cli.close()
        out, _ = p.communicate(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    err = open(err_path).read()
    assert p.returncode == 0, (p.returncode, out, err)
    stats = json.loads(out.strip().splitlines()[-1])
    assert stats["err"] == 0 and stats["frags"] == n and stats["batches"] > 4, stats
    assert "failed" not in err, err
    assert "runtime hip=" in err and "torch" not in err.split("runtime hip=")[1].split()[0], err
    bad = np.nonzero((res != exp_res) | (sig != exp_tag))[0]
    assert len(bad) == 0, [(int(j), int(res[j]), int(exp_res[j])) for j in bad[:10]]
    hist = {int(k): int(v) for k, v in zip(*np.unique(exp_res, return_counts=True))}
    assert hist.get(S, 0) > 3000 and hist.get(D, 0) > 1000 and hist.get(F, 0) > 1000 and hist.get(BAD, 0) > 100, hist


@pytest.mark.gpu
def test_stage_bench_shape_vs_reference_tile(ref):
    """The stage bench's own shape (tools/bench_verify_stage.py): its stream
    generator (1-4 signers, 10 % duplicates at short distances), 110,000 frags
    cut continuously into 36,000-frag batches (three full pipelined batches of
    ~64K signatures, one wave per SIMD each, and a remainder), the frags
    parsed inside the verify launch (the default), the area page-locked like
    the offload server's dcache.  Every result and opt_sig equals the
    sequential reference tile's over the same stream."""
    from bench_verify_stage import make_stream, stream_passes
    arena, frags, n_sigs = make_stream(110000, 0.1, seed=11)
    exp_res, exp_tag = ref_seq(ref, arena, frags)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 18)
    try:
        g.host_register(arena)
        ast = fa.AsyncStage(g, fa.TCache(), 36000, threads=8, device_parse=True)
        fr = np.ascontiguousarray(frags)
        res = np.zeros(len(fr), np.int8)
        sig = np.zeros(len(fr), np.uint64)
        stream_passes(ast, arena, fr, res, sig, 1, 36000)
        st = ast.stats()
        ast.close()
        pipe_l, one_l = g.launch_stats()
        g.host_unregister(arena)
    finally:
        g.close()
    assert st["batches"] == 4, st
    assert pipe_l >= 4, (pipe_l, one_l)                   # the batches ran on the pipelined kernel
    bad = np.nonzero((res != exp_res) | (sig != exp_tag))[0]
    assert len(bad) == 0, [(int(j), int(res[j]), int(exp_res[j])) for j in bad[:10]]
    hist = {int(k): int(v) for k, v in zip(*np.unique(exp_res, return_counts=True))}
    assert hist.get(S, 0) > 90000 and hist.get(D, 0) > 5000, hist


@pytest.mark.gpu
def test_stage_autoreg_keeps_callers_registration(gpu, monkeypatch):
    """One owner per page-locked range: with the stage's opt-in autoreg on, a
    frag area the caller registered itself stays registered after the stage
    is deleted (the caller's own unregister succeeds), and an area the stage
    registered is released by the stage.  (ROCm 7.2 answers a second
    hipHostRegister of a registered range with success, so the library asks
    the runtime first: fd_ed25519_gpu_host_is_registered.)"""
    monkeypatch.setenv("FD_ED25519_GPU_STAGE_AUTOREG", "1")
    fx = fixture_txns()
    for caller_registers in (True, False):
        arena, frags = _mk_frags([fx[k] for k in ["valid_txn_2sigs", "invalid_txn_same_1sig", "valid_txn_1sig"]])
        arena = np.concatenate([arena, np.zeros(8192, np.uint8)])
        if caller_registers:
            gpu.host_register(arena)
        assert fa.host_is_registered(arena) == caller_registers
        ast = fa.AsyncStage(gpu, fa.TCache(), 64, threads=1, device_parse=True)
        res = np.zeros(len(frags), np.int8); sig = np.zeros(len(frags), np.uint64)
        ast.submit(arena, len(arena), np.ascontiguousarray(frags), res, sig)
        while ast.pending():
            ast.poll(True)
        assert fa.host_is_registered(arena)               # registered while the stage holds it
        ast.close()
        assert list(res) == [S, F, S]
        assert fa.host_is_registered(arena) == caller_registers
        if caller_registers:
            gpu.host_unregister(arena)                    # raises if the stage had dropped it
        assert not fa.host_is_registered(arena)


@pytest.mark.gpu
def test_stage_device_parse_bad_frags(gpu):
    """The device parse classifies every sanity failure as the host parse
    does -- including a frag claiming more signatures than it can hold,
    which the verify grid's size relies on (FD_FRAG_SIG_BYTES)."""
    fx = fixture_txns()
    arena, frags = _mk_frags([fx["valid_txn_1sig"]] * len(BAD_KINDS) + [fx["valid_txn_2sigs"]])
    for i, k in enumerate(BAD_KINDS):
        _corrupt_frags(arena, frags, k, i)
    out = {}
    for devparse in (True, False):
        ast = fa.AsyncStage(gpu, fa.TCache(), 64, threads=1, device_parse=devparse)
        res = np.zeros(len(frags), np.int8); sig = np.zeros(len(frags), np.uint64)
        ast.submit(arena, len(arena), np.ascontiguousarray(frags), res, sig)
        while ast.pending():
            ast.poll(True)
        ast.close()
        out[devparse] = (res.copy(), sig.copy())
    assert list(out[True][0]) == [BAD, BAD, BAD, F, F, BAD, BAD, S, S]
    assert np.array_equal(out[True][0], out[False][0]) and np.array_equal(out[True][1], out[False][1])


@pytest.mark.gpu
def test_stage_device_parse_fields_outside_frag(gpu):
    """Device parse = host parse on frags whose fields point past the frag
    (one of them across a hole the copy plan does not send): BAD_FRAG in
    both, the valid frags around them verified."""
    arena, frags = _fields_outside_stream()
    out = {}
    for devparse in (True, False):
        ast = fa.AsyncStage(gpu, fa.TCache(), 64, threads=1, device_parse=devparse)
        res = np.zeros(len(frags), np.int8); sig = np.zeros(len(frags), np.uint64)
        ast.submit(arena, len(arena), np.ascontiguousarray(frags), res, sig)
        while ast.pending():
            ast.poll(True)
        ast.close()
        out[devparse] = (res.copy(), sig.copy())
    assert list(out[True][0]) == [S, BAD, BAD, S, BAD, D], list(out[True][0])
    assert np.array_equal(out[True][0], out[False][0]) and np.array_equal(out[True][1], out[False][1])


@pytest.mark.gpu
def test_stage_frag_areas_freed_between_batches(gpu):
    """The stage does not page-lock callers' frag areas by default (ADVICE
    r04): a frag area freed after its batch's poll and a new one (possibly at
    the same addresses) give correct results, and the caller can register
    the new area itself afterwards (it is not left registered by the stage)."""
    fx = fixture_txns()
    ast = fa.AsyncStage(gpu, fa.TCache(), 64, threads=1, device_parse=True)
    try:
        for rnd in range(3):
            names = ["valid_txn_2sigs", "invalid_txn_same_1sig", "valid_txn_1sig"]   # :219-264's F-then-S pair
            arena, frags = _mk_frags([fx[k] for k in names])
            arena = arena.copy()
            res = np.zeros(len(frags), np.int8); sig = np.zeros(len(frags), np.uint64)
            ast.tcache.reset()
            ast.submit(arena, len(arena), np.ascontiguousarray(frags), res, sig)
            while ast.pending():
                ast.poll(True)
            assert list(res) == [S, F, S], (rnd, list(res))
            gpu.host_register(arena)          # fails with AlreadyRegistered if the stage had kept it
            gpu.host_unregister(arena)
            del arena, frags
    finally:
        ast.close()


@pytest.mark.gpu
def test_stage_device_parse_signature_bound_edges(gpu):
    """The sz / 96 signature bound at its edge, device parse against host
    parse: a frag claiming exactly sz // 96 signatures is parsed and verified
    (its extra signatures are garbage, so it fails -- FAILED, or BAD_FRAG in
    both if the claimed signatures run past the frag span); one more is
    BAD_FRAG in both."""
    fx = fixture_txns()
    txns = [fx["valid_txn_1sig"], fx["valid_txn_2sigs"]] * 3
    kinds = ["claim_at_bound", "claim_past_bound", None] * 2
    arena, frags = _mk_frags(txns)
    for i, k in enumerate(kinds):
        _corrupt_frags(arena, frags, k, i)
    out = {}
    for devparse in (True, False):
        ast = fa.AsyncStage(gpu, fa.TCache(), 64, threads=1, device_parse=devparse)
        res = np.zeros(len(frags), np.int8); sig = np.zeros(len(frags), np.uint64)
        ast.submit(arena, len(arena), np.ascontiguousarray(frags), res, sig)
        while ast.pending():
            ast.poll(True)
        ast.close()
        out[devparse] = (res.copy(), sig.copy())
    assert np.array_equal(out[True][0], out[False][0]) and np.array_equal(out[True][1], out[False][1])
    r = out[True][0]
    assert r[1] == BAD and r[4] == BAD                     # past the bound
    assert r[0] in (F, BAD) and r[3] in (F, BAD)           # at the bound: parsed, fails
    assert r[2] == S and r[5] == S


@pytest.mark.gpu
@pytest.mark.parametrize("n", [60000, 70000])
def test_stage_device_parse_many_workgroups(gpu, n):
    """One device-parsed batch of 60,000 frags (235 parse workgroups, the
    pipelined verify kernel: at most one wave per SIMD) and of 70,000 (274
    workgroups, so the last workgroup's scan of the workgroup totals runs two
    rounds of 256; the one-shot kernels); frags cross every workgroup
    boundary.  The stage's results equal the host parse's, frag for frag
    (both replay the same tcache steps over the same stream: a pool of 2,500
    signed txns with 1-8 signatures, some corrupted, repeated)."""
    rng = np.random.default_rng(2024 + n)
    arena_u, frags_u = _random_frag_stream(rng, 2500, 2500)
    order = rng.integers(0, len(frags_u), size=n)
    frags = np.zeros(n, frags_u.dtype)
    frags["off"] = frags_u["off"][order]
    frags["sz"] = frags_u["sz"][order]
    big = fa.Ed25519Gpu(device_mask=1, max_batch=16 * n)
    out, stats = {}, {}
    try:
        for devparse in (True, False):
            if devparse:
                big.host_stats(reset=True)
            ast = fa.AsyncStage(big, fa.TCache(), n, threads=8, device_parse=devparse)
            res = np.zeros(n, np.int8); sig = np.zeros(n, np.uint64)
            ast.submit(arena_u, len(arena_u), np.ascontiguousarray(frags), res, sig)
            while ast.pending():
                ast.poll(True)
            stats[devparse] = ast.stats()
            if devparse:
                hs = big.host_stats()
            ast.close()
            out[devparse] = (res, sig)
    finally:
        big.close()
    bad = np.nonzero((out[True][0] != out[False][0]) | (out[True][1] != out[False][1]))[0]
    assert len(bad) == 0, [(int(j), int(out[True][0][j]), int(out[False][0][j])) for j in bad[:10]]
    hist = {int(k): int(v) for k, v in zip(*np.unique(out[True][0], return_counts=True))}
    st = stats[True]
    assert st["batches"] == 1 and st["replay_ns"] > 0, st          # the stage's own counters
    assert hs["h2d_bytes"] >= len(arena_u) // 2, hs                 # the device parse sent the frags' pages
    assert hist.get(S, 0) > 1000 and hist.get(D, 0) > 1000, hist


@pytest.mark.gpu
def test_stage_in_launch_parse_vs_parse_launch(monkeypatch, ref):
    """The pipelined path's in-launch parse (the verify launch's phase-A waves
    parse the batch's frags, look-back scan and all, then wait for the tiles
    holding their descriptors) against a parse launch first
    (FD_ED25519_GPU_APARSE=0), frag for frag, over one stream of five
    batches: 33,000 frags of 1-8 signatures with a third of them made
    BAD_FRAG in runs (so descriptors are sparse and a workgroup's descriptors
    come from tiles far from its own index), a 66,000-frag batch (above one
    wave per SIMD: a parse launch and the one-shot kernels, between pipelined
    batches), a batch with no valid frag (count 0), a batch of one frag and
    the first batch reversed."""
    rng = np.random.default_rng(4242)
    arena_u, frags_u = _random_frag_stream(rng, 2500, 2500)
    n, n_big = 33000, 66000
    order = rng.integers(0, len(frags_u), size=n_big)
    big = np.zeros(n_big, frags_u.dtype)
    big["off"] = frags_u["off"][order]
    big["sz"] = frags_u["sz"][order]
    frags = big[:n].copy()
    for s0 in range(0, n, 3000):                       # runs of frags past the arena: BAD_FRAG
        frags["off"][s0:s0 + int(rng.integers(200, 1500))] = len(arena_u) + 64
    allbad = frags[:700].copy()
    allbad["off"] = len(arena_u) + 64
    batches = [frags, big, allbad, frags[5:6].copy(), frags[::-1].copy()]
    out = {}
    for ap in ("1", "0"):
        monkeypatch.setenv("FD_ED25519_GPU_APARSE", ap)
        g = fa.Ed25519Gpu(device_mask=1, max_batch=16 * n_big)
        try:
            ast = fa.AsyncStage(g, fa.TCache(), n_big, threads=8, device_parse=True)
            res = [np.zeros(len(b), np.int8) for b in batches]
            sig = [np.zeros(len(b), np.uint64) for b in batches]
            for b, r, s in zip(batches, res, sig):
                ast.submit(arena_u, len(arena_u), np.ascontiguousarray(b), r, s)
            while ast.pending():
                ast.poll(True)
            ast.close()
            pipe_l, one_l = g.launch_stats()
            assert pipe_l > 0 and one_l > 0, (pipe_l, one_l)  # both kernels ran
        finally:
            g.close()
        out[ap] = (res, sig)
    for k in range(len(batches)):
        bad = np.nonzero((out["1"][0][k] != out["0"][0][k]) | (out["1"][1][k] != out["0"][1][k]))[0]
        assert len(bad) == 0, (k, [(int(j), int(out["1"][0][k][j]), int(out["0"][0][k][j])) for j in bad[:10]])
    exp = ref_seq_stream(ref, arena_u, batches)           # and both against the reference tile
    assert_vs_ref(out["1"][0], out["1"][1], exp, "in-launch parse")
    hist = {int(c): int(v) for c, v in zip(*np.unique(out["1"][0][0], return_counts=True))}
    assert hist.get(S, 0) > 1000 and hist.get(BAD, 0) > 3000, hist
    assert np.all(out["1"][0][2] == BAD)


@pytest.mark.gpu
def test_stage_in_launch_parse_two_contexts_concurrently(ref):
    """Two contexts on one GPU, each with its own stage, fed from two threads
    at once: their pipelined verify launches share the CUs, so a launch's
    workgroups are not all resident together.  The in-launch parse takes its
    tiles from a counter in order, so its waits still end; both streams
    (frags with runs of BAD_FRAG, so descriptors are sparse across tiles)
    give the results of one context alone."""
    import threading
    rng = np.random.default_rng(99)
    arena_u, frags_u = _random_frag_stream(rng, 2500, 2500)
    n = 30000
    streams = []
    for k in range(2):
        order = rng.integers(0, len(frags_u), size=n)
        fr = np.zeros(n, frags_u.dtype)
        fr["off"] = frags_u["off"][order]
        fr["sz"] = frags_u["sz"][order]
        for s0 in range(0, n, 2500):
            fr["off"][s0:s0 + int(rng.integers(300, 1800))] = len(arena_u) + 64
        streams.append([fr[j:j + 10000].copy() for j in range(0, n, 10000)] * 3)

    def run(g, batches, res, sig, errs):
        try:
            ast = fa.AsyncStage(g, fa.TCache(), 10000, threads=4, device_parse=True)
            for b, r, s in zip(batches, res, sig):          # nine batches: one more than STAGE_DEPTH
                if ast.pending() == fa.STAGE_DEPTH:
                    ast.poll(True)
                ast.submit(arena_u, len(arena_u), np.ascontiguousarray(b), r, s)
            while ast.pending():
                ast.poll(True)
            ast.close()
        except Exception as e:                          # noqa: BLE001
            errs.append(e)

    ctxs = [fa.Ed25519Gpu(device_mask=1, max_batch=16 * 10000) for _ in range(2)]
    try:
        out = {}
        for mode in ("alone", "together"):
            res = [[np.zeros(len(b), np.int8) for b in streams[k]] for k in range(2)]
            sig = [[np.zeros(len(b), np.uint64) for b in streams[k]] for k in range(2)]
            errs = []
            if mode == "alone":
                for k in range(2):
                    run(ctxs[k], streams[k], res[k], sig[k], errs)
            else:
                th = [threading.Thread(target=run, args=(ctxs[k], streams[k], res[k], sig[k], errs)) for k in range(2)]
                for t in th:
                    t.start()
                for t in th:
                    t.join(120)
                assert not any(t.is_alive() for t in th), "a stage did not finish"
            assert not errs, errs
            out[mode] = (res, sig)
        for k in range(2):
            for j in range(len(streams[k])):
                assert np.array_equal(out["alone"][0][k][j], out["together"][0][k][j]), (k, j)
                assert np.array_equal(out["alone"][1][k][j], out["together"][1][k][j]), (k, j)
            exp = ref_seq_stream(ref, arena_u, streams[k])   # each stream against the reference tile
            assert_vs_ref(out["together"][0][k], out["together"][1][k], exp, "stream %d" % k)
    finally:
        for g in ctxs:
            g.close()


@pytest.mark.gpu
def test_stage_in_launch_parse_small_signature_bound(monkeypatch, ref):
    """A pipelined frag batch whose host-side signature bound is tiny (30,000
    64-byte junk frags bound no signature) but whose parse has 118 tiles:
    the launch still gets a workgroup per tile to parse them, and the valid
    frags behind the junk verify -- against a parse launch first
    (FD_ED25519_GPU_APARSE=0), frag for frag."""
    rng = np.random.default_rng(7)
    arena_u, frags_u = _random_frag_stream(rng, 200, 200)
    junk = np.zeros(30000, frags_u.dtype)
    junk["off"] = rng.integers(0, len(arena_u) - 64, size=len(junk)).astype(np.uint32)
    junk["sz"] = 64
    batch = np.concatenate([junk, frags_u[:150]])
    out = {}
    for ap in ("1", "0"):
        monkeypatch.setenv("FD_ED25519_GPU_APARSE", ap)
        g = fa.Ed25519Gpu(device_mask=1, max_batch=16 * len(batch))
        try:
            ast = fa.AsyncStage(g, fa.TCache(), len(batch), threads=4, device_parse=True)
            res = np.zeros(len(batch), np.int8); sig = np.zeros(len(batch), np.uint64)
            ast.submit(arena_u, len(arena_u), np.ascontiguousarray(batch), res, sig)
            while ast.pending():
                ast.poll(True)
            ast.close()
        finally:
            g.close()
        out[ap] = (res, sig)
    assert np.array_equal(out["1"][0], out["0"][0]) and np.array_equal(out["1"][1], out["0"][1])
    # no junk frag verifies (most are BAD_FRAG: their fd_txn_t would lie outside the
    # frag, DESIGN §7's documented rule), so none inserts into the tcache; the valid
    # frags behind them then give the reference tile's results over those frags alone
    assert not np.any(out["1"][0][:len(junk)] == S)
    er, et = ref_seq(ref, arena_u, batch[len(junk):])
    assert_vs_ref([out["1"][0][len(junk):]], [out["1"][1][len(junk):]], [(er, et)], "valid frags behind junk")
    assert np.count_nonzero(out["1"][0][len(junk):] == S) > 50
