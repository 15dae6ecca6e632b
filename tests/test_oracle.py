"""CPU: the oracle (our C restatement, oracle/fd_ed25519_oracle.c) against the
golden fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import ctypes
import hashlib
from collections import Counter

import pytest

from golden_io import read_sha, read_sigs, read_txns


@pytest.mark.parametrize("fname", ["vectors_ref.bin", "synthetic.bin", "fuzz_seeds.bin"])
def test_oracle_codes_bit_exact(oracle, fname):
    recs = read_sigs(fname)
    assert recs
    for r in recs:
        a = oracle.fdo_verify(r["msg"], len(r["msg"]), r["sig"], r["pub"], 0)
        b = oracle.fdo_verify(r["msg"], len(r["msg"]), r["sig"], r["pub"], 1)
        assert (a, b) == (r["code"], r["code_ref"]), (fname, r["set"], r["tc_id"])
        if r["ok"] in (0, 1):   # accept/reject asserted by the reference's own tests
            assert (a == 0) == (r["ok"] == 1)


def test_golden_distribution_matches_survey():
    """The code histograms the survey recorded from the reference builds."""
    v = read_sigs("vectors_ref.bin")
    hist = lambda s, k: dict(Counter(x[k] for x in v if x["set"] == s))
    assert hist(1, "code") == {0: 84, -1: 36, -3: 13}
    assert hist(2, "code") == {0: 43, -1: 442, -2: 366, -3: 63}
    assert hist(2, "code_ref") == {0: 43, -1: 282, -2: 526, -3: 63}
    assert hist(4, "code") == {-1: 75, -2: 121}
    assert hist(4, "code_ref") == {-2: 196}
    assert hist(5, "code") == {0: 200}


@pytest.mark.parametrize("fname", ["txn_batches.bin", "cctv_batches.bin"])
def test_oracle_txn_batches(oracle, fname):
    for r in read_txns(fname):
        sigs = b"".join(r["sigs"]) or bytes(64)
        pubs = b"".join(r["pubs"]) or bytes(32)
        for fl, exp in ((0, r["code"]), (1, r["code_ref"])):
            assert oracle.fdo_verify_batch_single_msg(r["msg"], len(r["msg"]), sigs, pubs, r["n"], fl) == exp


def test_oracle_sha512_kat(oracle):
    out = ctypes.create_string_buffer(64)
    kats = read_sha()
    assert len(kats) > 100
    for m, md in kats:
        oracle.fdo_sha512(m, len(m), out)
        assert out.raw == md
        assert hashlib.sha512(m).digest() == md


def test_reference_scenarios_present():
    """test_cctv_batch (test_ed25519.c:1041-1082): every CCTV vector over
    message #7 at slot 1 of a 2- and a 4-signature batch, accept/reject as the
    reference test asserts; the 4 fuzz corpus seeds sign+verify to SUCCESS."""
    cb = read_txns("cctv_batches.bin")
    assert len(cb) == 206 and {r["n"] for r in cb} == {2, 4}
    cctv7 = [r for r in read_sigs("vectors_ref.bin") if r["set"] == 2 and r["msg"] == cb[0]["msg"]]
    assert len(cctv7) == 103
    for i, v in enumerate(cctv7):
        for r in cb[2 * i:2 * i + 2]:
            assert r["sigs"][1] == v["sig"] and r["pubs"][1] == v["pub"]
            assert (r["code"] == 0) == (v["ok"] == 1)
    fz = read_sigs("fuzz_seeds.bin")
    assert len(fz) == 4 and all(r["code"] == 0 and r["code_ref"] == 0 for r in fz)
