"""GPU: the reference's own remaining test scenarios and the full-size
config-3 batch (VERDICT r01 missing #4 / #5).

* test_cctv_batch (src/ballet/ed25519/test_ed25519.c:1041-1082): each CCTV
  vector over message #7 at slot 1 of a 2- and a 4-signature batch next to
  fresh valid signatures -- through the single-message drop-in (both code
  flavours) and as one descriptor batch + fd_ed25519_gpu_txn_reduce.
* corpus/fuzz_ed25519_sigverify seeds (fuzz_ed25519_sigverify.c:30-49).
* config 3 at full size: 1,048,576 descriptors, messages of 0..1232 bytes,
  through ONE context whose table scratch holds 262,144 signatures, so the
  batch runs as four chunked launches of the single-lane kernel.  Every
  descriptor's code is checked: the 16,384 distinct records (4,096 signed
  records, each also in three corrupted forms) get their expected codes from
  the oracle, and each of the 1M descriptors must equal its record's."""
import ctypes
import os
import sys

import numpy as np
import pytest

import firedancer_amd as fa
from golden_io import read_sigs, read_txns

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("flavour,key", [(fa.CODES_AVX512, "code"), (fa.CODES_REF, "code_ref")])
def test_cctv_batch_scenario_single_msg(gpu, flavour, key):
    recs = read_txns("cctv_batches.bin")
    gpu.set_codes(flavour)
    try:
        got = [gpu.verify_batch_single_msg(r["msg"], b"".join(r["sigs"]), b"".join(r["pubs"]), r["n"]) for r in recs]
    finally:
        gpu.set_codes(fa.CODES_AVX512)
    assert got == [r[key] for r in recs]


def test_cctv_batch_scenario_one_launch(gpu):
    recs = read_txns("cctv_batches.bin")
    flat = []
    for ti, r in enumerate(recs):
        for j in range(r["n"]):
            flat.append((r["msg"], r["sigs"][j], r["pubs"][j], ti))
    arena, desc, sz = fa.pack_batch(flat)
    codes = gpu.verify_batch(arena, sz, desc)
    per_txn = fa.txn_reduce(codes, desc)
    assert np.array_equal(per_txn, np.array([r["code"] for r in recs], np.int8))


def test_fuzz_corpus_seeds(gpu):
    recs = read_sigs("fuzz_seeds.bin")
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    assert np.array_equal(gpu.verify_batch(arena, sz, desc), np.zeros(len(recs), np.int8))
    for r in recs:
        assert gpu.verify(r["msg"], r["sig"], r["pub"]) == 0


def _config3_records(n_base=4096, seed=31):
    """n_base signed records (distinct keys, Uniform{0..1232}-B messages), each
    also as: message bit flipped, S high bit set (S >= l), S low-half bit
    flipped.  Returns (arena, unique descriptors [4 n_base])."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import synth
    rng = np.random.default_rng(seed)
    seeds = [rng.bytes(32) for _ in range(n_base)]
    sizes = rng.integers(0, 1233, size=n_base)
    msgs = [rng.bytes(int(z)) for z in sizes]
    kps = synth.keypairs(seeds, threads=16)
    sigs = synth.sign_many([kps[i] + (msgs[i],) for i in range(n_base)], threads=16)
    recs = []
    for i in range(n_base):
        m, s, p = msgs[i], sigs[i], kps[i][1]
        recs.append((m, s, p))
        mm = bytearray(m) if m else bytearray(b"\x00")
        mm[int(rng.integers(0, len(mm)))] ^= 1 << int(rng.integers(0, 8))
        recs.append((bytes(mm), s, p))
        s2 = bytearray(s); s2[63] |= 0x80
        recs.append((m, bytes(s2), p))
        s3 = bytearray(s); s3[32 + int(rng.integers(0, 16))] ^= 1 << int(rng.integers(0, 8))
        recs.append((m, bytes(s3), p))
    arena, desc, sz = fa.pack_batch(recs)
    return arena, desc, sz


def test_config3_full_size_chunked(oracle):
    n = 1 << 20
    arena, udesc, sz = _config3_records()
    u = len(udesc)
    exp_u = np.zeros(u, np.int8)
    oracle.fdo_verify_descs(arena.ctypes.data_as(ctypes.c_void_p), udesc.ctypes.data_as(ctypes.c_void_p), u,
                            exp_u.ctypes.data_as(ctypes.c_void_p), 0)
    hist = {int(k): int(v) for k, v in zip(*np.unique(exp_u, return_counts=True))}
    assert hist.get(0, 0) >= u // 4 - 8 and hist.get(-1, 0) >= u // 4 and hist.get(-3, 0) >= u // 4, hist
    pick = np.random.default_rng(5).integers(0, u, size=n)
    desc = udesc[pick].copy()
    desc["txn_idx"] = np.arange(n) & 0xffff
    g = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 18)   # table scratch for 256K: 4 chunked launches
    try:
        out = g.verify_batch(arena, sz, desc)
    finally:
        g.close()
    bad = np.nonzero(out != exp_u[pick])[0]
    assert len(bad) == 0, [(int(i), int(out[i]), int(exp_u[pick[i]])) for i in bad[:10]]
    # and a direct oracle sample on the expanded batch (not via the record map)
    for i in np.random.default_rng(9).choice(n, 1024, replace=False):
        d = desc[i]
        m = arena[d["msg_off"]:d["msg_off"] + d["msg_sz"]].tobytes()
        s = arena[d["sig_off"]:d["sig_off"] + 64].tobytes()
        p = arena[d["pub_off"]:d["pub_off"] + 32].tobytes()
        assert out[i] == oracle.fdo_verify(m, len(m), s, p, 0)


def test_pipe_variable_lengths_length_order(gpu, oracle):
    """The pipelined form on config-3-like traffic: three 64K batches of
    Uniform{0..1232}-B messages (a quarter each valid / message-flipped / S >= l
    / S-flipped), so phase A's in-workgroup length order permutes every full
    workgroup; every code is the oracle's."""
    import torch
    arena, udesc, sz = _config3_records(n_base=2048, seed=37)
    u = len(udesc)
    exp_u = np.zeros(u, np.int8)
    oracle.fdo_verify_descs(arena.ctypes.data_as(ctypes.c_void_p), udesc.ctypes.data_as(ctypes.c_void_p), u,
                            exp_u.ctypes.data_as(ctypes.c_void_p), 0)
    n = 65536
    rng = np.random.default_rng(11)
    picks = [rng.integers(0, u, size=n) for _ in range(3)]
    d_arena = torch.from_numpy(arena.copy()).cuda()
    d_descs = [torch.from_numpy(udesc[p].copy().view(np.uint8)).cuda() for p in picks]
    outs = [torch.full((n,), 99, dtype=torch.int8, device="cuda:0") for _ in picks]
    st = torch.cuda.Stream()
    for d, o in zip(d_descs, outs):
        gpu.pipe_dev(d_arena.data_ptr(), sz, d.data_ptr(), n, o.data_ptr(), stream=st.cuda_stream)
    gpu.pipe_flush_dev(stream=st.cuda_stream)
    torch.cuda.synchronize()
    for p, o in zip(picks, outs):
        got = o.cpu().numpy()
        bad = np.nonzero(got != exp_u[p])[0]
        assert len(bad) == 0, [(int(i), int(got[i]), int(exp_u[p[i]])) for i in bad[:10]]
