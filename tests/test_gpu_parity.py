"""GPU parity: the HIP path (through the C ABI) against the golden codes the
reference produced (tests/golden) and against the oracle on the same inputs.
Bar: bit-exact FD_ED25519_* codes for every descriptor."""
import numpy as np
import pytest

import firedancer_amd as fa
from golden_io import read_sigs, read_txns

pytestmark = pytest.mark.gpu


def _all_golden():
    return read_sigs("vectors_ref.bin") + read_sigs("synthetic.bin")


def test_golden_vectors_avx512_codes(gpu):
    recs = _all_golden()
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    gpu.set_codes(fa.CODES_AVX512)
    out = gpu.verify_batch(arena, sz, desc)
    exp = np.array([r["code"] for r in recs], dtype=np.int8)
    bad = np.nonzero(out != exp)[0]
    assert len(bad) == 0, [(recs[i]["set"], recs[i]["tc_id"], int(out[i]), int(exp[i])) for i in bad[:20]]


def test_golden_vectors_ref_codes(gpu):
    recs = _all_golden()
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    gpu.set_codes(fa.CODES_REF)
    try:
        out = gpu.verify_batch(arena, sz, desc)
    finally:
        gpu.set_codes(fa.CODES_AVX512)
    exp = np.array([r["code_ref"] for r in recs], dtype=np.int8)
    assert np.array_equal(out, exp)


def test_single_verify_dropin(gpu):
    recs = [r for r in read_sigs("vectors_ref.bin") if r["set"] == 1][:20]
    for r in recs:
        assert gpu.verify(r["msg"], r["sig"], r["pub"]) == r["code"]


def test_txn_batches_single_msg(gpu):
    for r in read_txns():
        got = gpu.verify_batch_single_msg(r["msg"], b"".join(r["sigs"]), b"".join(r["pubs"]), r["n"])
        assert got == r["code"], (r["n"], got, r["code"])


def test_txn_batches_as_one_descriptor_batch(gpu):
    """All multi-sig txns in ONE launch, then the host-side two-phase reduce."""
    txns = [t for t in read_txns() if 1 <= t["n"] <= 16]
    recs = []
    for ti, t in enumerate(txns):
        for j in range(t["n"]):
            recs.append((t["msg"], t["sigs"][j], t["pubs"][j], ti))
    arena, desc, sz = fa.pack_batch(recs)
    codes = gpu.verify_batch(arena, sz, desc)
    per_txn = fa.txn_reduce(codes, desc)
    assert np.array_equal(per_txn, np.array([t["code"] for t in txns], dtype=np.int8))


def test_unaligned_and_shared_fields(gpu, oracle):
    """Fields at every byte alignment, a message shared by many sigs, msg at the arena end."""
    recs = read_sigs("synthetic.bin")[:300]
    rng = np.random.default_rng(7)
    arena = bytearray()
    desc = np.zeros(len(recs), dtype=fa.DESC_DTYPE)
    for i, r in enumerate(recs):
        arena += bytes(int(rng.integers(0, 7)))
        so = len(arena); arena += r["sig"]
        arena += bytes(int(rng.integers(0, 5)))
        po = len(arena); arena += r["pub"]
        arena += bytes(int(rng.integers(0, 3)))
        mo = len(arena); arena += r["msg"]
        desc[i] = (so, po, mo, len(r["msg"]), i)
    sz = len(arena)
    a = np.frombuffer(bytes(arena) + bytes(16), np.uint8)
    out = gpu.verify_batch(a, sz, desc)
    assert np.array_equal(out, np.array([r["code"] for r in recs], np.int8))


def _corrupted_batch(n, seed):
    """n descriptors built from the 1024 valid config-1 sigs with a known corruption
    per index (expected code known by construction, checked against the oracle)."""
    base = [r for r in read_sigs("synthetic.bin") if r["set"] == 10]
    rng = np.random.default_rng(seed)
    recs, kinds = [], rng.integers(0, 4, n)
    for i in range(n):
        r = base[i % len(base)]
        msg, sig, pub = bytearray(r["msg"]), bytearray(r["sig"]), r["pub"]
        if kinds[i] == 1:
            msg[int(rng.integers(0, len(msg)))] ^= 1 << int(rng.integers(0, 8))
        elif kinds[i] == 2:
            sig[63] |= 0x80
        elif kinds[i] == 3:
            sig[32 + int(rng.integers(0, 16))] ^= 1 << int(rng.integers(0, 8))
        recs.append((bytes(msg), bytes(sig), pub))
    return recs, kinds


def test_config2_64k_properties_and_oracle_sample(gpu, oracle):
    n = 65536
    recs, kinds = _corrupted_batch(n, 11)
    arena, desc, sz = fa.pack_batch(recs)
    out = gpu.verify_batch(arena, sz, desc)
    assert np.all(out[kinds == 0] == 0)
    assert np.all(out[kinds == 1] == -3)
    assert np.all(out[kinds == 2] == -1)
    assert np.all(out[(kinds == 3)] == -3)
    idx = np.random.default_rng(3).choice(n, 1024, replace=False)
    for i in idx:
        m, s, p = recs[i]
        assert out[i] == oracle.fdo_verify(m, len(m), s, p, 0)


def test_async_submit_poll(gpu):
    recs = _all_golden()[:512]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    out = np.zeros(len(desc), np.int8)
    gpu.submit(arena, sz, desc, out)
    import time
    t0 = time.time()
    while not gpu.poll():
        assert time.time() - t0 < 60
        time.sleep(0.001)
    assert np.array_equal(out, np.array([r["code"] for r in recs], np.int8))


def test_device_pointer_entry_point(gpu):
    import torch
    recs = _all_golden()[:1000]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    d_arena = torch.from_numpy(arena.copy()).to("cuda:0")
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to("cuda:0")
    d_out = torch.zeros(len(desc), dtype=torch.int8, device="cuda:0")
    stream = torch.cuda.current_stream()
    gpu.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), len(desc), d_out.data_ptr(),
                         stream=stream.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), np.array([r["code"] for r in recs], np.int8))


def test_bad_descriptor(gpu):
    r = read_sigs("synthetic.bin")[0]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"])])
    desc[0]["msg_sz"] = 60000
    with pytest.raises(fa.GpuError):
        gpu.verify_batch(arena, sz, desc)


def test_empty_batch(gpu):
    out = gpu.verify_batch(np.zeros(16, np.uint8), 0, np.zeros(0, fa.DESC_DTYPE))
    assert len(out) == 0


L_ORDER = 2**252 + 27742317777372353535851937790883648493


def _words_to_int(w):
    return sum(int(x) << (32 * i) for i, x in enumerate(w))


def lat_euclid_check(k, u, v, n8):
    """The search's output is the one the exact extended Euclid on (8l, k)
    gives: at the first remainder r_i < 2^128, (u, v) = (r_i, t_i) up to sign
    when t_i is odd, else (r_{i-1} - j r_i, t_{i-1} - j t_i) for some j >= 0
    (fd_lattice_dev.h).  Pins every quotient of the Lehmer rounds, not only
    the lattice relation."""
    r0, t0, r1, t1 = n8, 0, k, 1
    while r1 >= 2**128:
        q = r0 // r1
        r0, r1, t0, t1 = r1, r0 - q * r1, t1, t0 - q * t1
    if t1 % 2:
        return (u, v) == ((r1, t1) if t1 > 0 else (-r1, -t1))
    j, rem = divmod(v - abs(t0), abs(t1))
    return rem == 0 and j >= 0 and u == (r0 - j * r1) * (1 if t0 > 0 else -1)


def test_lattice_device_random_and_adversarial_k(gpu):
    """The device short-vector search (fd_lattice_dev.h) on 200K random k and
    structured k: u = v k (mod 8l), v odd, 0 < v < l -- the conditions that make
    [v]([S]B - [k]A - R) == O equivalent to the reference's equation."""
    rng = np.random.default_rng(5)
    n = 200_000
    ks = [int.from_bytes(rng.bytes(32), "little") % L_ORDER for _ in range(n)]
    ks += [0, 1, 2, 3, L_ORDER - 1, L_ORDER - 2, 2**128 - 1, 2**128, 2**128 + 1, 2**127, 2**200, 2**252,
           (8 * L_ORDER // 3) % L_ORDER, (8 * L_ORDER // 5) % L_ORDER, 2**64, 12345]
    ks += [int.from_bytes(rng.bytes(32), "little") % (1 << int(rng.integers(1, 253))) for _ in range(4096)]
    kw = np.array([[(k >> (32 * j)) & 0xffffffff for j in range(8)] for k in ks], dtype=np.uint32)
    out = gpu.test_lattice(kw)
    n8 = 8 * L_ORDER
    bits = []
    for i, k in enumerate(ks):
        u = _words_to_int(out[i, 0:8]) * (-1 if out[i, 16] else 1)
        v = _words_to_int(out[i, 8:16])
        assert v % 2 == 1 and 0 < v < L_ORDER, (k, u, v)
        assert (u - v * k) % n8 == 0, (k, u, v)
        if (i < 50_000 or i >= n) and k:
            assert lat_euclid_check(k, u, v, n8), (k, u, v)
        bits.append(max(abs(u).bit_length(), v.bit_length()))
    # random k: the vectors are ~2^128 (what the ~130-doubling loop is sized for)
    assert max(bits[:n]) <= 140 and int(np.percentile(bits[:n], 99)) <= 131


def test_fresh_keys_reference_signed(gpu, oracle):
    """32K distinct keys / messages (so 32K distinct k, R, A), signed here by the
    reference fd_ed25519_sign (oracle/_ref), variable message lengths 0..1232,
    a quarter corrupted: codes == the reference fd_ed25519_verify's."""
    import ctypes, os
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libfdref_avx512.so")
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built (needs /root/reference in the dev container)")
    ref = ctypes.CDLL(so)
    ref.fdref_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    ref.fdref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
    ref.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
    rng = np.random.default_rng(99)
    n = 32768
    recs, exp = [], []
    for i in range(n):
        priv = rng.bytes(32)
        pub = ctypes.create_string_buffer(32); ref.fdref_public_from_private(pub, priv)
        msg = rng.bytes(int(rng.integers(0, 1233)))
        sig = ctypes.create_string_buffer(64); ref.fdref_sign(sig, msg, len(msg), pub.raw, priv)
        s, m = bytearray(sig.raw), bytearray(msg)
        kind = i & 3
        if kind == 1 and len(m):
            m[int(rng.integers(0, len(m)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            s[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))     # R bit flip
        elif kind == 3:
            s[32 + int(rng.integers(0, 31))] ^= 1 << int(rng.integers(0, 8))  # S bit flip
        recs.append((bytes(m), bytes(s), pub.raw))
        exp.append(ref.fdref_verify(bytes(m), len(m), bytes(s), pub.raw))
    arena, desc, sz = fa.pack_batch(recs)
    out = gpu.verify_batch(arena, sz, desc)
    exp = np.array(exp, dtype=np.int8)
    bad = np.nonzero(out != exp)[0]
    assert len(bad) == 0, [(int(i), int(out[i]), int(exp[i])) for i in bad[:10]]
    assert np.sum(exp == 0) >= n // 4


def test_sha512_batch_kats_and_random(gpu):
    """Batched SHA-512 kernel (fd_sha512_batch replacement) against the
    reference's SHA-512 KATs (fd_sha512_test_vector.c + CAVP, tests/golden)
    and hashlib on random lengths 0..3000 at every byte alignment."""
    import hashlib
    from golden_io import read_sha
    kats = read_sha()
    got = gpu.sha512_batch([m for m, _ in kats])
    for (m, h), g in zip(kats, got):
        assert g == h, (len(m),)
    rng = np.random.default_rng(21)
    msgs = [rng.bytes(int(rng.integers(0, 3001))) for _ in range(4000)]
    msgs += [bytes(n) for n in (0, 1, 111, 112, 119, 120, 127, 128, 129, 239, 240, 255, 256, 257)]
    got = gpu.sha512_batch(msgs)
    for m, g in zip(msgs, got):
        assert g == hashlib.sha512(m).digest(), (len(m),)


def test_sha256_batch_kats_and_random(gpu):
    """Batched SHA-256 kernel (fd_sha256_hash / fd_sha256_batch replacement,
    the shred Merkle path's hash) against the reference's SHA-256 KATs
    (fd_sha256_test_vector.c + CAVP, tests/golden/sha256_kat.bin) and hashlib
    on random lengths 0..3000 at arbitrary byte alignments, and the lengths
    around the padding boundary."""
    import hashlib
    from golden_io import read_sha
    kats = read_sha("sha256_kat.bin")
    assert len(kats) == 77
    got = gpu.sha256_batch([m for m, _ in kats])
    for (m, h), g in zip(kats, got):
        assert g == h, (len(m),)
    rng = np.random.default_rng(22)
    msgs = [rng.bytes(int(rng.integers(0, 3001))) for _ in range(4000)]
    msgs += [bytes(n) for n in (0, 1, 54, 55, 56, 57, 63, 64, 65, 118, 119, 120, 127, 128, 129)]
    got = gpu.sha256_batch(msgs)
    for m, g in zip(msgs, got):
        assert g == hashlib.sha256(m).digest(), (len(m),)


def test_pair_and_single_lane_kernels_agree(gpu):
    """Batches of at most one 256-signature workgroup per CU take the pair
    kernel (two lanes per signature for the decodes), larger ones the
    single-lane kernel; FD_ED25519_GPU_PAIR=0 forces the latter.  Both give
    the golden codes, and a batch one workgroup past the pair limit (single-lane
    kernel) matches the same records at pair size."""
    import os
    recs = _all_golden()
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    exp = np.array([r["code"] for r in recs], dtype=np.int8)
    os.environ["FD_ED25519_GPU_PAIR"] = "0"
    try:
        single = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 17)
    finally:
        del os.environ["FD_ED25519_GPU_PAIR"]
    try:
        # the single-lane kernel takes its descriptors in SHA-block-count order
        # (fd_len_sort_kernel, list form): the golden records span 0..~1.2K-byte
        # messages, so every bucket and both code flavours go through that path
        assert np.array_equal(single.verify_batch(arena, sz, desc), exp)
        single.set_codes(fa.CODES_REF)
        exp_ref = np.array([r["code_ref"] for r in recs], dtype=np.int8)
        assert np.array_equal(single.verify_batch(arena, sz, desc), exp_ref)
        # and twice over in a different order (codes land at the descriptor's index)
        perm = np.random.default_rng(3).permutation(np.concatenate([np.arange(len(desc)), np.arange(len(desc))]))
        single.set_codes(fa.CODES_AVX512)
        assert np.array_equal(single.verify_batch(arena, sz, desc[perm].copy()), exp[perm])
    finally:
        single.close()
    assert np.array_equal(gpu.verify_batch(arena, sz, desc), exp)
    # 256 x CUs signatures (pair kernel) vs 256 x CUs + 256 (single-lane kernel)
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n_pair = 256 * cus
    recs2, kinds = _corrupted_batch(n_pair + 256, 21)
    a2, d2, s2 = fa.pack_batch(recs2)
    g2 = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 17)   # one launch for the whole batch
    try:
        big = g2.verify_batch(a2, s2, d2)
        small = g2.verify_batch(a2, s2, d2[:n_pair])
    finally:
        g2.close()
    assert np.array_equal(big[:n_pair], small)
    assert np.all(big[kinds == 0] == 0) and np.all(big[kinds == 2] == -1)
