"""Hot-key cache (fd_ed25519_gpu_keycache_*): signatures whose public key is
cached are verified by a different kernel (comb table of the key, no
doublings); the codes must not change.  Oracles: the committed golden
records (reference AVX-512 and portable codes) with EVERY key cached --
including keys that fail to decode, non-canonical and small-order keys --
and with half of them cached (mixed batches split on the device); fresh
reference-signed signatures (valid and corrupted) over cached keys."""
import ctypes
import os
import sys

import numpy as np
import pytest

import firedancer_amd as fa
from golden_io import read_sigs, read_txns

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import synth  # noqa: E402


@pytest.fixture(scope="module")
def kgpu():
    g = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 16)
    g.keycache_reserve(8192)
    yield g
    g.close()


def _golden():
    return read_sigs("vectors_ref.bin") + read_sigs("synthetic.bin")


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [1.0, 0.5])
def test_golden_codes_with_cached_keys(kgpu, frac):
    recs = _golden()
    keys = sorted(set(r["pub"] for r in recs))
    rng = np.random.default_rng(5)
    cached = [k for k in keys if rng.random() < frac]
    kgpu.keycache_clear()
    assert kgpu.keycache_add(cached) == len(cached)
    assert kgpu.keycache_add(cached[:10]) == 0          # already cached
    assert kgpu.keycache_cnt() == len(cached)
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    for flavour, field in ((fa.CODES_AVX512, "code"), (fa.CODES_REF, "code_ref")):
        kgpu.set_codes(flavour)
        out = kgpu.verify_batch(arena, sz, desc)
        exp = np.array([r[field] for r in recs], np.int8)
        bad = np.nonzero(out != exp)[0]
        assert len(bad) == 0, [(int(i), recs[i]["set"], int(out[i]), int(exp[i])) for i in bad[:10]]
    kgpu.set_codes(fa.CODES_AVX512)


@pytest.mark.gpu
def test_txn_batches_with_cached_keys(kgpu):
    txns = read_txns()
    kgpu.keycache_clear()
    kgpu.keycache_add(sorted(set(p for t in txns for p in t["pubs"])))
    recs = []
    for ti, t in enumerate(txns):
        for j in range(t["n"]):
            recs.append((t["msg"], t["sigs"][j], t["pubs"][j], ti & 0xffff))
    arena, desc, sz = fa.pack_batch(recs)
    out = kgpu.verify_batch(arena, sz, desc)
    got = fa.txn_reduce(out, desc)
    exp = [t["code"] for t in txns if t["n"] > 0]
    assert [int(x) for x in got] == exp


@pytest.mark.gpu
def test_fresh_signatures_hot_keys(kgpu):
    """40,000 signatures by 600 cached signers (and 200 uncached ones), random
    messages 0..1232 B, a quarter corrupted: codes == the reference's."""
    so = os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so")
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built")
    ref = ctypes.CDLL(so)
    ref.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
    rng = np.random.default_rng(12)
    kps = synth.keypairs([rng.bytes(32) for _ in range(800)], threads=16)
    kgpu.keycache_clear()
    assert kgpu.keycache_add([p for _, p in kps[:600]]) == 600
    n = 40000
    items = []
    for i in range(n):
        s_, p_ = kps[int(rng.integers(0, 800))]
        items.append((s_, p_, rng.bytes(int(rng.integers(0, 1233)))))
    sigs = synth.sign_many(items, threads=16)
    recs, exp = [], []
    for i, ((_, p_, m), g) in enumerate(zip(items, sigs)):
        g, m = bytearray(g), bytearray(m)
        kind = i & 3
        if kind == 1 and len(m):
            m[int(rng.integers(0, len(m)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            g[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 3:
            g[32 + int(rng.integers(0, 31))] ^= 1 << int(rng.integers(0, 8))
        recs.append((bytes(m), bytes(g), p_))
        exp.append(ref.fdref_verify(bytes(m), len(m), bytes(g), p_))
    arena, desc, sz = fa.pack_batch(recs)
    out = kgpu.verify_batch(arena, sz, desc)
    exp = np.array(exp, np.int8)
    bad = np.nonzero(out != exp)[0]
    assert len(bad) == 0, [(int(i), int(out[i]), int(exp[i])) for i in bad[:10]]
    assert (exp == 0).sum() > n // 5


@pytest.mark.gpu
def test_all_cached_device_entry_bench_shape():
    """The bench's --hot-keys shape through the device-pointer entry: every
    signer cached, so the miss list is empty and only the split and the
    cached kernel do work (a launch whose split-kernel arguments carried a
    stale device-count pointer faulted here; the host now zeroes them)."""
    import torch
    sys.path.insert(0, REPO)
    import bench
    n = 16384
    arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=3, n_keys=256)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    try:
        keys = sorted(set(bench.desc_pub(arena, desc)))
        g.keycache_reserve(len(keys))
        assert g.keycache_add(keys) == len(keys) == 256
        d_arena = torch.from_numpy(arena).cuda()
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
        d_out = torch.full((n,), 99, dtype=torch.int8, device="cuda")
        st = torch.cuda.Stream()
        for _ in range(3):
            g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(d_out.cpu().numpy(), expect)
    finally:
        g.close()
