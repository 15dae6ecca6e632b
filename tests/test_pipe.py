"""GPU: the pipelined entry point fd_ed25519_gpu_pipe_dev (one launch = the
first phase of batch i beside the second phase of batch i-1).  Bar: every
batch's codes bit-exact with the reference's (golden records, both code
flavours), whatever the sizes of consecutive batches, with ordinary launches
interleaved, and at config-2 size."""
import numpy as np
import pytest
import torch

import firedancer_amd as fa
from golden_io import read_sigs, read_txns

pytestmark = pytest.mark.gpu


def _dev(recs):
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    return (torch.from_numpy(arena.copy()).to("cuda:0"), torch.from_numpy(desc.view(np.uint8).copy()).to("cuda:0"),
            sz, len(desc), torch.full((len(desc),), 99, dtype=torch.int8, device="cuda:0"))


def _golden():
    return read_sigs("vectors_ref.bin") + read_sigs("synthetic.bin")


def _run_pipe(g, batches, stream):
    for d_arena, d_desc, sz, n, d_out in batches:
        g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=stream.cuda_stream)
    g.pipe_flush_dev(stream=stream.cuda_stream)
    torch.cuda.synchronize()


@pytest.mark.parametrize("flavour,key", [(fa.CODES_AVX512, "code"), (fa.CODES_REF, "code_ref")])
def test_pipe_golden_sequence(gpu, flavour, key):
    recs = _golden()
    rng = np.random.default_rng(12)
    # batches of different sizes and contents, consecutive ones both larger and smaller
    sets = [recs, recs[:1000][::-1], recs[5:6], [recs[i] for i in rng.permutation(len(recs))[:3000]], recs[-700:]]
    batches = [_dev(s) for s in sets]
    st = torch.cuda.Stream()
    gpu.set_codes(flavour)
    try:
        _run_pipe(gpu, batches, st)
    finally:
        gpu.set_codes(fa.CODES_AVX512)
    for s, b in zip(sets, batches):
        assert np.array_equal(b[4].cpu().numpy(), np.array([r[key] for r in s], np.int8))


def test_pipe_with_ordinary_launches_between(gpu):
    recs = _golden()
    a, b, c = _dev(recs), _dev(recs[::-1]), _dev(recs[100:900])
    st = torch.cuda.current_stream()
    gpu.pipe_dev(a[0].data_ptr(), a[2], a[1].data_ptr(), a[3], a[4].data_ptr(), stream=st.cuda_stream)
    # an ordinary launch between pipe calls uses its own scratch
    gpu.verify_batch_dev(c[0].data_ptr(), c[2], c[1].data_ptr(), c[3], c[4].data_ptr(), stream=st.cuda_stream)
    gpu.pipe_dev(b[0].data_ptr(), b[2], b[1].data_ptr(), b[3], b[4].data_ptr(), stream=st.cuda_stream)
    gpu.pipe_flush_dev(stream=st.cuda_stream)
    torch.cuda.synchronize()
    for s, x in ((recs, a), (recs[::-1], b), (recs[100:900], c)):
        assert np.array_equal(x[4].cpu().numpy(), np.array([r["code"] for r in s], np.int8))


def test_pipe_txn_batches(gpu):
    txns = [t for t in read_txns() if 1 <= t["n"] <= 16] + read_txns("cctv_batches.bin")
    recs = []
    for ti, t in enumerate(txns):
        for j in range(t["n"]):
            recs.append((t["msg"], t["sigs"][j], t["pubs"][j], ti & 0xffff))
    arena, desc, sz = fa.pack_batch(recs)
    d = (torch.from_numpy(arena.copy()).cuda(), torch.from_numpy(desc.view(np.uint8).copy()).cuda(), sz, len(desc),
         torch.zeros(len(desc), dtype=torch.int8, device="cuda:0"))
    _run_pipe(gpu, [d], torch.cuda.Stream())
    codes = d[4].cpu().numpy()
    assert np.array_equal(fa.txn_reduce(codes, desc), np.array([t["code"] for t in txns], np.int8))


def test_pipe_config2_size_repeated(gpu, oracle):
    """64K descriptors with known corruptions, three batches in a row through
    the pipe (each batch's second phase runs beside the next one's first)."""
    from test_gpu_parity import _corrupted_batch
    n = 65536
    recs, kinds = _corrupted_batch(n, 23)
    arena, desc, sz = fa.pack_batch(recs)
    d_arena = torch.from_numpy(arena.copy()).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    outs = [torch.full((n,), 99, dtype=torch.int8, device="cuda:0") for _ in range(3)]
    st = torch.cuda.Stream()
    for o in outs:
        gpu.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, o.data_ptr(), stream=st.cuda_stream)
    gpu.pipe_flush_dev(stream=st.cuda_stream)
    torch.cuda.synchronize()
    ref = outs[0].cpu().numpy()
    assert np.all(ref[kinds == 0] == 0) and np.all(ref[kinds == 1] == -3) and np.all(ref[kinds == 2] == -1)
    assert np.all(ref[kinds == 3] == -3)
    for o in outs[1:]:
        assert np.array_equal(o.cpu().numpy(), ref)
    for i in np.random.default_rng(4).choice(n, 256, replace=False):
        m, s, p = recs[i]
        assert ref[i] == oracle.fdo_verify(m, len(m), s, p, 0)


def test_pipe_refuses_oversize_and_hot_keys(gpu):
    recs = _golden()[:10]
    a = _dev(recs)
    with pytest.raises(fa.GpuError):
        gpu.pipe_dev(a[0].data_ptr(), a[2], a[1].data_ptr(), (1 << 16) + 512, a[4].data_ptr())
    gpu.keycache_reserve(4)
    try:
        gpu.keycache_add([recs[0]["pub"]])
        with pytest.raises(fa.GpuError):
            gpu.pipe_dev(a[0].data_ptr(), a[2], a[1].data_ptr(), a[3], a[4].data_ptr())
    finally:
        gpu.keycache_clear()


@pytest.mark.parametrize("flavour,key", [(fa.CODES_AVX512, "code"), (fa.CODES_REF, "code_ref")])
def test_pipe_big_batches_kpre(flavour, key):
    """Batches above one wave per SIMD through pipe_dev (config 3's form):
    k = SHA-512(R||A||M) mod l for the whole batch in message-length order
    (fd_ed25519_kpre_kernel), then 64K chunks whose phase A reads k; every
    golden record (variable-length messages 0..1232 B, adversarial classes)
    tiled to 140K in random order, then 70K, then 5 -- codes bit-exact with
    the reference's across the calls and the flush."""
    recs = _golden()
    rng = np.random.default_rng(77)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=160000)
    try:
        sets = [[recs[i % len(recs)] for i in rng.permutation(140000)],
                [recs[i % len(recs)] for i in rng.permutation(70000)], recs[7:12]]
        batches = [_dev(s) for s in sets]
        st = torch.cuda.Stream()
        g.set_codes(flavour)
        _run_pipe(g, batches, st)
    finally:
        g.close()
    for s, b in zip(sets, batches):
        assert np.array_equal(b[4].cpu().numpy(), np.array([r[key] for r in s], np.int8))
