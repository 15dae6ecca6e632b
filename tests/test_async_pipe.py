"""GPU: the pipelined kernel behind the host-memory async pair
(fd_ed25519_gpu_submit / _poll, three batches in flight), the comb table
shared per device, and the pipe's failure paths (all-or-nothing scratch,
the key cache refusing changes while pipelined batches are in flight, the
phase-A wait's error word).  Bar: every batch's codes bit-exact with the
reference's (golden records), whatever the submit / poll interleaving."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import firedancer_amd as fa
from golden_io import read_sigs

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _golden():
    return read_sigs("vectors_ref.bin") + read_sigs("synthetic.bin")


def _host(recs):
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    return arena, desc, sz, np.full(len(desc), 99, np.int8), np.array([r["code"] for r in recs], np.int8)


def _sets():
    recs = _golden()
    rng = np.random.default_rng(31)
    return [recs, recs[::-1][:2000], recs[7:8], [recs[i] for i in rng.permutation(len(recs))[:3000]],
            recs[-900:], recs[100:1500], [recs[i] for i in rng.permutation(len(recs))]]


def test_async_queue_depth_in_flight(gpu):
    """Submit until BUSY (QUEUE_DEPTH in flight), complete the oldest, submit again:
    batches of different sizes and contents, all pipelined."""
    batches = [_host(s) for s in _sets()]
    p0, o0 = gpu.launch_stats()
    done, nxt = 0, 0
    while done < len(batches):
        while nxt < len(batches):
            a, d, sz, out, _ = batches[nxt]
            try:
                gpu.submit(a, sz, d, out)
            except fa.GpuError as e:
                assert "-104" in str(e)          # FD_ED25519_GPU_ERR_BUSY
                assert gpu.pending() == fa.QUEUE_DEPTH
                break
            nxt += 1
        assert gpu.poll(block=True)
        done += 1
    assert gpu.pending() == 0
    for a, d, sz, out, want in batches:
        assert np.array_equal(out, want)
    p1, o1 = gpu.launch_stats()
    assert o1 == o0                               # no one-shot launch
    assert len(batches) <= p1 - p0 <= len(batches) + 2   # one launch per batch + the final drains


def test_async_lone_batch_nonblocking_poll(gpu):
    """One batch and only non-blocking polls: it is drained once the GPU is idle."""
    a, d, sz, out, want = _host(_golden()[:777])
    gpu.submit(a, sz, d, out)
    for _ in range(200000):
        if gpu.poll():
            break
    else:
        pytest.fail("lone batch never completed")
    assert np.array_equal(out, want)


def test_async_oversize_batch_takes_one_shot_between_pipelined(gpu):
    """A batch above one wave per SIMD goes to the one-shot kernel; older
    pipelined batches still complete first and correctly."""
    from test_gpu_parity import _corrupted_batch
    small = [_host(s) for s in _sets()[:2]]
    recs, kinds = _corrupted_batch(65536, 5)
    recs = recs[:60000]                           # fits max_batch (64K); above 256 x CUs only if CUs < 235
    arena, desc, sz = fa.pack_batch(recs)
    big_out = np.full(len(desc), 99, np.int8)
    a, d, s_, out, want = small[0]
    gpu.submit(a, s_, d, out)
    gpu.submit(arena, sz, desc, big_out)
    a2, d2, s2, out2, want2 = small[1]
    gpu.submit(a2, s2, d2, out2)
    for _ in range(3):
        assert gpu.poll(block=True)
    assert np.array_equal(out, want) and np.array_equal(out2, want2)
    k = kinds[:60000]
    assert np.all(big_out[k == 0] == 0) and np.all(big_out[k == 1] == -3) and np.all(big_out[k == 2] == -1)


def test_sync_verify_refused_while_async_pending(gpu):
    a, d, sz, out, want = _host(_golden()[:50])
    gpu.submit(a, sz, d, out)
    with pytest.raises(fa.GpuError):
        gpu.verify_batch(a, sz, d)
    assert gpu.poll(block=True)
    assert np.array_equal(out, want)
    assert np.array_equal(gpu.verify_batch(a, sz, d), want)


def test_async_three_slots_one_gpu():
    """devices=[0,0,0]: every submit shards over three slots, each with its
    own pipe; three batches in flight."""
    g = fa.Ed25519Gpu(devices=[0, 0, 0], max_batch=1 << 14)
    try:
        batches = [_host(s) for s in _sets()[:5]]
        for b in batches[:3]:
            g.submit(b[0], b[2], b[1], b[3])
        for b in batches[3:]:
            assert g.poll(block=True)
            g.submit(b[0], b[2], b[1], b[3])
        while g.pending():
            assert g.poll(block=True)
        for a, d, sz, out, want in batches:
            assert np.array_equal(out, want)
        assert g.launch_stats()[1] == 0
    finally:
        g.close()


def test_comb_table_shared_per_device(gpu):
    """Two more contexts and a three-slot context on device 0 share the one
    5.9 GB comb table the session's context built: no new table, no 5.9 GB
    allocations, codes unchanged."""
    live0, refs0, builds0 = fa.ctab_stats(0)
    assert live0 == 1 and refs0 >= 1
    free0 = torch.cuda.mem_get_info(0)[0]
    g1 = fa.Ed25519Gpu(device_mask=1, max_batch=4096)
    g2 = fa.Ed25519Gpu(device_mask=1, max_batch=4096)
    g3 = fa.Ed25519Gpu(devices=[0, 0, 0], max_batch=4096)
    try:
        live, refs, builds = fa.ctab_stats(0)
        assert (live, refs, builds) == (1, refs0 + 5, builds0)
        used = free0 - torch.cuda.mem_get_info(0)[0]
        assert used < 3 * (1 << 30), used           # five slots' scratch, not 5 x 5.9 GB
        recs = _golden()[:1500]
        a, d, sz, out, want = _host(recs)
        for g in (g1, g2, g3):
            assert np.array_equal(g.verify_batch(a, sz, d), want)
    finally:
        g1.close(); g2.close(); g3.close()
    assert fa.ctab_stats(0)[:2] == (1, refs0)


def test_keycache_busy_while_pipelined_batches_in_flight(gpu):
    """keycache_add between pipe_dev calls would strand the
    in-flight batches; it is refused until they are drained."""
    recs = _golden()[:600]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    d_arena = torch.from_numpy(arena.copy()).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    out = torch.full((len(recs),), 99, dtype=torch.int8, device="cuda:0")
    st = torch.cuda.current_stream()
    gpu.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), len(recs), out.data_ptr(), stream=st.cuda_stream)
    r = gpu.lib.fd_ed25519_gpu_keycache_reserve(gpu.ctx, 16)
    assert r == -104                                # FD_ED25519_GPU_ERR_BUSY
    gpu.pipe_flush_dev(stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), np.array([x["code"] for x in recs], np.int8))
    gpu.keycache_reserve(16)
    try:
        assert gpu.keycache_add([recs[0]["pub"]]) == 1
        # a drain step is allowed with keys cached (phases B / C never read the key tables)
        gpu.pipe_flush_dev(stream=st.cuda_stream)
    finally:
        gpu.keycache_clear()


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, %(repo)r); sys.path.insert(0, %(tests)r)
import firedancer_amd as fa
from golden_io import read_sigs
recs = read_sigs("synthetic.bin")[:700]
arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
want = np.array([r["code"] for r in recs], np.int8)
g = fa.Ed25519Gpu(device_mask=1, max_batch=4096)
out = np.zeros(len(desc), np.int8)
try:
    g.submit(arena, sz, desc, out)
    print("FIRST_OK")
except fa.GpuError as e:
    print("FIRST_ERR", e)
out2 = np.zeros(len(desc), np.int8)
g.submit(arena, sz, desc, out2)
while g.pending():
    assert g.poll(block=True)
assert np.array_equal(out2, want)
print("SECOND_OK")
g.close()
"""


def test_pipe_scratch_all_or_nothing():
    """a failed allocation inside the pipe scratch leaves no
    half-made set behind: the batch is refused with ERR_OOM, the next one
    allocates the whole set and verifies correctly."""
    env = dict(os.environ, FD_ED25519_GPU_TEST_FAIL_ALLOC="2")
    p = subprocess.run([sys.executable, "-c", _CHILD % {"repo": REPO, "tests": os.path.join(REPO, "tests")}],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "FIRST_ERR" in p.stdout and "-101" in p.stdout, p.stdout   # FD_ED25519_GPU_ERR_OOM
    assert "SECOND_OK" in p.stdout


def test_lsort_wait_expiry_is_reported():
    """A diagnostic build whose phase-A length-order waits expire at once
    (tools/bin/lib_xlsort.so, -DFD_DIAG_LSORT_TIMEOUT): the pipelined batch
    that hit it is reported (pipe_status / its poll: FD_ED25519_GPU_ERR_LAUNCH)
    instead of returning codes from a partial order -- and ONLY that batch
    (the error word used to fail every later call on the slot):
    pipe_status clears, the one-shot kernels and later launches go on."""
    import ctypes
    path = os.path.join(REPO, "tools", "bin", "lib_xlsort.so")
    assert os.path.exists(path), "build tools/ (make -C tools) first"
    lib = ctypes.CDLL(path)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    lib.fd_ed25519_gpu_new.restype = vp
    lib.fd_ed25519_gpu_new.argtypes = [u64, u64]
    lib.fd_ed25519_gpu_pipe_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_pipe_flush_dev.argtypes = [vp, i32, vp]
    lib.fd_ed25519_gpu_pipe_status.argtypes = [vp, i32]
    lib.fd_ed25519_gpu_delete.argtypes = [vp]
    lib.fd_ed25519_verify_batch_gpu.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.fd_ed25519_gpu_submit.argtypes = [vp, vp, u64, vp, u64, vp]
    lib.fd_ed25519_gpu_poll_block.argtypes = [vp]
    recs = _golden()[:4096]                            # 16 full workgroups
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    want = np.array([r["code"] for r in recs], np.int8)
    d_arena = torch.from_numpy(arena.copy()).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    out = torch.zeros(len(recs), dtype=torch.int8, device="cuda:0")
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    c = lib.fd_ed25519_gpu_new(1, 4096)
    assert c
    try:
        st = torch.cuda.current_stream().cuda_stream
        assert lib.fd_ed25519_gpu_pipe_dev(c, 0, d_arena.data_ptr(), sz, d_desc.data_ptr(), len(recs),
                                           out.data_ptr(), st) == 0
        lib.fd_ed25519_gpu_pipe_flush_dev(c, 0, st)
        torch.cuda.synchronize()
        assert lib.fd_ed25519_gpu_pipe_status(c, 0) == -102          # FD_ED25519_GPU_ERR_LAUNCH
        assert lib.fd_ed25519_gpu_pipe_status(c, 0) == 0             # reported once, then cleared
        # the one-shot kernels are unaffected by the pipe's failure
        o1 = np.zeros(len(recs), np.int8)
        assert lib.fd_ed25519_verify_batch_gpu(c, p(arena), sz, p(desc), len(recs), p(o1)) == 0
        assert np.array_equal(o1, want)
        # an async pipelined batch that hits it fails alone; the next one-shot call still verifies
        o2 = np.zeros(len(recs), np.int8)
        assert lib.fd_ed25519_gpu_submit(c, p(arena), sz, p(desc), len(recs), p(o2)) == 0
        assert lib.fd_ed25519_gpu_poll_block(c) == -102
        o3 = np.zeros(len(recs), np.int8)
        assert lib.fd_ed25519_verify_batch_gpu(c, p(arena), sz, p(desc), len(recs), p(o3)) == 0
        assert np.array_equal(o3, want)
    finally:
        torch.cuda.synchronize()
        lib.fd_ed25519_gpu_delete(c)


def test_dev_and_async_pipe_calls_exclude_each_other(gpu):
    """the _dev pipe entry and the async queues share the slot's
    pipe state.  While a _dev batch sits between its phases, submit says BUSY
    (its phase C would run with no copy-out on the queue's stream); while
    async batches are pending, pipe_dev / pipe_flush_dev say BUSY.  Codes of
    both kinds stay exact when they alternate."""
    recs = _golden()[:1200]
    a, d, sz, _, want = _host(recs)
    d_arena = torch.from_numpy(a.copy()).cuda()
    d_desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out_dev = torch.full((len(recs),), 99, dtype=torch.int8, device="cuda:0")
    st = torch.cuda.current_stream()
    for rep in range(2):
        gpu.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), len(recs), out_dev.data_ptr(), stream=st.cuda_stream)
        out = np.full(len(recs), 99, np.int8)
        with pytest.raises(fa.GpuError, match="-104"):
            gpu.submit(a, sz, d, out)                       # a _dev batch holds the pipe
        gpu.pipe_flush_dev(stream=st.cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out_dev.cpu().numpy(), want)
        gpu.submit(a, sz, d, out)
        with pytest.raises(fa.GpuError, match="-104"):
            gpu.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), len(recs), out_dev.data_ptr(),
                         stream=st.cuda_stream)
        with pytest.raises(fa.GpuError, match="-104"):
            gpu.pipe_flush_dev(stream=st.cuda_stream)
        assert gpu.poll(block=True)
        assert np.array_equal(out, want)
        # the synchronous one-shot call is not a pipe user
        assert np.array_equal(gpu.verify_batch(a, sz, d), want)
