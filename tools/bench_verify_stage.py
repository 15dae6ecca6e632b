#!/usr/bin/env python3
"""bench_verify_stage.py -- §8(f) next-1/next-2: the verify tile's whole
per-frag logic on the GPU (fd_ed25519_gpu_verify_frags: frag -> descriptor
extraction, one batch verify, in-order tcache replay), one JSON line.

Workload: --frags frags (default 65,536) of synthetic signed Solana legacy
transactions (tools/synth.py, fresh keys), signature counts drawn from
{1 x5, 2 x2, 3, 4} (mean 1.8), --dup fraction of frags repeating an earlier
one (HA duplicates), laid out [payload][pad][fd_txn_t][u16 sz] in 64-byte
chunks like the dcache.  value = frags/s over the whole call from host
memory (includes the arena / descriptor copies to HBM and the host-side
parse and replay).  CPU baseline: the reference tile sequence
(fdref_verify_frags_seq: reference tcache + fd_ed25519_verify_batch_single_msg,
AVX-512 build) on ONE core -- the reference verify tile is single-threaded
(fd_verify.c) -- over a bounded sample."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def make_stream(n_frags, dup, seed=5):
    import synth
    rng = np.random.default_rng(seed)
    n_unique = int(n_frags * (1.0 - dup))
    cnts = [int(c) for c in rng.choice([1, 1, 1, 1, 1, 2, 2, 3, 4], size=n_unique)]
    txns = synth.build_txns(rng, n_unique, cnts, threads=16)
    order = list(range(n_unique))
    for _ in range(n_frags - n_unique):
        j = int(rng.integers(0, len(order)))
        order.insert(j + int(rng.integers(1, 8)), order[j])
    order = order[:n_frags]
    arena, frags = synth.pack_frags([txns[i] for i in order])
    return arena, frags, sum(cnts[i] for i in order)


def batch_schedule(total, batch, head=(), tail=()):
    """Batch sizes for a run of `total` frags from an idle stage: the `head`
    sizes first (a ramp: the first launch starts after a short copy and the
    link streams the next batches while the pipe fills), full `batch`es, then
    the `tail` sizes (fractions of `batch`: short last batches make the drain
    launches, which run one or two phases alone, short).  Sizes that do not
    fit are dropped from the tail first, then the head."""
    head = [int(h) for h in head if h > 0]
    tail = [max(1, int(batch * f)) for f in tail]
    while tail and sum(head) + sum(tail) > total:
        tail.pop(0)
    while head and sum(head) > total:
        head.pop()
    mid = total - sum(head) - sum(tail)
    sizes = head + [batch] * (mid // batch) + ([mid % batch] if mid % batch else []) + tail
    assert sum(sizes) == total and all(0 < z <= batch for z in sizes), (sizes, total, batch)
    return sizes


def stream_passes(ast, arena, fr, res, sig, passes, batch, head=(), tail=()):
    """`passes` passes over the frags fr as ONE stream into the async stage
    ast, like a tile that never stops: batches of `batch` frags cut
    continuously, so a batch may run from the end of one pass into the start
    of the next (a tile's batch boundaries fall anywhere in its stream; cut
    per pass, every pass would end in a remainder batch).  A batch that wraps
    goes in as its own copy of the frag records, and its results are put back
    in place when its poll returns.  Returns the seconds the stream took."""
    import firedancer_amd as fa
    n = len(fr)
    total, k = passes * n, 0
    sizes = batch_schedule(total, batch, head, tail)
    fifo = []
    t = time.perf_counter()
    while k < total or ast.pending():
        if k < total and ast.pending() < fa.STAGE_DEPTH:
            i, m = k % n, sizes.pop(0)
            if i + m <= n:
                ast.submit(arena, len(arena), fr[i:i + m], res[i:i + m], sig[i:i + m])
                fifo.append(None)
            else:
                n1 = n - i
                fb = np.ascontiguousarray(np.concatenate([fr[i:], fr[:m - n1]]))
                tr, ts = np.zeros(m, np.int8), np.zeros(m, np.uint64)
                ast.submit(arena, len(arena), fb, tr, ts)
                fifo.append((fb, tr, ts, i, n1))
            k += m
        else:
            ast.poll(True)
            w = fifo.pop(0)
            if w:
                fb, tr, ts, i, n1 = w
                res[i:], sig[i:] = tr[:n1], ts[:n1]
                res[:len(tr) - n1], sig[:len(tr) - n1] = tr[n1:], ts[n1:]
    return time.perf_counter() - t


def cpu_baseline(arena, frags, budget_s=10.0):
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp, ul = ctypes.c_void_p, ctypes.c_ulong
    lib.fdref_verify_frags_seq.argtypes = [vp, vp, ul, ul, ul, vp, vp]
    m = min(len(frags), 8192)
    fr = np.ascontiguousarray(np.stack([frags["off"][:m], frags["sz"][:m]], 1).astype(np.uint32))
    res = np.zeros(m, np.int8); tag = np.zeros(m, np.uint64)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    t0 = time.perf_counter(); done = 0
    while time.perf_counter() - t0 < budget_s:
        lib.fdref_verify_frags_seq(p(arena), p(fr), m, 16, 64, p(res), p(tag))
        done += m
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "frags/s", "cores": 1, "kind": "reference",
            "sample": "%d passes over the first %d frags (%.1f s): reference tcache + "
                      "fd_ed25519_verify_batch_single_msg (AVX-512 build), one thread like the tile" % (done // m, m, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=65536)
    ap.add_argument("--dup", type=float, default=0.1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    # 36,000 frags: 64.0K signatures at this stream's 1.78 per frag (+-195, 7.9 sigma under the
    # 65,536 one launch verifies in one wave per SIMD); profiles/r05/stage/ab_batch_size_stream.log
    ap.add_argument("--async-batch", type=int, default=36000)
    args = ap.parse_args()
    import firedancer_amd as fa

    t0 = time.perf_counter()
    arena, frags, n_sigs = make_stream(args.frags, args.dup)
    gen_s = time.perf_counter() - t0
    g = fa.Ed25519Gpu(device_mask=1, max_batch=1 << 18)
    stage = fa.VerifyStage(gpu=g, tcache=fa.TCache())
    for _ in range(args.warmup):
        stage.tcache.reset()
        res, _ = stage.verify_frags(arena, len(arena), frags)
    hist = {int(k): int(v) for k, v in zip(*np.unique(res, return_counts=True))}
    t_parse = time.perf_counter()
    for _ in range(3):
        fa.frags_to_descs(arena, len(arena), frags)
    parse_ms = (time.perf_counter() - t_parse) / 3 * 1e3
    times = []
    for _ in range(args.steps):
        stage.tcache.reset()
        t1 = time.perf_counter()
        stage.verify_frags(arena, len(arena), frags)
        times.append(time.perf_counter() - t1)
    dt = float(np.mean(times))
    # the asynchronous stage with the frags parsed on the GPU: --async-batch
    # frags per batch, QUEUE_DEPTH batches in flight (the pipelined kernel: one
    # phase of each per launch), over the same stream; and the same with the
    # one-shot kernels (FD_ED25519_GPU_ASYNC_PIPE=0) for the A/B
    ab = args.async_batch
    fr = np.ascontiguousarray(frags)

    def measure(pipe):
        """(frags/s, results, launches, breakdown) of the async stage: with the
        frag area page-locked by the caller (fd_ed25519_gpu_host_register, as a
        tile registers its dcache once), then left pageable"""
        os.environ["FD_ED25519_GPU_ASYNC_PIPE"] = "1" if pipe else "0"
        out = {}
        for mode in ("registered", "pageable"):
            big = fa.Ed25519Gpu(device_mask=1, max_batch=16 * ab)
            if mode == "registered":
                big.host_register(arena)
            ast = fa.AsyncStage(big, fa.TCache(), ab, threads=8, device_parse=True)
            res_a = np.zeros(len(frags), np.int8); sig_a = np.zeros(len(frags), np.uint64)
            calls = {"submit_s": 0.0, "poll_s": 0.0}

            def run_async():
                ast.tcache.reset()
                i = 0
                while i < len(fr) or ast.pending():
                    if i < len(fr) and ast.pending() < fa.STAGE_DEPTH:
                        j = min(len(fr), i + ab)
                        t = time.perf_counter()
                        ast.submit(arena, len(arena), fr[i:j], res_a[i:j], sig_a[i:j])
                        calls["submit_s"] += time.perf_counter() - t
                        i = j
                    else:
                        t = time.perf_counter()
                        ast.poll(True)
                        calls["poll_s"] += time.perf_counter() - t

            def run_stream(reps):
                """reps passes over the frags as ONE stream (no drain between
                passes, like a tile that never stops; batches cut across pass
                boundaries): the 16-deep tcache has forgotten a pass's frags
                long before they come again"""
                ast.tcache.reset()
                stream_passes(ast, arena, fr, res_a, sig_a, reps, ab)

            run_async()                       # first use: registration, buffers
            ast.stats(reset=True); big.host_stats(reset=True)
            calls["submit_s"] = calls["poll_s"] = 0.0
            t = []
            for _ in range(args.steps):
                t1 = time.perf_counter(); run_async(); t.append(time.perf_counter() - t1)
            dt_m = float(np.mean(t))
            st, hs = ast.stats(), big.host_stats()
            per = lambda ns: ns / args.steps / 1e6          # ms per run
            out[mode] = {
                "frags_per_s": args.frags / dt_m, "sigs_per_s": n_sigs / dt_m, "ms": dt_m * 1e3,
                "runs": len(t), "sigs_per_s_median": n_sigs / float(np.median(t)),
                "sigs_per_s_min_max": [n_sigs / max(t), n_sigs / min(t)],
                "caller_ms_per_run": {"submit": calls["submit_s"] / args.steps * 1e3,
                                      "poll_wait": calls["poll_s"] / args.steps * 1e3},
                "stage_ms_per_run": {k[:-3]: per(v) for k, v in st.items() if k.endswith("_ns")},
                "submit_path_ms_per_run": {k[:-3]: per(v) for k, v in hs.items() if k.endswith("_ns")},
                "h2d_gb_per_run": hs["h2d_bytes"] / args.steps / 1e9,
                "batches_per_run": st["batches"] / args.steps,
            }
            if mode == "registered":
                res_reg = res_a.copy()
                launches = big.launch_stats()
                t1 = time.perf_counter(); run_stream(args.steps); dt_s = time.perf_counter() - t1
                diff = int(np.count_nonzero(res_a != res_reg))
                assert diff <= 16, diff       # only a pass's first frags can meet the previous pass's last 16 tags
                out["streaming"] = {"frags_per_s": args.steps * args.frags / dt_s,
                                    "sigs_per_s": args.steps * n_sigs / dt_s, "ms_per_pass": dt_s / args.steps * 1e3,
                                    "passes": args.steps, "results_differing_from_single_pass": diff}
            else:
                assert np.array_equal(res_a, res_reg)
            ast.close()
            if mode == "registered":
                big.host_unregister(arena)
            big.close()
        os.environ.pop("FD_ED25519_GPU_ASYNC_PIPE", None)
        return out, res_reg, launches
    pipe_m, res_a, launches = measure(True)
    one_m, res_o, launches_o = measure(False)
    assert np.array_equal(res_a, res_o)
    line = {"metric": "verify-stage frags/sec (fd_ed25519_gpu_verify_frags, host frags)",
            "value": args.frags / dt, "unit": "frags/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt * 1e3, "higher_is_better": True, "dtype": "u32 limbs / u8 bytes",
            "data": "synthetic signed legacy txns (tools/synth.py), %.0f%% duplicates" % (100 * args.dup),
            "config": {"workload": "%d frags, %d signatures, tcache depth 16 / map 64" % (args.frags, n_sigs),
                       "arena_bytes": int(len(arena))},
            "sigs_per_s": n_sigs / dt, "host_parse_ms": parse_ms, "results": hist, "gen_s": gen_s,
            "async_device_parse": {"batch": ab, "in_flight": fa.QUEUE_DEPTH, "stage_depth": fa.STAGE_DEPTH, "kernel": "pipelined",
                                   "launches_pipe_oneshot": launches, **pipe_m,
                                   "results": {int(k): int(v) for k, v in zip(*np.unique(res_a, return_counts=True))},
                                   "note": "registered: the caller page-locked the frag area "
                                           "(fd_ed25519_gpu_host_register); pageable: not.  stage_ms_per_run: the "
                                           "caller's submit / poll and the completion worker's GPU polls, back-off "
                                           "waits and tcache replays; submit_path_ms_per_run: inside the GPU submits; "
                                           "streaming: --steps passes over the frags as one stream, no pipeline "
                                           "fill / drain between passes (registered)"},
            "async_device_parse_oneshot": {**one_m, "launches_pipe_oneshot": launches_o,
                                           "note": "FD_ED25519_GPU_ASYNC_PIPE=0: the same stage on the one-shot kernels"},
            "cpu_baseline": None if args.no_cpu else cpu_baseline(arena, frags)}
    print(json.dumps(line), flush=True)
    stage.close()


if __name__ == "__main__":
    main()
