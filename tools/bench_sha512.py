#!/usr/bin/env python3
"""bench_sha512.py -- §8(f) next-3: the standalone batched SHA-512 kernel
(fd_sha512_batch_gpu_dev) on device-resident messages, one JSON line.

Workload: --n messages (default 1,048,576) of --msg-sz bytes (default 200,
the config-2 message size; 1232 = the txn MTU), random bytes, packed back to
back (unaligned).  value = messages/s; also GB/s of message bytes and the
kernel's average launch time (HIP events on the launch stream).  CPU
baseline: the reference fd_sha512_hash (oracle/_ref, AVX2 core) on one pinned
thread per physical host core over a bounded sample."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def cpu_baseline(arena, msg, out_len, budget_s=5.0):
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so")
    if not os.path.exists(path):
        return None
    from firedancer_amd.hostcpu import baseline_cpus
    cpus, topo = baseline_cpus()
    threads = min(len(cpus), 256)
    cpu_arr = (ctypes.c_int * threads)(*cpus[:threads])
    lib = ctypes.CDLL(path)
    lib.fdref_sha512_msgs_pinned.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                             ctypes.c_ulong, ctypes.c_ulong, ctypes.c_void_p]
    m = min(len(msg), 65536)
    d = np.ascontiguousarray(msg[:m])
    out = np.zeros(64 * m, np.uint8)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.fdref_sha512_msgs_pinned(vp(arena), vp(d), m, vp(out), threads, 1, cpu_arr)
    t0 = time.perf_counter(); done = 0
    while time.perf_counter() - t0 < budget_s:
        lib.fdref_sha512_msgs_pinned(vp(arena), vp(d), m, vp(out), threads, 1, cpu_arr)
        done += m
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "msgs/s", "cores": threads, "kind": "reference",
            "per_core": done / dt / threads, "topology": topo,
            "sample": "%d passes x %d messages (%.1f s), fd_sha512_hash, %d pthreads pinned one per physical "
                      "core" % (done // m, m, dt, threads)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--msg-sz", type=int, default=200)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import torch
    import hashlib
    import firedancer_amd as fa

    n, sz = args.n, args.msg_sz
    rng = np.random.default_rng(3)
    arena = np.frombuffer(rng.bytes(n * sz + 16), np.uint8).copy()
    msg = np.zeros(n, fa.SHA_MSG_DTYPE)
    msg["off"] = np.arange(n, dtype=np.uint64) * sz
    msg["sz"] = sz
    g = fa.Ed25519Gpu(device_mask=1, max_batch=1024)
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(arena).to(dev)
    d_msg = torch.from_numpy(msg.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(64 * n, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)

    def step():
        g.sha512_batch_dev(d_arena.data_ptr(), n * sz, d_msg.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in np.random.default_rng(5).choice(n, 256, replace=False):
        m = arena[i * sz:(i + 1) * sz].tobytes()
        assert out[64 * i:64 * i + 64].tobytes() == hashlib.sha512(m).digest()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(st); step(); b.record(st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    blocks = (sz + 17 + 127) // 128
    line = {"metric": "SHA-512 messages/sec (batched, device-resident)", "value": n * args.steps / dt,
            "unit": "msgs/s", "n_gpus": 1, "steps": args.steps, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "dtype": "u64 (as u32 pairs)", "data": "synthetic random bytes",
            "config": {"workload": "%d messages x %d B, packed unaligned" % (n, sz), "blocks_per_msg": blocks},
            "kernel_ms": kms, "msg_GB_per_s": n * sz / (kms * 1e-3) / 1e9,
            "blocks_per_s": n * blocks / (kms * 1e-3),
            "cpu_baseline": None if args.no_cpu else cpu_baseline(arena, msg, 64 * n)}
    print(json.dumps(line), flush=True)
    g.close()


if __name__ == "__main__":
    main()
