"""Can the host feed 8 GPUs?  CPU bench of the submit paths' host work
(fd_ed25519_gpu_test_submit_host: per slot, its shard's copy plan and
rebased records on per-slot threads, exactly the code fd_ed25519_gpu_submit
and the frag path run before their copies; no device).

Workloads (synthetic layouts, contents irrelevant to the host work):
  desc:  config 2 per slot -- 65,536 descriptors of sig | pub | 200-B msg
         records packed back to back (bench.py's layout), nslot x 65,536 in all;
  frags: the verify stage's frags -- 35,000 per slot of 300..1,300 B back to
         back (a dcache-like arena).
copy 0: the plan alone (the DMA engines move the bytes); copy 1: the CPU also
memcpys the runs (what the host memory system would have to sustain if it
did the engines' work).  Prints one JSON line.

  python3 tools/bench_host_feed.py [--slots 1,2,4,8] [--iters 20]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import firedancer_amd as fa  # noqa: E402

DESC = fa.DESC_DTYPE
FRAG = np.dtype([("off", "<u4"), ("sz", "<u4")])


def desc_workload(n, msg_sz=200):
    rec = 96 + msg_sz
    off = np.arange(n, dtype=np.uint64) * rec
    d = np.zeros(n, DESC)
    d["sig_off"] = off
    d["pub_off"] = off + 64
    d["msg_off"] = off + 96
    d["msg_sz"] = msg_sz
    d["txn_idx"] = np.arange(n) & 0xffff
    arena = np.zeros(n * rec + 16, np.uint8)
    return arena, d


def frag_workload(n, rng):
    sz = rng.integers(300, 1301, size=n).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(sz)[:-1]])
    f = np.zeros(n, FRAG)
    f["off"] = off
    f["sz"] = sz
    arena = np.zeros(int(off[-1] + sz[-1]) + 16, np.uint8)
    return arena, f


def run(lib, kind, items, arena, nslot, iters, copy):
    ns = C.c_uint64(); by = C.c_uint64()
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    r = lib.fd_ed25519_gpu_test_submit_host(kind, p(items), len(items), p(arena), len(arena), nslot, iters, copy,
                                            C.byref(ns), C.byref(by))
    assert r == 0, r
    sec = ns.value / 1e9 / iters
    return {"items_per_s": len(items) / sec, "items_per_s_per_slot": len(items) / sec / nslot,
            "ms_per_batch": sec * 1e3, "bytes_per_batch": by.value, "host_read_GBps": by.value / sec / 1e9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--per-slot", type=int, default=65536)
    ap.add_argument("--frags-per-slot", type=int, default=35000)
    a = ap.parse_args()
    lib = fa.load_lib()
    lib.fd_ed25519_gpu_test_submit_host.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int,
                                                    C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(5)
    out = {"what": "host work of the multi-slot submit paths (copy plan + rebased records per slot, per-slot threads), "
                   "no device; copy=1 adds the CPU memcpy of the page runs",
           "cpu": os.cpu_count(), "sched_cpus": len(os.sched_getaffinity(0)), "desc": {}, "frags": {},
           "note": "no 8-GPU node measured: this is the host side alone"}
    for ns in [int(x) for x in a.slots.split(",")]:
        arena, d = desc_workload(ns * a.per_slot)
        for copy in (0, 1):
            out["desc"]["slots%d_copy%d" % (ns, copy)] = run(lib, 0, d, arena, ns, a.iters, copy)
        del arena, d
        arena, f = frag_workload(ns * a.frags_per_slot, rng)
        for copy in (0, 1):
            out["frags"]["slots%d_copy%d" % (ns, copy)] = run(lib, 1, f, arena, ns, a.iters, copy)
        del arena, f
    s8 = out["desc"].get("slots8_copy0")
    if s8:
        out["desc_8slot_vs_8x122M"] = s8["items_per_s"] / (8 * 122e6)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
