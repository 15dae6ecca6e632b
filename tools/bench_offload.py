#!/usr/bin/env python3
"""bench_offload.py -- the verify tile's side of the GPU offload link
(include/fd_verify_offload.h), measured end to end
across two processes.  Run `tools/gpu.sh offload`, which starts
firedancer_amd/fd_verify_offload_server (the process that owns the GPU)
and then this client, which never touches the GPU -- like the sandboxed
tile: it publishes --frags synthetic signed transactions (tools/synth.py,
1-4 signers, --dup duplicates) in seq order in bursts
(fd_verify_offload_publish_burst: as many as fit), reading results by seq
as they become ready (fd_verify_offload_results), and prints one JSON line: frags/s from
the first publish to the last result, result histogram, and the reference
tile on one core (fdref_verify_frags_seq, oracle/_ref) over a bounded sample
as cpu_baseline."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="/fd_verify_offload")
    ap.add_argument("--frags", type=int, default=65536)
    ap.add_argument("--dup", type=float, default=0.1)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import firedancer_amd as fa
    from bench_verify_stage import make_stream, cpu_baseline
    arena, frags, n_sigs = make_stream(args.frags, args.dup)
    t_join = time.time()
    while True:
        try:
            cli = fa.OffloadLink.join(args.name)
            break
        except Exception:
            if time.time() - t_join > 120:
                raise
            time.sleep(0.2)
    n = len(frags)
    depth = cli.depth
    res = np.zeros(n, np.int8)
    sig = np.zeros(n, np.uint64)
    fr = np.ascontiguousarray(frags)
    pub = nxt = 0
    t0 = time.perf_counter()
    while nxt < n:
        if pub < n:   # a result slot is reused when seq + depth is published: stay within depth of nxt
            pub += cli.publish_burst(arena, fr[pub:min(n, nxt + depth)])
        if nxt < pub:
            nxt += cli.results(nxt, res[nxt:pub], sig[nxt:pub])
    dt = time.perf_counter() - t0
    cli.halt()
    cli.close()
    hist = {int(k): int(v) for k, v in zip(*np.unique(res, return_counts=True))}
    line = {"metric": "verify-tile frags/sec through the GPU offload link (2 processes)", "value": n / dt,
            "unit": "frags/s", "n_gpus": 1, "higher_is_better": True, "ms_total": dt * 1e3,
            "data": "synthetic signed legacy txns (tools/synth.py), %.0f%% duplicates" % (100 * args.dup),
            "config": {"workload": "%d frags, %d signatures, published one by one by a client process without "
                                   "GPU access" % (n, n_sigs)},
            "sigs_per_s": n_sigs / dt, "results": hist,
            "cpu_baseline": None if args.no_cpu else cpu_baseline(arena, frags)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
