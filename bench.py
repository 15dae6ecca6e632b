#!/usr/bin/env python3
"""bench.py -- Ed25519 verifies/sec on MI355X (BASELINE.json metric), one JSON line.

Workload (BASELINE.json configs[1], "config 2"): per GPU, a 65,536-signature
batch with fixed 200-byte messages, all valid (the most work per signature),
inputs resident in HBM before the timed region.  One step = one pass of the
verify hot path (fd_ed25519_verify_batch_gpu_dev) over that batch.  With
--gpus N (torch.distributed.run, one process per GPU) every rank verifies its
own 64K batch: weak scaling, no collective on the data path (signatures are
independent; the barrier + MAX-over-ranks timing is the only exchange).

Synthetic data: 65,536 distinct keys and 200-byte random messages per rank
(fixed seed), RFC 8032-signed on the host by the benchmark input generator
tools/synth.py (our own code; the oracle is used only by cpu_baseline), one
arena record per signature.

Extra keys beside the contract fields:
  roofline     -- INT32 VALU multiply-add roofline of the verify kernel
                  (SURVEY.md §8(d)): achieved = W MAC/verify x verifies per launch
                  / mean launch time (HIP events on the launch stream),
                  peak = measured v_mad_u64_u32 rate (profiles/r01/valu_probe.json)
                  x 256 CU x 2.4 GHz; traffic = HBM bytes per launch from a
                  rocprofv3 PMC pass (profiles/r01/pmc_traffic.json, gfx950 FETCH_SIZE x2 correction) or null.
  cpu_baseline -- the reference fd_ed25519_verify (AVX-512 build when the host
                  has avx512ifma, else the portable build) compiled from the
                  reference sources (oracle/_ref), on a bounded sample of the
                  same descriptors, on this host's cores (rank 0, N=1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

# Algorithmic work per valid verify: W = 64 N_M + 36 N_S + 8 (N_M + N_S)
N_M, N_S = 1380.7, 1520.2
W_MAC = 64 * N_M + 36 * N_S + 8 * (N_M + N_S)
NOMINAL_GHZ = 2.4
N_CU = 256


def build_workload(n, msg_sz, seed):
    """n DISTINCT signatures (fresh key + msg_sz random bytes each, fixed seed),
    signed with RFC 8032 by the benchmark input generator tools/synth.py
    ([s]B in tools/bin/libsynth_sign.so on 16 host threads; pinned against
    the reference signer by tests/test_verify_stage.py)."""
    import firedancer_amd as fa
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import synth
    rng = np.random.default_rng(1234 + seed)
    seeds = [rng.bytes(32) for _ in range(n)]
    msgs = [rng.bytes(msg_sz) for _ in range(n)]
    kps = synth.keypairs(seeds, threads=16)
    sigs = synth.sign_many([(s_, p_, m_) for (s_, p_), m_ in zip(kps, msgs)], threads=16)
    recs = [(m_, g_, p_) for m_, g_, (_, p_) in zip(msgs, sigs, kps)]
    arena, desc, sz = fa.pack_batch(recs)
    return arena, desc, sz, "%d distinct keys and %d-B random messages (seed %d), RFC 8032-signed by " \
                            "tools/synth.py, all valid" % (n, msg_sz, 1234 + seed)


def valu_peak():
    """Measured v_mad_u64_u32 issue rate -> chip MAC/s at the nominal clock."""
    path = os.path.join(REPO, "profiles", "r01", "valu_probe.json")
    rate = None
    if os.path.exists(path):
        d = json.load(open(path))
        rates = [p["wave_instr_per_cu_per_clk"] for p in d["probes"] if p["instr"] == "v_mad_u64_u32"]
        rate = max(rates) if rates else None
    if rate is None:
        rate = 0.88   # measured on MI355X, 8 waves/SIMD (tools/valu_probe.hip)
    return rate * 64 * N_CU * NOMINAL_GHZ * 1e9


def pmc_traffic(n):
    path = os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("batch") != n:
        return None
    return d.get("hbm_bytes_per_launch")


def cpu_baseline(arena, desc, budget_s=10.0):
    """Reference fd_ed25519_verify on this host, bounded sample (oracle/_ref)."""
    has_ifma = "avx512ifma" in open("/proc/cpuinfo").read()
    flavour = "avx512" if has_ifma else "ref"
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_%s.so" % flavour)
    threads = min(16, os.cpu_count() or 1)
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.fdref_verify_descs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                       ctypes.c_ulong, ctypes.c_ulong]
    m = min(len(desc), 16384)
    d = np.ascontiguousarray(desc[:m])
    out = np.zeros(m, np.int8)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.fdref_verify_descs(vp(arena), vp(d), m, vp(out), threads, 1)   # warm-up pass
    assert np.all(out == 0), "reference rejected a valid benchmark signature"
    t0 = time.perf_counter(); done = 0
    while time.perf_counter() - t0 < budget_s:
        lib.fdref_verify_descs(vp(arena), vp(d), m, vp(out), threads, 1)
        done += m
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "verifies/s", "cores": threads, "kind": "reference",
            "sample": "%d passes x %d of the same config-2 descriptors (%.1f s), fd_ed25519_verify %s build, "
                      "%d pthreads" % (done // m, m, dt, "FD_HAS_AVX512" if has_ifma else "ref", threads)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--msg-sz", type=int, default=200)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import firedancer_amd as fa

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    n = args.batch
    arena, desc, sz, data_desc = build_workload(n, args.msg_sz, seed=rank)
    g = fa.Ed25519Gpu(device_mask=1 << local, max_batch=n)
    d_arena = torch.from_numpy(arena).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)

    def step():
        g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(),
                           stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    assert int((d_out == 0).sum()) == n, "verify rejected valid benchmark signatures"

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    assert int((d_out == 0).sum()) == n

    from firedancer_amd.dist import aggregate_throughput
    total, dt_max = aggregate_throughput(n * args.steps, dt, device=dev)
    value = total / dt_max

    if rank == 0:
        peak = valu_peak()
        achieved = W_MAC * n / (launch_ms * 1e-3)
        line = {
            "metric": "Ed25519 verifies/sec",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: " + data_desc,
            "config": {"workload": "config2: %d-signature batch per GPU, fixed %d-B messages, device-resident"
                                   % (n, args.msg_sz),
                       "batch_per_gpu": n, "msg_sz": args.msg_sz, "parallelism": "shard-per-gpu x%d" % world},
            "roofline": {"bound": "valu-int32", "achieved": achieved / 1e12, "peak": peak / 1e12,
                         "unit": "T MAC/s (32x32->64 multiply-adds, W=%.4g per verify)" % W_MAC,
                         "frac": achieved / peak, "traffic": pmc_traffic(n),
                         "kernel_ms": launch_ms},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(arena, desc, args.cpu_budget)
        print(json.dumps(line), flush=True)
    g.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
