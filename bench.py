#!/usr/bin/env python3
"""bench.py -- Ed25519 verifies/sec on MI355X (BASELINE.json metric), one JSON line.

Workload (BASELINE.json configs[1], "config 2"): per GPU, a 65,536-signature
batch with fixed 200-byte messages, all valid (the most work per signature),
inputs resident in HBM before the timed region.  One step = one pass of the
verify hot path (fd_ed25519_verify_batch_gpu_dev) over that batch.

Multi-GPU: `--gpus N` runs N ranks, one process per GPU.  Started without
WORLD_SIZE (plain `python bench.py --gpus N`), bench.py checks that N devices
are visible (exit 2 otherwise, before anything touches a GPU) and runs itself
under torch.distributed.run as a child process; started by
torch.distributed.run (the driver's form), WORLD_SIZE must equal N.  Every
rank verifies its own 64K batch: weak scaling, no collective on the data path
(signatures are independent, the reference scales the same way with N
independent verify tiles, src/app/fdctl/run/tiles/fd_verify.c:140-141); the
barrier + SUM(units) / MAX(time) over ranks is the only exchange.
`--stub` runs the same launcher and aggregation on CPU (gloo) for the tests.

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
                  rocprofv3 PMC pass of this very build (the newest profiles/rNN/
                  pmc_traffic.json whose code-object hash matches the loaded library's
                  fd_ed25519_gpu_build_id; gfx950 FETCH_SIZE x2 correction) or null.
  warmup_detail -- the untimed steps before the timed ones: prime steps (back-to-back
                  launches for --prime-ms, so the clock has left its idle ramp) and
                  the --warmup steps; build -- the library's build id.
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


def build_workload(n, msg_sz, seed, n_keys=None):
    """n signatures (fixed seed) over random messages, RFC 8032-signed by the
    benchmark input generator tools/synth.py ([s]B in tools/bin/libsynth_sign.so
    on 16 host threads; pinned against the reference signer by
    tests/test_verify_stage.py).  msg_sz: an int (fixed size) or None for
    Uniform{0..1232} (config 3).  n_keys distinct keys (default n)."""
    import firedancer_amd as fa
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import synth
    rng = np.random.default_rng(1234 + seed)
    n_keys = n_keys or n
    seeds = [rng.bytes(32) for _ in range(n_keys)]
    sizes = rng.integers(0, 1233, size=n) if msg_sz is None else np.full(n, msg_sz)
    msgs = [rng.bytes(int(z)) for z in sizes]
    kps = synth.keypairs(seeds, threads=16)
    sigs = synth.sign_many([kps[i % n_keys] + (msgs[i],) for i in range(n)], threads=16)
    recs = [(msgs[i], sigs[i], kps[i % n_keys][1]) for i in range(n)]
    arena, desc, sz = fa.pack_batch(recs)
    what = ("%d-B" % msg_sz) if msg_sz is not None else "Uniform{0..1232}-B"
    return arena, desc, sz, np.zeros(n, np.int8), "%d signatures by %d distinct keys over %s random messages " \
        "(seed %d), RFC 8032-signed by tools/synth.py, all valid" % (n, n_keys, what, 1234 + seed)


def desc_pub(arena, desc):
    return [arena[int(o):int(o) + 32].tobytes() for o in desc["pub_off"]]


def build_adversarial(n):
    """Config 4: every committed golden record (the reference's Wycheproof,
    CCTV and malleability vectors plus the generated adversarial classes,
    tests/golden) tiled to n descriptors; expected codes are the reference
    AVX-512 build's, checked after the run."""
    import firedancer_amd as fa
    from golden_io import read_sigs
    base = read_sigs("vectors_ref.bin") + read_sigs("synthetic.bin")
    recs = [base[i % len(base)] for i in range(n)]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    exp = np.array([r["code"] for r in recs], np.int8)
    hist = {int(k): int(v) for k, v in zip(*np.unique(exp, return_counts=True))}
    return arena, desc, sz, exp, "config-4 adversarial mix: %d golden records (reference vectors + generated " \
        "classes) tiled to %d, expected codes %s" % (len(base), n, hist)


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


def profile_rounds():
    """profiles/rNN directories, newest round first."""
    base = os.path.join(REPO, "profiles")
    rs = [d for d in os.listdir(base) if d.startswith("r") and d[1:].isdigit()] if os.path.isdir(base) else []
    return sorted(rs, key=lambda d: int(d[1:]), reverse=True)


def pmc_traffic(n, kernel, code):
    """HBM bytes per launch of this kernel at this batch size from the newest
    committed PMC summary (tools/gpu.sh profile -> tools/summarize_profile.py,
    profiles/rNN/pmc_traffic.json) that was measured on THIS build: its
    "build" entry's code hash must equal the loaded library's
    (fd_ed25519_gpu_build_id).  Returns (bytes or None, the file used or why
    none was)."""
    for r in profile_rounds():
        path = os.path.join(REPO, "profiles", r, "pmc_traffic.json")
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        if d.get("batch") != n or d.get("kernel") != kernel:
            continue
        if (d.get("build") or {}).get("code") != code:
            continue
        return d.get("hbm_bytes_per_launch"), "profiles/%s/pmc_traffic.json" % r
    return None, "no committed PMC profile of code object %s (%s, batch %d)" % (code, kernel, n)


def cpu_baseline(arena, desc, expect, budget_s=10.0):
    """Reference fd_ed25519_verify on this host (oracle/_ref), bounded sample:
    one pinned thread per physical core this process may use (BASELINE.md /
    SURVEY.md §8(d): N = physical cores, N stated), each verifying a
    contiguous shard of the same descriptors, warm-up pass, then whole passes
    until the budget is spent."""
    from firedancer_amd.hostcpu import baseline_cpus
    has_ifma = "avx512ifma" in open("/proc/cpuinfo").read()
    flavour = "avx512" if has_ifma else "ref"
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_%s.so" % flavour)
    if not os.path.exists(path):
        return None
    cpus, topo = baseline_cpus()
    threads = min(len(cpus), 256)
    cpu_arr = (ctypes.c_int * threads)(*cpus[:threads])
    lib = ctypes.CDLL(path)
    lib.fdref_verify_descs_pinned.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                              ctypes.c_ulong, ctypes.c_ulong, ctypes.c_void_p]
    m = min(len(desc), 65536)
    d = np.ascontiguousarray(desc[:m])
    out = np.zeros(m, np.int8)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.fdref_verify_descs_pinned(vp(arena), vp(d), m, vp(out), threads, 1, cpu_arr)   # warm-up pass
    if flavour == "avx512":
        assert np.array_equal(out, expect[:m]), "reference codes differ from the expected ones"
    t0 = time.perf_counter(); done = 0
    while time.perf_counter() - t0 < budget_s:
        lib.fdref_verify_descs_pinned(vp(arena), vp(d), m, vp(out), threads, 1, cpu_arr)
        done += m
    dt = time.perf_counter() - t0
    value = done / dt
    out = {"value": value, "unit": "verifies/s", "cores": threads, "kind": "reference",
           "per_core": value / threads, "topology": topo,
            "sample": "%d passes x %d of the same descriptors (%.1f s), fd_ed25519_verify %s build, "
                      "%d pthreads pinned one per physical core" % (done // m, m, dt,
                                                                    "FD_HAS_AVX512" if has_ifma else "ref", threads)}
    if threads < topo["machine_physical_cores"]:
        # the process may use fewer cores than the machine has (cgroup quota on the GPU box):
        # the all-cores figure is the measured per-core rate times the core count, labelled as such
        out["all_physical_cores_extrapolated"] = {
            "value": out["per_core"] * topo["machine_physical_cores"], "cores": topo["machine_physical_cores"],
            "note": "per-core rate measured on %d pinned cores x %d physical cores; not measured at that width"
                    % (threads, topo["machine_physical_cores"])}
    return out


def shred_cpu_baseline(recs, budget_s):
    """The reference FEC resolver's per-shred check (oracle/_ref fdref_shred_check:
    fd_shred_parse, the bmtree root from the inclusion proof, fd_ed25519_verify
    of the root, src/disco/shred/fd_fec_resolver.c:309-405) on ONE core, as the
    reference runs it inside its one shred tile: whole passes over the
    capture's shreds until the budget is spent."""
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_%s.so" %
                        ("avx512" if "avx512ifma" in open("/proc/cpuinfo").read() else "ref"))
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.fdref_shred_check.restype = ctypes.c_int
    lib.fdref_shred_check.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
    root = ctypes.create_string_buffer(32)
    for r in recs:                                                           # warm-up pass + check
        assert lib.fdref_shred_check(r["shred"], len(r["shred"]), r["leader"], root) == 0
    t0 = time.perf_counter(); done = 0
    while time.perf_counter() - t0 < budget_s:
        for r in recs:
            lib.fdref_shred_check(r["shred"], len(r["shred"]), r["leader"], root)
        done += len(recs)
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "shreds/s", "cores": 1, "kind": "reference",
            "sample": "%d passes over the %d valid shreds of the reference's demo capture (%.1f s), "
                      "fdref_shred_check on one core (the reference checks shreds in one tile)"
                      % (done // len(recs), len(recs), dt)}


def hostfed_main(args):
    """--path host-fed: the verifier fed from HOST memory, PCIe in the loop
    (VERDICT r03 next #3), one GPU, a line of its own (not the headline,
    which is device-resident).  Measured: H2D copy bandwidth from page-locked
    and from pageable memory; config 2 (64K x 200 B) and config 3 (1M,
    Uniform{0..1232} B) through fd_ed25519_verify_batch_gpu (synchronous,
    one-shot kernels: copy in, verify, codes out, one batch at a time) and
    through fd_ed25519_gpu_submit / _poll (QUEUE_DEPTH batches of at most
    64K in flight on the pipelined kernel, copies overlapping the kernels),
    from a pageable and from a page-locked arena; bytes per verify (the
    arena bytes the descriptors touch + the 16-B descriptor + the 1-B code)
    and the link-bound ceiling they imply."""
    # No torch here: the library and the HIP runtime it links are the process's
    # only GPU stack (torch's wheel bundles a second HIP / HSA runtime; with
    # both loaded, rocprofv3's finalizer faulted at exit).
    os.environ["FD_ED25519_GPU_NO_TORCH"] = "1"
    import firedancer_amd as fa
    out = {"metric": "host-fed Ed25519 verifies/sec (PCIe in the loop)", "unit": "verifies/s", "n_gpus": 1,
           "data": "synthetic (tools/synth.py), all valid"}
    # H2D bandwidth: 256 MB from page-locked (async copies) and from pageable memory
    fa.load_lib()                                        # the library (and the HIP runtime it links) first
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    nb = 256 << 20
    h_pin, d_buf = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipSetDevice(0) == 0
    assert hip.hipHostMalloc(ctypes.byref(h_pin), ctypes.c_size_t(nb), 0) == 0
    assert hip.hipMalloc(ctypes.byref(d_buf), ctypes.c_size_t(nb)) == 0
    h_page = np.ones(nb, np.uint8)
    bw = {}
    for name, src in (("pinned", h_pin.value), ("pageable", h_page.ctypes.data)):
        def copies(k):
            for _ in range(k):
                if name == "pinned":
                    assert hip.hipMemcpyAsync(d_buf, ctypes.c_void_p(src), ctypes.c_size_t(nb), 1, None) == 0
                else:
                    assert hip.hipMemcpy(d_buf, ctypes.c_void_p(src), ctypes.c_size_t(nb), 1) == 0
            assert hip.hipDeviceSynchronize() == 0
        copies(2)
        t = time.perf_counter()
        copies(8)
        bw[name] = 8 * nb / (time.perf_counter() - t) / 1e9
    out["h2d_GBps"] = bw
    hip.hipFree(d_buf)
    hip.hipHostFree(h_pin)
    del h_page
    res = {}
    want = [int(c) for c in os.environ.get("FD_HOSTFED_CONFIGS", "2,3").split(",")]
    skip = os.environ.get("FD_HOSTFED_SKIP", "").split(",")    # dev: sections left out (exit-crash bisection)
    for cfg, n, msg_sz in [c for c in ((2, 65536, 200), (3, 1 << 20, None)) if c[0] in want]:
        arena, desc, sz, expect, data_desc = build_workload(n, msg_sz, seed=0, n_keys=min(n, 65536))
        g = fa.Ed25519Gpu(device_mask=1, max_batch=min(n, 65536))
        r = {"workload": data_desc, "bytes_per_verify": (sz + 17 * n) / n}
        # synchronous one-shot calls over the whole batch (chunked by the library at max_batch)
        assert np.array_equal(g.verify_batch(arena, sz, desc), expect)
        t = time.perf_counter()
        k = 3
        for _ in range(k):
            o = g.verify_batch(arena, sz, desc)
        r["verify_batch_gpu_sync"] = k * n / (time.perf_counter() - t)
        assert np.array_equal(o, expect)
        # async pipelined stream of 64K batches, QUEUE_DEPTH in flight
        bs = 65536
        parts = [(i, min(bs, n - i)) for i in range(0, n, bs)]
        reps = max(4, 64 * bs // n)          # 64 batches at config 2, 64 chunks at config 3: fill and drain < 5 %

        def stream():
            outs = [np.zeros(c, np.int8) for _, c in parts] * reps
            todo = [(i, c, outs[j]) for j, (i, c) in enumerate(parts * reps)]
            pend = 0
            t0 = time.perf_counter()
            for i, c, o in todo:
                while pend >= fa.QUEUE_DEPTH:
                    assert g.poll(block=True); pend -= 1
                g.submit(arena, sz, desc[i:i + c], o)
                pend += 1
            while pend:
                assert g.poll(block=True); pend -= 1
            dt = time.perf_counter() - t0
            assert all(np.array_equal(o, expect[i:i + c]) for (i, c, o) in todo)
            return len(todo) and sum(c for _, c, _ in todo) / dt
        if "warm" not in skip:
            stream()
        r["submit_poll_pageable"] = stream()
        g.host_register(arena)
        if "warm" not in skip:
            stream()
        if "stats" not in skip:
            g.host_stats(reset=True)
        r["submit_poll_registered"] = stream()
        if "stats" not in skip:
            hs = g.host_stats()
            r["submit_path_ms_registered"] = {k[:-3]: v / 1e6 for k, v in hs.items() if k.endswith("_ns")}
            r["h2d_bytes_per_verify_registered"] = hs["h2d_bytes"] / (n * reps)
        g.host_unregister(arena)
        r["link_bound_verifies_per_s_pinned"] = bw["pinned"] * 1e9 / r["bytes_per_verify"]
        g.close()
        res["config%d" % cfg] = r
    out["configs"] = res
    out["value"] = res["config2"]["submit_poll_registered"] if "config2" in res else None
    out["note"] = ("value: config 2 through submit/poll from a page-locked arena; the headline line's value is "
                   "device-resident.  link_bound = pinned H2D GB/s / bytes_per_verify")
    print(json.dumps(out), flush=True)
    return 0


def notorch_main(args):
    """--path no-torch: the headline config-2 step (device-resident 64K x 200 B, one
    fd_ed25519_gpu_pipe_dev launch per step, codes checked after the run) with NO
    torch in the process: device memory, the stream and the timing events come
    from the HIP runtime the library links (/opt/rocm), through ctypes -- the
    runtime the C product (offload server, a C verify tile) runs on.  The
    headline line runs on torch's bundled runtime (torch imported first); this
    line puts the two side by side.  N=1, a line of its own."""
    os.environ["FD_ED25519_GPU_NO_TORCH"] = "1"
    import firedancer_amd as fa
    fa.load_lib()
    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    vp, sz_t = ctypes.c_void_p, ctypes.c_size_t
    n = args.batch or 65536
    assert n <= 65536, "--path no-torch runs the pipelined config-2 step (at most one wave per SIMD)"
    arena, desc, sz, expect, data_desc = build_workload(n, args.msg_sz, seed=0)
    assert hip.hipSetDevice(0) == 0

    def dmalloc(nb):
        p = vp()
        assert hip.hipMalloc(ctypes.byref(p), sz_t(nb)) == 0
        return p.value

    def h2d(d, a):
        assert hip.hipMemcpy(vp(d), vp(a.ctypes.data), sz_t(a.nbytes), 1) == 0

    d_arena, d_desc = dmalloc(arena.nbytes), dmalloc(desc.nbytes)
    h2d(d_arena, arena)
    h2d(d_desc, np.ascontiguousarray(desc))
    d_outs = [dmalloc(n), dmalloc(n)]
    stream = vp()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(stream), 1) == 0      # non-blocking, like torch's side stream
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    nstep = [0]

    def step():
        g.pipe_dev(d_arena, sz, d_desc, n, d_outs[nstep[0] & 1], stream=stream.value)
        nstep[0] += 1

    def sync():
        assert hip.hipStreamSynchronize(stream) == 0

    def event():
        e = vp()
        assert hip.hipEventCreate(ctypes.byref(e)) == 0
        return e

    def elapsed(a, b):
        ms = ctypes.c_float(0)
        assert hip.hipEventElapsedTime(ctypes.byref(ms), a, b) == 0
        return ms.value

    prime, t_prime = 0, time.perf_counter()
    while (time.perf_counter() - t_prime) * 1e3 < args.prime_ms:
        for _ in range(8):
            step()
        prime += 8
        sync()
    for _ in range(args.warmup):
        step()
    sync()
    ev0, ev1 = event(), event()
    t0 = time.perf_counter()
    hip.hipEventRecord(ev0, stream)
    for _ in range(args.steps):
        step()
    hip.hipEventRecord(ev1, stream)
    sync()
    dt = time.perf_counter() - t0
    region_ms = elapsed(ev0, ev1) / args.steps
    evs = [(event(), event()) for _ in range(min(args.steps, 50))]
    for a, b in evs:
        hip.hipEventRecord(a, stream)
        step()
        hip.hipEventRecord(b, stream)
    sync()
    launch_ms = float(np.mean([elapsed(a, b) for a, b in evs]))
    g.pipe_flush_dev(stream=stream.value)
    sync()
    for d in d_outs:
        o = np.zeros(n, np.int8)
        assert hip.hipMemcpy(vp(o.ctypes.data), vp(d), sz_t(n), 2) == 0
        assert np.array_equal(o, expect), "verify codes differ from the expected ones"
    value = n * args.steps / dt
    peak = valu_peak()
    line = {"metric": "Ed25519 verifies/sec (no torch in the process)", "value": value, "unit": "verifies/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "dtype": "u32", "data": "synthetic: " + data_desc,
            "config": {"workload": "config2: %d-signature batch, fixed %d-B messages, device-resident" % (n, args.msg_sz),
                       "batch_per_gpu": n},
            "roofline": {"bound": "valu-int32", "achieved": W_MAC * value / 1e12, "peak": peak / 1e12,
                         "frac": W_MAC * value / peak, "region_ms_per_launch": region_ms, "kernel_ms": launch_ms,
                         "kernel_frac": W_MAC * n / (launch_ms * 1e-3) / peak},
            "warmup_detail": {"prime_steps": prime, "warmup_steps": args.warmup},
            "build": fa.build_id(), "runtime": fa.runtime_info(), "torch_loaded": "torch" in sys.modules}
    g.close()
    for d in [d_arena, d_desc] + d_outs:
        hip.hipFree(vp(d))
    hip.hipStreamDestroy(stream)
    print(json.dumps(line), flush=True)
    return 0


def shred_main(args):
    """--path shred: shreds/s through fd_ed25519_gpu_shred_verify (the
    FEC resolver's first-shred check as a descriptor source).
    One step = one call over --batch shreds in HOST memory (the API takes host
    buffers): host walk (parse, proof bounds), Merkle roots on the GPU
    (fd_shred_root_kernel), one verify launch, codes back.  Reported beside
    it: the same with the roots hashed on the host thread
    (FD_ED25519_GPU_SHRED_HOST_HASH=1), the host walk alone, and the
    reference's one-core check."""
    import torch
    import firedancer_amd as fa
    from golden_io import read_shreds
    torch.cuda.set_device(0)
    base = [r for r in read_shreds() if r["tag"] < 1000 and r["result"] == 0]
    n = args.batch or 65536
    blob, spans, keys = bytearray(), [], []
    key_at = {}
    for i in range(n):
        r = base[i % len(base)]
        if r["leader"] not in key_at:
            key_at[r["leader"]] = len(blob); blob += r["leader"]
        keys.append(key_at[r["leader"]])
        spans.append((len(blob), len(r["shred"]))); blob += r["shred"]
    aux_off = (len(blob) + 63) & ~63
    arena = np.zeros(aux_off + 32 * n, np.uint8)
    arena[:len(blob)] = np.frombuffer(bytes(blob), np.uint8)
    spans = np.array(spans, fa.SPAN_DTYPE); keys = np.array(keys, np.uint32)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)

    def timed(env_host, steps):
        if env_host:
            os.environ["FD_ED25519_GPU_SHRED_HOST_HASH"] = "1"
        try:
            for _ in range(args.warmup):
                out = g.shred_verify(arena, len(arena), aux_off, 32 * n, spans, keys)
            assert np.all(out == 0), "shred codes differ from the reference's (all valid)"
            t0 = time.perf_counter()
            for _ in range(steps):
                g.shred_verify(arena, len(arena), aux_off, 32 * n, spans, keys)
            return (time.perf_counter() - t0) / steps
        finally:
            os.environ.pop("FD_ED25519_GPU_SHRED_HOST_HASH", None)

    t_gpu = timed(False, args.steps)
    t_host = timed(True, max(args.steps // 4, 3))
    host = arena.copy()
    t0 = time.perf_counter()
    walks = 3
    for _ in range(walks):
        fa.shred_walk(host, len(host), aux_off, 32 * n, spans, keys)
    t_walk = (time.perf_counter() - t0) / walks
    line = {"metric": "shreds_verified_per_s", "value": n / t_gpu, "unit": "shreds/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": t_gpu * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "reference demo capture",
            "config": {"workload": "fd_ed25519_gpu_shred_verify over %d shreds (the %d valid shreds of the "
                                   "reference's demo-shreds.pcap tiled), host memory in and out" % (n, len(base)),
                       "batch_per_gpu": n},
            "host_hash_variant": {"value": n / t_host, "ms_per_step": t_host * 1e3,
                                  "note": "FD_ED25519_GPU_SHRED_HOST_HASH=1: Merkle roots on the calling thread"},
            "host_walk_only": {"value": n / t_walk, "ms_per_step": t_walk * 1e3,
                               "note": "fa.shred_walk: parse + host roots, no GPU (one thread)"},
            "build": fa.build_id(), "cpu_baseline": None}
    if not args.no_cpu:
        line["cpu_baseline"] = shred_cpu_baseline(base, args.cpu_budget)
    g.close()
    print(json.dumps(line), flush=True)
    return 0


def launch_ranks(args):
    """--gpus N without WORLD_SIZE: run N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code.  The
    device count is read before anything initialises the GPU in this process
    (torch.cuda.device_count() does not, on this image); fewer devices than N
    is an error, never a silent single-GPU run."""
    import socket
    import subprocess
    if not args.stub:
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            print("bench.py: --gpus %d but only %d GPU(s) visible; refusing to run" % (args.gpus, have),
                  file=sys.stderr, flush=True)
            return 2
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    if os.environ.get("FD_MAPS_OUT"):
        # diagnostic: the process's mappings as Python exits (the C libraries'
        # finalizers run after this), to resolve the addresses of a crash at exit
        import atexit
        import shutil
        atexit.register(shutil.copyfile, "/proc/self/maps", os.environ["FD_MAPS_OUT"])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~40 ms of untimed launches first: the timed region then sees the clock the
    # GPU sustains under this load, not its ramp from idle
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4],
                    help="2: 64K valid 200-B sigs per GPU (headline); 3: 1M sigs in total, "
                         "Uniform{0..1232}-B messages, split over the GPUs (strong scaling); "
                         "4: the adversarial golden mix tiled to --batch per GPU")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--hot-keys", type=int, default=0,
                    help="config 2 / 3 with this many distinct signers, all in the hot-key cache "
                         "(vote-like traffic; fd_ed25519_gpu_keycache_*, 512 KB of HBM per key)")
    ap.add_argument("--msg-sz", type=int, default=200)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--prime-ms", type=float, default=150.0,
                    help="untimed back-to-back steps for this long before the warm-up steps: a GPU that was idle "
                         "runs its first ~100 ms at a ramping clock; the timed region should see the clock a "
                         "continuously fed verify stage runs at (reported as prime_steps)")
    ap.add_argument("--pipeline", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: each step is one fd_ed25519_gpu_pipe_dev launch (phase A of this batch, B of the "
                         "previous one, C of the one before: three batches in flight, every launch one batch of "
                         "work; the drain after the timed steps is timed and reported too); 0: each step is one "
                         "fd_ed25519_gpu_verify_batch_dev launch (the whole batch); -1 (default): 1 when the batch "
                         "is at most one wave per SIMD (256 x CUs signatures: config 2), else 0 (larger batches "
                         "already give every SIMD several waves, and the single-lane kernel packs them better)")
    ap.add_argument("--path", default="verify", choices=["verify", "shred", "host-fed", "no-torch"],
                    help="verify (default): the headline line above.  shred: the FEC resolver's first-shred check "
                         "(fd_ed25519_gpu_shred_verify: host walk, Merkle roots on the GPU, verify) over the "
                         "reference's demo capture tiled to --batch, from host memory, N=1; a line of its own "
                         "(not the headline metric) with the host-hash variant and the reference's one-core check "
                         "(oracle/_ref fdref_shred_check) beside it.  host-fed: configs 2 and 3 from HOST memory "
                         "(sync calls and the async submit/poll stream, pageable and page-locked) beside the H2D "
                         "bandwidth, N=1, a line of its own.  no-torch: the config-2 step with no torch in the "
                         "process (device memory, stream and events from the library's own HIP runtime), N=1")
    ap.add_argument("--stub", action="store_true",
                    help="CPU test mode (tests/test_bench_launch.py): gloo, a no-op step on a fixed count; "
                         "exercises the launcher, rank setup and SUM/MAX aggregation without a GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr, flush=True)
        sys.exit(2)
    if args.stub:
        sys.exit(stub_main(args, world, rank))
    if args.path == "shred":
        if world != 1:
            print("bench.py: --path shred runs on one GPU", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.exit(shred_main(args))
    if args.path == "host-fed":
        if world != 1:
            print("bench.py: --path host-fed runs on one GPU", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.exit(hostfed_main(args))
    if args.path == "no-torch":
        if world != 1:
            print("bench.py: --path no-torch runs on one GPU", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.exit(notorch_main(args))

    import torch
    import torch.distributed as dist
    import firedancer_amd as fa

    if torch.cuda.device_count() <= local:
        print("bench.py: rank %d needs GPU %d, %d visible" % (rank, local, torch.cuda.device_count()),
              file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group(backend="nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    if args.config == 3:
        total = args.batch or 1 << 20
        n = total // world + (1 if rank < total % world else 0)
        arena, desc, sz, expect, data_desc = build_workload(n, None, seed=rank,
                                                            n_keys=args.hot_keys or min(n, 65536))
    elif args.config == 4:
        n = args.batch or 65536
        arena, desc, sz, expect, data_desc = build_adversarial(n)
    else:
        n = args.batch or 65536
        arena, desc, sz, expect, data_desc = build_workload(n, args.msg_sz, seed=rank,
                                                            n_keys=args.hot_keys or None)
    g = fa.Ed25519Gpu(device_mask=1 << local, max_batch=n)
    if args.hot_keys:
        keys = sorted(set(desc_pub(arena, desc)))
        g.keycache_reserve(len(keys))
        g.keycache_add(keys)
        data_desc += "; all %d signers in the hot-key cache" % len(keys)
    d_arena = torch.from_numpy(arena).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    pair_max = 256 * torch.cuda.get_device_properties(dev).multi_processor_count   # the host's pair_max
    pipe = (args.pipeline == 1 or (args.pipeline == -1 and n <= pair_max)) and not args.hot_keys
    d_outs = [d_out, torch.zeros(n, dtype=torch.int8, device=dev)]
    nstep = [0]

    def step():
        # pipelined: step i's codes land in d_outs[i % 2] once the launches two
        # chunks later complete; a batch above one wave per SIMD (config 3) is
        # the library's k pre-pass + one launch per pair_max chunk, three chunks
        # in flight across launches and across steps
        if pipe:
            out = d_outs[nstep[0] & 1]
            g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=stream.cuda_stream)
            nstep[0] += 1
            return
        g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(),
                           stream=stream.cuda_stream)

    def settle():
        """codes of every launched batch final (pipeline: the pending phases
        of the last two batches); returns the drain's wall time in s"""
        t = time.perf_counter()
        if pipe:
            g.pipe_flush_dev(stream=stream.cuda_stream)
        torch.cuda.synchronize()
        t = time.perf_counter() - t
        for o in (d_outs if pipe else [d_out]):
            assert np.array_equal(o.cpu().numpy(), expect), "verify codes differ from the expected ones"
        return t

    prime = 0
    t_prime = time.perf_counter()
    while (time.perf_counter() - t_prime) * 1e3 < args.prime_ms:
        for _ in range(8):
            step()
        prime += 8
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # the timed region: K steps back to back, one HIP event pair around all of
    # them on the launch stream (an event record between launches costs the
    # GPU 3-4 us, tools/marker_probe.py: none inside the region)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    region_ms = ev0.elapsed_time(ev1) / args.steps    # average launch duration over the region, gaps included
    # after the region (untimed): each launch alone between two events, for
    # the kernel's own duration (kernel_ms, kernel_frac)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(min(args.steps, 50))]
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    drain = settle()

    from firedancer_amd.dist import aggregate_throughput
    total, dt_max = aggregate_throughput(n * args.steps, dt, device=dev)
    workload = {2: "config2: %d-signature batch per GPU, fixed %d-B messages, device-resident" % (n, args.msg_sz),
                3: "config3: %d signatures in total split over %d GPU(s), Uniform{0..1232}-B messages, "
                   "device-resident" % (args.batch or 1 << 20, world),
                4: "config4: adversarial golden mix, %d-descriptor batch per GPU, device-resident" % n}[args.config]
    value = total / dt_max

    kname = ("fd_ed25519_verify_pipe_kernel" if pipe else
             "fd_ed25519_verify_cached_kernel" if args.hot_keys else
             "fd_ed25519_verify_pair_kernel" if n <= pair_max and os.environ.get("FD_ED25519_GPU_PAIR") != "0"
             else "fd_ed25519_verify_kernel")
    if rank == 0:
        peak = valu_peak()
        # priced on the step (the wall-timed ms_per_step, launch gap included,
        # per GPU), as `value` is; the event-bracketed kernel time gives
        # kernel_frac beside it
        achieved = W_MAC * value / world
        kernel_achieved = W_MAC * n / (launch_ms * 1e-3)
        build = fa.build_id()
        traffic, traffic_src = pmc_traffic(n, kname, build.get("code")) if args.config == 2 else (None, "config 2 only")
        line = {
            "metric": "Ed25519 verifies/sec",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.config == 3 else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: " + data_desc,
            "config": {"workload": workload, "batch_per_gpu": n,
                       "msg_sz": args.msg_sz if args.config == 2 else None, "parallelism": "shard-per-gpu x%d" % world},
            "roofline": {"bound": "valu-int32", "achieved": achieved / 1e12, "peak": peak / 1e12,
                         "unit": "T MAC/s (32x32->64 multiply-adds, W=%.4g per verify)" % W_MAC,
                         "frac": achieved / peak, "traffic": traffic, "traffic_source": traffic_src,
                         "priced_on": "ms_per_step (wall clock per step, per GPU: W x value / n_gpus)",
                         "region_ms_per_launch": region_ms,
                         "region_ms_note": "HIP events on the launch stream around the timed region / steps: the "
                                           "average launch duration, inter-launch gaps included",
                         "kernel_ms": launch_ms, "kernel_frac": kernel_achieved / peak,
                         "kernel_frac_note": "the same W priced on the mean event-bracketed launch (no inter-launch "
                                             "gap), measured over up to 50 launches right after the timed region"},
            "cpu_baseline": None,
            "warmup_detail": {"prime_steps": prime, "prime_ms": args.prime_ms, "warmup_steps": args.warmup,
                              "untimed_steps_total": prime + args.warmup,
                              "note": "prime steps run back to back for prime_ms first (the clock ramps from idle), "
                                      "then the warmup steps; none of them is timed"},
            "build": build,
            "runtime": fa.runtime_info(),
        }
        if pipe:
            line["pipeline"] = {
                "api": "fd_ed25519_gpu_pipe_dev",
                "note": "each timed step is one launch running phase A (checks, SHA-512, lattice) of this batch, "
                        "phase B (decode + table of A and of R, check codes, top chain windows) of the "
                        "previous one and phase C (rest of the chain, [w]B, compare) of the one before: three "
                        "batches in flight, every launch one batch of work; the batches in flight when the timed "
                        "region starts were launched in the warm-up, the last two finish in the drain after it",
                "drain_ms": drain * 1e3,
                "value_with_drain": n * args.steps / (dt + drain),
            }
        # The same launch against the HBM roofline (not the bound: ~1/4 of the ~8 TB/s peak),
        # from the PMC-measured bytes per launch of this build's committed profile.
        t = traffic
        if t:
            gbs = t / (dt_max / args.steps) / 1e9
            line["roofline_hbm"] = {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s",
                                    "frac": gbs / 8000.0, "traffic": t}
        if args.config != 2:   # the roofline numerator W is defined for valid 200-B verifies only
            line["roofline"]["frac_note"] = "W-based numerator is for valid 200-B verifies (config 2)"
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(arena, desc, expect, args.cpu_budget)
        print(json.dumps(line), flush=True)
    g.close()
    if world > 1:
        dist.destroy_process_group()


def stub_main(args, world, rank):
    """--stub: the launcher / aggregation path on CPU (gloo), no GPU, no HIP.
    Each rank 'verifies' a fixed count per step (a short sleep stands in for
    the kernel); the line reports SUM of units over ranks / MAX of time."""
    import torch.distributed as dist
    from firedancer_amd.dist import aggregate_throughput
    if world > 1:
        dist.init_process_group(backend="gloo")
    n = args.batch or 1024
    for _ in range(args.warmup):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.002 * (1 + rank))
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    total, dt_max = aggregate_throughput(n * args.steps, dt)
    if rank == 0:
        print(json.dumps({"metric": "Ed25519 verifies/sec", "value": total / dt_max, "unit": "verifies/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": dt_max / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "stub": True, "units_total": total, "seconds_max": dt_max}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    main()
