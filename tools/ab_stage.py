"""ab_stage.py -- same-process A/B of verify-stage settings (dev tool): the
stage bench's frag stream (tools/bench_verify_stage.py make_stream), the
asynchronous device-parse stage over it as one stream (--passes passes, no
drain between them, like a tile that never stops), once per setting per
round, settings alternated over --rounds rounds; each setting's context is
created under its environment (read at context creation).  Prints the median
streaming rate per setting and checks every setting's results equal the
first's.

  python3 tools/ab_stage.py "A:" "B:FD_ED25519_GPU_PARSE_STREAM=1" [--frags N] [--rounds R]
  (a setting's BATCH=<frags> gives it its own batch size; HEAD=a/b/c its first
  batches' sizes in frags, TAIL=x/y its last batches' sizes as fractions of
  the batch -- bench_verify_stage.batch_schedule)
  --per-run: each measurement is ONE pass from an idle stage, fill and drain
  included (the stage bench's per-run figure), instead of --passes passes as
  one stream
"""
import argparse
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import firedancer_amd as fa  # noqa: E402
from bench_verify_stage import make_stream, stream_passes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("settings", nargs="+")
ap.add_argument("--frags", type=int, default=1 << 20)
ap.add_argument("--passes", type=int, default=4)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--batch", type=int, default=36000)
ap.add_argument("--per-run", action="store_true")
a = ap.parse_args()
arena, frags, n_sigs = make_stream(a.frags, 0.1)
fr = np.ascontiguousarray(frags)
specs = []
for sp in a.settings:
    name, _, env = sp.partition(":")
    specs.append((name, dict(kv.split("=", 1) for kv in env.split(",")) if env else {}))
# BATCH=<frags> in a setting: that setting's batch size (not an environment variable)
bsz = [int(env.pop("BATCH", a.batch)) for _, env in specs]
heads = [[int(x) for x in env.pop("HEAD").split("/")] if "HEAD" in env else [] for _, env in specs]
tails = [[float(x) for x in env.pop("TAIL").split("/")] if "TAIL" in env else [] for _, env in specs]
ctx = []
for (name, env), b in zip(specs, bsz):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=16 * b)
    if not ctx:
        g.host_register(arena)               # page-locked once (all contexts share the process's registration)
    st = fa.AsyncStage(g, fa.TCache(), b, threads=8, device_parse=True)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    ctx.append((g, st))
res = [np.zeros(len(fr), np.int8) for _ in specs]
sig = np.zeros(len(fr), np.uint64)


def stream(st, out, passes, k):
    st.tcache.reset()
    return passes * n_sigs / stream_passes(st, arena, fr, out, sig, passes, bsz[k], heads[k], tails[k])


passes = 1 if a.per_run else a.passes
for k, (g, st) in enumerate(ctx):
    stream(st, res[k], 1, k)                # warm
rates = [[] for _ in specs]
for r in range(a.rounds):
    order = range(len(specs)) if r % 2 == 0 else reversed(range(len(specs)))
    for k in order:
        rates[k].append(stream(ctx[k][1], res[k], passes, k))
for k, (name, env) in enumerate(specs):
    assert np.count_nonzero(res[k] != res[0]) <= 16, name
    print("%-10s %-50s %s median %.1f M sigs/s (mean %.1f, min %.1f max %.1f, %d runs)" % (
        name, ",".join(["%s=%s" % kv for kv in env.items()] + ["batch=%d" % bsz[k]] +
                       (["head=%s" % "/".join(map(str, heads[k]))] if heads[k] else []) +
                       (["tail=%s" % "/".join(map(str, tails[k]))] if tails[k] else [])),
        "per-run" if a.per_run else "streaming", statistics.median(rates[k]) / 1e6,
        statistics.mean(rates[k]) / 1e6, min(rates[k]) / 1e6, max(rates[k]) / 1e6, len(rates[k])), flush=True)
for i, (g, st) in enumerate(ctx):
    st.close()
    if i == 0:
        g.host_unregister(arena)
    g.close()
