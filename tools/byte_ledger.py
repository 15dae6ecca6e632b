"""byte_ledger.py -- the pipe kernel's HBM byte ledger per verify, reconciled
with the PMC counters ("Byte ledger").

Input: the JSON lines of `tools/gpu.sh bytes` over the product build and
six diagnostic builds of the same source (tools/build_var.sh; wrong codes
by design, AB_NOCHECK=1), each removing one class of traffic:
  notail   the entries' 32-B tail records neither stored nor read
  onee     every chain fetch reads row 0 of table 0 (L2-resident)
  nostore  the table stores skipped (the math kept)
  comb1    one comb addition instead of eleven
  nohand   no hand-off, partial-sum or check-code traffic between the phases
  noarena  phase A reads no descriptor and no arena byte
Measured bytes per verify = (2 FETCH_SIZE + WRITE_SIZE) x 1024 / n
(MI355X_MICROARCH.md: FETCH_SIZE tallies 128-B requests at 64 B).  Every
class is the product's bytes minus one diagnostic build's (the main-record
reads: onee's delta minus notail's); nothing is defined as a residual, so
the classes' sum against the counters' total is a check, and what is left
over is reported as "unattributed" (the status / window-count bytes, the
codes out, kernel arguments).  Algorithmic bytes come from the kernel's
layout and the digit distribution of the batch's scalars.

  python3 tools/byte_ledger.py bytes_ledger.jsonl [--n 65536] [--out ledger.json]

The builds (tools/bin is scratch; rebuild them from the tree):
  tools/build_var.sh prod6="" notail6="-DFD_DIAG_VTAB_NO_TAIL" onee6="-DFD_DIAG_VTAB_ONE_ENTRY" \
      nostore6="-DFD_DIAG_NO_VTAB_STORE" comb1_6="-DFD_DIAG_COMB_POS=1" nohand6="-DFD_DIAG_NO_HAND" \
      noarena6="-DFD_DIAG_NO_ARENA"
  gpurun ... 'AB_NOCHECK=1 TAG=ledger tools/gpu.sh bytes tools/bin/libvar_{prod6,notail6,onee6,nostore6,comb1_6,nohand6,noarena6}.so'
"""
import argparse
import json

ap = argparse.ArgumentParser()
ap.add_argument("jsonl")
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--out")
ap.add_argument("--fetches", type=float, default=66.6,
                help="table fetches per verify (2 per window; ~9 %% of waves run 34 windows)")
a = ap.parse_args()
rows = {}
for line in open(a.jsonl):
    d = json.loads(line)
    tag = d["tag"].replace("libvar_", "")
    rows[tag.rstrip("56").rstrip("_")] = d
n = a.n


def fb(d):    # corrected fetch bytes per verify
    return 2.0 * d["FETCH_SIZE"] * 1024.0 / n


def wb(d):
    return d["WRITE_SIZE"] * 1024.0 / n


p = rows["prod"]
F = a.fetches
p0 = F / 16.0           # digit 0 (biased nibble uniform over 16 values): the shared identity row
p1 = 3.0 * F / 16.0     # |d| <= 1: tails from the shared row (FD_OPT_TAIL1)
K = {"st": "table stores (16 x 128-B main + 14 x 32-B tail records; entry 1's tail is the shared zero tail)",
     "main": "table main-record reads (one 128-B line per fetch, zero digits from the shared row)",
     "tail": "table tail reads (32 B per fetch with |d| >= 2)",
     "comb": "comb reads (11 x 128-B entries)",
     "arena": "descriptor + arena reads (16 + 64 + 32 + 200 B)",
     "hand_r": "hand-off, partial-sum and check-code reads (phase B: 32 words, C: 25 words + 40-word sum + code)",
     "hand_w": "hand-off, partial-sum and check-code writes (phase A: 41 words, B: 40-word sum + code)"}
alg = {
    K["st"]: 2 * (8 * 128 + 7 * 32),
    K["main"]: (F - p0) * 128,
    K["tail"]: (F - p1) * 32,
    K["comb"]: 11 * 128,
    K["arena"]: 16 + 64 + 32 + 200,
    K["hand_r"]: 4 * (32 + 25 + 40) + 1,
    K["hand_w"]: 4 * (41 + 40) + 1,
}
meas = {
    K["st"]: wb(p) - wb(rows["nostore"]),
    K["main"]: (fb(p) - fb(rows["onee"])) - (fb(p) - fb(rows["notail"])),
    K["tail"]: fb(p) - fb(rows["notail"]),
    K["comb"]: (fb(p) - fb(rows["comb1"])) * 11.0 / 10.0,
    K["arena"]: fb(p) - fb(rows["noarena"]),
    K["hand_r"]: fb(p) - fb(rows["nohand"]),
    K["hand_w"]: wb(p) - wb(rows["nohand"]),
}
tot_m = fb(p) + wb(p)
unat = tot_m - sum(meas.values())
out = {"bytes_per_verify": {k: {"algorithmic": alg[k], "measured": meas[k], "ratio": meas[k] / alg[k]} for k in alg},
       "total": {"algorithmic": sum(alg.values()), "measured_sum_of_classes": sum(meas.values()),
                 "measured_2xFETCH_plus_WRITE": tot_m, "unattributed": unat,
                 "unattributed_frac": unat / tot_m,
                 "reconciles_within_5pct": abs(unat) <= 0.05 * tot_m},
       "builds": {k: {"FETCH_SIZE": v["FETCH_SIZE"], "WRITE_SIZE": v["WRITE_SIZE"], "dur_ms_median": v["dur_ms_median"],
                      "clock_ghz": v.get("clock_ghz")} for k, v in rows.items()},
       "note": "every class is a measured difference against one diagnostic build (no residual class); the tail "
               "class's notail delta is its reads only (FETCH); the store class is the nostore delta (all table "
               "stores, tails included); unattributed = the counters' total minus the classes' sum"}
s = json.dumps(out, indent=1)
print(s)
if a.out:
    open(a.out, "w").write(s + "\n")
