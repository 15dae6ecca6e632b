"""byte_ledger.py -- the pipe kernel's HBM byte ledger per verify, reconciled
with the PMC counters ("Byte ledger").

Input: the JSON lines of `tools/gpu.sh bytes` over the product build and
four diagnostic builds of the same source (tools/build_var.sh; wrong codes
by design, AB_NOCHECK=1), each removing one class of traffic:
  notail   the entries' 32-B tail records neither stored nor read
  onee     every chain fetch reads row 0 of table 0 (L2-resident)
  nostore  the table stores skipped (the math kept)
  comb1    one comb addition instead of eleven
Measured bytes per verify = (2 FETCH_SIZE + WRITE_SIZE) x 1024 / n
(MI355X_MICROARCH.md: FETCH_SIZE tallies 128-B requests at 64 B).  Each
class's measured bytes are the product's minus the diagnostic build's;
the remainder (arena, hand-offs, partial sums, codes) is what onee + comb1
leave.  Algorithmic bytes come from the kernel's layout
and the digit distribution of the batch's scalars.

  python3 tools/byte_ledger.py bytes_ledger.jsonl [--n 65536] [--out ledger.json]

The builds (tools/bin is scratch; rebuild them from the tree):
  tools/build_var.sh prod5="" notail5="-DFD_DIAG_VTAB_NO_TAIL" \
      onee5="-DFD_DIAG_VTAB_ONE_ENTRY" nostore5="-DFD_DIAG_NO_VTAB_STORE" comb1_5="-DFD_DIAG_COMB_POS=1"
  gpurun ... 'AB_NOCHECK=1 TAG=ledger tools/gpu.sh bytes tools/bin/libvar_{prod5,notail5,onee5,nostore5,comb1_5}.so'
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
    rows[tag.rstrip("5").rstrip("_")] = d
n = a.n


def fb(d):    # corrected fetch bytes per verify
    return 2.0 * d["FETCH_SIZE"] * 1024.0 / n


def wb(d):
    return d["WRITE_SIZE"] * 1024.0 / n


p = rows["prod"]
F = a.fetches
p0 = F / 16.0           # digit 0 (biased nibble uniform over 16 values): the shared identity row
p1 = 3.0 * F / 16.0     # |d| <= 1: tails from the shared row (FD_OPT_TAIL1)
alg = {
    "table stores (16 x 128-B main + 14 x 32-B tail records; entry 1's tail is the shared zero tail)":
        2 * (8 * 128 + 7 * 32),
    "table main-record reads (one 128-B line per fetch, zero digits from the shared row)": (F - p0) * 128,
    "table tail reads (32 B per fetch with |d| >= 2)": (F - p1) * 32,
    "comb reads (11 x 128-B entries)": 11 * 128,
    "arena + descriptor (16 + 64 + 32 + 200 B), hand-off / partial-sum / code reads": 16 + 64 + 32 + 200 + 4 * (8 + 8 + 16 + 24 + 2) + 160 + 2,
    "hand-off / partial-sum / code writes": 4 * 41 + 1 + 160 + 1 + 1,
}
meas = {
    "table stores (16 x 128-B main + 14 x 32-B tail records; entry 1's tail is the shared zero tail)":
        wb(p) - wb(rows["nostore"]),
    "table main-record reads (one 128-B line per fetch, zero digits from the shared row)":
        (fb(p) - fb(rows["onee"])) - (fb(p) - fb(rows["notail"])),
    "table tail reads (32 B per fetch with |d| >= 2)": fb(p) - fb(rows["notail"]),
    "comb reads (11 x 128-B entries)": (fb(p) - fb(rows["comb1"])) * 11.0 / 10.0,
    "arena + descriptor (16 + 64 + 32 + 200 B), hand-off / partial-sum / code reads":
        fb(rows["onee"]) - (fb(p) - fb(rows["comb1"])) * 11.0 / 10.0,
    "hand-off / partial-sum / code writes": wb(rows["nostore"]),
}
tot_m = fb(p) + wb(p)
out = {"bytes_per_verify": {k: {"algorithmic": alg[k], "measured": meas[k], "ratio": meas[k] / alg[k]} for k in alg},
       "total": {"algorithmic": sum(alg.values()), "measured_sum_of_classes": sum(meas.values()),
                 "measured_2xFETCH_plus_WRITE": tot_m},
       "builds": {k: {"FETCH_SIZE": v["FETCH_SIZE"], "WRITE_SIZE": v["WRITE_SIZE"], "dur_ms_median": v["dur_ms_median"],
                      "clock_ghz": v.get("clock_ghz")} for k, v in rows.items()},
       "note": "the tail class's notail delta also removes its 14 x 32-B stores from WRITE; the store class is the "
               "nostore delta (all table stores, tails included)"}
s = json.dumps(out, indent=1)
print(s)
if a.out:
    open(a.out, "w").write(s + "\n")
