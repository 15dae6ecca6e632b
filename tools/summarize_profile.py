#!/usr/bin/env python3
"""summarize_profile.py -- turn a `tools/gpu.sh profile` output directory
(gpurun_out/prof_<tag>) into the committed summaries under profiles/<tag>/:

  kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (verbatim)
  bench.json          the bench.py line of the same tree (un-profiled run)
  bench_driver_form.json  the same in the driver's form (--steps 20 --warmup 5), if run
  build.json          the library's build id (code-object hash + git) every file here is keyed to
  pmc_traffic.json    HBM bytes per verify-kernel launch from separate
                      FETCH_SIZE / WRITE_SIZE passes, with the gfx950
                      correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE x 2
                      for 16-B/lane reads; WRITE_SIZE as is)
  pmc_sq.json         SQ counters per launch and per wave (VALU instructions,
                      wave cycles, waits), GRBM_GUI_ACTIVE effective clock
  issue_probe.json    tools/issue_probe.hip output (per-instruction issue cost)

Usage: summarize_profile.py gpurun_out/prof_r01 profiles/r01
"""
import csv
import json
import os
import shutil
import statistics
import sys


VERIFY_KERNELS = ("fd_ed25519_verify_pipe_kernel", "fd_ed25519_verify_pair_kernel", "fd_ed25519_verify_kernel")


def verify_kernel(path):
    """The verify kernel the profiled bench launched (config 2: the pipe kernel by default)."""
    names = {r["Kernel_Name"] for r in csv.DictReader(open(path))}
    return next(k for k in VERIFY_KERNELS if k in names)


def pmc(path, kernel=None):
    kernel = kernel or verify_kernel(path)
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"] == kernel]
    by = {}
    for r in rows:
        d = by.setdefault(r["Dispatch_Id"], {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                             "grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                                             "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"])})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(by.values())


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    json.dump(bench, open(os.path.join(dst, "bench.json"), "w"))
    n = bench["config"]["batch_per_gpu"]
    build = bench.get("build")
    drv = os.path.join(src, "bench_driver_form.json")
    if os.path.exists(drv):
        d = json.loads(open(drv).read().strip().splitlines()[-1])
        assert d.get("build") == build, "driver-form bench ran a different build"
        json.dump(d, open(os.path.join(dst, "bench_driver_form.json"), "w"))
    json.dump(build, open(os.path.join(dst, "build.json"), "w"))

    fe = pmc(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"))
    wr = pmc(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"))
    fetch_kb = statistics.median(d["FETCH_SIZE"] for d in fe)
    write_kb = statistics.median(d["WRITE_SIZE"] for d in wr)
    hbm = (2.0 * fetch_kb + write_kb) * 1024.0
    traffic = {
        "build": build,
        "batch": n, "kernel": verify_kernel(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv")),
        "launches": len(fe),
        "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
        "hbm_bytes_per_launch": hbm, "hbm_bytes_per_verify": hbm / n,
        "note": "HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024, medians over the profiled launches of "
                "separate --pmc passes; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B "
                "requests at 64 B; the kernel's dominant reads are 16-B/lane table loads)",
    }
    json.dump(traffic, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)

    def mid(rows):   # a steady-state launch (a pipelined run's last launches drain it)
        return rows[len(rows) // 2]
    sq = mid(pmc(os.path.join(src, "pmc_sq", "pmc_counter_collection.csv")))
    gr = mid(pmc(os.path.join(src, "pmc_grbm", "pmc_counter_collection.csv")))
    iss_path = os.path.join(src, "pmc_issue", "pmc_counter_collection.csv")
    iss = mid(pmc(iss_path)) if os.path.exists(iss_path) else None
    waves = sq["SQ_WAVES"]
    out = {k: v for k, v in sq.items()}
    out.update({
        "build": build,
        "kernel": verify_kernel(os.path.join(src, "pmc_sq", "pmc_counter_collection.csv")),
        "valu_instr_per_wave": sq["SQ_INSTS_VALU"] / waves,
        "valu_instr_per_64_sigs": sq["SQ_INSTS_VALU"] / (n / 64.0),
        "wave_cycles_per_wave": 4.0 * sq["SQ_WAVE_CYCLES"] / waves,
        "wait_any_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
        "cycles_per_valu_instr": 4.0 * sq["SQ_WAVE_CYCLES"] / sq["SQ_INSTS_VALU"],
        "GRBM_GUI_ACTIVE": gr.get("GRBM_GUI_ACTIVE"),
        "effective_clock_ghz": gr.get("GRBM_GUI_ACTIVE", 0) / 8.0 / gr["dur_ns"],
        "note": "SQ_WAVE_CYCLES / SQ_WAIT_ANY count quad-cycles (x4 = cycles); the pipe kernel runs three "
                "waves per 64 signatures per launch (phases A, B, C of three batches), the pair kernel two (one "
                "exits after the decodes), the single-lane kernel one",
    })
    if iss:
        out["issue"] = {k: v for k, v in iss.items() if k.startswith("SQ_")}
        busy = iss.get("SQ_BUSY_CU_CYCLES")
        if busy:
            # per SIMD: VALU instructions per busy cycle (SQ_BUSY_CU_CYCLES: quad-cycles per CU, summed)
            out["issue"]["valu_instr_per_simd_cycle"] = iss["SQ_INSTS_VALU"] / (4.0 * busy * 4.0)
            out["issue"]["dual_issue_frac"] = iss.get("SQ_ACTIVE_INST_VALU2", 0) / max(iss.get("SQ_ACTIVE_INST_VALU", 1), 1)
    json.dump(out, open(os.path.join(dst, "pmc_sq.json"), "w"), indent=1)

    ip = os.path.join(src, "issue_probe.jsonl")
    if os.path.exists(ip):
        probes = [json.loads(l) for l in open(ip) if l.startswith("{")]
        json.dump({"tool": "tools/issue_probe.hip", "probes": probes}, open(os.path.join(dst, "issue_probe.json"), "w"),
                  indent=1)
    print(json.dumps({"bench": bench["value"], "kernel_ms": bench["roofline"]["kernel_ms"],
                      "hbm_bytes_per_launch": hbm, "valu_instr_per_64_sigs": out["valu_instr_per_64_sigs"],
                      "cycles_per_valu_instr": out["cycles_per_valu_instr"]}))


if __name__ == "__main__":
    main()
