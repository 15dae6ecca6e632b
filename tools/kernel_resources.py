#!/usr/bin/env python3
"""Per-kernel resource / occupancy report from the built code object's metadata.

Reads the amdhsa kernel metadata the assembler embeds (firedancer_amd/build/prod/
kern.opt.s, the exact code the library ships) and derives, per kernel, the
occupancy limits on gfx950: 512 VGPRs per lane per SIMD (unified arch + acc file,
allocation granule 8), 160 KB of LDS per CU, at most 8 waves per SIMD.  With the
SQ counters of profiles/r02/pmc_sq.json it adds the achieved mean waves per SIMD
of the profiled verify launch (SQ_WAVE_CYCLES counts quad-cycles).

  KR_ASM=<kern.opt.s> python3 tools/kernel_resources.py [out.json]   (default asm: the prod build,
                                                                   default out: /dev/stdout only; pass a path to write one)
"""
import json
import os
import sys

import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.environ.get('KR_ASM') or os.path.join(REPO, 'firedancer_amd', 'build', 'prod', 'kern.opt.s')
VGPR_FILE, VGPR_GRANULE, LDS_CU, MAX_WAVES, SIMDS_PER_CU, CUS = 512, 8, 160 * 1024, 8, 4, 256


def metadata(path):
    s = open(path).read()
    a = s.index(".amdgpu_metadata") + len(".amdgpu_metadata")
    b = s.index(".end_amdgpu_metadata", a)
    doc = s[a:b].split("\n...")[0]   # the YAML document ends at its "..." marker
    return yaml.safe_load(doc)["amdhsa.kernels"]


def limits(k):
    vg = k[".vgpr_count"] + k.get(".agpr_count", 0)
    vg_alloc = -(-vg // VGPR_GRANULE) * VGPR_GRANULE
    waves_vgpr = min(MAX_WAVES, VGPR_FILE // vg_alloc)
    wg = k[".max_flat_workgroup_size"]
    waves_per_wg = -(-wg // 64)
    lds = k[".group_segment_fixed_size"]
    wg_per_cu_lds = LDS_CU // lds if lds else None
    waves_lds = (wg_per_cu_lds * waves_per_wg) / SIMDS_PER_CU if lds else None
    lim = waves_vgpr if waves_lds is None else min(waves_vgpr, waves_lds)
    return {"vgpr": k[".vgpr_count"], "agpr": k.get(".agpr_count", 0), "vgpr_alloc": vg_alloc,
            "vgpr_spill": k.get(".vgpr_spill_count", 0), "sgpr": k[".sgpr_count"],
            "scratch_bytes": k[".private_segment_fixed_size"], "lds_bytes": lds,
            "workgroup": wg, "max_waves_per_simd_by_vgpr": waves_vgpr,
            "max_waves_per_simd_by_lds": waves_lds, "max_waves_per_simd": lim}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    if out is not None and not out.endswith(".json"):
        sys.exit("kernel_resources.py: the argument is the OUTPUT .json (the asm comes from KR_ASM or the prod build)")
    bid = os.path.join(os.path.dirname(ASM), "fd_build_id.h")
    build = None
    if os.path.exists(bid):
        t = open(bid).read().split('"')[1]
        build = dict(kv.split("=", 1) for kv in t.split())
    rep = {"source": os.path.relpath(ASM, REPO), "build": build, "model": "gfx950: 512 VGPRs/SIMD lane, granule 8; "
           "160 KB LDS/CU; 8 waves/SIMD; 4 SIMDs/CU; 256 CUs", "kernels": {}}
    for k in metadata(ASM):
        rep["kernels"][k[".name"]] = limits(k)
    pmc = os.environ.get("KR_PMC", "")          # a pmc_sq.json for the achieved waves per SIMD
    if pmc and os.path.exists(pmc):
        p = json.load(open(pmc))
        cyc = p["dur_ns"] * 1e-9 * p["effective_clock_ghz"] * 1e9
        rep["achieved"] = {
            "kernel": p["kernel"], "grid": p["grid"], "dur_ns": p["dur_ns"],
            "mean_waves_per_simd": 4.0 * p["SQ_WAVE_CYCLES"] / (cyc * SIMDS_PER_CU * CUS),
            "note": "SQ_WAVE_CYCLES (quad-cycles x4) / (launch cycles at the GRBM clock x 1,024 SIMDs); "
                    "config 2 pipelined = three waves per SIMD (phases A, B, C of three batches)",
        }
    if out:
        json.dump(rep, open(out, "w"), indent=1)
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
