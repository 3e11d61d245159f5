#!/usr/bin/env python
"""HBM traffic per launch from rocprofv3 PMC passes (scripts/gpu_pmc.sh with FETCH_SIZE and WRITE_SIZE in
separate passes), corrected as /opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes for gfx950:
FETCH_SIZE (KB) reports half the bytes of wide coalesced reads -> doubled; WRITE_SIZE (KB) is taken as is.
Writes a JSON {kernel: {fetch_kb, write_kb, hbm_bytes, valu}, "_workload": W} that bench.py reads for
roofline.traffic and the VALU roof -- only for a bench run of the same workload W ("cfg4", "cfg5", ...).

    python scripts/pmc_traffic.py gpurun_out/pmc profiles/round3/pmc/cfg4/pmc_traffic.json cfg4
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402


def short(name):
    n = name.split("::")[-1]
    n = n.split("<")[0]
    return n[2:] if n.startswith("k_") else n


def main(src, dst, workload):
    s = summarise(src)
    out = {}
    for k, cs in s.items():
        if "FETCH_SIZE" not in cs and "WRITE_SIZE" not in cs:
            continue
        f, w = cs.get("FETCH_SIZE", 0.0), cs.get("WRITE_SIZE", 0.0)
        e = {"kernel": k, "fetch_kb": round(f, 1), "write_kb": round(w, 1),
             "hbm_bytes": int(round((2.0 * f + w) * 1024.0))}
        if "SQ_INSTS_VALU" in cs and cs.get("GRBM_GUI_ACTIVE"):
            # VALU issue rate: wave64 VALU instructions per SIMD-cycle over the dispatch (GRBM_GUI_ACTIVE is
            # summed over the 8 XCDs; 1024 SIMDs).  Peak 0.5: a wave64 v_fma_f32 every 2 cycles per SIMD with
            # more than one wave resident (MI355X_MICROARCH.md, per-instruction cycle table).
            cyc = cs["GRBM_GUI_ACTIVE"] / 8.0
            rate = cs["SQ_INSTS_VALU"] / (1024.0 * cyc)
            e["valu"] = {"instructions": int(cs["SQ_INSTS_VALU"]), "cycles": int(cyc),
                         "issue_per_simd_cycle": round(rate, 4), "peak": 0.5, "frac": round(rate / 0.5, 4)}
            if cs.get("SQ_WAVE_CYCLES"):
                e["valu"]["lds_issue_wait_frac"] = round(cs.get("SQ_WAIT_INST_LDS", 0.0) / cs["SQ_WAVE_CYCLES"], 4)
            if cs.get("SQ_ACTIVE_INST_VALU"):
                # raw: SQ_ACTIVE_INST_VALU (summed over waves; ~1 per VALU instruction on the render kernels)
                e["valu"]["active_inst_valu"] = int(cs["SQ_ACTIVE_INST_VALU"])
        out[short(k)] = e
    out["_workload"] = workload
    out["_note"] = (f"per-launch means over the profiled launches (scripts/prof_render.py, {workload}); FETCH_SIZE x2 "
                    "per the gfx950 calibration, WRITE_SIZE as is; gathers and atomics are uncalibrated widths; "
                    "valu: SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) against 0.5 per SIMD-cycle")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    if len(sys.argv) != 4:
        sys.exit("usage: pmc_traffic.py SRC_DIR DST_JSON WORKLOAD (e.g. cfg4)")
    main(sys.argv[1], sys.argv[2], sys.argv[3])
