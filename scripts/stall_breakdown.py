#!/usr/bin/env python
"""Issue-slot breakdown of kernels from rocprofv3 PMC passes (scripts/gpu_pmc.sh; the SQ counters of
MI355X_MICROARCH.md 'rocprofv3 PMC slots'):

  SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready, not issued: the pipe
                   is busy or a dependency stalls it) + SQ_ACTIVE_INST_ANY (issuing)      [quad-cycles, per wave]

plus the instruction mix (VALU / SALU / LDS / SMEM / branch / VMEM counts), the VALU lane occupancy
(SQ_THREAD_CYCLES_VALU / 64 SQ_INSTS_VALU), waves resident per SIMD (4 SQ_WAVE_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8)) and the VALU cycles per SIMD-cycle at a per-form cost table (scripts/calib/valu_cost.hip).

    python scripts/stall_breakdown.py gpurun_out/r6a/stall_cfg4 profiles/round6/stall_cfg4.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402

SIMDS = 1024


def breakdown(cs):
    wc = cs.get("SQ_WAVE_CYCLES")
    if not wc:
        return None
    cyc = cs["GRBM_GUI_ACTIVE"] / 8.0   # per-XCD cycles of the dispatch (GRBM is summed over the 8 XCDs)
    e = {"cycles": int(cyc), "waves_per_simd": round(4.0 * wc / (SIMDS * cyc), 3),
         "wave_cycles_quad": int(wc)}
    parts = {"wait_any": cs.get("SQ_WAIT_ANY"), "wait_inst_any": cs.get("SQ_WAIT_INST_ANY"),
             "active_inst_any": cs.get("SQ_ACTIVE_INST_ANY")}
    if all(v is not None for v in parts.values()):
        e["frac_of_wave_cycles"] = {k: round(v / wc, 4) for k, v in parts.items()}
        e["frac_sum"] = round(sum(parts.values()) / wc, 4)
    if "SQ_WAIT_INST_LDS" in cs:
        e["wait_inst_lds_frac"] = round(cs["SQ_WAIT_INST_LDS"] / wc, 4)
    mix = {k[len("SQ_INSTS_"):].lower(): int(v) for k, v in cs.items() if k.startswith("SQ_INSTS_")}
    if mix:
        e["instructions"] = mix
    act = {k[len("SQ_ACTIVE_INST_"):].lower(): int(v) for k, v in cs.items() if k.startswith("SQ_ACTIVE_INST_")}
    if act:
        e["active_inst_quad_cycles"] = act
    if cs.get("SQ_INSTS_VALU"):
        v = cs["SQ_INSTS_VALU"]
        e["valu_per_simd_cycle"] = round(v / (SIMDS * cyc), 4)
        if cs.get("SQ_ACTIVE_INST_VALU"):
            e["active_valu_cycles_per_instr"] = round(4.0 * cs["SQ_ACTIVE_INST_VALU"] / v, 3)
            # VALU-pipe occupancy if each VALU instruction holds its SIMD for that many cycles
            e["valu_busy_frac_if_serial"] = round(4.0 * cs["SQ_ACTIVE_INST_VALU"] / (SIMDS * cyc), 4)
        if cs.get("SQ_THREAD_CYCLES_VALU"):
            e["valu_exec_lanes_per_instr"] = round(cs["SQ_THREAD_CYCLES_VALU"] / v, 2)
    return e


def main(src, dst):
    s = summarise(src)
    out = {}
    for k, cs in s.items():
        b = breakdown(cs)
        if b:
            out[k.split("::")[-1].split("(")[0]] = b
    out["_source"] = src
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    if len(sys.argv) != 3:
        sys.exit(__doc__)
    main(sys.argv[1], sys.argv[2])
