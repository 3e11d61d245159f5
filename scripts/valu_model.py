#!/usr/bin/env python
"""VALU-cycle model of k_render_bwd's walk (round 6): is the kernel's time its VALU issue?

Disassembles the built render object (build/obj/gsd_render.o), takes the no-background walk's first hand-off of
k_render_bwd<false> -- the four per-record phase-1 steps (the `row_newbcast:0..3` DPP forms) and the phase-2 block
that follows up to the hand-off's `ds_add_f64`s -- classifies every VALU instruction by its encoding form and prices
it with the per-form costs calibrated on the MI355X at five waves per SIMD (scripts/calib/valu_cost.hip,
profiles/round6/calib/valu_cost.txt).  With the counted wave steps of the bench scene (GSD_COUNT_WORK,
profiles/round5/work_counts_cfg4.json) that gives the VALU cycles per SIMD the walk needs, against the kernel's
measured duration in cycles (PMC GRBM_GUI_ACTIVE / 8, profiles/round6/stall_cfg4/stall_breakdown.json).

    python scripts/valu_model.py [--json out.json]
"""
import argparse
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "gaussian-splatting_deformable_amd", "build", "obj", "gsd_render.o")
LLVM = "/opt/rocm/lib/llvm/bin"
CALIB = os.path.join(ROOT, "profiles", "round6", "calib", "valu_cost.txt")


def calib(waves=5):
    """form name -> cycles per wave64 instruction at `waves` per SIMD."""
    out = {}
    for line in open(CALIB):
        m = re.match(r"(.+?)\s+waves/SIMD (\d+): ([\d.]+) cycles/instr", line)
        if m and int(m.group(2)) == waves:
            out[m.group(1).strip()] = float(m.group(3))
    return out


def disasm():
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", OBJ, os.path.join(d, "o")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                               f"--input={fb}", f"--output={co}", "--unbundle"])
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", co], text=True)


def kernel_lines(text, mangled):
    out, on = [], False
    for line in text.splitlines():
        if line.endswith(f"<{mangled}>:"):
            on = True
            continue
        if on:
            if not line.strip():
                break
            m = re.match(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//", line)
            if m:
                out.append((m.group(1), m.group(2)))
    return out


def form(op, args):
    """The calibration row an instruction is priced by (None: not a VALU instruction)."""
    if not op.startswith("v_"):
        return None
    if op in ("v_exp_f32_e32", "v_exp_f32"):
        return "v_exp_f32"
    if op in ("v_rcp_f32_e32", "v_rcp_f32"):
        return "v_rcp_f32"
    if "row_newbcast" in args:
        if op.startswith("v_mov"):
            return "v_mov_b32_dpp newbcast"
        if op.startswith("v_fmac"):
            return "v_fmac_f32_dpp newbcast"
        if op.startswith(("v_sub", "v_subrev")):
            return "v_sub_f32_dpp newbcast"
        return "v_mul_f32_dpp newbcast"
    if "row_ror" in args or "quad_perm" in args or "_dpp" in op:
        return "v_add_f32_dpp row_ror:8"
    if op.startswith("v_cmp"):
        return "v_cmp_ngt_f32_e64 s,0,v" if "f32" in op else "v_cmp_gt_i32_e64 s,v,v"
    if op.startswith("v_cndmask"):
        return "v_cndmask_b32_e64 0,v,s"
    if op.startswith("v_fmamk") or op.startswith("v_fmaak"):
        return "v_fmamk_f32 lit"
    if "0x" in args:   # a 32-bit literal: an 8-byte instruction
        return "v_min_f32_e32 lit,v"
    if op.endswith("_e64") or op.startswith(("v_fma_", "v_mad", "v_cvt_f64", "v_lshl_add", "v_add3", "v_bfe")):
        return "v_fma_f32 v,v,v"
    if op.startswith("v_fmac"):
        return "v_fmac_f32_e32 v,v"
    if op.startswith("v_mul"):
        return "v_mul_f32_e32 v,v"
    return "v_add_f32_e32 v,v"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    cost = calib(5)
    lines = kernel_lines(disasm(), "_ZN3gsd12k_render_bwdILb0EEEvNS_15RenderBwdParamsE")
    # the no-background walk is the second copy of the loop: take the first hand-off whose phase 1 has no background
    # FMA -- locate every `row_newbcast:0` step start and take the last one (the kBg = false instantiation is later)
    starts = [i for i, (op, args) in enumerate(lines) if op.startswith("v_sub_f32_dpp") and "row_newbcast:0 " in args]
    i0 = starts[-1]
    # the hand-off ends at its third ds_add_f64
    n_add, i1 = 0, i0
    while i1 < len(lines) and n_add < 3:
        n_add += lines[i1][0] == "ds_add_f64"
        i1 += 1
    block = lines[i0:i1]
    p2 = next(i for i, (op, _) in enumerate(block) if op.startswith("ds_read"))  # phase 2 starts at its reads
    def price(seg):
        n, cyc, by = 0, 0.0, {}
        for op, args in seg:
            f = form(op, args)
            if f is None:
                continue
            n += 1
            cyc += cost[f]
            by[f] = by.get(f, 0) + 1
        return n, cyc, by
    n1, c1, by1 = price(block[:p2])
    n2, c2, by2 = price(block[p2:])
    wc = json.load(open(os.path.join(ROOT, "profiles", "round5", "work_counts_cfg4.json")))["render_bwd"]
    sb = json.load(open(os.path.join(ROOT, "profiles", "round6", "stall_cfg4", "stall_breakdown.json")))["k_render_bwd"]
    steps = wc["wave_record_steps"]
    hand_offs = steps / 4.0            # an upper bound: a hand-off no lane took skips phase 2
    walk_cycles = (steps * c1 / 4.0 + hand_offs * c2) / 1024.0   # per SIMD
    res = {"phase1_per_step": {"valu": n1 / 4.0, "cycles": round(c1 / 4.0, 1)},
           "phase2_per_hand_off": {"valu": n2, "cycles": round(c2, 1)},
           "forms_phase1_per_4_steps": by1, "forms_phase2": by2,
           "wave_steps": steps, "walk_valu_cycles_per_simd": int(walk_cycles),
           "kernel_cycles": sb["cycles"], "walk_share_of_kernel": round(walk_cycles / sb["cycles"], 3),
           "pmc_valu_per_wave_step": round(sb["instructions"]["valu"] / steps, 1),
           "model_valu_per_wave_step_walk": round((n1 / 4.0) + n2 / 4.0, 1)}
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
