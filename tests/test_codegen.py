"""Generated-code checks on the built gfx950 code object (CPU only: disassembly, no GPU).

`fmac_bcast` in csrc/gsd_render.hip is hand-written inline asm (`v_fmac_f32_dpp ... row_newbcast`).  LLVM's hazard
recognizer does not look inside inline asm, and gfx9-family VALUs need two wait states between a VALU write of a
VGPR and a DPP read of it (the DPP source is src0).  The kernel is only correct if the compiler never places a VALU
write of the asm's src0 in the two instructions before it, so this test disassembles the library's render object
and checks every `v_fmac_f32_dpp`:
  - walking back from it, the instructions that supply its two wait states (an `s_nop N` supplies N + 1) must not
    be VALU instructions whose destination covers src0;
  - neither it nor the instruction before it may be a branch target (a predecessor off the straight line would
    escape the walk).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "gaussian-splatting_deformable_amd", "build", "obj", "gsd_render.o")
LLVM = "/opt/rocm/lib/llvm/bin"

_INSN = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>\s*$")


def _disassemble(tmp_path):
    fb, co = str(tmp_path / "fb.bin"), str(tmp_path / "dev.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", OBJ, str(tmp_path / "o")])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}",
                           "--unbundle"])
    return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", co], text=True)


def _regs(tok):
    """VGPR numbers named by an operand token: v7 -> {7}, v[6:7] -> {6, 7}; others -> empty."""
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _parse(text):
    insns, targets, funcs = [], set(), {}
    for line in text.splitlines():
        f = _FUNC.match(line)
        if f:
            funcs[f.group(2)] = int(f.group(1), 16)
            continue
        m = _INSN.match(line)
        if not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        insns.append((addr, op, [a.strip() for a in args.split(",")] if args else []))
        if op.startswith(("s_branch", "s_cbranch")):
            t = _TARGET.search(line)
            if t and t.group(1) in funcs:
                targets.add(funcs[t.group(1)] + int(t.group(2), 16))
    return insns, targets


def _hazards(insns, targets):
    bad, n_checked = [], 0
    for i, (addr, op, args) in enumerate(insns):
        if op != "v_fmac_f32_dpp":
            continue
        n_checked += 1
        src0 = _regs(args[1])
        if addr in targets or (i > 0 and insns[i - 1][0] in targets):
            bad.append((hex(addr), "branch target inside the wait-state window"))
            continue
        waits, j = 0, i - 1
        while waits < 2 and j >= 0:
            _, pop, pargs = insns[j]
            if pop == "s_nop":
                waits += int(pargs[0], 0) + 1
            else:
                if pop.startswith("v_") and pargs and _regs(pargs[0]) & src0:
                    bad.append((hex(addr), f"{pop} {', '.join(pargs)} writes src0 {args[1]}"))
                waits += 1
            j -= 1
    return bad, n_checked


@pytest.mark.skipif(not os.path.exists(OBJ), reason="library not built (build() / make -C .../csrc)")
@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-objdump"), reason="ROCm LLVM tools absent")
def test_fmac_dpp_source_hazard(tmp_path):
    insns, targets = _parse(_disassemble(tmp_path))
    bad, n = _hazards(insns, targets)
    assert n > 0, "no v_fmac_f32_dpp found: k_render_bwd no longer uses fmac_bcast (drop this test with it)"
    assert not bad, bad


def test_hazard_checker_flags_a_valu_write():
    """The checker itself: a VALU write of src0 one or two instructions ahead is a hazard, an s_nop 1 clears it."""
    mk = lambda a, op, args: (a, op, args)  # noqa: E731
    fm = ["v80", "v7", "v18", "row_newbcast:0"]
    seq = [mk(0, "v_mov_b32_e32", ["v7", "v3"]), mk(4, "v_mul_f32_e32", ["v9", "v9", "v9"]), mk(8, "v_fmac_f32_dpp", fm)]
    assert _hazards(seq, set())[0]
    seq = [mk(0, "v_mov_b32_e32", ["v[6:7]", "v[2:3]"]), mk(8, "v_fmac_f32_dpp", fm)]
    assert _hazards(seq, set())[0]
    seq = [mk(0, "v_mov_b32_e32", ["v7", "v3"]), mk(4, "s_nop", ["1"]), mk(8, "v_fmac_f32_dpp", fm)]
    assert not _hazards(seq, set())[0]
    seq = [mk(0, "ds_read_b128", ["v[4:7]", "v1"]), mk(4, "v_add_f32_e32", ["v9", "v9", "v9"]),
           mk(8, "v_fmac_f32_dpp", fm)]
    assert not _hazards(seq, set())[0]
    assert _hazards(seq, {8})[0]
