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


def _disassemble(tmp_path, obj=None):
    fb, co = str(tmp_path / "fb.bin"), str(tmp_path / "dev.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", obj or OBJ,
                           str(tmp_path / "o")])
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


# ---- the deformation network's LDS-DMA rings: every counted wait retires the copies its k-step reads ----
# The layer-fused kernels (gsd_mlp_train.hip) copy each k-step's weight fragments global -> LDS with inline-asm
# `global_load_lds_dwordx4` (invisible to the compiler) a fixed number of k-steps ahead, and end each k-step with
# `s_waitcnt vmcnt(N)` + `s_barrier`, N = the VMEM operations the source says were issued after the copies of the next
# k-step.  vmcnt retires in issue order, so the wait is safe iff at least N VMEM operations (copies, stores, loads,
# scratch -- all count) follow the last copy of the next k-step.  An operation the compiler merges or drops would make
# N too large and the barrier could pass with a slot still in flight.  This walks each ring phase of the built code
# (a phase ends at a full drain, vmcnt(0) + barrier): its copies, in issue order, are grouped per k-step (the size of
# a group: the copies between the phase's first and second counted waits), the phase's i-th counted wait needs group
# i (the prologue's wait needs k-step 0; k-step t's wait needs t + 1), and the count after that group's last copy
# must be >= N.  Loops (`#pragma unroll 1` over layers) appear once in the text; their k-steps issue the same
# operations on every iteration, so the text order is the issue order at every k-step boundary.
# (k_mlp_bwd_chain is not walked: its enc(x) pass starts a second ring without a drain, its copies younger than the
# main ring's prefetched ones, which this phase model does not describe; the 16-wide chain drains first)
_RING_KERNELS = ("_ZN3gsd15k_mlp_fwd_fusedILb1EEEvNS_14MlpFusedParamsE",
                 "_ZN3gsd15k_mlp_fwd_fusedILb0EEEvNS_14MlpFusedParamsE",
                 "_ZN3gsd17k_mlp_fwd_fused16ILb1EEEvNS_14MlpFusedParamsE",
                 "_ZN3gsd17k_mlp_fwd_fused16ILb0EEEvNS_14MlpFusedParamsE",
                 "_ZN3gsd17k_mlp_bwd_chain16ENS_14MlpChainParamsE")


def _kernel_insns(text, name):
    out, on = [], False
    for line in text.splitlines():
        f = _FUNC.match(line)
        if f:
            on = f.group(2) == name
            continue
        if on:
            m = _INSN.match(line)
            if m:
                out.append((m.group(1), m.group(2)))
    return out


def _vmcnt(op, args):
    if op != "s_waitcnt":
        return None
    m = re.search(r"vmcnt\((\d+)\)", args)
    return int(m.group(1)) if m else None


def _ring_violations(insns):
    """(index of the wait, N, VMEM ops after the needed copy) for every counted wait that does not retire its
    k-step's copies; plus the number of counted waits checked."""
    is_vmem = [op.startswith(("global_", "buffer_", "scratch_", "flat_")) for op, _ in insns]
    bad, checked = [], 0
    copies, waits = [], []   # the current phase's copy indices and counted waits (index, N)

    def close_phase():
        nonlocal checked
        if len(waits) < 2:
            return
        c = sum(1 for i in copies if waits[0][0] < i < waits[1][0])   # copies per k-step
        if c == 0:
            return
        for wi, (w, n) in enumerate(waits):
            grp = copies[wi * c: (wi + 1) * c]
            if len(grp) < c:   # the phase's tail: no copy group left to wait for
                break
            after = sum(1 for j in range(grp[-1] + 1, w) if is_vmem[j])
            checked += 1
            if after < n:
                bad.append((w, n, after))

    for i, (op, args) in enumerate(insns):
        if op == "global_load_lds_dwordx4":
            copies.append(i)
        n = _vmcnt(op, args)
        if n is None:
            continue
        # a counted wait or a drain: an s_barrier follows before any other memory operation
        barrier = False
        for o, a in insns[i + 1: i + 13]:
            if o == "s_barrier":
                barrier = True
                break
            if o.startswith(("global_", "buffer_", "scratch_", "flat_", "ds_")) or _vmcnt(o, a) is not None:
                break
        if not barrier:
            continue
        if n == 0:   # a drain: the phase ends here
            close_phase()
            copies, waits = [], []
        else:
            waits.append((i, n))
    close_phase()
    return bad, checked


CSRC = os.path.join(ROOT, "gaussian-splatting_deformable_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _check_build(tmp_path):
    """gsd_mlp_train.hip as the product compiles it, plus GSD_MLP_UNROLL_LAYERS: the layer loops unrolled, so the text
    order is the issue order (the product's `#pragma unroll 1` loops may be laid out rotated, which a text walk cannot
    follow); the k-steps, their operations and their counted waits are the same source."""
    obj = str(tmp_path / "mlp_check.o")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
                           "-fhip-fp32-correctly-rounded-divide-sqrt", "-DGSD_MLP_UNROLL_LAYERS", "-I", CSRC,
                           "-c", os.path.join(CSRC, "gsd_mlp_train.hip"), "-o", obj])
    return _disassemble(tmp_path, obj)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc absent")
@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-objdump"), reason="ROCm LLVM tools absent")
def test_mlp_ring_waits_retire_their_copies(tmp_path):
    text = _check_build(tmp_path)
    for name in _RING_KERNELS:
        insns = _kernel_insns(text, name)
        assert insns, f"{name} not in the object"
        bad, checked = _ring_violations(insns)
        assert checked >= 60, (name, checked)
        assert not bad, (name, bad[:5])


def test_ring_checker_flags_an_under_counted_wait():
    """The checker itself: a prologue of two 2-copy k-steps, then k-steps of 2 copies + 1 store; k-step t's wait may
    count the ops after k-step t + 1's copies (3: its store, then k-step t + 1's... in issue order) and no more."""
    def seq(n_end):
        s = [("global_load_lds_dwordx4", "")] * 4 + [("s_waitcnt", "vmcnt(2)"), ("s_barrier", "")]
        for _ in range(4):
            s += [("global_load_lds_dwordx4", "")] * 2 + [("global_store_dword", ""), ("s_waitcnt", f"vmcnt({n_end})"),
                                                          ("s_barrier", "")]
        return s + [("s_waitcnt", "vmcnt(0)"), ("s_barrier", "")]
    assert not _ring_violations(seq(3))[0]
    assert _ring_violations(seq(4))[0]
