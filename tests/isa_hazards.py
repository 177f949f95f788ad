"""Static wait-state checker for gfx950 code objects (used by tests/test_isa_hazards.py).

hipcc's hazard recognizer pads the instructions it generates, but treats an inline-asm statement as
one opaque instruction: it neither pads the hazards between the statement's own instructions nor,
for most rules, those between its instructions and the compiler's code on either side
(cdna_hip_programming.md section 5.7 item 2).  This module replays the producer -> consumer rules on
the disassembled instruction stream of a kernel, so a violation anywhere -- inside an asm block or at
its boundary -- is found.

The rule table is LLVM's own for gfx950, read off the compiler: every rule below is one that hipcc
was observed to pad in compiler-generated code (micro-kernels compiled for each producer / consumer
pair, and the shipped code object itself; the test checks that the whole compiler-generated part
of the library passes, which keeps the table from being stricter than the compiler).  Wait states
between two instructions are the instructions issued between them, an ``s_nop N`` counting N + 1.

    producer                        consumer (operand)                         wait states
    VALU writes SGPR / VCC          VALU reads it (mask, carry, constant)      2
    VALU writes SGPR / VCC          v_readlane / v_writelane lane select       4
    VALU writes SGPR                VMEM reads it (soffset, rsrc, saddr)       5
    VALU writes VCC                 v_div_fmas                                 4
    VALU writes EXEC                DPP                                        5
    VALU writes VGPR                DPP reads it as src0                       2
    VALU writes VGPR                v_readlane / v_readfirstlane src0          1
    v_pk_*_f32 writes VGPR          VALU reads it                              1
      (not after a producer with a cross-half op_sel / op_sel_hi: hipcc pads none there)
    v_writelane writes VGPR         VALU reads it                              1
    transcendental writes VGPR      non-transcendental VALU reads it           1
    v_dot* writes VGPR              VALU (other than a v_dot* srcC) or VMEM    3
    VMEM store, > 64-bit data       VALU writes a data VGPR                    2

Straight-line order is assumed: the window is cleared after an unconditional branch or s_endpgm
(the next instruction is reached only by a jump), and jumps into the middle of a window are not
followed.
"""
from __future__ import annotations

import os
import re
import subprocess
from dataclasses import dataclass, field

LLVM = "/opt/rocm/lib/llvm/bin"

_REG = re.compile(r"\b(v|s)\[(\d+):(\d+)\]|\b(v|s)(\d+)\b|\b(vcc_lo|vcc_hi|vcc|exec_lo|exec_hi|exec|m0)\b")
_TRANS = re.compile(r"^v_(sqrt|rsq|rcp|log|exp|sin|cos)(_iflag)?_(f16|f32|f64|bf16)")
_PKF32 = re.compile(r"^v_pk_(add|mul|fma|mov)_(f32|b32)")
_DOT = re.compile(r"^v_dot\d")
# a packed op whose lanes read across halves: a 1 in op_sel, or a 0 in op_sel_hi (the high lane reads
# a low half, e.g. a scalar broadcast from an SGPR pair); hipcc pads neither form
_OPSEL_LO = re.compile(r"\bop_sel:\[[^\]]*1|\bop_sel_hi:\[[^\]]*0")
_VMEM = re.compile(r"^(buffer|global|flat|scratch)_")
_DPP_MOD = re.compile(r"\b(quad_perm|row_shl|row_shr|row_ror|wave_shl|wave_shr|wave_rol|wave_ror|row_mirror|"
                      r"row_half_mirror|row_bcast|row_newbcast)\b")


def _regs(text: str) -> list[str]:
    out = []
    for m in _REG.finditer(text):
        if m.group(1):
            out += [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
        elif m.group(4):
            out.append(f"{m.group(4)}{m.group(5)}")
        else:
            r = m.group(6)
            out += {"vcc": ["vcc_lo", "vcc_hi"], "exec": ["exec_lo", "exec_hi"]}.get(r, [r])
    return out


def _sgpr_like(r: str) -> bool:
    return r.startswith("s") or r.startswith("vcc") or r.startswith("exec") or r == "m0"


@dataclass
class Ins:
    idx: int
    text: str
    op: str
    defs: list = field(default_factory=list)
    uses: list = field(default_factory=list)
    dpp_src0: list = field(default_factory=list)
    lane_sel: list = field(default_factory=list)
    srcc: list = field(default_factory=list)
    waits: int = 1

    @property
    def valu(self):
        return self.op.startswith("v_")

    @property
    def vmem(self):
        return bool(_VMEM.match(self.op))

    @property
    def dpp(self):
        return self.op.endswith("_dpp") or bool(_DPP_MOD.search(self.text))


def parse(line: str, idx: int) -> Ins:
    line = line.split("//")[0].strip()
    op, _, rest = line.partition(" ")
    ins = Ins(idx, line, op)
    if op == "s_nop":
        ins.waits = int(rest.strip(), 0) + 1
        return ins
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", rest)] if rest else []
    # modifiers after the last operand (op_sel:[..] wave_shr:1 offen ...) are not registers
    if ops:
        last = ops[-1].split()
        ops[-1] = last[0] if last else ""
    regs = [_regs(o) for o in ops]
    base = op.replace("_dpp", "").replace("_sdwa", "")
    if ins.vmem:
        if "load" in op and "lds" not in op and regs:
            ins.defs = regs[0]
            ins.uses = sum(regs[1:], [])
        else:
            ins.uses = sum(regs, [])
        return ins
    if op.startswith("s_"):
        if op.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_endpgm", "s_setprio", "s_sleep",
                          "s_trap", "s_sendmsg", "s_dcache", "s_icache", "s_setpc", "s_swappc")):
            ins.uses = sum(regs, [])
        else:
            ins.defs = regs[0] if regs else []
            ins.uses = sum(regs[1:], [])
            if op.startswith("s_cmp") or op.startswith("s_bitcmp"):
                ins.defs, ins.uses = [], sum(regs, [])
        return ins
    if op.startswith("ds_"):
        if ("read" in op or "load" in op or "bpermute" in op or "permute" in op) and regs:
            ins.defs, ins.uses = regs[0], sum(regs[1:], [])
        else:
            ins.uses = sum(regs, [])
        return ins
    if not ins.valu:
        ins.uses = sum(regs, [])
        return ins
    # VALU
    if base.startswith("v_cmpx"):
        ins.defs = ["exec_lo", "exec_hi"] + (regs[0] if base.endswith("_e64") and regs else [])
        ins.uses = sum(regs[1:] if base.endswith("_e64") else regs, [])
    elif base.startswith("v_cmp") and not base.endswith("_e64"):
        # llvm-objdump prints the implicit VCC destination first: "v_cmp_eq_u32_e32 vcc, v1, v2"
        srcs = regs[1:] if ops and ops[0] == "vcc" else regs
        ins.defs, ins.uses = ["vcc_lo", "vcc_hi"], sum(srcs, [])
    elif base.startswith("v_readlane") or base.startswith("v_readfirstlane"):
        ins.defs = regs[0]
        ins.uses = sum(regs[1:], [])
        ins.lane_sel = regs[2] if len(regs) > 2 else []
    elif base.startswith("v_writelane"):
        ins.defs = regs[0]
        ins.uses = sum(regs, [])                       # the old value too
        ins.lane_sel = regs[2] if len(regs) > 2 else []
    elif re.match(r"^v_(add|sub|subrev)_co_u32|^v_(addc|subb|subbrev)_co_u32|^v_div_scale|^v_(mad|mul)_[iu]64_[iu]32",
                  base):
        # vdst, sdst (carry out), srcs ...
        ins.defs = regs[0] + (regs[1] if len(regs) > 1 else [])
        ins.uses = sum(regs[2:], [])
    else:
        ins.defs = regs[0] if regs else []
        ins.uses = sum(regs[1:], [])
        if base.startswith("v_cndmask") and base.endswith("_e32"):
            ins.uses += ["vcc_lo", "vcc_hi"]
        if base.startswith("v_div_fmas"):
            ins.uses += ["vcc_lo", "vcc_hi"]
        if _DOT.match(base) and len(regs) >= 4:
            ins.srcc = regs[3]
    if ins.dpp and len(regs) > 1:
        ins.dpp_src0 = regs[1]
    return ins


@dataclass
class Violation:
    kernel: str
    rule: str
    need: int
    have: int
    producer: str
    consumer: str

    def __str__(self):
        return f"{self.kernel}: {self.rule}: {self.have} of {self.need} wait states: {self.producer!r} -> {self.consumer!r}"


def _rules(p: Ins, c: Ins):
    """(rule name, required wait states) for every hazard producer p creates for consumer c."""
    out = []
    pdef = set(p.defs)
    if not pdef:
        return out
    if p.valu:
        sg = {r for r in pdef if _sgpr_like(r) and not r.startswith("exec")}
        if sg:
            if c.valu and sg & set(c.uses):
                out.append(("VALU writes SGPR -> VALU reads it", 2))
            if c.lane_sel and sg & set(c.lane_sel):
                out.append(("VALU writes SGPR -> lane select", 4))
            if c.vmem and sg & set(c.uses):
                out.append(("VALU writes SGPR -> VMEM reads it", 5))
            if c.op.startswith("v_div_fmas") and {"vcc_lo", "vcc_hi"} & sg:
                out.append(("VALU writes VCC -> v_div_fmas", 4))
        if {"exec_lo", "exec_hi"} & pdef and c.valu and c.dpp:
            out.append(("VALU writes EXEC -> DPP", 5))
        vg = {r for r in pdef if r.startswith("v")}
        if vg:
            if c.valu and c.dpp and vg & set(c.dpp_src0):
                out.append(("VALU writes VGPR -> DPP src0", 2))
            if (c.op.startswith("v_readlane") or c.op.startswith("v_readfirstlane")) and vg & set(c.uses):
                out.append(("VALU writes VGPR -> v_readlane/readfirstlane", 1))
            if _PKF32.match(p.op) and not _OPSEL_LO.search(p.text) and c.valu and vg & set(c.uses):
                out.append(("v_pk_*_f32 writes VGPR -> VALU reads it", 1))
            if p.op.startswith("v_writelane") and c.valu and not c.op.startswith("v_writelane") and vg & set(c.uses):
                out.append(("v_writelane writes VGPR -> VALU reads it", 1))
            if _TRANS.match(p.op) and c.valu and not _TRANS.match(c.op) and vg & set(c.uses):
                out.append(("transcendental writes VGPR -> VALU reads it", 1))
            if _DOT.match(p.op) and vg & set(c.uses):
                same_dot_srcc = _DOT.match(c.op) and c.op == p.op and not (vg & (set(c.uses) - set(c.srcc)))
                if (c.valu and not same_dot_srcc) or c.vmem:
                    out.append(("v_dot writes VGPR -> other reader", 3))
    if p.vmem and "store" in p.op and re.search(r"(x3|x4|b96|b128)\b", p.op) and c.valu:
        data = set(_regs(p.text.split(",")[1])) if "," in p.text else set()
        if data & set(c.defs):
            out.append(("VMEM store data -> VALU overwrites it", 2))
    return out


def check_stream(kernel: str, lines: list[str], max_window: int = 8) -> list[Violation]:
    ins = [parse(l, i) for i, l in enumerate(lines)]
    viol = []
    window: list[Ins] = []
    for c in ins:
        waits = 0
        for p in reversed(window):
            for rule, need in _rules(p, c):
                if waits < need:
                    viol.append(Violation(kernel, rule, need, waits, p.text, c.text))
            waits += p.waits
            if waits >= 5:
                break
        window.append(c)
        if len(window) > max_window:
            window.pop(0)
        if c.op in ("s_branch", "s_endpgm", "s_setpc_b64"):
            window = []
    return viol


def disassemble(lib: str, workdir: str) -> dict[str, list[str]]:
    """kernel symbol -> instruction lines of the gfx950 code object inside lib."""
    fat, co = os.path.join(workdir, "fat.bin"), os.path.join(workdir, "co.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True,
                         check=True).stdout
    kernels, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            kernels[cur] = []
        elif cur and line.startswith("\t") and line.strip() and not line.strip().startswith(";"):
            kernels[cur].append(line.strip())
    return kernels
