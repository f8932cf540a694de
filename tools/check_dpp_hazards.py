"""Build-time check of the VALU-write -> DPP-read hazard in the engine's ISA.

gfx950 needs 2 wait states between a VALU instruction that writes a VGPR and a DPP
instruction that reads it as its DPP source (src0).  LLVM's hazard recognizer inserts
them for DPP it generates, but cannot see inside inline asm: the csrc kernels issue
v_fmac_f64_dpp row_newbcast groups from asm statements, and only some groups start with
their own s_nop.  This script scans the device assembly (``make asm`` -> /tmp/ryd_engine.s,
or a path given) in program order and fails if any DPP instruction's src0 was written by
a VALU instruction fewer than 2 wait states earlier (each intervening instruction is one
wait state, ``s_nop N`` is N + 1).  Control flow is followed by fall-through only; a
label resets the window (a branch target's predecessors end in a branch or s_cbranch,
whose own issue adds the wait states the DPP needs in practice, and the compiler's
recognizer covers the compiled side of the edge).

    python tools/check_dpp_hazards.py [asm.s]      # exit 1 and a listing on a hazard
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")
NEED = 2


def regs(tok: str):
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def operands(line: str):
    body = line.split(None, 1)
    if len(body) < 2:
        return []
    return [t.strip() for t in body[1].split(",")]


def vgpr_writes(mn: str, ops):
    """VGPRs written by a VALU instruction (its first operand), else empty."""
    if not mn.startswith("v_") or not ops:
        return set()
    if mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "v_cmpx")):
        return set()
    return regs(ops[0].split()[0])


def check(path: str):
    problems = []
    window = []          # (wait states, written vgprs, text) of recent instructions, newest last
    fn = "?"
    with open(path) as f:
        for ln, raw in enumerate(f, 1):
            line = raw.split(";")[0].strip()
            if not line:
                continue
            if line.endswith(":") and not line.startswith("."):
                if not line.startswith(".L") and not line.startswith("_L"):
                    fn = line[:-1]
                window = []
                continue
            if line.startswith("."):
                continue
            mn = line.split()[0]
            ops = operands(line)
            if "_dpp" in mn and ops and len(ops) >= 2:
                src0 = regs(ops[1].split()[0])
                ws = 0
                for w_states, wr, txt in reversed(window):
                    if ws >= NEED:
                        break
                    if wr & src0:
                        problems.append(f"{path}:{ln} [{fn}] {line}\n    reads v{sorted(src0)} written "
                                        f"{ws} wait state(s) earlier by: {txt}")
                        break
                    ws += w_states
            if mn == "s_nop":
                n = int(ops[0], 0) if ops else 0
                window.append((n + 1, set(), line))
            else:
                window.append((1, vgpr_writes(mn, ops), line))
            if len(window) > 8:
                window.pop(0)
    return problems


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/ryd_engine.s"
    probs = check(path)
    if probs:
        print(f"{len(probs)} VALU-write -> DPP-read hazard(s):")
        print("\n".join(probs[:50]))
        sys.exit(1)
    print(f"{path}: no VALU-write -> DPP-read hazard within {NEED} wait states")


if __name__ == "__main__":
    main()
