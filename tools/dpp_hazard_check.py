"""Check gfx950 assembly for the DPP read-after-VALU-write hazard.

A DPP instruction must not read (as its DPP source, src0) a VGPR written by a
VALU instruction in the previous two wait states.  The compiler guards the DPP
it generates itself; the hand-written `v_fmac_f64_dpp` asm in ba_bcr.hip is
invisible to it, so this script re-checks the final schedule.

usage: python tools/dpp_hazard_check.py file.s   (exit 1 on a hazard)
"""
import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(tok):
    m = REG.fullmatch(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return {int(m.group(3))}


def instructions(lines):
    for ln in lines:
        t = ln.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        yield t


def check(text):
    ins = list(instructions(text.splitlines()))
    bad = []
    for n, t in enumerate(ins):
        if "_dpp" not in t.split()[0]:
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        src0 = regs(ops[1].split()[0]) if len(ops) > 1 else set()
        waits = 0
        for back in range(n - 1, max(n - 4, -1), -1):
            p = ins[back]
            op = p.split()[0]
            if op.startswith("s_nop"):
                waits += int(p.split()[1], 0) + 1
            elif op.startswith("v_") and waits < 2:
                dst = regs(p.split(None, 1)[1].split(",")[0]) if len(p.split()) > 1 else set()
                if dst & src0:
                    bad.append((n, p, t))
                waits += 1
            else:
                waits += 1
            if waits >= 2:
                break
    return bad


if __name__ == "__main__":
    txt = open(sys.argv[1]).read()
    b = check(txt)
    for n, p, t in b[:20]:
        print(f"hazard at instruction {n}: '{p}' -> '{t}'")
    print(f"{sum(1 for i in instructions(txt.splitlines()) if '_dpp' in i.split()[0])} DPP instructions, {len(b)} hazards")
    sys.exit(1 if b else 0)
