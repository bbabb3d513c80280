#!/usr/bin/env python3
"""Check the DPP source hazard in hand-written inline asm (gfx950): a VALU instruction that
writes a VGPR needs 2 wait states before a DPP instruction reads that VGPR as its permuted
source.  The compiler does not look inside inline asm, so the kernels put an s_nop 1 into the
asm (fma8_row_bcast) or fence the source (dpp_ready); this script verifies the result in the
compiled ISA.

usage: hipcc --cuda-device-only -S -o x.s ... ; python tools/dpp_hazard_check.py x.s [symbol-substring]
Exit 1 when a DPP source was written by one of the two instructions issued before it."""
import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(tok):
    m = REG.fullmatch(tok.strip().rstrip(","))
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def main():
    lines = open(sys.argv[1]).read().split("\n")
    want = sys.argv[2] if len(sys.argv) > 2 else None
    fn, bad, checked = None, 0, 0
    window = []   # (wait states it provides, VGPRs it writes) of the last issued instructions
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            fn, window = m.group(1), []
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        args = t[len(op):].split(",")
        if want and (fn is None or want not in fn):
            continue
        if "_dpp" in op and op.startswith("v_"):
            src = regs(args[1]) if len(args) > 1 else set()
            ws = 0
            for w, wr in reversed(window):
                if ws >= 2:
                    break
                if wr & src:
                    print(f"{fn[:60]}: {t}  <- source written {ws} wait states before")
                    bad += 1
                    break
                ws += w
            checked += 1
        if op == "s_nop":
            window.append((int(t.split()[1], 0) + 1, set()))
        elif op.startswith("v_"):
            window.append((1, regs(args[0]) if args else set()))
        else:
            window.append((1, set()))
        window = window[-4:]
    print(f"{checked} DPP instructions checked, {bad} hazards")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
