"""ISA audit of the decode kernels (round-3 parity investigation).

usage: python tools/isa_audit.py FILE.s [...]   (hipcc --cuda-device-only -S output)

Checks, over the whole text in fall-through order:
  1. DPP reading a VGPR written by any VALU in the 2 preceding issue slots
     (gfx9 "VALU write VGPR -> DPP read" needs 2 wait states; s_nop N counts N+1);
  2. the same for VGPRs written inside inline asm (;;#ASMSTART..;;#ASMEND),
     which the compiler does not pad, read by DPP / readlane / permlane.
Prints every hit and a count per check.
"""
import re
import sys


def regs(s):
    out = set()
    for m in re.finditer(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b', s):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def audit(path):
    lines = open(path).read().split('\n')
    pend = []  # (defs, states left, from_asm)
    inasm = False
    hits = [0, 0]
    for i, line in enumerate(lines):
        t = line.strip()
        if t.startswith(';;#ASMSTART'):
            inasm = True
            continue
        if t.startswith(';;#ASMEND'):
            inasm = False
            continue
        if not t or t.startswith(';') or t.startswith('.') or t.endswith(':'):
            continue
        op = t.split()[0]
        parts = [p.strip() for p in t[len(op):].split(';')[0].split(',')]
        uses = regs(','.join(parts[1:])) if len(parts) > 1 else set()
        crosslane = '_dpp' in op or 'readlane' in op or 'permlane' in op or 'readfirstlane' in op
        if crosslane and not inasm:
            for defs, left, from_asm in pend:
                if defs & uses and ('_dpp' in op or from_asm):
                    print(f"{path}:{i + 1}: {t}  <- written {2 - left} state(s) before{' (inline asm)' if from_asm else ''}")
                    hits[1 if from_asm else 0] += 1
        w = int(parts[0], 0) + 1 if op == 's_nop' else 1
        if not inasm:
            pend = [(d, left - w, a) for d, left, a in pend if left - w > 0]
        if op.startswith('v_') and not op.startswith('v_cmp') and 'readlane' not in op and 'readfirstlane' not in op:
            pend.append((regs(parts[0]) if parts else set(), 2, inasm))
    return hits


if __name__ == "__main__":
    tot = [0, 0]
    for f in sys.argv[1:]:
        h = audit(f)
        tot = [a + b for a, b in zip(tot, h)]
    print(f"VALU-write -> DPP-read hazards: {tot[0]}; inline-asm output -> cross-lane read hazards: {tot[1]}")
