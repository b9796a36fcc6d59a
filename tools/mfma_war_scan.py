"""Scan gfx950 assembly for VGPR writes that follow an MFMA reading (or writing) the same register
closely -- the MFMA WAR / WAW hazards that hipcc's hazard recognizer resolves with s_nop for its own
VALU instructions but does not model for inline-asm outputs.

    python tools/mfma_war_scan.py file.s [...]

Per kernel: for every VGPR written inside an inline-asm block (;;#ASMSTART .. ;;#ASMEND), the wait-state
distance (instructions issued, s_nop N counting N + 1) back to the nearest MFMA whose SrcC / SrcA / SrcB /
vDst overlaps it, and the same minimum over compiler-generated VALU writes (which hipcc keeps at or above
the hardware requirement).  An asm write closer than every compiler write of the same kind is suspect.
"""
import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan(text, window=24):
    res = {}
    for name in re.findall(r"^(_Z\w+):", text, re.M):
        body = text[text.index(name + ":"):]
        body = body[:body.index("s_endpgm")]
        in_asm = False
        hist = []  # (wait-state position, kind, reg sets)
        posn = 0
        stats = {"asm": {}, "cc": {}}
        worst = []
        for line in body.splitlines():
            t = line.strip()
            if t.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if t.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
                continue
            op = t.split()[0]
            args = t[len(op):].split(";")[0]
            parts = [a.strip() for a in args.split(",")]
            if op.startswith("s_nop"):
                posn += int(t.split()[1], 0) + 1
                continue
            if op.startswith("v_mfma"):
                d, a, b, c = (regs(parts[i]) for i in range(4))
                hist.append((posn, d, a | b, c))
            elif op.startswith("v_") and parts and parts[0].startswith("v") and not op.startswith(("v_cmp", "v_readfirstlane", "v_readlane")):
                w = regs(parts[0])
                for (p0, d, ab, c) in reversed(hist):
                    dist = posn - p0
                    if dist > window:
                        break
                    for kind, rs in (("srcC", c), ("srcAB", ab), ("vdst", d)):
                        if w & rs:
                            key = "asm" if in_asm else "cc"
                            cur = stats[key].get(kind)
                            stats[key][kind] = dist if cur is None else min(cur, dist)
                            if in_asm:
                                worst.append((dist, kind, t))
                    # (only the nearest overlapping MFMA matters per kind; keep scanning older ones)
            posn += 1
            hist = [h for h in hist if posn - h[0] <= window]
        res[name] = (stats, sorted(worst)[:5])
    return res


if __name__ == "__main__":
    for f in sys.argv[1:]:
        for name, (stats, worst) in scan(open(f).read()).items():
            print(f, name[:60], stats, worst[:3])
