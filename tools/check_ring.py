#!/usr/bin/env python3
"""ISA check for the K1r register file (run by tests/test_abi.py on the built
library): after the prologue that fills v2..v129 with the unit, no
instruction of k1r_match_units / k1r_match_units64 may write those registers
except the gpr_idx-relative ring writes (`v_mov_b32 v2, ...` inside an
s_set_gpr_idx_on ... gpr_idx(DST) region), and neither kernel may spill.
Usage: tools/check_ring.py <disassembly of the code object>"""
import re
import sys


def kernels(text):
    cur, out = None, {}
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(_Z\w*k1r_match_units\w*)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if re.match(r"^[0-9a-f]+ <", line):
            cur = None
        if cur and line.startswith("\t"):
            out[cur].append(line.split("//")[0].strip())
    return out


def dst_regs(ins):
    parts = ins.split(None, 1)
    if len(parts) < 2 or not parts[0].startswith("v_") or parts[0].startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return []
    op = parts[1].split(",")[0].strip()
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def check(text):
    bad = []
    for name, ins in kernels(text).items():
        # from the first gpr-indexed access (after the prologue filled v2..v129)
        # to the last one (the epilogue may reuse the registers)
        regions = [i for i, x in enumerate(ins) if x.startswith("s_set_gpr_idx_on")]
        in_dst = False
        for x in ins[regions[0]:regions[-1] + 1]:
            if x.startswith("s_set_gpr_idx_on"):
                in_dst = "DST" in x
            elif x.startswith("s_set_gpr_idx_off"):
                in_dst = False
            elif any(2 <= r <= 129 for r in dst_regs(x)) and not (
                    in_dst and re.match(r"v_mov_b32(_e32)? v2,", x)):
                bad.append((name, x))
    return bad


if __name__ == "__main__":
    bad = check(open(sys.argv[1]).read())
    for b in bad:
        print(*b)
    sys.exit(1 if bad else 0)
