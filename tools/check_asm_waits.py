#!/usr/bin/env python3
"""Guard for memory operations issued from inline asm (run by
tests/test_abi.py on the built library).

Round 2 lost a GPU box to an inline-asm load whose destination register the
compiler released on a loop-exit path while the load was still in flight
(DESIGN.md 4.2).  Two checks close that class:

  * source (lint_source): every `asm` block in the .hip sources that issues a
    memory load into a register (ds_read*, global_load*, buffer_load*,
    flat_load*, s_load*, except the LDS-DMA form global_load_lds_*) must wait
    for it inside the same block (s_waitcnt lgkmcnt(0) / vmcnt(0) after the
    load), so no register of the block is live across an outstanding load;
  * code object (check): an LDS-DMA (global_load_lds_*) writes LDS, not a
    register, so it may stay in flight across instructions -- but on every
    control-flow path from it to s_endpgm an `s_waitcnt vmcnt(0)` must drain
    it, or the workgroup's LDS could be handed to the next workgroup while the
    DMA still writes into it.  The path analysis runs over the disassembly's
    CFG (branch targets <kernel+0xOFF>, fall-through).

Usage: tools/check_asm_waits.py <disassembly> [sources...]"""
import re
import sys

_HDR = re.compile(r"^([0-9a-f]+) <(\w+)>:")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<(\w+)\+0x([0-9a-f]+)>")


def kernels(text):
    """name -> (base address, [(address, instruction text)])."""
    out, cur = {}, None
    for line in text.splitlines():
        m = _HDR.match(line)
        if m:
            cur = m.group(2)
            out[cur] = (int(m.group(1), 16), [])
            continue
        if cur and line.startswith("\t"):
            a = _ADDR.search(line)
            if a:
                out[cur][1].append((int(a.group(1), 16), line.split("//")[0].strip(), line))
    return out


def _succ(i, ins, base, index):
    """Successor instruction indices of instruction i."""
    _, op, raw = ins[i]
    mnem = op.split()[0] if op else ""
    if mnem == "s_endpgm":
        return []
    tg = None
    if mnem.startswith(("s_branch", "s_cbranch")):
        m = _TGT.search(raw)
        if m:
            tg = index.get(base + int(m.group(2), 16))
    if mnem == "s_branch":
        return [tg] if tg is not None else []
    nxt = [i + 1] if i + 1 < len(ins) else []
    return nxt + ([tg] if tg is not None else [])


def check(text):
    """[(kernel, message)] for LDS-DMA operations that can reach s_endpgm undrained."""
    bad = []
    for name, (base, ins) in kernels(text).items():
        index = {a: i for i, (a, _, _) in enumerate(ins)}
        starts = [i for i, (_, op, _) in enumerate(ins) if op.startswith("global_load_lds")]
        for s in starts:
            seen, work = set(), [s]
            while work:
                i = work.pop()
                for j in _succ(i, ins, base, index):
                    if j in seen:
                        continue
                    seen.add(j)
                    op = ins[j][1]
                    if op.startswith("s_waitcnt") and "vmcnt(0)" in op:
                        continue  # drained on this path
                    if op.startswith("s_endpgm"):
                        bad.append((name, f"LDS-DMA at {ins[s][0]:#x} reaches s_endpgm at {ins[j][0]:#x} undrained"))
                        continue
                    work.append(j)
    return bad


def check_k4_bitmap(text, at=784):
    """[(kernel, message)] unless every K4 bitmap `ds_or_b32 ... offset:<at>`
    (kK4MapAt: a batch's element-start bitmap) lies between its clear (the
    previous access at that offset is a ds_write_b32) and its read (the next one
    is a ds_read_b32): the compiler barriers in k4_body keep that order, and a
    reorder would read a half-built bitmap."""
    bad, found = [], 0
    tag = f"offset:{at}"
    for name, (base, ins) in kernels(text).items():
        if "k4_decompress" not in name:
            continue
        acc = [(i, op.split()[0]) for i, (_, op, _) in enumerate(ins) if op.startswith("ds_") and tag in op]
        for k, (i, mn) in enumerate(acc):
            if mn != "ds_or_b32":
                continue
            found += 1
            prev = acc[k - 1][1] if k else None
            nxt = acc[k + 1][1] if k + 1 < len(acc) else None
            if prev != "ds_write_b32" or nxt != "ds_read_b32":
                bad.append((name, f"bitmap ds_or at {ins[i][0]:#x}: previous {prev}, next {nxt}"))
    if not found:
        bad.append(("k4", "no K4 bitmap ds_or_b32 found"))
    return bad


_ASM = re.compile(r"\basm\s+(?:volatile\s*)?\(", re.S)
_LOAD = re.compile(r"\b(ds_read\w*|global_load\w*|buffer_load\w*|flat_load\w*|s_load\w*|s_buffer_load\w*)\b")


def _asm_strings(src):
    """The instruction text of every asm(...) statement: its leading string literals."""
    for m in _ASM.finditer(src):
        i, depth = m.end(), 1
        while i < len(src) and depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        body = src[m.end():i - 1]
        head = body.split(":", 1)[0]
        yield src[:m.start()].count("\n") + 1, "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', head))


def lint_source(path):
    """[(file:line, message)] for asm loads into registers not waited in-block."""
    bad = []
    src = open(path).read()
    for line, text in _asm_strings(src):
        for m in _LOAD.finditer(text):
            mn = m.group(1)
            if mn.startswith("global_load_lds"):
                continue  # LDS destination: covered by check() on the code object
            cnt = "lgkmcnt(0)" if mn.startswith(("ds_", "s_")) else "vmcnt(0)"
            rest = text[m.end():]
            if not re.search(r"s_waitcnt[^\\]*" + re.escape(cnt), rest):
                bad.append((f"{path}:{line}", f"{mn} not waited ({cnt}) inside its asm block"))
    return bad


if __name__ == "__main__":
    bad = check(open(sys.argv[1]).read())
    for p in sys.argv[2:]:
        bad += lint_source(p)
    for b in bad:
        print(*b)
    sys.exit(1 if bad else 0)
