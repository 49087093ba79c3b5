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

Two more close the classes round 6 met:

  * check_m0 (code object): s_set_gpr_idx_on writes m0, which the compiler
    reserves and does not take as an asm clobber; from every s_set_gpr_idx_off
    of the K1r kernels, nothing may read m0 (or a copy of it) before m0 is
    written again;
  * lint_scc (source): an asm statement whose SALU instructions write SCC must
    list "scc" as clobbered -- one that did not was scheduled between a compare
    and its branch and broke the decoder (profiles/r06s_*).

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


_M0_IMPLICIT = ("global_load_lds", "buffer_load_dword_lds", "s_movrel", "v_movrel", "s_sendmsg",
                "ds_read_addtid", "ds_write_addtid", "ds_gws", "s_set_gpr_idx_on")


def _operands(op):
    parts = op.split(None, 1)
    return [x.strip() for x in parts[1].split(",")] if len(parts) > 1 else []


_RANGE = re.compile(r"^s\[(\d+):(\d+)\]$")
# instructions whose first operand is read, not written
_NO_DST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_setpc", "s_set_gpr_idx", "s_store", "s_buffer_store",
           "s_sendmsg", "s_setreg", "s_waitcnt", "s_nop", "s_endpgm", "s_barrier", "s_sleep", "s_dcache",
           "s_ttrace", "s_setprio", "s_trap", "s_icache", "s_memtime", "s_memrealtime")


def _regs(tok):
    """SGPR / m0 names an operand token covers ('s[4:5]' -> s4, s5)."""
    tok = tok.split()[0] if tok else tok
    m = _RANGE.match(tok or "")
    if m:
        return {f"s{k}" for k in range(int(m.group(1)), int(m.group(2)) + 1)}
    return {tok} if tok and (tok == "m0" or re.fullmatch(r"s\d+", tok)) else set()


def _dst_src(op):
    mn = op.split()[0] if op else ""
    ops = _operands(op)
    if not ops:
        return mn, set(), set()
    writes = mn.startswith(("s_", "v_readlane", "v_readfirstlane")) and not mn.startswith(_NO_DST)
    if writes:
        return mn, _regs(ops[0]), set().union(*[_regs(x) for x in ops[1:]]) if len(ops) > 1 else set()
    return mn, set(), set().union(*[_regs(x) for x in ops])


def check_m0(text, names=("k1r_match_units",)):
    """[(kernel, message)] where a value in m0 could be read after the
    register-index asm changed it.  s_set_gpr_idx_on writes m0, which the
    compiler reserves and does not take as an asm clobber, so the REG_* asm
    (snappy_kernels.hip) leaves m0 holding the index: from every
    s_set_gpr_idx_off, on every CFG path, nothing may read m0 -- or an SGPR
    copied from it -- before m0 is written again.  Reads: m0 as a source
    operand (v_writelane / v_readlane lane select, s_mov from it) and the
    instructions that use m0 implicitly (LDS-DMA, movrel, s_sendmsg, ...)."""
    bad, found = [], 0
    for name, (base, ins) in kernels(text).items():
        if not any(n in name for n in names):
            continue
        index = {a: i for i, (a, _, _) in enumerate(ins)}
        for s0 in (i for i, (_, op, _) in enumerate(ins) if op.startswith("s_set_gpr_idx_off")):
            found += 1
            seen, work = set(), [(s0, frozenset({"m0"}))]
            while work:
                i, dirty = work.pop()
                for j in _succ(i, ins, base, index):
                    op = ins[j][1]
                    mn, dst, srcs = _dst_src(op)
                    d = set(dirty)
                    if mn in ("s_mov_b32", "s_mov_b64") and srcs and srcs <= d:
                        d |= dst  # a copy of the index (or the index put back): tracked, not a use
                    elif mn.startswith(_M0_IMPLICIT) and "m0" in d and not mn.startswith("s_set_gpr_idx_on"):
                        bad.append((name, f"{mn} at {ins[j][0]:#x} uses m0 left by s_set_gpr_idx_off at {ins[s0][0]:#x}"))
                        continue
                    elif srcs & d:
                        bad.append((name, f"{op} at {ins[j][0]:#x} reads m0 (or its copy) left by s_set_gpr_idx_off "
                                          f"at {ins[s0][0]:#x}"))
                        continue
                    else:
                        d -= dst  # written again
                        if mn.startswith("s_set_gpr_idx_on"):
                            d.discard("m0")
                    if not d:
                        continue
                    key = (j, frozenset(d))
                    if key in seen:
                        continue
                    seen.add(key)
                    work.append((j, frozenset(d)))
    if not found:
        bad.append(("k1r", "no s_set_gpr_idx_off found"))
    return bad


# SALU that write SCC: an asm statement holding one must list "scc" as clobbered,
# or the compiler may schedule it between its own compare and branch
_SCC_WRITERS = re.compile(r"\bs_(?:cmp\w*|cmpk\w*|add_\w+|addc_\w+|addk_\w+|sub_\w+|subb_\w+|and\w*|or\w*|xor\w*|"
                          r"nand\w*|nor\w*|xnor\w*|not_\w+|lshl\w*|lshr\w*|ashr\w*|bfe_\w+|min_\w+|max_\w+|abs\w*|"
                          r"bcnt\w*|bitcmp\w*|quadmask\w*|wqm\w*)\b")


def _asm_sections(body):
    """An asm statement's template, outputs, inputs, clobbers: split at the colons
    outside string literals and parentheses (labels inside the template have colons)."""
    out, cur, depth, q, k = [], [], 0, False, 0
    while k < len(body):
        c = body[k]
        if q:
            cur.append(c)
            if c == "\\":
                cur.append(body[k + 1])
                k += 1
            elif c == '"':
                q = False
        elif c == '"':
            q = True
            cur.append(c)
        elif c in "([{":
            depth += 1
            cur.append(c)
        elif c in ")]}":
            depth -= 1
            cur.append(c)
        elif c == ":" and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(c)
        k += 1
    out.append("".join(cur))
    return out


def lint_scc(path):
    """[(file:line, message)] for asm statements that write SCC without the clobber."""
    bad = []
    src = open(path).read()
    for m in _ASM.finditer(src):
        i, depth = m.end(), 1
        while i < len(src) and depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        parts = _asm_sections(src[m.end():i - 1])
        text = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', parts[0]))
        w = _SCC_WRITERS.search(text)
        if not w:
            continue
        clob = parts[3] if len(parts) > 3 else ""
        if '"scc"' not in clob:
            bad.append((f"{path}:{src[:m.start()].count(chr(10)) + 1}", f"{w.group(0)} writes SCC; \"scc\" not clobbered"))
    return bad


_ASM = re.compile(r"\basm\s*(?:volatile\s*)?\(", re.S)
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
