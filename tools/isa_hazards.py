"""Scan gfx950 assembly for MFMA hazards the compiler cannot see (MFMAs written as inline asm).

Follows every control-flow path from each MFMA (fall-through and branch targets) and reports, with the wait states
in between:
  RAW  an instruction that reads or writes (WAW) an MFMA's destination fewer than `--raw` wait states after it
  WARC an instruction that writes an MFMA's SrcC register fewer than `--warc` wait states after the MFMA
  PRE  a VALU that writes an MFMA A/B/C source fewer than 2 wait states before it
Wait states: each instruction counts 1, `s_nop N` counts N+1. Another MFMA reading the destination as SrcC (the
same accumulator chain) is exempt from RAW. Usage: python tools/isa_hazards.py file.s kernel_substring [...]
"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        k = m.group(1)
        if m.group(4) is not None:
            out.add(f"{k}{m.group(4)}")
        else:
            out.update(f"{k}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(lines):
    """-> list of (text, is_asm, op, dst_regs, src_regs, waits)."""
    out, in_asm = [], False
    for raw in lines:
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(";") or s.endswith(":") or s.startswith("."):
            if s.endswith(":"):
                out.append((s, False, "label", set(), set(), 0))
            continue
        s = s.split(";")[0].strip()
        op, _, rest = s.partition(" ")
        ops = [o.strip() for o in rest.split(",")] if rest else []
        waits = 1
        if op == "s_nop":
            waits = int(ops[0], 0) + 1
        if op.startswith("v_") or op.startswith("ds_") or op.startswith("buffer_") or op.startswith("global_"):
            if op.startswith("buffer_store") or op.startswith("global_store") or op.startswith("ds_write") \
                    or op.startswith("ds_store"):
                dst, src = set(), set().union(*[regs(o) for o in ops]) if ops else set()
            else:
                dst = regs(ops[0]) if ops else set()
                src = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
        else:
            dst, src = set(), set()
        out.append((s, in_asm, op, dst, src, waits, ops))
    return out


def _successors(ins):
    """Per instruction index: the indices execution may reach next (fall-through and branch targets)."""
    labels = {it[0][:-1]: k for k, it in enumerate(ins) if it[2] == "label"}
    succ = []
    for k, it in enumerate(ins):
        op = it[2]
        nxt = [k + 1] if k + 1 < len(ins) else []
        if op == "s_branch":
            nxt = [labels[it[6][0]]] if it[6][0] in labels else []
        elif op.startswith("s_cbranch"):
            if it[6][0] in labels:
                nxt = nxt + [labels[it[6][0]]]
        elif op == "s_endpgm":
            nxt = []
        succ.append(nxt)
    return succ


def scan(ins, raw_ws=12, warc_ws=7):
    """Follows every path (both sides of each branch) from each MFMA until `raw_ws` wait states have passed."""
    succ = _successors(ins)
    hits = set()
    for i, it in enumerate(ins):
        if not it[2].startswith("v_mfma"):
            continue
        ops = it[6]
        d = regs(ops[0])
        a, b, c = regs(ops[1]), regs(ops[2]), regs(ops[3]) if len(ops) > 3 else set()
        # PRE: a VALU write to a source too close before (layout order; these kernels' writes are block-local)
        ws = 0
        for j in range(i - 1, max(-1, i - 8), -1):
            jt = ins[j]
            if jt[2] == "label":
                continue
            if jt[2].startswith("v_") and not jt[2].startswith("v_mfma") and jt[3] & (a | b | c) and ws < 2:
                hits.add(("PRE", i, j, ws))
            ws += jt[5]
        stack, seen = [(n, 0) for n in succ[i]], set()
        while stack:
            j, ws = stack.pop()
            if (j, ws) in seen or ws >= max(raw_ws, warc_ws):
                continue
            seen.add((j, ws))
            jt = ins[j]
            op = jt[2]
            if op.startswith("v_mfma"):
                jops = jt[6]
                jd, jc = regs(jops[0]), regs(jops[3]) if len(jops) > 3 else set()
                if (regs(jops[1]) | regs(jops[2])) & d and ws < raw_ws:
                    hits.add(("RAW-AB", i, j, ws))
                if jc & d and jc != d and ws < raw_ws:
                    hits.add(("RAW-C", i, j, ws))
                if jd & d and jd != d and ws < raw_ws:
                    hits.add(("WAW", i, j, ws))
            elif op.startswith(("v_", "ds_", "buffer_", "global_")):
                if (jt[4] & d or jt[3] & d) and ws < raw_ws:
                    hits.add(("RAW", i, j, ws))
                if op.startswith("v_") and jt[3] & c and ws < warc_ws:
                    hits.add(("WARC", i, j, ws))
            for n in succ[j]:
                stack.append((n, ws + jt[5]))
    return sorted(hits, key=lambda h: (h[1], h[2]))


def kernel_lines(text, name):
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", text, re.M)
    if not m:
        raise SystemExit(f"{name} not found")
    end = text.index(".Lfunc_end", m.end())   # (blocks may be laid out after an s_endpgm)
    return text[m.end():end].splitlines()


def main():
    text = open(sys.argv[1]).read()
    bad = 0
    for name in sys.argv[2:]:
        ins = parse(kernel_lines(text, name))
        for kind, i, j, ws in scan(ins):
            src = "asm" if ins[j][1] else "COMPILER"
            print(f"{name}: {kind} ws={ws} [{src}] after `{ins[i][0]}`\n      -> `{ins[j][0]}`")
            bad += 1
    print(f"{bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
