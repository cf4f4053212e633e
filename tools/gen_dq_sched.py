#!/usr/bin/env python3
"""Generate the VALU placement of the one-wave-per-SIMD dQ kernel (csrc/attention.hip, attn_bwd_dq_hs_kernel).

Per 32-key half-tile a wave issues 24 v_mfma_f32_32x32x16_bf16 in the order
  gaps 0-7: S^T (0-3) / dP^T (4-7) chains of query block 0 | 8-11: dQ^T of block 1 (previous half) |
  12-19: chains of block 1 | 20-23: dQ^T of block 0,
and per query block 40 VALU ops: 16 exp2 (E), 16 multiplies dS = P dP (M), 8 bf16 pair conversions (C). The
schedule is periodic (24 gaps); block 1's ops wrap into the next half. Rules: E one gap after the S chain's last
MFMA, M two gaps after the dP chain's last MFMA and in a later gap than its E, C after both M of its pair; at most
2 exps and 4 VALU ops per gap; a block's pack of elements 0-7 (C 0-3) is complete one gap before its first dQ^T
MFMA, elements 8-15 (C 4-7) one gap before its third. Output (stdout): the C++ table DQ_SCHED[24][4] of op codes
(kind << 6 | block << 5 | index; 0xff = none); the placement is listed on stderr.
"""
import sys

NG = 24
START_E = {0: 5, 1: 17}      # S chains at gaps 0-3 / 12-15
START_M = {0: 9, 1: 21}      # dP chains at gaps 4-7 / 16-19
DQ = {0: 20, 1: 8 + NG}      # first dQ^T gap that reads the block's packs


def main():
    cap_e = [0] * NG
    slots = [[] for _ in range(NG)]
    placed = {}
    for qb in (1, 0):        # block 1 wraps into the next half: place it first
        tE, tM, tC = {}, {}, {}
        g = START_E[qb]
        while len(tC) < 8:
            gi = g % NG
            s = slots[gi]
            for j in range(8):                       # conversions first: they free the pipeline tail
                if j not in tC and 2 * j + 1 in tM and len(s) < 4:
                    tC[j] = g
                    s.append(("C", qb, j))
            for e in range(16):
                if e in tE and e not in tM and tE[e] < g and g >= START_M[qb] and len(s) < 4:
                    tM[e] = g
                    s.append(("M", qb, e))
            for j in range(8):
                if j not in tC and 2 * j + 1 in tM and len(s) < 4:
                    tC[j] = g
                    s.append(("C", qb, j))
            for e in range(16):
                if e not in tE and cap_e[gi] < 2 and len(s) < 4:
                    tE[e] = g
                    cap_e[gi] += 1
                    s.append(("E", qb, e))
            g += 1
            assert g < START_E[qb] + 2 * NG, "does not fit"
        assert max(tC[j] for j in range(4)) < DQ[qb], (qb, tC)
        assert max(tC[j] for j in range(4, 8)) < DQ[qb] + 2, (qb, tC)
        placed[qb] = (tE, tM, tC)
    code = {"E": 0, "M": 1, "C": 2}
    # Order within each gap (the periodic stream, gap 23 before gap 0): a conversion after the multiplies of its
    # pair, and no op directly after the op whose result it reads when that op is an exp (trans use) or a
    # multiply read by a conversion: the compiler pads both with an s_nop 0 and does not count the asm MFMA
    # between gaps. Each gap takes the first permutation without such a pair, given the previous gap's last op.
    import itertools

    def reads(a, b):   # does op b read op a's result?
        if a[1] != b[1]:
            return False
        return (a[0] == "E" and b[0] == "M" and a[2] == b[2]) or \
            (a[0] == "M" and b[0] == "C" and a[2] in (2 * b[2], 2 * b[2] + 1))

    def padded(prev, nxt):
        return prev is not None and reads(prev, nxt) and prev[0] in ("E", "M")

    for _ in range(2):   # second pass: gap 0 sees gap 23's final order
        for g in range(NG):
            prev = slots[g - 1][-1] if slots[g - 1] else None
            best = None
            for perm in itertools.permutations(slots[g]):
                if any(reads(perm[j], perm[i]) for i in range(len(perm)) for j in range(i + 1, len(perm))):
                    continue                       # a consumer before its producer
                chain = [prev] + list(perm)
                pads = sum(padded(chain[i], chain[i + 1]) for i in range(len(perm)))
                if best is None or pads < best[0]:
                    best = (pads, list(perm))
            slots[g] = best[1]
    pads = sum(padded(slots[g - 1][-1] if slots[g - 1] else None, slots[g][0]) for g in range(NG) if slots[g]) + \
        sum(padded(slots[g][i], slots[g][i + 1]) for g in range(NG) for i in range(len(slots[g]) - 1))
    print(f"// hazard pads left: {pads}", file=sys.stderr)
    rows = []
    for g, s in enumerate(slots):
        print(f"// gap {g:2d}: " + " ".join(f"{k}{qb}.{i}" for k, qb, i in s), file=sys.stderr)
        ops = [(code[k] << 6) | (qb << 5) | i for k, qb, i in s] + [0xFF] * (4 - len(s))
        rows.append("{" + ", ".join(f"0x{o:02x}" for o in ops) + "}")
    print("constexpr unsigned char DQ_SCHED[24][4] = {\n    " + ",\n    ".join(rows) + "};")


if __name__ == "__main__":
    main()
