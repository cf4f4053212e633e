#!/usr/bin/env python3
"""Generate the VALU placement of the one-wave-per-SIMD attention forward (csrc/attention.hip, attn_fwd_hs_kernel).

Per 32-key half a wave issues 16 v_mfma_f32_32x32x16_bf16 and 4 v_mfma_f32_16x16x32_bf16 row sums in the order
  gaps 0-3: S^T chain of query block 0 | 4, 5, 7, 8: O^T += V^T P^T of block 1 (previous half), 6 / 9 its row sums |
  10-13: S^T chain of block 1 | 14, 15, 17, 18: O^T of block 0, 16 / 19 its row sums,
and per query block 24 VALU ops: 16 exp2 (E) and 8 bf16 pair conversions (C, elements 2c, 2c+1), plus per half two
v_add_f32 per block (A) that add the half's row-sum partial into the running f32 sums >= 12 wait states after the
block's second row-sum MFMA. The schedule is periodic (20 gaps); block 1's ops wrap into the next half. Rules: E from
two gaps after the chain's last MFMA (its first exps last in their gap: with the gap's LDS read issued right behind
the MFMA that gives the 12 wait states the chain's result needs), C in a later gap than the exps it reads; a 32x32x16
gap carries <= 24 issue cycles (E 8, C 5: <= 2 E), a 16x16x32 gap <= 8 (one op); a block's packs of elements 0-7
(C 0-3) complete before its first PV MFMA, elements 8-15 (C 4-7) before its third. Within a gap the op order avoids an
op directly after the exp it reads (the compiler pads that with an s_nop 0). Output (stdout): the C++ table
FW_SCHED_R[20][4] (kind << 6 | block << 5 | index; 0xff = none); the placement is listed on stderr.
"""
import itertools, sys
# gap kinds per half (20 gaps)
KIND = ["S0"]*4 + ["P1","P1","R1","P1","P1","R1"] + ["S1"]*4 + ["P0","P0","R0","P0","P0","R0"]
NG = len(KIND)
big = [k[0] in "SP" for k in KIND]
# per block: chain end gap, first PV gap reading s2=0 packs, first PV gap reading s2=1 packs
CHAIN_END = {0: 3, 1: 13}
PV0 = {0: 14, 1: 4 + NG}
PV1 = {0: 17, 1: 7 + NG}
START_E = {0: CHAIN_END[0] + 2, 1: CHAIN_END[1] + 2}
COST = {"E": 8, "C": 5}
def cap(g):
    return 24 if big[g % NG] else 8
def main():
    used = [0]*NG; ne = [0]*NG
    slots = [[] for _ in range(NG)]
    for qb in (1, 0):
        tE, tC = {}, {}
        g = START_E[qb]
        while len(tC) < 8:
            gi = g % NG; s = slots[gi]
            for j in range(8):
                if j not in tC and 2*j in tE and 2*j+1 in tE and max(tE[2*j], tE[2*j+1]) < g and used[gi] + COST["C"] <= cap(g):
                    tC[j] = g; used[gi] += COST["C"]; s.append(("C", qb, j))
            for e in range(16):
                if e not in tE and ne[gi] < (2 if big[gi] else 1) and used[gi] + COST["E"] <= cap(g):
                    tE[e] = g; ne[gi] += 1; used[gi] += COST["E"]; s.append(("E", qb, e))
            g += 1
            assert g < START_E[qb] + 2*NG
        c0 = max(tC[j] for j in range(4)); c1 = max(tC[j] for j in range(4, 8))
        print(f"// block {qb}: E {min(tE.values())}..{max(tE.values())}, C0-3 by {c0} (PV {PV0[qb]}), C4-7 by {c1} (PV {PV1[qb]})", file=sys.stderr)
        assert c0 < PV0[qb] and c1 < PV1[qb], (qb, tC)
        # next chain of this block writes S[qb] at its chain start (gap CHAIN_END-3 + NG): all E/C done before
        assert max(max(tE.values()), max(tC.values())) < CHAIN_END[qb] - 3 + NG
    def reads(a, b):
        if a is None or a[1] != b[1] or a[0] != "E": return False
        return b[0] == "C" and a[2] in (2*b[2], 2*b[2]+1)
    def cost(sl):
        pads, late = 0, 0
        for g in range(NG):
            prev = sl[g - 1][-1] if sl[g - 1] else None
            for i, op in enumerate(sl[g]):
                if reads(prev, op):
                    pads += 1
                prev = op
                if op[0] == "E" and START_E[op[1]] == g:
                    late -= i
        return (late, pads)
    for _ in range(4):   # coordinate descent over the gaps' orders
        for g in range(NG):
            best = None
            for perm in itertools.permutations(slots[g]):
                trial = slots[:g] + [list(perm)] + slots[g + 1:]
                c = cost(trial)
                if best is None or c < best[0]:
                    best = (c, list(perm))
            slots[g] = best[1]
    print(f"// (late, pads): {cost(slots)}", file=sys.stderr)
    # the row-sum partials of a half (two 16x16x32 MFMAs from a zero accumulator) are added into the running f32 sums
    # by two v_add_f32 >= 12 wait states after the second MFMA: block 1 (MFMAs at 6, 9) at gaps 12 / 13, block 0
    # (16, 19) in the next half's gaps 2 / 3
    for g, qb, j in ((12, 1, 0), (13, 1, 1), (2, 0, 0), (3, 0, 1)):
        slots[g].append(("A", qb, j))
    CAP = max(len(s) for s in slots)
    code = {"E": 0, "A": 1, "C": 2}
    rows = []
    for g, s in enumerate(slots):
        print(f"// gap {g:2d} {KIND[g]}: " + " ".join(f"{k}{qb}.{i}" for k, qb, i in s), file=sys.stderr)
        ops = [(code[k] << 6) | (qb << 5) | i for k, qb, i in s] + [0xFF]*(CAP - len(s))
        rows.append("{" + ", ".join(f"0x{o:02x}" for o in ops) + "}")
    print(f"constexpr unsigned char FW_SCHED_R[{NG}][{CAP}] = {{\n    " + ",\n    ".join(rows) + "};")
if __name__ == "__main__":
    main()
