#!/usr/bin/env python3
"""Generate the VALU placement of the one-wave-per-SIMD attention forward (csrc/attention.hip, attn_fwd_hs_kernel).

Per 32-key half a wave issues 16 v_mfma_f32_32x32x16_bf16 in the order
  gaps 0-3: S^T chain of query block 0 | 4-7: O^T += V^T P^T of block 1 (previous half) |
  8-11: S^T chain of block 1 | 12-15: O^T += V^T P^T of block 0,
and per query block 40 VALU ops: 16 exp2 (E), 16 row-sum adds (A, element i into partial sum i & 3), 8 bf16 pair
conversions (C, elements 2c, 2c+1). The schedule is periodic (16 gaps); block 1's ops wrap into the next half. Rules:
E from two gaps after the chain's last MFMA, A and C in a later gap than the exps they read, at most 2 exps and 5 ops
per gap; a block's packs of elements 0-7 (C 0-3) complete one gap before its first PV MFMA, elements 8-15 (C 4-7)
one gap before its third. Within a gap the op order avoids an op directly after the exp it reads (the compiler pads
that with an s_nop 0 and does not count the asm MFMA between gaps). Output (stdout): the C++ table FW_SCHED[16][5]
(kind << 6 | block << 5 | index; 0xff = none); the placement is listed on stderr.
"""
import itertools
import sys

NG = 16
START_E = {0: 5, 1: 13}      # S chains at gaps 0-3 / 8-11
PV = {0: 12, 1: 4 + NG}      # first PV gap that reads the block's packs
CAP_E, CAP = 2, 5


def main():
    cap_e = [0] * NG
    slots = [[] for _ in range(NG)]
    for qb in (1, 0):        # block 1 wraps into the next half: place it first
        tE, tA, tC = {}, {}, {}
        g = START_E[qb]
        while len(tC) < 8 or len(tA) < 16:
            gi = g % NG
            s = slots[gi]
            for j in range(8):                       # conversions first: they gate the PV MFMAs
                if j not in tC and 2 * j in tE and 2 * j + 1 in tE and max(tE[2 * j], tE[2 * j + 1]) < g and \
                        len(s) < CAP:
                    tC[j] = g
                    s.append(("C", qb, j))
            for e in range(16):
                if e in tE and e not in tA and tE[e] < g and len(s) < CAP - (1 if len(tC) < 8 else 0):
                    tA[e] = g
                    s.append(("A", qb, e))
            for e in range(16):
                if e not in tE and cap_e[gi] < CAP_E and len(s) < CAP:
                    tE[e] = g
                    cap_e[gi] += 1
                    s.append(("E", qb, e))
            g += 1
            assert g < START_E[qb] + 2 * NG, "does not fit"
        assert max(tC[j] for j in range(4)) < PV[qb], (qb, tC)
        assert max(tC[j] for j in range(4, 8)) < PV[qb] + 2, (qb, tC)
        assert max(tA.values()) < START_E[qb] + NG, (qb, tA)   # done before the block's next chain's exps
    code = {"E": 0, "A": 1, "C": 2}

    def reads(a, b):   # does op b read op a's result?
        if a[1] != b[1] or a[0] != "E":
            return False
        return (b[0] == "A" and a[2] == b[2]) or (b[0] == "C" and a[2] in (2 * b[2], 2 * b[2] + 1))

    for _ in range(2):   # second pass: gap 0 sees gap 15's final order
        for g in range(NG):
            prev = slots[g - 1][-1] if slots[g - 1] else None
            best = None
            for perm in itertools.permutations(slots[g]):
                chain = [prev] + list(perm)
                pads = sum(1 for i in range(len(perm)) if chain[i] is not None and reads(chain[i], chain[i + 1]))
                if best is None or pads < best[0]:
                    best = (pads, list(perm))
            slots[g] = best[1]
    pads = sum(1 for g in range(NG) for i, op in enumerate(slots[g])
               if reads((slots[g - 1][-1] if i == 0 else slots[g][i - 1]) if (i or slots[g - 1]) else ("X", 0, 0), op))
    print(f"// hazard pads left: {pads}", file=sys.stderr)
    rows = []
    for g, s in enumerate(slots):
        print(f"// gap {g:2d}: " + " ".join(f"{k}{qb}.{i}" for k, qb, i in s), file=sys.stderr)
        ops = [(code[k] << 6) | (qb << 5) | i for k, qb, i in s] + [0xFF] * (CAP - len(s))
        rows.append("{" + ", ".join(f"0x{o:02x}" for o in ops) + "}")
    print(f"constexpr unsigned char FW_SCHED[{NG}][{CAP}] = {{\n    " + ",\n    ".join(rows) + "};")


if __name__ == "__main__":
    main()
