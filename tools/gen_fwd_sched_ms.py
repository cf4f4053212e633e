#!/usr/bin/env python3
"""Generate the VALU placement of the attention forward with MFMA row sums (csrc/attention.hip, LCI_FWD_MSUM).

Per 32-key half a wave issues 20 v_mfma_f32_32x32x16_bf16 in the order
  gaps 0-3: S^T chain of query block 0 | 4-7: O^T += V^T P^T of block 1 (previous half) | 8-9: row sums of block 1
  (ones . P^T, one per k-step) | 10-13: S^T chain of block 1 | 14-17: O^T of block 0 | 18-19: row sums of block 0,
and per query block 24 VALU ops: 16 exp2 (E) and 8 bf16 pair conversions (C, elements 2c, 2c+1); the row sum is the
MFMA's, so the 16 row-sum adds of tools/gen_fwd_sched.py are gone. Periodic (20 gaps); block 1's ops wrap into the next
half. Rules: E from two gaps after the chain's last MFMA, C in a later gap than both exps it reads, <= 2 exps and
<= 3 ops per gap; a block's packs of elements 0-7 (C 0-3) complete one gap before its first PV MFMA, elements 8-15
(C 4-7) one gap before its third; within a gap no op directly after the exp it reads. Output (stdout): the C++
table FW_SCHED_MS[20][3] (kind << 6 | block << 5 | index; 0xff = none) and FW_MS_START_E1; placement on stderr.
"""
import itertools
import sys

NG = 20
START_E = {0: 5, 1: 15}      # S chains at gaps 0-3 / 10-13
PV = {0: 14, 1: 4 + NG}      # first PV gap that reads the block's packs (k-step 0); k-step 1 two gaps later
CAP_E, CAP = 2, 3


def main():
    cap_e = [0] * NG
    slots = [[] for _ in range(NG)]
    for qb in (1, 0):
        tE, tC = {}, {}
        g = START_E[qb]
        while len(tC) < 8:
            gi = g % NG
            s = slots[gi]
            for j in range(8):
                if j not in tC and 2 * j in tE and 2 * j + 1 in tE and max(tE[2 * j], tE[2 * j + 1]) < g and \
                        len(s) < CAP:
                    tC[j] = g
                    s.append(("C", qb, j))
            for e in range(16):
                if e not in tE and cap_e[gi] < CAP_E and len(s) < CAP:
                    tE[e] = g
                    cap_e[gi] += 1
                    s.append(("E", qb, e))
            g += 1
            assert g < START_E[qb] + 2 * NG, "does not fit"
        assert max(tC[j] for j in range(4)) < PV[qb], (qb, tC)
        assert max(tC[j] for j in range(4, 8)) < PV[qb] + 2, (qb, tC)
        assert max(tC.values()) < START_E[qb] + NG - 5, (qb, tC)   # before the block's next chain
    code = {"E": 0, "C": 2}

    def reads(a, b):
        return a[1] == b[1] and a[0] == "E" and b[0] == "C" and a[2] in (2 * b[2], 2 * b[2] + 1)

    for _ in range(2):
        for g in range(NG):
            prev = slots[g - 1][-1] if slots[g - 1] else None
            best = None
            for perm in itertools.permutations(slots[g]):
                chain = [prev] + list(perm)
                pads = sum(1 for i in range(len(perm)) if chain[i] is not None and reads(chain[i], chain[i + 1]))
                if best is None or pads < best[0]:
                    best = (pads, list(perm))
            slots[g] = best[1]
    rows = []
    for g, s in enumerate(slots):
        print(f"// gap {g:2d}: " + " ".join(f"{k}{qb}.{i}" for k, qb, i in s), file=sys.stderr)
        ops = [(code[k] << 6) | (qb << 5) | i for k, qb, i in s] + [0xFF] * (CAP - len(s))
        rows.append("{" + ", ".join(f"0x{o:02x}" for o in ops) + "}")
    print(f"constexpr int FW_MS_START_E1 = {START_E[1]};")
    print(f"constexpr unsigned char FW_SCHED_MS[{NG}][{CAP}] = {{\n    " + ",\n    ".join(rows) + "};")


if __name__ == "__main__":
    main()
