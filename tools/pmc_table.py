"""Per-kernel median counters from rocprofv3 --pmc counter_collection CSVs: python tools/pmc_table.py <dir...> [substr]"""
import csv
import glob
import sys
from collections import defaultdict

dirs = [d for d in sys.argv[1:] if not d.startswith("@")]
sub = next((d[1:] for d in sys.argv[1:] if d.startswith("@")), "")
vals = defaultdict(lambda: defaultdict(list))
for d in dirs:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if sub not in n:
                continue
            key = (n.split("(")[0][-32:], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
    print(k, {c: f"{v:.4g}" for c, v in sorted(med.items())})
    cyc = med.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in med:
        print("    MFMA busy %.3f  VALU busy %.3f" % (med["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc),
                                                   4 * med.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * cyc)))
    if "SQ_WAIT_ANY" in med:
        tot = med["SQ_WAIT_ANY"] + med["SQ_WAIT_INST_ANY"] + med["SQ_ACTIVE_INST_ANY"]
        print("    wait_any %.2f wait_inst %.2f active %.2f (of wave cycles); lds bank conflict / insts_lds %.2f" % (
            med["SQ_WAIT_ANY"] / tot, med["SQ_WAIT_INST_ANY"] / tot, med["SQ_ACTIVE_INST_ANY"] / tot,
            med["SQ_LDS_BANK_CONFLICT"] / max(1, med["SQ_INSTS_LDS"])))
