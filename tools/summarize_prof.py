#!/usr/bin/env python3
"""Summarize a tools/profile_bench.sh run: per-kernel average duration (kernel trace) and HBM traffic
(PMC passes) for the liblci kernels.

Traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled.
Only dispatches after the first `skip_frac` of the run are counted (warm-up includes MIOpen's find phase).

    python tools/summarize_prof.py gpurun_out/prof_r01 > profiles/r01_rocprof_summary.md
    python tools/summarize_prof.py gpurun_out/prof_r01 0.5 profiles/traffic.json [workload]   # + HBM bytes

Directory layouts: tools/profile_bench.sh (trace/, fetch/, write/) or tools/gpu_round.sh (trace/, pmc_FETCH_SIZE/,
pmc_WRITE_SIZE/, pmc_SQ_WAVES/). The SQ pass gives, per kernel (MI355X_MICROARCH.md §rocprofv3 PMC slots,
per-instruction constants): cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs), MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles), VALU busy = 4 SQ_ACTIVE_INST_VALU (quad-cycles) / (1024 x cycles),
executed MFMA FLOP = SQ_INSTS_MFMA x 32768 (v_mfma_f32_32x32x16_bf16; x 16384 for the 16x16x32 attention kernels),
effective clock = cycles / duration.
"""
import csv
import os
import sys
from collections import defaultdict


# KernelTimer name (bench.py) -> the liblci kernels it launches (rocprofv3 names carry template arguments)
TIMER_KERNELS = {"conv3": r"conv3_fwd\w*_kernel", "conv3_wgrad": r"conv3_wgrad\w*_kernel",
                 "attn_bwd_dkdv": r"attn_bwd_dkdv\w*_kernel", "attn_bwd_dq": r"attn_bwd_dq\w*_kernel",
                 "attn_fwd": r"(?<!win_)attn_fwd\w*_kernel", "gemm_bt": r"gemm_bt_kernel", "window_attn_bwd": r"win_attn_bwd\w*_kernel",
                 "window_attn_fwd": r"win_attn_fwd\w*_kernel", "selective_scan_bwd": r"scan_bwd\w*_kernel",
                 "linear_wgrad": r"linear_wgrad\w*_kernel"}


def short(name):
    for key in ("attn_fwd", "attn_bwd_dkdv", "attn_bwd_dq", "attn_bwd_delta", "patch_embed", "scan", "window", "fft_",
                "fftconv", "hyena", "dwconv", "conv3", "inorm", "ln_fwd", "ln_bwd", "linear_", "gelu_", "upsample2x", "hf_",
                "gemm_bt", "win_", "longconv", "row_dot"):
        if key in name:
            return name.split("(")[0].replace("void ", "")
    return None


def load_trace(path):
    rows = list(csv.DictReader(open(path)))
    return rows


def sq_summary(d, skip_frac):
    p = os.path.join(d, "pmc_SQ_WAVES", "run_counter_collection.csv")
    if not os.path.exists(p):
        return None
    rows = list(csv.DictReader(open(p)))
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        per[(r["Dispatch_Id"], r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
        per[(r["Dispatch_Id"], r["Kernel_Name"])]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    keys = sorted(per, key=lambda k: int(k[0]))
    acc = defaultdict(lambda: defaultdict(float))
    for k in keys[int(len(keys) * skip_frac):]:
        n = short(k[1])
        if not n:
            continue
        c = per[k]
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        a = acc[n]
        a["n"] += 1
        a["ns"] += c["_ns"]
        a["cyc"] += cyc
        a["mfma"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["valu"] += 4 * c["SQ_ACTIVE_INST_VALU"]
        # FLOP per MFMA instruction: 16x16x32 kernels (the *16 attention kernels) 16384, 32x32x16 32768
        a["flop"] += (16384 if ("dkdv16" in k[1] or "dq16" in k[1] or "fwd16" in k[1]) else 32768) * c["SQ_INSTS_MFMA"]
    out = {}
    for n, a in acc.items():
        out[n] = {"n": int(a["n"]), "ms": a["ns"] / a["n"] / 1e6, "clock": a["cyc"] / a["ns"],
                  "mfma": a["mfma"] / (1024 * a["cyc"]), "valu": a["valu"] / (1024 * a["cyc"]),
                  "flop": a["flop"] / a["n"]}
    return out


def main():
    d = sys.argv[1]
    skip_frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    tr = load_trace(os.path.join(d, "trace", "run_kernel_trace.csv"))
    start = int(len(tr) * skip_frac)
    dur = defaultdict(list)
    for r in tr[start:]:
        n = short(r["Kernel_Name"])
        if n:
            dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    counters = {}
    for c in ("fetch", "write"):
        p = os.path.join(d, c, "run_counter_collection.csv")
        if not os.path.exists(p):
            p = os.path.join(d, "pmc_" + {"fetch": "FETCH_SIZE", "write": "WRITE_SIZE"}[c], "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        rows = list(csv.DictReader(open(p)))
        acc = defaultdict(list)
        for r in rows[int(len(rows) * skip_frac):]:
            n = short(r["Kernel_Name"])
            if n:
                acc[n].append(float(r["Counter_Value"]))
        counters[c] = acc
    if len(sys.argv) > 3:   # per-kernel HBM bytes per launch as JSON (bench.py's roofline.traffic)
        import json
        import re
        out = {}
        for n in dur:
            f = counters.get("fetch", {}).get(n)
            w = counters.get("write", {}).get(n)
            if f and w:
                out[n] = {"read_bytes": 2.0 * sum(f) / len(f) * 1024, "write_bytes": sum(w) / len(w) * 1024,
                          "avg_ms": sum(dur[n]) / len(dur[n]), "launches": len(dur[n])}
        # per KernelTimer name (bench.py's roofline kernel): the launch-weighted mean over the kernels it launches
        timers = {}
        for t, pat in TIMER_KERNELS.items():
            hits = [v for k, v in out.items() if re.search(pat, k)]
            if hits:
                nl = sum(v["launches"] for v in hits)
                timers[t] = {"bytes_per_call": sum(v["launches"] * (v["read_bytes"] + v["write_bytes"]) for v in hits) / nl,
                             "kernels": sorted(k for k, v in out.items() if re.search(pat, k)), "launches": nl}
        path, wl = sys.argv[3], (sys.argv[4] if len(sys.argv) > 4 else "vit_p2_512")
        doc = json.load(open(path)) if os.path.exists(path) else {}
        doc.pop("kernels", None); doc.pop("source", None)
        doc["note"] = ("per workload: HBM bytes per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                       "that workload (FETCH_SIZE x2, the gfx950 correction; KiB -> bytes); `timers` = per KernelTimer "
                       "name, launch-weighted over the kernels it launches")
        prev = doc.setdefault("workloads", {}).get(wl, {})
        # timers this run did not produce (tools/fft_traffic.py's fftconv_fwd / _bwd entries) are kept
        kept = {k: v for k, v in prev.get("timers", {}).items() if k not in timers}
        entry = {"source": d, "kernels": out, "timers": {**kept, **timers}}
        if "fft_source" in prev:
            entry["fft_source"] = prev["fft_source"]
        doc["workloads"][wl] = entry
        json.dump(doc, open(path, "w"), indent=1)
    print(f"# rocprofv3 summary: {d}\n")
    print(f"Kernel-trace dispatches counted: the last {100 * (1 - skip_frac):.0f}% of the run "
          f"({len(tr) - start} of {len(tr)} dispatches).\n")
    print("| kernel | dispatches | avg ms | min ms | max ms | HBM read MB/launch (2x FETCH_SIZE) | HBM write MB/launch |")
    print("|---|---|---|---|---|---|---|")
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        f = counters.get("fetch", {}).get(n)
        w = counters.get("write", {}).get(n)
        fm = f"{2 * sum(f) / len(f) / 1024:.1f}" if f else "n/a"
        wm = f"{sum(w) / len(w) / 1024:.1f}" if w else "n/a"
        print(f"| {n} | {len(v)} | {sum(v) / len(v):.3f} | {min(v):.3f} | {max(v):.3f} | {fm} | {wm} |")
    sq = sq_summary(d, skip_frac)
    if sq:
        print("\nSQ counter pass (MFMA / VALU busy per SIMD-cycle, executed MFMA FLOP per launch, effective clock):\n")
        print("| kernel | dispatches | avg ms | clock GHz | MFMA busy | VALU busy | executed TFLOP/launch | executed TFLOP/s |")
        print("|---|---|---|---|---|---|---|---|")
        for n, v in sorted(sq.items(), key=lambda kv: -kv[1]["ms"] * kv[1]["n"]):
            print(f"| {n} | {v['n']} | {v['ms']:.3f} | {v['clock']:.2f} | {v['mfma']:.3f} | {v['valu']:.3f} | "
                  f"{v['flop'] / 1e12:.2f} | {v['flop'] / v['ms'] / 1e9:.0f} |")
    print("\nrocprofv3 --stats top kernels (whole run, includes warm-up / MIOpen find):\n")
    st = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))))
    st.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print("| kernel | calls | total ms | avg ms | % |")
    print("|---|---|---|---|---|")
    for r in st[:12]:
        print(f"| {r['Name'][:80]} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.1f} | "
              f"{float(r['AverageNs']) / 1e6:.3f} | {float(r['Percentage']):.1f} |")


if __name__ == "__main__":
    main()
