#!/usr/bin/env python3
"""HBM traffic per FFT-conv call at the C4 shape (hyena.py:32-51 fftconv_ref; 768 rows x L = 262144, f32), for the
C4 bench line's roofline.traffic: the fftconv_fwd / fftconv_bwd KernelTimer names each launch several kernels
(column passes, row pass, inverse column passes, the dD row dot), so their bytes per call are summed over the
dispatches between marker kernels.

    run (GPU box, one pass per counter):
      rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/fetch -o run -- python3 tools/fft_traffic.py
      rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT/write -o run -- python3 tools/fft_traffic.py
    parse (anywhere):
      python3 tools/fft_traffic.py --parse OUT [profiles/traffic.json]

The run does one untimed fwd + bwd (allocations, twiddles), then NCALL forward calls and NCALL backward calls of
kernels.fftconv, each followed by a torch.cuda._sleep marker dispatch. Bytes = 2 x FETCH_SIZE (the gfx950 correction,
MI355X_MICROARCH.md) + WRITE_SIZE, per dispatch, summed per call.
"""
import csv
import json
import os
import sys

NCALL = 3
B, H, HD, L = 2, 6, 64, 262144


def run():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(0)
    u = torch.randn(B * H, HD, L, device="cuda", generator=g).requires_grad_(True)
    k = (torch.randn(HD, L, device="cuda", generator=g) * torch.exp(-torch.linspace(0, 8, L, device="cuda")))
    k.requires_grad_(True)
    D = torch.randn(HD, device="cuda", generator=g).requires_grad_(True)
    y = kernels.fftconv(u, k, D)
    gy = torch.randn_like(y)
    torch.autograd.grad(y, [u, k, D], gy)
    torch.cuda.synchronize()

    def marker():
        torch.cuda.synchronize()
        torch.cuda._sleep(100)
        torch.cuda.synchronize()

    marker()
    for _ in range(NCALL):
        y = kernels.fftconv(u, k, D)
        marker()
    for _ in range(NCALL):
        # the backward alone: the graph's forward ran above (outside the marked segments), retain it for repeats
        torch.autograd.grad(y, [u, k, D], gy, retain_graph=True)
        marker()
    print("fft_traffic run ok", flush=True)


def _rows(d):
    p = os.path.join(d, "run_counter_collection.csv")
    rows = list(csv.DictReader(open(p)))
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
    rows.sort(key=lambda r: int(r[key]))
    return rows


def _segments(rows):
    segs, cur, started = [], [], False
    for r in rows:
        name = r["Kernel_Name"]
        if "sleep" in name.lower() or "spin" in name.lower():
            if started:
                segs.append(cur)
            cur, started = [], True
            continue
        if started:
            cur.append((name, float(r["Counter_Value"])))
    return segs


def parse(out_dir, traffic_path=None):
    fetch, write = _segments(_rows(os.path.join(out_dir, "fetch"))), _segments(_rows(os.path.join(out_dir, "write")))
    assert len(fetch) == len(write) == 2 * NCALL, (len(fetch), len(write))
    res = {}
    for which, sl in (("fftconv_fwd", slice(0, NCALL)), ("fftconv_bwd", slice(NCALL, 2 * NCALL))):
        tot = []
        for fs, ws in zip(fetch[sl], write[sl]):
            lib = [i for i, (n, _) in enumerate(fs) if "lci::" in n]
            tot.append(sum(2.0 * fs[i][1] * 1024 + ws[i][1] * 1024 for i in lib))
            kern = sorted({fs[i][0].split("(")[0] for i in lib})
        rows = B * H * HD
        alg = (8.0 if which == "fftconv_fwd" else 16.0) * rows * L
        per = {}   # per-kernel bytes of the first call (read = 2 x FETCH_SIZE, write)
        fs, ws = fetch[sl][0], write[sl][0]
        for i, (nm, _) in enumerate(fs):
            if "lci::" in nm:
                key = f"{i}:{nm.split('(')[0]}"
                per[key] = {"read": 2.0 * fs[i][1] * 1024, "write": ws[i][1] * 1024}
                print(f"  {which} {key:60s} read {per[key]['read'] / 1e9:7.3f} GB  write {per[key]['write'] / 1e9:7.3f} GB")
        res[which] = {"bytes_per_call": sum(tot) / len(tot), "algorithmic_bytes": alg, "per_kernel": per,
                      "ratio_to_algorithmic": sum(tot) / len(tot) / alg, "kernels": kern, "calls": len(tot)}
        print(f"{which}: {res[which]['bytes_per_call'] / 1e9:.3f} GB per call, algorithmic {alg / 1e9:.3f} GB "
              f"({res[which]['ratio_to_algorithmic']:.2f}x); kernels {kern}")
    if traffic_path:
        doc = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
        wl = doc.setdefault("workloads", {}).setdefault("vit_hyena_p2_1024", {"source": out_dir, "kernels": {},
                                                                              "timers": {}})
        wl["fft_source"] = f"{out_dir} (tools/fft_traffic.py: {B * H * HD} rows x L={L}, the C4 call)"
        wl.setdefault("timers", {}).update(res)
        json.dump(doc, open(traffic_path, "w"), indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--parse":
        parse(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        run()
