#!/usr/bin/env python3
"""Tune the torch Linear / matmul GEMMs of a bench workload with PyTorch-ROCm TunableOp on top of the shipped table.

Runs `bench.run_workload(workload)` for one warm-up + one timed step with TunableOp tuning ON, starting from
long_context_biomedical_imaging_amd/tunableop_gfx950.csv, and writes the merged table (old + newly tuned shapes) to
--out. Copy that file over the shipped table after checking it. Usage (GPU box):
    python tools/tune_gemms.py --workload vit_mamba_p2_256 --out gpurun_out/tune/c5.csv [--max-ms 15]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--table", default=None, help="start table (default: the shipped one)")
    ap.add_argument("--max-ms", type=int, default=15, help="max tuning duration per solution candidate (ms)")
    ap.add_argument("--max-iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None)
    a = ap.parse_args()
    import bench
    from long_context_biomedical_imaging_amd import trainer
    import torch.cuda.tunable as tunable
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_max_tuning_duration(a.max_ms)
    tunable.set_max_tuning_iterations(a.max_iters)
    tunable.set_filename(os.path.abspath(a.out))
    print("read start table:", tunable.read_file(a.table or trainer.TUNED_GEMMS), file=sys.stderr, flush=True)
    batch = a.batch or (2 if a.workload in ("vit_p2_512", "vit_hyena_p2_512", "vit_hyena_p2_1024") else 1)
    res = bench.run_workload(a.workload, batch, 1, 1, 0, 1, dev, kernel_timer=False)
    print("step ms", res["ms_per_step"] if res else None, file=sys.stderr, flush=True)
    tunable.write_file(os.path.abspath(a.out))
    print("wrote", a.out, len(tunable.get_results()), "results", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
