"""Print a bench JSON line's step time, roofline and per-kernel breakdown (liblci kernels timed with HIP events)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.load(open(path))
    print(f"== {path}: {d['ms_per_step']} ms/step, {d['value']:.0f} {d['unit']}, peak {d.get('peak_memory_gb')} GB")
    print("   roofline:", json.dumps(d.get("roofline")))
    tot = 0.0
    for n, v in sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms_per_step"]):
        tot += v["ms_per_step"]
        rate = {x: v[x] for x in ("tflops", "gbs") if x in v}
        print(f"   {n:28s} {v['ms_per_step']:8.2f} ms/step  calls {v['calls_per_step']:6.1f}  avg {v['avg_ms']:.3f} {rate}")
    print(f"   total liblci {tot:.1f} ms/step")
