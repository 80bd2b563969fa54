"""Print the headline numbers of a bench.py JSON line (value, ms/step, stages, paths, top kernels)."""
import json
import sys

rec = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
print(f"value {rec['value']:.0f} {rec['unit']}  ms/step {rec['ms_per_step']:.3f}  n_gpus {rec['n_gpus']}  "
      f"frames/step {rec['config']['frames_per_step']:.0f}")
print("stages", {k: round(v, 3) for k, v in rec.get("stages_rank0", {}).items()}, "paths", rec.get("paths_rank0"))
ks = rec.get("kernels_rank0", {})
for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["ms_per_step"])[:8]:
    print(f"  {k:18s} mean {1000 * v['mean_ms']:9.2f} us  x{v['launches_per_step']:4d}  per-step {v['ms_per_step']:8.3f} ms"
          f"  {v['achieved_gbs'] or 0:8.1f} GB/s")
