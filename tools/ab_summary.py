"""Summarise an alternated A/B log of tools/gpu_probe.py lines (dev tool):
mean ms_fused per (scene, lib) and each lib's ratio to the first lib of the scene.
usage: ab_summary.py LOG.jsonl [key]   (key: the field naming the variant, default "lib")"""
import collections
import json
import sys

path = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "lib"
runs = collections.defaultdict(list)
order = []
for line in open(path):
    if not line.startswith("{"):
        continue
    r = json.loads(line)
    k = (r.get("scene"), str(r.get(key)))
    if k not in runs:
        order.append(k)
    runs[k].append(r["ms_fused"])
base = {}
for scene, lib in order:
    ms = runs[(scene, lib)]
    mean = sum(ms) / len(ms)
    base.setdefault(scene, mean)
    print(f"{scene:10s} {lib:12s} n={len(ms)} mean={mean:9.3f} ms  ratio={mean / base[scene]:.4f}  "
          f"runs={[round(x, 2) for x in ms]}")
