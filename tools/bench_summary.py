"""One line per bench JSON: label, it/s and each kernel class's ms per launch and GB/s."""
import json
import sys

path, label = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
line = [l for l in open(path) if l.startswith("{")][-1]
d = json.loads(line)
ks = d.get("kernels", {})
parts = [f"{n}={v['ms'] / max(v['launches'], 1):.3f}ms/{v['GBps'] / 1e3:.2f}" for n, v in
         sorted(ks.items(), key=lambda kv: -kv[1]["ms"])[:8]]
print(f"{label:28s} {d['value']:9.2f} it/s  " + " ".join(parts))
