"""Per-kernel averages of the counters in the rocprofv3 PMC passes gpurun_out/<prefix>1..N
(tools/gpu/pmc_kernel.sh): one line per kernel name with each counter's mean per launch.
FETCH_SIZE / WRITE_SIZE are in KB per launch as rocprofv3 reports them (the gfx950
correction for 16-B/lane loads is left to the reader: MI355X_MICROARCH.md, HBM)."""
import csv
import glob
import re
import sys
from collections import defaultdict

prefix = sys.argv[1]
per = defaultdict(float)  # (file, kernel, dispatch, counter) -> value summed over its rows
for f in sorted(glob.glob(prefix + "*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:70]
        per[(f, name, r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
vals = defaultdict(lambda: defaultdict(list))
for (f, name, _d, cn), v in per.items():
    vals[name][cn].append(v)
for name, cs in sorted(vals.items()):
    parts = [f"{c}={sum(v) / len(v):.4g}(n={len(v)})" for c, v in sorted(cs.items())]
    print(name + ": " + " ".join(parts))
