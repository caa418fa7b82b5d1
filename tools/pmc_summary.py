"""Summarise rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE runs of the same
bench command) into profiles/pmc_summary.json: per kernel the mean counters per dispatch
and the HBM traffic per launch, corrected as MI355X_MICROARCH.md "HBM" prescribes:
bytes = (FETCH_SIZE + WRITE_SIZE) * 1024, with FETCH_SIZE doubled for kernels whose reads
are 16-byte-per-lane streaming loads (gfx950 reports half of those).

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv STATS.csv OUT.json
"""
import csv
import json
import sys
from collections import defaultdict

# rocprof kernel name -> (bench kernel class, reads are 16-B/lane streams)
KMAP = {"k_gemm_tn": ("gemm_tn", True), "k_gemm_nn": ("gemm_nn", True),
        "k_gemm_nn_dot": ("gemm_nn_dot", True), "k_spmm": ("spmm", False),
        "k_fb_a": ("findbasis", True), "k_fb_b": ("findbasis", True), "k_fb_c": ("findbasis", True)}


def load(path, counter):
    vals = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter:
            vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(fetch_csv, write_csv, stats_csv, out_json):
    fe, wr = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    stats = {row["Name"]: row for row in csv.DictReader(open(stats_csv))}
    out = {"source": {"fetch": fetch_csv, "write": write_csv, "stats": stats_csv},
           "note": "FETCH_SIZE/WRITE_SIZE are KiB; fetch doubled for 16-B/lane streaming reads (gfx950)",
           "kernels": {}, "rocprof_kernels": {}}
    for name in sorted(set(fe) | set(wr)):
        f = sum(fe[name]) / max(len(fe[name]), 1)
        w = sum(wr[name]) / max(len(wr[name]), 1)
        cls, wide = KMAP.get(name, (name, False))
        traffic = ((2.0 if wide else 1.0) * f + w) * 1024.0
        st = stats.get(name)
        out["rocprof_kernels"][name] = {"dispatches": len(fe[name]), "fetch_kib_mean": f, "write_kib_mean": w,
                                        "fetch_corrected": wide, "traffic_bytes_per_launch": traffic,
                                        "avg_duration_ns": float(st["AverageNs"]) if st else None}
        if name in ("k_gemm_tn", "k_gemm_nn", "k_gemm_nn_dot", "k_spmm"):
            out["kernels"][cls] = {"traffic_bytes_per_launch": traffic, "rocprof_kernel": name}
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out["rocprof_kernels"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
