"""Summarise rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE runs of the same
bench command) into profiles/pmc_summary.json: per kernel class the HBM traffic per launch,
corrected as MI355X_MICROARCH.md "HBM" prescribes: bytes = (FETCH_SIZE + WRITE_SIZE) * 1024,
with FETCH_SIZE doubled for kernels whose reads are 16-byte-per-lane streaming loads (gfx950
reports half of those).  Template instantiations of one kernel (k_nn_tn_w<32, 7, 2>, ...)
are pooled into their bench class: traffic per launch = total corrected bytes / launches,
the same averaging bench.py uses for the achieved rate.

With the bench line of the same command (BENCH.json, optional) each class also gets
`ratio` = PMC traffic per launch / algorithmic bytes per launch (the bench's per-class byte
tally), which bench.py multiplies by its own bytes per launch for roofline.traffic.  The PMC
run must cover whole restart cycles (as bench.py's steps do) so both averages are taken over
the same mix of projection widths.

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv STATS.csv OUT.json [BENCH.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict

# kernel base name -> (bench class, reads are 16-B/lane streams)
#   spmm: CSR values/keys are 2-8 B per lane and X pairs 16 B -> left uncorrected
KMAP = {"k_gemm_tn": ("gemm_tn", True), "k_gemm_nn": ("gemm_nn", True),
        "k_gemm_nn_dot": ("gemm_nn_dot", True), "k_nn_tn": ("nn_tn", True), "k_nn_tn_w": ("nn_tn", True),
        "k_spmm": ("spmm", False), "k_spmm_pair": ("spmm", False),
        # template SpMM: X pairs are 16-B/lane loads (the 1-B template ids are 0.4 % of the bytes)
        "k_spmm_tplr": ("spmm", True), "k_spmm_tpl": ("spmm", True), "k_spmm_sell": ("spmm", False),
        # lane-shared template and plane-march SpMM: X pairs as 16-B/lane loads
        "k_spmm_tpl3": ("spmm", True), "k_spmm_march": ("spmm", True), "k_spmm_march7": ("spmm", True),
        "k_spmm_march27": ("spmm", True),
        "k_fb_a": ("findbasis", True), "k_fb_a01": ("findbasis", True), "k_fb_b2": ("findbasis", True),
        "k_fb_ca": ("findbasis", True), "k_gemm_nn_gram": ("gemm_nn_dot", True),
        "k_fbg_gram": ("findbasis", True), "k_fbg_a": ("findbasis", True), "k_fbg_b": ("findbasis", True),
        "k_fbg_gram_m": ("findbasis", False), "k_fbg_b_m": ("findbasis", False)}


def base(name):
    m = re.search(r"migmres::(k_[a-z0-9_]+)", name) or re.search(r"\b(k_[a-z0-9_]+)", name)
    return m.group(1) if m else name


def load(path, counter):
    vals = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter:
            vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(fetch_csv, write_csv, stats_csv, out_json, bench_json=None):
    fe, wr = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    stats = {row["Name"]: row for row in csv.DictReader(open(stats_csv))}
    out = {"source": {"fetch": fetch_csv, "write": write_csv, "stats": stats_csv},
           "note": "FETCH_SIZE/WRITE_SIZE are KiB; fetch doubled for 16-B/lane streaming reads (gfx950)",
           "kernels": {}, "rocprof_kernels": {}}
    pool = defaultdict(lambda: [0.0, 0])
    for name in sorted(set(fe) | set(wr)):
        nf, nw = len(fe[name]), len(wr[name])
        f = sum(fe[name]) / max(nf, 1)
        w = sum(wr[name]) / max(nw, 1)
        b = base(name)
        cls, wide = KMAP.get(b, (b, False))
        traffic = ((2.0 if wide else 1.0) * f + w) * 1024.0
        st = stats.get(name)
        out["rocprof_kernels"][name] = {"class": cls, "dispatches": nf, "fetch_kib_mean": f, "write_kib_mean": w,
                                        "fetch_corrected": wide, "traffic_bytes_per_launch": traffic,
                                        "avg_duration_ns": float(st["AverageNs"]) if st else None}
        if b in KMAP:
            pool[cls][0] += traffic * nf
            pool[cls][1] += nf
    alg = {}
    if bench_json:
        line = [ln for ln in open(bench_json).read().splitlines() if ln.strip().startswith("{")][-1]
        b = json.loads(line)
        out["source"]["bench"] = bench_json
        for cls, v in b.get("kernels", {}).items():
            if v.get("GBps") and v.get("launches"):
                alg[cls] = v["GBps"] * 1e9 * v["ms"] / 1e3 / v["launches"]
    for cls, (tot, n) in pool.items():
        out["kernels"][cls] = {"traffic_bytes_per_launch": tot / max(n, 1), "dispatches": n}
        if cls in alg:
            out["kernels"][cls]["algorithmic_bytes_per_launch"] = alg[cls]
            out["kernels"][cls]["ratio"] = tot / max(n, 1) / alg[cls]
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
