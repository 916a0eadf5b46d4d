"""Reduce the two rocprofv3 --pmc passes of tools/pmc_gateup.py to
profiles/pmc_gate_up.json: HBM bytes per gate/up launch with the gfx950 corrections
of MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of 16 B/lane streaming reads:
x2; WRITE_SIZE exact; both in KiB)."""
import csv
import json
import os
import sys

KERNEL = "gemv_dec_kernel<8, 1, 3, 0, 1, 1, 8>"


def mean_counter(path):
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    vals = [float(r["Counter_Value"]) for r in rows]
    return sum(vals) / len(vals), len(vals), rows[0]["Counter_Name"]


def main(out_dir="gpurun_out", dst="profiles/pmc_gate_up.json"):
    f, nf, cf = mean_counter(os.path.join(out_dir, "pmc_fetch", "pmc_counter_collection.csv"))
    w, nw, cw = mean_counter(os.path.join(out_dir, "pmc_write", "pmc_counter_collection.csv"))
    hbm = f * 1024 * 2 + w * 1024
    alg = 2 * 9216 * 2304 * 2 + 8 * 2304 * 2 + 8 * 9216 * 2
    res = {"kernel": KERNEL + " (decode gate/up GEGLU, M=8, N=18432, K=2304)",
           "launches": nf, "FETCH_SIZE_KiB_mean": f, "WRITE_SIZE_KiB_mean": w,
           "correction": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE is half of 16B/lane reads)",
           "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": round(hbm / alg, 4),
           "workload": "26 distinct weight sets rotated (2.2 GB > 256 MiB Infinity Cache), tools/pmc_gateup.py"}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
