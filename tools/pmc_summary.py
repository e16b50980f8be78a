"""Summarize rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/<tag>_pmc_<workload>.json.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: rocprofv3 reports
both in KiB, and on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
(16 B/lane) coalesced streaming read (MI355X_MICROARCH.md §HBM), so it is doubled.
Usage: python tools/pmc_summary.py <tag> <workload> <kernel-substring> <algorithmic-bytes-per-launch>
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(path, kernel):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    tag, workload, kernel, alg = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    out = os.path.join(REPO, "gpurun_out")
    fetch, nf = mean_counter(os.path.join(out, f"pmc_{workload}_FETCH_SIZE_{tag}", "run_counter_collection.csv"), kernel)
    write, nw = mean_counter(os.path.join(out, f"pmc_{workload}_WRITE_SIZE_{tag}", "run_counter_collection.csv"), kernel)
    hbm = 2 * fetch * 1024 + write * 1024
    res = {"workload": workload, "kernel": kernel, "tag": tag, "dispatches": [nf, nw],
           "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": hbm / alg,
           "method": "separate rocprofv3 --pmc passes; 2*FETCH_SIZE (gfx950 16-B stream calibration) + WRITE_SIZE"}
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    path = os.path.join(REPO, "profiles", f"{tag}_pmc_{workload}.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
