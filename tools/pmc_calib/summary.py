"""FETCH_SIZE / WRITE_SIZE per known byte count for each access form of pmc_calib.hip:
python tools/pmc_calib/summary.py <tag> -> profiles/<tag>_pmc_calibration.json.
Every calibration kernel reads (or writes) 2^30 bytes once; the ratio is counter bytes
(KiB x 1024) / 2^30, so 0.5 = the counter reports half the bytes (double it)."""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "gpurun_out")
BYTES = 1 << 30


def per_kernel(path):
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"].replace("float __vector(2)", "v2f").replace("float __vector(4)", "v4f").split("(")[0]
            acc.setdefault(name, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(tag):
    res = {"tag": tag, "bytes_per_kernel": BYTES, "method": "rocprofv3 --pmc <counter> -- tools/pmc_calib/pmc_calib, "
           "one counter per pass; ratio = counter KiB * 1024 / bytes the kernel reads or writes", "forms": {}}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(OUT, f"pmc_calib_{counter}_{tag}", "run_counter_collection.csv")
        for k, v in sorted(per_kernel(path).items()):
            res["forms"].setdefault(k, {})[counter + "_ratio"] = v * 1024 / BYTES
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    out = os.path.join(REPO, "profiles", f"{tag}_pmc_calibration.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
