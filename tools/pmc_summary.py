"""Summarize rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/<tag>_pmc_<label>.json.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: rocprofv3 reports
both in KiB, and on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
(16 B/lane) coalesced streaming read (MI355X_MICROARCH.md §HBM), so it is doubled.

Usage:
  python tools/pmc_summary.py <tag>      every pass of tools/gpu_pmc.sh <tag>, algorithmic
                                         bytes taken from the same round's bench lines
                                         (gpurun_out/bench_<w>_<tag>.json); the summaries carry
                                         bench.code_tag() so bench.py uses them only for this code
  python tools/pmc_summary.py <tag> <pmc-dir-workload> <kernel-substring> <alg-bytes> [label]
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")


def mean_counter(path, kernel, every_grid=False):
    """mean counter value over the kernel's dispatches with its most common grid (the
    steady-state launches: priming launches of the step kernel have other grids), or over
    every dispatch (every_grid: the step groups' slice launches, whose grids cycle with the
    level windows -- their mean over many windows is the steady-state mean)"""
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                rows.append((row["Grid_Size"], float(row["Counter_Value"])))
    if not rows:
        return None, 0
    grids = {}
    for g, _ in rows:
        grids[g] = grids.get(g, 0) + 1
    g = max(grids, key=grids.get)
    vals = [v for gg, v in rows if every_grid or gg == g]
    return sum(vals) / len(vals), len(vals)


def summarize(tag, workload, kernel, alg, label=None, every_grid=False):
    label = label or workload
    fetch, nf = mean_counter(os.path.join(OUT, f"pmc_{workload}_FETCH_SIZE_{tag}", "run_counter_collection.csv"), kernel,
                             every_grid)
    write, nw = mean_counter(os.path.join(OUT, f"pmc_{workload}_WRITE_SIZE_{tag}", "run_counter_collection.csv"), kernel,
                             every_grid)
    if fetch is None or write is None:
        print(f"{label}: no dispatches of {kernel!r}", file=sys.stderr)
        return None
    hbm = 2 * fetch * 1024 + write * 1024
    sys.path.insert(0, REPO)
    import bench

    res = {"workload": label, "kernel": kernel, "tag": tag, "code_tag": bench.code_tag(), "dispatches": [nf, nw],
           "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": hbm / alg,
           "method": "separate rocprofv3 --pmc passes; 2*FETCH_SIZE (gfx950 16-B stream calibration) + WRITE_SIZE"}
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", f"{tag}_pmc_{label}.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return res


def bench_line(tag, workload):
    with open(os.path.join(OUT, f"bench_{workload}_{tag}.json")) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def main():
    tag = sys.argv[1]
    if len(sys.argv) > 2:
        summarize(tag, sys.argv[2], sys.argv[3], float(sys.argv[4]), sys.argv[5] if len(sys.argv) > 5 else None)
        return
    for w in ("c5full", "c5", "c4"):
        if not os.path.exists(os.path.join(OUT, f"pmc_{w}_FETCH_SIZE_{tag}")):
            continue
        b = bench_line(tag, w)
        r = b["roofline"]
        if r.get("step_group", r.get("steps_per_launch", 1)) > 1:  # step groups: the slice and block kernels
            for k in r["kernels"]:
                name = k["kernel"].split("<")[0]
                summarize(tag, w, name, k["algorithmic_bytes_per_launch"], f"{w}_{name}", every_grid=True)
        else:
            summarize(tag, w, "k_lvl_step", r["algorithmic_bytes_per_launch"], w)
        summarize(tag, w, "k_upols_step", b["per_block_step"]["algorithmic_bytes_per_launch"], w + "_plain")
        if b.get("offline"):
            o = b["offline"]
            summarize(tag, w, o["kernel"].split("<")[0], o["algorithmic_bytes_per_launch"], w + "_offline")
    if not os.path.exists(os.path.join(OUT, f"pmc_c2_FETCH_SIZE_{tag}")):
        return
    b = bench_line(tag, "c2")
    summarize(tag, "c2", "k_c2c_lds<4096", b["roofline"]["algorithmic_bytes_per_launch"], "c2")


if __name__ == "__main__":
    main()
