"""GPU busy time per streaming step from a rocprofv3 kernel trace (run_kernel_trace.csv) of a
bench.py run with step groups: the block launches of the main handle (the k_lvl_block grid with
the most GPU time) and every k_lvl_slices launch between the first and the last of them; the
union of their [start, end) intervals divided by the number of block launches. The two kernels
run side by side on two streams, so per-kernel average durations add up to more than a step;
this is the figure bench.py's roofline.kernel_avg_ms (the step pair) is compared against.

    python tools/step_busy.py <run_kernel_trace.csv> [algorithmic_bytes_per_step]

With a trace of a NEO_BENCH_MARK=1 run the figure is taken over the streaming timed region alone
(between the last marker add and the marker mul after it, as tools/trace_region.py), i.e. the
same steps bench.py's wall clock times; otherwise over every block launch of the main handle
(which includes the instrumented, latency and host round-trip runs).
"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
region = None
small = [i for i, r in enumerate(rows) if int(r["Grid_Size_X"]) <= 512]
adds = [i for i in small if "OnSelf_add" in rows[i]["Kernel_Name"]]
if adds:
    muls = [i for i in small if "MulFunctor" in rows[i]["Kernel_Name"] and i > adds[-1]]
    if muls:
        region = (int(rows[adds[-1]]["End_Timestamp"]), int(rows[muls[0]]["Start_Timestamp"]))
        rows = [r for r in rows if region[0] <= int(r["Start_Timestamp"]) < region[1]]
blk = [r for r in rows if "k_lvl_block" in r["Kernel_Name"]]
tot = collections.Counter()
for r in blk:
    tot[r["Grid_Size_X"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
grid = tot.most_common(1)[0][0]  # the main handle's launches: the most GPU time
blk = [r for r in blk if r["Grid_Size_X"] == grid]
iv = lambda r: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
b = sorted(iv(r) for r in blk)
lo, hi = b[0][0], b[-1][1]
sl = sorted(iv(r) for r in rows if "k_lvl_slices" in r["Kernel_Name"] and lo <= int(r["Start_Timestamp"]) <= hi)
busy, cur = 0, None
for s, e in sorted(b + sl):
    if cur is None or s > cur[1]:
        if cur:
            busy += cur[1] - cur[0]
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
busy += cur[1] - cur[0]
# the whole marked region: every kernel in it (block and slices launches of this handle; the
# marker kernels at its edges), clipped to the region, so a slices launch that began before the
# first block or ends after the last one counts where it runs
def union(ivs, lo_, hi_):
    tot, c = 0, None
    for s_, e_ in sorted((max(s_, lo_), min(e_, hi_)) for s_, e_ in ivs):
        if e_ <= s_:
            continue
        if c is None or s_ > c[1]:
            if c:
                tot += c[1] - c[0]
            c = [s_, e_]
        else:
            c[1] = max(c[1], e_)
    return tot + (c[1] - c[0] if c else 0)
reg = {}
if region:
    all_iv = [iv(r) for r in rows]
    ours = [iv(r) for r in rows if "k_lvl_block" in r["Kernel_Name"] or "k_lvl_slices" in r["Kernel_Name"]]
    reg = {"region_busy_us_per_step": union(ours, *region) / len(b) / 1e3,
           "region_idle_us": (region[1] - region[0] - union(all_iv, *region)) / 1e3}
out = {"trace": sys.argv[1], "timed_region_only": region is not None,
       "region_us": (region[1] - region[0]) / 1e3 if region else None, "block_grid": int(grid), "block_launches": len(b), "slice_launches": len(sl),
       "busy_ns": busy, "busy_us_per_step": busy / len(b) / 1e3,
       "block_avg_us": sum(e - s for s, e in b) / len(b) / 1e3,
       "slices_avg_us": sum(e - s for s, e in sl) / max(len(sl), 1) / 1e3,
       **reg,
       "note": "busy_us_per_step: union of the main block launches and the slices launches that start between the "
               "first and the last of them / block launches (undercounts: a slices launch begun before the first "
               "block is left out); region_busy_us_per_step: every block and slices interval clipped to the marked "
               "region / block launches; region_idle_us: the region's time with no kernel at all"}
if len(sys.argv) > 2:
    by = float(sys.argv[2])
    out["algorithmic_bytes_per_step"] = by
    out["achieved_gbs"] = by / (out["busy_us_per_step"] * 1e-6) / 1e9
print(json.dumps(out))
