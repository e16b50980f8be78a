#!/usr/bin/env python3
"""Key numbers of a round's bench lines (gpurun_out/bench_<w>_<tag>.json) for DESIGN.md §6:
python tools/summarize_round.py <tag>"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def line(tag, w):
    p = os.path.join(REPO, "gpurun_out", f"bench_{w}_{tag}.json")
    if not os.path.exists(p):
        return None
    return json.loads(open(p).read().strip().splitlines()[-1])


def main(tag):
    for w in ("c5full", "c5fulls128", "c5", "c5s128", "c4", "c3", "c5full_n2", "c2"):
        d = line(tag, w)
        if d is None:
            continue
        r = d["roofline"]
        out = {"value": round(d["value"], 1), "us_per_step": round(d["ms_per_step"] * 1e3, 2),
               "gpu_us": round((d.get("gpu_ms_per_step") or 0) * 1e3, 2), "frac": round(r["frac"], 3),
               "traffic_over_alg": round(r["traffic_over_algorithmic"], 3) if r.get("traffic_over_algorithmic") else None}
        if d.get("steady"):
            out["steady"] = round(d["steady"]["value"], 1)
            out["steady_frac"] = round(d["steady"]["frac"], 3)
            out["steady_over_headline"] = round(1 / d["steady"]["value_over_headline"], 3)
        lat = d.get("latency")
        if lat:
            out["rt_p50_p99"] = (round(lat["host_roundtrip_p50_us"], 1), round(lat["host_roundtrip_p99_us"], 1))
            if lat.get("paced"):
                p = lat["paced"]
                out["paced_rt_p50_p99"] = (round(p["host_roundtrip_p50_us"], 1), round(p["host_roundtrip_p99_us"], 1))
                out["paced_value"] = round(p["value"], 1)
        if d.get("parity"):
            out["parity"] = d["parity"]["parity_err"]
        if d.get("per_block_step"):
            out["plain"] = (round(d["per_block_step"]["value"], 1), round(d["per_block_step"]["frac"], 3))
        if d.get("offline"):
            out["offline"] = round(d["offline"]["value"], 1)
        if d.get("ir_change"):
            out["ir_change_ms"] = round(d["ir_change"]["total_ms"], 1)
        if d.get("latency_mode") and d["latency_mode"].get("available"):
            lm = d["latency_mode"]
            out["latency_mode"] = (round(lm["host_roundtrip_p50_us"], 2), round(lm["host_roundtrip_p99_us"], 2),
                                   lm["gpu_step_p50_us"], round(lm["value"], 1))
        if d.get("cpu_baseline"):
            out["cpu"] = (round(d["cpu_baseline"].get("threads_1", 0), 2), round(d["cpu_baseline"]["value"], 1),
                          d["cpu_baseline"]["cores"])
        if d.get("per_rank_ms"):
            out["per_rank_us"] = [round(x * 1e3, 2) for x in d["per_rank_ms"]]
        if d.get("c2_fft"):
            out["c2_frac"] = round(d["c2_fft"]["roofline"]["frac"], 3)
        print(w, json.dumps(out))
        if d.get("host_io"):
            for k, v in d["host_io"].items():
                if isinstance(v, dict):
                    keys = ("msamples_s", "p50_us", "p99_us", "frame_p50_us", "frame_p99_us", "shared_scratch")
                    print("   host_io", k, json.dumps({kk: v[kk] for kk in keys if kk in v}))


if __name__ == "__main__":
    main(sys.argv[1])
