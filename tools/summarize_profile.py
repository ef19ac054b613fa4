#!/usr/bin/env python3
"""Summarise a rocprofv3 run of bench.py (tools/gpu_profile.sh) into
profiles/<tag>_summary.json: kernel-trace durations of the library's
kernels (the dominant one first) and the FETCH_SIZE-derived HBM read bytes
per launch of the dominant kernel (x1024 B per KB unit, x2 gfx950
wide-read correction, MI355X_MICROARCH.md §HBM)."""
import csv
import json
import os
import re
import sys


def short(name):
    """Kernel name without its parameter list."""
    return re.sub(r"\((rure_amd::BatchDev|unsigned|int|long|void\*).*$", "", name)


def main(tag, kernel_substr="rure_amd::"):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "gpurun_out", tag)
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    ks = sorted([r for r in stats if kernel_substr in r["Name"]], key=lambda r: -float(r["TotalDurationNs"]))
    bench = json.loads(open(os.path.join(src, "bench_trace.json")).read().strip().splitlines()[-1])
    # the kernel the bench line's roofline names comes first (C3's line also
    # times the shootout pipeline, whose replace kernels add up to more)
    named = str(bench.get("roofline", {}).get("kernel", ""))
    for i, r in enumerate(ks):
        kid = short(r["Name"]).split("::")[-1].split("<")[0]
        if kid and kid in named:
            ks.insert(0, ks.pop(i))
            break
    pmc = list(csv.DictReader(open(os.path.join(src, "pmc", "pmc_counter_collection.csv"))))
    fetch = [float(r["Counter_Value"]) for r in pmc
             if ks and r["Kernel_Name"] == ks[0]["Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    # the bench line's roofline entry for the dominant kernel (the C3 line
    # carries one per phase: roofline = the variant kernel, roofline_strip =
    # the lexer, which reads the raw text, not the stripped stream)
    roof = bench.get("roofline", {})
    if ks:
        kid = re.sub(r"_kernel.*$", "", short(ks[0]["Name"]).split("::")[-1])
        for k, v in bench.items():
            if k.startswith("roofline") and isinstance(v, dict) and kid in str(v.get("kernel", "")):
                roof = v
                break
    alg = roof.get("alg_bytes_per_launch")
    import datetime
    out = {
        "tag": tag,
        "generated_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
        "kernel": ks[0]["Name"] if ks else None,
        "calls": int(ks[0]["Calls"]) if ks else 0,
        "avg_ns": float(ks[0]["AverageNs"]) if ks else None,
        "min_ns": float(ks[0]["MinNs"]) if ks else None,
        "max_ns": float(ks[0]["MaxNs"]) if ks else None,
        "fetch_size_kb_avg": sum(fetch) / len(fetch) if fetch else None,
        "hbm_read_bytes_per_launch": (sum(fetch) / len(fetch)) * 1024 * 2 if fetch else None,
        "bench_kernel_ms_events": roof.get("kernel_ms", bench.get("kernel_ms")),
        "alg_bytes_per_launch": alg,
        "bench_value_GBps": bench["value"],
        "bench_config": bench["config"],
        "note": "FETCH_SIZE (KB) x 1024 x 2: gfx950 reports half of wide streaming reads",
        "library_kernels": [{"name": short(r["Name"]), "calls": int(r["Calls"]),
                             "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"])}
                            for r in ks[:8]],
    }
    if out["hbm_read_bytes_per_launch"] and alg:
        out["traffic_over_alg"] = out["hbm_read_bytes_per_launch"] / alg
    # every roofline of the bench line (C3: the variant kernel and the strip
    # lexer) from the launches of its workload alone: the kernel trace's
    # dispatches of that kernel with the largest grid (the shootout pipeline
    # and the warm-up ramp launch the same kernels over smaller inputs), and
    # the FETCH_SIZE rows of the same grid
    trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    out["rooflines"] = {}
    for key, v in bench.items():
        if not (key.startswith("roofline") and isinstance(v, dict) and v.get("alg_bytes_per_launch")):
            continue
        kid = str(v.get("kernel", "")).split("(")[-1].split(":")[0].split("_kernel")[0].strip()
        rows = [r for r in trace if "rure_amd::" in r["Kernel_Name"] and kid and kid + "_kernel" in r["Kernel_Name"]]
        if not rows:
            continue
        grid = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        g = max(grid(r) for r in rows)
        main = [r for r in rows if grid(r) == g]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in main]
        avg = sum(durs) / len(durs)
        fk = [float(r["Counter_Value"]) for r in pmc
              if kid + "_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE" and int(r["Grid_Size"]) == g]
        a = v["alg_bytes_per_launch"]
        ent = {"kernel": short(main[0]["Kernel_Name"]), "grid": g, "launches": len(main),
               "avg_ns": round(avg, 1), "alg_bytes_per_launch": a,
               "achieved_GBps": round(a / avg, 1), "peak_GBps": v.get("peak"),
               "frac": round(a / avg / float(v.get("peak") or 8000.0), 4),
               "bench_kernel_ms_events": v.get("kernel_ms")}
        if fk:
            ent["hbm_read_bytes_per_launch"] = sum(fk) / len(fk) * 1024 * 2
            ent["traffic_over_alg"] = round(ent["hbm_read_bytes_per_launch"] / a, 4)
        out["rooflines"][key] = ent
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    with open(os.path.join(root, "profiles", tag + "_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    # keep the raw kernel stats CSV next to it
    with open(os.path.join(root, "profiles", tag + "_kernel_stats.csv"), "w") as f:
        f.write(open(os.path.join(src, "trace", "run_kernel_stats.csv")).read())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
