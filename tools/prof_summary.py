"""Summarise a rocprofv3 `--kernel-trace --stats` run of bench.py for the roofline:

    python tools/prof_summary.py --stats <dir>/..._kernel_stats.csv --bench <bench json of the same run>
        --command "python3 bench.py --gpus 1 --steps 20 --warmup 5" --workload c2 --out profiles/r03_profile_c2.json

Writes the K1 kernel's call count and average duration over EVERY call of the profiled command (no
call dropped), the bench line that same profiled process printed (its ms_per_step includes the
tracer's overhead, so avg_ms <= ms_per_step holds for the same invocation), and the roofline fraction
bytes / avg / 8 TB/s. bench.py reads the newest such file and reports it next to its HIP-event figure.
With --trace (the same run's kernel_trace.csv) it also reports the launches of the timed region alone:
bench.py dispatches its pre-warm launches (their count is in its JSON line), W warm-up launches, then
the K timed ones (then the per-launch probes), so
launches P+W .. P+W+K-1 in dispatch order (P pre-warm) are the ones ms_per_step covers; the process's first launch
(cold code and TLB) is the slowest of all and is not among them.
"""
from __future__ import annotations

import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--command", required=True)
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--kernel", default="xxh3_wave_kernel")
    ap.add_argument("--out", required=True)
    ap.add_argument("--trace", default=None, help="the same run's kernel_trace.csv")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.stats)) if a.kernel in r["Name"]]
    assert rows, f"no {a.kernel} row in {a.stats}"
    calls = sum(int(r["Calls"]) for r in rows)
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    bench = None
    for line in open(a.bench):
        line = line.strip()
        if line.startswith("{"):
            bench = json.loads(line)
    assert bench is not None, "no bench JSON line"
    nbytes = bench["config"]["bytes_per_gpu"]
    avg_ms = total_ns / calls / 1e6
    res = {"workload": a.workload, "kernel": rows[0]["Name"], "calls": calls, "avg_ms": round(avg_ms, 5),
           "min_ms": round(min(float(r["MinNs"]) for r in rows) / 1e6, 5),
           "max_ms": round(max(float(r["MaxNs"]) for r in rows) / 1e6, 5),
           "command": a.command, "stats_csv": a.stats.split("/")[-1],
           "bytes_per_launch": nbytes, "achieved_GBs": round(nbytes / (avg_ms / 1e3) / 1e9, 1),
           "frac": round(nbytes / (avg_ms / 1e3) / 1e9 / 8000.0, 4),
           "same_run_bench": {"ms_per_step": bench["ms_per_step"], "value": bench["value"],
                              "kernel_ms_events": bench["roofline"]["kernel_ms"],
                              "kernel_ms_back_to_back": bench["roofline"].get("kernel_ms_back_to_back")}}
    res["avg_le_ms_per_step"] = avg_ms <= bench["ms_per_step"]
    if a.trace:
        tr = sorted((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                    for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"])
        # bench.py's untimed pre-warm launches (r05) come first, then W warm-up, then the K timed ones
        skip = int(bench.get("prewarm", {}).get("launches", 0)) + a.warmup
        timed = [d for _, d in tr[skip:skip + a.steps]]
        assert len(timed) == a.steps, "trace holds fewer launches than pre-warm + warm-up + steps"
        t_ms = sum(timed) / len(timed) / 1e6
        res["timed_region"] = {"launches": f"{skip}..{skip + a.steps - 1} in dispatch order",
                               "avg_ms": round(t_ms, 5), "frac": round(nbytes / (t_ms / 1e3) / 1e9 / 8000.0, 4),
                               "avg_le_ms_per_step": t_ms <= bench["ms_per_step"],
                               "first_launch_ms": round(tr[0][1] / 1e6, 5)}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
