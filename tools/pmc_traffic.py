"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per K1 launch.

    python tools/pmc_traffic.py --fetch <dir_fetch> --write <dir_write> --workload c2 \
        --algorithmic-bytes 6553600000 --out profiles/r01_traffic_c2.json

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming read (16 B/lane
loads, TCC_EA0_RDREQ x 64 B with 128-B requests), so it is doubled; WRITE_SIZE is exact for 16-B
streaming stores (our 16-B digest stores are uncalibrated but negligible). The two counters are
collected in separate passes (they do not fit one TCC pass).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def counter_values(d: str, counter: str, kernel_substr: str) -> list[float]:
    vals = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(p) as f:
            for row in csv.DictReader(f):
                if kernel_substr in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write")
    ap.add_argument("--kernel", default="xxh3_wave_kernel")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--algorithmic-bytes", type=float, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = counter_values(a.fetch, "FETCH_SIZE", a.kernel)
    write = counter_values(a.write, "WRITE_SIZE", a.kernel) if a.write else []
    if not fetch:
        raise SystemExit(f"no FETCH_SIZE rows for {a.kernel} under {a.fetch}")
    f_kib = statistics.median(fetch)
    w_kib = statistics.median(write) if write else 0.0
    read_bytes = f_kib * 1024 * 2  # gfx950: FETCH_SIZE = 1/2 of a wide streaming read
    write_bytes = w_kib * 1024
    res = {
        "workload": a.workload,
        "kernel": a.kernel,
        "dispatches": len(fetch),
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib if write else None,
        "hbm_read_bytes_per_launch": read_bytes,
        "hbm_write_bytes_per_launch": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes,
        "algorithmic_bytes_per_launch": a.algorithmic_bytes,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / a.algorithmic_bytes,
        "correction": "read = FETCH_SIZE*1024*2 (gfx950 half-count on 16-B/lane streams), write = WRITE_SIZE*1024",
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE ({os.path.basename(a.out)})",
    }
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
