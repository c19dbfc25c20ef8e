"""Per-(variant, case) averages of the K1 PMC passes of tools/k1_pmc.sh: dispatches of one kernel come
in runs of 23 (3 warm-up + 20 timed) per probe case, in PROBE_CASES order.

    python tools/k1_pmc_summary.py gpurun_out/k1pmc cdc_packed,cdc_256
"""
import csv
import os
import sys
from collections import defaultdict


def main():
    root, cases = sys.argv[1], sys.argv[2].split(",")
    rows = defaultdict(lambda: defaultdict(list))
    for p in sorted(os.listdir(root)):
        f = os.path.join(root, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        disp = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if "xxh3_wave_kernel" not in r["Kernel_Name"]:
                continue
            d = disp[int(r["Dispatch_Id"])]
            d["k"] = r["Kernel_Name"].split("<")[1].split(">")[0]
            d["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            d[r["Counter_Name"]] = float(r["Counter_Value"])
        seen = defaultdict(int)
        for i in sorted(disp):
            d = disp[i]
            case = cases[(seen[d["k"]] // 23) % len(cases)]
            seen[d["k"]] += 1
            for c, v in d.items():
                if c != "k":
                    rows[(d["k"], case)][c].append(v)
    for key in sorted(rows):
        m = {c: sum(v) / len(v) for c, v in rows[key].items()}
        print(key, f"dur {m.pop('dur'):.1f} us")
        g = m.get("GRBM_GUI_ACTIVE")
        for c in sorted(m):
            extra = ""
            if c == "SQ_ACTIVE_INST_VALU" and g:
                extra = f"  VALU issue {4 * m[c] / (g / 8 * 1024):.2f} of the SIMDs' (quad-cycles x4 / SIMD-cycles)"
            if c == "TA_TA_BUSY_sum" and g:
                extra = f"  TA busy {m[c] / (g / 8 * 256):.2f} per TA"
            print(f"    {c:32s} {m[c]:16.4g}{extra}")


if __name__ == "__main__":
    main()
