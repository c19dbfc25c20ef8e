"""Average each PMC counter per kernel over a rocprofv3 counter_collection.csv (one or more files)."""
import csv
import sys
from collections import defaultdict

tot, cnt, dur = defaultdict(float), defaultdict(set), defaultdict(list)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:60]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])].add((path, r["Dispatch_Id"]))
        dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (k, c), v in sorted(tot.items()):
    n = len(cnt[(k, c)])
    print(f"{k:60s} {c:24s} {v / n:16.1f}  (n={n}, avg dur {sum(dur[k]) / len(dur[k]) / 1e3:.1f} us)")
