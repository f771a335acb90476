"""Print the kernel timeline of the last bench step from a rocprofv3 kernel trace (tools/trace_overlap.sh):
kernel, queue, start / end / duration in us relative to the previous step's preprocess backward."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "preprocess_bwd" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["End_Timestamp"])
skip = sys.argv[2].split(",") if len(sys.argv) > 2 else []
for r in rows[a + 1:b + 1]:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsr::", "")[:40]
    if any(k in n for k in skip):
        continue
    s = (int(r["Start_Timestamp"]) - t0) / 1000
    e = (int(r["End_Timestamp"]) - t0) / 1000
    print(f"{n:40s} q{r.get('Queue_Id', '?'):>3} {s:8.1f} {e:8.1f} {e - s:7.1f}")
