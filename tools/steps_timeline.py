"""Kernel timeline of bench steps from a rocprofv3 kernel trace: the last
STEPS steps (a step starts at k_add_link), one line per kernel, plus the
per-step wall time and busy time."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if "k_add_link" in x["Kernel_Name"]]
idx.append(len(r))
for w in range(len(idx) - 1 - steps, len(idx) - 1):
    i0, i1 = idx[w], idx[w + 1]
    t0 = int(r[i0]["Start_Timestamp"])
    busy = 0
    for x in r[i0:i1]:
        s = int(x["Start_Timestamp"]) - t0
        e = int(x["End_Timestamp"]) - t0
        busy += e - s
        n = x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:6.1f}  {n[-48:]}")
    end = int(r[i1]["Start_Timestamp"]) if i1 < len(r) else int(r[i1 - 1]["End_Timestamp"])
    print(f"busy {busy / 1e3:.1f} us, wall {(end - t0) / 1e3:.1f} us\n")
