"""Print the kernel timeline of one bench step from a rocprofv3 kernel trace
(steps start at k_add_keys / k_add_link)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if "k_add_keys" in x["Kernel_Name"]
       or "k_add_link" in x["Kernel_Name"]]
i0, i1 = idx[which], idx[which + 1]
t0 = int(r[i0]["Start_Timestamp"])
busy = 0
for x in r[i0:i1]:
    s = int(x["Start_Timestamp"]) - t0
    e = int(x["End_Timestamp"]) - t0
    busy += e - s
    name = x["Kernel_Name"].replace("(anonymous namespace)::", "")
    if "rocprim" in name:
        name = "rocprim::" + name.split("detail::")[2][:40]
    print("%8.1f %8.1f %7.1f  %-60s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3,
                                        name[:60], x["Grid_Size_X"]))
print("busy %.1f us, wall %.1f us" % (busy / 1e3,
      (int(r[i1]["Start_Timestamp"]) - t0) / 1e3))
