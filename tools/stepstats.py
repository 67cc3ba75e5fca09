"""Kernel statistics of a bench run's last STEPS steps from a rocprofv3
kernel trace, in the format of rocprofv3's own kernel_stats.csv.

rocprofv3 --stats averages every dispatch of the process, including the
pre-population and settle rounds (1M-entry pulls), so its averages for the
round kernels are not the bench's.  A step starts at k_add_link; the last
STEPS steps of the trace are the bench's timed region when the profiled
bench runs with --no-profile (no stage-timed pass after it) or, with
--stage-pass P, the P steps of the stage-timed pass (the roofline's source).

usage: python tools/stepstats.py TRACE.csv STEPS [--skip-last M] > out.csv
"""
import argparse
import csv
import statistics
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("steps", type=int)
    ap.add_argument("--skip-last", type=int, default=0,
                    help="ignore the trace's last M steps")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    # (pipelined calls after the first: k_apply_link, the previous call's
    # deferred apply beside this call's filing)
    starts = [i for i, x in enumerate(rows)
              if "k_add_link" in x["Kernel_Name"] or "k_apply_link" in x["Kernel_Name"]]
    # a step runs from its k_add_link to the next one; the trace's last step
    # ends at its last round kernel (a round's apply or terminal pull, a
    # queue group's tallies and epoch delivery), so that what runs after the
    # timed region (the bench's queue-size check k_count_requests, the
    # runtime's result copies) is not counted
    tail = ("k_rapply", "k_rfinish", "k_round_future", "k_put_result", "k_tally",
            "k_track_", "k_rrank")
    end = len(rows)
    while end > starts[-1] + 1 and not any(t in rows[end - 1]["Kernel_Name"] for t in tail):
        end -= 1
    starts.append(end)
    hi = len(starts) - 1 - a.skip_last
    lo = hi - a.steps
    if lo < 0:
        sys.exit(f"trace holds {len(starts) - 1} steps, asked for {a.steps}")
    dur = defaultdict(list)
    for x in rows[starts[lo]:starts[hi]]:
        dur[x["Kernel_Name"]].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
    tot = sum(sum(v) for v in dur.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage",
                "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2),
                    min(v), max(v), statistics.pstdev(v)])


if __name__ == "__main__":
    main()
