"""HBM traffic per launch of each bench stage from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE, collected in separate runs by scripts/gpu_pmc.sh).

Units and corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE / WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts half
the bytes of a wide coalesced read, so fetched bytes = 2 x FETCH_SIZE (the
guide's calibration is for 16-B-per-lane streaming; other access widths are
uncalibrated and the raw values are kept beside the corrected ones).
Only the last `--steps` dispatches of each kernel (the bench's timed steps)
are used.  Writes {stage: {...}} JSON (bench.py reads "hbm_bytes").
"""
import argparse
import csv
import json
from collections import defaultdict

STAGES = {
    "scan": ["k_rscan"],
    "select": ["k_rhist"],
    "emit": ["k_remit"],
    "rank": ["k_rrank"],
    "apply": ["k_rapply"],
    "future": ["k_round_future"],
    "add_link": ["k_add_link"],
    "add_chain": ["k_add_chain"],
    # (bench.py's default launch: the add chain beside the scan, then the
    # batch's slots scanned)
    "chain_scan": ["k_chain_scan", "k_scan_fix"],
    # (pipelined calls: the previous call's deferred apply beside this call's
    # filing, one launch; "apply" and "add_link" then count only the other
    # phases' launches -- pre-population, settle -- not the bench's steps)
    "apply_link": ["k_apply_link"],
}
CALIB = ["stream16", "rand64", "rand32", "rand16", "rand8"]
STREAMING = {"scan", "select", "future"}
# walkers that also stream columns with 16-B-per-lane loads: bytes per slot
# (k_remit: the quantized keys 8 + meta 4), counted 2x; the rest of their
# fetch 1x
STREAM_PART = {"emit": 12, "chain_scan": 32}


def calib_rates(stats_csv, out):
    """add each pattern's measured rate (rocprofv3 --stats of fetch_calib):
    GB/s of its known bytes and 64-B memory requests per second"""
    names = {"stream16": "stream16(", "rand64": "rand_rec<4>", "rand32": "rand_rec<2>",
             "rand16": "rand16(", "rand8": "rand8("}
    for r in csv.DictReader(open(stats_csv)):
        for k, pat in names.items():
            if pat in r["Name"] and k in out:
                ns = float(r["AverageNs"])
                if k == "stream16" and int(r["Calls"]) > 3:
                    continue  # the evict passes share the name
                out[k]["avg_ns"] = ns
                out[k]["GBps"] = round(out[k]["known_bytes"] / ns, 1)
                req = out[k]["fetch_size_bytes"] / 64.0
                out[k]["requests_per_s"] = round(req / (ns * 1e-9))
    return out


def calibrate(fetch_csv, known_json):
    """bytes-per-FETCH_SIZE-byte factors from tools/fetch_calib: per
    repetition six stream16 dispatches (the 2nd is the measured 512 MiB, the
    others 2 GiB evict passes) and one of each random-access kernel"""
    known = json.load(open(known_json))
    rows = sorted(csv.DictReader(open(fetch_csv)), key=lambda x: int(x["Dispatch_Id"]))
    by = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        key = ("rand64" if "rand_rec<4>" in name else "rand32" if "rand_rec<2>" in name
               else "rand16" if name.startswith("rand16") else "rand8"
               if name.startswith("rand8") else "stream16" if name.startswith("stream16")
               else None)
        if key:
            by[key].append(float(r["Counter_Value"]) * 1024.0)
    by["evict"] = [v for i, v in enumerate(by["stream16"]) if i % 6 != 1]
    by["stream16"] = [v for i, v in enumerate(by["stream16"]) if i % 6 == 1]
    known = dict(known, evict=known["evict_pass_bytes"])
    out = {}
    for name in CALIB + ["evict"]:
        got = by.get(name, [])
        avg = sum(got) / max(len(got), 1)
        out[name] = {"known_bytes": known[name], "fetch_size_bytes": round(avg),
                     "dispatches": len(got),
                     "known_per_counted": known[name] / avg if avg else None}
    return out


def per_kernel(path, steps):
    vals = defaultdict(list)
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda x: int(x["Dispatch_Id"]))
    for r in rows:
        name = r["Kernel_Name"]
        for ks in STAGES.values():
            for k in ks:
                if k + "(" in name or k + "_t<" in name or name.endswith(k):
                    vals[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: v[-steps:] for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", default="gpurun_out/pmc_FETCH_SIZE/run_counter_collection.csv")
    ap.add_argument("--write", default="gpurun_out/pmc_WRITE_SIZE/run_counter_collection.csv")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--out", default="profiles/traffic_r03.json")
    ap.add_argument("--calib", default=None,
                    help="tools/fetch_calib FETCH_SIZE csv (with --known): print factors")
    ap.add_argument("--known", default=None)
    ap.add_argument("--slots", type=int, default=1 << 20,
                    help="client slots of the profiled bench (STREAM_PART)")
    ap.add_argument("--calib-stats", default=None,
                    help="rocprofv3 --stats csv of the same calibration run: rates")
    a = ap.parse_args()
    if a.calib:
        out = calibrate(a.calib, a.known)
        if a.calib_stats:
            out = calib_rates(a.calib_stats, out)
        json.dump(out, open(a.out, "w"), indent=1)
        for k, v in out.items():
            print(k, v)
        return
    fe = per_kernel(a.fetch, a.steps)
    wr = per_kernel(a.write, a.steps)
    out = {}
    for stage, ks in STAGES.items():
        f = sum(sum(fe.get(k, [])) / max(len(fe.get(k, [])), 1) for k in ks)
        w = sum(sum(wr.get(k, [])) / max(len(wr.get(k, [])), 1) for k in ks)
        # calibrated on known byte counts (tools/fetch_calib.hip, profiles/
        # r02_fetch_calib.json): FETCH_SIZE counts 64 B per memory request; a
        # coalesced stream requests 128 B (bytes = 2 x FETCH_SIZE), a random
        # access of <= 64 B one 64-B request (bytes = FETCH_SIZE).  Streaming
        # stages take 2x; the walkers' random accesses 1x, k_remit's streamed
        # key columns 2x (STREAM_PART); the all-streamed bound is kept beside
        fac = 2.0 if stage in STREAMING else 1.0
        hbm = fac * f + w
        if stage in STREAM_PART and f > 0:
            # the streamed columns' raw count is half their bytes
            streamed_raw = min(f, STREAM_PART[stage] * a.slots / 2.0)
            hbm = 2.0 * streamed_raw + (f - streamed_raw) + w
        out[stage] = {"fetch_size_bytes_raw": round(f), "write_size_bytes": round(w),
                      "hbm_bytes": round(hbm), "fetch_factor": fac,
                      "hbm_bytes_if_all_streamed": round(2 * f + w),
                      "kernels": ks, "launches_averaged": a.steps}
    if out.get("chain_scan", {}).get("fetch_size_bytes_raw"):
        # the timed steps ran the add chain beside the scan: k_rscan and
        # k_add_chain ran only outside them (pre-population, settle rounds)
        out.pop("scan", None)
        out.pop("add_chain", None)
    if out.get("apply_link", {}).get("fetch_size_bytes_raw"):
        # pipelined steps: the apply ran beside the next call's filing;
        # k_rapply and k_add_link ran alone only outside them
        out.pop("apply", None)
        out.pop("add_link", None)
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in out.items():
        print(f"{k:10s} fetch(raw) {v['fetch_size_bytes_raw']/1e6:8.2f} MB  write {v['write_size_bytes']/1e6:8.2f} MB  hbm(corr) {v['hbm_bytes']/1e6:8.2f} MB")


if __name__ == "__main__":
    main()
