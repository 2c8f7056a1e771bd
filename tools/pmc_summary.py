"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md's HBM section prescribes, written to a JSON
summary that bench.py reads for roofline.traffic.

    python tools/pmc_summary.py gpurun_out/prof_r02 profiles/r02_pmc.json
    python tools/pmc_summary.py --symbols SRC OUT "what was profiled"

--symbols keys every kernel by its base symbol (template instantiations
pooled, launch-weighted), reading SRC/pmc_fetch_h and SRC/pmc_write_h: the
form bench.py's headline roofline reads (profiles/r03_pmc_headline.json).

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch.  FETCH_SIZE counts 64 B per
128-B memory request on gfx950 (half the bytes of a coalesced streaming
read); the factor 2 was re-checked for this engine's 8-byte-per-lane loads
with tools/micro/rescan.hip (known D bytes: 256 rows x 9000 x 8 B = 18000 KiB
-> FETCH_SIZE 9063 KiB), see the 'calibration' entry.  WRITE_SIZE is taken
as reported (exact for streaming stores; this engine's scattered 8-byte
column stores are uncalibrated)."""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict

NAMES = {"k_dnj_select": "dnj_select", "k_dnj_plan": "dnj_find", "k_dnj_scan": "dnj_scan",
         "k_dnj_join": "update", "k_dnj_join_pf": "update", "k_dnj_requeue": "dnj_requeue",
         "k_dnj_fold": "dnj_fold", "k_dnj_sphase": "dnj_sphase", "k_dnj_scan_v": "dnj_scan"}
# the NJ passes (tools/perf_dnj.py 10000 nj), when present
NJ_NAMES = {"k_nj_argmin": "nj_argmin", "k_nj_join": "nj_update", "k_nj_pop": "nj_pop"}


def per_kernel(path):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.match(r"(?:void )?(\w+)", r["Kernel_Name"])
        d[m.group(1)].append(float(r["Counter_Value"]) * 1024.0)
    return d


def by_symbol(src, out, what):
    def pooled(path):
        d = defaultdict(list)
        for r in csv.DictReader(open(path)):
            m = re.match(r"(?:void )?(\w+)", r["Kernel_Name"])
            d[m.group(1)].append(float(r["Counter_Value"]) * 1024.0)
        return d
    fetch = pooled(f"{src}/pmc_fetch_h/run_counter_collection.csv")
    write = pooled(f"{src}/pmc_write_h/run_counter_collection.csv")
    kernels = {}
    for k, v in fetch.items():
        f = 2.0 * statistics.mean(v)
        w = statistics.mean(write.get(k, [0.0]))
        kernels[k] = {"launches": len(v), "fetch_bytes_per_launch": round(f, 1),
                      "write_bytes_per_launch": round(w, 1), "hbm_bytes_per_launch": round(f + w, 1)}
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of {what}; "
                     f"FETCH_SIZE x2 per MI355X_MICROARCH.md (calibration in profiles/r02_pmc.json)",
           "kernels": kernels}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


def main():
    if sys.argv[1] == "--symbols":
        return by_symbol(sys.argv[2], sys.argv[3], sys.argv[4])
    src, out = sys.argv[1], sys.argv[2]
    fetch = per_kernel(f"{src}/pmc_fetch/run_counter_collection.csv")
    write = per_kernel(f"{src}/pmc_write/run_counter_collection.csv")
    kernels = {}

    def add(names, fetch, write):
        for k, label in names.items():
            if k not in fetch:
                continue
            f = 2.0 * statistics.mean(fetch[k])
            w = statistics.mean(write.get(k, [0.0]))
            kernels[label] = {"kernel": k, "launches": len(fetch[k]), "fetch_bytes_per_launch": round(f, 1),
                              "write_bytes_per_launch": round(w, 1), "hbm_bytes_per_launch": round(f + w, 1)}
    add(NAMES, fetch, write)
    import os
    if os.path.exists(f"{src}/pmc_fetch_nj/run_counter_collection.csv"):
        add(NJ_NAMES, per_kernel(f"{src}/pmc_fetch_nj/run_counter_collection.csv"),
            per_kernel(f"{src}/pmc_write_nj/run_counter_collection.csv"))
    cal = {}
    cal_csv = f"{src}/pmc_cal/run_counter_collection.csv"
    for r in (csv.DictReader(open(cal_csv)) if os.path.exists(cal_csv) else []):
        if "k_rescan<256, 8, false>" in r["Kernel_Name"] and r["Grid_Size"] == "327680":
            cal.setdefault("fetch_kib", []).append(float(r["Counter_Value"]))
    calib = None
    if not cal and os.path.exists(out):
        calib = json.load(open(out)).get("calibration")  # keep the last measured calibration
    if cal:
        kib = statistics.mean(cal["fetch_kib"])
        calib = {"kernel": "tools/micro/rescan.hip k_rescan<256,8,false>, 256 rows x 9000 f64",
                 "known_read_kib": 256 * 9000 * 8 / 1024.0, "fetch_size_kib": round(kib, 1),
                 "ratio": round(kib / (256 * 9000 * 8 / 1024.0), 4)}
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                     f"tools/perf_dnj.py 10000 dnj|nj exact (the CLI default); FETCH_SIZE x2 per MI355X_MICROARCH.md",
           "kernels": kernels, "calibration": calib}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
