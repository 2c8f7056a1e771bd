"""The dist kernel's clock and issue mix from one rocprofv3 --pmc pass
(tools/profile_r06.sh clk): GRBM_GUI_ACTIVE over the dispatch's duration gives
the clock the chip held while the kernel ran (the counter sums the 8 XCDs'
GPU-busy cycles), SQ_BUSY_CYCLES / SQ_WAVE_CYCLES / SQ_INSTS_VALU /
SQ_VALU_MFMA_BUSY_CYCLES the issue mix.  Per dispatch of k_snp_mfma3 / k_snp_mfma2, then the
mean.

    python tools/pmc_clock.py gpurun_out/prof_r06/pmc_clk profiles/r06_dist_clock.json
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict


def main():
    src, out = sys.argv[1], sys.argv[2]
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f"{src}/run_counter_collection.csv")):
        m = re.match(r"(?:void )?(\w+)", r["Kernel_Name"])
        if not m or m.group(1) not in ("k_snp_mfma2", "k_snp_mfma3"):
            continue
        d = disp[r["Dispatch_Id"]]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k in ("Start_Timestamp", "End_Timestamp"):
            if k in r:
                d[k] = float(r[k])
    rows = []
    for d in disp.values():
        dur = (d.get("End_Timestamp", 0) - d.get("Start_Timestamp", 0)) * 1e-9
        if dur <= 0 or "GRBM_GUI_ACTIVE" not in d:
            continue
        row = {"dur_s": dur, **{k: v for k, v in d.items() if not k.endswith("Timestamp")}}
        row["clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8.0 / dur / 1e9
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            # busy cycles summed over the chip's 1024 SIMDs, against the cycles the chip ran
            row["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
        rows.append(row)
    mean = {k: statistics.mean(r[k] for r in rows) for k in rows[0]} if rows else {}
    res = {"source": f"rocprofv3 --pmc (one pass) of tools/perf_dist.py 50000 5000000, dispatches of k_snp_mfma3 / k_snp_mfma2 "
                     f"({src})", "dispatches": rows, "mean": mean,
           "reading": "clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration: the clock the chip held while the fp4 MFMA "
                      "kernel ran (2.4 GHz nominal); mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x "
                      "those cycles"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
