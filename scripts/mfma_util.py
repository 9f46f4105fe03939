"""MFMA utilisation per kernel from a rocprofv3 --pmc pass of
scripts/prof_prefill.py (counters SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_VALU_MFMA_MOPS_F16, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) and the kernel
trace of the same command:

    MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
    clock    = (GRBM_GUI_ACTIVE / 8) / kernel time (trace median)

    python scripts/mfma_util.py <counter_collection.csv> <kernel_trace.csv> [flop_per_launch]
"""
import collections
import csv
import re
import statistics
import sys


def short(name: str) -> str:
    return re.sub(r"\(.*", "", name)[:90]


def main():
    pmc_path, trace_path = sys.argv[1], sys.argv[2]
    flop = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0 * 16384 * 4096 * 4096
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(pmc_path)):
        per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_path)):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for k, c in per.items():
        if not c.get("SQ_VALU_MFMA_BUSY_CYCLES") or max(c["SQ_VALU_MFMA_BUSY_CYCLES"]) == 0 or k not in dur:
            continue
        t = statistics.median(dur[k])
        gui = statistics.median(c["GRBM_GUI_ACTIVE"]) / 8
        util = statistics.median(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / (gui * 1024)
        print(f"{k}\n    launches={len(dur[k])} median {t * 1e6:.1f} us  MfmaUtil {100 * util:.1f} %  "
              f"clock {gui / t / 1e9:.2f} GHz  -> {flop / t / 1e12:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
