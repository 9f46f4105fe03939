"""Median per-dispatch counter values per kernel from rocprofv3 csv directories (a --kernel-trace
directory first, then --pmc directories), one row per kernel: trace duration and every counter.
   python scripts/counter_table.py <trace_dir> <pmc_dir> [<pmc_dir> ...]"""
import collections
import csv
import glob
import re
import statistics
import sys


def short(name: str) -> str:
    return re.sub(r"\(.*", "", name)[:60]


def main():
    dirs = sys.argv[1:]
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{dirs[0]}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs[1:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(dur):
        if statistics.median(dur[k]) < 50:   # the GEMMs only
            continue
        print(f"{k}\n    trace median {statistics.median(dur[k]):.1f} us over {len(dur[k])}")
        for c, v in sorted(vals.get(k, {}).items()):
            print(f"    {c:32s} {statistics.median(v):.6g}")


if __name__ == "__main__":
    main()
