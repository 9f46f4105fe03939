"""Per-token kernel census of the HIP-graph decode step from a rocprofv3 kernel trace.

  rocprofv3 --kernel-trace -d DIR -- python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline
  python scripts/decode_anatomy.py DIR [--steps 4]

A decode step ends with the greedy pick of the logits (k_greedy_final, or torch's ArgMax reduction
for bench.py --greedy two-stage/torch); the last `--steps` complete steps (pick to pick) are
averaged.  Under the tracer every dispatch carries its own
extra cost, so the absolute times are inflated; the launch COUNT per step is exact.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if "k_greedy_final" in r[2]] or \
        [i for i, r in enumerate(rows) if "ArgMax" in r[2]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} greedy-pick dispatches found")
    sel = ends[-(a.steps + 1):]
    per = defaultdict(lambda: [0, 0.0])
    walls, counts = [], []
    for s0, s1 in zip(sel[:-1], sel[1:]):
        chunk = rows[s0 + 1:s1 + 1]
        walls.append((chunk[-1][1] - rows[s0][1]) / 1000.0)
        counts.append(len(chunk))
        for t0, t1, name in chunk:
            e = per[name]
            e[0] += 1
            e[1] += (t1 - t0) / 1000.0
    n = len(walls)
    print(f"decode step under the tracer: wall {sum(walls) / n:.1f} us, {sum(counts) / n:.1f} dispatches per step "
          f"(mean of the last {n} steps)")
    tot = 0.0
    for name, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        tot += t / n
        print(f"{c / n:7.1f} x {t / c:8.2f} us = {t / n:8.1f} us  {name[:130]}")
    print(f"summed kernel time per step {tot:.1f} us")


if __name__ == "__main__":
    main()
