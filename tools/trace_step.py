"""Per-kernel timeline of decode steps from a rocprofv3 --kernel-trace CSV.

Usage: python tools/trace_step.py <run_kernel_trace.csv> [n_steps]
Finds the decode steps (sampler launch -> next sampler launch), then prints per
kernel kind: launches per step, mean duration, mean gap in front of it (end of the
previous kernel -> its start) and its share of the step; then the median step's
first kernels in order.
"""
import collections
import csv
import statistics
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("t5g::", "")[:58]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           f'{r.get("Grid_Size_X", "")}x{r.get("Grid_Size_Y", "")}x{r.get("Grid_Size_Z", "")}') for r in rows]
    starts = [i for i, k in enumerate(ks) if k[0].startswith("sampler_kernel")]
    steps = [(starts[i], starts[i + 1]) for i in range(len(starts) - 1)]
    steps = steps[2:-1] if len(steps) > 6 else steps
    if not steps:
        print("no decode steps found")
        return
    steps = steps[:int(sys.argv[2]) if len(sys.argv) > 2 else 400]
    walls = [(ks[b][1] - ks[a][1]) / 1e3 for a, b in steps]
    print(f"steps {len(steps)}  step wall median {statistics.median(walls):.1f} us  "
          f"min {min(walls):.1f}  max {max(walls):.1f}")
    agg_d, agg_g, agg_n = collections.defaultdict(float), collections.defaultdict(float), collections.defaultdict(int)
    for a, b in steps:
        prev_end = ks[a - 1][2] if a > 0 else ks[a][1]
        for k in ks[a:b]:
            key = (k[0], k[3])
            agg_d[key] += (k[2] - k[1]) / 1e3
            agg_g[key] += (k[1] - prev_end) / 1e3
            agg_n[key] += 1
            prev_end = max(prev_end, k[2])
    ns = len(steps)
    print(f"per step: kernel busy {sum(agg_d.values()) / ns:.1f} us, gaps {sum(agg_g.values()) / ns:.1f} us, "
          f"launches {sum(agg_n.values()) / ns:.0f}")
    print(f"{'kernel':58s} {'grid':>14s} {'n/step':>6s} {'dur':>7s} {'gap':>6s} {'us/step':>8s}")
    for key in sorted(agg_d, key=lambda k: -(agg_d[k] + agg_g[k])):
        print(f"{key[0]:58s} {key[1]:>14s} {agg_n[key] / ns:6.1f} {agg_d[key] / agg_n[key]:7.2f} "
              f"{agg_g[key] / agg_n[key]:6.2f} {(agg_d[key] + agg_g[key]) / ns:8.1f}")
    med = sorted(range(ns), key=lambda i: walls[i])[ns // 2]
    a, b = steps[med]
    print(f"\nmedian step ({walls[med]:.1f} us), first 30 kernels:")
    prev_end = ks[a][1]
    for k in ks[a:min(b, a + 30)]:
        print(f"  {k[0]:58s} {k[3]:>14s} dur {(k[2] - k[1]) / 1e3:7.2f}  gap {(k[1] - prev_end) / 1e3:6.2f}")
        prev_end = max(prev_end, k[2])


if __name__ == "__main__":
    main()
