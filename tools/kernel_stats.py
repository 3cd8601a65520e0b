"""Per-kernel durations of the TIMED dispatches of a rocprofv3 kernel trace.

rocprofv3's own `--stats` summary averages every dispatch of a kernel in the process: warm-up, clock-settle and
contract-check launches included.  bench.py brackets each timed region with two dispatches of
`bf_trace_mark_kernel` (bf_trace_mark, include/bf.h); this script keeps only the dispatches that START after a
region's first mark and END before its second, and summarises them per kernel name in rocprof's `kernel_stats` CSV
columns (+ MedianNs, Region).

    python tools/kernel_stats.py <kernel_trace.csv> [out.csv]      # prints the table, writes the CSV if given

Regions are numbered in trace order: bench.py times the headline first, then its `secondary` cases in the order of
the JSON line.
"""
import csv
import statistics
import sys

MARK = "bf_trace_mark_kernel"


def read_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def timed_regions(rows):
    """[(start_ns, end_ns, [(start, end, name), ...])] between consecutive pairs of marks."""
    marks = [r for r in rows if MARK in r[2]]
    regions = []
    for i in range(0, len(marks) - 1, 2):
        t0, t1 = marks[i][1], marks[i + 1][0]
        regions.append((t0, t1, [r for r in rows if r[0] >= t0 and r[1] <= t1 and MARK not in r[2]]))
    return regions


def summarise(dispatches):
    """name -> dict(Calls, TotalDurationNs, AverageNs, MinNs, MaxNs, StdDev, MedianNs), busiest first."""
    by = {}
    for s, e, name in dispatches:
        by.setdefault(name, []).append(e - s)
    out = {}
    total = sum(sum(v) for v in by.values()) or 1
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        out[name] = {"Calls": len(d), "TotalDurationNs": sum(d), "AverageNs": sum(d) / len(d),
                     "Percentage": 100.0 * sum(d) / total, "MinNs": min(d), "MaxNs": max(d),
                     "StdDev": statistics.pstdev(d) if len(d) > 1 else 0.0, "MedianNs": statistics.median(d)}
    return out


def region_stats(trace_csv):
    """[{kernel name -> stats}] per timed region, in trace order."""
    return [summarise(d) for _, _, d in timed_regions(read_trace(trace_csv))]


def dominant(stats, contains=None):
    """(name, stats) of the busiest kernel of a region (optionally whose name contains `contains`)."""
    for name, s in stats.items():
        if contains is None or contains in name:
            return name, s
    return None, None


def write_csv(regions, path):
    cols = ["Region", "Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "Percentage", "MinNs", "MaxNs",
            "StdDev"]
    with open(path, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(cols)
        for i, reg in enumerate(regions):
            for name, s in reg.items():
                w.writerow([i, name] + [round(s[c], 3) if isinstance(s[c], float) else s[c] for c in cols[2:]])


def main():
    regions = region_stats(sys.argv[1])
    for i, reg in enumerate(regions):
        for name, s in reg.items():
            print(f"region {i}: {s['Calls']:4d} x {name[:110]}: avg {s['AverageNs'] / 1e3:9.2f} us  median "
                  f"{s['MedianNs'] / 1e3:9.2f} us  min {s['MinNs'] / 1e3:9.2f}  max {s['MaxNs'] / 1e3:9.2f}")
    if len(sys.argv) > 2:
        write_csv(regions, sys.argv[2])


if __name__ == "__main__":
    main()
