"""Print the top kernels of a rocprofv3 *_kernel_stats.csv: total ms, calls, percent (names shortened)."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
div = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0  # e.g. number of steps
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / div:.2f} ms (/{div:g})")
for r in rows[:n]:
    name = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    print(f"{float(r['TotalDurationNs']) / 1e6 / div:9.3f} ms {int(r['Calls']) / div:7.1f} calls {float(r['Percentage']):6.2f}%  {name[:110]}")
