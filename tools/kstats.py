"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv: name, calls, total ms, avg us, %."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    print(f"{r['Name'][:90]:90s} {r['Calls']:>7s} {float(r['TotalDurationNs'])/1e6:9.2f} ms "
          f"{float(r['AverageNs'])/1e3:9.1f} us {r['Percentage'][:5]}")
