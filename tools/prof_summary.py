"""Summarise a rocprofv3 --kernel-trace run of bench.py: per-kernel totals over the LAST
timed step (between the last two Adam launches) and over the whole run."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof'
rows = list(csv.DictReader(open(f'{d}/run_kernel_trace.csv')))
idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
a, b = idx[-2] + 1, idx[-1] + 1
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[a:b]:
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][:80]
    agg[n][0] += 1
    agg[n][1] += dur
tot = sum(v[1] for v in agg.values())
wall = (int(rows[b - 1]['End_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3
print(f'| kernel (one train step) | calls | us | % |\n|---|---|---|---|')
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f'| `{n}` | {c} | {t:.1f} | {100 * t / tot:.1f} |')
print(f'\nkernel time per step {tot / 1e3:.2f} ms; first-to-last dispatch span {wall / 1e3:.2f} ms')
