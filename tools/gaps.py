"""Idle gaps between consecutive kernels of the last timed train step in a rocprofv3
--kernel-trace run (python tools/gaps.py gpurun_out/prof_gen [min_us]): the largest gaps with
the kernels on either side, to find host-side stalls (syncs, launch-bound stretches)."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_gen'
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
rows = sorted(csv.DictReader(open(f'{d}/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
rows = rows[idx[-2] + 1: idx[-1] + 1]
name = lambda r: r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][:60]
gaps = []
for a, b in zip(rows, rows[1:]):
    g = (int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3
    gaps.append((g, name(a), name(b)))
tot = sum(g for g, _, _ in gaps if g > 0)
print(f'kernels {len(rows)}, total gap {tot:.1f} us, gaps > {min_us} us: '
      f'{sum(g for g, _, _ in gaps if g > min_us):.1f} us')
for g, a, b in sorted(gaps, reverse=True)[:25]:
    print(f'{g:9.1f}  {a}  ->  {b}')
