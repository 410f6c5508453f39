"""Summarise a rocprofv3 --kernel-trace run of bench.py: per-kernel totals over ONE timed train
step and the first-to-last dispatch span of that step.

python tools/prof_summary.py DIR [TOP] [--adams-per-step N]

A step is cut between two consecutive generator Adam launches. A GAN step (config 3/5) launches
two Adams (generator, then discriminator), so with N = 2 the slice runs from the generator Adam
of step k-1 to the generator Adam of step k: the discriminator phase of step k-1 and the
generator phase of step k, i.e. one whole step's kernels. N is detected from the bench log line
count when not given: 2 when both adam grid sizes occur, else 1."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument('dir', nargs='?', default='gpurun_out/prof')
ap.add_argument('top', nargs='?', type=int, default=40)
ap.add_argument('--adams-per-step', type=int, default=None)
args = ap.parse_args()

rows = list(csv.DictReader(open(f'{args.dir}/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name'] or 'adam_dev_kernel' in r['Kernel_Name']]
n_adam = args.adams_per_step
if n_adam is None:
    sizes = {r.get('Grid_Size', r.get('Grid_Size_X', '')) for r in (rows[i] for i in idx)}
    n_adam = 2 if len(sizes) > 1 else 1
a, b = idx[-1 - 2 * n_adam] + 1, idx[-1 - n_adam] + 1
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[a:b]:
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][:80]
    agg[n][0] += 1
    agg[n][1] += dur
tot = sum(v[1] for v in agg.values())
wall = (int(rows[b - 1]['End_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3
print(f'| kernel (one train step, {n_adam} Adam launch(es) per step) | calls | us | % |\n|---|---|---|---|')
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:args.top]:
    print(f'| `{n}` | {c} | {t:.1f} | {100 * t / tot:.1f} |')
print(f'\nkernel time per step {tot / 1e3:.2f} ms over {sum(v[0] for v in agg.values())} launches; '
      f'first-to-last dispatch span {wall / 1e3:.2f} ms')
