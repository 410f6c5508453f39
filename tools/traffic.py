"""HBM traffic of the conv family (the bench's roofline kernel family) from rocprofv3 PMC passes.

    python tools/traffic.py --fetch gpurun_out/pmcF --write gpurun_out/pmcW --steps 3 \
        --config gen --out profiles/r01/traffic_gen.json

--fetch / --write: output dirs of `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs (one
counter block per pass) of `bench.py --steps S --warmup W --no-roofline`; --steps = S + W (every
train step the profiled process ran). Corrections as in MI355X_MICROARCH.md "HBM": counters are in
KiB; FETCH_SIZE is doubled ONLY for the kernels whose reads are 16-byte-per-lane (dwordx4) loads,
the access width the guide calibrates (gfx950 tallies their 128-B requests at 64 B); the kernels
that read with 4-byte loads (the fixed-order slab reductions, the one-channel post conv, the
first-layer forward) are left uncorrected, as the guide leaves other widths uncalibrated. Both
lists are written into the output. The result is per train step and per conv-family ABI call
(bench.py reads it into roofline.traffic)."""
import argparse
import collections
import csv
import json
import re

# kernels launched by the conv / convtr / conv2d ABI entry points (csrc/conv1d.hip, disc.hip)
# (csrc/resblock.hip's fused residual-block kernels are conv ABI calls too: encx_resblock_*)
FAMILY = re.compile(r'conv_fwd_kernel|pw_kernel|pw_wgrad_kernel|conv_poly_kernel|conv_wgrad|wgrad_reduce|conv_fwd_reduce|'
                    r'conv_poly_reduce|conv_fold_edges|LdConvFlat|LdPolyFlat|c2_|rb_fwd_kernel|rb_bwd_kernel|'
                    r'rb_dgrad_kernel|rb_wgrad_kernel|rb_wgrad_reduce')


def per_dispatch(d, counter):
    out = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f'{d}/run_counter_collection.csv')):
        if r['Counter_Name'] != counter:
            continue
        key = int(r['Dispatch_Id'])
        out[key] += float(r['Counter_Value'])
        names[key] = r['Kernel_Name']
    return out, names


# conv-family kernels whose operand reads are dwordx4 (ld4u / f32x4) loads
WIDE = re.compile(r'conv_fwd_kernel|conv_poly_kernel|conv_wgrad_kernel|pw_kernel|pw_wgrad_kernel|'
                  r'LdConvFlat|LdPolyFlat|c2_fwd_rw|c2_dgrad_rw|c2_wgrad_rw|c2_fwdr|c2_dgradr|c2_wgrad3|'
                  r'c2_dgrad_narrow')


def family_kib(d, counter, split=False):
    vals, names = per_dispatch(d, counter)
    tot, wide, n = 0.0, 0.0, 0
    kinds = {'wide': set(), 'narrow': set()}
    for k, v in vals.items():
        if FAMILY.search(names[k]):
            tot += v
            n += 1
            w = bool(WIDE.search(names[k]))
            wide += v if w else 0.0
            kinds['wide' if w else 'narrow'].add(re.sub(r'[<(].*', '', names[k].replace('(anonymous namespace)::', '')).replace('void ', ''))
    return (tot, wide, n, kinds) if split else (tot, n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--fetch', required=True)
    ap.add_argument('--write', required=True)
    ap.add_argument('--steps', type=int, required=True)
    ap.add_argument('--config', default='gen')
    ap.add_argument('--calls-per-step', type=int, default=None,
                    help='conv-family ABI calls per step (bench roofline "launches" / steps)')
    ap.add_argument('--out', required=True)
    args = ap.parse_args()
    f_kib, f_wide, nf, kinds = family_kib(args.fetch, 'FETCH_SIZE', split=True)
    w_kib, nw = family_kib(args.write, 'WRITE_SIZE')
    fetch = (f_kib + f_wide) * 1024 / args.steps  # x2 on the wide-load kernels only
    write = w_kib * 1024 / args.steps
    res = {'config': args.config, 'fetch_bytes_per_step': fetch, 'write_bytes_per_step': write,
           'hbm_bytes_per_step': fetch + write, 'kernel_dispatches_per_step': nf / args.steps,
           'fetch_bytes_per_step_uncorrected': f_kib * 1024 / args.steps,
           # every conv-family kernel's FETCH_SIZE doubled (the upper bound if the narrow-load
           # kernels' requests are tallied at half size too; their width is uncalibrated)
           'hbm_bytes_per_step_conservative': 2 * f_kib * 1024 / args.steps + write,
           'correction': 'FETCH_SIZE x2 on the dwordx4-load kernels only (gfx950), KiB -> bytes',
           'fetch_x2_kernels': sorted(kinds['wide']), 'fetch_uncorrected_kernels': sorted(kinds['narrow']),
           'steps_profiled': args.steps}
    if args.calls_per_step:
        res['abi_calls_per_step'] = args.calls_per_step
        res['hbm_bytes_per_call'] = (fetch + write) / args.calls_per_step
        res['hbm_bytes_per_call_conservative'] = res['hbm_bytes_per_step_conservative'] / args.calls_per_step
    json.dump(res, open(args.out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
