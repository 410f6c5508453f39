"""HBM traffic of the conv family (the bench's roofline kernel family) from rocprofv3 PMC passes.

    python tools/traffic.py --fetch gpurun_out/pmcF --write gpurun_out/pmcW --steps 3 \
        --config gen --out profiles/r01/traffic_gen.json

--fetch / --write: output dirs of `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs (one
counter block per pass) of `bench.py --steps S --warmup W --no-roofline`; --steps = S + W (every
train step the profiled process ran). Corrections, calibrated on this GPU (tools/mb/fetch_calib.hip,
profiles/r05/fetch_calibration.md: 512 MiB read once with 16-B aligned, 16-B unaligned, 8-B and 4-B
loads, and written with 16-B and 4-B stores): counters are in KiB; FETCH_SIZE reports half the bytes
read for EVERY load width (so x2 on every kernel), WRITE_SIZE the bytes written exactly. The result
is per train step and per conv-family ABI call (bench.py reads it into roofline.traffic)."""
import argparse
import collections
import csv
import json
import re

# kernels launched by the conv / convtr / conv2d ABI entry points (csrc/conv1d.hip, disc.hip)
# (csrc/resblock.hip's fused residual-block kernels are conv ABI calls too: encx_resblock_*)
# (round 6: the v2 kernels, and the short-T layers' im2col / epilogue kernels with their hipBLASLt
# GEMMs, `Cijk_*`; the LSTM weight grads' library GEMMs carry the same names and are counted in
# too, an overcount of their few tens of MB per step)
FAMILY = re.compile(r'conv_fwd_kernel|conv_fwd2_kernel|pw_kernel|pw_wgrad_kernel|conv_poly_kernel|conv_poly2_kernel|'
                    r'conv_wgrad|wgrad_reduce|conv_fwd_reduce|conv_poly_reduce|conv_fold_edges|LdConvFlat|LdPolyFlat|'
                    r'c2_|rb_fwd_kernel|rb_bwd_kernel|rb_dgrad_kernel|rb_wgrad_kernel|rb_wgrad_reduce|im2col_kernel|'
                    r'gemm_epi_kernel|wg_transpose_kernel|wg_colsum|Cijk_')


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


def family_kib(d, counter):
    """-> (KiB over the conv-family dispatches, dispatch count, kernel names)."""
    vals, names = per_dispatch(d, counter)
    tot, n, kinds = 0.0, 0, set()
    for k, v in vals.items():
        if FAMILY.search(names[k]):
            tot += v
            n += 1
            kinds.add(re.sub(r'[<(].*', '', names[k].replace('(anonymous namespace)::', '')).replace('void ', ''))
    return tot, n, kinds


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
    f_kib, nf, kinds = family_kib(args.fetch, 'FETCH_SIZE')
    w_kib, nw, _ = family_kib(args.write, 'WRITE_SIZE')
    fetch = 2 * f_kib * 1024 / args.steps  # calibrated: x2 for every load width (gfx950)
    write = w_kib * 1024 / args.steps
    res = {'config': args.config, 'fetch_bytes_per_step': fetch, 'write_bytes_per_step': write,
           'hbm_bytes_per_step': fetch + write, 'kernel_dispatches_per_step': nf / args.steps,
           'fetch_bytes_per_step_uncorrected': f_kib * 1024 / args.steps,
           'correction': 'FETCH_SIZE x2 on every kernel (calibrated for 16-B aligned / unaligned, 8-B and '
                         '4-B loads: profiles/r05/fetch_calibration.md), WRITE_SIZE x1; KiB -> bytes',
           'kernels': sorted(kinds),
           'steps_profiled': args.steps}
    if args.calls_per_step:
        res['abi_calls_per_step'] = args.calls_per_step
        res['hbm_bytes_per_call'] = (fetch + write) / args.calls_per_step
    json.dump(res, open(args.out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
