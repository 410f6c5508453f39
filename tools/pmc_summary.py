"""Summarise rocprofv3 --pmc CSVs per kernel (last timed step of a bench run):
python tools/pmc_summary.py gpurun_out/pmc1 [gpurun_out/pmc2 ...]
FETCH_SIZE is doubled for every kernel: on gfx950 it reports half the bytes read for 16-B aligned,
16-B unaligned, 8-B and 4-B loads alike (tools/mb/fetch_calib.hip, profiles/r05/fetch_calibration.md)."""
import collections
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))



def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    seen = set()
    for r in csv.DictReader(open(f'{d}/run_counter_collection.csv')):
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][:70]
        per[name][r['Counter_Name']] += float(r['Counter_Value'])
        key = (r['Dispatch_Id'], name)
        if key not in seen:
            seen.add(key)
            cnt[name] += 1
            per[name]['_ns'] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            per[name]['_lds'] = float(r['LDS_Block_Size'])
            per[name]['_vgpr'] = float(r['VGPR_Count']) + float(r['Accum_VGPR_Count'])
    return per, cnt


def main():
    tabs = [load(d) for d in sys.argv[1:]]
    per, cnt = tabs[0]
    for p, _ in tabs[1:]:
        for k, v in p.items():
            for c, x in v.items():
                if not c.startswith('_'):
                    per[k][c] += x
    rows = sorted(per.items(), key=lambda kv: -kv[1]["_ns"])[:int(os.environ.get("PMC_TOP", "28"))]
    print('| kernel | calls | us/call | mfma busy | wait any | wait inst | lds conf | vgpr | lds B | fetch MB/call | '
          'write MB/call | HBM GB/s |')
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k, v in rows:
        n = cnt[k]
        wc = v.get('SQ_WAVE_CYCLES', 0) or 1
        # SQ_WAVE_CYCLES counts quad-cycles summed over waves; MFMA busy counts cycles per SIMD
        mb = v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0)
        gui = v.get('GRBM_GUI_ACTIVE', 0)
        busy = mb / (gui / 8 * 256 * 4) if gui else float('nan')
        fetch = v.get('FETCH_SIZE', 0) / n / 1024 * 2  # KB -> MB; x2: gfx950 counts half (calibrated)
        write = v.get('WRITE_SIZE', 0) / n / 1024
        gbs = (fetch + write) / max(v['_ns'] / n / 1e3, 1e-9) * 1e3  # MB per us = TB/s -> GB/s
        print(f"| `{k}` | {n} | {v['_ns'] / n / 1e3:.1f} | {busy:.2f} | {v.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
              f"{v.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | "
              f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, v.get('SQ_LDS_IDX_ACTIVE', 0)):.2f} | {v['_vgpr']:.0f} | "
              f"{v['_lds']:.0f} | {fetch:.1f} | {write:.1f} | {gbs:.0f} |")


if __name__ == '__main__':
    main()
