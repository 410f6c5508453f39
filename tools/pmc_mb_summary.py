"""Per-kernel-variant wave-state / MFMA / LDS counter summary of tools/gpu_pmc_mb.sh output:
python tools/pmc_mb_summary.py gpurun_out/pmcmb1 gpurun_out/pmcmb2"""
import collections
import csv
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    seen = set()
    for r in csv.DictReader(open(f'{d}/run_counter_collection.csv')):
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
        name = name[:name.index('>(') + 1] if '>(' in name else name.split('(')[0]
        per[name][r['Counter_Name']] += float(r['Counter_Value'])
        key = (r['Dispatch_Id'], name)
        if key not in seen:
            seen.add(key)
            cnt[name] += 1
            per[name]['_ns'] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            per[name]['_vgpr'] = float(r['VGPR_Count']) + float(r.get('Accum_VGPR_Count', 0) or 0)
            per[name]['_lds'] = float(r['LDS_Block_Size'])
    return per, cnt


def main():
    p1, c1 = load(sys.argv[1])
    p2, _ = load(sys.argv[2]) if len(sys.argv) > 2 else ({}, None)
    print('| kernel | us/call | vgpr | LDS B | MFMA busy | wait any | wait inst | active | LDS conf | VALU/MFMA | LDS/MFMA | SALU/MFMA | VMEM/MFMA |')
    print('|---|---|---|---|---|---|---|---|---|---|---|---|---|')
    for k in sorted(p1, key=lambda k: -p1[k]['_ns'] / c1[k]):
        v, w, n = p1[k], p2.get(k, {}), c1[k]
        mf = w.get('SQ_INSTS_MFMA', 0)
        if not v.get('SQ_VALU_MFMA_BUSY_CYCLES') or not mf:
            continue
        wc = v['SQ_WAVE_CYCLES'] or 1
        gui = v.get('GRBM_GUI_ACTIVE', 0)
        busy = v['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * 256 * 4) if gui else float('nan')
        print(f"| `{k}` | {v['_ns'] / n / 1e3:.1f} | {v['_vgpr']:.0f} | {v['_lds']:.0f} | {busy:.2f} | "
              f"{v['SQ_WAIT_ANY'] / wc:.2f} | {v['SQ_WAIT_INST_ANY'] / wc:.2f} | {v['SQ_ACTIVE_INST_ANY'] / wc:.2f} | "
              f"{v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_LDS_IDX_ACTIVE']):.2f} | "
              f"{w.get('SQ_INSTS_VALU', 0) / mf:.2f} | {w.get('SQ_INSTS_LDS', 0) / mf:.2f} | "
              f"{w.get('SQ_INSTS_SALU', 0) / mf:.2f} | {w.get('SQ_INSTS_VMEM_RD', 0) / mf:.3f} |")


if __name__ == '__main__':
    main()
