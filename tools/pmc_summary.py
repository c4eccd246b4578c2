"""Per-launch PMC summary of the verify kernels from tools/pmc_passes.sh output.

    python tools/pmc_summary.py gpurun_out/pmc > profiles/rNN_curve_pmc.json

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is
doubled (the curve kernel's table reads are 16 B/lane gathers, an access width
the guide leaves uncalibrated: the doubled figure is an upper estimate).
Infinity-Cache hits are counted too (fabric-side counters).
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, tag):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for fn in glob.glob(os.path.join(d, tag, '*counter_collection.csv')):
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                k = r['Kernel_Name'].split('(')[0]
                if k.startswith('void '):
                    k = k[5:]
                per[k][r['Counter_Name']].append(float(r['Counter_Value']))
    return per


def main(d):
    out = {'source': d, 'kernels': {}}
    merged = collections.defaultdict(dict)
    for tag in ('fetch', 'write', 'sq1', 'sq2', 'l2'):
        for k, counters in load(d, tag).items():
            for c, vals in counters.items():
                # one value per dispatch after summing over XCD/SE instances
                merged[k][c] = sum(vals) / max(1, len(vals))
    for k, c in merged.items():
        if not k.startswith('pv::k_'):
            continue
        e = dict(c)
        if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
            e['hbm_read_bytes'] = 2 * c['FETCH_SIZE'] * 1024
            e['hbm_write_bytes'] = c['WRITE_SIZE'] * 1024
            e['hbm_bytes_per_launch'] = e['hbm_read_bytes'] + e['hbm_write_bytes']
        if 'TCC_HIT_sum' in c and 'TCC_MISS_sum' in c:
            e['l2_hit_rate'] = c['TCC_HIT_sum'] / max(1.0, c['TCC_HIT_sum'] + c['TCC_MISS_sum'])
        if 'GRBM_GUI_ACTIVE' in c:
            e['gpu_cycles_per_xcd'] = c['GRBM_GUI_ACTIVE'] / 8
        out['kernels'][k] = e
    # the generic batches' curve kernel: k_curve_half (default), else the grouped k_curve<false>
    names = sorted(out['kernels'], key=lambda k: not k.startswith('pv::k_curve_half'))
    curve_k = next((k for k in names if k.startswith('pv::k_curve') and 'true' not in k), None)
    out['curve_kernel'] = curve_k
    out['hbm_bytes_per_launch'] = out['kernels'].get(curve_k, {}).get('hbm_bytes_per_launch')
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
