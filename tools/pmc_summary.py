"""Per-launch PMC summary of the verify kernels from tools/pmc_passes.sh output.

    python tools/pmc_summary.py gpurun_out/pmc [units] > profiles/rNN_curve_pmc.json

units (optional): the verifies / checks one launch of the dominant kernel
processed; adds hbm_bytes_per_unit so a bench line can scale the traffic to
its own launch size.

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
    """kernel -> counter -> values over the dispatches of the kernel's LARGEST
    grid (a bench run also launches the small latency calls; those are not the
    bench line's launch)"""
    rows = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(d, tag, '*counter_collection.csv')):
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                k = r['Kernel_Name'].split('(')[0]
                if k.startswith('void '):
                    k = k[5:]
                rows[k].append((int(r.get('Grid_Size') or 0), r['Counter_Name'], float(r['Counter_Value'])))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, rs in rows.items():
        g = max(x[0] for x in rs)
        for grid, c, v in rs:
            if grid == g:
                per[k][c].append(v)
    return per


def main(d, units=None):
    out = {'source': d, 'kernels': {}}
    merged = collections.defaultdict(dict)
    for tag in ('fetch', 'write', 'sq1', 'sq2', 'l2'):
        for k, counters in load(d, tag).items():
            for c, vals in counters.items():
                # one value per dispatch after summing over XCD/SE instances
                merged[k][c] = sum(vals) / max(1, len(vals))
    for k, c in merged.items():
        if not (k.startswith('pv::k_') or k.startswith('pvbls::k_')):
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
    bls_k = next((k for k in out['kernels'] if k.startswith('pvbls::k_bls_verify')), None)
    if bls_k:
        out['check_kernel'] = bls_k
        if curve_k is None:
            # the lane-pair check kernel and the sigma-prep kernel that feeds it
            parts = [out['kernels'][k].get('hbm_bytes_per_launch') for k in out['kernels']
                     if k == bls_k or k.startswith('pvbls::k_bls_sigprep')]
            out['hbm_bytes_per_launch'] = None if None in parts else sum(parts)
    if units:
        out['units_per_launch'] = units
        if out['hbm_bytes_per_launch'] is not None:
            out['hbm_bytes_per_unit'] = out['hbm_bytes_per_launch'] / units
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
