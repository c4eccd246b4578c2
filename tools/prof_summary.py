"""Per-kernel duration summary from a rocprofv3 output (csv dir or rocpd .db)."""
import collections
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
    sym = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
    cols = [r[1] for r in c.execute('pragma table_info(%s)' % sym)]
    namecol = 'kernel_name' if 'kernel_name' in cols else 'display_name'
    rows = c.execute('select s.%s, d.start, d."end" from %s d join %s s on d.kernel_id = s.id' % (namecol, disp, sym))
    return [(n, (e - s) / 1e6) for n, s, e in rows]


def from_csv(d):
    out = []
    for fn in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                out.append((r['Kernel_Name'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6))
    return out


def main(path):
    rows = from_db(path) if path.endswith('.db') else from_csv(path)
    agg = collections.defaultdict(list)
    for n, ms in rows:
        agg[n].append(ms)
    print('%-60s %6s %12s %12s %12s' % ('kernel', 'calls', 'avg_ms', 'min_ms', 'total_ms'))
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        short = n.split('(')[0][:60]
        print('%-60s %6d %12.4f %12.4f %12.3f' % (short, len(v), sum(v) / len(v), min(v), sum(v)))


if __name__ == '__main__':
    main(sys.argv[1])
