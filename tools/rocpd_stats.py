"""Kernel statistics from a rocprofv3 SQLite output (run_results.db: rocprofv3
on this image writes rocpd databases by default), in the layout of the
round-1 --stats summaries: per kernel calls, total / avg / min / max duration.

    python tools/rocpd_stats.py DIR_OR_DB [--timeline KERNEL_SUBSTR]

--timeline also prints every dispatch of the matching kernel (start, end,
duration, stream), to read pipelined launches (overlapping intervals)."""
import glob
import os
import sqlite3
import sys


def main():
    p = sys.argv[1]
    db = p if p.endswith('.db') else glob.glob(os.path.join(p, '**', '*.db'), recursive=True)[0]
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute('select name, count(*), sum(duration), avg(duration), min(duration), max(duration) '
                       'from kernels group by name order by sum(duration) desc').fetchall()
    tot = sum(r[2] for r in rows)
    print('# {}  (durations in us)'.format(db))
    print('{:<34} {:>6} {:>12} {:>10} {:>10} {:>10} {:>6}'.format('kernel', 'calls', 'total', 'avg', 'min', 'max', '%'))
    for name, n, s, a, lo, hi in rows:
        short = name.split('(')[0]
        print('{:<34} {:>6} {:>12.1f} {:>10.1f} {:>10.1f} {:>10.1f} {:>6.2f}'.format(
            short[:34], n, s / 1e3, a / 1e3, lo / 1e3, hi / 1e3, 100.0 * s / tot))
    if '--timeline' in sys.argv:
        sub = sys.argv[sys.argv.index('--timeline') + 1]
        ev = cur.execute('select start, end, duration, stream from kernels where name like ? order by start',
                         ('%' + sub + '%',)).fetchall()
        if ev:
            t0 = ev[0][0]
            print('# dispatches of *{}*: start end duration (us) stream'.format(sub))
            for s, e, d, st in ev:
                print('{:12.1f} {:12.1f} {:10.1f} {}'.format((s - t0) / 1e3, (e - t0) / 1e3, d / 1e3, st))


if __name__ == '__main__':
    main()
