"""Kernel statistics from a rocprofv3 --kernel-trace --stats database (rocpd
SQLite, the image's default output format): per kernel the calls, total and
average duration, and the average over the dispatches of its LARGEST grid (the
bench line's launch; the small latency calls of the same run are excluded).

    python tools/rocpd_stats.py gpurun_out/<dir>/run_results.db > profiles/rNN_..._kernel_stats.txt
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute('select name, duration, grid_x * grid_y * grid_z from kernels').fetchall()
    per = {}
    for name, dur, grid in rows:
        per.setdefault(name.split('(')[0], []).append((float(dur), int(grid)))
    total = sum(d for v in per.values() for d, _ in v)
    print('{:<48} {:>7} {:>12} {:>11} {:>7} {:>14} {:>9}'.format(
        'kernel', 'calls', 'total_ms', 'avg_ms', 'pct', 'big_grid_avg_ms', 'big_calls'))
    for name, v in sorted(per.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
        tot = sum(d for d, _ in v)
        g = max(x for _, x in v)
        big = [d for d, x in v if x == g]
        # rocpd durations are in ns
        print('{:<48} {:>7} {:>12.3f} {:>11.4f} {:>7.2f} {:>14.4f} {:>9}'.format(
            name[:48], len(v), tot / 1e6, tot / len(v) / 1e6, 100 * tot / total, sum(big) / len(big) / 1e6, len(big)))


if __name__ == '__main__':
    main(sys.argv[1])
