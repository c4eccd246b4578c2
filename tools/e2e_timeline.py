"""Kernel timeline of the last pv_verify_batch call from a rocprofv3
--kernel-trace csv directory (tools/e2e_trace.py under rocprofv3).  Copies are
not used: rocprofiler-sdk drops async-copy completion callbacks on this image
(it times out waiting for them), so a copy timeline is incomplete.  The last
call = from the k_hash launch (or the fused k_chunk_half launch) of its first
chunk (the last `chunks` per-chunk grids).  Prints the events, the GPU kernel-busy union and the kernel
overlap between consecutive chunks (two compute streams).
    python tools/e2e_timeline.py DIR [chunks]"""
import csv
import glob
import os
import sys


def main(d, chunks=9):
    ev = []
    for fn in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(fn)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0]))
    ev.sort()
    # per-chunk grids: k_curve_half (hash / lattice / curve schedule) or
    # k_chunk_half (fused chunks, host_fused 1; no k_hash before them)
    curves = [i for i, e in enumerate(ev) if 'k_curve' in e[2] or 'k_chunk_half' in e[2]]
    first_curve = curves[-chunks]
    prev = curves[-chunks - 1] if len(curves) > chunks else -1
    hashes = [i for i in range(prev + 1, first_curve) if 'k_hash' in ev[i][2]]
    start = max(hashes) if hashes else first_curve
    last = ev[start:]
    t0 = last[0][0]
    print('# last call: {} chunks; start end dur (us) kernel'.format(chunks))
    for s, e, n in last:
        print('{:10.1f} {:10.1f} {:8.1f} {}'.format((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, n))
    spans = sorted((s, e) for s, e, _ in last)
    busy, cs, ce, gaps = 0, spans[0][0], spans[0][1], []
    for s, e in spans[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(round((s - ce) / 1e3, 1))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    span = (max(e for _, e in spans) - t0) / 1e3
    ov = 0
    cv = [(s, e) for s, e, n in last if 'k_curve' in n]
    hs = [(s, e) for s, e, n in last if 'k_hash' in n or 'k_lattice' in n]
    for s, e in hs:
        for a, b in cv:
            ov += max(0, min(e, b) - max(s, a))
    print('# kernel span {:.1f} us, kernel-busy union {:.1f} us ({:.1%}), idle gaps (us) {}'.format(
        span, busy / 1e3, busy / 1e3 / span, gaps))
    print('# hash/lattice time overlapped with a curve grid of another chunk: {:.1f} us'.format(ov / 1e3))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 9)
