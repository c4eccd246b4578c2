"""Sum rocprofv3 --pmc counter_collection.csv rows per (kernel, counter) and
print one table per variant directory: python tools/pmc_table.py DIR [kernel-substr]"""
import collections
import csv
import glob
import os
import sys


def load(path):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            k = r['Kernel_Name']
            tot[(k, r['Counter_Name'])] += float(r['Counter_Value'])
            disp[k].add(r['Dispatch_Id'])
    return tot, disp


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else 'curve_half'
    for f in sorted(glob.glob(os.path.join(root, '*', '*counter_collection.csv'))):
        tot, disp = load(f)
        print('==', os.path.basename(os.path.dirname(f)))
        for (k, c), v in sorted(tot.items()):
            if sub in k:
                print('  {:28s} {:>16.0f}   per dispatch {:>14.0f}'.format(c, v, v / max(1, len(disp[k]))))


if __name__ == '__main__':
    main()
