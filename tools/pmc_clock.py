"""Clock of each dispatch of a kernel from a pmc_clock.sh CSV: GRBM_GUI_ACTIVE / XCDs / duration."""
import csv
import glob
import os
import sys

root, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else 'curve_half')
for f in sorted(glob.glob(os.path.join(root, '*', '*counter_collection.csv'))):
    rows = {}
    for r in csv.DictReader(open(f)):
        if sub not in r['Kernel_Name']:
            continue
        d = rows.setdefault(r['Dispatch_Id'], {'ns': int(r['End_Timestamp']) - int(r['Start_Timestamp'])})
        d[r['Counter_Name']] = d.get(r['Counter_Name'], 0) + float(r['Counter_Value'])
    print('==', os.path.basename(os.path.dirname(f)))
    for k, d in sorted(rows.items(), key=lambda x: int(x[0])):
        ghz = d.get('GRBM_GUI_ACTIVE', 0) / 8 / d['ns']
        print('  dispatch {} {:.3f} ms  clock {:.3f} GHz (GUI_ACTIVE/8)  GRBM_COUNT/8/ns {:.3f}'.format(
            k, d['ns'] / 1e6, ghz, d.get('GRBM_COUNT', 0) / 8 / d['ns']))
