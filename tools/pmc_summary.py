"""Median of every PMC counter per kernel over rocprofv3 --pmc passes:
python tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ... > profiles/rNN_pmc_summary.txt"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    vals[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))
    for k in sorted(vals):
        if not k.startswith(('void bsls::', 'bsls::')):
            continue
        print(k[:72])
        for c in sorted(vals[k]):
            v = vals[k][c]
            print('   %-28s %18.1f  (rows %d)' % (c, statistics.median(v), len(v)))


if __name__ == '__main__':
    main(sys.argv[1:])
