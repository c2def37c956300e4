"""Average every collected counter per kernel over the rocprofv3 passes under DIR.
    python tools/pmc_table.py DIR [kernel-substring]"""
import collections, csv, glob, os, sys

d, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else '')
acc = collections.defaultdict(list)
for p in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
    for r in csv.DictReader(open(p)):
        if sub in r['Kernel_Name']:
            name = r['Kernel_Name'].split('(')[0].replace('void ', '')
            acc[(name, r['Counter_Name'])].append(float(r['Counter_Value']))
kernels = sorted({k for k, _ in acc})
counters = sorted({c for _, c in acc})
print('counter'.ljust(44) + ''.join(k[-34:].rjust(36) for k in kernels))
for c in counters:
    row = [acc.get((k, c)) for k in kernels]
    print(c.ljust(44) + ''.join(('{:.4g}'.format(sum(v) / len(v)) if v else '-').rjust(36) for v in row))
