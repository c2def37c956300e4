import csv, collections, sys, glob
for f in sorted(glob.glob(sys.argv[1] + '/*/p_counter_collection.csv')):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if sys.argv[2] not in r['Kernel_Name']:
            continue
        key = (r['Kernel_Name'][:40])
        d.setdefault(r['Dispatch_Id'], {})[r['Counter_Name']] = float(r['Counter_Value'])
    last = list(d.values())[-1] if d else {}
    print(f, {k: '%.4g' % v for k, v in last.items()})
