# Summarise rocprofv3 --pmc CSVs: per kernel, counters averaged over dispatches.
import csv, collections, sys, glob
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r['Kernel_Name'].split('(')[0]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    for k, v in agg.items():
        n = len(disp[k])
        print(path.split('/')[-2], k, n, " ".join("%s=%.4g" % (c, x / n) for c, x in sorted(v.items())))
