import csv,sys,glob
for d in sys.argv[1:]:
    f=glob.glob(d+'/**/*kernel_stats.csv',recursive=True)
    rows=list(csv.DictReader(open(f[0])))
    print(d)
    for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:8]:
        print('  %-60s n=%5s avg %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
