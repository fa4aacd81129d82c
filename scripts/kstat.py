import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in sys.argv[3:]):
        print(sys.argv[2], r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
