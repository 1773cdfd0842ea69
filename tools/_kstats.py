import csv, glob, re, sys, json
for d in sys.argv[1:]:
    f = glob.glob(d + '/**/*kernel_stats.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    j = json.loads(open(d + '.json').read().strip().splitlines()[-1])
    print(d, 'value', round(j['value'], 2), 'ms/step', round(j['ms_per_step'], 3))
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:9]:
        m = re.search(r'(k_\w+)', r['Name'])
        print('   %-18s avg_us=%8.1f  pct=%5.1f' % (m.group(1) if m else r['Name'][:18], float(r['AverageNs']) / 1e3, float(r['Percentage'])))
