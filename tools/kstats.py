"""Summarise a rocprofv3 kernel_stats.csv (our kernels only)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r['Name']
    if 'at::' in n or 'rocblas' in n or 'Cijk' in n or 'rocclr' in n:
        continue
    print('%-72s %5s %9.2f ms %9.1f us avg %9.1f max' % (n[:72], r['Calls'], int(r['TotalDurationNs']) / 1e6,
                                                         float(r['AverageNs']) / 1e3, float(r['MaxNs']) / 1e3))
