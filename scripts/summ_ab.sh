#!/bin/bash
# Summarise an A/B directory: every bench line's value, then the grouped kernels of its one-stream trace.
d=$1
for f in $d/*.json; do python3 -c "
import json,sys
d=json.load(open('$f')); print('%-28s %.4e %s' % ('$(basename $f .json)', d['value'], d['config'].get('launch_order','')))
" 2>/dev/null; done
[ -f $d/trace_s1/run_kernel_stats.csv ] && python3 - $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + '/trace_s1/run_kernel_stats.csv')):
    n = r['Name']
    if any(k in n for k in ['k_group', 'k_search', 'k_emit']):
        print('%-60s %6s %8.1f us' % (n[:60], r['Calls'], float(r['AverageNs']) / 1000))
PY
[ -f $d/pytest_grouped.log ] && tail -1 $d/pytest_grouped.log
true
