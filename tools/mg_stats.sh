#!/bin/bash
# print the MultiGet kernels' average durations of a tools/mg_profile.sh run: tools/mg_stats.sh TAG
for c in wide lsm; do python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$1/$c/${c}_kernel_stats.csv')):
    if 'mg' in r['Name'] or 'multiget' in r['Name']: print('$c', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"; done
