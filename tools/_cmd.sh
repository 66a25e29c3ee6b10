set -u
export TMPDIR=/tmp
O=gpurun_out/r03lat; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/dbg/single_frame.py > $O/lat.log 2>&1 || exit $?
grep "^{" $O/lat.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'zfft' in r['Name'] or 'copy' in r['Name'].lower(): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
