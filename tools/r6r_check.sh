# FETCH_SIZE against known request sizes (contiguous stream, 64..512-B random rows)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 60 ./tools/bin/fetch_probe > $O/requested.json || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o run --output-format csv -- ./tools/bin/fetch_probe > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 tools/fetch_probe_summary.py $O/pmc $O/requested.json | tee $O/fetch_probe.json
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- ./tools/bin/fetch_probe > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
python3 -c "
import csv, glob
for r in csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv', recursive=True)[0])):
    print(r['Name'][:40], r['Calls'], r['AverageNs'], r['MinNs'])
" | tee $O/kernel_times.txt
rm -rf $O/pmc $O/kt
