set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_d
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python tools/gram_only_time.py spot 20000 f64 2 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); python -c "
import csv; r=list(csv.DictReader(open('$f')))
for x in r: print('%-90s n=%5s avg_ns=%10.1f' % (x['Name'][:90], x['Calls'], float(x['AverageNs'])))"
