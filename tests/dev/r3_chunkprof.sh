# chunk resolver: diag counters, then per-kernel times (rocprofv3 kernel trace) of the A/B run
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cprof
timeout -k 10 200 python -u tests/dev/diag_chunk.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof -o run -- python3 tests/dev/ab_resolvers.py chunk > gpurun_out/cprof/ab.txt 2>&1
rc=$?; tail -3 gpurun_out/cprof/ab.txt
f=$(find gpurun_out/cprof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r, key=lambda x:-float(x['TotalDurationNs']))[:10]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1000,1), 'us avg')
"
exit $rc
