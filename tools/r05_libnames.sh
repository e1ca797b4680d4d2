#!/bin/bash
# kernel names / durations of the library GEMMs at the config-2 shapes (rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/libnames; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 tools/nt_library_compare.py --only cfg2 --iters 10 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
cat $O/run.log | grep -v amdgpu.ids
f=$(find $O -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows: print(r['Name'][:110], r['Calls'], r['AverageNs'])
"
