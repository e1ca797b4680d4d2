#!/bin/bash
# coord_map_fwd with the weights staged through LDS: parity tests, the kernel's duration
# (rocprofv3 --stats of a short config-2 / config-5 run), bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cmap; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_scale.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in cfg2 cfg5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
    python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$wl.log 2>&1 || exit $?
  f=$(find $O/prof_$wl -name "run_kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'coord_map' in r['Name'] or 'reduce_rows' in r['Name']: print('$wl', r['Name'][:40], r['Calls'], r['AverageNs'])
"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_$i.log 2>&1 || exit $?
  echo "cfg2 #$i $(grep -o '"value": [0-9.]*' $O/c2_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c2_$i.log)"
done
