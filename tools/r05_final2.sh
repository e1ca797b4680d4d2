#!/bin/bash
# the round's last measurement set, plus the config-5 confirmation of the tile-43 split change
set -o pipefail
bash tools/r05_measure.sh tests r05j || exit $?
O=gpurun_out/r05j; 
for v in 1 0; do
  SCA_TNB_MODEL=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_model$v.log 2>&1 || exit $?
  echo "cfg5 model=$v $(grep -o '"value": [0-9.]*' $O/c5_model$v.log)"
done
bash tools/r05_measure.sh prof r05j || exit $?
