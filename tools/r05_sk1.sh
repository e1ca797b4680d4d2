#!/bin/bash
set -o pipefail
O=gpurun_out/sk1; mkdir -p $O
timeout -k 10 400 python -u tools/tn_library_compare.py --only "cfg2" --splits 0 --tnb-tiles 0 --ksplit-tiles 46 --ksplit-splits 1,2 > $O/tn.log 2>&1; rc=$?; grep "ksplit" $O/tn.log | grep "us"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    SCA_TNR_SK=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/sk${v}_$i.log 2>&1 || exit $?
    echo "cfg2 tnr_sk=$v #$i $(grep -o '"value": [0-9.]*' $O/sk${v}_$i.log)"
  done
done
