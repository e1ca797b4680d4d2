#!/bin/bash
set -o pipefail
O=gpurun_out/r05tn5
mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "[$name] rc=$rc"; tail -n ${TAILN:-4} "$O/$name.log" | cut -c1-300; return $rc; }
step ours 400 python -u tools/tn_library_compare.py || exit 1
step lib 300 python -u tools/tn_library_compare.py --library || exit 1
