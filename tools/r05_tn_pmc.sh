#!/bin/bash
# MFMA busy / clock of the weight-gradient kernels at the config-5 attention shape (isolated launches)
export TMPDIR=/tmp
O=gpurun_out/r05tnpmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O -o sq -- python3 tools/tn_library_compare.py --only "${ONLY:-cfg5 attn}" --profile "ksplit36 sk=3,bmm" --iters 3 > $O/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 $O/run.log
python3 tools/tn_pmc2.py $O
