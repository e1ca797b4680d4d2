set -o pipefail
timeout -k 10 120 python -u tools/gemm_stamps.py > gpurun_out/stamps.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/stamps.log
bash tools/tn_pmc.sh r03_tnpmc 2>&1 | tail -60
