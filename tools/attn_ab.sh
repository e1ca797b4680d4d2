# fused vs split attention backward, microbenchmark at the workload shape
mkdir -p gpurun_out
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn_f.log 2>&1 || exit $?
timeout -k 10 120 python - > gpurun_out/attn_s.log 2>&1 <<PY || exit $?
import sys, runpy
sys.argv = ["tools/attn_bench.py"]
sys.path.insert(0, ".")
from scattennet_amd import _lib as L
L.lib().sca_attn_bwd_fused(0)
runpy.run_path("tools/attn_bench.py", run_name="__main__")
PY
echo fused; grep "us" gpurun_out/attn_f.log; echo split; grep "us" gpurun_out/attn_s.log
