"""Run bench.py with module attributes of scattennet_amd.ops / keypoint_module / layers
overridden first (A/B experiments without product switches):

    python tools/bench_var.py "ops._FAN_OUT=False" [more assignments] -- [bench.py args]
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")  # as bench.py, before torch initialises HIP
from scattennet_amd import keypoint_module, layers, ops  # noqa: E402,F401

argv = sys.argv[1:]
cut = argv.index("--") if "--" in argv else len(argv)
for stmt in argv[:cut]:
    exec(stmt, {"ops": ops, "keypoint_module": keypoint_module, "layers": layers})
sys.argv = [os.path.join(ROOT, "bench.py")] + argv[cut + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
