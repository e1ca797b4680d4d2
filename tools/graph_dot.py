"""Summarise a DEBUG_HIP_GRAPH_DOT_PRINT dump: node id, the executor's StreamId, kernel, parents.

    python tools/graph_dot.py gpurun_out/dot/graph_*_dot_print_1
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
nodes = {}
for m in re.finditer(r'"(graph_\d+_node_\d+)"\[[^\]]*label="(\d+)\n([^\n]*)\n(?:StreamId:(\d+))?', s):
    nodes[m.group(1)] = (int(m.group(2)), m.group(3), m.group(4))
par = collections.defaultdict(list)
for m in re.finditer(r'"(graph_\d+_node_\d+)"\s*->\s*"(graph_\d+_node_\d+)"', s):
    par[m.group(2)].append(m.group(1))


def short(k):
    k = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", k)
    return k[:40]


for key, (i, k, sid) in sorted(nodes.items(), key=lambda kv: kv[1][0]):
    ps = ",".join(str(nodes[p][0]) for p in par[key] if p in nodes)
    print(f"{i:4d} s{sid} {short(k):40s} <- {ps}")
