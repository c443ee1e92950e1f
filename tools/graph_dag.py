"""Dump the DAG of bench.py's captured step: every node of the hipGraph (kernel name for kernel nodes) and every edge,
read back through the HIP graph API (hipGraphGetNodes / hipGraphGetEdges / hipGraphKernelNodeGetParams) from the
graph StepGraph captured.  Runs bench.py's main with the given arguments and writes JSON to --out.

    python tools/graph_dag.py --out gpurun_out/dag.json -- --steps 3 --warmup 3 --no-cpu-baseline --no-fp32
    python tools/graph_dag.py --analyze gpurun_out/dag.json
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


class Dim3(ctypes.Structure):
    _fields_ = [('x', ctypes.c_uint32), ('y', ctypes.c_uint32), ('z', ctypes.c_uint32)]


class KernelNodeParams(ctypes.Structure):
    _fields_ = [('blockDim', Dim3), ('extra', ctypes.c_void_p), ('func', ctypes.c_void_p), ('gridDim', Dim3),
                ('kernelParams', ctypes.c_void_p), ('sharedMemBytes', ctypes.c_uint32)]


def extract(raw_graph):
    hip = ctypes.CDLL('libamdhip64.so')
    hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p
    hip.hipKernelNameRefByPtr.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    g = ctypes.c_void_p(raw_graph)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    idx = {nodes[i]: i for i in range(n.value)}
    out_nodes = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t))
        name = ''
        grid = None
        if t.value == 0:
            p = KernelNodeParams()
            if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nodes[i]), ctypes.byref(p)) == 0:
                nm = hip.hipKernelNameRefByPtr(p.func, None)
                name = nm.decode() if nm else hex(p.func or 0)
                grid = [p.gridDim.x, p.gridDim.y, p.gridDim.z]
        out_nodes.append({'id': i, 'type': t.value, 'name': name, 'grid': grid})
    m = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(g, None, None, ctypes.byref(m)) == 0
    fr = (ctypes.c_void_p * m.value)()
    to = (ctypes.c_void_p * m.value)()
    assert hip.hipGraphGetEdges(g, fr, to, ctypes.byref(m)) == 0
    edges = [[idx[fr[i]], idx[to[i]]] for i in range(m.value)]
    return {'nodes': out_nodes, 'edges': edges}


def analyze(path):
    d = json.load(open(path))
    nodes, edges = d['nodes'], d['edges']
    n = len(nodes)
    preds = [[] for _ in range(n)]
    succs = [[] for _ in range(n)]
    for a, b in edges:
        preds[b].append(a)
        succs[a].append(b)
    # longest path (in node count) and width profile: level = longest chain of predecessors
    order, indeg = [], [len(p) for p in preds]
    ready = [i for i in range(n) if indeg[i] == 0]
    while ready:
        i = ready.pop()
        order.append(i)
        for j in succs[i]:
            indeg[j] -= 1
            if indeg[j] == 0:
                ready.append(j)
    level = [0] * n
    for i in order:
        for j in succs[i]:
            level[j] = max(level[j], level[i] + 1)
    forks = [i for i in range(n) if len(succs[i]) > 1]
    joins = [i for i in range(n) if len(preds[i]) > 1]
    short = lambda i: (nodes[i]['name'].split('(')[0].replace('void ', '').replace('(anonymous namespace)::', '')[:48]
                       or f'type{nodes[i]["type"]}')
    print(f'{n} nodes, {len(edges)} edges, roots {sum(1 for p in preds if not p)}, depth {max(level) + 1}')
    for i in forks:
        print(f'fork  node {i:4d} level {level[i]:4d} {short(i)} -> ' + ', '.join(f'{j}:{short(j)}' for j in succs[i]))
    for i in joins:
        print(f'join  node {i:4d} level {level[i]:4d} {short(i)} <- ' + ', '.join(f'{j}:{short(j)}' for j in preds[i]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out')
    ap.add_argument('--analyze')
    ap.add_argument('--replay-timing', action='store_true',
                    help='after the capture, time hipGraphLaunch on the host (return of replay()) against the device')
    ap.add_argument('rest', nargs=argparse.REMAINDER)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
        return
    os.environ['SSSEG_GRAPH_KEEP'] = '1'
    import bench
    from ssseg import graph as sgraph
    orig = sgraph.StepGraph.__init__

    def patched(self, *args, **kw):
        orig(self, *args, **kw)
        if not getattr(sgraph, '_dag_written', False):
            sgraph._dag_written = True
            d = extract(self.graph.raw_cuda_graph())
            with open(a.out, 'w') as f:
                json.dump(d, f)
            print(f'graph_dag: {len(d["nodes"])} nodes, {len(d["edges"])} edges -> {a.out}', file=sys.stderr)
            if a.replay_timing:
                import time
                import torch
                torch.cuda.synchronize()
                for k in range(6):
                    t0 = time.perf_counter()
                    self.graph.replay()
                    t1 = time.perf_counter()
                    torch.cuda.synchronize()
                    t2 = time.perf_counter()
                    print(f'graph_dag replay {k}: host launch {1e3 * (t1 - t0):.2f} ms, launch+sync {1e3 * (t2 - t0):.2f} ms',
                          file=sys.stderr)

    sgraph.StepGraph.__init__ = patched
    rest = a.rest[1:] if a.rest and a.rest[0] == '--' else a.rest
    sys.argv = ['bench.py'] + rest
    bench.main()


if __name__ == '__main__':
    main()
