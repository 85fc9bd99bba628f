"""Sub-train-job DAG helpers for the planned "ensemble of sub-train-jobs" feature
(reference rafiki/utils/graph.py:1-60, unused there and broken: it raises an undefined
``InvalidDAGException``).  Same functions, working: Kahn's algorithm with a deterministic order,
cycle detection via the leftover-node check.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List


class InvalidDAGError(Exception):
    pass


def build_dag(sub_train_jobs, ensemble=None) -> Dict[str, List[str]]:
    """Every sub-train-job feeds the ensemble model's sub-train-job (if one is given)."""
    ens = None
    if ensemble is not None:
        ens = next((s for s in sub_train_jobs if s.model_id == ensemble.id), None)
    adj = {}
    for s in sub_train_jobs:
        adj[s.id] = [] if ens is None or s.id == ens.id else [ens.id]
    return adj


def get_children(node, adj):
    return list(adj[node])


def get_parents(node, adj):
    return [n for n, kids in adj.items() if node in kids]


def get_nodes_with_zero_incoming_degrees(adj):
    indeg = {n: 0 for n in adj}
    for kids in adj.values():
        for k in kids:
            indeg[k] = indeg.get(k, 0) + 1
    return sorted(n for n, d in indeg.items() if d == 0)


def topological_order(adj) -> List[str]:
    nodes = set(adj)
    for kids in adj.values():
        nodes.update(kids)
    indeg = {n: 0 for n in nodes}
    for kids in adj.values():
        for k in kids:
            indeg[k] += 1
    q = deque(sorted(n for n in nodes if indeg[n] == 0))
    out = []
    while q:
        n = q.popleft()
        out.append(n)
        for k in sorted(adj.get(n, [])):
            indeg[k] -= 1
            if indeg[k] == 0:
                q.append(k)
    if len(out) != len(nodes):
        raise InvalidDAGError('graph has a cycle')
    return out


def validate_dag(adj) -> bool:
    try:
        topological_order(adj)
        return True
    except InvalidDAGError:
        return False
