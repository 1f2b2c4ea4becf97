"""Supply-network helpers, restating utils.py:87-130 of the reference.

check_connections (utils.py:87-92), create_network (94-102), get_stage (105-120),
get_retailers (124-130). Host-side only: they shape the EnvSpec.
"""
import numpy as np


def check_connections(connections):
    """Downstream nodes must have larger indices than their upstream node (utils.py:87-92)."""
    for node, children in connections.items():
        for child in (children or []):
            if child < node:
                raise Exception("Downstream node cannot have a smaller index number than upstream node")


def create_network(connections):
    """Adjacency matrix network[parent][child] = 1, sized by the largest key (utils.py:94-102)."""
    n = max(connections.keys()) + 1
    net = np.zeros((n, n))
    for parent, children in connections.items():
        for child in (children or []):
            net[parent][child] = 1
    return net


def get_stage(node, network):
    """Number of hops from node 0 (utils.py:105-120); raises on a disconnected node."""
    if node == 0:
        return 0
    depth = 0
    for _ in range(len(network) + 1):
        ups = [i for i in range(len(network)) if network[i][node] == 1]
        if not ups:
            break
        node = ups[0]
        depth += 1
        if node == 0:
            return depth
    raise Exception("Infinite Loop")


def get_retailers(network):
    """Nodes with no downstream connection (utils.py:124-130)."""
    return [i for i in range(len(network)) if not any(network[i])]
