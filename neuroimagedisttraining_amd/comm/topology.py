"""Decentralised-FL topologies as row-stochastic mixing matrices (reference
``fedml_core/distributed/topology/{base,symmetric,asymmetric}_topology_manager.py``).

* symmetric: ring (Watts-Strogatz k=2, p=0) union Watts-Strogatz(k=neighbor_num, p=0) links, self loops,
  rows normalised;
* asymmetric: the symmetric graph plus ``out_directed_neighbor`` random directed links per node.

The mixing matrix ``W`` is what the MI355X D-PSGD path consumes directly: one client-stacked GEMM
``theta_new = W_local @ theta`` (rows = local clients, cols = all clients gathered over RCCL), instead of the
reference's per-neighbour Python loops.  Graph construction is written directly in numpy (no networkx needed;
for p=0 Watts-Strogatz is the k-nearest-neighbour ring lattice).
"""
from __future__ import annotations

import abc

import numpy as np


def ring_lattice(n, k):
    """Adjacency of a ring lattice where each node links to its k//2 neighbours on each side (WS with p=0)."""
    a = np.zeros((n, n), dtype=np.float32)
    half = max(0, int(k) // 2)
    for i in range(n):
        for d in range(1, half + 1):
            a[i, (i + d) % n] = 1
            a[i, (i - d) % n] = 1
    np.fill_diagonal(a, 0)
    return a


class BaseTopologyManager(abc.ABC):
    @abc.abstractmethod
    def generate_topology(self):
        ...

    @abc.abstractmethod
    def get_in_neighbor_idx_list(self, node_index):
        ...

    @abc.abstractmethod
    def get_out_neighbor_idx_list(self, node_index):
        ...

    @abc.abstractmethod
    def get_in_neighbor_weights(self, node_index):
        ...

    @abc.abstractmethod
    def get_out_neighbor_weights(self, node_index):
        ...


def _row_normalise(a):
    return (a / a.sum(1, keepdims=True)).astype(np.float32)


class SymmetricTopologyManager(BaseTopologyManager):
    def __init__(self, n, neighbor_num=2):
        self.n = n
        self.neighbor_num = neighbor_num
        self.topology = np.zeros((0, 0), dtype=np.float32)

    def generate_topology(self):
        a = np.maximum(ring_lattice(self.n, 2), ring_lattice(self.n, self.neighbor_num))
        np.fill_diagonal(a, 1)
        self.topology = _row_normalise(a)
        return self.topology

    def get_in_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    get_out_neighbor_weights = get_in_neighbor_weights

    def get_in_neighbor_idx_list(self, node_index):
        w = self.get_in_neighbor_weights(node_index)
        return [j for j, v in enumerate(w) if v > 0 and j != node_index]

    get_out_neighbor_idx_list = get_in_neighbor_idx_list


class AsymmetricTopologyManager(BaseTopologyManager):
    def __init__(self, n, undirected_neighbor_num=3, out_directed_neighbor=3, seed=None):
        self.n = n
        self.undirected_neighbor_num = undirected_neighbor_num
        self.out_directed_neighbor = out_directed_neighbor
        self.rng = np.random.RandomState(seed) if seed is not None else np.random
        self.topology = np.zeros((0, 0), dtype=np.float32)

    def generate_topology(self):
        a = np.maximum(ring_lattice(self.n, 2), ring_lattice(self.n, self.undirected_neighbor_num))
        for i in range(self.n):
            cand = [j for j in range(self.n) if j != i and a[i, j] == 0]
            if cand:
                pick = self.rng.choice(cand, min(len(cand), self.out_directed_neighbor), replace=False)
                a[i, pick] = 1
        np.fill_diagonal(a, 1)
        self.topology = _row_normalise(a)
        return self.topology

    def get_in_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[:, node_index]

    def get_out_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    def get_in_neighbor_idx_list(self, node_index):
        w = self.get_in_neighbor_weights(node_index)
        return [j for j, v in enumerate(w) if v > 0 and j != node_index]

    def get_out_neighbor_idx_list(self, node_index):
        w = self.get_out_neighbor_weights(node_index)
        return [j for j, v in enumerate(w) if v > 0 and j != node_index]


def mixing_matrix(kind, n, round_idx=0, client_idx=None, neighbors=None, seed=0):
    """Neighbour-averaging matrices of the reference's decentralised baselines (``dpsgd_api.py:116-139``):
    ``ring`` (self + 2 ring neighbours), ``full`` (everyone), ``random`` (self + ``neighbors`` clients drawn with
    ``np.random.seed(round + client)``).  Rows are uniform over the chosen set."""
    w = np.zeros((n, n), dtype=np.float32)
    for i in range(n):
        if kind == "ring":
            s = {i, (i - 1) % n, (i + 1) % n}
        elif kind == "full":
            s = set(range(n))
        elif kind == "random":
            rs = np.random.RandomState(round_idx + i + seed)
            k = min(n - 1, int(neighbors or 1))
            s = {i} | set(rs.choice([j for j in range(n) if j != i], k, replace=False).tolist())
        else:
            raise ValueError(kind)
        w[i, sorted(s)] = 1.0 / len(s)
    return w
