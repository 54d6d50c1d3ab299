"""Resource placement over the ranks of a node (the routing above the engines).

Each engine owns the resources whose *engine id* e satisfies ``e % N == rank``
(``sf_config.shard_count`` / ``shard_index``; its local row is ``e // N``).
By default a resource's engine id is its own id, so rank ``res % N`` holds it.
A Zipf trace then leaves the rank that happens to hold the busiest resources
with far more events than the mean (1.62x for config 3 at
N = 8), and with weak scaling the node runs at that rank's pace.

Resources are independent on the decision path (one ClusterNode per
resource, ClusterBuilderSlot.java:83-114; SystemRule's node-wide reads go
through the exchange, sf_sysx.h), so any resource -> rank map decides
exactly the same verdicts.  ``Placement.balanced`` moves the top-K resources
by the previous batch's counts: longest-processing-time first, each to the
rank with the least load so far (the remaining resources' load counted at
their default ranks), and gives each moved resource a fresh engine id
``R_pad + N * j + rank`` (j-th resource moved to that rank) past every
default id, so no default id changes.  The caller (bench.py, the Java
EventBatcher) renames events and rules with ``engine_id``; the engine is
unchanged."""
from __future__ import annotations

import numpy as np


class Placement:
    def __init__(self, R: int, N: int, moved: np.ndarray | None = None, moved_rank: np.ndarray | None = None):
        self.R, self.N = int(R), int(N)
        self.R_pad = -(-self.R // self.N) * self.N
        self.moved = np.zeros(0, np.int64) if moved is None else np.asarray(moved, np.int64)
        self.moved_rank = np.zeros(0, np.int64) if moved_rank is None else np.asarray(moved_rank, np.int64)
        eid = np.arange(self.R, dtype=np.int64)
        slot = np.zeros(self.N, np.int64)
        for r_, k in zip(self.moved, self.moved_rank):
            eid[r_] = self.R_pad + self.N * slot[k] + k
            slot[k] += 1
        self.eid = eid
        self.extra = int(slot.max()) if self.moved.size else 0

    @staticmethod
    def balanced(counts: np.ndarray, N: int, K: int = 4096) -> "Placement":
        """The top-K resources of ``counts`` (events per resource, the previous
        batch) spread over N ranks, LPT greedy against the others' load."""
        counts = np.asarray(counts, np.int64)
        R = counts.size
        if N <= 1:
            return Placement(R, N)
        K = min(K, R)
        top = np.argsort(-counts, kind="stable")[:K]
        rest = counts.copy()
        rest[top] = 0
        load = np.bincount(np.arange(R) % N, weights=rest, minlength=N).astype(np.float64)
        rank = np.empty(K, np.int64)
        for i, r_ in enumerate(top):
            k = int(np.argmin(load))
            rank[i] = k
            load[k] += counts[r_]
        return Placement(R, N, top, rank)

    def engine_id(self, res) -> np.ndarray:
        return self.eid[np.asarray(res, np.int64)]

    def owner(self, res) -> np.ndarray:
        return self.engine_id(res) % self.N

    def local_rows(self) -> int:
        """max_resources of each rank's engine (its rows e // N)."""
        return self.R_pad // self.N + self.extra

    def loads(self, counts) -> np.ndarray:
        """Events per rank for per-resource ``counts``."""
        return np.bincount(self.owner(np.arange(self.R)), weights=np.asarray(counts, np.float64),
                           minlength=self.N)
