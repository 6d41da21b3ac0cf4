"""Synthetic graph datasets (node classification) + per-client graph views for federated GNNs.

Shapes follow the datasets named by the reference configs (`conf/fed_gnn/*`, `conf/fed_aas/*`:
Coauthor_CS, Cora, PubMed, DBLP, Yelp, AmazonProducts, Reddit): node count, feature width,
class count and average degree. Graphs are stochastic-block-model-like
(edges mostly within a class), features are class-dependent sparse bag-of-words + noise.

Per-client views reproduce the reference's `GraphWorker` edge rules
(`worker/graph_worker.py:179-241,252-269`):
* training nodes are split among clients (node-split federated GNN);
* client k keeps in-client edges (both ends in T_k; Bernoulli-dropped with `edge_drop_rate`),
  cross-client edges (src in T_k, dst in another client's training set) and validation edges;
* with `share_feature`, layer 0 propagates over local edges only, layers ≥ 1 over all kept
  edges with other clients' boundary embeddings substituted (zeros where unavailable,
  `_get_cross_deivce_embedding`); without it every layer uses local edges only.
Propagation uses GCN normalisation D^-½(A+I)D^-½ of each client's edge set; the K clients'
edge sets are concatenated with a client offset so one gather/scatter covers the cohort.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch


def _coalesce(src: torch.Tensor, dst: torch.Tensor, n: int):
    key = torch.unique(src.long() * n + dst.long())
    return (key // n), (key % n)


@dataclass
class EdgeSet:
    """Concatenated normalised edges of K client graphs over N nodes (flat ids k*N+i)."""

    src: torch.Tensor  # int64 [E]
    dst: torch.Tensor  # int64 [E]
    val: torch.Tensor  # fp32 [E]
    K: int
    N: int

    def csr(self) -> "CSRPair":
        """CSR of Â (rows = dst, over K·N flat rows, or N when the graph is shared) and of Âᵀ
        (for the backward), built once per edge set for the native SpMM kernel."""
        cached = getattr(self, "_csr", None)
        if cached is None:
            rows = self.N * self.K
            cached = CSRPair(*_to_csr(self.dst, self.src, self.val, rows), *_to_csr(self.src, self.dst, self.val, rows))
            object.__setattr__(self, "_csr", cached)
        return cached


@dataclass
class CSRPair:
    rowptr: torch.Tensor
    col: torch.Tensor
    val: torch.Tensor
    rowptr_t: torch.Tensor
    col_t: torch.Tensor
    val_t: torch.Tensor


def _to_csr(row: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n_rows: int):
    order = torch.argsort(row, stable=True)
    counts = torch.bincount(row, minlength=n_rows)
    rowptr = torch.zeros(n_rows + 1, dtype=torch.int32, device=row.device)
    rowptr[1:] = counts.cumsum(0).to(torch.int32)
    return rowptr, col[order].to(torch.int32), val[order].float()


def gcn_norm(src: torch.Tensor, dst: torch.Tensor, n: int):
    """Self loops + symmetric normalisation (PyG `gcn_norm`); messages flow src -> dst."""
    loops = torch.arange(n, device=src.device)
    s = torch.cat([src, loops])
    d = torch.cat([dst, loops])
    deg = torch.zeros(n, device=src.device).index_add_(0, d, torch.ones_like(d, dtype=torch.float32))
    dinv = deg.clamp(min=1).rsqrt()
    return s, d, dinv[s] * dinv[d]


class GraphDataset:
    def __init__(self, spec, seed: int, device, dtype=torch.float32):
        self.spec = spec
        self.device = torch.device(device)
        self.dtype = dtype
        N, C, F = spec.num_nodes, spec.num_classes, spec.num_features
        g = torch.Generator().manual_seed(seed * 9973 + 5)
        self.num_nodes = N
        y = torch.randint(0, C, (N,), generator=g)
        E = max(N, N * max(spec.avg_degree, 2) // 2)
        E = min(E, 20_000_000)
        u = torch.randint(0, N, (E,), generator=g)
        # 80 % of edges stay within the source node's class
        by_class = [torch.nonzero(y == c).flatten() for c in range(C)]
        same = torch.rand(E, generator=g) < 0.8
        v = torch.randint(0, N, (E,), generator=g)
        for c in range(C):
            sel = same & (y[u] == c)
            cnt = int(sel.sum())
            if cnt and by_class[c].numel():
                v[sel] = by_class[c][torch.randint(0, by_class[c].numel(), (cnt,), generator=g)]
        keep = u != v
        u, v = u[keep], v[keep]
        src, dst = _coalesce(torch.cat([u, v]), torch.cat([v, u]), N)  # undirected
        self.src, self.dst = src, dst
        # features: class-specific active words + random words
        words = max(F // (4 * C), 1)
        proto = torch.zeros(C, F)
        for c in range(C):
            proto[c, torch.randint(0, F, (words,), generator=g)] = 1.0
        x = proto[y] * 1.0 + (torch.rand(N, F, generator=g) < (2.0 / max(F, 1))).float()
        x = x / x.sum(1, keepdim=True).clamp(min=1)
        self.x = x.to(self.device, dtype)
        self.labels_cpu = y.to(torch.int32)
        self.labels_dev = self.labels_cpu.to(self.device)
        perm = torch.randperm(N, generator=g)
        ntr, nva = int(0.6 * N), int(0.2 * N)
        self.train_nodes = perm[:ntr].sort().values
        self.val_nodes = perm[ntr : ntr + nva].sort().values
        self.test_nodes = perm[ntr + nva :].sort().values
        self.n = ntr
        # the "labels" used by the partitioners are those of the training nodes
        self.labels = self.labels_cpu[self.train_nodes]
        fs, fd, fv = gcn_norm(src, dst, N)
        self.full = EdgeSet(fs.to(self.device), fd.to(self.device), fv.to(self.device), 1, N)
        self.views: ClientGraphViews | None = None

    # partitioners work on positions inside train_nodes -> map to node ids
    def node_ids(self, positions: torch.Tensor) -> torch.Tensor:
        return self.train_nodes[positions.long()]

    def gather_labels(self, idx):
        return self.labels_dev.index_select(0, idx.reshape(-1).long()).reshape(idx.shape)

    def labels_for(self, idx):
        return self.gather_labels(idx)

    # ---- trainer hooks (input_kind == "graph")
    def batch(self, idx: torch.Tensor) -> "GraphBatch":
        v = self.views
        assert v is not None, "client graph views not built (GraphWorker._before_training)"
        return GraphBatch(self.x, v.l0, v.l1, idx, v, self.comm)

    comm = None

    @torch.no_grad()
    def evaluate(self, trainer, theta_rows: torch.Tensor, shard=(0, 1)):
        """Full-graph inference of M models; accuracy/loss over the rank's share of test nodes."""
        from ..engine.params import BoundParams
        from ..models.layers import RunCtx
        from ..ops import functional as Fn

        M = theta_rows.shape[0]
        rank, world = shard
        nodes = self.test_nodes.to(self.device)
        nodes = nodes[rank * nodes.numel() // world : (rank + 1) * nodes.numel() // world]
        compute = theta_rows.to(trainer.compute_dtype)
        params = BoundParams(trainer.layout, compute, None, K=M)
        ctx = RunCtx(params, None, training=False)
        seeds = nodes.unsqueeze(0).expand(M, -1)
        logits = trainer.model.forward(GraphBatch(self.x, self.full, self.full, seeds, None), ctx)
        labels = self.gather_labels(seeds)
        valid = torch.full((M,), seeds.shape[1], dtype=torch.int32, device=self.device)
        loss, correct = Fn.cross_entropy(logits.contiguous(), labels, valid)
        n_total = self.test_nodes.numel()
        return loss * seeds.shape[1], correct, n_total


class ClientGraphViews:
    """Edge sets of a cohort of clients (wave), built once per wave on device."""

    def __init__(self, ds: GraphDataset, owner: torch.Tensor, clients: list[int], share_feature: bool,
                 edge_drop_rate: float | None, seed: int):
        N = ds.num_nodes
        dev = ds.device
        self.ds = ds
        self.clients = clients
        self.K = len(clients)
        self.share_feature = share_feature
        src, dst = ds.src, ds.dst
        val_mask = torch.zeros(N, dtype=torch.bool)
        val_mask[ds.val_nodes] = True
        is_train = owner >= 0
        l0_s, l0_d, l1_s, l1_d = [], [], [], []
        self.stats = []
        keep_masks = []
        for i, c in enumerate(clients):
            own = owner == c
            in_client = own[src] & own[dst]
            orig_in = int(in_client.sum())
            if edge_drop_rate:
                g = torch.Generator().manual_seed(seed * 7919 + c)
                in_client &= torch.rand(in_client.shape, generator=g) >= edge_drop_rate
            cross = own[src] & is_train[dst] & ~own[dst]
            val_e = val_mask[src] & val_mask[dst]
            local = in_client | val_e
            full = local | cross
            self.stats.append({"original_in_client_training_edge_cnt": orig_in,
                               "in_client_training_edge_cnt": int(in_client.sum()),
                               "cross_client_training_edge_cnt": int(cross.sum()),
                               "training_node_cnt": int(own.sum()),
                               "validation_node_cnt": int(val_mask.sum())})
            # messages flow src -> dst; a client aggregates into its own nodes
            s0, d0, v0 = gcn_norm(dst[local], src[local], N)
            s1, d1, v1 = gcn_norm(dst[full], src[full], N)
            l0_s.append((s0, d0, v0))
            l1_s.append((s1, d1, v1))
            keep_masks.append(own)
        self.l0 = self._concat(l0_s, N, dev)
        self.l1 = self._concat(l1_s if share_feature else l0_s, N, dev)
        # halo substitution plan for layers >= 1 (reference `_get_cross_deivce_embedding`):
        # own training nodes keep their embedding; other clients' boundary nodes that this
        # client's kept edges touch get the owner's embedding; every other node gets zero.
        boundary = torch.zeros(N, dtype=torch.bool)
        cross_all = is_train[src] & is_train[dst] & (owner[src] != owner[dst])
        boundary[src[cross_all]] = True  # training nodes with an edge into another client
        self.boundary_nodes = torch.nonzero(boundary).flatten()
        self.owner = owner
        own_rows = torch.stack(keep_masks)  # [K, N]
        remote = torch.zeros((self.K, N), dtype=torch.bool)
        for i, c in enumerate(clients):
            own = owner == c
            cross = own[src] & is_train[dst] & ~own[dst]
            req = torch.zeros(N, dtype=torch.bool)
            req[dst[cross]] = True
            remote[i] = req & boundary
        self.keep = own_rows.to(dev)
        self.remote = remote.to(dev)
        self.boundary_nodes_dev = self.boundary_nodes.to(dev)
        pos = torch.full((N,), -1, dtype=torch.int64)
        for i, c in enumerate(clients):
            pos[owner == c] = i
        self.client_pos = pos.to(dev)
        self.boundary_cnt = [int((own_rows[i] & boundary).sum()) for i in range(self.K)]

    @staticmethod
    def _concat(parts, N, dev) -> EdgeSet:
        src = torch.cat([p[0] + i * N for i, p in enumerate(parts)])
        dst = torch.cat([p[1] + i * N for i, p in enumerate(parts)])
        val = torch.cat([p[2] for p in parts])
        return EdgeSet(src.to(dev), dst.to(dev), val.to(dev), len(parts), N)


def propagate(h: torch.Tensor, es: EdgeSet) -> torch.Tensor:
    """out[k, i] = Σ_j Â_k[i, j] h[k, j]  (h [K, N, F]); differentiable gather + index_add."""
    K, N, F = h.shape
    from ..ops import backend

    if backend.using_hip(h):  # native CSR SpMM (csrc/attention.hip: spmm_kernel)
        from ..ops import functional as Fn

        csr = es.csr()
        if es.K == 1:  # one graph shared by the K models
            return Fn.spmm(h, csr)
        return Fn.spmm(h.reshape(1, K * N, F), csr).view(K, N, F)
    if es.K == 1 and K > 1:  # one graph shared by K models (evaluation): fold K into features
        flat = h.permute(1, 0, 2).reshape(N, K * F)
        msg = flat.index_select(0, es.src) * es.val.to(h.dtype)[:, None]
        out = torch.zeros_like(flat).index_add_(0, es.dst, msg)
        return out.view(N, K, F).permute(1, 0, 2)
    flat = h.reshape(K * N, F)
    msg = flat.index_select(0, es.src) * es.val.to(h.dtype)[:, None]
    out = torch.zeros_like(flat).index_add_(0, es.dst, msg)
    return out.view(K, N, F)


def substitute_halo(h: torch.Tensor, views: "ClientGraphViews", comm=None) -> torch.Tensor:
    """Layer ≥ 1 input of client k: own training nodes keep h[k]; other clients' boundary
    nodes that k's cross edges reach get the OWNER's embedding (detached: the reference ships
    them through the server without gradient); every other node is zeroed.
    Across ranks the boundary rows are merged with one all-reduce (M6/M8 → collective)."""
    K, N, F = h.shape
    hd = h.detach()
    # boundary embeddings as computed by their owners (rows of the owning client)
    pos = views.client_pos  # [N] row of the owning client in this cohort (-1 if remote/none)
    bnd = views.boundary_nodes_dev
    table = torch.zeros((N, F), dtype=h.dtype, device=h.device)
    local_owned = pos[bnd] >= 0
    rows = bnd[local_owned]
    if rows.numel():
        table[rows] = hd[pos[rows].long(), rows]
    if comm is not None and comm.world > 1:
        comm.all_reduce_(table)
    keep = views.keep.unsqueeze(-1)
    remote = views.remote.unsqueeze(-1)
    return torch.where(keep, h, torch.where(remote, table.unsqueeze(0).expand(K, N, F), torch.zeros_like(h)))


@dataclass
class GraphBatch:
    x: torch.Tensor  # [N, F] shared node features
    l0: EdgeSet
    l1: EdgeSet
    seeds: torch.Tensor | None  # [K, B] node ids whose logits are returned (None = all)
    views: "ClientGraphViews | None" = None  # halo plan (None: no substitution)
    comm: object = None
