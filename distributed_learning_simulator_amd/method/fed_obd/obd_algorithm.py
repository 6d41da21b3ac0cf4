"""Opportunistic Block Dropout (FedOBD, arXiv 2208.05174) — block discovery + selection.

Reference `method/fed_obd/obd_algorithm.py`:
* blocks = module groups matching {AlbertTransformer, AlbertEmbeddings, Bottleneck,
  TransformerEncoderLayer} or the sibling sequences (BN, ReLU, Conv), (BN, Conv), (Conv, BN),
  plus every top-most parameterised submodule not overlapping a block; the blocks must cover
  exactly all parameters (`:8-86`);
* per client: score_b = ‖θ_b − θ_g,b‖₂ / |b|; visit score groups in descending order, add a
  block iff the running total stays ≤ (1 − dropout_rate)·P (`:88-127`).

Cohort form: per-(client, block) Σ Δ² for all K clients in ONE segmented-reduction launch
(`block_sq_norms` kernel), the O(#blocks) greedy selection on the host, then the unselected
blocks are zeroed in the upload rows with one masked multiply.
"""

from __future__ import annotations

import torch

from ...engine.params import ParamLayout
from ...ops import fl
from ...utils.logging import get_logger

CONTAINER_BLOCKS = {"AlbertTransformer", "AlbertEmbeddings", "Bottleneck", "TransformerEncoderLayer"}
SEQ_PATTERNS = [("BatchNorm2d", "ReLU", "Conv2d"), ("BatchNorm2d", "Conv2d"), ("Conv2d", "BatchNorm2d")]


def get_module_blocks(root) -> list[list]:
    blocks: list[list] = []

    def visit(m):
        if m.kind in CONTAINER_BLOCKS:
            blocks.append([m])
            return
        ch = m.children
        i = 0
        while i < len(ch):
            for pat in SEQ_PATTERNS:
                n = len(pat)
                if i + n <= len(ch) and all(ch[i + j].kind == pat[j] for j in range(n)):
                    blocks.append(ch[i : i + n])
                    i += n
                    break
            else:
                visit(ch[i])
                i += 1

    visit(root)
    return blocks


def _overlap(a: str, b: str) -> bool:
    return a == b or a.startswith(b + ".") or b.startswith(a + ".")


class BlockStructure:
    """Block → parameter names / element ids over the flat layout."""

    def __init__(self, model, layout: ParamLayout, device):
        blocks = get_module_blocks(model.root)
        names_in_blocks = [[m.name for m in b] for b in blocks]
        for m in list(model.root.modules())[1:]:
            if not m.all_params():
                continue
            if any(_overlap(m.name, bn) for blk in names_in_blocks for bn in blk):
                continue
            blocks.append([m])
            names_in_blocks.append([m.name])
        self.block_names = names_in_blocks
        index = layout.index()
        self.block_params: list[list[str]] = [[p for m in b for p in m.all_params()] for b in blocks]
        covered = [p for ps in self.block_params for p in ps]
        if sorted(covered) != sorted(index.keys()):
            missing = set(index) - set(covered)
            extra = set(covered) - set(index)
            raise RuntimeError(f"block coverage mismatch: missing {missing} extra {extra}")
        ids = torch.full((layout.padded_size,), -1, dtype=torch.int32)
        seg_block = torch.zeros(len(layout.entries), dtype=torch.long)
        seg_pos = {e.name: i for i, e in enumerate(layout.entries)}
        sizes = []
        for bi, ps in enumerate(self.block_params):
            n = 0
            for p in ps:
                e = index[p]
                ids[e.offset : e.offset + e.numel] = bi
                seg_block[seg_pos[p]] = bi
                n += e.numel
            sizes.append(n)
        self.num_blocks = len(self.block_params)
        self.block_ids = ids.to(device)
        self.block_sizes = torch.tensor(sizes, dtype=torch.int64)
        self.block_sizes_dev = self.block_sizes.to(device)
        self.offsets = torch.zeros(self.num_blocks + 1, dtype=torch.int64)
        self.segment_block = seg_block.to(device)  # tensor index -> block index
        self.num_params = layout.num_params


class OpportunisticBlockDropoutAlgorithm:
    def __init__(self, dropout_rate: float):
        self.dropout_rate = dropout_rate
        self.structure: BlockStructure | None = None

    def ensure_blocks(self, model, layout, device, log: bool = False) -> BlockStructure:
        if self.structure is None:
            self.structure = BlockStructure(model, layout, device)
            if log:
                get_logger().info("identify %d blocks in model", self.structure.num_blocks)
                for b in self.structure.block_names:
                    get_logger().debug("block %s", b)
        return self.structure

    def select_blocks(self, delta_rows: torch.Tensor) -> torch.Tensor:
        """delta_rows [K, P] -> bool block mask [K, nblocks] (same greedy as the reference)."""
        st = self.structure
        sq = fl.block_sq_norms(delta_rows, st.offsets, st.block_ids)
        mean = (sq.sqrt() / st.block_sizes_dev.float()).cpu()
        threshold = (1 - self.dropout_rate) * st.num_params
        sizes = st.block_sizes.tolist()
        K, nb = mean.shape
        mask = torch.zeros((K, nb), dtype=torch.bool)
        for k in range(K):
            groups: dict[float, list[int]] = {}
            for b, v in enumerate(mean[k].tolist()):
                groups.setdefault(v, []).append(b)
            partial = 0
            for v in sorted(groups.keys(), reverse=True):
                if partial > threshold:
                    break
                for b in groups[v]:
                    if partial + sizes[b] > threshold:
                        continue
                    partial += sizes[b]
                    mask[k, b] = True
        return mask.to(delta_rows.device)
