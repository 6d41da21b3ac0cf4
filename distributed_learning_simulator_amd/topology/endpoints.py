"""Endpoints: the worker↔server transport of the cohort runtime.

Reference: `ClientEndpoint.send/get/has_data/close`,
`ServerEndpoint.send/get/broadcast/worker_num/close` over pickled Pipes, plus the
quantising subclasses in `topology/quantized_endpoint.py:14-116`.

Here a "send" never leaves the device. The client endpoint converts a `CohortMessage` into
wire format *in place* (quantise → the receiver's dequantised view) and records the exact
wire bytes per client; the server endpoint's `get` finishes decoding; `broadcast` applies
downlink compression and charges bytes per receiving client. Byte counts follow the
reference's `get_message_size` rule on the wire payload.

Fixed reference defects: B2 — `get` passes `None` (skipped client) through
and decodes once; B3 — client-side quantisation applies to the *uploaded payload* whatever
its kind (Δ or θ), which is what FedPAQ's analysis charges (`analyze_log.py:263-272`).
"""

from __future__ import annotations

import torch

from ..message import CohortMessage
from ..ops import compress, fl
from ..utils.logging import get_logger


class _Ctx:
    def __init__(self, layout, device, seed: int):
        self.layout = layout
        self.device = device
        self.seed = seed
        self.seg_ids = layout.segment_ids(device)
        self.seg_sizes = layout.segment_sizes(device)
        self.meta = compress.LayoutMeta.of(layout, device)
        self.dense_bytes = layout.num_params * 4


class ClientEndpoint:
    def __init__(self, **kwargs):
        self.kwargs = kwargs
        self.ctx: _Ctx | None = None
        self.bytes_sent = 0
        self.messages_sent = 0
        self.dequant_server_data = False

    def bind(self, layout, device, seed: int) -> None:
        self.ctx = _Ctx(layout, device, seed)

    def _dense_wire(self, msg: CohortMessage) -> list[int]:
        if "wire_bytes" in msg.extra:  # sender-side sparse encodings (error feedback top-k)
            return list(msg.extra["wire_bytes"])
        if msg.block_mask is not None:
            sizes = msg.extra["block_param_sizes"]  # [nblocks] logical elements
            sel = (msg.block_mask.float() * sizes.float()[None, :]).sum(1)
            return [int(v) * 4 for v in sel.tolist()]
        return [self.ctx.dense_bytes] * msg.size

    def encode(self, msg: CohortMessage, seed: int) -> CohortMessage:
        msg.wire_bytes = self._dense_wire(msg)
        return msg

    def send(self, msg: CohortMessage, seed: int = 0) -> CohortMessage:
        msg = self.encode(msg, seed)
        self.bytes_sent += int(sum(msg.wire_bytes))
        self.messages_sent += msg.size
        return msg

    def receive_broadcast(self, params: torch.Tensor) -> torch.Tensor:
        return params

    def close(self) -> None:
        pass


class ServerEndpoint:
    def __init__(self, **kwargs):
        self.kwargs = kwargs
        self.ctx: _Ctx | None = None
        self.bytes_broadcast = 0
        self.quant_broadcast = False

    def bind(self, layout, device, seed: int) -> None:
        self.ctx = _Ctx(layout, device, seed)

    def get(self, msg: CohortMessage | None, defer_payload: bool = False) -> CohortMessage | None:
        """Receive: a packed payload is decoded here, unless the consumer dequantises it
        itself (`defer_payload`: FedAvg's fused accumulation)."""
        if msg is not None and msg.payload is not None and not defer_payload:
            msg.dense()
        return msg

    def encode_broadcast(self, params: torch.Tensor, seed: int) -> tuple[torch.Tensor, int]:
        return params, self.ctx.dense_bytes

    def broadcast(self, params: torch.Tensor, n_receivers: int, seed: int = 0) -> tuple[torch.Tensor, int]:
        """Returns (what receivers reconstruct, total bytes for n_receivers)."""
        received, per = self.encode_broadcast(params, seed)
        total = per * n_receivers
        self.bytes_broadcast += total
        return received, total

    def close(self) -> None:
        pass


# ------------------------------------------------------------------ quantised
def _attach(msg: CohortMessage, payload) -> CohortMessage:
    """The upload becomes the packed payload: the dense rows are no longer part of the message
    (kept only as the receiver's decode target)."""
    msg.payload = payload
    msg.extra["decode_into"] = msg.data
    msg.data = None
    msg.wire_bytes = payload.row_bytes()
    return msg


class QuantClientEndpoint(ClientEndpoint):
    """Quantise uploads into a wire payload; optionally dequantise server data."""

    def quantize(self, msg: CohortMessage, seed: int) -> CohortMessage:
        raise NotImplementedError

    def encode(self, msg, seed):
        return self.quantize(msg, seed)


class QuantServerEndpoint(ServerEndpoint):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.quant_broadcast = bool(kwargs.get("quant_broadcast", False))


class StochasticQuantClientEndpoint(QuantClientEndpoint):
    """FedPAQ / fed_obd_sq upload: 255-level stochastic quantisation into an 8-bit payload
    (reference `quantized_endpoint.py:74-77`)."""

    levels = 255

    def quantize(self, msg, seed):
        seeds = fl.row_seeds(seed, msg.client_ids)
        p = compress.pack_stochastic(msg.data, self.ctx.meta, seeds, msg.extra.get("segment_mask"), self.levels)
        return _attach(msg, p)


class StochasticQuantServerEndpoint(QuantServerEndpoint):
    levels = 255

    def encode_broadcast(self, params, seed):
        if not self.quant_broadcast:
            return params, self.ctx.dense_bytes
        p = compress.pack_stochastic(params.unsqueeze(0), self.ctx.meta, fl.row_seeds(seed, [-1]), None, self.levels)
        return p.decode()[0], p.row_bytes()[0]


class NNADQClientEndpoint(QuantClientEndpoint):
    """FedOBD upload quantiser (reference `quantized_endpoint.py:86-101`); logs the
    compression ratio with the phrase the reference's analyser parses
    ("worker NNABQ compression ratio", `analyze_log.py:131-134`)."""

    def __init__(self, weight: float | None = None, **kwargs):
        super().__init__(**kwargs)
        self.weight = weight

    def quantize(self, msg, seed):
        if self.weight is None:
            return super().quantize(msg, seed)
        dense = self._dense_wire(msg)
        p = compress.pack_nnadq(msg.data, self.ctx.meta, self.weight, msg.extra.get("segment_mask"))
        msg = _attach(msg, p)
        for cid, w, d in zip(msg.client_ids, msg.wire_bytes, dense):
            get_logger().debug("worker %d NNABQ compression ratio is %s", cid, w / max(d, 1))
        msg.extra["compression_ratio"] = [w / max(d, 1) for w, d in zip(msg.wire_bytes, dense)]
        return msg


class NNADQServerEndpoint(QuantServerEndpoint):
    def __init__(self, weight: float | None = None, **kwargs):
        super().__init__(**kwargs)
        self.weight = weight

    def encode_broadcast(self, params, seed):
        if not self.quant_broadcast or self.weight is None:
            return params, self.ctx.dense_bytes
        p = compress.pack_nnadq(params.unsqueeze(0), self.ctx.meta, self.weight)
        wire = p.row_bytes()[0]
        get_logger().info("broadcast NNABQ compression ratio is %s", wire / self.ctx.dense_bytes)
        return p.decode()[0], wire
