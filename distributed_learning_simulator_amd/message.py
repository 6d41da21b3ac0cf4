"""FL protocol payloads and the byte-accounting rule.

Single-client dataclasses keep the reference's API (`message.py:10-49`):
`Message`, `ParameterMessageBase`, `ParameterMessage` (+`complete`),
`ParameterFileMessage`, `DeltaParameterMessage` (+`restore`). `get_message_size` is the
reference's accounting rule (`message.py:52-62`): sum of element_size*numel over every
tensor reachable from the message.

`CohortMessage` is the MI355X-native form: one object carries the uploads of all K clients
resident on a rank as a flat device tensor `[K, P]` (no pickling, no host copy). Its
`wire_bytes` list holds, per client, what `get_message_size` would report for that client's
single-client message *in wire format* (quantised / packed payloads), so the comm
bytes/round metric follows the reference's rule exactly.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field, fields
from typing import Any

import torch

TensorDict = dict[str, torch.Tensor]


@dataclass(kw_only=True)
class Message:
    other_data: dict = field(default_factory=dict)
    in_round: bool = False
    end_training: bool = False


@dataclass(kw_only=True)
class ParameterMessageBase(Message):
    dataset_size: int = 0


@dataclass(kw_only=True)
class ParameterMessage(ParameterMessageBase):
    parameter: TensorDict

    def complete(self, other_parameter: TensorDict) -> None:
        for k, v in other_parameter.items():
            if k not in self.parameter:
                self.parameter[k] = v


@dataclass(kw_only=True)
class ParameterFileMessage(ParameterMessageBase):
    path: str


@dataclass(kw_only=True)
class DeltaParameterMessage(ParameterMessageBase):
    delta_parameter: TensorDict

    def restore(self, parameter: TensorDict) -> ParameterMessage:
        new_parameter = {k: v.clone() for k, v in parameter.items()}
        for k, v in self.delta_parameter.items():
            new_parameter[k] = new_parameter[k] + v.to(new_parameter[k].device)
        msg = ParameterMessage(parameter=new_parameter)
        for f in fields(self):
            if f.name != "delta_parameter":
                setattr(msg, f.name, getattr(self, f.name))
        msg.parameter = new_parameter
        return msg


def _count_tensors(obj: Any) -> int:
    if isinstance(obj, torch.Tensor):
        return obj.element_size() * obj.numel()
    if isinstance(obj, dict):
        return sum(_count_tensors(v) for v in obj.values())
    if isinstance(obj, (list, tuple, set)):
        return sum(_count_tensors(v) for v in obj)
    if hasattr(obj, "__dataclass_fields__"):
        return sum(_count_tensors(getattr(obj, f.name)) for f in fields(obj))
    return 0


def get_message_size(msg: Any) -> int:
    """Reference rule (`message.py:52-62`): Σ element_size·numel of all tensors."""
    if isinstance(msg, CohortMessage):
        return int(sum(msg.wire_bytes))
    cnt = _count_tensors(msg)
    assert cnt > 0
    return cnt


@dataclass(kw_only=True)
class FlatParameterMessage(ParameterMessageBase):
    """Server result / broadcast: the global model as one flat device tensor [P_pad]."""

    parameter: torch.Tensor
    layout: Any = None

    def parameter_dict(self) -> TensorDict:
        return self.layout.unflatten(self.parameter)


@dataclass(kw_only=True)
class CohortMessage(Message):
    """Uploads of K co-resident clients.

    kind: "parameter" (data = θ_k), "delta" (data = θ_k − θ_g), "gradient" (per-step).
    data: dense decoded payload [K, P] on device (what the server-side algorithm consumes).
    mask: optional [K, P] element mask (FedDropoutAvg) or None.
    block_mask: optional [K, n_blocks] bool (FedOBD selected blocks) or None.
    """

    client_ids: list[int]
    dataset_sizes: torch.Tensor  # [K] float64/float32 on device
    kind: str = "delta"
    data: torch.Tensor | None = None
    mask: torch.Tensor | None = None
    block_mask: torch.Tensor | None = None
    wire_bytes: list[int] = field(default_factory=list)
    layout: Any = None  # engine.params.ParamLayout
    extra: dict = field(default_factory=dict)
    # quantised uploads travel as a packed wire buffer (ops/compress.QuantPayload): `data` is
    # None until the receiver decodes it (`dense()`), or never when the server's accumulation
    # dequantises the payload directly
    payload: Any = None

    @property
    def size(self) -> int:
        return len(self.client_ids)

    def dense(self) -> torch.Tensor:
        """Decoded [K, P] rows (decodes a pending payload in place, once)."""
        if self.data is None and self.payload is not None:
            self.data = self.payload.decode(out=self.extra.pop("decode_into", None))
            self.payload = None
        return self.data

    def client_message(self, i: int) -> ParameterMessageBase:
        """Materialise client i as a reference-style single-client message (API parity,
        tests, analysis). Not used on the hot path."""
        assert self.layout is not None and self.data is not None
        tensors = self.layout.unflatten(self.data[i])
        n = int(self.dataset_sizes[i].item())
        common = dict(
            dataset_size=n,
            other_data=copy.deepcopy(self.other_data),
            in_round=self.in_round,
            end_training=self.end_training,
        )
        if self.kind == "delta":
            return DeltaParameterMessage(delta_parameter=tensors, **common)
        return ParameterMessage(parameter=tensors, **common)
