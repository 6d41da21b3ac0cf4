"""FedOBD / FedOBD-SQ — reference `method/fed_obd/{__init__,worker,server,phase}.py`.

Two-phase protocol:
* stage 1 (rounds 1..`round`, `random_client_number` clients): upload only the
  opportunistically selected blocks of Δ (fixed B4: Δ of the selected blocks, averaged per
  block over the clients that sent it), NNADQ- (fed_obd) or stochastically (fed_obd_sq)
  quantised; the server broadcasts the quantised global model (`quant_broadcast`);
* after round `round` (or an early-stop plateau) the server flags `phase_two`;
* stage 2 (all clients, `second_phase_epoch` epochs): aggregation after EVERY local epoch
  (in-round, `check_acc` ⇒ evaluate), the last epoch sets `end_training` ⇒ server ends.
Stage 2 runs as `second_phase_epoch` one-epoch mini-rounds over the cohort (the optimizer
state is cleared at every load, as `util/model.py:9-20` does for reuse_learning_rate) with a
cosine schedule over the stage-2 epochs.
"""

from __future__ import annotations

from enum import Enum, auto

import torch

from ...algorithm.fed_avg_algorithm import FedAVGAlgorithm
from ...message import CohortMessage
from ...server.aggregation_server import AggregationServer
from ...topology.endpoints import (NNADQClientEndpoint, NNADQServerEndpoint, StochasticQuantClientEndpoint,
                                   StochasticQuantServerEndpoint)
from ...utils.logging import get_logger
from ...worker.aggregation_worker import AggregationWorker
from ..algorithm_factory import CentralizedAlgorithmFactory
from .obd_algorithm import OpportunisticBlockDropoutAlgorithm


class Phase(Enum):
    STAGE_ONE = auto()
    STAGE_TWO = auto()
    END = auto()


class FedOBDWorker(AggregationWorker):
    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        self.obd = OpportunisticBlockDropoutAlgorithm(float(config.algorithm_kwargs["dropout_rate"]))
        self.phase = Phase.STAGE_ONE
        self.endpoint.dequant_server_data = True
        self._stage2_epoch = 0
        self._second_phase_epoch = int(config.algorithm_kwargs.get("second_phase_epoch", 1))

    def local_epochs(self) -> int:
        return 1 if self.phase == Phase.STAGE_TWO else self._epochs

    def state_dict(self) -> dict:
        return {"phase": self.phase.value, "stage2_epoch": self._stage2_epoch}

    def load_state_dict(self, state: dict) -> None:
        self.phase = Phase(state.get("phase", Phase.STAGE_ONE.value))
        self._stage2_epoch = int(state.get("stage2_epoch", 0))
        if self.phase == Phase.STAGE_TWO:
            self.disable_choose_model_by_validation()

    def run_round(self, round_num, theta_g, client_ids):
        last = getattr(self.session.server, "last_result", None)
        if self.phase == Phase.STAGE_ONE and last is not None and last.other_data.get("phase_two"):
            get_logger().warning("switch to phase 2")
            self.phase = Phase.STAGE_TWO
            self.disable_choose_model_by_validation()  # reference fed_obd/worker.py:35
        if self.phase == Phase.STAGE_TWO:
            self._stage2_epoch += 1
        yield from super().run_round(round_num, theta_g, client_ids)

    def build_schedule(self, round_num, wave):
        if self.phase != Phase.STAGE_TWO:
            return super().build_schedule(round_num, wave)
        return self.trainer.build_schedule(
            self.shards(wave), 1, seed=self.config.seed * 100_003 + round_num * 1009 + self._stage2_epoch * 31, client_ids=list(wave),
            epoch_offset=self._stage2_epoch - 1, total_epochs=self._second_phase_epoch)

    def _get_sent_data(self, wave, theta_g, stats) -> CohortMessage:
        msg = super()._get_sent_data(wave, theta_g, stats)  # Δ rows
        st = self.obd.ensure_blocks(self.session.model, self.session.layout, msg.data.device,
                                    log=self.session.is_main)
        if self.phase == Phase.STAGE_ONE:
            bmask = self.obd.select_blocks(msg.data)
            msg.data.mul_(bmask[:, st.block_ids.clamp(min=0).long()] & (st.block_ids >= 0)[None, :])
            msg.block_mask = bmask
            msg.extra["block_ids"] = st.block_ids
            msg.extra["block_param_sizes"] = st.block_sizes_dev
            msg.extra["segment_mask"] = bmask[:, st.segment_block]
            return msg
        msg.in_round = True
        msg.other_data["check_acc"] = True
        if self._stage2_epoch >= self._second_phase_epoch:
            msg.end_training = True
        return msg


class FedOBDServer(AggregationServer):
    def __init__(self, config, endpoint, algorithm=None, session=None, **kwargs):
        super().__init__(config, endpoint, algorithm=algorithm or FedAVGAlgorithm(), session=session, **kwargs)
        self.phase = Phase.STAGE_ONE
        self.endpoint.quant_broadcast = True
        self.last_result = None
        # a plateau switches FedOBD to stage 2 instead of ending training
        self._obd_early_stop, self.early_stop = self.early_stop, False

    def state_dict(self) -> dict:
        return {**super().state_dict(), "phase": self.phase.value}

    def load_state_dict(self, state: dict) -> None:
        super().load_state_dict(state)
        self.phase = Phase(state.get("phase", Phase.STAGE_ONE.value))
        if self.phase != Phase.STAGE_ONE:
            self._algorithm.num_blocks = 0

    def _select_workers(self):
        if self.phase != Phase.STAGE_ONE:
            return list(range(self.worker_number))
        return super()._select_workers()

    def _get_stat_key(self):
        if not self.performance_stat:
            return super()._get_stat_key()
        return max(self.performance_stat.keys()) + 1

    def _before_start(self):
        msg = super()._before_start()
        # ranks hosting no client must still join the per-block collectives
        obd = OpportunisticBlockDropoutAlgorithm(float(self.config.algorithm_kwargs["dropout_rate"]))
        st = obd.ensure_blocks(self.session.model, self.session.layout, self.session.device)
        self._algorithm.num_blocks = st.num_blocks
        self._algorithm.block_ids = st.block_ids
        return msg

    def _aggregate_worker_data(self):
        result = super()._aggregate_worker_data()
        self._compute_stat = self.phase == Phase.STAGE_ONE or "check_acc" in result.other_data
        if result.end_training:
            self.phase = Phase.END
        if self.phase == Phase.STAGE_ONE:
            if self.round_number >= self.config.round or (self._obd_early_stop and self._convergent()):
                get_logger().warning("switch to phase 2")
                self.phase = Phase.STAGE_TWO
                self._algorithm.num_blocks = 0  # full-model Δ uploads from now on
                result.other_data["phase_two"] = True
                result.in_round = False
        elif self.phase == Phase.STAGE_TWO:
            result.in_round = True
        return result

    def _stopped(self) -> bool:
        return self.phase == Phase.END


def _register():
    CentralizedAlgorithmFactory.register_algorithm(
        algorithm_name="fed_obd",
        client_cls=FedOBDWorker,
        server_cls=FedOBDServer,
        client_endpoint_cls=NNADQClientEndpoint,
        server_endpoint_cls=NNADQServerEndpoint,
    )
    CentralizedAlgorithmFactory.register_algorithm(
        algorithm_name="fed_obd_sq",
        client_cls=FedOBDWorker,
        server_cls=FedOBDServer,
        client_endpoint_cls=StochasticQuantClientEndpoint,
        server_endpoint_cls=StochasticQuantServerEndpoint,
    )


_register()
