"""sign-SGD with majority vote [Bernstein et al. 2018] — the reference ships only configs
(`conf/sign_sgd/*.yaml`, `distributed_algorithm: sign_SGD`) and the per-step gradient
exchange substrate `worker/gradient_worker.py:29-131` (flatten grads → send → receive
aggregated gradient → momentum/dampening/nesterov SGD). No server was registered; this is
the intended method.

Per optimizer step, for every client k (all clients hold the same model: identical seeded
init, identical updates):
  g_k = ∇_k + wd·θ                       (`gradient_worker.py:13-26`)
  bits_k = 1[g_k ≥ 0]                    (1-bit pack kernel, P/8 bytes on the wire)
  votes = Σ_k (2·bits_k − 1)             (vote kernel + ONE int32 all-reduce over ranks)
  θ ← SGD(θ, sign(votes))                (fused SGD kernel on the single shared row)
Clients are processed in waves inside a step when they do not fit at once (votes
accumulate; the model is fixed during the step). Wire accounting per step: every active
client uploads ceil(P/8) bytes and receives the ceil(P/8)-byte majority.
"""

from __future__ import annotations

import json
import os
import time

import torch

from ...engine.trainer import TrainStats
from ...message import FlatParameterMessage
from ...ops import fl, quant
from ...server.aggregation_server import AggregationServer
from ...utils.logging import get_logger
from ...worker.aggregation_worker import AggregationWorker
from ..algorithm_factory import CentralizedAlgorithmFactory


class SignSGDWorker(AggregationWorker):
    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        self.epoch_stat: dict = {}

    def train_round_sync(self, round_num: int, theta_g: torch.Tensor, clients: list[int], on_epoch=None):
        """All clients of the job train one round of `epoch` epochs with a majority-vote
        exchange after every step. Returns (final θ, bytes up, bytes down)."""
        tr = self.trainer
        sess = self.session
        comm = sess.comm
        P = tr.layout.padded_size
        nbytes = (tr.layout.num_params + 7) // 8
        b = tr.buffers
        tr.load_global(theta_g, 1)
        tr.reset_optimizer(1)
        local = sess.local_clients(clients)
        cap = tr.capacity
        # every rank must run the same number of steps: schedule over the GLOBAL max shard
        all_sizes = [sess.practitioners[c].dataset_size(sess.dc.spec.name) for c in clients]
        B = tr.hyper.batch_size
        steps_per_epoch = max(1, max((n + B - 1) // B for n in all_sizes))
        shards = self.shards(local) if local else []
        sched = tr.build_schedule(shards, self.local_epochs(), seed=self.config.seed * 100_003 + round_num,
                                  min_steps_per_epoch=steps_per_epoch, client_ids=local) if local else None
        epochs = self.local_epochs()
        S = steps_per_epoch * epochs
        stats = TrainStats(epochs, max(len(local), 1), tr.device)
        up = down = 0
        wd = tr.hyper.weight_decay
        theta0 = b.theta[:1]
        step_in_epoch = 0
        e = 0
        for s in range(S):
            votes = torch.zeros(P, dtype=torch.int32, device=tr.device)
            n_active = 0
            if sched is not None and s < sched.steps:
                # schedule for local clients may have fewer steps than the global max
                for w0 in range(0, len(local), cap):
                    w1 = min(len(local), w0 + cap)
                    K = w1 - w0
                    idx = sched.idx[s, w0:w1]
                    valid = sched.counts[s, w0:w1]
                    x = tr._gather(sess.dc.train, idx)
                    y = sess.dc.train.gather_labels(idx)
                    loss, correct = tr.forward_loss(K, x, y, valid, shared=True)
                    loss.sum().backward()
                    with torch.no_grad():
                        g = b.grad[:K]
                        if wd:
                            g.add_(theta0, alpha=wd)
                        active = sched.active[s, w0:w1]
                        votes += quant.sign_vote(quant.sign_pack(g), P, active)
                        vf = valid.float()
                        ee = min(e, epochs - 1)
                        stats.loss_sum[ee, w0:w1] += loss.detach() * vf
                        stats.correct[ee, w0:w1] += correct
                        stats.samples[ee, w0:w1] += vf
                        n_active += int(active.sum().item()) if comm.world == 1 else 0
            comm.all_reduce_(votes)
            with torch.no_grad():
                majority = torch.sign(votes.float()).unsqueeze(0)
                lr = torch.full((1,), tr.hyper.lr_at_epoch(e, epochs), device=tr.device)
                one = torch.ones(1, dtype=torch.bool, device=tr.device)
                first = torch.tensor([s == 0], device=tr.device)
                fl.sgd_step(theta0, majority, b.state1[:1], lr, one, first, 0.0, tr.hyper.momentum,
                            tr.hyper.dampening, tr.hyper.nesterov, b.shadow[:1] if b.shadow is not None else None)
            n_clients_step = len(clients)  # every client uploads its 1-bit sign each step
            up += n_clients_step * nbytes
            down += n_clients_step * nbytes
            step_in_epoch += 1
            if step_in_epoch == steps_per_epoch:
                step_in_epoch = 0
                if on_epoch is not None:
                    on_epoch(e, stats)
                e += 1
        self.last_stats = stats
        return b.theta[0].clone(), up, down


class SignSGDServer(AggregationServer):
    """Drives the synchronous rounds (the per-step exchange lives in the worker)."""

    def run_rounds(self, session, theta_recv):
        worker = session.worker
        while not self._stopped():
            r = self.round_number
            t0 = time.perf_counter()
            selected = list(self.selected)

            def on_epoch(e, stats):
                loss, acc = stats.epoch_metrics(e)
                worker.epoch_stat[e + 1] = {"loss": float(loss.mean()), "accuracy": float(acc.mean())}

            theta, up, down = worker.train_round_sync(r, theta_recv, selected, on_epoch)
            result = FlatParameterMessage(parameter=theta, layout=session.layout)
            theta_recv, _ = self.send_result(result)
            session.record_round(r, t0, selected, up, down)
        if session.is_main:
            os.makedirs(worker.save_dir, exist_ok=True)
            with open(os.path.join(worker.save_dir, "epoch_stat.json"), "wt", encoding="utf8") as f:
                json.dump(worker.epoch_stat, f)


CentralizedAlgorithmFactory.register_algorithm(
    algorithm_name="sign_SGD", client_cls=SignSGDWorker, server_cls=SignSGDServer)
