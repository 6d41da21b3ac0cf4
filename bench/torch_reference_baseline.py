"""Reference-equivalent baseline on the same GPU: the reference's execution model in plain PyTorch.

The reference (`simulation_lib/training.py:105-125`, `worker/aggregation_worker.py`,
`algorithm/fed_avg_algorithm.py:39-52`) trains its clients one at a time inside a process per
GPU: each client loads the global state dict into a torch.nn model, builds a fresh SGD
optimizer, runs its local epochs in eager fp32 (`conf/global.yaml` use_amp: false) and hands its
parameters to the server, which averages them in fp64. The reference itself cannot run here
(its engine, `cyy_torch_toolbox`, is not installed and there is no network), so this script
re-creates exactly that loop with stock PyTorch-ROCm (MIOpen convs, rocBLAS/hipBLASLt GEMMs) to
give the headline config (BASELINE.json config 2: FedAvg, 100 clients, ResNet-18 CIFAR stem,
5 local epochs, batch 64, SGD lr 0.1 momentum 0.9, cosine) a measured reference-style number.

`--clients-timed C` trains C of the round's clients and scales the time to the whole round
(clients are identical in size, so the per-client time is constant). Output: one JSON line.

    python bench/torch_reference_baseline.py --clients-timed 8 --warmup-clients 1
"""

from __future__ import annotations

import argparse
import json
import sys
import threading
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + self.shortcut(x))


class ResNet18(nn.Module):
    """CIFAR-stem ResNet-18 (11,173,962 parameters, the same count models/zoo.py pins)."""

    def __init__(self, classes: int = 10) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        layers, cin = [], 64
        for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
            layers += [BasicBlock(cin, cout, stride), BasicBlock(cout, cout, 1)]
            cin = cout
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(512, classes)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = self.layers(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


class DenseNet40(nn.Module):
    """DenseNet-40 (growth 12, stem 24, BN-ReLU-Conv layers, 1x1 transitions + 2x2 average
    pool; 1,059,298 parameters as models/zoo.py pins), written the usual torch.cat way."""

    def __init__(self, classes: int = 10, growth: int = 12) -> None:
        super().__init__()
        c = 2 * growth
        self.conv1 = nn.Conv2d(3, c, 3, 1, 1, bias=False)
        self.blocks = nn.ModuleList()
        self.trans = nn.ModuleList()
        for b in range(3):
            layers = nn.ModuleList()
            for _ in range(12):
                layers.append(nn.ModuleDict({"bn": nn.BatchNorm2d(c), "conv": nn.Conv2d(c, growth, 3, 1, 1, bias=False)}))
                c += growth
            self.blocks.append(layers)
            if b < 2:
                self.trans.append(nn.ModuleDict({"bn": nn.BatchNorm2d(c), "conv": nn.Conv2d(c, c, 1, bias=False)}))
        self.bn = nn.BatchNorm2d(c)
        self.fc = nn.Linear(c, classes)

    def forward(self, x):
        x = self.conv1(x)
        for b, layers in enumerate(self.blocks):
            for lay in layers:
                x = torch.cat([x, lay["conv"](F.relu(lay["bn"](x)))], 1)
            if b < 2:
                t = self.trans[b]
                x = F.avg_pool2d(t["conv"](F.relu(t["bn"](x))), 2)
        x = F.relu(self.bn(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


class Bottleneck(nn.Module):
    def __init__(self, cin: int, width: int, stride: int) -> None:
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return F.relu(out + (x if self.down is None else self.down(x)))


class ResNet50(nn.Module):
    """ImageNet ResNet-50 (25,557,032 parameters, as models/zoo.py pins)."""

    def __init__(self, classes: int = 1000) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        blocks, cin = [], 64
        for width, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            for i in range(n):
                blocks.append(Bottleneck(cin, width, stride if i == 0 else 1))
                cin = width * 4
        self.layers = nn.Sequential(*blocks)
        self.fc = nn.Linear(2048, classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.layers(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def signsgd_step_time(args, dev):
    """sign-SGD (BASELINE config 4) in the reference's style: every step each of the 128 clients
    computes its gradient on its next batch of 128 images in turn (sequential eager fp32), the
    signs are summed into a majority vote and the shared model takes one step. Times
    `--clients-timed` client gradients of one step, scaled to 128 clients x 8 steps per round."""
    model = ResNet50().to(dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    images = torch.randn(args.batch, 3, 224, 224, generator=g).to(dev)
    labels = torch.randint(0, 1000, (args.batch,), generator=g).to(dev)
    params = [p for p in model.parameters()]
    vote = [torch.zeros_like(p) for p in params]

    def client_grad():
        model.zero_grad(set_to_none=True)
        F.cross_entropy(model(images), labels).backward()
        for v, p in zip(vote, params):
            v.add_(torch.sign(p.grad))

    for _ in range(args.warmup_clients):
        client_grad()
        print("[baseline] warmup client done", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(args.clients_timed):
        client_grad()
        print(f"[baseline] client {c + 1}/{args.clients_timed} {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.clients_timed
    with torch.no_grad():
        for v, p in zip(vote, params):
            p.add_(torch.sign(v), alpha=-0.001)
    return dt, sum(p.numel() for p in params)


class TransformerClassifier(nn.Module):
    """Transformer-base text classifier as models/zoo.py TransformerClassificationModel: token
    embedding x sqrt(d) + sinusoidal PE, 6 post-norm nn.TransformerEncoderLayer (d 512, 8 heads,
    FFN 2048, ReLU, dropout 0.1), masked mean over the sequence, linear head (AG-News: 4 classes)."""

    def __init__(self, vocab=30000, d=512, heads=8, layers=6, ffn=2048, classes=4, max_len=128) -> None:
        super().__init__()
        self.d = d
        self.emb = nn.Embedding(vocab, d, padding_idx=0)
        pos = torch.arange(max_len).unsqueeze(1)
        div = torch.exp(torch.arange(0, d, 2) * (-torch.log(torch.tensor(10000.0)) / d))
        pe = torch.zeros(max_len, d)
        pe[:, 0::2] = torch.sin(pos * div)
        pe[:, 1::2] = torch.cos(pos * div)
        self.register_buffer("pe", pe)
        layer = nn.TransformerEncoderLayer(d, heads, ffn, dropout=0.1, batch_first=True)
        self.encoder = nn.TransformerEncoder(layer, layers, enable_nested_tensor=False)
        self.fc = nn.Linear(d, classes)

    def forward(self, tokens):
        pad = tokens == 0
        x = self.emb(tokens) * self.d ** 0.5 + self.pe[: tokens.shape[1]]
        x = self.encoder(x, src_key_padding_mask=pad)
        keep = (~pad).unsqueeze(-1).float()
        return self.fc((x * keep).sum(1) / keep.sum(1).clamp(min=1))


def train_client(model, global_state, images, labels, args):
    model.load_state_dict(global_state)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr if args.lr else (0.01 if args.model == "transformer" else 0.1),
                          momentum=0.9)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=args.epoch)
    n = images.shape[0]
    for _ in range(args.epoch):
        perm = torch.randperm(n, device=images.device)
        for s in range(0, n, args.batch):
            idx = perm[s:s + args.batch]
            loss = F.cross_entropy(model(images[idx]), labels[idx])
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
        sched.step()
    return {k: v.detach().clone() for k, v in model.state_dict().items()}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--clients-timed", type=int, default=8)
    ap.add_argument("--warmup-clients", type=int, default=1)
    ap.add_argument("--epoch", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.0, help="0: the config's (0.1 CNNs, 0.01 FedOBD Transformer)")
    ap.add_argument("--train-size", type=int, default=50000)
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--model", default="ResNet18", choices=["ResNet18", "densenet40", "transformer", "resnet50"])
    ap.add_argument("--no-benchmark", action="store_true", help="torch.backends.cudnn.benchmark off")
    args = ap.parse_args()

    # MIOpen auto-tuning per shape: on for ResNet-18 (11 conv shapes); DenseNet-40 has ~80 distinct
    # conv shapes (every layer a new input width, plus the ragged last batch) and its exhaustive
    # search alone ran > 8 minutes, so it runs with PyTorch's default (off)
    # (ResNet-50 at batch 128 x 224²: the search had not finished its first client in 10 minutes)
    torch.backends.cudnn.benchmark = args.model == "ResNet18" and not args.no_benchmark
    t_start = time.perf_counter()

    def beat():  # keeps a long MIOpen kernel search visibly alive
        while True:
            time.sleep(30)
            print(f"[baseline] alive {time.perf_counter() - t_start:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    dev = torch.device("cuda:0")
    if args.model == "resnet50":
        args.batch = 128
        per_client_step, n_params = signsgd_step_time(args, dev)
        s_round = per_client_step * 128 * 8  # 128 clients, 8 vote steps per round (10 % shards)
        print(json.dumps({
            "metric": "FL rounds/sec (sign-SGD, 128 clients, ResNet-50, ImageNet-shaped) — reference-style PyTorch eager",
            "value": 1.0 / s_round, "unit": "rounds/s", "s_per_round": s_round, "s_per_client_step": per_client_step,
            "samples_per_s": args.batch / per_client_step, "clients_timed": args.clients_timed, "dtype": "fp32",
            "params": n_params, "miopen_benchmark": torch.backends.cudnn.benchmark,
            "config": {"model": "resnet50", "clients": 128, "steps_per_round": 8, "per_client_batch": 128},
            "torch": torch.__version__, "device": torch.cuda.get_device_name(0),
        }), flush=True)
        return
    g = torch.Generator(device="cpu").manual_seed(0)
    if args.model == "transformer":
        # BASELINE config 3: AG-News-shaped (120k samples over 100 clients, L 128, lengths in
        # [L/4, L], token 0 = padding), 50 clients trained per FedOBD round
        per_client = 120000 // 100
        lengths = torch.randint(32, 129, (per_client,), generator=g)
        images = torch.randint(1, 30000, (per_client, 128), generator=g)
        images[torch.arange(128).view(1, -1) >= lengths.view(-1, 1)] = 0
        images = images.to(dev)
        labels = torch.randint(0, 4, (per_client,), generator=g).to(dev)
        model = TransformerClassifier().to(dev)
    else:
        per_client = args.train_size // args.clients
        images = torch.randn(per_client, 3, 32, 32, generator=g).to(dev)
        labels = torch.randint(0, 10, (per_client,), generator=g).to(dev)
        fmt = torch.channels_last if args.channels_last else torch.contiguous_format
        images = images.contiguous(memory_format=fmt)
        model = (ResNet18() if args.model == "ResNet18" else DenseNet40()).to(dev).to(memory_format=fmt)
    global_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    n_params = sum(p.numel() for p in model.parameters())

    for c in range(args.warmup_clients):
        # (first client: MIOpen finds / compiles its kernels — minutes for DenseNet's many shapes)
        train_client(model, global_state, images, labels, args)
        print(f"[baseline] warmup client {c + 1} done", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    acc = None
    t0 = time.perf_counter()
    for c in range(args.clients_timed):
        state = train_client(model, global_state, images, labels, args)
        print(f"[baseline] client {c + 1}/{args.clients_timed} {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        # server side: fp64 weighted accumulation of the upload (fed_avg_algorithm.py:39-52)
        if acc is None:
            acc = {k: v.double() * per_client for k, v in state.items() if v.is_floating_point()}
        else:
            for k in acc:
                acc[k] += state[k].double() * per_client
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s_per_client = dt / args.clients_timed
    round_clients = 50 if args.model == "transformer" else args.clients  # FedOBD: 50 of 100 per round
    s_round = s_per_client * round_clients
    print(json.dumps({
        "metric": ("FL rounds/sec (FedOBD stage 1 training, 100 clients / 50 per round, Transformer-base, "
                   "AG-News-shaped) — reference-style PyTorch eager" if args.model == "transformer" else
                   f"FL rounds/sec (FedAvg, {args.clients} clients, "
                   f"{'ResNet-18' if args.model == 'ResNet18' else 'DenseNet-40'}, CIFAR-10-shaped) — "
                   "reference-style PyTorch eager"),
        "value": 1.0 / s_round, "unit": "rounds/s", "s_per_round": s_round, "s_per_client": s_per_client,
        "samples_per_s": per_client * args.epoch / s_per_client, "clients_timed": args.clients_timed,
        "dtype": "fp32", "params": n_params, "channels_last": args.channels_last,
        "miopen_benchmark": torch.backends.cudnn.benchmark,
        "config": {"model": args.model, "clients": args.clients, "local_epochs": args.epoch,
                   "per_client_batch": args.batch, "per_client_samples": per_client},
        "torch": torch.__version__, "device": torch.cuda.get_device_name(0),
    }), flush=True)


if __name__ == "__main__":
    main()
