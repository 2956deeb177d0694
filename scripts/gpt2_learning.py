#!/usr/bin/env python
"""Does GPT-2 FetchSGD learn?  A learning curve on the learnable synthetic
PersonaChat text (``--synthetic_text bigram``: 1,024 tokens, 4 successors
each -- LM loss ~10.8 nats at init, ln 4 = 1.39 once the chain is learnt).

Runs the reference's GPT-2 training round (gpt2_train.py:88-99, 115-167:
lm_coef * LM + mc_coef * MC loss, FetchSGD server) through the engine for
``--rounds`` rounds at a constant LR and prints one JSON line every
``--every`` rounds: the mean training loss of those rounds and the
validation LM nll / MC accuracy / ppl (gpt2_train.py test_gpt2).

Usage: python scripts/gpt2_learning.py [--rounds 200] [--every 20] [--mode sketch] [--out f.jsonl]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(extra, size="mini", device="cuda"):
    from commefficient_amd.models.gpt2 import GPT2DoubleHeads
    from commefficient_amd.parallel import dist
    from commefficient_amd.parallel.fed_model import FedModel
    from commefficient_amd.parallel.server import FedOptimizer
    from commefficient_amd.train.gpt2 import get_data_loaders
    from commefficient_amd.train.losses import gpt2_loss_train, gpt2_loss_val
    from commefficient_amd.utils.args import parse_args
    argv = ["--dataset_name", "PERSONA", "--model", "GPT2DoubleHeads", "--synthetic",
            "--synthetic_text", "bigram", "--num_clients", "1000", "--num_workers", "8",
            "--local_batch_size", "4", "--valid_batch_size", "8", "--device", device,
            "--dtype", "bf16" if device == "cuda" else "fp32", "--gpt2_size", size, "--num_epochs", "1",
            "--seed", "21"] + extra
    args = parse_args(argv=argv, probe_port=False)
    ctx = dist.init(device)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    dims = {"tiny": {"n_layer": 2, "n_embd": 64, "n_head": 2},
            "mini": {"n_layer": 2, "n_embd": 256, "n_head": 4}}.get(size, {})
    model = GPT2DoubleHeads("gpt2", **dims)
    args.len_tokenizer = model.model.config.vocab_size
    train_loader, test_loader = get_data_loaders(args, ctx.device)
    fed = FedModel(model, gpt2_loss_train, args, gpt2_loss_val, num_clients=args.num_clients)
    opt = FedOptimizer(torch.optim.SGD(model.parameters(), lr=args.lr_scale or 0.1), args, fed)
    return args, fed, opt, train_loader, test_loader


def validate(fed, test_loader, args, batches=8):
    fed.train(False)
    nl, ac = [], []
    for i, batch in enumerate(test_loader):
        if i >= batches:
            break
        nll, acc = fed(batch)[:2]
        nl.append(nll)
        ac.append(acc)
    fed.train(True)
    nll = torch.cat(nl).mean().item()
    return nll, torch.cat(ac).mean().item()


def curve(rounds, every, extra, size="mini", log=print, device="cuda"):
    args, fed, opt, train_loader, test_loader = build(extra, size, device)
    rows = []
    nll, acc = validate(fed, test_loader, args)
    rows.append({"round": 0, "train_loss": None, "val_nll": nll, "val_acc": acc,
                 "val_ppl": math.exp(min(nll, 50))})
    log(json.dumps(rows[-1]))
    done, acc_loss, t0 = 0, [], time.time()
    while done < rounds:
        for batch in train_loader:
            if done >= rounds:
                break
            if len(batch) < args.num_workers * args.local_batch_size:
                continue
            loss = fed(batch)[0]
            opt.step()
            acc_loss.append(loss.mean())
            done += 1
            if done % every == 0:
                nll, acc = validate(fed, test_loader, args)
                rows.append({"round": done, "train_loss": torch.stack(acc_loss).mean().item(),
                             "val_nll": nll, "val_acc": acc, "val_ppl": math.exp(min(nll, 50)),
                             "s_per_round": (time.time() - t0) / done})
                acc_loss = []
                log(json.dumps(rows[-1]))
    return rows


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=200)
    p.add_argument("--every", type=int, default=20)
    p.add_argument("--size", default="mini")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--mode", default="sketch", choices=["sketch", "uncompressed", "true_topk"])
    p.add_argument("--out", default=None)
    p.add_argument("--device", default="cuda")
    p.add_argument("--stock", action="store_true",
                   help="HF embedding + F.cross_entropy instead of the native ones (A/B)")
    b = p.parse_args()
    if b.stock:
        from commefficient_amd.ops import transformer as tx
        from commefficient_amd.train import losses
        tx._embed_native_ok = lambda tr, ids: False
        losses._NATIVE_LM_CE[0] = False
    extra = ["--mode", b.mode, "--local_momentum", "0", "--virtual_momentum", "0.9",
             "--lr_scale", str(b.lr)]
    if b.mode == "sketch":
        extra += ["--error_type", "virtual", "--num_rows", "5", "--num_cols", "500000", "--k", "50000"]
    elif b.mode == "true_topk":
        extra += ["--error_type", "virtual", "--k", "50000"]
    out = open(b.out, "a") if b.out else None

    def log(line):
        print(line, flush=True)
        if out is not None:
            out.write(json.dumps({"mode": b.mode, "size": b.size, "lr": b.lr, **json.loads(line)}) + "\n")
            out.flush()
    curve(b.rounds, b.every, extra, b.size, log, b.device)


if __name__ == "__main__":
    main()
