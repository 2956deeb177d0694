"""GPT-2 federated training driver (the reference's gpt2_train.py:115-365).

Double-heads GPT-2 (LM + multiple choice) on PersonaChat, one client per
personality, linear LR decay from ``lr_scale`` (default 4e-2) to 0, per-round
logging, HF ``save_pretrained`` of the server weights after each epoch,
validation reporting nll / acc / ppl = exp(mean nll) (gpt2_train.py:149-253).
``--finetune`` only evaluates a saved model (gpt2_train.py:308-309).
With ``--synthetic`` PersonaChat-shaped token data is generated (no tokenizer
or downloads needed); otherwise the reference on-disk layout is read with a
local HF tokenizer directory given by ``--model_checkpoint``.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from ..data.fed_persona import SPECIAL_TOKENS, FedPERSONA, SyntheticPersona
from ..data.persona_loader import PersonaFedLoader, PersonaValLoader
from ..models.gpt2 import ATTR_TO_SPECIAL_TOKEN, GPT2DoubleHeads
from ..parallel import dist
from ..parallel.fed_model import FedModel
from ..parallel.server import FedOptimizer
from ..utils import (ScalarWriter, TableLogger, Timer, linear_decay_lambda, make_logdir,
                     steps_per_epoch)
from ..utils.trace import RoundProfiler
from .losses import gpt2_loss_train, gpt2_loss_val
from .cv import restore_driver_state, save_checkpoint


def get_data_loaders(args, device, tokenizer=None):
    if args.synthetic:
        n_pers = args.num_clients or 1000
        text = getattr(args, "synthetic_text", "uniform")
        # the model's base vocabulary (GPT-2 50,257, OpenAI-GPT 40,478), before the
        # 5 special tokens the synthetic records append
        n_tok = getattr(args, "len_tokenizer", None)
        vocab = n_tok - len(SPECIAL_TOKENS) if n_tok else 50257
        tr = SyntheticPersona(num_personalities=n_pers, num_candidates=args.num_candidates,
                              max_history=args.max_history, train=True, do_iid=args.do_iid,
                              num_clients=args.num_clients, seed=args.seed, text=text, vocab=vocab)
        te = SyntheticPersona(num_personalities=n_pers, num_candidates=args.num_candidates,
                              max_history=args.max_history, train=False, seed=args.seed,
                              n_val=max(args.valid_batch_size * args.num_workers, 200), text=text,
                              vocab=vocab)
    else:
        tr = FedPERSONA(tokenizer, args.num_candidates, args.max_history,
                        args.personality_permutations, args.dataset_dir, "PERSONA", None,
                        args.do_iid, args.num_clients, train=True, download=True, seed=args.seed)
        te = FedPERSONA(tokenizer, -1, args.max_history, 1, args.dataset_dir, "PERSONA",
                        None, train=False)
    train = PersonaFedLoader(tr, args.num_workers, args.local_batch_size, device, args.seed,
                             workers=getattr(args, "train_dataloader_workers", 0))
    test = PersonaValLoader(te, args.valid_batch_size * args.num_workers, device)
    return train, test


def run_batches(model, opt, sched, loader, training, args, writer=None, log_step0=0,
                profiler=None, progress=None):
    model.train(training)
    losses, accs = [], []
    ctx = dist.ctx()
    if training:
        spe = steps_per_epoch(args.local_batch_size, loader.dataset, args.num_workers)
        t0 = time.time()
        # resumed mid-epoch: the sampler skips the rounds already processed
        start = progress["iter"] if progress is not None else 0
        if progress is not None:
            progress["epoch_done"] = True
        for i, batch in enumerate(loader, start=start):
            if i >= spe:
                break
            if args.max_rounds and model.round_idx >= args.max_rounds:
                if progress is not None:
                    progress["epoch_done"] = False
                break
            if progress is not None:
                progress["iter"] = i + 1
            sched.step()
            if args.local_batch_size == -1:
                if len(np.unique(batch.client_ids)) < args.num_workers:
                    continue
            elif len(batch) < args.num_workers * args.local_batch_size:
                continue
            loss, acc, dl, ul = model(batch)
            opt.step()
            if profiler is not None:
                profiler.step()
            if (args.checkpoint_every and progress is not None
                    and model.round_idx % args.checkpoint_every == 0):
                save_checkpoint(model, args, progress)
            losses.append(loss)
            accs.append(acc)
            if writer is not None and ctx.is_main:
                writer.add_scalar("training/loss", loss.mean().item(), log_step0 + i)
            if args.log_every and (i + 1) % args.log_every == 0 and ctx.is_main:
                print("round {} loss {:.4f} ({:.2f} s/round)".format(
                    model.round_idx, loss.mean().item(), (time.time() - t0) / (i + 1)))
            if args.do_test and i >= 2:
                break
    else:
        for i, batch in enumerate(loader):
            nll, acc = model(batch)[:2]
            losses.append(nll)
            accs.append(acc)
            if args.do_test and i >= 2:
                break
    if not losses:
        return float("nan"), float("nan")
    return torch.cat(losses).mean().item(), torch.cat(accs).mean().item()


def main(args):
    ctx = dist.init(args.device, port=args.port)
    timer = Timer()
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    if args.lr_scale is None:
        args.lr_scale = 4e-2
    args.dataset_name = "PERSONA"
    tokenizer = None
    if not args.synthetic:
        from transformers import AutoTokenizer
        tokenizer = AutoTokenizer.from_pretrained(args.model_checkpoint)
        tokenizer.add_special_tokens(ATTR_TO_SPECIAL_TOKEN)
    size = "tiny" if args.do_test else args.gpt2_size
    dims = {"tiny": {"n_layer": 2, "n_embd": 64, "n_head": 2},
            # smallest shape on the native junction + attention kernels
            "mini": {"n_layer": 2, "n_embd": 256, "n_head": 4}}.get(size, {})
    # (--test: a random-init model of the checkpoint's family -- GPT-2 or
    # OpenAI-GPT, gpt2_train.py:262-267 -- not the checkpoint itself)
    family = "gpt2" if "gpt2" in args.model_checkpoint else "openai-gpt"
    model = GPT2DoubleHeads(args.model_checkpoint if not args.do_test else family, **dims)
    if tokenizer is not None:
        model.model.resize_token_embeddings(len(tokenizer))
    args.len_tokenizer = model.model.config.vocab_size
    train_loader, test_loader = get_data_loaders(args, ctx.device, tokenizer)
    if args.num_clients is None:
        args.num_clients = train_loader.dataset.num_clients
    opt = torch.optim.SGD(model.parameters(), lr=1)
    fed = FedModel(model, gpt2_loss_train, args, gpt2_loss_val, num_clients=args.num_clients)
    fopt = FedOptimizer(opt, args, fed)
    spe = steps_per_epoch(args.local_batch_size, train_loader.dataset, args.num_workers)
    sched = torch.optim.lr_scheduler.LambdaLR(fopt, lr_lambda=linear_decay_lambda(args, spe))
    progress = {"epoch": 0, "iter": 0}
    if args.resume:
        # weights, server / client state, accounting, dropout seed streams,
        # sampler position and LR-schedule step (the cv driver's sidecar format)
        sd = torch.load(args.resume, map_location="cpu", weights_only=True)
        fed.load_fed_state_dict(sd)
        progress = restore_driver_state(sd, train_loader, sched)
    progress["loader"] = train_loader
    progress["sched"] = sched
    log_dir = make_logdir(args)
    writer = ScalarWriter(log_dir) if ctx.is_main else None
    if ctx.is_main:
        print("Finished initializing in {:.2f} seconds".format(timer()))
    logger = TableLogger()
    profiler = RoundProfiler(getattr(args, "profile_dir", None), ctx.rank,
                             getattr(args, "profile_rounds", 5))
    if args.do_finetune:
        nll, acc = run_batches(fed, None, None, test_loader, False, args)
        if ctx.is_main:
            print({"nll": nll, "acc": acc, "ppl": math.exp(nll)})
        return fed
    for epoch in range(progress["epoch"], math.ceil(args.num_epochs)):
        if epoch != progress["epoch"]:
            progress["epoch"], progress["iter"] = epoch, 0
        d0 = fed.accountant.client_download.sum().item()
        u0 = fed.accountant.client_upload.sum().item()
        tl, ta = run_batches(fed, fopt, sched, train_loader, True, args, writer, epoch * int(spe),
                             profiler, progress)
        ttime = timer()
        down = (fed.accountant.client_download.sum().item() - d0) / 2 ** 20
        up = (fed.accountant.client_upload.sum().item() - u0) / 2 ** 20
        if ctx.is_main:
            fed.save_pretrained(log_dir)
        nll, acc = run_batches(fed, None, None, test_loader, False, args)
        if ctx.is_main:
            logger.append({"epoch": epoch + 1, "train_time": ttime, "train_loss": tl,
                           "val_nll": nll, "val_acc": acc, "val_ppl": math.exp(min(nll, 50)),
                           "down (MiB)": round(down), "up (MiB)": round(up),
                           "total_time": timer.total_time})
            if writer is not None:
                writer.add_scalar("validation/nll", nll, epoch)
                writer.add_scalar("validation/acc", acc, epoch)
                writer.add_scalar("validation/ppl", math.exp(min(nll, 50)), epoch)
        if progress.get("epoch_done", True):
            progress["epoch"], progress["iter"] = epoch + 1, 0
        if args.max_rounds and fed.round_idx >= args.max_rounds:
            break
    profiler.close(fed.timer)
    train_loader.close()  # the record worker processes, if any
    fed.finalize()
    if args.do_checkpoint:
        save_checkpoint(fed, args, progress)
    if writer is not None:
        writer.close()
    return fed
