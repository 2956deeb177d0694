"""CV federated training driver (the reference's cv_train.py:85-421).

``main(args)`` = spawn/init -> seeds -> data -> model (+ Fixup / finetune
param groups) -> ``FedModel`` / ``FedOptimizer`` -> LambdaLR triangular
schedule -> epochs of train + val rounds with TableLogger rows, scalar logs,
byte totals -> checkpoint (``checkpoint_path + model + '.pt'`` state_dict,
the reference format, plus a ``.fedstate.pt`` sidecar for resume).

Fixed reference quirks: --eval_before_start works
(#6); an epoch runs exactly ``spe * fraction`` rounds (#16); the NaN check
runs one round behind through a pinned-memory copy instead of a host sync
per round.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from .. import models
from ..data import FedEMNIST, FedImageNet, FedCIFAR10, FedCIFAR100, make_synthetic
from ..data.device_loader import DeviceFedLoader, DeviceValLoader
from ..data.transforms import host_transforms
from ..parallel import dist
from ..parallel.fed_model import FedModel
from ..parallel.server import FedOptimizer
from ..utils import (ScalarWriter, TableLogger, Timer, make_logdir, num_classes_of_dataset,
                     steps_per_epoch, triangular_lambda, union)
from ..utils.trace import RoundProfiler
from .losses import cv_loss

DATASETS = {"CIFAR10": FedCIFAR10, "CIFAR100": FedCIFAR100, "EMNIST": FedEMNIST,
            "ImageNet": FedImageNet}


def get_datasets(args):
    name = args.dataset_name or "CIFAR10"
    args.dataset_name = name
    if args.synthetic:
        hard = getattr(args, "synthetic_difficulty", "easy") == "hard"
        tr = make_synthetic(name, train=True, do_iid=args.do_iid, num_clients=args.num_clients,
                            size=args.synthetic_size, seed=args.seed, hard=hard)
        te = make_synthetic(name, train=False, size=args.synthetic_size, seed=args.seed,
                            hard=hard)
        return tr, te
    cls = DATASETS[name]
    tr = cls(args.dataset_dir, name, None, args.do_iid, args.num_clients, train=True,
             download=True, seed=args.seed)
    te = cls(args.dataset_dir, name, None, train=False, download=False)
    return tr, te


def get_data_loaders(args, device):
    train_ds, test_ds = get_datasets(args)
    if hasattr(train_ds, "arrays"):
        out_bf16 = args.dtype == "bf16"
        aug = args.dataset_name in ("CIFAR10", "CIFAR100")
        train_loader = DeviceFedLoader(train_ds, args.num_workers, args.local_batch_size, device,
                                       seed=args.seed, augment=aug, out_bf16=out_bf16)
        test_loader = DeviceValLoader(test_ds, args.valid_batch_size * args.num_workers, device,
                                      out_bf16=out_bf16)
    else:  # folder datasets (ImageNet): host decode path
        from ..data.host_loader import host_fed_loaders
        train_loader, test_loader = host_fed_loaders(args, train_ds, test_ds,
                                                     host_transforms(args.dataset_name))
    return train_loader, test_loader


def build_param_groups(args, model):
    if args.model.startswith("Fixup"):
        nps = list(model.named_parameters())
        bias = [p for n, p in nps if "bias" in n]
        scale = [p for n, p in nps if "scale" in n]
        other = [p for n, p in nps if not ("bias" in n or "scale" in n)]
        return [{"params": bias, "lr": 0.1}, {"params": scale, "lr": 0.1},
                {"params": other, "lr": 1}]
    if args.do_finetune:
        sd = torch.load(args.finetune_path + args.model + ".pt", map_location="cpu",
                        weights_only=True)
        model.load_state_dict(sd)
        for p in model.parameters():
            p.requires_grad = False
        return list(model.finetune_parameters())
    return list(model.parameters())


class LagNaNCheck:
    """Detects a NaN round loss one round late, without a per-round sync."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.prev = None

    def push(self, loss_vec: torch.Tensor) -> bool:
        bad = False
        if self.prev is not None:
            ev, host = self.prev
            ev.synchronize()
            bad = bool(host.item())
        flag = torch.isnan(loss_vec).any()
        if self.device.type == "cuda":
            host = torch.empty((), dtype=torch.bool, pin_memory=True)
            host.copy_(flag, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self.prev = (ev, host)
        else:
            self.prev = (_Done(), flag)
        return bad


class _Done:
    def synchronize(self):
        pass


def run_batches(model, opt, lr_scheduler, loader, training, epoch_fraction, args, nan_check=None,
                profiler=None, progress=None):
    if not training and epoch_fraction != 1:
        raise ValueError("Must do full epochs for val")
    model.train(training)
    losses, accs = [], []
    ds = loader.dataset
    rounds = 0
    if training:
        spe = steps_per_epoch(args.local_batch_size, ds, args.num_workers)
        t0 = time.time()
        # resumed mid-epoch: the sampler skips the rounds already processed
        start = progress["iter"] if progress is not None else 0
        if progress is not None:
            progress["epoch_done"] = True
        for i, batch in enumerate(loader, start=start):
            if i >= spe * epoch_fraction:
                break
            if args.max_rounds and model.round_idx >= args.max_rounds:
                if progress is not None:
                    progress["epoch_done"] = False
                break
            if progress is not None:
                progress["iter"] = i + 1  # loader rounds consumed in this epoch
            lr_scheduler.step()
            if lr_scheduler.get_last_lr()[0] == 0:
                opt.step()  # reference "HACK STEP": no pending round -> only sets fedavg LR
            cids = batch.client_ids if hasattr(batch, "client_ids") else batch[0].numpy()
            if args.local_batch_size == -1:
                if len(np.unique(cids)) < args.num_workers:
                    print("SKIPPING BATCH: NOT ENOUGH CLIENTS ({} < {})".format(
                        len(np.unique(cids)), args.num_workers))
                    continue
            elif len(cids) < args.num_workers * args.local_batch_size:
                print("SKIPPING BATCH: NOT ENOUGH DATA ({} < {})".format(
                    len(cids), args.num_workers * args.local_batch_size))
                continue
            loss, acc, _dl, _ul = model(batch)
            if nan_check is not None and nan_check.push(loss):
                print("LOSS IS NAN, TERMINATING TRAINING")
                if progress is not None:
                    progress["nan"] = True
                return float("nan"), float("nan")
            opt.step()
            if profiler is not None:
                profiler.step()
            losses.append(loss)
            accs.append(acc)
            rounds += 1
            if (args.checkpoint_every and progress is not None
                    and model.round_idx % args.checkpoint_every == 0):
                save_checkpoint(model, args, progress)
            if args.log_every and rounds % args.log_every == 0 and dist.ctx().is_main:
                print("round {} lr {:.5f} loss {:.4f} acc {:.4f} ({:.1f} rounds/s)".format(
                    model.round_idx, lr_scheduler.get_last_lr()[0], loss.mean().item(),
                    acc.mean().item(), rounds / (time.time() - t0)))
            if args.do_test:
                break
        if progress is not None:
            progress["rounds"] = rounds
    else:
        for batch in loader:
            if len(batch) < args.valid_batch_size:
                print("SKIPPING VAL BATCH: TOO SMALL")
                continue
            loss, acc = model(batch)[:2]
            losses.append(loss)
            accs.append(acc)
            if args.do_test:
                break
    if not losses:
        return float("nan"), float("nan")
    return torch.cat(losses).mean().item(), torch.cat(accs).mean().item()


def train(model, opt, lr_scheduler, train_loader, test_loader, args, writer, loggers=(),
          timer=None, progress=None):
    """``progress``: {"epoch", "iter", "loader", "sched"} -- where training
    stands (restored by --resume, saved in the .fedstate.pt sidecar)."""
    timer = timer or Timer()
    if progress is None:
        progress = {"epoch": 0, "iter": 0}
    progress["loader"] = train_loader
    progress["sched"] = lr_scheduler
    ctx = dist.ctx()
    nan_check = LagNaNCheck(model.device)
    profiler = RoundProfiler(getattr(args, "profile_dir", None), ctx.rank,
                             getattr(args, "profile_rounds", 5))
    total_down = total_up = 0.0
    acct = model.accountant
    summary = {}
    if args.eval_before_start:
        test_loss, test_acc = run_batches(model, None, None, test_loader, False, 1, args)
        timer()
        if ctx.is_main:
            print("Test acc at epoch 0: {:0.4f}".format(test_acc))
    for epoch in range(progress["epoch"], math.ceil(args.num_epochs)):
        if epoch != progress["epoch"]:
            progress["epoch"], progress["iter"] = epoch, 0
        frac = args.num_epochs - epoch if epoch == math.ceil(args.num_epochs) - 1 else 1
        d0 = acct.client_download.sum().item()
        u0 = acct.client_upload.sum().item()
        train_loss, train_acc = run_batches(model, opt, lr_scheduler, train_loader, True, frac,
                                            args, nan_check, profiler, progress)
        if progress.get("nan") or (math.isnan(train_loss) and progress.get("rounds", 0) > 0):
            print("TERMINATING TRAINING DUE TO NAN LOSS")
            return summary
        train_time = timer()
        down_mb = (acct.client_download.sum().item() - d0) / (1024 * 1024)
        up_mb = (acct.client_upload.sum().item() - u0) / (1024 * 1024)
        total_down += down_mb
        total_up += up_mb
        test_loss, test_acc = run_batches(model, None, None, test_loader, False, 1, args)
        test_time = timer()
        lr = lr_scheduler.get_last_lr()[0]
        stats = {"train_time": train_time, "train_loss": train_loss, "train_acc": train_acc,
                 "test_loss": test_loss, "test_acc": test_acc, "down (MiB)": round(down_mb),
                 "up (MiB)": round(up_mb), "total_time": timer.total_time}
        summary = union({"epoch": epoch + 1, "lr": lr}, stats)
        if ctx.is_main:
            for lg in loggers:
                lg.append(summary)
            if writer is not None:
                for tag, v in (("Loss/train", train_loss), ("Loss/test", test_loss),
                               ("Acc/train", train_acc), ("Acc/test", test_acc),
                               ("Time/train", train_time), ("Time/test", test_time),
                               ("Time/total", timer.total_time), ("Lr", lr)):
                    writer.add_scalar(tag, v, epoch)
        if progress.get("epoch_done", True):
            progress["epoch"], progress["iter"] = epoch + 1, 0  # epoch complete
        if args.max_rounds and model.round_idx >= args.max_rounds:
            break
    profiler.close(model.timer)
    if ctx.is_main:
        nc = train_loader.dataset.num_clients
        print("Total Download (MiB): {:0.2f}".format(total_down))
        print("Total Upload (MiB): {:0.2f}".format(total_up))
        print("Avg Download Per Client: {:0.2f}".format(total_down / nc))
        print("Avg Upload Per Client: {:0.2f}".format(total_up / nc))
        if getattr(model, "skipped_rounds", 0):
            print("Rounds dropped by --skip_nonfinite: {}".format(model.skipped_rounds))
    return summary


def driver_state(progress) -> dict:
    """Epoch / in-epoch position, sampler RNG and LR-schedule step."""
    if not progress:
        return {}
    out = {"epoch": int(progress["epoch"]), "iter": int(progress["iter"])}
    ld = progress.get("loader")
    if ld is not None and hasattr(ld, "state_dict"):
        out["loader"] = ld.state_dict(pos=progress["iter"])
        out["loader"]["epoch"] = int(progress["epoch"])
    elif ld is not None and hasattr(getattr(ld, "batch_sampler", None), "state_dict"):
        out["loader"] = {"sampler": ld.batch_sampler.state_dict(pos=progress["iter"]),
                         "epoch": int(progress["epoch"])}
    sch = progress.get("sched")
    if sch is not None:
        out["sched_steps"] = int(sch.last_epoch)
    return out


def restore_driver_state(sd: dict, loader, sched) -> dict:
    """Inverse of ``driver_state``: position the sampler and the schedule."""
    drv = sd.get("driver") or {}
    progress = {"epoch": int(drv.get("epoch", 0)), "iter": int(drv.get("iter", 0))}
    ls = drv.get("loader")
    if ls is not None:
        if hasattr(loader, "load_state_dict"):
            loader.load_state_dict(ls)
        elif hasattr(getattr(loader, "batch_sampler", None), "load_state_dict"):
            loader.batch_sampler.load_state_dict(ls["sampler"])
    if "sched_steps" in drv:
        while sched.last_epoch < drv["sched_steps"]:
            sched.step()
    return progress


def save_checkpoint(model: FedModel, args, progress=None):
    # every rank joins the gathers of the sharded server state and the
    # per-client rows; rank 0 writes
    fs = model.fed_state_dict()
    if not dist.ctx().is_main:
        return
    path = args.checkpoint_path + args.model + ".pt"
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save(model.state_dict(), path)
    fs["driver"] = driver_state(progress)
    torch.save(fs, args.checkpoint_path + args.model + ".fedstate.pt")
    print("saved", path)


def main(args, loggers=()):
    """``loggers``: extra per-epoch row sinks (``.append(dict)``), e.g. the
    convergence script's JSONL curve, next to the TableLogger."""
    ctx = dist.init(args.device, port=args.port)
    timer = Timer()
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if args.do_test:
        args.num_cols, args.num_rows, args.k = 10, 1, 10
    if args.do_finetune:
        num_classes = num_classes_of_dataset(args.finetuned_from)
        num_new = num_classes_of_dataset(args.dataset_name)
    else:
        num_classes = num_classes_of_dataset(args.dataset_name or "CIFAR10")
        num_new = None
    train_loader, test_loader = get_data_loaders(args, ctx.device)
    if args.num_clients is None:
        args.num_clients = train_loader.dataset.num_clients
    model = models.build_model(args, num_classes, num_new)
    groups = build_param_groups(args, model)
    opt = torch.optim.SGD(groups, lr=1)
    fed = FedModel(model, cv_loss, args, cv_loss, num_clients=args.num_clients)
    fopt = FedOptimizer(opt, args, fed)
    spe = steps_per_epoch(args.local_batch_size, train_loader.dataset, args.num_workers)
    if args.lr_scale is None:
        args.lr_scale = 0.4
    sched = torch.optim.lr_scheduler.LambdaLR(fopt, lr_lambda=triangular_lambda(args, spe))
    progress = None
    if args.resume:
        sd = torch.load(args.resume, map_location="cpu", weights_only=True)
        fed.load_fed_state_dict(sd)
        progress = restore_driver_state(sd, train_loader, sched)
    log_dir = make_logdir(args)
    writer = ScalarWriter(log_dir) if (args.use_tensorboard and ctx.is_main) else None
    if ctx.is_main:
        print("Finished initializing in {:.2f} seconds".format(timer()))
    progress = progress or {"epoch": 0, "iter": 0}
    train(fed, fopt, sched, train_loader, test_loader, args, writer,
          loggers=(TableLogger(),) + tuple(loggers), timer=timer, progress=progress)
    fed.finalize()
    if args.do_checkpoint:
        save_checkpoint(fed, args, progress)
    if writer is not None:
        writer.close()
    if fed.timer.enabled and ctx.is_main:
        print("phase ms:", fed.timer.summary())
    return fed
