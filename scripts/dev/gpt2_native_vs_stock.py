#!/usr/bin/env python
"""One GPT-2 (mini) training round with the native embedding + LM cross-
entropy vs the stock ones (HF embedding, F.cross_entropy), from the same
weights and batch: relative difference of the round's weight update, per
parameter group (a check that the native pieces compute the same gradient)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(native: bool):
    import importlib.util
    from commefficient_amd.ops import transformer as tx
    from commefficient_amd.train import losses
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpt2_learning.py")
    spec = importlib.util.spec_from_file_location("gl", path)
    gl = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gl)
    orig = tx._embed_native_ok
    if not native:
        tx._embed_native_ok = lambda tr, ids: False
    losses._NATIVE_LM_CE[0] = native
    try:
        args, fed, opt, tl, _ = gl.build(["--mode", "uncompressed", "--error_type", "none",
                                          "--local_momentum", "0", "--virtual_momentum", "0",
                                          "--lr_scale", "0.1", "--weight_decay", "0"], "mini")
        w0 = fed.w.clone()
        it = iter(tl)
        for _ in range(2):
            fed(next(it))
            opt.step()
        torch.cuda.synchronize()
        names = [n for n, p in fed.model.named_parameters() if p.requires_grad]
        return (fed.w - w0).clone(), fed.flat, names
    finally:
        tx._embed_native_ok = orig
        losses._NATIVE_LM_CE[0] = True


def main():
    dn, flat, names = run(True)
    ds, _, _ = run(False)
    print(f"whole update: rel diff {((dn - ds).norm() / ds.norm()).item():.3e}, |update| {ds.norm().item():.3e}")
    for nm, o, n in zip(names, flat.offsets, flat.numels):
        a, b = dn[o:o + n], ds[o:o + n]
        if b.norm() > 0 and ("wte" in nm or "wpe" in nm or "lm_head" in nm or "ln_f" in nm or ".0." in nm):
            print(f"{nm:40s} rel {((a - b).norm() / b.norm()).item():.3e}  |b| {b.norm().item():.3e}")


if __name__ == "__main__":
    main()
