"""End-to-end driver runs on CPU (synthetic data): the reference's ``--test``
smoke mode (utils.py:106, cv_train.py:329-336) for every
federated mode, checkpoint + resume, torch.profiler tracing, and the GPT-2
driver on the tiny architecture."""
import json
import os

import pytest
import torch

import fed_train

BASE = ["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", "600",
        "--num_clients", "30", "--num_workers", "5", "--local_batch_size", "-1",
        "--device", "cpu", "--dtype", "fp32", "--num_epochs", "1", "--valid_batch_size", "16",
        "--port", "29611"]

MODES = {
    "sketch": ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
               "--virtual_momentum", "0.9", "--num_rows", "3", "--num_cols", "500", "--k", "50",
               "--num_blocks", "2"],
    "true_topk": ["--mode", "true_topk", "--error_type", "virtual", "--local_momentum", "0",
                  "--virtual_momentum", "0.9", "--k", "100"],
    "local_topk": ["--mode", "local_topk", "--error_type", "local", "--local_momentum", "0.9",
                   "--k", "100"],
    "fedavg": ["--mode", "fedavg", "--error_type", "none", "--local_momentum", "0",
               "--num_fedavg_epochs", "2", "--fedavg_batch_size", "10"],
    "uncompressed": ["--mode", "uncompressed", "--error_type", "none", "--local_momentum", "0.9"],
}


@pytest.mark.parametrize("mode", list(MODES))
def test_cv_driver_test_mode(mode, tmp_path, monkeypatch, capsys):
    monkeypatch.chdir(tmp_path)
    fed = fed_train.main(BASE + MODES[mode] + ["--test", "--max_rounds", "2"])
    assert fed.round_idx >= 1
    out = capsys.readouterr().out
    assert "Total Upload (MiB)" in out
    assert torch.isfinite(fed.w).all()


def test_cv_driver_checkpoint_resume_and_profile(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    ck = str(tmp_path / "ck") + os.sep
    base = [a if a != "1" or i == 0 or BASE[i - 1] != "--num_epochs" else "4"
            for i, a in enumerate(BASE)]  # --test runs one round per epoch
    args = base + MODES["sketch"] + ["--test", "--model", "ResNet9", "--max_rounds", "3",
                                     "--checkpoint", "--checkpoint_path", ck,
                                     "--profile_dir", str(tmp_path / "prof"),
                                     "--profile_rounds", "1"]
    fed = fed_train.main(args)
    sd = torch.load(ck + "ResNet9.pt", map_location="cpu", weights_only=True)
    assert "n.prep.conv.weight" in sd
    side = ck + "ResNet9.fedstate.pt"
    assert os.path.exists(side)
    assert os.path.exists(tmp_path / "prof" / "rank0" / "kernels.txt")
    traces = [f for f in os.listdir(tmp_path / "prof" / "rank0") if f.endswith(".json")]
    assert traces
    # resume continues the round counter and the server state
    fed2 = fed_train.main(base + MODES["sketch"] + ["--test", "--max_rounds", "5",
                                                    "--resume", side])
    assert fed2.round_idx > fed.round_idx


def test_gpt2_driver_tiny_synthetic(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    argv = ["--dataset_name", "PERSONA", "--model", "GPT2DoubleHeads", "--synthetic",
            "--synthetic_size", "64", "--num_clients", "16", "--num_workers", "4",
            "--local_batch_size", "2", "--valid_batch_size", "2", "--device", "cpu",
            "--dtype", "fp32", "--gpt2_size", "tiny", "--mode", "sketch",
            "--error_type", "virtual", "--local_momentum", "0", "--virtual_momentum", "0.9",
            "--num_rows", "3", "--num_cols", "2000", "--k", "200", "--num_epochs", "1",
            "--max_rounds", "2", "--num_results_train", "1", "--port", "29612"]
    fed = fed_train.main(argv)
    assert fed.round_idx == 2
    assert torch.isfinite(fed.w).all()


def test_openai_gpt_double_heads_driver_tiny_synthetic(tmp_path, monkeypatch):
    """OpenAI-GPT double heads (M9; the reference picks it for any checkpoint
    name without "gpt2", gpt2_train.py:262-267) through the GPT-2 driver: a
    tiny random-init OpenAIGPTDoubleHeadsModel (eager attention, its own 40,478
    + 5 vocabulary) trains two FetchSGD rounds; validation nll starts at
    ~ln(40,483)."""
    import math
    monkeypatch.chdir(tmp_path)
    argv = ["--dataset_name", "PERSONA", "--model", "GPT2DoubleHeads", "--synthetic",
            "--synthetic_size", "64", "--num_clients", "16", "--num_workers", "4",
            "--local_batch_size", "2", "--valid_batch_size", "2", "--device", "cpu",
            "--dtype", "fp32", "--gpt2_size", "tiny", "--mode", "sketch",
            "--model_checkpoint", "openai-gpt",
            "--error_type", "virtual", "--local_momentum", "0", "--virtual_momentum", "0.9",
            "--num_rows", "3", "--num_cols", "2000", "--k", "200", "--num_epochs", "1",
            "--max_rounds", "2", "--num_results_train", "1", "--port", "29614"]
    fed = fed_train.main(argv)
    m = fed.model.model
    assert type(m).__name__ == "OpenAIGPTDoubleHeadsModel"
    assert m.config.vocab_size == 40478 + 5
    assert fed.round_idx == 2
    assert torch.isfinite(fed.w).all()
    from commefficient_amd.train.gpt2 import get_data_loaders
    _, te = get_data_loaders(fed.args, torch.device("cpu"))
    batch = next(iter(te))
    fed.train(False)
    nll = fed(batch)[0].mean().item()
    assert abs(nll - math.log(40483)) < 1.0, nll


@pytest.mark.parametrize("stop", [3, 5])
def test_resume_reproduces_uninterrupted_run(stop, tmp_path, monkeypatch):
    """Checkpoint after ``stop`` rounds (mid-epoch: 3; epoch boundary: 5 of
    5 rounds/epoch), resume, finish: the weights, server state and byte totals
    equal those of one uninterrupted run (sampler position, augmentation keys,
    LR schedule and accounting all restored)."""
    monkeypatch.chdir(tmp_path)
    base = ["--dataset_name", "CIFAR10", "--synthetic", "--synthetic_size", "40",
            "--num_clients", "20", "--num_workers", "4", "--local_batch_size", "2",
            "--device", "cpu", "--dtype", "fp32", "--num_epochs", "2", "--valid_batch_size", "16",
            "--port", "29613", "--mode", "true_topk", "--error_type", "virtual",
            "--local_momentum", "0", "--virtual_momentum", "0.9", "--k", "5000",
            "--lr_scale", "0.1", "--pivot_epoch", "1"]
    full = fed_train.main(base + ["--max_rounds", "8"])
    ck = str(tmp_path / "ck") + os.sep
    fed_train.main(base + ["--max_rounds", str(stop), "--checkpoint", "--checkpoint_path", ck])
    res = fed_train.main(base + ["--max_rounds", "8", "--resume", ck + "ResNet9.fedstate.pt"])
    assert res.round_idx == full.round_idx == 8
    torch.testing.assert_close(res.w, full.w, rtol=0, atol=0)
    torch.testing.assert_close(res.server.V, full.server.V, rtol=0, atol=0)
    torch.testing.assert_close(res.accountant.client_download, full.accountant.client_download)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [
    ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
     "--virtual_momentum", "0.9", "--num_rows", "5", "--num_cols", "20000", "--k", "2000"],
    ["--mode", "local_topk", "--error_type", "local", "--local_momentum", "0.9",
     "--virtual_momentum", "0", "--k", "2000"],
    ["--mode", "uncompressed", "--error_type", "none", "--local_momentum", "0",
     "--virtual_momentum", "0.9", "--microbatch_size", "2"],
])
def test_gpt2_driver_native_kernels_gpu(mode, tmp_path, monkeypatch):
    """GPT-2 driver rounds on the GPU with the native transformer path
    (junction kernels, fused attention, unpadded tokens, gradient sinks,
    side-stream weight gradients) in a linear (merged) and two per-client
    modes: finite weights that moved, finite losses."""
    monkeypatch.chdir(tmp_path)
    argv = ["--dataset_name", "PERSONA", "--model", "GPT2DoubleHeads", "--synthetic",
            "--synthetic_size", "64", "--num_clients", "16", "--num_workers", "4",
            "--local_batch_size", "2", "--valid_batch_size", "2", "--device", "cuda",
            "--dtype", "bf16", "--gpt2_size", "mini", "--num_epochs", "1",
            "--max_rounds", "3", "--num_results_train", "1", "--port", "29614"] + mode
    fed = fed_train.main(argv)
    assert fed.round_idx == 3
    assert torch.isfinite(fed.w).all()


def test_gpt2_resume_reproduces_uninterrupted_run(tmp_path, monkeypatch):
    """GPT-2 driver (tiny, dropout on): checkpoint mid-epoch, resume, finish ==
    one uninterrupted run, bitwise (sampler position, LR step, server state,
    dropout generators all restored)."""
    monkeypatch.chdir(tmp_path)
    base = ["--dataset_name", "PERSONA", "--model", "GPT2DoubleHeads", "--synthetic",
            "--num_clients", "16", "--num_workers", "4", "--local_batch_size", "2",
            "--valid_batch_size", "2", "--device", "cpu", "--dtype", "fp32", "--gpt2_size", "tiny",
            "--mode", "true_topk", "--error_type", "virtual", "--local_momentum", "0",
            "--virtual_momentum", "0.9", "--k", "500", "--num_epochs", "1",
            "--num_results_train", "1", "--port", "29615"]
    full = fed_train.main(base + ["--max_rounds", "4"])
    ck = str(tmp_path / "ck") + os.sep
    fed_train.main(base + ["--max_rounds", "2", "--checkpoint", "--checkpoint_path", ck])
    res = fed_train.main(base + ["--max_rounds", "4", "--resume",
                                 ck + "GPT2DoubleHeads.fedstate.pt"])
    assert res.round_idx == full.round_idx == 4
    torch.testing.assert_close(res.w, full.w, rtol=0, atol=0)
    torch.testing.assert_close(res.server.V, full.server.V, rtol=0, atol=0)


@pytest.mark.gpu
def test_gpt2_small_fetchsgd_learns_bigram_text():
    """The full-size GPT-2 of the GPT-2 config (12 layers x 768, 124M
    parameters) learns under FetchSGD (5 x 500,000 sketch, k = 50,000,
    virtual momentum 0.9) on the learnable bigram text: validation LM nll
    10.95 at init, 8.9 after 100 rounds at LR 0.05 on MI355X
    (profiles/r6_gpt2_small_learning.jsonl: 7.97 at round 125; LR 0.02 / 0.1
    reach 9.59 / 7.64 by round 150).  The first ~25 rounds' TRAINING loss
    sits above the init value (momentum + error-feedback transient: 11.02
    averaged over rounds 1-25 at LR 0.05) -- what the 13-round
    bench_configs run shows as loss_last > ln 50257."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                        "gpt2_learning.py")
    spec = importlib.util.spec_from_file_location("gpt2_learning", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    extra = ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
             "--virtual_momentum", "0.9", "--num_rows", "5", "--num_cols", "500000", "--k", "50000",
             "--lr_scale", "0.05"]
    rows = mod.curve(100, 25, extra, "small", log=print)
    first = rows[0]["val_nll"]
    best = min(r["val_nll"] for r in rows[1:])
    assert first > 10.5, rows
    assert best < first - 1.2, rows
    assert rows[-1]["val_nll"] < rows[1]["val_nll"], rows


@pytest.mark.gpu
def test_gpt2_fetchsgd_learns_bigram_text():
    """GPT-2 under FetchSGD learns (reference objective gpt2_train.py:88-99,
    server fed_aggregator.py:568-613): on the learnable synthetic PersonaChat
    text (``--synthetic_text bigram``: 1,024 tokens with 4 successors each,
    LM nll ln 50262 = 10.8 at init, ln 4 = 1.39 at the optimum) a mini GPT-2
    (2 layers x 256) with a 5 x 500,000 sketch and k = 50,000 brings the
    validation LM nll down by more than 3 nats within 200 rounds of 8 clients
    (curves: profiles/r4_gpt2_learning.jsonl, gpurun_out/r5g2learn: native
    embedding + CE and the stock ones track each other within the noise)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                        "gpt2_learning.py")
    spec = importlib.util.spec_from_file_location("gpt2_learning", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    extra = ["--mode", "sketch", "--error_type", "virtual", "--local_momentum", "0",
             "--virtual_momentum", "0.9", "--num_rows", "5", "--num_cols", "500000", "--k", "50000",
             "--lr_scale", "0.3"]
    rows = mod.curve(200, 20, extra, "mini", log=print)
    # (the validation nll at this constant LR moves by ~1 nat between
    # evaluations -- e.g. 8.55 / 7.09 / 7.22 / 8.20 / 6.95 at rounds 40-120 on
    # MI355X -- so the bound is on the best evaluation, with a looser one on
    # the mean of the last three)
    first = rows[0]["val_nll"]
    last = sum(r["val_nll"] for r in rows[-3:]) / 3
    best = min(r["val_nll"] for r in rows[1:])
    assert best < first - 3.0, rows
    assert last < first - 2.5, rows
    assert rows[-1]["train_loss"] < rows[1]["train_loss"], rows
