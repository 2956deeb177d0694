"""Federated data layer: FedDataset/FedSampler semantics (reference
data_utils/fed_dataset.py, fed_sampler.py), on-disk formats (SURVEY.md
Appendix D) and the device loader."""
import json
import os

import numpy as np
import pytest
import torch

from commefficient_amd.data import FedCIFAR10, FedEMNIST, FedSampler, make_synthetic
from commefficient_amd.data.device_loader import DeviceFedLoader, DeviceValLoader
from commefficient_amd.data.fed_persona import (FedPERSONA, SyntheticPersona, collate,
                                                build_input_from_segments)


def test_noniid_split_matches_reference_formula():
    ds = make_synthetic("CIFAR10", train=True, num_clients=30, size=1003)
    ipc = ds.images_per_client  # natural clients (classes): 101 x 3 + 100 x 7
    dpc = ds.data_per_client
    assert len(dpc) == 30 and dpc.sum() == 1003
    # each natural client split into 3 equal parts, remainder to the last
    for nat, n in enumerate(ipc):
        part = dpc[nat * 3:(nat + 1) * 3]
        assert list(part[:2]) == [n // 3, n // 3] and part[2] == n // 3 + n % 3
    # non-iid: every client's examples come from one class
    r = np.arange(1003)
    cl = ds.client_of(r)
    tgt = ds.train_targets[ds.data_index(r)]
    for c in range(30):
        assert len(np.unique(tgt[cl == c])) == 1


def test_iid_split():
    ds = make_synthetic("CIFAR10", train=True, do_iid=True, num_clients=7, size=100)
    dpc = ds.data_per_client
    assert dpc.sum() == 100 and dpc.max() - dpc.min() <= 1 and list(dpc[-2:]) == [15, 15]


@pytest.mark.parametrize("lbs", [-1, 3])
def test_sampler_semantics(lbs):
    ds = make_synthetic("CIFAR10", train=True, num_clients=20, size=200)
    s = FedSampler(ds, 4, lbs, seed=0)
    seen = []
    for r in s:
        cl = ds.client_of(r)
        u, cnt = np.unique(cl, return_counts=True)
        assert len(u) <= 4
        if lbs != -1:
            assert cnt.max() <= lbs
        else:
            assert all(c == ds.data_per_client[x] for x, c in zip(u, cnt))
        seen.append(r)
    allr = np.concatenate(seen)
    assert sorted(allr.tolist()) == list(range(200))  # epoch covers every example once
    # same seed -> same rounds on every rank
    a = [x.tolist() for x in FedSampler(ds, 4, lbs, seed=9)]
    b = [x.tolist() for x in FedSampler(ds, 4, lbs, seed=9)]
    assert a == b


def test_cifar_on_disk_format_roundtrip(tmp_path):
    rng = np.random.RandomState(0)
    tr_x = rng.randint(0, 256, (60, 32, 32, 3)).astype(np.uint8)
    tr_y = np.repeat(np.arange(10), 6)
    te_x = rng.randint(0, 256, (20, 32, 32, 3)).astype(np.uint8)
    te_y = rng.randint(0, 10, 20)
    FedCIFAR10.write_split(str(tmp_path), tr_x, tr_y, te_x, te_y, 10)
    assert json.load(open(tmp_path / "stats.json")) == {"images_per_client": [6] * 10,
                                                        "num_val_images": 20}
    ds = FedCIFAR10(str(tmp_path), "CIFAR10", None, False, 20, train=True)
    cid, img, tgt = ds[13]
    assert cid == 4 and tgt == 2 and img.shape == (32, 32, 3)  # class 2, first half
    assert np.array_equal(img, tr_x[13])
    te = FedCIFAR10(str(tmp_path), "CIFAR10", None, train=False)
    cid, img, tgt = te[5]
    assert cid == -1 and tgt == te_y[5]


def test_emnist_pt_format(tmp_path):
    os.makedirs(tmp_path / "train")
    os.makedirs(tmp_path / "test")
    for i in range(3):
        torch.save({"x": torch.rand(4, 28, 28), "y": torch.full((4,), i)},
                   tmp_path / "train" / f"client{i}.pt")
    torch.save({"x": torch.rand(5, 28, 28), "y": torch.arange(5)}, tmp_path / "test" / "test.pt")
    json.dump({"images_per_client": [4, 4, 4], "num_val_images": 5},
              open(tmp_path / "stats.json", "w"))
    ds = FedEMNIST(str(tmp_path), "EMNIST", None, False, 3, train=True)
    x, y = ds.arrays()
    assert x.shape == (12, 28, 28, 1) and x.dtype == np.uint8 and list(y[::4]) == [0, 1, 2]


def test_device_loader_cpu():
    ds = make_synthetic("CIFAR10", train=True, num_clients=20, size=200)
    ld = DeviceFedLoader(ds, 5, -1, "cpu", seed=1)
    rb = next(iter(ld))
    assert len(np.unique(rb.client_ids)) == 5
    x, y = rb.take(np.arange(len(rb)))
    assert x.shape == (len(rb), 3, 32, 32) and y.shape == (len(rb),)
    # the same example gets the same augmentation whether taken alone or in a group
    x1, _ = rb.take(np.array([3]))
    torch.testing.assert_close(x1[0], x[3])
    te = make_synthetic("CIFAR10", train=False, size=200)
    vb = next(iter(DeviceValLoader(te, 16, "cpu")))
    assert (vb.client_ids == -1).all()


class _Tok:
    def tokenize(self, s):
        return s.split()

    def convert_tokens_to_ids(self, toks):
        if isinstance(toks, str):
            toks = [toks]
        return [abs(hash(t)) % 1000 if not t.startswith("<") else 1000 + ["<bos>", "<eos>",
                "<speaker1>", "<speaker2>", "<pad>"].index(t) for t in toks]


def test_persona_formats(tmp_path):
    dialog = {"personality": ["i like cats", "i am tall"],
              "utterances": [{"history": ["hi"], "candidates": ["no", "hello there"]},
                             {"history": ["hi", "hello there", "how are you"],
                              "candidates": ["bad", "fine thanks"]}]}
    for i in range(2):
        json.dump([dialog], open(tmp_path / f"client{i}.json", "w"))
    json.dump([dialog], open(tmp_path / "validation.json", "w"))
    json.dump({"dialogs_per_client": [1, 1], "train_utterances_per_dialog": [2, 2],
               "val_utterances_per_dialog": [2]}, open(tmp_path / "stats.json", "w"))
    ds = FedPERSONA(_Tok(), 2, 2, 1, str(tmp_path), "PERSONA", None, False, None, train=True)
    assert len(ds) == 4 and list(ds.data_per_client) == [2, 2]
    cid, rec = ds[3]
    assert cid == 1 and rec["mc_labels"] == 1 and len(rec["input_ids"]) == 2
    ids, mc, lab, mcl, tt = collate([rec, ds[0][1]])
    assert ids.shape[:2] == (2, 2) and (lab[0, 0] == -100).all()  # only gold has lm labels
    gold = lab[0, 1]
    assert (gold != -100).sum() == len("fine thanks".split()) + 1  # reply + <eos>
    val = FedPERSONA(_Tok(), -1, 2, 1, str(tmp_path), "PERSONA", None, train=False)
    assert len(val) == 2 and val[1][0] == -1


def test_build_input_segments_token_types():
    inst = build_input_from_segments([[5, 6]], [[7], [8, 9]], [10], [1, 2, 3, 4], lm_labels=True)
    # the reply is always spoken by speaker2 (fed_persona.py:338-342)
    assert inst["input_ids"] == [1, 5, 6, 4, 7, 3, 8, 9, 4, 10, 2]
    assert inst["token_type_ids"] == [3, 3, 3, 4, 4, 3, 3, 3, 4, 4, 4]
    assert inst["lm_labels"][-2:] == [10, 2] and inst["mc_token_ids"] == 10


def test_synthetic_persona_shapes():
    ds = SyntheticPersona(num_personalities=10, dialogs_per_client=2, utterances_per_dialog=3)
    assert len(ds) == 60 and ds.num_clients == 10
    cid, rec = ds[7]
    assert cid == 1 and len(rec["input_ids"]) == 2


def test_prepare_cifar_from_binary_release(tmp_path):
    """CIFAR-10/100 binary records -> the reference layout (one client per
    class) -> readable by FedCIFAR10/100."""
    import json as _json
    from commefficient_amd.data.image_datasets import FedCIFAR10, FedCIFAR100
    rng = np.random.RandomState(0)
    for cls, sub, files, lb, ncls in ((FedCIFAR10, "cifar-10-batches-bin",
                                       [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"],
                                       1, 10),
                                      (FedCIFAR100, "cifar-100-binary", ["train.bin", "test.bin"],
                                       2, 100)):
        root = tmp_path / sub
        root.mkdir(parents=True)
        for fn in files:
            n = 30
            lab = rng.randint(0, ncls, size=(n, lb)).astype(np.uint8)
            px = rng.randint(0, 256, size=(n, 3072)).astype(np.uint8)
            np.concatenate([lab, px], 1).tofile(str(root / fn))
        ds = cls(str(tmp_path), cls.__name__[3:], None, False, None, train=True, download=True)
        x, y = ds.arrays()
        assert x.shape[1:] == (32, 32, 3) and x.dtype == np.uint8
        stats = _json.load(open(tmp_path / "stats.json"))
        assert len(stats["images_per_client"]) == ncls and sum(stats["images_per_client"]) == len(y)
        for p in tmp_path.iterdir():  # next dataset in a clean dir
            if p.is_file():
                p.unlink()


def test_prepare_femnist_from_leaf_json(tmp_path):
    import json as _json
    from commefficient_amd.data.image_datasets import FedEMNIST
    rng = np.random.RandomState(1)
    for split, users in (("train", ["w0", "w1", "w2"]), ("test", ["w0", "w3"])):
        (tmp_path / split).mkdir()
        data = {"users": users, "num_samples": [], "user_data": {}}
        for u in users:
            n = rng.randint(2, 5)
            data["user_data"][u] = {"x": rng.rand(n, 784).tolist(), "y": rng.randint(0, 62, n).tolist()}
        (tmp_path / split / "all_data_0.json").write_text(_json.dumps(data))
    ds = FedEMNIST(str(tmp_path), "EMNIST", None, False, None, train=True, download=True)
    x, y = ds.arrays()
    assert x.shape[1:] == (28, 28, 1) and x.dtype == np.uint8
    assert len(ds.images_per_client) == 3 and int(np.sum(ds.images_per_client)) == len(y)
    te = FedEMNIST(str(tmp_path), "EMNIST", None, False, None, train=False)
    assert len(te.arrays()[1]) == ds.num_val_images


def test_persona_loader_workers_match_inline():
    """--train_dataloader_workers: the rounds built in forked worker
    processes (prefetched ahead) are the rounds built inline, tensor for
    tensor, in the same order."""
    from commefficient_amd.data.persona_loader import PersonaFedLoader
    ds = SyntheticPersona(num_personalities=40, num_candidates=2, max_history=2, train=True,
                          num_clients=40, seed=3)
    outs = {}
    for workers in (0, 2):
        ld = PersonaFedLoader(ds, 4, 3, "cpu", seed=7, workers=workers)
        rounds = []
        for i, rb in enumerate(ld):
            if i >= 5:
                break
            pos = np.arange(len(rb))[::-1].copy()  # a permuted selection
            rounds.append((rb.client_ids.copy(), rb.take(pos)))
        ld.close()
        outs[workers] = rounds
    assert len(outs[0]) == len(outs[2]) == 5
    for (c0, t0), (c2, t2) in zip(outs[0], outs[2]):
        assert np.array_equal(c0, c2)
        for a, b in zip(t0, t2):
            if torch.is_tensor(a):
                assert torch.equal(a, b)
            else:
                assert np.array_equal(np.asarray(a), np.asarray(b))
