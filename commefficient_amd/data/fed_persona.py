"""PersonaChat federated dataset (one client per personality) and a synthetic
PersonaChat-shaped generator.

Reference: /root/reference/CommEfficient/data_utils/fed_persona.py:31-392
(SURVEY.md §2.7 D4, Appendix D).  On-disk layout (same files):
``client{i}.json`` (list of dialogs ``{"personality": [...], "utterances":
[{"history": [...], "candidates": [...]}, ...]}``), ``validation.json``,
``stats.json`` ``{dialogs_per_client, train_utterances_per_dialog,
val_utterances_per_dialog}``.

Model inputs per utterance (``build_input_from_segments``): for each of the
last ``num_candidates`` candidates, ``<bos> persona <speaker?> history...
<speaker?> reply <eos>`` with token types, ``mc_token_ids`` = last position,
``lm_labels`` on the gold (last) reply only; ``mc_labels`` = index of the
gold candidate.  Ignored labels are -100 (the HF convention; the reference's
pytorch_transformers used -1).

Differences by design: utterances are tokenised once per client and cached
(the reference re-reads and re-tokenises a client's JSON for every item,
fed_persona.py:218-221); all personality permutations are returned, fixing
Appendix C #11 (the reference returns only the last one).
"""
from __future__ import annotations

import json
import os
import random
from itertools import chain
from typing import List, Optional

import numpy as np
import torch

from .fed_dataset import FedDataset

SPECIAL_TOKENS = ["<bos>", "<eos>", "<speaker1>", "<speaker2>", "<pad>"]
MODEL_INPUTS = ["input_ids", "mc_token_ids", "lm_labels", "mc_labels", "token_type_ids"]
IGNORE = -100


def build_input_from_segments(persona, history, reply, special_ids, lm_labels=False,
                              with_eos=True):
    bos, eos, speaker1, speaker2 = special_ids[:4]
    sequence = [[bos] + list(chain(*persona))] + [list(h) for h in history]
    sequence += [list(reply) + ([eos] if with_eos else [])]
    sequence = [sequence[0]] + [[speaker2 if (len(sequence) - i) % 2 == 0 else speaker1] + s
                                for i, s in enumerate(sequence[1:])]
    inst = {"input_ids": list(chain(*sequence)),
            "token_type_ids": [speaker2 if i % 2 else speaker1
                               for i, s in enumerate(sequence) for _ in s]}
    inst["mc_token_ids"] = len(inst["input_ids"]) - 1
    inst["lm_labels"] = [IGNORE] * len(inst["input_ids"])
    if lm_labels:
        inst["lm_labels"] = ([IGNORE] * sum(len(s) for s in sequence[:-1]) + [IGNORE]
                             + sequence[-1][1:])
    return inst


def utterance_to_inputs(persona, history, candidates, special_ids, num_candidates, max_history,
                        train=True):
    n = len(candidates)
    if num_candidates > 0 and train:
        n = min(num_candidates, n)
    cands = candidates[-n:]
    hist = history[-(2 * max_history + 1):]
    rec = {k: [] for k in ("input_ids", "mc_token_ids", "lm_labels", "token_type_ids")}
    for j, c in enumerate(cands):
        inst = build_input_from_segments(persona, hist, c, special_ids, lm_labels=(j == n - 1))
        for k in rec:
            rec[k].append(inst[k])
    rec["mc_labels"] = n - 1
    return rec


def collate(records: List[dict], pad_id: int = 0):
    """Pad to the longest sequence -> (input_ids[B,C,L], mc_token_ids[B,C],
    lm_labels[B,C,L], mc_labels[B], token_type_ids[B,C,L])."""
    B = len(records)
    C = len(records[0]["input_ids"])
    L = max(len(s) for r in records for s in r["input_ids"])
    # numpy fill, one torch wrap per tensor (per-sequence torch.tensor calls
    # were half of a round's host batch assembly)
    ids = np.full((B, C, L), pad_id, dtype=np.int64)
    tt = np.full((B, C, L), pad_id, dtype=np.int64)
    lab = np.full((B, C, L), IGNORE, dtype=np.int64)
    mc = np.zeros((B, C), dtype=np.int64)
    mcl = np.zeros(B, dtype=np.int64)
    for b, r in enumerate(records):
        for c in range(C):
            n = len(r["input_ids"][c])
            ids[b, c, :n] = r["input_ids"][c]
            tt[b, c, :n] = r["token_type_ids"][c]
            lab[b, c, :n] = r["lm_labels"][c]
            mc[b, c] = r["mc_token_ids"][c]
        mcl[b] = r["mc_labels"]
    return tuple(torch.from_numpy(a) for a in (ids, mc, lab, mcl, tt))


def label_positions(lab: torch.Tensor) -> torch.Tensor:
    """[B, R] flat positions p = c*L + l of the tokens whose NEXT token is a
    labelled LM target (lab[b, c, l+1] != -100), in order; -1 pads rows to the
    batch's largest count R.  Lets the loss run the LM head on the R labelled
    positions of an example instead of all C*L (the reference's HF model
    computes logits for every position, gpt2_train.py:88-99; only the gold
    reply is labelled, ~15 of ~260 positions per example)."""
    B, C, L = lab.shape
    nxt = torch.zeros(B, C, L, dtype=torch.bool)
    nxt[:, :, :-1] = lab[:, :, 1:] != IGNORE
    m = nxt.reshape(B, C * L)
    cnt = m.sum(1)
    R = max(1, int(cnt.max())) if B else 1
    order = torch.argsort((~m).to(torch.int8), dim=1, stable=True)[:, :R]
    keep = torch.arange(R).unsqueeze(0) < cnt.unsqueeze(1)
    return torch.where(keep, order, torch.full_like(order, -1))


def personachat_collate_fn(records):
    """DataLoader collate: records are (client_id, record-dict)."""
    cids = torch.tensor([r[0] for r in records], dtype=torch.long)
    return (cids,) + collate([r[1] for r in records])


class FedPERSONA(FedDataset):
    """Utterance-level federated PersonaChat, natural client = personality."""

    def __init__(self, tokenizer, num_candidates, max_history, personality_permutations,
                 *args, **kwargs):
        self.tokenizer = tokenizer
        self.num_candidates = num_candidates
        self.max_history = max_history
        self.personality_permutations = personality_permutations
        super().__init__(*args, **kwargs)
        self._cache = {}
        if self.type == "val":
            with open(os.path.join(self.dataset_dir, "validation.json")) as f:
                self.raw_val_set = json.load(f)
            self._val_index = [(d, u) for d, dl in enumerate(self.raw_val_set)
                               for u in range(len(dl["utterances"]))]

    @property
    def special_ids(self):
        return self.tokenizer.convert_tokens_to_ids(SPECIAL_TOKENS)

    def prepare_datasets(self, download=False):
        raise FileNotFoundError(
            f"{self.stats_fn()} not found: split PersonaChat into the reference layout "
            "(client{i}.json, validation.json, stats.json) or use --synthetic")

    def _load_meta(self, train):
        with open(self.stats_fn()) as f:
            st = json.load(f)
        self.dialogs_per_client = np.array(st["dialogs_per_client"])
        self.train_utterances_per_dialog = np.array(st["train_utterances_per_dialog"])
        self.val_utterances_per_dialog = np.array(st["val_utterances_per_dialog"])
        cs = np.concatenate([[0], np.cumsum(self.dialogs_per_client)])
        self.images_per_client = np.array([self.train_utterances_per_dialog[cs[i]:cs[i + 1]].sum()
                                           for i in range(len(self.dialogs_per_client))])
        self.num_val_images = int(self.val_utterances_per_dialog.sum())

    @property
    def data_per_client(self):
        if self.do_iid:
            return super().data_per_client
        return self.images_per_client if self._num_clients in (None, len(self.images_per_client)) \
            else super().data_per_client

    def _tok(self, obj):
        if isinstance(obj, str):
            return self.tokenizer.convert_tokens_to_ids(self.tokenizer.tokenize(obj))
        return [self._tok(o) for o in obj]

    def _client(self, nat):
        if nat not in self._cache:
            with open(os.path.join(self.dataset_dir, f"client{nat}.json")) as f:
                raw = json.load(f)
            self._cache[nat] = [{"personality": self._tok(d["personality"]),
                                 "utterances": [{"history": self._tok(u["history"]),
                                                 "candidates": self._tok(u["candidates"])}
                                                for u in d["utterances"]]} for d in raw]
            if len(self._cache) > 4096:
                self._cache.pop(next(iter(self._cache)))
        return self._cache[nat]

    def _get_train_item(self, nat, idx_within_client):
        dialogs = self._client(nat)
        for d in dialogs:
            if idx_within_client < len(d["utterances"]):
                return self._record(d["personality"], d["utterances"][idx_within_client], True)
            idx_within_client -= len(d["utterances"])
        raise IndexError

    def _record(self, persona, utt, train):
        persona = list(persona)
        recs = []
        for _ in range(max(1, self.personality_permutations)):
            random.shuffle(persona)
            recs.append(utterance_to_inputs(persona, utt["history"], utt["candidates"],
                                            self.special_ids, self.num_candidates,
                                            self.max_history, train))
        return recs[-1] if len(recs) == 1 else recs

    def _get_val_item(self, idx):
        d, u = self._val_index[idx]
        dl = self.raw_val_set[d]
        utt = {"history": self._tok(dl["utterances"][u]["history"]),
               "candidates": self._tok(dl["utterances"][u]["candidates"])}
        return self._record(self._tok(dl["personality"]), utt, False)


def _hash64(key, ctr):
    """SplitMix64 of (key, counter): a counter-based generator, vectorised
    over ``ctr``."""
    with np.errstate(over="ignore"):
        z = (np.uint64(key) * np.uint64(0x9E3779B97F4A7C15)
             + np.asarray(ctr, dtype=np.uint64) * np.uint64(0xBF58476D1CE4E5B9))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


class SyntheticPersona(FedDataset):
    """PersonaChat-shaped token data built like the reference's records
    (/root/reference/CommEfficient/data_utils/fed_persona.py:245-258,330-358):
    clients = personalities with a few dialogs each; a persona of
    ``persona_sents`` (5) sentences; utterance u of a dialog sees the u-th
    history of that dialog -- the 2u+1 previous turns, truncated to the last
    ``2 * max_history + 1`` -- and ``num_candidates`` candidate replies (gold
    last).  Token ids < ``vocab`` and the 5 special tokens are
    ``vocab .. vocab+4`` (as after ``add_special_tokens_``).

    Length assumption (no PersonaChat copy is available here, so parity of
    the length distribution is unpinned): every sentence is 8..19 GPT-2 BPE
    tokens, uniform (mean 13.5, the typical length of a PersonaChat turn), so
    with max_history 2 the model input is ~70..240 tokens -- past the
    128-token short attention kernels, as real PersonaChat inputs are."""

    TEXTS = ("uniform", "bigram")
    BIGRAM_VOCAB, BIGRAM_FANOUT = 1024, 4

    def __init__(self, num_personalities=1000, dialogs_per_client=2, utterances_per_dialog=7,
                 num_candidates=2, max_history=2, vocab=50257, train=True, do_iid=False,
                 num_clients=None, seed=0, sent_len=(8, 20), n_val=500, persona_sents=5,
                 text="uniform"):
        """``text``: "uniform" -- i.i.d. uniform tokens (the throughput
        benches: nothing to learn beyond the special tokens); "bigram" -- a
        learnable language, the same for train and validation: 1,024 of the
        vocabulary's tokens, each followed by one of 4 fixed successors chosen
        uniformly (LM loss from ~ln 50257 = 10.8 at init down to ln 4 = 1.39
        once the chain is learnt; tests/test_drivers.py)."""
        assert text in self.TEXTS, text
        self.text = text
        if text == "bigram":
            lang = np.random.RandomState(seed * 7919 + 0xB16)
            self._sub = np.sort(lang.choice(vocab, self.BIGRAM_VOCAB, replace=False)).astype(np.int64)
            self._succ = lang.randint(0, self.BIGRAM_VOCAB, size=(self.BIGRAM_VOCAB, self.BIGRAM_FANOUT))
        self.num_candidates, self.max_history, self.vocab = num_candidates, max_history, vocab
        self._np, self._dpc, self._upd = num_personalities, dialogs_per_client, utterances_per_dialog
        self._n_val = n_val
        self._rng = np.random.RandomState(seed + (0 if train else 1))
        self._sent_len = sent_len
        super().__init__("", "PERSONA", None, do_iid, num_clients, train=train, seed=seed)
        self.special_ids = [vocab + i for i in range(5)]
        self._personas = [self._sents(persona_sents) for _ in range(num_personalities)]

    def _meta_ready(self):
        return True

    def _load_meta(self, train):
        self.images_per_client = np.full(self._np, self._dpc * self._upd)
        self.num_val_images = self._n_val

    def _walk(self, lens, start, choice):
        """Bigram sentences: sentence i starts at sub-vocabulary token start[i]
        and takes successor choice[i, t] at step t; returns token id lists."""
        L = int(max(lens))
        cur = np.asarray(start, dtype=np.int64) % self.BIGRAM_VOCAB
        seq = np.empty((len(lens), L), dtype=np.int64)
        seq[:, 0] = cur
        for t in range(1, L):
            cur = self._succ[cur, choice[:, t] % self.BIGRAM_FANOUT]
            seq[:, t] = cur
        ids = self._sub[seq]
        return [ids[i, :n].tolist() for i, n in enumerate(lens)]

    def _sents(self, n):
        lo, hi = self._sent_len
        if self.text == "bigram":
            lens = [self._rng.randint(lo, hi) for _ in range(n)]
            return self._walk(lens, self._rng.randint(0, self.BIGRAM_VOCAB, size=n),
                              self._rng.randint(0, self.BIGRAM_FANOUT, size=(n, hi)))
        return [self._rng.randint(0, self.vocab, size=self._rng.randint(lo, hi)).tolist()
                for _ in range(n)]

    def _rec(self, key, persona, train, u):
        """Deterministic record of item ``key``, utterance ``u`` of its dialog:
        every random number comes from one vectorised counter hash (a per-item
        RandomState took ~40 us to construct, the round's batch assembly ~15 ms
        at 32 items)."""
        lo, hi = self._sent_len
        n_hist = min(2 * int(u) + 1, 2 * self.max_history + 1)
        n_sent = n_hist + max(2, self.num_candidates)
        lens = lo + (_hash64(key, np.arange(1, n_sent + 1)) % np.uint64(hi - lo)).astype(np.int64)
        if self.text == "bigram":
            start = _hash64(key, np.arange(500, 500 + n_sent)).astype(np.int64) & 0xffff
            choice = (_hash64(key, np.arange(1000, 1000 + n_sent * hi)) % np.uint64(self.BIGRAM_FANOUT))
            sents = self._walk(lens.tolist(), start, choice.astype(np.int64).reshape(n_sent, hi))
        else:
            toks = (_hash64(key, np.arange(1000, 1000 + int(lens.sum()))) % np.uint64(self.vocab))
            toks = toks.astype(np.int64).tolist()
            sents, o = [], 0
            for n in lens.tolist():
                sents.append(toks[o:o + n])
                o += n
        return utterance_to_inputs(persona, sents[:n_hist], sents[n_hist:], self.special_ids,
                                   self.num_candidates, self.max_history, train)

    def _get_train_item(self, nat, idx_within_client):
        return self._rec(nat * 100003 + idx_within_client, self._personas[nat], True,
                         idx_within_client % self._upd)

    def _get_val_item(self, idx):
        return self._rec(10 ** 9 + idx, self._personas[idx % self._np], False, idx % self._upd)

    def __getitem__(self, idx):
        out = super().__getitem__(idx)
        return out[0], out[1]
