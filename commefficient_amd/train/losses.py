"""Loss functions in the engine's per-example form.

``loss_fn(model, inputs: tuple, targets, args) -> (per_example_loss[n], [metric[n], ...])``

The engine sums per-example losses for merged clients and averages them per
client otherwise, so one definition serves both paths.  CV: cross-entropy +
top-1 correctness (reference cv_train.py:31-84 ``compute_loss_ce`` /
``Correct``).  GPT-2: see models/gpt2.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.nn import cross_entropy_correct
from ..ops import transformer as _tx


class _unpacked_sequences:
    """HF transformers (>= 4.5x) checks every causal-mask forward without an
    attention mask for "packed" sequences (several sequences in one row, told
    apart by position-id jumps) with ``(mask[:, -1] == 0).all()`` -- a
    device->host sync in the middle of each forward, which stalls the host's
    launch queue (GPT-2 PersonaChat round: ~5 ms of GPU idle per round).  Our
    rows are single sequences (position ids 0..L-1), for which that check
    returns None; this context skips it for the duration of our own forward."""

    def __enter__(self):
        try:
            from transformers import masking_utils as mu
        except ImportError:  # older transformers: no such check
            self.mu = None
            return self
        self.mu = mu
        self.orig = getattr(mu, "find_packed_sequence_indices", None)
        if self.orig is not None:
            mu.find_packed_sequence_indices = lambda position_ids: None
        return self

    def __exit__(self, *exc):
        if self.mu is not None and self.orig is not None:
            self.mu.find_packed_sequence_indices = self.orig
        return False


def gpt2_hidden_states(m, input_ids, token_type_ids, args=None, lengths=None):
    """Final hidden states of the double-heads model's transformer: the native
    junction kernels (ops/transformer.py; with host ``lengths`` only the real
    tokens run through the token-wise ops) unless ``--transformer hf`` or the
    config is outside what they cover (then the HF module forward)."""
    tr = m.transformer
    if getattr(args, "transformer", "native") == "native" and _tx.native_ok(tr, input_ids):
        return _tx.gpt2_hidden(tr, input_ids, token_type_ids,
                               lengths if getattr(args, "unpad", "on") == "on" else None)
    with _unpacked_sequences():
        return tr(input_ids=input_ids, token_type_ids=token_type_ids, use_cache=False)[0]


def cv_loss(model, inputs, targets, args):
    fused = getattr(model, "loss", None)
    if callable(fused) and len(inputs) == 1:
        # model-provided head + loss (ResNet-9: one native kernel each way)
        per_ex, correct = fused(inputs[0], targets)
        return per_ex, [correct]
    logits = model(*inputs)
    # one fused kernel on GPU (loss, correctness and the logits gradient)
    per_ex, correct = cross_entropy_correct(logits, targets)
    return per_ex, [correct]


def gpt2_loss_train(model, inputs, targets, args, groups=None):
    """inputs = (input_ids[B,C,L], mc_token_ids[B,C], lm_labels[B,C,L], token_type_ids[B,C,L]),
    targets = mc_labels[B].  Per-example ``lm_coef*lm + mc_coef*mc`` whose mean
    over a client's examples is the reference objective (gpt2_train.py:88-99):
    HF's lm loss is ONE token-weighted mean over every labelled token of the
    client's (micro)batch, so example e carries ``n_g * tokloss_e / ntok_g``
    (n_g examples and ntok_g labelled tokens of its client g in this call).
    ``groups``: per-example client slot of a merged multi-client batch (None:
    one client).  With --microbatch_size the token mean is per microbatch, as
    in the reference (fed_worker.py:266-287)."""
    input_ids, mc_token_ids, lm_labels, token_type_ids = inputs[:4]
    m = model.model if hasattr(model, "model") and not hasattr(model, "transformer") else model
    B = input_ids.shape[0]
    if len(inputs) > 4 and hasattr(m, "transformer") and hasattr(m, "multiple_choice_head"):
        # LM head only at the labelled positions (data/fed_persona.py
        # label_positions): same loss, ~1/17 of the vocabulary GEMM + softmax
        tok_sum, ntok, mc_logits = _lm_at_labels(m, input_ids, mc_token_ids, lm_labels,
                                                  token_type_ids, inputs[4], args,
                                                  inputs[5] if len(inputs) > 5 else None)
    else:
        lm_logits, mc_logits = _double_heads(m, input_ids, token_type_ids, mc_token_ids, args)
        shift_logits = lm_logits[..., :-1, :].float()
        shift_labels = lm_labels[..., 1:]
        tok = F.cross_entropy(shift_logits.reshape(-1, shift_logits.size(-1)),
                              shift_labels.reshape(-1), ignore_index=-100,
                              reduction="none").view(B, -1)
        mask = (shift_labels.reshape(B, -1) != -100).float()
        tok_sum = (tok * mask).sum(1)
        ntok = mask.sum(1)
    lm = token_weighted(tok_sum, ntok, groups)
    # (one native kernel each way on GPU: loss, top-1 and the logits gradient)
    mc, acc = cross_entropy_correct(mc_logits.float(), targets)
    return args.lm_coef * lm + args.mc_coef * mc, [acc]


def _double_heads(m, input_ids, token_type_ids, mc_token_ids, args, last_only=False):
    """(lm_logits, mc_logits) of HF's double-heads forward (``last_only``: LM
    logits of the last candidate only)."""
    if hasattr(m, "transformer") and hasattr(m, "multiple_choice_head"):
        hid = gpt2_hidden_states(m, input_ids, token_type_ids, args)
        mc_logits = m.multiple_choice_head(hid, mc_token_ids).squeeze(-1)
        lm_logits = m.lm_head(hid[:, -1] if last_only else hid)
        return lm_logits, mc_logits
    with _unpacked_sequences():
        out = m(input_ids=input_ids, token_type_ids=token_type_ids, mc_token_ids=mc_token_ids,
                use_cache=False)
    return (out.logits[:, -1] if last_only else out.logits), out.mc_logits


_NATIVE_LM_CE = [True]  # (tests compare against the stock cross-entropy)


def _lm_at_labels(m, input_ids, mc_token_ids, lm_labels, token_type_ids, lm_pos, args=None,
                  lengths=None):
    """(per-example sum of LM token losses, labelled-token count, mc logits)
    with the LM head evaluated only at ``lm_pos`` [B, R] (-1 = pad)."""
    hid = gpt2_hidden_states(m, input_ids, token_type_ids, args, lengths)  # [B, C, L, H]
    B, C, L, H = hid.shape
    mc_logits = m.multiple_choice_head(hid, mc_token_ids).squeeze(-1)
    valid = lm_pos >= 0
    p = lm_pos.clamp_min(0)
    h = torch.gather(hid.reshape(B, C * L, H), 1, p.unsqueeze(-1).expand(-1, -1, H))
    logits = _tx.lm_head(m, h)                                           # [B, R, V]
    tgt = torch.gather(lm_labels.reshape(B, C * L), 1, (p + 1).clamp_max(C * L - 1))
    tgt = torch.where(valid, tgt, torch.full_like(tgt, -100))
    if logits.is_cuda and _NATIVE_LM_CE[0]:
        # one native pass over the bf16 logits: loss, and the unit gradient for
        # backward (rows labelled -100: zero), no fp32 copy of the logits
        tok = cross_entropy_correct(logits.reshape(-1, logits.shape[-1]),
                                    tgt.reshape(-1).contiguous())[0].view(B, -1)
    else:
        tok = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), tgt.reshape(-1),
                              ignore_index=-100, reduction="none").view(B, -1)
    mask = (tgt != -100).float()
    return (tok * mask).sum(1), mask.sum(1), mc_logits


def token_weighted(tok_sum: torch.Tensor, ntok: torch.Tensor, groups=None) -> torch.Tensor:
    """Per-example terms whose per-group MEAN is sum(tok_sum)/sum(ntok) of the group."""
    B = tok_sum.shape[0]
    if groups is None:
        return tok_sum * (B / ntok.sum().clamp_min(1.0))
    # a client's examples are contiguous: local ids 0.. by run (no host sync)
    g = groups.long()
    g = torch.cat([g.new_zeros(1), (g[1:] != g[:-1]).long()]).cumsum(0) if B else g
    ng = torch.zeros(max(B, 1), device=tok_sum.device)
    tg = torch.zeros_like(ng)
    ng.index_add_(0, g, torch.ones_like(ntok))
    tg.index_add_(0, g, ntok.detach())
    return tok_sum * (ng[g] / tg[g].clamp_min(1.0))


def gpt2_loss_val(model, inputs, targets, args):
    """Validation: (nll of the LM on the gold reply, mc accuracy) (gpt2_train.py:55-87)."""
    input_ids, mc_token_ids, lm_labels, token_type_ids = inputs[:4]
    m = model.model if hasattr(model, "model") and not hasattr(model, "transformer") else model
    # the gold candidate is the last one (PERSONA collate order)
    lm_last, mc_logits = _double_heads(m, input_ids, token_type_ids, mc_token_ids, args,
                                       last_only=True)
    B = input_ids.shape[0]
    lg = lm_last[:, :-1, :].float()
    lb = lm_labels[:, -1, 1:]
    tok = F.cross_entropy(lg.reshape(-1, lg.size(-1)), lb.reshape(-1), ignore_index=-100,
                          reduction="none").view(B, -1)
    mask = (lb != -100).float()
    nll = (tok * mask).sum(1) / mask.sum(1).clamp_min(1.0)
    acc = (mc_logits.argmax(-1) == targets).float()
    return nll, [acc]
