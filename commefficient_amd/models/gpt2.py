"""GPT-2 / OpenAI-GPT double-heads models for PersonaChat-style federated training.

The reference loads ``pytorch_transformers.GPT2DoubleHeadsModel`` (LM head tied
to ``wte`` + multiple-choice head) and adds 5 special tokens
(/root/reference/CommEfficient/gpt2_train.py:4-6,26-32,101-112,262-273), giving
124,444,417 trainable parameters.  Here the same HF ``transformers``
architecture is built from its config with random init (no network, no
pretrained checkpoints in this environment), with SDPA attention so the
attention runs on the ROCm fused kernels.  The training loss matches
gpt2_train.py:88-99 (``lm_coef * lm + mc_coef * mc``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

SPECIAL_TOKENS = ["<bos>", "<eos>", "<speaker1>", "<speaker2>", "<pad>"]
ATTR_TO_SPECIAL_TOKEN = {"bos_token": "<bos>", "eos_token": "<eos>", "pad_token": "<pad>",
                         "additional_special_tokens": ["<speaker1>", "<speaker2>"]}


def build_double_heads(model_checkpoint: str = "gpt2", n_special: int = 5, n_layer=None,
                       n_embd=None, n_head=None, n_positions=None):
    import os
    from transformers import (GPT2Config, GPT2DoubleHeadsModel, OpenAIGPTConfig,
                              OpenAIGPTDoubleHeadsModel)
    is_gpt2 = "gpt2" in model_checkpoint
    if os.path.isdir(model_checkpoint):  # a local HF directory (e.g. --finetune)
        cls = GPT2DoubleHeadsModel if is_gpt2 else OpenAIGPTDoubleHeadsModel
        return cls.from_pretrained(model_checkpoint)
    cfg = GPT2Config() if is_gpt2 else OpenAIGPTConfig()
    for k, v in (("n_layer", n_layer), ("n_embd", n_embd), ("n_head", n_head),
                 ("n_positions", n_positions)):
        if v is not None:
            setattr(cfg, k, v)
    if is_gpt2:  # (HF's OpenAI-GPT has no SDPA attention: it keeps the eager one)
        try:
            cfg._attn_implementation = "sdpa"
        except Exception:
            pass
    if is_gpt2 and cfg.activation_function == "gelu_new":
        # the same tanh-approximation GELU as one fused kernel each way
        # (torch's gelu(approximate="tanh")) instead of HF's ~8 elementwise ops
        cfg.activation_function = "gelu_pytorch_tanh"
    model = (GPT2DoubleHeadsModel if is_gpt2 else OpenAIGPTDoubleHeadsModel)(cfg)
    if n_special:
        model.resize_token_embeddings(cfg.vocab_size + n_special, mean_resizing=False)
    return model


class GPT2DoubleHeads(nn.Module):
    """Registry wrapper so ``--model GPT2DoubleHeads`` works like the CV models."""

    def __init__(self, model_checkpoint="gpt2", **kw):
        super().__init__()
        self.model = build_double_heads(model_checkpoint, **{k: v for k, v in kw.items()
                                                             if k in ("n_layer", "n_embd",
                                                                      "n_head", "n_positions",
                                                                      "n_special")})

    def forward(self, *a, **kw):
        return self.model(*a, **kw)

    def save_pretrained(self, d):
        self.model.save_pretrained(d)


def double_heads_loss(model, batch, lm_coef=1.0, mc_coef=1.0):
    """(loss, lm_loss, mc_loss, mc_correct_frac) for one PersonaChat batch
    ``(input_ids[B,C,L], mc_token_ids[B,C], lm_labels[B,C,L], mc_labels[B], token_type_ids[B,C,L])``."""
    input_ids, mc_token_ids, lm_labels, mc_labels, token_type_ids = batch
    m = model.model if isinstance(model, GPT2DoubleHeads) else model
    out = m(input_ids=input_ids, token_type_ids=token_type_ids, mc_token_ids=mc_token_ids)
    lm_logits, mc_logits = out.logits, out.mc_logits
    # shift for next-token prediction; -100 labels are ignored (pad / persona)
    shift_logits = lm_logits[..., :-1, :].contiguous()
    shift_labels = lm_labels[..., 1:].contiguous()
    lm_loss = F.cross_entropy(shift_logits.view(-1, shift_logits.size(-1)).float(),
                              shift_labels.view(-1), ignore_index=-100)
    mc_loss = F.cross_entropy(mc_logits.float(), mc_labels)
    acc = (mc_logits.argmax(dim=-1) == mc_labels).float().mean()
    return lm_coef * lm_loss + mc_coef * mc_loss, lm_loss, mc_loss, acc
