"""BERT-base extractive QA (SQuAD 1.1 shape) PyTorchTrial: the 5th BASELINE config
("BERT-base SQuAD-shape PyTorchTrial slots_per_trial=8, aggregation_frequency>1 +
checkpoint/resume"), mirroring ``examples/nlp/bert_squad_pytorch/model_def.py`` of the reference
(AdamW, linear warmup/decay per batch, max_grad_norm clipping, global batch 96, seq 384).

The encoder is written for MI355X rather than taken from HuggingFace (``impl: hf`` still selects
the HF module for comparison): Q/K/V are one fused [3H, H] GEMM, attention is PyTorch SDPA (CK /
AOTriton flash kernels on ROCm) reading Q/K/V as strided views of the fused output, and every
Linear -> dropout -> +residual -> LayerNorm, Linear -> GELU and bias-gradient reduction runs on the
fused ``det_transformer.hip`` kernels (``determined_1_amd/ops/transformer.py``).  Parameter
initialisation and the forward math match ``transformers.BertForQuestionAnswering``;
``load_hf_state_dict`` maps HF checkpoints onto the fused layout (tests pin the two
implementations to the same outputs).  Weights are random-init bert-base-uncased geometry
(12 x 768, 12 heads) — no network for pretrained checkpoints; data is ``SyntheticSQuAD``.
"""
import math
from types import SimpleNamespace
from typing import Any, Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.synthetic import SyntheticSQuAD
from determined_1_amd.ops import transformer as tfops


class BertEncoderConfig:
    def __init__(self, vocab_size: int = 30522, hidden_size: int = 768, num_hidden_layers: int = 12,
                 num_attention_heads: int = 12, intermediate_size: int = 3072, hidden_dropout_prob: float = 0.1,
                 attention_probs_dropout_prob: float = 0.1, max_position_embeddings: int = 512,
                 type_vocab_size: int = 2, layer_norm_eps: float = 1e-12, initializer_range: float = 0.02,
                 pad_token_id: int = 0, hidden_act: str = "gelu") -> None:
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.intermediate_size = intermediate_size
        self.hidden_dropout_prob = hidden_dropout_prob
        self.attention_probs_dropout_prob = attention_probs_dropout_prob
        self.max_position_embeddings = max_position_embeddings
        self.type_vocab_size = type_vocab_size
        self.layer_norm_eps = layer_norm_eps
        self.initializer_range = initializer_range
        self.pad_token_id = pad_token_id
        if hidden_act not in ("gelu", "gelu_new"):
            raise ValueError(f"hidden_act {hidden_act!r}: the fused encoder implements gelu and gelu_new")
        self.hidden_act = hidden_act

    @classmethod
    def from_hparams(cls, hp: Dict[str, Any]) -> "BertEncoderConfig":
        return cls(hidden_size=int(hp.get("hidden_size", 768)), num_hidden_layers=int(hp.get("num_hidden_layers", 12)),
                   num_attention_heads=int(hp.get("num_attention_heads", 12)),
                   intermediate_size=int(hp.get("intermediate_size", 3072)),
                   vocab_size=int(hp.get("vocab_size", 30522)),
                   hidden_dropout_prob=float(hp.get("hidden_dropout_prob", 0.1)),
                   attention_probs_dropout_prob=float(hp.get("attention_probs_dropout_prob", 0.1)))


class _LN(nn.Module):
    """LayerNorm parameters (HF names ``weight``/``bias``); the math lives in the fused ops."""

    def __init__(self, h: int, eps: float) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(h))
        self.bias = nn.Parameter(torch.zeros(h))
        self.eps = eps


class _Dense(nn.Module):
    def __init__(self, fan_in: int, fan_out: int) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.empty(fan_out, fan_in))
        self.bias = nn.Parameter(torch.zeros(fan_out))


class BertEmbeddings(nn.Module):
    def __init__(self, c: BertEncoderConfig) -> None:
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden_size, padding_idx=c.pad_token_id)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = _LN(c.hidden_size, c.layer_norm_eps)
        self.p = c.hidden_dropout_prob

    def forward(self, input_ids: torch.Tensor, token_type_ids: Optional[torch.Tensor]) -> torch.Tensor:
        # one lookup-and-sum launch with a graph-safe backward on the GPU (ops/csrc/det_embed.hip)
        e = tfops.bert_embeddings(input_ids, token_type_ids, self.word_embeddings.weight,
                                  self.token_type_embeddings.weight, self.position_embeddings.weight,
                                  self.word_embeddings.padding_idx)
        e = tfops.layer_norm(e, self.LayerNorm.weight, self.LayerNorm.bias, self.LayerNorm.eps)
        return F.dropout(e, self.p, self.training)


class BertLayer(nn.Module):
    """attention (fused QKV GEMM + SDPA) -> Linear/dropout/+x/LN -> Linear+GELU -> Linear/dropout/+a/LN"""

    def __init__(self, c: BertEncoderConfig) -> None:
        super().__init__()
        H = c.hidden_size
        self.nh = c.num_attention_heads
        self.hd = H // c.num_attention_heads
        self.qkv = _Dense(H, 3 * H)
        self.attn_out = _Dense(H, H)
        self.attn_ln = _LN(H, c.layer_norm_eps)
        self.ffn_in = _Dense(H, c.intermediate_size)
        self.ffn_out = _Dense(c.intermediate_size, H)
        self.ffn_ln = _LN(H, c.layer_norm_eps)
        self.p = c.hidden_dropout_prob
        self.p_attn = c.attention_probs_dropout_prob
        self.gelu_approx = "tanh" if c.hidden_act == "gelu_new" else "none"

    def forward(self, x: torch.Tensor, mask_bias: Optional[torch.Tensor],
                acc: Optional[tfops.SharedWeightGrads] = None) -> torch.Tensor:
        """``acc``: weight-gradient accumulator when this layer is applied repeatedly (ALBERT)."""
        B, S, H = x.shape
        # x and a are each read by a Linear and as a residual: the two gradients meet in one GEMM
        lx, la = tfops.ResidualGradLink(), tfops.ResidualGradLink()
        qkv = tfops.linear(x, self.qkv.weight, self.qkv.bias, acc=acc, link=lx)  # [B, S, 3H]
        ctx = tfops.qkv_self_attention(qkv, self.nh, mask_bias, self.p_attn, self.training)
        a = tfops.linear_dropout_add_layernorm(ctx, self.attn_out.weight, self.attn_out.bias, x, self.attn_ln.weight,
                                               self.attn_ln.bias, self.p, self.attn_ln.eps, self.training, acc=acc,
                                               link=lx)
        i = tfops.linear_gelu(a, self.ffn_in.weight, self.ffn_in.bias, self.gelu_approx, acc=acc, link=la)
        return tfops.linear_dropout_add_layernorm(i, self.ffn_out.weight, self.ffn_out.bias, a, self.ffn_ln.weight,
                                                  self.ffn_ln.bias, self.p, self.ffn_ln.eps, self.training, acc=acc,
                                                  link=la)


class BertForQA(nn.Module):
    """``transformers.BertForQuestionAnswering`` semantics on the fused MI355X encoder."""

    def __init__(self, c: BertEncoderConfig) -> None:
        super().__init__()
        self.config = c
        self.embeddings = BertEmbeddings(c)
        self.layers = nn.ModuleList(BertLayer(c) for _ in range(c.num_hidden_layers))
        self.qa_outputs = nn.Linear(c.hidden_size, 2)
        self.apply(self._init)

    def _init(self, m: nn.Module) -> None:  # HF BertPreTrainedModel._init_weights
        std = self.config.initializer_range
        if isinstance(m, (nn.Linear, _Dense)):
            nn.init.normal_(m.weight, 0.0, std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)
            if m.padding_idx is not None:
                with torch.no_grad():
                    m.weight[m.padding_idx].zero_()

    def forward(self, input_ids: torch.Tensor, token_type_ids: Optional[torch.Tensor] = None,
                attention_mask: Optional[torch.Tensor] = None, start_positions: Optional[torch.Tensor] = None,
                end_positions: Optional[torch.Tensor] = None) -> SimpleNamespace:
        x = self.embeddings(input_ids, token_type_ids)
        mask_bias = None
        if attention_mask is not None:  # additive [B, 1, 1, S] like HF's extended attention mask
            mask_bias = (1.0 - attention_mask[:, None, None, :].to(x.dtype)) * torch.finfo(x.dtype).min
        for layer in self.layers:
            x = layer(x, mask_bias)
        logits = self.qa_outputs(x)
        start_logits, end_logits = (t.squeeze(-1).contiguous() for t in logits.split(1, dim=-1))
        loss = None
        if start_positions is not None and end_positions is not None:
            ignored = start_logits.shape[1]
            s = start_positions.clamp(0, ignored)
            e = end_positions.clamp(0, ignored)
            loss = (F.cross_entropy(start_logits.float(), s, ignore_index=ignored)
                    + F.cross_entropy(end_logits.float(), e, ignore_index=ignored)) / 2
        return SimpleNamespace(loss=loss, start_logits=start_logits, end_logits=end_logits)


def hf_encoder_state(sd: Dict[str, torch.Tensor], num_layers: int) -> Dict[str, torch.Tensor]:
    """Embeddings + encoder layers of a ``transformers`` BERT state dict in the fused layout."""
    out = {}
    for k, v in sd.items():
        if k.startswith("bert.embeddings."):
            if "position_ids" in k or "token_type_ids" in k:
                continue
            out[k[len("bert."):]] = v
    for i in range(num_layers):
        pre = f"bert.encoder.layer.{i}."
        for t in ("weight", "bias"):
            out[f"layers.{i}.qkv.{t}"] = torch.cat([sd[pre + f"attention.self.{m}.{t}"] for m in ("query", "key", "value")])
            out[f"layers.{i}.attn_out.{t}"] = sd[pre + f"attention.output.dense.{t}"]
            out[f"layers.{i}.attn_ln.{t}"] = sd[pre + f"attention.output.LayerNorm.{t}"]
            out[f"layers.{i}.ffn_in.{t}"] = sd[pre + f"intermediate.dense.{t}"]
            out[f"layers.{i}.ffn_out.{t}"] = sd[pre + f"output.dense.{t}"]
            out[f"layers.{i}.ffn_ln.{t}"] = sd[pre + f"output.LayerNorm.{t}"]
    return out


def load_hf_state_dict(model: BertForQA, sd: Dict[str, torch.Tensor]) -> None:
    """Load a ``transformers`` BertForQuestionAnswering state dict into the fused layout."""
    out = hf_encoder_state(sd, model.config.num_hidden_layers)
    out.update({k: v for k, v in sd.items() if k.startswith("qa_outputs.")})
    model.load_state_dict(out)


def bert_config(hp: Dict[str, Any]) -> Any:
    from transformers import BertConfig

    return BertConfig(
        hidden_size=int(hp.get("hidden_size", 768)),
        num_hidden_layers=int(hp.get("num_hidden_layers", 12)),
        num_attention_heads=int(hp.get("num_attention_heads", 12)),
        intermediate_size=int(hp.get("intermediate_size", 3072)),
        max_position_embeddings=512,
        attn_implementation="sdpa",
    )
