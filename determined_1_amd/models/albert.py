"""ALBERT (xxlarge-v2 geometry) extractive QA PyTorchTrial on the fused MI355X encoder.

Mirrors the reference's ``examples/nlp/albert_squad_pytorch`` (``model_def.py`` ``AlbertSQuADPyTorch``;
``distributed_8gpu.yaml``: albert-xxlarge-v2, seq 384, global batch 16, aggregation_frequency 3,
AdamW with linear warmup/decay, max_grad_norm 1.0).  That example carries the reference's only
published throughput numbers (``README.md:25-29``: 2 examples/s on one V100-16GB, 15.8 on 8,
92.75 on 64), which ``scripts/bench_albert.py`` measures against.

Architecture (``transformers.AlbertForQuestionAnswering`` semantics, ``load_hf_state_dict`` maps
HF checkpoints onto this layout and the CPU tests pin both to the same outputs):
  * factorised embeddings: word/position/token-type tables of width E=128, LayerNorm(E), then one
    ``embedding_hidden_mapping_in`` Linear E -> H;
  * ONE transformer layer (fused QKV GEMM, MFMA attention, Linear+dropout+residual+LayerNorm and
    Linear+tanh-GELU on ``det_transformer.hip``) applied ``num_hidden_layers`` times with shared
    weights — the 12 per-use weight gradients accumulate in one buffer through the dW GEMMs
    themselves (``tfops.SharedWeightGrads``: beta = 1, no elementwise sums), so each shared
    parameter produces one gradient per backward and lands in the arena / all-reduce bucket once;
  * QA head Linear(H, 2).
Weights are random-init (no network for pretrained checkpoints); data is ``SyntheticSQuAD``.
"""
from types import SimpleNamespace
from typing import Any, Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.bert import BertEncoderConfig, BertLayer, _LN
from determined_1_amd.models.synthetic import SyntheticSQuAD
from determined_1_amd.ops import transformer as tfops

# albert-xxlarge-v2 config.json geometry
XXLARGE_V2 = dict(vocab_size=30000, embedding_size=128, hidden_size=4096, num_hidden_layers=12,
                  num_attention_heads=64, intermediate_size=16384, hidden_act="gelu_new",
                  hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


class AlbertConfig(BertEncoderConfig):
    def __init__(self, embedding_size: int = 128, **kw: Any) -> None:
        kw.setdefault("vocab_size", 30000)
        kw.setdefault("hidden_act", "gelu_new")
        super().__init__(**kw)
        self.embedding_size = embedding_size

    @classmethod
    def from_hparams(cls, hp: Dict[str, Any]) -> "AlbertConfig":
        c = dict(XXLARGE_V2)
        for k in c:
            if k in hp:
                c[k] = type(c[k])(hp[k])
        return cls(**c)


class AlbertEmbeddings(nn.Module):
    def __init__(self, c: AlbertConfig) -> None:
        super().__init__()
        E = c.embedding_size
        self.word_embeddings = nn.Embedding(c.vocab_size, E, padding_idx=c.pad_token_id)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, E)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, E)
        self.LayerNorm = _LN(E, c.layer_norm_eps)
        self.p = c.hidden_dropout_prob

    def forward(self, input_ids: torch.Tensor, token_type_ids: Optional[torch.Tensor]) -> torch.Tensor:
        S = input_ids.shape[1]
        pos = torch.arange(S, device=input_ids.device)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        e = self.word_embeddings(input_ids) + self.token_type_embeddings(token_type_ids) + self.position_embeddings(pos)
        e = tfops.layer_norm(e, self.LayerNorm.weight, self.LayerNorm.bias, self.LayerNorm.eps)
        return F.dropout(e, self.p, self.training)


class AlbertForQA(nn.Module):
    """``transformers.AlbertForQuestionAnswering`` semantics (one layer group, inner_group_num 1)."""

    def __init__(self, c: AlbertConfig) -> None:
        super().__init__()
        self.config = c
        self.embeddings = AlbertEmbeddings(c)
        self.embedding_hidden_mapping_in = nn.Linear(c.embedding_size, c.hidden_size)
        self.layer = BertLayer(c)  # shared across all num_hidden_layers applications
        self.qa_outputs = nn.Linear(c.hidden_size, 2)
        self.apply(self._init)

    def _init(self, m: nn.Module) -> None:  # HF AlbertPreTrainedModel._init_weights
        std = self.config.initializer_range
        if isinstance(m, nn.Linear) or type(m).__name__ == "_Dense":
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
        e = self.embeddings(input_ids, token_type_ids)
        x = tfops.linear(e, self.embedding_hidden_mapping_in.weight, self.embedding_hidden_mapping_in.bias)
        mask_bias = None
        if attention_mask is not None:
            mask_bias = (1.0 - attention_mask[:, None, None, :].to(x.dtype)) * torch.finfo(x.dtype).min
        acc = tfops.SharedWeightGrads()  # one dW buffer per shared weight, accumulated by GEMM beta=1
        for _ in range(self.config.num_hidden_layers):
            x = self.layer(x, mask_bias, acc)
        logits = self.qa_outputs(x)
        start_logits, end_logits = (t.squeeze(-1).contiguous() for t in logits.split(1, dim=-1))
        loss = None
        if start_positions is not None and end_positions is not None:
            ignored = start_logits.shape[1]
            s = start_positions.clamp(0, ignored)
            e2 = end_positions.clamp(0, ignored)
            loss = (F.cross_entropy(start_logits.float(), s, ignore_index=ignored)
                    + F.cross_entropy(end_logits.float(), e2, ignore_index=ignored)) / 2
        return SimpleNamespace(loss=loss, start_logits=start_logits, end_logits=end_logits)


def load_hf_state_dict(model: AlbertForQA, sd: Dict[str, torch.Tensor]) -> None:
    """Load a ``transformers`` AlbertForQuestionAnswering state dict into the fused layout."""
    out = {}
    for k, v in sd.items():
        if k.startswith("albert.embeddings."):
            if "position_ids" in k or "token_type_ids" in k:
                continue
            out[k[len("albert."):]] = v
        elif k.startswith("albert.encoder.embedding_hidden_mapping_in."):
            out[k[len("albert.encoder."):]] = v
        elif k.startswith("qa_outputs."):
            out[k] = v
    pre = "albert.encoder.albert_layer_groups.0.albert_layers.0."
    for t in ("weight", "bias"):
        out[f"layer.qkv.{t}"] = torch.cat([sd[pre + f"attention.{m}.{t}"] for m in ("query", "key", "value")])
        out[f"layer.attn_out.{t}"] = sd[pre + f"attention.dense.{t}"]
        out[f"layer.attn_ln.{t}"] = sd[pre + f"attention.LayerNorm.{t}"]
        out[f"layer.ffn_in.{t}"] = sd[pre + f"ffn.{t}"]
        out[f"layer.ffn_out.{t}"] = sd[pre + f"ffn_output.{t}"]
        out[f"layer.ffn_ln.{t}"] = sd[pre + f"full_layer_layer_norm.{t}"]
    model.load_state_dict(out)
