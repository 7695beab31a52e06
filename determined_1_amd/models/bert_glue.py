"""BERT sentence-pair classification (GLUE MRPC shape) PyTorchTrial on the fused MI355X encoder.

Mirrors the reference's ``examples/nlp/bert_glue_pytorch`` (``model_def.py`` ``BertPytorch``:
bert-base, AdamW with linear warmup/decay stepped per batch, seq 128, global batch 24 (192 on 8
slots), per-batch acc / F1 metrics as ``glue_compute_metrics('mrpc')``).  The model follows
``transformers.BertForSequenceClassification`` (pooler = tanh(Linear(h[CLS])), dropout,
classifier; cross-entropy, or MSE for a single regression output) on the same fused encoder as
``models/bert.py``; ``load_hf_state_dict`` maps HF checkpoints and the CPU tests pin the outputs.
Random-init weights and ``SyntheticGLUEPairs`` data (no network for bert-base-uncased / GLUE).
"""
from types import SimpleNamespace
from typing import Any, Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.bert import BertEmbeddings, BertEncoderConfig, BertLayer, _Dense, hf_encoder_state
from determined_1_amd.models.synthetic import SyntheticGLUEPairs
from determined_1_amd.ops import transformer as tfops


class BertForSequenceClassification(nn.Module):
    def __init__(self, c: BertEncoderConfig, num_labels: int = 2) -> None:
        super().__init__()
        self.config = c
        self.num_labels = num_labels
        self.embeddings = BertEmbeddings(c)
        self.layers = nn.ModuleList(BertLayer(c) for _ in range(c.num_hidden_layers))
        self.pooler = _Dense(c.hidden_size, c.hidden_size)
        self.p = c.hidden_dropout_prob
        self.classifier = nn.Linear(c.hidden_size, num_labels)
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

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                token_type_ids: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None) -> SimpleNamespace:
        x = self.embeddings(input_ids, token_type_ids)
        mask_bias = None
        if attention_mask is not None:
            mask_bias = (1.0 - attention_mask[:, None, None, :].to(x.dtype)) * torch.finfo(x.dtype).min
        for layer in self.layers:
            x = layer(x, mask_bias)
        pooled = torch.tanh(tfops.linear(x[:, 0].contiguous(), self.pooler.weight, self.pooler.bias))
        logits = self.classifier(F.dropout(pooled, self.p, self.training))
        loss = None
        if labels is not None:
            if self.num_labels == 1:
                loss = F.mse_loss(logits.squeeze(-1).float(), labels.float())
            else:
                loss = F.cross_entropy(logits.float(), labels)
        return SimpleNamespace(loss=loss, logits=logits)


def load_hf_state_dict(model: BertForSequenceClassification, sd: Dict[str, torch.Tensor]) -> None:
    """Load a ``transformers`` BertForSequenceClassification state dict into the fused layout."""
    out = hf_encoder_state(sd, model.config.num_hidden_layers)
    out["pooler.weight"] = sd["bert.pooler.dense.weight"]
    out["pooler.bias"] = sd["bert.pooler.dense.bias"]
    out["classifier.weight"] = sd["classifier.weight"]
    out["classifier.bias"] = sd["classifier.bias"]
    model.load_state_dict(out)


def glue_pair_metrics(logits: torch.Tensor, labels: torch.Tensor) -> Dict[str, torch.Tensor]:
    """``glue_compute_metrics('mrpc')`` per batch: accuracy, F1 of the positive class, their mean."""
    preds = logits.argmax(-1)
    acc = (preds == labels).float().mean()
    tp = ((preds == 1) & (labels == 1)).sum().float()
    fp = ((preds == 1) & (labels == 0)).sum().float()
    fn = ((preds == 0) & (labels == 1)).sum().float()
    f1 = 2 * tp / (2 * tp + fp + fn).clamp(min=1.0)
    return {"acc": acc, "f1": f1, "acc_and_f1": (acc + f1) / 2}
