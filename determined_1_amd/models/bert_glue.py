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


class BertGLUETrial(det_torch.PyTorchTrial):
    """``BertPytorch`` of the reference's bert_glue_pytorch example."""

    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.seq_len = int(hp.get("max_seq_length", 128))
        cfg = BertEncoderConfig.from_hparams(hp)
        self.model = context.wrap_model(BertForSequenceClassification(cfg, int(hp.get("num_labels", 2))))
        no_decay = ("bias", "LayerNorm.weight", "_ln.weight")
        wd = float(hp.get("weight_decay", 0.0))
        groups = [
            {"params": [p for n, p in self.model.named_parameters() if not any(k in n for k in no_decay)], "weight_decay": wd},
            {"params": [p for n, p in self.model.named_parameters() if any(k in n for k in no_decay)], "weight_decay": 0.0},
        ]
        self.opt = context.wrap_optimizer(torch.optim.AdamW(groups, lr=float(hp.get("learning_rate", 2e-5)),
                                                            eps=float(hp.get("adam_epsilon", 1e-8))))
        total = int(hp.get("num_training_steps", 459))
        warm = int(hp.get("num_warmup_steps", 0))

        def lr_lambda(step: int) -> float:  # transformers.get_linear_schedule_with_warmup
            if step < warm:
                return float(step) / max(1, warm)
            return max(0.0, float(total - step) / max(1, total - warm))

        self.sched = context.wrap_lr_scheduler(torch.optim.lr_scheduler.LambdaLR(self.opt, lr_lambda),
                                               det_torch.LRScheduler.StepMode.STEP_EVERY_BATCH)
        amp = hp.get("amp", "O0")
        if amp and amp != "O0":
            self.model, self.opt = context.configure_apex_amp(self.model, self.opt, opt_level=amp)

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        ids, am, tt, labels = batch
        out = self.model(input_ids=ids, attention_mask=am, token_type_ids=tt, labels=labels)
        self.context.backward(out.loss)
        self.context.step_optimizer(self.opt)
        m = glue_pair_metrics(out.logits, labels)
        m["loss"] = out.loss
        return m

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        ids, am, tt, labels = batch
        out = self.model(input_ids=ids, attention_mask=am, token_type_ids=tt, labels=labels)
        m = glue_pair_metrics(out.logits, labels)
        m["validation_loss"] = out.loss
        return m

    def build_training_data_loader(self) -> det_torch.DataLoader:
        hp = self.context.get_hparams()
        ds = SyntheticGLUEPairs(int(hp.get("train_records", 3668)), self.seq_len, int(hp.get("vocab_size", 30522)))
        return det_torch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size(), num_workers=2,
                                    drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        hp = self.context.get_hparams()
        ds = SyntheticGLUEPairs(int(hp.get("validation_records", 408)), self.seq_len, int(hp.get("vocab_size", 30522)),
                                seed=1)
        return det_torch.DataLoader(ds, batch_size=self.context.get_per_slot_batch_size(), num_workers=2)
