"""ALBERT-xxlarge-v2 SQuAD 2.0 fine-tuning trial (reference examples/nlp/albert_squad_pytorch):
the networks and helpers come from the ``determined_1_amd.models.albert`` library  Synthetic SQuAD-shaped features (no network here).

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
from typing import Any, Dict, Optional

import torch

from determined_1_amd.models.synthetic import SyntheticSQuAD
from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.albert import AlbertConfig, AlbertForQA, XXLARGE_V2


class AlbertSQuADTrial(det_torch.PyTorchTrial):
    """``AlbertSQuADPyTorch`` (reference ``examples/nlp/albert_squad_pytorch/model_def.py``):
    AdamW (weight_decay 0, eps 1e-8), linear warmup then linear decay per batch, max_grad_norm."""

    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.seq_len = int(hp.get("max_seq_length", 384))
        self.model = context.wrap_model(AlbertForQA(AlbertConfig.from_hparams(hp)))
        no_decay = ("bias", "LayerNorm.weight", "_ln.weight")
        wd = float(hp.get("weight_decay", 0.0))
        groups = [
            {"params": [p for n, p in self.model.named_parameters() if not any(k in n for k in no_decay)], "weight_decay": wd},
            {"params": [p for n, p in self.model.named_parameters() if any(k in n for k in no_decay)], "weight_decay": 0.0},
        ]
        self.opt = context.wrap_optimizer(torch.optim.AdamW(groups, lr=float(hp.get("learning_rate", 5e-5)),
                                                            eps=float(hp.get("adam_epsilon", 1e-8))))
        total = int(hp.get("num_training_steps", 16500))
        warm = int(hp.get("num_warmup_steps", 1620))

        def lr_lambda(step: int) -> float:
            if step < warm:
                return float(step) / max(1, warm)
            return max(0.0, float(total - step) / max(1, total - warm))

        self.sched = context.wrap_lr_scheduler(torch.optim.lr_scheduler.LambdaLR(self.opt, lr_lambda),
                                               det_torch.LRScheduler.StepMode.STEP_EVERY_BATCH)
        amp = hp.get("amp", "O2")
        if amp and amp != "O0":
            self.model, self.opt = context.configure_apex_amp(self.model, self.opt, opt_level=amp)
        self.max_grad_norm = float(hp.get("max_grad_norm", 1.0))

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        ids, tt, am, s, e = batch
        out = self.model(input_ids=ids, token_type_ids=tt, attention_mask=am, start_positions=s, end_positions=e)
        self.context.backward(out.loss)
        self.context.step_optimizer(
            self.opt, clip_grads=det_torch.ClipGradsNorm(self.max_grad_norm) if self.max_grad_norm > 0 else None)
        return {"loss": out.loss}

    def evaluate_batch(self, batch: Any) -> Dict[str, Any]:
        ids, tt, am, s, e = batch
        out = self.model(input_ids=ids, token_type_ids=tt, attention_mask=am)
        ps = out.start_logits.argmax(-1)
        pe = out.end_logits.argmax(-1)
        exact = ((ps == s) & (pe == e)).float().mean()
        inter = (torch.minimum(pe, e) - torch.maximum(ps, s) + 1).clamp(min=0).float()
        plen = (pe - ps + 1).clamp(min=1).float()
        glen = (e - s + 1).float()
        return {"exact_match": exact, "f1": (2 * inter / (plen + glen)).mean()}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        n = int(self.context.get_hparams().get("train_records", 132198))
        vocab = int(self.context.get_hparams().get("vocab_size", XXLARGE_V2["vocab_size"]))
        return det_torch.DataLoader(SyntheticSQuAD(n, self.seq_len, vocab_size=vocab),
                                    batch_size=self.context.get_per_slot_batch_size(), num_workers=2, drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        n = int(self.context.get_hparams().get("validation_records", 512))
        vocab = int(self.context.get_hparams().get("vocab_size", XXLARGE_V2["vocab_size"]))
        return det_torch.DataLoader(SyntheticSQuAD(n, self.seq_len, vocab_size=vocab, seed=1),
                                    batch_size=self.context.get_per_slot_batch_size(), num_workers=2)



AlbertSQuADPyTorch = AlbertSQuADTrial  # the reference example's class name
