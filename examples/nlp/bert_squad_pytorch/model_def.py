"""BERT-base SQuAD fine-tuning trial (reference examples/nlp/bert_squad_pytorch): see
determined_1_amd/models/bert.py.

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
from typing import Any, Dict, Optional

import torch

from determined_1_amd.models.synthetic import SyntheticSQuAD
from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.bert import BertEncoderConfig, BertForQA, bert_config


class BertSQuADTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.seq_len = int(hp.get("max_seq_length", 384))
        if hp.get("impl", "native") == "hf":
            from transformers import BertForQuestionAnswering

            model = BertForQuestionAnswering(bert_config(hp))
        else:
            model = BertForQA(BertEncoderConfig.from_hparams(hp))
        self.model = context.wrap_model(model)
        no_decay = ("bias", "LayerNorm.weight", "_ln.weight")
        wd = float(hp.get("weight_decay", 0.0))
        groups = [
            {"params": [p for n, p in self.model.named_parameters() if not any(k in n for k in no_decay)], "weight_decay": wd},
            {"params": [p for n, p in self.model.named_parameters() if any(k in n for k in no_decay)], "weight_decay": 0.0},
        ]
        self.opt = context.wrap_optimizer(torch.optim.AdamW(groups, lr=float(hp.get("learning_rate", 3e-5)),
                                                            eps=float(hp.get("adam_epsilon", 1e-8))))
        total = int(hp.get("num_training_steps", 15000))
        warm = int(hp.get("num_warmup_steps", 0))

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
        # token-overlap F1 of predicted vs gold spans
        inter = (torch.minimum(pe, e) - torch.maximum(ps, s) + 1).clamp(min=0).float()
        plen = (pe - ps + 1).clamp(min=1).float()
        glen = (e - s + 1).float()
        f1 = (2 * inter / (plen + glen)).mean()
        return {"exact_match": exact, "f1": f1}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        n = int(self.context.get_hparams().get("train_records", 88000))
        vocab = int(self.context.get_hparams().get("vocab_size", 30522))
        return det_torch.DataLoader(SyntheticSQuAD(n, self.seq_len, vocab_size=vocab),
                                    batch_size=self.context.get_per_slot_batch_size(), num_workers=2, drop_last=True)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        n = int(self.context.get_hparams().get("validation_records", 1024))
        vocab = int(self.context.get_hparams().get("vocab_size", 30522))
        return det_torch.DataLoader(SyntheticSQuAD(n, self.seq_len, vocab_size=vocab, seed=1),
                                    batch_size=self.context.get_per_slot_batch_size(), num_workers=2)



BertSQuADPyTorch = BertSQuADTrial  # the reference example's class name
