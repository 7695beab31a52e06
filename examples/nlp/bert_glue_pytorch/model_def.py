"""BERT GLUE (MRPC) fine-tuning trial (reference examples/nlp/bert_glue_pytorch): see
determined_1_amd/models/bert_glue.py.  Synthetic MRPC-shaped sentence pairs (no network here).

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
from typing import Any, Dict, Optional

import torch

from determined_1_amd.models.bert import BertEmbeddings, BertEncoderConfig, BertLayer, _Dense, hf_encoder_state
from determined_1_amd.models.synthetic import SyntheticGLUEPairs
from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.bert_glue import BertForSequenceClassification, glue_pair_metrics


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



BertPytorch = BertGLUETrial  # the reference example's class name
