"""DARTS recurrent-cell search on Penn Treebank as hyperparameter search (reference
examples/hp_search_benchmarks/darts_penntreebank_pytorch): the networks and helpers come from the ``determined_1_amd.models.darts_rnn`` library

This file is the experiment's user code (it is what a checkpoint's ``code/`` holds): the
Trial -- data, optimizer, training and evaluation steps -- lives here; the network building
blocks are imported from the framework's model library, as the reference examples import theirs
from torchvision / transformers.
"""
import logging
import math
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch
from determined_1_amd.models.darts_rnn import BatchifiedStream, BpttBatchSampler, DARTSRNNModel, SGDThenASGD, SyntheticCorpus, collate_shifted, genotype_from_hparams


class _EvalHistory(det_torch.PyTorchCallback):
    """Checkpointed optimizer-switch bookkeeping."""

    def __init__(self, trial: "DARTSRNNTrial") -> None:
        self.trial = trial

    def state_dict(self) -> Dict[str, Any]:
        return {"history": list(self.trial.eval_history), "last_loss": self.trial.last_loss}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.trial.eval_history = list(sd.get("history", []))
        self.trial.last_loss = sd.get("last_loss")



class DARTSRNNTrial(det_torch.PyTorchTrial):
    def __init__(self, context: det_torch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.hp = hp
        self.corpus = SyntheticCorpus(int(hp.get("vocab_size", 10000)), int(hp.get("train_tokens", 929589)),
                                      int(hp.get("valid_tokens", 73760)))
        emsize = int(hp.get("emsize", 850))
        self.net = DARTSRNNModel(self.corpus.vocab, emsize, int(hp.get("nhid", emsize)),
                                 int(hp.get("nhidlast", emsize)), float(hp.get("dropout", 0.75)),
                                 float(hp.get("dropouth", 0.25)), float(hp.get("dropoutx", 0.75)),
                                 float(hp.get("dropouti", 0.2)), float(hp.get("dropoute", 0.1)),
                                 genotype_from_hparams(hp))
        self.model = context.wrap_model(self.net)
        self.lr = float(hp.get("learning_rate", 20.0))
        self.bptt = int(hp.get("bptt", 35))
        self.opt = context.wrap_optimizer(SGDThenASGD(self.model.parameters(), self.lr,
                                                      float(hp.get("weight_decay", 8e-7))))
        self.clip = float(hp.get("clip_gradients_l2_norm", 0.25))
        self.hidden = None  # type: Optional[List[torch.Tensor]]
        self.eval_history = []  # type: List[float]
        self.last_loss = None  # type: Optional[float]
        self._last_epoch = -1

    def build_callbacks(self) -> Dict[str, det_torch.PyTorchCallback]:
        return {"eval_history": _EvalHistory(self)}

    def build_training_data_loader(self) -> det_torch.DataLoader:
        ds = BatchifiedStream(self.corpus.train, self.context.get_per_slot_batch_size())
        return det_torch.DataLoader(ds, batch_sampler=BpttBatchSampler(len(ds), self.bptt,
                                                                       int(self.hp.get("max_seq_length_delta", 20))),
                                    collate_fn=collate_shifted)

    def build_validation_data_loader(self) -> det_torch.DataLoader:
        ds = BatchifiedStream(self.corpus.valid, int(self.hp.get("eval_batch_size", 10)))
        return det_torch.DataLoader(ds, batch_sampler=BpttBatchSampler(len(ds), self.bptt, 0, valid=True),
                                    collate_fn=collate_shifted)

    def _maybe_switch(self) -> None:
        nonmono = int(self.hp.get("nonmono", 5))
        if (self.opt.optim_name == "SGD" and self.last_loss is not None and len(self.eval_history) > nonmono + 1
                and self.last_loss > min(self.eval_history[:-(nonmono + 1)])):
            logging.info("validation stopped improving: switching to averaged SGD")
            self.opt.set_optim("ASGD")

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        if epoch_idx != self._last_epoch and epoch_idx > int(self.hp.get("optimizer_switch_epoch", 75)):
            self._maybe_switch()
        self._last_epoch = epoch_idx
        x, y = batch
        for g in self.opt.param_groups:
            g["lr"] = self.lr * x.shape[0] / self.bptt
        if self.hidden is None or batch_idx == 0 or self.hidden[0].shape[1] != x.shape[1]:
            self.hidden = self.net.init_hidden(x.shape[1])
        hidden = [h.detach() for h in self.hidden]
        log_prob, hidden, raws, drops = self.model(x, hidden, return_h=True)
        self.hidden = hidden
        raw_loss = F.nll_loss(log_prob.reshape(-1, log_prob.shape[2]), y)
        loss = raw_loss
        alpha, beta = float(self.hp.get("alpha", 0.0)), float(self.hp.get("beta", 1e-3))
        if alpha > 0:
            loss = loss + alpha * drops[-1].pow(2).mean()
        if beta > 0 and raws[-1].shape[0] > 1:
            loss = loss + beta * (raws[-1][1:] - raws[-1][:-1]).pow(2).mean()
        self.context.backward(loss)
        self.context.step_optimizer(self.opt, clip_grads=det_torch.ClipGradsNorm(self.clip) if self.clip > 0 else None)
        return {"loss": loss, "raw_loss": raw_loss, "perplexity": torch.exp(raw_loss.detach().float().clamp(max=50))}

    def evaluate_full_dataset(self, data_loader: torch.utils.data.DataLoader) -> Dict[str, Any]:
        saved = None
        if self.opt.optim_name == "ASGD":
            saved = {}
            for p in self.net.parameters():
                ax = self.opt.averaged(p)
                if ax is not None:
                    saved[p] = p.detach().clone()
                    p.data.copy_(ax)
        self.net.eval()
        total, n = 0.0, 0
        bsz = int(self.hp.get("eval_batch_size", 10))
        hidden = self.net.init_hidden(bsz)
        with torch.no_grad():
            for x, y in data_loader:
                x, y = self.context.to_device((x, y))
                log_prob, hidden = self.net(x, hidden)
                total += float(F.nll_loss(log_prob.reshape(-1, log_prob.shape[2]), y)) * x.shape[0]
                n += x.shape[0]
        self.net.train()
        if saved:
            for p, v in saved.items():
                p.data.copy_(v)
        loss = total / max(1, n)
        self.last_loss = loss
        self.eval_history.append(min([loss] + self.eval_history))
        return {"loss": loss, "perplexity": math.exp(min(loss, 50.0))}

