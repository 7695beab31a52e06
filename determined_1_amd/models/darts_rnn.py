"""DARTS recurrent cell language model (Penn Treebank) trained from a hyperparameter genotype.

Mirrors the reference's ``examples/hp_search_benchmarks/darts_penntreebank_pytorch``
(``model_def.py:58-303`` ``DARTSRNNTrial``, ``data.py`` variable-length BPTT batching,
``optimizer.py`` ``HybridSGD``): each of the 8 intermediate nodes of the DARTS recurrent cell
(Liu et al. 2019) reads one earlier state (``node{i}_edge``) through one activation
(``node{i}_op`` in {tanh, relu, sigmoid, identity}); the searchers tune those categoricals.
Training keeps the AWD-LSTM recipe of the original: embedding / locked (variational) dropouts,
tied decoder, BPTT windows of random length with the learning rate scaled by
``seq_len / bptt``, temporal activation regularisation (``beta``), gradient clipping, and a switch
from SGD to averaged SGD once validation stops improving for ``nonmono`` evaluations
(after ``optimizer_switch_epoch``).  PTB cannot be downloaded here: ``SyntheticCorpus`` (a sparse
random Markov chain over a 10k vocabulary) stands in.

MI355X-first execution of the recurrence (a launch-bound chain of small GEMMs):
  * the input half of the initial projection ``W0`` runs ONCE for the whole window as one
    [T*B, ninp] x [ninp, 2*nhid] GEMM (the input dropout mask is constant over time);
  * node GEMMs are grouped by dependency wave: nodes that read the same earlier state are one
    GEMM against their column-concatenated weights (the reference genotype runs 6 GEMMs per
    step instead of 9); the concatenation happens once per forward, not per step;
  * the dropout mask on the hidden input of every node (``dropouth``) is applied once per
    state, not once per consumer.
"""
import logging
import math
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_1_amd import pytorch as det_torch

ACTIVATIONS = ("tanh", "relu", "sigmoid", "identity")
INIT_RANGE = 0.04


def _act(name: str, x: torch.Tensor) -> torch.Tensor:
    if name == "tanh":
        return torch.tanh(x)
    if name == "relu":
        return torch.relu(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "identity":
        return x
    raise ValueError(f"unknown activation {name!r} (one of {ACTIVATIONS})")


def genotype_from_hparams(hp: Dict[str, Any], nodes: int = 8) -> List[Tuple[str, int]]:
    """``node{i}_op`` / ``node{i}_edge`` -> [(activation, input state)], state 0 = cell input
    state, state i = node i (reference ``model_def.py:111-119``)."""
    out = []
    for i in range(1, nodes + 1):
        op, pred = str(hp[f"node{i}_op"]), int(hp[f"node{i}_edge"])
        if op not in ACTIVATIONS:
            raise ValueError(f"node {i}: unknown op {op!r} (one of {ACTIVATIONS})")
        if not 0 <= pred < i:
            raise ValueError(f"node {i}: input {pred} must be in [0, {i - 1}]")
        out.append((op, pred))
    return out


def _waves(genotype: Sequence[Tuple[str, int]]) -> List[List[Tuple[int, List[int]]]]:
    """Schedule: list of waves; each wave is a list of (pred state, [node indices reading it]).
    A node joins the first wave after the one that produced its input."""
    level = {0: 0}
    for i, (_, pred) in enumerate(genotype, start=1):
        level[i] = level[pred] + 1
    waves = []  # type: List[List[Tuple[int, List[int]]]]
    for lv in range(1, max(level.values()) + 1):
        groups = {}  # type: Dict[int, List[int]]
        for i in range(1, len(genotype) + 1):
            if level[i] == lv:
                groups.setdefault(genotype[i - 1][1], []).append(i)
        waves.append(sorted(groups.items()))
    return waves


class DARTSCell(nn.Module):
    """DARTS recurrent cell: s0 = highway(x, h_prev); s_i = highway(s_pred(i)); h = mean(s_1..s_8),
    where highway(s) = s + sigmoid(c) * (act(h) - s) with [c, h] = s @ W_i."""

    def __init__(self, ninp: int, nhid: int, dropouth: float, dropoutx: float,
                 genotype: Sequence[Tuple[str, int]]) -> None:
        super().__init__()
        self.nhid, self.ninp = nhid, ninp
        self.dropouth, self.dropoutx = dropouth, dropoutx
        self.genotype = list(genotype)
        self.W0 = nn.Parameter(torch.empty(ninp + nhid, 2 * nhid).uniform_(-INIT_RANGE, INIT_RANGE))
        self.Ws = nn.ParameterList([nn.Parameter(torch.empty(nhid, 2 * nhid).uniform_(-INIT_RANGE, INIT_RANGE))
                                    for _ in self.genotype])
        self.waves = _waves(self.genotype)

    def forward(self, x: torch.Tensor, h0: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """x [T, B, ninp], h0 [1, B, nhid] -> (outputs [T, B, nhid], last hidden [1, B, nhid])."""
        T, B, _ = x.shape
        nhid = self.nhid
        if self.training:
            x_mask = torch.empty(B, self.ninp, device=x.device, dtype=x.dtype).bernoulli_(1 - self.dropoutx)
            x = x * (x_mask / (1 - self.dropoutx))
            h_mask = torch.empty(B, nhid, device=x.device, dtype=x.dtype).bernoulli_(1 - self.dropouth)
            h_mask = h_mask / (1 - self.dropouth)
        else:
            h_mask = None
        # input half of W0 for the whole window in one GEMM
        xw = torch.mm(x.reshape(T * B, self.ninp), self.W0[:self.ninp]).view(T, B, 2 * nhid)
        w0h = self.W0[self.ninp:]
        grouped = [[(pred, nodes, torch.cat([self.Ws[i - 1] for i in nodes], dim=1) if len(nodes) > 1
                     else self.Ws[nodes[0] - 1]) for pred, nodes in wave] for wave in self.waves]
        h = h0[0]
        outs = []
        for t in range(T):
            hm = h * h_mask if h_mask is not None else h
            ch = torch.addmm(xw[t], hm, w0h)
            c, hh = ch.split(nhid, dim=1)
            s0 = torch.lerp(h, torch.tanh(hh), torch.sigmoid(c))
            states = {0: s0}
            masked = {}  # type: Dict[int, torch.Tensor]
            for wave in grouped:
                for pred, nodes, w in wave:
                    sp = states[pred]
                    if pred not in masked:
                        masked[pred] = sp * h_mask if h_mask is not None else sp
                    y = torch.mm(masked[pred], w).view(B, len(nodes), 2, nhid)
                    for j, i in enumerate(nodes):
                        states[i] = torch.lerp(sp, _act(self.genotype[i - 1][0], y[:, j, 1]), torch.sigmoid(y[:, j, 0]))
            h = torch.stack([states[i] for i in range(1, len(self.genotype) + 1)], 0).mean(0)
            outs.append(h)
        return torch.stack(outs, 0), h.unsqueeze(0)


def locked_dropout(x: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """Variational dropout: one mask per sequence, shared over time (x [T, B, C])."""
    if not training or p <= 0:
        return x
    m = torch.empty(1, x.shape[1], x.shape[2], device=x.device, dtype=x.dtype).bernoulli_(1 - p)
    return x * (m / (1 - p))


def embedded_dropout(embed: nn.Embedding, words: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """Drop whole word types (rows of the embedding matrix) for this batch."""
    w = embed.weight
    if training and p > 0:
        m = torch.empty(w.shape[0], 1, device=w.device, dtype=w.dtype).bernoulli_(1 - p)
        w = w * (m / (1 - p))
    return F.embedding(words, w)


class DARTSRNNModel(nn.Module):
    """Embedding -> DARTS cell -> tied decoder -> log-softmax."""

    def __init__(self, ntoken: int, ninp: int, nhid: int, nhidlast: int, dropout: float, dropouth: float,
                 dropoutx: float, dropouti: float, dropoute: float, genotype: Sequence[Tuple[str, int]]) -> None:
        super().__init__()
        if nhidlast != ninp or nhid != nhidlast:
            raise ValueError("the DARTS cell LM ties the decoder: emsize == nhid == nhidlast required")
        self.encoder = nn.Embedding(ntoken, ninp)
        self.rnn = DARTSCell(ninp, nhid, dropouth, dropoutx, genotype)
        self.decoder = nn.Linear(ninp, ntoken)
        self.decoder.weight = self.encoder.weight
        self.nhid, self.ntoken = nhid, ntoken
        self.dropout, self.dropouti, self.dropoute = dropout, dropouti, dropoute
        nn.init.uniform_(self.encoder.weight, -0.1, 0.1)
        nn.init.zeros_(self.decoder.bias)

    def init_hidden(self, bsz: int) -> List[torch.Tensor]:
        return [torch.zeros(1, bsz, self.nhid, device=self.encoder.weight.device, dtype=self.encoder.weight.dtype)]

    def forward(self, words: torch.Tensor, hidden: List[torch.Tensor], return_h: bool = False) -> Any:
        emb = embedded_dropout(self.encoder, words, self.dropoute, self.training)
        emb = locked_dropout(emb, self.dropouti, self.training)
        raw, h = self.rnn(emb, hidden[0])
        out = locked_dropout(raw, self.dropout, self.training)
        log_prob = F.log_softmax(self.decoder(out.reshape(-1, out.shape[2])), dim=-1).view(out.shape[0], out.shape[1], -1)
        if return_h:
            return log_prob, [h], [raw], [out]
        return log_prob, [h]


class SGDThenASGD(torch.optim.Optimizer):
    """SGD that can switch to averaged SGD (reference ``optimizer.py`` ``HybridSGD``).

    The outer param groups are the ones LR schedulers edit; they are copied into the active inner
    optimizer before every step (the reference's scheduler edited the outer groups only, which the
    inner optimizers never saw).  ``state_dict`` is the active optimizer's; an ASGD state (its
    groups carry ``t0``) restores into ASGD mode."""

    def __init__(self, params: Any, lr: float, weight_decay: float = 0.0, lambd: float = 0.0, alpha: float = 0.75,
                 t0: float = 0.0) -> None:
        params = list(params)
        super().__init__(params, dict(lr=lr, weight_decay=weight_decay))
        self.SGD = torch.optim.SGD(params, lr=lr, weight_decay=weight_decay)
        self.ASGD = torch.optim.ASGD(params, lr=lr, lambd=lambd, alpha=alpha, t0=t0, weight_decay=weight_decay)
        self.optim_name = "SGD"
        self.optim = self.SGD  # type: torch.optim.Optimizer

    def set_optim(self, name: str) -> None:
        if name not in ("SGD", "ASGD"):
            raise ValueError(name)
        self.optim_name = name
        self.optim = self.SGD if name == "SGD" else self.ASGD

    def state_dict(self) -> Dict[str, Any]:
        return self.optim.state_dict()

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self.set_optim("ASGD" if "t0" in state_dict["param_groups"][0] else "SGD")
        self.optim.load_state_dict(state_dict)

    @torch.no_grad()
    def step(self, closure: Any = None) -> Any:
        for outer, inner in zip(self.param_groups, self.optim.param_groups):
            inner["lr"] = outer["lr"]
        return self.optim.step(closure)

    def averaged(self, p: torch.Tensor) -> Optional[torch.Tensor]:
        st = self.ASGD.state.get(p, {})
        return st.get("ax")


class SyntheticCorpus:
    """Token stream from a sparse random Markov chain: every word has ``fanout`` successors with
    Zipf-like probabilities, so a language model can reach a perplexity well below the vocabulary
    size.  ``train`` / ``valid`` are 1-D int64 tensors like the reference's ``Corpus``."""

    def __init__(self, vocab: int = 10000, train_tokens: int = 929589, valid_tokens: int = 73760, fanout: int = 8,
                 seed: int = 0) -> None:
        rng = np.random.RandomState(seed)
        self.vocab = vocab
        succ = rng.randint(0, vocab, size=(vocab, fanout))
        probs = 1.0 / np.arange(1, fanout + 1)
        probs /= probs.sum()
        self.train = torch.from_numpy(self._walk(succ, probs, train_tokens, rng))
        self.valid = torch.from_numpy(self._walk(succ, probs, valid_tokens, rng))

    @staticmethod
    def _walk(succ: np.ndarray, probs: np.ndarray, n: int, rng: np.random.RandomState) -> np.ndarray:
        choice = rng.choice(len(probs), size=n, p=probs)
        out = np.empty(n, dtype=np.int64)
        tok = int(rng.randint(0, succ.shape[0]))
        for i in range(n):
            tok = int(succ[tok, choice[i]])
            out[i] = tok
        return out


class BatchifiedStream(torch.utils.data.Dataset):
    """[N] token stream -> [N // B, B] (column b is the b-th contiguous slice); item t is row t."""

    def __init__(self, tokens: torch.Tensor, batch_size: int) -> None:
        n = tokens.numel() // batch_size
        self.data = tokens[:n * batch_size].view(batch_size, n).t().contiguous()

    def __len__(self) -> int:
        return self.data.shape[0]

    def __getitem__(self, i: int) -> torch.Tensor:
        return self.data[i]


class BpttBatchSampler:
    """Consecutive row windows of random length ~ N(bptt, 5) (bptt/2 with probability 0.05),
    clipped to [5, bptt + max_delta]; validation uses exactly ``bptt`` (reference ``data.py``
    ``BatchSamp``).  A window of length L yields L + 1 rows: inputs and shifted targets."""

    def __init__(self, n_rows: int, bptt: int, max_delta: int, valid: bool = False, seed: int = 0) -> None:
        self.n = n_rows - 2
        self.bptt, self.max_delta, self.valid = bptt, max_delta, valid
        self.rng = np.random.RandomState(seed)

    def __len__(self) -> int:
        return max(1, self.n // self.bptt)

    def _seq_len(self, i: int) -> int:
        if self.valid:
            return min(self.bptt, self.n - 1 - i)
        base = self.bptt if self.rng.random_sample() < 0.95 else self.bptt / 2.0
        L = min(max(5, int(self.rng.normal(base, 5))), self.bptt + self.max_delta)
        return min(L, self.n - 1 - i)

    def __iter__(self) -> Iterator[List[int]]:
        i = 0
        while i < self.n:
            L = self._seq_len(i)
            if L <= 0:
                break
            yield list(range(i, i + L + 1))
            i += L


def collate_shifted(rows: List[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
    """L + 1 rows of [B] -> (inputs [L, B], targets [L * B])."""
    x = torch.stack(rows)
    return x[:-1].contiguous(), x[1:].reshape(-1)
