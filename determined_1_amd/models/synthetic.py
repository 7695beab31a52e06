"""Synthetic datasets of the benchmark shapes (no network: no ImageNet / CIFAR / SQuAD here).

``SyntheticImages`` mimics a decoded-image pipeline: a fixed pool of random uint8 HWC images in
*pinned* host memory.  ``__getitems__`` (torch>=2 batched fetch) returns contiguous batches as
zero-copy views of the pinned pool, so the only per-batch host work is the DMA the
``DevicePrefetcher`` issues; normalisation to bf16 NCHW-channels_last happens on the GPU in one
``det_u8_normalize`` kernel pass.
"""
from typing import Any, List, Optional, Sequence, Tuple

import torch
import torch.utils.data as tud

IMAGENET_MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
IMAGENET_STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)


class SyntheticImages(tud.Dataset):
    def __init__(self, length: int, image_size: int = 224, channels: int = 3, num_classes: int = 1000,
                 pool: int = 512, seed: int = 0, pin: bool = True) -> None:
        g = torch.Generator().manual_seed(seed)
        self.length = int(length)
        self.pool = min(pool, self.length)
        imgs = torch.randint(0, 256, (self.pool, image_size, image_size, channels), dtype=torch.uint8, generator=g)
        labels = torch.randint(0, num_classes, (self.pool,), dtype=torch.int64, generator=g)
        if pin and torch.cuda.is_available():
            imgs = imgs.pin_memory()
            labels = labels.pin_memory()
        self.images = imgs
        self.labels = labels

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, torch.Tensor]:
        j = i % self.pool
        return self.images[j], self.labels[j]

    def __getitems__(self, idx: Sequence[int]) -> Tuple[torch.Tensor, torch.Tensor]:
        n = len(idx)
        j0 = idx[0] % self.pool
        contiguous = all(idx[k] == idx[0] + k for k in range(n)) and j0 + n <= self.pool
        if contiguous:
            return self.images[j0:j0 + n], self.labels[j0:j0 + n]
        sel = torch.tensor([i % self.pool for i in idx], dtype=torch.int64)
        return self.images.index_select(0, sel), self.labels.index_select(0, sel)


class SyntheticImageClasses(tud.Dataset):
    """Learnable uint8 image classification data in the layout CIFAR-10 / ImageNet decoders
    produce (HWC uint8).  Sample ``i`` is its class template (contrast 20 around 128) plus one of
    1024 noise patterns (std 60: the 1:3 signal-to-noise of ``SyntheticClassification``), with the
    label and pattern drawn from a hash of ``i`` -- every index is a distinct image, nothing is
    materialised up front (trial start-up stays in milliseconds), and ``__getitems__`` builds a
    whole batch ``(uint8 [N,H,W,C], int64 [N])`` with four vector ops in int16, so the host does
    no per-sample work and normalisation runs on the GPU (``ops.functional.u8_normalize``).
    Use with ``collate_fn=passthrough_collate``."""

    BANK = 1024

    def __init__(self, length: int, image_size: int = 32, channels: int = 3, num_classes: int = 10,
                 noise: float = 60.0, seed: int = 0, template_seed: int = 1234) -> None:
        self.length = int(length)
        self.num_classes = num_classes
        self.seed = int(seed)
        self.shape = (image_size, image_size, channels)
        self.noise = noise
        self.template_seed = template_seed
        self._table: Optional[torch.Tensor] = None

    def _build(self) -> torch.Tensor:
        """Every (class, noise pattern) image, uint8 [num_classes * BANK, H, W, C]: built once on
        first use (~70 ms for CIFAR's shape), then a batch is a single gather."""
        gt = torch.Generator().manual_seed(self.template_seed)
        templates = (128.0 + 20.0 * torch.randn((self.num_classes,) + self.shape, generator=gt)).to(torch.int16)
        g = torch.Generator().manual_seed(self.seed * 1000003 + 29)
        bank = (self.noise * torch.randn((self.BANK,) + self.shape, generator=g)).to(torch.int16)
        table = (templates.view(self.num_classes, 1, -1) + bank.view(1, self.BANK, -1)).clamp_(0, 255)
        return table.to(torch.uint8).view((self.num_classes * self.BANK,) + self.shape)

    def __len__(self) -> int:
        return self.length

    def _keys(self, ii: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        h = (ii * 2654435761 + self.seed * 40503) & 0x7FFFFFFF  # Knuth multiplicative hash
        return (h >> 7) % self.num_classes, h % self.BANK

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, torch.Tensor]:
        x, y = self.__getitems__([i])
        return x[0], y[0]

    def __getitems__(self, idx: Sequence[int]) -> Tuple[torch.Tensor, torch.Tensor]:
        if self._table is None:
            self._table = self._build()
        labels, pick = self._keys(torch.as_tensor(list(idx), dtype=torch.int64))
        return self._table.index_select(0, labels * self.BANK + pick), labels


from determined_1_amd.pytorch._data import passthrough_collate  # noqa: E402,F401  (re-export)


class SyntheticTokens(tud.Dataset):
    """BERT/SQuAD-shaped synthetic batches: input_ids, attention_mask, token_type_ids,
    start/end positions."""

    def __init__(self, length: int, seq_len: int = 384, vocab: int = 30522, seed: int = 0, pool: int = 256) -> None:
        g = torch.Generator().manual_seed(seed)
        self.length = int(length)
        self.pool = min(pool, self.length)
        self.input_ids = torch.randint(0, vocab, (self.pool, seq_len), generator=g)
        self.attention_mask = torch.ones(self.pool, seq_len, dtype=torch.int64)
        self.token_type_ids = torch.zeros(self.pool, seq_len, dtype=torch.int64)
        self.token_type_ids[:, seq_len // 2:] = 1
        self.start = torch.randint(0, seq_len, (self.pool,), generator=g)
        self.end = torch.clamp(self.start + torch.randint(0, 16, (self.pool,), generator=g), max=seq_len - 1)

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int) -> List[torch.Tensor]:
        j = i % self.pool
        return [self.input_ids[j], self.attention_mask[j], self.token_type_ids[j], self.start[j], self.end[j]]


class SyntheticClassification(tud.Dataset):
    """Learnable synthetic classification data: each class has a fixed random template and a
    sample is ``template[label] + noise``, so accuracy rises with training (stands in for MNIST /
    CIFAR-10, which cannot be downloaded here).

    Labels are drawn once per index and noise comes from a fixed pool indexed by a hash of the
    sample index, so ``__getitems__`` builds a whole batch with two gathers instead of one
    generator + ``randn`` per sample (which dominated short ASHA trials' validation passes)."""

    NOISE_POOL = 1024

    def __init__(self, length: int, shape: Sequence[int], num_classes: int = 10, noise: float = 1.0,
                 seed: int = 0, template_seed: int = 1234) -> None:
        self.length = int(length)
        self.shape = tuple(shape)
        self.num_classes = num_classes
        self.noise = noise
        self.seed = seed
        gt = torch.Generator().manual_seed(template_seed)
        self.templates = torch.randn((num_classes,) + self.shape, generator=gt)
        g = torch.Generator().manual_seed(seed * 1000003 + 17)
        self.labels = torch.randint(0, num_classes, (self.length,), generator=g)
        pool = min(self.NOISE_POOL, self.length)
        self.noise_pool = noise * torch.randn((pool,) + self.shape, generator=g)
        self._mul = 2654435761 % pool or 1  # Knuth multiplicative hash over the pool

    def __len__(self) -> int:
        return self.length

    def _noise_index(self, idx: torch.Tensor) -> torch.Tensor:
        return (idx * self._mul + self.seed) % self.noise_pool.shape[0]

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, torch.Tensor]:
        y = self.labels[i]
        j = int(self._noise_index(torch.tensor(i)))
        return self.templates[y] + self.noise_pool[j], y.clone()

    def __getitems__(self, idx: Sequence[int]) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        ii = torch.as_tensor(list(idx), dtype=torch.int64)
        y = self.labels.index_select(0, ii)
        x = self.templates.index_select(0, y) + self.noise_pool.index_select(0, self._noise_index(ii))
        return list(zip(x.unbind(0), y.unbind(0)))


class SyntheticSQuAD(tud.Dataset):
    """SQuAD-shaped extractive-QA features (input_ids, token_type_ids, attention_mask,
    start/end positions) for BERT throughput runs; random tokens, answer span inside the context."""

    def __init__(self, length: int, seq_len: int = 384, vocab_size: int = 30522, seed: int = 0) -> None:
        self.length = int(length)
        self.seq_len = seq_len
        self.vocab = vocab_size
        self.seed = seed

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, ...]:
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        L = self.seq_len
        q = min(64, L // 4)  # question length (64 at SQuAD's 384; short sequences for tiny test models)
        span = min(30, (L - q) // 4)
        ids = torch.randint(min(1000, self.vocab // 2), self.vocab, (L,), generator=g)
        ids[0], ids[q - 1], ids[L - 1] = min(101, self.vocab - 1), min(102, self.vocab - 1), min(102, self.vocab - 1)
        tt = torch.zeros(L, dtype=torch.int64)
        tt[q:] = 1
        am = torch.ones(L, dtype=torch.int64)
        s = int(torch.randint(q, L - span - 1, (1,), generator=g))
        e = s + int(torch.randint(0, span, (1,), generator=g))
        return ids, tt, am, torch.tensor(s), torch.tensor(e)


class SyntheticGLUEPairs(tud.Dataset):
    """MRPC-shaped sentence-pair classification features (input_ids, attention_mask,
    token_type_ids, label) with a learnable rule: label 1 pairs repeat a span of sentence A inside
    sentence B (a paraphrase stand-in), label 0 pairs do not.  Variable sentence lengths exercise
    the padding mask."""

    def __init__(self, length: int, seq_len: int = 128, vocab_size: int = 30522, seed: int = 0) -> None:
        self.length = int(length)
        self.seq_len = seq_len
        self.vocab = vocab_size
        self.seed = seed

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int) -> Tuple[torch.Tensor, ...]:
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        L = self.seq_len
        la = int(torch.randint(L // 8, L // 2 - 2, (1,), generator=g))
        lb = int(torch.randint(L // 8, L - la - 3, (1,), generator=g))
        a = torch.randint(1000, self.vocab, (la,), generator=g)
        b = torch.randint(1000, self.vocab, (lb,), generator=g)
        label = int(torch.randint(0, 2, (1,), generator=g))
        if label == 1:
            n = min(la, lb, 8)
            b[:n] = a[:n]
        ids = torch.zeros(L, dtype=torch.int64)
        tt = torch.zeros(L, dtype=torch.int64)
        am = torch.zeros(L, dtype=torch.int64)
        seq = torch.cat([torch.tensor([101]), a, torch.tensor([102]), b, torch.tensor([102])])
        ids[:seq.numel()] = seq
        am[:seq.numel()] = 1
        tt[la + 2:seq.numel()] = 1
        return ids, am, tt, torch.tensor(label)
