"""Small models of the reference's tutorials / test fixtures.

* ``OneVarModel``: y = w*x with one weight, the analytic fixture of
  ``harness/tests/experiment/fixtures/pytorch_onevar_model.py`` (with data = label = 1 and MSE loss,
  one SGD step gives w' = w + 2*lr*(1 - w)).
* ``XORNet``: 2-2-1 MLP of ``fixtures/pytorch_xor_model.py``.
* ``MNISTNet``: the CNN of ``examples/tutorials/mnist_pytorch/model_def.py``.
* ``CIFAR10CNN``: the CNN of ``examples/computer_vision/cifar10_pytorch/model_def.py:42-122``.
"""
import os

import torch
import torch.nn as nn


class OneVarModel(nn.Module):
    def __init__(self, init_w: float = 0.0) -> None:
        super().__init__()
        self.w = nn.Parameter(torch.tensor([init_w], dtype=torch.float32))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x * self.w


class XORNet(nn.Module):
    def __init__(self, hidden_size: int = 2) -> None:
        super().__init__()
        self.main = nn.Sequential(nn.Linear(2, hidden_size), nn.Sigmoid(), nn.Linear(hidden_size, 1), nn.Sigmoid())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.main(x)


class Flatten(nn.Module):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x.reshape(x.shape[0], -1)


class MNISTNet(nn.Module):
    def __init__(self, n_filters1: int = 32, n_filters2: int = 64, dropout1: float = 0.25,
                 dropout2: float = 0.5) -> None:
        super().__init__()
        self.net = nn.Sequential(
            nn.Conv2d(1, n_filters1, 3, 1), nn.ReLU(),
            nn.Conv2d(n_filters1, n_filters2, 3), nn.ReLU(),
            nn.MaxPool2d(2), nn.Dropout(dropout1), Flatten(),
            nn.Linear(144 * n_filters2, 128), nn.ReLU(), nn.Dropout(dropout2),
            nn.Linear(128, 10), nn.LogSoftmax(dim=1),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)


class CIFAR10CNN(nn.Module):
    """The reference's CIFAR-10 network (``cifar10_pytorch/model_def.py:47-65``).  On an MI355X the
    whole forward and backward run on ``ops/cnn.py`` (csrc/det_cnn.hip: ~20 launches per training
    batch); ``DET_NATIVE_CNN=0`` keeps the torch layers.  The logits come back fp32 on that path."""

    def __init__(self, layer1_dropout: float = 0.25, layer2_dropout: float = 0.25, layer3_dropout: float = 0.5,
                 num_classes: int = 10) -> None:
        super().__init__()
        self.native = os.environ.get("DET_NATIVE_CNN", "1") != "0" and num_classes == 10
        self.net = nn.Sequential(
            nn.Conv2d(3, 32, kernel_size=(3, 3)), nn.ReLU(),
            nn.Conv2d(32, 32, kernel_size=(3, 3)), nn.ReLU(),
            nn.MaxPool2d((2, 2)), nn.Dropout2d(layer1_dropout),
            nn.Conv2d(32, 64, (3, 3), padding=1), nn.ReLU(),
            nn.Conv2d(64, 64, (3, 3)), nn.ReLU(),
            nn.MaxPool2d((2, 2)), nn.Dropout2d(layer2_dropout),
            Flatten(),
            nn.Linear(2304, 512), nn.ReLU(), nn.Dropout(layer3_dropout),
            nn.Linear(512, num_classes),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.native and x.is_cuda:
            from determined_1_amd.ops import cnn

            layers = [self.net[i] for i in (0, 2, 6, 8, 13, 16)]
            params = [t for m in layers for t in (m.weight, m.bias)]
            if cnn.supported(x, params):
                ps = (self.net[5].p, self.net[11].p, self.net[15].p)
                return cnn.cifar_cnn(x, params, ps, self.training)
        return self.net(x)
