"""Small models of the reference's tutorials / test fixtures.

* ``OneVarModel``: y = w*x with one weight, the analytic fixture of
  ``harness/tests/experiment/fixtures/pytorch_onevar_model.py`` (with data = label = 1 and MSE loss,
  one SGD step gives w' = w + 2*lr*(1 - w)).
* ``XORNet``: 2-2-1 MLP of ``fixtures/pytorch_xor_model.py``.
* ``MNISTNet``: the CNN of ``examples/tutorials/mnist_pytorch/model_def.py``.
* ``CIFAR10CNN``: the CNN of ``examples/computer_vision/cifar10_pytorch/model_def.py:42-122``.
"""
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
    def __init__(self, layer1_dropout: float = 0.25, layer2_dropout: float = 0.25, layer3_dropout: float = 0.5,
                 num_classes: int = 10) -> None:
        super().__init__()
        self.net = nn.Sequential(
            nn.Conv2d(3, 32, kernel_size=(3, 3)), nn.ReLU(),
            nn.Conv2d(32, 32, kernel_size=(3, 3)), nn.ReLU(),
            nn.MaxPool2d((2, 2)), nn.Dropout(layer1_dropout),
            nn.Conv2d(32, 64, (3, 3), padding=1), nn.ReLU(),
            nn.Conv2d(64, 64, (3, 3)), nn.ReLU(),
            nn.MaxPool2d((2, 2)), nn.Dropout2d(layer2_dropout),
            Flatten(),
            nn.Linear(2304, 512), nn.ReLU(), nn.Dropout(layer3_dropout),
            nn.Linear(512, num_classes),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)
