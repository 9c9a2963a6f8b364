"""Agent models of the reference (parameter layout = §8 row a13).

Module names, Sequential indices and construction order match
DIST/models.py:8-57 / DEC/models.py:6-51, so state_dict keys, shapes, the
flattened layout of AgentBank rows and the default-init RNG stream are the
reference's:  conv.0, conv.2 (5x5 convs, padding 2, 2x2 max-pool after each),
linear.0 (flat -> hidden), ReLU, linear.2 (hidden -> 10), Softmax.  As in the
reference there is no activation after the convs and the Softmax output goes
into CrossEntropyLoss.  Forward/backward run through PyTorch-ROCm.
"""
from __future__ import annotations

import torch
from torch import nn


def _conv_trunk(in_channels: int) -> nn.Sequential:
    layers = []
    for cin, cout in ((in_channels, 32), (32, 64)):
        layers += [nn.Conv2d(cin, cout, kernel_size=5, padding=2, bias=True), nn.MaxPool2d((2, 2))]
    return nn.Sequential(*layers)


def _classifier(flat: int, hidden: int, classes: int = 10) -> nn.Sequential:
    return nn.Sequential(nn.Linear(flat, hidden), nn.ReLU(), nn.Linear(hidden, classes), nn.Softmax(dim=1))


class _CNN(nn.Module):
    IN_CHANNELS = 1
    FLAT = 3136
    HIDDEN = 512

    def __init__(self):
        super().__init__()
        self.conv = _conv_trunk(self.IN_CHANNELS)
        self.linear = _classifier(self.FLAT, self.HIDDEN)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.conv(x)
        return self.linear(h.reshape(h.shape[0], -1))


class Model1(_CNN):
    """MNIST / FashionMNIST CNN, 1,663,370 parameters (DIST/models.py:8-30)."""


class Model3(_CNN):
    """CIFAR-10 CNN, 1,105,098 parameters (DIST/models.py:36-57)."""

    IN_CHANNELS = 3
    FLAT = 4096
    HIDDEN = 256


MODELS = {"Model1": Model1, "Model3": Model3}


def select_model(name: str, device) -> nn.Module:
    """Simulator/Server.select_global_model (DIST/simulators.py:31-38): the
    reference exits on an unknown name; here it raises SystemExit likewise."""
    if name not in MODELS:
        raise SystemExit("Error: unrecognized model")
    return MODELS[name]().to(device)
