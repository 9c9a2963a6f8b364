"""Gossip agent (DIST/clients.py) on the HIP engine.

The model's parameters and grads are views into one row of an AgentBank
(HBM); the optimizer is BankSGD (one fused HIP kernel per step instead of
torch.optim.SGD); `consensus` is the weighted neighbour sum computed by the
CSR mix kernel.  Forward/backward/inference run through PyTorch-ROCm.
"""
from typing import Dict, List, Tuple

import numpy as np
import torch
from torch import nn
from torch.utils.data import DataLoader

import _engine  # noqa: F401
from dolhip import ops
from dolhip.agent import BankAgent, BankSGD, engine_device
from dolhip.data import DatasetSplit


class Client(BankAgent):
    def __init__(self, args, train_set, test_set, idxs, model):
        self.args = args
        self.loaders = self.train_val_test(train_set, test_set, idxs)
        self.criterion = nn.CrossEntropyLoss()
        self.device = engine_device(args)
        self._init_bank(model, self.device)
        self.history = {}
        self.rounds = 1
        self.optimizer = BankSGD(self, lr=args.lr, momentum=args.momentum)

    def train_val_test(self, train_set, test_set, idxs):
        """10 % validation split drawn with the global numpy RNG (DIST/clients.py:19-32)."""
        val_size = max(int(len(idxs) / 10), 1)
        val = set(np.random.choice(list(idxs), val_size, replace=False))
        train = list(set(idxs) - val)
        bs = self.args.local_bs
        return {
            "train": DataLoader(DatasetSplit(train_set, train), batch_size=bs, shuffle=True),
            "val": DataLoader(DatasetSplit(train_set, val), batch_size=bs, shuffle=True),
            "test": DataLoader(test_set, batch_size=bs, shuffle=True),
        }

    def local_update(self, global_round):
        """local_ep epochs of momentum SGD (DIST/clients.py:34-59)."""
        epoch_loss = 0.0
        hist = []
        for it in range(self.args.local_ep):
            train_acc, losses = 0.0, []
            total = len(self.loaders["train"].dataset)
            for images, labels in self.loaders["train"]:
                self.zero_grad()
                images, labels = images.to(self.device), labels.to(self.device)
                log_probs = self.model(images)
                loss = self.criterion(log_probs, labels)
                loss.backward()
                pred = torch.max(log_probs, 1)[1].view(-1)
                correct = torch.sum(torch.eq(pred, labels)).item()
                self.optimizer.step()
                losses.append(loss.item())
                train_acc += correct / total
            val_acc, val_loss = self.inference("val")
            train_loss = sum(losses) / len(losses)
            self.report(it, train_loss, train_acc, val_acc, val_loss)
            hist.append({"iter": it, "train_loss": train_loss, "train_acc": train_acc,
                         "val_acc": val_acc, "val_loss": val_loss})
            epoch_loss += train_loss / self.args.local_ep
        self.history.setdefault(global_round, {})["train_hist"] = hist
        self.rounds += 1
        return epoch_loss

    def consensus(self, Ni: List[Tuple[torch.Tensor, Dict[str, torch.Tensor]]]) -> Dict[str, torch.Tensor]:
        """sum_j a_ij * x_j over the (a_ij, state_dict_j) pairs of Neighbors
        (DIST/clients.py:61-69): new tensors, +0 start, ascending pair order.
        One CSR-mix kernel per key; the simulators' batched path mixes every
        agent at once instead (AgentBank.mix)."""
        own = self.model.state_dict()
        out = {}
        vals = torch.tensor([float(a) for a, _ in Ni], dtype=torch.float32, device=self.device)
        deg = len(Ni)
        rowptr = torch.tensor([0, deg], dtype=torch.int32, device=self.device)
        col = torch.arange(deg, dtype=torch.int32, device=self.device)
        for key, ref in own.items():
            y = torch.empty(1, ref.numel(), dtype=torch.float32, device=self.device)
            if deg == 0:
                y.zero_()
            else:
                X = torch.stack([sd[key].reshape(-1) for _, sd in Ni]).to(self.device, torch.float32)
                ops.mix_csr(X, y, rowptr, col, vals)
            out[key] = y.view(ref.shape)
        return out

    def inference(self, dataset):
        """(accuracy, mean batch loss) (DIST/clients.py:71-86)."""
        self.model.eval()
        nb, loss, total, correct = 0.0, 0.0, 0.0, 0.0
        with torch.no_grad():
            for images, labels in self.loaders[dataset]:
                images, labels = images.to(self.device), labels.to(self.device)
                outputs = self.model(images)
                loss += self.criterion(outputs, labels).item()
                pred = torch.max(outputs, 1)[1].view(-1)
                correct += torch.sum(torch.eq(pred, labels)).item()
                total += len(labels)
                nb += 1
        return correct / total, loss / nb

    def report(self, it, train_loss, train_acc, val_acc, val_loss):
        if self.args.verbose:
            print("| Local Epoch : {:2d} | Train Loss: {:2.3f} | Train Acc: {:4.2f}% | Val Loss: {:2.3f} | "
                  "Val Acc: {:4.2f}% |".format(it + 1, train_loss, train_acc * 100, val_loss, val_acc * 100))
