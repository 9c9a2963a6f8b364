"""Federated clients (DEC/clients.py) on the HIP engine.

Parameters, grads, momentum and ADMM duals live in rows of an AgentBank.
`update_weights` runs each batch as PyTorch-ROCm forward/backward followed by
ONE fused HIP kernel for gradient term + momentum SGD (dol_prox_admm_sgd_f32).
If a subclass overrides `update_model` (the reference's plugin convention:
`Foo_Server` pairs with `Foo_Client`), the reference's two-call sequence
update_model(...) + optimizer.step() is kept instead.
"""
from typing import Dict, Optional, Union

import torch
from torch import nn
from torch.utils.data import DataLoader

import _engine  # noqa: F401
from dolhip import ops
from dolhip.agent import BankAgent, BankSGD, RowState, engine_device
from dolhip.data import DatasetSplit

Theta = Union[Dict[str, torch.Tensor], RowState, torch.Tensor]


class Client(BankAgent):
    # the gradient term this class fuses into the step: None / "prox" / "admm"
    TERM: Optional[str] = None

    def __init__(self, args, train_set, test_set, idxs, model):
        self.args = args
        self.loaders = self.train_val_test(train_set, test_set, idxs)
        self.criterion = nn.CrossEntropyLoss()
        self.device = engine_device(args)
        self._init_bank(model, self.device)
        self.history = []
        self.optimizer = BankSGD(self, lr=args.lr, momentum=args.momentum)
        self._theta = None  # device copy of the round's theta (flat)

    def train_val_test(self, train_set, test_set, idxs):
        """First 10 % of the user's indices validate (DEC/clients.py:158-176)."""
        bs = self.args.local_bs
        if test_set:
            return {"train": None,
                    "test": DataLoader(DatasetSplit(test_set, range(len(test_set))), batch_size=bs, shuffle=False)}
        idxs = list(idxs)
        val_size = max(int(len(idxs) / 10), 1)
        return {"train": DataLoader(DatasetSplit(train_set, idxs[val_size:]), batch_size=bs, shuffle=True),
                "test": DataLoader(DatasetSplit(train_set, idxs[:val_size]), batch_size=bs, shuffle=False)}

    # ------------------------------------------------------------------ theta
    def theta_vector(self, theta: Theta) -> torch.Tensor:
        """theta as one flat fp32 device vector in this bank's layout."""
        if isinstance(theta, torch.Tensor) and theta.dim() == 1:
            return theta
        if isinstance(theta, RowState):
            return theta.flat()
        if self._theta is None:
            self._theta = torch.empty(self.bank.P, dtype=torch.float32, device=self.device)
        return self.bank.flatten(theta, out=self._theta)

    def theta_dict(self, theta: Theta):
        if isinstance(theta, torch.Tensor):
            return self.bank.unflatten(theta)
        return theta

    def _fused(self) -> bool:
        return type(self).update_model is _DEFAULT_UPDATE_MODEL.get(type(self).TERM)

    # ------------------------------------------------------------------ local training
    def _forward_backward(self, images, labels):
        images, labels = images.to(self.device), labels.to(self.device)
        self.zero_grad()
        log_probs = self.model(images)
        loss = self.criterion(log_probs, labels)
        loss.backward()
        pred = torch.max(log_probs, 1)[1].view(-1)
        return loss, torch.sum(torch.eq(pred, labels)).item()

    def update_weights(self, theta: Theta, global_round):
        """w <- theta; local_ep epochs; validation; duals (DEC/clients.py:178-195)."""
        th = self.theta_vector(theta)
        with torch.no_grad():
            self.flat_params().copy_(th)
        fused = self._fused()
        th_dict = None if fused else self.theta_dict(theta)
        epoch_loss = 0.0
        for it in range(self.args.local_ep):
            train_acc, losses = 0.0, []
            total = len(self.loaders["train"].dataset)
            for images, labels in self.loaders["train"]:
                if fused:
                    loss, corr = self._forward_backward(images, labels)
                    self.optimizer.step(theta=th if self.TERM else None, alpha=self.TERM == "admm",
                                        rho=self.args.rho or 0.0)
                else:
                    loss, corr = self.update_model(images, labels, th_dict)
                    self.optimizer.step()
                losses.append(loss.item())
                train_acc += corr / total
            val_acc, val_loss = self.inference("test")
            train_loss = sum(losses) / len(losses)
            self.report(global_round, it, train_loss, train_acc, val_acc, val_loss)
            self.history.append({"global_round": global_round, "epoch": it, "train_loss": train_loss,
                                 "train_acc": train_acc, "val_acc": val_acc, "val_loss": val_loss})
            epoch_loss += train_loss / self.args.local_ep
        self.update_duals(th if fused else th_dict)
        return self.state_view(), epoch_loss

    def update_model(self, images, labels, theta):
        pass

    def update_duals(self, theta):
        pass

    def inference(self, dataset):
        """(accuracy, SUM of batch losses) (DEC/clients.py:203-217)."""
        self.model.eval()
        loss, total, correct = 0.0, 0.0, 0.0
        with torch.no_grad():
            for images, labels in self.loaders[dataset]:
                images, labels = images.to(self.device), labels.to(self.device)
                outputs = self.model(images)
                loss += self.criterion(outputs, labels).item()
                pred = torch.max(outputs, 1)[1].view(-1)
                correct += torch.sum(torch.eq(pred, labels)).item()
                total += len(labels)
        return correct / total, loss

    def report(self, global_round, it, train_loss, train_acc, val_acc, val_loss):
        if self.args.verbose and (it % 9 == 0):
            print("| Local Epoch : {:2d} | Train Loss: {:.3f} | Train Acc: {:.2f}% | Val Loss: {:.3f} | "
                  "Val Acc: {:.2f}% |".format(it + 1, train_loss, train_acc * 100, val_loss, val_acc * 100))


class FedAvg_Client(Client):
    """No extra term (DEC/clients.py:85-95)."""

    TERM = None

    def update_model(self, images, labels, theta):
        return self._forward_backward(images, labels)


class FedProx_Client(Client):
    """grad += rho * (w - theta) (DEC/clients.py:101-115)."""

    TERM = "prox"

    def update_model(self, images, labels, theta):
        loss, correct = self._forward_backward(images, labels)
        b, i = self.bank, self.row
        ops.prox_grad(b.buffer("grad")[i:i + 1], b.buffer("x")[i:i + 1], self.theta_vector(theta),
                      self.args.rho, P=b.P)
        return loss, correct


class FedAdmm_Client(Client):
    """grad += alpha + rho * (w - theta); alpha += rho * (w - theta) after the
    local epochs (DEC/clients.py:118-144).  alpha lives in the bank's 'alpha'
    row; `self.alpha` is a dict of views into it (updated in place)."""

    TERM = "admm"

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.bank.buffer("alpha", zero=True)[self.row].zero_()

    def attach(self, bank, row):
        super().attach(bank, row)
        bank.buffer("alpha", zero=True)

    @property
    def alpha(self) -> Dict[str, torch.Tensor]:
        return self.bank.row_views(self.row, "alpha")

    def update_model(self, images, labels, theta):
        loss, correct = self._forward_backward(images, labels)
        b, i = self.bank, self.row
        ops.prox_grad(b.buffer("grad")[i:i + 1], b.buffer("x")[i:i + 1], self.theta_vector(theta),
                      self.args.rho, alpha=b.buffer("alpha")[i:i + 1], P=b.P)
        return loss, correct

    def update_duals(self, theta):
        """alpha += rho (w - theta) (DEC/clients.py:141-144); the kernel also
        leaves ||w - theta||^2 (fp64, fixed order) in self.resid_sq for the
        server's per-round metrics (not part of the reference)."""
        b, i = self.bank, self.row
        if getattr(self, "resid_sq", None) is None:
            self.resid_sq = torch.zeros(1, dtype=torch.float64, device=b.device)
        ops.admm_dual(b.buffer("alpha")[i:i + 1], b.buffer("x")[i:i + 1], self.theta_vector(theta),
                      self.args.rho, resid_sq=self.resid_sq, P=b.P)


_DEFAULT_UPDATE_MODEL = {None: FedAvg_Client.update_model, "prox": FedProx_Client.update_model,
                         "admm": FedAdmm_Client.update_model}
