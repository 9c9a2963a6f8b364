"""Federated servers (DEC/servers.py) on the HIP engine.

Same plugin convention as the reference: `Foo_Server` trains `Foo_Client`
(class looked up by name, DEC/servers.py:22).  The N clients' parameters are
rows of one AgentBank; the global model is a separate 1-row bank whose row is
theta.  `average_weights` is the ordered mean kernel over bank rows in the
sampled order (bit-identical to the reference's sequential sum / m).
"""
import copy
import time

import numpy as np
import torch
from tqdm import tqdm

import _engine  # noqa: F401
from dolhip import ops
from dolhip.agent import RowState, engine_device
from dolhip.bank import AgentBank, layout_of
from dolhip.models import select_model
from utils import get_dataset, exp_details, setup_seed
import clients as _clients
from clients import FedAvg_Client, FedAdmm_Client, FedProx_Client  # noqa: F401


def _client_class(server_cls_name: str):
    name = server_cls_name.replace("_Server", "_Client")
    cls = getattr(_clients, name, None) or globals().get(name)
    if cls is None:
        raise KeyError(name)  # the reference fails the same way (globals()[...])
    return cls


class Server(object):
    def __init__(self, args):
        self.args = args
        self.history = []
        self.metrics = []  # per-round primal / dual metrics (FedADMM), beside the reference's history
        self.global_round = 0
        setup_seed(args.seed)
        model = self.select_global_model(self.args.model, self.args.device)
        train_dataset, test_dataset, user_groups = get_dataset(args)
        cls = _client_class(type(self).__name__)
        self.global_client = cls(args=self.args, train_set=None, test_set=test_dataset,
                                 idxs=range(len(test_dataset)), model=copy.deepcopy(model))
        self.clients = []
        for idx in range(self.args.num_users):
            self.clients.append(cls(args=self.args, train_set=train_dataset, test_set=None,
                                    idxs=user_groups[idx], model=copy.deepcopy(model)))
        self.device = engine_device(args)
        self.bank = AgentBank(self.args.num_users, layout_of(model), self.device)
        for i, c in enumerate(self.clients):
            c.attach(self.bank, i)
        if args.verbose:
            exp_details(args)
            print("random seed =", args.seed)
            print()
            print(model)

    def select_global_model(self, model, device):
        return select_model(model, device if device is not None else "cuda")

    def average_weights(self, w):
        """Ordered uniform average (DEC/servers.py:42-48): new tensors, sum in
        list order, true fp32 division by len(w).  Rows of this server's bank
        are averaged in place of copies; other state dicts are staged."""
        if len(w) == 0:
            raise IndexError("list index out of range")  # as w[0] in the reference
        if all(isinstance(s, RowState) and s.bank is w[0].bank for s in w):
            bank = w[0].bank
            out = torch.empty(bank.P, dtype=torch.float32, device=bank.device)
            bank.ordered_mean([s.row for s in w], out=out)
            return bank.unflatten(out)
        keys = list(w[0].keys())
        ref = w[0]
        out = {}
        for k in keys:
            X = torch.stack([sd[k].reshape(-1) for sd in w]).to(torch.float32)
            if X.device.type != "cuda":
                X = X.to(self.device)
            order = torch.arange(len(w), dtype=torch.int32, device=X.device)
            out[k] = ops.ordered_mean(X, order).view(ref[k].shape)
        return out

    def run(self, frac, rounds):
        start_time = time.time()
        m = max(int(frac * self.args.num_users), 1)
        test_acc, test_loss = [], []
        train_loss = []
        for _ in tqdm(range(rounds)):
            print(f"\n | Global Training Round : {self.global_round + 1} |\n")
            idxs_users = np.random.choice(range(self.args.num_users), m, replace=False)
            local_weights, local_losses = [], []
            theta = self.global_client.flat_params()  # read-only for the whole round
            for i, idx in enumerate(idxs_users):
                if self.args.verbose:
                    print(" | #{:2d}: {:2d} |".format(i + 1, idx))
                lsum, loss = self.clients[idx].update_weights(global_round=self.global_round, theta=theta)
                local_weights.append(lsum)  # a live bank-row view: stable until the next round
                local_losses.append(loss)
            loss_avg = sum(local_losses) / len(local_losses)
            train_loss.append(loss_avg)
            self._record_metrics(idxs_users)
            mean_acc_all, _ = self.avg_trainig_calculator()
            self.update_global_model(local_weights)
            test_acc_1, test_loss_1 = self.global_client.inference("test")
            test_acc.append(test_acc_1)
            test_loss.append(test_loss_1)
            mean_train_loss = np.mean(np.array(train_loss))
            print("\ntest accuracy:{:.2f}%\n".format(100 * test_acc_1))
            print(f" \nAvg Training Stats after {self.global_round + 1} global rounds:")
            print("Training Loss : {:.3f}".format(mean_train_loss))
            self.history.append({"round": self.global_round, "test_acc": test_acc_1, "test_loss": test_loss_1,
                                 "train_loss": mean_train_loss, "train_acc": mean_acc_all})
            self.global_round += 1
        print("\n Total Run Time: {0:0.4f}".format(time.time() - start_time))
        print(f" \n Results after {rounds} global rounds of training:")
        print("|---- Test Accuracy: {:.2f}%".format(100 * test_acc[-1]))

    def _record_metrics(self, idxs_users):
        """Per-round primal / dual metrics of the sampled clients, kept
        in self.metrics so the reference's `history` schema is unchanged:
        primal_resid_sq = sum_k ||w_k - theta||^2 (pre-round theta, from the
        dual kernel), dual_sq = sum_k ||alpha_k||^2 (FedADMM only)."""
        cs = [self.clients[int(i)] for i in idxs_users]
        if not cs or getattr(cs[0], "TERM", None) != "admm":
            return
        b = cs[0].bank
        rows = torch.as_tensor([c.row for c in cs], device=b.device)
        alpha = b.buffer("alpha")[rows, : b.P].double()
        resid = torch.stack([c.resid_sq[0] for c in cs]).sum()
        self.metrics.append({"round": self.global_round, "primal_resid_sq": float(resid),
                             "dual_sq": float((alpha * alpha).sum())})

    def tarining(self):
        pass

    def avg_trainig_calculator(self):
        """Mean train-split accuracy/loss over ALL clients (DEC/servers.py:85-93)."""
        avg_acc, avg_loss = 0.0, 0.0
        self.global_client.model.eval()
        n = self.args.num_users
        if self.args.skip_train_eval:
            return float("nan"), float("nan")
        for c in range(n):
            acc, loss = self.clients[c].inference("train")
            avg_acc += acc / n
            avg_loss += loss / n
        return avg_acc, avg_loss

    def update_global_model(self, local_weights):
        theta = self.average_weights(local_weights)
        g = self.global_client
        with torch.no_grad():
            g.bank.flatten(theta, out=g.flat_params())

    def plot(self):
        """Per-client local-epoch curves (DEC/servers.py:95-120): an s x s block of
        clients (s = ceil(sqrt(n))), each with a loss panel (train / val) and,
        one grid row below it, an accuracy panel (train / val), from the
        client's `history` rows that `update_weights` appends.  The reference
        offsets the accuracy row by a literal 10 (= s at its n = 100) and runs
        past the last client for non-square n (IndexError); here the offset is
        s and the cells after the last client stay empty.  Clients never
        sampled have no history and get empty panels, as the reference's
        `except: pass` gives."""
        import math

        import matplotlib.pyplot as plt
        import pandas as pd

        n = self.args.num_users
        s = math.ceil(math.sqrt(n))
        fig, axs = plt.subplots(2 * s, s, figsize=(s * 2, s * 4), sharex=True, sharey="row", squeeze=False)
        axs = axs.flat
        for block in range(s):
            for j in range(s):
                c = block * s + j
                if c >= n:
                    break
                loss_ax, acc_ax = axs[2 * block * s + j], axs[(2 * block + 1) * s + j]
                hist = pd.DataFrame(self.clients[c].history)
                loss_ax.set_title("Client #%d" % (c + 1))
                loss_ax.set(xlabel="rounds", ylabel="loss")
                acc_ax.set(xlabel="rounds", ylabel="accuracy")
                loss_ax.label_outer()
                acc_ax.label_outer()
                if {"train_loss", "val_loss"} <= set(hist.columns):
                    loss_ax.plot(hist["train_loss"], "b", label="train")
                    loss_ax.plot(hist["val_loss"], "r", label="val")
                    loss_ax.legend()
                if {"train_acc", "val_acc"} <= set(hist.columns):
                    acc_ax.plot(hist["train_acc"], "k", label="train")
                    acc_ax.plot(hist["val_acc"], "g", label="val")
                    acc_ax.legend()
        plt.show()
        return fig


class FedAdmm_Server(Server):
    """Averages the plain local weights, as the reference (DEC/servers.py:121-127)."""


class FedAvg_Server(Server):
    """DEC/servers.py:129-135."""


class FedProx_Server(Server):
    """DEC/servers.py:137-143."""
