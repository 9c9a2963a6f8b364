"""dolhip — MI355X (gfx950) engine for the per-round consensus step of
AlirezaMoseni/Distributed-Optimization-and-Learning.

Layers:
  _native   ctypes binding of libdol_hip.so (C-ABI: include/dol_hip.h)
  ops       tensor-level wrappers (validation, current torch stream)
  graph     communication_graph / Neighbors-as-CSR / ring plan (host)
  bank      AgentBank: stacked [N, ld] agent state in HBM, module views
  parallel  agent sharding over ranks: ring halo exchange, global mean
The reference-shaped APIs live beside this package:
  weighted_average/  (Simulator, DecFedAvg, FedLCon, Client, ...)
  primal_dual/       (Server, FedAvg_/FedProx_/FedAdmm_Server/_Client)
"""
from ._native import DolNativeError, build, lib  # noqa: F401
from . import ops, graph, bank  # noqa: F401
from .bank import AgentBank  # noqa: F401
from .graph import MixingPlan, communication_graph, csr_from_dense  # noqa: F401

__version__ = "0.1.0"
