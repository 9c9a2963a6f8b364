"""bench.py's config-5 round (ER W draw + device Neighbors + fused MLP step +
bit-exact mix, 1024 agents x 101,770) for the current environment; one JSON
line with the round and its phases (r06 MLP load-order experiments).
  python tools/cfg5_round_ab.py"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)

import torch  # noqa: E402

r = bench.config5_round(torch.device("cuda"), reps=20)
print(json.dumps({"f1_keep": os.environ.get("DOL_MLP_F1_KEEP", "0"),
                  "dw1_reverse": os.environ.get("DOL_MLP_DW1_REVERSE", "0"),
                  "ms_per_round": r["ms_per_round"], "ms_seq": r["ms_per_round_sequential"],
                  "phase_ms": r["phase_ms"]}), flush=True)
