"""Secondary mixing workloads (BASELINE configs 3 and 5): rounds/s and GB/s of
one X <- W X round for ring / random-regular / (optional) dense W.

  python tools/bench_configs.py [--agents 1024 8192] [--params 1048576] [--reps 10]
Prints one JSON line per (topology, N).  Algorithmic bytes = 2*N*P*4 (each
row read once, written once), as in the headline."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def time_plan(plan, X, Y, P, reps):
    for _ in range(2):
        plan.apply(X, Y, P=P)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        plan.apply(X, Y, P=P)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def mlp_round(N, d, h, c, B, p_edge, reps, dev, mix="split3"):
    """BASELINE config 5: a NEW Erdos-Renyi W every round (drawn on the device,
    graph.erdos_renyi_stochastic_hip), mixed on the dense matrix-core path
    (mix='split3') or bit-exactly by the LDS-gather CSR kernel after a device
    Neighbors pass (mix='csr'), then one fused local step of every agent's MLP
    (dol_mlp_step_f32)."""
    from dolhip.bank import AgentBank
    from dolhip.mlp import BatchedMLP, mlp_layout
    bank = AgentBank(N, mlp_layout(d, h, c), dev)
    mlp = BatchedMLP(bank, d, h, c)
    bank.buffer("x").normal_(0, 0.05)
    bank.buffer("y").zero_()
    bank.buffer("mom", zero=True)
    gen = torch.Generator(device=dev).manual_seed(2028)
    state = {"round": 0, "W": torch.empty(N, N, device=dev)}

    def draw():  # a new W every round: one HIP kernel (graph_draw.hip), seeded per round
        state["round"] += 1
        W = G.erdos_renyi_stochastic_hip(N, p_edge, 2028 * 1000003 + state["round"], dev, out=state["W"])
        if mix == "csr":
            state["plan"] = G.MixingPlan.from_dense(W, dense_kernel="csr", reuse=state.get("plan"))
        else:
            state["plan"] = G.MixingPlan.from_dense(W)
    X = torch.randn(N, B, d, device=dev)
    y = torch.randint(0, c, (N, B), device=dev)
    ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
          for k in ("graph", "local", "mix")}

    def one(k=None):
        r = (lambda nm, i: ev[nm][k][i].record()) if k is not None else (lambda nm, i: None)
        r("graph", 0)
        draw()
        r("graph", 1)
        r("local", 0)
        mlp.step(X, y, lr=0.05, momentum=0.5, first_step=False)   # fused fwd+CE+bwd+SGD (one kernel)
        r("local", 1)
        r("mix", 0)
        bank.mix(state["plan"])
        r("mix", 1)
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(reps):
        one(k)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    ms = {k: sum(a.elapsed_time(b) for a, b in v) / reps for k, v in ev.items()}

    # the pre-fusion path (torch.bmm fwd/bwd + the fused SGD kernel), same data, for comparison
    def unfused():
        mlp.step_unfused(X, y, lr=0.05, momentum=0.5, first_step=False)
    for _ in range(2):
        unfused()
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    for _ in range(reps):
        unfused()
    e_.record()
    torch.cuda.synchronize()
    ms["local_unfused"] = s_.elapsed_time(e_) / reps
    # the torch form of the same draw (nine kernels), for comparison
    G.erdos_renyi_stochastic(N, p_edge, gen)
    torch.cuda.synchronize()
    s_.record()
    for _ in range(reps):
        G.erdos_renyi_stochastic(N, p_edge, gen)
    e_.record()
    torch.cuda.synchronize()
    ms["graph_torch"] = s_.elapsed_time(e_) / reps

    P = bank.P
    flops_fb = 2.0 * N * B * (d * h + h * c) * 3  # fwd + two backward GEMMs per layer
    local_bytes = N * (4 * P + B * d) * 4           # w, mom in + out, X in (compulsory)
    out = {"workload": "config5: time-varying ER p=%.2f (new W per round, on device) %s mix + fused MLP "
                       "%d-%d-%d local step" % (p_edge, "bit-exact LDS-gather CSR" if mix == "csr" else
                                                "dense MFMA (split3)", d, h, c), "mix_path": mix,
           "agents": N, "params": P, "batch": B, "ms_per_round": el * 1e3, "rounds_per_s": 1 / el, "kernel_ms": ms,
           "mix_TFLOPs": 2.0 * N * N * P / (ms["mix"] / 1e3) / 1e12,
           "local_TFLOPs": flops_fb / (ms["local"] / 1e3) / 1e12,
           "local_GBps": local_bytes / (ms["local"] / 1e3) / 1e9,
           "local_frac_of_8TBps": local_bytes / (ms["local"] / 1e3) / 1e9 / 8000.0,
           "local_speedup_vs_unfused": ms["local_unfused"] / ms["local"]}
    print(json.dumps(out), flush=True)
    del bank, mlp, state, X, y
    torch.cuda.empty_cache()


def dgd_round(N, P, topo, objective, momentum, steps, reps, dev):
    """BASELINE config 3: one fused DGD round (mix + local momentum-SGD steps on a
    separable synthetic loss) over all agents; algorithmic bytes = N*P*4 *
    (x read + y write + target read [+ momentum read + write])."""
    from dolhip.synthetic import SeparableDGD
    if topo == "ring":
        torch.manual_seed(2028)
        plan = G.MixingPlan(G.communication_csr("circle", "stochastic", N)[0], dev)
    else:
        plan = G.MixingPlan(G.random_regular_csr(N, int(topo[2:]), seed=2028), dev)
    prob = SeparableDGD(plan, P, objective=objective, lr=0.01, momentum=momentum, local_steps=steps, seed=7)
    for _ in range(2):
        prob.round()
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    for _ in range(reps):
        prob.round()
    e_.record()
    torch.cuda.synchronize()
    ms = s_.elapsed_time(e_) / reps
    alg = N * P * 4 * (3 + (2 if momentum else 0))
    print(json.dumps({"workload": "config3: fused DGD round (mix + %d local step%s)" % (steps, "s" * (steps > 1)),
                      "topology": topo, "kernel": plan.kind, "objective": objective, "momentum": momentum,
                      "agents": N, "params": P, "ms_per_round": ms, "rounds_per_s": 1e3 / ms,
                      "algorithmic_bytes": alg, "GBps": alg / (ms / 1e3) / 1e9,
                      "frac_of_8TBps": alg / (ms / 1e3) / 1e9 / 8000.0}), flush=True)
    del prob, plan
    torch.cuda.empty_cache()


def dgd_pm_round(N, P, topo, objective, momentum, steps, reps, dev):
    """Config 3's fused round on the parameter-major bank (dol_dgd_csr_pm_f32):
    XT, YT, TT (targets), MT (momentum) all [P, round_up(N, 4)]; algorithmic
    bytes as dgd_round."""
    from dolhip import ops
    if topo == "ring":
        torch.manual_seed(2028)
        c = G.communication_csr("circle", "stochastic", N)[0]
    else:
        c = G.random_regular_csr(N, int(topo[2:]), seed=2028)
    ld = (N + 3) // 4 * 4
    g = torch.Generator(device=dev).manual_seed(7)
    XT, TT = (torch.empty(P, ld, device=dev).normal_(generator=g) for _ in range(2))
    YT = torch.empty_like(XT)
    MT = torch.zeros_like(XT) if momentum else None
    rp = torch.as_tensor(c.rowptr, dtype=torch.int32, device=dev)
    col = torch.as_tensor(c.col, dtype=torch.int32, device=dev)
    val = torch.as_tensor(c.val, dtype=torch.float32, device=dev)
    state = {"first": True}

    def one():
        ops.dgd_csr_pm(XT, YT, rp, col, val, TT, MT, objective=objective, steps=steps, lr=0.01, momentum=momentum,
                       first_step=state["first"])
        state["first"] = False
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    for _ in range(reps):
        one()
    e_.record()
    torch.cuda.synchronize()
    ms = s_.elapsed_time(e_) / reps
    alg = N * P * 4 * (3 + (2 if momentum else 0))
    print(json.dumps({"workload": "config3: fused DGD round (mix + %d local step%s), parameter-major bank"
                                  % (steps, "s" * (steps > 1)),
                      "topology": topo + "-pm", "kernel": "csr_pm + DGD epilogue", "objective": objective,
                      "momentum": momentum, "agents": N, "params": P, "ms_per_round": ms, "rounds_per_s": 1e3 / ms,
                      "algorithmic_bytes": alg, "GBps": alg / (ms / 1e3) / 1e9,
                      "frac_of_8TBps": alg / (ms / 1e3) / 1e9 / 8000.0}), flush=True)
    del XT, TT, YT, MT
    torch.cuda.empty_cache()


def pm_round(N, P, topo, reps, dev, X, Y):
    """One X <- W X round on the parameter-major bank (XT[p][j], p-row stride
    round_up(N, 4)), reusing X / Y's memory as XT / YT."""
    from dolhip import ops
    if topo == "ring":
        torch.manual_seed(2028)
        c = G.communication_csr("circle", "stochastic", N)[0]
    else:
        c = G.random_regular_csr(N, int(topo[2:]), seed=2028)
    ld = (N + 3) // 4 * 4
    yoff = int(os.environ.get("PM_YOFF", "0"))  # floats: YT's start relative to Y's (HBM channel placement probe)
    XT = X.view(-1)[: P * ld].view(P, ld)
    YT = Y.view(-1)[yoff: yoff + P * ld].view(P, ld)
    rp = torch.as_tensor(c.rowptr, dtype=torch.int32, device=dev)
    col = torch.as_tensor(c.col, dtype=torch.int32, device=dev)
    val = torch.as_tensor(c.val, dtype=torch.float32, device=dev)
    for _ in range(2):
        ops.mix_csr_pm(XT, YT, rp, col, val)
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    for _ in range(reps):
        ops.mix_csr_pm(XT, YT, rp, col, val)
    e_.record()
    torch.cuda.synchronize()
    ms = s_.elapsed_time(e_) / reps
    alg = 2 * N * P * 4
    print(json.dumps({"topology": topo + "-pm", "kernel": "csr_pm (parameter-major bank)", "agents": N, "params": P,
                      "yoff": yoff, "x_ptr_mod_2M": XT.data_ptr() % (1 << 21), "y_minus_x": YT.data_ptr() - XT.data_ptr(),
                      "nnz": int(c.nnz), "ms_per_launch": ms, "rounds_per_s": 1e3 / ms,
                      "GBps": alg / (ms / 1e3) / 1e9, "frac_of_8TBps": alg / (ms / 1e3) / 1e9 / 8000.0}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, nargs="*", default=[1024, 8192])
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--topologies", nargs="+", default=["ring", "ring-eps5", "rr4", "dense-er0.1"])
    ap.add_argument("--dense-max-agents", type=int, default=2048)
    ap.add_argument("--mlp", type=int, nargs="*", default=[1024], help="agent counts for the config-5 MLP round")
    ap.add_argument("--mlp-mix", nargs="+", default=["split3", "csr"], help="config-5 mix paths")
    ap.add_argument("--dgd", type=int, nargs="*", default=[1024], help="agent counts for the config-3 DGD round")
    ap.add_argument("--dgd-topologies", nargs="+", default=["ring", "rr4"])
    ap.add_argument("--dgd-pm", type=int, nargs="*", default=[1024],
                    help="agent counts for the config-3 round on the parameter-major bank")
    a = ap.parse_args()
    dev = torch.device("cuda")
    P = a.params
    for N in a.mlp:
        for mix in a.mlp_mix:
            mlp_round(N, 784, 128, 10, 32, 0.1, a.reps, dev, mix=mix)
    for N in a.dgd:
        for topo in a.dgd_topologies:
            dgd_round(N, P, topo, "least_squares", 0.5, 1, a.reps, dev)
            dgd_round(N, P, topo, "logistic", 0.0, 1, a.reps, dev)
    for N in a.dgd_pm:
        for topo in a.dgd_topologies:
            dgd_pm_round(N, P, topo, "least_squares", 0.5, 1, a.reps, dev)
            dgd_pm_round(N, P, topo, "logistic", 0.0, 1, a.reps, dev)
    for N in a.agents:
        ld = row_stride(P)
        X = torch.empty(N, ld, device=dev).normal_()
        Y = torch.empty_like(X)
        for topo in a.topologies:
            if topo.endswith("-pm"):  # the parameter-major bank: XT [P, N] (dol_mix_csr_pm_f32)
                pm_round(N, P, topo[:-3], a.reps, dev, X, Y)
                continue
            t0 = time.time()
            steps = 1
            extra = {}
            if topo.startswith("ring"):
                torch.manual_seed(2028)
                plan = G.MixingPlan.from_graph(G.communication_graph("circle", "stochastic", N)[0], dev)
                if "-eps" in topo:
                    steps = int(topo.split("-eps")[1])
            elif topo.startswith("rr"):
                plan = G.MixingPlan(G.random_regular_csr(N, int(topo[2:]), seed=2028), dev)
            elif topo.startswith("dense-er"):
                if N > a.dense_max_agents:
                    continue
                p_edge = float(topo[len("dense-er"):])
                gen = torch.Generator().manual_seed(2028)
                A = (torch.rand(N, N, generator=gen) < p_edge).float()
                A.fill_diagonal_(0)
                R = torch.rand(N, N, generator=gen) * A
                R /= R.sum(0).clamp_min(1e-30)
                plan = G.MixingPlan.from_graph(R.T.contiguous(), dev, dense=True)
                extra["flops"] = 2.0 * N * N * P
            else:
                raise SystemExit(f"unknown topology {topo}")
            build_s = time.time() - t0
            if steps > 1:
                def run():
                    plan.apply_steps(X, Y, steps, P=P)
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s_.record()
                for _ in range(a.reps):
                    run()
                e_.record()
                torch.cuda.synchronize()
                ms = s_.elapsed_time(e_) / a.reps
            else:
                ms = time_plan(plan, X, Y, P, a.reps)
            alg = 2 * N * P * 4
            rec = {"topology": topo, "kernel": plan.kind, "agents": N, "params": P, "nnz": plan.csr.nnz,
                   "rounds_per_launch": steps, "ms_per_launch": ms, "rounds_per_s": steps * 1e3 / ms,
                   "GBps": alg / (ms / 1e3) / 1e9, "frac_of_8TBps": alg / (ms / 1e3) / 1e9 / 8000.0,
                   "plan_build_s": build_s}
            if plan.kind == "csr":  # the naive (nnz + N) * P * 4 figure beside the 2 * N * P * 4 one
                rec["GBps_naive_nnz_plus_n"] = (plan.csr.nnz + N) * P * 4 / (ms / 1e3) / 1e9
            if "flops" in extra:
                tf = extra["flops"] / (ms / 1e3) / 1e12
                rec.update({"TFLOPs": tf, "mfma_util_vs_157TF": tf / 157.3})
            print(json.dumps(rec), flush=True)
        del X, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
