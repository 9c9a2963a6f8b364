"""Headline benchmark: consensus rounds/s at 8192 agents x 2^20 params.

One step = one synchronous gossip round X <- W X over all agents (FedLCon's
inner step, DIST/simulators.py:190-196), W = communication_graph("circle",
"stochastic", 8192) seeded 2028 (the reference's own construction, ring
kernel).  Inputs are synthetic fp32 (randn), resident in HBM before timing.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Without a launcher, `--gpus N > 1` starts the N ranks itself (child
processes, before any GPU call) and relays rank 0's line; a run whose joined
world differs from --gpus exits non-zero.  The line's `parallel` field lists
the world size, backend and device each rank saw.

Strong scaling: the 8192 agents are split into contiguous blocks, one per
rank; each round exchanges the two boundary rows with the neighbouring ranks
(RCCL send/recv) while the interior rows are mixed.

Rank 0 prints ONE JSON line.  `roofline` prices the dominant kernel (the
ring mix) from HIP events around every launch in the timed region;
`cpu_baseline` times the reference-structured torch-CPU round
(oracle/ref_cpu.py) on this host on a bounded sample (N=1 only).
Secondaries (N=1, skipped with --no-primal-dual): FedADMM round (config 4),
FedLCon eps = 5 fused pass, random 4-regular mix on the parameter-major bank,
the Erdos-Renyi mix on the matrix cores (split3) and bit-exact, and a whole
config-5 round (ER draw + device Neighbors + fused MLP local step + exact mix).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "distributed-optimization-and-learning_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

def _log(msg: str) -> None:
    """Progress on stderr (stdout carries only the one JSON line), with the
    device's free memory once CUDA is up (a leg that OOMs names what held it)."""
    free = ""
    try:
        if torch.cuda.is_initialized():
            f, _ = torch.cuda.mem_get_info()
            free = f" [free {f / 2**30:.1f} GiB, torch {torch.cuda.memory_allocated() / 2**30:.1f} GiB]"
    except Exception:  # noqa: BLE001 -- diagnostics only
        pass
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}{free}", file=sys.stderr, flush=True)


METRIC = "consensus rounds/sec at 8192 agents x 1M params (1/8 GPU) + % of HBM peak"
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--agents", type=int, default=8192)
    ap.add_argument("--params", type=int, default=1 << 20)
    ap.add_argument("--cpu-agents", type=int, nargs="+", default=[64, 256, 1024],
                    help="CPU baseline sample sizes (agents; SURVEY 8d)")
    ap.add_argument("--cpu-seconds", type=float, default=4.0, help="CPU seconds per sample below 512 agents")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline (profiling runs)")
    ap.add_argument("--no-copy", action="store_true", help="skip the copy-kernel calibration")
    ap.add_argument("--map-ring", type=int, default=1, help="1: the ring's x / y as mapped blocks (dol_bank_alloc, the bank default); 0: torch's allocator")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_ring_8192x1M.json"))
    ap.add_argument("--no-primal-dual", action="store_true", help="skip the secondary measurements (primal/dual round, FedLCon eps=5, dense ER mix)")
    ap.add_argument("--pd-steps", type=int, default=10)
    ap.add_argument("--launch-check", action="store_true",
                    help="only bring the ranks up: every rank joins the process group and rank 0 prints the "
                         "world each rank saw (the launcher's own test; no kernels, no GPU needed under gloo)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` without a launcher: start
    N copies of this script as child processes, one rank each (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their
    environment, exactly what torch.distributed.run sets), relay rank 0's JSON
    line, and return non-zero if any rank fails or the line reports a world
    other than N.  This process never touches the GPU (no HIP call before or
    after the children start; they are children, not an exec).  A rank that
    dies takes the others down at once instead of leaving them in a
    collective until its timeout."""
    import signal
    import subprocess
    import threading
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    lines: list = []

    def relay(stream):  # rank 0's stdout: the JSON line (anything else goes to stderr)
        for raw in stream:
            s = raw.decode(errors="replace").rstrip("\n")
            if s.startswith("{"):
                lines.append(s)
            else:
                print(s, file=sys.stderr, flush=True)

    def stop_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_end = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    reader = None
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", ROLE_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       DOL_BENCH_LAUNCHER="bench.py --gpus (child processes)")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                          stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                          start_new_session=True))
        reader = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
        reader.start()
        failed = None
        while failed is None and any(p.poll() is None for p in procs):
            for r, p in enumerate(procs):
                if p.poll() not in (None, 0):
                    failed = (r, p.returncode)
                    break
            time.sleep(0.2)
        if failed is None:
            failed = next(((r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0), None)
        if failed is not None:
            _log(f"ERROR: rank {failed[0]} exited with {failed[1]}; stopping the other ranks")
            stop_all()
            return failed[1] if failed[1] > 0 else 1
    except BaseException:
        stop_all()
        raise
    reader.join(timeout=10)
    if len(lines) != 1:
        _log(f"ERROR: rank 0 printed {len(lines)} JSON lines, expected one")
        return 1
    got = json.loads(lines[0]).get("n_gpus")
    if got != n:
        _log(f"ERROR: the line reports n_gpus={got}, launched {n} ranks")
        return 1
    print(lines[0], flush=True)
    return 0


def rank_infos(world: int, rank: int, local: int, backend: str, device) -> list:
    """What every rank saw (world size, rank, backend, device), gathered to all
    ranks: the line's `parallel` field, so a run that came up with fewer ranks
    than asked cannot pass for an N-GPU number."""
    me = {"rank": rank, "local_rank": local, "world_size": world,
          "backend": dist.get_backend() if world > 1 else "none", "device": str(device), "pid": os.getpid(),
          "launcher": os.environ.get("DOL_BENCH_LAUNCHER", "torch.distributed.run" if world > 1 else "none")}
    if world == 1:
        return [me]
    out = [None] * world
    dist.all_gather_object(out, me)
    return out


def launch_check(args, world: int, rank: int, local: int, backend: str) -> int:
    """--launch-check: join the group, gather what each rank saw, rank 0 prints
    one JSON line in the bench line's shape (n_gpus, parallel); no kernels."""
    from dolhip import parallel
    if world > 1:
        dev = None
        if backend == "nccl":
            dev = torch.device("cuda", int(os.environ.get("DOL_DEVICE_MAP", local)))
            torch.cuda.set_device(dev)
        parallel.init_process_group(backend, device=dev)
    infos = rank_infos(world, rank, local, backend, "cpu" if backend == "gloo" else f"cuda:{local}")
    if os.environ.get("DOL_BENCH_FAIL_RANK") == str(rank):  # tests: a rank that dies after joining
        os._exit(3)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "steps": 0,
                          "parallel": {"world_size": world, "backend": infos[0]["backend"], "ranks": infos}}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def ring_weights(n: int):
    """W = communication_graph('circle', 'stochastic', n) after manual_seed(2028), built
    sparse (bit-identical, tests/test_graph_host.py) so 8 ranks don't each hold a dense W."""
    from dolhip import graph as G
    torch.manual_seed(2028)
    rw = G.communication_csr("circle", "stochastic", n)[0].ring_weights()  # = csr_from_dense(communication_graph(...))
    assert rw is not None
    return rw


def copy_peak(device, X=None, Y=None, P=None, gib: float = 8.0, reps: int = 20) -> dict:
    """HBM calibration: the best of three copies on this box, each timed with
    HIP events — a flat nontemporal copy over 2 x `gib` GiB and over 2 x 16 GiB,
    and (given the bench's own [N, ld] buffers) a copy in the ring kernel's tile
    kernel's own access pattern over the same rows (dol_stream_copy_rows_f32:
    the ring kernel with the stencil replaced by the row itself).  Each copy's
    rate is its FASTEST of `reps` launches (a ceiling; the mean is reported
    beside it).  Returns every rate and the winner; `frac_of_measured_copy`
    divides the ring kernel's mean rate by the winner."""
    from dolhip import ops

    def timed(fn, nbytes):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(device)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for s, e in ev:
            s.record()
            fn()
            e.record()
        torch.cuda.synchronize(device)
        ms = [s.elapsed_time(e) for s, e in ev]
        return nbytes / (min(ms) / 1e3) / 1e9, nbytes / (sum(ms) / len(ms) / 1e3) / 1e9

    out, mean = {}, {}
    if X is not None:
        out["ring_kernel_pattern_copy"], mean["ring_kernel_pattern_copy"] = timed(
            lambda: ops.stream_copy_rows(X, Y, P=P), 2 * X.shape[0] * P * 4)
    for g in (gib, 16.0):
        n = int(g * (1 << 30) / 4)
        a = torch.empty(n, dtype=torch.float32, device=device).normal_()
        b = torch.empty_like(a)
        k = f"flat_nt_copy_{int(g)}GiB"
        out[k], mean[k] = timed(lambda: ops.stream_copy(a, b), 2 * n * 4)
        del a, b
        torch.cuda.empty_cache()
    best = max(out, key=out.get)
    return {"GBps": out[best], "variant": best, "statistic": "fastest launch", "all_GBps": out,
            "all_GBps_mean": mean}


def cpu_baseline(sizes, P: int, seconds: float, full_agents: int):
    """The reference-structured torch-CPU round (oracle/ref_cpu.py: the O(N^2)
    Neighbors scan + consensus + load_state_dict) at each N in `sizes` (SURVEY
    §8d: 64, 256, 1024 agents x 2^20), and the vectorised torch-CPU ring round
    beside it, on the threads this process may use (os.sched_getaffinity; the
    box's CPU share).  `value` extrapolates the largest N per byte to
    `full_agents` (optimistic for the reference: its scan grows as N^2)."""
    from oracle import ref_cpu
    from dolhip import graph as G
    # the box's CPU share: OMP_NUM_THREADS (16 per GPU on the pool, where
    # os.cpu_count() and the affinity mask report the whole machine); else the
    # affinity mask
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = int(os.environ.get("OMP_NUM_THREADS") or aff)
    torch.set_num_threads(threads)
    per_n, vec_n = {}, {}
    for n in sizes:
        _log(f"cpu baseline: {n} agents x {P} on {threads} threads")
        torch.manual_seed(2028)
        W = G.communication_graph("circle", "stochastic", n)[0]
        X = torch.randn(n, P)
        # a warm-up round at every size, then >= 2 timed rounds (>= `seconds` below 512 agents)
        rounds, sec = ref_cpu.time_rounds(W, X, min_seconds=seconds if n < 512 else 0.0,
                                          max_rounds=50 if n < 512 else 2, warmup=True)
        per_n[n] = {"rounds": rounds, "seconds": sec, "rounds_per_s": rounds / sec,
                    "GBps": 2 * n * P * 4 * rounds / sec / 1e9}
        rw = G.csr_from_dense(W).ring_weights()
        vr, vsec = ref_cpu.time_vectorized(X, torch.from_numpy(rw[0]), torch.from_numpy(rw[1]),
                                           min_seconds=seconds / 3)
        vec_n[n] = {"rounds": vr, "seconds": vsec, "rounds_per_s": vr / vsec, "GBps": 2 * n * P * 4 * vr / vsec / 1e9}
        del W, X
    big = max(sizes)
    value = per_n[big]["rounds_per_s"] * big / full_agents
    # the reference's round is O(N^2) in its Neighbors scan and O(N) in the
    # consensus work: least-squares fit of seconds/round = a N^2 + b N over the
    # samples, evaluated at full_agents (the per-byte `value` ignores the N^2 part)
    fit = _fit_n2_n({n: per_n[n]["rounds_per_s"] for n in sizes}, full_agents) if len(sizes) >= 2 else None
    return {
        "value": value,
        "unit": "rounds/s",
        "cores": threads,
        "os_cpu_count": os.cpu_count(),
        "affinity_cpus": aff,
        "kind": "port",
        "per_agents": per_n,
        "fit_a_n2_plus_b_n": fit,
        "vectorized": {"value": vec_n[big]["rounds_per_s"] * big / full_agents, "unit": "rounds/s", "cores": threads,
                       "kind": "port", "per_agents": vec_n,
                       "sample": "vectorized torch-CPU ring round (oracle/ref_cpu.py: roll + mul + add over the whole "
                                 "matrix); value per-byte extrapolated from the largest N"},
        "sample": (f"reference-structured torch-CPU round (Neighbors scan + consensus + load_state_dict, "
                   f"oracle/ref_cpu.py), circle/stochastic, N in {list(sizes)} x {P} params on {threads} threads; "
                   f"value = the N={big} rate x {big}/{full_agents} (per-byte extrapolation to {full_agents} agents)"),
    }


def _fit_n2_n(samples: dict, n_full: int):
    """Non-negative least squares seconds/round = a n^2 + b n (a, b >= 0: a
    round cannot get cheaper with more agents) over {n: rounds_per_s},
    evaluated at n_full.  Timing noise can no longer push a or b below zero
    and so move the extrapolated CPU rate either way."""
    from scipy.optimize import nnls
    ns = sorted(samples)
    A = np.array([[n * n, n] for n in ns], dtype=np.float64)
    t = np.array([1.0 / samples[n] for n in ns])
    scale = A.max(axis=0)  # column scaling: n^2 and n differ by orders of magnitude
    coef, resid = nnls(A / scale, t)
    a, b = coef / scale
    t_full = a * n_full ** 2 + b * n_full
    return {"rounds_per_s": 1.0 / t_full if t_full > 0 else None, "seconds_per_round": t_full,
            "a_s_per_agent2": float(a), "b_s_per_agent": float(b), "residual_s": float(resid),
            "samples": {int(n): float(1.0 / samples[n]) for n in ns}}


def cpu_secondaries(P: int, full_agents: int, admm_sizes=(64, 256), cfg5_sizes=(64, 128, 256),
                    cfg5_agents: int = 1024):
    """CPU legs beside the secondaries (reference-structured torch-CPU code in
    oracle/ref_cpu.py, same threads as cpu_baseline):
      * FedADMM: FedAdmm_Client.update_weights (autograd least-squares loss +
        the ADMM term + SGD momentum, 10 local steps) + update_duals + the
        server's deepcopy + average_weights (DEC/clients.py:36-53,125-144,
        DEC/servers.py:42-48) over n clients x P; the per-client cost does not
        depend on n, so `value` = the largest n's rate x n / full_agents;
      * config 5: every agent's 784-128-10 MLP step (nn.Module, CrossEntropyLoss,
        SGD momentum, batch 32; DIST/clients.py:34-59) + the consensus round
        with a new ER p = 0.1 W (Neighbors scan + consensus + load_state_dict);
        the local steps grow as n and Neighbors + consensus as n^2, so `value`
        = the non-negative least-squares fit seconds/round = a n^2 + b n over
        the three samples, evaluated at cfg5_agents (the largest sample's rate
        scaled by (n / cfg5_agents)^2, the r03 bound, is reported beside it).
    Every size runs a warm-up round, then 2 timed rounds."""
    from oracle import ref_cpu
    threads = torch.get_num_threads()
    adm = {}
    for n in admm_sizes:
        _log(f"cpu FedADMM: {n} clients x {P}")
        r, sec = ref_cpu.time_admm_rounds(n, P, rounds=2, warmup=True)
        adm[n] = {"rounds": r, "seconds": sec, "rounds_per_s": r / sec, "ms_per_client": sec / r / n * 1e3}
    big = max(admm_sizes)
    c5 = {}
    for n in cfg5_sizes:
        _log(f"cpu config 5: {n} agents")
        r, sec = ref_cpu.time_config5_rounds(n, rounds=2, warmup=True)
        c5[n] = {"rounds": r, "seconds": sec, "rounds_per_s": r / sec}
    b5 = max(cfg5_sizes)
    fit5 = _fit_n2_n({n: v["rounds_per_s"] for n, v in c5.items()}, cfg5_agents)
    fit5["n2_bound_rounds_per_s"] = c5[b5]["rounds_per_s"] * (b5 / cfg5_agents) ** 2
    if fit5["rounds_per_s"] is None:  # degenerate samples: the per-byte-squared bound instead
        fit5["rounds_per_s"] = fit5["n2_bound_rounds_per_s"]
    return {
        "fedadmm": {"value": adm[big]["rounds_per_s"] * big / full_agents, "unit": "rounds/s", "cores": threads,
                    "kind": "port", "per_clients": adm,
                    "sample": f"reference-structured torch-CPU FedADMM round (oracle/ref_cpu.py AdmmClient + "
                              f"average_weights), 10 local steps, n in {list(admm_sizes)} x {P}; value = the n={big} "
                              f"rate x {big}/{full_agents} (per client, linear)"},
        "config5": {"value": fit5["rounds_per_s"], "unit": "rounds/s", "cores": threads,
                    "kind": "port", "per_agents": c5, "fit_a_n2_plus_b_n": fit5,
                    "sample": f"reference-structured torch-CPU config-5 round (oracle/ref_cpu.py "
                              f"time_config5_rounds: per-agent nn.Module MLP step + ER W Neighbors/consensus), n in "
                              f"{list(cfg5_sizes)}, warm-up + 2 rounds each; value = the non-negative least-squares fit "
                              f"seconds/round = a n^2 + b n evaluated at n={cfg5_agents}"},
    }


def primal_dual_round(N: int, P: int, world: int, rank: int, device, steps: int, local_steps: int = 10):
    """Secondary measurement (BASELINE config 4, primal/dual side): one FedADMM
    round of dolhip.synthetic.SeparableADMM on least squares over ALL N agents
    (frac = 1), `local_steps` local momentum-SGD steps per client in registers:
    the fused client round (dol_admm_ls_round_f32: w = theta, ADMM gradient +
    SGD steps, dual ascent, ||w - theta||^2 / ||alpha||^2 partials) over the
    local agent block, then the server mean — local ordered sum + all_reduce
    (RCCL) + / N ("fast"; DEC/servers.py:42-48's order is the "exact" mode).
    Bit-exact against the reference's own FedAdmm_Server on a least-squares
    model (tests/test_admm_gpu.py).  Timed like the headline (barrier, max over
    ranks); each kernel's share from HIP events."""
    from dolhip import ops
    from dolhip.synthetic import SeparableADMM
    prob = SeparableADMM(N, P, rho=0.1, lr=0.1, momentum=0.5, local_steps=local_steps, frac=1.0, seed=2028,
                         device=device, mean="fast")
    fused = prob.fused  # client round + this rank's ordered sum in one pass (dol_admm_ls_round_mean_f32)
    names = ("round_mean",) if fused else ("client_round", "mean")
    ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
          for k in names}
    rnd, rnd_mean = ops.admm_ls_round, prob._round_mean
    state = {"k": None}

    def timed_round(*a, **kw):
        k = state["k"]
        if k is not None:
            ev["client_round"][k][0].record()
        rnd(*a, **kw)
        if k is not None:
            ev["client_round"][k][1].record()
            ev["mean"][k][0].record()

    def timed_round_mean(*a, **kw):
        k = state["k"]
        if k is not None:
            ev["round_mean"][k][0].record()
        out = rnd_mean(*a, **kw)
        if k is not None:
            ev["round_mean"][k][1].record()
        return out

    prob._round = timed_round
    prob._round_mean = timed_round_mean
    prob.round()  # warm-up (first momentum step)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        state["k"] = k
        prob.round()
        if not fused:
            ev["mean"][k][1].record()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    n = prob.n
    row_bytes = n * P * 4
    # compulsory bytes: client round reads t, alpha, buf and writes w, alpha, buf; the mean reads w, writes theta
    # (fused: the new w rows are summed in registers, theta read once and written once)
    alg = ({"round_mean": 6 * row_bytes + 2 * P * 4} if fused else
           {"client_round": 6 * row_bytes, "mean": row_bytes + P * 4})
    kern = {}
    for nm in alg:
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev[nm]]))
        kern[nm] = {"ms": ms, "GBps": alg[nm] / (ms / 1e3) / 1e9, "frac": alg[nm] / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS,
                    "algorithmic_bytes": alg[nm]}
    two_kernel = None
    if fused:
        # the same round on the two-kernel path (client round, then the ordered
        # sum re-reading the rows), same buffers, for comparison
        state["k"] = None
        prob.fused = False
        prob.round()
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(3):
            prob.round()
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        tk = torch.tensor([(time.perf_counter() - t1) / 3], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(tk, op=dist.ReduceOp.MAX)
        prob.fused = True
        two_kernel = {"ms_per_round": float(tk.item()) * 1e3,
                      "what": "dol_admm_ls_round_f32 + ordered sum (the mean re-reads the new rows), host-timed"}
    exact = None
    if world > 1:
        # the bit-exact server mean across ranks (DEC/servers.py:42-48's order):
        # one all_to_all of the sampled rows to column blocks, an ordered sum per
        # block, one all_gather (parallel.global_mean_exact); host-timed, max over ranks
        from dolhip import parallel as par
        order = [int(g) for g in prob.sample()]
        out_t = torch.empty_like(prob.theta)
        par.global_mean_exact(prob.w, prob.lo, prob.hi, order, P, out=out_t)
        torch.cuda.synchronize(device)
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(3):
            par.global_mean_exact(prob.w, prob.lo, prob.hi, order, P, out=out_t)
        torch.cuda.synchronize(device)
        dist.barrier()
        ex = torch.tensor([(time.perf_counter() - t1) / 3], dtype=torch.float64, device=device)
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        exact = {"ms": float(ex.item()) * 1e3, "sampled": len(order),
                 "bytes_moved_per_rank": prob.n * P * 4 * (world - 1) // world,
                 "what": "global_mean_exact: all_to_all of the sampled rows to column blocks + ordered sum + all_gather"}
    hist = prob.history
    columns = None
    if world > 1:
        # the parameter-sharded problem: every rank runs all
        # sampled agents on its column block, theta exact, no collective per round
        del prob
        torch.cuda.empty_cache()
        colp = SeparableADMM(N, P, rho=0.1, lr=0.1, momentum=0.5, local_steps=local_steps, frac=1.0, seed=2028,
                             device=device, shard="columns")
        colp.round()
        torch.cuda.synchronize(device)
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(steps):
            colp.round()
        torch.cuda.synchronize(device)
        dist.barrier()
        tc = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=device)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        cms = float(tc.item()) / steps * 1e3
        colp.history  # (collective: the metric partials summed across ranks)
        columns = {"rounds_per_s": 1e3 / cms, "ms_per_round": cms, "columns_per_rank": colp.Pl,
                   "GBps_per_rank": (6 * N * colp.Pl + 2 * colp.Pl) * 4 / (cms / 1e3) / 1e9,
                   "what": "SeparableADMM(shard='columns'): dol_admm_ls_round_mean_f32 over all sampled agents on "
                           "this rank's parameter columns, theta bit-exact (DEC/servers.py:42-48's order), no "
                           "collective on the round path"}
        prob = colp
    out = {"rounds_per_s": steps / el, "ms_per_round": el / steps * 1e3, "agents": N, "params": P,
           "local_steps": local_steps, "kernels": kern, "fused_round_mean": fused, "two_kernel_round": two_kernel,
           "exact_mean": exact, "column_sharded_exact": columns,
           "primal_resid_sq_last": hist[-1]["primal_resid_sq"], "dual_sq_last": hist[-1]["dual_sq"],
           "what": "FedADMM least-squares round over all agents: fused client round (w = theta, %d momentum-SGD "
                   "steps with the ADMM term, dual ascent) with this rank's ordered sum of the new rows in the "
                   "same pass, + all_reduce mean at world > 1" % local_steps}
    del prob
    torch.cuda.empty_cache()
    return out


def dgd_rounds(device, N: int = 1024, P: int = 1 << 20, reps: int = 10):
    """Secondary (BASELINE config 3: synthetic least-squares / logistic, 1024
    agents x 2^20, ring + random-regular W, mixing-bound): one decentralised
    gradient-descent round (DIST/simulators.py:147-162: consensus, then one
    local momentum-SGD step, DIST/clients.py:43-49) through the product
    classes -- SeparableDGD on the agent-major bank (ring: the fused
    dol_dgd_ring_f32) and SeparableDGDPM on the parameter-major bank (random
    4-regular: dol_dgd_csr_pm_f32) -- each one HBM pass, bit-exact against the
    oracle (tests/test_dgd_gpu.py, tests/test_pmajor_gpu.py).  Algorithmic
    bytes N*P*4 * (x + y + target [+ momentum in + out])."""
    from dolhip import graph as G
    from dolhip.synthetic import SeparableDGD, SeparableDGDPM
    torch.manual_seed(2028)
    ring_plan = G.MixingPlan(G.communication_csr("circle", "stochastic", N)[0], device)
    rr_plan = G.MixingPlan(G.random_regular_csr(N, 4, seed=2028), device)
    out = {}
    for name, cls, plan in (("ring", SeparableDGD, ring_plan), ("rr4_pm", SeparableDGDPM, rr_plan)):
        for objective, mom in (("least_squares", 0.9), ("logistic", 0.0)):
            prob = cls(plan, P, objective=objective, lr=0.01, momentum=mom, local_steps=1, seed=7)
            for _ in range(2):
                prob.round()
            torch.cuda.synchronize(device)
            _warm(prob.round, seconds=0.1)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                prob.round()
            e.record()
            torch.cuda.synchronize(device)
            ms = s.elapsed_time(e) / reps
            alg = N * P * 4 * (3 + (2 if mom else 0))
            out[f"{name}_{objective}"] = {"ms_per_round": ms, "rounds_per_s": 1e3 / ms, "momentum": mom,
                                          "GBps": alg / (ms / 1e3) / 1e9,
                                          "frac": alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS,
                                          "class": cls.__name__}
            del prob
            torch.cuda.empty_cache()
    return {"agents": N, "params": P, "local_steps": 1, "rounds": out,
            "what": "config 3 DGD round: mix + one local SGD step in one pass (ring: agent-major bank; random "
                    "4-regular: parameter-major bank), least squares with momentum 0.9 and logistic without"}


def _warm(fn, seconds: float = 0.25) -> None:
    """Run fn() back to back for ~seconds before a short leg is timed: after an
    idle gap the GPU's clocks take tens of ms to ramp, and a 10-rep leg of
    ~1 ms calls otherwise lands inside the ramp (split3 at 1024 agents: 1.25
    ms per round timed from idle, 1.11 ms timed right after other work, same
    process; tools/dense_heat_probe.py, profiles/r04p_dense_clock_ramp.jsonl)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()


def _events_ms(fn, reps: int) -> float:
    """Mean ms of `reps` calls of fn() between two events on the current stream."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


RING_STEPS_KERNELS = {1: "ring_steps_kernel (register tiles)", 2: "ring_stream_kernel", 3: "ring_stream_dma_kernel",
                      4: "ring_stream_dma_kernel (block-synchronised)",
                      5: "ring_stream_dma_kernel (64-row tiles, column-tile-fastest sweep)"}


def fedlcon_eps_round(device, ring, N: int, P: int, eps: int = 5, reps: int = 10):
    """Secondary (N = 1): FedLCon's eps consensus rounds as one fused pass over
    the headline's buffers, through the product call: an AgentBank over
    ring.x / ring.y and the ring MixingPlan of the same W, bank.mix(plan,
    steps=eps) exactly as weighted_average/simulators.py:233 calls it.  The
    first call tunes the kernel for these buffers (ops.mix_ring_steps); every
    variant's time and the library default's are reported beside the result."""
    from dolhip import graph as G, ops
    from dolhip.bank import AgentBank
    torch.manual_seed(2028)
    plan = G.MixingPlan(G.communication_csr("circle", "stochastic", N)[0], device)
    assert plan.kind == "ring"
    bank = AgentBank(N, P, device, ld=ring.x.stride(0))
    bank.adopt("x", ring.x, replaceable=True)
    bank.adopt("y", ring.y, replaceable=True)  # dead contents: the destination check may swap them
    # first uses: the destination check of each (source, destination) pair
    # (AgentBank.mix; a slow destination is replaced) and the eps
    # kernel's tuning for each buffer pair -- until a call adds no check
    for _ in range(8):
        probes = len(bank.pair_probes)
        bank.mix(plan, steps=eps)
        if len(bank.pair_probes) == probes:
            break
    bank.mix(plan, steps=eps)
    torch.cuda.synchronize(device)
    ms_pass = _events_ms(lambda: bank.mix(plan, steps=eps), reps)
    entry = ops.ring_steps_choice(bank.x, bank.buffer("y"), eps, P=P, n_rows=N)
    choice = entry["choice"] if entry else 0
    bufs = [bank.x, bank.buffer("y")]

    def alternating(variant):  # as bank.mix: each pass writes the other buffer
        def run():
            ops.mix_ring_steps(bufs[0], bufs[1], plan.w_prev, plan.w_next, eps, P=P, n_rows=N, variant=variant)
            bufs.reverse()
        return run
    # the untuned library default on the same buffers, alternating like the product call
    ms_default = _events_ms(alternating(0), reps)
    # the pass per direction (one destination matrix of a pair can be the slow one)
    a, b = bank.x, bank.buffer("y")
    direction_ms = {"x_to_y": _events_ms(lambda: ops.mix_ring_steps(a, b, plan.w_prev, plan.w_next, eps, P=P, n_rows=N,
                                                                    variant=choice), reps),
                    "y_to_x": _events_ms(lambda: ops.mix_ring_steps(b, a, plan.w_prev, plan.w_next, eps, P=P, n_rows=N,
                                                                    variant=choice), reps)}
    ring.x, ring.y = bank.x, bank.buffer("y")  # (the buffers swapped an even or odd number of times)
    return {"eps": eps, "rounds_per_s": eps * 1e3 / ms_pass, "ms_per_pass": ms_pass,
            "GBps_per_pass": 2 * N * P * 4 / (ms_pass / 1e3) / 1e9,
            "frac_per_pass": 2 * N * P * 4 / (ms_pass / 1e3) / 1e9 / HBM_PEAK_GBPS,
            "kernel": RING_STEPS_KERNELS.get(choice, "library default"),
            "variant_ms": {str(k): v for k, v in (entry["ms"] if entry else {}).items()},
            "default_ms_per_pass": ms_default, "direction_ms": direction_ms,
            "destination_checks": bank.pair_probes,
            "call": "AgentBank.mix(plan, steps=5) (FedLCon.run's call)",
            "what": "FedLCon eps=5 consensus rounds fused into one HBM pass, bit-identical; the kernel tuned by the "
                    "product path for the bank's buffers on first use"}


def random_regular_pm_round(device, X, Y, N: int, P: int, reps: int = 10):
    """Secondary (BASELINE config 3's random-regular mix at the headline size):
    X <- W X for a random 4-regular W on the parameter-major bank
    (dol_mix_csr_pm_f32), reusing the headline's buffers as XT [P, N] / YT.
    The call is the product one (ops.mix_csr_pm, nseg=None): its first use on
    these buffers tunes the stage order (the best order follows where the
    pages landed, profiles/r03_pm_stage_order.txt); the library default's
    time is reported beside it."""
    from dolhip import graph as G, ops
    c = G.random_regular_csr(N, 4, seed=2028)
    XT = X.view(-1)[: P * N].view(P, N)
    YT = Y.view(-1)[: P * N].view(P, N)
    rp = torch.as_tensor(c.rowptr, device=device)
    col = torch.as_tensor(c.col, device=device)
    val = torch.as_tensor(c.val, device=device)
    for _ in range(2):
        ops.mix_csr_pm(XT, YT, rp, col, val)
    torch.cuda.synchronize(device)
    ms = _events_ms(lambda: ops.mix_csr_pm(XT, YT, rp, col, val), reps)
    entry = ops.pm_stage_order_choice(XT, YT, N, P=P)
    ms_default = _events_ms(lambda: ops.mix_csr_pm(XT, YT, rp, col, val, nseg=0), reps)
    # the same call in the other direction (a parameter-major DGD alternates XT / YT; DESIGN §4.4:
    # some pairs of allocations are slower one way)
    ms_reverse = _events_ms(lambda: ops.mix_csr_pm(YT, XT, rp, col, val), reps)
    gbps = 2 * N * P * 4 / (ms / 1e3) / 1e9
    return {"agents": N, "params": P, "degree": 4, "ms_per_round": ms, "rounds_per_s": 1e3 / ms, "GBps": gbps,
            "frac": gbps / HBM_PEAK_GBPS, "kernel": "csr_pm_kernel (parameter-major bank)",
            "stage_order": entry["choice"] if entry else 0,
            "stage_order_ms": {str(k): v for k, v in (entry["ms"] if entry else {}).items()},
            "default_ms_per_round": ms_default, "reverse_direction_ms": ms_reverse,
            "what": "random 4-regular W mix on the parameter-major bank, bit-identical to the reference consensus"}


def dense_mix_round(device, N: int = 1024, P: int = 101770, reps: int = 10):
    """Secondary (BASELINE config 5's mixing, N = 1): X <- W X with an Erdos-Renyi
    p = 0.1 stochastic W (graph.erdos_renyi_stochastic, drawn on the device) on
    the split3 bf16-MFMA kernel (dense_split.hip), P = the 784-128-10 MLP's
    parameter count.  Includes the per-round operand split; flop = 2 N^2 P."""
    from dolhip import graph as G, ops
    from dolhip.bank import row_stride
    gen = torch.Generator(device=device).manual_seed(2028)
    W = G.erdos_renyi_stochastic(N, 0.1, gen)
    X = torch.empty(N, row_stride(P), device=device).normal_(generator=gen)
    Y = torch.empty_like(X)
    work = torch.empty(ops.dense_split3_workspace_bytes(N, N, P, 0), dtype=torch.uint8, device=device)
    ops.mix_dense_split3(W, X, Y, P=P, work=work)
    _warm(lambda: ops.mix_dense_split3(W, X, Y, P=P, work=work))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        ops.mix_dense_split3(W, X, Y, P=P, work=work)
    e.record()
    torch.cuda.synchronize(device)
    ms = s.elapsed_time(e) / reps
    tf = 2.0 * N * N * P / (ms / 1e3) / 1e12
    del W, X, Y, work
    torch.cuda.empty_cache()
    return {"agents": N, "params": P, "ms_per_round": ms, "rounds_per_s": 1e3 / ms, "TFLOPs_f32_equiv": tf,
            "vs_f32_matrix_peak_157TF": tf / 157.3, "bf16_mfma_util": 6 * tf / 2516.6,
            "what": "dense ER p=0.1 W mix on bf16 MFMA at fp32 accuracy (three-piece split, six products), "
                    "split pass included"}


def er_exact_mix_round(device, N: int = 1024, P: int = 101770, reps: int = 10):
    """Secondary (BASELINE config 5's mixing, N = 1), bit-exact: the same
    Erdos-Renyi p = 0.1 W drawn on the device each round (dol_er_stochastic_f32),
    its Neighbors selection on the device (dol_dense_to_csr_f32 + the
    chunk-major packing) and the LDS-gather CSR mix (dol_mix_csr_slab_f32) --
    the reference's consensus bit for bit; draw + CSR build included in the
    round time, the mix kernel timed separately."""
    from dolhip import graph as G
    from dolhip.bank import row_stride
    gen = torch.Generator(device=device).manual_seed(2028)
    X = torch.empty(N, row_stride(P), device=device).normal_(generator=gen)
    Y = torch.empty_like(X)
    Wbuf = torch.empty(N, N, device=device)
    st = {"plan": None, "r": 0}

    def draw():
        st["r"] += 1
        W = G.erdos_renyi_stochastic_hip(N, 0.1, 2028 * 1000003 + st["r"], device, out=Wbuf)
        st["plan"] = G.MixingPlan.from_dense(W, dense_kernel="csr", reuse=st["plan"],
                                           balance=True)  # the config-5 product path's pack
    draw()
    st["plan"].apply(X, Y, P=P)
    _warm(lambda: (draw(), st["plan"].apply(X, Y, P=P)))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    for _ in range(reps):
        draw()
        st["plan"].apply(X, Y, P=P)
    ev[1].record()
    ev[2].record()
    for _ in range(reps):
        st["plan"].apply(X, Y, P=P)
    ev[3].record()
    torch.cuda.synchronize(device)
    ms_round = ev[0].elapsed_time(ev[1]) / reps
    ms_mix = ev[2].elapsed_time(ev[3]) / reps
    nnz = int(st["plan"].rowptr[-1].item())
    del X, Y, Wbuf, st
    torch.cuda.empty_cache()
    return {"agents": N, "params": P, "nnz": nnz, "ms_per_round": ms_round, "rounds_per_s": 1e3 / ms_round,
            "mix_ms": ms_mix, "lds_GBps": nnz * P * 4 / (ms_mix / 1e3) / 1e9,
            "kernel": "csr_slab_kernel (LDS-gather CSR) + dense_to_csr + slab_pack",
            "what": "a time-varying ER p=0.1 W (drawn each round by the device hash kernel; dense_er_mix draws its W with the torch generator, same distribution), mixed bit-exactly (reference consensus order); "
                    "W draw + device Neighbors + packing included in ms_per_round"}


def config5_round_sharded(device, world: int, rank: int, N: int = 1024, reps: int = 10):
    """Config 5 over `world` ranks: dolhip.synthetic.TimeVaryingMLPGossip with
    torch.distributed up -- each rank's agent block takes the fused MLP step,
    one all_to_all moves the bank to parameter-column blocks, every rank mixes
    all N agents on its columns with the round's W (drawn from the shared seed
    on every rank, on a side stream during the local step), one all_to_all
    moves it back.  Bit-identical to one GPU
    (tests/test_parallel_gpu.py::test_config5_rounds_across_ranks_match_one_gpu).
    Timed like the headline: barrier, max over ranks."""
    from dolhip.synthetic import TimeVaryingMLPGossip
    d, h, c, B = 784, 128, 10, 32
    sim = TimeVaryingMLPGossip(N, d, h, c, p_edge=0.1, lr=0.05, momentum=0.5, seed=2028, device=device)
    gen = torch.Generator(device=device).manual_seed(2028 + rank)
    sim.batch(torch.empty(sim.n_local, B, d, device=device).normal_(generator=gen),
              torch.randint(0, c, (sim.n_local, B), device=device, generator=gen))
    for _ in range(2):
        sim.round()
    torch.cuda.synchronize(device)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        sim.round()
    torch.cuda.synchronize(device)
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item()) / reps
    out = {"agents": N, "params": sim.P, "batch": B, "mlp": f"{d}-{h}-{c}", "ms_per_round": el * 1e3,
           "rounds_per_s": 1.0 / el, "ranks": world, "agents_per_rank": sim.n_local, "columns_per_rank": sim.tr.Pc,
           "overlap_chunks": sim.overlap_chunks,
           "what": "config 5 over ranks (TimeVaryingMLPGossip): fused MLP step on each rank's agents in pieces, each "
                   "piece's all_to_all to parameter-column blocks posted while the next piece steps, bit-exact ER mix "
                   "per block (same W on every rank), all_to_all back"}
    del sim
    torch.cuda.empty_cache()
    return out


def config5_round(device, N: int = 1024, reps: int = 10):
    """Secondary (BASELINE config 5, N = 1): one whole round of the
    time-varying-graph MLP workload -- a new Erdos-Renyi p = 0.1 W drawn on the
    device, the device Neighbors selection + slab packing, one fused local step
    of every agent's 784-128-10 MLP (dol_mlp_step_f32: forward, CE, backward,
    momentum SGD; synthetic batch of 32 per agent) and the bit-exact mix of the
    parameter rows (dol_mix_csr_slab_f32).  Phases timed with events on the
    launch stream; ms_per_round by the host clock over `reps` rounds."""
    from dolhip import graph as G
    from dolhip.bank import AgentBank
    from dolhip.mlp import BatchedMLP, mlp_layout
    d, h, c, B = 784, 128, 10, 32
    bank = AgentBank(N, mlp_layout(d, h, c), device)
    mlp = BatchedMLP(bank, d, h, c)
    gen = torch.Generator(device=device).manual_seed(2028)
    bank.buffer("x").normal_(0, 0.05, generator=gen)
    bank.buffer("y").zero_()
    bank.buffer("mom", zero=True)
    X = torch.empty(N, B, d, device=device).normal_(generator=gen)
    y = torch.randint(0, c, (N, B), device=device, generator=gen)
    Wbuf = torch.empty(N, N, device=device)
    st = {"plan": None, "r": 0}
    ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
          for k in ("graph", "local", "mix")}

    def one(k=None):
        rec = (lambda nm, i: ev[nm][k][i].record()) if k is not None else (lambda nm, i: None)
        st["r"] += 1
        rec("graph", 0)
        W = G.erdos_renyi_stochastic_hip(N, 0.1, 2028 * 1000003 + st["r"], device, out=Wbuf)
        st["plan"] = G.MixingPlan.from_dense(W, dense_kernel="csr", reuse=st["plan"], balance=True)  # as the product path packs
        rec("graph", 1)
        rec("local", 0)
        mlp.step(X, y, lr=0.05, momentum=0.5, first_step=False)
        rec("local", 1)
        rec("mix", 0)
        bank.mix(st["plan"])
        rec("mix", 1)
    for _ in range(2):
        one()
    _warm(one)
    t0 = time.perf_counter()
    for k in range(reps):
        one(k)
    torch.cuda.synchronize(device)
    el_seq = (time.perf_counter() - t0) / reps
    ms = {k: sum(a.elapsed_time(b) for a, b in v) / reps for k, v in ev.items()}
    P = bank.P
    del bank, mlp, Wbuf, st
    torch.cuda.empty_cache()
    # the product path: dolhip.synthetic.TimeVaryingMLPGossip, the W draw + CSR
    # build on a side stream during the local step
    from dolhip.synthetic import TimeVaryingMLPGossip
    sim = TimeVaryingMLPGossip(N, d, h, c, p_edge=0.1, lr=0.05, momentum=0.5, seed=2028, device=device)
    sim.batch(X, y)
    for _ in range(2):
        sim.round()
    _warm(sim.round)
    t0 = time.perf_counter()
    for _ in range(reps):
        sim.round()
    torch.cuda.synchronize(device)
    el = (time.perf_counter() - t0) / reps
    del sim
    out = {"agents": N, "params": P, "batch": B, "mlp": f"{d}-{h}-{c}", "ms_per_round": el * 1e3,
           "rounds_per_s": 1.0 / el, "ms_per_round_sequential": el_seq * 1e3, "phase_ms": ms,
           "local_GBps": N * (4 * P + B * d) * 4 / (ms["local"] / 1e3) / 1e9,
           "what": "config 5 round (dolhip.synthetic.TimeVaryingMLPGossip): ER p=0.1 W drawn on device + device "
                   "Neighbors/packing on a side stream, fused MLP local step (momentum SGD) on fp32 MFMA, bit-exact "
                   "LDS-gather CSR mix of the parameter rows; phase_ms from the same round run sequentially"}
    del X, y
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start the N ranks ourselves (before any GPU call)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a line timed on fewer (or more) ranks than asked would pass for the wrong N
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world} ranks joined", file=sys.stderr, flush=True)
        sys.exit(2)
    # DOL_DEVICE_MAP=0 puts every rank on cuda:0 and DOL_DIST_BACKEND=gloo stages
    # halos through host memory: a rehearsal of the N>1 path on a 1-GPU box
    backend = os.environ.get("DOL_DIST_BACKEND", "nccl")
    if args.launch_check:
        sys.exit(launch_check(args, world, rank, local, backend))
    device = torch.device("cuda", int(os.environ.get("DOL_DEVICE_MAP", local)))
    torch.cuda.set_device(device)
    import dolhip
    from dolhip import parallel
    from dolhip.parallel import ShardedRing
    if world > 1:
        # bounded timeout on every collective + RCCL async error handling: a
        # stuck rank fails the run instead of hanging it
        parallel.init_process_group(backend, device=device if backend == "nccl" else None)
    infos = rank_infos(world, rank, local, backend, device)

    dolhip.lib()
    N, P = args.agents, args.params
    wp, wn = ring_weights(N)
    # --map-ring 1 (default): the headline's two buffers are mapped physical
    # blocks, like every bank matrix of >= 1 GiB (bank.device_matrix; in one
    # process 10.69 vs 10.90 ms for torch-allocated ones,
    # profiles/r05d_alloc_ab.jsonl), at every world size (r06): across ranks the
    # two boundary rows are copied into torch-allocated send buffers before the
    # RCCL send (ShardedRing.stage_sends), so every N runs on the same memory
    ring = ShardedRing(N, P, wp, wn, device, mapped=bool(args.map_ring))
    g = torch.Generator(device=device).manual_seed(2028 + rank)
    ring.x.normal_(generator=g)
    ring.y.zero_()

    # device warm-up (not a step): ~0.3 s of the ring-pattern copy kernel over the
    # same rows lifts the clocks out of their idle ramp before the W warm-up steps
    # (a short timed region that starts cold runs slow: profiles/r04p_dense_clock_ramp.jsonl)
    from dolhip import ops as _ops
    _warm(lambda: _ops.stream_copy_rows(ring.x, ring.y, P=P), seconds=0.3)
    ring.y.zero_()
    _log(f"ring {N} x {P}: warm-up")
    for _ in range(args.warmup):
        ring.step()
    torch.cuda.synchronize(device)

    # kernel events: around every launch of the dominant kernel
    K = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    ring.kernel_events = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for k in range(K):
        if world == 1:
            ev[k][0].record()
            ring.step()
            ev[k][1].record()
        else:
            ring.kernel_events = ev[k]
            ring.step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    kern_rows = ring.n_local if world == 1 else ring.n_local - 2
    alg_bytes = 2 * kern_rows * P * 4  # each row read once + written once
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9

    # secondary (N = 1): FedLCon's eps = 5 consensus rounds per local update
    # (DIST/simulators.py:190-196) as ONE temporally blocked pass over the same
    # X, through the call FedLCon.run makes (weighted_average/simulators.py:233
    # -> AgentBank.mix(plan, steps=eps) -> MixingPlan.apply_steps ->
    # ops.mix_ring_steps, whose kernel the product path tunes on first use for
    # the bank's buffers); the headline above stays one round per step
    fedlcon = None
    if world == 1 and not args.no_primal_dual:
        fedlcon = fedlcon_eps_round(device, ring, N, P)

    # secondary (N = 1): config 3's random 4-regular mix at the headline size on
    # the parameter-major bank, in the headline's buffers
    _log("headline done")
    rr_pm = None
    if world == 1 and not args.no_primal_dual and N <= 8192:
        rr_pm = random_regular_pm_round(device, ring.x, ring.y, N, P)
        # the same-box yardstick: the headline ring kernel moves the same bytes
        rr_pm["ring_kernel_ms_same_box"] = kern_ms
        rr_pm["ring_over_pm"] = kern_ms / rr_pm["ms_per_round"]
    _log("random-regular pm done")
    calib = None
    if not args.no_copy:
        calib = copy_peak(device, ring.x, ring.y, P)
    del ring.x, ring.y
    gc.collect()  # the legs' banks may sit in reference cycles: release their mapped blocks now
    torch.cuda.empty_cache()
    _log("calibration done")
    pd_round = None
    if not args.no_primal_dual:
        pd_round = primal_dual_round(N, P, world, rank, device, args.pd_steps)
    _log("primal/dual round done")
    dense = exact = None
    if world == 1 and not args.no_primal_dual:
        dense = dense_mix_round(device)
        exact = er_exact_mix_round(device)
    _log("dense ER done")
    cfg5 = None
    secondary_errors = []
    if not args.no_primal_dual:
        if world == 1:
            cfg5 = config5_round(device)
        else:  # a secondary: an error here must not cost the headline line
            try:
                cfg5 = config5_round_sharded(device, world, rank)
            except (RuntimeError, ValueError) as e:  # recorded at the line's top level, not hidden
                cfg5 = {"error": f"{type(e).__name__}: {e}"[:300]}
                secondary_errors.append({"leg": "config5_round", "error": cfg5["error"]})
                _log(f"ERROR: config-5 round over ranks failed: {cfg5['error']}")
    _log("config 5 round done")
    dgd = None
    if world == 1 and not args.no_primal_dual:
        dgd = dgd_rounds(device)
    _log("config 3 rounds done")

    traffic = None
    traffic_src = None
    if os.path.exists(args.traffic_file):
        try:
            tr = json.load(open(args.traffic_file))
            if tr.get("agents") == N and tr.get("params") == P and tr.get("n_gpus", 1) == world:
                traffic = tr.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(args.traffic_file, ROOT)
        except (OSError, ValueError):
            traffic = None

    from dolhip import ops
    from dolhip.bank import retired_va
    bank_va = retired_va()
    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(args.cpu_agents, P, args.cpu_seconds, N)
            if not args.no_primal_dual:
                sec = cpu_secondaries(P, N)
                if pd_round is not None:
                    pd_round["cpu_baseline"] = sec["fedadmm"]
                    pd_round["vs_cpu"] = pd_round["rounds_per_s"] / sec["fedadmm"]["value"]
                if cfg5 is not None:
                    cfg5["cpu_baseline"] = sec["config5"]
                    cfg5["vs_cpu"] = cfg5["rounds_per_s"] / sec["config5"]["value"]
        value = K / elapsed
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rounds/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (randn agent parameters, seed 2028)",
            "config": {
                "workload": f"ring gossip mix X <- W X, {N} agents x {P} params, W = "
                            f"communication_graph('circle','stochastic',{N}) seed 2028",
                "agents": N,
                "params": P,
                "topology": "circle",
                "mode": "stochastic",
                "parallelism": f"agent-shard x{world}" + ((" + RCCL halo send/recv" if backend == "nccl" else
                                                           f" + {backend} halo send/recv (rehearsal)") if world > 1 else ""),
            },
            "parallel": {"world_size": world, "backend": infos[0]["backend"],
                         "distinct_devices": len({(i["device"]) for i in infos}),
                         "launcher": infos[0]["launcher"], "ranks": infos},
            "roofline": {
                "bound": "hbm",
                "kernel": ("ring_mix_kernel" if os.environ.get("DOL_RING_DMA", "1") == "0" else
                           "ring_mix_dma_kernel<4, NoEpi, true, false>" if os.environ.get("DOL_RING_NTI", "1") != "0" else
                           "ring_mix_dma_kernel<4, NoEpi>"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": alg_bytes,
                "kernel_ms": kern_ms,
                "copy_kernel_GBps": calib["GBps"] if calib else None,
                "copy_calibration": calib,
                "frac_of_measured_copy": (achieved / calib["GBps"]) if calib else None,
            },
            "cpu_baseline": cpu,
            "primal_dual_round": pd_round,
            "fedlcon_eps5": fedlcon,
            "random_regular_pm": rr_pm,
            "dense_er_mix": dense,
            "er_exact_mix": exact,
            "config5_round": cfg5,
            "config3_dgd": dgd,
            "secondary_errors": secondary_errors,
            "tuned_launches": ops.tuned_choices(),
            "bank_retired_va": bank_va,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
