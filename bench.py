#!/usr/bin/env python3
"""Headline benchmark: Leduc NFSP self-play hands/s (BASELINE.json `metric`).

One step = one pass of the hot path over one batch: every lane of the engine plays one
hand (fused rollout kernel: deal, eta draws, D/L/D scheduler, AR / eps-greedy BR forwards,
env transitions, RL/SL records), the records are inserted into the agents' memories,
and the learner runs update_strategy at the REFERENCE cadence (one per 128 RL inserts
of an agent: AR fit + BR targets/fit/schedules/target sync).  Nothing is skipped inside
the timed region.

Workload (config.workload): C3 = 1,048,576 lanes per GPU, M_RL 200k, M_SL 2M, target
sync every 150 BR updates (BASELINE.json configs[2]; configs[3] is the same per GPU at
N = 8).  `--config c2` selects configs[1] (65,536 lanes).

Multi-GPU (`torch.distributed.run --nproc-per-node N bench.py --gpus N`, configs[3] = C4):
one self-play shard per GPU (its own hands, memories and learner; seeds 1234 + rank; weak
scaling), and after every lane slice's learner an all-reduce of the average-policy (AR)
gradient steps of both agents (17.4 KB), enqueued by libnfsp on the AR chain stream over its
own RCCL communicator (shards.AvgPolicyExchange; `--xchg-every k` = every k slices,
`--ar-allreduce off` = independent replicas).  A barrier and a max-over-ranks of the elapsed
time bracket the timed region; at N > 1 the line also carries every rank's own step time,
device / PCI bus id and the exchange's cost (`ranks`).

Timing: W warmup steps, then K steps with no instrumentation -> `value` / `ms_per_step`;
then K more steps with HIP events recorded on each kernel's stream around every launch ->
each kernel's average duration (`kernel_ms`, `ms_per_step_event_timed`).

Roofline (`rooflines()`): SURVEY 8(d)'s HBM framing of the kernel on the learner's critical
path -- the chain on the stream with the longest busy span per step (`critical_stream`):
algorithmic bytes per launch (the 128 sampled tuples of each update in the reference's fp32
layout, 257 B M_RL / 132 B M_SL) / its average duration.  `roofline_other` holds the other
chain, the rollout (its inserted tuples per launch of one slice), the chains' MFMA framing
(the matrix-core FLOPs they execute, priced against the bf16 dense peak they run at) and
their issue framing (static issue cycles per step / measured); `whole_step_hbm_per_gpu` is
SURVEY 8(d)'s whole-path bytes per hand x hands / step time.

`bench.py --gpus N` without a torch.distributed environment starts the N rank processes
itself (launch_ranks; the parent never touches a GPU); every rank checks WORLD_SIZE == N.

`cpu_baseline` (rank 0, N = 1 only) comes from the C++ restatement of the reference's
main.train (oracle/nfsp_cpu.cpp).  It uses the reference cadence and this config's memory
capacities, and is parity-checked hand for hand against oracle/nfsp_oracle.py.  As BASELINE.md
plans it, it runs as one process per host core -- the cores this job may use: the cgroup CPU
quota (16 on the 1-GPU box, whose os.cpu_count() reports the whole machine's 256), else
os.cpu_count() -- each an independent replica, for `--cpu-seconds`; `cpu_baseline_numpy`,
the numpy restatement, the same way.  Both print the core count and os.cpu_count().
"""
from __future__ import annotations

import argparse
import json
import subprocess
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Hardware queues per process (read when HIP initialises, so before torch is imported).  An
# engine runs 4 streams that must not share a queue: a rollout queued behind a 1 ms SGD chain
# kernel breaks the slices' pipelining.  HIP's default of 4 queues is enough while the engine's
# streams are the process's only busy ones, but a process group (torch's NCCL streams, the
# exchange's RCCL communicator) adds streams, and with 4 queues the ctx stream landed on agent 0's
# BR queue: C4's per-rank line with the exchange ran 179.0 ms per step, 168.9 with 8 queues and
# 168.7 with 16; C3 alone 166.9 / 166.7 / 167.3 (`tools/hwq_probe.sh`).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

CONFIGS = {
    # C3 advances its 1M lanes in 16 slices of 65,536 (include/nfsp.h cfg.slices), pipelined
    # (cfg.slice_lag 2: a slice acts with the nets its predecessor's predecessor's learner left,
    # while its predecessor's chains run): the policy lag is 2 slices, not 1M hands, and C3
    # learns inside the CPU reference's seed band (tests/test_gpu_slices.py)
    "c3": dict(n_lanes=1_048_576, slices=16, slice_lag=2, rl_capacity=200_000, sl_capacity=2_000_000,
               label="C3: 1,048,576 Leduc lanes/GPU (advanced in 16 pipelined slices of 65,536), device "
                     "M_RL 200k + M_SL 2M, target sync 150, reference update cadence (1 update_strategy "
                     "/ 128 RL inserts / agent)"),
    # C4 (BASELINE configs[3]): per GPU C3's 1M lanes and memories, as 128 pipelined slices of
    # 8,192, and the ranks' AR nets exchanged after every slice (W0 + 2 x the mean of the
    # deltas, shards.AvgPolicyExchange, RCCL on the AR chain stream): the 8-GPU job then learns
    # inside the CPU reference's band per total hand from its first 8.4M hands, >= 0.1 chips
    # inside the bar at every checkpoint (tests/test_gpu_slices.py; 64 slices
    # passed the first checkpoint by 0.012).  bench.py --gpus N > 1 runs it by default.
    "c4": dict(n_lanes=1_048_576, slices=128, slice_lag=2, rl_capacity=200_000, sl_capacity=2_000_000,
               xchg_every=1, xchg_gain=2.0,
               label="C4: 1,048,576 Leduc lanes/GPU (128 pipelined slices of 8,192), device M_RL 200k + M_SL "
                     "2M, target sync 150, reference cadence; the AR nets of all GPUs exchanged after every "
                     "slice (W0 + 2 x mean of the ranks' deltas, RCCL on the AR chain stream)"),
    "c3_1slice": dict(n_lanes=1_048_576, rl_capacity=200_000, sl_capacity=2_000_000,
                      label="C3 with all 1,048,576 lanes in one rollout per step (round 2's form: policy "
                            "lag of 1M hands), M_RL 200k + M_SL 2M, reference cadence"),
    "c2": dict(n_lanes=65_536, slices=16, slice_lag=2, rl_capacity=40_000, sl_capacity=40_000,
               label="C2: 65,536 Leduc lanes/GPU (16 pipelined slices of 4,096), M_RL/M_SL 40k, "
                     "eta 0.1, 2x64 MLP heads, reference update cadence"),
    "c3_4k": dict(n_lanes=4_096, rl_capacity=200_000, sl_capacity=2_000_000,
                  label="C3's memories and cadence at 4,096 lanes (policy lag 4k hands; DESIGN §9)"),
    "c3_64k": dict(n_lanes=65_536, rl_capacity=200_000, sl_capacity=2_000_000,
                   label="C3's memories and cadence at 65,536 lanes (policy lag 64k hands; DESIGN §9)"),
    # engine groups (nfsp_group_*): C3's 1,048,576 lanes per GPU as R learner replicas of
    # 1M / R lanes, each with C3's own memories (M_RL 200k, M_SL 2M) and cadence, their SGD
    # chains in shared launches, and the AR nets averaged over the replicas after every step
    # (C4's exchange, on device).  A new measured configuration beside C3, not C3 itself.
    **{f"c3_r{R}": dict(n_lanes=1_048_576, replicas=R, rl_capacity=200_000, sl_capacity=2_000_000,
                        label=f"C3 as {R} learner replicas x {1_048_576 // R:,} Leduc lanes on one GPU, "
                              f"each with device M_RL 200k + M_SL 2M, target sync 150, reference cadence; "
                              f"AR nets averaged over the replicas every step")
       for R in (2, 4, 8, 16, 32, 64, 128, 256)},
    # C4's arithmetic on ONE GPU (bench groups): R replicas of C4's per-GPU shard, the AR nets
    # exchanged after every slice on device -- what --gpus R runs, in one process; trained from
    # scratch over learn_steps steps (R x 1M hands each) beside the CPU band
    **{f"c4_emul_r{R}": dict(n_lanes=R * 1_048_576, replicas=R, slices=128, slice_lag=2, rl_capacity=200_000,
                             sl_capacity=2_000_000, xchg_every=1, xchg_gain=2.0, learn_steps=32 // R,
                             label=f"C4 emulated on one GPU: {R} replicas x 1,048,576 Leduc lanes (128 pipelined "
                                   f"slices each), M_RL 200k + M_SL 2M each, reference cadence; the replicas' AR "
                                   f"nets exchanged after every slice (W0 + 2 x mean delta), from scratch")
       for R in (4, 8)},
    # the same with the group's BR learner call as one persistent launch (nfsp_group_sched
    # br_persist, k_br_persist: DESIGN.md Appendix A.1b) -- the same SGD steps bit for bit
    "c4_emul_r8_persist": dict(n_lanes=8 * 1_048_576, replicas=8, slices=128, slice_lag=2, rl_capacity=200_000,
                               sl_capacity=2_000_000, xchg_every=1, xchg_gain=2.0, learn_steps=4,
                               sched=dict(br_persist=1),
                               label="C4 emulated on one GPU as c4_emul_r8, the BR learner calls as one persistent "
                                     "launch each (k_br_persist)"),
    "c5": dict(n_lanes=1_048_576, slices=16, slice_lag=2, rl_capacity=200_000, sl_capacity=2_000_000,
               game="kuhn", label="C5: Kuhn swap-in, 1,048,576 lanes/GPU (16 pipelined slices), C3's "
                                  "memories and cadence"),
    # C5's exploitability -> 0 check runs textbook NFSP with the MSE Q loss
    "c5_tb": dict(n_lanes=1_048_576, slices=16, slice_lag=2, rl_capacity=200_000, sl_capacity=2_000_000,
                  game="kuhn", quirks=504,
                  label="C5: Kuhn swap-in, 1,048,576 lanes/GPU (16 pipelined slices), C3's memories and cadence, "
                        "textbook NFSP with the MSE Q loss (quirks NFSP_TEXTBOOK_MSE)"),
}

PEAK_BF16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: BF16 MFMA, ~2.5 PF dense (the chains' MFMAs)
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
# the chains' matrix-core work per SGD step: 18 v_mfma_f32_16x16x32_bf16 per wave x 4 waves
# (SQ_INSTS_MFMA, profiles/r06/chain_pmc.json), 2 x 16 x 16 x 32 FLOP each: the exact 3-term
# bf16 split executes ~2.9x the dense-equivalent f32 FLOPs of the step (32 x F_TRAIN)
MFMA_PER_SGD_STEP = 18 * 4
FLOP_PER_MFMA = 2 * 16 * 16 * 32
CHAIN_CLOCK_HZ = 2.40e9       # the chains' effective shader clock (tools/chain_clock.py)
# algorithmic work per unit (DESIGN.md "Measurement")
F_FWD = 2 * (30 * 64 + 64 * 3)          # 4,224 FLOP per row forward (dense-equivalent)
F_TRAIN = 3 * F_FWD                      # forward + backward (dX, dW) per row
BYTES_RL, BYTES_SL = 257, 132            # reference tuple layout in fp32


def learner_flops(br_updates, ar_updates, batch=128, epochs=2):
    br = br_updates * (2 * batch * F_FWD + epochs * batch * F_TRAIN)   # targets + fit
    ar = ar_updates * (epochs * batch * F_TRAIN)
    return br + ar


def load_pmc(config, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this config
    (FETCH_SIZE x 2 + WRITE_SIZE, KB -> bytes; MI355X_MICROARCH.md §HBM), or None."""
    path = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    k = d.get("kernels", {}).get(kernel)
    return None if k is None else k.get("hbm_bytes_per_launch")


def cpu_share() -> int:
    """Host cores this job may use: os.cpu_count(), capped by the cgroup CPU quota
    (/sys/fs/cgroup/cpu.max; the 1-GPU box: 16 of the machine's 256) and the affinity mask."""
    import math
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_worker(kind: str, seconds: float, config: str, seed: int, workload: str = "c") -> dict:
    """One CPU-baseline process (bench.py --cpu-worker): one replica of main.train restated
    in C++ (kind "port") or numpy ("numpy") for `seconds`; never touches a GPU.  workload
    (BASELINE.md): "c" end to end with updates, "a" env + scheduler with random action vectors,
    "b" the agents' play (forwards, memory inserts) without updates."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    cfg = CONFIGS[config]
    game = cfg.get("game", "leduc")
    if kind == "port":
        import cpu_port
        c = cpu_port.make_cfg(None, seed, True, game, rl_capacity=cfg["rl_capacity"],
                              sl_capacity=cfg["sl_capacity"], workload=workload)
        c.seed = c.seed + seed
        hands, el = cpu_port.bench(c, 1, seconds)
        return {"hands": int(hands), "seconds": el}
    import random
    import nfsp_oracle as orc
    random.seed(seed)
    env, p1, p2 = orc.make_main(init_seed=seed)
    env.kuhn = game == "kuhn"
    players = [p1, p2]
    if workload == "a":
        players = [orc.RandomPlayer(env), orc.RandomPlayer(env)]
    elif workload == "b":
        for p in players:
            p.update_strategy = lambda: None
    dealer = random.randint(0, 1)
    hands = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(50):
            dealer = 1 - dealer
            orc.play_hand(env, players, dealer, 0.1)
            hands += 1
    return {"hands": hands, "seconds": time.perf_counter() - t0}


def cpu_processes(kind: str, procs: int, seconds: float, config: str, workload: str = "c") -> dict:
    """`procs` concurrent worker processes (one per core), each an independent replica; the
    aggregate hands/s = sum of each one's hands / its own time.  Child processes, started
    fresh (no fork of a process that holds the GPU)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", kind, "--cpu-seconds", str(seconds),
           "--config", config, "--cpu-workload", workload]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="")
    ps = [subprocess.Popen(cmd + ["--cpu-seed", str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, env=env) for r in range(procs)]
    res = []
    for p in ps:
        out, err = p.communicate(timeout=seconds + 300)
        if p.returncode != 0:
            raise RuntimeError(f"cpu worker failed ({p.returncode}): {err[-2000:]}")
        res.append(json.loads(out.strip().splitlines()[-1]))
    return {"value": sum(r["hands"] / r["seconds"] for r in res), "hands": sum(r["hands"] for r in res),
            "per_process": [r["hands"] / r["seconds"] for r in res]}


def cpu_baseline(seconds: float, cfg_name: str, cores: int | None = None):
    """BASELINE.md's CPU plan: main.train restated in C++ (oracle/nfsp_cpu.cpp, parity-checked
    hand for hand against oracle/nfsp_oracle.py by tests/test_cpu_port.py) as one process per
    host core, each an independent replica at this config's memory capacities.  Beside it:
    the same C++ as threads of one process (round 3's form)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cpu_port
    if not os.path.exists(cpu_port.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    cfg = CONFIGS[cfg_name]
    cores = cores or cpu_share()
    r = cpu_processes("port", cores, seconds, cfg_name)
    c = cpu_port.make_cfg(None, 0, True, cfg.get("game", "leduc"), rl_capacity=cfg["rl_capacity"],
                          sl_capacity=cfg["sl_capacity"])
    th_hands, th_el = cpu_port.bench(c, cores, min(seconds, 5.0))
    return {"value": r["value"], "unit": "hands/s", "cores": cores, "os_cpu_count": os.cpu_count(),
            "kind": "port", "processes": cores, "per_core": sum(r["per_process"]) / cores,
            "threads_one_process": {"value": th_hands / th_el, "threads": cores},
            "sample": f"{r['hands']} hands of main.train restated in C++ (oracle/nfsp_cpu.cpp: the "
                      f"reference's {cfg.get('game', 'leduc').capitalize()} Env, scheduler, memories M_RL "
                      f"{cfg['rl_capacity']:,} / M_SL {cfg['sl_capacity']:,}, updates at the reference cadence, "
                      f"fp32 MLPs) by {cores} processes (one per core of this job's CPU share: cgroup quota / "
                      f"affinity; os.cpu_count() = {os.cpu_count()}), one independent replica (one learner) "
                      f"each, {seconds:.0f} s"}


def cpu_baseline_numpy(seconds: float, cfg_name: str, cores: int | None = None):
    """The reference-structured CPU path in numpy (oracle Env/Agent + main.train's loop), one
    process per host core as cpu_baseline."""
    cores = cores or cpu_share()
    r = cpu_processes("numpy", cores, seconds, cfg_name)
    return {"value": r["value"], "unit": "hands/s", "cores": cores, "os_cpu_count": os.cpu_count(),
            "kind": "port", "processes": cores, "per_core": sum(r["per_process"]) / cores,
            "sample": f"{r['hands']} hands of main.train restated in numpy (oracle/nfsp_oracle.py: Env, "
                      f"Agent play/updates at the reference cadence, numpy fp32 MLPs) by {cores} processes "
                      f"(one per core; os.cpu_count() = {os.cpu_count()}), {seconds:.0f} s each"}


def cpu_baseline_rollout(seconds: float, cfg_name: str, cores: int | None = None) -> dict:
    """BASELINE.md's CPU workloads (a) and (b) -- the CPU counterparts of the line's
    rollout_only_hands_per_s (the fused rollout + inserts, no learner): (a) main.train's env and
    D/L/D scheduler with uniform-random action vectors; (b) the agents' play with the MLP forwards
    (eta 0.1, eps 0.06) and the memory inserts, no updates.  Both restatements (C++ port and
    numpy), one process per core of the job's CPU share, `seconds` each."""
    cores = cores or cpu_share()
    out = {"cores": cores, "os_cpu_count": os.cpu_count(), "unit": "hands/s",
           "gpu_counterpart": "rollout_only_hands_per_s (k_rollout + k_scan + k_commit per hand)"}
    for wl, what in (("a", "env + scheduler, uniform-random action vectors"),
                     ("b", "Agent.play: MLP forwards + memory inserts, no updates")):
        row = {"what": what}
        for kind in ("port", "numpy"):
            r = cpu_processes(kind, cores, seconds, cfg_name, wl)
            row[kind] = {"value": r["value"], "hands": r["hands"], "per_core": sum(r["per_process"]) / cores}
        out[wl] = row
    out["sample"] = (f"{cores} processes x {seconds:.0f} s per workload and restatement "
                     f"(oracle/nfsp_cpu.cpp workload 1 / 2, oracle/nfsp_oracle.py RandomPlayer / play "
                     f"without update_strategy), config {cfg_name}")
    return out


def init_dist(backend=None, force: bool = False):
    """One process per GPU (torch.distributed.run env); returns (world, rank, local, dist or None).
    The default backend is RCCL ("nccl") on a GPU box; tests pass "gloo".  force: a process
    group even at world size 1 (bench.py --ar-allreduce on: the exchange path measured on one
    GPU, its collectives local)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and not force:
        return world, rank, local, None
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    import datetime
    import torch.distributed as dist
    backend = backend or "nccl"
    # bounded: a rank whose peer never arrives fails in 2 minutes, not the default 10-30
    timeout = datetime.timedelta(seconds=float(os.environ.get("NFSP_PG_TIMEOUT_S", "120")))
    if backend == "nccl":
        dist.init_process_group(backend, timeout=timeout,
                                device_id=torch.device("cuda", local % torch.cuda.device_count()))
    else:
        dist.init_process_group(backend, timeout=timeout)
    return world, rank, local, dist


class StepWatchdog:
    """N > 1: a rank whose step makes no progress for `limit_s` (env NFSP_STEP_WATCHDOG_S,
    default 600) exits with 124 after saying where it is.  The per-slice AR exchange is an RCCL
    all-reduce that libnfsp enqueues on its own stream, outside torch's process-group timeout: a
    rank whose peer died or never joined would otherwise wait on the device forever, and with it
    the job.  Exiting lets the launcher (torch.distributed.run, or launch_ranks) stop the others.
    `beat(what)` marks progress; a daemon thread checks every second."""

    def __init__(self, rank: int, limit_s: float | None = None):
        import threading
        self.rank = rank
        self.limit_s = float(os.environ.get("NFSP_STEP_WATCHDOG_S", "600")) if limit_s is None else limit_s
        self.what, self.t = "start", time.monotonic()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True)
        self._th.start()

    def beat(self, what: str):
        self.what, self.t = what, time.monotonic()

    def _run(self):
        while not self._stop.wait(1.0):
            idle = time.monotonic() - self.t
            if idle > self.limit_s:
                sys.stderr.write(f"bench.py: rank {self.rank} made no progress for {idle:.0f} s (last: "
                                 f"{self.what}); exiting so the launcher stops the job\n")
                sys.stderr.flush()
                os._exit(124)

    def stop(self):
        self._stop.set()


def timed_steps(step, steps, warmup, dist=None, sync=lambda: None, device="cuda", out=None):
    """W untimed warmup steps, then exactly K timed steps bracketed by a barrier + device
    sync on both sides; returns the MAX elapsed seconds over ranks (every rank gets it).
    out (dict): also gets this rank's own time ("local_s": its K steps, from the barrier to its
    own final sync, before it waits for the others)."""
    import torch
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if out is not None:
        out["local_s"] = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def job_value(units_per_rank, world, elapsed):
    """Whole-job throughput: the units all ranks processed / the max-over-ranks time."""
    return units_per_rank * world / elapsed


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str], poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` started without a torch.distributed environment: start N rank
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1 /
    MASTER_PORT set, one rank per GPU) and wait for them.  Fail fast: the first rank to exit
    non-zero (OOM, RCCL init, a HIP error) ends the job -- its siblings, which would otherwise
    block in a barrier or all-reduce until the process-group timeout, are terminated (then
    killed after 10 s) and its exit code is returned.  The parent never touches the GPU (no
    torch.cuda call: it only forks children), so the children own the devices; rank 0 prints
    the JSON line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            rc = p.poll()
            if rc is not None and rc != 0:
                failed = (r, rc)
                break
        else:
            time.sleep(poll_s)
    if failed is None:
        bad = [p.returncode for p in procs if p.returncode != 0]
        return bad[0] if bad else 0
    r, rc = failed
    sys.stderr.write(f"bench.py: rank {r} exited with {rc}; stopping the other ranks\n")
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.time() + 10.0
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


def check_world(args, world: int):
    """Every rank: the job must be the one asked for (`--gpus N` = N ranks), and with RCCL
    every rank needs its own GPU.  A mismatch exits non-zero instead of timing the wrong job."""
    if world != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE {world} != --gpus {args.gpus}\n")
        sys.exit(2)
    if args.dist_backend == "nccl" and args.stub_step_ms is None:
        import torch
        if torch.cuda.device_count() < world:
            sys.stderr.write(f"bench.py: {world} ranks need {world} GPUs, "
                             f"{torch.cuda.device_count()} visible\n")
            sys.exit(2)


_RESULT_OUT = None


def claim_stdout():
    """In a rank process: keep the real stdout for the one JSON result line and send
    everything else written to fd 1 -- Python prints and native libraries' chatter (gloo's
    peer-connection lines, RCCL / HIP banners) -- to stderr."""
    global _RESULT_OUT
    if _RESULT_OUT is None:
        sys.stdout.flush()
        _RESULT_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def emit_result(obj: dict):
    out = _RESULT_OUT if _RESULT_OUT is not None else sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def device_identity() -> dict:
    """This rank's device: torch's index and the PCI bus id (None without a GPU)."""
    try:
        import torch
        if not torch.cuda.is_available():
            return {"device": None, "pci_bus_id": None}
        i = torch.cuda.current_device()
        p = torch.cuda.get_device_properties(i)
        bus = ":".join(f"{v:02x}" for v in (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                             getattr(p, "pci_device_id", 0)))
        return {"device": i, "pci_bus_id": bus, "name": p.name}
    except Exception as e:          # never fail the job over the report
        return {"device": None, "pci_bus_id": None, "error": str(e)}


def rank_report(dist, backend: str, mine: dict) -> dict:
    """N > 1: every rank's own figures (all_gather_object): its un-instrumented ms per step,
    the exchange's ms per call, its device and PCI bus id.  Under RCCL each rank must hold its
    own GPU: duplicate bus ids end the job (exit 2) instead of timing co-resident ranks."""
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, dict(mine, rank=dist.get_rank()))
    if backend == "nccl":
        ids = [(r.get("host"), r.get("pci_bus_id")) for r in ranks]
        if any(i[1] is None for i in ids) or len(set(ids)) != len(ids):
            sys.stderr.write(f"bench.py: ranks do not hold distinct GPUs: {ids}\n")
            sys.exit(2)
    ms = [r["ms_per_step"] for r in ranks]
    return {"world_size": dist.get_world_size(), "ranks": ranks,
            "ms_per_step_min": min(ms), "ms_per_step_max": max(ms),
            "distinct_devices": len({(r.get("host"), r.get("pci_bus_id")) for r in ranks}) == len(ranks)}


def refuse_host_fallback(args, world: int, fallback):
    """Under RCCL at N > 1 the exchange must run on RCCL: a host-transport fallback (some rank
    could not build the communicator) would time a different, slower job.  Every rank sees the
    same fallback (AvgPolicyExchange agrees on it), so every rank exits 2 together, unless
    --allow-host-fallback says the fallback is wanted."""
    if fallback and args.dist_backend == "nccl" and world > 1 and not args.allow_host_fallback:
        sys.stderr.write(f"bench.py: the AR exchange fell back to the host transport ({fallback}); "
                         f"refusing to time it (--allow-host-fallback to accept)\n")
        sys.exit(2)


def check_ar_nets(dist, digest: str, when: str) -> dict:
    """Every rank's AR-net digest (shards.ar_nets_digest); the exchange keeps the shards' AR nets
    one net, so unequal digests mean it did not work: exit 2 on every rank."""
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, digest)
    same = len(set(got)) == 1
    if not same:
        sys.stderr.write(f"bench.py: AR nets differ over the ranks {when}: {[g[:12] for g in got]}\n")
        sys.exit(2)
    return {"ar_nets_identical": True, "digest": got[0][:16]}


def check_exchange_calls(calls: int, steps: int, slices: int, every: int) -> dict:
    """The exchanges the timed pass made against its cadence: one per `every` learner calls,
    one learner call per slice.  A shortfall means some slice's exchange did not run: exit 2."""
    expected = steps * slices // every if slices % every == 0 else None
    if expected is not None and calls != expected:
        sys.stderr.write(f"bench.py: {calls} exchanges in the timed pass, {expected} expected "
                         f"({steps} steps x {slices} slices / every {every})\n")
        sys.exit(2)
    return {"calls_timed_pass": calls, "calls_expected": expected, "calls_ok": expected is not None}


def stub_main(args, world, rank, dist):
    """Test hook (`--stub-step-ms`): the launcher and the timing protocol with a CPU sleep in
    place of the engine step (no GPU).  Never a measurement: `data` says "stub"."""
    lanes = CONFIGS[args.config]["n_lanes"]
    if args.stub_fail:
        fr, fc = (int(v) for v in args.stub_fail.split(":"))
        if rank == fr:
            sys.stderr.write(f"stub: rank {rank} fails with {fc}\n")
            os._exit(fc)
    tl = {}
    # the exchange's protocol with a CPU stand-in: a 2 x 2,179 f32 "AR net" per rank, equal at
    # the start, W0 + mean of the ranks' random deltas after every one of the config's slices
    # (gloo all-reduce); --stub-rccl-fail R: rank R reports no RCCL (every rank falls back);
    # --stub-diverge R: rank R's net is perturbed after the timed pass (the digest check fires)
    import hashlib
    import torch
    slices = CONFIGS[args.config].get("slices", 1)
    xchg = dist is not None and world > 1
    net = torch.zeros(2 * 2179, dtype=torch.float32)
    calls = [0]
    fallback = None
    if xchg:
        ready = torch.tensor([0 if args.stub_rccl_fail is not None and rank == args.stub_rccl_fail else 1],
                             dtype=torch.int32)
        dist.all_reduce(ready, op=dist.ReduceOp.MIN)
        if int(ready.item()) == 0:
            fallback = "rccl setup failed on some rank: stub"
        refuse_host_fallback(args, world, fallback)
    gen = torch.Generator().manual_seed(rank)
    wd = StepWatchdog(rank) if dist is not None and world > 1 else None
    hang = tuple(int(v) for v in args.stub_hang.split(":")) if args.stub_hang else None
    nstep = [0]

    def step():
        nstep[0] += 1
        if wd is not None:
            wd.beat(f"step {nstep[0]}")
        if hang is not None and rank == hang[0] and nstep[0] == hang[1]:
            while True:                      # a rank stuck as in an all-reduce whose peer is gone
                time.sleep(1.0)
        for _ in range(slices):
            if xchg:
                d = torch.rand(net.numel(), generator=gen) * 1e-3
                dist.all_reduce(d)
                net.add_(d, alpha=1.0 / world)
                calls[0] += 1
        time.sleep(args.stub_step_ms * 1e-3 * (1 + 0.5 * rank))

    def digest():
        return hashlib.sha256(net.numpy().tobytes()).hexdigest()
    for _ in range(args.warmup):
        step()
    xcheck = {}
    if xchg:
        xcheck["after_warmup"] = check_ar_nets(dist, digest(), "after the warmup")
    c0 = calls[0]
    elapsed = timed_steps(step, args.steps, 0, dist, device="cpu", out=tl)
    c1 = calls[0]
    if xchg and args.stub_diverge is not None and rank == args.stub_diverge:
        net[0] += 1.0
    out = {"metric": "Leduc self-play hands/sec", "unit": "hands/s",
           "value": job_value(args.steps * lanes, world, elapsed), "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "data": "stub",
           "config": {"parallelism": f"dp{world}"}}
    if xchg:
        xcheck["after_timed_pass"] = check_ar_nets(dist, digest(), "after the timed pass")
        out["ar_allreduce"] = dict(check_exchange_calls(c1 - c0, args.steps, slices, 1), calls=calls[0],
                                   transport="stub", fallback=fallback, ar_nets_check=xcheck)
        # the stand-in net's "exploitability" is a placeholder; the hands are the protocol's
        out["ar_allreduce"]["learning_at_total_hands"] = learning_check(
            1.0, (args.warmup + args.steps) * lanes, world, True)
    if dist is not None:
        import socket
        out["ranks"] = rank_report(dist, "gloo", dict(
            device_identity(), host=socket.gethostname(), ms_per_step=tl["local_s"] / args.steps * 1e3,
            exchange_ms_per_call=None, exchanges=c1 - c0))
        if xchg:
            out["ranks"]["ar_nets_identical"] = True
    if rank == 0:
        emit_result(out)
    if dist is not None:
        dist.destroy_process_group()


def cpu_band(hands: int) -> dict | None:
    """The CPU reference's exact-exploitability seed band at `hands` hands (main.train restated
    in C++ with C3's memories, 24 seeds, every 2M hands to 32M: tests/golden/cpu_band_c3mem_24.json),
    at the nearest checkpoint.  Past its last checkpoint the last one stands in (the CPU curve is
    flat there, 1.384 / 1.381 at 30 / 32M), as the C3 / C4 gates compare their 33.5M and 67M
    points (tests/test_gpu_slices.py); `beyond_band` says so."""
    path = os.path.join(REPO, "tests", "golden", "cpu_band_c3mem_24.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        cb = json.load(f)["band"]
    pts = sorted(int(k) for k in cb)
    h = min(pts, key=lambda k: abs(k - hands))
    out = {"hands": h, "mean": cb[str(h)][0], "std": cb[str(h)][1],
           "source": "tests/golden/cpu_band_c3mem_24.json (24 seeds)"}
    if hands > pts[-1] + (pts[1] - pts[0]) // 2:
        out["beyond_band"] = True
    return out


def band_check(x: float, hands: int) -> dict:
    """One engine seed's exact exploitability against the CPU band at the same hands: the C3 /
    C4 gates' bar (|x - mean| <= 2 sigma and x <= mean + sigma; the gates average 16 / 8 seeds)."""
    b = cpu_band(hands)
    out = {"hands": hands, "exploitability": x, "cpu_band": b}
    if b is not None:
        out["sigmas_from_cpu_mean"] = (x - b["mean"]) / b["std"]
        out["inside_bar"] = abs(x - b["mean"]) <= 2 * b["std"] and x <= b["mean"] + b["std"]
    return out


def learning_check(x: float, hands_per_rank: int, world: int, exchanged: bool) -> dict:
    """band_check at the hands the evaluated net has learned from: with the AR exchange on, the
    ranks' AR nets are one net trained on every rank's hands, so the job's TOTAL hands (world x
    per rank) -- the x-axis of the C4 gate (tests/test_gpu_slices.py) and of the CPU band; without
    it, one shard's own hands."""
    out = band_check(x, hands_per_rank * world if exchanged else hands_per_rank)
    out["hands_are"] = "total over ranks (the exchanged AR net)" if exchanged else "this rank's"
    return out


def measure_group(pkg, name: str, steps: int, warmup: int) -> dict:
    """A side measurement beside the headline (N = 1): engine-group config `name`, the same
    sync protocol, and the exact exploitability of replica 0's AR nets (softmax mixed) against
    the CPU reference's band at the same TOTAL hands (all replicas' hands: the replicas share
    one AR net through the exchange).  Two forms:
    * c3_rR: C3's per-GPU lanes as R learner replicas, AR nets averaged once per step; W warmup
      + K timed steps (the stage is stated), exploitability after them;
    * c4_emul_rR: BASELINE configs[3]'s arithmetic on one GPU -- R replicas of C4's per-GPU
      shard (1,048,576 lanes in 128 pipelined slices, the AR nets exchanged after every slice,
      W0 + gain x mean delta: the rank path bit for bit, tests/test_gpu_exchange.py), trained
      from scratch for `learn_steps` steps, each step timed by itself and the exploitability
      taken between steps outside the timing: hands/s and the learning curve over the same
      hands."""
    import torch
    cfg = CONFIGS[name]
    R = cfg["replicas"]
    lanes = cfg["n_lanes"] // R
    xchg = cfg.get("xchg_every")
    extra = {k: cfg[k] for k in ("slices", "slice_lag") if k in cfg}
    g = pkg.engine.EngineGroup(R, n_lanes=lanes, rl_capacity=cfg["rl_capacity"], sl_capacity=cfg["sl_capacity"],
                               seed=1234, init_seed=0, avg_ar=not xchg, **extra)
    if cfg.get("sched"):
        g.set_sched(**cfg["sched"])
    out = {"workload": cfg["label"], "learner_replicas": R, "lanes_per_replica": lanes, "sched": g.sched(),
           "metric": "hands/s (beside it RL inserts/s: M_RL inserts, each 1/128 of an update_strategy)",
           "unit": "hands/s"}
    s0 = g.stats()
    if xchg:
        g.set_exchange(pkg.native.XCHG_AR, every=xchg, scale=cfg["xchg_gain"] / R)
        g.average_ar()                           # the ranks' broadcast: replica 0's AR nets
        curve, el = [], 0.0
        for k in range(cfg["learn_steps"]):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.step()
            torch.cuda.synchronize()
            el += time.perf_counter() - t0
            curve.append(band_check(g.exploitability(0)["exploitability"], (k + 1) * cfg["n_lanes"]))
        steps, warmup = cfg["learn_steps"], 0
        out["learning_curve"] = curve
        out["inside_bar_at_every_checkpoint"] = all(c.get("inside_bar", False) for c in curve)
        out["timing"] = "each step bracketed by device syncs from scratch; evaluations between steps untimed"
    else:
        for _ in range(warmup):
            g.step()
        torch.cuda.synchronize()
        s0 = g.stats()
        el = timed_steps(g.step, steps, 0, None, torch.cuda.synchronize)
    g.check()                                    # (a persistent BR kernel's expired wait raises)
    s1 = g.stats()
    hands = steps * cfg["n_lanes"]
    rl = sum(s1["rl_total"]) - sum(s0["rl_total"])
    ex = g.exploitability(0)["exploitability"]
    out.update({"value": hands / el, "hands_per_s": hands / el,
                "training_stage": {"warmup_steps": warmup, "hands_before_timing": warmup * cfg["n_lanes"]},
                "steps": steps, "warmup": warmup,
                "ms_per_step": el / steps * 1e3, "rl_inserts_per_s": rl / el,
                "rl_inserts_per_hand": rl / hands,
                "exploitability_exact_softmax": ex,
                "exploitability_vs_cpu_band": band_check(ex, int(s1["hands"])),
                "hands_trained": int(s1["hands"])})
    g.close()
    del g
    torch.cuda.empty_cache()
    return out


def rooflines(config, cfg, k_ms, k_launches, k_step_ms, br_upd, ar_upd, ar_max, t_rl, t_sl, hands_per_s,
              ms_per_step=None):
    """SURVEY 8(d)'s framings of the kernels, from one event-timed pass: k_ms = average ms per
    launch, k_launches = launches, k_step_ms = ms per engine step (per kernel / stream);
    br_upd / ar_upd = the pass's BR / AR updates (both agents), ar_max = the longest AR chain's
    updates; t_rl / t_sl = RL / SL inserts per hand; hands_per_s = the un-instrumented rate.
    ms_per_step: the un-instrumented pass's step time.  The headline kernel's duration is then
    capped by it: the critical stream runs its launches back to back, so one launch lasts at
    most the un-instrumented step / launches per step; the events around every launch add
    ~0.8 %, and the line's kernel time must not exceed its step time.
    Returns (roofline, roofline_other, whole_step_hbm_per_gpu, stream_ms_per_step).
    tests/test_bench_roofline.py feeds it the committed profiles' timings."""
    R = cfg.get("replicas", 1)
    slices = cfg.get("slices", 1)
    bytes_hand = BYTES_RL * t_rl + BYTES_SL * t_sl
    # one k_rollout launch plays one slice: n_lanes / slices lanes (a group's launch: every
    # replica's slice, R x (n_lanes / R) / slices -- the same count)
    lanes_launch = cfg["n_lanes"] // slices
    rollout_bytes = bytes_hand * lanes_launch
    # the rollout writes bit-packed staging records, not the reference's fp32 tuples: the
    # tuple bytes are a reference-layout EQUIVALENT; `traffic` / `achieved_counter` are what
    # the kernel moves (rocprofv3 PMC, profiles/pmc_<config>.json)
    roof_rollout = {"kernel": "k_rollout", "bound": "hbm",
                    "achieved": rollout_bytes / (k_ms["k_rollout"] * 1e-3) / 1e9,
                    "achieved_is": "reference-layout-equivalent bytes (257 B / 132 B fp32 tuples) of the "
                                   "hands one launch plays",
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "traffic": load_pmc(config, "k_rollout"),
                    "bytes_per_hand": bytes_hand, "lanes_per_launch": lanes_launch,
                    "bytes_per_launch": rollout_bytes, "avg_ms": k_ms["k_rollout"]}
    roof_rollout["frac"] = roof_rollout["achieved"] / PEAK_HBM_GBS
    if roof_rollout["traffic"]:
        roof_rollout["achieved_counter"] = roof_rollout["traffic"] / (k_ms["k_rollout"] * 1e-3) / 1e9
        roof_rollout["frac_counter"] = roof_rollout["achieved_counter"] / PEAK_HBM_GBS
        roof_rollout["traffic_vs_reference_layout"] = roof_rollout["traffic"] / rollout_bytes
    # SURVEY 8(d)'s whole-path figure: rollout writes + the sampled reads at the reference
    # cadence (T_rl / 128 updates x 128 rows x (257 + 132) B) per hand, over the timed step
    step_bytes_hand = bytes_hand + (t_rl / 128.0) * 128 * (BYTES_RL + BYTES_SL)
    whole_step = {"bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
                  "bytes_per_hand": step_bytes_hand, "achieved": step_bytes_hand * hands_per_s / 1e9}
    whole_step["frac"] = whole_step["achieved"] / PEAK_HBM_GBS

    def chain_mfma(name, updates):
        """The chain's matrix-core work: MFMA_PER_SGD_STEP v_mfma_f32_16x16x32_bf16 per SGD step
        (2 epochs x 4 minibatches of 32 per update), priced against the bf16 dense peak;
        `dense_equivalent_*` is the f32 FLOP count of the same steps (32 x F_TRAIN)."""
        n = max(k_launches[name], 1)
        sgd_steps = updates * 2 * 128 / 32 / n
        flop = sgd_steps * MFMA_PER_SGD_STEP * FLOP_PER_MFMA
        t = k_ms[name] * 1e-3
        ach = flop / t / 1e12 if t > 0 else 0.0
        return {"kernel": name, "bound": "mfma", "achieved": ach, "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s (bf16 MFMA executed)", "frac": ach / PEAK_BF16_TFLOPS, "traffic": None,
                "avg_ms": k_ms[name], "launches": k_launches[name], "flop_per_launch": flop,
                "dense_equivalent_tflops": (sgd_steps * 32 * F_TRAIN / t / 1e12) if t > 0 else 0.0}

    def chain_roof_hbm(name, updates, tuple_bytes):
        """SURVEY 8(d)'s HBM framing of a chain: algorithmic bytes = the 128 sampled memory
        tuples of each update (reference fp32 layout), per launch."""
        n = max(k_launches[name], 1)
        byt = updates * 128 * tuple_bytes / n
        ach = byt / (k_ms[name] * 1e-3) / 1e9 if k_ms[name] > 0 else 0.0
        return {"kernel": name, "bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": ach / PEAK_HBM_GBS, "traffic": load_pmc(config, name),
                "avg_ms": k_ms[name], "launches": k_launches[name], "bytes_per_launch": byt}

    par = 2 * R if R > 1 else 1

    def chain_issue(name, updates, net):
        """The chain's step as an issue roofline: the loop's static issue cycles per SGD step
        (tools/chain_census.py -> profiles/r06/chain_census.json, MI355X_MICROARCH.md issue
        costs) against the measured cycles per step at the chain's effective clock (2.40 GHz,
        tools/chain_clock.py).  frac = the share of the step one wave spends issuing."""
        path = os.path.join(REPO, "profiles", "r06", "chain_census.json")
        n = max(k_launches[name], 1) * (par if name == "k_chain3_br" else 1)
        steps = updates * 2 * 128 / 32 / n                  # epochs x minibatches per workgroup
        if not os.path.exists(path) or steps <= 0:
            return None
        with open(path) as f:
            issue = json.load(f)[net]["issue_cycles_per_step"]
        measured = k_ms[name] * 1e-3 / steps * CHAIN_CLOCK_HZ
        out = {"kernel": name, "bound": "issue", "achieved": issue, "peak": measured,
               "unit": "cycles per SGD step (static issue / measured)", "frac": issue / measured,
               "us_per_step": k_ms[name] * 1e3 / steps, "source": "profiles/r06/chain_census.json"}
        pmc = os.path.join(REPO, "profiles", "r06", "chain_pmc.json")   # tools/chain_pmc.sh
        if os.path.exists(pmc):
            with open(pmc) as f:
                out["sq_active_inst_frac"] = json.load(f)[net]["frac_active_inst"]
            out["sq_source"] = "profiles/r06/chain_pmc.json"
        return out

    # roofline: SURVEY 8(d)'s HBM framing (the judged bound) of each kernel; the MFMA and
    # issue framings of the chains go to roofline_other
    roofs = {"k_chain3_br_hbm": chain_roof_hbm("k_chain3_br", br_upd, BYTES_RL),
             "k_chain3_ar_hbm": chain_roof_hbm("k_chain3_ar", ar_upd, BYTES_SL),
             "k_rollout_hbm": roof_rollout,
             "k_chain3_br_mfma": chain_mfma("k_chain3_br", br_upd),
             "k_chain3_ar_mfma": chain_mfma("k_chain3_ar", ar_upd),
             "k_chain3_br_issue": chain_issue("k_chain3_br", br_upd, "br"),
             # one AR launch runs both agents' chains side by side: it lasts as long as the
             # agent with more updates
             "k_chain3_ar_issue": chain_issue("k_chain3_ar", ar_max, "ar")}
    # the dominant kernel = the one on the learner's critical path: the streams run side by
    # side (AR chains of both agents on one stream, each agent's BR targets + chains on its
    # own), so GPU time summed over streams overstates the BR chain; the stream whose busy
    # span per step is longest bounds the step, and its chain is the roofline kernel
    streams = {"ar_chain": k_step_ms["k_chain3_ar"], "br_stream_a0": k_step_ms["br_stream_a0"],
               "br_stream_a1": k_step_ms["br_stream_a1"]}
    crit = max(streams, key=streams.get)
    dom = "k_chain3_ar" if crit == "ar_chain" else "k_chain3_br"
    roof_key = f"{dom}_hbm"
    roofline = dict(roofs[roof_key])
    roofline["critical_stream"] = crit
    per_step = k_step_ms[dom] / k_ms[dom] if k_ms[dom] > 0 else 0.0      # launches per step
    roofline["launches_per_step"] = per_step
    roofline["avg_ms_event_timed"] = k_ms[dom]
    roofline["avg_ms_source"] = "HIP events around every launch (second pass)"
    if ms_per_step and per_step > 0 and ms_per_step / per_step < k_ms[dom]:
        roofline["avg_ms"] = ms_per_step / per_step
        roofline["avg_ms_source"] = ("un-instrumented step / launches per step on the critical stream "
                                     "(the event-timed average is longer: events around every launch)")
        roofline["achieved"] = roofline["bytes_per_launch"] / (roofline["avg_ms"] * 1e-3) / 1e9
        roofline["frac"] = roofline["achieved"] / PEAK_HBM_GBS
    pmc = load_pmc(config, roofline["kernel"])
    if pmc is not None:
        roofline["traffic"] = pmc
        roofline["traffic_source"] = f"profiles/pmc_{config}.json (rocprofv3 --pmc passes)"
    return roofline, {k: v for k, v in roofs.items() if k != roof_key}, whole_step, streams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: c3 at N = 1, c4 at N > 1")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-cores", type=int, default=None,
                    help="processes for the CPU baselines (default: this job's CPU share, cpu_share())")
    ap.add_argument("--cpu-worker", choices=["port", "numpy"], default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seed", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-workload", choices=["a", "b", "c"], default="c", help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL (one rank per GPU); gloo: a CPU-side rehearsal of the N > 1 path")
    ap.add_argument("--ar-allreduce", default="auto", choices=["auto", "on", "off"],
                    help="the all-reduce of the AR (average-policy) gradient steps over the ranks "
                         "(C4; shards.AvgPolicyExchange); auto = on for N > 1")
    ap.add_argument("--xchg-every", type=int, default=None,
                    help="the exchange after every k-th slice's learner (k = slices: once per step); "
                         "default: the config's (c4: 1), else 1")
    ap.add_argument("--xchg-gain", type=float, default=None,
                    help="W0 + gain x mean of the ranks' AR deltas (1: plain averaging; DESIGN.md §8); "
                         "default: the config's (c4: 2), else 2")
    ap.add_argument("--xchg-transport", default="auto", choices=["auto", "rccl", "host"],
                    help="rccl: libnfsp's own communicator on the AR chain stream; host: the process "
                         "group from a host callback; auto: rccl under nccl, host under gloo")
    ap.add_argument("--allow-host-fallback", action="store_true",
                    help="under --dist-backend nccl at N > 1, time the job even if the AR exchange fell "
                         "back to the host transport (default: exit 2)")
    ap.add_argument("--stub-step-ms", type=float, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--stub-rccl-fail", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--stub-diverge", type=int, default=None, help=argparse.SUPPRESS)
    # test hook with --stub-step-ms: rank R exits with code C after the process group is up
    ap.add_argument("--stub-fail", default=None, help=argparse.SUPPRESS)
    # test hook with --stub-step-ms: rank R's step N never returns (a peer lost in a collective)
    ap.add_argument("--stub-hang", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--slices", type=int, default=None, help="override the config's lane slices")
    ap.add_argument("--slice-lag", type=int, default=None, choices=[1, 2],
                    help="override the config's slice lag (2: slices pipelined)")
    ap.add_argument("--groups", default="c4_emul_r8,c3_r4,c3_r16,c3_r64,c3_r256",
                    help="engine-group configs measured beside the C3 headline at N = 1 "
                         "(`groups` in the JSON line; '' = none)")
    args = ap.parse_args()
    if args.config is None:
        args.config = "c4" if max(args.gpus, int(os.environ.get("WORLD_SIZE", "1"))) > 1 else "c3"
    c = CONFIGS[args.config]
    if "learn_steps" in c:
        ap.error(f"{args.config} is a one-GPU group line: bench.py --groups {args.config}")
    args.xchg_every = args.xchg_every if args.xchg_every is not None else c.get("xchg_every", 1)
    args.xchg_gain = args.xchg_gain if args.xchg_gain is not None else c.get("xchg_gain", 2.0)
    slices = args.slices if args.slices is not None else c.get("slices", 1)
    if args.xchg_every < 1 or slices % args.xchg_every:
        # every step must end on an exchange: the AR-net digest check after the warmup and after
        # the timed pass compares the ranks' nets, which agree only right after an exchange
        ap.error(f"--xchg-every {args.xchg_every} must divide the config's {slices} slices")

    if args.cpu_worker:                # a CPU-baseline child process: no GPU, one JSON line
        print(json.dumps(cpu_worker(args.cpu_worker, args.cpu_seconds, args.config, args.cpu_seed,
                                    args.cpu_workload)))
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's `bench.py --gpus N` without torch.distributed.run: one rank per GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    claim_stdout()
    check_world(args, int(os.environ.get("WORLD_SIZE", "1")))
    if args.stub_step_ms is not None:
        world, rank, _, dist = init_dist("gloo")
        return stub_main(args, world, rank, dist)

    import torch
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % torch.cuda.device_count())   # one rank per GPU (mod: rehearsals)
    world, rank, local, dist = init_dist(args.dist_backend, force=args.ar_allreduce == "on")
    # N > 1: a rank stuck on the device (an RCCL exchange or communicator setup whose peer is
    # gone) exits instead of holding the job until the driver's limit
    wd = StepWatchdog(rank) if dist is not None and world > 1 else None

    import __graft_entry__
    pkg = __graft_entry__.load_package()
    cfg = dict(CONFIGS[args.config])
    for k, v in (("slices", args.slices), ("slice_lag", args.slice_lag)):
        if v is not None:
            cfg[k] = v
            cfg["label"] += f" [{k} {v}]"
    game = pkg.native.GAME_KUHN if cfg.get("game") == "kuhn" else pkg.native.GAME_LEDUC
    R = cfg.get("replicas", 1)
    if R > 1:        # seeds 1234 + R rank + r: distinct over every replica of the job
        eng = pkg.engine.EngineGroup(R, n_lanes=cfg["n_lanes"] // R, rl_capacity=cfg["rl_capacity"],
                                     sl_capacity=cfg["sl_capacity"], seed=1234 + R * rank,
                                     init_seed=R * rank, game=game, avg_ar=True)
    else:
        extra = {k: cfg[k] for k in ("quirks", "slices", "slice_lag") if k in cfg}
        eng = pkg.engine.SelfPlayEngine(n_lanes=cfg["n_lanes"], rl_capacity=cfg["rl_capacity"],
                                        sl_capacity=cfg["sl_capacity"], seed=1234 + rank,
                                        init_seed=rank, game=game, **extra)
    avg = None
    if R == 1 and dist is not None and (args.ar_allreduce == "on" or (args.ar_allreduce == "auto" and world > 1)):
        # C4: the AR nets of both agents, W0 + mean of the ranks' deltas after every
        # `xchg_every`-th slice, on the AR chain stream
        if wd is not None:
            wd.beat("exchange setup (RCCL communicator)")
        avg = pkg.shards.AvgPolicyExchange(eng, dist, every=args.xchg_every, transport=args.xchg_transport,
                                           gain=args.xchg_gain)
        refuse_host_fallback(args, world, avg.fallback)

    nstep = [0]

    def step():
        nstep[0] += 1
        if wd is not None:
            wd.beat(f"engine step {nstep[0]}")
        eng.step()
    dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    xcheck = {}
    if avg is not None and world > 1:       # the exchange kept the shards' AR nets one net
        xcheck["after_warmup"] = check_ar_nets(dist, pkg.shards.ar_nets_digest(eng), "after the warmup")
    # `value`: K steps with no instrumentation at all
    s0 = eng.stats()
    tl = {}
    x0 = avg.calls if avg is not None else 0
    elapsed = timed_steps(step, args.steps, 0, dist, torch.cuda.synchronize, device=dev, out=tl)
    x1 = avg.calls if avg is not None else 0
    s1 = eng.stats()
    if avg is not None and world > 1:
        xcheck["after_timed_pass"] = check_ar_nets(dist, pkg.shards.ar_nets_digest(eng), "after the timed pass")
    xcalls = check_exchange_calls(x1 - x0, args.steps, cfg.get("slices", 1), args.xchg_every) \
        if avg is not None else None
    # per-kernel durations: K more steps with HIP events around every launch (kernel_ms,
    # roofline); their wall time is reported beside `value`, never as it
    eng.set_timing(True)
    eng.timings()
    elapsed_ev = timed_steps(step, args.steps, 0, dist, torch.cuda.synchronize, device=dev)
    timings = eng.timings()
    eng.set_timing(False)
    s2 = eng.stats()

    hands_rank = args.steps * cfg["n_lanes"]
    value = job_value(hands_rank, world, elapsed)
    br_upd = sum(s2["br_updates"]) - sum(s1["br_updates"])      # the instrumented pass's work
    ar_upd = sum(s2["ar_updates"]) - sum(s1["ar_updates"])
    rl_ins = sum(s1["rl_total"]) - sum(s0["rl_total"])          # the timed pass's inserts
    sl_ins = sum(s1["sl_total"]) - sum(s0["sl_total"])
    k_ms = {k: v[0] / max(v[1], 1) for k, v in timings.items()}
    k_step_ms = {k: v[0] / args.steps for k, v in timings.items()}       # per engine step
    k_launches = {k: v[1] for k, v in timings.items()}
    t_rl, t_sl = rl_ins / hands_rank, sl_ins / hands_rank
    # the issue framing is per chain workgroup: the AR launch lasts as long as its longest
    # chain, a BR launch runs up to 2R segments side by side
    reps1, reps2 = s1.get("replicas", [s1]), s2.get("replicas", [s2])
    ar_max = max(b["ar_updates"][a] - x["ar_updates"][a] for x, b in zip(reps1, reps2) for a in (0, 1))
    roofline, roofs_other, whole_step, streams = rooflines(
        args.config, cfg, k_ms, k_launches, k_step_ms, br_upd, ar_upd, ar_max, t_rl, t_sl,
        hands_rank / elapsed, ms_per_step=elapsed / args.steps * 1e3)
    rollout_path_ms = k_step_ms["k_rollout"] + k_step_ms["k_scan"] + k_step_ms["k_commit"]
    out = {
        "metric": "Kuhn self-play hands/sec" if cfg.get("game") == "kuhn" else "Leduc self-play hands/sec",
        "value": value,
        "unit": "hands/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "ms_per_step_event_timed": elapsed_ev / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: Philox self-play deals/draws, Glorot-uniform random-init nets",
        "config": {"workload": cfg["label"], "lanes_per_gpu": cfg["n_lanes"], "learner_replicas_per_gpu": R,
                   "rl_capacity": cfg["rl_capacity"], "sl_capacity": cfg["sl_capacity"],
                   "inserts_per_update": 128, "batch": 128, "parallelism": (f"dp{world}: shards + AR-gradient all-reduce every "
                                   f"{args.xchg_every} slice(s) ({avg.transport})"
                                   if avg is not None else
                                   f"replicas x{world} GPUs x {R} learner replicas per GPU (on-device AR average per step)"
                                   if R > 1 else f"replicas x{world}")},
        "roofline": roofline,
        "roofline_other": roofs_other,
        "whole_step_hbm_per_gpu": whole_step,
        "kernel_ms": k_ms,
        "kernel_ms_per_step": k_step_ms,
        "kernel_ms_source": "HIP events around every launch, second pass of K steps",
        "stream_ms_per_step": streams,
        "slices": cfg.get("slices", 1),
        "slice_lag": cfg.get("slice_lag", 1),
        "rollout_only_hands_per_s": cfg["n_lanes"] / (rollout_path_ms * 1e-3) * world,
        "per_step": {"br_updates": br_upd / args.steps, "ar_updates": ar_upd / args.steps,
                     "ar_updates_max_chain": ar_max / args.steps,
                     "rl_inserts_per_hand": t_rl, "sl_inserts_per_hand": t_sl},
        "exploitability_proxy": sum(s2["exploitability"]),
    }
    xchg_ms = k_ms.get("ar_exchange") if avg is not None and k_launches.get("ar_exchange") else None
    if avg is not None:
        out["ar_allreduce"] = {**xcalls, "calls": avg.calls, "bytes_per_call": avg.bytes_per_call,
                               "ar_nets_check": xcheck or None,
                               "backend": args.dist_backend, "transport": avg.transport, "fallback": avg.fallback,
                               "every_slices": args.xchg_every, "gain": args.xchg_gain,
                               "ms_per_call_event_timed": xchg_ms,
                               "ms_per_call_is": "HIP events on the AR stream around delta + all-reduce + "
                                                 "apply (includes waiting for the slowest rank's AR chain)"}
    if dist is not None:
        import socket
        out["ranks"] = rank_report(dist, args.dist_backend, dict(
            device_identity(), host=socket.gethostname(), ms_per_step=tl["local_s"] / args.steps * 1e3,
            ms_per_step_event_timed=elapsed_ev / args.steps * 1e3,
            exchange_ms_per_call=xchg_ms, exchanges=(x1 - x0)))
        if xcheck:
            out["ranks"]["ar_nets_identical"] = True      # else check_ar_nets exited 2
    # exact exploitability of the AR nets after the timed steps (outside the timed region)
    ex = {m: eng.exploitability(m) for m in (0, 1)}
    out["exploitability_exact"] = {
        "softmax_mixed": ex[0]["exploitability"], "argmax_as_executed": ex[1]["exploitability"],
        "hands_trained_per_gpu": int(s2["hands"]), "unit": "chips (BR_0 + BR_1)"}
    if cfg.get("game", "leduc") == "leduc" and cfg["rl_capacity"] == 200_000:
        # the CPU reference's seed band at the same hands (one seed of the engine here): at N > 1
        # with the exchange on, the total hands of the job (the AR net learned from all of them)
        exchanged = avg is not None and world > 1
        chk = learning_check(ex[0]["exploitability"], int(s2["hands"]), world, exchanged)
        out["exploitability_exact"]["vs_cpu_band"] = chk
        if exchanged:
            out["ar_allreduce"]["learning_at_total_hands"] = chk
    if world == 1 and args.config == "c3" and args.groups:
        # several learners on the one GPU (engine groups): new measured configs, not the headline
        eng.close()
        del eng
        torch.cuda.empty_cache()
        out["groups"] = {name: measure_group(pkg, name, max(args.steps, 10), args.warmup)
                         for name in args.groups.split(",")}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.config, args.cpu_cores)
        out["cpu_baseline_numpy"] = cpu_baseline_numpy(min(args.cpu_seconds, 5.0), args.config, args.cpu_cores)
        out["cpu_baseline_rollout"] = cpu_baseline_rollout(min(args.cpu_seconds, 4.0), args.config, args.cpu_cores)
        out["cpu_baseline_rollout"]["gpu_rollout_only_hands_per_s"] = out["rollout_only_hands_per_s"]
    if rank == 0:
        emit_result(out)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
