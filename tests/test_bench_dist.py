"""bench.py's multi-GPU protocol on CPU (gloo, world size 2): one process per rank, a barrier
and device sync around exactly K timed steps, the MAX elapsed over ranks, and the whole-job
value = units of all ranks / that time (bench.py timed_steps / job_value).  The GPU engine
itself is replaced by a CPU step of known, rank-dependent duration."""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, REPO)
    import bench
    w, r, _, dist = bench.init_dist(backend="gloo")
    calls = []
    dt = 0.02 * (1 + rank)                  # rank 1 is the slow one

    def step():
        calls.append(1)
        time.sleep(dt)
    elapsed = bench.timed_steps(step, steps=4, warmup=2, dist=dist, device="cpu")
    q.put((r, w, len(calls), elapsed, bench.job_value(100 * 4, w, elapsed)))
    dist.destroy_process_group()


def _bench(args, env_extra=None, timeout=180):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    return r.returncode, lines, r.stderr


def test_gpus_flag_launches_the_ranks():
    """`bench.py --gpus 2` with no torch.distributed environment (how the driver may call it)
    starts two rank processes itself; rank 0 prints one line for the whole 2-rank job."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--stub-step-ms", "20",
                             "--config", "c2"])
    assert rc == 0, err
    assert len(lines) == 1, lines
    # stdout holds the result line only: the ranks send every other write to fd 1 (gloo's
    # "Rank k is connected" lines, library banners) to stderr
    stdout = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1",
                             "--warmup", "0", "--stub-step-ms", "1"], capture_output=True, text=True,
                            timeout=120, env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}).stdout
    assert len(stdout.splitlines()) == 1 and json.loads(stdout)["n_gpus"] == 2, stdout
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    # rank 1 sleeps 1.5x as long: the job time is the slow rank's
    assert out["ms_per_step"] >= 30.0
    assert abs(out["value"] - 2 * 3 * 65_536 / (out["ms_per_step"] * 3e-3)) < 1e-6 * out["value"]
    # N > 1 explains itself: every rank's own step time, device / PCI bus id, exchange cost
    rk = out["ranks"]
    assert rk["world_size"] == 2 and [r["rank"] for r in rk["ranks"]] == [0, 1]
    ms = [r["ms_per_step"] for r in rk["ranks"]]
    assert 20.0 <= ms[0] < ms[1] and ms[1] >= 30.0
    assert rk["ms_per_step_min"] == ms[0] and rk["ms_per_step_max"] == ms[1]
    assert out["ms_per_step"] >= ms[1]            # the job waits for the slowest rank
    for r in rk["ranks"]:
        for k in ("device", "pci_bus_id", "host", "exchange_ms_per_call", "exchanges"):
            assert k in r, (k, r)


def test_one_rank_line_has_no_rank_report():
    rc, lines, err = _bench(["--steps", "2", "--warmup", "0", "--stub-step-ms", "5"])
    assert rc == 0, err
    assert len(lines) == 1 and lines[0]["n_gpus"] == 1 and "ranks" not in lines[0]


def test_world_size_mismatch_refused():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero instead of timing a
    different job than the one asked for."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--stub-step-ms", "1"],
                            env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2 and not lines
    assert "WORLD_SIZE 1 != --gpus 2" in err


def test_failing_rank_ends_the_job_fast():
    """A rank that dies (here: rank 1 exits 3 once the group is up) ends the whole job with its
    exit code within seconds: the launcher stops rank 0, which is blocked in the timed
    region's barrier, instead of waiting for the process-group timeout."""
    t0 = time.time()
    rc, lines, err = _bench(["--gpus", "2", "--steps", "50", "--warmup", "1", "--stub-step-ms", "20",
                             "--stub-fail", "1:3"], env_extra={"NFSP_PG_TIMEOUT_S": "600"})
    assert rc == 3, err
    assert not lines
    assert "rank 1 exited with 3" in err
    assert time.time() - t0 < 60


def test_two_rank_timing_protocol():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, n0, e0, v0), (r1, w1, n1, e1, v1) = res
    assert (r0, r1, w0, w1) == (0, 1, 2, 2)
    assert n0 == n1 == 6                      # warmup 2 + exactly 4 timed steps on every rank
    assert e0 == e1                           # every rank sees the max over ranks
    assert e0 >= 4 * 0.04                     # ... which is the slow rank's time
    assert v0 == v1 == 800 / e0               # whole-job units / max time


def test_n2_line_proves_its_exchange():
    """N > 1 with the exchange on (the stub's CPU stand-in of the AR nets, exchanged after every
    slice over gloo): the line carries the exchanges the timed pass made against its cadence and
    the ranks' AR-net digests, equal after the warmup and after the timed pass."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--stub-step-ms", "5",
                             "--config", "c2"])
    assert rc == 0, err
    x = lines[0]["ar_allreduce"]
    assert x["calls_timed_pass"] == x["calls_expected"] == 3 * 16 and x["calls_ok"]
    assert x["fallback"] is None
    chk = x["ar_nets_check"]
    assert chk["after_warmup"]["ar_nets_identical"] and chk["after_timed_pass"]["ar_nets_identical"]
    assert lines[0]["ranks"]["ar_nets_identical"] is True
    # the exchanged AR net is scored at the job's TOTAL hands: 2 ranks x (1 + 3) steps x 65,536
    lt = x["learning_at_total_hands"]
    assert lt["hands"] == 2 * 4 * 65_536 and lt["hands_are"].startswith("total")
    assert lt["cpu_band"]["hands"] == 0 or lt["cpu_band"]["hands"] % 2_000_000 == 0


def test_n1_line_has_no_exchange_fields():
    rc, lines, err = _bench(["--steps", "2", "--warmup", "1", "--stub-step-ms", "2", "--config", "c2"])
    assert rc == 0, err
    assert "ar_allreduce" not in lines[0]


def test_learning_check_x_axis():
    """bench.learning_check: per-rank hands without the exchange, world x hands with it."""
    import bench
    a = bench.learning_check(1.3, 8_388_608, 8, False)
    b = bench.learning_check(1.3, 8_388_608, 8, True)
    assert a["hands"] == 8_388_608 and a["cpu_band"]["hands"] == 8_000_000
    assert b["hands"] == 67_108_864 and b["cpu_band"]["beyond_band"] is True


def test_xchg_every_must_divide_the_slices():
    """an --xchg-every that does not divide the slices would leave a step's last
    slices unexchanged, and the AR-net digest check would end the job; it is refused up front."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--stub-step-ms", "2",
                             "--config", "c2", "--xchg-every", "3"])
    assert rc == 2 and not lines
    assert "must divide" in err
    rc, lines, err = _bench(["--steps", "1", "--warmup", "0", "--stub-step-ms", "2", "--config", "c2",
                             "--xchg-every", "4"])
    assert rc == 0, err


def test_host_fallback_refused_under_rccl():
    """A rank that cannot set up RCCL makes every rank fall back to the host transport; under
    --dist-backend nccl at N > 1 the job then exits 2 instead of timing the slower job ..."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "2", "--warmup", "0", "--stub-step-ms", "2",
                             "--config", "c2", "--stub-rccl-fail", "1"])
    assert rc == 2 and not lines, err
    assert "refusing to time it" in err
    # ... unless the fallback is asked for; the line then says so
    rc, lines, err = _bench(["--gpus", "2", "--steps", "2", "--warmup", "0", "--stub-step-ms", "2",
                             "--config", "c2", "--stub-rccl-fail", "1", "--allow-host-fallback"])
    assert rc == 0, err
    assert lines[0]["ar_allreduce"]["fallback"].startswith("rccl setup failed")


def test_diverged_ar_nets_end_the_job():
    """Ranks whose AR nets differ after the timed pass (rank 1's perturbed) exit 2: no line."""
    rc, lines, err = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--stub-step-ms", "2",
                             "--config", "c2", "--stub-diverge", "1"])
    assert rc == 2 and not lines, err
    assert "AR nets differ over the ranks after the timed pass" in err


def test_stuck_rank_ends_the_job():
    """a rank stuck in a step (here: rank 1's second step never returns, as in
    an exchange whose peer is gone -- libnfsp's RCCL all-reduce is outside torch's process-group
    timeout) exits 124 once its step watchdog (NFSP_STEP_WATCHDOG_S) sees no progress, and the
    launcher stops the other rank: the job ends with 124 in seconds, with no result line."""
    t0 = time.time()
    rc, lines, err = _bench(["--gpus", "2", "--steps", "4", "--warmup", "1", "--stub-step-ms", "5",
                             "--config", "c2", "--stub-hang", "1:2"],
                            env_extra={"NFSP_STEP_WATCHDOG_S": "3", "NFSP_PG_TIMEOUT_S": "600"})
    assert rc == 124, err
    assert not lines
    assert "rank 1 made no progress" in err and "last: step 2" in err
    assert time.time() - t0 < 60


def test_eight_rank_job_like_the_drivers_scale_run():
    """The driver's N = 8 invocation (`bench.py --gpus 8`, C4's arithmetic per rank: 128 slices,
    the AR exchange after every slice) rehearsed with 8 gloo ranks on the CPU: one line, dp8,
    the whole-job value over the slowest rank's time, every rank reported, every exchange made
    and the ranks' AR nets identical after it, the learning check at the job's total hands."""
    rc, lines, err = _bench(["--gpus", "8", "--steps", "2", "--warmup", "1", "--stub-step-ms", "5"],
                            timeout=300)
    assert rc == 0, err
    assert len(lines) == 1, lines
    out = lines[0]
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    lanes = 1_048_576
    assert abs(out["value"] - 8 * 2 * lanes / (out["ms_per_step"] * 2e-3)) < 1e-6 * out["value"]
    rk = out["ranks"]
    assert rk["world_size"] == 8 and [r["rank"] for r in rk["ranks"]] == list(range(8))
    assert out["ms_per_step"] >= rk["ms_per_step_max"]
    x = out["ar_allreduce"]
    assert x["calls_timed_pass"] == x["calls_expected"] == 2 * 128 and x["calls_ok"]
    assert x["ar_nets_check"]["after_timed_pass"]["ar_nets_identical"]
    assert x["learning_at_total_hands"]["hands"] == 8 * 3 * lanes
