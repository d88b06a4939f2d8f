"""bench.py's multi-GPU protocol on CPU (gloo, world size 2): one process per rank, a barrier
and device sync around exactly K timed steps, the MAX elapsed over ranks, and the whole-job
value = units of all ranks / that time (bench.py timed_steps / job_value).  The GPU engine
itself is replaced by a CPU step of known, rank-dependent duration."""
import multiprocessing as mp
import os
import socket
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
