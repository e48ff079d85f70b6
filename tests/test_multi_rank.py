"""CPU, world_size 2 (gloo): the replica bench's multi-rank logic — every rank times its own
videos, the job time is the max over ranks, value counts all ranks' frames (weak scaling) —
exactly the code bench.py runs over RCCL on the GPU box."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed = 2.0 + rank            # rank 1 is the slow one
    t = bench.max_over_ranks(elapsed, torch.device("cpu"))
    v = bench.whole_job_frames_per_s(world, 49, 3, t)
    dist.barrier()
    q.put((rank, t, v))
    dist.destroy_process_group()


def test_two_rank_replica_timing_is_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, v in out:
        assert t == pytest.approx(3.0)
        assert v == pytest.approx(2 * 49 * 3 / 3.0)


def test_single_process_is_identity():
    import bench
    assert bench.max_over_ranks(1.25, torch.device("cpu")) == 1.25
    assert bench.whole_job_frames_per_s(1, 49, 2, 0.5) == pytest.approx(196.0)


def test_bench_self_launches_n_workers():
    """bench.py --gpus 2 without a launcher's WORLD_SIZE starts 2 fresh worker processes (the
    GPU work stubbed by a CPU sleep of 20 ms x (rank+1) per step, gloo): rank 0 prints one line
    that saw 2 distinct ranks and the slower rank's time."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--stub-cpu", "--steps", "5", "--warmup", "0"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks"] == [0, 1]
    assert res["ms_per_step"] >= 40.0          # rank 1 sleeps 40 ms per step
    assert res["value"] == pytest.approx(2 * 49 * 5 / (res["ms_per_step"] * 5 / 1000.0))
    assert res["per_gpu_frames_per_s"] == pytest.approx(res["value"] / 2)


def test_train_bench_self_launches_n_workers():
    """tools/train_bench.py --gpus 2 starts 2 worker processes itself (the training step stubbed
    by a CPU sleep of 20 ms x (rank+1), gloo): one line, 2 ranks, the slower rank's time."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "train_bench.py"), "--gpus", "2",
                        "--stub-cpu", "--steps", "5", "--batch", "5", "--accum", "4"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks"] == [0, 1]
    assert res["ms_per_step"] >= 40.0
    assert res["value"] == pytest.approx(2 * 5 * 4 * 5 / (res["ms_per_step"] * 5 / 1000.0))
