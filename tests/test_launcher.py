"""Supervised launcher: a crashed rank and a hung rank are detected, the
whole group is restarted, and the job resumes from its checkpoint on the next attempt
(loopback fake communicator, world size 2, CPU)."""
import json
import os

import pytest
import torch

from flink_tensorflow_amd.parallel.fake import FakeCommunicator
from flink_tensorflow_amd.parallel.launcher import WorkerFailure, launch


def _train(rank, world, attempt, ckpt_dir, fault):
    """10 'steps' of an all-reduced counter with a checkpoint after every step; the fault
    fires once, on attempt 0 at step 4 on rank 1."""
    from flink_tensorflow_amd.parallel import comm
    from flink_tensorflow_amd.parallel.launcher import heartbeat

    path = os.path.join(ckpt_dir, f"rank{rank}.json")
    step, total = 0, 0.0
    if os.path.exists(path):
        with open(path) as f:
            st = json.load(f)
        step, total = st["step"], st["total"]
    resumed_from = step
    while step < 10:
        if attempt == 0 and rank == 1 and step == 4:
            if fault == "crash":
                os._exit(3)
            if fault == "hang":
                import time

                time.sleep(600)
        t = torch.tensor([float(rank + 1)])
        comm.get().all_reduce(t)
        total += float(t)
        step += 1
        with open(path, "w") as f:
            json.dump({"step": step, "total": total}, f)
        heartbeat(f"step {step}")
    return {"total": total, "resumed_from": resumed_from}


@pytest.mark.parametrize("fault", ["crash", "hang"])
def test_restart_after_failure(tmp_path, fault):
    rep = launch(_train, 2, args=(str(tmp_path), fault), communicator=FakeCommunicator, max_restarts=1, heartbeat_timeout=15.0,
                 timeout=120)
    assert rep.attempts == 2 and len(rep.failures) == 1
    assert ("exited with code 3" in rep.failures[0]) if fault == "crash" else ("missed heartbeats" in rep.failures[0])
    for r in rep.results:
        assert r["total"] == 30.0  # 10 steps x (1 + 2), nothing lost or double counted
        assert r["resumed_from"] >= 4


def test_gives_up_after_max_restarts(tmp_path):
    with pytest.raises(WorkerFailure):
        launch(_boom, 2, communicator=FakeCommunicator, max_restarts=1, timeout=60)


def _boom(rank, world, attempt):
    raise RuntimeError("boom")


def _silent_exit(rank, world, attempt):
    if rank == 1:
        os._exit(0)  # exits "successfully" without posting a result
    return rank


def test_clean_exit_without_result_is_a_failure():
    with pytest.raises(WorkerFailure, match="without a result"):
        launch(_silent_exit, 2, communicator=FakeCommunicator, max_restarts=0, timeout=60)


# ---------------------------------------------------------------- bench.py self-launch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, timeout=240):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=ROOT)


def test_bench_spawns_its_own_ranks():
    """``python bench.py --gpus 2`` outside any launcher starts 2 rank processes itself
    (torch.distributed.run as a child), they rendezvous and rank 0 prints the world."""
    p = _bench("--gpus", "2", "--rehearse-fake-comm", "--launch-check")
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["world_size"] == 2 and out["comm_world_size"] == 2
    assert out["ranks"] == [0, 1] and out["pids_distinct"]


def test_bench_refuses_missing_gpus():
    """Asking for more GPUs than are visible fails loudly instead of measuring fewer."""
    if torch.cuda.device_count() >= 2:
        pytest.skip("box has 2+ GPUs")
    p = _bench("--gpus", "2", timeout=120)
    assert p.returncode != 0
    assert "refusing" in p.stderr


def test_sysfs_gpu_count_reads_kfd_topology(tmp_path, monkeypatch):
    """GPUs are counted from the KFD topology (nodes with SIMDs), narrowed by a visibility
    mask, without loading any GPU library."""
    from flink_tensorflow_amd.utils.gpus import sysfs_gpu_count

    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):  # CPU nodes have simd_count 0
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simds}\nmem_banks_count 1\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert sysfs_gpu_count(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert sysfs_gpu_count(str(tmp_path)) == 1
    assert sysfs_gpu_count(str(tmp_path / "missing")) == 0


def test_window_timeline_splits_fill_from_steady_state():
    """tools/window_timeline.py: a two-lane window whose batches complete every 3 ms after a
    7 ms first batch reports the 3 ms period and the fill as a constant overhead."""
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "window_timeline.py")
    spec = importlib.util.spec_from_file_location("window_timeline", path)
    wt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(wt)
    tl = [{"lane": i % 2, "n": 256, "submit_ms": 0.1 * i, "h2d_ms": 0.2, "start_ms": 0.1 + 3.0 * max(0, i - 1),
           "done_ms": 7.0 + 3.0 * i} for i in range(20)]
    r = wt.analyse(tl, elapsed=7.0 + 3.0 * 19 + 0.1)
    assert abs(r["period_ms"] - 3.0) < 1e-9 and r["batches"] == 20
    assert abs(r["overhead_ms"] - (r["elapsed_ms"] - 60.0)) < 1e-9 and 3.9 < r["overhead_ms"] < 4.2
