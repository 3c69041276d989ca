"""CPU: bench.py's multi-GPU harness (VERDICT r1 missing #2). `python bench.py --gpus N` started by
hand launches the N ranks itself (enf_launch.py: torch.distributed.run child processes, before
anything touches a device); each rank times its share, the wall time is the max over ranks and
`value` aggregates all ranks' samples. Exercised here with gloo and a CPU stand-in step
(--selftest-cpu); on the GPU box the same harness runs on RCCL with the enf_flow_apply step."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def run_bench(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--selftest-cpu", "--no-cpu", "--steps", "3",
                        "--warmup", "1", "--N", "1000", *args], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_single_rank_line():
    out = run_bench()
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup"] == 1
    # the settle phase is reported in the line (the CPU stand-in step never settles a GPU clock)
    assert out["settle"]["launches"] == 0 and "steady clock" in out["settle"]["why"]
    assert out["distributed"]["world_size"] == 1 and len(out["distributed"]["per_rank_kernel_ms"]) == 1
    assert out["value"] == pytest.approx(1000 * 3 / (out["ms_per_step"] * 3 / 1e3), rel=1e-6)


def test_bench_launches_two_ranks():
    out = run_bench("--gpus", "2")
    assert out["n_gpus"] == 2
    d = out["distributed"]
    assert d["world_size"] == 2 and d["backend"] == "gloo" and d["data_path_collective"] is None
    assert len(d["per_rank_kernel_ms"]) == 2 and all(v > 0 for v in d["per_rank_kernel_ms"])
    # whole-job aggregate: both ranks' samples over the max-over-ranks wall time
    assert out["value"] == pytest.approx(2 * 1000 * 3 / (out["ms_per_step"] * 3 / 1e3), rel=1e-6)
    assert out["scaling"] == "weak" and out["config"]["N_total"] == 2000
    # the config-5 leg at N = 2: minibatch shares tile every batch, the ranks agree, and the step the GPU
    # run times is the graph-captured libenf RCCL (EnfComm) data-parallel step
    t = out["train"]
    assert t["n_gpus"] == 2 and t["ranks_agree"] and len(t["per_rank_s"]) == 2
    assert "EnfComm" in t["step"] and "captured in the HIP graph" in t["step"]


@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_bench_strong_scaling_line(gpus):
    """--scaling strong: the N = 1000 columns are split over the ranks in contiguous shards
    (1000 = 333 + 333 + 334 at three ranks), value = N x steps / the max-over-ranks time, "scaling": "strong"."""
    out = run_bench("--gpus", str(gpus), "--scaling", "strong", "--no-train")
    assert out["n_gpus"] == gpus and out["scaling"] == "strong"
    c = out["config"]
    assert c["N_total"] == 1000 and c["N_per_gpu"] == 1000 // gpus  # (rank 0: [0, 1000 // gpus))
    assert "in all, split over" in c["workload"]
    assert out["value"] == pytest.approx(1000 * 3 / (out["ms_per_step"] * 3 / 1e3), rel=1e-6)


def test_bench_world_mismatch_is_an_error():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--selftest-cpu", "--gpus", "2", "--no-cpu"],
                       capture_output=True, text=True, timeout=120, env={**os.environ, **env}, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def run_bench_train(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench_train.py"), "--selftest-cpu", "--steps", "7",
                        "--N", "1003", "--nbatches", "4", *args], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_bench_train_launches_ranks(gpus):
    """bench_train.py --gpus N starts N ranks itself; the ranks' minibatch shares tile every batch
    (asserted inside each rank) and all ranks apply the same update."""
    out = run_bench_train("--gpus", str(gpus))
    assert out["n_gpus"] == gpus and len(out["per_rank_s"]) == gpus
    assert out["ranks_agree"] and out["config"]["parallelism"] == f"dp{gpus}"
