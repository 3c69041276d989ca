"""One process per GPU for bench.py / bench_train.py (harness plumbing, not product).

``python bench.py --gpus N`` started by hand (no WORLD_SIZE in the environment) starts N ranks
itself: ``python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1``
on the same script and arguments, as CHILD processes, and the parent exits with their exit code.
The parent never touches the GPU (no torch.cuda call happens before this point), so no GPU-
initialised process is replaced or forked. Under the driver's own ``torch.distributed.run`` launch
WORLD_SIZE is set and each process simply is one rank.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks_if_needed(n: int, script: str, argv: List[str]) -> Optional[int]:
    """Return None if this process is a rank (WORLD_SIZE set, or n == 1); otherwise run n ranks of
    ``script argv`` under torch.distributed.run and return their exit code."""
    if n <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def rank_env():
    """(world, rank, local_rank) from torch.distributed.run's environment (1, 0, 0 without it)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def check_world(gpus: int, world: int) -> None:
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
