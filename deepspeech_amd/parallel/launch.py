"""Single-node launcher: N worker processes, one per GPU, without torchrun.

``python bench.py --gpus 8`` (and ``deepspeech_amd.train --gpus 8``) start here when no
launcher has set ``WORLD_SIZE``. The parent never touches the GPU (it does not even import
torch): it only picks a rendezvous port, starts N copies of the same command line as child
processes with the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT), forwards their output, and exits with the first
failing rank's code after stopping the others (exact PIDs, never a pattern). Each child then
initialises RCCL through ``parallel/dist.py`` exactly as under torchrun. No process is ever
replaced (exec) — the parent stays alive until every rank has exited.

The reference has no multi-device launch at all: its tower-mean ``average_gradients``
(src/deepSpeech_train.py:193-228) is dead code (call site commented out at :451-454).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")


def launcher_world() -> Optional[int]:
    """World size set by an outer launcher (torchrun / this module), None if there is none."""
    w = os.environ.get("WORLD_SIZE")
    return int(w) if w not in (None, "") else None


def check_world(requested: Optional[int]) -> int:
    """Resolve the world size of this process against ``--gpus``: under a launcher the two
    must agree (a silent mismatch would report the wrong n_gpus); without one, the request."""
    outer = launcher_world()
    if outer is None:
        return 1 if requested is None else int(requested)
    if requested is not None and int(requested) != outer:
        raise SystemExit("--gpus %d does not match the launcher's WORLD_SIZE=%d" % (requested, outer))
    return outer


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_local(nproc: int, argv: Sequence[str], extra_env: Optional[dict] = None,
                poll_s: float = 0.2) -> int:
    """Run ``argv`` as ``nproc`` ranks on this node; return the job's exit code (0 if every
    rank succeeded, else the first failing rank's code; a rank killed by a signal reports
    128 + signal). A failing rank stops the rest: SIGTERM, then SIGKILL after 10 s."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs: List[subprocess.Popen] = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        # dmabuf IPC only on this platform (RCCL / CUDA-tensor sharing between ranks)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(list(argv), env=env))
    code = 0
    alive = set(range(nproc))
    try:
        while alive:
            for r in sorted(alive):
                rc = procs[r].poll()
                if rc is None:
                    continue
                alive.discard(r)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    sys.stderr.write("[launch] rank %d exited with %d; stopping the other ranks\n" % (r, rc))
                    _stop([procs[k] for k in alive])
            if alive:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        _stop([p for p in procs if p.poll() is None])
        raise
    return code


def _stop(procs: List[subprocess.Popen], grace_s: float = 10.0) -> None:
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    deadline = time.time() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def maybe_spawn(requested: Optional[int], script: str, argv: Sequence[str]) -> Optional[int]:
    """If no launcher is active and ``requested`` > 1, run ``script argv`` as that many ranks
    and return the job's exit code; otherwise return None (this process is a rank: go on)."""
    return maybe_spawn_cmd(requested, [sys.executable, "-u", script] + list(argv))


def maybe_spawn_cmd(requested: Optional[int], cmd: Sequence[str]) -> Optional[int]:
    """maybe_spawn for a whole command line (``python -m deepspeech_amd.train ...``)."""
    if launcher_world() is not None or requested is None or int(requested) <= 1:
        return None
    return spawn_local(int(requested), list(cmd))
