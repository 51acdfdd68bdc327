"""Per-platform process environment (reference: src/setenvs.py, which pins KMP/OMP/MKL
threads for Intel KNL / Broadwell before the TF session starts).

MI355X equivalents, applied BEFORE torch is imported (the reference applied its settings
after importing TensorFlow, so its OMP values could not take effect — quirk noted in
SURVEY §5.6; the CLI shims deepSpeech_train.py / deepSpeech_test.py call this first):

  mi355x  HSA_ENABLE_IPC_MODE_LEGACY=0   dmabuf IPC for RCCL / cross-process tensors
          HIP_FORCE_DEV_KERNARG=1        kernel arguments in device memory (lower launch
                                         latency for the many small launches of a step)
          TORCH_NCCL_HIGH_PRIORITY=1     RCCL on high-priority streams, so bucketed gradient
                                         all-reduces overlap BPTT instead of queuing behind it
          OMP_NUM_THREADS                host threads for the loader / featurizer (8)
          NCCL_MAX_NCHANNELS=32          RCCL CU footprint (see below)
          GPU_MAX_HW_QUEUES=8            hardware queues per process. A data-parallel step uses
                                         the main stream, the weight-gradient side stream, the
                                         bucket-ordering stream and RCCL's streams: with HIP's
                                         default of 4 queues two of them share one and the
                                         weight-gradient GEMMs serialise behind the BPTT
                                         (measured at world size 1 with the DP machinery forced
                                         on: 10.01-10.08 ms/step at 4 queues, 9.39-9.43 at 8,
                                         9.35-9.45 without DP; profiles/r2_dp_readiness.md)
          DEBUG_HIP_FORCE_GRAPH_QUEUES=1 replay a captured step graph (Trainer step graphs) on
                                         one queue: HIP otherwise spreads a graph's parallel
                                         branches over extra queues joined by barrier packets,
                                         which made a 100-frame step 3.37 ms against 1.78 on
                                         one queue (200 / 400 / 1000 frames: 2.44 / 4.85 / 7.94
                                         against 2.43 / 3.67 / 8.08; profiles/r5_step_graphs.md)

RCCL channel budget. Each RCCL channel is one workgroup that stays resident for the whole
collective. The persistent recurrence needs P*groups co-resident workgroups, one per CU:
200 of the 256 CUs at the headline shape (8 groups x 25), and the weight-gradient GEMMs
use the rest. If a bucket's all-reduce is in flight when a recurrence launches, its
workgroups wait for CUs held by RCCL channels (they never deadlock: the collective does not
depend on the recurrence, and every recurrence spin is bounded, tests/test_dp_gpu.py), so
the channel count is what the recurrence can lose: 256 - 200 = 56 free CUs, minus room for
the side-stream GEMM tiles -> at most 32 channels. 32 channels x ~2 channels per xGMI link
direction still cover the 7 links of the 8-GPU mesh.
  knl/bdw the reference's Intel settings, kept for command-line compatibility.

Existing values in the environment win (setdefault), so a launcher can override — except
GPU_MAX_HW_QUEUES, which is raised to at least 8 (a lower preset value is replaced).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

PLATFORMS: Dict[str, Dict[str, str]] = {
    "mi355x": {
        "HSA_ENABLE_IPC_MODE_LEGACY": "0",
        "HIP_FORCE_DEV_KERNARG": "1",
        "TORCH_NCCL_HIGH_PRIORITY": "1",
        "OMP_NUM_THREADS": "8",
        "NCCL_MAX_NCHANNELS": "32",
        "GPU_MAX_HW_QUEUES": "8",
        "DEBUG_HIP_FORCE_GRAPH_QUEUES": "1",
    },
    "bdw": {
        "KMP_BLOCKTIME": "1", "KMP_SETTINGS": "1", "OMP_NUM_THREADS": "8", "MKL_NUM_THREADS": "8",
        "OMP_DYNAMIC": "false", "KMP_AFFINITY": "granularity=fine,verbose,compact,1,0",
    },
    "knl": {
        "KMP_BLOCKTIME": "0", "KMP_SETTINGS": "1", "OMP_NUM_THREADS": "8", "MKL_NUM_THREADS": "8",
        "OMP_DYNAMIC": "false", "KMP_AFFINITY": "granularity=fine,verbose,explicit,proclist=[4-67]",
    },
}


def platform_from_argv(argv: List[str], default: str = "mi355x") -> str:
    for i, a in enumerate(argv[:-1]):
        if a == "--platform":
            return argv[i + 1]
        if a.startswith("--platform="):
            return a.split("=", 1)[1]
    return default


def setenvs(argv: Optional[List[str]] = None, platform: Optional[str] = None) -> Dict[str, str]:
    """Apply the platform's environment (existing variables are kept). Returns what was set."""
    import sys
    plat = platform or platform_from_argv(list(argv if argv is not None else sys.argv))
    if plat not in PLATFORMS:
        raise ValueError("unknown platform %r (expected one of %s)" % (plat, sorted(PLATFORMS)))
    applied = {}
    for k, v in PLATFORMS[plat].items():
        if k in _AT_LEAST and k in os.environ:
            # a floor, not a default: machines export HIP's own default of 4 queues, which
            # is exactly what a DP step must not run with (see GPU_MAX_HW_QUEUES above).
            # DS2_KEEP_HW_QUEUES=1 keeps an exported value as it is (A/B of the queue count,
            # scripts/ab_queues.sh)
            if os.environ.get("DS2_KEEP_HW_QUEUES") == "1":
                continue
            try:
                if int(os.environ[k]) >= int(v):
                    continue
            except ValueError:
                pass
            os.environ[k] = v
            applied[k] = v
        elif k not in os.environ:
            os.environ[k] = v
            applied[k] = v
    return applied


_AT_LEAST = ("GPU_MAX_HW_QUEUES",)
