"""Environment for several processes sharing one GPU (rehearsals, same-GPU tests).

HIP gives every process GPU_MAX_HW_QUEUES hardware queues (4 by default).  Once the processes
on one GPU hold more queues than the GPU can keep mapped, the scheduler time-slices them: the
4-rank same-GPU MLP rehearsal ran at 16.9 M samples/s with 4 queues per process and at 452 M
with 2 (profiles/r06_ranks), and a 4-rank ResNet-18 step took ~45 s instead of ~0.03 s.  One
process per GPU, the deployment shape, is unaffected.

Not used for the elastic workers (scripts/elastic_demo.py). With 2 queues each, a surviving
worker stopped answering CheckUp while its update kernel spun for the dead peer until the
exchange's 10 s timeout, and the master evicted that healthy worker (r06_full5). The same
silence later came back with HIP's 4 queues (r06_full7). Its cause was a step graph destroyed
while a replay was still in flight: the destructor waits with the GIL held. Trainers now retire
replaced graphs and free them only after a sync (utils/graphs.py).
"""
from __future__ import annotations

QUEUE_BUDGET = 8  # hardware queues in total across the processes sharing a GPU


def share_gpu_env(env: dict, procs_per_gpu: int) -> dict:
    """Cap GPU_MAX_HW_QUEUES in ``env`` (in place, returned) for ``procs_per_gpu`` processes on
    one GPU: at most QUEUE_BUDGET in total, never above the value already set.  Two or fewer
    processes keep HIP's default."""
    if procs_per_gpu > 2:
        cap = max(1, QUEUE_BUDGET // procs_per_gpu)
        if int(env.get("GPU_MAX_HW_QUEUES") or 4) > cap:
            env["GPU_MAX_HW_QUEUES"] = str(cap)
    return env
