"""bench.py's RCCL rank branch (the code the driver's multi-GPU SCALE run executes) run end to end on
one GPU: torch.distributed.run with one process, the nccl (RCCL) process group, the RCCL unique id
broadcast, a one-part z-slab Partition, ParBilinearForm over a one-rank communicator, the timed
Mults with their barriers and the cross-rank reductions of the results."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("workload", ["c2", "c4"])
def test_bench_rank_branch_one_rank(workload):
    args = ["--gpus", "1", "--rank-path", "1", "--workload", workload, "--steps", "5", "--warmup", "2",
            "--no-cpu-baseline", "--deadline", "240"]
    if workload == "c2":
        args += ["--c2-n", "24"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["ms_per_step"] > 0
    assert "RCCL" in line["config"]["parallelism"], line["config"]["parallelism"]
    assert line["roofline"]["kernel_ms_avg"] > 0
    # the stages the rank branch passes through, in order (bench.py's watchdog log)
    log = r.stderr
    stages = ["init_process_group", "assemble", "kernel timing", "timed Mults", "reduce results", "teardown"]
    pos = [log.find(s) for s in stages]
    assert all(p >= 0 for p in pos) and pos == sorted(pos), log[-2000:]
