"""bench.py's contract (the driver parses its last line): the JSON keys of a single-GPU line, a
loopback group line and the per-member emulation line, on a small C2 mesh.  The numbers are not
checked here (profiles/ holds the measurements); the shape of the output and its consistency are."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=240):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                         text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_bench_help_lists_the_options():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], cwd=ROOT, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0
    for opt in ("--gpus", "--steps", "--warmup", "--workload", "--schedule", "--loopback", "--member", "--deadline"):
        assert opt in out.stdout


def test_par_launch_label_follows_the_graph_mode(monkeypatch):
    """The N > 1 line names the launch form par_form.cpp's par_graph() picks (CPU, no GPU)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    monkeypatch.delenv("ECM2_PAR_GRAPH", raising=False)
    assert "direct" in b.par_launch_label("serial", -1)
    assert "graph" in b.par_launch_label("overlap", -1)
    assert "graph" in b.par_launch_label("serial", 1) and "direct" in b.par_launch_label("overlap", 0)
    monkeypatch.setenv("ECM2_PAR_GRAPH", "1")
    assert "graph" in b.par_launch_label("serial", -1)
    monkeypatch.setenv("ECM2_PAR_GRAPH", "0")
    assert "direct" in b.par_launch_label("overlap", -1)


SMALL = ["--workload", "c2", "--c2-n", "12", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--full-layout", "0"]


@pytest.mark.gpu
def test_bench_single_gpu_line():
    b = run_bench(*SMALL)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in b, k
    assert b["n_gpus"] == 1 and b["steps"] == 3 and b["warmup"] == 1 and b["value"] > 0
    assert b["dtype"] == "f64" and b["config"]["ndofs"] == (2 * 12 + 1) ** 3
    r = b["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3)
    assert r["traffic"] is None  # a pin belongs to the default size only
    # value = ndofs * steps / time
    assert b["value"] == pytest.approx(b["config"]["ndofs"] / (b["ms_per_step"] * 1e-3) / 1e6, rel=1e-3)
    assert b["config"]["numbering"].startswith("structured") and b["config"]["mesh"] == "affine"
    # the one-GPU line carries the marginal Jacobi-PCG iteration (MDoF*iter/s)
    # (an iteration holds one apply kernel; against ms_per_step it need not be slower at this launch-bound
    # size: the device-driven loop enqueues iterations ahead, the timed Mults are host-issued one by one)
    assert b["pcg_iteration"]["iterations"] == 20
    assert b["pcg_iteration"]["iteration_ms"] > b["roofline"]["kernel_ms_avg"]
    # and one ex16p SDIRK33 step (configs[4]'s unit of work) on the same mesh
    st = b["sdirk_step"]
    assert st["stage_solves"] == 3 and st["converged"] and st["pcg_iterations"] > 3 and st["step_ms"] > st["solves_ms"]
    # the same run's variants: the reference's numbering (same layout: AFFINE with the k(T) snapshot on a
    # brick-tiled mesh), a trilinear mesh (TRILINEAR) and the drop-in configuration (+ MFEM Jacobians)
    assert b["entity_numbering"]["value"] > 0 and b["entity_numbering"]["qdata_layout"] == "affine_ts"
    assert b["trilinear"]["value"] > 0 and b["trilinear"]["qdata_layout"] == "trilinear"
    assert b["drop_in"]["value"] > 0 and b["drop_in"]["qdata_layout"] == "trilinear"
    # the snapshot forms without a per-point stream: the Pennes operator (both laws of one field) and
    # ex16p's M + dt K(u_alpha_gf)
    assert b["pennes"]["snapshot"] == {"on": True, "mass_values": 2, "law_at_point": True}
    assert b["ex16"]["snapshot"] == {"on": True, "mass_values": 2, "law_at_point": False}
    assert b["pennes"]["qdata_layout"] == b["ex16"]["qdata_layout"] == "affine_tsm"
    assert b["pennes"]["roofline"]["traffic"] is None and b["pennes"]["value"] > 0  # (pins: default size only)
    s = run_bench(*SMALL, "--variants", "0", "--coefficient-snapshot", "0")
    assert s["value"] > 0 and "entity_numbering" not in s
    assert b["config"]["qdata_layout"] == "affine_ts" and s["config"]["qdata_layout"] == "affine"
    e = run_bench(*SMALL, "--numbering", "entity", "--variants", "0")
    assert e["config"]["numbering"].startswith("entity") and "entity_numbering" not in e


@pytest.mark.gpu
def test_bench_loopback_group_and_member_lines():
    g = run_bench(*SMALL, "--loopback", "2")
    assert g["value"] > 0 and "loopback" in g["config"]["parallelism"]
    m = run_bench(*SMALL, "--loopback", "2", "--member", "-1")
    assert m["emulated_n_gpus"] == 2 and len(m["member_ms"]) == 2 and m["members"] == [0, 1]
    assert m["slowest_member_ms"] == max(m["member_ms"]) and m["emulated_value"] > 0
    assert m["pcg"] is None
    p = run_bench(*SMALL, "--loopback", "2", "--member", "-1", "--pcg-iters", "5")
    assert len(p["pcg"]["member_iteration_ms"]) == 2 and p["pcg"]["slowest_member_iteration_ms"] > 0
    s = run_bench(*SMALL, "--variants", "0", "--pcg-iters", "5")
    assert s["pcg_iteration"]["iteration_ms"] > s["roofline"]["kernel_ms_avg"]  # (as in the single-GPU line)


def _timed_region_worker(rank, port, out):
    """One rank of bench.py's timed region over gloo: rank 1's Mults take 20 ms each, rank 0's nothing."""
    import importlib.util
    import time
    import types
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    fake = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda: None))
    delay = 0.02 if rank == 1 else 0.0
    dt = b.time_mults(lambda x, y: time.sleep(delay), None, None, 5, 1, 2, dist, fake)
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # as bench.py reduces the ranks' times
    with open(os.path.join(out, f"r{rank}.json"), "w") as f:
        json.dump({"dt": dt, "max": float(t[0])}, f)
    dist.destroy_process_group()


def test_timed_region_is_per_rank_and_maxed(tmp_path):
    """bench.py time_mults: the opening barrier aligns the ranks, a rank's time ends at its own last
    synchronize (the closing barrier brackets the region but is not in it), the line takes the MAX."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_timed_region_worker, args=(port, str(tmp_path)), nprocs=2, join=True)
    r0 = json.load(open(tmp_path / "r0.json"))
    r1 = json.load(open(tmp_path / "r1.json"))
    assert r1["dt"] >= 5 * 0.02 and r0["dt"] < 0.05  # rank 0 does not wait for rank 1 inside its time
    assert r0["max"] == r1["max"] == r1["dt"]
