"""The C++ examples over the C ABI: native callers that link libecm2pa.so through
include/ecm2_pa.h alone.  examples/heat_step.cpp runs ex16's PA heat step (Mass + Diffusion with
a k(T) coefficient, SDIRK33, constrained Jacobi-PCG) on the reference's fichera fixture and
checks its known answers (1^T M 1 = 7, K 1 = 0, a decaying maximum); examples/par_heat.cpp runs
ex16p's parallel form (z-slab partition, loopback group) and checks its Mult and two SDIRK
steps against the serial form."""
import os
import subprocess

import pytest

from helpers import GOLDEN, ROOT

EXAMPLES = os.path.join(ROOT, "examples")
BINARY = os.path.join(EXAMPLES, "heat_step")
PAR_BINARY = os.path.join(EXAMPLES, "par_heat")


def _build():
    subprocess.run(["make", "-s", "-C", EXAMPLES], check=True, timeout=300)
    assert os.access(BINARY, os.X_OK) and os.access(PAR_BINARY, os.X_OK)


def _run(*args, timeout=120):
    return subprocess.run([BINARY, os.path.join(GOLDEN, "fichera.mesh"), *map(str, args)], cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_example_builds_and_fails_loudly_without_gpu():
    """Compiles and links against the header + library; with no device the first compute
    entry point returns ECM2_ERR_HIP and the program stops (no CPU fallback)."""
    _build()
    import ecm2_amd as E
    if E.load_library().ecm2_device_count() > 0:
        pytest.skip("a GPU is visible")
    r = _run(1, 2, 1)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "mesh " in r.stdout and "boundary dofs" in r.stdout  # host setup ran
    assert "no HIP device" in r.stderr
    r = subprocess.run([PAR_BINARY, "2", "4", "1"], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("refine,order", [(1, 1), (2, 2)])
def test_example_heat_step_on_gpu(refine, order):
    if not os.access(BINARY, os.X_OK):
        _build()
    r = _run(refine, order, 5)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.rstrip().endswith("PASS")
    assert r.stdout.count("converged 1") == 5


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("2", "8", "1", "1"), ("4", "12", "2", "1"), ("3", "10", "2", "0")])
def test_example_par_heat_on_gpu(args):
    if not os.access(PAR_BINARY, os.X_OK):
        _build()
    r = subprocess.run([PAR_BINARY, *args], cwd=ROOT, capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.rstrip().endswith("PASS")


@pytest.mark.gpu
@pytest.mark.parametrize("decomp", ["1", "0"])
def test_example_par_heat_rccl_one_rank(decomp):
    """The one-process-per-GPU flow (RCCL id, ecm2_par_form_mult, RCCL-summed PCG dots) with one
    rank on the box's GPU; WORLD_SIZE > 1 needs a node with that many GPUs."""
    if not os.access(PAR_BINARY, os.X_OK):
        _build()
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([PAR_BINARY, "rccl", "8", "2", decomp], cwd=ROOT, capture_output=True, text=True,
                       timeout=120, env=env)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.rstrip().endswith("rank 0 of 1: PASS")
