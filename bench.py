#!/usr/bin/env python3
"""bench.py -- MDoF/s of the PA diffusion+mass Mult (hex, H1 p=2) on MI355X.

Metric (BASELINE.json): "MDoF/s on PA diffusion+mass Mult, hex p=2; % HBM roofline at
1/2/4/8 GPUs".  One *step* = one operator Mult y = A x (L-vector in, L-vector out;
tests/benchmarks/bench_assembly_levels.cpp:281-286 counts ndofs per Mult) with x, y and the
operator resident in HBM.

Workload (default): BASELINE configs[3], the north-star configuration -- Cartesian 108^3,
H1 p = 2, 10,218,313 DoF, z-slab partitioned over the ranks with the shared-DoF exchange over
RCCL (one rank per GPU; strong scaling).  --workload c2 runs configs[1] (Cartesian 50^3 per
GPU, weak scaling), c3 configs[2] (fichera refined, + PCG), c5 configs[4] (68^3, p = 4).

Coefficients are the bioheat ones: alpha = rho*c_eff(x) (FunctionCoefficient projected at the
quadrature points) and beta = gamma*dt*k(T) with T an H1 grid function (the Pennes law,
evaluated on the device at Assemble).  Inputs are synthetic (no data files).

Roofline fields: `achieved` / `frac` = HBM bytes the dominant kernel actually
moves per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE pin of this workload and layout, with its
provenance) / its HIP-event time / 8 TB/s -- or, without a pin, the formulation's minimum
bytes (stored qdata + x + y + map) as a lower bound; `alg_ratio` = SURVEY §8(d)'s fixed
algorithmic bytes (56 B per quadrature point) / the same time / 8 TB/s, which exceeds 1
when the compressed (AFFINE) layout stores less than the formula counts.

Beside the timed Mults (outside the timed region), the one-GPU line also carries the same
run's variants (the reference's numbering, a trilinear mesh, the drop-in configuration, the full
per-point layout, the Pennes and ex16p coefficient paths), the marginal Jacobi-PCG iteration
(`pcg_iteration`, the device-driven loop) and one ex16p SDIRK33 step (`sdirk_step`), and the CPU
oracle baseline.
"""
import argparse
import importlib.util
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
PEAK_FP64_TFLOPS = 78.6  # MI355X FP64 vector (and matrix) peak, dense


def alg_flops(order, ne):
    """SURVEY §8(d)'s algorithmic flops of one Mult (2 x the sum-factorised MACs per element:
    diffusion 2D^3Q + 3D^2Q^2 + 3Q^3D + 9Q^3 + 3Q^3D + 3Q^2D^2 + 3D^3Q, mass 2(D^3Q + D^2Q^2 + DQ^3)
    + Q^3); C4: 10.29 GF, C5: 14.62 GF."""
    D, Q = order + 1, order + 2
    dif = 2 * D**3 * Q + 3 * D**2 * Q**2 + 3 * Q**3 * D + 9 * Q**3 + 3 * Q**3 * D + 3 * Q**2 * D**2 + 3 * D**3 * Q
    mas = 2 * (D**3 * Q + D**2 * Q**2 + D * Q**3) + Q**3
    return 2.0 * (dif + mas) * ne
METRIC = "MDoF/s on PA diffusion+mass Mult, hex p=2; % HBM roofline at 1/2/4/8 GPUs"


def load_pkg():
    if "ecm2_amd" in sys.modules:
        return sys.modules["ecm2_amd"]
    pkg_dir = os.path.join(ROOT, "cardiac-ablation-ecm2_amd")
    spec = importlib.util.spec_from_file_location("ecm2_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ecm2_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


class Deadline:
    """Per-rank watchdog: if the run is not done after `seconds`, print this rank's last stage
    and exit non-zero (no re-exec, no retry)."""

    def __init__(self, seconds, rank):
        self.rank, self.stage, self.t0 = rank, "start", time.time()
        self._done = threading.Event()
        if seconds > 0:
            threading.Thread(target=self._watch, args=(seconds,), daemon=True).start()

    def at(self, stage):
        self.stage = stage
        print(f"[bench rank {self.rank}] {time.time() - self.t0:7.1f}s {stage}", file=sys.stderr, flush=True)

    def done(self):
        self._done.set()

    def _watch(self, seconds):
        if not self._done.wait(seconds):
            print(f"bench.py rank {self.rank}: deadline of {seconds:.0f}s exceeded; last stage: {self.stage}",
                  file=sys.stderr, flush=True)
            os._exit(3)


def alpha_fn(P):
    return 3.6e6 * (1.0 + 0.1 * np.sin(3.0 * P[..., 0]))


def temperature_fn(X):
    return 37.0 + 20.0 * np.exp(-10.0 * np.sum(X * X, axis=-1))


K_SCALE, K_SLOPE, K_TREF = 0.5 * 0.05, 0.0012, 37.0  # gamma*dt*k0, dk/dT / k0, T0


def bioheat_coefficients(E, torch, mesh, fes, part=None):
    """alpha = rho*c_eff(x) at quadrature points (FunctionCoefficient projection) and the
    temperature grid function T (L-vector) for beta = gamma*dt*k(T)."""
    q1d = fes.order + 2
    X = fes.dof_coords()
    T = temperature_fn(X)
    if part is None:
        P = mesh.quadrature_points(q1d)
        alpha = alpha_fn(P).reshape(fes.ne, -1)
    else:
        P = E.quadrature_points_subset(mesh, q1d, part.elems)
        alpha = alpha_fn(P).reshape(part.ne_local, -1)
        T = T[part.local_to_global]
    return torch.as_tensor(alpha).cuda(), torch.as_tensor(T).cuda()


def bench_integrators(E):
    """The timed form's integrators: MassIntegrator(QuadratureCoefficient(alpha)) (the projected
    FunctionCoefficient rho*c_eff(x)) and DiffusionIntegrator(AffineGridFunctionCoefficient(T, ...))
    (gamma*dt*k(T) of the H1 temperature field)."""
    mass = lambda a: E.MassIntegrator(E.QuadratureCoefficient(a))
    diff = lambda T: E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, K_SCALE, K_SLOPE, K_TREF))
    return mass, diff


def bench_form(E, torch, mesh, fes, keep, kernel=0, scatter="partials", compress_geometry=True,
               element_order="auto", geometry_input="nodes", coefficient_snapshot=True):
    """The serial form every bench line times (and tests/test_gpu_timed_forms.py pins against the
    oracle at the timed size): Mass(rho*c_eff(x)) + Diffusion(gamma*dt*k(T)) on `fes`, assembled.
    element_order "faces": the reference's numbering, the form derives its order from the map alone.
    geometry_input "jacobians": MFEM's GeometricFactors::JACOBIANS array, as the binding passes it.
    The coefficient tensors are appended to `keep` (they must outlive the form's Assemble)."""
    a, T = bioheat_coefficients(E, torch, mesh, fes)
    keep.extend([a, T])
    mass, diff = bench_integrators(E)
    f = E.BilinearForm(fes, kernel=kernel, element_order=os.environ.get("ECM2_ELEMENT_ORDER", element_order),
                       scatter=scatter, compress_geometry=compress_geometry,
                       bricks=int(os.environ.get("ECM2_BRICKS", "-1")),  # A/B: p >= 3 brick depth
                       geometry="jacobians" if geometry_input == "jacobians" else "nodes",
                       coefficient_snapshot=coefficient_snapshot)
    if geometry_input == "jacobians":
        # MFEM's GeometricFactors::JACOBIANS (NQ x 3 x 3 x NE), as the binding passes it; the form
        # fits it to trilinear maps (or checks it affine) at Assemble and keeps it for re-assembly
        f.SetJacobians(mesh.jacobians(fes.order + 2))
    f.AddDomainIntegrator(mass(a))
    f.AddDomainIntegrator(diff(T))
    f.Assemble()
    return f


PERFUSION = (3.6e6, 0.05 * 3.6e3, 6.4e-3, 0.02, 37.0, 50.0)  # rho_c, gamma dt c_b, w0, a, T0, T_stop


def bench_law_form(E, torch, mesh, fes, keep, case):
    """The coefficient-snapshot forms whose mass is not a quadrature coefficient (bench sub-objects):
    pennes -- Mass(rho c + gamma dt c_b w_b(T)) + Diffusion(gamma dt k(T)) of one H1 temperature field
    (the Pennes perfusion law with coagulation shut-off at T_stop, evaluated at the point); ex16 --
    ex16p's implicit operator M + dt K(u_alpha_gf), u_alpha_gf = kappa + alpha u formed at the dofs and
    passed as a GridFunctionCoefficient (examples/ex16p.cpp:450-466), the mass coefficient 1."""
    T = torch.as_tensor(temperature_fn(fes.dof_coords())).cuda()
    f = E.BilinearForm(fes)
    if case == "pennes":
        keep.append(T)
        f.AddDomainIntegrator(E.MassIntegrator(E.PerfusionCoefficient(T, *PERFUSION)))
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, K_SCALE, K_SLOPE, K_TREF)))
    else:
        ua = 0.05 * (0.5 + 0.01 * T)  # dt (kappa + alpha u)
        keep.append(ua)
        f.AddDomainIntegrator(E.MassIntegrator(E.ConstantCoefficient(1.0)))
        f.AddDomainIntegrator(E.DiffusionIntegrator(E.GridFunctionCoefficient(ua)))
    f.Assemble()
    return f


def qdata_layout(E, form):
    """Quadrature-data layout of a (local) form: affine | affine_ts (AFFINE with the k(T)
    coefficient snapshot; affine_tsm: and the mass per element) | affine_e | affine_e_ts(m) (the p >= 3
    bricks' snapshot) | trilinear | trilinear_e | blocked | native."""
    lay = {E.QLAYOUT_NATIVE: "native", E.QLAYOUT_BLOCKED: "blocked", E.QLAYOUT_AFFINE: "affine",
           E.QLAYOUT_AFFINE_E: "affine_e", E.QLAYOUT_TRILINEAR: "trilinear",
           E.QLAYOUT_TRILINEAR_E: "trilinear_e"}[form.info()["layout"]]
    if lay in ("affine", "affine_e") and hasattr(form, "CoefficientSnapshot") and form.CoefficientSnapshot():
        lay += "_ts"
        if hasattr(form, "SnapshotInfo") and form.SnapshotInfo()[1] == 2:
            lay += "m"  # the mass stored per element: no per-point stream
    return lay


def min_bytes(form, ne, nd, n_true):
    """The formulation's minimum HBM bytes per Mult: its stored qdata read once, x read and y
    written once, one int32 map entry per element dof."""
    return form.qdata_bytes() + 16.0 * n_true + 4.0 * ne * nd


def time_mults(apply, x, y, steps, warmup, world, dist, torch):
    for _ in range(warmup):
        apply(x, y)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        apply(x, y)
    torch.cuda.synchronize()
    # this rank's K steps end at its own synchronize; the closing barrier still brackets the region
    # (no rank leaves before every rank's steps are done), but its own latency -- an RCCL all-reduce
    # and a synchronize, tens of microseconds at 8 ranks against a ~1.3 ms region of 20 C4 Mults --
    # is not a Mult's.  The caller takes the MAX of these per-rank times over the ranks.
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    return t1 - t0


def kernel_ms(forms, apply, x, y, steps, torch, settle_s=0.06, world=1, dist=None):
    """HIP events around the dominant (fused apply) kernel(s) of each Mult, on the stream they
    are launched on (a pass of its own, outside the timed loop); ms per Mult.  It runs right
    before the timed loop and first keeps the GPU busy for `settle_s` of untimed Mults: after
    any idle of a few ms the first ~50 Mults run up to 17-30% slower while the power
    management settles (profiles/r2_ramp_c4.json, r2_ramp_c5.json), so both this pass and the
    timed steps that follow it see the sustained rate of a PCG loop."""
    # the settle count is rank 0's and identical on every rank: a distributed Mult is collective
    for _ in range(4):
        apply(x, y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        apply(x, y)
    torch.cuda.synchronize()
    n = max(1, min(5000, int(settle_s / max((time.perf_counter() - t0) / 8, 1e-6))))
    if dist is not None:
        t = torch.tensor([n], dtype=torch.int64, device="cuda")
        dist.broadcast(t, 0)
        n = int(t.item())
    for i in range(n):
        apply(x, y)
        if i % 64 == 63:
            torch.cuda.synchronize()  # bounded host run-ahead; no idle long enough to matter
    for f in forms:
        f.timing(True)
    for _ in range(steps):
        apply(x, y)
    torch.cuda.synchronize()
    kms = sum(f.timing_get()[0] for f in forms)
    for f in forms:
        f.timing(False)
    return kms / steps


PART_NAME = {"slabs": "z-slabs", "boxes": "boxes", "bricks": "brick runs"}


def member_bench(args, E, torch, group, xs, ys, ndofs, workload, dl):
    """--loopback N --member R: member R's rows of the partitioned operator alone, captured in
    one HIP graph and replayed -- the stages, streams and kernels one RCCL rank runs on its own
    GPU (interior elements beside the exchange + boundary elements, then the shared-dof sums),
    with the exchange as device-local copies instead of xGMI transfers.  The slowest member's
    time gives the emulated N-GPU rate (ndofs / that time); every member's time is printed."""
    n = len(group.forms)
    members = list(range(n)) if args.member < 0 else [args.member]
    group.Mult(xs, ys)  # RAP: every member's ghost contributions, which a member's P^T receive copies
    torch.cuda.synchronize()
    use_graph = args.member_graph if args.member_graph >= 0 else (
        args.par_graph if args.par_graph >= 0 else int(args.schedule == "overlap"))
    runs, graphs = {}, []
    for r in members:
        for _ in range(3):
            group.MultMember(r, xs, ys)
        torch.cuda.synchronize()
        if use_graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=torch.cuda.Stream()):
                group.MultMember(r, xs, ys)
            graphs.append(g)
            runs[r] = g.replay
        else:
            runs[r] = (lambda rr: (lambda: group.MultMember(rr, xs, ys)))(r)
    # members interleaved over several passes, each member's time the median of its passes: one
    # member timed once carries +-10% run-to-run noise, and the slowest of eight picks it up
    # (profiles/r3_member_emul.txt)
    passes = 3 if len(members) > 1 else 1
    samples = {r: [] for r in members}
    for p in range(passes):
        for r in members:
            dl.at(f"member {r} pass {p}")
            run = runs[r]
            t0 = time.perf_counter()
            k = 0
            while time.perf_counter() - t0 < 0.06:  # settle the clock (kernel_ms)
                run()
                k += 1
                if k % 64 == 0:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(args.steps):
                run()
            ev1.record()
            torch.cuda.synchronize()
            samples[r].append(ev0.elapsed_time(ev1) / args.steps)
    per = [sorted(samples[r])[len(samples[r]) // 2] for r in members]
    del runs, graphs
    worst = max(per)
    pcg = None
    if args.pcg_iters:
        # one rank's solver iteration: its Mult, its vector passes on its true dofs, two dots
        # through a real (one-rank) RCCL all-reduce and the per-iteration read-back
        it_ms = {r: [] for r in members}
        for p in range(passes):
            for r in members:
                dl.at(f"member {r} pcg pass {p}")
                it_ms[r].append(pcg_iteration_ms(torch, E.Operator(group, member=r),
                                                 group.forms[r].true_size, args.pcg_iters))
        pm = [sorted(it_ms[r])[len(it_ms[r]) // 2] for r in members]
        pcg = {"iterations": args.pcg_iters, "member_iteration_ms": [round(v, 5) for v in pm],
               "slowest_member_iteration_ms": round(max(pm), 5),
               "note": "marginal time per Jacobi-PCG iteration of each member as one rank's operator "
                       "(ecm2_operator_from_par_member: the member's Mult, its vector passes, both dots through "
                       "ncclAllReduce on a one-rank communicator, the device-driven loop); a real N-rank "
                       "all-reduce over xGMI adds its hops on top"}
    print(json.dumps({"emulated_n_gpus": n, "workload": workload, "ndofs": ndofs,
                      "member_ms": [round(v, 5) for v in per], "members": members,
                      "member_passes_ms": [[round(v, 5) for v in samples[r]] for r in members],
                      "slowest_member_ms": round(worst, 5),
                      "partition": PART_NAME[args.partition],
                      "decomposition": group.forms[0].part.decomposition,
                      "coefficient_snapshot": [bool(f.CoefficientSnapshot()) for f in group.forms],
                      "emulated_value": round(ndofs / (worst * 1e-3) / 1e6, 2), "unit": "MDoF/s",
                      "pcg": pcg,
                      "note": f"one member's Mult alone on one GPU, exchange by device copies: a rank's Mult short "
                              f"of the xGMI transfer time; members interleaved over {passes} passes, the median "
                              "pass per member"}), flush=True)


def sdirk_step(E, torch, mesh, fes, keep, ode_type=23, dt=0.01):
    """configs[4]'s unit of work: one implicit step of ex16p's ConductionOperator (examples/ex16p.cpp:
    373-470, SDIRK33 ode.cpp:834-859) -- SetParameters(u) re-assembles T = M + c dt K(u) and K(u)
    (K = DiffusionIntegrator(k(T)) through the snapshot kernel, M = MassIntegrator(rho c_eff(x) /
    3.6e6: ex16's unit capacity)), then the three stage solves (constrained Jacobi-PCG, rel_tol 1e-8 as
    ex16p, Dirichlet on the boundary).  One untimed step first; the timed step starts from its result."""
    a, T = bioheat_coefficients(E, torch, mesh, fes)
    a = a / 3.6e6
    keep.extend([a, T])
    c = E.ode_implicit_coeff(ode_type)
    Tf, Kf = E.BilinearForm(fes), E.BilinearForm(fes)
    Tf.AddDomainIntegrator(E.MassIntegrator(E.QuadratureCoefficient(a)))
    Tf.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, 0.5 * c * dt, K_SLOPE, K_TREF)))
    Kf.AddDomainIntegrator(E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, 0.5, K_SLOPE, K_TREF)))
    ess = torch.as_tensor(fes.boundary_dofs()).cuda()
    u = T.clone()
    out = {}
    for timed in (False, True):
        T.copy_(u)  # SetParameters(u): the coefficient field is the current state
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Tf.Assemble()
        Kf.Assemble()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ns, it, conv = E.ode_step(ode_type, E.Operator(Tf), E.Operator(Kf), dt, u, ess=ess, rel_tol=1e-8, max_iter=500)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if timed:
            out = {"ode": "SDIRK33", "dt": dt, "step_ms": round((t2 - t0) * 1e3, 3),
                   "reassembly_ms": round((t1 - t0) * 1e3, 3), "solves_ms": round((t2 - t1) * 1e3, 3),
                   "stage_solves": ns, "pcg_iterations": it, "converged": conv,
                   "ms_per_iteration": round((t2 - t1) * 1e3 / max(it, 1), 4),
                   "note": "ex16p's step: SetParameters (re-Assemble T = M + c dt K(u) and K(u)) + three constrained "
                           "Jacobi-PCG stage solves (rel_tol 1e-8, boundary dofs held); wall time"}
    return out


def pcg_iteration_ms(torch, op, n, iters):
    """Marginal wall time per Jacobi-PCG iteration of `op` (an Operator, or a BilinearForm's own
    PCG): (t(2K) - t(K)) / K for solves of K and 2K iterations (no essential dofs, rel_tol 1e-30 so
    every iteration runs), after one untimed solve -- the per-solve setup (the Jacobi diagonal, the
    first residual and its read-backs) cancels."""
    b = torch.empty(n, dtype=torch.float64, device="cuda")
    b.uniform_(-1.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(3))
    x = torch.empty_like(b)
    op.PCG(b, x, rel_tol=1e-30, max_iter=iters, jacobi=True)
    torch.cuda.synchronize()
    t = []
    for k in (iters, 2 * iters):
        t0 = time.perf_counter()
        it, _ = op.PCG(b, x, rel_tol=1e-30, max_iter=k, jacobi=True)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
        assert it == k, (it, k)
    return (t[1] - t[0]) / iters


def pmc_pin(workload, world, layout):
    """Pinned PMC traffic of this workload's dominant kernel in this layout (profiles/pmc_pin.py)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}_n{world}_{layout}.json")
    if not os.path.exists(path):
        return None, None
    try:
        pin = json.load(open(path))
    except Exception:
        return None, None
    prov = {k: pin.get(k) for k in ("kernel", "commit", "date", "source", "correction")}
    prov["file"] = os.path.relpath(path, ROOT)
    return pin.get("hbm_bytes_per_launch"), prov


def roofline(workload, world, layout, kms, alg_bytes, mbytes, stream, use_pin=True, flops=None):
    # a pin holds the traffic of one configuration (the workload's default size, one kernel per
    # GPU): anything else reports the formulation's minimum bytes instead
    traffic, prov = pmc_pin(workload, world, layout) if use_pin else (None, None)
    moved = traffic if traffic else mbytes
    achieved = moved / (kms * 1e-3) / 1e9
    return {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": PEAK_HBM_GBS,
        "unit": "GB/s",
        "frac": round(achieved / PEAK_HBM_GBS, 4),
        "traffic": traffic,
        "achieved_basis": ("PMC bytes moved per launch (pin)" if traffic else
                           "formulation minimum bytes per launch (no PMC pin: a lower bound of the bytes moved)"),
        "traffic_provenance": prov,
        "kernel_ms_avg": round(kms, 5),
        "algorithmic_bytes_per_launch": alg_bytes,
        "alg_ratio": round(alg_bytes / (kms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "min_bytes_per_launch": mbytes,
        "stream_copy_gbs": stream[0] if stream else None,
        "stream_read_gbs": stream[1] if stream else None,
        "frac_of_stream": round(achieved / max(stream), 4) if stream else None,
        # the second roof: SURVEY §8(d)'s algorithmic FP64 flops per launch over the same time (the
        # compressed layouts and the coefficient snapshot leave kernels between the two roofs)
        "fp64": ({"achieved": round(flops / (kms * 1e-3) / 1e12, 2), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                  "frac": round(flops / (kms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, 4),
                  "algorithmic_flops_per_launch": flops} if flops else None),
    }


def par_launch_label(schedule, par_graph):
    """The distributed Mult's launch form as par_form.cpp's par_graph() resolves it: --par-graph,
    else ECM2_PAR_GRAPH, else the schedule's default (serial: direct launches, overlap: graph)."""
    env = os.environ.get("ECM2_PAR_GRAPH")
    graph = par_graph == 1 if par_graph >= 0 else (env != "0" if env is not None else schedule != "serial")
    return (f"{schedule} schedule, "
            + ("hip-graph replay per Mult (RCCL exchange captured)" if graph else "direct stream launches per Mult"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c4")
    ap.add_argument("--c2-n", type=int, default=50,
                    help="c2: elements per edge of the per-GPU Cartesian block (configs[1] = 50)")
    ap.add_argument("--c3-refine", type=int, default=6,
                    help="c3: uniform refinements of fichera.mesh (6 -> 14.9M DoF, 5 -> 1.88M)")
    ap.add_argument("--kernel", choices=["auto", "tpe", "wpe", "unfused", "line"], default="auto")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--geometry", choices=["compressed", "full"], default="compressed",
                    help="compressed: AFFINE qdata on parallelepiped meshes (default); full: per-point layout")
    ap.add_argument("--coefficient-snapshot", type=int, default=1, choices=[0, 1],
                    help="1: k(T) evaluated in the kernel from a snapshot of T (p = 2 AFFINE lattice forms, "
                         "ecm2_pa_form_set_coefficient_snapshot); 0: W beta stored per point")
    ap.add_argument("--full-layout", type=int, default=1,
                    help="1 (N = 1): also time the full per-point qdata layout in this run (full_layout sub-object)")
    ap.add_argument("--variants", type=int, default=1, choices=[0, 1, 2],
                    help="1 (N = 1, c2/c4/c5): also time, in this run, the reference's own numbering "
                         "(entity_numbering sub-object), a trilinear mesh (trilinear), the drop-in configuration "
                         "(drop_in) and the snapshot forms without a per-point stream (pennes, ex16); 2: the "
                         "last two only")
    ap.add_argument("--numbering", choices=["structured", "entity"], default="structured",
                    help="c2/c4/c5 main line: lattice dof numbering on a lexicographic mesh (structured) or the "
                         "reference's own (entity: MakeCartesian3D's space-filling-curve element order, "
                         "FiniteElementSpace vertex/edge/face/interior numbering, element order derived by the form)")
    ap.add_argument("--mesh", choices=["affine", "trilinear"], default="affine",
                    help="c2/c4/c5 main line: the Cartesian mesh (affine) or its interior vertices moved (trilinear)")
    ap.add_argument("--geometry-input", choices=["nodes", "jacobians"], default="nodes",
                    help="c2/c4/c5 main line: geometry given as element corners (nodes) or as MFEM's "
                         "GeometricFactors::JACOBIANS array (what the reference-side binding passes)")
    ap.add_argument("--coefficients", choices=["bioheat", "pennes", "ex16"], default="bioheat",
                    help="serial main line's coefficients: bioheat (rho c_eff(x) projected + gamma dt k(T), the "
                         "headline), pennes or ex16 (the snapshot forms of the pennes / ex16 sub-objects)")
    ap.add_argument("--loopback", type=int, default=1,
                    help="N>1 on one GPU: N subdomains in this process (validation of the partitioned path)")
    ap.add_argument("--partition", choices=["slabs", "boxes", "bricks"], default="slabs",
                    help="N > 1: z-slabs (CartesianPartitioning along z), px x py x pz boxes (2x2x2 at N = 8) "
                         "or equal runs of whole 4x4x4 bricks (partition_bricks: balanced to one brick)")
    ap.add_argument("--member", type=int, default=None,
                    help="with --loopback N (z-slabs, OVERLAP): time member R's rows alone, as one rank runs "
                         "them on its own GPU (HIP graph); -1 = every member, the slowest sets the emulated rate")
    ap.add_argument("--schedule", choices=["serial", "overlap"], default="serial",
                    help="distributed Mult schedule (ecm2_par_form_set_schedule)")
    ap.add_argument("--par-graph", type=int, default=-1, choices=[-1, 0, 1],
                    help="distributed Mult: 1 HIP graph per Mult, 0 direct launches, -1 the schedule's default")
    ap.add_argument("--member-graph", type=int, default=-1, choices=[-1, 0, 1],
                    help="--member: 1 replay one HIP graph per Mult, 0 launch the stages directly, "
                         "-1 as the RCCL form would (--par-graph, else the schedule's default)")
    ap.add_argument("--pcg-iters", type=int, default=-1,
                    help="also time K Jacobi-PCG iterations (no ess, rel_tol 1e-30): on one GPU the serial "
                         "form's solver; with --member the member as one rank's operator (its dots through "
                         "a one-rank RCCL all-reduce, ecm2_operator_from_par_member).  Default: 20 on the "
                         "one-GPU line, 0 otherwise")
    ap.add_argument("--sdirk", type=int, default=1, choices=[0, 1],
                    help="one-GPU line: also time one ex16p SDIRK33 step on this workload's mesh (sdirk_step)")
    ap.add_argument("--rank-path", type=int, default=0, choices=[0, 1],
                    help="1 with --gpus 1 (under torch.distributed.run): take the RCCL rank branch the N > 1 run "
                         "takes -- process group, RCCL unique id broadcast, one-part z-slab Partition, "
                         "ParBilinearForm over a one-rank communicator, cross-rank reductions -- so a one-GPU "
                         "test executes that code before a multi-GPU run does")
    ap.add_argument("--deadline", type=float, default=900.0,
                    help="seconds after which a rank prints its last stage and exits non-zero (0: none)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.pcg_iters < 0:
        args.pcg_iters = 20 if (world == 1 and args.loopback <= 1 and args.workload != "c3") else 0
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dl = Deadline(args.deadline, rank)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dl.at("import torch")
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    par = world > 1 or args.rank_path == 1  # the RCCL rank branch (one process per GPU)
    if par:
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dl.at("init_process_group")
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local_rank % max(1, torch.cuda.device_count())))
    E = load_pkg()
    E.load_library()
    scatter = os.environ.get("ECM2_SCATTER", "partials")  # A/B: partials | atomic
    kernel = {"auto": E.KERNEL_AUTO, "tpe": E.KERNEL_TPE, "wpe": E.KERNEL_WPE, "unfused": E.KERNEL_UNFUSED,
              "line": E.KERNEL_LINE}[args.kernel]
    decomp = os.environ.get("ECM2_DECOMP", "overlap")

    compress = args.geometry == "compressed"
    order = 4 if args.workload == "c5" else 2
    if args.workload == "c2":
        n = args.c2_n
        nx = ny = n
        nz_total = n * world
        scaling = "weak"
        workload = (f"configs[1]: inline-hex refined to Cartesian {n}x{n}x{nz_total} ({n}^3 per GPU), H1 p=2, "
                    "Mass(rho*c)+Diffusion(gamma*dt*k(T)) PA Mult")
    elif args.workload == "c3":
        scaling = "strong"
        workload = (f"configs[2]: fichera.mesh refined {args.c3_refine}x, H1 p=2, nonlinear Pennes k(T) "
                    "re-assembled on the device, Jacobi-PCG")
    elif args.workload == "c4":
        nx = ny = nz_total = 108
        scaling = "strong"
        workload = ("configs[3]: Cartesian 108^3 (10.2M DoF) z-slab split over the GPUs, H1 p=2, "
                    "Mass(rho*c)+Diffusion(gamma*dt*k(T)) PA Mult")
    else:
        nx = ny = nz_total = 68
        scaling = "strong"
        workload = "configs[4]: Cartesian 68^3 (20.3M DoF) z-slab split over the GPUs, H1 p=4, Mass+Diffusion PA Mult"
    dl.at("mesh and space")
    if args.workload == "c3":
        if world > 1 or args.loopback > 1:
            raise SystemExit("c3 is the single-GPU PCG configuration")
        mesh = E.Mesh(os.path.join(ROOT, "tests", "golden", "fichera.mesh"))
        for _ in range(args.c3_refine):
            mesh.UniformRefinement()
        fes = E.H1Space(mesh, order)
    else:
        mesh, fes = cartesian_space(E, nx, ny, nz_total, order, args.numbering, args.mesh)
    variant = variant_key(args)
    nsub = world if par else args.loopback
    mass, diff = bench_integrators(E)
    form = None
    keep = []

    def serial_form(compress_geometry, mesh=mesh, fes=fes, numbering=args.numbering, geo=args.geometry_input):
        if args.coefficients != "bioheat":
            keep.extend(list(bioheat_coefficients(E, torch, mesh, fes)))  # (the CPU baseline's operator)
            return bench_law_form(E, torch, mesh, fes, keep, args.coefficients)
        return bench_form(E, torch, mesh, fes, keep, kernel=kernel, scatter=scatter,
                          compress_geometry=compress_geometry,
                          element_order="faces" if numbering == "entity" and args.workload != "c3" else "auto",
                          geometry_input=geo, coefficient_snapshot=bool(args.coefficient_snapshot))

    def sub_measure(f, fes_s, tag, note, use_pin=True):
        """Time another serial form of this workload in this run (same steps, same clock
        settling): value, step and kernel time, roofline (the pin of its own variant)."""
        xs = torch.empty(fes_s.ndofs, dtype=torch.float64, device="cuda")
        xs.uniform_(-1.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(1))
        ys = torch.empty_like(xs)
        kf = kernel_ms([f], f.Mult, xs, ys, args.steps, torch)
        dtf = time_mults(f.Mult, xs, ys, args.steps, args.warmup, 1, None, torch)
        lay = qdata_layout(E, f)
        lat, units, runs = f.AddressingInfo()
        lslot, xruns = f.PlanInfo()
        nsh, nslots = f.ScatterInfo()
        return {"qdata_layout": lay,
                "plan": {"lattice_slot_units": lslot, "explicit_dof_runs": xruns, "shared_dofs": nsh,
                         "partial_slots": nslots},
                "value": round(fes_s.ndofs * args.steps / dtf / 1e6, 2),
                "ms_per_step": round(dtf / args.steps * 1e3, 5),
                "lattice_units": [lat, units], "summation_runs": runs,
                "roofline": roofline(args.workload + tag, 1, lay, kf, f.algorithmic_bytes(),
                                     min_bytes(f, fes_s.ne, nd, fes_s.ndofs), None, use_pin=pin_ok and use_pin,
                                     flops=alg_flops(order, fes_s.ne)),
                "note": note}

    dl.at("assemble")
    if nsub <= 1 and not par:
        form = serial_form(compress)
        alpha, T = keep[0], keep[1]
        n_true = fes.ndofs
        apply = form.Mult
        timed_forms = [form]
        ne_own = fes.ne
    else:
        # z-slab partition (CartesianPartitioning along z, mesh.cpp:8966)
        if args.partition == "boxes":
            f = {1: (1, 1, 1), 2: (1, 1, 2), 4: (1, 2, 2), 8: (2, 2, 2), 16: (2, 2, 4)}.get(nsub)
            if f is None:
                raise SystemExit(f"--partition boxes: no box factorisation for {nsub} parts")
            er = E.partition_boxes(mesh, f)
        elif args.partition == "bricks":
            er = E.partition_bricks(mesh, nsub)
        else:
            er = E.partition_slabs_z(mesh, nsub)
        if par:
            rid = [E.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(rid, src=0)
            part = E.Partition(fes, er, rank, world, decomposition=decomp)
            pform = E.ParBilinearForm(part, rccl_id=rid[0], kernel=kernel, scatter=scatter,
                                      compress_geometry=compress, schedule=args.schedule, graph=args.par_graph)
            alpha, T = bioheat_coefficients(E, torch, mesh, fes, part)
            pform.AddDomainIntegrator(mass(alpha))
            pform.AddDomainIntegrator(diff(T))
            pform.Assemble()
            n_true = part.n_owned
            apply = pform.Mult
            timed_forms = [pform]
            ne_own = part.ne_owned
        else:
            # --loopback: all subdomains in this process on one GPU (exchange by device copies)
            forms = []
            for r in range(nsub):
                part = E.Partition(fes, er, r, nsub, decomposition=decomp)
                pf = E.ParBilinearForm(part, kernel=kernel, scatter=scatter, compress_geometry=compress,
                                       schedule=args.schedule)
                alpha, T = bioheat_coefficients(E, torch, mesh, fes, part)
                keep += [alpha, T, part]
                pf.AddDomainIntegrator(mass(alpha))
                pf.AddDomainIntegrator(diff(T))
                pf.Assemble()
                forms.append(pf)
            group = E.ParGroup(forms)
            xs = [torch.empty(f.true_size, dtype=torch.float64, device="cuda").uniform_(-1, 1) for f in forms]
            ys = [torch.empty_like(v) for v in xs]
            if args.member is not None:
                member_bench(args, E, torch, group, xs, ys, fes.ndofs, workload, dl)
                return
            n_true = sum(f.true_size for f in forms)
            apply = lambda _x, _y: group.Mult(xs, ys)
            timed_forms = forms
            ne_own = fes.ne

    x = torch.empty(n_true, dtype=torch.float64, device="cuda")
    x.uniform_(-1.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(1 + rank))
    y = torch.empty_like(x)
    torch.cuda.synchronize()

    dl.at("kernel timing")
    pdist = dist if par else None
    if par:
        dist.barrier()  # all ranks settle together
    kms = kernel_ms(timed_forms, apply, x, y, args.steps, torch, world=world, dist=pdist)
    dl.at("timed Mults")
    dt = time_mults(apply, x, y, args.steps, args.warmup, world, pdist, torch)
    abytes = sum(f.algorithmic_bytes() for f in timed_forms)
    nd = (order + 1) ** 3
    mbytes = sum(min_bytes(f, f.part.ne_local if hasattr(f, "part") else fes.ne, nd, f.true_size
                           if hasattr(f, "true_size") else n_true) for f in timed_forms)
    qbytes = sum(f.qdata_bytes() for f in timed_forms)
    layout = qdata_layout(E, timed_forms[0])
    pcg = c3_pcg(E, torch, fes, form) if args.workload == "c3" else None
    reasm = reassembly_ms(torch, form) if (form is not None and args.workload != "c3") else None
    pcg_it = (pcg_iteration_ms(torch, form, fes.ndofs, args.pcg_iters)
              if (args.pcg_iters and form is not None and world == 1 and args.loopback <= 1) else None)
    sdirk = (sdirk_step(E, torch, mesh, fes, keep)
             if (args.sdirk and form is not None and world == 1 and args.loopback <= 1 and args.workload != "c3")
             else None)

    # aggregate over ranks: total true dofs, max time; kernel ms per Mult (interior + boundary
    # launches of one Mult when partitioned); bytes per GPU
    tot = torch.tensor([float(n_true), dt, abytes, kms, qbytes, mbytes], dtype=torch.float64, device="cuda")
    if par:
        dl.at("reduce results")
        s = tot.clone()
        for i in (0, 2, 4, 5):
            dist.all_reduce(s[i:i + 1], op=dist.ReduceOp.SUM)
        for i in (1, 3):
            dist.all_reduce(s[i:i + 1], op=dist.ReduceOp.MAX)
        tot = s
    ndofs_total, tmax, bytes_total, kavg_ms, qbytes_total, mbytes_total = [float(v) for v in tot.cpu()]
    pin_ok = (args.loopback <= 1 and (args.workload != "c2" or args.c2_n == 50)
              and (args.workload != "c3" or args.c3_refine == 6))
    value = ndofs_total * args.steps / tmax / 1e6
    lattice = timed_forms[0].AddressingInfo()

    subs = {}
    serial_main = not par and args.loopback <= 1 and args.workload != "c3"
    if serial_main and args.full_layout and compress:
        dl.at("full layout")
        del apply
        ff = serial_form(False)
        subs["full_layout"] = sub_measure(
            ff, fes, variant, "same run, same mesh and numbering, per-point qdata (56 B per quadrature point: the "
                              "layout SURVEY §8(d)'s algorithmic bytes describe, so its alg_ratio is a roofline fraction)")
        del ff
    if (serial_main and args.variants == 1 and args.numbering == "structured" and args.mesh == "affine"
            and args.coefficients == "bioheat"):
        dl.at("entity numbering")
        me, fe_ = cartesian_space(E, nx, ny, nz_total, order, "entity", "affine")
        fv = serial_form(compress, me, fe_, "entity")
        subs["entity_numbering"] = sub_measure(
            fv, fe_, "ent", "same run, same mesh geometry, the reference's own numbering: MakeCartesian3D's "
                            "space-filling-curve element order (sfc_ordering = true) and FiniteElementSpace's "
                            "vertex/edge/face/interior dofs (what a drop-in BilinearFormExtension receives as "
                            "gather_map), element order derived by the form from the map alone")
        del fv
        dl.at("trilinear mesh")
        mt, ft = cartesian_space(E, nx, ny, nz_total, order, "structured", "trilinear")
        fv = serial_form(compress, mt, ft, "structured")
        subs["trilinear"] = sub_measure(
            fv, ft, "tri", "same run, interior vertices moved by up to 0.15 h (genuinely trilinear hexes, as "
                           "an unstructured cardiac mesh): the AFFINE compression does not apply; the TRILINEAR "
                           "layout stores the elements' trilinear-map coefficients and the kernel evaluates J, "
                           "adj(J) and det J at every quadrature point (the per-point layout is full_layout's)")
        del fv, me, fe_, mt, ft
        dl.at("drop-in configuration")
        md, fd = cartesian_space(E, nx, ny, nz_total, order, "entity", "trilinear")
        fv = serial_form(compress, md, fd, "entity", "jacobians")
        subs["drop_in"] = sub_measure(
            fv, fd, "enttrijac", "same run, the configuration a drop-in ECM2PABilinearFormExtension executes "
                                 "(INTEGRATION.md): the reference's own numbering (SFC element order, entity dofs), "
                                 "non-affine hexes (interior vertices moved by up to 0.15 h) and the geometry as MFEM's "
                                 "GeometricFactors::JACOBIANS array (set_jacobians, fitted to trilinear maps at "
                                 "Assemble)")
        del fv, md, fd
    if (serial_main and args.variants in (1, 2) and args.numbering == "structured" and args.mesh == "affine"
            and args.coefficients == "bioheat"):
        for case, note in (("pennes", "same run, same mesh and numbering as the main line, the Pennes operator with "
                                      "both coefficients laws of one H1 temperature field: Mass(rho c + gamma dt c_b "
                                      "w_b(T), perfusion shut-off at T_stop) + Diffusion(gamma dt k(T)); the snapshot "
                                      "kernel applies both laws at the point and stores one mass value per element "
                                      "(no per-point stream)"),
                           ("ex16", "same run, same mesh and numbering, ex16p's implicit operator M + dt K(u_alpha_gf) "
                                    "with u_alpha_gf = kappa + alpha u formed at the dofs and passed as a "
                                    "GridFunctionCoefficient (examples/ex16p.cpp:450-466); one mass value per "
                                    "element")):
            dl.at(f"{case} form")
            fv = bench_law_form(E, torch, mesh, fes, keep, case)
            sub = sub_measure(fv, fes, {"pennes": "pen", "ex16": "ex16"}[case], note)  # (its own pin)
            sub["snapshot"] = dict(zip(("on", "mass_values", "law_at_point"), fv.SnapshotInfo()))
            subs[case] = sub
            del fv

    if rank == 0:
        dl.at("stream copy peak")
        stream = stream_copy_peak(E, torch)
        cpu = None
        if not args.no_cpu_baseline and not par and args.loopback <= 1:
            dl.at("cpu baseline")
            cpu = cpu_baseline(fes, mesh, alpha, T, args.cpu_baseline_seconds, args.workload)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MDoF/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (generated Cartesian hex mesh, bioheat coefficients, uniform random x)",
            "config": {
                "workload": workload,
                "ndofs": int(ndofs_total),
                "elements": int(fes.ne),
                "order": order, "q1d": order + 2,
                "launch": "stream launches" if not par else par_launch_label(args.schedule, args.par_graph),
                "kernel": ["auto", "tpe", "wpe", "unfused", "line"][timed_forms[0].info()["kernel"]],
                "qdata_layout": layout,
                "numbering": ("entity (the reference's FiniteElementSpace numbering)" if args.workload == "c3" or
                              args.numbering == "entity" else "structured (dof lattice of the Cartesian mesh)"),
                "mesh": args.mesh if args.workload != "c3" else "fichera (affine after refinement)",
                "lattice_units": list(lattice[:2]), "summation_runs": lattice[2],
                "qdata_bytes_stored": qbytes_total / world,
                "parallelism": (f"domain decomposition, {PART_NAME[args.partition]} x{world} ({decomp}, {args.schedule} schedule), RCCL shared-DoF exchange"
                                if par else
                                (f"loopback {PART_NAME[args.partition]} x{args.loopback} on one GPU" if args.loopback > 1 else "single GPU")),
            },
            "roofline": roofline(args.workload + variant, world, layout, kavg_ms, bytes_total / world,
                                 mbytes_total / world, stream, use_pin=pin_ok, flops=alg_flops(order, ne_own)),
            "cpu_baseline": cpu,
        }
        if sdirk is not None:
            line["sdirk_step"] = sdirk
        if pcg_it is not None:
            line["pcg_iteration"] = {"iterations": args.pcg_iters, "iteration_ms": round(pcg_it, 5),
                                     "mdof_iter_per_s": round(fes.ndofs / (pcg_it * 1e-3) / 1e6, 1),
                                     "note": "marginal time per Jacobi-PCG iteration on the serial form (ecm2_pcg_solve: the "
                                             "device-driven loop), no ess: Mult + two fused vector passes "
                                             "(step_r with (B r, r), update_xd) + (A d, d), folded into "
                                             "the Mult's element energies on the snapshot kernel, a dot "
                                             "pass otherwise"}
        if reasm is not None:
            line["reassembly_ms"] = reasm  # Assemble after a k(T) change, plan kept (outside the timed region)
        line.update(subs)
        if pcg is not None:
            line["pcg"] = pcg
        print(json.dumps(line), flush=True)
    dl.at("teardown")
    if par:
        # release the forms (ncclCommDestroy of the operator's communicator) on every rank
        # while all ranks are alive, then tear down torch's process group
        del apply, timed_forms, pform
        import gc
        gc.collect()
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
    dl.done()


def variant_key(args):
    """Suffix of the PMC pin of the main line's variant: '' structured affine, 'ent', 'tri', 'jac'
    (geometry as MFEM Jacobians) and their combinations ('enttrijac': the drop-in configuration)."""
    if args.workload == "c3":
        return ""
    return (("ent" if args.numbering == "entity" else "") + ("tri" if args.mesh == "trilinear" else "")
            + ("jac" if args.geometry_input == "jacobians" else "")
            + {"bioheat": "", "pennes": "pen", "ex16": "ex16"}[args.coefficients])


def cartesian_space(E, nx, ny, nz, order, numbering, shape):
    """The Cartesian box mesh and its H1 space.  structured: lexicographic elements, lattice dofs;
    entity: the reference's MakeCartesian3D (space-filling-curve element order) and its
    FiniteElementSpace numbering.  trilinear: every interior vertex moved by a seeded uniform
    offset of up to 0.15 h per coordinate (non-affine hexes)."""
    mesh = E.Mesh.MakeCartesian3D(nx, ny, nz, 1.0, ny / nx, nz / nx, sfc_ordering=(numbering == "entity"))
    if shape == "trilinear":
        V = mesh.vertices()
        h = 1.0 / nx
        hi = np.array([1.0, ny / nx, nz / nx])
        inner = np.all((V > 0.5 * h) & (V < hi - 0.5 * h), axis=1)
        V[inner] += 0.15 * h * np.random.default_rng(7).uniform(-1, 1, (int(inner.sum()), 3))
        mesh.set_vertices(V)
    fes = E.H1Space(mesh, order, E.NUMBERING_ENTITY if numbering == "entity" else E.NUMBERING_STRUCTURED)
    return mesh, fes


def reassembly_ms(torch, form, reps=5):
    """Device re-assembly after a k(T) change (row f1: the coefficient snapshot or projection and the
    qdata setup; the merge plan and addressing are kept), ms per Assemble."""
    form.Assemble()  # warm
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        form.Assemble()
    ev1.record()
    torch.cuda.synchronize()
    return round(ev0.elapsed_time(ev1) / reps, 3)


def c3_pcg(E, torch, fes, form, max_iter=100):
    """C3 extras: device re-assembly after a k(T) change (coefficient projection
    + qdata setup) and a Jacobi-PCG solve on the constrained operator, as MDoF*iter/s."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    form.Assemble()  # warm
    torch.cuda.synchronize()
    ev0.record()
    reps = 5
    for _ in range(reps):
        form.Assemble()
    ev1.record()
    torch.cuda.synchronize()
    reasm_ms = ev0.elapsed_time(ev1) / reps
    ess = torch.as_tensor(fes.boundary_dofs()).cuda()
    b = torch.empty(fes.ndofs, dtype=torch.float64, device="cuda")
    b.uniform_(-1.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(2))
    x = torch.empty_like(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it, nrm = form.PCG(b, x, ess=ess, rel_tol=1e-30, max_iter=max_iter, jacobi=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stop = (f"stopped at max_iter = {max_iter}" if it >= max_iter else
            f"converged to rel_tol 1e-30 after {it} of max_iter = {max_iter} iterations")
    return {"iterations": it, "max_iter": max_iter, "seconds": round(dt, 4),
            "mdof_iter_per_s": round(fes.ndofs * it / dt / 1e6, 1), "reassembly_ms": round(reasm_ms, 3),
            "note": f"Jacobi-PCG with rel_tol 1e-30 ({stop}); MDoF*iter/s over the whole solve (its setup -- the "
                    "Jacobi diagonal, the first residual -- included), with the DIAG_ONE constraint passes and the "
                    "device-driven stopping test"}


def stream_copy_peak(E, torch, nbytes=1 << 30, reps=20):
    """Measured HBM stream rates on this GPU with the library's 16-byte nontemporal kernels:
    (copy: read + write bytes / time, read-only: bytes / time), reported beside the 8 TB/s
    spec peak (SURVEY §8(d) 'Bounding roofline'); frac_of_stream uses the larger."""
    a = torch.empty(nbytes // 8, dtype=torch.float64, device="cuda").uniform_()
    b = torch.empty_like(a)
    for _ in range(3):
        E.stream_copy(a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        E.stream_copy(a, b)
    e1.record()
    torch.cuda.synchronize()
    rate = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del b
    # read-only stream of the same buffer (the PA kernels move ~93% reads)
    out = torch.empty(256 * 64 * 256, dtype=torch.float64, device="cuda")
    for _ in range(3):
        E.stream_read(a, out)
    e0.record()
    for _ in range(reps):
        E.stream_read(a, out)
    e1.record()
    torch.cuda.synchronize()
    rrate = nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, out
    return round(rate, 1), round(rrate, 1)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        return subprocess.check_output(["uname", "-m"], text=True).strip()
    except Exception:
        return "unknown"


# the reference's own CPU PA Mult, 8 OpenMP threads, survey container
REFERENCE_OMP8 = {"c2": 28.4, "c3": 23.3, "c4": 27.5, "c5": 45.8}


def cpu_baseline(fes, mesh, alpha, T, seconds, workload):
    """The oracle (CPU restatement of the reference PA path, 'port') on the same workload,
    timed on this host's cores for a bounded number of Mults (~`seconds` of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    order = fes.order
    q1d = order + 2
    en = mesh.element_nodes()
    gm = fes.gather_map()
    Tq = O.interp_evector(T.cpu().numpy()[gm], order, q1d)
    beta = K_SCALE * (1.0 + K_SLOPE * (Tq - K_TREF))
    op = O.OracleOperator(en, gm, fes.ndofs, order, alpha=alpha.cpu().numpy(), beta=beta)
    x = np.random.default_rng(1).uniform(-1, 1, fes.ndofs)
    op.mult(x)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        op.mult(x)
        n += 1
        if time.perf_counter() - t0 >= seconds or n >= 1000:
            break
    dt = time.perf_counter() - t0
    return {
        "value": round(fes.ndofs * n / dt / 1e6, 3),
        "unit": "MDoF/s",
        "cores": O.num_threads(),
        "cores_note": (f"OpenMP threads = OMP_NUM_THREADS ({os.environ.get('OMP_NUM_THREADS', 'unset')}): the "
                       f"host-core share of one GPU on this box (os.cpu_count() = {os.cpu_count()} is the whole "
                       "multi-GPU host's, shared by 8 GPUs' jobs)"),
        "kind": "port",
        "cpu_model": cpu_model(),
        "sample": f"{n} oracle PA Mults (gather, mass, diffusion, CSR scatter; OpenMP) on the same "
                  f"{fes.ndofs}-DoF mesh, {dt:.1f} s",
        "reference_cpu_omp8": {"value": REFERENCE_OMP8.get(workload), "unit": "MDoF/s",
                               "note": "the reference's own PA Mult, Device('omp'), 8 threads of the survey "
                                       "container's Intel Xeon (BASELINE.md); not run on this host"},
    }


if __name__ == "__main__":
    main()
