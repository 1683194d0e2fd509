#!/usr/bin/env python3
"""bench.py -- MDoF/s of the PA diffusion+mass Mult (hex, H1 p=2) on MI355X.

Metric (BASELINE.json): "MDoF/s on PA diffusion+mass Mult, hex p=2; % HBM roofline at
1/2/4/8 GPUs".  One *step* = one operator Mult y = A x (L-vector in, L-vector out;
tests/benchmarks/bench_assembly_levels.cpp:281-286 counts ndofs per Mult) with x, y
and the operator resident in HBM.  Workload: BASELINE configs[1] -- inline-hex refined
to ~1M DoF (Cartesian 50^3, p = 2, 1,030,301 DoF) per GPU; with N GPUs the global
mesh is 50 x 50 x 50N, z-slab partitioned, one rank per GPU (weak scaling) with the
shared-DoF exchange over RCCL.  --workload c4 runs configs[3] (Cartesian 108^3,
10.2M DoF, split over the ranks: strong scaling).

Coefficients are the bioheat ones: alpha = rho*c_eff(x) (FunctionCoefficient projected
at the quadrature points) and beta = gamma*dt*k(T) with T an H1 grid function (the
Pennes law, evaluated on the device at Assemble).  Inputs are synthetic (no data files).
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2")
    ap.add_argument("--c2-n", type=int, default=50,
                    help="c2: elements per edge of the per-GPU Cartesian block (experiments; configs[1] = 50)")
    ap.add_argument("--c3-refine", type=int, default=6,
                    help="c3: uniform refinements of fichera.mesh (6 -> 14.9M DoF, 5 -> 1.88M)")
    ap.add_argument("--kernel", choices=["auto", "tpe", "wpe", "unfused", "line"], default="auto")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: capture one Mult in a HIP graph and replay it per step (single process)")
    ap.add_argument("--geometry", choices=["compressed", "full"], default="compressed",
                    help="compressed: AFFINE qdata on parallelepiped meshes (default); full: per-point layout")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="measurement aid: run ONE rank (--emulate-rank) of an N-rank partition alone, "
                         "exchanges replaced by same-size device copies (values not the operator's)")
    ap.add_argument("--emulate-rank", type=int, default=1)
    ap.add_argument("--loopback", type=int, default=1,
                    help="N>1 on one GPU: N subdomains in this process (validation of the partitioned path)")
    args = ap.parse_args()

    if args.emulate_world > 1:
        os.environ["ECM2_EMULATE_EXCHANGE"] = "1"
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank % max(1, torch.cuda.device_count())))
    E = load_pkg()
    E.load_library()
    scatter = os.environ.get("ECM2_SCATTER", "partials")  # A/B knob: partials | atomic
    kernel = {"auto": E.KERNEL_AUTO, "tpe": E.KERNEL_TPE, "wpe": E.KERNEL_WPE, "unfused": E.KERNEL_UNFUSED,
              "line": E.KERNEL_LINE}[args.kernel]

    compress = args.geometry == "compressed"
    order = 4 if args.workload == "c5" else 2
    if args.workload == "c2":
        n = args.c2_n
        nx = ny = n
        nz_total = n * max(world, args.emulate_world)
        scaling = "weak"
        workload = f"configs[1]: inline-hex refined to Cartesian {n}x{n}x{nz_total} ({n}^3 per GPU), H1 p=2, Mass(rho*c)+Diffusion(gamma*dt*k(T)) PA Mult"
    elif args.workload == "c3":
        scaling = "strong"
        workload = (f"configs[2]: fichera.mesh refined {args.c3_refine}x, H1 p=2, nonlinear Pennes k(T) "
                    "re-assembled on the device, Jacobi-PCG")
    elif args.workload == "c4":
        nx = ny = nz_total = 108
        scaling = "strong"
        workload = "configs[3]: Cartesian 108^3 (10.2M DoF) split over GPUs, H1 p=2, Mass+Diffusion PA Mult"
    else:
        nx = ny = nz_total = 68
        scaling = "strong"
        workload = "configs[4]: Cartesian 68^3 (20.3M DoF) split over GPUs, H1 p=4, Mass+Diffusion PA Mult"
    if args.workload == "c3":
        if world > 1 or args.loopback > 1:
            raise SystemExit("c3 is the single-GPU PCG configuration")
        mesh = E.Mesh(os.path.join(ROOT, "tests", "golden", "fichera.mesh"))
        for _ in range(args.c3_refine):
            mesh.UniformRefinement()
        fes = E.H1Space(mesh, order)
    else:
        mesh = E.Mesh.MakeCartesian3D(nx, ny, nz_total, 1.0, ny / nx, nz_total / nx)
        fes = E.H1Space(mesh, order, E.NUMBERING_STRUCTURED)
    nsub = world if world > 1 else max(args.loopback, args.emulate_world)
    mass = lambda a: E.MassIntegrator(E.QuadratureCoefficient(a))
    diff = lambda T: E.DiffusionIntegrator(E.AffineGridFunctionCoefficient(T, K_SCALE, K_SLOPE, K_TREF))
    if nsub <= 1:
        alpha, T = bioheat_coefficients(E, torch, mesh, fes)
        form = E.BilinearForm(fes, kernel=kernel, element_order=os.environ.get("ECM2_ELEMENT_ORDER", "auto"),
                              scatter=scatter, compress_geometry=compress)
        form.AddDomainIntegrator(mass(alpha))
        form.AddDomainIntegrator(diff(T))
        form.Assemble()
        n_true = fes.ndofs
        apply = form.Mult
        timed_forms = [form]
    else:
        # z-slab partition (CartesianPartitioning along z, mesh.cpp:8966)
        er = E.partition_slabs_z(mesh, nsub)
        if world > 1 or args.emulate_world > 1:
            if args.emulate_world > 1:
                rid, prank, pworld = [None], args.emulate_rank, args.emulate_world
            else:
                rid = [E.rccl_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(rid, src=0)
                prank, pworld = rank, world
            part = E.Partition(fes, er, prank, pworld, decomposition=os.environ.get("ECM2_DECOMP", "overlap"))
            pform = E.ParBilinearForm(part, rccl_id=rid[0], kernel=kernel, scatter=scatter,
                                      compress_geometry=compress)
            alpha, T = bioheat_coefficients(E, torch, mesh, fes, part)
            pform.AddDomainIntegrator(mass(alpha))
            pform.AddDomainIntegrator(diff(T))
            pform.Assemble()
            n_true = part.n_owned
            apply = pform.Mult
            timed_forms = [pform]
        else:
            # --loopback: all subdomains in this process on one GPU (exchange by device copies)
            forms, keep = [], []
            for r in range(nsub):
                part = E.Partition(fes, er, r, nsub, decomposition=os.environ.get("ECM2_DECOMP", "overlap"))
                pf = E.ParBilinearForm(part, kernel=kernel, scatter=scatter, compress_geometry=compress)
                alpha, T = bioheat_coefficients(E, torch, mesh, fes, part)
                keep += [alpha, T]
                pf.AddDomainIntegrator(mass(alpha))
                pf.AddDomainIntegrator(diff(T))
                pf.Assemble()
                forms.append(pf)
            group = E.ParGroup(forms)
            xs = [torch.empty(f.true_size, dtype=torch.float64, device="cuda").uniform_(-1, 1) for f in forms]
            ys = [torch.empty_like(v) for v in xs]
            n_true = sum(f.true_size for f in forms)
            apply = lambda _x, _y: group.Mult(xs, ys)
            timed_forms = forms

    x = torch.empty(n_true, dtype=torch.float64, device="cuda")
    x.uniform_(-1.0, 1.0, generator=torch.Generator(device="cuda").manual_seed(1 + rank))
    y = torch.empty_like(x)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        apply(x, y)
    torch.cuda.synchronize()
    step = lambda: apply(x, y)
    if args.graph and world == 1:
        # one Mult (all its launches) as a HIP graph, replayed per step
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            apply(x, y)
        graph.replay()
        torch.cuda.synchronize()
        step = graph.replay
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # second, instrumented pass: HIP events around the dominant (fused apply) kernel on
    # the stream it is launched on (kept out of the timed loop above)
    for f in timed_forms:
        f.timing(True)
    for _ in range(args.steps):
        apply(x, y)
    torch.cuda.synchronize()
    kms = sum(f.timing_get()[0] for f in timed_forms)
    for f in timed_forms:
        f.timing(False)
    abytes = sum(f.algorithmic_bytes() for f in timed_forms)
    qbytes = sum(f.qdata_bytes() for f in timed_forms)
    pcg = c3_pcg(E, torch, fes, form) if args.workload == "c3" else None

    # aggregate over ranks: total true dofs, max time; kernel ms per Mult (summed over
    # the apply launches of one Mult: interior + boundary blocks when partitioned)
    tot = torch.tensor([float(n_true), dt, abytes, kms / args.steps, qbytes],
                       dtype=torch.float64, device="cuda")
    if world > 1:
        s = tot.clone()
        dist.all_reduce(s[0:1], op=dist.ReduceOp.SUM)
        dist.all_reduce(s[2:3], op=dist.ReduceOp.SUM)
        dist.all_reduce(s[4:5], op=dist.ReduceOp.SUM)
        dist.all_reduce(s[1:2], op=dist.ReduceOp.MAX)
        dist.all_reduce(s[3:4], op=dist.ReduceOp.MAX)
        tot = s
    ndofs_total, tmax, bytes_total, kavg_ms, qbytes_total = [float(v) for v in tot.cpu()]
    value = ndofs_total * args.steps / tmax / 1e6

    if rank == 0:
        achieved = bytes_total / world / (kavg_ms * 1e-3) / 1e9
        traffic = None
        # pinned PMC traffic of this workload, kernel family and qdata layout (profiles/pmc_pin.py)
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}_n{world}_{qdata_layout(E, timed_forms[0])}.json")
        if os.path.exists(pmc) and args.loopback <= 1 and args.emulate_world <= 1:  # pins are single-form profiles
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        stream = stream_copy_peak(E, torch)
        cpu = None
        if not args.no_cpu_baseline and world == 1 and args.loopback <= 1 and args.emulate_world <= 1:
            cpu = cpu_baseline(fes, mesh, alpha, T, args.cpu_baseline_seconds)
        line = {
            "metric": "MDoF/s on PA diffusion+mass Mult, hex p=2; % HBM roofline at 1/2/4/8 GPUs",
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
                "launch": "hip-graph replay per Mult" if (args.graph and world == 1) else "stream launches",
                "kernel": ["auto", "tpe", "wpe", "unfused", "line"][timed_forms[0].info()["kernel"]],
                "qdata_layout": qdata_layout(E, timed_forms[0]),
                "qdata_bytes_stored": qbytes_total / world,
                "parallelism": f"domain-decomposition z-slabs x{world}, RCCL shared-DoF exchange" if world > 1
                else (f"EMULATED rank {args.emulate_rank} of {args.emulate_world} z-slabs alone on one GPU "
                      "(exchanges = same-size local copies; measurement aid, not a scaling number)"
                      if args.emulate_world > 1 else
                      (f"loopback z-slabs x{args.loopback} on one GPU" if args.loopback > 1 else "single GPU")),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": traffic,
                "kernel_ms_avg": round(kavg_ms, 5),
                "stream_copy_gbs": stream,
                "frac_of_stream": round(achieved / stream, 4) if stream else None,
                "algorithmic_bytes_per_launch": bytes_total / world,
                # real HBM rate of the dominant kernel (PMC bytes / its time): with AFFINE qdata
                # the kernel moves fewer bytes than the SURVEY's fixed formula counts, so
                # "frac" can exceed 1; this is the bandwidth actually drawn
                "traffic_gbs": round(traffic / (kavg_ms * 1e-3) / 1e9, 1) if traffic else None,
                "traffic_frac": round(traffic / (kavg_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4) if traffic else None,
            },
            "cpu_baseline": cpu,
        }
        if pcg is not None:
            line["pcg"] = pcg
        print(json.dumps(line), flush=True)
    if world > 1:
        # release the forms (ncclCommDestroy of the operator's communicator) on every rank
        # while all ranks are alive, then tear down torch's process group
        del step, apply, timed_forms, pform
        import gc
        gc.collect()
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()


def qdata_layout(E, form):
    """Quadrature-data layout of a (local) form: affine | blocked | native."""
    return {E.QLAYOUT_NATIVE: "native", E.QLAYOUT_BLOCKED: "blocked",
            E.QLAYOUT_AFFINE: "affine", E.QLAYOUT_AFFINE_E: "affine_e"}[form.info()["layout"]]


def c3_pcg(E, torch, fes, form, max_iter=200):
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
    it, nrm = form.PCG(b, x, ess=ess, rel_tol=1e-30, max_iter=max_iter, jacobi=True)  # fixed iteration count
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"iterations": it, "seconds": round(dt, 4), "mdof_iter_per_s": round(fes.ndofs * it / dt / 1e6, 1),
            "reassembly_ms": round(reasm_ms, 3),
            "note": "fixed max_iter with rel_tol 1e-30 (timing); includes the per-iteration 8-byte "
                    "convergence read-back and the DIAG_ONE constraint passes"}


def stream_copy_peak(E, torch, nbytes=1 << 30, reps=20):
    """Measured HBM STREAM-copy rate on this GPU (read + write bytes / time) with the
    library's 16-byte nontemporal copy kernel, reported beside the 8 TB/s spec peak
    (SURVEY §8(d) 'Bounding roofline')."""
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
    del a, b
    return round(rate, 1)


def cpu_baseline(fes, mesh, alpha, T, seconds):
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
        "kind": "port",
        "sample": f"{n} oracle PA Mults (gather, mass, diffusion, CSR scatter; OpenMP) on the same "
                  f"{fes.ndofs}-DoF mesh, {dt:.1f} s",
    }


if __name__ == "__main__":
    main()
