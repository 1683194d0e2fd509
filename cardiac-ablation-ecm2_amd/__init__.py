"""cardiac-ablation-ecm2_amd -- Python binding of the MI355X PA diffusion+mass operator.

The product is the C-ABI shared library ``lib/libecm2pa.so`` (C++ host code +
hand-written gfx950 HIP kernels; header ``include/ecm2_pa.h``).  This module is a
thin ctypes mirror of the reference's user-facing names so that tests and the
benchmark read like the reference's own drivers:

    reference (MFEM)                                   here
    Mesh::MakeCartesian3D / Mesh(file)                 Mesh.MakeCartesian3D / Mesh(path)
    Mesh::UniformRefinement                            Mesh.UniformRefinement
    H1_FECollection + FiniteElementSpace               H1Space
    BilinearForm + SetAssemblyLevel(PARTIAL)           BilinearForm (PARTIAL only)
    AddDomainIntegrator(MassIntegrator(Q))             AddDomainIntegrator(MassIntegrator(Q))
    Assemble / Mult / AssembleDiagonal                 Assemble / Mult / AssembleDiagonal
    ConstrainedOperator + CGSolver (+ Jacobi)          BilinearForm.PCG

Vectors are torch CUDA float64 tensors (torch is plumbing: device memory and
streams).  There is no CPU fallback: without the built library or without a GPU
every compute call raises ``ECM2Error``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libecm2pa.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ecm2_pa.h")

MASS, DIFFUSION = 0, 1
COEFF_CONSTANT, COEFF_QUAD, COEFF_GRIDFUNC_AFFINE, COEFF_GRIDFUNC_PERFUSION = 0, 1, 2, 3
COEFF_QUAD_VECTOR, COEFF_QUAD_SYMMATRIX, COEFF_QUAD_MATRIX = 4, 5, 6
COEFF_CONST_VECTOR, COEFF_CONST_SYMMATRIX, COEFF_CONST_MATRIX = 7, 8, 9
COEFF_GRIDFUNC = 10
KERNEL_AUTO, KERNEL_TPE, KERNEL_WPE, KERNEL_UNFUSED, KERNEL_LINE = 0, 1, 2, 3, 4
NUMBERING_ENTITY, NUMBERING_STRUCTURED = 0, 1
ORDER_NATIVE, ORDER_BRICK, ORDER_MORTON = 0, 1, 2
SCATTER_PARTIALS, SCATTER_ATOMIC = 0, 1
QLAYOUT_NATIVE, QLAYOUT_BLOCKED, QLAYOUT_AFFINE, QLAYOUT_AFFINE_E, QLAYOUT_TRILINEAR = 0, 1, 2, 3, 4  # info()['layout']
QLAYOUT_NATIVE9 = 5  # a general matrix diffusion coefficient's 9-entry qdata
QLAYOUT_TRILINEAR_E = 6  # TRILINEAR for the p >= 3 line / brick kernels
DECOMP_RAP, DECOMP_OVERLAP = 0, 1  # Partition decomposition
_SCATTER = {"partials": SCATTER_PARTIALS, "atomic": SCATTER_ATOMIC}


class ECM2Error(RuntimeError):
    pass


_lib = None


def load_library(path: str = LIB_PATH):
    """Load the in-tree HIP library (import torch first so one HIP runtime is used)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ECM2Error(f"HIP extension not built: {path} missing (run __graft_entry__.build())")
    try:
        import torch  # noqa: F401  -- share torch's libamdhip64 / librccl
    except Exception:
        pass
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    vp, ip, dp, i32, f64 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_double
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "ecm2_last_error": (ctypes.c_char_p, []),
        "ecm2_version": (i32, []),
        "ecm2_device_count": (i32, []),
        "ecm2_mesh_cartesian": (i32, [i32, i32, i32, f64, f64, f64, pp]),
        "ecm2_mesh_cartesian_ex": (i32, [i32, i32, i32, f64, f64, f64, i32, pp]),
        "ecm2_mesh_read": (i32, [ctypes.c_char_p, pp]),
        "ecm2_mesh_refine_uniform": (i32, [vp]),
        "ecm2_mesh_info": (i32, [vp, ip, ip]),
        "ecm2_mesh_get_vertices": (i32, [vp, vp]),
        "ecm2_mesh_set_vertices": (i32, [vp, vp]),
        "ecm2_mesh_get_elements": (i32, [vp, vp]),
        "ecm2_mesh_get_element_nodes": (i32, [vp, vp]),
        "ecm2_mesh_get_attributes": (i32, [vp, vp]),
        "ecm2_mesh_set_attributes": (i32, [vp, vp]),
        "ecm2_pa_form_add_integrator_marked": (i32, [vp, i32, i32, vp, vp, vp, i32]),
        "ecm2_pa_form_set_attributes": (i32, [vp, vp]),
        "ecm2_mesh_quadrature_points": (i32, [vp, i32, vp]),
        "ecm2_mesh_destroy": (None, [vp]),
        "ecm2_h1space_create": (i32, [vp, i32, i32, pp]),
        "ecm2_h1space_info": (i32, [vp, ip, ip, ip]),
        "ecm2_h1space_get_gather_map": (i32, [vp, vp]),
        "ecm2_h1space_boundary_dofs": (i32, [vp, vp, ip]),
        "ecm2_h1space_element_order": (i32, [vp, vp]),
        "ecm2_h1space_dof_coords": (i32, [vp, vp, vp]),
        "ecm2_h1space_destroy": (None, [vp]),
        "ecm2_pa_form_create": (i32, [i32, i32, i32, vp, i32, pp]),
        "ecm2_pa_form_set_element_nodes": (i32, [vp, vp]),
        "ecm2_pa_form_set_jacobians": (i32, [vp, vp]),
        "ecm2_pa_form_add_integrator": (i32, [vp, i32, i32, vp, vp]),
        "ecm2_stream_copy": (i32, [vp, vp, ctypes.c_long, vp]),
        "ecm2_stream_read": (i32, [vp, ctypes.c_long, vp, ctypes.c_long, vp]),
        "ecm2_pa_form_set_kernel": (i32, [vp, i32]),
        "ecm2_pa_form_set_scatter": (i32, [vp, i32]),
        "ecm2_pa_form_scatter_info": (i32, [vp, vp, vp]),
        "ecm2_pa_form_set_bricks": (i32, [vp, i32]),
        "ecm2_pa_form_set_geometry_compression": (i32, [vp, i32]),
        "ecm2_pa_form_set_coefficient_snapshot": (i32, [vp, i32]),
        "ecm2_pa_form_coefficient_snapshot": (i32, [vp, ip]),
        "ecm2_pa_form_energy_parts": (i32, [vp, ip]),
        "ecm2_pa_form_flux_diagonal": (i32, [vp, ip]),
        "ecm2_pa_form_qdata_bytes": (i32, [vp, dp]),
        "ecm2_pa_form_brick_info": (i32, [vp, ip, ip]),
        "ecm2_pa_form_addressing_info": (i32, [vp, ip, ip, ctypes.POINTER(ctypes.c_long)]),
        "ecm2_pa_form_plan_info": (i32, [vp, ip, ctypes.POINTER(ctypes.c_long)]),
        "ecm2_pa_form_set_element_order": (i32, [vp, vp]),
        "ecm2_mesh_element_order": (i32, [vp, i32, vp]),
        "ecm2_pa_form_assemble": (i32, [vp, vp]),
        "ecm2_pa_form_mult": (i32, [vp, vp, vp, vp]),
        "ecm2_pa_form_mult_transpose": (i32, [vp, vp, vp, vp]),
        "ecm2_pa_form_add_mult": (i32, [vp, vp, vp, f64, vp]),
        "ecm2_pa_form_assemble_diagonal": (i32, [vp, vp, vp]),
        "ecm2_pa_form_restriction_mult": (i32, [vp, vp, vp, vp]),
        "ecm2_pa_form_restriction_mult_transpose": (i32, [vp, vp, vp, vp]),
        "ecm2_pa_form_integrator_add_mult": (i32, [vp, i32, vp, vp, vp]),
        "ecm2_pa_form_get_qdata": (i32, [vp, i32, vp, vp]),
        "ecm2_pa_form_info": (i32, [vp, ip, ip, ip, ip, ip, ip]),
        "ecm2_pa_form_timing": (i32, [vp, i32]),
        "ecm2_pa_form_timing_get": (i32, [vp, dp, ctypes.POINTER(ctypes.c_long)]),
        "ecm2_pa_form_algorithmic_bytes": (i32, [vp, dp]),
        "ecm2_pa_form_destroy": (None, [vp]),
        "ecm2_pcg_solve": (i32, [vp, vp, i32, vp, vp, f64, f64, i32, i32, ip, dp, vp]),
        "ecm2_pcg_last_converged": (i32, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older build (same-box A/B of library versions); tests check the exports
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int):
    if rc != 0:
        msg = _lib.ecm2_last_error().decode(errors="replace")
        err = ECM2Error(f"ecm2 error {rc}: {msg}")
        err.code = rc
        raise err


def pcg_last_converged() -> bool:
    """IterativeSolver::GetConverged() of this thread's last PCG solve (BilinearForm.PCG,
    Operator.PCG): False after CGSolver's (B r, r) < 0 or (A d, d) == 0 stops and at max_iter."""
    return bool(load_library().ecm2_pcg_last_converged())


def _np_ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def _dev_ptr(t) -> ctypes.c_void_p:
    if t is None:
        return ctypes.c_void_p(0)
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise ECM2Error("expected a torch CUDA tensor")
    if not t.is_contiguous():
        raise ECM2Error("expected a contiguous tensor")
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream=None) -> ctypes.c_void_p:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def stream_read(a, out, stream=None):
    """Read-only HBM stream over a (out: >= 4,194,304 doubles of per-thread sums)."""
    _check(load_library().ecm2_stream_read(_dev_ptr(a), a.numel(), _dev_ptr(out), out.numel(), _stream(stream)))


def stream_copy(a, b, stream=None):
    """b = a through the library's 16-byte nontemporal copy kernel (HBM STREAM measurement)."""
    _check(load_library().ecm2_stream_copy(_dev_ptr(a), _dev_ptr(b), a.numel(), _stream(stream)))


def declared_symbols(header: str = HEADER_PATH) -> list:
    """Function names declared in include/ecm2_pa.h."""
    import re
    txt = open(header).read()
    return sorted(set(re.findall(r"\b(ecm2_[a-z0-9_]+)\s*\(", txt)))


# ----------------------------------------------------------------------------
# Mesh / space (setup side)
# ----------------------------------------------------------------------------
class Mesh:
    """Trilinear hexahedral mesh (Mesh::MakeCartesian3D / Mesh(file) / UniformRefinement)."""

    def __init__(self, path: Optional[str] = None, _handle=None):
        lib = load_library()
        h = ctypes.c_void_p()
        if _handle is not None:
            h = _handle
        else:
            _check(lib.ecm2_mesh_read(path.encode(), ctypes.byref(h)))
        self._h = h

    @classmethod
    def MakeCartesian3D(cls, nx, ny, nz, sx=1.0, sy=1.0, sz=1.0, sfc_ordering=False):
        """Mesh::MakeCartesian3D.  sfc_ordering=True is the reference's default (elements along
        a generalized Hilbert curve); False (lexicographic elements) is this module's default."""
        lib = load_library()
        h = ctypes.c_void_p()
        _check(lib.ecm2_mesh_cartesian_ex(nx, ny, nz, sx, sy, sz, 1 if sfc_ordering else 0, ctypes.byref(h)))
        return cls(_handle=h)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ecm2_mesh_destroy(self._h)
            self._h = None

    def UniformRefinement(self):
        _check(_lib.ecm2_mesh_refine_uniform(self._h))

    def _info(self):
        nv, ne = ctypes.c_int(), ctypes.c_int()
        _check(_lib.ecm2_mesh_info(self._h, ctypes.byref(nv), ctypes.byref(ne)))
        return nv.value, ne.value

    def GetNV(self):
        return self._info()[0]

    def GetNE(self):
        return self._info()[1]

    def vertices(self) -> np.ndarray:
        out = np.empty((self.GetNV(), 3), np.float64)
        _check(_lib.ecm2_mesh_get_vertices(self._h, _np_ptr(out)))
        return out

    def set_vertices(self, v: np.ndarray):
        v = np.ascontiguousarray(v, np.float64)
        assert v.shape == (self.GetNV(), 3)
        _check(_lib.ecm2_mesh_set_vertices(self._h, _np_ptr(v)))

    def elements(self) -> np.ndarray:
        out = np.empty((self.GetNE(), 8), np.int32)
        _check(_lib.ecm2_mesh_get_elements(self._h, _np_ptr(out)))
        return out

    def GetAttributes(self) -> np.ndarray:
        """Element attributes [ne] (Mesh::GetAttribute)."""
        out = np.empty(self.GetNE(), np.int32)
        _check(_lib.ecm2_mesh_get_attributes(self._h, _np_ptr(out)))
        return out

    def SetAttributes(self, attr):
        """Mesh::SetAttribute for every element (then Mesh::SetAttributes)."""
        a = np.ascontiguousarray(attr, np.int32)
        assert a.shape == (self.GetNE(),)
        _check(_lib.ecm2_mesh_set_attributes(self._h, _np_ptr(a)))

    def element_order(self, kind: int) -> np.ndarray:
        """0 native, 1 brick (Cartesian only), 2 Morton order of centroids."""
        out = np.empty(self.GetNE(), np.int32)
        _check(_lib.ecm2_mesh_element_order(self._h, kind, _np_ptr(out)))
        return out

    def quadrature_points(self, q1d: int) -> np.ndarray:
        """Physical Gauss-Legendre points [ne][q1d^3][3] (FunctionCoefficient projection points)."""
        out = np.empty((self.GetNE(), q1d ** 3, 3), np.float64)
        _check(_lib.ecm2_mesh_quadrature_points(self._h, q1d, _np_ptr(out)))
        return out

    def jacobians(self, q1d: int, device="cuda"):
        """GeometricFactors::JACOBIANS of the trilinear elements at the q1d^3 Gauss-Legendre
        points (mesh.cpp:15220-15273): a torch float64 tensor in MFEM's layout NQ x 3 x 3 x NE,
        J(q, i, j, e) = d x_i / d xi_j, q lexicographic (qx fastest) -- the array the reference-side
        binding hands ecm2_pa_form_set_jacobians.  Computed with torch on
        `device` from the corners (the caller's data, not the product path)."""
        import torch
        t, _ = np.polynomial.legendre.leggauss(q1d)
        t = 0.5 * (t + 1.0)
        z = torch.as_tensor(self.element_nodes(), device=device)  # [e][i][corner], corner = cx + 2 cy + 4 cz
        # d N_c / d xi_j at every point: N_c = prod_k (xi_k if c_k else 1 - xi_k)
        dN = np.zeros((q1d ** 3, 8, 3))
        for q in range(q1d ** 3):
            xi = (t[q % q1d], t[(q // q1d) % q1d], t[q // (q1d * q1d)])
            for c in range(8):
                ck = (c & 1, (c >> 1) & 1, (c >> 2) & 1)
                f = [xi[k] if ck[k] else 1.0 - xi[k] for k in range(3)]
                for j in range(3):
                    g = 1.0 if ck[j] else -1.0
                    dN[q, c, j] = g * np.prod([f[k] for k in range(3) if k != j])
        dN = torch.as_tensor(dN, device=device)
        # J[e][j][i][q] flattened is MFEM's J(q, i, j, e)
        return torch.einsum("eic,qcj->ejiq", z, dN).contiguous()

    def element_nodes(self) -> np.ndarray:
        """Lexicographic corner coordinates [ne][3][8]."""
        out = np.empty((self.GetNE(), 3, 8), np.float64)
        _check(_lib.ecm2_mesh_get_element_nodes(self._h, _np_ptr(out)))
        return out


class H1Space:
    """H1_FECollection(order) + FiniteElementSpace on a hex mesh (lexicographic element dofs)."""

    def __init__(self, mesh: Mesh, order: int, numbering: int = NUMBERING_ENTITY):
        h = ctypes.c_void_p()
        _check(load_library().ecm2_h1space_create(mesh._h, order, numbering, ctypes.byref(h)))
        self._h = h
        self.mesh = mesh
        self.order = order
        nd, ne, ndl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(_lib.ecm2_h1space_info(h, ctypes.byref(nd), ctypes.byref(ne), ctypes.byref(ndl)))
        self.ndofs, self.ne, self.nd = nd.value, ne.value, ndl.value

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ecm2_h1space_destroy(self._h)
            self._h = None

    def GetVSize(self):
        return self.ndofs

    GetTrueVSize = GetVSize

    def gather_map(self) -> np.ndarray:
        out = np.empty((self.ne, self.nd), np.int32)
        _check(_lib.ecm2_h1space_get_gather_map(self._h, _np_ptr(out)))
        return out

    def element_order_faces(self) -> np.ndarray:
        """4x4x4 face-linked bricks first (ecm2_h1space_element_order): internal position -> element."""
        out = np.empty(self.ne, np.int32)
        _check(_lib.ecm2_h1space_element_order(self._h, _np_ptr(out)))
        return out

    def boundary_dofs(self) -> np.ndarray:
        n = ctypes.c_int(0)
        _check(_lib.ecm2_h1space_boundary_dofs(self._h, None, ctypes.byref(n)))
        out = np.empty(n.value, np.int32)
        if n.value:
            _check(_lib.ecm2_h1space_boundary_dofs(self._h, _np_ptr(out), ctypes.byref(n)))
        return out

    GetEssentialTrueDofs = boundary_dofs

    def dof_coords(self) -> np.ndarray:
        out = np.empty((self.ndofs, 3), np.float64)
        _check(_lib.ecm2_h1space_dof_coords(self._h, self.mesh._h, _np_ptr(out)))
        return out


# ----------------------------------------------------------------------------
# Coefficients and integrators
# ----------------------------------------------------------------------------
class ConstantCoefficient:
    def __init__(self, value: float):
        self.value = float(value)


class QuadratureCoefficient:
    """Values at the quadrature points, torch CUDA float64 [ne][nq] (CoefficientVector)."""

    def __init__(self, values):
        self.values = values


class VectorCoefficient:
    """DiffusionIntegrator(VectorCoefficient): the diagonal conductivity diag(v).  values: a
    3-vector (VectorConstantCoefficient) or torch CUDA float64 [ne][nq][3] at the quadrature points."""

    def __init__(self, values):
        self.values = values


class MatrixCoefficient:
    """DiffusionIntegrator(MatrixCoefficient): anisotropic conductivity M.  values: a 3x3 matrix
    (MatrixConstantCoefficient) or torch CUDA float64 [ne][nq][3][3] at the quadrature points
    (row-major M(i, j)); symmetric=True (SymmetricMatrixCoefficient) keeps the 6 entries
    (11,12,13,22,23,33), else the general 9-entry qdata (bilininteg_diffusion_kernels.cpp:297-348)."""

    def __init__(self, values, symmetric=False):
        self.values, self.symmetric = values, bool(symmetric)


class GridFunctionCoefficient:
    """GridFunctionCoefficient (coefficient.cpp:250-253): the H1 field T (CUDA L-vector on the form's
    own space) interpolated at the quadrature points, no law -- e.g. ex16p's kappa + alpha u formed at
    the dofs (examples/ex16p.cpp:450-466)."""

    def __init__(self, T):
        self.T = T


class AffineGridFunctionCoefficient:
    """scale * (1 + slope * (T(x) - t_ref)) with T an H1 grid function (CUDA L-vector).

    The Pennes conductivity law k(T) = k0 (1 + a (T - T0)) times gamma*dt."""

    def __init__(self, T, scale=1.0, slope=0.0, t_ref=0.0):
        self.T, self.scale, self.slope, self.t_ref = T, float(scale), float(slope), float(t_ref)


class PerfusionCoefficient:
    """Pennes heat capacity + perfusion of an implicit stage's mass coefficient, from an H1
    temperature grid function T (CUDA L-vector):
        alpha(T) = rho_c + gdt_cb * w_b(T),   w_b(T) = w0 * max(0, 1 + a (T - t0)) for T < t_stop,
    0 at or above t_stop (perfusion shut-down in coagulated tissue)."""

    def __init__(self, T, rho_c, gdt_cb, w0, a=0.0, t0=37.0, t_stop=1e300):
        self.T = T
        self.params = tuple(float(v) for v in (rho_c, gdt_cb, w0, a, t0, t_stop))


def _check_points(c, v, tails, ne, nq, flat_ok=False):
    """A per-quadrature-point coefficient tensor must be CUDA float64, contiguous-able, shaped
    (ne, nq) + one of `tails` (flat_ok: or ne * nq values in any shape): the kernels read it as
    [ne][nq][dim] doubles, so anything else would be misread (or read out of bounds) on the GPU."""
    import torch
    name = type(c).__name__
    if not isinstance(v, torch.Tensor) or not v.is_cuda or v.dtype != torch.float64:
        raise ECM2Error(f"{name}: expected a CUDA float64 tensor, got {type(v).__name__} "
                        f"{getattr(v, 'dtype', '')}")
    if flat_ok:
        if ne is not None and v.numel() != ne * nq:
            raise ECM2Error(f"{name}: {v.numel()} values, the form has {ne} x {nq} quadrature points")
        if not v.is_contiguous():
            raise ECM2Error(f"{name}: the values must be contiguous")
        return
    shp = tuple(v.shape)
    if len(shp) < 2 or shp[2:] not in tails or (ne is not None and shp[:2] != (ne, nq)):
        raise ECM2Error(f"{name}: expected shape ({ne}, {nq}) + one of {tails}, got {shp}")


def _check_field(c, T, ndofs):
    """A grid-function coefficient's field must be a CUDA float64 L-vector of the form's space (the
    local [owned | ghost] L-vector for a partitioned form): the snapshot and coefficient kernels read
    ndofs doubles from it."""
    import torch
    name = type(c).__name__
    if not isinstance(T, torch.Tensor) or not T.is_cuda or T.dtype != torch.float64:
        raise ECM2Error(f"{name}: expected a CUDA float64 tensor, got {type(T).__name__} {getattr(T, 'dtype', '')}")
    if ndofs is not None and T.numel() != ndofs:
        raise ECM2Error(f"{name}: {T.numel()} values, the form's L-vector has {ndofs}")
    if not T.is_contiguous():
        raise ECM2Error(f"{name}: the field must be contiguous")


def _integrator_args(c, keep, ne=None, nq=None, ndofs=None):
    """(coefficient kind, data pointer, params pointer) of a coefficient for the C ABI; ne, nq: the
    form's elements and quadrature points per element (checked against per-point tensors); ndofs: its
    L-vector size (checked against grid-function fields)."""
    if isinstance(c, (GridFunctionCoefficient, AffineGridFunctionCoefficient, PerfusionCoefficient)):
        _check_field(c, c.T, ndofs)
    if isinstance(c, ConstantCoefficient):
        arr = (ctypes.c_double * 1)(c.value)
        keep.append(arr)
        return COEFF_CONSTANT, ctypes.cast(arr, ctypes.c_void_p), None
    if isinstance(c, QuadratureCoefficient):
        _check_points(c, c.values, ((),), ne, nq, flat_ok=True)
        keep.append(c.values)
        return COEFF_QUAD, _dev_ptr(c.values), None
    if isinstance(c, GridFunctionCoefficient):
        keep.append(c.T)
        return COEFF_GRIDFUNC, _dev_ptr(c.T), None
    if isinstance(c, AffineGridFunctionCoefficient):
        keep.append(c.T)
        params = (ctypes.c_double * 3)(c.scale, c.slope, c.t_ref)
        keep.append(params)
        return COEFF_GRIDFUNC_AFFINE, _dev_ptr(c.T), ctypes.cast(params, ctypes.c_void_p)
    if isinstance(c, (VectorCoefficient, MatrixCoefficient)):
        v = c.values
        vec = isinstance(c, VectorCoefficient)
        if hasattr(v, "is_cuda"):  # per quadrature point, device
            # the kernels read [ne][nq][dim] float64: anything else would be misread on the GPU
            _check_points(c, v, ((3,),) if vec else ((3, 3), (9,)), ne, nq)
            if vec:
                keep.append(v.contiguous())
                return COEFF_QUAD_VECTOR, _dev_ptr(keep[-1]), None
            m = v.reshape(v.shape[0], v.shape[1], 3, 3)
            if c.symmetric:
                m = m[..., [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
            keep.append(m.contiguous())
            return (COEFF_QUAD_SYMMATRIX if c.symmetric else COEFF_QUAD_MATRIX), _dev_ptr(keep[-1]), None
        a = np.asarray(v, np.float64)
        if vec:
            arr = (ctypes.c_double * 3)(*a.reshape(3))
            kind = COEFF_CONST_VECTOR
        elif c.symmetric:
            a = a.reshape(3, 3)
            arr = (ctypes.c_double * 6)(a[0, 0], a[0, 1], a[0, 2], a[1, 1], a[1, 2], a[2, 2])
            kind = COEFF_CONST_SYMMATRIX
        else:
            arr = (ctypes.c_double * 9)(*a.reshape(9))
            kind = COEFF_CONST_MATRIX
        keep.append(arr)
        return kind, ctypes.cast(arr, ctypes.c_void_p), None
    if isinstance(c, PerfusionCoefficient):
        keep.append(c.T)
        params = (ctypes.c_double * 6)(*c.params)
        keep.append(params)
        return COEFF_GRIDFUNC_PERFUSION, _dev_ptr(c.T), ctypes.cast(params, ctypes.c_void_p)
    raise ECM2Error(f"unsupported coefficient {type(c).__name__}")


class MassIntegrator:
    kind = MASS

    def __init__(self, coeff=None):
        self.coeff = coeff if coeff is not None else ConstantCoefficient(1.0)


class DiffusionIntegrator:
    kind = DIFFUSION

    def __init__(self, coeff=None):
        self.coeff = coeff if coeff is not None else ConstantCoefficient(1.0)


class AssemblyLevel:
    PARTIAL = "partial"


class BilinearForm:
    """BilinearForm at AssemblyLevel::PARTIAL backed by the HIP PA form."""

    def __init__(self, fes: H1Space, kernel: int = KERNEL_AUTO, q1d: int = 0, geometry: str = "nodes",
                 element_order: str = "auto", scatter: str = "partials", bricks: int = -1,
                 compress_geometry: bool = True, coefficient_snapshot: bool = True):
        self.fes = fes
        self._integs = []
        self._kernel = kernel
        self._keep = []
        gm = fes.gather_map()
        h = ctypes.c_void_p()
        _check(load_library().ecm2_pa_form_create(fes.ne, fes.order, fes.ndofs, _np_ptr(gm), q1d, ctypes.byref(h)))
        self._h = h
        if geometry == "nodes":
            en = fes.mesh.element_nodes()
            _check(_lib.ecm2_pa_form_set_element_nodes(h, _np_ptr(en)))
        _check(_lib.ecm2_pa_form_set_kernel(h, kernel))
        _check(_lib.ecm2_pa_form_set_scatter(h, _SCATTER[scatter]))
        _check(_lib.ecm2_pa_form_set_bricks(h, bricks))
        _check(_lib.ecm2_pa_form_set_geometry_compression(h, 1 if compress_geometry else 0))
        _check(_lib.ecm2_pa_form_set_coefficient_snapshot(h, 1 if coefficient_snapshot else 0))
        if element_order == "native" and fes.ne > 0:
            ident = np.arange(fes.ne, dtype=np.int32)  # kept alive across the call
            _check(_lib.ecm2_pa_form_set_element_order(h, _np_ptr(ident)))
        elif fes.ne > 0:
            # "auto": Cartesian meshes -> the mesh's 4x4x4 brick order; otherwise the form
            # derives face-linked bricks from the element->dof map at Assemble
            perm = None
            if element_order in ("auto", "brick"):
                try:
                    perm = fes.mesh.element_order(ORDER_BRICK)
                except ECM2Error:
                    if element_order == "brick":
                        raise
            elif element_order == "morton":
                perm = fes.mesh.element_order(ORDER_MORTON)
            elif element_order != "faces":
                raise ECM2Error(f"unknown element order {element_order!r}")
            if perm is not None:
                _check(_lib.ecm2_pa_form_set_element_order(h, _np_ptr(perm)))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ecm2_pa_form_destroy(self._h)
            self._h = None

    def SetAssemblyLevel(self, level):
        if level != AssemblyLevel.PARTIAL:
            raise ECM2Error("only AssemblyLevel::PARTIAL is implemented")

    def SetJacobians(self, J):
        """GeometricFactors::JACOBIANS (NQ x 3 x 3 x NE, torch CUDA)."""
        self._keep.append(J)
        _check(_lib.ecm2_pa_form_set_jacobians(self._h, _dev_ptr(J)))

    def AddDomainIntegrator(self, integ, elem_marker=None):
        """BilinearForm::AddDomainIntegrator(integ[, elem_marker]): with a marker (0 / 1 per
        attribute) the integrator acts on the elements whose attribute a has elem_marker[a-1]."""
        info = self.info()
        kind, data, params = _integrator_args(integ.coeff, self._keep, info["ne"], info["q1d"] ** 3, info["ndofs"])
        if elem_marker is None:
            _check(_lib.ecm2_pa_form_add_integrator(self._h, integ.kind, kind, data, params))
        else:
            mk = np.ascontiguousarray(elem_marker, np.int32)
            _check(_lib.ecm2_pa_form_add_integrator_marked(self._h, integ.kind, kind, data, params, _np_ptr(mk),
                                                           mk.size))
            self._marked = True
        self._integs.append(integ)

    def Assemble(self, stream=None):
        if getattr(self, "_marked", False):  # the mesh's current attributes, as the reference reads them
            attr = np.ascontiguousarray(self.fes.mesh.GetAttributes())
            _check(_lib.ecm2_pa_form_set_attributes(self._h, _np_ptr(attr)))
        _check(_lib.ecm2_pa_form_assemble(self._h, _stream(stream)))

    def ScatterInfo(self):
        """(shared dofs, partial slots) of the fused kernel's deterministic scatter."""
        n, m = ctypes.c_int(), ctypes.c_long()
        _check(_lib.ecm2_pa_form_scatter_info(self._h, ctypes.byref(n), ctypes.byref(m)))
        return n.value, m.value

    def AddressingInfo(self):
        """(lattice, units, n_runs) after Assemble: of the fused kernel's units (p <= 2 blocks,
        p >= 3 bricks), those that compute their dofs from the lattice instead of reading the
        gather map; runs of the summation plan."""
        n, u, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
        _check(_lib.ecm2_pa_form_addressing_info(self._h, ctypes.byref(n), ctypes.byref(u), ctypes.byref(r)))
        return n.value, u.value, r.value

    def PlanInfo(self):
        """(lattice-slot units, explicit-dof summation runs) after Assemble."""
        n, r = ctypes.c_int(), ctypes.c_long()
        _check(_lib.ecm2_pa_form_plan_info(self._h, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value

    def BrickInfo(self):
        """(bricks, depth bz) of the p >= 3 brick kernel after Assemble (0, 0: none)."""
        n, bz = ctypes.c_int(), ctypes.c_int()
        _check(_lib.ecm2_pa_form_brick_info(self._h, ctypes.byref(n), ctypes.byref(bz)))
        return n.value, bz.value

    def Mult(self, x, y, stream=None):
        _check(_lib.ecm2_pa_form_mult(self._h, _dev_ptr(x), _dev_ptr(y), _stream(stream)))

    def MultTranspose(self, x, y, stream=None):
        _check(_lib.ecm2_pa_form_mult_transpose(self._h, _dev_ptr(x), _dev_ptr(y), _stream(stream)))

    def AddMult(self, x, y, a=1.0, stream=None):
        """y += a A x (Operator::AddMult)."""
        _check(_lib.ecm2_pa_form_add_mult(self._h, _dev_ptr(x), _dev_ptr(y), float(a), _stream(stream)))

    def SetKernel(self, kernel: int):
        _check(_lib.ecm2_pa_form_set_kernel(self._h, kernel))

    def SetGeometryCompression(self, on: bool):
        _check(_lib.ecm2_pa_form_set_geometry_compression(self._h, 1 if on else 0))

    def SetCoefficientSnapshot(self, on: bool):
        """Interpolate the diffusion coefficient's field snapshot in the kernel (see ecm2_pa.h)."""
        _check(_lib.ecm2_pa_form_set_coefficient_snapshot(self._h, 1 if on else 0))

    def CoefficientSnapshot(self) -> bool:
        v = ctypes.c_int()
        _check(_lib.ecm2_pa_form_coefficient_snapshot(self._h, ctypes.byref(v)))
        return bool(v.value)

    def SnapshotInfo(self):
        """(snapshot taken, mass values 0 none / 1 per point / 2 per element, laws applied at the point)."""
        v = [ctypes.c_int() for _ in range(3)]
        _check(_lib.ecm2_pa_form_snapshot_info(self._h, *[ctypes.byref(a) for a in v]))
        return bool(v[0].value), v[1].value, bool(v[2].value)

    def FluxDiagonal(self) -> bool:
        """Axis-aligned elements: the snapshot kernel applies adj(J) adj(J)^T / det J as a diagonal."""
        v = ctypes.c_int()
        _check(_lib.ecm2_pa_form_flux_diagonal(self._h, ctypes.byref(v)))
        return bool(v.value)

    def EnergyParts(self):
        """Partials of x^T A x the Mult writes when PCG folds its den = (A d, d) into it (0: a dot pass)."""
        v = ctypes.c_int()
        _check(_lib.ecm2_pa_form_energy_parts(self._h, ctypes.byref(v)))
        return v.value

    def AssembleDiagonal(self, diag, stream=None):
        _check(_lib.ecm2_pa_form_assemble_diagonal(self._h, _dev_ptr(diag), _stream(stream)))

    def RestrictionMult(self, x, xe, stream=None):
        _check(_lib.ecm2_pa_form_restriction_mult(self._h, _dev_ptr(x), _dev_ptr(xe), _stream(stream)))

    def RestrictionMultTranspose(self, xe, y, stream=None):
        _check(_lib.ecm2_pa_form_restriction_mult_transpose(self._h, _dev_ptr(xe), _dev_ptr(y), _stream(stream)))

    def IntegratorAddMultPA(self, kind, xe, ye, stream=None):
        _check(_lib.ecm2_pa_form_integrator_add_mult(self._h, kind, _dev_ptr(xe), _dev_ptr(ye), _stream(stream)))

    def qdata(self, kind) -> np.ndarray:
        info = self.info()
        nq = info["q1d"] ** 3
        nc = (9 if info["layout"] == QLAYOUT_NATIVE9 else 6) if kind == DIFFUSION else 1
        out = np.empty((self.fes.ne, nc, nq), np.float64)
        _check(_lib.ecm2_pa_form_get_qdata(self._h, kind, _np_ptr(out), _stream()))
        return out

    def info(self) -> dict:
        v = [ctypes.c_int() for _ in range(6)]
        _check(_lib.ecm2_pa_form_info(self._h, *[ctypes.byref(a) for a in v]))
        return dict(zip(["ne", "ndofs", "d1d", "q1d", "kernel", "layout"], [a.value for a in v]))

    def timing(self, enable: bool):
        _check(_lib.ecm2_pa_form_timing(self._h, 1 if enable else 0))

    def timing_get(self):
        ms, n = ctypes.c_double(), ctypes.c_long()
        _check(_lib.ecm2_pa_form_timing_get(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def algorithmic_bytes(self) -> float:
        b = ctypes.c_double()
        _check(_lib.ecm2_pa_form_algorithmic_bytes(self._h, ctypes.byref(b)))
        return b.value

    def qdata_bytes(self) -> float:
        """Bytes of quadrature data stored (after Assemble)."""
        b = ctypes.c_double()
        _check(_lib.ecm2_pa_form_qdata_bytes(self._h, ctypes.byref(b)))
        return b.value

    def PCG(self, b, x, ess=None, rel_tol=1e-12, abs_tol=0.0, max_iter=1000, jacobi=True, stream=None):
        """ConstrainedOperator(DIAG_ONE) + CGSolver(+OperatorJacobiSmoother); returns (iters, final_norm)."""
        it, nrm = ctypes.c_int(), ctypes.c_double()
        n_ess = 0 if ess is None else int(ess.numel())
        _check(_lib.ecm2_pcg_solve(self._h, _dev_ptr(ess) if n_ess else None, n_ess, _dev_ptr(b), _dev_ptr(x),
                                   rel_tol, abs_tol, max_iter, 1 if jacobi else 0,
                                   ctypes.byref(it), ctypes.byref(nrm), _stream(stream)))
        return it.value, nrm.value


# ----------------------------------------------------------------------------
# Distributed form (ParMesh partition + ParBilinearForm over RCCL)
# ----------------------------------------------------------------------------
_PAR_SIGS = {
    "ecm2_partition_slabs_z": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "ecm2_partition_bricks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "ecm2_partition_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_partition_info": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int)] * 6),
    "ecm2_partition_get": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 7),
    "ecm2_partition_destroy": (None, [ctypes.c_void_p]),
    "ecm2_rccl_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "ecm2_par_form_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_par_form_add_integrator": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    "ecm2_par_form_add_integrator_marked": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "ecm2_par_form_set_attributes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ecm2_par_form_set_kernel": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ecm2_par_form_set_scatter": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ecm2_par_form_set_bricks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ecm2_par_form_set_schedule": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ecm2_par_form_addressing_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                                      ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_long)]),
    "ecm2_par_form_set_geometry_compression": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ecm2_par_form_qdata_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "ecm2_par_form_coefficient_snapshot": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "ecm2_par_form_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "ecm2_rccl_p2p_selftest": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    "ecm2_partition_create_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_partition_decomposition": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                                    ctypes.POINTER(ctypes.c_int)]),
    "ecm2_par_form_assemble": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ecm2_par_form_mult": (ctypes.c_int, [ctypes.c_void_p] * 4),
    "ecm2_par_form_mult_transpose": (ctypes.c_int, [ctypes.c_void_p] * 4),
    "ecm2_partition_exchange_schedule": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                        ctypes.POINTER(ctypes.c_int)]),
    "ecm2_par_group_mult": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "ecm2_par_group_mult_rccl": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p]),
    "ecm2_par_group_mult_member": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p]),
    "ecm2_par_form_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ecm2_par_form_timing_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_long)]),
    "ecm2_par_form_algorithmic_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "ecm2_par_form_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "ecm2_par_form_destroy": (None, [ctypes.c_void_p]),
    "ecm2_mesh_quadrature_points_subset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                          ctypes.c_int, ctypes.c_void_p]),
    "ecm2_par_form_assemble_diagonal": (ctypes.c_int, [ctypes.c_void_p] * 3),
    "ecm2_par_group_diagonal": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "ecm2_operator_from_pa_form": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_operator_from_par_form": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_operator_from_par_group": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_operator_from_par_member": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_void_p)]),
    "ecm2_operator_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "ecm2_operator_mult": (ctypes.c_int, [ctypes.c_void_p] * 4),
    "ecm2_operator_pcg": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double),
                                         ctypes.c_void_p]),
    "ecm2_ode_implicit_coeff": (ctypes.c_double, [ctypes.c_int]),
    "ecm2_ode_step": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]),
    "ecm2_operator_destroy": (None, [ctypes.c_void_p]),
}


def _par_lib():
    lib = load_library()
    if not getattr(lib, "_ecm2_par_ready", False):
        for name, (res, args) in _PAR_SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype, fn.argtypes = res, args
        lib._ecm2_par_ready = True
    return lib


def partition_slabs_z(mesh: Mesh, nranks: int) -> np.ndarray:
    """Mesh::CartesianPartitioning along z: element -> rank."""
    out = np.empty(mesh.GetNE(), np.int32)
    _check(_par_lib().ecm2_partition_slabs_z(mesh._h, nranks, _np_ptr(out)))
    return out


def partition_boxes(mesh: Mesh, parts) -> np.ndarray:
    """Mesh::CartesianPartitioning(nxyz) (mesh.cpp:8966-9003): element -> rank = i_x + px (i_y +
    py i_z), i_d = clip(floor(n_d (c_d - vmin_d) / (vmax_d - vmin_d)), 0, n_d - 1) with c the
    element centre and [vmin, vmax] the vertices' bounding box; parts = (px, py, pz).  A centre
    that lies exactly on a box boundary (ties of the exact arithmetic, e.g. 10 elements split 4
    ways) goes to the upper box, as the exact formula says (a relative 1e-12 nudge absorbs the
    rounding of the centroid)."""
    n = np.array([int(v) for v in parts])
    c = mesh.element_nodes().mean(axis=2)  # [e][3] centres (the trilinear map at the reference centre)
    V = mesh.vertices()
    lo, hi = V.min(axis=0), V.max(axis=0)
    span = np.where(hi > lo, hi - lo, 1.0)
    t = n * (c - lo) / span
    idx = np.clip(np.floor(t + 1e-12 * np.maximum(1.0, np.abs(t))), 0, n - 1).astype(np.int64)
    return np.ascontiguousarray(idx[:, 0] + n[0] * (idx[:, 1] + n[1] * idx[:, 2]), np.int32)


def partition_bricks(mesh: Mesh, nranks: int, cell: int = 4) -> np.ndarray:
    """Equal runs of whole cell^3 element bricks of a Cartesian mesh in lexicographic (x-fastest)
    brick order, element -> rank (ecm2_partition_bricks).  Every part is a union of the 4 x 4 x 4
    bricks the fused kernels assemble (bricks.hpp aligns them at the part's minimum corner), and
    the parts' brick counts differ by at most one (z-slabs differ by a whole layer).  (Not a
    reference partitioner: the reference offers METIS and Mesh::CartesianPartitioning; Partition
    accepts any element -> rank map.  Measured against z-slabs: DESIGN.md §6.)"""
    out = np.empty(mesh.GetNE(), np.int32)
    _check(_par_lib().ecm2_partition_bricks(mesh._h, nranks, cell, _np_ptr(out)))
    return out


def quadrature_points_subset(mesh: Mesh, q1d: int, elems: np.ndarray) -> np.ndarray:
    elems = np.ascontiguousarray(elems, np.int32)
    out = np.empty((elems.size, q1d ** 3, 3), np.float64)
    _check(_par_lib().ecm2_mesh_quadrature_points_subset(mesh._h, q1d, _np_ptr(elems), elems.size, _np_ptr(out)))
    return out


class Partition:
    """Local view of one rank: [owned | ghost] local L-vector, [interior | boundary]
    elements, neighbour exchange lists (ParFiniteElementSpace / P)."""

    def __init__(self, fes: H1Space, elem_rank: np.ndarray, rank: int, nranks: int, decomposition: str = "overlap"):
        """decomposition: "overlap" (owned + ghost elements, one exchange per Mult; default) or
        "rap" (the reference's P^T A P over owned elements, two exchanges)."""
        lib = _par_lib()
        er = np.ascontiguousarray(elem_rank, np.int32)
        h = ctypes.c_void_p()
        dec = {"rap": DECOMP_RAP, "overlap": DECOMP_OVERLAP}[decomposition]
        _check(lib.ecm2_partition_create_ex(fes._h, fes.mesh._h, _np_ptr(er), rank, nranks, dec, ctypes.byref(h)))
        self._h = h
        self.fes, self.rank, self.nranks = fes, rank, nranks
        d, no = ctypes.c_int(), ctypes.c_int()
        _check(lib.ecm2_partition_decomposition(h, ctypes.byref(d), ctypes.byref(no)))
        self.decomposition, self.ne_owned = ("rap", "overlap")[d.value], no.value
        v = [ctypes.c_int() for _ in range(6)]
        _check(lib.ecm2_partition_info(h, *[ctypes.byref(a) for a in v]))
        self.ne_local, self.ne_interior, self.n_owned, self.n_ghost, self.n_nbrs, self.n_send = [a.value for a in v]
        nd = fes.nd
        self.elems = np.empty(self.ne_local, np.int32)
        self.local_to_global = np.empty(self.n_owned + self.n_ghost, np.int32)
        self.gather_map = np.empty((self.ne_local, nd), np.int32)
        self.nbrs = np.empty(self.n_nbrs, np.int32)
        self.send_off = np.empty(self.n_nbrs + 1, np.int32)
        self.send_idx = np.empty(max(self.n_send, 1), np.int32)
        self.recv_off = np.empty(self.n_nbrs + 1, np.int32)
        _check(lib.ecm2_partition_get(h, _np_ptr(self.elems), _np_ptr(self.local_to_global), _np_ptr(self.gather_map),
                                      _np_ptr(self.nbrs), _np_ptr(self.send_off), _np_ptr(self.send_idx),
                                      _np_ptr(self.recv_off)))
        self.send_idx = self.send_idx[: self.n_send]

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ecm2_partition_destroy(self._h)
            self._h = None

    @property
    def owned_global(self):
        return self.local_to_global[: self.n_owned]

    XBUF_X_TRUE, XBUF_SENDBUF, XBUF_XGHOST, XBUF_YGHOST, XBUF_RECVBUF = 0, 1, 2, 3, 4

    def exchange_schedule(self, transpose: bool) -> np.ndarray:
        """The transfers of P (False) or P^T (True) both transports issue: rows (peer, send,
        buffer, offset, count) -- ecm2_partition_exchange_schedule."""
        lib = _par_lib()
        n = ctypes.c_int(0)
        _check(lib.ecm2_partition_exchange_schedule(self._h, 1 if transpose else 0, None, ctypes.byref(n)))
        out = np.empty((n.value, 5), np.int32)
        if n.value:
            _check(lib.ecm2_partition_exchange_schedule(self._h, 1 if transpose else 0, _np_ptr(out), ctypes.byref(n)))
        return out


def rccl_p2p_selftest(graph: bool, n: int = 4096) -> float:
    """Max error of a one-rank RCCL self send/recv, direct or graph-captured."""
    e = ctypes.c_double()
    _check(_par_lib().ecm2_rccl_p2p_selftest(1 if graph else 0, n, ctypes.byref(e)))
    return e.value


def rccl_unique_id() -> bytes:
    buf = (ctypes.c_ubyte * 128)()
    _check(_par_lib().ecm2_rccl_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return bytes(buf)


class ParBilinearForm:
    """ParBilinearForm(PARTIAL): y_true = P^T A_local P x_true.  rccl_id=None -> loopback
    group member (use ParGroup.Mult); otherwise one process per GPU over RCCL."""

    def __init__(self, part: Partition, rccl_id: Optional[bytes] = None, kernel: int = KERNEL_AUTO, q1d: int = 0,
                 scatter: str = "partials", bricks: int = -1, compress_geometry: bool = True,
                 schedule: str = "serial", graph: int = -1):
        lib = _par_lib()
        self.part = part
        self._q1d = q1d
        self._keep = []
        en = np.ascontiguousarray(part.fes.mesh.element_nodes()[part.elems]) if part.ne_local else np.zeros((1, 3, 8))
        idbuf = None
        if rccl_id is not None:
            idbuf = (ctypes.c_ubyte * 128).from_buffer_copy(rccl_id)
            self._keep.append(idbuf)
        h = ctypes.c_void_p()
        _check(lib.ecm2_par_form_create(part._h, _np_ptr(en), q1d,
                                        ctypes.cast(idbuf, ctypes.c_void_p) if idbuf is not None else None,
                                        ctypes.byref(h)))
        self._h = h
        _check(lib.ecm2_par_form_set_kernel(h, kernel))
        _check(lib.ecm2_par_form_set_scatter(h, _SCATTER[scatter]))
        _check(lib.ecm2_par_form_set_bricks(h, bricks))
        _check(lib.ecm2_par_form_set_schedule(h, {"serial": 0, "overlap": 1}[schedule], graph))
        _check(lib.ecm2_par_form_set_geometry_compression(h, 1 if compress_geometry else 0))
        self.true_size = part.n_owned

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ecm2_par_form_destroy(self._h)
            self._h = None

    def AddDomainIntegrator(self, integ, elem_marker=None):
        kind, data, params = _integrator_args(integ.coeff, self._keep, self.part.ne_local,
                                              (self._q1d or self.part.fes.order + 2) ** 3,
                                              self.part.n_owned + self.part.n_ghost)
        if elem_marker is None:
            _check(_par_lib().ecm2_par_form_add_integrator(self._h, integ.kind, kind, data, params))
        else:
            mk = np.ascontiguousarray(elem_marker, np.int32)
            _check(_par_lib().ecm2_par_form_add_integrator_marked(self._h, integ.kind, kind, data, params,
                                                                  _np_ptr(mk), mk.size))
            self._marked = True

    def Assemble(self, stream=None):
        if getattr(self, "_marked", False):
            attr = np.ascontiguousarray(self.part.fes.mesh.GetAttributes()[self.part.elems])
            _check(_par_lib().ecm2_par_form_set_attributes(self._h, _np_ptr(attr)))
        _check(_par_lib().ecm2_par_form_assemble(self._h, _stream(stream)))

    def Mult(self, x, y, stream=None):
        _check(_par_lib().ecm2_par_form_mult(self._h, _dev_ptr(x), _dev_ptr(y), _stream(stream)))

    def MultTranspose(self, x, y, stream=None):
        _check(_par_lib().ecm2_par_form_mult_transpose(self._h, _dev_ptr(x), _dev_ptr(y), _stream(stream)))

    def SetKernel(self, kernel: int):
        _check(_par_lib().ecm2_par_form_set_kernel(self._h, kernel))

    def SetGeometryCompression(self, on: bool):
        _check(_par_lib().ecm2_par_form_set_geometry_compression(self._h, 1 if on else 0))

    def AssembleDiagonal(self, d, stream=None):
        """Diagonal of P^T A P on this rank's true dofs (collective over the RCCL ranks)."""
        _check(_par_lib().ecm2_par_form_assemble_diagonal(self._h, _dev_ptr(d), _stream(stream)))

    def timing(self, enable: bool):
        _check(_par_lib().ecm2_par_form_timing(self._h, 1 if enable else 0))

    def timing_get(self):
        ms, n = ctypes.c_double(), ctypes.c_long()
        _check(_par_lib().ecm2_par_form_timing_get(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def algorithmic_bytes(self) -> float:
        b = ctypes.c_double()
        _check(_par_lib().ecm2_par_form_algorithmic_bytes(self._h, ctypes.byref(b)))
        return b.value

    def qdata_bytes(self) -> float:
        b = ctypes.c_double()
        _check(_par_lib().ecm2_par_form_qdata_bytes(self._h, ctypes.byref(b)))
        return b.value

    def CoefficientSnapshot(self) -> bool:
        v = ctypes.c_int()
        _check(_par_lib().ecm2_par_form_coefficient_snapshot(self._h, ctypes.byref(v)))
        return bool(v.value)

    def AddressingInfo(self):
        """(lattice, units, n_runs) of the rank's local form (see BilinearForm.AddressingInfo)."""
        n, u, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
        _check(_par_lib().ecm2_par_form_addressing_info(self._h, ctypes.byref(n), ctypes.byref(u), ctypes.byref(r)))
        return n.value, u.value, r.value

    def info(self) -> dict:
        n, k, lay = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(_par_lib().ecm2_par_form_info(self._h, ctypes.byref(n), ctypes.byref(k)))
        _check(_par_lib().ecm2_par_form_layout(self._h, ctypes.byref(lay)))
        return {"n_true": n.value, "kernel": k.value, "layout": lay.value}


class ParGroup:
    """All subdomains of one partition in this process on one GPU (loopback transport)."""

    def __init__(self, forms):
        self.forms = list(forms)

    def Mult(self, xs, ys, stream=None):
        n = len(self.forms)
        fa = (ctypes.c_void_p * n)(*[f._h.value for f in self.forms])
        xa = (ctypes.c_void_p * n)(*[_dev_ptr(x).value for x in xs])
        ya = (ctypes.c_void_p * n)(*[_dev_ptr(y).value for y in ys])
        _check(_par_lib().ecm2_par_group_mult(ctypes.cast(fa, ctypes.c_void_p), n, ctypes.cast(xa, ctypes.c_void_p),
                                              ctypes.cast(ya, ctypes.c_void_p), _stream(stream)))

    def MultRccl(self, xs, ys, stream=None):
        """Mult with every exchange row sent through RCCL (a one-rank communicator to itself)."""
        n = len(self.forms)
        fa = (ctypes.c_void_p * n)(*[f._h.value for f in self.forms])
        xa = (ctypes.c_void_p * n)(*[_dev_ptr(x).value for x in xs])
        ya = (ctypes.c_void_p * n)(*[_dev_ptr(y).value for y in ys])
        _check(_par_lib().ecm2_par_group_mult_rccl(ctypes.cast(fa, ctypes.c_void_p), n, ctypes.cast(xa, ctypes.c_void_p),
                                                   ctypes.cast(ya, ctypes.c_void_p), _stream(stream)))

    def MultMember(self, r, xs, ys, stream=None):
        """Member r's rows alone (y[r] only), on the streams and in the stage order one RCCL rank
        uses: what one rank's Mult costs on its own GPU, short of the xGMI transfer."""
        n = len(self.forms)
        fa = (ctypes.c_void_p * n)(*[f._h.value for f in self.forms])
        xa = (ctypes.c_void_p * n)(*[_dev_ptr(x).value for x in xs])
        ya = (ctypes.c_void_p * n)(*[_dev_ptr(y).value for y in ys])
        _check(_par_lib().ecm2_par_group_mult_member(ctypes.cast(fa, ctypes.c_void_p), n, r,
                                                     ctypes.cast(xa, ctypes.c_void_p),
                                                     ctypes.cast(ya, ctypes.c_void_p), _stream(stream)))

    def AssembleDiagonal(self, ds, stream=None):
        n = len(self.forms)
        fa = (ctypes.c_void_p * n)(*[f._h.value for f in self.forms])
        da = (ctypes.c_void_p * n)(*[_dev_ptr(d).value for d in ds])
        _check(_par_lib().ecm2_par_group_diagonal(ctypes.cast(fa, ctypes.c_void_p), n, ctypes.cast(da, ctypes.c_void_p),
                                                  _stream(stream)))

    @property
    def offsets(self):
        """Offsets of the members' true vectors in the group's concatenated true vector."""
        return np.cumsum([0] + [f.true_size for f in self.forms])


class Operator:
    """The solvers' view of a form (the reference's Operator, operator.hpp:24-110): a serial
    BilinearForm, one RCCL rank's ParBilinearForm (collective solvers), or a ParGroup
    (vectors = concatenated true vectors of its members)."""

    def __init__(self, form, member=None):
        """member (ParGroup only): that member alone as one rank's operator on its own GPU
        (measurement; ecm2_operator_from_par_member)."""
        lib = _par_lib()
        h = ctypes.c_void_p()
        if member is not None:
            if not isinstance(form, ParGroup):
                raise ECM2Error("member= needs a ParGroup")
            n = len(form.forms)
            fa = (ctypes.c_void_p * n)(*[f._h.value for f in form.forms])
            _check(lib.ecm2_operator_from_par_member(ctypes.cast(fa, ctypes.c_void_p), n, int(member),
                                                     ctypes.byref(h)))
        elif isinstance(form, BilinearForm):
            _check(lib.ecm2_operator_from_pa_form(form._h, ctypes.byref(h)))
        elif isinstance(form, ParBilinearForm):
            _check(lib.ecm2_operator_from_par_form(form._h, ctypes.byref(h)))
        elif isinstance(form, ParGroup):
            n = len(form.forms)
            fa = (ctypes.c_void_p * n)(*[f._h.value for f in form.forms])
            _check(lib.ecm2_operator_from_par_group(ctypes.cast(fa, ctypes.c_void_p), n, ctypes.byref(h)))
        else:
            raise ECM2Error(f"no operator for {type(form).__name__}")
        self._h = h
        self.form = form  # keeps the form(s) alive while the operator exists
        n = ctypes.c_int()
        _check(lib.ecm2_operator_size(h, ctypes.byref(n)))
        self.size = n.value

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ecm2_operator_destroy(self._h)
            self._h = None

    def Mult(self, x, y, stream=None):
        _check(_par_lib().ecm2_operator_mult(self._h, _dev_ptr(x), _dev_ptr(y), _stream(stream)))

    def PCG(self, b, x, ess=None, rel_tol=1e-12, abs_tol=0.0, max_iter=1000, jacobi=True, stream=None):
        """ConstrainedOperator(DIAG_ONE) + CGSolver(+OperatorJacobiSmoother); returns (iters, final_norm)."""
        it, nrm = ctypes.c_int(), ctypes.c_double()
        n_ess = 0 if ess is None else int(ess.numel())
        _check(_par_lib().ecm2_operator_pcg(self._h, _dev_ptr(ess) if n_ess else None, n_ess, _dev_ptr(b), _dev_ptr(x),
                                            rel_tol, abs_tol, max_iter, 1 if jacobi else 0,
                                            ctypes.byref(it), ctypes.byref(nrm), _stream(stream)))
        return it.value, nrm.value


ODE_BACKWARD_EULER, ODE_SDIRK23_L, ODE_SDIRK33, ODE_IMPLICIT_MIDPOINT, ODE_SDIRK23, ODE_SDIRK34 = 21, 22, 23, 32, 33, 34


def ode_implicit_coeff(ode_type: int) -> float:
    """Stage coefficient c of ODESolver type (ode.cpp:77-91): stages solve (M + c dt K) k = -K u."""
    c = _par_lib().ecm2_ode_implicit_coeff(ode_type)
    if c == 0.0:
        raise ECM2Error(f"unsupported implicit ODE solver type {ode_type}")
    return c


def ode_step(ode_type: int, T: Operator, K: Operator, dt: float, u, ess=None, rel_tol=1e-10, max_iter=500,
             jacobi=True, stream=None):
    """One implicit step of M du/dt = -K u (ex16 ConductionOperator, slope form) on device vector u
    (in place).  T must be M + c dt K with c = ode_implicit_coeff(ode_type).
    Returns (stage solves, total PCG iterations, converged)."""
    ns, it, conv = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    n_ess = 0 if ess is None else int(ess.numel())
    _check(_par_lib().ecm2_ode_step(ode_type, T._h, K._h, dt, _dev_ptr(u), _dev_ptr(ess) if n_ess else None, n_ess,
                                    rel_tol, max_iter, 1 if jacobi else 0, ctypes.byref(ns), ctypes.byref(it),
                                    ctypes.byref(conv), _stream(stream)))
    return ns.value, it.value, bool(conv.value)
