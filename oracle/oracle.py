"""oracle.py -- ctypes wrapper of the C restatement (pa_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / the timed CPU "port",
never by the product path.  See pa_oracle.c for the reference citations and
DESIGN.md ("Oracle") for how the restatement is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    _KEEP.clear()  # lib() is evaluated before the arguments of each call expression
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        i32, f64, vp = ctypes.c_int, ctypes.c_double, ctypes.c_void_p
        sig = {
            "orc_gauss_legendre": (None, [i32, vp, vp]),
            "orc_gauss_lobatto": (None, [i32, vp, vp]),
            "orc_basis_eval": (None, [i32, vp, f64, vp, vp]),
            "orc_dof_to_quad": (None, [i32, i32, vp, vp]),
            "orc_cube_weights": (None, [i32, vp]),
            "orc_default_q1d": (i32, [i32]),
            "orc_geom": (None, [i32, i32, vp, vp, vp, vp]),
            "orc_diffusion_setup": (None, [i32, i32, vp, vp, vp, i32, vp]),
            "orc_mass_setup": (None, [i32, i32, vp, vp, vp, i32, vp]),
            "orc_interp_evector": (None, [i32, i32, i32, vp, vp]),
            "orc_mass_apply": (None, [i32, i32, i32, vp, vp, vp, vp]),
            "orc_diffusion_apply": (None, [i32, i32, i32, vp, vp, vp, vp, vp]),
            "orc_restriction_mult": (None, [i32, i32, vp, vp, vp]),
            "orc_restriction_build_csr": (None, [i32, i32, i32, vp, vp, vp]),
            "orc_restriction_mult_transpose": (None, [i32, vp, vp, vp, vp]),
            "orc_pa_mult": (None, [i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
            "orc_fa_mult": (None, [i32, i32, i32, vp, vp, i32, vp, i32, vp, i32, vp, vp, vp]),
            "orc_pa_diagonal_e": (None, [i32, i32, i32, vp, vp, vp, vp, vp]),
            "orc_diffusion_setup_m": (i32, [i32, i32, vp, vp, vp, i32, i32, vp]),
            "orc_diffusion_apply_n": (None, [i32, i32, i32, vp, vp, vp, i32, vp, vp]),
            "orc_pa_diagonal_e_n": (None, [i32, i32, i32, vp, vp, vp, vp, i32, vp]),
            "orc_fa_mult_m": (None, [i32, i32, i32, vp, vp, i32, vp, i32, vp, i32, i32, vp, vp, vp]),
            "orc_pcg": (i32, [i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp,
                              f64, f64, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
            "orc_num_threads": (i32, []),
        }
        for n, (r, a) in sig.items():
            f = getattr(_lib, n)
            f.restype, f.argtypes = r, a
    return _lib


_KEEP = []


def _p(a):
    """Pointer to a numpy array; the array is kept alive until the next _release()
    (a bare c_void_p does not hold a reference, so temporaries would be freed)."""
    if a is None:
        return None
    _KEEP.append(a)
    return ctypes.c_void_p(a.ctypes.data)


def _release():
    _KEEP.clear()


def _f64(a):
    return np.ascontiguousarray(a, np.float64)


def _i32(a):
    return np.ascontiguousarray(a, np.int32)


# ---- 1D tables --------------------------------------------------------------
def gauss_legendre(n):
    x, w = np.empty(n), np.empty(n)
    lib().orc_gauss_legendre(n, _p(x), _p(w))
    return x, w


def gauss_lobatto(n):
    x, w = np.empty(n), np.empty(n)
    lib().orc_gauss_lobatto(n, _p(x), _p(w))
    return x, w


def basis_eval(p, nodes, y):
    nodes = _f64(nodes)
    u, d = np.empty(p + 1), np.empty(p + 1)
    lib().orc_basis_eval(p, _p(nodes), float(y), _p(u), _p(d))
    return u, d


def default_q1d(p):
    return lib().orc_default_q1d(p)


def dof_to_quad(p, q1d):
    """B, G as [Q, D] arrays (B[q, d] = B[q + Q*d] of the reference)."""
    B = np.empty(q1d * (p + 1))
    G = np.empty(q1d * (p + 1))
    lib().orc_dof_to_quad(p, q1d, _p(B), _p(G))
    return B.reshape(p + 1, q1d).T.copy(), G.reshape(p + 1, q1d).T.copy()


def cube_weights(q1d):
    W = np.empty(q1d ** 3)
    lib().orc_cube_weights(q1d, _p(W))
    return W


# ---- independent structured mesh (oracle-side) ------------------------------
def cartesian_mesh(nx, ny, nz, sx=1.0, sy=1.0, sz=1.0, order=2, transform=None):
    """Cartesian hex mesh with lattice dof numbering, built independently of the product.

    Returns (enodes [ne][3][8] lexicographic corners, gather_map [ne][nd], ndofs,
    dof_coords [ndofs][3]).  Element order is lexicographic (Make3D, mesh.cpp:3777-3790).
    transform(xyz)->xyz (vectorised) maps vertices (e.g. the non-aligned mesh of
    test_pa_coeff.cpp:22-42)."""
    p, D = order, order + 1
    ix, iy, iz = np.meshgrid(np.arange(nx + 1), np.arange(ny + 1), np.arange(nz + 1), indexing="ij")
    V = np.stack([ix / nx * sx, iy / ny * sy, iz / nz * sz], axis=-1)  # [nx+1,ny+1,nz+1,3]
    if transform is not None:
        V = transform(V.reshape(-1, 3)).reshape(V.shape)
    ex, ey, ez = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij")
    ex, ey, ez = (a.transpose(2, 1, 0).ravel() for a in (ex, ey, ez))  # x fastest
    ne = nx * ny * nz
    enodes = np.empty((ne, 3, 8))
    for a in range(8):
        ax, ay, az = a & 1, (a >> 1) & 1, a >> 2
        enodes[:, :, a] = V[ex + ax, ey + ay, ez + az, :]
    NX, NY, NZ = p * nx + 1, p * ny + 1, p * nz + 1
    gm = np.empty((ne, D ** 3), np.int32)
    for k in range(D):
        for j in range(D):
            for i in range(D):
                gm[:, (k * D + j) * D + i] = (p * ex + i) + NX * ((p * ey + j) + NY * (p * ez + k))
    ndofs = NX * NY * NZ
    nodes, _ = gauss_lobatto(D)
    coords = np.zeros((ndofs, 3))
    for k in range(D):
        for j in range(D):
            for i in range(D):
                xi = (nodes[i], nodes[j], nodes[k])
                pt = np.zeros((ne, 3))
                for a in range(8):
                    ax, ay, az = a & 1, (a >> 1) & 1, a >> 2
                    N = (xi[0] if ax else 1 - xi[0]) * (xi[1] if ay else 1 - xi[1]) * (xi[2] if az else 1 - xi[2])
                    pt += N * enodes[:, :, a]
                coords[gm[:, (k * D + j) * D + i]] = pt
    return enodes, gm, ndofs, coords


# ---- geometry / setup -------------------------------------------------------
def geom(enodes, q1d):
    enodes = _f64(enodes)
    ne = enodes.shape[0]
    nq = q1d ** 3
    X = np.empty((ne, 3, nq))
    J = np.empty((ne, 3, 3, nq))   # [e][j][i][q]
    detJ = np.empty((ne, nq))
    lib().orc_geom(ne, q1d, _p(enodes), _p(X), _p(J), _p(detJ))
    return X, J, detJ


def _coef(c, ne, nq):
    if np.isscalar(c):
        return np.array([float(c)]), 1
    c = _f64(c)
    assert c.size == ne * nq
    return c, 0


def diffusion_setup(J, W, coef, q1d):
    ne, nq = J.shape[0], q1d ** 3
    c, cc = _coef(coef, ne, nq)
    D = np.empty((ne, 6, nq))
    lib().orc_diffusion_setup(ne, q1d, _p(_f64(W)), _p(_f64(J)), _p(c), cc, _p(D))
    return D


def mass_setup(detJ, W, coef, q1d):
    ne, nq = detJ.shape[0], q1d ** 3
    c, cc = _coef(coef, ne, nq)
    M = np.empty((ne, nq))
    lib().orc_mass_setup(ne, q1d, _p(_f64(W)), _p(_f64(detJ)), _p(c), cc, _p(M))
    return M


def interp_evector(xe, p, q1d):
    xe = _f64(xe)
    ne = xe.shape[0]
    out = np.empty((ne, q1d ** 3))
    lib().orc_interp_evector(ne, p, q1d, _p(xe), _p(out))
    return out


# ---- restriction ------------------------------------------------------------
def restriction_mult(gm, x):
    gm = _i32(gm)
    ne, nd = gm.shape
    xe = np.empty((ne, nd))
    lib().orc_restriction_mult(ne, nd, _p(gm), _p(_f64(x)), _p(xe))
    return xe


def build_csr(gm, ndofs):
    gm = _i32(gm)
    ne, nd = gm.shape
    off = np.empty(ndofs + 1, np.int32)
    idx = np.empty(ne * nd, np.int32)
    lib().orc_restriction_build_csr(ne, nd, ndofs, _p(gm), _p(off), _p(idx))
    return off, idx


def restriction_mult_transpose(off, idx, ye):
    ndofs = off.size - 1
    y = np.empty(ndofs)
    lib().orc_restriction_mult_transpose(ndofs, _p(_i32(off)), _p(_i32(idx)), _p(_f64(ye)), _p(y))
    return y


def mass_apply(B, M, xe):
    Q, D = B.shape
    ne = xe.shape[0]
    Bf = _f64(B.T.ravel())  # B[q + Q*d]
    ye = np.zeros_like(_f64(xe))
    lib().orc_mass_apply(ne, D, Q, _p(Bf), _p(_f64(M)), _p(_f64(xe)), _p(ye))
    return ye


def diffusion_apply(B, G, Dd, xe):
    Q, D = B.shape
    ne = xe.shape[0]
    ye = np.zeros_like(_f64(xe))
    lib().orc_diffusion_apply(ne, D, Q, _p(_f64(B.T.ravel())), _p(_f64(G.T.ravel())), _p(_f64(Dd)),
                              _p(_f64(xe)), _p(ye))
    return ye


def diffusion_setup_m(J, W, coef, cdim, q1d):
    """PADiffusionSetup3D for a vector / matrix coefficient (cdim 3, 6, 9): coef [ne][nq][cdim] or
    the cdim constant values; returns D [ne][nD][nq], nD = 9 (general) or 6 (symmetric)."""
    ne, nq = J.shape[0], q1d ** 3
    c = _f64(coef)
    const = 1 if c.size == cdim else 0
    assert const or c.size == ne * nq * cdim
    D = np.empty((ne, 9 if cdim == 9 else 6, nq))
    lib().orc_diffusion_setup_m(ne, q1d, _p(_f64(W)), _p(_f64(J)), _p(c), cdim, const, _p(D))
    return D


def diffusion_apply_n(B, G, Dd, xe):
    """The diffusion AddMultPA on 6- or 9-entry qdata (Dd [ne][nD][nq])."""
    Q, D = B.shape
    ne = xe.shape[0]
    ye = np.zeros_like(_f64(xe))
    lib().orc_diffusion_apply_n(ne, D, Q, _p(_f64(B.T.ravel())), _p(_f64(G.T.ravel())), _p(_f64(Dd)), Dd.shape[1],
                                _p(_f64(xe)), _p(ye))
    return ye


class OracleOperator:
    """y = R^T (M_alpha + K_beta) R x on the CPU (the reference's PA path, restated).

    alpha / beta: scalar, per-quadrature array [ne][nq], or None (integrator absent).
    beta_dim 3 / 6 / 9: beta is a vector / symmetric matrix (11,12,13,22,23,33) / general matrix
    (row-major) coefficient, [ne][nq][beta_dim] or its beta_dim constant values."""

    def __init__(self, enodes, gm, ndofs, order, alpha=None, beta=None, q1d=None, beta_dim=1):
        self.enodes = _f64(enodes)
        self.gm = _i32(gm)
        self.ne = self.gm.shape[0]
        self.ndofs = int(ndofs)
        self.p = order
        self.q1d = q1d or default_q1d(order)
        self.B, self.G = dof_to_quad(order, self.q1d)
        self.W = cube_weights(self.q1d)
        X, J, detJ = geom(self.enodes, self.q1d)
        self.X, self.J, self.detJ = X, J, detJ
        self.alpha, self.beta = alpha, beta
        self.M = mass_setup(detJ, self.W, alpha, self.q1d) if alpha is not None else None
        self.beta_dim = beta_dim
        if beta is None:
            self.D = None
        elif beta_dim == 1:
            self.D = diffusion_setup(J, self.W, beta, self.q1d)
        else:
            self.D = diffusion_setup_m(J, self.W, beta, beta_dim, self.q1d)
        self.off, self.idx = build_csr(self.gm, self.ndofs)
        nd = self.gm.shape[1]
        self._xe = np.empty((self.ne, nd))
        self._ye = np.empty((self.ne, nd))
        self._Bf = _f64(self.B.T.ravel())
        self._Gf = _f64(self.G.T.ravel())

    @classmethod
    def from_jacobians(cls, J, gm, ndofs, order, alpha=None, beta=None, q1d=None):
        """The same operator on a mesh given by its Jacobians at the quadrature points -- J [ne][3 (j)][3 (i)]
        [nq], GeometricFactors::JACOBIANS' memory order (mesh.cpp:15220-15273) -- e.g. a curved mesh whose
        high-order nodes the test turned into J; the setups are PADiffusionSetup3D / the mass setup on
        that J (bilininteg_diffusion_kernels.cpp:243-367, bilininteg_mass_pa.cpp:60-78)."""
        self = cls.__new__(cls)
        self.gm = _i32(gm)
        self.ne = self.gm.shape[0]
        self.ndofs = int(ndofs)
        self.p = order
        self.q1d = q1d or default_q1d(order)
        self.B, self.G = dof_to_quad(order, self.q1d)
        self.W = cube_weights(self.q1d)
        J = _f64(J)
        assert J.shape == (self.ne, 3, 3, self.q1d ** 3)
        self.enodes, self.X, self.J = None, None, J
        self.detJ = np.ascontiguousarray(np.linalg.det(np.transpose(J, (0, 3, 2, 1))))  # det of J[i][j]
        self.alpha, self.beta, self.beta_dim = alpha, beta, 1
        self.M = mass_setup(self.detJ, self.W, alpha, self.q1d) if alpha is not None else None
        self.D = diffusion_setup(J, self.W, beta, self.q1d) if beta is not None else None
        self.off, self.idx = build_csr(self.gm, self.ndofs)
        nd = self.gm.shape[1]
        self._xe = np.empty((self.ne, nd))
        self._ye = np.empty((self.ne, nd))
        self._Bf = _f64(self.B.T.ravel())
        self._Gf = _f64(self.G.T.ravel())
        return self

    def mult(self, x):
        if self.D is not None and self.D.shape[1] == 9:  # MultInternal with the general qdata
            xe = restriction_mult(self.gm, x)
            ye = diffusion_apply_n(self.B, self.G, self.D, xe)
            if self.M is not None:
                ye += mass_apply(self.B, self.M, xe)
            return restriction_mult_transpose(self.off, self.idx, ye)
        y = np.empty(self.ndofs)
        lib().orc_pa_mult(self.ne, self.p, self.q1d, self.ndofs, _p(self.gm), _p(self.off), _p(self.idx),
                          _p(self._Bf), _p(self._Gf), _p(self.M), _p(self.D), _p(_f64(x)), _p(y),
                          _p(self._xe), _p(self._ye))
        return y

    def mult_markers(self, x, attr, mass_marker=None, diff_marker=None):
        """MultInternal with attribute markers (bilinearform_ext.cpp:527-560 + AddMultWithMarkers
        :807-847, AddWithMarkers_ :753-774): each integrator's AddMultPA into a zeroed E-vector,
        added element by element where attr > 0 and marker[attr - 1] != 0 (no marker: all)."""
        attr = np.asarray(attr)
        xe = restriction_mult(self.gm, x)
        ye = np.zeros_like(xe)
        for marker, app in ((mass_marker, self.M is not None and (lambda v: mass_apply(self.B, self.M, v))),
                            (diff_marker, self.D is not None and (lambda v: diffusion_apply(self.B, self.G, self.D, v)))):
            if not app:
                continue
            tmp = app(xe)
            if marker is None:
                ye += tmp
                continue
            mk = np.asarray(marker)
            keep = np.array([a > 0 and mk[a - 1] != 0 for a in attr])
            ye[keep] += tmp[keep]
        return restriction_mult_transpose(self.off, self.idx, ye)

    def fa_mult(self, x, with_diag=False):
        """Legacy element-matrix assembly path (independent of sum factorisation)."""
        y = np.empty(self.ndofs)
        diag = np.empty(self.ndofs) if with_diag else None
        am, amc = _coef(self.alpha, self.ne, self.q1d ** 3) if self.alpha is not None else (None, 0)
        if self.beta is not None and self.beta_dim > 1:
            bd = _f64(self.beta)
            bdc = 1 if bd.size == self.beta_dim else 0
        else:
            bd, bdc = _coef(self.beta, self.ne, self.q1d ** 3) if self.beta is not None else (None, 0)
        lib().orc_fa_mult_m(self.ne, self.p, self.q1d, _p(self.enodes), _p(self.gm), self.ndofs,
                            _p(am), amc, _p(bd), self.beta_dim, bdc, _p(_f64(x)), _p(y), _p(diag))
        return (y, diag) if with_diag else y

    def diagonal(self):
        nd = self.gm.shape[1]
        de = np.zeros((self.ne, nd))
        Q = self.q1d
        nD = self.D.shape[1] if self.D is not None else 6
        lib().orc_pa_diagonal_e_n(self.ne, self.p + 1, Q, _p(self._Bf), _p(self._Gf), _p(self.M), _p(self.D), nD,
                                  _p(de))
        return np.bincount(self.gm.ravel(), weights=de.ravel(), minlength=self.ndofs)

    def diagonal_markers(self, attr, integrators):
        """PABilinearFormExtension::AssembleDiagonal with markers (bilinearform_ext.cpp:370-411):
        localY = 0; for each (kind, marker) in AddDomainIntegrator order, the integrator's
        AssembleDiagonalPA adds into localY, then a marked integrator zeroes the elements it
        excludes in that SHARED localY (earlier integrators' contributions there included);
        finally AbsMultTranspose.  integrators: [("mass" | "diffusion", marker or None), ...]."""
        attr = np.asarray(attr)
        nd = self.gm.shape[1]
        de = np.zeros((self.ne, nd))
        Q = self.q1d
        for kind, marker in integrators:
            Dm = self.M if kind == "mass" else None
            Dd = self.D if kind == "diffusion" else None
            lib().orc_pa_diagonal_e(self.ne, self.p + 1, Q, _p(self._Bf), _p(self._Gf), _p(Dm), _p(Dd), _p(de))
            if marker is not None:
                mk = np.asarray(marker)
                drop = np.array([not (a > 0 and mk[a - 1] != 0) for a in attr])
                de[drop] = 0.0
        return np.bincount(self.gm.ravel(), weights=de.ravel(), minlength=self.ndofs)

    def pcg(self, b, ess, rel_tol=1e-12, abs_tol=0.0, max_iter=1000, jacobi=True):
        ess = _i32(ess)
        dinv = None
        if jacobi:
            d = self.diagonal()
            d[ess] = 1.0
            dinv = 1.0 / d
        x = np.empty(self.ndofs)
        fn = ctypes.c_double()
        st = ctypes.c_int()
        it = lib().orc_pcg(self.ne, self.p, self.q1d, self.ndofs, _p(self.gm), _p(self.off), _p(self.idx),
                           _p(self._Bf), _p(self._Gf), _p(self.M), _p(self.D), _p(ess), ess.size,
                           _p(dinv), _p(_f64(b)), _p(x), rel_tol, abs_tol, max_iter, ctypes.byref(fn),
                           ctypes.byref(st))
        # CGSolver's outcome: 1 converged, 2 max_iter, 3 (B r, r) < 0, 4 (A d, d) == 0, 5 non-finite
        self.last_pcg_status = st.value
        return x, it, fn.value


def quad_points(enodes, q1d):
    """Physical coordinates of the quadrature points, [ne][nq][3]."""
    X, _, _ = geom(enodes, q1d)
    return np.transpose(X, (0, 2, 1)).copy()


def num_threads():
    return lib().orc_num_threads()
