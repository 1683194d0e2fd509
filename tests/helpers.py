"""Test helpers: coefficient functions and mesh fixtures shared by CPU and GPU tests.

Coefficients restate tests/unit/fem/test_pa_coeff.cpp:45-58 (coeffFunction) and the
non-aligned Cartesian mesh of test_pa_coeff.cpp:22-42; the bioheat coefficients
follow SURVEY §8(d) (alpha = rho*c_eff, beta = gamma*dt*k(T)).
"""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

# Relative tolerance of every FP64 parity check: ||y - y_ref||_inf / ||y_ref||_inf.
RTOL = 1e-12


def nonaligned(V):
    """MakeCartesianNonaligned vertex remap (test_pa_coeff.cpp:33-39)."""
    V = np.array(V, dtype=np.float64, copy=True)
    V[:, 1] += 0.2 * V[:, 0]
    V[:, 2] += 0.3 * V[:, 0]
    return V


def coeff_function(P):
    """coeffFunction, 3D branch (test_pa_coeff.cpp:45-58)."""
    return np.sin(8.0 * np.pi * P[..., 0]) * np.cos(6.0 * np.pi * P[..., 1]) * np.sin(4.0 * np.pi * P[..., 2]) + 2.0


def alpha_bioheat(P):
    """rho*c_eff = 3.6e6 (1 + 0.1 sin 3x)  [J/(m^3 K)], heat capacity + gamma*dt*w_b*c_b folded in."""
    return 3.6e6 * (1.0 + 0.1 * np.sin(3.0 * P[..., 0]))


def temperature(P):
    """T = 37 + 20 exp(-10 |p|^2) (ablation hot spot)."""
    return 37.0 + 20.0 * np.exp(-10.0 * np.sum(P * P, axis=-1))


def k_of_T(T):
    """Pennes conductivity law k(T) = 0.5 (1 + 0.0012 (T - 37))."""
    return 0.5 * (1.0 + 0.0012 * (T - 37.0))


def relerr(y, yref):
    y, yref = np.asarray(y), np.asarray(yref)
    den = np.abs(yref).max()
    return float(np.abs(y - yref).max() / (den if den > 0 else 1.0))


def read_mfem_mesh(path):
    """Independent numpy parser of an MFEM v1.0 hex mesh (for the reference's data fixtures).

    Returns (vertices [nv][3], elements [ne][8] native order)."""
    lines = []
    for raw in open(path):
        s = raw.split("#")[0].strip()
        if s:
            lines.append(s)
    assert lines[0].startswith("MFEM mesh v1.0")
    i, V, E = 1, None, None
    while i < len(lines):
        key = lines[i]
        if key == "elements":
            n = int(lines[i + 1])
            E = np.array([[int(t) for t in lines[i + 2 + k].split()[2:]] for k in range(n)], np.int32)
            i += 2 + n
        elif key == "boundary":
            n = int(lines[i + 1])
            i += 2 + n
        elif key == "vertices":
            n = int(lines[i + 1])
            V = np.array([[float(t) for t in lines[i + 3 + k].split()] for k in range(n)])
            i += 3 + n
        else:
            i += 1
    return V, E


LEX_TO_NATIVE = [0, 1, 3, 2, 4, 5, 7, 6]


def element_nodes_from(V, E):
    """Lexicographic corner coordinates [ne][3][8] from native-order elements."""
    en = np.empty((E.shape[0], 3, 8))
    for a in range(8):
        en[:, :, a] = V[E[:, LEX_TO_NATIVE[a]]]
    return en


def load_pkg():
    """Register the package (directory name has hyphens) as `ecm2_amd`; idempotent."""
    if "ecm2_amd" in sys.modules:
        return sys.modules["ecm2_amd"]
    pkg_dir = os.path.join(ROOT, "cardiac-ablation-ecm2_amd")
    spec = importlib.util.spec_from_file_location("ecm2_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ecm2_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


for _d in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if _d not in sys.path:
        sys.path.insert(0, _d)
load_pkg()


def vector_coeff_function(P):
    """vectorCoeffFunction, 3D (test_pa_coeff.cpp:58-70): [..., 3]."""
    return np.stack([np.sin(np.pi * P[..., 1]), np.sin(2.5 * np.pi * P[..., 0]), np.sin(6.1 * np.pi * P[..., 2])], -1)


def symmetric_matrix_coeff_function(P):
    """symmetricMatrixCoeffFunction, 3D (test_pa_coeff.cpp:105-125): (11,12,13,22,23,33) [..., 6]."""
    x, y, z = P[..., 0], P[..., 1], P[..., 2]
    return np.stack([np.sin(np.pi * y), np.cos(2.5 * np.pi * x), np.sin(4.9 * np.pi * z),
                     np.sin(6.1 * np.pi * y), np.cos(6.1 * np.pi * z), np.sin(6.1 * np.pi * z)], -1)


def asymmetric_matrix_coeff_function(P):
    """asymmetricMatrixCoeffFunction, 3D (test_pa_coeff.cpp:84-103): row-major M(i, j) [..., 9]."""
    x, y, z = P[..., 0], P[..., 1], P[..., 2]
    return np.stack([1.1 + np.sin(np.pi * y), np.cos(2.5 * np.pi * x), np.sin(4.9 * np.pi * z),
                     np.cos(np.pi * x), 1.1 + np.sin(6.1 * np.pi * y), np.cos(6.1 * np.pi * z),
                     np.sin(1.5 * np.pi * y), np.cos(2.9 * np.pi * x), 1.1 + np.sin(6.1 * np.pi * z)], -1)


def anisotropic_coefficients(P, ctype, seed=0):
    """test_pa_coeff.cpp coeffType 3..6: (values, dim) -- 3 vector function, 4 symmetric matrix
    function, 5 asymmetric matrix function, 6 a constant random matrix with 2 added on its diagonal."""
    if ctype == 3:
        return vector_coeff_function(P), 3
    if ctype == 4:
        return symmetric_matrix_coeff_function(P), 6
    if ctype == 5:
        return asymmetric_matrix_coeff_function(P), 9
    m = np.random.default_rng(seed).uniform(0, 1, (3, 3)) + 2.0 * np.eye(3)
    return m.reshape(9), 9
