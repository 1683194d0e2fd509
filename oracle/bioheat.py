"""bioheat.py -- CPU restatement of the bioheat coefficient laws (TEST INFRASTRUCTURE ONLY).

Imported by tests/ as the checker of the device coefficient kernels, never by the product.

* Projection of an H1 temperature grid function to the quadrature points: the reference's
  GridFunctionCoefficient -> CoefficientVector::Project (fem/coefficient.cpp:2052-2070) ->
  QuadratureFunction::ProjectGridFunction (fem/qfunction.cpp:73-98), i.e. the E-vector of T
  interpolated with the tensor basis B (oracle.interp_evector).
* The laws composed with it are the bioheat application's (the fork's Pennes
  code is not in the reference snapshot), so their parity is UNPINNED: these functions
  restate the formulas the library documents (include/ecm2_pa.h, ECM2_COEFF_GRIDFUNC_*),
  not reference code.
"""
import numpy as np

import oracle as O


def temperature_at_quadrature(T, gather_map, order, q1d):
    """T(x_q) [ne][nq] of the H1 L-vector T (GridFunctionCoefficient projection)."""
    return O.interp_evector(np.asarray(T)[gather_map], order, q1d)


def affine_law(Tq, scale, slope, t_ref):
    """ECM2_COEFF_GRIDFUNC_AFFINE: scale (1 + slope (T - t_ref)) -- the conductivity
    k(T) = k0 (1 + a (T - T0)) times gamma dt."""
    return scale * (1.0 + slope * (Tq - t_ref))


def perfusion_law(Tq, rho_c, gdt_cb, w0, a, t0, t_stop):
    """ECM2_COEFF_GRIDFUNC_PERFUSION: alpha(T) = rho_c + gdt_cb w_b(T) with
    w_b(T) = w0 max(0, 1 + a (T - t0)) below t_stop, 0 at or above it."""
    r = 1.0 + a * (Tq - t0)
    wb = np.where((Tq < t_stop) & (r > 0.0), w0 * r, 0.0)
    return rho_c + gdt_cb * wb
