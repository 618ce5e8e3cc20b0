"""Parity metrics shared by the tests (tolerances are stated where used).

All comparisons are normalised per energy group: groups span ~1e-10..1e1 in
magnitude (Planck spectrum), so a global relative error would hide errors in
the faint groups.
"""
import numpy as np


def per_group_rel(a, b, group_axis):
    """max_g  max|a - b| over group g / max|b| over group g."""
    a = np.moveaxis(np.asarray(a, dtype=np.float64), group_axis, 0)
    b = np.moveaxis(np.asarray(b, dtype=np.float64), group_axis, 0)
    G = a.shape[0]
    num = np.abs(a - b).reshape(G, -1).max(axis=1)
    den = np.abs(b).reshape(G, -1).max(axis=1)
    den = np.where(den > 0, den, 1.0)
    return float((num / den).max())


def flux_rel(F_a, F_b, psi_ref, mu, wt):
    """F = sum_i mu_i w_i psi_i cancels to ~0 in equilibrium, so its error is
    measured against the scale of the summands: max_c sum_i |mu_i w_i psi_i|
    per group."""
    scale = np.einsum("i,igc->gc", np.abs(mu * wt), np.abs(psi_ref)).max(axis=1)
    scale = np.where(scale > 0, scale, 1.0)
    return float((np.abs(F_a - F_b).max(axis=1) / scale).max())
