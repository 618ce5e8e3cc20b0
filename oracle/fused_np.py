"""Upwind-frame, time-fused numpy restatement -- TEST INFRASTRUCTURE ONLY.

A second, independently derived CPU restatement of the reference's sweep
(src/solver.cpp:319-823), written in the form the MI355X kernel uses:

* every (direction, group) line is stored in its own *upwind frame*: cell
  k = 0 is the inflow cell (physical cell N-1-k for mu < 0), and each cell
  holds (e_in, e_out) = the upwind / downwind node.  With |mu| the 2x2 cell
  systems of BE / CN / BDF become sign-independent (solver.cpp:327-399 vs
  :362-399 etc. are mirror images);
* the four BDF2 substeps of one full step (solver.cpp:721-753) are fused
  per cell: the sweep carries X = (p_up, x_BE0, x_CN, x_BE2, x_BDF), where
  p_up is the previous cell's step-start downwind node (prev_ends of the
  upwind cell, solver.cpp:449/483/542/581) and x_* are the four substeps'
  upwind scalars.  half_ends (solver.cpp:733) is H = CN result for mu < 0
  lines and the BE-predictor result for mu > 0 lines (the last full copy is
  taken after the last mu < 0 CN cell).

It is checked against the loop-order C oracle (rt_oracle.c) in tests; the
two were written independently, so agreement pins the algebra of both.
"""
from __future__ import annotations

import numpy as np

C_LIGHT = 299.79245800


class LineSet:
    """Per-line constants of the lines of one half (mu < 0 or mu > 0)."""

    def __init__(self, mu_signed, sigma, Bg, cor1, cor2, cor3, V, dx, dt, ts_method, use_correction):
        self.mu = np.asarray(mu_signed, dtype=np.float64)
        self.m = np.abs(self.mu)
        self.sigma = np.asarray(sigma, dtype=np.float64)   # rho*kappa
        self.B = np.asarray(Bg, dtype=np.float64)
        self.dx = dx
        self.dt = dt
        self.ts = ts_method
        tau = dt / 2.0 if ts_method == 3 else dt
        self.tau = tau
        c = C_LIGHT
        # emission + correction source S = Sc + Sl * (e_in + e_out) (psi = mean of the nodes)
        half = 0.5 * c * tau * dx
        self.Sc = half * self.sigma * self.B
        if use_correction:
            beta = V / c
            self.Sc = self.Sc + half * ((np.asarray(cor2) * self.mu) * beta - np.asarray(cor3) * self.mu ** 2 * beta ** 2)
            self.Sl = half * np.asarray(cor1) * self.mu * beta * 0.5
        else:
            self.Sl = np.zeros_like(self.m)
        hd = 0.5 * dx
        self.hd = hd
        # BE(tau)  (solver.cpp:319-404)
        a = 1.0 + c * tau * self.sigma
        b = c * tau * self.m
        d = (a * dx + b) / 2.0
        self.be = dict(b=b, inv=self._inv(d, b / 2.0))
        # CN(tau)  (solver.cpp:407-490)
        t = 0.5 * c * tau * self.sigma
        A = 0.5 * c * self.m * tau
        Bp, Cp = 1.0 + t, 1.0 - t
        d = 0.5 * (A + Bp * dx)
        self.cn = dict(A=A, k1=0.5 * (Cp * dx - A), k2=0.5 * A, inv=self._inv(d, A / 2.0))
        # BDF(tau, const_B with the full dt)  (solver.cpp:493-587)
        t = c * self.sigma * tau / 6.0
        Ab = 1.0 + t
        Bc = c * self.m * dt / 6.0
        Cb = 1.0 - 4.0 * t
        D = t
        d = 0.5 * (Ab * dx + Bc)
        self.bdf = dict(Bc=Bc, q1=0.5 * (Cb * dx - 4.0 * Bc), q2=2.0 * Bc, q3=0.5 * (Bc + D * dx), q4=0.5 * Bc,
                        inv=self._inv(d, 0.5 * Bc))

    @staticmethod
    def _inv(d, o):
        # [[d, o], [-o, d]]^-1 = [[d, -o], [o, d]] / (d^2 + o^2)
        det = d * d + o * o
        return (d / det, -o / det, o / det, d / det)

    def source(self, ein, eout):
        return self.Sc + self.Sl * (ein + eout)

    def be_cell(self, ein, eout, x):
        S = self.source(ein, eout)
        r_in = S + self.be["b"] * x + self.hd * ein
        r_out = S + self.hd * eout
        i00, i01, i10, i11 = self.be["inv"]
        return i00 * r_in + i01 * r_out, i10 * r_in + i11 * r_out

    def cn_cell(self, ein, eout, xp, xh):
        S = self.source(ein, eout)
        k1, k2, A = self.cn["k1"], self.cn["k2"], self.cn["A"]
        r_in = S + k1 * ein - k2 * eout + A * (xp + xh)
        r_out = S + k2 * ein + k1 * eout
        i00, i01, i10, i11 = self.cn["inv"]
        return i00 * r_in + i01 * r_out, i10 * r_in + i11 * r_out

    def bdf_cell(self, ein, eout, hin, hout, pin, pout, x, xh, xp):
        S = self.source(ein, eout)
        q = self.bdf
        r_in = S + q["q1"] * hin - q["q2"] * hout - q["q3"] * pin - q["q4"] * pout + q["Bc"] * (x + 4.0 * xh + xp)
        r_out = S + q["q2"] * hin + q["q1"] * hout + q["q4"] * pin - q["q3"] * pout
        i00, i01, i10, i11 = q["inv"]
        return i00 * r_in + i01 * r_out, i10 * r_in + i11 * r_out


def sweep_step(ls: LineSet, E: np.ndarray, bdry: np.ndarray, negative_half: bool) -> np.ndarray:
    """One full step (1 substep for BE/CN, the 4 fused substeps for BDF2) of
    the lines in `ls`, state E (lines, N, 2) in the upwind frame, updated in
    place.  bdry (nsub, lines) are the per-substep inflow values.  Returns the
    per-substep outflow scalars (nsub, lines) = the carried values after the
    last cell (what reflective partners read, solver.cpp:677-684)."""
    L, N, _ = E.shape
    if ls.ts == 1:
        x = bdry[0].copy()
        for k in range(N):
            e_in, e_out = ls.be_cell(E[:, k, 0], E[:, k, 1], x)
            E[:, k, 0], E[:, k, 1] = e_in, e_out
            x = e_out
        return x[None]
    if ls.ts == 2:
        xh = bdry[0].copy()
        pup = bdry[0].copy()
        for k in range(N):
            p_out = E[:, k, 1].copy()
            e_in, e_out = ls.cn_cell(E[:, k, 0], E[:, k, 1], pup, xh)
            E[:, k, 0], E[:, k, 1] = e_in, e_out
            xh, pup = e_out, p_out
        return xh[None]
    # BDF2: X = (pup, x0, xh, x2, x3)
    x0 = bdry[0].copy()
    xh = bdry[1].copy()
    x2 = bdry[2].copy()
    x3 = bdry[3].copy()
    for k in range(N):
        p_in, p_out = E[:, k, 0].copy(), E[:, k, 1].copy()
        if k == 0:
            xp1, xp3, hup = bdry[1], bdry[3], bdry[3]
        else:
            xp1 = xp3 = pup
            hup = xh if negative_half else x0
        e1 = ls.be_cell(p_in, p_out, x0)
        e2 = ls.cn_cell(e1[0], e1[1], xp1, xh)
        h = e2 if negative_half else e1
        e3 = ls.be_cell(e2[0], e2[1], x2)
        e4 = ls.bdf_cell(e3[0], e3[1], h[0], h[1], p_in, p_out, x3, hup, xp3)
        E[:, k, 0], E[:, k, 1] = e4
        x0, xh, x2, x3, pup = e1[1], e2[1], e3[1], e4[1], p_out
    return np.stack([x0, xh, x2, x3])


class FusedSolver:
    """Whole-run driver over the reference's configuration dict (oracle.parse_prm)."""

    def __init__(self, params: dict, mu, B, kappa, cor1, cor2, cor3, psi_source):
        self.p = params
        M, G, N = params["M"], params["G"], params["N"]
        self.M, self.G, self.N = M, G, N
        self.mu = np.asarray(mu)
        h = M // 2
        # line l = i' + h*g within a half; i' counts |mu| upwards from the centre
        self.idx = {}
        for half in (0, 1):
            ii = [(h - 1 - ip) if half == 0 else (h + ip) for ip in range(h)]
            I = np.array([[i for i in ii] for _ in range(G)]).ravel()          # (G*h,) direction
            Gi = np.repeat(np.arange(G), h)                                    # group
            self.idx[half] = (I, Gi)
        sigma = params["rho"] * np.asarray(kappa)
        ts = params["ts_method"]
        self.nsub = 4 if ts == 3 else 1
        self.lines = {}
        self.E = {}
        for half in (0, 1):
            I, Gi = self.idx[half]
            self.lines[half] = LineSet(self.mu[I], sigma[Gi], np.asarray(B)[Gi], np.asarray(cor1)[Gi],
                                       np.asarray(cor2)[Gi], np.asarray(cor3)[Gi], params["V"], params["dx"],
                                       params["dt"], ts, bool(params["use_correction"]))
            self.E[half] = np.repeat(np.asarray(B)[Gi][:, None, None], N, axis=1).repeat(2, axis=2).astype(np.float64)
        self.psi_source = np.asarray(psi_source)  # (M, G)

    def step(self):
        p = self.p
        nsub = self.nsub
        # mu < 0 lines: right boundary (solver.cpp:639-664)
        I, Gi = self.idx[0]
        if p["bc_right"] == 1:
            b = self.psi_source[I, Gi]
        else:
            b = np.zeros(len(I))
        out_neg = sweep_step(self.lines[0], self.E[0], np.repeat(b[None], nsub, axis=0), True)
        # mu > 0 lines: left boundary (solver.cpp:665-692; 0 falls through to source)
        I, Gi = self.idx[1]
        if p["bc_left"] == 2:
            bd = out_neg  # same (i', g) ordering in both halves
        else:
            bd = np.repeat(self.psi_source[I, Gi][None], nsub, axis=0)
        sweep_step(self.lines[1], self.E[1], bd, False)

    def ends(self) -> np.ndarray:
        """(M, G, N, 2) in the reference's physical frame."""
        M, G, N = self.M, self.G, self.N
        out = np.empty((M, G, N, 2))
        for half in (0, 1):
            I, Gi = self.idx[half]
            E = self.E[half]
            if half == 0:   # physical cell c = N-1-k; e_in is the right node
                out[I, Gi, :, 1] = E[:, ::-1, 0]
                out[I, Gi, :, 0] = E[:, ::-1, 1]
            else:
                out[I, Gi, :, 0] = E[:, :, 0]
                out[I, Gi, :, 1] = E[:, :, 1]
        return out
