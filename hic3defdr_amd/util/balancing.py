"""Knight-Ruiz matrix balancing for the simulated replicates (reference
hic3defdr/util/balancing.py:5-208; algorithm: Knight & Ruiz, IMA J. Numer.
Anal. 2013, with Juicer's "sum factor" rescale), used before a simulated
data set is analysed (README.md:586-614).

Host code (scipy.sparse), off the hot path: a few hundred sparse mat-vecs
per matrix. Organised as a Newton outer iteration (`_KR.solve`) around a
box-constrained conjugate-gradient inner solve (`_KR.inner`); the arithmetic
(the (n, 1) column shapes, the order of the products and the clamps) is the
published one the reference transcribes, so the bias vectors agree with the
reference's to rounding (tests/test_simulation.py pins them at 1e-9)."""
import numpy as np
import scipy.sparse as sparse


def _symmetrised(array):
    """The symmetric matrix of the upper triangle of `array` (CSR)."""
    up = sparse.triu(sparse.csr_matrix(array))
    return (up + up.transpose() - sparse.diags([up.diagonal()], [0])).tocsr()


def _col_dot(a, b):
    # inner product of two (n, 1) columns as a (1, 1) matrix product
    return np.dot(a.T, b)


class _KR(object):
    """State of one balancing run on the non-empty rows `A` of the matrix."""

    def __init__(self, A, x0, tol, lo, hi, verbose):
        self.A = A
        self.lo, self.hi = lo, hi
        self.verbose = verbose
        self.target = tol ** 2           # stop once |1 - x (A x)|^2 <= target
        self.floor_eta = 0.5 * tol
        self.x = np.ones((A.shape[0], 1)) if x0 is None else x0
        self.history = []

    def _scaled_rowsums(self):
        self.v = self.x * self.A.dot(self.x)
        self.r = 1 - self.v
        return float(_col_dot(self.r, self.r)[0, 0])

    def _hit_box(self, y, step, y_try):
        """CG left the box [lo, hi]: the largest multiple of `step` that
        keeps y inside (None: stay inside, continue)."""
        if np.min(y_try) <= self.lo:
            if self.lo == 0:
                return y
            down = np.where(step < 0)
            return y + np.min((self.lo - y[down]) / step[down]) * step
        if np.max(y_try) >= self.hi:
            up = np.where(y_try > self.hi)
            # the builtin min, as the transcription (the values are 1-D here)
            return y + min((self.hi - y[up]) / step[up]) * step
        return None

    def inner(self, rho, tol_in):
        """Preconditioned CG on (diag(x) A diag(x) + diag(v)) y = 1 from
        y = 1; returns (y, the inner iterations, the last rho)."""
        x, v, A = self.x, self.v, self.A
        y = np.ones_like(x)
        k, rho_prev, p = 0, None, None
        z = None
        while rho > tol_in:
            k += 1
            if k == 1:
                z = self.r / v
                p = z.copy()
                rho = _col_dot(self.r, z)
            else:
                p = z + (rho / rho_prev) * p
            w = x * A.dot(x * p) + v * p
            alpha = rho / _col_dot(p, w)
            step = alpha * p
            y_try = y + step
            clamped = self._hit_box(y, step, y_try)
            if clamped is not None:
                return clamped, k, rho
            y = y_try
            self.r = self.r - alpha * w
            rho_prev = rho
            z = self.r / v
            rho = _col_dot(self.r, z)
        return y, k, rho

    def solve(self, max_iter):
        g, eta_cap = 0.9, 0.1
        eta = eta_cap
        rho = self._scaled_rowsums()
        res_sq = res_prev = rho
        if self.verbose:
            print('it in. it res')
        outer = 0
        while res_sq > self.target:
            if max_iter is not None and outer > max_iter:
                break
            outer += 1
            y, k, rho = self.inner(rho, max(eta ** 2 * res_sq, self.target))
            self.x = self.x * y
            rho = self._scaled_rowsums()
            res_sq = rho
            ratio, res_prev = res_sq / res_prev, res_sq
            norm = np.sqrt(res_sq)
            # forcing term of the inexact Newton step (Eisenstat-Walker)
            eta_last, eta = eta, g * ratio
            if g * eta_last ** 2 > 0.1:
                eta = max(eta, g * eta_last ** 2)
            eta = max(min(eta, eta_cap), self.floor_eta / norm)
            if self.verbose:
                print('{} {} {:.3e}'.format(outer, k, norm))
                self.history.append(norm)
        return self.x


def kr_balance(array, tol=1e-6, x0=None, delta=0.1, ddelta=3, fl=1,
               max_iter=3000):
    """Returns (balanced CSR, bias, residual norms) as the reference
    (balancing.py:5-208): `array` is symmetrised from its upper triangle,
    empty rows sit out the iteration and get bias 0, the scaling vector is
    rescaled so the balanced matrix keeps the original total, and bias is
    its inverse. The balanced matrix is upper triangular when the input
    was; fl == 1 prints the convergence table."""
    upper_input = sparse.tril(array, k=-1).nnz == 0
    full = _symmetrised(array)
    rows = full.getnnz(1) > 0
    kr = _KR(full[rows, :][:, rows], x0, tol, delta, ddelta, fl == 1)
    x = kr.solve(max_iter)
    scale = np.zeros(rows.shape, dtype=float)
    scale[rows] = np.squeeze(x)

    def apply(s):
        d = sparse.diags([s], [0])
        return d.dot(full).dot(d)
    scale *= np.sqrt(full.sum() / apply(scale).sum())
    balanced = apply(scale)
    nz = scale != 0
    scale[nz] = 1 / scale[nz]
    if upper_input:
        balanced = sparse.triu(balanced).tocsr()
    return balanced, scale, np.array(kr.history)
