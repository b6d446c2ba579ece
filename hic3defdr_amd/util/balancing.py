"""Knight-Ruiz matrix balancing (reference hic3defdr/util/balancing.py:5-208;
Knight & Ruiz, IMA J. Numer. Anal. 2013), used to produce bias vectors for
simulated replicates before they are analysed (README.md:586-614).

Host code (scipy.sparse): a few hundred sparse mat-vecs per matrix, outside
the hot path. The inner conjugate-gradient step and the outer Newton update
follow the published algorithm with the reference's constants (eta_max 0.1,
g 0.9, delta/Delta clamps, the "sum factor" rescale of Juicer)."""
import numpy as np
import scipy.sparse as sparse


def _symmetric_from_upper(array):
    up = sparse.triu(sparse.csr_matrix(array))
    return (up + up.transpose() - sparse.diags([up.diagonal()], [0])).tocsr()


def kr_balance(array, tol=1e-6, x0=None, delta=0.1, ddelta=3, fl=1,
               max_iter=3000):
    """Returns (balanced CSR, bias, residual norms). ``array`` is symmetrised
    from its upper triangle; empty rows are dropped for the iteration and get
    bias 0. bias is the inverse of the KR scaling vector, rescaled so the
    balanced matrix keeps the original total (reference :179-201); the
    balanced matrix is upper triangular when the input was."""
    triu = sparse.tril(array, k=-1).nnz == 0
    full = _symmetric_from_upper(array)
    nz = full.getnnz(1) > 0
    A = full[nz, :][:, nz]
    n = A.shape[0]
    x = np.ones((n, 1)) if x0 is None else x0
    g, eta_max = 0.9, 0.1
    eta = eta_max
    stop_tol = tol * 0.5
    rt = tol ** 2
    v = x * A.dot(x)
    rk = 1 - v
    rho_km1 = float(np.dot(rk.T, rk)[0, 0])
    rout = rold = rho_km1
    res = []
    it = 0
    if fl == 1:
        print('it in. it res')
    while rout > rt:
        if max_iter is not None and it > max_iter:
            break
        it += 1
        k = 0
        y = np.ones((n, 1))
        innertol = max(eta ** 2 * rout, rt)
        rho_km2 = None
        # inner CG on (diag(x) A diag(x) + diag(v)) y = 1, kept inside
        # [delta, Delta] by a step clamp
        while rho_km1 > innertol:
            k += 1
            if k == 1:
                z = rk / v
                p = z.copy()
                rho_km1 = np.dot(rk.T, z)
            else:
                p = z + (rho_km1 / rho_km2) * p
            w = x * A.dot(x * p) + v * p
            alpha = rho_km1 / np.dot(p.T, w)
            ap = alpha * p
            ynew = y + ap
            if np.min(ynew) <= delta:
                if delta == 0:
                    break
                neg = np.where(ap < 0)
                y = y + np.min((delta - y[neg]) / ap[neg]) * ap
                break
            if np.max(ynew) >= ddelta:
                big = np.where(ynew > ddelta)
                y = y + min((ddelta - y[big]) / ap[big]) * ap
                break
            y = ynew
            rk = rk - alpha * w
            rho_km2 = rho_km1
            z = rk / v
            rho_km1 = np.dot(rk.T, z)
        x = x * y
        v = x * A.dot(x)
        rk = 1 - v
        rho_km1 = float(np.dot(rk.T, rk)[0, 0])
        rout = rho_km1
        rat = rout / rold
        rold = rout
        res_norm = np.sqrt(rout)
        eta_0 = eta
        eta = g * rat
        if g * eta_0 ** 2 > 0.1:
            eta = max(eta, g * eta_0 ** 2)
        eta = max(min(eta, eta_max), stop_tol / res_norm)
        if fl == 1:
            print('{} {} {:.3e}'.format(it, k, res_norm))
            res.append(res_norm)
    bias = np.zeros(nz.shape, dtype=float)
    bias[nz] = np.squeeze(x)
    # Juicer's sum factor: the balanced matrix keeps the original total
    d = sparse.diags([bias], [0])
    bias *= np.sqrt(full.sum() / d.dot(full).dot(d).sum())
    d = sparse.diags([bias], [0])
    balanced = d.dot(full).dot(d)
    bias[bias != 0] = 1 / bias[bias != 0]
    if triu:
        balanced = sparse.triu(balanced).tocsr()
    return balanced, bias, np.array(res)
