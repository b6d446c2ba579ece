"""Synthetic Hi-C generator in the reference's on-disk input layout.

The demo data of the reference (``hic3defdr/util/demo_data.py:8``, a Dropbox
URL) is not reachable offline, so every workload in this repo is synthetic.
The generator follows SURVEY.md §8(d):

- upper-triangular CSR per replicate with distances up to ``dmax + 50``;
- mean ``mu(d) = 400 * (d + 1) ** -1`` with 0.2 % "loop" pixels at x5;
- replicate depth factor ``0.8 + 0.1 k``; 1 % of pixels x2 in the second and
  later conditions;
- per-bin bias ``exp(N(0, 0.25))`` with 1 % of bins at 0.05 (fails
  ``bias_thresh``);
- counts ``NB(n = 1/0.05, p = n / (n + mu * b_i * b_j))``;
- loop clusters: 3x3 blocks written as the reference's sparse cluster JSON
  (``hic3defdr/util/clusters.py:116-136`` format: list of lists of [i, j]).

Layout (``README.md:259-301`` of the reference): ``<base>/<rep>/<chrom>_raw.npz``
(``scipy.sparse.save_npz``), ``<base>/<rep>/<chrom>_kr.bias`` (``np.savetxt``),
``<base>/clusters/<cond>_<chrom>.json``.

Only numpy/scipy are imported so the golden-generation script can run this
module under the reference's own interpreter.
"""
import json
import os

import numpy as np
import scipy.sparse as sp


def default_design(n_per_cond=(2, 2), cond_names=None):
    """Replicate names and a boolean design matrix ``(R, C)``."""
    if cond_names is None:
        cond_names = ['ES', 'NPC', 'XC', 'YC', 'ZC'][:len(n_per_cond)]
    reps, design = [], []
    for c, (name, n) in enumerate(zip(cond_names, n_per_cond)):
        for k in range(n):
            reps.append('%s_%d' % (name, k + 1))
            row = [False] * len(n_per_cond)
            row[c] = True
            design.append(row)
    return reps, list(cond_names), np.array(design, dtype=bool)


def band_pixels(n_bins, max_d):
    """Row/col of every upper-triangular pixel with ``0 <= col-row <= max_d``."""
    r, c = [], []
    for d in range(0, min(max_d, n_bins - 1) + 1):
        i = np.arange(0, n_bins - d, dtype=np.int64)
        r.append(i)
        c.append(i + d)
    return np.concatenate(r), np.concatenate(c)


def generate_chrom(rng, n_bins, max_d, design, disp=0.05, loop_frac=0.002,
                   diff_frac=0.01, bad_bin_frac=0.01):
    """One chromosome: returns (list of CSR per replicate, bias (n_bins, R))."""
    R = design.shape[0]
    cond_of_rep = design.argmax(axis=1)
    r, c = band_pixels(n_bins, max_d)
    d = c - r
    base = 400.0 * (d + 1.0) ** -1.0
    loopy = rng.random(r.size) < loop_frac
    base = base * np.where(loopy, 5.0, 1.0)
    diff = rng.random(r.size) < diff_frac
    mats, biases = [], []
    for k in range(R):
        bias = np.exp(rng.normal(0, 0.25, n_bins))
        bias[rng.random(n_bins) < bad_bin_frac] = 0.05
        cond_eff = np.where(diff, 2.0, 1.0) if cond_of_rep[k] >= 1 else 1.0
        mu = base * cond_eff * bias[r] * bias[c] * (0.8 + 0.1 * k)
        n = 1.0 / disp
        p = n / (n + mu)
        x = rng.negative_binomial(n, p)
        keep = x > 0
        m = sp.coo_matrix((x[keep], (r[keep], c[keep])),
                          shape=(n_bins, n_bins)).tocsr()
        mats.append(m)
        biases.append(bias)
    return mats, np.array(biases).T


def generate_clusters(rng, n_bins, max_d, n_clusters, min_d=10):
    """Random 3x3 loop clusters with ``min_d <= col-row <= max_d``."""
    clusters = []
    for _ in range(n_clusters):
        d = int(rng.integers(min_d, max(min_d + 1, max_d - 2)))
        i = int(rng.integers(0, max(1, n_bins - d - 3)))
        clusters.append([[i + a, i + d + b] for a in range(3) for b in range(3)
                         if 0 <= i + a < n_bins and i + d + b < n_bins])
    return clusters


def write_dataset(base, chrom_sizes, dist_thresh_max=200, n_per_cond=(2, 2),
                  seed=0, disp=0.05, clusters_per_chrom=None, extra_d=50):
    """Writes a synthetic dataset and returns a dict of constructor kwargs.

    ``chrom_sizes`` maps chromosome name -> number of bins.
    """
    rng = np.random.default_rng(seed)
    reps, conds, design = default_design(n_per_cond)
    for rep in reps:
        os.makedirs(os.path.join(base, rep), exist_ok=True)
    os.makedirs(os.path.join(base, 'clusters'), exist_ok=True)
    for chrom, n_bins in chrom_sizes.items():
        mats, bias = generate_chrom(rng, n_bins, dist_thresh_max + extra_d,
                                    design, disp=disp)
        for k, rep in enumerate(reps):
            sp.save_npz(os.path.join(base, rep, '%s_raw.npz' % chrom), mats[k])
            np.savetxt(os.path.join(base, rep, '%s_kr.bias' % chrom),
                       bias[:, k])
        n_cl = clusters_per_chrom if clusters_per_chrom is not None \
            else max(3, n_bins // 50)
        for cond in conds:
            cl = generate_clusters(rng, n_bins, dist_thresh_max, n_cl)
            with open(os.path.join(base, 'clusters',
                                   '%s_%s.json' % (cond, chrom)), 'w') as fh:
                json.dump(cl, fh)
    return {
        'raw_npz_patterns': [os.path.join(base, r, '<chrom>_raw.npz')
                             for r in reps],
        'bias_patterns': [os.path.join(base, r, '<chrom>_kr.bias')
                          for r in reps],
        'chroms': list(chrom_sizes),
        'reps': reps,
        'conds': conds,
        'design': design,
        'loop_patterns': {c: os.path.join(base, 'clusters',
                                          '%s_<chrom>.json' % c)
                          for c in conds},
    }


# mm10 chr1..chr19, chrX at 10 kb (bins): BASELINE.json configs[2] (cfg3)
MM10_BINS = [19535, 18211, 16007, 15649, 15171, 14950, 14546, 12930, 12459,
             13069, 12208, 12013, 12042, 12490, 10404, 9820, 9499, 9070, 6143,
             17102]


def _write_genome_chrom(args):
    base, i, n_bins, seed, dmax, n_per_cond = args
    chrom = 'chr%d' % (i + 1)
    reps, conds, design = default_design(n_per_cond)
    rng = np.random.default_rng([seed, i])
    mats, bias = generate_chrom(rng, n_bins, dmax + 50, design)
    for k, rep in enumerate(reps):
        sp.save_npz(os.path.join(base, rep, '%s_raw.npz' % chrom), mats[k])
        np.savetxt(os.path.join(base, rep, '%s_kr.bias' % chrom), bias[:, k])
    for cond in conds:
        cl = generate_clusters(rng, n_bins, dmax, max(3, n_bins // 50))
        with open(os.path.join(base, 'clusters', '%s_%s.json' % (cond, chrom)),
                  'w') as fh:
            json.dump(cl, fh)
    return chrom


def write_genome(base, bins, seed=3, workers=8, dmax=200, n_per_cond=(2, 2)):
    """A whole genome (chromosome i = 'chr<i+1>' of bins[i] bins, each drawn
    from its own seed [seed, i]) in the reference's input layout -- per
    replicate NPZ + bias files, loop-cluster JSON -- written by a process pool
    (cfg3 end to end: tools/run_e2e.py, tests/test_gpu_cfg3.py). Returns the
    constructor kwargs as write_dataset."""
    from concurrent.futures import ProcessPoolExecutor
    reps, conds, design = default_design(n_per_cond)
    for rep in reps:
        os.makedirs(os.path.join(base, rep), exist_ok=True)
    os.makedirs(os.path.join(base, 'clusters'), exist_ok=True)
    # largest chromosomes first so the pool's tail is short
    order = sorted(range(len(bins)), key=lambda i: -bins[i])
    jobs = [(base, i, bins[i], seed, dmax, tuple(n_per_cond)) for i in order]
    if workers > 1:
        with ProcessPoolExecutor(workers) as ex:
            list(ex.map(_write_genome_chrom, jobs))
    else:
        for j in jobs:
            _write_genome_chrom(j)
    chroms = ['chr%d' % (i + 1) for i in range(len(bins))]
    return dict(
        raw_npz_patterns=[os.path.join(base, r, '<chrom>_raw.npz') for r in reps],
        bias_patterns=[os.path.join(base, r, '<chrom>_kr.bias') for r in reps],
        chroms=chroms, reps=reps, conds=conds, design=design,
        loop_patterns={c: os.path.join(base, 'clusters', '%s_<chrom>.json' % c)
                       for c in conds})


def draw_band(n_bins, n_per_cond, dmax, seed=0, chrom_index=0, disp=0.05,
              workers=8, keys=False):
    """The disp pixels of one chromosome drawn directly in the distance band,
    no files (the cfg3 / cfg4 shapes, where writing NPZ files for a whole
    genome would dominate): the generator model above with unit size
    factors -- mu(d) = 400 (d+1)^-1, 0.2 % loops x5, 1 % differential x2 in
    conditions >= 1, per-bin bias exp(N(0, .25)), depth 0.8 + 0.1 (k mod 4),
    NB(1/disp) -- and disp_idx as prepare_data computes it with unit size
    factors: every condition's mean of raw / (b_i b_j) >= 1 and d >= 4.
    The streams are seeded by (seed, chrom_index) -- one for the band, one
    per replicate (SeedSequence children), the replicates drawn on `workers`
    threads (numpy's bulk draws release the GIL) -- so a rank can draw just
    its own chromosomes and every world size sees the same genome. Returns
    (raw (n, R) int32, f (n, R) f64, dist (n,) int32); with ``keys`` also
    (row (n,) int32, bias (n_bins, R)): f = (bias[row] * bias[row + dist])
    * 1 (unit size factors), what the distance re-shard rebuilds f from."""
    import concurrent.futures
    R = int(sum(n_per_cond))
    kids = np.random.SeedSequence([seed, chrom_index]).spawn(R + 1)
    rng = np.random.default_rng(kids[0])
    cond = np.repeat(np.arange(len(n_per_cond)), n_per_cond)
    top = min(dmax, n_bins - 1)
    d = np.concatenate([np.full(n_bins - k, k, dtype=np.int32)
                        for k in range(top + 1)])
    r = np.concatenate([np.arange(n_bins - k, dtype=np.int32)
                        for k in range(top + 1)])
    c = r + d
    base = 400.0 / (d + 1.0)
    base *= np.where(rng.random(d.size) < 0.002, 5.0, 1.0)
    diff = rng.random(d.size) < 0.01
    raw = np.empty((d.size, R), dtype=np.int32)
    f = np.empty((d.size, R))
    bias = np.empty((n_bins, R))
    n = 1.0 / disp

    def replicate(k):
        g = np.random.default_rng(kids[k + 1])
        b = np.exp(g.normal(0, 0.25, n_bins))
        bias[:, k] = b
        bb = b[r] * b[c]
        mu = base * np.where(diff & (cond[k] >= 1), 2.0, 1.0) * bb * \
            (0.8 + 0.1 * (k % 4))
        raw[:, k] = g.negative_binomial(n, n / (n + mu))
        f[:, k] = bb
    with concurrent.futures.ThreadPoolExecutor(max(1, min(workers, R))) as ex:
        list(ex.map(replicate, range(R)))
    keep = d >= 4
    for ci in range(len(n_per_cond)):
        keep &= (raw[:, cond == ci] / f[:, cond == ci]).mean(axis=1) >= 1.0
    out = (np.ascontiguousarray(raw[keep]), np.ascontiguousarray(f[keep]),
           np.ascontiguousarray(d[keep]))
    if keys:
        out += (np.ascontiguousarray(r[keep]), bias)
    return out


def draw_genome(bins_list, n_per_cond, dmax, seed=0, indices=None,
                workers=8, keys=False):
    """draw_band for the chromosomes `indices` (default all) of a genome
    given as a list of bin counts, drawn concurrently (each chromosome has
    its own generator; numpy draws release the GIL). Returns the list of
    (raw, f, dist) in `indices` order."""
    import concurrent.futures
    idx = list(range(len(bins_list))) if indices is None else list(indices)
    with concurrent.futures.ThreadPoolExecutor(max(1, min(workers,
                                                          len(idx)))) as ex:
        # (the chromosomes in parallel, each one's replicates serially)
        return list(ex.map(lambda i: draw_band(bins_list[i], n_per_cond, dmax,
                                               seed=seed, chrom_index=i,
                                               workers=1, keys=keys),
                           idx))
