"""HiC3DeFDR class shell (reference hic3defdr/analysis/constructor.py:12-86)."""
import os
import pickle

import pandas as pd

from hic3defdr_amd.analysis.core import CoreHiC3DeFDR
from hic3defdr_amd.analysis.analysis import AnalyzingHiC3DeFDR
from hic3defdr_amd.analysis.simulation import SimulatingHiC3DeFDR


class HiC3DeFDR(CoreHiC3DeFDR, AnalyzingHiC3DeFDR, SimulatingHiC3DeFDR):
    """Main object for a hic3defdr analysis (MI355X-native hot path).

    Same constructor as the reference (``constructor.py:62-86``):

    raw_npz_patterns : list of str
        ``scipy.sparse.save_npz`` contact matrices per replicate, with
        ``<chrom>`` placeholders.
    bias_patterns : list of str
        ``np.savetxt`` bias vectors per replicate, with ``<chrom>``.
    chroms : list of str
    design : pd.DataFrame or str
        Boolean (replicates x conditions); a string is read with
        ``pd.read_csv(design, index_col=0)``.
    outdir : str
    dist_thresh_min, dist_thresh_max : int
    bias_thresh : float
    mean_thresh : float
    loop_patterns : dict of str, optional
        condition -> sparse cluster JSON pattern with ``<chrom>``.
    res : int, optional
    """

    def __init__(self, raw_npz_patterns, bias_patterns, chroms, design, outdir,
                 dist_thresh_min=4, dist_thresh_max=200, bias_thresh=0.1,
                 mean_thresh=1.0, loop_patterns=None, res=None):
        self.raw_npz_patterns = raw_npz_patterns
        self.bias_patterns = bias_patterns
        self.chroms = chroms
        if type(design) == str:
            self.design = pd.read_csv(design, index_col=0)
        else:
            self.design = design
        self.outdir = outdir
        self.dist_thresh_min = dist_thresh_min
        self.dist_thresh_max = dist_thresh_max
        self.bias_thresh = bias_thresh
        self.mean_thresh = mean_thresh
        self.loop_patterns = loop_patterns
        self.res = res
        state = self.__dict__.copy()
        del state['outdir']
        os.makedirs(self.outdir, exist_ok=True)
        with open(self.picklefile, 'wb') as handle:
            pickle.dump(state, handle, -1)
