from hic3defdr_amd.analysis.constructor import HiC3DeFDR  # noqa: F401
