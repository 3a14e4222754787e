"""The GRM's slab reduce fused into the persistent tile kernel (GBM_GRM_FUSED, csrc/grm.hip
SliceBounds::fuse): the unit that draws a tile's last ticket sums the tile's loci-range slabs into G in
range order, from 0.0, as grm_slab_reduce_kernel does — so G must be the SAME BITS as with the separate
reduce, for every split, ragged shapes (the edge columns), and G += accumulation (the streamed fit).
The GRM is the product of reference src/gwas.jl:124 (GenomicBreedingCore.grmsimple)."""
import numpy as np
import pytest

import gbm
import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


@pytest.mark.parametrize("n,p,split", [
    (1030, 1234, "4,2,1,1"),  # ragged last tile column of 6 (edge kernel beside the tiles)
    (4999, 600, None),        # the planner's split, C2-like ragged n
    (1100, 2049, "3,1"),      # last column of 76: masked tiles, no edge
    (700, 5000, "1,1,1,1,1,1,1,1"),
    (2048, 3000, None),       # whole tiles, no edge
])
def test_grm_fused_reduce_same_bits(gbm_env, n, p, split):
    X = oracle.synth_genotypes(n * 3 + p, n, p)
    gbm_env.setenv("GBM_GRM_CARRY", "0")
    if split:
        gbm_env.setenv("GBM_GRM_SPLIT", split)
    gbm_env.setenv("GBM_GRM_FUSED", "0")
    G0, q0 = gbm.grm(X)
    gbm_env.setenv("GBM_GRM_FUSED", "1")
    assert gbm.load_library().gbm_dev_grm_slices(n, p) > 1
    G1, q1 = gbm.grm(X)
    G2, _ = gbm.grm(X)  # tickets and slabs reused by a second call
    Gr, qr = oracle.grm(X)
    assert q0 == q1 == qr
    assert np.array_equal(G0, G1) and np.array_equal(G1, G2)
    assert rel(G1, Gr) < 1e-12


def test_gblup_fused_matches_oracle(gbm_env):
    gbm_env.setenv("GBM_GRM_FUSED", "1")
    n, p = 1030, 3000
    X = oracle.synth_genotypes(21, n, p)
    Y = oracle.synth_phenotypes(X, 22, ntraits=2)
    b_hat, y_pred, mu, q = gbm.gblup_arrays(X, Y, lambda_=1.0)
    ref = oracle.gblup_fit(X, Y, 1.0)
    assert q == ref["q"] and rel(y_pred, ref["y_pred"]) < 1e-9 and rel(b_hat, ref["b_hat"]) < 1e-6


def test_streamed_accumulating_fit_fused_same_bits(gbm_env):
    """Loci-streamed fit: every chunk's GRM is added into G (accum); the fused epilogue adds the old G
    tile first, as the reduce kernel does."""
    n, p, chunk = 700, 5000, 1500
    X = oracle.synth_genotypes(77, n, p)
    Y = oracle.synth_phenotypes(X, 78, ntraits=2)
    gbm_env.setenv("GBM_HOST_CHUNK", str(chunk))
    gbm_env.setenv("GBM_STREAM_CHUNK", str(chunk))
    gbm_env.setenv("GBM_GRM_FUSED", "0")
    r = gbm.gblup_arrays(X, Y)
    gbm_env.setenv("GBM_GRM_FUSED", "1")
    s = gbm.gblup_arrays(X, Y)
    for a, b in zip(s, r):
        assert np.array_equal(np.asarray(a), np.asarray(b))
